#!/bin/bash
# Tree-code kernel time against resident waves per SIMD (LDS padding lowers it).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pad in ${PADS:-0 10000 20000}; do
  SRHIP_JIT_LDS_PAD=$pad timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/occ_$pad.json 2> gpurun_out/occ_$pad.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/occ_$pad.json'));print('pad $pad', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
