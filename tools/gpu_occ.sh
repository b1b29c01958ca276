#!/bin/bash
# occupancy sensitivity of the tree-code eval kernel (config #2): extra LDS per
# workgroup lowers the resident workgroups per CU (28 KB each by default: 5)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pad in ${PADS:-0 5000 14000 26000}; do
  SRHIP_JIT_LDS_PAD=$pad timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 10 > gpurun_out/occ.log 2>&1 || exit $?
  tail -1 gpurun_out/occ.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pad', $pad, 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
done
