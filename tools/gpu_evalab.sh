#!/bin/bash
# loss tree code (config #2): kernel time, three runs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for k in 1 2 3; do
  SRHIP_DEBUG_PASSES=1 timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || exit $?
  tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), 'ms/step', round(d['ms_per_step'],3), 'value', d['value'])"
done
