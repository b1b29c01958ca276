#!/bin/bash
# loss tree code (config #2): XCD-aligned tree groups and the LDS tile budget
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { echo "== $*"; env "$@" SRHIP_DEBUG_PASSES=1 timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/knob.log 2>&1 || exit $?;
        grep "tree-code" gpurun_out/knob.log | tail -1; tail -1 gpurun_out/knob.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), 'ms/step', round(d['ms_per_step'],3))"; }
run SRHIP_XCD_NTG=0
run SRHIP_XCD_NTG=1
run SRHIP_XCD_NTG=0 SRHIP_EVAL_LDS=56
run SRHIP_XCD_NTG=1 SRHIP_EVAL_LDS=56
run SRHIP_XCD_NTG=1 SRHIP_EVAL_LDS=100
