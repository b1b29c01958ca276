#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { echo "== $*"; env "$@" SRHIP_DEBUG_PASSES=1 timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/nt.log 2>&1 || exit $?;
        grep "tree-code" gpurun_out/nt.log | tail -1; tail -1 gpurun_out/nt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"; }
run SRHIP_TREE_NT=0
run SRHIP_TREE_NT=5
run SRHIP_TREE_NT=6
run SRHIP_TREE_NT=3
run SRHIP_TREE_NT=0
