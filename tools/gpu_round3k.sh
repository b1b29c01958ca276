#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/out_copy.py 16 16:after > gpurun_out/out_copy3.txt 2>&1 || exit 1
cat gpurun_out/out_copy3.txt
timeout -k 10 300 python -u tools/step_overhead.py > gpurun_out/step_overhead.txt 2>&1 || exit 1
cat gpurun_out/step_overhead.txt
