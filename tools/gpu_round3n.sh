#!/bin/bash
# round 3 final: GPU suite, smoke, bench, bench profile, gradient kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_run.sh suite smoke bench || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof2 -o gp -- python3 tools/prof_grad.py 5 > gpurun_out/prof_grad_final.json 2> gpurun_out/prof_grad_final.err || exit 1
cut -c1-300 gpurun_out/prof_grad_final.json
find gpurun_out/gprof2 -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200
bash tools/gpu_run.sh profile || exit $?
