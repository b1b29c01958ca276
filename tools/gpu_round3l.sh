#!/bin/bash
# round 3: finalize with 16 slots per workgroup; config #3 output call in bench_configs
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u tools/step_overhead.py > gpurun_out/step_overhead.txt 2>&1 || exit 1
cat gpurun_out/step_overhead.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin -o fin -- python3 tools/prof_target.py 10 > gpurun_out/fin.log 2>&1 || exit 1
find gpurun_out/fin -name "*kernel_stats.csv" | head -1 | xargs cut -c1-180
timeout -k 10 400 python -u tools/bench_configs.py --only 1,3 > gpurun_out/configs13.jsonl 2>&1 || exit 1
cat gpurun_out/configs13.jsonl
