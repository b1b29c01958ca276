#!/bin/bash
# GPU tests, per-operator microbench, bench line — stop at the first crash/hang
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/microbench.py > gpurun_out/microbench.log 2>&1 || exit $?
cat gpurun_out/microbench.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
