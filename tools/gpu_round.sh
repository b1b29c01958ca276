#!/bin/bash
# tests → bench → profile, stopping at the first crash/hang (not at test failures)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then TAG=$PROFILE bash tools/gpu_profile.sh || exit $?; fi
