#!/bin/bash
# GPU test suite only (no bench); output streamed to gpurun_out/pytest_gpu.log
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TMO:-600} python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
exit $rc
