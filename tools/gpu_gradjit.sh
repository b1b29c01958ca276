#!/bin/bash
# Gradient tree code: GPU tests, then the config #5 shard gradient timing
# (tools/prof_grad.py) with per-pass times.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_jit_grad_gpu.py tests/test_gradients.py tests/test_constant_optimization.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gradjit.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gradjit.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SRHIP_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/prof_grad.py 3 > gpurun_out/prof_grad.log 2>&1 || exit $?
tail -6 gpurun_out/prof_grad.log
