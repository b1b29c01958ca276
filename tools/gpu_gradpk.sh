#!/bin/bash
# gradient tree code: packed vs scalar (config #5 shard), plus the gradient GPU tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_jit_grad_gpu.py tests/test_gradients.py tests/test_constant_optimization.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gradpk.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gradpk.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for pk in 1 0 1; do SRHIP_JIT_PACKED=$pk timeout -k 10 200 python3 tools/prof_grad.py 3 > gpurun_out/gradpk.log 2>&1 || exit $?; echo "packed=$pk $(tail -1 gpurun_out/gradpk.log | cut -c1-220)"; done
