#!/bin/bash
# zero-copy results: GPU suite subset + per-call overhead with and without
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_gpu_parity.py tests/test_jit_grad_gpu.py tests/test_constant_optimization.py tests/test_search.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_zc.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_zc.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 4 ]; then exit $rc; fi
for z in 1 0 1; do echo "== SRHIP_ZERO_COPY=$z"; SRHIP_ZERO_COPY=$z timeout -k 10 300 python3 tools/step_overhead.py || exit $?; done
