#!/bin/bash
# multi-part tree code: GPU tests for the tree code, then configs #1/#3/#5 throughput
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py tests/test_full_size.py tests/test_configs_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_parts.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_parts.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SRHIP_DEBUG_PASSES=1 timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/configs.log 2> gpurun_out/configs_err.log || exit $?
cat gpurun_out/configs.log; grep "tree-code part\|pass" gpurun_out/configs_err.log | tail -12
