#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_jit_grad_gpu.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gradjit.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_gradjit.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/bench_constopt.py > gpurun_out/constopt.log 2>&1 || exit $?
SRHIP_GJIT=0 timeout -k 10 300 python3 tools/bench_constopt.py >> gpurun_out/constopt.log 2>&1 || exit $?
cat gpurun_out/constopt.log
