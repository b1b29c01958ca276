#!/bin/bash
# round 3: gradient accumulation by fma into the constant accumulators
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_grad_gpu.py tests/test_constant_optimization.py tests/test_configs_gpu.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/pytest_3m.log 2>&1 || { tail -30 gpurun_out/pytest_3m.log; exit 1; }
tail -2 gpurun_out/pytest_3m.log
timeout -k 10 200 python -u tools/prof_grad.py 5 > gpurun_out/prof_grad_accfma.json 2>&1 || exit 1
SRHIP_GJIT_ACC_FMA=0 timeout -k 10 200 python -u tools/prof_grad.py 5 > gpurun_out/prof_grad_noaccfma.json 2>&1 || exit 1
cat gpurun_out/prof_grad_accfma.json gpurun_out/prof_grad_noaccfma.json | cut -c1-400
timeout -k 10 300 python -u tools/debug_grads.py > gpurun_out/debug_grads.txt 2>&1 || exit 1
grep -E "==|beyond" gpurun_out/debug_grads.txt
