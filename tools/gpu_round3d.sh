#!/bin/bash
# round 3: self-cleaning finalize (per-call overhead), constant-map set_constants, gradient diagnostics
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_jit_gpu.py tests/test_constant_optimization.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_3d.log 2>&1 || { tail -30 gpurun_out/pytest_3d.log; exit 1; }
tail -3 gpurun_out/pytest_3d.log
timeout -k 10 200 python -u tools/step_overhead.py > gpurun_out/step_overhead.txt 2>&1 || exit 1
cat gpurun_out/step_overhead.txt
timeout -k 10 300 python -u tools/prof_constopt.py > gpurun_out/constopt_profile.txt 2>&1 || exit 1
head -25 gpurun_out/constopt_profile.txt
timeout -k 10 400 python -u tools/debug_grads.py > gpurun_out/debug_grads.txt 2>&1 || exit 1
cat gpurun_out/debug_grads.txt
