#!/bin/bash
# round 3: tail split of the tree-code grid (A/B + parity), host copy throughput
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/pytest_3g.log 2>&1 || { tail -30 gpurun_out/pytest_3g.log; exit 1; }
tail -2 gpurun_out/pytest_3g.log
timeout -k 10 400 python -u tools/ab_env.py --ntrees 512,1024,2048,4096 --steps 30 '' 'SRHIP_JIT_TAIL=0' > gpurun_out/ab_tail.txt 2>&1 || exit 1
cat gpurun_out/ab_tail.txt
timeout -k 10 200 python -u tools/step_overhead.py > gpurun_out/step_overhead.txt 2>&1 || exit 1
cat gpurun_out/step_overhead.txt
timeout -k 10 120 ./tools/hostcopy > gpurun_out/hostcopy.txt 2>&1 || exit 1
cat gpurun_out/hostcopy.txt
