#!/bin/bash
# round 3: gradient results kept in the routine registers; small-shard tree groups
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_jit_grad_gpu.py tests/test_constant_optimization.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_3i.log 2>&1 || { tail -30 gpurun_out/pytest_3i.log; exit 1; }
tail -2 gpurun_out/pytest_3i.log
timeout -k 10 200 python -u tools/prof_grad.py 5 > gpurun_out/prof_grad_keepva.json 2>&1 || exit 1
SRHIP_GJIT_KEEP_VA=0 timeout -k 10 200 python -u tools/prof_grad.py 5 > gpurun_out/prof_grad_nokeep.json 2>&1 || exit 1
cat gpurun_out/prof_grad_keepva.json gpurun_out/prof_grad_nokeep.json | cut -c1-400
timeout -k 10 400 python -u tools/ab_env.py --ntrees 512,1024 --steps 30 '' 'SRHIP_MIN_PER_GROUP=128' 'SRHIP_MIN_PER_GROUP=96' 'SRHIP_MIN_PER_GROUP=128 SRHIP_JIT_TAIL=0' > gpurun_out/ab_mpg.txt 2>&1 || exit 1
cat gpurun_out/ab_mpg.txt
