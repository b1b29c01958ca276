#!/bin/bash
# round 3: split finalize; workgroup size at the strong-scaling shard sizes; config #3 output call
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_jit_gpu.py tests/test_full_size.py tests/test_distributed_gpu.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/pytest_3j.log 2>&1 || { tail -30 gpurun_out/pytest_3j.log; exit 1; }
tail -2 gpurun_out/pytest_3j.log
timeout -k 10 200 python -u tools/step_overhead.py > gpurun_out/step_overhead.txt 2>&1 || exit 1
cat gpurun_out/step_overhead.txt
timeout -k 10 500 python -u tools/ab_env.py --ntrees 512,4096 --steps 30 '' 'SRHIP_FIN_SLICES=1' 'SRHIP_JIT_WAVES=8' > gpurun_out/ab_waves.txt 2>&1 || exit 1
cat gpurun_out/ab_waves.txt
timeout -k 10 300 python -u tools/out_copy.py 16 > gpurun_out/out_copy2.txt 2>&1 || exit 1
cat gpurun_out/out_copy2.txt
timeout -k 10 300 python -u tools/bench_configs.py --only 3 > gpurun_out/configs3.jsonl 2>&1 || exit 1
cat gpurun_out/configs3.jsonl
