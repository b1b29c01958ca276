#!/bin/bash
# config #5 shard: tree-code workgroup waves (parity tests with SRHIP_JIT_WAVES=8 + A/B)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SRHIP_JIT_WAVES=8 timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_jit_gpu.py tests/test_full_size.py tests/test_distributed_gpu.py tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/pytest_waves.log 2>&1 || { tail -30 gpurun_out/pytest_waves.log; exit 1; }
tail -2 gpurun_out/pytest_waves.log
AB_CFG=5 timeout -k 10 600 python -u tools/ab_env.py --ntrees 16384 --steps 5 '' 'SRHIP_JIT_WAVES=8' > gpurun_out/ab_cfg5_auto.txt 2>&1 || { cat gpurun_out/ab_cfg5_auto.txt; exit 1; }
cat gpurun_out/ab_cfg5_auto.txt
timeout -k 10 300 python -u tools/ab_env.py --ntrees 4096,512 --steps 20 '' > gpurun_out/ab_cfg2_auto.txt 2>&1 || exit 1
cat gpurun_out/ab_cfg2_auto.txt
