#!/bin/bash
# round 3: workgroup size at the strong-scaling shard sizes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_env.py --ntrees 512,1024,4096 --steps 30 '' 'SRHIP_JIT_WAVES=8' 'SRHIP_JIT_WAVES=2' > gpurun_out/ab_waves.txt 2>&1 || exit 1
cat gpurun_out/ab_waves.txt
