#!/bin/bash
# workgroup target of the tree-group planner at the strong-scaling shard sizes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in ${TARGETS:-8192 4096 2048 16384}; do
  echo "== SRHIP_TARGET_WG=$t"
  SRHIP_TARGET_WG=$t timeout -k 10 200 python3 tools/step_overhead.py > gpurun_out/twg.log 2>&1 || exit $?
  cat gpurun_out/twg.log
done
