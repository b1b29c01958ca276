#!/bin/bash
# tiles per workgroup of the loss tree code at the strong-scaling shard sizes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for nt in 0 2 3 6; do
  echo "== SRHIP_TREE_NT=$nt (0: planner)"
  SRHIP_TREE_NT=$nt timeout -k 10 300 python3 tools/step_overhead.py || exit $?
done
