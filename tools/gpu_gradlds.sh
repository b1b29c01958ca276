#!/bin/bash
# gradient tree code: LDS tile budget sweep on the config #5 shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in ${BUDGETS:-40 52 64 80}; do
  SRHIP_GJIT_LDS=$b SRHIP_DEBUG_PASSES=1 timeout -k 10 120 python3 tools/prof_grad.py 2 > gpurun_out/gradlds_$b.log 2>&1 || exit $?
  echo "budget $b KiB: $(tail -1 gpurun_out/gradlds_$b.log)"; grep "part" gpurun_out/gradlds_$b.log | tail -2
done
