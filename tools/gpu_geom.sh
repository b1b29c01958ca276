#!/bin/bash
# Geometry sweep at the N = 8 shard sizes (tools/geom_sweep.py), one process per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/geom.jsonl; : > $out
run() { env "$@" timeout -k 10 120 python3 tools/geom_sweep.py $KIND $N 20 >> $out 2>>gpurun_out/geom.err || exit $?; }
KIND=rows N=1 run SRHIP_DEBUG_PASSES=1
for N in 8 4; do
  KIND=rows
  run SRHIP_DEBUG_PASSES=1
  for t in 8192 16384 32768; do for m in 16 32 64; do run SRHIP_TARGET_WG=$t SRHIP_MIN_PER_GROUP=$m; done; done
  for nt in 1 2 4 8; do run SRHIP_TREE_NT=$nt; done
  run SRHIP_JIT_TAIL=0
done
KIND=trees N=8
run SRHIP_DEBUG_PASSES=1
for t in 8192 16384 32768; do for m in 8 16 32 64; do run SRHIP_TARGET_WG=$t SRHIP_MIN_PER_GROUP=$m; done; done
for nt in 2 4 8 16; do run SRHIP_TREE_NT=$nt; done
echo done; wc -l $out
