# launch-geometry knobs at the N = 8 shard sizes (tools/geom_sweep.py, one process per setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/geom
for r in 1 2; do
  for mpg in 64 16 32 128; do
    for kind in trees rows; do
      SRHIP_MIN_PER_GROUP=$mpg timeout -k 10 200 python3 tools/geom_sweep.py $kind 8 20 >> gpurun_out/geom/sweep.jsonl 2>> gpurun_out/geom/err.log || { echo "sweep failed"; exit 1; }
      tail -1 gpurun_out/geom/sweep.jsonl
    done
  done
done
