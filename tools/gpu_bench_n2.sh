#!/bin/bash
# Rehearsal of bench.py's N > 1 paths on a one-GPU box: two ranks on GPU 0
# over gloo (SRHIP_BENCH_SHARED_GPU=1), row shards and tree shards; then the
# N = 1 bench line. The N = 2 numbers are not a measurement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export SRHIP_BENCH_SHARED_GPU=1
timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --rs-steps 2 > gpurun_out/bench_n2_rows.json 2> gpurun_out/bench_n2_rows.err || { tail -20 gpurun_out/bench_n2_rows.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 2 --shard trees --steps 5 --warmup 2 --no-row-shard > gpurun_out/bench_n2_trees.json 2> gpurun_out/bench_n2_trees.err || { tail -20 gpurun_out/bench_n2_trees.err; exit 1; }
unset SRHIP_BENCH_SHARED_GPU
timeout -k 10 400 python3 bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_n2_rows", "bench_n2_trees", "bench_n1"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["n_gpus"], round(d["value"] / 1e12, 3), "T", round(d["ms_per_step"], 3), "ms", d["config"]["parallelism"][:60],
          "row_shard", d["row_shard"] and round(d["row_shard"]["ms_per_step"], 1))
PY
