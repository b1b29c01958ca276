#!/bin/bash
# Configs #3 (Float64: tree code vs SRHIP_JIT64=0 interpreter) and #5 on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/configs_r4.jsonl; : > $out
SRHIP_JIT64=0 timeout -k 10 300 python3 tools/bench_configs.py --only 3 >> $out 2>> gpurun_out/configs_r4.err || exit $?
timeout -k 10 300 python3 tools/bench_configs.py --only 3 >> $out 2>> gpurun_out/configs_r4.err || exit $?
timeout -k 10 400 python3 tools/bench_configs.py --only 5 >> $out 2>> gpurun_out/configs_r4.err || exit $?
cat $out
timeout -k 10 300 python3 tools/shard_probe.py 10 > gpurun_out/shard_probe_r4b.json 2> gpurun_out/shard_probe_r4b.err || exit $?
python3 - <<'PY'
import json
p = json.loads(open("gpurun_out/shard_probe_r4b.json").read())
for k in ("strided", "balanced", "strided_precise"):
    print(k, [(round(s["wall_ms"], 3), s.get("redone_tiles")) for s in p[k]["shards"]])
print("full", p["full"], "precise full", p["strided_precise"]["full"])
PY
