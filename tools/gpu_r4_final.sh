#!/bin/bash
# Round-4 validation after the tree-code bar change: GPU suite + smoke, then
# the N = 8 shard probe (tree and row shards; tools/shard_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_suite.sh || exit $?
timeout -k 10 300 python3 tools/shard_probe.py 10 > gpurun_out/shard_probe_r4c.json 2> gpurun_out/shard_probe_r4c.err || exit $?
python3 - <<'PY'
import json
p = json.loads(open("gpurun_out/shard_probe_r4c.json").read())
for k in ("strided", "balanced", "strided_precise"):
    print(k, round(p[k]["max_wall_ms"], 3), [(round(s["wall_ms"], 3), s.get("redone_tiles")) for s in p[k]["shards"]])
print("full", round(p["full"]["wall_ms"], 3), "strided proj", round(p["strided"]["projected_speedup_wall"], 2),
      "rows", {k: round(v["projected_speedup_wall_no_allreduce"], 2) for k, v in p["rows"].items()})
PY
