#!/bin/bash
# Tree-group-major block mapping A/B (SRHIP_TG_MAJOR, jit_template.hip block_of
# rotate 3): config #2, its N = 8 row and tree shards; then the loop check
# (identical sums) under it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/tgmajor.jsonl; : > $out
SRHIP_TG_MAJOR=1 timeout -k 10 120 python3 tools/dynloop_check.py > gpurun_out/tgm_check.jsonl 2>&1 || { cat gpurun_out/tgm_check.jsonl; exit 1; }
for rep in 1 2; do
  for tg in 0 1; do
    for kn in "rows 1" "rows 8" "trees 8"; do
      SRHIP_TG_MAJOR=$tg timeout -k 10 120 python3 tools/geom_sweep.py $kn 30 >> $out 2>>gpurun_out/tgmajor.err || exit $?
    done
  done
done
cat gpurun_out/tgm_check.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/tgmajor.jsonl"):
    d = json.loads(l); print(d["kind"], d["N"], d["knobs"], d["kernel_ms"], d["wall_ms"])
PY
