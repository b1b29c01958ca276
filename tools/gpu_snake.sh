#!/bin/bash
# Wave deal A/B (jit.cpp wave_snake): tree-code GPU tests, then config #2 and
# its N = 8 shards with SRHIP_JIT_WAVE_SNAKE=0 / 1 (tools/geom_sweep.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py tests/test_jit_out_gpu.py \
  tests/test_jit_losses_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_snake.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_snake.log | tail -2
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/snake.jsonl; : > $out
for rep in 1 2; do
  for sn in 0 1; do
    for kn in "rows 1" "rows 8" "trees 8" "rows 4"; do
      SRHIP_JIT_WAVE_SNAKE=$sn timeout -k 10 120 python3 tools/geom_sweep.py $kn 30 >> $out 2>>gpurun_out/snake.err || exit $?
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/snake.jsonl"):
    d = json.loads(l); print(d["kind"], d["N"], d["knobs"], d["kernel_ms"], d["wall_ms"])
PY
