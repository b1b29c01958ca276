#!/bin/bash
# Round 4: dynamic tree dealing (jit_template.hip next_tree) — the affected GPU
# tests, then the N=8 shard probe and bench.py config #2 with SRHIP_JIT_DYNAMIC
# 1 (default) and 0 (the static deal); each step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py tests/test_jit_losses_gpu.py \
  tests/test_full_size.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_dyn.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for d in 1 0; do
  SRHIP_JIT_DYNAMIC=$d timeout -k 10 300 python3 tools/shard_probe.py 10 > gpurun_out/shard_probe_dyn$d.json 2> gpurun_out/shard_probe_dyn$d.err || exit $?
  SRHIP_JIT_DYNAMIC=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 10 --no-cpu --no-row-shard > gpurun_out/bench_dyn$d.json 2> gpurun_out/bench_dyn$d.err || exit $?
  python3 - "$d" <<'PY'
import json, sys
d = sys.argv[1]
p = json.loads(open(f"gpurun_out/shard_probe_dyn{d}.json").read())
b = json.loads(open(f"gpurun_out/bench_dyn{d}.json").read().strip().splitlines()[-1])
print(f"dyn={d} bench ms/step {b['ms_per_step']:.4f} kernel {b['roofline']['kernel_ms']:.4f}; full {p['full']['kernel_ms']:.3f}",
      "strided shards", [round(s["kernel_ms"], 3) for s in p["strided"]["shards"]], "proj", round(p["strided"]["projected_speedup_wall"], 2),
      "balanced proj", round(p["balanced"]["projected_speedup_wall"], 2))
PY
done
