#!/bin/bash
# Round 4 validation: tree-code GPU tests (loss, gradient, per-row output,
# full size), then the printf driver probes P / Q when those builds exist.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py tests/test_jit_losses_gpu.py \
  tests/test_jit_out_gpu.py tests/test_jit64_gpu.py tests/test_full_size.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r4.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for V in P Q; do
  lib=symbolicregression.jl_amd/lib/libsrhip_$V.so
  [ -f $lib ] || continue
  SRHIP_LIB=$PWD/$lib timeout -k 10 100 python3 tools/debug_driver.py 8 256 > gpurun_out/dbg$V.txt 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/shard_probe.py 10 > gpurun_out/shard_probe_r4.json 2> gpurun_out/shard_probe_r4.err || exit $?
python3 - <<'PY'
import json
p = json.loads(open("gpurun_out/shard_probe_r4.json").read())
print("full", p["full"]["wall_ms"], "strided proj", round(p["strided"]["projected_speedup_wall"], 2),
      "rows", {k: round(v["projected_speedup_wall_no_allreduce"], 2) for k, v in p["rows"].items()})
PY
echo done
