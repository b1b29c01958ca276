# First-tile failure prepass (SRHIP_JIT_PREPASS) A/B: bench line and the
# fixed-cost probe's row sizes, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/prepass
for r in 1 2; do
  for v in 1 0; do
    SRHIP_JIT_PREPASS=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/prepass/bench_$v.json 2>> gpurun_out/prepass/err.log || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/prepass/bench_$v.json').read().strip().splitlines()[-1]); print('prepass=$v bench', round(d['value']/1e12,3), round(d['roofline']['kernel_ms'],4))"
    SRHIP_JIT_PREPASS=$v timeout -k 10 300 python3 tools/fixed_cost_probe.py 10 > gpurun_out/prepass/fc_$v.jsonl 2>> gpurun_out/prepass/err.log || { echo "probe $v failed"; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
for l in open(f"gpurun_out/prepass/fc_{v}.jsonl"):
    d = json.loads(l)
    if d.get("variant") == "default" and d.get("set") in ("4096", "512"):
        print("prepass=%s %s rows %7d %.4f ms" % (v, d["set"], d["rows"], d["kernel_ms"]))
PY
  done
done
