# SRHIP_JIT_STICKY_TREE A/B over the fixed-cost probe's sets and row counts (interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/sticky
for r in 1 2; do
  for v in 1 0; do
    SRHIP_JIT_STICKY_TREE=$v timeout -k 10 300 python3 tools/fixed_cost_probe.py 10 > gpurun_out/sticky/fc_${v}_$r.jsonl 2>> gpurun_out/sticky/err.log || { echo "probe $v failed"; exit 1; }
    python3 - "$v" "$r" <<'PY'
import json, sys
v, r = sys.argv[1], sys.argv[2]
out = []
for l in open(f"gpurun_out/sticky/fc_{v}_{r}.jsonl"):
    d = json.loads(l)
    if d.get("variant") == "default" and d.get("set") in ("4096", "512"):
        out.append("%s/%dk %.4f" % (d["set"], d["rows"] // 1000, d["kernel_ms"]))
print("sticky=%s: " % v + "  ".join(out))
PY
  done
done
