# HBM fetch (FETCH_SIZE pass) and kernel time of the bench command under
# staging / mapping variants: tools/fetch_probe.sh <variant>... (default,
# NTX = SRHIP_JIT_NTX=1, TG_MAJOR = SRHIP_TG_MAJOR=1, RG_XCD0 = SRHIP_RG_XCD=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/fetch && export TMPDIR=/tmp
for v in "$@"; do
  case $v in default) E="";; NTX) E="SRHIP_JIT_NTX=1";; TG_MAJOR) E="SRHIP_TG_MAJOR=1";; RG_XCD0) E="SRHIP_RG_XCD=0";; *) echo "unknown $v"; exit 2;; esac
  env $E timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fetch/$v -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-row-shard > gpurun_out/fetch/$v.json 2> gpurun_out/fetch/$v.err || { echo "$v failed"; exit 1; }
  env $E timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/fetch/${v}_t.json 2>> gpurun_out/fetch/$v.err || { echo "$v bench failed"; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, json, sys, collections
v = sys.argv[1]
acc = collections.defaultdict(float)
for f in glob.glob(f"gpurun_out/fetch/{v}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("sr_jit_eval"):
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
d = json.loads(open(f"gpurun_out/fetch/{v}_t.json").read().strip().splitlines()[-1])
print(json.dumps(dict(variant=v, fetch_mb=2 * 1024 * sum(acc.values()) / max(1, len(acc)) / 1e6,
                      kernel_ms=d["roofline"]["kernel_ms"], value_T=d["value"] / 1e12)))
PY
done
