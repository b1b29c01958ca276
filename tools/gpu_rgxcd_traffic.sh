#!/bin/bash
# HBM traffic of the tree-code kernel with row groups dealt per XCD (SRHIP_RG_XCD=1) or not
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rgx
export TMPDIR=/tmp
for x in 0 1; do
  SRHIP_RG_XCD=$x timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 10 > gpurun_out/rgx/b$x.log 2>&1 || exit $?
  tail -1 gpurun_out/rgx/b$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('RG_XCD=$x kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
  SRHIP_RG_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rgx/f$x -o f -- python3 bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>> gpurun_out/rgx/err.txt || exit $?
  SRHIP_RG_XCD=$x timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/rgx/w$x -o w -- python3 bench.py --steps 3 --warmup 1 --no-cpu > /dev/null 2>> gpurun_out/rgx/err.txt || exit $?
  python3 - <<PY
import csv, glob
for k in ("f", "w"):
    v = [float(r["Counter_Value"]) for f in glob.glob("gpurun_out/rgx/%s$x/*counter_collection.csv" % k) for r in csv.DictReader(open(f)) if "sr_jit_eval" in r["Kernel_Name"]]
    print("RG_XCD=$x", k, "KB per dispatch", sum(v) / 5)
PY
done
