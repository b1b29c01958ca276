#!/bin/bash
# Kernel-trace A/B of the shared-subtree columns (jit.h Columns): bench.py
# under rocprofv3 --kernel-trace --stats for each SRHIP_JIT_GCOLS value given
# (default: 64 0 16 32) -> gpurun_out/kt/g<N>/ (kernel stats, bench JSON).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/kt
export TMPDIR=/tmp
for g in ${@:-64 0 16 32}; do
  SRHIP_JIT_GCOLS=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt/g$g -o kt -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/kt/g$g.json 2> gpurun_out/kt/g$g.err || exit $?
  python3 - "$g" <<'PY'
import csv, sys
g = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/kt/g{g}/kt_kernel_stats.csv")))
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    print(f"gcols={g} {r['Name'][:48]:48s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e6:.4f} ms")
PY
done
