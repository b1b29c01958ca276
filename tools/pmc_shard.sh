#!/bin/bash
# PMC passes of the loss tree code at two shard sizes (NTREES=512 vs 4096):
# tools/pmc_shard.sh -> gpurun_out/pmc_shard/<n>_<pass>/...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_shard; mkdir -p $OUT
pass() { n=$1; name=$2; shift 2
  NTREES=$n timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/${n}_$name -o $name -- python3 tools/prof_target.py 5 >> $OUT/log.txt 2>&1 || { echo "pass $n $name failed"; exit 1; }
}
for n in 512 4096; do
  pass $n p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
  pass $n p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_IFETCH SQ_WAVES SQ_ACTIVE_INST_MISC
  pass $n p3 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_MISSES GRBM_GUI_ACTIVE
done
python3 - <<'PY'
import csv, glob, collections, os
for n in (512, 4096):
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for f in glob.glob(f"gpurun_out/pmc_shard/{n}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "sr_jit_eval" not in r.get("Kernel_Name", ""): continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    # per dispatch: counter rows are per (dispatch, counter) after rocprofv3 aggregation over dimensions
    d = {k: tot[k] / max(1, cnt[k]) for k in tot}
    print(n, {k: f"{v:.4g}" for k, v in sorted(d.items())})
PY
