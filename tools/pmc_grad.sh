#!/bin/bash
# PMC passes of the gradient tree code on config #5's shard (tools/prof_grad.py):
# tools/pmc_grad.sh -> gpurun_out/pmc_grad/<pass>/..., summary on stdout
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_grad; mkdir -p $OUT
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 tools/prof_grad.py 2 >> $OUT/log.txt 2>&1 || { echo "pass $name failed"; exit 1; }
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
pass p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_IFETCH SQ_WAVES SQ_INSTS_VALU_TRANS_F32
pass p3 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_MISSES GRBM_GUI_ACTIVE
pass p4 FETCH_SIZE
pass p5 WRITE_SIZE
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_grad/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sr_jit_grad" not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = {k: tot[k] / max(1, n[k]) for k in tot}
print("per sr_jit_grad dispatch:", {k: f"{v:.4g}" for k, v in sorted(d.items())})
if d.get("GRBM_GUI_ACTIVE") and d.get("SQ_ACTIVE_INST_VALU"):
    print("valu_busy_4cyc", d["SQ_ACTIVE_INST_VALU"] * 4 / (d["GRBM_GUI_ACTIVE"] * 1024))
PY
