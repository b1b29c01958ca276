"""Per-dispatch averages of the PMC passes of tools/gpu_prof_jit.sh for the
tree-code kernel (sr_jit_eval*) or the interpreter's eval kernel, plus the
kernel trace's average duration, and the derived ratios DESIGN.md quotes."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
want = os.environ.get("KERNEL", "sr_jit_eval")
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "pmc*", "*counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if want in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d in per.values():
        for k, v in d.items():
            vals[k].append(v)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
kt = glob.glob(os.path.join(out, "kt", "*kernel_stats.csv"))
dur = None
if kt:
    for r in csv.DictReader(open(kt[0])):
        if want in r["Name"]:
            dur = float(r["AverageNs"]) / 1e6
# the exact kernel symbol the passes measured (the most dispatched match)
names = defaultdict(int)
for f in glob.glob(os.path.join(out, "pmc*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if want in r["Kernel_Name"]:
            names[r["Kernel_Name"]] += 1
exact = max(names, key=names.get) if names else want
res = {"kernel": exact, "avg_ms_kernel_trace": dur, "counters_per_dispatch": avg}
# the library the passes ran: bench.py attaches this summary to its JSON line
# only when its own run launched the same kernel from the same libsrhip.so
import hashlib  # noqa: E402
_lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd", "lib", "libsrhip.so")
if os.path.exists(_lib):
    res["lib_sha256"] = hashlib.sha256(open(_lib, "rb").read()).hexdigest()
# the same average over the bench's timed steps only (the last STEPS dispatches;
# the first warmup calls run on a cold instruction cache)
ktr = glob.glob(os.path.join(out, "kt", "*kernel_trace.csv"))
if ktr:
    d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(ktr[0]))
               if want in r["Kernel_Name"])
    steps = int(os.environ.get("STEPS", "20"))
    if len(d) >= steps:
        res["avg_ms_timed_steps"] = sum(e - b for b, e in d[-steps:]) / steps / 1e6
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VALU"):
        if k in avg:
            res[f"{k}/WAVE_CYCLES"] = avg[k] / wc
if "GRBM_GUI_ACTIVE" in avg and "SQ_INSTS_VALU" in avg:
    cyc = avg["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
    res["gpu_cycles"] = cyc
    res["valu_busy_2cyc"] = avg["SQ_INSTS_VALU"] * 2 / (cyc * 1024)
    if "SQ_ACTIVE_INST_VALU" in avg:
        # quad-cycles the SIMDs' VALUs work (≈ 1.05 per wave64 instruction,
        # packed or not): the share of the 1024 SIMDs' cycles the VALU is busy
        res["valu_busy_4cyc"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024)
        res["quad_cycles_per_valu_inst"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_INSTS_VALU"]
if "FETCH_SIZE" in avg:
    # KB; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950
    # (MI355X_MICROARCH.md, HBM): doubled
    res["hbm_bytes_per_launch"] = (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024
if "valu_busy_4cyc" in res:
    res["valu_busy"] = res["valu_busy_4cyc"]
elif "valu_busy_2cyc" in res:
    res["valu_busy"] = res["valu_busy_2cyc"]
res["workload"] = os.environ.get("WORKLOAD", "config#2")
print(json.dumps(res, indent=1))
