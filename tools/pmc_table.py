"""Print mean per-dispatch eval_kernel counters of a tools/pmc_micro.sh run."""
import csv, collections, sys
from pathlib import Path
src = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in sorted(src.glob("*/*counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if "eval_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]][(p.name, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v.values()) / len(v):16.4g}")
