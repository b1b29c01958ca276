"""Per-call kernel timeline of one eval_loss call (GPU box, under rocprofv3
--kernel-trace): the config #2 batch (4096 trees, bench.py's seed) on ROWS
rows, K calls with a host sync between them. Run under the kernel trace,
then `python tools/call_timeline.py --parse <kernel_trace.csv>` prints, per
call, the span from the first kernel's start to the last kernel's end, the
summed kernel durations and the gaps, and the per-kernel averages — the
per-call fixed cost of a row shard."""
import csv
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def run(rows, k):
    sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
    import numpy as np

    import srhip
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, rows)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    for _ in range(3):
        prog.eval_loss(ds, K.LOSS["L2"])
    for _ in range(k):
        prog.eval_loss(ds, K.LOSS["L2"])
        time.sleep(0.002)  # a gap the parser splits calls on
    print(json.dumps({"rows": rows, "calls": k}))


def parse(path, k):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48])
                for r in csv.DictReader(open(path)))
    calls, cur = [], []
    for e in ev:
        if cur and e[0] - cur[-1][1] > 1_000_000:  # > 1 ms idle: the next call
            calls.append(cur)
            cur = []
        cur.append(e)
    calls.append(cur)
    calls = calls[-k:]
    spans = [(c[-1][1] - c[0][0]) / 1e3 for c in calls]
    busy = [sum(e[1] - e[0] for e in c) / 1e3 for c in calls]
    per = defaultdict(list)
    for c in calls:
        for e in c:
            per[e[2]].append((e[1] - e[0]) / 1e3)
    out = {"calls": len(calls), "span_us_median": sorted(spans)[len(spans) // 2],
           "kernels_us_median": sorted(busy)[len(busy) // 2],
           "gaps_us_median": sorted(s - b for s, b in zip(spans, busy))[len(spans) // 2],
           "launches_per_call": len(calls[-1]),
           "per_kernel_us": {n: sum(v) / len(v) for n, v in per.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--parse":
        parse(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 10)
    else:
        run(int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 10)
