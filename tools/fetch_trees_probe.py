"""HBM fetch of the loss tree code against the size of its code: the config #2
batch (bench.py's 4096 trees, seed 1000, 1M rows) and its first 2048 / 1024 /
512 trees, each evaluated 3 times, in that order. Run under
`rocprofv3 --pmc FETCH_SIZE --kernel-trace`: the counter CSV's dispatches come
in this order (tools/fetch_trees_probe.py --parse <csv> prints the table)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SETS = (4096, 2048, 1024, 512)
REPS = 3


def parse(path):
    import csv
    import collections
    acc = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        acc[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    ev = [d for d in sorted(acc) if name[d].startswith("sr_jit_eval")]
    ev = ev[-len(SETS) * REPS:]
    for k, n in enumerate(SETS):
        v = [acc[d] for d in ev[k * REPS:(k + 1) * REPS]]
        print(json.dumps(dict(trees=n, fetch_kb=v, fetch_mb_corrected=2 * sum(v) / len(v) * 1024 / 1e6)))


def main():
    sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
    import numpy as np
    import srhip
    from srhip import constants as K
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    progs = {n: srhip.Program(ctx, srhip.flatten(trees[:n], o, dtype=np.float32), np.float32) for n in SETS}
    for n in SETS:
        for _ in range(REPS):
            progs[n].eval_loss(ds, K.LOSS["L2"])
            print(json.dumps(dict(trees=n, kernel=ctx.last_kernel_name(), kernel_ms=ctx.last_kernel_time()[0],
                                  code_bytes=progs[n].jit_info()["code_bytes"])), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        main()
