"""Step-by-step GPU probe of the evaluation path (prints after every call)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle")]
import numpy as np
import srhip
from srhip import Node, constants as K
from srhip.engine import Context, DeviceDataset, Program

t0 = time.time()
def say(*a):
    print(f"[{time.time() - t0:6.2f}s]", *a, flush=True)

step = sys.argv[1]
o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
say("lib", srhip._lib.LIB_PATH)
say("devices", srhip.device_count())
ctx = Context(0); say("context")
if step in ("leaf", "const", "cos"):
    tree = {"leaf": Node("x1"), "const": o.make_binary("+", Node("x1"), Node(val=2.0)),
            "cos": o.make_unary("cos", Node("x1"))}[step]
    trees, n = [tree], 4
else:
    trees, n = srhip.random_population(int(sys.argv[2]), o, 5, np.float32, seed=1), 1000
X = np.random.default_rng(0).standard_normal((5, n)).astype(np.float32)
ds = DeviceDataset(ctx, X, X[0].copy()); say("dataset", ds.info())
prog = Program(ctx, srhip.flatten(trees, o, np.float32), np.float32); say("program", prog.info()[:2])
if step == "loss":
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"]); say("eval_loss", s[:4], ok[:8], ctx.last_kernel_time())
else:
    out, ok = prog.eval_tree_array(ds); say("eval_tree_array", out.ravel()[:4], ok[:8], ctx.last_kernel_time())
