"""Generate tests/golden/golden.npz — committed input/output vectors of the
scoring path (run: python tests/golden/make_golden.py).

The Julia reference cannot run in this image (no `julia`, DynamicExpressions.jl
not vendored — SURVEY.md §8c), so the expected outputs are produced by the
CPU restatement in oracle/, which is itself pinned by the reference's
known-answer tests (tests/test_reference_kats.py). The fixtures freeze that
pinned behaviour: tests/test_golden.py re-derives them on the CPU (oracle
regression) and checks the engine against them on the GPU.

Cases (BASELINE.json configs, scaled to fixture size):
  cfg1_f32   README quickstart shape: X = randn(Float32, 5, 100),
             y = 2cos(x4) + x1^2 - 2, ops [+,*,/,-] / [cos,exp]   (README.md:41-48)
  cfg2_f32   config #2 op set at 1000 rows
  cfg3_f64   config #3: [+,-,*,/,safe_pow] / [safe_log,safe_sqrt,cos,exp],
             X ~ U(-3, 3) (mixed sign, NaN-heavy)
  grid_f32 / grid_f64
             every supported operator on LinRange(-100, 100, 99) (Configure.jl:3-26)
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle")]
import oracle  # noqa: E402
import srhip  # noqa: E402
from srhip import Node  # noqa: E402

ALL_BIN = ["+", "-", "*", "/", "pow", "greater", "logical_or", "logical_and", "mod", "max", "min"]
ALL_UNA = ["neg", "square", "cube", "exp", "abs", "log", "log2", "log10", "log1p", "sqrt", "sin", "cos",
           "tan", "sinh", "cosh", "tanh", "atan", "asinh", "acosh", "atanh_clip", "erf", "erfc", "gamma",
           "relu", "round", "floor", "ceil", "sign", "inv"]


def pack(prefix, trees, options, X, y, T, out):
    flat = srhip.flatten(trees, options, dtype=T)
    yhat, ok = oracle.eval_trees(flat, X, dtype=T)
    sums, losses, lok = oracle.eval_loss_batch(flat, X, y, dtype=T)
    out.update({
        f"{prefix}/binops": np.array(options.binary_operators, dtype="U16"),
        f"{prefix}/unaops": np.array(options.unary_operators, dtype="U16"),
        f"{prefix}/node_off": flat.node_off, f"{prefix}/kind": flat.kind, f"{prefix}/arg": flat.arg,
        f"{prefix}/const_off": flat.const_off, f"{prefix}/consts": flat.consts.astype(T),
        f"{prefix}/X": X.astype(T), f"{prefix}/y": y.astype(T),
        f"{prefix}/out": yhat, f"{prefix}/ok": ok,
        f"{prefix}/loss_sum": sums, f"{prefix}/loss": losses, f"{prefix}/loss_ok": lok,
    })


def grid_trees(options, T):
    """op(x1) and op(x1, x2), op(x1, c), op(c, x1) for every operator."""
    trees = []
    for i in range(1, len(options.unary_operators) + 1):
        trees.append(Node(i, Node(feature=1)))
    for i in range(1, len(options.binary_operators) + 1):
        trees.append(Node(i, Node(feature=1), Node(feature=2)))
        trees.append(Node(i, Node(feature=1), Node(val=T(0.7))))
        trees.append(Node(i, Node(val=T(-1.3)), Node(feature=2)))
    return trees


def main():
    out = {}
    rng = np.random.default_rng(2024)
    # cfg1: README quickstart data
    o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"])
    X = rng.standard_normal((5, 100)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    pack("cfg1_f32", srhip.random_population(64, o, 5, np.float32, seed=11), o, X, y, np.float32, out)
    # cfg2 op set
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    X = rng.standard_normal((5, 1000)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    pack("cfg2_f32", srhip.random_population(128, o, 5, np.float32, seed=12), o, X, y, np.float32, out)
    # cfg3: NaN-heavy float64
    o = srhip.Options(binary_operators=["+", "-", "*", "/", "pow"],
                      unary_operators=["log", "sqrt", "cos", "exp"])
    X = rng.uniform(-3, 3, (5, 300))
    y = rng.standard_normal(300)
    pack("cfg3_f64", srhip.random_population(256, o, 5, np.float64, seed=13), o, X, y, np.float64, out)
    # every operator on the legality grid
    o = srhip.Options(binary_operators=ALL_BIN, unary_operators=ALL_UNA)
    g = np.linspace(-100, 100, 99)
    X = np.stack([g, g[::-1] * 0.37, g * 0.01])
    for T, name in ((np.float32, "grid_f32"), (np.float64, "grid_f64")):
        pack(name, grid_trees(o, T), o, X.astype(T), np.zeros(99, T), T, out)
    np.savez_compressed(Path(__file__).with_name("golden.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
