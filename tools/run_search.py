"""EquationSearch with the reference's DEFAULT Options on the engine
(srhip.evolution: every island's candidates in one launch per round).

  python tools/run_search.py config1 [--iterations 40]   README quickstart:
      X = randn(Float32, 5, 100), y = 2cos(x4) + x1² − 2, [+,*,/,-] / [cos,exp],
      npopulations = 20, niterations = 40 (BASELINE config #1)
  python tools/run_search.py config4 [--iterations 2]    10 features × 100k rows,
      npopulations = 64, default Options otherwise (BASELINE config #4, one GPU)

Prints one JSON line per iteration (progress) and a final JSON line: evals,
evals/s, s/iteration, launches, the engine's share of the wall time, and the
hall of fame as flattened trees (kind / arg / constants) so that
tests/test_search_records.py can recheck every stored loss on the CPU oracle
(this tool never loads the oracle). The reference prints evals/s in its
progress line (src/SymbolicRegression.jl:871-896)."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import evolution as E  # noqa: E402


def data(cfg):
    if cfg == "config1":
        rng = np.random.default_rng(0)
        X = rng.standard_normal((5, 100)).astype(np.float32)
        o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], npopulations=20)
    else:
        rng = np.random.default_rng(41)
        X = rng.standard_normal((10, 100_000)).astype(np.float32)
        o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], npopulations=64)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    return X, y, o


class TimedEngine(E.EngineEvaluator):
    """The engine evaluator, printing a progress line every ~20 s, and timing
    each request kind: calls, trees, host seconds inside the call (flatten,
    program build, launch, wait) and the device time of its kernels (HIP
    events of the context, srhip Context.last_kernel_time)."""

    def __init__(self, *a):
        super().__init__(*a)
        self.t_last = time.perf_counter()
        self.calls = 0
        self.kinds = {k: {"calls": 0, "trees": 0, "host_s": 0.0, "kernel_ms": 0.0}
                      for k in ("losses", "losses_rows", "optimize")}

    def _timed(self, kind, n, fn):
        self.calls += 1
        now = time.perf_counter()
        if now - self.t_last > 20:
            print(json.dumps({"progress_calls": self.calls}), flush=True)
            self.t_last = now
        out = fn()
        k = self.kinds[kind]
        k["host_s"] += time.perf_counter() - now
        k["calls"] += 1
        k["trees"] += n
        if kind != "optimize":
            k["kernel_ms"] += float(srhip.get_context(0).last_kernel_time()[0])
        return out

    def losses(self, trees):
        return self._timed("losses", len(trees), lambda: super(TimedEngine, self).losses(trees))

    def losses_rows(self, trees, rows):
        return self._timed("losses_rows", len(trees), lambda: super(TimedEngine, self).losses_rows(trees, rows))

    def optimize(self, trees, noise):
        return self._timed("optimize", len(trees), lambda: super(TimedEngine, self).optimize(trees, noise))

    def report(self):
        out = {}
        for kind, k in self.kinds.items():
            if k["calls"]:
                out[kind] = dict(k, host_ms_per_call=1e3 * k["host_s"] / k["calls"],
                                 kernel_ms_per_call=k["kernel_ms"] / k["calls"] if kind != "optimize" else None,
                                 trees_per_call=k["trees"] / k["calls"])
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["config1", "config4"])
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--batching", action="store_true",
                    help="Options(batching=true, batch_size=50): score_func_batch's per-candidate row samples, "
                         "all candidates of a round in one launch (srhip_eval_loss_rowsets)")
    a = ap.parse_args()
    X, y, o = data(a.config)
    if a.batching:
        o.batching = True
    nit = a.iterations or (40 if a.config == "config1" else 2)
    ds = srhip.Dataset(X, y)
    ev = TimedEngine(ds, o)
    t0 = time.perf_counter()
    hof, st = srhip.equation_search(X, y, o, niterations=nit, seed=a.seed, evaluator=ev, verbose=True)
    wall = time.perf_counter() - t0
    front = hof.pareto()
    flat = srhip.flatten([m.tree for m in front], o, dtype=np.float32)
    rec = {"tool": "run_search", "config": a.config, "npopulations": o.npopulations, "niterations": nit,
           "rows": int(X.shape[1]), "nfeat": int(X.shape[0]), "options": "defaults (fast_cycle=false, "
           "crossover_probability=0.066, tournament_selection_p=0.86, use_frequency, optimizer_probability=0.14)",
           "batching": bool(o.batching), "wall_s": wall, **{k: v for k, v in st.items() if k != "result"},
           "engine_by_kind": ev.report(),
           "hall_of_fame": [{"complexity": srhip.compute_complexity(m.tree, o), "loss": m.loss, "score": m.score,
                             "equation": srhip.string_tree(m.tree, o)} for m in front],
           "flat": {"node_off": flat.node_off.tolist(), "kind": flat.kind.tolist(), "arg": flat.arg.tolist(),
                    "const_off": flat.const_off.tolist(), "consts": [float(c) for c in flat.consts]}}
    line = json.dumps(rec)
    print(line, flush=True)
    if a.out:
        Path(a.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
