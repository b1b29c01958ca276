"""Row-sharded evaluation across ranks (config #5's partition), world_size 2
over gloo on CPU: each rank computes its shard's partial sums (with the
oracle — no GPU here), the host combine step all-reduces them, and the result
must equal the single-process evaluation of all rows."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import srhip
from srhip.distributed import (combine_row_shards, merge_tree_shards, pack_grad_partials, pack_partials,
                               shard_range, shard_trees, unpack_grad_partials, unpack_partials)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_range_covers_rows():
    for n in (0, 1, 7, 1000, 10_000_001):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1


def test_pack_roundtrip():
    sums = np.array([1.5, np.nan, 3.0])
    ok = np.array([True, False, True])
    s, w, k = unpack_partials(pack_partials(sums, 10.0, ok))
    assert w == 10.0 and list(k) == [True, False, True]
    assert s[0] == 1.5 and np.isnan(s[1]) and s[2] == 3.0


def test_tree_shards_cover_and_merge_in_order():
    for nt in (0, 1, 5, 4096, 4097):
        for world in (1, 2, 3, 8):
            parts = [shard_trees(nt, r, world) for r in range(world)]
            allidx = np.sort(np.concatenate(parts)) if parts else np.zeros(0)
            assert np.array_equal(allidx, np.arange(nt))  # every tree exactly once
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1
            vals = merge_tree_shards([p * 10.0 for p in parts], nt)  # results computed per shard
            assert np.array_equal(vals, np.arange(nt) * 10.0)      # land back in tree order
    with pytest.raises(ValueError):
        merge_tree_shards([np.zeros(3), np.zeros(3)], 5)


def test_grad_pack_roundtrip():
    sums = np.array([1.5, np.nan, 3.0])
    ok = np.array([True, False, True])
    co = np.array([0, 2, 3, 5])
    g = np.array([0.5, -1.0, np.nan, 2.0, 4.0])
    buf = pack_grad_partials(sums, g, 7.0, ok, co)
    assert np.all(np.isfinite(buf))  # a failed tree's NaNs never reach the all-reduce
    s, gg, w, k = unpack_grad_partials(buf + buf, 3, co)  # two identical shards
    assert w == 14.0 and list(k) == [True, False, True]
    np.testing.assert_array_equal(gg[[0, 1, 3, 4]], 2 * g[[0, 1, 3, 4]])
    assert np.isnan(gg[2]) and np.isnan(s[1])


def _problem():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(40, o, 5, np.float64, seed=5)
    rng = np.random.default_rng(6)
    X = rng.standard_normal((5, 5001))
    y = 2 * np.cos(X[3]) + X[0] ** 2 - 2
    w = np.abs(rng.standard_normal(5001))
    return o, trees, X, y, w


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "symbolicregression.jl_amd"), str(root / "oracle"), str(root / "tests")]
    import torch.distributed as dist

    import oracle
    from srhip.distributed import torch_all_reduce_sum

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o, trees, X, y, w = _problem()
    flat = srhip.flatten(trees, o, dtype=np.float64)
    b, e = shard_range(X.shape[1], rank, world)
    sums, _, ok = oracle.eval_loss_batch(flat, X[:, b:e], y[b:e], w[b:e], dtype=np.float64)
    s, W, k = combine_row_shards(sums, float(w[b:e].sum()), ok, torch_all_reduce_sum())
    q.put((rank, s, W, k))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_row_sharded_gloo_world2_matches_single_process():
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
    import oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    o, trees, X, y, w = _problem()
    flat = srhip.flatten(trees, o, dtype=np.float64)
    ref_s, _, ref_ok = oracle.eval_loss_batch(flat, X, y, w, dtype=np.float64)
    for _, s, W, k in res:
        assert np.array_equal(k, ref_ok)
        assert abs(W - w.sum()) < 1e-9 * w.sum()
        np.testing.assert_allclose(s[k], ref_s[k], rtol=1e-12)


class OracleShardProgram:
    """Test stand-in for srhip.Program on one row shard: loss and
    Σ w·∂ℓ/∂c (L2) of every tree on the CPU oracle."""

    def __init__(self, cands, options, X, y):
        self.flat = srhip.flatten(cands, options, dtype=np.float64)
        self.X, self.y = X, y
        self.consts = np.asarray(self.flat.consts, dtype=np.float64)

    def set_constants(self, c):
        self.consts = np.asarray(c, dtype=np.float64)

    def _trees(self):
        co = self.flat.const_off
        for t in range(self.flat.ntrees):
            k, a, _ = self.flat.tree(t)
            yield t, k, a, self.consts[co[t]:co[t + 1]]

    def eval_loss_grad(self, dev, kind, params):
        import oracle
        sums, grads, ok = [], [], []
        for t, k, a, c in self._trees():
            out, g, good = oracle.eval_grad_consts(k, a, c, self.X, len(c))
            r = out - self.y
            sums.append(float(r @ r) if good else np.nan)
            grads.append(2.0 * (g @ r) if good else np.full(len(c), np.nan))
            ok.append(bool(good))
        return (np.asarray(sums), np.concatenate(grads) if grads else np.zeros(0), float(self.X.shape[1]),
                np.asarray(ok))

    def eval_loss(self, dev, kind, params):
        s, _, w, ok = self.eval_loss_grad(dev, kind, params)
        return s, w, ok


def _copt_problem():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(11)
    X = rng.standard_normal((3, 301))
    y = 2.5 * np.cos(1.3 * X[0]) + 0.7 * X[1]
    trees = srhip.random_population(24, o, 3, np.float64, seed=12)
    return o, X, y, trees


def _copt_worker(rank, world, port, q, shared=False):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "symbolicregression.jl_amd"), str(root / "oracle"), str(root / "tests")]
    import torch.distributed as dist

    from srhip.distributed import RowShardedEvaluator, shared_rng, torch_all_reduce_sum
    from test_distributed import OracleShardProgram, _copt_problem

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o, X, y, trees = _copt_problem()
    b, e = shard_range(X.shape[1], rank, world)
    red = torch_all_reduce_sum()
    ds = srhip.Dataset(X, y)

    def factory(cands):
        return RowShardedEvaluator(OracleShardProgram(cands, o, X[:, b:e], y[b:e]), None, o.elementwise_loss, red,
                                   np.float64)

    # shared: no rng given, the ranks agree on rank 0's broadcast seed
    rng = shared_rng(None) if shared else np.random.default_rng(5)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=rng, evaluator_factory=factory)
    q.put((rank, res.losses, res.converged))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_constant_optimization_row_sharded_gloo_world2():
    """optimize_constants_batch over 2 row shards (gradients all-reduced)
    takes the same steps as over all rows in one process."""
    from test_constant_optimization import OracleEvaluator

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_copt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    o, X, y, trees = _copt_problem()
    ref = srhip.optimize_constants_batch(srhip.Dataset(X, y), trees, o, rng=np.random.default_rng(5),
                                         evaluator_factory=lambda c: OracleEvaluator(c, o, X, y))
    (_, l0, c0), (_, l1, c1) = res
    np.testing.assert_array_equal(l0, l1)  # both ranks agree exactly
    assert np.array_equal(c0, ref.converged)
    np.testing.assert_allclose(l0, ref.losses, rtol=1e-7)


@pytest.mark.timeout(120)
def test_constant_optimization_row_sharded_unseeded_ranks_agree():
    """With no rng given, every rank must still build the same perturbed
    restarts: rank 0's seed is broadcast (srhip.distributed.shared_rng)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_copt_worker, args=(r, world, port, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (_, l0, c0), (_, l1, c1) = res
    np.testing.assert_array_equal(l0, l1)
    np.testing.assert_array_equal(c0, c1)


def test_balanced_tree_shards_cover_and_balance():
    """bench.py's default N > 1 partition (shard_trees_balanced, LPT on the
    estimated cost): every tree on exactly one rank, the ranks' estimated
    costs within one costliest tree of each other, the same on every rank."""
    import srhip
    from srhip.distributed import shard_trees_balanced, tree_cost

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(1000, o, 5, np.float32, seed=3, maxsize=30)
    costs = np.array([tree_cost(t, o) for t in trees])
    for world in (1, 2, 3, 8):
        parts = [shard_trees_balanced(trees, o, r, world) for r in range(world)]
        assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(len(trees)))
        loads = [costs[p].sum() for p in parts]
        assert max(loads) - min(loads) <= costs.max() + 1e-9
        assert all(np.array_equal(p, shard_trees_balanced(trees, o, r, world)) for r, p in enumerate(parts))
