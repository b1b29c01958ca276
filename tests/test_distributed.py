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
from srhip.distributed import combine_row_shards, pack_partials, shard_range, unpack_partials


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
