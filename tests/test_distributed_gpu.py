"""Row-sharded product path on the engine (config #5's partition), world_size 2
with both ranks on device 0 and the gloo backend for the all-reduce:

* eval_loss_row_sharded: each rank uploads its row shard and evaluates all
  trees on it; the combined losses / did_succeed equal the single-process
  engine result (fp64 partial sums, summation order aside) and the oracle's;
* optimize_constants_row_sharded: loss AND ∂L/∂c partials all-reduced per
  step (RowShardedEvaluator); both ranks agree exactly and match the
  single-process optimiser on the engine.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
import srhip
from numerics import assert_close_conditioned, loss_spread

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem(T=np.float32):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(21)
    X = rng.standard_normal((20, 200_003)).astype(T)
    y = (T(2) * np.cos(X[3]) + X[0] * X[0] - T(2)).astype(T)
    trees = srhip.random_population(700, o, 20, T, seed=22)
    return o, X, y, trees


def _copt_problem():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(31)
    X = rng.standard_normal((4, 50_001))
    y = 2.5 * np.cos(1.3 * X[0]) + 0.7 * X[1]
    trees = srhip.random_population(64, o, 4, np.float64, seed=32)
    return o, X, y, trees


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "symbolicregression.jl_amd"), str(root / "oracle"), str(root / "tests")]
    os.environ["SRHIP_DEVICE"] = "0"
    import torch.distributed as dist

    from srhip.distributed import eval_loss_row_sharded, optimize_constants_row_sharded
    from test_distributed_gpu import _copt_problem, _problem

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, X, y, trees = _problem()
        losses, ok = eval_loss_row_sharded(trees, srhip.Dataset(X, y), o, device=0)
        o2, X2, y2, trees2 = _copt_problem()
        res = optimize_constants_row_sharded(trees2, srhip.Dataset(X2, y2), o2, rng=np.random.default_rng(5),
                                             device=0)
        q.put((rank, losses, ok, res.losses, res.converged))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_row_sharded_engine_world2_on_one_gpu(gpu_ctx):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # loss evaluation: both ranks, single-process engine, oracle
    o, X, y, trees = _problem()
    ref_l, ref_ok = srhip.eval_loss_batch_ok(trees, srhip.Dataset(X, y), o)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    _, or_l, or_ok = oracle.eval_loss_batch(flat, X, y, dtype=np.float32, nthreads=16)
    for _, l, k, _, _ in res:
        assert np.array_equal(k, ref_ok) and np.array_equal(k, or_ok)
        m = k & np.isfinite(ref_l)
        # the shards regroup the Float32 per-tile partial sums: within the
        # north_star's 1e-5 of the single-process engine and of the oracle
        np.testing.assert_allclose(l[m], ref_l[m], rtol=1e-5)
        # against the oracle: the north_star's 1e-5, or (a tree outside it)
        # within 4x the oracle's own spread under ulp-scale perturbations
        rel = np.abs(l[m] - or_l[m]) / np.abs(or_l[m])
        out = np.flatnonzero(m)[~(rel <= 1e-5)]
        if out.size:
            sp = loss_spread([trees[i] for i in out], o, X, y, None, np.float32, nperturb=3) / X.shape[1]
            assert_close_conditioned(l[out], or_l[out], sp, rtol=1e-5, factor=4.0, msg="row-sharded vs oracle")
    np.testing.assert_array_equal(res[0][1], res[1][1])
    # constant optimisation with all-reduced gradients
    o2, X2, y2, trees2 = _copt_problem()
    ref = srhip.optimize_constants_batch(srhip.Dataset(X2, y2), trees2, o2, rng=np.random.default_rng(5))
    (_, _, _, l0, c0), (_, _, _, l1, c1) = res
    np.testing.assert_array_equal(l0, l1)
    np.testing.assert_array_equal(c0, c1)
    assert np.mean(c0 == ref.converged) >= 0.95
    both = c0 & ref.converged
    np.testing.assert_allclose(l0[both], ref.losses[both], rtol=1e-6)


def test_packed_partials_equal_host_packing(gpu_ctx):
    """srhip_eval_loss_packed (device buffer for the RCCL all-reduce) writes
    exactly pack_partials(srhip_eval_loss(...)): per-tree sums and failure
    flags (static failures included) and Σw."""
    import torch

    from srhip import constants as K
    from srhip.distributed import pack_partials

    o, X, y, trees = _problem()
    trees = trees[:600] + [srhip.Node(val=np.float32(np.inf)), srhip.Node(val=np.float32(1.5))]
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X[:, :50_001], y[:50_001])
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    buf = torch.full((2 * len(trees) + 1,), -7.0, dtype=torch.float64, device=f"cuda:{ctx.device}")
    prog.eval_loss_packed(ds, K.LOSS["L2"], buf.data_ptr())
    ctx.sync()
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
    np.testing.assert_array_equal(buf.cpu().numpy(), pack_partials(s, w, ok))
    assert not ok[600] and ok[601]


def _empty_shard_worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "symbolicregression.jl_amd"), str(root / "oracle"), str(root / "tests")]
    os.environ["SRHIP_DEVICE"] = "0"
    import torch.distributed as dist

    from srhip.distributed import eval_loss_row_sharded
    from test_distributed_gpu import _problem

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, X, y, trees = _problem()
        # one row over two ranks: rank 1's shard is empty (shard_range)
        losses, ok = eval_loss_row_sharded(trees[:600], srhip.Dataset(X[:, :1], y[:1]), o, device=0)
        q.put((rank, losses, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(200)
def test_row_sharded_world2_with_an_empty_shard(gpu_ctx):
    """A rank whose row shard is empty evaluates nothing (every tree's result
    is its static verdict) and still joins the all-reduce: the combined
    result equals the single-process engine's on the one row."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=150) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o, X, y, trees = _problem()
    ref_l, ref_ok = srhip.eval_loss_batch_ok(trees[:600], srhip.Dataset(X[:, :1], y[:1]), o)
    for _, l, k in res:
        np.testing.assert_array_equal(k, ref_ok)
        np.testing.assert_allclose(l[k], ref_l[k], rtol=1e-6)


def test_empty_dataset_tree_code_batch(gpu_ctx):
    """Zero rows with a batch large enough for tree code: no launch, every
    tree succeeds with a zero sum unless it fails statically; a non-finite
    constant root fails only when there are rows, so it
    succeeds here (eval_loss and the packed device buffer agree)."""
    import torch

    from srhip import constants as K
    from srhip.distributed import pack_partials

    o, X, y, trees = _problem()
    trees = trees[:600] + [srhip.Node(val=np.float32(np.inf))]
    ds = srhip.DeviceDataset(gpu_ctx, X[:, :0], y[:0])
    prog = srhip.Program(gpu_ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
    assert ok.all() and w == 0.0
    assert np.all(s == 0.0)
    buf = torch.full((2 * len(trees) + 1,), -7.0, dtype=torch.float64, device=f"cuda:{gpu_ctx.device}")
    prog.eval_loss_packed(ds, K.LOSS["L2"], buf.data_ptr())
    gpu_ctx.sync()
    np.testing.assert_array_equal(buf.cpu().numpy(), pack_partials(s, w, ok))


def test_packed_rejects_a_buffer_on_another_device(gpu_ctx):
    """srhip_eval_loss_packed refuses host memory (and, on a multi-GPU box,
    a buffer of another device) with SRHIP_ERR_INVALID instead of writing it
    from the wrong device's stream."""
    import torch

    from srhip import constants as K

    o, X, y, trees = _problem()
    ds = srhip.DeviceDataset(gpu_ctx, X[:, :1000], y[:1000])
    prog = srhip.Program(gpu_ctx, srhip.flatten(trees[:8], o, dtype=np.float32), np.float32)
    host = torch.zeros(2 * 8 + 1, dtype=torch.float64)
    with pytest.raises(Exception):
        prog.eval_loss_packed(ds, K.LOSS["L2"], host.data_ptr())
    if torch.cuda.device_count() > 1:
        other = (gpu_ctx.device + 1) % torch.cuda.device_count()
        buf = torch.zeros(2 * 8 + 1, dtype=torch.float64, device=f"cuda:{other}")
        with pytest.raises(Exception):
            prog.eval_loss_packed(ds, K.LOSS["L2"], buf.data_ptr())
