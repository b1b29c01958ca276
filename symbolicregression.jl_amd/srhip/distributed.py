"""Multi-GPU evaluation on one node (one process per GPU, torch.distributed).

Two partitions, as SURVEY.md §8e describes:

* trees / islands: every rank scores its own trees against a full dataset
  replica; no collective on the data path (see bench.py).
* rows (large datasets, config #5): every rank holds a contiguous row shard
  and computes per-tree partial sums Σ w·ℓ over it; one all-reduce of
  [ntrees × 2 + 1] fp64 (sum, failure count per tree, Σw) over RCCL (xGMI)
  combines them. did_succeed is the AND over shards (failure counts add up),
  the loss is ΣΣ / ΣΣw — identical to the single-device result up to fp64
  summation order.

Constant optimisation on a row-sharded dataset (config #5) needs the
gradient too: `combine_grad_shards` all-reduces [Σw·ℓ, failures, Σw·∂ℓ/∂c
of every constant, Σw] in one buffer, and `RowShardedEvaluator` plugs that
into `optimize_constants_batch` (each rank runs the same lockstep optimiser
on identical, all-reduced values, so every rank takes the same steps).

Trees of one batch are split over ranks by `shard_trees` (strided, so every
rank gets a similar cost mix) and put back in order by `merge_tree_shards`
(bench.py's strong-scaling run).

The combine steps are plain host logic on top of any all-reduce, so they are
tested with the gloo backend on CPU (tests/test_distributed.py) and on the
engine with both ranks on one GPU (tests/test_distributed_gpu.py).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row shard [begin, end) of rank (sizes differ by at most 1)."""
    base, extra = divmod(n, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def shard_trees(ntrees: int, rank: int, world: int) -> np.ndarray:
    """Indices of the trees rank evaluates: every world-th tree from rank on
    (random populations are unordered, so strided shards carry similar cost)."""
    return np.arange(rank, ntrees, world, dtype=np.int64)


# Estimated device cost of an operator per row (SIMD cycles of its tree code,
# tools/census.py on config #2: a packed + - * about 1, exp 5, sin / cos 7,
# IEEE division 8; leaves are register reads). Other operators count as a
# transcendental.
OP_COST = {"+": 1.0, "-": 1.0, "*": 1.0, "/": 8.0, "cos": 7.0, "sin": 7.0, "exp": 5.0, "neg": 0.5,
           "abs": 0.5, "square": 1.0, "cube": 2.0}


def tree_cost(tree, options) -> float:
    """The tree's estimated evaluation cost per row (OP_COST over its nodes)."""
    stack, c = [tree], 0.0
    while stack:
        t = stack.pop()
        if t.degree == 1:
            c += OP_COST.get(options.unary_operators[t.op - 1], 7.0)
            stack.append(t.l)
        elif t.degree == 2:
            c += OP_COST.get(options.binary_operators[t.op - 1], 7.0)
            stack += [t.l, t.r]
        else:
            c += 0.1
    return c


def shard_trees_balanced(trees, options, rank: int, world: int) -> np.ndarray:
    """Indices of the trees rank evaluates, partitioned by estimated cost:
    most expensive first, each to the rank with the least cost so far (LPT;
    ties to the lower rank), so the slowest rank — which sets the step time of
    a strong-scaling run — carries about 1/world of the work. Deterministic:
    every rank computes the same partition."""
    costs = np.array([tree_cost(t, options) for t in trees])
    order = np.argsort(-costs, kind="stable")
    load = np.zeros(world)
    owner = np.empty(len(trees), dtype=np.int64)
    for i in order:
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += costs[i]
    return np.flatnonzero(owner == rank)


def merge_tree_shards(parts, ntrees: int) -> np.ndarray:
    """Per-rank result arrays (in shard_trees order, rank 0 first) back into
    tree order."""
    parts = list(parts)
    world = len(parts)
    out = np.empty(ntrees, dtype=np.result_type(*[np.asarray(p).dtype for p in parts]) if parts else np.float64)
    for r, p in enumerate(parts):
        idx = shard_trees(ntrees, r, world)
        if len(p) != len(idx):
            raise ValueError(f"rank {r} returned {len(p)} results for {len(idx)} trees")
        out[idx] = p
    return out


def pack_partials(sums: np.ndarray, wsum: float, ok: np.ndarray) -> np.ndarray:
    """[sum_0, fail_0, sum_1, fail_1, ..., Σw] (failed trees contribute 0)."""
    nt = len(sums)
    buf = np.zeros(2 * nt + 1, dtype=np.float64)
    buf[0:2 * nt:2] = np.where(ok, sums, 0.0)
    buf[1:2 * nt:2] = np.where(ok, 0.0, 1.0)
    buf[-1] = wsum
    return buf


def unpack_partials(buf: np.ndarray):
    nt = (len(buf) - 1) // 2
    fails = buf[1:2 * nt:2]
    ok = fails == 0
    sums = np.where(ok, buf[0:2 * nt:2], np.nan)
    return sums, float(buf[-1]), ok


def combine_row_shards(sums: np.ndarray, wsum: float, ok: np.ndarray,
                       all_reduce_sum: Callable[[np.ndarray], np.ndarray]):
    """Combine one rank's shard partials with everyone else's."""
    return unpack_partials(all_reduce_sum(pack_partials(sums, wsum, ok)))


def pack_grad_partials(sums: np.ndarray, grads: np.ndarray, wsum: float, ok: np.ndarray,
                       const_off: np.ndarray) -> np.ndarray:
    """[sum_t, fail_t per tree ..., Σw·∂ℓ/∂c per constant ..., Σw]; a failed
    tree contributes 0 to its sums and gradients and 1 to its failure count."""
    nt, nc = len(sums), len(grads)
    buf = np.zeros(2 * nt + nc + 1, dtype=np.float64)
    buf[0:2 * nt:2] = np.where(ok, sums, 0.0)
    buf[1:2 * nt:2] = np.where(ok, 0.0, 1.0)
    bad = np.repeat(~np.asarray(ok, dtype=bool), np.diff(const_off))
    buf[2 * nt:2 * nt + nc] = np.where(bad, 0.0, grads)
    buf[-1] = wsum
    return buf


def unpack_grad_partials(buf: np.ndarray, ntrees: int, const_off: np.ndarray):
    nc = int(const_off[-1])
    sums, wsum, ok = unpack_partials(np.concatenate([buf[:2 * ntrees], buf[-1:]]))
    grads = buf[2 * ntrees:2 * ntrees + nc].copy()
    grads[np.repeat(~ok, np.diff(const_off))] = np.nan
    return sums, grads, wsum, ok


def combine_grad_shards(sums, grads, wsum, ok, const_off, all_reduce_sum: Callable[[np.ndarray], np.ndarray]):
    """Combine one rank's (Σw·ℓ, Σw·∂ℓ/∂c, Σw, ok) of its row shard with the
    other ranks' in one all-reduce (SURVEY.md §5 "constant-gradient
    all-reduce"): ∂L/∂c = ΣΣ w·∂ℓ/∂c / ΣΣ w, did_succeed = AND over shards."""
    red = all_reduce_sum(pack_grad_partials(sums, grads, wsum, ok, const_off))
    return unpack_grad_partials(red, len(sums), const_off)


class RowShardedEvaluator:
    """Evaluator for `optimize_constants_batch` over a row-sharded dataset:
    the candidates are compiled on this rank's shard, loss and gradient
    partials are all-reduced (src/ConstantOptimization.jl:12-19,43 with the
    dataset split across GPUs). `program_factory(candidates)` returns an
    object with set_constants / eval_loss / eval_loss_grad (srhip.Program on
    the shard; tests pass an oracle-backed stand-in)."""

    def __init__(self, prog, dev, loss, all_reduce_sum: Callable[[np.ndarray], np.ndarray], T):
        self.prog, self.dev, self.loss, self.red, self.T = prog, dev, loss, all_reduce_sum, T
        self.const_off = np.asarray(prog.flat.const_off)

    def _set(self, consts):
        self.prog.set_constants(np.asarray(consts).astype(self.T, copy=False))

    def loss_grad(self, consts):
        from .constant_optimization import _finish, _grad_finish

        self._set(consts)
        sums, grads, wsum, ok = self.prog.eval_loss_grad(self.dev, self.loss.kind, self.loss.params)
        s, g, W, k = combine_grad_shards(sums, grads, wsum, ok, self.const_off, self.red)
        return _finish(s, W, k), _grad_finish(g, W, k, self.const_off)

    def loss_only(self, consts):
        from .constant_optimization import _finish

        self._set(consts)
        sums, wsum, ok = self.prog.eval_loss(self.dev, self.loss.kind, self.loss.params)
        s, W, k = combine_row_shards(sums, wsum, ok, self.red)
        return _finish(s, W, k)


def torch_all_reduce_sum(device: Optional[str] = None, group=None):
    """all_reduce(SUM) over torch.distributed (RCCL with device='cuda',
    gloo with device='cpu')."""
    import torch
    import torch.distributed as dist

    def f(buf: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(buf)
        if device:
            t = t.to(device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t.cpu().numpy()

    return f


class DeviceRowShard:
    """Row-sharded eval_loss (config #5 at N GPUs). With the nccl backend
    (RCCL over xGMI) srhip_eval_loss_packed writes [Σw·ℓ, failed] per tree +
    Σw into a torch tensor on this rank's GPU and one all_reduce(SUM)
    combines the shards on the tensor itself, no host round trip. Any other
    backend (gloo: CPU tests, ranks sharing one GPU) takes the host path: the
    per-tree results of srhip_eval_loss, packed on the host (pack_partials)
    and all-reduced as a CPU tensor, so no torch GPU support is needed.
    step() returns the reduced buffer (device tensor or numpy array) and
    records the evaluation and all-reduce times of the call (host clock
    around a synchronised stream / collective)."""

    def __init__(self, prog, dev, loss, group=None):
        self.prog, self.dev, self.loss, self.group = prog, dev, loss, group
        self.nt = prog.ntrees
        self.eval_ms = self.reduce_ms = 0.0
        self.buf = self.host = None
        import torch.distributed as dist

        # no process group (one GPU): the shard is the whole dataset, nothing
        # to reduce, and no torch device state (torch's HIP runtime must be
        # loaded before libsrhip's when both are used: bench.py, tests)
        self.backend = dist.get_backend(group) if dist.is_available() and dist.is_initialized() else None
        if self.backend == "nccl":
            import torch

            self.buf = torch.zeros(2 * self.nt + 1, dtype=torch.float64, device=f"cuda:{dev.ctx.device}")

    def step(self):
        import time

        import torch
        import torch.distributed as dist

        t0 = time.perf_counter()
        if self.backend != "nccl":
            sums, wsum, ok = self.prog.eval_loss(self.dev, self.loss.kind, self.loss.params)
            packed = pack_partials(sums, wsum, ok)
            t1 = time.perf_counter()
            if self.backend is not None:
                t = torch.from_numpy(packed)
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                packed = t.numpy()
            self.host = packed
            self.eval_ms, self.reduce_ms = (t1 - t0) * 1e3, (time.perf_counter() - t1) * 1e3
            return self.host
        self.prog.eval_loss_packed(self.dev, self.loss.kind, self.buf.data_ptr(), self.loss.params)
        self.dev.ctx.sync()
        t1 = time.perf_counter()
        dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)
        torch.cuda.synchronize(self.buf.device)
        t2 = time.perf_counter()
        self.eval_ms, self.reduce_ms = (t1 - t0) * 1e3, (t2 - t1) * 1e3
        return self.buf

    def result(self):
        """(losses Σw·ℓ/Σw as float64 with NaN for failed trees, did_succeed) of the last step."""
        sums, wsum, ok = unpack_partials(self.host if self.buf is None else self.buf.cpu().numpy())
        with np.errstate(invalid="ignore", divide="ignore"):
            return sums / wsum, ok


def eval_loss_row_sharded(trees, dataset, options, device: Optional[int] = None, group=None):
    """eval_loss for many trees with the dataset's rows sharded over the ranks
    of the default process group. `dataset` is the full Dataset (X on host);
    each rank uploads only its shard. Returns (losses in T, did_succeed)."""
    import torch.distributed as dist

    from .dataset import Dataset
    from .interface import compile_trees

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    rb, re = shard_range(dataset.n, rank, world)
    shard = Dataset(dataset.X, dataset.y, dataset.weights, row_range=(rb, re))
    dev = shard.device(device)
    prog = compile_trees(trees, options, dataset.T, dev.ctx.device)
    # nccl: partials packed on the device and all-reduced there; other
    # backends: packed on the host and all-reduced as a CPU tensor (DeviceRowShard)
    rs = DeviceRowShard(prog, dev, options.elementwise_loss, group)
    rs.step()
    loss, tok = rs.result()
    T = dataset.T
    out = loss.astype(T)
    out[~tok] = T(np.inf)
    return out, tok


def shared_rng(rng=None, group=None) -> np.random.Generator:
    """One generator state on every rank: with rng None, rank 0 draws a seed
    and broadcasts it; a given rng must already be seeded identically on every
    rank (the caller's contract). The row-sharded optimiser needs this: each
    rank builds the perturbed restarts (ConstantOptimization.jl:46-54) itself,
    and partials all-reduced at different constants would describe no
    candidate."""
    import torch.distributed as dist

    if rng is not None:
        return rng
    seed = [int(np.random.SeedSequence().entropy % (1 << 63))] if dist.get_rank(group) == 0 else [None]
    dist.broadcast_object_list(seed, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return np.random.default_rng(seed[0])


def optimize_constants_row_sharded(trees, dataset, options, rng=None, device: Optional[int] = None, group=None):
    """optimize_constants_batch with the dataset's rows sharded over the ranks
    of the process group: every rank uploads its shard, compiles the
    candidates on it, and all-reduces loss and gradient partials per step
    (RowShardedEvaluator). All ranks return the same result: with rng None
    the ranks share one broadcast seed (`shared_rng`); a given rng must be
    seeded identically on every rank."""
    import torch.distributed as dist

    from .constant_optimization import optimize_constants_batch
    from .dataset import Dataset
    from .interface import compile_trees

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    rb, re = shard_range(dataset.n, rank, world)
    shard = Dataset(dataset.X, dataset.y, dataset.weights, row_range=(rb, re))
    dev = shard.device(device)
    backend = dist.get_backend(group)
    red = torch_all_reduce_sum("cuda" if backend == "nccl" else None, group)

    def factory(cands):
        return RowShardedEvaluator(compile_trees(cands, options, dataset.T, dev.ctx.device), dev,
                                   options.elementwise_loss, red, dataset.T)

    return optimize_constants_batch(dataset, trees, options, rng=shared_rng(rng, group), evaluator_factory=factory)
