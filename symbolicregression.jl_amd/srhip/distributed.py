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

The combine step is plain host logic on top of any all-reduce, so it is
tested with the gloo backend on CPU (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row shard [begin, end) of rank (sizes differ by at most 1)."""
    base, extra = divmod(n, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


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
    loss = options.elementwise_loss
    sums, wsum, ok = prog.eval_loss(dev, loss.kind, loss.params)
    backend = dist.get_backend(group)
    red = torch_all_reduce_sum("cuda" if backend == "nccl" else None, group)
    tsum, twsum, tok = combine_row_shards(sums, wsum, ok, red)
    T = dataset.T
    with np.errstate(invalid="ignore", divide="ignore"):
        out = (tsum / twsum).astype(T)
    out[~tok] = T(np.inf)
    return out, tok
