"""`Dataset{T}` (src/Dataset.jl:24-64) with a device-resident copy.

X has the reference's shape (nfeatures, n) — X[f, i] is feature f of row i —
y is (n,), weights optional. avg_y and baseline_loss follow the reference;
the device copy (srhip_dataset) is made on first use and reused by every
evaluation (uploaded once, src/LossFunctions.jl:122-126 is the first user).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .engine import DeviceDataset, get_context


class Dataset:
    def __init__(self, X: np.ndarray, y: np.ndarray, weights: Optional[np.ndarray] = None,
                 varMap: Optional[Sequence[str]] = None, row_range: Optional[tuple] = None):
        X = np.asarray(X)
        y = np.asarray(y)
        if X.ndim != 2:
            raise ValueError("X must be (nfeatures, n)")
        self.X = X
        self.y = y
        self.nfeatures, self.n = X.shape
        self.weighted = weights is not None
        self.weights = None if weights is None else np.asarray(weights)
        self.varMap = list(varMap) if varMap is not None else [f"x{i + 1}" for i in range(self.nfeatures)]
        T = np.result_type(X.dtype, y.dtype)
        self.T = T.type
        # avg_y, src/Dataset.jl:56-60 (computed in T like the reference)
        if self.weighted:
            self.avg_y = T.type(np.sum(y * self.weights, dtype=T) / np.sum(self.weights, dtype=T))
        else:
            self.avg_y = T.type(np.sum(y, dtype=T) / T.type(self.n))
        self.baseline_loss = T.type(1)  # src/Dataset.jl:61
        self.row_range = row_range  # (row_begin, row_end) shard of this process, or None
        self._dev = {}

    def device(self, device: Optional[int] = None) -> DeviceDataset:
        ctx = get_context(device)
        d = self._dev.get(ctx.device)
        if d is None:
            rb, re = self.row_range if self.row_range is not None else (0, self.n)
            d = DeviceDataset(ctx, self.X, self.y, self.weights, rb, re)
            self._dev[ctx.device] = d
        return d
