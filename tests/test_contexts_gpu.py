"""Contexts and threads (srhip.h conventions): a program
runs on its own context, a dataset is shared by every context of its device.
The Julia binding relies on this: each thread (one island per
Threads.@spawn, src/SearchUtils.jl:33-45) creates its programs in its own
context and scores them on one uploaded Dataset.

* a program created in context B evaluates a dataset uploaded through
  context A, bit for bit as in one context (loss, ∂L/∂c, eval_tree_array);
* two host threads, each with its own context and program, run
  eval_loss_grad concurrently on one dataset: every result equals the
  serial one (ctypes releases the GIL inside the C call, so the calls
  overlap);
* srhip_eval_loss_batch_ctx scores in the given context.
"""
import ctypes as C
import threading

import numpy as np
import pytest

import srhip
from srhip import constants as K
from srhip._lib import lib
from srhip.engine import _p, _trees_struct

pytestmark = pytest.mark.gpu


def _free(*objs):
    """Destroy programs / datasets now (before their context is closed)."""
    for o in objs:
        if o is not None:
            o.__del__()


CFG = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


def _data(n=200_000, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    return X, y


def test_program_in_other_context_runs_on_shared_dataset(gpu_ctx):
    o = srhip.Options(**CFG)
    X, y = _data()
    trees = srhip.random_population(700, o, 5, np.float32, seed=11)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    a, b = srhip.Context(0), srhip.Context(0)
    ds = pa = pb = small = None
    try:
        ds = srhip.DeviceDataset(a, X, y)
        pa, pb = srhip.Program(a, flat, np.float32), srhip.Program(b, flat, np.float32)
        sa, wa, oka = pa.eval_loss(ds, K.LOSS["L2"])
        sb, wb, okb = pb.eval_loss(ds, K.LOSS["L2"])
        assert wa == wb and np.array_equal(oka, okb) and np.array_equal(sa[oka], sb[okb])
        ga = pa.eval_loss_grad(ds, K.LOSS["L2"])
        gb = pb.eval_loss_grad(ds, K.LOSS["L2"])
        assert np.array_equal(ga[3], gb[3]) and np.array_equal(ga[0][ga[3]], gb[0][gb[3]])
        np.testing.assert_array_equal(ga[1], gb[1])
        small = srhip.DeviceDataset(a, X[:, :3000], y[:3000])
        oa, _ = pa.eval_tree_array(small)
        ob, _ = pb.eval_tree_array(small)
        np.testing.assert_array_equal(oa, ob)
        # the timing of a call is reported by the context that ran it (the program's)
        assert b.last_kernel_time()[1] >= 1
    finally:
        _free(pa, pb, ds, small)
        a.close()
        b.close()


def test_threads_with_own_contexts_run_concurrently(gpu_ctx):
    o = srhip.Options(**CFG)
    X, y = _data()
    shared = srhip.DeviceDataset(gpu_ctx, X, y)
    nthreads, reps = 4, 6
    ctxs = [srhip.Context(0) for _ in range(nthreads)]
    progs, serial = [], []
    try:
        for k in range(nthreads):
            trees = [t for t in srhip.random_population(400, o, 5, np.float32, seed=100 + k)
                     if srhip.get_constants(t)]
            p = srhip.Program(ctxs[k], srhip.flatten(trees, o, dtype=np.float32), np.float32)
            progs.append(p)
            serial.append(p.eval_loss_grad(shared, K.LOSS["L2"]))
        errors, results = [], [[None] * reps for _ in range(nthreads)]
        start = threading.Barrier(nthreads)

        def work(k):
            try:
                start.wait()
                for r in range(reps):
                    results[k][r] = progs[k].eval_loss_grad(shared, K.LOSS["L2"])
            except Exception as e:  # reported below
                errors.append((k, e))

        th = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errors, errors
        for k in range(nthreads):
            s0, g0, w0, ok0 = serial[k]
            for r in range(reps):
                s, g, w, ok = results[k][r]
                assert w == w0 and np.array_equal(ok, ok0)
                np.testing.assert_array_equal(s[ok], s0[ok0])
                np.testing.assert_array_equal(g, g0)
    finally:
        _free(*progs, shared)
        for c in ctxs:
            c.close()


def test_eval_loss_batch_ctx_uses_given_context(gpu_ctx):
    o = srhip.Options(**CFG)
    X, y = _data(50_000)
    trees = srhip.random_population(64, o, 5, np.float32, seed=5)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    ds = srhip.DeviceDataset(gpu_ctx, X, y)
    other = srhip.Context(0)
    try:
        consts = np.ascontiguousarray(flat.consts, dtype=np.float32)
        tr = _trees_struct(flat, consts)
        sums = np.zeros(len(trees))
        ok = np.zeros(len(trees), dtype=np.uint8)
        w = C.c_double(0)
        rc = lib().srhip_eval_loss_batch_ctx(other.handle, ds.handle, C.byref(tr), K.LOSS["L2"], None, None, 0,
                                             _p(sums), C.byref(w), _p(ok))
        assert rc == 0
        ref_p = srhip.Program(gpu_ctx, flat, np.float32)
        ref_s, ref_w, ref_ok = ref_p.eval_loss(ds, K.LOSS["L2"])
        _free(ref_p)
        assert w.value == ref_w and np.array_equal(ok.astype(bool), ref_ok)
        np.testing.assert_array_equal(sums[ref_ok], ref_s[ref_ok])
        assert other.last_kernel_time()[1] >= 1  # ran in `other`
    finally:
        _free(ds)
        other.close()
