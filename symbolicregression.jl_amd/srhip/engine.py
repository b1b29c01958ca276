"""Thin object layer over the C ABI: device contexts, device datasets and
compiled programs. Everything here calls libsrhip.so; nothing computes on
the CPU."""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import numpy as np

from . import constants as K
from ._lib import SrhipError, Trees, check, lib
from .node import FlatTrees

_ctx_lock = threading.Lock()
_contexts: dict = {}


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data  # an int: ctypes passes it as void*, cheaper than data_as


def dtype_code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt == np.float32:
        return K.F32
    if dt == np.float64:
        return K.F64
    from ._lib import Unsupported

    raise Unsupported(-2, f"dtype {dt} is not supported by the engine (Float32/Float64 only)")


def device_count() -> int:
    n = C.c_int32(0)
    lib().srhip_device_count(C.byref(n))
    return n.value


class Context:
    """One device + stream (srhip_open). Calls through one context are
    serialised by the library."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().srhip_open(int(device), C.byref(h)))
        self.handle = h
        self.device = int(device)

    def close(self):
        if self.handle:
            lib().srhip_close(self.handle)
            self.handle = None

    def last_kernel_time(self):
        ms = C.c_double(0)
        n = C.c_int32(0)
        check(lib().srhip_last_kernel_time(self.handle, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def sync(self):
        check(lib().srhip_sync(self.handle))

    def last_bailed(self) -> int:
        """Trees of the last eval whose tree code handed a tile back."""
        return self.last_jit_events()[0]

    def last_kernel_name(self) -> str:
        """The main evaluation kernel this thread launched last (srhip_last_kernel_name)."""
        buf = C.create_string_buffer(128)
        check(lib().srhip_last_kernel_name(buf, 128))
        return buf.value.decode()

    def last_tree_code(self) -> int:
        """Trees the last eval ran as tree code (srhip_last_tree_code)."""
        n = C.c_int32(0)
        check(lib().srhip_last_tree_code(self.handle, C.byref(n)))
        return n.value

    def last_jit_events(self):
        """(trees handed back to the interpreter, tiles redone with the
        PRECISE routines) of the last eval."""
        n = C.c_int32(0)
        r = C.c_int64(0)
        check(lib().srhip_last_bailed(self.handle, C.byref(n), C.byref(r)))
        return n.value, r.value


def default_device() -> int:
    return int(os.environ.get("SRHIP_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def get_context(device: Optional[int] = None) -> Context:
    d = default_device() if device is None else int(device)
    with _ctx_lock:
        c = _contexts.get(d)
        if c is None:
            c = Context(d)
            _contexts[d] = c
        return c


class DeviceDataset:
    """srhip_dataset: rows [row_begin, row_end) of X (nfeatures, n), y, w
    resident on one device."""

    def __init__(self, ctx: Context, X: np.ndarray, y: np.ndarray, w: Optional[np.ndarray] = None,
                 row_begin: int = 0, row_end: Optional[int] = None):
        if X.ndim != 2:
            raise ValueError("X must be (nfeatures, n)")
        dt = np.result_type(X.dtype, y.dtype)
        code = dtype_code(dt)
        nfeat, n = X.shape
        if X.flags.c_contiguous:
            layout, Xa = K.X_FEATURE_MAJOR, np.ascontiguousarray(X, dtype=dt)
        else:  # Fortran order = Julia's column-major (nfeatures, n)
            layout, Xa = K.X_JULIA, np.asfortranarray(X, dtype=dt)
        ya = np.ascontiguousarray(y, dtype=dt)
        wa = None if w is None else np.ascontiguousarray(w, dtype=dt)
        if ya.shape != (n,) or (wa is not None and wa.shape != (n,)):
            raise AssertionError("Dataset dimensions are invalid")  # Configure.jl:53-60
        rb = int(row_begin)
        re = n if row_end is None else int(row_end)
        h = C.c_void_p()
        check(lib().srhip_dataset_create(ctx.handle, code, layout, _p(Xa), _p(ya), _p(wa), n, nfeat, rb,
                                         re, C.byref(h)))
        self.handle = h
        self.ctx = ctx
        self.dtype = dt
        self.nfeat = nfeat
        self.rows = re - rb
        self.weighted = w is not None

    def info(self):
        rows = C.c_int64()
        nf = C.c_int32()
        sw = C.c_double()
        syw = C.c_double()
        fin = C.c_int32()
        check(lib().srhip_dataset_info(self.handle, C.byref(rows), C.byref(nf), C.byref(sw), C.byref(syw),
                                       C.byref(fin)))
        return dict(rows=rows.value, nfeat=nf.value, sum_w=sw.value, sum_yw=syw.value, x_finite=bool(fin.value))

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().srhip_dataset_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class Program:
    """srhip_program: a compiled, device-resident batch of trees.
    varying_constants (SRHIP_PROGRAM_VARYING_CONSTANTS): the caller will set
    new constants, so Float32 tree code reads them from memory from the start."""

    def __init__(self, ctx: Context, flat: FlatTrees, dtype, varying_constants: bool = False,
                 interpreted: bool = False):
        self.ctx = ctx
        self.dtype = np.dtype(dtype)
        self.flat = flat
        consts = np.ascontiguousarray(flat.consts, dtype=self.dtype)
        self._keep = (flat.node_off, flat.kind, flat.arg, flat.const_off, consts)
        tr = Trees(
            flat.ntrees,
            flat.node_off.ctypes.data_as(C.POINTER(C.c_int32)),
            flat.kind.ctypes.data_as(C.POINTER(C.c_uint8)),
            flat.arg.ctypes.data_as(C.POINTER(C.c_uint16)),
            flat.const_off.ctypes.data_as(C.POINTER(C.c_int32)),
            consts.ctypes.data_as(C.c_void_p),
        )
        h = C.c_void_p()
        check(lib().srhip_program_create_ex(ctx.handle, dtype_code(self.dtype), C.byref(tr),
                                            (K.PROGRAM_VARYING_CONSTANTS if varying_constants else 0)
                                            | (K.PROGRAM_INTERPRETED if interpreted else 0), C.byref(h)))
        self.handle = h
        self.ntrees = flat.ntrees

    def info(self):
        nt = C.c_int32()
        tot = C.c_int64()
        nodes = np.zeros(max(self.ntrees, 1), dtype=np.int32)
        check(lib().srhip_program_info(self.handle, C.byref(nt), C.byref(tot), _p(nodes)))
        return nt.value, tot.value, nodes[: nt.value]

    def jit_info(self):
        """Tree code of this program (srhip_program_jit_info)."""
        nt, nf = C.c_int32(), C.c_int32()
        nb = C.c_int64()
        mc, ml = C.c_double(), C.c_double()
        check(lib().srhip_program_jit_info(self.handle, C.byref(nt), C.byref(nf), C.byref(nb), C.byref(mc),
                                           C.byref(ml)))
        return dict(ntrees=nt.value, nfast=nf.value, code_bytes=nb.value, ms_codegen=mc.value, ms_load=ml.value)

    def grad_jit_info(self):
        """Gradient tree code of this program (srhip_program_grad_jit_info)."""
        nt, nr = C.c_int32(), C.c_int32()
        nb = C.c_int64()
        mc, ml = C.c_double(), C.c_double()
        check(lib().srhip_program_grad_jit_info(self.handle, C.byref(nt), C.byref(nr), C.byref(nb), C.byref(mc),
                                                C.byref(ml)))
        return dict(ntrees=nt.value, nrejected=nr.value, code_bytes=nb.value, ms_codegen=mc.value,
                    ms_load=ml.value)

    def update_stats(self):
        """How set_constants applied new constants: {"inplace": n, "rebuilt": n}."""
        a, b = C.c_int64(), C.c_int64()
        check(lib().srhip_program_update_stats(self.handle, C.byref(a), C.byref(b)))
        return dict(inplace=a.value, rebuilt=b.value)

    def set_constants(self, consts: np.ndarray):
        c = np.ascontiguousarray(consts, dtype=self.dtype)
        if c.shape != (int(self.flat.const_off[-1]),):
            raise ValueError("constant vector has the wrong length")
        check(lib().srhip_program_set_constants(self.handle, _p(c)))

    def eval_loss(self, ds: DeviceDataset, loss_kind: int, params=None, row_idx=None):
        nt = self.ntrees
        sums = np.empty(max(nt, 1), dtype=np.float64)  # the library writes every tree's entry
        ok = np.empty(max(nt, 1), dtype=np.uint8)
        wsum = C.c_double(0)
        par = None if params is None else np.asarray(params, dtype=np.float64)
        idx = None if row_idx is None else np.ascontiguousarray(row_idx, dtype=np.int64)
        nidx = 0 if idx is None else len(idx)
        check(lib().srhip_eval_loss(ds.handle, self.handle, int(loss_kind), _p(par), _p(idx), nidx, _p(sums),
                                    C.byref(wsum), _p(ok)))
        return sums[:nt], wsum.value, ok[:nt].view(bool)  # 0/1 bytes: a view, no copy

    def eval_loss_rowsets(self, ds: DeviceDataset, loss_kind: int, row_idx, params=None):
        """srhip_eval_loss_rowsets: tree t on its own rows row_idx[t] (an
        (ntrees, batch_size) integer array): (Σ w·ℓ per tree, Σ w per tree, ok)."""
        nt = self.ntrees
        idx = np.ascontiguousarray(row_idx, dtype=np.int64)
        if idx.ndim != 2 or idx.shape[0] != nt:
            raise ValueError("row_idx must be (ntrees, batch_size)")
        sums = np.empty(max(nt, 1), dtype=np.float64)
        wsum = np.empty(max(nt, 1), dtype=np.float64)
        ok = np.empty(max(nt, 1), dtype=np.uint8)
        par = None if params is None else np.asarray(params, dtype=np.float64)
        check(lib().srhip_eval_loss_rowsets(ds.handle, self.handle, int(loss_kind), _p(par), _p(idx), idx.shape[1],
                                            _p(sums), _p(wsum), _p(ok)))
        return sums[:nt], wsum[:nt], ok[:nt].view(bool)

    def eval_loss_packed(self, ds: DeviceDataset, loss_kind: int, d_out: int, params=None):
        """srhip_eval_loss_packed: [Σw·ℓ, failed] per tree + Σw written to the
        device buffer at address d_out (2·ntrees + 1 float64, e.g. a torch
        tensor's data_ptr()), enqueued on the context's stream (ctx.sync()
        before another stream reads it)."""
        par = None if params is None else np.asarray(params, dtype=np.float64)
        check(lib().srhip_eval_loss_packed(ds.handle, self.handle, int(loss_kind), _p(par), C.c_void_p(int(d_out))))

    def eval_loss_grad(self, ds: DeviceDataset, loss_kind: int, params=None):
        """(Σ w·ℓ per tree, Σ w·∂ℓ/∂c per constant [const_off order], Σw, ok)."""
        nt = self.ntrees
        nc = int(self.flat.const_off[-1])
        sums = np.zeros(max(nt, 1), dtype=np.float64)
        grads = np.zeros(max(nc, 1), dtype=np.float64)
        ok = np.zeros(max(nt, 1), dtype=np.uint8)
        wsum = C.c_double(0)
        par = None if params is None else np.asarray(params, dtype=np.float64)
        check(lib().srhip_eval_loss_grad(ds.handle, self.handle, int(loss_kind), _p(par), _p(sums), _p(grads),
                                         C.byref(wsum), _p(ok)))
        return sums[:nt], grads[:nc], wsum.value, ok[:nt].astype(bool)

    def eval_grad_tree_array(self, ds: DeviceDataset):
        """(ŷ [ntrees][rows], ∂ŷ/∂c [total consts][rows], ok)."""
        nt = self.ntrees
        nc = int(self.flat.const_off[-1])
        val = np.empty((nt, ds.rows), dtype=self.dtype)
        grad = np.empty((nc, ds.rows), dtype=self.dtype)
        ok = np.zeros(max(nt, 1), dtype=np.uint8)
        check(lib().srhip_eval_grad_tree_array(ds.handle, self.handle, _p(val), _p(grad), _p(ok)))
        return val, grad, ok[:nt].astype(bool)

    def eval_tree_array(self, ds: DeviceDataset):
        nt = self.ntrees
        out = np.empty((nt, ds.rows), dtype=self.dtype)
        ok = np.zeros(max(nt, 1), dtype=np.uint8)
        check(lib().srhip_eval_tree_array(ds.handle, self.handle, _p(out), _p(ok)))
        return out, ok[:nt].astype(bool)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().srhip_program_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def _trees_struct(flat: FlatTrees, consts: np.ndarray) -> Trees:
    return Trees(
        flat.ntrees,
        flat.node_off.ctypes.data_as(C.POINTER(C.c_int32)),
        flat.kind.ctypes.data_as(C.POINTER(C.c_uint8)),
        flat.arg.ctypes.data_as(C.POINTER(C.c_uint16)),
        flat.const_off.ctypes.data_as(C.POINTER(C.c_int32)),
        consts.ctypes.data_as(C.c_void_p),
    )


def jit_compile(flat: FlatTrees, fast: bool = True, grad: bool = False, memc: bool = False, loss=None,
                out: bool = False, text: bool = True):
    """Tree compiler without a device (srhip_jit_compile, or with grad=True
    srhip_jit_compile_grad: the reverse-mode gradient tree code; memc: the
    memory-constant loss tree code; loss: a Loss other than L2, through
    srhip_jit_compile_loss; out: the per-row output code of
    srhip_eval_tree_array): (code bytes, assembly text, {tree id: byte
    offset})."""
    f64 = np.dtype(flat.consts.dtype) == np.float64
    consts = np.ascontiguousarray(flat.consts, dtype=np.float64 if f64 else np.float32)
    tr = _trees_struct(flat, consts)
    nb, nt, no = C.c_int64(0), C.c_int64(0), C.c_int64(0)

    def call(*bufs):
        if f64 and grad:  # the Float64 gradient tree code (jit64.cpp GradGen64)
            kind, param = (0, 0.0) if loss is None else (int(loss.kind), float(loss.param))
            return lib().srhip_jit_compile_loss(C.byref(tr), 1, 8, kind, param, bufs[0], C.byref(nb), bufs[1],
                                                C.byref(nt), bufs[2], C.byref(no))
        if f64 and loss is not None:  # the Float64 tree compiler with another loss's tail
            return lib().srhip_jit_compile_loss(C.byref(tr), 0, 8, int(loss.kind), float(loss.param),
                                                bufs[0], C.byref(nb), bufs[1], C.byref(nt), bufs[2], C.byref(no))
        if f64:  # the Float64 tree compiler (jit64.cpp), L2 or per-row outputs
            return lib().srhip_jit_compile(C.byref(tr), 8 | (4 if out else 0), bufs[0], C.byref(nb), bufs[1],
                                           C.byref(nt), bufs[2], C.byref(no))
        if loss is not None:
            return lib().srhip_jit_compile_loss(C.byref(tr), int(grad), int(fast), int(loss.kind), float(loss.param),
                                                bufs[0], C.byref(nb), bufs[1], C.byref(nt), bufs[2], C.byref(no))
        if grad:
            return lib().srhip_jit_compile_grad(C.byref(tr), bufs[0], C.byref(nb), bufs[1], C.byref(nt), bufs[2],
                                                C.byref(no))
        return lib().srhip_jit_compile(C.byref(tr), int(fast) | (2 if memc else 0) | (4 if out else 0) |
                                       (0 if text else 16), bufs[0],
                                       C.byref(nb), bufs[1],
                                       C.byref(nt), bufs[2], C.byref(no))

    rc = call(None, None, None)
    if rc != -1:
        check(rc)
    buf = np.zeros(max(nb.value, 1), dtype=np.uint8)
    txt = C.create_string_buffer(max(nt.value, 1))
    offs = np.zeros(max(no.value, 1), dtype=np.int32)
    check(call(_p(buf), txt, _p(offs)))
    pairs = offs[: no.value].reshape(-1, 2)
    return bytes(buf[: nb.value]), txt.value.decode(), {int(t): int(o) for t, o in pairs}


def debug_constant_map(flat: FlatTrees, new_consts, dtype, grad: bool = False, keep_layout: bool = False):
    """srhip_debug_constant_map (no device): (trees that differ from a fresh
    compile after writing new_consts through the constant map, trees the
    update recompiled, 1 if it needed a rebuild). keep_layout: the images of
    a program whose constants change (failing trees keep their code)."""
    dt = np.dtype(dtype)
    consts = np.ascontiguousarray(flat.consts, dtype=dt)
    new = np.ascontiguousarray(new_consts, dtype=dt)
    tr = _trees_struct(flat, consts)
    mm, rc, rl = C.c_int64(), C.c_int64(), C.c_int32()
    check(lib().srhip_debug_constant_map(C.byref(tr), dtype_code(dt), int(grad) | (2 if keep_layout else 0), _p(new),
                                         C.byref(mm), C.byref(rc),
                                         C.byref(rl)))
    return mm.value, rc.value, rl.value


__all__ = ["Context", "DeviceDataset", "Program", "get_context", "device_count", "SrhipError", "jit_compile",
           "debug_constant_map"]
