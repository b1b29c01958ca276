"""ctypes binding of libsrhip.so (include/srhip.h).

The product path always goes through this library: if it cannot be loaded,
every entry point raises instead of falling back to any CPU code.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG_ROOT = Path(__file__).resolve().parent.parent  # symbolicregression.jl_amd/
LIB_PATH = Path(os.environ.get("SRHIP_LIB", _PKG_ROOT / "lib" / "libsrhip.so"))

# status codes (include/srhip.h)
OK = 0
ERR_INVALID = -1
ERR_UNSUPPORTED = -2
ERR_DEVICE = -3
ERR_NOMEM = -4


class SrhipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"srhip error {code}: {msg}")
        self.code = code


class Unsupported(SrhipError):
    """The call is outside the engine's coverage (the Julia shim would fall
    back to the reference CPU path)."""


class Trees(C.Structure):
    _fields_ = [
        ("ntrees", C.c_int32),
        ("node_off", C.POINTER(C.c_int32)),
        ("kind", C.POINTER(C.c_uint8)),
        ("arg", C.POINTER(C.c_uint16)),
        ("const_off", C.POINTER(C.c_int32)),
        ("consts", C.c_void_p),
    ]


class ConstOptOptions(C.Structure):
    """srhip_constopt_options (include/srhip.h)."""
    _fields_ = [
        ("algorithm", C.c_int32),
        ("iterations", C.c_int32),
        ("nrestarts", C.c_int32),
        ("loss_kind", C.c_int32),
        ("loss_params", C.POINTER(C.c_double)),
        ("start_noise", C.POINTER(C.c_double)),
        ("seed", C.c_uint64),
    ]


# srhip_constopt_eval_fn
CONSTOPT_EVAL_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_double),
                               C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double))

_lib = None
_load_error: Exception | None = None

# (name, argtypes) — every symbol declared in include/srhip.h
SIGNATURES = {
    "srhip_version": [],
    "srhip_last_error": [],
    "srhip_device_count": [C.POINTER(C.c_int32)],
    "srhip_open": [C.c_int32, C.POINTER(C.c_void_p)],
    "srhip_close": [C.c_void_p],
    "srhip_op_lookup": [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)],
    "srhip_op_eval": [C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_double, C.POINTER(C.c_double)],
    "srhip_last_kernel_name": [C.c_char_p, C.c_int32],
    "srhip_dataset_create": [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.POINTER(C.c_void_p)],
    "srhip_dataset_destroy": [C.c_void_p],
    "srhip_dataset_info": [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                           C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32)],
    "srhip_program_create": [C.c_void_p, C.c_int32, C.POINTER(Trees), C.POINTER(C.c_void_p)],
    "srhip_program_create_ex": [C.c_void_p, C.c_int32, C.POINTER(Trees), C.c_uint32, C.POINTER(C.c_void_p)],
    "srhip_program_destroy": [C.c_void_p],
    "srhip_program_info": [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_void_p],
    "srhip_program_set_constants": [C.c_void_p, C.c_void_p],
    "srhip_eval_loss": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int64,
                        C.c_void_p, C.POINTER(C.c_double), C.c_void_p],
    "srhip_eval_loss_packed": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p],
    "srhip_eval_loss_batch": [C.c_void_p, C.POINTER(Trees), C.c_int32, C.c_void_p, C.c_void_p,
                              C.c_int64, C.c_void_p, C.POINTER(C.c_double), C.c_void_p],
    "srhip_eval_loss_batch_ctx": [C.c_void_p, C.c_void_p, C.POINTER(Trees), C.c_int32, C.c_void_p, C.c_void_p,
                                  C.c_int64, C.c_void_p, C.POINTER(C.c_double), C.c_void_p],
    "srhip_eval_loss_rowsets": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int64,
                                C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_eval_loss_batch_rowsets_ctx": [C.c_void_p, C.c_void_p, C.POINTER(Trees), C.c_int32, C.c_void_p,
                                          C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_eval_tree_array": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_eval_loss_grad": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.POINTER(C.c_double), C.c_void_p],
    "srhip_eval_grad_tree_array": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_last_kernel_time": [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32)],
    "srhip_sync": [C.c_void_p],
    "srhip_program_jit_info": [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                               C.POINTER(C.c_double), C.POINTER(C.c_double)],
    "srhip_program_update_stats": [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "srhip_program_grad_jit_info": [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                    C.POINTER(C.c_double), C.POINTER(C.c_double)],
    "srhip_last_bailed": [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)],
    "srhip_last_tree_code": [C.c_void_p, C.POINTER(C.c_int32)],
    "srhip_jit_compile": [C.POINTER(Trees), C.c_int32, C.c_void_p, C.POINTER(C.c_int64), C.c_char_p,
                          C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int64)],
    "srhip_jit_compile_grad": [C.POINTER(Trees), C.c_void_p, C.POINTER(C.c_int64), C.c_char_p,
                               C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int64)],
    "srhip_jit_compile_loss": [C.POINTER(Trees), C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_void_p,
                               C.POINTER(C.c_int64), C.c_char_p, C.POINTER(C.c_int64), C.c_void_p,
                               C.POINTER(C.c_int64)],
    "srhip_constopt_profile": [C.POINTER(C.c_double), C.c_int32],
    "srhip_optimize_constants_batch": [C.c_void_p, C.c_void_p, C.POINTER(Trees), C.POINTER(ConstOptOptions),
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_optimize_constants_cb": [C.POINTER(Trees), C.c_int32, C.POINTER(ConstOptOptions), CONSTOPT_EVAL_FN,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "srhip_debug_constant_map": [C.POINTER(Trees), C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int64), C.POINTER(C.c_int32)],
}


def lib():
    """The loaded library; raises if libsrhip.so is missing (no fallback)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise _load_error
    try:
        L = C.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - exercised only without a build
        _load_error = ImportError(
            f"libsrhip.so not loadable from {LIB_PATH}: {e}. Build it with "
            "`make -C symbolicregression.jl_amd/csrc` (or __graft_entry__.build())."
        )
        raise _load_error
    for name, argtypes in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = C.c_int32
    L.srhip_last_error.restype = C.c_char_p
    _lib = L
    return L


def check(rc: int) -> None:
    if rc == OK:
        return
    msg = lib().srhip_last_error().decode(errors="replace")
    if rc == ERR_UNSUPPORTED:
        raise Unsupported(rc, msg)
    raise SrhipError(rc, msg)
