"""The C ABI surface (no GPU needed): libsrhip.so loads, exports every symbol
include/srhip.h declares, and its tables agree with the Python mirror."""
import ctypes as C
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = (ROOT / "include" / "srhip.h").read_text()


def header_defines(prefix):
    return {m.group(1): int(m.group(2)) for m in re.finditer(rf"#define {prefix}(\w+)\s+\(?(-?\d+)\)?", HEADER)}


def header_functions():
    return sorted(set(re.findall(r"^(?:int32_t|const char\*)\s+(srhip_\w+)\(", HEADER, re.M)))


def test_header_ids_match_python_constants():
    import srhip.constants as K

    bops = header_defines("SRHIP_BOP_")
    uops = header_defines("SRHIP_UOP_")
    losses = header_defines("SRHIP_LOSS_")
    assert bops == K.BOP
    assert uops == K.UOP
    assert losses == K.LOSS
    nb = int(re.search(r"#define SRHIP_NUM_BOPS (\d+)", HEADER).group(1))
    nu = int(re.search(r"#define SRHIP_NUM_UOPS (\d+)", HEADER).group(1))
    nl = int(re.search(r"#define SRHIP_NUM_LOSSES (\d+)", HEADER).group(1))
    assert nb == len(K.BOPS) and nu == len(K.UOPS) and nl == len(K.LOSSES)


def test_library_exports_every_declared_symbol():
    from srhip import _lib

    L = _lib.lib()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/srhip.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(declared)


def test_version_and_errors_without_device():
    from srhip import _lib

    L = _lib.lib()
    assert L.srhip_version() == 1
    # invalid-argument path needs no device
    rc = L.srhip_open(0, None)
    assert rc == _lib.ERR_INVALID
    assert b"null" in L.srhip_last_error()


def test_op_lookup_matches_python_table():
    import srhip.constants as K
    from srhip import _lib

    L = _lib.lib()
    for name, (arity, ident) in K.OP_NAMES.items():
        a, i = C.c_int32(), C.c_int32()
        assert L.srhip_op_lookup(name.encode(), C.byref(a), C.byref(i)) == 0, name
        assert (a.value, i.value) == (arity, ident), name
    assert L.srhip_op_lookup(b"asin", None, None) == _lib.ERR_UNSUPPORTED
    assert b"asin" in L.srhip_last_error()


def test_unsupported_operator_raises_in_mirror():
    import srhip

    o = srhip.Options(binary_operators=["+"], unary_operators=["asin"])
    with pytest.raises(srhip.Unsupported):
        o.engine_operator_ids()
