"""Tree compiler (csrc/jit.cpp) on the CPU: its machine code is what the LLVM
assembler makes of its own assembly text, instruction for instruction.

The tree compiler writes gfx950 machine code directly (no assembler at run
time). Every encoding it can emit appears in random programs of several
operator sets; the test assembles the text mirror with llvm-mc
(/opt/rocm/lib/llvm/bin) and compares the bytes. The GPU tests
(tests/test_jit_gpu.py) check what the code computes."""
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

import srhip
from srhip.engine import jit_compile

LLVM = Path("/opt/rocm/lib/llvm/bin")
OPSETS = [
    (["+", "-", "*", "/"], ["cos", "exp"]),  # config #2: FAST path with guards
    (["+", "-", "*", "/"], ["sin", "cos", "exp", "neg", "square", "cube", "abs"]),
    (["+", "*", "/", "-", "^", "max", "min", "mod"], ["safe_log", "safe_sqrt", "tanh", "relu", "inv", "sign"]),
]


def assemble(text: str) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        s, o, b = (os.path.join(td, n) for n in ("t.s", "t.o", "t.bin"))
        Path(s).write_text(".text\n" + text)
        subprocess.run([str(LLVM / "llvm-mc"), "-triple", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-filetype=obj",
                        s, "-o", o], check=True, capture_output=True)
        subprocess.run([str(LLVM / "llvm-objcopy"), "-O", "binary", "--only-section=.text", o, b], check=True)
        return Path(b).read_bytes()


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("k", range(len(OPSETS)))
def test_machine_code_equals_llvm_mc(k):
    b_ops, u_ops = OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(300, o, 7, np.float32, seed=11 + k)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    for fast, memc in ((True, False), (False, False), (True, True)):
        code, text, offs = jit_compile(flat, fast=fast, memc=memc)
        assert len(offs) >= 0.7 * len(trees), f"only {len(offs)} of {len(trees)} trees compiled"
        ref = assemble(text)
        assert len(ref) == len(code)
        if ref != code:
            a = np.frombuffer(code, dtype=np.uint32)
            r = np.frombuffer(ref, dtype=np.uint32)
            i = int(np.flatnonzero(a != r)[0])
            lines = [ln for ln in text.splitlines() if not ln.startswith(";")]
            raise AssertionError(f"word {i}: jit {a[i]:#010x} vs llvm-mc {r[i]:#010x} near '{lines[:]}'"[:400])


@pytest.mark.parametrize("k", range(len(OPSETS)))
def test_threaded_code_generation_equals_serial(k):
    """build()'s code generation on several host threads (every tree at a
    provisional address, the layout, every tree again at its final address)
    gives the serial generator's bytes and offsets exactly."""
    b_ops, u_ops = OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    flat = srhip.flatten(srhip.random_population(1500, o, 7, np.float32, seed=71 + k), o, dtype=np.float32)
    for fast, memc in ((True, False), (False, False), (True, True)):
        code_t, _, offs_t = jit_compile(flat, fast=fast, memc=memc)
        code_p, text_p, offs_p = jit_compile(flat, fast=fast, memc=memc, text=False)
        assert text_p == ""
        assert offs_p == offs_t and code_p == code_t


def test_every_tree_of_config2_compiles():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(1000, o, 5, np.float32, seed=0)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    code, _, offs = jit_compile(flat)
    assert len(offs) >= 990
    assert all(v % 64 == 0 for v in offs.values())
    print(f"{len(offs)} trees, {len(code) / len(offs):.0f} bytes per tree")


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
def test_shared_subtree_columns_equal_llvm_mc():
    """Config #2's shared subtrees (cos(x_f), exp(cos(x_f)), x_i / x_j, ...) are
    read from their columns with global loads (jit.h Columns::gkey): the code
    holds them, its bytes are llvm-mc's, and memory-constant code (whose
    driver passes no column base) holds none."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    flat = srhip.flatten(srhip.random_population(1500, o, 5, np.float32, seed=1000), o, dtype=np.float32)
    code, text, offs = jit_compile(flat)
    assert text.count("global_load_dwordx4") > 500 and "s_waitcnt vmcnt(0)" in text
    assert assemble(text) == code
    _, text_m, _ = jit_compile(flat, memc=True)
    assert "global_load_dwordx4" not in text_m


def test_memory_constant_code_loads_every_constant():
    """Memory-constant tree code (set_constants without new code): no
    literal of the tree's constants remains in its code, and every constant
    is loaded from its program instruction (s_load_dword ..., 8 pc + 4)."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    x1, x2 = srhip.Node("x1"), srhip.Node("x2")
    c = [np.float32(v) for v in (1.2345678, -0.7654321, 3.3333333)]
    t = o.make_binary("+", o.make_binary("*", srhip.Node(val=c[0]), o.make_unary("cos", x1)),
                      o.make_binary("/", x2, srhip.Node(val=c[1])))
    t = o.make_binary("-", t, o.make_unary("exp", o.make_binary("*", x2, srhip.Node(val=c[2]))))
    flat = srhip.flatten([t], o, dtype=np.float32)
    for fast in (True, False):
        _, lit_text, _ = jit_compile(flat, fast=fast)
        _, text, offs = jit_compile(flat, fast=fast, memc=True)
        assert offs
        hexes = {hex(int(np.float32(v).view(np.uint32))) for v in c}
        assert any(h in lit_text for h in hexes)
        assert not any(h in text for h in hexes), "a constant compiled in as a literal"
        loads = [ln for ln in text.splitlines() if ln.startswith("s_load_dword s")]
        assert len(loads) == 3, loads


GRAD_OPSETS = [
    (["+", "-", "*", "/"], ["cos", "exp"]),  # config #5
    (["+", "-", "*", "/"], ["sin", "cos", "exp", "neg", "square", "cube", "abs"]),
    (["+", "-", "*", "/", "^"], ["safe_log", "safe_sqrt", "cos", "exp"]),  # config #3's operators
]


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("k", range(len(GRAD_OPSETS)))
def test_gradient_machine_code_equals_llvm_mc(k):
    """The reverse-mode gradient tree code (csrc/jit_grad.cpp): same check."""
    b_ops, u_ops = GRAD_OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(300, o, 7, np.float32, seed=21 + k)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    code, text, offs = jit_compile(flat, grad=True)
    assert len(offs) >= 0.9 * len(trees), f"only {len(offs)} of {len(trees)} trees compiled"
    ref = assemble(text)
    assert len(ref) == len(code)
    if ref != code:
        a = np.frombuffer(code, dtype=np.uint32)
        r = np.frombuffer(ref, dtype=np.uint32)
        i = int(np.flatnonzero(a != r)[0])
        raise AssertionError(f"word {i}: jit {a[i]:#010x} vs llvm-mc {r[i]:#010x}")


TRANS = ("v_rcp_f32", "v_exp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32")


def trans_forwarding_hazards(text: str):
    """Instructions that read a transcendental's destination VGPR right
    after it: gfx950 needs one wait state in between (a read without it sees
    the register's old value; round 5's safe_log / safe_sqrt reverse rules
    did this and their gradients came out wrong on the GPU only)."""
    import re
    ins = [ln.strip() for ln in text.splitlines()
           if ln.strip() and not ln.strip().startswith(";") and not ln.strip().endswith(":")]
    bad = []
    for a, b in zip(ins, ins[1:]):
        if not a.startswith(TRANS):
            continue
        dst = a.split()[1].rstrip(",")
        srcs = b.split(None, 1)[1].split(",")[1:] if len(b.split(None, 1)) > 1 else []
        if b.startswith("v_") and any(re.fullmatch(re.escape(dst), s.strip().split()[0]) for s in srcs if s.strip()):
            bad.append((a, b))
    return bad


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("k", range(len(GRAD_OPSETS)))
def test_float64_gradient_machine_code_equals_llvm_mc(k):
    """The Float64 reverse-mode gradient tree code (jit64.cpp GradGen64): same
    check, and every tree of these operator sets compiles."""
    b_ops, u_ops = GRAD_OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(300, o, 7, np.float64, seed=51 + k)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    code, text, offs = jit_compile(flat, grad=True)
    assert len(offs) >= 0.95 * len(trees), f"only {len(offs)} of {len(trees)} trees compiled"
    ref = assemble(text)
    assert len(ref) == len(code)
    if ref != code:
        a = np.frombuffer(code, dtype=np.uint32)
        r = np.frombuffer(ref, dtype=np.uint32)
        i = int(np.flatnonzero(a != r)[0])
        raise AssertionError(f"word {i}: jit {a[i]:#010x} vs llvm-mc {r[i]:#010x}")
    assert not trans_forwarding_hazards(text)


@pytest.mark.parametrize("k", range(len(GRAD_OPSETS)))
def test_gradient_code_has_no_transcendental_forwarding_hazard(k):
    b_ops, u_ops = GRAD_OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    flat = srhip.flatten(srhip.random_population(300, o, 7, np.float32, seed=31 + k), o, dtype=np.float32)
    _, text, offs = jit_compile(flat, grad=True)
    assert offs
    assert trans_forwarding_hazards("v_rcp_f32_e32 v1, v2\nv_mul_f32_e32 v3, v4, v1") != []  # the check itself
    bad = trans_forwarding_hazards(text)
    assert not bad, bad[:3]


@pytest.mark.parametrize("k", range(len(OPSETS)))
def test_loss_code_has_no_transcendental_forwarding_hazard(k):
    b_ops, u_ops = OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    flat = srhip.flatten(srhip.random_population(300, o, 7, np.float32, seed=41 + k), o, dtype=np.float32)
    for fast, memc in ((True, False), (False, False), (True, True)):
        _, text, _ = jit_compile(flat, fast=fast, memc=memc)
        bad = trans_forwarding_hazards(text)
        assert not bad, bad[:3]


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
def test_gradient_shared_subtree_columns_equal_llvm_mc():
    """Config #5-like gradient programs read their shared constant-free
    subtrees (cos(x_f), exp(x_f), ...) from columns (jit.h kGradGbase): the
    code holds the global loads, its bytes are llvm-mc's, and as many trees
    compile as without columns (a tree whose columns exhaust the register
    pool falls back to its own code)."""
    import os
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(1000, o, 20, np.float32, seed=5)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    code, text, offs = jit_compile(flat, grad=True)
    assert text.count("global_load_dwordx4") > 300 and "s_waitcnt vmcnt(0)" in text
    assert assemble(text) == code
    os.environ["SRHIP_GJIT_GCOLS"] = "0"
    try:
        code0, text0, offs0 = jit_compile(flat, grad=True)
    finally:
        del os.environ["SRHIP_GJIT_GCOLS"]
    assert "global_load_dwordx4" not in text0
    assert len(offs) == len(offs0)
    calls, calls0 = text.count("s_swappc_b64"), text0.count("s_swappc_b64")
    print(f"routine calls {calls} with columns, {calls0} without")
    assert calls < 0.9 * calls0


def test_gradient_code_covers_config5_trees():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(2000, o, 20, np.float32, seed=5)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    code, _, offs = jit_compile(flat, grad=True)
    assert len(offs) >= 0.97 * len(trees), f"{len(offs)} of {len(trees)}"
    print(f"{len(offs)} of {len(trees)} trees, {len(code) / len(offs):.0f} bytes per tree")


LOSS_CASES = [srhip.L1DistLoss(), srhip.HuberLoss(0.7), srhip.L1EpsilonInsLoss(0.3), srhip.L2EpsilonInsLoss(0.25),
              srhip.QuantileLoss(0.8)]


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("loss", LOSS_CASES + [srhip.PeriodicLoss(2.0)], ids=lambda l: f"kind{l.kind}")
def test_float64_gradient_loss_seeds_equal_llvm_mc(loss):
    """The Float64 gradient tree code seeded by another loss's ℓ and dℓ/dr
    routines (jit64.cpp GradGen64::emit_loss_seed): machine code = llvm-mc's."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "cos", "exp"])
    flat = srhip.flatten(srhip.random_population(100, o, 5, np.float64, seed=61), o, dtype=np.float64)
    code, text, offs = jit_compile(flat, grad=True, loss=loss)
    assert len(offs) >= 95
    assert assemble(text) == code


@pytest.mark.parametrize("loss", LOSS_CASES, ids=lambda l: f"kind{l.kind}")
def test_loss_tails_equal_llvm_mc(loss):
    """Tree code of the non-L2 elementwise losses: the loss tree code's tile
    tail (FAST and PRECISE) and the gradient tree code's seed w·ℓ'(r) call the
    loss's routines with its Float64 parameter in s_k:s_kh; same byte check."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(120, o, 5, np.float32, seed=31 + loss.kind)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    bits = int(np.float64(loss.param).view(np.uint64))
    for grad, fast in ((False, True), (False, False), (True, False)):
        code, text, offs = jit_compile(flat, fast=fast, grad=grad, loss=loss)
        assert len(offs) >= 0.9 * len(trees), f"grad={grad}: only {len(offs)} of {len(trees)} trees compiled"
        assert f"s_mov_b32 s90, {hex(bits >> 32)}" in text or (bits >> 32) == 0
        ref = assemble(text)
        assert ref == code, f"grad={grad} fast={fast}: machine code differs from llvm-mc"
        if grad:  # two routine calls per tile beyond the L2 code's: ℓ and ℓ'
            _, l2text, _ = jit_compile(flat, fast=fast, grad=True)
            assert text.count("s_swappc_b64") == l2text.count("s_swappc_b64") + 2 * len(offs)


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
def test_every_loss_has_gradient_tree_code():
    """Since round 6 every elementwise loss has gradient routines in both
    dtypes (Float32 Periodic: g_periodic / d_periodic; Float64 LP: d_lp with
    only the pow's temporaries live): the Float64 LP gradient code compiles
    and equals llvm-mc's bytes."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "cos", "exp"])
    flat64 = srhip.flatten(srhip.random_population(100, o, 5, np.float64, seed=61), o, dtype=np.float64)
    code, text, offs = jit_compile(flat64, grad=True, loss=srhip.LPDistLoss(2.5))
    assert len(offs) >= 95
    assert assemble(text) == code


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
def test_float32_periodic_gradient_code_equals_llvm_mc():
    """Float32 PeriodicLoss gradient tree code (round 6): the seed calls
    g_periodic (ℓ without the loss code's hand-back) and d_periodic (ℓ' =
    k·sin(r·k), device_ops.h periodic_g_f32); machine code = llvm-mc's."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    flat = srhip.flatten(srhip.random_population(120, o, 5, np.float32, seed=33), o, dtype=np.float32)
    code, text, offs = jit_compile(flat, grad=True, loss=srhip.PeriodicLoss(2.0))
    assert len(offs) >= 0.9 * 120
    assert assemble(text) == code


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("memc", [False, True])
def test_output_code_equals_llvm_mc(memc):
    """The per-row output tree code of srhip_eval_tree_array (Options::out):
    PRECISE only, no y load, one global_store_dwordx4 of the root block per
    tile, no early exit; same byte check."""
    b_ops, u_ops = OPSETS[1]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(200, o, 6, np.float32, seed=41)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    code, text, offs = jit_compile(flat, fast=False, memc=memc, out=True)
    assert len(offs) >= 0.7 * len(trees)
    assert text.count("global_store_dwordx4") == len(offs)
    assert "s_cmp_lg_u32 s83" not in text  # no FAST verdict
    assert assemble(text) == code


F64_OPSETS = [
    (["+", "-", "*", "/", "^"], ["safe_log", "safe_sqrt", "cos", "exp"]),  # config #3
    (["+", "-", "*", "/", "max", "min"], ["neg", "abs", "square", "cube", "sin", "tanh", "relu"]),
]


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("k", range(len(F64_OPSETS)))
def test_float64_tree_code_equals_llvm_mc(k):
    """The Float64 tree compiler (csrc/jit64.cpp): same byte check; the
    shallow trees of config #3's operator set compile."""
    b_ops, u_ops = F64_OPSETS[k]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(300, o, 5, np.float64, seed=51 + k)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    code, text, offs = jit_compile(flat)
    assert len(offs) >= 0.6 * len(trees), f"only {len(offs)} of {len(trees)} trees compiled"
    assert "v_add_f64" in text or "v_mul_f64" in text
    assert assemble(text) == code


@pytest.mark.skipif(not (LLVM / "llvm-mc").exists(), reason="llvm-mc not installed")
@pytest.mark.parametrize("what", ["out", "L1", "HUBER", "LP", "PERIODIC", "QUANTILE"])
def test_float64_output_and_loss_tree_code_equals_llvm_mc(what):
    """The Float64 tree compiler's per-row output code (the root block stored
    per tile) and its tile tails for the other losses (a loss routine of the
    Float64 interpreter's elem_loss): same byte check, and every shallow tree
    of config #3's operator set still compiles."""
    b_ops, u_ops = F64_OPSETS[0]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    trees = srhip.random_population(200, o, 5, np.float64, seed=71)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    _, _, base = jit_compile(flat)
    if what == "out":
        code, text, offs = jit_compile(flat, out=True)
        assert "global_store_dwordx4" in text
    else:
        loss = srhip.SupervisedLoss(srhip.constants.LOSS[what], 2.5 if what in ("LP", "PERIODIC") else 0.7)
        code, text, offs = jit_compile(flat, loss=loss)
        assert "s_swappc_b64" in text
    assert set(offs) == set(base)
    assert assemble(text) == code
