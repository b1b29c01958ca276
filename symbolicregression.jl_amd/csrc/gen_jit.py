#!/usr/bin/env python3
"""Generate the operator routines of the tree compiler (jit.cpp) for gfx950.

The tree compiler turns every tree of a large batch into straight-line CDNA4
machine code (one code block per tree, values in VGPRs, no dispatch). Cheap
operators (+ - * neg abs square cube) are emitted inline by jit.cpp; every
other operator is a *routine* called with s_swappc_b64: operands in the fixed
VGPR blocks A and B (R rows each), result in A, non-finite marker in CHK.

Routine bodies are not hand-written: each is compiled by hipcc from the same
C++ operator code as the interpreters (device_ops.h: bop / uop / mark /
fast_sincos_f32) inside a tiny kernel whose state is pinned to fixed registers
with inline-asm constraints, and cut out of the compiler's assembly (the
machinery of gen_asm_interp.py). Results are therefore bit-identical to the
interpreters' for the same transcendental build.

Two regions are emitted with the same layout, routine k at the same offset in
both: FAST (exp / sin / cos in Float32, SR_PRECISE_TRANSC=0) and PRECISE
(Float64-evaluated, the default build). A tree switches region by adding a
constant to the call target (s_mdelta), which is how a tile is redone
precisely when a fast-mode guard fires (jit.cpp).

Outputs (argv[2] = output directory):
  jit_routines_r<R>.inc  SR_JIT_ROUTINES_TEXT: asm of the routines kernel
  jit_layout_r<R>.h      register map, routine table, call clobbers
Usage: gen_jit.py <hipcc> <outdir> [R]
"""
import os
import re
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_asm_interp as G  # noqa: E402

UOPS, BOPS = G.UOPS, G.BOPS
LOSSY_UOPS, LOSSY_LHS, LOSSY_RHS = G.LOSSY_UOPS, G.LOSSY_LHS, G.LOSSY_RHS


class JitRegs:
    """Fixed registers of tree code (jit.cpp mirrors these through jit_layout.h)."""

    def __init__(self, R):
        self.R = R
        assert R == 4, "the tree compiler is laid out for 4 rows per lane"
        self.A, self.B, self.CHK = 32, 36, 40
        self.LANE, self.LSUM, self.LANE4, self.CHKSAVE = 41, 42, 43, 44
        self.GCAN, self.GMIN, self.GEXP = 45, 46, 47
        self.GT, self.Y = 48, 52  # guard temp block, y / loss block
        self.POOL0, self.NPOOL = 56, 8  # value blocks v56..v87
        self.GTRIG = self.POOL0 + self.NPOOL * R  # guard: max |x| of sin / cos of a FAST-derived value
        self.VEND = self.GTRIG + 1  # first register above tree-code state
        # SGPR state of tree code (pinned in the routine snippets so that no
        # routine uses them as temporaries)
        self.S = dict(tile=64, nt=65, partial=66, tilebytes=67, woff=68, status=69, flag=70, rr=72, tgt=74,
                      rt=76, mdelta=78, fastok=79, eps=80, k=81, pe=82, mode=83, x0=84, x1=85, x2=86, x3=87,
                      kh=90)  # kh: high word of a loss routine's Float64 parameter (low word in k)
        self.SPAIRS = {"flag", "rr", "tgt", "rt"}

    def vstate(self):
        g = [("a", self.A, self.R), ("b", self.B, self.R), ("chk", self.CHK, 1)]
        # everything else of tree-code state, pinned as one list
        rest = list(range(self.CHK + 1, self.VEND))
        return g, rest

    def sregs(self):
        out = []
        for n, r in self.S.items():
            out.append((n, r))
            if n in self.SPAIRS:
                out.append((n + "_hi", r + 1))
        return out


# Routine temporaries: s0..s22 and v0..v29. s23 is the prefetching tree
# loop's next code offset (jit_template.hip SR_JIT_LOOP_PF_TEXT), v30 / v31
# the loop's LDS tile / counter addresses: all live across every call.
ROUTINE_S_END, ROUTINE_V_END = 23, 30
# SGPRs held live across a loss routine besides tree-code state: s23, the
# memory constants (s24..s39), the hand-written loop's state (s40..s63) and
# the registers above the state, so that its temporaries stay in s0..s22
LOSS_PINNED_S = list(range(23, 64)) + [88, 89] + list(range(91, 102))


def sgpr_pinned(name):
    """Routines compiled with LOSS_PINNED_S held live: the losses, and the
    Float64 pow and logs of PRECISE Float32 ^ and log10 (SGPR temporaries would otherwise
    reach s23+)."""
    return name.startswith(("l_", "d_", "g_", "b_pow", "u_log", "u_sin_pd", "u_cos_pd"))


def snippet_source(rg, routines):
    R = rg.R
    _, rest = rg.vstate()
    out = ["#define SRHIP_INLINE_ALL 1", '#include "interp.h"', "using namespace srhip; using namespace srhip::interp;",
           "namespace {", "struct St {", f"  float a[{R}]; float b[{R}]; float chk;", f"  unsigned v[{len(rest)}];"]
    for n, _ in rg.sregs():
        out.append(f"  unsigned s_{n};")
    out.append("};")

    def pins(kind):
        lines = []
        regs = [(f"a[{i}]", rg.A + i) for i in range(R)] + [(f"b[{i}]", rg.B + i) for i in range(R)]
        regs += [("chk", rg.CHK)] + [(f"v[{i}]", r) for i, r in enumerate(rest)]
        for i in range(0, len(regs), 8):
            ch = regs[i:i + 8]
            if kind == "in":
                lines.append('  asm volatile("; IN ' + " ".join(f"v{r}" for _, r in ch) + '" : ' +
                             ", ".join(f'"={{v{r}}}"(s.{e})' for e, r in ch) + ");")
            else:
                lines.append('  asm volatile("; OUT" :: ' + ", ".join(f'"{{v{r}}}"(s.{e})' for e, r in ch) + ");")
        ss = rg.sregs()
        for i in range(0, len(ss), 8):
            ch = ss[i:i + 8]
            if kind == "in":
                lines.append('  asm volatile("; IN ' + " ".join(f"s{r}" for _, r in ch) + '" : ' +
                             ", ".join(f'"={{s{r}}}"(s.s_{n})' for n, r in ch) + ");")
            else:
                lines.append('  asm volatile("; OUT" :: ' + ", ".join(f'"{{s{r}}}"(s.s_{n})' for n, r in ch) + ");")
        return lines

    for name, body in routines:
        out.append(f'extern "C" __global__ void __launch_bounds__(64) sr_h_{name}() {{')
        out.append("  St s;")
        out += pins("in")
        if sgpr_pinned(name):
            # a loss routine runs inside the hand-written tree loop (its state
            # in s40..s57) and between the tiles of memory-constant code (its
            # constants in s24..s39): LOSS_PINNED_S are held live across it, so
            # the compiler keeps its temporaries in s0..s22
            zs = LOSS_PINNED_S
            out.append(f"  unsigned zz[{len(zs)}];")
            for i in range(0, len(zs), 8):
                out.append('  asm volatile("; IN ' + " ".join(f"s{zs[j]}" for j in range(i, min(i + 8, len(zs)))) +
                           '" : ' + ", ".join(f'"={{s{zs[j]}}}"(zz[{j}])'
                                                                for j in range(i, min(i + 8, len(zs)))) + ");")
            out.append("  __builtin_amdgcn_sched_barrier(0);")  # nothing scheduled ahead of the pins
        out.append("  float& chk = s.chk; (void)chk;")
        out.append(f"  constexpr int R = {R}; (void)R;")
        out.append("  " + body)
        out += pins("out")
        if sgpr_pinned(name):
            zs = LOSS_PINNED_S
            for i in range(0, len(zs), 8):
                out.append('  asm volatile("; OUT" :: ' + ", ".join(f'"{{s{zs[j]}}}"(zz[{j}])'
                                                                 for j in range(i, min(i + 8, len(zs)))) + ");")
        out.append("}")
    out.append("}  // namespace")
    return "\n".join(out) + "\n"


def rows(expr):
    return f"_Pragma(\"unroll\") for (int r = 0; r < R; ++r) {{ {expr} }}"


def rows_serial(expr):
    """The R rows one after the other, the scheduler fenced between them: the
    registers of one row's evaluation at a time (the Float64 pow / cos of the
    parametric losses do not fit the routine temporaries four rows at once)."""
    return " ".join("{ constexpr int r = %d; %s } __builtin_amdgcn_sched_barrier(0);" % (r, expr) for r in range(4))


# sin / cos routines that hand arguments beyond the fast reduction back to the
# caller (the tree is then re-evaluated by the interpreter) instead of doing
# the large-argument reduction themselves.
TRIG_BAIL = False

# Operators emitted inline by jit.cpp (no routine).
INLINE_BOPS = {"ADD", "SUB", "MUL"}
INLINE_UOPS = {"NEG", "ABS", "SQUARE", "CUBE"}


def losses():
    """SRHIP_LOSS_* of include/srhip.h: {name: id}."""
    txt = open(G.INCLUDE).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define SRHIP_LOSS_(\w+)\s+(\d+)", txt)}


LOSSES = losses()
# no loss routine: L2 is inline (LPDistLoss{n} with an integer n has one: its
# power-by-squaring loop runs over the wave-uniform n in SGPRs)
NO_LOSS_ROUTINE = {"L2"}


def routine_list():
    """(name, body, trig) of every routine: one per operator not emitted inline,
    and one per elementwise loss but L2 (r in A -> ℓ(r) in A, the parameter in
    s_k: device_ops.h elem_loss with ŷ = r, y = 0, so r - 0 = r exactly)."""
    rs = []
    for u in sorted(UOPS, key=lambda k: UOPS[k]):
        if u in INLINE_UOPS:
            continue
        if u in ("SIN", "COS") and TRIG_BAIL:
            body = ("float qm = 0.0f; " +
                    rows(f"float qa; s.a[r] = dev::fast_sincos_f32(s.a[r], {1 if u == 'COS' else 0}, qa); "
                         "qm = __builtin_fmaxf(qm, qa);") +
                    " const unsigned long long fl = __builtin_amdgcn_ballot_w64(!(qm <= dev::kTrigQMax));"
                    " s.s_flag = (unsigned)fl; s.s_flag_hi = (unsigned)(fl >> 32);")
            rs.append((f"u_{u.lower()}", body, True))
        elif u in ("SIN", "COS"):  # the whole range: one ballot for the rows, then big_sincos_f32
            wc = 1 if u == "COS" else 0
            body = (f"float v[R]; float qmax = 0.0f; "
                    f"for (int r = 0; r < R; ++r) {{ float qa; v[r] = dev::fast_sincos_f32(s.a[r], {wc}, qa); "
                    f"qmax = __builtin_fmaxf(qmax, qa); }} "
                    f"if (__builtin_amdgcn_ballot_w64(!(qmax <= dev::kTrigQMax)) != 0) {{ "
                    # one row at a time: the full reduction's registers are not multiplied by R
                    f"for (int r = 0; r < R; ++r) if (__builtin_amdgcn_ballot_w64(dev::trig_big(s.a[r])) != 0) {{ "
                    f"const float o = dev::big_sincos_f32(s.a[r], {wc}); v[r] = dev::trig_big(s.a[r]) ? o : v[r]; }} }} "
                    f"for (int r = 0; r < R; ++r) s.a[r] = v[r];")
            rs.append((f"u_{u.lower()}", body, False))
            # the complete routine under another name: the hand-scheduled FAST
            # body (manual_trig) branches to it when an argument needs more
            # than the fast reduction
            rs.append((f"u_{u.lower()}_full", body, False))
        else:
            mk = "chk = mark(s.a[r], chk); " if u in LOSSY_UOPS else ""
            rs.append((f"u_{u.lower()}", rows(f"{mk}s.a[r] = dev::uop<SRHIP_UOP_{u}>(s.a[r]);"), False))
            if u == "EXP":  # the compiled body beside the hand-scheduled one (tests: SRHIP_JIT_MANUAL=0)
                rs.append(("u_exp_full", rows(f"{mk}s.a[r] = dev::uop<SRHIP_UOP_{u}>(s.a[r]);"), False))
    # the gradient tree code's forward sin / cos (jit_grad.cpp): the value in A
    # (u_sin / u_cos's, bit for bit) and the reverse pass's factor in B — cos x
    # for sin, sin x for cos (device_ops.h sincos_pd_f32) — so that the
    # reverse pass multiplies instead of calling the other routine
    if not TRIG_BAIL:
        for u in ("SIN", "COS"):
            wc = 1 if u == "COS" else 0
            body = (f"float v[R]; float dv[R]; float qmax = 0.0f; "
                    f"for (int r = 0; r < R; ++r) {{ float qa; v[r] = dev::sincos_pd_f32(s.a[r], {wc}, dv[r], qa); "
                    f"qmax = __builtin_fmaxf(qmax, qa); }} "
                    f"if (__builtin_amdgcn_ballot_w64(!(qmax <= dev::kTrigQMax)) != 0) {{ "
                    f"for (int r = 0; r < R; ++r) if (__builtin_amdgcn_ballot_w64(dev::trig_big(s.a[r])) != 0) {{ "
                    f"const bool bg = dev::trig_big(s.a[r]); const float o = dev::big_sincos_f32(s.a[r], {wc}); "
                    f"v[r] = bg ? o : v[r]; const float od = dev::big_sincos_f32(s.a[r], {1 - wc}); "
                    f"dv[r] = bg ? od : dv[r]; }} }} "
                    f"for (int r = 0; r < R; ++r) {{ s.a[r] = v[r]; s.b[r] = dv[r]; }}")
            rs.append((f"u_{u.lower()}_pd", body, False))
    for b in sorted(BOPS, key=lambda k: BOPS[k]):
        if b in INLINE_BOPS:
            continue
        mk = ("chk = mark(s.a[r], chk); " if b in LOSSY_LHS else "") + \
             ("chk = mark(s.b[r], chk); " if b in LOSSY_RHS else "")
        # Float64 pow (PRECISE Float32 ^) does not fit the temporaries four rows at once
        rw = rows_serial if b == "POW" else rows
        rs.append((f"b_{b.lower()}", rw(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(s.a[r], s.b[r]);"), False))
        if b == "DIV":  # the compiled IEEE division, where manual_div sends rows out of its range
            rs.append(("b_div_full", rows(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(s.a[r], s.b[r]);"), False))
    # constant-operand variants: the constant in SGPR s_k (no VGPR moves of a
    # literal); the constant itself was checked at compile time, not marked
    for b in sorted(BOPS, key=lambda k: BOPS[k]):
        if b in INLINE_BOPS:
            continue
        imm = "const float imm = __int_as_float((int)s.s_k); "
        mk = "chk = mark(s.a[r], chk); " if b in LOSSY_LHS else ""
        rw = rows_serial if b == "POW" else rows
        rs.append((f"b_{b.lower()}_rc", imm + rw(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(s.a[r], imm);"), False))
        mk = "chk = mark(s.a[r], chk); " if b in LOSSY_RHS else ""
        rs.append((f"b_{b.lower()}_lc", imm + rw(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(imm, s.a[r]);"), False))
        if b == "DIV":
            rs.append(("b_div_lc_full", imm + rows(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(imm, s.a[r]);"), False))
    for name in sorted(LOSSES, key=lambda k: LOSSES[k]):
        if name in NO_LOSS_ROUTINE:
            continue
        imm = ("const double imm = __builtin_bit_cast(double, ((unsigned long long)s.s_kh << 32) | "
               "(unsigned long long)s.s_k); ")
        if name == "PERIODIC":  # Cody-Waite cos; a row beyond it hands the tile back (the bail flag)
            body = (imm + "bool big = false; " +
                    rows_serial("bool b; const double x = (double)s.a[r] * (6.28318530717958647692 / imm); "
                                "const double c = dev::cw_cos(x, b); big = big || b; s.a[r] = (float)(1.0 - c);") +
                    " const unsigned long long fl = __builtin_amdgcn_ballot_w64(big);"
                    " s.s_flag = (unsigned)fl; s.s_flag_hi = (unsigned)(fl >> 32);")
            rs.append((f"l_{name.lower()}", body, True))
            continue
        rs.append((f"l_{name.lower()}",
                   imm + rows_serial(f"s.a[r] = dev::elem_loss<float>(SRHIP_LOSS_{name}, imm, s.a[r], 0.0f);"),
                   False))
    # dℓ/dr of the same losses (the gradient tree code's seed, jit_grad.cpp)
    for name in sorted(LOSSES, key=lambda k: LOSSES[k]):
        if name in NO_LOSS_ROUTINE:
            continue
        imm = ("const double imm = __builtin_bit_cast(double, ((unsigned long long)s.s_kh << 32) | "
               "(unsigned long long)s.s_k); ")
        if name == "PERIODIC":  # no OCML sin (its registers): device_ops.h periodic_g_f32
            rs.append(("d_periodic", imm + rows_serial(
                "s.a[r] = (float)dev::periodic_g_f32((double)s.a[r], imm, true);"), False))
            # and the gradient code's ℓ without the loss code's hand-back
            rs.append(("g_periodic", imm + rows_serial(
                "s.a[r] = (float)dev::periodic_g_f32((double)s.a[r], imm, false);"), False))
            continue
        rs.append((f"d_{name.lower()}",
                   imm + rows_serial(f"s.a[r] = dev::elem_dloss<float>(SRHIP_LOSS_{name}, imm, s.a[r], 0.0f);"),
                   False))
    return rs


def manual_trig(kind):
    """FAST sin / cos for the 4 rows of A, hand-scheduled: the same operations
    (bit for bit) as hipcc's code for dev::fast_sincos_f32 — reduction by pi
    (three-part pi/2), odd polynomial, sign from the parity of n — with the
    two row pairs interleaved on packed f32 instructions, n rounded with the
    1.5*2^23 shift (its low mantissa bit is n's parity) and no s_nop. Any
    |t| > kTrigQMax (before rounding: a superset of the rows the full
    routine treats specially) branches to the full routine, which starts
    over from A (untouched until the last instructions)."""
    cos = kind == "cos"
    L = ["s_mov_b32 s0, 0x3ea2f983", "s_mov_b32 s20, 0x4702dc00"]  # 1/pi, kTrigQMax = 33500
    if cos:  # t = x/pi - 1/2
        L += ["v_pk_fma_f32 v[0:1], v[32:33], s[0:1], -0.5 op_sel_hi:[1,0,0]",
              "v_pk_fma_f32 v[2:3], v[34:35], s[0:1], -0.5 op_sel_hi:[1,0,0]"]
    else:    # t = x/pi
        L += ["v_pk_mul_f32 v[0:1], v[32:33], s[0:1] op_sel_hi:[1,0]",
              "v_pk_mul_f32 v[2:3], v[34:35], s[0:1] op_sel_hi:[1,0]"]
    L += ["s_mov_b32 s2, 0x4b400000",                       # 1.5 * 2^23
          "v_max3_f32 v24, |v0|, |v1|, |v2|",
          "v_max_f32_e64 v24, v24, |v3|",
          "v_cmp_lt_f32_e32 vcc, s20, v24",
          "s_mov_b32 s4, 0xcb400000",
          "v_pk_add_f32 v[4:5], v[0:1], s[2:3] op_sel_hi:[1,0]",   # t + 1.5*2^23: n in the low bits
          "v_pk_add_f32 v[6:7], v[2:3], s[2:3] op_sel_hi:[1,0]",
          "s_cbranch_vccnz @FULL@",
          "v_pk_add_f32 v[8:9], v[4:5], s[4:5] op_sel_hi:[1,0]",   # n = rint(t)
          "v_pk_add_f32 v[10:11], v[6:7], s[4:5] op_sel_hi:[1,0]",
          "s_mov_b32 s6, 0xbfc90fd8"]
    if cos:  # m = 2n + 1
        L += ["v_pk_fma_f32 v[8:9], v[8:9], 2.0, 1.0 op_sel_hi:[1,0,0]",
              "v_pk_fma_f32 v[10:11], v[10:11], 2.0, 1.0 op_sel_hi:[1,0,0]"]
    else:    # m = 2n
        L += ["v_pk_add_f32 v[8:9], v[8:9], v[8:9]",
              "v_pk_add_f32 v[10:11], v[10:11], v[10:11]"]
    L += ["s_mov_b32 s8, 0xb4a8885a",
          "v_pk_fma_f32 v[12:13], v[8:9], s[6:7], v[32:33] op_sel_hi:[1,0,1]",   # r = x - m*pi/2 (3 parts)
          "v_pk_fma_f32 v[14:15], v[10:11], s[6:7], v[34:35] op_sel_hi:[1,0,1]",
          "s_mov_b32 s10, 0xa7c234c4",
          "v_pk_fma_f32 v[12:13], v[8:9], s[8:9], v[12:13] op_sel_hi:[1,0,1]",
          "v_pk_fma_f32 v[14:15], v[10:11], s[8:9], v[14:15] op_sel_hi:[1,0,1]",
          "s_mov_b32 s12, 0x362ee8a0",
          "v_pk_fma_f32 v[12:13], v[8:9], s[10:11], v[12:13] op_sel_hi:[1,0,1]",
          "v_pk_fma_f32 v[14:15], v[10:11], s[10:11], v[14:15] op_sel_hi:[1,0,1]",
          "v_mov_b32_e32 v28, 0xb94fb8ba",
          "v_pk_mul_f32 v[16:17], v[12:13], v[12:13]",                          # s = r^2
          "v_pk_mul_f32 v[18:19], v[14:15], v[14:15]",
          "s_mov_b32 s16, 0x3c08876e",
          "v_pk_fma_f32 v[20:21], v[16:17], s[12:13], v[28:29] op_sel_hi:[1,0,0]",
          "v_pk_fma_f32 v[22:23], v[18:19], s[12:13], v[28:29] op_sel_hi:[1,0,0]",
          "s_mov_b32 s18, 0xbe2aaaa6",
          "v_pk_fma_f32 v[20:21], v[20:21], v[16:17], s[16:17] op_sel_hi:[1,1,0]",
          "v_pk_fma_f32 v[22:23], v[22:23], v[18:19], s[16:17] op_sel_hi:[1,1,0]",
          "v_pk_fma_f32 v[20:21], v[20:21], v[16:17], s[18:19] op_sel_hi:[1,1,0]",
          "v_pk_fma_f32 v[22:23], v[22:23], v[18:19], s[18:19] op_sel_hi:[1,1,0]",
          "v_pk_mul_f32 v[20:21], v[16:17], v[20:21]",
          "v_pk_mul_f32 v[22:23], v[18:19], v[22:23]"]
    neg = " neg_lo:[0,1,1] neg_hi:[0,1,1]" if cos else ""
    # the sign (-1)^n: n's parity (low bit of t + 1.5*2^23) shifted to bit 31
    # and added, which flips the sign bit exactly as a xor would
    L += [f"v_pk_fma_f32 v[20:21], v[20:21], v[12:13], v[12:13]{neg}",
          f"v_pk_fma_f32 v[22:23], v[22:23], v[14:15], v[14:15]{neg}",
          "v_lshl_add_u32 v32, v4, 31, v20",
          "v_lshl_add_u32 v33, v5, 31, v21",
          "v_lshl_add_u32 v34, v6, 31, v22",
          "v_lshl_add_u32 v35, v7, 31, v23"]
    return L


def manual_div_rk(rg):
    """a / c for a constant divisor c (s_k) through its correctly rounded
    reciprocal y = RN(1/c) (s_x1, computed by the host): q = a*y,
    r = fma(-c, q, a), q' = fma(r, y, q) — the IEEE quotient whenever |a| and
    |c| lie in [2^-60, 2^60] (tools/check_div_const.c: 1.7e10 quotients, no
    mismatch; the host only uses this routine for such c). A row outside
    that range (0, Inf, NaN, extreme exponents) sends all four to the IEEE
    routine b_div_rc."""
    k, y = rg.S["k"], rg.S["x1"]
    return ["v_max3_f32 v0, |v32|, |v33|, |v34|",
            "v_min3_f32 v1, |v32|, |v33|, |v34|",
            "s_mov_b32 s0, 0x5d800000",           # 2^60
            "v_max_f32_e64 v0, v0, |v35|",
            "v_min_f32_e64 v1, v1, |v35|",
            "s_mov_b32 s1, 0x21800000",           # 2^-60
            "v_cmp_gt_f32_e64 s[2:3], s0, v0",
            "v_cmp_lt_f32_e64 s[4:5], s1, v1",
            "s_and_b64 s[2:3], s[2:3], s[4:5]",
            "s_andn2_b64 s[2:3], exec, s[2:3]",
            "s_cbranch_scc1 .Lsrdk_fb_%=",
            f"v_mul_f32_e32 v4, s{y}, v32",
            f"v_mul_f32_e32 v5, s{y}, v33",
            f"v_mul_f32_e32 v6, s{y}, v34",
            f"v_mul_f32_e32 v7, s{y}, v35",
            f"v_fma_f32 v8, -s{k}, v4, v32",
            f"v_fma_f32 v9, -s{k}, v5, v33",
            f"v_fma_f32 v10, -s{k}, v6, v34",
            f"v_fma_f32 v11, -s{k}, v7, v35",
            f"v_fma_f32 v32, v8, s{y}, v4",
            f"v_fma_f32 v33, v9, s{y}, v5",
            f"v_fma_f32 v34, v10, s{y}, v6",
            f"v_fma_f32 v35, v11, s{y}, v7",
            f"s_setpc_b64 s[{rg.S['rr']}:{rg.S['rr'] + 1}]",
            ".Lsrdk_fb_%=:",
            "s_branch @DIVRC@"]


def manual_exp():
    """FAST exp for the 4 rows of A, bit for bit hipcc's Float32 exp
    (SR_PRECISE_TRANSC=0: clamp to [-104, 89], n = rint(c*log2e),
    f = fma(c, log2e, -n) + c*log2e_lo, ldexp(v_exp_f32(f), n)) on every tile
    the FAST path keeps. Tree code runs this body only under its exp guard
    (jit.cpp: a tile with some |x| > 87, or a non-finite x, which the input
    mark catches, is redone with the PRECISE routines), so for a kept tile
    |x| <= 87: the clamp is the identity, rint(t) is (t + 1.5*2^23) - 1.5*2^23
    (round to nearest even, |t| < 2^22), and 2^f * 2^n is a normal number,
    i.e. its bits are those of 2^f plus n << 23 — the low bits of
    t + 1.5*2^23 shifted left by 23. Two rows per v_pk_*_f32 instruction.
    The input is marked (chk) as in the compiled body: (x0, x1)*0 + (x2, x3)
    is finite iff the four rows are. The mark is load-bearing: for an x the
    exp guard rejects this body returns garbage, possibly a signalling NaN;
    a later FAST exp would turn that NaN finite (its payload added by the
    n << 23 step), and v_max3 of an sNaN drops the guard accumulators'
    earlier values (measured: config #2 trees 1000 and 2800 kept such a
    tile), so a non-finite exp input must redo the tile itself."""
    return ["s_mov_b32 s2, 0x3fb8aa3b",            # log2(e)
            "s_mov_b32 s4, 0x4b400000",            # 1.5 * 2^23
            "v_pk_mul_f32 v[0:1], v[32:33], s[2:3] op_sel_hi:[1,0]",   # t = x*log2e
            "v_pk_mul_f32 v[2:3], v[34:35], s[2:3] op_sel_hi:[1,0]",
            "s_mov_b32 s6, 0x32a57060",            # log2(e) - RN32(log2(e))
            "v_pk_add_f32 v[4:5], v[0:1], s[4:5] op_sel_hi:[1,0]",     # s = t + 1.5*2^23: n in the low bits
            "v_pk_add_f32 v[6:7], v[2:3], s[4:5] op_sel_hi:[1,0]",
            "v_pk_add_f32 v[0:1], v[4:5], s[4:5] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]",   # n = rint(t)
            "v_pk_add_f32 v[2:3], v[6:7], s[4:5] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]",
            "v_pk_fma_f32 v[8:9], v[32:33], s[2:3], v[0:1] op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]",
            "v_pk_fma_f32 v[10:11], v[34:35], s[2:3], v[2:3] op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]",
            "v_pk_fma_f32 v[8:9], s[6:7], v[32:33], v[8:9] op_sel_hi:[0,1,1]",
            "v_pk_fma_f32 v[10:11], s[6:7], v[34:35], v[10:11] op_sel_hi:[0,1,1]",
            "v_exp_f32_e32 v8, v8",
            "v_exp_f32_e32 v9, v9",
            "v_exp_f32_e32 v10, v10",
            "v_exp_f32_e32 v11, v11",
            "v_pk_fma_f32 v[12:13], v[32:33], 0, v[34:35] op_sel_hi:[1,0,1]",
            "v_fmac_f32_e32 v40, 0, v12",
            "v_fmac_f32_e32 v40, 0, v13",
            "v_lshl_add_u32 v32, v4, 23, v8",
            "v_lshl_add_u32 v33, v5, 23, v9",
            "v_lshl_add_u32 v34, v6, 23, v10",
            "v_lshl_add_u32 v35, v7, 23, v11"]


def manual_div(rg):
    """a / b (A / B) for the 4 rows: when every |a| and |b| lies in
    [2^-45, 2^45], v_div_scale_f32 leaves both unchanged (no exponent
    difference of 96, no denormal reciprocal or quotient), v_div_fmas_f32 is a
    plain fma and v_div_fixup_f32 returns its input, so hipcc's IEEE sequence
    reduces to rcp, e = 1 - b*r, r += e*r, q = a*r, e = a - b*q, q += e*r,
    e = a - b*q, q += e*r — the same roundings, here two rows per v_pk_*_f32
    instruction. Rows out of the range (0, Inf, extreme exponents) send all
    four to the compiled routine (b_div_full), which marks b; so b needs no
    mark here: an infinite b (whose quotient would lose it) never takes
    this path, and a NaN b gives a NaN quotient."""
    neg0 = " neg_lo:[1,0,0] neg_hi:[1,0,0]"
    return ["v_max3_f32 v0, |v32|, |v33|, |v34|",
            "v_min3_f32 v1, |v32|, |v33|, |v34|",
            "v_max3_f32 v0, v0, |v35|, |v36|",
            "v_min3_f32 v1, v1, |v35|, |v36|",
            "v_max3_f32 v0, v0, |v37|, |v38|",
            "v_min3_f32 v1, v1, |v37|, |v38|",
            "s_mov_b32 s0, 0x56000000",           # 2^45
            "v_max_f32_e64 v0, v0, |v39|",
            "v_min_f32_e64 v1, v1, |v39|",
            "s_mov_b32 s1, 0x29000000",           # 2^-45
            "v_cmp_gt_f32_e64 s[2:3], s0, v0",
            "v_cmp_lt_f32_e64 s[4:5], s1, v1",
            "s_and_b64 s[2:3], s[2:3], s[4:5]",
            "s_andn2_b64 s[2:3], exec, s[2:3]",
            "s_cbranch_scc1 @DIVFULL@",
            "v_rcp_f32_e32 v2, v36",
            "v_rcp_f32_e32 v3, v37",
            "v_rcp_f32_e32 v4, v38",
            "v_rcp_f32_e32 v5, v39",
            "v_pk_fma_f32 v[6:7], v[36:37], v[2:3], 1.0 op_sel_hi:[1,1,0]" + neg0,
            "v_pk_fma_f32 v[8:9], v[38:39], v[4:5], 1.0 op_sel_hi:[1,1,0]" + neg0,
            "v_pk_fma_f32 v[2:3], v[6:7], v[2:3], v[2:3]",
            "v_pk_fma_f32 v[4:5], v[8:9], v[4:5], v[4:5]",
            "v_pk_mul_f32 v[10:11], v[32:33], v[2:3]",
            "v_pk_mul_f32 v[12:13], v[34:35], v[4:5]",
            "v_pk_fma_f32 v[6:7], v[36:37], v[10:11], v[32:33]" + neg0,
            "v_pk_fma_f32 v[8:9], v[38:39], v[12:13], v[34:35]" + neg0,
            "v_pk_fma_f32 v[10:11], v[6:7], v[2:3], v[10:11]",
            "v_pk_fma_f32 v[12:13], v[8:9], v[4:5], v[12:13]",
            "v_pk_fma_f32 v[6:7], v[36:37], v[10:11], v[32:33]" + neg0,
            "v_pk_fma_f32 v[8:9], v[38:39], v[12:13], v[34:35]" + neg0,
            "v_pk_fma_f32 v[32:33], v[6:7], v[2:3], v[10:11]",
            "v_pk_fma_f32 v[34:35], v[8:9], v[4:5], v[12:13]"]


def manual_div_lc(rg):
    """c / a for the constant c in s_k (the odd half of an SGPR pair, so the
    packed instructions pick it with op_sel) and the 4 rows of A: manual_div's
    sequence with c as the numerator, under the same range condition on c and
    every |a|; otherwise the compiled routine (b_div_lc_full), which marks
    a (here unmarked, as b in manual_div)."""
    k = rg.S["k"]
    assert k % 2 == 1
    cp = f"s[{k - 1}:{k}]"
    neg0 = " neg_lo:[1,0,0] neg_hi:[1,0,0]"
    return [f"v_max3_f32 v0, |v32|, |v33|, |s{k}|",
            f"v_min3_f32 v1, |v32|, |v33|, |s{k}|",
            "v_max3_f32 v0, v0, |v34|, |v35|",
            "v_min3_f32 v1, v1, |v34|, |v35|",
            "s_mov_b32 s0, 0x56000000",           # 2^45
            "s_mov_b32 s1, 0x29000000",           # 2^-45
            "v_cmp_gt_f32_e64 s[2:3], s0, v0",
            "v_cmp_lt_f32_e64 s[4:5], s1, v1",
            "s_and_b64 s[2:3], s[2:3], s[4:5]",
            "s_andn2_b64 s[2:3], exec, s[2:3]",
            "s_cbranch_scc1 @LCFULL@",
            "v_rcp_f32_e32 v2, v32",
            "v_rcp_f32_e32 v3, v33",
            "v_rcp_f32_e32 v4, v34",
            "v_rcp_f32_e32 v5, v35",
            "v_pk_fma_f32 v[6:7], v[32:33], v[2:3], 1.0 op_sel_hi:[1,1,0]" + neg0,
            "v_pk_fma_f32 v[8:9], v[34:35], v[4:5], 1.0 op_sel_hi:[1,1,0]" + neg0,
            "v_pk_fma_f32 v[2:3], v[6:7], v[2:3], v[2:3]",
            "v_pk_fma_f32 v[4:5], v[8:9], v[4:5], v[4:5]",
            f"v_pk_mul_f32 v[10:11], {cp}, v[2:3] op_sel:[1,0]",
            f"v_pk_mul_f32 v[12:13], {cp}, v[4:5] op_sel:[1,0]",
            f"v_pk_fma_f32 v[6:7], v[32:33], v[10:11], {cp} op_sel:[0,0,1]" + neg0,
            f"v_pk_fma_f32 v[8:9], v[34:35], v[12:13], {cp} op_sel:[0,0,1]" + neg0,
            "v_pk_fma_f32 v[10:11], v[6:7], v[2:3], v[10:11]",
            "v_pk_fma_f32 v[12:13], v[8:9], v[4:5], v[12:13]",
            f"v_pk_fma_f32 v[6:7], v[32:33], v[10:11], {cp} op_sel:[0,0,1]" + neg0,
            f"v_pk_fma_f32 v[8:9], v[34:35], v[12:13], {cp} op_sel:[0,0,1]" + neg0,
            "v_pk_fma_f32 v[32:33], v[6:7], v[2:3], v[10:11]",
            "v_pk_fma_f32 v[34:35], v[8:9], v[4:5], v[12:13]"]


def compile_bodies(hipcc, rg, routines, extra):
    src = snippet_source(rg, [(n, b) for n, b, _ in routines])
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "routines.hip")
        open(sp, "w").write(src)
        ap = os.path.join(td, "routines.s")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
               "-S", "-I", HERE, sp, "-o", ap] + extra
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            raise SystemExit("gen_jit: routine compile failed")
        asm = open(ap).read()
    bodies = {}
    for n, _, _ in routines:
        try:
            if not G.pins_first(asm, n):  # a pinned register used as a temporary before its pin
                raise SystemExit("code placed ahead of the register pins")
            bodies[n] = G.extract(asm, n)
        except SystemExit as e:  # a body the block cannot hold (memory operands, calls): no routine
            sys.stderr.write(f"gen_jit: routine {n} skipped ({e})\n")
    return bodies


def label_sizes(lines_by_name, order):
    """Assemble every body standalone; return its byte size."""
    T = []
    for n in order:
        T.append(f".Lsr_start_{n}_%=:")
        T += lines_by_name[n]
        T.append(f".Lsr_end_{n}_%=:")
    T.insert(0, ".Lsr_base_%=:")
    offs = G.label_offsets(T)
    return {n: offs[f"end_{n}"] - offs[f"start_{n}"] for n in order}


def build(hipcc, outdir, R):
    rg = JitRegs(R)
    routines = routine_list()
    fast = compile_bodies(hipcc, rg, routines, ["-DSR_PRECISE_TRANSC=0"])
    prec = compile_bodies(hipcc, rg, routines, [])
    names = [n for n, _, _ in routines if n in fast and n in prec]
    manual = set()
    if "b_div_rc" in names:  # hand-written, the same in both regions (IEEE exact)
        fast["b_div_rk"] = prec["b_div_rk"] = manual_div_rk(rg)
        names.insert(names.index("b_div_rc") + 1, "b_div_rk")
    if os.environ.get("SR_JIT_MANUAL_DIV", "1") != "0" and "b_div_full" in names:
        fast["b_div"] = prec["b_div"] = manual_div(rg)  # exact: the same in both regions
        manual.add("b_div")
        if "b_div_lc_full" in names:
            fast["b_div_lc"] = prec["b_div_lc"] = manual_div_lc(rg)
            manual.add("b_div_lc")
    if os.environ.get("SR_JIT_MANUAL_EXP", "1") != "0" and "u_exp" in names:
        fast["u_exp"] = manual_exp()
        manual.add("u_exp")
    if os.environ.get("SR_JIT_MANUAL_TRIG", "1") != "0":
        for k in ("sin", "cos"):
            if f"u_{k}_full" in names:
                fast[f"u_{k}"] = manual_trig(k)
                manual.add(f"u_{k}")
    trig = {n for n, _, t in routines if t}
    vstate = set(range(rg.A, rg.VEND))
    sstate = {r for _, r in rg.sregs()}
    # a loss routine runs between the tiles of memory-constant tree code, whose
    # constants live in s24..s39 (jit.cpp Gen::SC0): one whose SGPR temporaries
    # reach them (logcosh, logitdist: Float64 constants) is left out, and that
    # loss runs interpreted (SR_JIT_LOSS_ROUTINE -1)
    # (and one whose VGPR temporaries run into the state block: LP's Float64 pow)
    # A loss routine is compiled with LOSS_PINNED_S held live (snippet_source):
    # the compiler may still borrow one of them, but saves it to a VGPR lane
    # first and restores it before the routine ends (v_writelane /
    # v_readlane), so those are not temporaries of the routine.
    pinned = set(LOSS_PINNED_S)
    for n in [n for n in names if n.startswith(("l_", "d_", "g_"))]:
        used, vused = set(), set()
        for d in (fast, prec):
            used |= G.regs_used(d[n], G.REG_S) - sstate - pinned
            vused |= G.regs_used(d[n], G.REG_V) - vstate
        if any(r >= ROUTINE_S_END for r in used) or any(r >= ROUTINE_V_END for r in vused):
            sys.stderr.write(f"gen_jit: loss routine {n} left out (SGPR temps {sorted(r for r in used if r >= ROUTINE_S_END)}, "
                             f"VGPR temps up to v{max(vused, default=0)})\n")
            names.remove(n)
    vtemp, stemp = set(), set()
    for d in (fast, prec):
        for n in names:
            vtemp |= G.regs_used(d[n], G.REG_V) - vstate
            stemp |= G.regs_used(d[n], G.REG_S) - sstate - (pinned if sgpr_pinned(n) else set())
    if vtemp & vstate or stemp & sstate:
        raise SystemExit("gen_jit: temp/state overlap")
    if max(vtemp, default=0) >= ROUTINE_V_END:
        over = sorted({n for d in (fast, prec) for n in names
                       if max(G.regs_used(d[n], G.REG_V) - vstate, default=0) >= ROUTINE_V_END})
        raise SystemExit(f"gen_jit: routine VGPR temps reach v{max(vtemp)} (v{ROUTINE_V_END}+ held by the tree loop): {over}")
    if max(stemp, default=0) >= ROUTINE_S_END:
        over = sorted({n for d in (fast, prec) for n in names
                       if max(G.regs_used(d[n], G.REG_S) - sstate - (pinned if sgpr_pinned(n) else set()),
                              default=0) >= ROUTINE_S_END})
        raise SystemExit(f"gen_jit: routine SGPR temps reach s{max(stemp)} (s{ROUTINE_S_END}+ held by the tree loop): {over}")

    def with_ret(lines, n, t):
        body = list(lines)
        while body and body[0].startswith("s_nop"):
            body.pop(0)
        out = [l.replace("%=", f"{t}") for l in body]
        # a trig routine's bail flag is tested by the caller (tree code)
        out.append(f"s_setpc_b64 s[{rg.S['rr']}:{rg.S['rr'] + 1}]")
        return out

    fb = {n: with_ret(fast[n], n, "f") for n in names}
    pb = {n: with_ret(prec[n], n, "p") for n in names}
    def sized(bodies):
        return {n: [l.replace("@FULL@", f".Lsr_start_{n}_full_%=").replace("@DIVRC@", ".Lsr_start_b_div_rc_%=")
                    .replace("@DIVFULL@", ".Lsr_start_b_div_full_%=").replace("@LCFULL@", ".Lsr_start_b_div_lc_full_%=")
                    for l in b] for n, b in bodies.items()}
    fs, ps = label_sizes(sized(fb), names), label_sizes(sized(pb), names)
    fb = {n: [l.replace("@FULL@", f".Lsrent_fast_{n}_full").replace("@DIVRC@", ".Lsrent_fast_b_div_rc")
              .replace("@DIVFULL@", ".Lsrent_fast_b_div_full").replace("@LCFULL@", ".Lsrent_fast_b_div_lc_full")
              for l in b] for n, b in fb.items()}
    pb = {n: [l.replace("@DIVRC@", ".Lsrent_prec_b_div_rc").replace("@DIVFULL@", ".Lsrent_prec_b_div_full")
              .replace("@LCFULL@", ".Lsrent_prec_b_div_lc_full") for l in b] for n, b in pb.items()}
    slot = {n: (max(fs[n], ps[n]) + 63) // 64 * 64 for n in names}
    text = ["s_endpgm"]
    for region, bodies, sizes in (("fast", fb, fs), ("prec", pb, ps)):
        text.append(".p2align 8")
        text.append(f".globl sr_rt_{region}")
        text.append(f"sr_rt_{region}:")
        for n in names:
            text.append(f".globl sr_rt_{region}_{n}")
            text.append(f"sr_rt_{region}_{n}:")
            text.append(f".Lsrent_{region}_{n}:")  # local entry label (branch target)
            text += bodies[n]
            pad = slot[n] - sizes[n]
            assert pad % 4 == 0
            if pad:
                text.append(f".fill {pad // 4}, 4, 0xbf800000")  # s_nop 0
    os.makedirs(outdir, exist_ok=True)
    inc = os.path.join(outdir, f"jit_routines_r{R}.inc")
    with open(inc, "w") as f:
        f.write(f"// Generated by gen_jit.py (R={R}); do not edit.\n#pragma once\n#define SR_JIT_ROUTINES_TEXT \\\n")
        for ln in text:
            f.write('  "' + ln.replace("\\", "\\\\").replace('"', '\\"') + '\\n" \\\n')
        f.write('  ""\n')
    # layout header
    uop_rt = {UOPS[u]: f"u_{u.lower()}" for u in UOPS}
    bop_rt = {BOPS[b]: f"b_{b.lower()}" for b in BOPS}
    hp = os.path.join(outdir, f"jit_layout_r{R}.h")
    clob_v = sorted(vtemp | (vstate - {rg.CHK, rg.LANE, rg.LSUM, rg.LANE4}))
    clob_s = sorted(stemp | (sstate - {rg.S[k] for k in ("tile", "nt", "partial", "tilebytes", "woff", "fastok",
                                                          "status", "x0")}))
    with open(hp, "w") as f:
        f.write(f"// Generated by gen_jit.py (R={R}); do not edit.\n#pragma once\n")
        f.write(f"#define SR_JIT_R {R}\n")
        for k, v in (("A", rg.A), ("B", rg.B), ("CHK", rg.CHK), ("LANE", rg.LANE), ("LSUM", rg.LSUM),
                     ("LANE4", rg.LANE4), ("CHKSAVE", rg.CHKSAVE), ("GCAN", rg.GCAN), ("GMIN", rg.GMIN),
                     ("GEXP", rg.GEXP), ("GTRIG", rg.GTRIG), ("GT", rg.GT), ("Y", rg.Y), ("POOL0", rg.POOL0),
                     ("NPOOL", rg.NPOOL),
                     ("VEND", rg.VEND)):
            f.write(f"#define SR_JIT_V_{k} {v}\n")
        for k, v in rg.S.items():
            f.write(f"#define SR_JIT_S_{k.upper()} {v}\n")
        f.write("// routine of each unary / binary operator (-1: inline or not available)\n")
        def rid(n):
            return names.index(n) if n in names else -1
        f.write("#define SR_JIT_UOP_ROUTINE {" + ", ".join(
            str(-1 if u_name.upper()[2:] in INLINE_UOPS else rid(u_name))
            for _, u_name in sorted(uop_rt.items())) + "}\n")
        f.write("#define SR_JIT_BOP_ROUTINE {" + ", ".join(
            str(-1 if b_name.upper()[2:] in INLINE_BOPS else rid(b_name))
            for _, b_name in sorted(bop_rt.items())) + "}\n")
        for suf in ("rc", "lc"):
            f.write(f"#define SR_JIT_BOP_ROUTINE_{suf.upper()} {{" + ", ".join(
                str(-1 if b_name.upper()[2:] in INLINE_BOPS else rid(f"{b_name}_{suf}"))
                for _, b_name in sorted(bop_rt.items())) + "}\n")
        f.write("// routine of each elementwise loss, by SRHIP_LOSS_* (-1: L2, inline)\n")
        f.write("#define SR_JIT_LOSS_ROUTINE {" + ", ".join(
            str(-1 if n in NO_LOSS_ROUTINE else rid(f"l_{n.lower()}")) for n in sorted(LOSSES, key=lambda k: LOSSES[k])) + "}\n")
        f.write("// ℓ routine of each elementwise loss in the gradient tree code (the loss routine, but\n"
                "// Periodic's without the hand-back)\n")
        f.write("#define SR_JIT_GRAD_LOSS_ROUTINE {" + ", ".join(
            str(-1 if n in NO_LOSS_ROUTINE else rid("g_periodic" if n == "PERIODIC" else f"l_{n.lower()}"))
            for n in sorted(LOSSES, key=lambda k: LOSSES[k])) + "}\n")
        f.write("// dℓ/dr routine of each elementwise loss (-1: L2, inline, or left out)\n")
        f.write("#define SR_JIT_DLOSS_ROUTINE {" + ", ".join(
            str(-1 if n in NO_LOSS_ROUTINE else rid(f"d_{n.lower()}")) for n in sorted(LOSSES, key=lambda k: LOSSES[k])) + "}\n")
        f.write("// the gradient forward's sin / cos with the reverse factor in B (-1: not built)\n")
        f.write(f"#define SR_JIT_SINCOS_PD_ROUTINE {{{rid('u_sin_pd')}, {rid('u_cos_pd')}}}\n")
        f.write(f"#define SR_JIT_NUM_ROUTINES {len(names)}\n")
        f.write("#define SR_JIT_ROUTINE_NAMES {" + ", ".join(f'"{n}"' for n in names) + "}\n")
        f.write("#define SR_JIT_ROUTINE_TRIG {" + ", ".join("1" if n in trig else "0" for n in names) + "}\n")
        # routines whose FAST and PRECISE bodies are the same code (labels aside)
        # and small: tree code may copy them in place of a call (jit.cpp)
        def norm(lines):
            return [re.sub(r"_[fp]\b", "", l) for l in lines]
        inl = [n for n in names if norm(fb[n]) == norm(pb[n]) and fs[n] <= 512 and
               not any(k in l for l in fb[n][:-1] for k in ("s_getpc", "s_setpc", "s_swappc", "s_endpgm"))]
        f.write("#define SR_JIT_ROUTINE_INLINE {" + ", ".join("1" if n in inl else "0" for n in names) + "}\n")
        f.write("#define SR_JIT_ROUTINE_BODY_BYTES {" + ", ".join(str(fs[n] - 4) for n in names) + "}\n")
        f.write("#define SR_JIT_CLOBBERS " + ", ".join([f'"v{r}"' for r in clob_v] + [f'"s{r}"' for r in clob_s]
                                                          + ['"vcc"', '"scc"', '"m0"']) + "\n")
        # memory-constant tree code (jit.cpp Gen::memc): its constants in s24..s39
        f.write("#define SR_JIT_CLOBBERS_MEMC SR_JIT_CLOBBERS, " + ", ".join(f'"s{r}"' for r in range(24, 40)) + "\n")
        # gradient tree code (jit_grad.cpp): the same routines, a larger value
        # pool, per-constant accumulators, constants in SGPRs
        g = dict(GPOOL0=56, GNPOOL=20, GACC=136, NGACC=16, SC0=24, SCPTR=78, SGPTR=84)
        assert g["GPOOL0"] + 4 * g["GNPOOL"] == g["GACC"]
        assert max(stemp) < g["SC0"] and g["SC0"] % 4 == 0
        for k, v in g.items():
            f.write(f"#define SR_JIT_G_{k} {v}\n")
        gin_v = {rg.CHK, rg.LANE, rg.LSUM, rg.LANE4}
        # + one above the accumulators: the FAST forward's sin / cos argument guard (jit_grad.cpp VGTRIG_G)
        gclob_v = sorted((vtemp | set(range(rg.A, g["GACC"] + g["NGACC"] + 1))) - gin_v)
        gin_s = {rg.S[k] for k in ("tile", "nt", "partial", "tilebytes", "woff", "status")} | \
            {g["SCPTR"], g["SCPTR"] + 1, g["SGPTR"], g["SGPTR"] + 1}
        gclob_s = sorted((stemp | sstate | set(range(g["SC0"], g["SC0"] + g["NGACC"]))) - gin_s)
        f.write("#define SR_JIT_GRAD_CLOBBERS " + ", ".join([f'"v{r}"' for r in gclob_v] + [f'"s{r}"' for r in gclob_s]
                                                               + ['"vcc"', '"scc"', '"m0"']) + "\n")
        f.write(f"// routine VGPR temps v{min(vtemp)}..v{max(vtemp)}, SGPR temps {sorted(stemp)}\n")
        f.write("// routine sizes (fast / precise bytes): " +
                ", ".join(f"{n} {fs[n]}/{ps[n]}" for n in names) + "\n")


if __name__ == "__main__":
    hipcc, outdir = sys.argv[1], sys.argv[2]
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    build(hipcc, outdir, R)
