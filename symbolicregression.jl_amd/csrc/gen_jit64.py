#!/usr/bin/env python3
"""Generate the operator routines of the Float64 tree compiler (jit64.cpp).

The Float64 counterpart of gen_jit.py: every tree of a Float64 batch becomes
straight-line gfx950 machine code (jit64.cpp); + - * neg abs square cube are
emitted inline, every other operator is a routine called with s_swappc_b64,
operands in the fixed VGPR blocks A and B (2 rows per lane, one Float64 per
row: v[32:35], v[36:39]), result in A, non-finite marker in CHK (a Float64,
v[40:41]). The bodies are compiled by hipcc from the Float64 operator code of
device_ops.h (dev::uop / dev::bop / mark), the same code as the Float64
interpreter, inside a tiny kernel whose state is pinned to fixed registers,
and cut out of the compiler's assembly (gen_asm_interp.extract). Results are
therefore the interpreter's bit for bit. There is one region (Float64 has no
FAST path). Routines whose compiled code reads memory or calls (the extractor
refuses them) are left out: trees that use those operators stay interpreted.

Outputs (argv[2] = output directory):
  jit64_routines.inc  SR_JIT64_ROUTINES_TEXT: asm of the routines kernel
  jit64_layout.h      register map, routine table, call clobbers
Usage: gen_jit64.py <hipcc> <outdir>
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_asm_interp as G  # noqa: E402

UOPS, BOPS = G.UOPS, G.BOPS
LOSSY_UOPS, LOSSY_LHS, LOSSY_RHS = G.LOSSY_UOPS, G.LOSSY_LHS, G.LOSSY_RHS
LOSSES = {m.group(1): int(m.group(2)) for m in
          re.finditer(r"#define SRHIP_LOSS_(\w+)\s+(\d+)", open(G.INCLUDE).read())}
NO_LOSS_ROUTINE = {"L2"}  # L2 inline
INLINE_BOPS = {"ADD", "SUB", "MUL"}
INLINE_UOPS = {"NEG", "ABS", "SQUARE", "CUBE"}


class Regs64:
    """Fixed registers of Float64 tree code (jit64.cpp mirrors these through
    jit64_layout.h). R = 2 rows per lane: a 128-row tile is 1 KiB per column,
    the byte layout of the Float32 tree code's 256-row tiles."""
    R = 2
    A, B, CHK = 32, 36, 40        # double a[2], b[2]; double chk (v[40:41])
    LANE, LANE2, LSUM = 42, 43, 44  # LDS lane address; 2·lane (row in tile); double lsum (v[44:45])
    GT, Y = 48, 52                # temp block, y / residual block
    POOL0, NPOOL = 56, 8          # value blocks v56..v87 (4 VGPRs = 2 rows each)
    VEND = 88
    S = dict(tile=64, nt=65, partial=66, tilebytes=67, woff=68, status=69, rr=72, tgt=74, rt=76, k=81, pe=82,
             base=86, kh=90)
    SPAIRS = {"rr", "tgt", "rt", "base"}

    def vpins(self):
        pins = [("a[0]", "v[32:33]"), ("a[1]", "v[34:35]"), ("b[0]", "v[36:37]"), ("b[1]", "v[38:39]"),
                ("chk", "v[40:41]")]
        rest = [r for r in range(self.CHK + 2, self.VEND)]
        return pins + [(f"v[{i}]", f"v{r}") for i, r in enumerate(rest)], rest

    def sregs(self):
        out = []
        for n, r in self.S.items():
            out.append((n, r))
            if n in self.SPAIRS:
                out.append((n + "_hi", r + 1))
        return out


# Registers of the hand-written Float64 tree loop (jit64_template.hip
# SR_JIT64_LOOP_TEXT) live across every tree-code call: s46..s57 its state,
# s60 / s61 the tree and slot, s[88:89] the code area, s[94:95] its return;
# and every SGPR above the routine temporaries that no state names (the
# gradient tree code's constant / partial pointers s[78:79], s[84:85]
# among them). Held live across each routine (the compiler may borrow one
# only saved to a VGPR lane and restored), so routine SGPR temporaries stay
# in s0..s45 — which lets the LogCosh / LogitDist / erfc routines in (round 5;
# with fewer pins their exp / log1p constants went to s70..s85); VGPR
# temporaries stay below v88 (the loop's LDS tile / counter addresses).
LOOP64_PINNED_S = (list(range(46, 64)) + [70, 71, 78, 79, 80, 83, 84, 85, 88, 89] + list(range(91, 94)) +
                   list(range(94, 102)))
ROUTINE64_S_END, ROUTINE64_V_END = 46, 88


def snippet_source(rg, routines):
    pins, rest = rg.vpins()
    out = ["#define SRHIP_INLINE_ALL 1", '#include "interp.h"', "using namespace srhip; using namespace srhip::interp;",
           "namespace {", "struct St {", "  double a[2]; double b[2]; double chk;", f"  unsigned v[{len(rest)}];"]
    for n, _ in rg.sregs():
        out.append(f"  unsigned s_{n};")
    out.append("};")

    def pin_lines(kind):
        lines = []
        for i in range(0, len(pins), 8):
            ch = pins[i:i + 8]
            if kind == "in":
                lines.append('  asm volatile("; IN ' + " ".join(r for _, r in ch) + '" : ' +
                             ", ".join(f'"={{{r}}}"(s.{e})' for e, r in ch) + ");")
            else:
                lines.append('  asm volatile("; OUT" :: ' + ", ".join(f'"{{{r}}}"(s.{e})' for e, r in ch) + ");")
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
        out += pin_lines("in")
        zs = LOOP64_PINNED_S
        out.append(f"  unsigned zz[{len(zs)}];")
        for i in range(0, len(zs), 8):
            out.append('  asm volatile("; IN ' + " ".join(f"s{zs[j]}" for j in range(i, min(i + 8, len(zs)))) +
                       '" : ' + ", ".join(f'"={{s{zs[j]}}}"(zz[{j}])'
                                                            for j in range(i, min(i + 8, len(zs)))) + ");")
        out.append("  __builtin_amdgcn_sched_barrier(0);")  # the body after every pin
        out.append("  double& chk = s.chk; (void)chk;")
        out.append("  constexpr int R = 2; (void)R;")
        out.append("  " + body)
        out += pin_lines("out")
        for i in range(0, len(zs), 8):
            out.append('  asm volatile("; OUT" :: ' + ", ".join(f'"{{s{zs[j]}}}"(zz[{j}])'
                                                             for j in range(i, min(i + 8, len(zs)))) + ");")
        out.append("}")
    out.append("}  // namespace")
    return "\n".join(out) + "\n"


def rows(expr):
    return f"_Pragma(\"unroll\") for (int r = 0; r < R; ++r) {{ {expr} }}"


def routine_list():
    """(name, body): one per operator not emitted inline; constant-operand
    variants with the Float64 constant in s_k (low word) : s_kh (high word)."""
    rs = []
    for u in sorted(UOPS, key=lambda k: UOPS[k]):
        if u in INLINE_UOPS:
            continue
        mk = "chk = mark(s.a[r], chk); " if u in LOSSY_UOPS else ""
        rs.append((f"u_{u.lower()}", rows(f"{mk}s.a[r] = dev::uop<SRHIP_UOP_{u}>(s.a[r]);")))
    imm = ("const double imm = __builtin_bit_cast(double, ((unsigned long long)s.s_kh << 32) | "
           "(unsigned long long)s.s_k); ")
    for b in sorted(BOPS, key=lambda k: BOPS[k]):
        if b in INLINE_BOPS:
            continue
        mk = ("chk = mark(s.a[r], chk); " if b in LOSSY_LHS else "") + \
             ("chk = mark(s.b[r], chk); " if b in LOSSY_RHS else "")
        rs.append((f"b_{b.lower()}", rows(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(s.a[r], s.b[r]);")))
        mk = "chk = mark(s.a[r], chk); " if b in LOSSY_LHS else ""
        rs.append((f"b_{b.lower()}_rc", imm + rows(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(s.a[r], imm);")))
        mk = "chk = mark(s.a[r], chk); " if b in LOSSY_RHS else ""
        rs.append((f"b_{b.lower()}_lc", imm + rows(f"{mk}s.a[r] = dev::bop<SRHIP_BOP_{b}>(imm, s.a[r]);")))
    # elementwise losses but L2 (inline): r in A -> ℓ(r) in A, the parameter
    # (Float64 bits) in s_k : s_kh — device_ops.h elem_loss with ŷ = r, y = 0
    # (r - 0 = r exactly), the Float64 interpreter's loss code
    for name in sorted(LOSSES, key=lambda k: LOSSES[k]):
        if name in NO_LOSS_ROUTINE:
            continue
        rs.append((f"l_{name.lower()}",
                   imm + rows(f"s.a[r] = dev::elem_loss<double>(SRHIP_LOSS_{name}, imm, s.a[r], 0.0);")))
    # dℓ/dr of the same losses (the Float64 gradient tree code's seed, jit64.cpp GradGen64);
    # LP's Float64 pow runs its two rows one after the other (scheduler fenced between them:
    # both at once exceed the routine registers)
    for name in sorted(LOSSES, key=lambda k: LOSSES[k]):
        if name in NO_LOSS_ROUTINE:
            continue
        body = f"s.a[r] = dev::elem_dloss<double>(SRHIP_LOSS_{name}, imm, s.a[r], 0.0);"
        if name == "LP":  # elem_dloss's value with only pow's temporaries live, one row at a time
            rs.append(("d_lp", imm + "const double pm1 = imm - 1.0; " + rows(
                "{ const double a = s.a[r]; const double v = imm * dev::elem_loss<double>(SRHIP_LOSS_LP, pm1, a, 0.0); "
                "s.a[r] = a == 0.0 ? v * 0.0 : __builtin_copysign(v, a); }")))
            continue
        rs.append((f"d_{name.lower()}", imm + rows(body)))
    return rs


def compile_bodies(hipcc, rg, routines):
    src = snippet_source(rg, routines)
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "routines64.hip")
        open(sp, "w").write(src)
        ap = os.path.join(td, "routines64.s")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
               "-S", "-I", HERE, sp, "-o", ap]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            raise SystemExit("gen_jit64: routine compile failed")
        asm = open(ap).read()
    bodies = {}
    for n, _ in routines:
        try:
            if not G.pins_first(asm, n):  # a pinned register used as a temporary before its pin
                raise SystemExit("code placed ahead of the register pins")
            bodies[n] = G.extract(asm, n)
        except SystemExit as e:  # memory operands, calls: no routine (the operator stays interpreted)
            sys.stderr.write(f"gen_jit64: routine {n} left out ({e})\n")
    return bodies


def build(hipcc, outdir):
    rg = Regs64()
    routines = routine_list()
    bodies = compile_bodies(hipcc, rg, routines)
    names = [n for n, _ in routines if n in bodies]
    _, rest = rg.vpins()
    vstate = set(range(rg.A, rg.VEND))
    sstate = {r for _, r in rg.sregs()}
    # a routine whose temporaries would live in tree-code state (or reach the
    # SGPRs above the state) is left out too
    pinned = set(LOOP64_PINNED_S)  # borrowed ones are saved to a VGPR lane and restored
    for n in list(names):
        vt = G.regs_used(bodies[n], G.REG_V) - vstate
        st = G.regs_used(bodies[n], G.REG_S) - sstate - pinned
        if any(r >= ROUTINE64_V_END for r in vt) or any(r >= ROUTINE64_S_END for r in st):
            sys.stderr.write(f"gen_jit64: routine {n} left out (VGPRs up to v{max(vt, default=0)}, "
                             f"SGPRs up to s{max(st, default=0)})\n")
            names.remove(n)
    vtemp, stemp = set(), set()
    for n in names:
        vtemp |= G.regs_used(bodies[n], G.REG_V) - vstate
        stemp |= G.regs_used(bodies[n], G.REG_S) - sstate - pinned
    assert max(stemp, default=0) < ROUTINE64_S_END and max(vtemp, default=0) < ROUTINE64_V_END
    text = ["s_endpgm", ".p2align 8", ".globl sr_rt64", "sr_rt64:"]
    for n in names:
        body = list(bodies[n])
        while body and body[0].startswith("s_nop"):
            body.pop(0)
        text += [f".globl sr_rt64_{n}", f"sr_rt64_{n}:", ".p2align 6" if False else ""]
        text = [t for t in text if t]
        text += [l.replace("%=", "d") for l in body]
        text.append(f"s_setpc_b64 s[{rg.S['rr']}:{rg.S['rr'] + 1}]")
        text.append(".p2align 6")
    os.makedirs(outdir, exist_ok=True)
    with open(os.path.join(outdir, "jit64_routines.inc"), "w") as f:
        f.write("// Generated by gen_jit64.py; do not edit.\n#pragma once\n#define SR_JIT64_ROUTINES_TEXT \\\n")
        for ln in text:
            f.write('  "' + ln.replace("\\", "\\\\").replace('"', '\\"') + '\\n" \\\n')
        f.write('  ""\n')
    uop_rt = {UOPS[u]: f"u_{u.lower()}" for u in UOPS}
    bop_rt = {BOPS[b]: f"b_{b.lower()}" for b in BOPS}

    def rid(n):
        return names.index(n) if n in names else -1
    # clobbers of a tree-code call: routine temporaries and every tree-code
    # register but the driver's inputs / outputs
    clob_v = sorted(vtemp | (vstate - {rg.CHK, rg.CHK + 1, rg.LANE, rg.LANE2, rg.LSUM, rg.LSUM + 1}))
    clob_s = sorted(stemp | set(range(20, 22)) |
                    (sstate - {rg.S[k] for k in ("tile", "nt", "partial", "tilebytes", "woff", "status")}))
    with open(os.path.join(outdir, "jit64_layout.h"), "w") as f:
        f.write("// Generated by gen_jit64.py; do not edit.\n#pragma once\n")
        for k in ("A", "B", "CHK", "LANE", "LANE2", "LSUM", "GT", "Y", "POOL0", "NPOOL", "VEND"):
            f.write(f"#define SR_JIT64_V_{k} {getattr(rg, k)}\n")
        for k, v in rg.S.items():
            f.write(f"#define SR_JIT64_S_{k.upper()} {v}\n")
        f.write("#define SR_JIT64_UOP_ROUTINE {" + ", ".join(
            str(-1 if u[2:].upper() in INLINE_UOPS else rid(u)) for _, u in sorted(uop_rt.items())) + "}\n")
        f.write("#define SR_JIT64_BOP_ROUTINE {" + ", ".join(
            str(-1 if b[2:].upper() in INLINE_BOPS else rid(b)) for _, b in sorted(bop_rt.items())) + "}\n")
        for suf in ("rc", "lc"):
            f.write(f"#define SR_JIT64_BOP_ROUTINE_{suf.upper()} {{" + ", ".join(
                str(-1 if b[2:].upper() in INLINE_BOPS else rid(f"{b}_{suf}")) for _, b in sorted(bop_rt.items()))
                + "}\n")
        f.write("#define SR_JIT64_LOSS_ROUTINE {" + ", ".join(
            str(-1 if n in NO_LOSS_ROUTINE else rid(f"l_{n.lower()}")) for n in sorted(LOSSES, key=lambda k: LOSSES[k])) + "}\n")
        f.write("#define SR_JIT64_DLOSS_ROUTINE {" + ", ".join(
            str(-1 if n in NO_LOSS_ROUTINE else rid(f"d_{n.lower()}")) for n in sorted(LOSSES, key=lambda k: LOSSES[k])) + "}\n")
        f.write(f"#define SR_JIT64_NUM_ROUTINES {len(names)}\n")
        f.write("#define SR_JIT64_ROUTINE_NAMES {" + ", ".join(f'"{n}"' for n in names) + "}\n")
        f.write("#define SR_JIT64_CLOBBERS " + ", ".join([f'"v{r}"' for r in clob_v] + [f'"s{r}"' for r in clob_s]
                                                         + ['"vcc"', '"scc"']) + "\n")
        # Float64 gradient tree code (jit64.cpp GradGen64): the same routines, a
        # larger value pool, the tree's constants as VGPR pairs (the routines'
        # SGPR temporaries reach s45), one Float64 accumulator pair per constant;
        # its inputs: s[78:79] the tree's constants, s[84:85] its ∂L/∂c partials
        g = dict(POOL0=56, NPOOL=20, C0=136, ACC=168, NACC=16, SCPTR=78, SGPTR=84)
        assert g["POOL0"] + 4 * g["NPOOL"] == g["C0"] and g["C0"] + 2 * g["NACC"] == g["ACC"]
        for k, v in g.items():
            f.write(f"#define SR_JIT64_G_{k} {v}\n")
        gin_v = {rg.CHK, rg.CHK + 1, rg.LANE, rg.LANE2, rg.LSUM, rg.LSUM + 1}
        gclob_v = sorted((vtemp | set(range(rg.A, g["ACC"] + 2 * g["NACC"]))) - gin_v)
        gin_s = {rg.S[k] for k in ("tile", "nt", "partial", "tilebytes", "woff", "status")} | \
            {g["SCPTR"], g["SCPTR"] + 1, g["SGPTR"], g["SGPTR"] + 1}
        assert not gin_s & (stemp | {20, 21})
        gclob_s = sorted((stemp | set(range(20, 22)) | sstate) - gin_s)
        f.write("#define SR_JIT64_GRAD_CLOBBERS " + ", ".join([f'"v{r}"' for r in gclob_v] + [f'"s{r}"' for r in gclob_s]
                                                              + ['"vcc"', '"scc"']) + "\n")
        f.write(f"// routine VGPR temps {sorted(vtemp)}, SGPR temps {sorted(stemp)}\n")


if __name__ == "__main__":
    build(sys.argv[1], sys.argv[2])
