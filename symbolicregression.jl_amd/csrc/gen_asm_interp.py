#!/usr/bin/env python3
"""Generate the direct-threaded interpreter block of the f32 eval kernel.

The C++ interpreter (interp.h) dispatches each program instruction with a
uniform binary-search branch tree: ~7 compares + 7 branches + ~14 SALU per
instruction, on a CU whose single scalar unit is shared by its 4 SIMDs. For
the +,-,*,/ mix that costs more than the VALU work of the instruction (8 rows
per lane). This script builds a *threaded* interpreter instead:

  * every opcode has a handler; the dispatch is
        s_lshl/s_and (opcode) -> s_add/s_addc (table slot) -> s_setpc_b64
    into a table of `s_branch handler` entries: 2 jumps and 5 SALU;
  * the program lives in two VGPRs (lane j = instruction j, as in
    run_program_v), read with v_readlane one instruction ahead;
  * handler BODIES are not hand-written: each one is compiled by hipcc from the
    same C++ operator code as the C++ interpreter (device_ops.h: bop/uop/mark,
    fast_sincos_f32) inside a tiny kernel whose interpreter state is pinned to
    fixed registers with inline-asm constraints; the body is cut out of the
    compiler's assembly. Arithmetic, instruction order within a row and hazard
    nops are therefore the compiler's own: results are bit-identical to the
    C++ interpreter.
  * anything the threaded block does not handle (operators outside the
    handled set, |x| > 105615 for sin/cos) "bails": the block returns a flag
    and the C++ kernel re-runs that (tree, tile) with run_program.

Output: a header defining SR_TI_TEXT (the asm string), SR_TI_CLOBBERS and
the register map used by eval_kernel.h. Usage:
    gen_asm_interp.py <hipcc> <out.inc> [R] [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
INCLUDE = os.path.join(HERE, "..", "..", "include", "srhip.h")


def enums():
    txt = open(INCLUDE).read()
    uops = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define SRHIP_UOP_(\w+)\s+(\d+)", txt)}
    bops = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define SRHIP_BOP_(\w+)\s+(\d+)", txt)}
    return uops, bops


UOPS, BOPS = enums()
NUM_UOPS, NUM_BOPS = len(UOPS), len(BOPS)
MAX_SLOTS = 16
OP_END, OP_LDX, OP_LDC, OP_PUSH0 = 0, 1, 2, 3
OP_POP0 = OP_PUSH0 + MAX_SLOTS
OP_UN0 = OP_POP0 + MAX_SLOTS
OP_BIN0 = OP_UN0 + NUM_UOPS
VARIANTS = ["AX", "XA", "AC", "CA", "AT", "TA", "XX", "XC", "CX"]
NUM_OPCODES = OP_BIN0 + len(VARIANTS) * NUM_BOPS
D = 2  # stack slots of the shallow kernel (kShallowSlots)

# Operators with handlers: all but the five whose inline code is large
# (pow, mod, atanh_clip's mod, gamma, tan): those bail to the C++ interpreter.
H_BOPS = [b for b in BOPS if b not in ("POW", "MOD")]
H_UOPS = [u for u in UOPS if u not in ("ATANH_CLIP", "GAMMA", "TAN")]
LOSSY_UOPS = {"EXP", "TANH", "ATAN", "ERF", "ERFC", "SIGN", "INV"}
LOSSY_LHS = {"POW", "GREATER", "LOGICAL_OR", "LOGICAL_AND", "MAX", "MIN"}
LOSSY_RHS = {"DIV", "POW", "GREATER", "LOGICAL_OR", "LOGICAL_AND", "MOD", "MAX", "MIN"}


class RegMap:
    """Fixed registers of the threaded block for R rows per lane."""

    def __init__(self, R):
        self.R = R
        b = 32
        # acc, tmp, the two X buffers (ping-pong: the X operand of the next
        # instruction is read while this one runs), slots. The XX second
        # operand goes to tmp: the compiler emits every POP right before the
        # AT/TA instruction that consumes tmp, so tmp is dead at an XX.
        self.acc, self.tmp, self.xa, self.xb = b, b + R, b + 2 * R, b + 3 * R
        self.x2 = self.tmp
        self.slot = [b + (4 + k) * R for k in range(D)]
        top = b + (4 + D) * R
        self.chk, self.lane = top, top + 1
        self.vstate_end = top + 2
        # SGPRs: scratch, table (2), target (2), trig flag (2), instruction
        # records of parity A and B (4 + 4: next table slot, next X offset,
        # immediate, pad), record base (2), record offset, bail
        self.s_t, self.s_tbl, self.s_tgt, self.s_flag = 67, 68, 70, 74
        self.s_rec = {"a": 76, "b": 80}
        self.s_rbase, self.s_roff, self.s_bail = 84, 86, 87
        self.s_exit = 72  # address of the block's exit (handlers are > 128 KiB apart)

    def imm_sgpr(self, par):
        return self.s_rec[par] + 2

    def vstate(self):
        """(name, first reg, count) of every VGPR state register group."""
        R = self.R
        g = [("acc", self.acc, R), ("tmp", self.tmp, R), ("xa", self.xa, R), ("xb", self.xb, R)]
        g += [(f"slot{k}", self.slot[k], R) for k in range(D)]
        g += [("chk", self.chk, 1), ("lane", self.lane, 1)]
        return g

    def sstate(self):
        out = [("st", self.s_t), ("tbl0", self.s_tbl), ("tbl1", self.s_tbl + 1), ("tgt0", self.s_tgt),
               ("tgt1", self.s_tgt + 1), ("flag0", self.s_flag), ("flag1", self.s_flag + 1)]
        for par in ("a", "b"):
            out += [(f"r{par}{k}", self.s_rec[par] + k) for k in range(4)]
        out += [("rbase0", self.s_rbase), ("rbase1", self.s_rbase + 1), ("roff", self.s_roff),
                ("bail", self.s_bail), ("exit0", self.s_exit), ("exit1", self.s_exit + 1)]
        return out


# ---------------------------------------------------------------------------
# 1. handler snippets (C++), compiled by hipcc

def snippet_source(rm, handlers):
    R = rm.R
    out = ["#define SRHIP_INLINE_ALL 1", '#include "interp.h"', "using namespace srhip; using namespace srhip::interp;",
           "namespace {", "struct St {"]
    for name, base, cnt in rm.vstate():
        out.append(f"  float {name}[{cnt}];" if cnt > 1 else
                   f"  {'float' if name == 'chk' else 'unsigned'} {name};")
    for name, _ in rm.sstate():
        out.append(f"  unsigned s_{name};")
    out.append("};")
    # IN: define every state register (pinned); OUT: use every one of them.
    def pin_lines(kind):
        lines = []
        for name, base, cnt in rm.vstate():
            regs = [(f"{name}[{i}]" if cnt > 1 else name, base + i) for i in range(cnt)]
            for i in range(0, len(regs), 8):
                chunk = regs[i:i + 8]
                if kind == "in":
                    ops = ", ".join(f'"={{v{r}}}"(s.{e})' for e, r in chunk)
                    lines.append(f'  asm volatile("; IN" : {ops});')
                else:
                    ops = ", ".join(f'"{{v{r}}}"(s.{e})' for e, r in chunk)
                    lines.append(f'  asm volatile("; OUT" :: {ops});')
        ss = rm.sstate()
        for i in range(0, len(ss), 8):
            chunk = ss[i:i + 8]
            if kind == "in":
                ops = ", ".join(f'"={{s{r}}}"(s.s_{n})' for n, r in chunk)
                lines.append(f'  asm volatile("; IN" : {ops});')
            else:
                ops = ", ".join(f'"{{s{r}}}"(s.s_{n})' for n, r in chunk)
                lines.append(f'  asm volatile("; OUT" :: {ops});')
        return lines
    for hname, body, par in handlers:
        out.append(f'extern "C" __global__ void __launch_bounds__(64) sr_h_{hname}() {{')
        out.append("  St s;")
        out += pin_lines("in")
        out.append(f"  const float imm = __int_as_float((int)s.s_r{par}2); (void)imm;")
        out.append("  float& chk = s.chk; (void)chk;")
        out.append(f"  constexpr int R = {R}; (void)R;")
        out.append("  " + body)
        out += pin_lines("out")
        out.append("}")
    out.append("}  // namespace")
    return "\n".join(out) + "\n"


def rows(expr):
    return f"_Pragma(\"unroll\") for (int r = 0; r < R; ++r) {{ {expr} }}"


def handler_bodies(basic_only=False):
    """(opcode, name, body C++, needs_x, needs_x2, trig) for every handled opcode
    (basic_only: the BASIC operator set only, the rest bails)."""
    hs = []
    hs.append((OP_LDX, "ldx", rows("s.acc[r] = s.{X}[r];"), True, False, False))
    hs.append((OP_LDC, "ldc", rows("s.acc[r] = imm;"), False, False, False))
    for k in range(D):
        hs.append((OP_PUSH0 + k, f"push{k}", rows(f"s.slot{k}[r] = s.acc[r];"), False, False, False))
        hs.append((OP_POP0 + k, f"pop{k}", rows(f"s.tmp[r] = s.slot{k}[r];"), False, False, False))
    for u in H_UOPS:
        code = OP_UN0 + UOPS[u]
        if u in ("SIN", "COS"):
            # fast path only while every row's |n| <= kTrigQMax (device_ops.h)
            body = ("float qm = 0.0f; " +
                    rows(f"float qa; s.acc[r] = dev::fast_sincos_f32(s.acc[r], {1 if u == 'COS' else 0}, qa); "
                         "qm = __builtin_fmaxf(qm, qa);") +
                    " const unsigned long long fl = __builtin_amdgcn_ballot_w64(!(qm <= dev::kTrigQMax));"
                    " s.s_flag0 = (unsigned)fl; s.s_flag1 = (unsigned)(fl >> 32);")
            hs.append((code, f"un_{u.lower()}", body, False, False, True))
        else:
            mk = "chk = mark(s.acc[r], chk); " if u in LOSSY_UOPS else ""
            hs.append((code, f"un_{u.lower()}",
                       rows(f"{mk}s.acc[r] = dev::uop<SRHIP_UOP_{u}>(s.acc[r]);"), False, False, False))
    for b in H_BOPS:
        LL, LR = b in LOSSY_LHS, b in LOSSY_RHS
        f = f"dev::bop<SRHIP_BOP_{b}>"
        for vi, v in enumerate(VARIANTS):
            code = OP_BIN0 + vi * NUM_BOPS + BOPS[b]
            mk = ""
            if v == "AX":
                mk, e = ("chk = mark(s.acc[r], chk); " if LL else ""), f"{f}(s.acc[r], s.{{X}}[r])"
            elif v == "XA":
                mk, e = ("chk = mark(s.acc[r], chk); " if LR else ""), f"{f}(s.{{X}}[r], s.acc[r])"
            elif v == "AC":
                mk, e = ("chk = mark(s.acc[r], chk); " if LL else ""), f"{f}(s.acc[r], imm)"
            elif v == "CA":
                mk, e = ("chk = mark(s.acc[r], chk); " if LR else ""), f"{f}(imm, s.acc[r])"
            elif v == "AT":
                mk = ("chk = mark(s.acc[r], chk); " if LL else "") + ("chk = mark(s.tmp[r], chk); " if LR else "")
                e = f"{f}(s.acc[r], s.tmp[r])"
            elif v == "TA":
                mk = ("chk = mark(s.tmp[r], chk); " if LL else "") + ("chk = mark(s.acc[r], chk); " if LR else "")
                e = f"{f}(s.tmp[r], s.acc[r])"
            elif v == "XX":
                e = f"{f}(s.{{X}}[r], s.tmp[r])"  # second X operand read into tmp
            elif v == "XC":
                e = f"{f}(s.{{X}}[r], imm)"
            else:  # CX
                e = f"{f}(imm, s.{{X}}[r])"
            nx = v in ("AX", "XA", "XX", "XC", "CX")
            hs.append((code, f"b{b.lower()}_{v.lower()}", rows(f"{mk}s.acc[r] = {e};"), nx, v == "XX", False))
    # code layout: the BASIC operator set (srhip_internal.h) first, so that the
    # common handlers share instruction-cache lines; the rest after it
    basic_u = {"NEG", "SQUARE", "CUBE", "EXP", "ABS", "LOG", "SQRT", "SIN", "COS"}
    basic_b = {"ADD", "SUB", "MUL", "DIV"}

    def is_basic(h):
        u = h[1].upper()
        if u in ("LDX", "LDC") or u.startswith(("PUSH", "POP")):
            return True
        if u.startswith("UN_"):
            return u[3:] in basic_u
        return u[1:].split("_")[0] in basic_b
    if basic_only:
        return [h for h in hs if is_basic(h)]
    return [h for h in hs if is_basic(h)] + [h for h in hs if not is_basic(h)]


# ---------------------------------------------------------------------------
# 2. extraction

REG_V = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
REG_S = re.compile(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]")
BAD = ("s_swappc", "s_setpc", "s_getpc", "scratch_", "buffer_", "global_", "flat_", "s_load", "s_store",
       "s_buffer", "s_dcache", "s_endpgm", "s_sendmsg", "ds_", "s_waitcnt")


def pins_first(asm_text, name):
    """False if handler `name` writes a register ahead of the "; IN <regs>"
    marker that pins it (live from the routine's entry in the tree code): the
    compiler, which sees the register defined only at the marker, took it for
    a free temporary there. Markers without a register list are not checked."""
    m = re.search(rf"^sr_h_{name}:.*?$(.*?)^\.Lfunc_end", asm_text, re.S | re.M)
    if not m:
        raise SystemExit(f"gen_asm_interp: handler {name} not found in compiler output")
    written_s, written_v, in_marker = set(), set(), False
    for ln in m.group(1).splitlines():
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_marker = True
            continue
        if s.startswith(";;#ASMEND"):
            in_marker = False
            continue
        if in_marker:
            if s.startswith("; IN "):
                regs = s[5:].split()
                if (regs_used(regs, REG_S) & written_s) or (regs_used(regs, REG_V) & written_v):
                    return False
            continue
        s = s.split(";")[0].strip()
        parts = s.split(None, 1)
        if not s or s.startswith(".") or len(parts) < 2:
            continue
        if parts[0].startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_nop", "v_cmpx")):
            continue
        dst = parts[1].split(",")[0]
        written_s |= regs_used([dst], REG_S)
        written_v |= regs_used([dst], REG_V)
    return True


def extract(asm_text, name):
    m = re.search(rf"^sr_h_{name}:.*?$(.*?)^\.Lfunc_end", asm_text, re.S | re.M)
    if not m:
        raise SystemExit(f"gen_asm_interp: handler {name} not found in compiler output")
    # the compiler may place cold blocks after the kernel's s_endpgm: every
    # s_endpgm becomes a branch to the handler's end (the last one is dropped)
    body = m.group(1).rstrip().splitlines()
    while body and not body[-1].strip().split(";")[0]:
        body.pop()
    if body and body[-1].strip().startswith("s_endpgm"):
        body.pop()
    body = [("s_branch .LBBsrend" if ln.strip().startswith("s_endpgm") else ln) for ln in body]
    if any(ln == "s_branch .LBBsrend" for ln in body):
        body.append(".LBBsrend:")
    lines, in_marker = [], False
    for ln in body:
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_marker = True
            continue
        if s.startswith(";;#ASMEND"):
            in_marker = False
            continue
        s = s.split(";")[0].rstrip()  # (a loop header label carries a trailing comment)
        if in_marker or not s or s.startswith(".") and not s.endswith(":"):
            continue
        if re.match(r"^\.LBB\w+:$", s):
            lines.append(s)
            continue
        for bad in BAD:
            if bad in s:
                raise SystemExit(f"gen_asm_interp: handler {name} contains '{bad}': {s}")
        lines.append(s)
    # a branch to the very next line (left where a trailing s_endpgm was) goes
    lines = [s for k, s in enumerate(lines)
             if not (s.startswith("s_branch ") and k + 1 < len(lines) and lines[k + 1] == s.split()[1] + ":")]
    # handler-local labels -> unique per handler (and per asm instance via %=)
    lbl = {}
    for s in lines:
        if s.endswith(":"):
            lbl[s[:-1]] = f".Lsr{name}_{len(lbl)}_%="
    out = []
    for s in lines:
        for k, v in lbl.items():
            s = re.sub(re.escape(k) + r"\b", v, s)
        out.append(s)
    return out


def regs_used(lines, pat):
    used = set()
    for s in lines:
        if s.endswith(":"):
            continue
        for m in pat.finditer(s):
            if m.group(1) is not None:
                used.add(int(m.group(1)))
            else:
                used.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return used


# ---------------------------------------------------------------------------
# 3. the threaded block

def build(hipcc, out_path, R, extra):
    rm = RegMap(R)
    # R = 16 pins 130 VGPRs of state: the large handlers (acosh, ...) crash
    # the compiler's scheduler there, and only the BASIC set matters for speed
    hs = handler_bodies(basic_only=R > 8)
    variants = []  # (opcode, parity, name, body, needs_x, needs_x2, trig)
    for code, n, body, nx, nx2, trig in hs:
        for par, xname in (("a", "xa"), ("b", "xb")):
            variants.append((code, par, f"{n}_{par}", body.replace("{X}", xname), nx, nx2, trig))
    src = snippet_source(rm, [(n, b, par) for _, par, n, b, *_ in variants])
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "handlers.hip")
        open(sp, "w").write(src)
        ap = os.path.join(td, "handlers.s")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
               "-S", "-I", HERE, sp, "-o", ap] + extra
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            raise SystemExit("gen_asm_interp: handler compile failed")
        asm = open(ap).read()
    bodies = {n: extract(asm, n) for _, _, n, *_ in variants}

    vstate = set(range(rm.acc, rm.vstate_end))
    sstate = {r for _, r in rm.sstate()}
    vtemp, stemp = set(), set()
    for n, lines in bodies.items():
        vtemp |= regs_used(lines, REG_V) - vstate
        stemp |= regs_used(lines, REG_S) - sstate
    vtemp |= {0, 1}  # glue: LDS addresses
    if vtemp & vstate:
        raise SystemExit("gen_asm_interp: temp/state VGPR overlap")

    s = rm
    nrd = R // 4  # ds_read_b128 per R-row operand
    T = []
    a = T.append

    def lds_read(dst, addr_v):
        # R rows per lane: chunk c of 4 rows at +1024*c bytes (interp.h lds_rows)
        for c in range(nrd):
            off = f" offset:{1024 * c}" if c else ""
            a(f"ds_read_b128 v[{dst + 4 * c}:{dst + 4 * c + 3}], v{addr_v}{off}")

    def rec(par, k):
        return s.s_rec[par] + k

    # Records (ti_records_kernel): record 0 of a tree = {h(0), xo(0)}, record
    # i+1 = {h(i+1), xo(i+1), imm(i)} with h(j) the byte offset (from
    # .Lsr_base) of instruction j's handler in the parity j&1 and xo(j) the LDS
    # byte offset of its X operand. Instruction i runs in parity (i&1) with
    # record i+1 in that parity's SGPRs; it loads record i+2 into the other
    # parity's SGPRs and X(i+1) into the other X buffer, and jumps straight to
    # the next handler: everything it waits for was issued one instruction ago.
    a(f"s_getpc_b64 s[{s.s_tbl}:{s.s_tbl + 1}]")
    a(".Lsr_pc_%=:")
    a(f"s_add_u32 s{s.s_tbl}, s{s.s_tbl}, .Lsr_base_%=-.Lsr_pc_%=")
    a(f"s_addc_u32 s{s.s_tbl + 1}, s{s.s_tbl + 1}, 0")
    a(f"s_mov_b32 s{s.s_bail}, 0")
    a(f"s_add_u32 s{s.s_exit}, s{s.s_tbl}, .Lsr_done_%=-.Lsr_base_%=")
    a(f"s_mov_b32 s{s.s_exit + 1}, s{s.s_tbl + 1}")
    # the handler offsets were measured on a standalone assembly of this text:
    # check two of them against the assembled layout, else run the C++ path
    # (biased by 2^20 so that no value is an inline constant: sizes are fixed)
    a(f"s_mov_b32 s{s.s_t}, .Lsr_h_end_%=-.Lsr_base_%=+0x100000")
    a(f"s_cmp_lg_u32 s{s.s_t}, @HOFF_END@")
    a("s_cbranch_scc1 .Lsr_bail_%=")
    a(f"s_mov_b32 s{s.s_t}, .Lsr_done_%=-.Lsr_base_%=+0x100000")
    a(f"s_cmp_lg_u32 s{s.s_t}, @HOFF_DONE@")
    a("s_cbranch_scc1 .Lsr_bail_%=")
    a(f"s_add_u32 s{s.s_t}, s{s.s_tbl}, @SPAN@")  # the block in one 4 GiB page:
    a("s_cbranch_scc1 .Lsr_bail_%=")             # the target's high word is constant
    a(f"s_mov_b32 s{s.s_tgt + 1}, s{s.s_tbl + 1}")
    a(f"s_load_dwordx4 s[{rec('b', 0)}:{rec('b', 3)}], s[{s.s_rbase}:{s.s_rbase + 1}], 0x0")
    a(f"s_load_dwordx4 s[{rec('a', 0)}:{rec('a', 3)}], s[{s.s_rbase}:{s.s_rbase + 1}], 0x10")
    a(f"s_mov_b32 s{s.s_roff}, 32")
    a("s_waitcnt lgkmcnt(0)")
    a(f"v_add_u32_e32 v0, s{rec('b', 1)}, v{s.lane}")
    lds_read(s.xa, 0)
    a(f"s_and_b32 s{s.s_t}, s{rec('b', 0)}, @MASK@")
    a(f"s_add_u32 s{s.s_tgt}, s{s.s_tbl}, s{s.s_t}")
    a(f"s_setpc_b64 s[{s.s_tgt}:{s.s_tgt + 1}]")
    a(".Lsr_base_%=:")
    a(".Lsr_h_end_%=:")
    a(f"s_setpc_b64 s[{s.s_exit}:{s.s_exit + 1}]")
    a(".Lsr_bail_%=:")
    a(f"s_mov_b32 s{s.s_bail}, 1")
    a(f"s_setpc_b64 s[{s.s_exit}:{s.s_exit + 1}]")
    for code, par, n, body, nx, nx2, trig in variants:
        other = "b" if par == "a" else "a"
        xother = s.xb if par == "a" else s.xa
        a(f".Lsr_h_{n}_%=:")
        a("s_waitcnt lgkmcnt(0)")  # this record + this X (issued one instruction ago)
        if nx2:  # second X operand (its byte offset is the immediate), read now
            a(f"v_add_u32_e32 v1, s{rec(par, 2)}, v{s.lane}")
            lds_read(s.x2, 1)
            a("s_waitcnt lgkmcnt(0)")
        a(f"s_load_dwordx4 s[{rec(other, 0)}:{rec(other, 3)}], s[{s.s_rbase}:{s.s_rbase + 1}], s{s.s_roff}")
        a(f"s_add_u32 s{s.s_roff}, s{s.s_roff}, 16")
        a(f"v_add_u32_e32 v0, s{rec(par, 1)}, v{s.lane}")
        lds_read(xother, 0)  # X operand of the NEXT instruction (offset 0 if none)
        a(f"s_and_b32 s{s.s_t}, s{rec(par, 0)}, @MASK@")  # next handler (masked: never
        a(f"s_add_u32 s{s.s_tgt}, s{s.s_tbl}, s{s.s_t}")   # a jump outside the block)
        body_lines = list(bodies[n])
        while body_lines and body_lines[0].startswith("s_nop"):
            body_lines.pop(0)
        for ln in body_lines:
            a(ln)
        if trig:
            a(f"s_cmp_lg_u64 s[{s.s_flag}:{s.s_flag + 1}], 0")
            a(f"s_cbranch_scc1 .Lsr_tb_{n}_%=")
        a(f"s_setpc_b64 s[{s.s_tgt}:{s.s_tgt + 1}]")
        if trig:  # bail stub within branch range
            a(f".Lsr_tb_{n}_%=:")
            a(f"s_mov_b32 s{s.s_bail}, 1")
            a(f"s_setpc_b64 s[{s.s_exit}:{s.s_exit + 1}]")
    a(".Lsr_done_%=:")
    a("s_waitcnt lgkmcnt(0)")  # the last record load and X prefetch may be in flight

    # handler offsets from a standalone assembly of the block (same encoding)
    handled = {(p_, code): n for code, p_, n, *_ in variants}
    # placeholders large enough to be literals, then iterate to a fixed point
    subst = {"@HOFF_END@": "0x1ffff0", "@HOFF_DONE@": "0x1ffff0", "@SPAN@": "0x1ffff0", "@MASK@": "0x1ffff0"}
    for _ in range(4):
        offs = label_offsets([_subst(ln, subst) for ln in T])
        span = 1
        while span < offs["done"] + 64:
            span *= 2
        new = {"@HOFF_END@": hex(offs["h_end"] + 0x100000), "@HOFF_DONE@": hex(offs["done"] + 0x100000),
               "@SPAN@": hex(span), "@MASK@": hex(span - 4)}
        if new == subst:
            break
        subst = new
    else:
        raise SystemExit("gen_asm_interp: handler layout did not converge")
    T = [_subst(ln, subst) for ln in T]
    if label_offsets(T) != offs:
        raise SystemExit("gen_asm_interp: handler offsets changed after substitution")
    hoff = []
    for par in ("a", "b"):
        for code in range(256):
            n = "end" if code == OP_END else handled.get((par, code))
            hoff.append(offs[f"h_{n}"] if n else offs["bail"])
    hp = out_path.replace(".inc", "_hoff.h")
    with open(hp, "w") as f:
        f.write(f"// Generated by gen_asm_interp.py (R={R}): byte offset from the block's base of the\n"
                "// handler of (parity, opcode), index parity*256 + opcode; unhandled = bail.\n#pragma once\n")
        f.write(f"#define SR_TI_HOFF_INIT {{{', '.join(str(v) for v in hoff)}}}\n")

    # clobbers: every register the block writes besides its outputs
    outs_v = set(range(s.acc, s.acc + R)) | {s.chk}
    ins_v = {s.lane}
    clob_v = sorted((vtemp | vstate) - outs_v - ins_v)
    clob_s = sorted((stemp | sstate) - {s.s_bail, s.s_rbase, s.s_rbase + 1})
    clob = [f'"v{r}"' for r in clob_v] + [f'"s{r}"' for r in clob_s] + ['"vcc"', '"scc"']
    hdr = [f"// Generated by gen_asm_interp.py (R={R}); do not edit.",
           "#pragma once",
           f"#define SR_TI_R {R}",
           f"#define SR_TI_NUM_OPCODES {NUM_OPCODES}",
           f"#define SR_TI_OP_BIN0 {OP_BIN0}",
           "#define SR_TI_TEXT \\"]
    for ln in T:
        for l2 in ln.split("\n"):
            hdr.append('  "' + l2.replace("\\", "\\\\").replace('"', '\\"') + '\\n" \\')
    hdr.append("  \"\"")
    hdr.append("#define SR_TI_CLOBBERS " + ", ".join(clob))
    outs = [f'"={{v{s.acc + i}}}"(acc[{i}])' for i in range(R)]
    outs += [f'"+{{v{s.chk}}}"(chk)', f'"={{s{s.s_bail}}}"(bail)']
    hdr.append("#define SR_TI_OUTPUTS(acc, chk, bail) " + ", ".join(outs))
    ins = [f'"{{s[{s.s_rbase}:{s.s_rbase + 1}]}}"(recs)', f'"{{v{s.lane}}}"(lane)']
    hdr.append("#define SR_TI_INPUTS(recs, lane) " + ", ".join(ins))
    hdr.append(f"// handlers: {len(variants)} (+end, bail), VGPR temps {min(vtemp)}..{max(vtemp)}, "
               f"SGPR temps {sorted(stemp)}")
    open(out_path, "w").write("\n".join(hdr) + "\n")


def _subst(ln, subst):
    for k, v in subst.items():
        ln = ln.replace(k, v)
    return ln


def label_offsets(T):
    """Assemble the block standalone (labels made symbols) and return the offset
    of every .Lsr_<name>_%= label from .Lsr_base_%=."""
    txt = "\n".join(T).replace("%=", "0")
    txt = re.sub(r"\.Lsr_", "srlab_", txt)
    llvm = "/opt/rocm/lib/llvm/bin"
    with tempfile.TemporaryDirectory() as td:
        sp, op = os.path.join(td, "blk.s"), os.path.join(td, "blk.o")
        open(sp, "w").write("\t.text\n" + txt + "\n")
        r = subprocess.run([os.path.join(llvm, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                            "-mcpu=gfx950", "-c", sp, "-o", op], capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            raise SystemExit("gen_asm_interp: standalone assembly failed")
        r = subprocess.run([os.path.join(llvm, "llvm-objdump"), "-t", op], capture_output=True, text=True,
                           check=True)
    sym = {}
    for ln in r.stdout.splitlines():
        parts = ln.split()
        if parts and parts[-1].startswith("srlab_"):
            sym[parts[-1][len("srlab_"):-1]] = int(parts[0], 16)  # strip the trailing %= ("0")
    base = sym["base_"]
    return {k.rstrip("_"): v - base for k, v in sym.items()}


if __name__ == "__main__":
    hipcc, out = sys.argv[1], sys.argv[2]
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    build(hipcc, out, R, sys.argv[4:])
