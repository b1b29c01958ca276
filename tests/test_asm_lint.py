"""Static lint of every inline-asm statement in csrc/ (VERDICT r04 weak 7).

Round 4's illegal memory access came from an asm block
(`s_getpc_b64; s_add_u32; s_addc_u32`) that wrote SCC without declaring it:
a carry chain of the compiler spanned the block and a pointer came out 2^32
off. Rule checked here: an asm statement whose text writes SCC (a scalar ALU
instruction that sets it) or transfers control into code that may
(s_swappc_b64 / s_setpc_b64 into tree code or routines) must list "scc" in
its clobbers, directly or through a clobber macro that the generators emit
with "scc". Statements that only hold a code blob (their text starts with
s_endpgm: never executed inline) are exempt."""
import re
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "symbolicregression.jl_amd" / "csrc"

# scalar instructions that write SCC (SOP1 / SOP2 / SOPC / SOPK arithmetic and logic)
SCC_WRITERS = re.compile(
    r"\bs_(add|addc|sub|subb)_[ui]32\b|\bs_cmp|\bs_cselect|\bs_(and|or|xor|andn2|orn2|nand|nor|xnor)_b(32|64)\b"
    r"|\bs_(lshl|lshr|ashr)\w*|\bs_bfe_|\bs_(min|max)_[ui]32\b|\bs_abs_i32\b|\bs_not_b|\bs_bitcmp|\bs_mul_hi"
    r"|\bs_(and|or|xor)_saveexec|\bs_swappc_b64\b|\bs_setpc_b64\b")

# clobber macros and the generator that defines each (must emit "scc")
MACROS = {"SR_JIT_CLOBBERS": "gen_jit.py", "SR_JIT_CLOBBERS_MEMC": "gen_jit.py", "SR_JIT_GRAD_CLOBBERS": "gen_jit.py",
          "SR_JIT64_CLOBBERS": "gen_jit64.py", "SR_JIT64_GRAD_CLOBBERS": "gen_jit64.py",
          "SR_TI_CLOBBERS": "gen_asm_interp.py"}


def _statements(text, holders=False):
    """(line, whole statement text) of each asm(...) / asm volatile(...); a
    statement that is a kernel's whole body (`{ asm volatile(X); }`, the
    routine holders) is skipped unless holders=True."""
    for m in re.finditer(r"\basm\s+(?:volatile\s*)?\(", text):
        if not holders and re.search(r"\(\)\s*\{\s*$", text[max(0, m.start() - 40):m.start()]):
            continue
        i, depth = m.end(), 1
        while depth and i < len(text):
            c = text[i]
            if c == '"':
                i += 1
                while text[i] != '"':
                    i += 2 if text[i] == "\\" else 1
            elif c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
            i += 1
        yield text.count("\n", 0, m.start()) + 1, text[m.end():i - 1]


def _template_and_clobbers(stmt):
    parts, depth, cur, in_str = [], 0, "", False
    i = 0
    while i < len(stmt):  # split on top-level colons (outside strings and brackets)
        c = stmt[i]
        if in_str:
            cur += c
            if c == "\\":
                cur += stmt[i + 1]
                i += 1
            elif c == '"':
                in_str = False
        elif c == '"':
            in_str, cur = True, cur + c
        elif c in "([{":
            depth, cur = depth + 1, cur + c
        elif c in ")]}":
            depth, cur = depth - 1, cur + c
        elif c == ":" and depth == 0 and not (i + 1 < len(stmt) and stmt[i + 1] == ":"):
            parts.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    parts.append(cur)
    return parts[0], (parts[3] if len(parts) > 3 else "")


def _macro_has_scc(name):
    """The generated header when present (gen/), else the generator's
    statement that writes the #define (with the list it joins)."""
    for hdr in (CSRC / "gen").glob("*"):
        if hdr.suffix in (".h", ".inc"):
            for ln in hdr.read_text(errors="ignore").splitlines():
                if ln.startswith(f"#define {name} "):
                    return '"scc"' in ln or (name == "SR_JIT_CLOBBERS_MEMC" and _macro_has_scc("SR_JIT_CLOBBERS"))
    src = (CSRC / MACROS[name]).read_text()
    i = src.find(f"#define {name} ")
    return i >= 0 and "scc" in src[max(0, i - 600):i + 400]


def test_every_scc_writing_asm_declares_scc():
    bad, checked = [], 0
    for path in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list(CSRC.glob("*.cpp"))):
        for line, stmt in _statements(path.read_text()):
            tmpl, clob = _template_and_clobbers(stmt)
            strings = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', tmpl)).replace("\\n", "\n")
            if strings.lstrip().startswith("s_endpgm"):
                continue  # a code holder, never executed inline
            macro_text = re.sub(r'"(?:[^"\\]|\\.)*"', "", tmpl)
            if not SCC_WRITERS.search(strings) and not re.search(r"\bSR_\w+TEXT\b", macro_text):
                continue
            checked += 1
            ok = '"scc"' in clob or any(m in clob and _macro_has_scc(m) for m in MACROS)
            if not ok:
                bad.append(f"{path.name}:{line}")
    assert checked >= 10, checked  # the lint sees the code-area, call and loop blocks
    assert not bad, "asm writing SCC without an \"scc\" clobber: " + ", ".join(bad)


def test_the_lint_catches_the_round4_bug():
    stmt = next(_statements('asm volatile("s_getpc_b64 s[88:89]\\n" "s_add_u32 s88, s88, x@rel32@lo+4\\n"'
                            '"s_addc_u32 s89, s89, x@rel32@hi+12" : "={s[88:89]}"(area) : : );'))[1]
    tmpl, clob = _template_and_clobbers(stmt)
    assert SCC_WRITERS.search("".join(re.findall(r'"((?:[^"\\]|\\.)*)"', tmpl)).replace("\\n", "\n"))
    assert '"scc"' not in clob


def test_clobber_macros_declare_scc():
    for name in MACROS:
        assert _macro_has_scc(name), name


def test_routine_temporaries_stay_clear_of_the_tree_loop():
    """The hand-written prefetching tree loop (jit_template.hip
    SR_JIT_LOOP_PF_TEXT) keeps the next tree's code offset in s23 and its LDS
    addresses in v30 / v31 across every tree-code call: no routine may use them
    as temporaries (round 5: a LogCosh routine that did faulted the GPU). A
    loss routine may borrow s23 only saved to and restored from a VGPR lane."""
    hdr = (CSRC / "gen" / "jit_layout_r4.h").read_text()
    m = re.search(r"// routine VGPR temps v0\.\.v(\d+), SGPR temps \[([0-9, ]*)\]", hdr)
    assert m, "layout header lost its temporaries line"
    assert int(m.group(1)) < 30
    assert max(int(s) for s in m.group(2).split(",")) < 23
    inc = (CSRC / "gen" / "jit_routines_r4.inc").read_text()
    lines = re.findall(r'^\s*"([^"\n]*)\\n"', inc, re.M)
    bodies, cur = {}, None
    for ln in lines:
        m = re.match(r"(sr_rt_(?:fast|prec)_\w+):$", ln)
        if m:
            cur = m.group(1)
            bodies[cur] = []
        elif cur and not ln.startswith((".globl", ".L", ".p2align", ".fill")):
            bodies[cur].append(ln)
    assert len(bodies) > 50
    borrowed = 0
    for name, body in bodies.items():
        uses = [ln for ln in body if re.search(r"\bs23\b", ln)]
        if not uses:
            continue
        borrowed += 1
        # saved first, restored last, from the same lane
        assert re.match(r"v_writelane_b32 (v\d+), s23, (\d+)$", uses[0]), (name, uses[0])
        v, lane = re.match(r"v_writelane_b32 (v\d+), s23, (\d+)$", uses[0]).groups()
        assert uses[-1] == f"v_readlane_b32 s23, {v}, {lane}", (name, uses[-1])
        # the loss routines, and the gradient forward's sin / cos with the reverse factor (u_*_pd:
        # two large-argument reductions inline), compiled with LOSS_PINNED_S held live
        assert name.startswith(("sr_rt_fast_l_", "sr_rt_prec_l_", "sr_rt_fast_d_", "sr_rt_prec_d_",
                                "sr_rt_fast_u_sin_pd", "sr_rt_prec_u_sin_pd", "sr_rt_fast_u_cos_pd",
                                "sr_rt_prec_u_cos_pd", "sr_rt_fast_g_", "sr_rt_prec_g_")), name
    assert borrowed <= 12


def test_float64_routine_temporaries_stay_clear_of_the_tree_loop():
    """The hand-written Float64 tree loop (jit64_template.hip
    SR_JIT64_LOOP_TEXT) keeps its state in s46..s57, s60/s61, s[88:89],
    s[94:95] and v88/v89 across every call (round 5: LogCosh / LogitDist
    routines with temporaries up to s51 sent its tree walk astray)."""
    hdr = (CSRC / "gen" / "jit64_layout.h").read_text()
    m = re.search(r"// routine VGPR temps \[([0-9, ]*)\], SGPR temps \[([0-9, ]*)\]", hdr)
    assert m, "layout header lost its temporaries line"
    assert max(int(v) for v in m.group(1).split(",")) < 88
    assert max(int(s) for s in m.group(2).split(",")) < 46
    clob = re.search(r"#define SR_JIT64_CLOBBERS (.*)", hdr).group(1)
    for r in list(range(46, 58)) + [60, 61, 88, 89, 94, 95]:
        assert f'"s{r}"' not in clob, r
