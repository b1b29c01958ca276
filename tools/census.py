"""Per-opcode VALU budget of the loss tree code.

Compiles a batch to tree code on the CPU (srhip_jit_compile, no device),
places it in the large code-object template as the runtime does
(csrc/jit.cpp build), disassembles the image with llvm-objdump and walks
each tree's FAST main path for one interior tile: the tree code, the
routines it calls (their main path: range checks pass, no bail), the L2
tail. Instruction classes are priced with the issue costs measured by
tools/issue_rate.hip (profiles/r03a_issue_rate.txt): SIMD cycles per wave64
instruction at >= 2 waves per SIMD.

Prints the per-opcode budget (instructions and SIMD cycles per tree-tile,
summed over the batch) and a predicted kernel time:
  cycles per launch = sum over trees of cycles(tree) x tiles per row group
                      x row groups, / (1024 SIMDs x f_clk)

With --grad the gradient tree code (jit_grad.cpp) of config #5's shard is
walked instead (forward, loss, reverse pass of one interior tile; defaults
16384 trees x 20 features x 1.25M rows), routines by name, the tree's own
code split into forward ("tree") and everything after the loss ("reverse").

Usage: python tools/census.py [--ntrees 4096] [--grad] [--json out.json]
"""
import argparse
import collections
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin/"
GEN = ROOT / "symbolicregression.jl_amd" / "csrc" / "gen"

# SIMD cycles per wave64 instruction, >= 2 waves per SIMD (profiles/r03a_issue_rate.txt)
COST = {
    "pk": 4.25,      # v_pk_{add,mul,fma}_f32, v_pk_mov_b32
    "f32": 2.2,      # v_{add,sub,subrev,mul,fma,fmac}_f32 (VOP2 / VOP3), v_mov_b32, v_xor_b32, v_add_u32
    "trans": 8.1,    # v_exp/rcp/log/sqrt/rsq/sin/cos_f32: 8 cycles, NOT hidden behind other VALU
    "f64": 4.2,      # v_fma_f64, v_mul_f64, v_add_f64
    "other": 4.2,    # integer, v_max3/min3, v_cmp, v_cndmask, conversions
}
F32 = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|mac)_f32|^v_mov_b32|^v_xor_b32|^v_add_u32")
TRANS = re.compile(r"^v_(exp|rcp|log|sqrt|rsq|sin|cos)_f32")


def vclass(m):
    if m.startswith("v_pk_"):
        return "pk"
    if F32.match(m):
        return "f32"
    if TRANS.match(m):
        return "trans"
    if m.endswith("_f64") and re.match(r"^v_(fma|mul|add)_f64", m):
        return "f64"
    return "other"


def readelf_syms(path):
    out = subprocess.run([LLVM + "llvm-readelf", "-s", "--wide", str(path)], capture_output=True, text=True,
                         check=True).stdout
    syms = {}
    for ln in out.splitlines():
        p = ln.split()
        if len(p) >= 8 and p[0].endswith(":") and p[0][:-1].isdigit():
            syms[p[7]] = int(p[1], 16)
    return syms


def text_section(path):
    out = subprocess.run([LLVM + "llvm-readelf", "-S", "--wide", str(path)], capture_output=True, text=True,
                         check=True).stdout
    for ln in out.splitlines():
        m = re.search(r"\]\s+\.text\s+PROGBITS\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", ln)
        if m:
            return int(m.group(1), 16), int(m.group(2), 16)
    raise SystemExit("no .text")


def disassemble(path):
    out = subprocess.run([LLVM + "llvm-objdump", "-d", "--mcpu=gfx950", str(path)], capture_output=True, text=True,
                         check=True).stdout
    ins = {}
    for ln in out.splitlines():
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):\s*([0-9A-F ]+?)\s*(<.*>)?$", ln)
        if m:
            words = m.group(3).split()
            ins[int(m.group(2), 16)] = (m.group(1).strip(), 4 * len(words), int(words[0], 16))
    return ins


BYPLACE = collections.Counter()


def walk(ins, entry, fast0, names=None, attrib=None, max_steps=100000, grad_split=False, epi=None):
    """One interior tile of one tree: (prologue counts, tile counts).
    attrib (Counter) collects SIMD cycles per routine name / 'tree'. With epi
    (a Counter) the walk goes on after the tile loop and counts the tree's
    epilogue there."""
    pro, tile = collections.Counter(), collections.Counter()
    where = ["tree"]
    cur = pro
    pc = entry
    scc = False
    sreg = {79: 1, 68: 0}  # fastok = 1, unweighted
    ret_stack = []
    tile_start = None
    prev_cmp_tile = False
    steps = 0
    while steps < max_steps:
        steps += 1
        txt, size, word0 = ins[pc]
        m = txt.split()[0]
        nxt = pc + size
        ops = txt[len(m):].replace(",", " ").split()
        if m.startswith("v_") or m.startswith("ds_"):
            cur[m] += 1
            if attrib is not None and cur is tile and m.startswith("v_"):
                attrib[where[-1]] += COST[vclass(m)]
                BYPLACE[(where[-1], m)] += 1
        else:
            cur["S:" + m] += 1
        if m == "s_mov_b32" and ops[0].startswith("s") and ops[0][1:].isdigit():
            try:
                sreg[int(ops[0][1:])] = int(ops[1], 0)
            except ValueError:
                pass
        if m == "s_cselect_b32":
            d = int(ops[0][1:])
            sreg[d] = int(ops[1], 0) if scc else int(ops[2], 0)
        if m.startswith("s_cmp"):
            a, b = ops[0], ops[1]
            def val(x):
                if x.startswith("s[") or not x.startswith("s"):
                    try:
                        return int(x, 0)
                    except ValueError:
                        return 0
                return sreg.get(int(x[1:]), None)
            if m == "s_cmp_ge_u32" and a == "s64":
                scc = False  # tiles remain
                prev_cmp_tile = True
            elif m == "s_cmp_lt_u32" and a == "s64":
                if epi is None:
                    scc = True   # loop back: the tile ends here
                    return pro, tile
                scc = False  # the last tile: walk on through the tree's epilogue
                cur = epi
            elif m == "s_cmp_eq_u32" and a == "s82":
                scc = False  # not the last tile
            elif m == "s_cmp_lg_u64":
                scc = False  # no bail
            else:
                va, vb = val(a), val(b)
                if va is None or vb is None:
                    scc = False
                elif m == "s_cmp_eq_u32":
                    scc = va == vb
                elif m == "s_cmp_lg_u32":
                    scc = va != vb
                else:
                    scc = False
        if m == "s_andn2_b64" and ops[1] == "exec":
            scc = False  # a routine's range check passes
        if m in ("s_cbranch_scc1", "s_cbranch_scc0", "s_branch", "s_cbranch_vccnz", "s_cbranch_vccz",
                 "s_cbranch_execz", "s_cbranch_execnz"):
            off = word0 & 0xffff
            off = off - 0x10000 if off & 0x8000 else off  # simm16, in dwords
            target = nxt + 4 * off
            take = {"s_cbranch_scc1": scc, "s_cbranch_scc0": not scc, "s_branch": True,
                    "s_cbranch_vccnz": False, "s_cbranch_vccz": True, "s_cbranch_execz": False,
                    "s_cbranch_execnz": True}[m]
            pc = target if take else nxt
            if tile_start is None and prev_cmp_tile:
                tile_start = pc  # the tile label follows the `tiles remain` test
                cur = tile
            prev_cmp_tile = False
            continue
        if m == "s_swappc_b64":
            # target: s[74:75] = base + offset (FAST region)
            ret_stack.append(nxt)
            pc = call_target
            where.append(names.get(call_target, hex(call_target)) if names else "routine")
            continue
        if m == "s_add_u32" and ops[0] == "s74" and ops[1] == "s86":
            call_target = fast0 + int(ops[2], 0)
        if grad_split and m == "s_cmp_eq_u32" and ops[0] == "s68" and where == ["tree"]:
            where[0] = "reverse"  # the loss tail: everything after it is loss + reverse pass
        if m == "s_setpc_b64":
            if ret_stack:
                pc = ret_stack.pop()
                where.pop()
                continue
            return pro, tile  # the tree returned (failed or done)
        if m == "s_endpgm":
            return pro, tile
        pc = nxt
    raise RuntimeError("walk did not finish")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntrees", type=int, default=0)
    ap.add_argument("--seed", type=int, default=-1)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--nfeat", type=int, default=0)
    ap.add_argument("--grad", action="store_true", help="the gradient tree code of config #5's shard")
    ap.add_argument("--fclk", type=float, default=2.4e9)
    ap.add_argument("--json", default="")
    ap.add_argument("--by-place", action="store_true", help="per routine / tree-code opcode counts")
    args = ap.parse_args()
    dflt = dict(ntrees=16384, seed=5, rows=1_250_000, nfeat=20) if args.grad else \
        dict(ntrees=4096, seed=1000, rows=1_000_000, nfeat=5)
    for k, v in dflt.items():
        if getattr(args, k) in (0, -1):
            setattr(args, k, v)
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    if args.grad:  # tools/prof_grad.py's batch
        trees = srhip.random_population(args.ntrees, o, args.nfeat, np.float32, seed=args.seed)
    else:
        trees = srhip.random_population(args.ntrees, o, args.nfeat, np.float32, seed=args.seed, maxsize=30)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    tmpl = GEN / "jit_tmpl_l.hsaco"
    syms = readelf_syms(tmpl)
    taddr, toff = text_section(tmpl)
    area = syms["sr_jit_code"]
    fo = toff + (area - taddr)
    fast0 = syms["sr_rt_fast"]
    names = {v: k[len("sr_rt_fast_"):] for k, v in syms.items() if k.startswith("sr_rt_fast_")}
    attrib = collections.Counter()
    tot_tile, tot_pro, tot_epi = collections.Counter(), collections.Counter(), collections.Counter()
    per_tree = []
    # one code area at a time (a large batch fills several, as at run time)
    left = list(range(len(trees)))
    ncomp = 0
    while left:
        sub = srhip.flatten([trees[t] for t in left], o, dtype=np.float32)
        code, _, offs = srhip.engine.jit_compile(sub, fast=True, grad=args.grad)
        if not offs:
            break
        img = bytearray(tmpl.read_bytes())
        img[fo:fo + len(code)] = code
        with tempfile.NamedTemporaryFile(suffix=".hsaco", delete=False) as f:
            f.write(img)
            path = f.name
        ins = disassemble(path)
        for t, off in sorted(offs.items()):
            pro, tile = walk(ins, area + off, fast0, names, attrib, grad_split=args.grad, epi=tot_epi)
            tot_tile.update(tile)
            tot_pro.update(pro)
            per_tree.append(sum(COST[vclass(k)] * v for k, v in tile.items() if k.startswith("v_")))
        ncomp += len(offs)
        done = set(offs)
        left = [t for k, t in enumerate(left) if k not in done]
        if args.grad is False:
            break  # the loss code of config #2 fits one area
    offs = range(ncomp)
    nodes = int(flat.nodes.sum())
    # budget
    rows_budget = []
    tot_cyc = 0.0
    for k, v in tot_tile.most_common():
        if not k.startswith("v_"):
            continue
        c = COST[vclass(k)] * v
        tot_cyc += c
        rows_budget.append((k, vclass(k), v, c))
    print(f"{len(offs)} trees compiled, {nodes} nodes; per interior tile (256 rows) of every tree:")
    print(f"{'instruction':34s} {'class':6s} {'count':>9s} {'SIMD-cyc':>10s} {'share':>7s}")
    for k, cl, v, c in rows_budget:
        print(f"{k:34s} {cl:6s} {v:9d} {c:10.0f} {100 * c / tot_cyc:6.1f}%")
    if args.by_place:
        for (pl, m), v in sorted(BYPLACE.items(), key=lambda z: (z[0][0], -z[1])):
            print(f"  {pl:12s} {m:28s} {v:8d} {COST[vclass(m)] * v:10.0f}")
    nval = sum(v for k, v in tot_tile.items() if k.startswith("v_"))
    nsalu = sum(v for k, v in tot_tile.items() if k.startswith("S:"))
    nds = sum(v for k, v in tot_tile.items() if k.startswith("ds_"))
    by_class = collections.Counter()
    for k, cl, v, c in rows_budget:
        by_class[cl] += c
    tiles = (args.rows + 255) // 256
    pred_ms = tot_cyc * tiles / (1024 * args.fclk) * 1e3
    # VALU instructions per launch (the PMC counter's unit: wave-instructions)
    pred_valu = nval * tiles
    print("SIMD cycles by place: " + ", ".join(f"{k} {v:.0f} ({100 * v / tot_cyc:.1f}%)"
                                               for k, v in attrib.most_common()))
    print(f"VALU per tile of all trees: {nval} (ds {nds - nval if False else nds}, salu+branch {nsalu})")
    print("SIMD cycles by class: " + ", ".join(f"{k} {v:.0f} ({100 * v / tot_cyc:.1f}%)" for k, v in by_class.most_common()))
    def cyc(cn):
        return sum(COST[vclass(k)] * v for k, v in cn.items() if k.startswith("v_"))
    print(f"per call of every tree (once per row group): prologue {cyc(tot_pro):.0f} SIMD-cycles "
          f"({sum(v for k, v in tot_pro.items() if k.startswith('v_'))} VALU, "
          f"{sum(v for k, v in tot_pro.items() if k.startswith('S:'))} SALU/branch), epilogue {cyc(tot_epi):.0f} "
          f"({sum(v for k, v in tot_epi.items() if k.startswith('v_'))} VALU, "
          f"{sum(v for k, v in tot_epi.items() if k.startswith('S:'))} SALU/branch, "
          f"{tot_epi.get('S:s_nop', 0)} s_nop); per tile {tot_cyc:.0f}")
    print(f"predicted VALU-issue time for {args.rows} rows: {pred_ms:.3f} ms at f_clk {args.fclk / 1e9:.2f} GHz; "
          f"{pred_valu / 1e9:.3f}e9 VALU wave-instructions per launch (tile bodies only)")
    if args.json:
        Path(args.json).write_text(json.dumps(dict(
            ntrees=len(offs), nodes=nodes, cost_model=COST, budget=[dict(ins=k, cls=cl, count=v, cycles=c)
                                                                    for k, cl, v, c in rows_budget],
            by_class=dict(by_class), by_place=dict(attrib), predicted_ms=pred_ms, valu_per_launch=pred_valu,
            salu_per_tile=nsalu, ds_per_tile=nds), indent=1))


if __name__ == "__main__":
    main()
