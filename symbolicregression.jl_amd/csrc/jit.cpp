// jit.cpp — the tree compiler: accumulator-machine programs (compile.cpp) →
// straight-line gfx950 machine code, one block per tree, loaded per program.
//
// Why: the threaded interpreter pays, per node, a scalar record load, an
// s_setpc dispatch and an LDS read of the next X operand whether or not it is
// needed (2 KiB of LDS per wave-instruction, the LDS array's 256 B/clk is the
// bound for + - * trees: DESIGN.md §3). Tree code has none of that: values
// live in VGPR blocks chosen by a register allocator, the features a tree
// uses are read from LDS once per tile, constants are instruction literals,
// + - * neg abs square cube are single VALU instructions, every other
// operator is a routine (gen_jit.py: hipcc-compiled device_ops.h code with
// pinned registers) entered with s_swappc_b64.
//
// Tree code (R = 4 rows per lane, tiles of 256 rows, LDS layout of the driver
// in jit_template.hip): for each tile from s_tile to s_nt: read y and the
// used features, run the operators, mark the root, add the tile's L2 sum in
// the order of eval_kernel.h's tile_loss, stop at the first non-finite tile.
//
// FAST path (trees whose operators are + - * / neg abs square cube exp sin
// cos): exp / sin / cos run their Float32 routines (<= 1-2 ulp), and guards
// catch every row where that could change did_succeed against the Float64-
// evaluated routines: a cancellation |a ± b| <= 2^-14 (|a|+|b|)
// or a magnitude below 2^-120 on a transcendental-derived value that can
// make a divisor exactly 0, and |x| > 87 at exp (overflow / underflow
// thresholds). A tile whose guards fire, or that fails, is redone at once
// with the PRECISE routines (same code, call targets shifted to the PRECISE
// region); only what the PRECISE pass says is kept.
#include "jit.h"

#include <elf.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "jit_asm.h"

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw Error(SRHIP_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));  \
  } while (0)

namespace srhip {
namespace jit {
namespace {

using namespace detail;


// ---- IR ------------------------------------------------------------------------
enum { O_VAL = 0, O_X = 1, O_C = 2 };
struct Opnd {
  int k = O_VAL;
  int v = -1;        // value id (O_VAL) or feature (O_X)
  uint32_t c = 0;    // constant bits (O_C)
  int pc = -1;       // O_C: the program instruction whose immediate holds it (memory-constant code)
  bool der = false;  // O_X: a derived column (v is its column, not a dataset feature)
};
struct IrOp {
  bool un = false;
  int op = 0;
  Opnd a, b;
  int rid = -1;      // routine, -1: inline
  int krid = -1;     // constant-operand routine variant (constant in s_k), -1: none
  bool taint = false, zs = false;
  int consumer = -1, cpos = 0;
};

constexpr uint32_t kFastUops = (1u << SRHIP_UOP_NEG) | (1u << SRHIP_UOP_ABS) | (1u << SRHIP_UOP_SQUARE) |
                               (1u << SRHIP_UOP_CUBE) | (1u << SRHIP_UOP_EXP) | (1u << SRHIP_UOP_SIN) |
                               (1u << SRHIP_UOP_COS);
constexpr uint32_t kFastBops = (1u << SRHIP_BOP_ADD) | (1u << SRHIP_BOP_SUB) | (1u << SRHIP_BOP_MUL) |
                               (1u << SRHIP_BOP_DIV);

bool is_inline(const IrOp& o) {
  return o.un ? (o.op == SRHIP_UOP_NEG || o.op == SRHIP_UOP_ABS || o.op == SRHIP_UOP_SQUARE || o.op == SRHIP_UOP_CUBE)
              : (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB || o.op == SRHIP_BOP_MUL);
}

uint32_t fbits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

// Derived columns of a build (jit.h Columns): the column of u(x_f), -1 when
// u(x_f) is not derived
// the loss routine of the tile tail can hand a tile back (the Float32
// Periodic routine's Cody-Waite range, gen_jit.py)
bool loss_bails(int loss) {
  return loss > SRHIP_LOSS_L2 && loss < SRHIP_NUM_LOSSES && kLossRoutine[loss] >= 0 && kRoutineTrig[kLossRoutine[loss]];
}

struct DerivedMap {
  const Columns* cols = nullptr;
  // shared-subtree columns (Columns::gkey): key -> g, column gbase + g of the
  // tree code; empty: none (memory-constant or per-row output code)
  std::unordered_map<std::string, int> gidx;
  int gbase = 1 << 30;
  void set_shared(const Columns& c) {
    gidx.clear();
    for (int g = 0; g < c.ngcol; ++g) gidx.emplace(c.gkey[g], g);
    gbase = c.gbase();
  }
  int col(int op, int f) const {
    if (!cols) return -1;
    const uint32_t key = ((uint32_t)op << 16) | (uint32_t)f;
    for (int k = 0; k < cols->nder; ++k)
      if (cols->der[k] == key) return cols->nraw + k;
    return -1;
  }
};

// operators that tree code runs as routines (the derivable ones)
bool is_routine_uop(int op) {
  return !(op == SRHIP_UOP_NEG || op == SRHIP_UOP_ABS || op == SRHIP_UOP_SQUARE || op == SRHIP_UOP_CUBE);
}

// Program (compile.cpp) → IR: the accumulator machine with register renaming;
// u(x_f) of a derived column becomes a read of that column.
bool build_ir(const Ins<float>* p, std::vector<IrOp>& ops, Opnd& root, const DerivedMap* dm = nullptr) {
  ops.clear();
  Opnd acc, tmp, slot[kMaxSlots];
  for (int pc = 0;; ++pc) {
    if (pc > 4096) return false;
    const uint32_t code = p[pc].code;
    const int opc = (int)(code & 0xffu);
    const int f = (int)(code >> 16);
    const float imm = p[pc].imm;
    auto X = [&](int ff) { Opnd o; o.k = O_X; o.v = ff; return o; };
    auto C = [&](float c) { Opnd o; o.k = O_C; o.c = fbits(c); o.pc = pc; return o; };
    auto val = [&](IrOp o) {
      ops.push_back(o);
      Opnd r; r.k = O_VAL; r.v = (int)ops.size() - 1;
      return r;
    };
    if (opc == OP_END) { root = acc; return true; }
    if (opc == OP_LDX) { acc = X(f); continue; }
    if (opc == OP_LDC) { acc = C(imm); continue; }
    if (opc >= OP_PUSH0 && opc < OP_PUSH0 + kMaxSlots) { slot[opc - OP_PUSH0] = acc; continue; }
    if (opc >= OP_POP0 && opc < OP_POP0 + kMaxSlots) { tmp = slot[opc - OP_POP0]; continue; }
    if (opc >= OP_UN0 && opc < OP_BIN0) {
      if (dm && acc.k == O_X && !acc.der) {
        const int c = dm->col(opc - OP_UN0, acc.v);
        if (c >= 0) { acc = X(c); acc.der = true; continue; }
      }
      IrOp o; o.un = true; o.op = opc - OP_UN0; o.a = acc;
      if (acc.k != O_VAL && !(o.un && is_inline(o) && acc.k == O_X)) {
        // a unary operator on a leaf (only with constant folding off): keep it simple
        if (acc.k == O_C) return false;
      }
      acc = val(o);
      continue;
    }
    const int v = (opc - OP_BIN0) / SRHIP_NUM_BOPS;
    const int b = (opc - OP_BIN0) % SRHIP_NUM_BOPS;
    IrOp o; o.un = false; o.op = b;
    uint32_t g;
    std::memcpy(&g, &imm, 4);
    switch (v) {
      case V_AX: o.a = acc; o.b = X(f); break;
      case V_XA: o.a = X(f); o.b = acc; break;
      case V_AC: o.a = acc; o.b = C(imm); break;
      case V_CA: o.a = C(imm); o.b = acc; break;
      case V_AT: o.a = acc; o.b = tmp; break;
      case V_TA: o.a = tmp; o.b = acc; break;
      case V_XX: o.a = X(f); o.b = X((int)g); break;
      case V_XC: o.a = X(f); o.b = C(imm); break;
      case V_CX: o.a = C(imm); o.b = X(f); break;
      default: return false;
    }
    if (o.a.k == O_C && o.b.k == O_C) return false;
    acc = val(o);
  }
}

// ---- shared subtrees (jit.h Columns::gkey) -----------------------------------------
// The canonical text of an IR value's subtree in raw features, e.g.
// "b3(u11(x3),x0)" for cos(x4) / x1 (an LDS-derived column spelled as its
// u(x_f)), or "" when the subtree reads a constant: constants differ from
// tree to tree, so only constant-free subtrees are shared.
static std::string leaf_key(const Opnd& q, const Columns* cols) {
  if (q.k != O_X) return "";
  if (!q.der) return "x" + std::to_string(q.v);
  if (cols && q.v >= cols->nraw && q.v < cols->nraw + cols->nder) {
    const uint32_t d = cols->der[q.v - cols->nraw];
    return "u" + std::to_string(d >> 16) + "(x" + std::to_string(d & 0xffffu) + ")";
  }
  return "";  // a shared-subtree column (keys are taken before the substitution)
}
// Per value: its key, and the SIMD cycles per 256-row tile that its subtree's
// operators cost as FAST tree code and as PRECISE code (tools/census.py's
// prices: a routine ~120 FAST, ~260 PRECISE; + - * neg abs square cube ~8),
// its postfix stack depth and whether it holds a routine.
struct SubtreeInfo {
  std::vector<std::string> key;
  std::vector<int> fast, precise, depth;
  std::vector<char> routine;
};
static void subtree_keys(const std::vector<IrOp>& ops, const Columns* cols, SubtreeInfo& si) {
  const size_t n = ops.size();
  si.key.assign(n, std::string());
  si.fast.assign(n, 0);
  si.precise.assign(n, 0);
  si.depth.assign(n, 1);
  si.routine.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const IrOp& o = ops[i];
    const bool inl = is_inline(o);
    int f = inl ? 8 : 120, p = inl ? 8 : 260;
    bool r = !inl;
    auto part = [&](const Opnd& q, int* d) {
      *d = 1;
      if (q.k != O_VAL) {
        if (q.k == O_X && q.der) *d = 2;  // u(x_f): feature then operator
        return leaf_key(q, cols);
      }
      f += si.fast[q.v];
      p += si.precise[q.v];
      r = r || si.routine[q.v];
      *d = si.depth[q.v];
      return si.key[q.v];
    };
    int da = 1, db = 0;
    const std::string ka = part(o.a, &da);
    if (ka.empty()) continue;
    if (o.un) {
      si.key[i] = "u" + std::to_string(o.op) + "(" + ka + ")";
    } else {
      const std::string kb = part(o.b, &db);
      if (kb.empty()) continue;
      // + and * commute exactly in IEEE arithmetic: one key for both orders
      const bool comm = o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_MUL;
      si.key[i] = "b" + std::to_string(o.op) + "(" + (comm && kb < ka ? kb + "," + ka : ka + "," + kb) + ")";
    }
    si.fast[i] = f;
    si.precise[i] = p;
    si.routine[i] = r;
    si.depth[i] = o.un ? da : std::max(da, db + 1);
  }
}
// The postfix node stream (srhip_trees kinds / args, raw features) of a value.
static void subtree_postfix(const std::vector<IrOp>& ops, const Opnd& q, const Columns* cols,
                            std::vector<uint8_t>& kind, std::vector<uint16_t>& arg) {
  if (q.k == O_X) {
    if (!q.der) {
      kind.push_back(SRHIP_NODE_FEATURE);
      arg.push_back((uint16_t)q.v);
    } else {
      const uint32_t d = cols->der[q.v - cols->nraw];
      kind.push_back(SRHIP_NODE_FEATURE);
      arg.push_back((uint16_t)(d & 0xffffu));
      kind.push_back(SRHIP_NODE_UNARY);
      arg.push_back((uint16_t)(d >> 16));
    }
    return;
  }
  const IrOp& o = ops[q.v];
  subtree_postfix(ops, o.a, cols, kind, arg);
  if (!o.un) subtree_postfix(ops, o.b, cols, kind, arg);
  kind.push_back(o.un ? SRHIP_NODE_UNARY : SRHIP_NODE_BINARY);
  arg.push_back((uint16_t)o.op);
}
// Every maximal shared subtree of the IR becomes a read of its column (O_X,
// der, column gbase + g); the operations that only it used are dropped.
// Returns false (IR unchanged) when the tree holds none.
static bool substitute_shared(std::vector<IrOp>& ops, Opnd& root, const DerivedMap& dm) {
  if (dm.gidx.empty()) return false;
  SubtreeInfo si;
  subtree_keys(ops, dm.cols, si);
  bool any = false;
  std::vector<char> live(ops.size(), 0);
  std::function<void(Opnd&)> rw = [&](Opnd& q) {
    if (q.k != O_VAL) return;
    if (!si.key[q.v].empty()) {
      auto it = dm.gidx.find(si.key[q.v]);
      if (it != dm.gidx.end()) {
        Opnd x;
        x.k = O_X;
        x.v = dm.gbase + it->second;
        x.der = true;
        q = x;
        any = true;
        return;
      }
    }
    live[q.v] = 1;
    IrOp& o = ops[q.v];
    rw(o.a);
    if (!o.un) rw(o.b);
  };
  rw(root);
  if (!any) return false;
  std::vector<int> nid(ops.size(), -1);
  std::vector<IrOp> out;
  for (size_t i = 0; i < ops.size(); ++i) {
    if (!live[i]) continue;
    IrOp o = ops[i];
    if (o.a.k == O_VAL) o.a.v = nid[o.a.v];
    if (!o.un && o.b.k == O_VAL) o.b.v = nid[o.b.v];
    nid[i] = (int)out.size();
    out.push_back(o);
  }
  if (root.k == O_VAL) root.v = nid[root.v];
  ops.swap(out);
  return true;
}

// ---- code generation of one tree --------------------------------------------------
struct Gen {
  Asm& as;
  const Tmpl& T;
  uint64_t base_va;     // address of this tree's first instruction
  bool fast_opt;
  std::vector<IrOp> ops;
  Opnd root;
  bool fast = false;    // this tree has a guarded FAST path
  bool g_can = false, g_min = false, g_exp = false, g_trig = false, has_trig = false, has_call = false;
  // allocation state
  enum { L_NONE = -1, L_A = 100, L_B = 101 };
  std::vector<int> loc;          // per value
  int pool_owner[NPOOL];         // -1 free, value id, or 1000 + feature
  int a_owner = -1, b_owner = -1;
  int xblk[256];
  int xlast[256];
  bool xinl[256];                // feature read by an inline operator or as the root
  bool xdirect = false;          // call operands that are features: ds_read straight into A / B
  std::vector<int> feats;        // features in first-use order
  int load_idx[256];             // load number (0 = y)
  int nloads = 0, waited = 0;
  std::vector<int> next_call;    // first call index > i
  int L_tile = -1, L_done = -1, L_redo = -1, L_bail = -1;
  std::string why;
  bool out = false;              // per-row output code (Options::out)
  int out_rreg = -1;             // the root block of the tile (out mode)
  // shared-subtree columns (jit.h Columns): O_X columns from gbase on are read
  // from device memory — s[36:37] = column 0 at this row group's first row,
  // s38 = the column stride in bytes (the driver's, jit_template.hip) — with
  // one global load each at the tile start; gwaited: their vmcnt wait is done
  int gbase = 1 << 30;
  bool gwaited = true;
  // the global loads of the tile in issue order: column f is load gidx[f] of
  // gnum; loads return in issue order (gfx9 vmcnt), so its wait is
  // vmcnt(gnum - 1 - gidx[f]) and later columns may still be in flight
  int gidx[256];
  int gnum = 0, gdone = 0;
  bool gany = false;   // the tree reads shared-subtree columns
  // SRHIP_JIT_GPREFETCH=1 (read per build): the next tile's column loads
  // issued at the end of the current one instead of at its start; measured
  // no faster (config #2 2.589 vs 2.563 ms, interleaved, profiles/r06_ab_build1.jsonl)
  bool gprefetch = [] { const char* e = std::getenv("SRHIP_JIT_GPREFETCH"); return e && e[0] == '1'; }();
  int L_reload = -1;   // issue this tile's column loads, then the tile (a FAST redo)
  // The column loads of tile S_TILE into their pool blocks (xblk): issued
  // before the tile runs — for the first tile in the prologue, for the next
  // one at the end of the current tile (their latency under its tail and the
  // next tile's LDS reads) — and again before a redone tile.
  void emit_gloads() {
    as.vop2(VOP2_LSHLREV_B32, "v_lshlrev_b32_e32", VGT, K(2), VLANE4);  // lane·16
    as.sop2(SOP2_LSHL_B32, "s_lshl_b32", 0, S(S_TILE), K(10));         // tile·1024
    as.sop2(SOP2_ADD_U32, "s_add_u32", 0, S(S_GCOL), S(0));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", 1, S(S_GCOL + 1), K(0));
    for (size_t j = 0; j < feats.size(); ++j) {
      const int f = feats[j];
      if (!is_g(f)) continue;
      const uint32_t g = (uint32_t)(f - gbase);
      int sb = 0;
      if (g > 0) {
        as.sop2(SOP2_MUL_I32, "s_mul_i32", 2, S(S_GSTRIDE), K(g));
        as.sop2(SOP2_MUL_HI_U32, "s_mul_hi_u32", 3, S(S_GSTRIDE), K(g));
        as.sop2(SOP2_ADD_U32, "s_add_u32", 2, S(0), S(2));
        as.sop2(SOP2_ADDC_U32, "s_addc_u32", 3, S(1), S(3));
        sb = 2;
      }
      as.global_load_dwordx4(VPOOL0 + R * (int)j, VGT, sb, 0);
    }
  }
  static constexpr int S_GCOL = 36, S_GSTRIDE = 38;
  bool is_g(int v) const { return v >= gbase; }

  // SRHIP_JIT_TRIG_FULL=1 (tests): sin / cos through the complete compiled
  // routines instead of the hand-scheduled FAST bodies
  bool trig_full = false;
  // SRHIP_JIT_MANUAL=0 (tests): sin, cos, exp and / through the compiled
  // routines instead of the hand-scheduled packed bodies (gen_jit.py manual_*)
  bool manual_off = false;
  bool off_exp = false, off_trig = false, off_div = false;
  static int div_rk() {
    static const int r = [] {
      for (int k = 0; k < kNumRoutines; ++k)
        if (std::string(kRoutineName[k]) == "b_div_rk") return k;
      return -1;
    }();
    return r;
  }
  static int full_routine(int rid) {
    const std::string want = std::string(kRoutineName[rid]) + "_full";
    for (int k = 0; k < kNumRoutines; ++k)
      if (want == kRoutineName[k]) return k;
    return rid;
  }
  bool inline_ok = false;  // copy mode-independent small routines into the tree code
  // + - * (and square / cube, residuals, the root check) two rows per
  // instruction on v_pk_*_f32; block moves on v_pk_mov_b32
  bool packed = true, pkmov = true;
  // memory-constant code (Options::memc): every constant operand is an SGPR
  // s[SC0 + k], loaded in the prologue from the immediate of its program
  // instruction (s[SPROG:SPROG+1] = the tree's program in device memory), so
  // srhip_program_set_constants' in-place program update is all a new
  // constant set needs
  static constexpr int SC0 = 24, NSC = 16, SPROG = 56;
  bool memc = false;
  int loss = SRHIP_LOSS_L2;       // the tile tail's elementwise loss (Options::loss)
  uint64_t lparam = 0;            // its Float64 parameter's bits
  std::vector<int> cpcs;          // program instruction of constant slot k
  int cslot(const Opnd& q) {
    for (size_t k = 0; k < cpcs.size(); ++k)
      if (cpcs[k] == q.pc) return (int)k;
    cpcs.push_back(q.pc);
    return (int)cpcs.size() - 1;
  }
  int creg(const Opnd& q) const {
    for (size_t k = 0; k < cpcs.size(); ++k)
      if (cpcs[k] == q.pc) return SC0 + (int)k;
    throw Error(SRHIP_ERR_INVALID, "jit: constant without a slot");
  }
  Gen(Asm& a, const Tmpl& t, uint64_t va, bool f) : as(a), T(t), base_va(va), fast_opt(f) {
    const char* e = std::getenv("SRHIP_JIT_INLINE");  // measured no faster: off by default
    inline_ok = e && e[0] == '1';
    const char* xd = std::getenv("SRHIP_JIT_XDIRECT");
    xdirect = !(xd && xd[0] == '0');  // measured 1 % faster on config #2
    const char* pk = std::getenv("SRHIP_JIT_PACKED");
    packed = !(pk && pk[0] == '0');
    const char* pm = std::getenv("SRHIP_JIT_PKMOV");
    pkmov = !(pm && pm[0] == '0');
    const char* tf = std::getenv("SRHIP_JIT_TRIG_FULL");
    trig_full = tf && tf[0] == '1';
    const char* mo = std::getenv("SRHIP_JIT_MANUAL");
    manual_off = mo && mo[0] == '0';
    // SRHIP_JIT_MANUAL_OFF=exp,trig,div (debugging): only these through the compiled routines
    if (const char* mf = std::getenv("SRHIP_JIT_MANUAL_OFF")) {
      const std::string l(mf);
      off_exp = l.find("exp") != std::string::npos;
      off_trig = l.find("trig") != std::string::npos;
      off_div = l.find("div") != std::string::npos;
    }
  }

  uint64_t cur_va() const { return base_va + as.bytes(); }
  // sin / cos of a value that carries FAST rounding: the result's phase error
  // grows with |x| (a 1-ulp change of x = 2^14 moves it by 2^-9), so such
  // arguments are guarded like a cancellation
  static bool trig_guard_on() {  // SRHIP_JIT_TRIG_GUARD=0 (experiments): no such guard
    static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_TRIG_GUARD"); return !(e && e[0] == '0'); }();
    return on;
  }
  bool trig_of_tainted(const IrOp& o) const {
    static const bool zs_only = [] { const char* e = std::getenv("SRHIP_JIT_TRIG_GUARD_ZS"); return e && e[0] == '1'; }();
    return o.un && (o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS) && o.a.k == O_VAL && ops[o.a.v].taint &&
           (o.zs || !zs_only);
  }
  // Loss-parity guards (round 4; thresholds from
  // tools/fast_guard_sim.py): FAST rounding in a value that reaches a divisor
  // is amplified without bound near the divisor's zeros, and those rows carry
  // most of the loss (a 1/d pole: the relative loss error grows like ε/d_min).
  // A sin / cos of a FAST-derived u on a divisor path redoes the tile when
  // |result| < 2^-k·|u| (its relative condition |u·tan u| above 2^k), as a
  // cancellation does (|a ± b| <= 2^-k (|a| + |b|)), k = SRHIP_JIT_CAN_LOG2
  // (default 7); an exp of a FAST-derived u when |u| > 16 (relative error
  // amplified |u|-fold); a sin / cos of a FAST-derived u when |u| > 2^10
  // (absolute error |u|·ε).
  static bool loss_guards_on() {  // SRHIP_JIT_LOSS_GUARDS=0 (experiments): the round-3 guards only
    static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_LOSS_GUARDS"); return !(e && e[0] == '0'); }();
    return on;
  }
  static uint32_t can_eps_bits() {  // 2^-k
    static const uint32_t b = [] {
      const char* e = std::getenv("SRHIP_JIT_CAN_LOG2");
      const int k = e ? std::max(1, std::min(100, std::atoi(e))) : (loss_guards_on() ? 7 : 14);
      return (uint32_t)(127 - k) << 23;
    }();
    return b;
  }
  static uint32_t exp_scale_bits() {  // 87 / 2^k, k = SRHIP_JIT_EXP_GUARD_LOG2 (default 4: |x| > 16)
    static const uint32_t b = [] {
      const char* e = std::getenv("SRHIP_JIT_EXP_GUARD_LOG2");
      const int k = e ? std::max(0, std::min(6, std::atoi(e))) : 4;
      return fbits(87.0f / (float)(1 << k));
    }();
    return b;
  }
  bool trig_small(const IrOp& o) const { return loss_guards_on() && trig_of_tainted(o) && o.zs; }
  bool exp_tainted(const IrOp& o) const {
    return loss_guards_on() && o.un && o.op == SRHIP_UOP_EXP && o.a.k == O_VAL && ops[o.a.v].taint;
  }
  int reg_of_loc(int l) const { return l == L_A ? VA : l == L_B ? VB : VPOOL0 + R * l; }

  bool analyze() {
    const int n = (int)ops.size();
    // routines, consumers
    for (int i = 0; i < n; ++i) {
      IrOp& o = ops[i];
      if (!is_inline(o)) {
        o.rid = o.un ? kUopRoutine[o.op] : kBopRoutine[o.op];
        if (o.rid < 0) { why = "operator without routine"; return false; }
        if (trig_full && o.un && (o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS)) o.rid = full_routine(o.rid);
        if (manual_off && ((o.un && (o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS || o.op == SRHIP_UOP_EXP)) ||
                           (!o.un && o.op == SRHIP_BOP_DIV)))
          o.rid = full_routine(o.rid);
        if ((off_exp && o.un && o.op == SRHIP_UOP_EXP) || (off_trig && o.un && (o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS)) ||
            (off_div && !o.un && o.op == SRHIP_BOP_DIV))
          o.rid = full_routine(o.rid);
        has_call = true;
        // a constant operand rides in s_k: the routine variant takes the other one in A
        if (!o.un && o.b.k == O_C && o.a.k != O_C && kBopRoutineRC[o.op] >= 0) o.krid = kBopRoutineRC[o.op];
        if (!o.un && o.a.k == O_C && o.b.k != O_C && kBopRoutineLC[o.op] >= 0) o.krid = kBopRoutineLC[o.op];
        if ((manual_off || off_div) && o.krid >= 0 && !o.un && o.op == SRHIP_BOP_DIV) o.krid = full_routine(o.krid);
        if (kRoutineTrig[o.rid]) has_trig = true;
      }
      for (int s = 0; s < 2; ++s) {
        const Opnd& q = s ? o.b : o.a;
        if (s && o.un) break;
        if (q.k == O_VAL) { ops[q.v].consumer = i; ops[q.v].cpos = s; }
      }
    }
    // a loss routine that hands a tile back (Float32 Periodic beyond its Cody-Waite range)
    if (!out && loss_bails(loss)) has_trig = true;
    if (memc) {
      cpcs.clear();
      for (const IrOp& o : ops) {
        if (o.a.k == O_C) cslot(o.a);
        if (!o.un && o.b.k == O_C) cslot(o.b);
      }
      if (root.k == O_C) cslot(root);
      for (const IrOp& o : ops)
        if ((o.a.k == O_C && o.a.pc < 0) || (!o.un && o.b.k == O_C && o.b.pc < 0)) { why = "constant without a program slot"; return false; }
      if ((int)cpcs.size() > NSC) { why = "more constants than memory-constant SGPRs"; return false; }
    }
    // FAST eligibility, taint, zero sensitivity
    bool elig = fast_opt, trans = false;
    for (auto& o : ops) {
      if (o.un ? !((kFastUops >> o.op) & 1u) : !((kFastBops >> o.op) & 1u)) elig = false;
      if (o.un && (o.op == SRHIP_UOP_EXP || o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS)) trans = true;
    }
    fast = elig && trans;
    for (int i = 0; i < n; ++i) {
      IrOp& o = ops[i];
      o.taint = o.un && (o.op == SRHIP_UOP_EXP || o.op == SRHIP_UOP_SIN || o.op == SRHIP_UOP_COS);
      if (o.a.k == O_VAL && ops[o.a.v].taint) o.taint = true;
      if (!o.un && o.b.k == O_VAL && ops[o.b.v].taint) o.taint = true;
    }
    for (int i = n - 1; i >= 0; --i) {
      IrOp& o = ops[i];
      auto mark = [&](const Opnd& q) {
        if (q.k == O_VAL) ops[q.v].zs = true;
      };
      if (!o.un) {
        if (o.op == SRHIP_BOP_DIV) {
          mark(o.b);
          if (o.zs) mark(o.a);
        } else if (o.zs && (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB || o.op == SRHIP_BOP_MUL)) {
          mark(o.a);
          mark(o.b);
        }
      } else if (o.zs && (o.op == SRHIP_UOP_NEG || o.op == SRHIP_UOP_ABS || o.op == SRHIP_UOP_SQUARE ||
                          o.op == SRHIP_UOP_CUBE || o.op == SRHIP_UOP_SIN)) {
        mark(o.a);
      }
    }
    if (fast) {
      for (auto& o : ops) {
        if (o.un && o.op == SRHIP_UOP_EXP) g_exp = true;
        if (trig_of_tainted(o) && trig_guard_on()) g_trig = true;
        if (trig_small(o)) g_can = true;  // its guard shares the cancellation accumulator
        if (o.taint && o.zs) {
          if (!o.un && (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB)) g_can = true;
          if ((!o.un && (o.op == SRHIP_BOP_MUL || o.op == SRHIP_BOP_DIV)) ||
              (o.un && (o.op == SRHIP_UOP_SQUARE || o.op == SRHIP_UOP_CUBE)))
            g_min = true;
        }
      }
    }
    // features: first use order, last use
    for (int f = 0; f < 256; ++f) { xblk[f] = -1; xlast[f] = -1; load_idx[f] = -1; xinl[f] = false; }
    auto usef = [&](const Opnd& q, int i) {
      if (q.k != O_X) return true;
      if (q.v < 0 || q.v > 255) return false;
      if (xlast[q.v] < 0) feats.push_back(q.v);
      xlast[q.v] = i;
      return true;
    };
    for (int i = 0; i < n; ++i) {
      if (!usef(ops[i].a, i)) return false;
      if (!ops[i].un && !usef(ops[i].b, i)) return false;
      if (ops[i].rid < 0 || !xdirect) {
        if (ops[i].a.k == O_X) xinl[ops[i].a.v] = true;
        if (!ops[i].un && ops[i].b.k == O_X) xinl[ops[i].b.v] = true;
      }
    }
    if (!usef(root, n)) return false;
    if (root.k == O_X) xinl[root.v] = true;
    for (int f : feats)
      if (is_g(f)) xinl[f] = true;  // a shared-subtree column is loaded once, at the tile start
    {
      std::vector<int> pre;
      for (int f : feats)
        if (xinl[f]) pre.push_back(f);
      feats = pre;  // the features preloaded into register blocks at the tile start
    }
    if ((int)feats.size() > NPOOL) { why = "more features than register blocks"; return false; }
    for (int f : feats)
      if (!is_g(f) && (1 + f) * TILE * 4 + 3 * 4 * 64 > 65535) { why = "feature offset beyond the DS immediate"; return false; }
    next_call.assign(n + 1, n);
    for (int i = n - 1; i >= 0; --i) next_call[i] = ops[i].rid >= 0 ? i : next_call[i + 1];
    loc.assign(n, L_NONE);
    return true;
  }

  // ---- emission helpers ----
  Src opsrc(const Opnd& q, int e) const {
    if (q.k == O_C) return memc ? S(creg(q)) : K(q.c);
    if (q.k == O_X) return V(VPOOL0 + R * xblk[q.v] + e);
    return V(reg_of_loc(loc[q.v]) + e);
  }
  bool opnd_is_vgpr(const Opnd& q) const { return q.k != O_C; }

  void wait_for(const Opnd& q) {
    if (q.k != O_X) return;
    if (is_g(q.v)) {
      const int k = gidx[q.v];
      if (k >= gdone) {
        as.waitcnt_vm(gnum - 1 - k);
        gdone = k + 1;
        gwaited = gdone == gnum;
      }
      return;
    }
    const int li = load_idx[q.v];
    if (li >= waited) {
      as.waitcnt_lgkm(nloads - 1 - li);
      waited = li + 1;
    }
  }
  void wait_all() {
    if (waited < nloads) {
      as.waitcnt_lgkm(0);
      waited = nloads;
    }
    if (!gwaited) { as.waitcnt_vm(0); gwaited = true; gdone = gnum; }
  }
  int free_block() const {
    for (int k = 0; k < NPOOL; ++k)
      if (pool_owner[k] == -1) return k;
    return -1;
  }
  void mov_block(int dst, const Src (&src)[R]) {
    bool blk = src[0].enc >= 256;
    for (int e = 1; e < R; ++e) blk = blk && src[e].enc == src[0].enc + e;
    if (blk) { mov_block_reg(dst, src[0].enc - 256); return; }
    for (int e = 0; e < R; ++e) as.vop1(VOP1_MOV, "v_mov_b32_e32", dst + e, src[e]);
  }
  void mov_block_reg(int dst, int srcreg) {
    if (pkmov) {
      for (int e = 0; e < R; e += 2)
        as.vop3p(VOP3P_MOV_B32, "v_pk_mov_b32", dst + e, V(srcreg + e), V(srcreg + e), nullptr, 2, 7, 0, 0);
      return;
    }
    for (int e = 0; e < R; ++e) as.vop1(VOP1_MOV, "v_mov_b32_e32", dst + e, V(srcreg + e));
  }
  // a source of a packed instruction for rows e, e+1: a VGPR pair, an inline
  // constant, or the constant in s[20:21] (pk_const puts it there first)
  static Src pks(const Src& s) { return s.lit ? S(S_PKC) : s; }
  void pk_const(const Src& s) {
    if (s.lit) as.sop1(SOP1_MOV, "s_mov_b32", S_PKC, K(s.val), "s" + std::to_string(S_PKC));
  }
  // block d = a (op) b, two rows per instruction; a constant feeds both halves
  void pk_block(int opc, const char* nm, int d, const Src (&a)[R], const Src (&b)[R], bool negb) {
    pk_const(a[0]);
    pk_const(b[0]);
    int hi = 4 | (a[0].enc >= 256 ? 1 : 0) | (b[0].enc >= 256 ? 2 : 0), lo = 0;
    // a constant in an odd SGPR (memory-constant code): the aligned pair below it, high half to both lanes
    auto odd = [&](const Src& x, int bit) {
      if (x.enc < 102 && !x.lit && (x.enc & 1)) { lo |= bit; hi |= bit; return S(x.enc - 1); }
      return pks(x);
    };
    for (int e = 0; e < R; e += 2) {
      const Src pa = odd(a[e], 1), pb = odd(b[e], 2);
      as.vop3p(opc, nm, d + e, pa, pb, nullptr, lo, hi, negb ? 2 : 0, negb ? 2 : 0);
    }
  }
  // a call operand into block `dst` (A or B): features not preloaded (or all
  // of them with xdirect) are read from the LDS tile, other operands moved
  bool load_x_direct(const Opnd& q) const { return q.k == O_X && !is_g(q.v) && (xdirect || xblk[q.v] < 0); }
  void operand_to(int dst, const Opnd& q, bool* issued) {
    if (load_x_direct(q)) {
      as.ds_read_b128(dst, VLANE, (1 + q.v) * TILE * 4);
      ++nloads;
      *issued = true;
      return;
    }
    Src sq[R];
    for (int e = 0; e < R; ++e) sq[e] = opsrc(q, e);
    mov_block(dst, sq);
  }
  void wait_direct(bool issued) {
    if (issued) { as.waitcnt_lgkm(0); waited = nloads; }
  }

  // value v leaves its location (its last use)
  void release_val(int v) {
    const int l = loc[v];
    if (l == L_A) { if (a_owner == v) a_owner = -1; }
    else if (l == L_B) { if (b_owner == v) b_owner = -1; }
    else if (l >= 0 && pool_owner[l] == v) pool_owner[l] = -1;
  }
  void release_x(int f, int i) {
    if (xlast[f] == i && xblk[f] >= 0 && pool_owner[xblk[f]] == 1000 + f) pool_owner[xblk[f]] = -1;
  }
  bool evict(int owner_slot_loc, int keep_a, int keep_b) {
    int& own = owner_slot_loc == L_A ? a_owner : b_owner;
    if (own < 0 || own == keep_a || own == keep_b) return true;
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted (evict)"; return false; }
    mov_block_reg(VPOOL0 + R * k, owner_slot_loc == L_A ? VA : VB);
    pool_owner[k] = own;
    loc[own] = k;
    own = -1;
    return true;
  }

  // s[86:87] = the FAST routine region (set once per tree entry); a PRECISE
  // tile adds the region offset D to it, the next FAST tile takes it off
  void set_base() {
    as.sop1(SOP1_GETPC, "s_getpc_b64", S_BASE, Src{0, false, 0}, "");
    if (as.want_text) as.lines.back() = "s_getpc_b64 s[" + std::to_string(S_BASE) + ":" + std::to_string(S_BASE + 1) + "]";
    const uint64_t pc_next = cur_va();
    const int64_t rel = (int64_t)(T.fast0 - pc_next);
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_BASE, S(S_BASE), K((uint32_t)(uint64_t)rel));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", S_BASE + 1, S(S_BASE + 1), K((uint32_t)((uint64_t)rel >> 32)));
  }
  void shift_base(bool up) {
    as.sop2(up ? SOP2_ADD_U32 : SOP2_SUB_U32, up ? "s_add_u32" : "s_sub_u32", S_BASE, S(S_BASE), K((uint32_t)T.delta));
    as.sop2(up ? SOP2_ADDC_U32 : SOP2_SUBB_U32, up ? "s_addc_u32" : "s_subb_u32", S_BASE + 1, S(S_BASE + 1), K(0));
  }
  void call_routine(int rid) {
    static const size_t inline_max = [] {  // SRHIP_JIT_INLINE_MAX: only bodies up to this many bytes
      const char* e = std::getenv("SRHIP_JIT_INLINE_MAX");
      return e ? (size_t)std::atoi(e) : (size_t)1 << 30;
    }();
    if (inline_ok && !T.body[rid].empty() && T.body[rid].size() * 4 <= inline_max) {  // a copy of the body
      for (uint32_t w : T.body[rid]) as.raw(w);
      as.sopp(0x00, "s_nop", 0);  // a trans result read right after the body
      return;
    }
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_TGT, S(S_BASE), K((uint32_t)(T.rt_va[rid] - T.fast0)));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", S_TGT + 1, S(S_BASE + 1), K(0));
    as.sop1(SOP1_SWAPPC, "s_swappc_b64", S_RR, S(S_TGT), "s[" + std::to_string(S_RR) + ":" + std::to_string(S_RR + 1) + "]");
    if (as.want_text)
      as.lines.back() = "s_swappc_b64 s[" + std::to_string(S_RR) + ":" + std::to_string(S_RR + 1) + "], s[" +
                        std::to_string(S_TGT) + ":" + std::to_string(S_TGT + 1) + "]";
    if (kRoutineTrig[rid]) {
      as.sopc(SOPC_LG_U64, "s_cmp_lg_u64", S(S_FLAG), K(0),
              "s[" + std::to_string(S_FLAG) + ":" + std::to_string(S_FLAG + 1) + "]");
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_bail);
    }
  }

  bool emit_call(int i) {
    IrOp& o = ops[i];
    if (o.krid >= 0) return emit_call_k(i);
    const int va_ = o.a.k == O_VAL ? o.a.v : -1;
    const int vb_ = (!o.un && o.b.k == O_VAL) ? o.b.v : -1;
    wait_for(o.a);
    if (!o.un) wait_for(o.b);
    // routines keep B: a unary call leaves its owner there
    if (!evict(L_A, va_, vb_) || (!o.un && !evict(L_B, va_, vb_))) return false;
    // move the operands into A (lhs) and B (rhs)
    const int la = va_ >= 0 ? loc[va_] : L_NONE;
    const int lb = vb_ >= 0 ? loc[vb_] : L_NONE;
    bool issued = false;
    if (o.un) {
      if (la != L_A) operand_to(VA, o.a, &issued);
    } else if (la == L_B && lb == L_A) {
      mov_block_reg(VGT, VA);
      mov_block_reg(VA, VB);
      mov_block_reg(VB, VGT);
    } else if (la == L_B) {
      mov_block_reg(VA, VB);
      operand_to(VB, o.b, &issued);
    } else if (lb == L_A) {
      mov_block_reg(VB, VA);
      operand_to(VA, o.a, &issued);
    } else {
      if (la != L_A) operand_to(VA, o.a, &issued);
      if (lb != L_B) operand_to(VB, o.b, &issued);
    }
    wait_direct(issued);
    // the operands are consumed
    if (va_ >= 0) release_val(va_);
    if (vb_ >= 0) release_val(vb_);
    if (o.a.k == O_X) release_x(o.a.v, i);
    if (!o.un && o.b.k == O_X) release_x(o.b.v, i);
    a_owner = -1;
    if (!o.un) b_owner = -1;
    if (fast && o.un && o.op == SRHIP_UOP_EXP) {  // max |x| over the rows, two per instruction
      // a FAST-derived x counts 87/16 times its size: |x| > 16 fires the 87 check
      int src = VA;
      if (exp_tainted(o)) {
        Src a4[R], k4[R];
        for (int e = 0; e < R; ++e) { a4[e] = V(VA + e); k4[e] = K(exp_scale_bits()); }  // 87/16 = 5.4375
        pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", VGT, a4, k4, false);
        src = VGT;
      }
      for (int e = 0; e < R; e += 2) {
        const Src g = V(VGEXP), x0 = V(src + e), x1 = V(src + e + 1);
        as.vop3(VOP3_MAX3_F32, "v_max3_f32", VGEXP, g, x0, &x1, 6, 0);
      }
    }
    if (fast && g_trig && trig_of_tainted(o))
      for (int e = 0; e < R; e += 2) {
        const Src g = V(VGTRIG), x0 = V(VA + e), x1 = V(VA + e + 1);
        as.vop3(VOP3_MAX3_F32, "v_max3_f32", VGTRIG, g, x0, &x1, 6, 0);
      }
    const bool tsmall = fast && trig_small(o);
    if (tsmall) mov_block_reg(VGT, VA);  // u, for the condition check after the call
    call_routine(o.rid);
    loc[i] = L_A;
    a_owner = i;
    if (tsmall) {  // fires when 2^-k·|u| - |sin/cos u| > 0 (or NaN)
      for (int e = 0; e < R; ++e) {
        const Src u = V(VGT + e), eps = S(S_EPS), r = V(VA + e);
        as.vop3(VOP3_FMA_F32, "v_fma_f32", VGT + e, u, eps, &r, 5, 4);
      }
      for (int e = 0; e < R; e += 2) {
        const Src g = V(VGCAN), t0 = V(VGT + e), t1 = V(VGT + e + 1);
        as.vop3(VOP3_MAX3_F32, "v_max3_f32", VGCAN, g, t0, &t1, 0, 0);
      }
    }
    if (fast && o.taint && o.zs && !o.un && o.op == SRHIP_BOP_DIV) guard_min(VA);
    return true;
  }

  // a binary operator with one constant operand: the constant in s_k, the
  // other operand in A, B untouched
  bool emit_call_k(int i) {
    IrOp& o = ops[i];
    const bool kr = o.b.k == O_C;
    const Opnd& q = kr ? o.a : o.b;
    const int vq = q.k == O_VAL ? q.v : -1;
    wait_for(q);
    if (!evict(L_A, vq, -1)) return false;
    const int lq = vq >= 0 ? loc[vq] : L_NONE;
    if (lq != L_A) {
      bool issued = false;
      operand_to(VA, q, &issued);
      wait_direct(issued);
    }
    if (vq >= 0) release_val(vq);
    if (q.k == O_X) release_x(q.v, i);
    if (vq >= 0 && lq == L_B) b_owner = -1;
    a_owner = -1;
    const uint32_t cb = kr ? o.b.c : o.a.c;
    if (memc) as.sop1(SOP1_MOV, "s_mov_b32", S_K, S(creg(kr ? o.b : o.a)), "s" + std::to_string(S_K));
    else as.sop1(SOP1_MOV, "s_mov_b32", S_K, K(cb), "s" + std::to_string(S_K));
    int rid = o.krid;
    float cf;
    std::memcpy(&cf, &cb, 4);
    const float ac = std::fabs(cf);
    // (memory-constant code: the constant may change, so no host reciprocal)
    if (!memc && kr && o.op == SRHIP_BOP_DIV && div_rk() >= 0 && ac >= 0x1p-60f && ac <= 0x1p60f) {
      // the reciprocal-and-correction routine (IEEE exact for admitted a; gen_jit.py manual_div_rk)
      const volatile float one = 1.0f;
      const float y = one / cf;  // correctly rounded (SSE division, no contraction)
      uint32_t yb;
      std::memcpy(&yb, &y, 4);
      as.sop1(SOP1_MOV, "s_mov_b32", S_RECIP, K(yb), "s" + std::to_string(S_RECIP));
      rid = div_rk();
    }
    call_routine(rid);
    loc[i] = L_A;
    a_owner = i;
    if (fast && o.taint && o.zs && o.op == SRHIP_BOP_DIV) guard_min(VA);
    return true;
  }

  void guard_min(int reg) {
    for (int e = 0; e < R; e += 2) {
      const Src g = V(VGMIN), x0 = V(reg + e), x1 = V(reg + e + 1);
      as.vop3(VOP3_MIN3_F32, "v_min3_f32", VGMIN, g, x0, &x1, 6, 0);
    }
  }

  bool emit_inline(int i) {
    IrOp& o = ops[i];
    wait_for(o.a);
    if (!o.un) wait_for(o.b);
    const bool gcan = fast && o.taint && o.zs && !o.un && (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB);
    const bool gmin = fast && o.taint && o.zs &&
                      ((!o.un && o.op == SRHIP_BOP_MUL) || (o.un && (o.op == SRHIP_UOP_SQUARE || o.op == SRHIP_UOP_CUBE)));
    if (gcan) {  // t = |a| + |b| before the operands are overwritten
      Src ka, kb;
      for (const Opnd* q : {&o.a, &o.b}) {
        if (q->k != O_C) continue;
        if (memc) as.sop2(SOP2_AND_B32, "s_and_b32", S_K, S(creg(*q)), K(0x7fffffffu));
        else as.sop1(SOP1_MOV, "s_mov_b32", S_K, K(q->c & 0x7fffffffu), "s" + std::to_string(S_K));
      }
      for (int e = 0; e < R; ++e) {
        ka = o.a.k == O_C ? S(S_K) : opsrc(o.a, e);
        kb = o.b.k == O_C ? S(S_K) : opsrc(o.b, e);
        as.vop3(VOP3_ADD_F32, "v_add_f32_e64", VGT + e, ka, kb, nullptr, 3, 0);
      }
    }
    // operand registers (read below), then release dying operands
    Src a[R], b[R];
    for (int e = 0; e < R; ++e) {
      a[e] = opsrc(o.a, e);
      if (!o.un) b[e] = opsrc(o.b, e);
    }
    const int va_ = o.a.k == O_VAL ? o.a.v : -1;
    const int vb_ = (!o.un && o.b.k == O_VAL) ? o.b.v : -1;
    int freed = -1;
    auto rel = [&](int v) {
      if (v < 0) return;
      const int l = loc[v];
      release_val(v);
      if (l >= 0 && freed < 0) freed = l;
    };
    rel(va_);
    rel(vb_);
    if (o.a.k == O_X) { const int k = xblk[o.a.v]; release_x(o.a.v, i); if (pool_owner[k] == -1 && freed < 0) freed = k; }
    if (!o.un && o.b.k == O_X) { const int k = xblk[o.b.v]; release_x(o.b.v, i); if (pool_owner[k] == -1 && freed < 0) freed = k; }
    // destination: the operand block of the consuming routine when no call
    // comes in between, else a freed or free pool block
    int dst = L_NONE;
    if (o.consumer >= 0 && ops[o.consumer].rid >= 0 && next_call[i + 1] == o.consumer) {
      const bool lhs = o.cpos == 0 || ops[o.consumer].krid >= 0;
      if (lhs && a_owner < 0) dst = L_A;
      if (!lhs && b_owner < 0) dst = L_B;
    }
    if (dst == L_NONE) dst = freed >= 0 ? freed : free_block();
    if (dst == L_NONE) { why = "register pool exhausted"; return false; }
    const int d = reg_of_loc(dst);
    const bool ca = o.a.k == O_C, cb = !o.un && o.b.k == O_C;
    const bool pk_bin = packed && !o.un && !(ca && cb) &&
                        (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB || o.op == SRHIP_BOP_MUL);
    const bool pk_un = packed && o.un && !ca && (o.op == SRHIP_UOP_SQUARE || o.op == SRHIP_UOP_CUBE);
    if (pk_bin) {
      if (o.op == SRHIP_BOP_MUL) pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", d, a, b, false);
      else pk_block(VOP3P_ADD_F32, "v_pk_add_f32", d, a, b, o.op == SRHIP_BOP_SUB);
    } else if (pk_un) {
      if (o.op == SRHIP_UOP_SQUARE) {
        pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", d, a, a, false);
      } else {  // CUBE = (x*x)*x
        const int tt = (d == a[0].enc - 256) ? VGT : d;
        Src t2[R];
        for (int e = 0; e < R; ++e) t2[e] = V(tt + e);
        pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", tt, a, a, false);
        pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", d, t2, a, false);
      }
    }
    for (int e = 0; e < R && !pk_bin && !pk_un; ++e) {
      if (o.un) {
        switch (o.op) {
          case SRHIP_UOP_NEG: as.vop2(VOP2_XOR_B32, "v_xor_b32_e32", d + e, K(0x80000000u), a[e].enc - 256); break;
          case SRHIP_UOP_ABS: as.vop2(VOP2_AND_B32, "v_and_b32_e32", d + e, K(0x7fffffffu), a[e].enc - 256); break;
          case SRHIP_UOP_SQUARE: as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", d + e, a[e], a[e].enc - 256); break;
          default: {  // CUBE = (x*x)*x
            const int tt = (d + e == a[e].enc - 256) ? VGT + e : d + e;
            as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", tt, a[e], a[e].enc - 256);
            as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", d + e, V(tt), a[e].enc - 256);
          }
        }
      } else {
        switch (o.op) {
          case SRHIP_BOP_ADD:
          case SRHIP_BOP_MUL: {
            const int opc = o.op == SRHIP_BOP_ADD ? VOP2_ADD_F32 : VOP2_MUL_F32;
            const char* nm = o.op == SRHIP_BOP_ADD ? "v_add_f32_e32" : "v_mul_f32_e32";
            if (cb) as.vop2(opc, nm, d + e, b[e], a[e].enc - 256);
            else as.vop2(opc, nm, d + e, a[e], b[e].enc - 256);
            break;
          }
          default:  // SUB
            if (cb) as.vop2(VOP2_SUBREV_F32, "v_subrev_f32_e32", d + e, b[e], a[e].enc - 256);
            else if (ca) as.vop2(VOP2_SUB_F32, "v_sub_f32_e32", d + e, a[e], b[e].enc - 256);
            else as.vop2(VOP2_SUB_F32, "v_sub_f32_e32", d + e, a[e], b[e].enc - 256);
        }
      }
    }
    if (o.un && (o.a.k == O_C)) { why = "unary operator on a constant"; return false; }
    loc[i] = dst;
    if (dst == L_A) a_owner = i;
    else if (dst == L_B) b_owner = i;
    else pool_owner[dst] = i;
    if (gcan) {
      for (int e = 0; e < R; ++e) {
        const Src t_ = V(VGT + e), eps = S(S_EPS), r = V(d + e);
        as.vop3(VOP3_FMA_F32, "v_fma_f32", VGT + e, t_, eps, &r, 4, 4);
      }
      for (int e = 0; e < R; e += 2) {
        const Src g = V(VGCAN), t0 = V(VGT + e), t1 = V(VGT + e + 1);
        as.vop3(VOP3_MAX3_F32, "v_max3_f32", VGCAN, g, t0, &t1, 0, 0);
      }
    }
    if (gmin) guard_min(d);
    return true;
  }

  bool emit_tree(const std::vector<IrOp>& ir, const Opnd& rt) {
    ops = ir;
    root = rt;
    if (!analyze()) return false;
    for (int k = 0; k < NPOOL; ++k) pool_owner[k] = -1;
    L_tile = as.label();
    L_done = as.label();
    L_redo = as.label();
    L_bail = as.label();
    const uint32_t D = (uint32_t)T.delta;
    // ---- prologue
    as.sop1(SOP1_MOV, "s_mov_b32", S_STATUS, K(0), "s" + std::to_string(S_STATUS));
    for (size_t k = 0; k < cpcs.size(); ++k) {  // memory-constant code: s_load_dword s[SC0+k], the immediate
      const uint32_t off = (uint32_t)cpcs[k] * 8u + 4u;
      as.put(0xc0020000u | ((uint32_t)(SC0 + k) << 6) | (uint32_t)(SPROG >> 1));
      as.put(off);
      if (as.want_text)
        as.lines.push_back("s_load_dword s" + std::to_string(SC0 + k) + ", s[" + std::to_string(SPROG) + ":" +
                           std::to_string(SPROG + 1) + "], " + hex32(off));
    }
    if (!cpcs.empty()) as.waitcnt_lgkm(0);
    if (g_can) as.sop1(SOP1_MOV, "s_mov_b32", S_EPS, K(can_eps_bits()), "s" + std::to_string(S_EPS));  // 2^-k
    if (has_call) set_base();
    if (fast) {
      as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_FASTOK), K(0));
      as.sop2(SOP2_CSELECT, "s_cselect_b32", S_MODE, K(1), K(0));
      as.sop2(SOP2_CSELECT, "s_cselect_b32", S_K, K(D), K(0));
      as.sop2(SOP2_ADD_U32, "s_add_u32", S_BASE, S(S_BASE), S(S_K));
      as.sop2(SOP2_ADDC_U32, "s_addc_u32", S_BASE + 1, S(S_BASE + 1), K(0));
    } else {
      as.sop1(SOP1_MOV, "s_mov_b32", S_MODE, K(1), "s" + std::to_string(S_MODE));
      if (has_call) shift_base(true);
    }
    as.sopc(SOPC_GE_U32, "s_cmp_ge_u32", S(S_TILE), S(S_NT));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_done);
    // the pool blocks of the preloaded features and columns (first-use order),
    // the columns' load order
    gany = false;
    gnum = 0;
    for (size_t j = 0; j < feats.size(); ++j) {
      xblk[feats[j]] = (int)j;
      if (is_g(feats[j])) { gany = true; gidx[feats[j]] = gnum++; }
    }
    if (gany && gprefetch) {
      L_reload = as.label();
      as.bind(L_reload);
      emit_gloads();
    }
    // ---- tile
    as.bind(L_tile);
    if (gany && !gprefetch) emit_gloads();  // each tile issues its own column loads
    if (fast || has_trig) as.vop1(VOP1_MOV, "v_mov_b32_e32", VCHKSAVE, V(VCHK));  // for a redo / bail
    if (g_can) as.vop1(VOP1_MOV, "v_mov_b32_e32", VGCAN, K(0xbf800000u));   // -1
    if (g_min) as.vop1(VOP1_MOV, "v_mov_b32_e32", VGMIN, K(0x3f800000u));   // 1
    if (g_exp) as.vop1(VOP1_MOV, "v_mov_b32_e32", VGEXP, K(0));
    if (g_trig) as.vop1(VOP1_MOV, "v_mov_b32_e32", VGTRIG, K(0));
    a_owner = b_owner = -1;
    for (int k = 0; k < NPOOL; ++k) pool_owner[k] = -1;
    nloads = 0;
    waited = 0;
    if (!out) {  // y (no y column in out mode)
      as.ds_read_b128(VY, VLANE, 0);
      ++nloads;
    }
    for (size_t j = 0; j < feats.size(); ++j) {
      const int f = feats[j];
      pool_owner[j] = 1000 + f;
      if (is_g(f)) continue;  // in flight since the tile's column loads (emit_gloads)
      load_idx[f] = nloads++;
      as.ds_read_b128(VPOOL0 + R * (int)j, VLANE, (1 + f) * TILE * 4);
    }
    gwaited = !gany;
    gdone = 0;
    std::fill(loc.begin(), loc.end(), (int)L_NONE);
    for (int i = 0; i < (int)ops.size(); ++i) {
      if (ops[i].rid >= 0) { if (!emit_call(i)) return false; }
      else if (!emit_inline(i)) return false;
    }
    // root value
    int rreg;
    if (root.k == O_VAL) rreg = reg_of_loc(loc[root.v]);
    else if (root.k == O_X) { wait_for(root); rreg = VPOOL0 + R * xblk[root.v]; }
    else {
      for (int e = 0; e < R; ++e) as.vop1(VOP1_MOV, "v_mov_b32_e32", VGT + e, memc ? S(creg(root)) : K(root.c));
      rreg = VGT;
    }
    if (packed && rreg != VGT) {
      // (r0, r1)·0 + (r2, r3) is finite iff the four rows are: one packed fma, two into chk
      const Src r01 = V(rreg), r23 = V(rreg + 2), z = K(0);
      as.vop3p(VOP3P_FMA_F32, "v_pk_fma_f32", VGT, r01, z, &r23, 0, 5, 0, 0);
      for (int e = 0; e < 2; ++e) {
        const Src r = V(VGT + e), c = V(VCHK);
        as.vop3(VOP3_FMA_F32, "v_fma_f32", VCHK, r, z, &c, 0, 0);
      }
    } else {
      for (int e = 0; e < R; ++e) {
        const Src r = V(rreg + e), z = K(0), c = V(VCHK);
        as.vop3(VOP3_FMA_F32, "v_fma_f32", VCHK, r, z, &c, 0, 0);
      }
    }
    wait_all();
    if (out) {  // out mode: the root block is stored by emit_tail_out
      out_rreg = rreg;
      return true;
    }
    // ---- FAST-mode verdict: a failure or a guard redoes the tile precisely
    if (fast) {
      const int L_skip = as.label();
      as.sopc(SOPC_LG_U32, "s_cmp_lg_u32", S(S_MODE), K(0));
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_skip);
      as.vopc(VOPC_U_F32, "v_cmp_u_f32_e32", V(VCHK), VCHK);
      as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_redo);
      // the guards fire on NaN too: a FAST exp of an argument the exp guard
      // rejects returns garbage, possibly a signalling NaN, which poisons the
      // max3 / min3 accumulators of later guards (v_max3 of an sNaN is NaN)
      if (g_can) {
        as.vopc(VOPC_NGT_F32, "v_cmp_ngt_f32_e32", K(0), VGCAN);  // !(0 > max): a cancellation or NaN
        as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_redo);
      }
      if (g_min) {
        as.vopc(VOPC_NLE_F32, "v_cmp_nle_f32_e32", K(0x03800000u), VGMIN);  // !(2^-120 <= min|v|)
        as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_redo);
      }
      if (g_exp) {
        as.vopc(VOPC_NGE_F32, "v_cmp_nge_f32_e32", K(0x42ae0000u), VGEXP);  // !(87 >= max|x|)
        as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_redo);
      }
      if (g_trig) {
        static const uint32_t lim = [] {  // 2^k, k = SRHIP_JIT_TRIG_GUARD_LOG2 (default 14)
          const char* e = std::getenv("SRHIP_JIT_TRIG_GUARD_LOG2");
          const int k = e ? std::max(1, std::min(100, std::atoi(e))) : (loss_guards_on() ? 10 : 14);
          return (uint32_t)(127 + k) << 23;
        }();
        as.vopc(VOPC_NGE_F32, "v_cmp_nge_f32_e32", K(lim), VGTRIG);  // !(2^k >= max|x|)
        as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_redo);
      }
      as.bind(L_skip);
    }
    // ---- L2 loss of the tile: the residuals here, their squares in emit_tail
    if (packed) {
      Src r[R], y[R];
      for (int e = 0; e < R; ++e) { r[e] = V(rreg + e); y[e] = V(VY + e); }
      pk_block(VOP3P_ADD_F32, "v_pk_add_f32", VY, r, y, true);
    } else {
      for (int e = 0; e < R; ++e) as.vop2(VOP2_SUB_F32, "v_sub_f32_e32", VY + e, V(rreg + e), VY + e);
    }
    return true;
  }

  // second half of the tile: weights (s_woff != 0), mask, sums, loop
  // the last, partial tile: rows past `partial` add 0 (block `reg` zeroed there)
  void emit_mask(int reg) {
    const int L_nomask = as.label();
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_PE, S(S_TILE), K(1));
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_PE), S(S_NT));
    as.branch(SOPP_SCC0, "s_cbranch_scc0", L_nomask);
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_PARTIAL), K((uint32_t)TILE));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_nomask);
    for (int e = 0; e < R; ++e) {
      as.sop2(SOP2_SUB_I32, "s_sub_i32", S_PE, S(S_PARTIAL), K((uint32_t)e));
      as.vopc(VOPC_GT_I32, "v_cmp_gt_i32_e32", S(S_PE), VLANE4);
      as.sopp(0x00, "s_nop", 1);  // VALU-written VCC read as a VALU mask: 2 wait states
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", reg + e, K(0), reg + e, ", vcc");
    }
    as.bind(L_nomask);
  }

  // call a routine of the PRECISE region whatever the mode (the loss: the
  // interpreter's elem_loss in Float64-evaluated form, bit for bit)
  void call_precise(int rid) {
    as.sop1(SOP1_GETPC, "s_getpc_b64", S_TGT, Src{0, false, 0}, "");
    if (as.want_text) as.lines.back() = "s_getpc_b64 s[" + std::to_string(S_TGT) + ":" + std::to_string(S_TGT + 1) + "]";
    const uint64_t pc_next = cur_va();
    const int64_t rel = (int64_t)(T.rt_va[rid] + T.delta - pc_next);
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_TGT, S(S_TGT), K((uint32_t)(uint64_t)rel));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", S_TGT + 1, S(S_TGT + 1), K((uint32_t)((uint64_t)rel >> 32)));
    as.sop1(SOP1_SWAPPC, "s_swappc_b64", S_RR, S(S_TGT), "s[" + std::to_string(S_RR) + ":" + std::to_string(S_RR + 1) + "]");
    if (as.want_text)
      as.lines.back() = "s_swappc_b64 s[" + std::to_string(S_RR) + ":" + std::to_string(S_RR + 1) + "], s[" +
                        std::to_string(S_TGT) + ":" + std::to_string(S_TGT + 1) + "]";
  }

  // the tile tail of a loss other than L2: ℓ(r) of the residual block VY by
  // the loss routine, weighted, masked and summed as eval_kernel.h's
  // tile_loss does ((ℓ0 + ℓ2) + (ℓ1 + ℓ3)), then the loop
  void emit_tail_loss() {
    mov_block_reg(VA, VY);
    as.sop1(SOP1_MOV, "s_mov_b32", S_K, K((uint32_t)lparam), "s" + std::to_string(S_K));
    as.sop1(SOP1_MOV, "s_mov_b32", S_KH, K((uint32_t)(lparam >> 32)), "s" + std::to_string(S_KH));
    call_precise(kLossRoutine[loss]);
    if (loss_bails(loss)) {  // a row beyond the routine's range: the tree goes back to the interpreter
      as.sopc(SOPC_LG_U64, "s_cmp_lg_u64", S(S_FLAG), K(0),
              "s[" + std::to_string(S_FLAG) + ":" + std::to_string(S_FLAG + 1) + "]");
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_bail);
    }
    mov_block_reg(VY, VA);
    const int L_unw = as.label(), L_sum = as.label();
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_WOFF), K(0));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", VGT, S(S_WOFF), VLANE);
    as.ds_read_b128(VGT, VGT, 0);
    as.waitcnt_lgkm(0);
    {
      Src y[R], w[R];
      for (int e = 0; e < R; ++e) { y[e] = V(VY + e); w[e] = V(VGT + e); }
      if (packed) pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", VY, w, y, false);
      else for (int e = 0; e < R; ++e) as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", VY + e, V(VGT + e), VY + e);
    }
    as.bind(L_unw);
    emit_mask(VY);
    as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY, V(VY), VY + 2);
    as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY + 1, V(VY + 1), VY + 3);
    as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY, V(VY), VY + 1);
    as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VLSUM, V(VLSUM), VY);
    as.bind(L_sum);
  }

  // out mode: the tile's root block to the tree's output rows (lane ℓ holds
  // rows 4ℓ .. 4ℓ+3 of the tile: one coalesced 1 KiB global_store_dwordx4 per
  // wave at s[S_OUT:S_OUT+1] + 16ℓ), then the next tile's rows. Rows past the
  // last are written too: they lie in the output's padding (stride n_pad).
  void emit_store_out() {
    const int voff = VGCAN;  // free without the FAST path: 16ℓ
    as.vop2(VOP2_LSHLREV_B32, "v_lshlrev_b32_e32", voff, K(2), VLANE4);
    as.put(0xdc7c8000u);  // global_store_dwordx4 voff, v[rreg:rreg+3], s[S_OUT:S_OUT+1]
    as.put((uint32_t)voff | ((uint32_t)out_rreg << 8) | ((uint32_t)S_OUT << 16));
    if (as.want_text)
      as.lines.push_back("global_store_dwordx4 v" + std::to_string(voff) + ", v[" + std::to_string(out_rreg) + ":" +
                         std::to_string(out_rreg + 3) + "], s[" + std::to_string(S_OUT) + ":" +
                         std::to_string(S_OUT + 1) + "]");
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_OUT, S(S_OUT), K((uint32_t)(TILE * 4)));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", S_OUT + 1, S(S_OUT + 1), K(0));
  }

  // second half of the tile: squares (weighted when s_woff != 0), mask, sums, loop
  void emit_tail() {
    if (out) {
      emit_store_out();
    } else if (loss != SRHIP_LOSS_L2) {
      emit_tail_loss();
    } else {
      const int L_unw = as.label(), L_sum = as.label();
      as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_WOFF), K(0));
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
      // weighted: w * r^2 per row (eval_kernel.h tile_loss), masked, then summed
      as.vop2(VOP2_ADD_U32, "v_add_u32_e32", VGT, S(S_WOFF), VLANE);
      as.ds_read_b128(VGT, VGT, 0);
      Src y[R], w[R];
      for (int e = 0; e < R; ++e) { y[e] = V(VY + e); w[e] = V(VGT + e); }
      if (packed) pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", VY, y, y, false);
      else for (int e = 0; e < R; ++e) as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", VY + e, V(VY + e), VY + e);
      as.waitcnt_lgkm(0);
      if (packed) pk_block(VOP3P_MUL_F32, "v_pk_mul_f32", VY, w, y, false);
      else for (int e = 0; e < R; ++e) as.vop2(VOP2_MUL_F32, "v_mul_f32_e32", VY + e, V(VGT + e), VY + e);
      emit_mask(VY);
      as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY, V(VY), VY + 2);
      as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY + 1, V(VY + 1), VY + 3);
      as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VY, V(VY), VY + 1);
      as.vop2(VOP2_ADD_F32, "v_add_f32_e32", VLSUM, V(VLSUM), VY);
      as.branch(SOPP_BRANCH, "s_branch", L_sum);
      // unweighted: the residuals masked, squared and accumulated by fma
      as.bind(L_unw);
      emit_mask(VY);
      for (int e = 0; e < R; ++e) {
        const Src r = V(VY + e), l = V(VLSUM);
        as.vop3(VOP3_FMA_F32, "v_fma_f32", VLSUM, r, r, &l, 0, 0);
      }
      as.bind(L_sum);
    }
    // a failed tile ends the tree (out mode: every tile is stored)
    if (!out) {
      as.vopc(VOPC_U_F32, "v_cmp_u_f32_e32", V(VCHK), VCHK);
      as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_done);
    }
    // after a redone tile the call's remaining tiles run PRECISE directly
    // (a tree whose guards fire on one tile mostly fires on the next: poles,
    // large arguments); SRHIP_JIT_STICKY=0: the next tile starts FAST again
    static const bool sticky = [] { const char* e = std::getenv("SRHIP_JIT_STICKY"); return !(e && e[0] == '0'); }();
    if (fast && !sticky) {
      const int L_keep = as.label();
      as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_FASTOK), K(0));
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_keep);
      as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(S_MODE), K(0));
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_keep);
      as.sop1(SOP1_MOV, "s_mov_b32", S_MODE, K(0), "s" + std::to_string(S_MODE));
      shift_base(false);
      as.bind(L_keep);
    }
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", VLANE, S(S_TILEBYTES), VLANE);
    as.sop2(SOP2_ADD_U32, "s_add_u32", S_TILE, S(S_TILE), K(1));
    as.sopc(SOPC_LT_U32, "s_cmp_lt_u32", S(S_TILE), S(S_NT));
    if (gany && gprefetch) {  // the next tile's column loads before it starts
      as.branch(SOPP_SCC0, "s_cbranch_scc0", L_done);
      emit_gloads();
      as.branch(SOPP_BRANCH, "s_branch", L_tile);
    } else {
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_tile);
    }
    as.bind(L_done);
    as.sop1(SOP1_SETPC, "s_setpc_b64", 0, S(S_RT), "");
    if (as.want_text) as.lines.back() = "s_setpc_b64 s[" + std::to_string(S_RT) + ":" + std::to_string(S_RT + 1) + "]";
    if (fast) {
      as.bind(L_redo);
      as.sop2(SOP2_ADD_U32, "s_add_u32", S_X0, S(S_X0), K(1));  // redo counter (driver output)
      as.vop1(VOP1_MOV, "v_mov_b32_e32", VCHK, V(VCHKSAVE));
      as.sop1(SOP1_MOV, "s_mov_b32", S_MODE, K(1), "s" + std::to_string(S_MODE));
      shift_base(true);
      as.branch(SOPP_BRANCH, "s_branch", (gany && gprefetch) ? L_reload : L_tile);  // the columns' blocks were reused
    }
    if (has_trig) {
      as.bind(L_bail);
      as.waitcnt_lgkm(0);
      if (gany) as.waitcnt_vm(0);  // no column load may land after the tree has returned
      as.vop1(VOP1_MOV, "v_mov_b32_e32", VCHK, V(VCHKSAVE));
      as.sop1(SOP1_MOV, "s_mov_b32", S_STATUS, K(1), "s" + std::to_string(S_STATUS));
      as.sop1(SOP1_SETPC, "s_setpc_b64", 0, S(S_RT), "");
      if (as.want_text) as.lines.back() = "s_setpc_b64 s[" + std::to_string(S_RT) + ":" + std::to_string(S_RT + 1) + "]";
    }
  }
};

}  // namespace

// One tree: returns false (nothing appended) when it cannot be compiled.
static bool gen_tree(const Ins<float>* prog, const Tmpl& T, bool fast_opt, bool text, std::vector<uint32_t>& out,
                     std::vector<std::string>* lines, uint64_t area_va, int32_t* off, bool* is_fast,
                     std::string* why, const DerivedMap& dm, bool memc, int loss = SRHIP_LOSS_L2,
                     uint64_t lparam = 0, bool out_mode = false) {
  std::vector<IrOp> ir;
  Opnd root;
  if (!build_ir(prog, ir, root, &dm)) { *why = "program not translatable"; return false; }
  const size_t start = (out.size() + 15) / 16 * 16;  // 64-byte aligned entries
  // shared subtrees read from their columns; a tree whose code then does not
  // fit (its columns and features exceed the register blocks) computes them
  std::vector<IrOp> ir0;
  Opnd root0 = root;
  const bool shared = !memc && !out_mode && !dm.gidx.empty();
  if (shared) ir0 = ir;
  const bool subst = shared && substitute_shared(ir, root, dm);
  Asm as;
  for (int attempt = 0;; ++attempt) {
    as = Asm();
    as.want_text = text;
    Gen g(as, T, area_va + start * 4, fast_opt && loss != SRHIP_LOSS_PERIODIC && !out_mode);
    g.out = out_mode;
    g.memc = memc;
    g.loss = loss;
    g.lparam = lparam;
    if (subst && attempt == 0) g.gbase = dm.gbase;
    if (!g.emit_tree(ir, root)) {
      if (subst && attempt == 0) {
        ir = ir0;
        root = root0;
        continue;
      }
      *why = g.why;
      return false;
    }
    g.emit_tail();
    *is_fast = g.fast;
    break;
  }
  as.finish();
  while (out.size() < start) {  // s_nop padding
    out.push_back(0xbf800000u);
    if (lines) lines->push_back("s_nop 0");
  }
  out.insert(out.end(), as.w.begin(), as.w.end());
  if (lines) {
    lines->push_back("; tree code at " + std::to_string(start * 4));
    lines->insert(lines->end(), as.lines.begin(), as.lines.end());
  }
  *off = (int32_t)(start * 4);
  return true;
}

// One loaded code object per part: a batch whose code exceeds one code area
// (8 MiB) is split into consecutive slot ranges, one launch each.
struct ModulePart {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr, fn_w = nullptr, fn_derive = nullptr;
  hipFunction_t fn_dl = nullptr, fn_dlw = nullptr;  // the hand-written tree loop (sr_jit_eval_dl / _dlm)
  hipFunction_t fn_dlp = nullptr, fn_dlpw = nullptr;  // its prefetching variant (literal code)
  int32_t* d_off = nullptr;  // [nslots] code offsets
  int slot0 = 0, nslots = 0;
};
struct Module {
  Columns cols;
  bool memc = false;
  bool bails = false;  // its tree code can hand a tree back (rerun_bailed reads the flags)
  bool out = false;  // per-row output code: fn runs sr_jit_out(_m)
  std::vector<ModulePart> parts;
  uint32_t* d_bail = nullptr;  // [nslots + 2]: bail flags of all slots, bail count, PRECISE redo count
  int nslots = 0;
};

bool available() { return templates().ok; }
// an operator routine that hands tiles back (gen_jit.py TRIG_BAIL): every module's
bool can_bail() {
  for (int k = 0; k < kNumRoutines; ++k) {
    bool is_loss = false;
    for (int l = 0; l < SRHIP_NUM_LOSSES; ++l) is_loss = is_loss || kLossRoutine[l] == k;
    if (kRoutineTrig[k] && !is_loss) return true;
  }
  return false;
}
bool module_bails(const Module* m) { return m && m->bails; }
const char* unavailable_reason() { return templates().why.c_str(); }

// Host threads for code generation (SRHIP_JIT_THREADS, default min(16,
// hardware threads); 1: serial).
static int codegen_threads() {
  static const int n = [] {
    const char* e = std::getenv("SRHIP_JIT_THREADS");
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    return e ? std::max(1, std::atoi(e)) : std::min(16, hw);
  }();
  return n;
}
template <typename F>
static void parallel_for(size_t n, F&& body) {
  const int nth = (int)std::min<size_t>((size_t)codegen_threads(), (n + 63) / 64);
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (;;) {
      const size_t b = next.fetch_add(64);
      if (b >= n) return;
      for (size_t k = b; k < std::min(n, b + 64); ++k) body(k);
    }
  };
  std::vector<std::thread> th;
  for (int i = 1; i < nth; ++i) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

// codegen on several host threads: every tree at a provisional address (its
// size does not depend on the address: the routine-base offsets are literals
// either way), the layout in order, then every placed tree again at its final
// address; the result is the serial codegen's word for word (false: a size
// changed, the caller runs the serial one).
static bool codegen_par(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, size_t from,
                        const Options& opt, std::vector<uint32_t>& words, std::vector<int32_t>& offs,
                        std::vector<int32_t>& ok_trees, std::vector<int32_t>& rest, Stats* st, const Tmpl& T,
                        const Columns& cols, size_t* stop) {
  DerivedMap dm;
  dm.cols = &cols;
  dm.set_shared(cols);
  const size_t n = cand.size() - from;
  struct R { std::vector<uint32_t> w; bool ok = false, fast = false; std::string why; size_t start = 0; };
  std::vector<R> res(n);
  parallel_for(n, [&](size_t k) {
    const int32_t t = cand[from + k];
    R& r = res[k];
    int32_t off;
    r.ok = cb.tree_off[t] >= 0 && gen_tree(&cb.code[cb.tree_off[t]], T, opt.fast, false, r.w, nullptr, T.area_va, &off,
                                           &r.fast, &r.why, dm, opt.memc, opt.loss, opt.lparam, opt.out);
  });
  size_t pos = words.size(), end = n;
  for (size_t k = 0; k < n; ++k) {
    if (!res[k].ok) continue;
    const size_t start = (pos + 15) / 16 * 16;
    if ((start + res[k].w.size()) * 4 > T.area_bytes) { end = k; break; }
    res[k].start = start;
    pos = start + res[k].w.size();
  }
  bool same = true;
  parallel_for(end, [&](size_t k) {
    R& r = res[k];
    if (!r.ok) return;
    const size_t sz = r.w.size();
    r.w.clear();
    int32_t off;
    bool f;
    std::string why;
    const int32_t t = cand[from + k];
    if (!gen_tree(&cb.code[cb.tree_off[t]], T, opt.fast, false, r.w, nullptr, T.area_va + r.start * 4, &off, &f, &why,
                  dm, opt.memc, opt.loss, opt.lparam, opt.out) ||
        r.w.size() != sz)
      same = false;
  });
  if (!same) return false;
  static const bool dbg = std::getenv("SRHIP_JIT_DEBUG") != nullptr;
  for (size_t k = 0; k < end; ++k) {
    const R& r = res[k];
    if (!r.ok) {
      rest.push_back(cand[from + k]);
      if (st) st->nrejected++;
      if (dbg) std::fprintf(stderr, "jit: tree %d not compiled: %s\n", cand[from + k], r.why.c_str());
      continue;
    }
    words.resize(r.start, 0xbf800000u);  // s_nop padding to the 64-byte entry
    words.insert(words.end(), r.w.begin(), r.w.end());
    ok_trees.push_back(cand[from + k]);
    offs.push_back((int32_t)(r.start * 4));
    if (st) { st->ntrees++; st->nfast += r.fast ? 1 : 0; }
  }
  *stop = end == n ? cand.size() : from + end;
  return true;
}

// Trees that compile are appended to ok_trees / offs, the others to `rest`; a
// tree that no longer fits in the area ends the call (returns its position in
// cand; cand.size() when all were done).
static size_t codegen(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, size_t from,
                      const Options& opt, std::vector<uint32_t>& words, std::vector<std::string>* lines,
                      std::vector<int32_t>& offs, std::vector<int32_t>& ok_trees, std::vector<int32_t>& rest,
                      Stats* st, const Tmpl& T, const Columns& cols) {
  if (!lines && cand.size() - from >= 512 && codegen_threads() > 1) {
    const size_t w0 = words.size(), o0 = offs.size(), k0 = ok_trees.size(), r0 = rest.size();
    const Stats s0 = st ? *st : Stats();
    size_t stop = 0;
    if (codegen_par(cb, cand, from, opt, words, offs, ok_trees, rest, st, T, cols, &stop)) return stop;
    words.resize(w0);  // a size changed with the address: the serial layout below
    offs.resize(o0);
    ok_trees.resize(k0);
    rest.resize(r0);
    if (st) *st = s0;
  }
  DerivedMap dm;
  dm.cols = &cols;
  dm.set_shared(cols);
  for (size_t k = from; k < cand.size(); ++k) {
    const int32_t t = cand[k];
    int32_t off = -1;
    bool f = false;
    std::string why;
    const size_t before = words.size();
    const size_t lbefore = lines ? lines->size() : 0;
    const bool okc = cb.tree_off[t] >= 0 &&
                     gen_tree(&cb.code[cb.tree_off[t]], T, opt.fast, opt.text, words, lines, T.area_va, &off, &f, &why, dm, opt.memc,
                              opt.loss, opt.lparam, opt.out);
    if (okc && words.size() * 4 > T.area_bytes) {  // area full: the next part takes it
      words.resize(before);
      if (lines) lines->resize(lbefore);
      return k;
    }
    if (okc) {
      ok_trees.push_back(t);
      offs.push_back(off);
      if (st) { st->ntrees++; st->nfast += f ? 1 : 0; }
    } else {
      words.resize(before);
      if (lines) lines->resize(lbefore);
      rest.push_back(t);
      if (st) st->nrejected++;
      static const bool dbg = std::getenv("SRHIP_JIT_DEBUG") != nullptr;
      if (dbg) std::fprintf(stderr, "jit: tree %d not compiled: %s\n", t, why.c_str());
    }
  }
  return cand.size();
}

// SRHIP_JIT_PART_GLOBAL=1 (experiments): per-tree partials always straight to global memory
bool part_global() {
  static const bool g = [] { const char* e = std::getenv("SRHIP_JIT_PART_GLOBAL"); return e && e[0] == '1'; }();
  return g;
}
bool has_loss_routine(int loss) {
  return loss == SRHIP_LOSS_L2 || (loss >= 0 && loss < SRHIP_NUM_LOSSES && kLossRoutine[loss] >= 0);
}
int choose_waves(int nraw) {
  static const int forced = [] {
    const char* e = std::getenv("SRHIP_JIT_WAVES");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : 0;
  }();
  if (forced) return forced;
  static const int wide = [] {  // SRHIP_JIT_WIDE_FEATURES: the feature count from which 8 waves
    const char* e = std::getenv("SRHIP_JIT_WIDE_FEATURES");
    return e ? std::max(1, std::atoi(e)) : 10;
  }();
  return nraw >= wide ? 8 : 4;
}
// 94 VGPRs: 5 waves per SIMD, 20 per CU; the CU's 160 KiB shared by its workgroups
size_t lds_per_workgroup(int waves) {
  const int per_cu = std::max(1, 20 / std::max(1, waves));
  return (size_t)160 * 1024 / (size_t)per_cu;
}

// The shared-subtree columns of a batch (jit.h Columns::gkey): the
// constant-free subtrees holding a routine, counted per occurrence in the
// trees' IR (after the LDS columns). Largest first, a subtree is kept when
// its occurrences save more FAST tree-code cycles than twice what the derive
// pass spends on it PRECISE (count·(fast − 16) > 2·precise: a read costs a
// load and a block); a kept subtree's occurrences are taken off the subtrees
// inside it. At most SRHIP_JIT_GCOLS (default 32; 0: none) columns, the most
// profitable ones (32: config #2 2.66 ms against 2.68 at 16 and 3.00 at 64 with the derive pass, profiles/r06_gcols_ab.txt); none for per-row output or memory-constant code (their
// constants change; their drivers pass no column base).
// precise: the tree code runs its routines PRECISE (the gradient code's
// forward), so an occurrence saves the PRECISE price; env: the cap's variable.
static void plan_shared(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, bool on, Columns& c,
                        bool precise = false, const char* env = "SRHIP_JIT_GCOLS", int dflt = 32) {
  const char* ge = std::getenv(env);  // read per build: A/B tests
  const int gmax = ge ? std::max(0, std::min(kMaxGlobalCols, std::atoi(ge))) : dflt;
  const int room = std::min(gmax, 255 - c.gbase());
  if (!on || room <= 0) return;
  struct Info {
    int count = 0, fast = 0, precise = 0, size = 0;
    std::vector<std::string> kids;
    std::vector<uint8_t> kind;
    std::vector<uint16_t> arg;
  };
  std::unordered_map<std::string, Info> info;
  DerivedMap dm;
  dm.cols = &c;
  std::vector<IrOp> ir;
  Opnd root;
  SubtreeInfo si;
  for (int32_t t : cand) {
    if (cb.tree_off[t] < 0 || !build_ir(&cb.code[cb.tree_off[t]], ir, root, &dm)) continue;
    subtree_keys(ir, &c, si);
    for (size_t i = 0; i < ir.size(); ++i) {
      if (si.key[i].empty() || !si.routine[i] || si.depth[i] > 8) continue;
      Info& I = info[si.key[i]];
      if (I.count++ == 0) {
        I.fast = precise ? si.precise[i] : si.fast[i];
        I.precise = si.precise[i];
        I.size = (int)si.key[i].size();
        for (const Opnd* q : {&ir[i].a, &ir[i].b}) {
          if (q == &ir[i].b && ir[i].un) break;
          if (q->k == O_VAL && !si.key[q->v].empty()) I.kids.push_back(si.key[q->v]);
        }
        Opnd v;
        v.k = O_VAL;
        v.v = (int)i;
        subtree_postfix(ir, v, &c, I.kind, I.arg);
      }
    }
  }
  std::vector<std::pair<const std::string*, Info*>> order;
  for (auto& kv : info) order.push_back({&kv.first, &kv.second});
  std::sort(order.begin(), order.end(), [](const auto& a, const auto& b) {
    return a.second->size != b.second->size ? a.second->size > b.second->size : *a.first < *b.first;
  });
  std::function<void(const std::string&, int)> absorb = [&](const std::string& k, int n) {
    auto it = info.find(k);
    if (it == info.end()) return;
    it->second.count -= n;
    for (const std::string& kid : it->second.kids) absorb(kid, n);
  };
  std::vector<std::pair<int64_t, const std::string*>> kept;
  for (auto& e : order) {
    const Info& I = *e.second;
    const int64_t gain = (int64_t)I.count * (I.fast - 16) - 2 * (int64_t)I.precise;
    if (I.count < 2 || gain <= 0) continue;
    kept.push_back({gain, e.first});
    for (const std::string& kid : I.kids) absorb(kid, I.count);
  }
  std::stable_sort(kept.begin(), kept.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  if ((int)kept.size() > room) kept.resize(room);
  c.goff.assign(1, 0);
  for (auto& kv : kept) {
    const Info& I = info[*kv.second];
    c.gkey.push_back(*kv.second);
    c.gkind.insert(c.gkind.end(), I.kind.begin(), I.kind.end());
    c.garg.insert(c.garg.end(), I.arg.begin(), I.arg.end());
    c.goff.push_back((int32_t)c.gkind.size());
  }
  c.ngcol = (int)kept.size();
  if (std::getenv("SRHIP_JIT_DEBUG"))
    for (size_t g = 0; g < kept.size(); ++g)
      std::fprintf(stderr, "jit: shared column %zu: %s gain %lld\n", g, kept[g].second->c_str(), (long long)kept[g].first);
}

// The derived columns of a batch: every u(x_f) (u a routine operator) used by
// at least SRHIP_JIT_DERIVE_MIN (default 4) trees' code, most used first, as
// many as leave room for four row tiles in the workgroup's LDS; nraw = the
// raw features still read after the substitution.
static Columns plan_columns(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, const Options& opt) {
  Columns c;
  std::vector<IrOp> ir;
  Opnd root;
  struct Cnt { uint32_t key; int n; };
  std::vector<Cnt> cnt;
  static const int min_uses = [] { const char* e = std::getenv("SRHIP_JIT_DERIVE_MIN"); return e ? std::max(1, std::atoi(e)) : 4; }();
  static const bool env_on = [] { const char* e = std::getenv("SRHIP_JIT_DERIVE"); return !(e && e[0] == '0'); }();
  const bool on = opt.derive && env_on;
  for (int32_t t : cand) {
    if (cb.tree_off[t] < 0 || !build_ir(&cb.code[cb.tree_off[t]], ir, root)) continue;
    for (const IrOp& o : ir) {
      if (o.un && o.a.k == O_X && !o.a.der && is_routine_uop(o.op) && on) {
        const uint32_t key = ((uint32_t)o.op << 16) | (uint32_t)o.a.v;
        auto it = std::find_if(cnt.begin(), cnt.end(), [&](const Cnt& q) { return q.key == key; });
        if (it == cnt.end()) cnt.push_back({key, 1}); else ++it->n;
      }
    }
  }
  std::stable_sort(cnt.begin(), cnt.end(), [](const Cnt& a, const Cnt& b) { return a.n > b.n; });
  std::vector<uint32_t> chosen;
  for (const Cnt& q : cnt)
    if (q.n >= min_uses && (int)chosen.size() < kMaxDerived) chosen.push_back(q.key);
  // raw features read after the substitution
  auto raw_max = [&](const std::vector<uint32_t>& ch) {
    Columns tmp;
    tmp.nraw = 1 << 14;  // out of the feature range: no clash with raw features while scanning
    tmp.nder = (int)ch.size();
    for (size_t k = 0; k < ch.size(); ++k) tmp.der[k] = ch[k];
    DerivedMap dm;
    dm.cols = &tmp;
    int m = -1;
    for (int32_t t : cand) {
      if (cb.tree_off[t] < 0 || !build_ir(&cb.code[cb.tree_off[t]], ir, root, &dm)) continue;
      for (const IrOp& o : ir) {
        if (o.a.k == O_X && !o.a.der) m = std::max(m, o.a.v);
        if (!o.un && o.b.k == O_X && !o.b.der) m = std::max(m, o.b.v);
      }
      if (root.k == O_X && !root.der) m = std::max(m, root.v);
    }
    return m + 1;
  };
  // room: four tiles (SRHIP_JIT_DERIVE_TILES) of (y, raw, derived) in the
  // workgroup's LDS, less the partials' share
  static const int dtiles = [] { const char* e = std::getenv("SRHIP_JIT_DERIVE_TILES"); return e ? std::max(1, std::atoi(e)) : 4; }();
  const size_t tile_bytes = (size_t)dtiles * (size_t)(64 * SR_JIT_R) * sizeof(float);
  c.waves = choose_waves(raw_max({}));  // from the raw features before any substitution
  const size_t lds_wg = lds_per_workgroup(c.waves);
  const size_t budget = lds_wg - (part_global() ? 0 : std::min<size_t>(lds_wg / 8, 4096));
  while (true) {
    const int nraw = raw_max(chosen);
    const size_t cols = 1 + (size_t)nraw + chosen.size();  // y, raw, derived (w, when weighted, may cost a tile)
    if (chosen.empty() || (cols * tile_bytes <= budget && nraw + (int)chosen.size() <= 60)) {
      c.nraw = nraw;
      break;
    }
    chosen.pop_back();  // the least used one goes
  }
  c.nder = (int)chosen.size();
  for (int k = 0; k < c.nder; ++k) c.der[k] = chosen[k];
  plan_shared(cb, cand, on && !opt.out && !opt.memc, c);
  return c;
}

Columns plan_grad_columns(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand) {
  Columns c;
  c.nraw = kGradGbase;  // raw features stay below (the gradient code's DS immediates end at feature 62)
  static const bool env_on = [] { const char* e = std::getenv("SRHIP_JIT_DERIVE"); return !(e && e[0] == '0'); }();
  // 64: config #5's shard gradient 42.2 ms against 42.8 at 32 and 45.9 without (interleaved,
  // tools/ab_build.py --grad, profiles/r06_grad_gcols_ab.txt)
  plan_shared(cb, cand, env_on, c, /*precise=*/true, "SRHIP_GJIT_GCOLS", 64);
  return c;
}

bool compile_only(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, const Options& opt,
                  std::vector<uint8_t>* bytes, std::string* text, std::vector<int32_t>* offsets, Stats* st) {
  const Templates& TT = templates();
  if (!TT.ok) throw Error(SRHIP_ERR_UNSUPPORTED, std::string("jit templates unavailable: ") + TT.why);
  std::vector<uint32_t> words;
  std::vector<std::string> lines;
  std::vector<int32_t> offs, okt, rest;
  const Columns cols = plan_columns(cb, cand, opt);
  codegen(cb, cand, 0, opt, words, opt.text ? &lines : nullptr, offs, okt, rest, st, TT.large, cols);
  if (bytes) {
    bytes->resize(words.size() * 4);
    std::memcpy(bytes->data(), words.data(), bytes->size());
  }
  if (text) {
    text->clear();
    for (auto& l : lines) { *text += l; *text += '\n'; }
  }
  if (offsets) {
    offsets->clear();
    for (size_t k = 0; k < okt.size(); ++k) {
      offsets->push_back(okt[k]);
      offsets->push_back(offs[k]);
    }
  }
  return !okt.empty();
}

Module* build(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list,
              std::vector<int32_t>& rest, const Options& opt, Stats* st) {
  const Templates& TT = templates();
  if (!TT.ok) { rest = cand; return nullptr; }
  auto t0 = std::chrono::steady_clock::now();
  const Columns cols = plan_columns(cb, cand, opt);
  constexpr int kMaxParts = 8;
  struct Chunk { std::vector<uint32_t> words; std::vector<int32_t> offs, slots; const Tmpl* T; };
  std::vector<Chunk> chunks;
  size_t pos = 0, bytes = 0;
  while (pos < cand.size()) {
    Chunk ch;
    ch.T = &TT.large;
    const size_t next = codegen(cb, cand, pos, opt, ch.words, nullptr, ch.offs, ch.slots, rest, st, TT.large, cols);
    if (next == pos) {  // one tree larger than the area
      rest.push_back(cand[pos]);
      if (st) st->nrejected++;
      pos = next + 1;
      continue;
    }
    if ((int)chunks.size() + 1 == kMaxParts && next < cand.size()) {  // the rest stays interpreted
      for (size_t k = next; k < cand.size(); ++k) rest.push_back(cand[k]);
      if (st) st->nrejected += (int)(cand.size() - next);
      pos = cand.size();
    } else {
      pos = next;
    }
    if (ch.slots.empty()) continue;
    if (ch.words.size() * 4 <= TT.small.area_bytes) {  // relayout for the small template's addresses
      Chunk sm;
      sm.T = &TT.small;
      std::vector<int32_t> rs;
      codegen(cb, ch.slots, 0, opt, sm.words, nullptr, sm.offs, sm.slots, rs, nullptr, TT.small, cols);
      if (sm.slots != ch.slots) throw Error(SRHIP_ERR_INVALID, "jit: small-template relayout differs");
      ch = std::move(sm);
    }
    bytes += ch.words.size() * 4;
    chunks.push_back(std::move(ch));
  }
  if (chunks.empty()) return nullptr;
  auto t1 = std::chrono::steady_clock::now();
  Module* m = new Module();
  m->cols = cols;
  m->memc = opt.memc;
  m->bails = can_bail() || (!opt.out && loss_bails(opt.loss));
  m->out = opt.out;
  try {
    for (Chunk& ch : chunks) {
      ModulePart pt;
      pt.slot0 = m->nslots;
      pt.nslots = (int)ch.slots.size();
      m->parts.push_back(pt);
      ModulePart& q = m->parts.back();
      std::vector<uint8_t> img(ch.T->img, ch.T->img + ch.T->size);
      std::memcpy(img.data() + ch.T->area_off, ch.words.data(), ch.words.size() * 4);
      HIP_CHECK(hipModuleLoadData(&q.mod, img.data()));
      if (opt.out) {  // no weighted variant: the output kernel reads no y / w
        HIP_CHECK(hipModuleGetFunction(&q.fn, q.mod, opt.memc ? "sr_jit_out_m" : "sr_jit_out"));
        q.fn_w = q.fn;
        // the same with the trees dealt from an LDS counter (jit_template.hip jit_eval_body DYN)
        HIP_CHECK(hipModuleGetFunction(&q.fn_dl, q.mod, opt.memc ? "sr_jit_out_md" : "sr_jit_out_d"));
      } else {
        HIP_CHECK(hipModuleGetFunction(&q.fn, q.mod, opt.memc ? "sr_jit_eval_m" : "sr_jit_eval"));
        HIP_CHECK(hipModuleGetFunction(&q.fn_w, q.mod, opt.memc ? "sr_jit_eval_mw" : "sr_jit_eval_w"));
        HIP_CHECK(hipModuleGetFunction(&q.fn_dl, q.mod, opt.memc ? "sr_jit_eval_dlm" : "sr_jit_eval_dl"));
        HIP_CHECK(hipModuleGetFunction(&q.fn_dlw, q.mod, opt.memc ? "sr_jit_eval_dlmw" : "sr_jit_eval_dlw"));
        if (!opt.memc) {
          HIP_CHECK(hipModuleGetFunction(&q.fn_dlp, q.mod, "sr_jit_eval_dlp"));
          HIP_CHECK(hipModuleGetFunction(&q.fn_dlpw, q.mod, "sr_jit_eval_dlpw"));
        }
      }
      HIP_CHECK(hipModuleGetFunction(&q.fn_derive, q.mod, "sr_jit_derive"));
      for (hipFunction_t f : {q.fn, q.fn_w, q.fn_dl, q.fn_dlw, q.fn_dlp, q.fn_dlpw})
        if (f)
          HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
      HIP_CHECK(hipMalloc((void**)&q.d_off, ch.offs.size() * sizeof(int32_t)));
      HIP_CHECK(hipMemcpy(q.d_off, ch.offs.data(), ch.offs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      m->nslots += pt.nslots;
      jit_list.insert(jit_list.end(), ch.slots.begin(), ch.slots.end());
    }
    HIP_CHECK(hipMalloc((void**)&m->d_bail, (size_t)(m->nslots + 2) * sizeof(uint32_t)));
    // clean from the start: each call's finalize leaves the counters clean again
    HIP_CHECK(hipMemset(m->d_bail, 0, (size_t)(m->nslots + 2) * sizeof(uint32_t)));
  } catch (...) {
    destroy(m);
    throw;
  }
  auto t2 = std::chrono::steady_clock::now();
  if (st) {
    st->ms_codegen = std::chrono::duration<double, std::milli>(t1 - t0).count();
    st->ms_load = std::chrono::duration<double, std::milli>(t2 - t1).count();
    st->code_bytes = bytes;
    st->nparts = (int)chunks.size();
  }
  return m;
}

void destroy(Module* m) {
  if (!m) return;
  for (ModulePart& q : m->parts) {
    if (q.d_off) (void)hipFree(q.d_off);
    if (q.mod) (void)hipModuleUnload(q.mod);
  }
  if (m->d_bail) (void)hipFree(m->d_bail);
  delete m;
}

uint32_t* bail_flags(Module* m) { return m->d_bail; }
const Columns& columns(const Module* m) { return m->cols; }
bool memc(const Module* m) { return m && m->memc; }
int nslots(const Module* m) { return m->nslots; }
int nparts(const Module* m) { return m ? (int)m->parts.size() : 0; }
void part(const Module* m, int k, int* slot0, int* nslots) {
  *slot0 = m->parts[k].slot0;
  *nslots = m->parts[k].nslots;
}

struct JitArgs {
  EvalArgs<float> e;
  const int32_t* code_off;
  uint32_t* bail;
  uint32_t* counters;
  int fast;
  int part_lds;
  int nraw, nder;
  uint32_t der[kMaxDerived];
  const float* dcols;
  int nbig, ts;
  int dyn;
  const float* gcols;  // [ngcol][n_pad] shared-subtree columns of this call, or null
};
struct DeriveArgs {
  const float* X;
  int64_t n_pad;
  int nder;
  uint32_t der[kMaxDerived];
  float* out;
};

hipError_t launch_derive(Module* m, const float* X, int64_t n_pad, float* out, hipStream_t stream) {
  if (m->cols.nder == 0) return hipSuccess;
  DeriveArgs da;
  da.X = X;
  da.n_pad = n_pad;
  da.nder = m->cols.nder;
  std::memcpy(da.der, m->cols.der, sizeof(da.der));
  da.out = out;
  size_t sz = sizeof(da);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &da, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const unsigned gx = (unsigned)std::min<int64_t>(1024, (n_pad / 4 + 255) / 256);
  return hipModuleLaunchKernel(m->parts[0].fn_derive, std::max(gx, 1u), (unsigned)m->cols.nder, 1, 256, 1, 1, 0,
                               stream, nullptr, cfg);
}

int64_t flag_words(Module* m) { return (int64_t)m->nslots + 2; }

hipError_t reset_flags(Module* m, hipStream_t stream) {
  return hipMemsetAsync(m->d_bail, 0, (size_t)(m->nslots + 2) * sizeof(uint32_t), stream);
}

// (reserved: JitArgs::dyn)
bool dynamic_trees() { return false; }

// Loss tree code runs under sr_jit_eval_dl(w) / _dlm(w) (memory constants),
// whose tree loop is hand-written (jit_template.hip SR_JIT_LOOP_TEXT): the
// waves of a workgroup take their trees from an LDS counter, so the workgroup
// is not held by the wave that drew the costly trees (or the trees whose tiles
// are redone PRECISE). Same sums bit for bit (wave_sum's order); interleaved
// A/B (tools/loop_ab.py, profiles/r04_loop_ab.jsonl): config #2 3.380 →
// 3.247 ms, its 125k-row shard 0.546 → 0.506, a 512-tree shard 0.515 → 0.503.
// SRHIP_JIT_DYNLOOP=0 (read per launch): the compiled static loop.
static bool dynloop() {
  const char* e = std::getenv("SRHIP_JIT_DYNLOOP");
  return !(e && e[0] == '0');
}

bool partials4(Module* m, int k) {
  const ModulePart& q = m->parts[k];
  return q.fn_dl && !m->out && dynloop();
}

hipError_t launch(Module* m, int k, const EvalPlan& plan, const EvalArgs<float>& a, bool fast, const float* dcols,
                  hipStream_t stream, const float* gcols) {
  const ModulePart& q = m->parts[k];
  if (a.nlist != q.nslots) return hipErrorInvalidValue;
  if (m->out && (a.w != nullptr || a.out == nullptr || a.out_stride < a.n_pad)) return hipErrorInvalidValue;
  JitArgs ja;
  ja.e = a;
  ja.code_off = q.d_off;
  ja.bail = m->d_bail + q.slot0;
  ja.counters = m->d_bail + m->nslots;
  ja.fast = (fast && !m->out) ? 1 : 0;
  ja.nraw = m->cols.nraw;
  ja.nder = m->cols.nder;
  std::memcpy(ja.der, m->cols.der, sizeof(ja.der));
  ja.dcols = dcols;
  // shared-subtree columns: tree code reads them (jit_template.hip passes
  // s[36:37] = gcols + row0, s38 = n_pad·4)
  if (m->cols.ngcol > 0 && (!gcols || (uint64_t)a.n_pad * 4u > 0xffffffffu)) return hipErrorInvalidValue;
  ja.gcols = m->cols.ngcol > 0 ? gcols : nullptr;
  ja.nbig = plan.nbig >= 0 ? plan.nbig : a.nrg;
  ja.ts = plan.nbig >= 0 ? plan.ts : plan.ntiles;
  // Sticky PRECISE per tree across row groups (prefetching hand-written loop):
  // a tree redone PRECISE in one row group runs PRECISE in the later ones.
  // It pays with few row groups and costs with many (the trees then run
  // PRECISE where FAST would have held): 4096 config #2 trees, interleaved
  // A/B (profiles/r04_sticky_tree_sizes.jsonl, r04_sticky_tree_ab.jsonl):
  // 30k rows 0.248 → 0.190 ms, 100k 0.449 → 0.449, 250k 0.956 → 0.951, 500k
  // 1.734 → 1.762, 1M 3.28 → 3.39. Round 6 (shared subtrees; profiles/
  // r06_sticky_tree.txt): 4096 trees on 10k rows 0.120 → 0.105 ms, 30k 0.217
  // → 0.191, 62.5k even, 125k +1 %, 250k +3 %; 512 trees even. So it is on
  // for at most 48 row groups (≈ 48k rows); SRHIP_JIT_STICKY_TREE=1 / 0 (read
  // per launch) forces it on / off. The mark is bit 1 of the tree's flag word
  // (bit 0: failed), which the finalize ignores.
  {
    const char* e = std::getenv("SRHIP_JIT_STICKY_TREE");
    ja.dyn = (e && e[0] == '1') ? 1 : (e && e[0] == '0') ? 0 : (a.nrg <= 48 ? 1 : 0);
  }
  if (ja.nraw > a.nfeat) return hipErrorInvalidValue;
  if (ja.nbig > a.nrg || ja.ts < 1 || ja.ts > plan.ntiles) return hipErrorInvalidValue;
  // partials in LDS when they take little room next to the tiles (measured
  // faster on config #2: one coalesced write-out instead of a store per tree)
  const size_t part_bytes = (size_t)a.tpb * sizeof(Part<float>);
  ja.part_lds = part_bytes <= 8192 && !part_global() ? 1 : 0;
  size_t sz = sizeof(ja);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ja, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const unsigned grid = a.rotate >= 2 ? (unsigned)((a.nrg + 7) / 8 * 8) * (unsigned)a.ntg
                                      : (unsigned)a.nrg * (unsigned)a.ntg;
  // SRHIP_JIT_LDS_PAD (experiments): extra LDS per workgroup, i.e. fewer resident waves
  static const unsigned pad = [] { const char* e = std::getenv("SRHIP_JIT_LDS_PAD"); return e ? (unsigned)std::atoi(e) : 0u; }();
  // LDS: the row tiles (+ the partials when part_lds)
  const size_t narr = 1 + (size_t)(ja.nraw + ja.nder) + (a.w ? 1 : 0);
  const size_t lds = narr * (size_t)plan.ntiles * (size_t)plan.tile * sizeof(float) + (ja.part_lds ? part_bytes : 0) + 16;
  // the hand-written loop keeps its tree counter in the last 16 bytes
  hipFunction_t fn = a.w ? q.fn_w : q.fn;
  if (m->out && q.fn_dl && dynloop()) fn = q.fn_dl;
  const char* name = m->out ? (m->memc ? (fn == q.fn_dl ? "sr_jit_out_md" : "sr_jit_out_m")
                                       : (fn == q.fn_dl ? "sr_jit_out_d" : "sr_jit_out"))
                            : m->memc ? (a.w ? "sr_jit_eval_mw" : "sr_jit_eval_m") : (a.w ? "sr_jit_eval_w" : "sr_jit_eval");
  if (q.fn_dl && !m->out && dynloop()) {
    fn = a.w ? q.fn_dlw : q.fn_dl;
    name = m->memc ? (a.w ? "sr_jit_eval_dlmw" : "sr_jit_eval_dlm") : (a.w ? "sr_jit_eval_dlw" : "sr_jit_eval_dl");
  }
  // literal code: the loop that claims the next tree and loads its flag and
  // code offset before running this one (interleaved A/B, profiles/
  // r04_loop_ab.jsonl: config #2 3.247 → 3.231 ms, a 512-tree shard 0.503 →
  // 0.483); SRHIP_JIT_PREFETCH=0 (read per launch): without
  static const auto prefetch = [] { const char* e = std::getenv("SRHIP_JIT_PREFETCH"); return !(e && e[0] == '0'); };
  if (q.fn_dlp && !m->out && dynloop() && prefetch()) {
    fn = a.w ? q.fn_dlpw : q.fn_dlp;
    name = a.w ? "sr_jit_eval_dlpw" : "sr_jit_eval_dlp";
  }
  note_kernel(name);
  return hipModuleLaunchKernel(fn, grid, 1, 1, (unsigned)plan.threads, 1, 1, (unsigned)lds + pad, stream, nullptr, cfg);
}

}  // namespace jit
}  // namespace srhip
