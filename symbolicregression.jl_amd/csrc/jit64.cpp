// jit64.cpp — the Float64 tree compiler: every shallow tree of a Float64
// batch becomes straight-line gfx950 machine code, the counterpart of jit.cpp
// for Dataset{Float64} (BASELINE config #3: NaN-heavy Float64 evaluation).
//
// Float64 has no FAST path: the routines are the Float64 interpreter's
// operator code (gen_jit64.py), so losses and did_succeed are the
// interpreter's. Layout (jit64_layout.h): R = 2 rows per lane, a 128-row tile
// is 1 KiB per column (the byte layout of the Float32 tiles), a value block is
// 4 VGPRs (two Float64), 8 pool blocks, the routine operands in A = v[32:35]
// and B = v[36:39], the non-finite marker CHK = v[40:41] (Float64), the lane's
// loss sum LSUM = v[44:45].
//
// Tree code of one tree:
//   prologue  routine base (s_getpc), status 0
//   tile      y and the features inline operators read, from the LDS tile
//             (ds_read_b128: two rows); + - * neg abs square cube inline
//             (v_add_f64 / v_mul_f64, sign bits on the high word), every other
//             operator by routine; the root marked into CHK (fma(v, 0, chk):
//             NaN for a non-finite value, as the interpreter's mark); the
//             residual, masked past the last row, squared (weighted) into LSUM;
//             a failed tile ends the tree (DynamicExpressions' early exit)
//   epilogue  s_setpc_b64 back to the driver (jit64_template.hip)
// Constants are literals of the code (an SGPR pair per use, or s_k : s_kh for
// a routine's constant operand): a program whose constants are set again runs
// on the interpreter (api.cpp update_constants).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "jit.h"
#include "jit_asm.h"
#include "gen/jit64_layout.h"

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw Error(SRHIP_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));  \
  } while (0)

extern "C" const unsigned char srhip_jit64_tmpl[];
extern "C" const unsigned char srhip_jit64_tmpl_end[];

namespace srhip {
namespace jit {
namespace {

using detail::Asm;
using detail::K;
using detail::S;
using detail::Src;
using detail::V;

constexpr int R2 = 2, TILE2 = 64 * R2;
constexpr int A2 = SR_JIT64_V_A, B2 = SR_JIT64_V_B, CHK2 = SR_JIT64_V_CHK, LANE2 = SR_JIT64_V_LANE;
constexpr int LROW2 = SR_JIT64_V_LANE2, LSUM2 = SR_JIT64_V_LSUM, GT2 = SR_JIT64_V_GT, Y2 = SR_JIT64_V_Y;
constexpr int POOL2 = SR_JIT64_V_POOL0, NPOOL2 = SR_JIT64_V_NPOOL;
constexpr int T_TILE = SR_JIT64_S_TILE, T_NT = SR_JIT64_S_NT, T_PARTIAL = SR_JIT64_S_PARTIAL;
constexpr int T_TILEBYTES = SR_JIT64_S_TILEBYTES, T_WOFF = SR_JIT64_S_WOFF, T_STATUS = SR_JIT64_S_STATUS;
constexpr int T_RR = SR_JIT64_S_RR, T_TGT = SR_JIT64_S_TGT, T_RT = SR_JIT64_S_RT, T_K = SR_JIT64_S_K;
constexpr int T_PE = SR_JIT64_S_PE, T_BASE = SR_JIT64_S_BASE, T_KH = SR_JIT64_S_KH;
constexpr int T_C = 20;  // s[20:21]: the Float64 constant of an inline operator (a routine temporary)
constexpr int kNum64 = SR_JIT64_NUM_ROUTINES;
const int kUop64[SRHIP_NUM_UOPS] = SR_JIT64_UOP_ROUTINE;
const int kBop64[SRHIP_NUM_BOPS] = SR_JIT64_BOP_ROUTINE;
const int kBop64RC[SRHIP_NUM_BOPS] = SR_JIT64_BOP_ROUTINE_RC;
const int kBop64LC[SRHIP_NUM_BOPS] = SR_JIT64_BOP_ROUTINE_LC;
const char* const kName64[kNum64] = SR_JIT64_ROUTINE_NAMES;
const int kLoss64[SRHIP_NUM_LOSSES] = SR_JIT64_LOSS_ROUTINE;
const int kDLoss64[SRHIP_NUM_LOSSES] = SR_JIT64_DLOSS_ROUTINE;
constexpr int T_OUT = 92;  // s[92:93]: out mode, the tree's output rows of the current tile

// gfx950 encodings used here and not by jit.cpp (checked against llvm-mc by tests/test_jit.py)
enum : int {
  VOP3_FMA_F64 = 0x1cc, VOP3_ADD_F64 = 0x280, VOP3_MUL_F64 = 0x281, VOPC_U_F64 = 0x68,
  VOP1_MOV = 0x01, VOP2_CNDMASK = 0x00, VOP2_LSHLREV_B32 = 0x12, VOP2_AND_B32 = 0x13, VOP2_XOR_B32 = 0x15, VOP2_ADD_U32 = 0x34,
  VOP3P_MOV_B32 = 0x33, VOPC_GT_I32 = 0xc4,
  SOP1_MOV = 0x00, SOP1_GETPC = 0x1c, SOP1_SETPC = 0x1d, SOP1_SWAPPC = 0x1e,
  SOP2_ADD_U32 = 0x00, SOP2_SUB_I32 = 0x03, SOP2_ADDC_U32 = 0x04,
  SOPC_EQ_U32 = 0x06, SOPC_GE_U32 = 0x09, SOPC_LT_U32 = 0x0a,
  SOPP_BRANCH = 0x02, SOPP_SCC0 = 0x04, SOPP_SCC1 = 0x05, SOPP_VCCNZ = 0x07,
};

// ---- the template ------------------------------------------------------------------
struct Tmpl64 {
  const uint8_t* img = nullptr;
  size_t size = 0, area_off = 0, area_bytes = 0;
  uint64_t area_va = 0, rt0 = 0;
  uint64_t rt_va[kNum64] = {};
  bool ok = false;
  std::string why;
};

bool parse_tmpl64(const uint8_t* img, size_t size, Tmpl64* t) {
  t->img = img;
  t->size = size;
  if (size < sizeof(Elf64_Ehdr)) { t->why = "template too small"; return false; }
  Elf64_Ehdr eh;
  std::memcpy(&eh, img, sizeof(eh));
  if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_shoff + (size_t)eh.e_shnum * sizeof(Elf64_Shdr) > size) {
    t->why = "template is not an ELF64 image";
    return false;
  }
  std::vector<Elf64_Shdr> sh(eh.e_shnum);
  std::memcpy(sh.data(), img + eh.e_shoff, sh.size() * sizeof(Elf64_Shdr));
  const Elf64_Shdr* symtab = nullptr;
  for (auto& s : sh)
    if (s.sh_type == SHT_SYMTAB) symtab = &s;
  if (!symtab || symtab->sh_link >= sh.size()) { t->why = "template has no symbol table"; return false; }
  const Elf64_Shdr& strtab = sh[symtab->sh_link];
  uint64_t code_va = 0, area_fn_va = 0, area_fn_size = 0;
  int found = 0;
  for (size_t i = 0; i < symtab->sh_size / sizeof(Elf64_Sym); ++i) {
    Elf64_Sym sym;
    std::memcpy(&sym, img + symtab->sh_offset + i * sizeof(Elf64_Sym), sizeof(sym));
    if (sym.st_name >= strtab.sh_size) continue;
    const std::string n(reinterpret_cast<const char*>(img + strtab.sh_offset + sym.st_name));
    if (n == "sr_jit64_code") { code_va = sym.st_value; found |= 1; }
    else if (n == "sr_jit64_area") { area_fn_va = sym.st_value; area_fn_size = sym.st_size; found |= 2; }
    else if (n == "sr_rt64") { t->rt0 = sym.st_value; found |= 4; }
    else if (n.rfind("sr_rt64_", 0) == 0) {
      for (int k = 0; k < kNum64; ++k)
        if (n.compare(8, std::string::npos, kName64[k]) == 0) t->rt_va[k] = sym.st_value;
    }
  }
  if (found != 7) { t->why = "template symbols missing"; return false; }
  for (int k = 0; k < kNum64; ++k)
    if (!t->rt_va[k]) { t->why = std::string("routine missing: ") + kName64[k]; return false; }
  const Elf64_Shdr* text = nullptr;
  for (auto& s : sh)
    if (s.sh_type == SHT_PROGBITS && (s.sh_flags & SHF_EXECINSTR) && code_va >= s.sh_addr &&
        code_va < s.sh_addr + s.sh_size)
      text = &s;
  if (!text) { t->why = "code area outside .text"; return false; }
  t->area_va = code_va;
  t->area_off = (size_t)(code_va - text->sh_addr + text->sh_offset);
  const uint64_t end = area_fn_va + area_fn_size;
  if (end <= code_va + 64 || end > text->sh_addr + text->sh_size) { t->why = "bad area size"; return false; }
  t->area_bytes = (size_t)(end - code_va) - 64;
  if (t->area_off + t->area_bytes > size) { t->why = "area beyond the image"; return false; }
  t->ok = true;
  return true;
}

const Tmpl64& tmpl64() {
  static Tmpl64 T;
  static std::once_flag once;
  std::call_once(once, [] { parse_tmpl64(srhip_jit64_tmpl, (size_t)(srhip_jit64_tmpl_end - srhip_jit64_tmpl), &T); });
  return T;
}

// ---- IR ------------------------------------------------------------------------------
enum { Q_VAL = 0, Q_X = 1, Q_C = 2 };
struct Q {
  int k = Q_VAL;
  int v = -1;      // value id or feature
  uint64_t c = 0;  // constant bits
};
struct Op64 {
  bool un = false;
  int op = 0;
  Q a, b;
  int rid = -1, krid = -1;  // routine; constant-operand variant (constant in s_k : s_kh)
};

bool inline64(const Op64& o) {
  return o.un ? (o.op == SRHIP_UOP_NEG || o.op == SRHIP_UOP_ABS || o.op == SRHIP_UOP_SQUARE || o.op == SRHIP_UOP_CUBE)
              : (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB || o.op == SRHIP_BOP_MUL);
}

bool build_ir64(const Ins<double>* p, std::vector<Op64>& ops, Q& root) {
  ops.clear();
  Q acc, tmp, slot[kMaxSlots];
  for (int pc = 0;; ++pc) {
    if (pc > 4096) return false;
    const uint32_t code = p[pc].code;
    const int opc = (int)(code & 0xffu);
    const int f = (int)(code >> 16);
    uint64_t bits;
    std::memcpy(&bits, &p[pc].imm, 8);
    auto X = [&](int ff) { Q q; q.k = Q_X; q.v = ff; return q; };
    auto C = [&]() { Q q; q.k = Q_C; q.c = bits; return q; };
    auto val = [&](const Op64& o) { ops.push_back(o); Q q; q.k = Q_VAL; q.v = (int)ops.size() - 1; return q; };
    if (opc == OP_END) { root = acc; return true; }
    if (opc == OP_LDX) { acc = X(f); continue; }
    if (opc == OP_LDC) { acc = C(); continue; }
    if (opc >= OP_PUSH0 && opc < OP_PUSH0 + kMaxSlots) { slot[opc - OP_PUSH0] = acc; continue; }
    if (opc >= OP_POP0 && opc < OP_POP0 + kMaxSlots) { tmp = slot[opc - OP_POP0]; continue; }
    if (opc >= OP_UN0 && opc < OP_BIN0) {
      if (acc.k == Q_C) return false;
      Op64 o;
      o.un = true;
      o.op = opc - OP_UN0;
      o.a = acc;
      acc = val(o);
      continue;
    }
    const int v = (opc - OP_BIN0) / SRHIP_NUM_BOPS;
    Op64 o;
    o.op = (opc - OP_BIN0) % SRHIP_NUM_BOPS;
    switch (v) {
      case V_AX: o.a = acc; o.b = X(f); break;
      case V_XA: o.a = X(f); o.b = acc; break;
      case V_AC: o.a = acc; o.b = C(); break;
      case V_CA: o.a = C(); o.b = acc; break;
      case V_AT: o.a = acc; o.b = tmp; break;
      case V_TA: o.a = tmp; o.b = acc; break;
      case V_XX: o.a = X(f); o.b = X((int)bits); break;
      case V_XC: o.a = X(f); o.b = C(); break;
      case V_CX: o.a = C(); o.b = X(f); break;
      default: return false;
    }
    if (o.a.k == Q_C && o.b.k == Q_C) return false;
    acc = val(o);
  }
}

// ---- code generation of one tree -----------------------------------------------------
struct Gen64 {
  Asm& as;
  const Tmpl64& T;
  uint64_t base_va;
  std::vector<Op64> ops;
  Q root;
  int n = 0;
  std::vector<int> last, loc;  // last reader of a value (n: the root), its pool block (-1: none)
  int owner[NPOOL2];           // -1 free, value id, 1000 + feature
  int xblk[256], xlast[256], load_idx[256];
  std::vector<int> feats;      // features inline operators read, in first-use order
  int nloads = 0, waited = 0, max_feat = -1;
  bool has_call = false;
  int L_tile = -1, L_done = -1;
  std::string why;
  Opts64 opt;  // out mode / loss of this build

  Gen64(Asm& a, const Tmpl64& t, uint64_t va, const Opts64& o) : as(a), T(t), base_va(va), opt(o) {}
  uint64_t cur_va() const { return base_va + as.bytes(); }
  static int blk(int k) { return POOL2 + 4 * k; }

  bool analyze() {
    n = (int)ops.size();
    last.assign(n, -1);
    loc.assign(n, -1);
    for (int f = 0; f < 256; ++f) { xblk[f] = -1; xlast[f] = -1; load_idx[f] = -1; }
    auto usef = [&](const Q& q, int i, bool inl) {
      if (q.k != Q_X) return true;
      if (q.v < 0 || q.v > 62) { why = "feature offset beyond the DS immediate"; return false; }
      max_feat = std::max(max_feat, q.v);
      if (inl) {
        if (xlast[q.v] < 0) feats.push_back(q.v);
        xlast[q.v] = std::max(xlast[q.v], i);
      }
      return true;
    };
    for (int i = 0; i < n; ++i) {
      Op64& o = ops[i];
      const bool inl = inline64(o);
      if (!inl) {
        if (!o.un && o.b.k == Q_C) o.krid = kBop64RC[o.op];
        if (!o.un && o.a.k == Q_C) o.krid = kBop64LC[o.op];
        o.rid = o.un ? kUop64[o.op] : kBop64[o.op];
        if (o.rid < 0 && o.krid < 0) { why = "operator without a Float64 routine"; return false; }
        if (o.rid < 0 && !(o.a.k == Q_C || o.b.k == Q_C)) { why = "operator without a Float64 routine"; return false; }
        has_call = true;
      }
      if (!usef(o.a, i, inl)) return false;
      if (!o.un && !usef(o.b, i, inl)) return false;
      if (o.a.k == Q_VAL) last[o.a.v] = i;
      if (!o.un && o.b.k == Q_VAL) last[o.b.v] = i;
    }
    if (!usef(root, n, true)) return false;
    if (root.k == Q_VAL) last[root.v] = n;
    if (!opt.out && opt.loss != SRHIP_LOSS_L2) {  // the loss routine of the tile tail
      if (opt.loss < 0 || opt.loss >= SRHIP_NUM_LOSSES || kLoss64[opt.loss] < 0) { why = "no Float64 loss routine"; return false; }
      has_call = true;
    }
    if ((int)feats.size() > NPOOL2) { why = "more features than register blocks"; return false; }
    return true;
  }

  // ---- emission helpers
  static std::string pr(int r) { return "v[" + std::to_string(r) + ":" + std::to_string(r + 1) + "]"; }
  static std::string pname(const Src& s) {
    if (s.enc >= 256) return pr(s.enc - 256);
    if (s.enc < 102) return "s[" + std::to_string(s.enc) + ":" + std::to_string(s.enc + 1) + "]";
    return s.enc == 128 ? "0" : s.name();
  }
  // VOP3 on Float64 register pairs (neg bit i negates source i)
  void vop3d(int op, const char* nm, int vdst, const Src& s0, const Src& s1, const Src* s2, int neg) {
    as.put(0xd0000000u | ((uint32_t)op << 16) | (uint32_t)vdst);
    as.put(((uint32_t)(neg & 7) << 29) | ((uint32_t)(s2 ? s2->enc : 0) << 18) | ((uint32_t)s1.enc << 9) |
           (uint32_t)s0.enc);
    if (!as.want_text) return;
    auto f = [&](const Src& s, int i) { return ((neg >> i) & 1 ? "-" : "") + pname(s); };
    as.t(std::string(nm) + " " + pr(vdst) + ", " + f(s0, 0) + ", " + f(s1, 1) + (s2 ? ", " + f(*s2, 2) : ""));
  }
  void movd(int dst, int src) {  // one Float64 (a register pair)
    as.vop3p(VOP3P_MOV_B32, "v_pk_mov_b32", dst, V(src), V(src), nullptr, 2, 7, 0, 0);
  }
  void mov_block(int dst, int src) {
    if (dst == src) return;
    movd(dst, src);
    movd(dst + 2, src + 2);
  }
  void const_to_s(int sreg, uint64_t bits) {
    as.sop1(SOP1_MOV, "s_mov_b32", sreg, K((uint32_t)bits), "s" + std::to_string(sreg));
    as.sop1(SOP1_MOV, "s_mov_b32", sreg + 1, K((uint32_t)(bits >> 32)), "s" + std::to_string(sreg + 1));
  }
  void wait_for(int f) {
    const int li = load_idx[f];
    if (li >= waited) {
      as.waitcnt_lgkm(nloads - 1 - li);
      waited = li + 1;
    }
  }
  void wait_all() {
    if (waited < nloads) { as.waitcnt_lgkm(0); waited = nloads; }
  }
  int free_block() const {
    for (int k = 0; k < NPOOL2; ++k)
      if (owner[k] == -1) return k;
    return -1;
  }
  void free_at(int i) {  // values and features whose last reader is step i
    for (int k = 0; k < NPOOL2; ++k) {
      const int w = owner[k];
      if (w >= 0 && w < 1000 && last[w] == i) owner[k] = -1;
      if (w >= 1000 && xlast[w - 1000] == i) owner[k] = -1;
    }
  }
  // block register of an operand for inline use (-1: a constant, in s[T_C:T_C+1])
  int opnd_reg(const Q& q) {
    if (q.k == Q_VAL) return blk(loc[q.v]);
    if (q.k == Q_X) { wait_for(q.v); return blk(xblk[q.v]); }
    const_to_s(T_C, q.c);
    return -1;
  }
  // a call operand into block A or B: a value block, a feature from the LDS
  // tile, or a constant (both rows)
  void operand_to(int dst, const Q& q) {
    if (q.k == Q_VAL) { mov_block(dst, blk(loc[q.v])); return; }
    if (q.k == Q_X) {
      as.ds_read_b128(dst, LANE2, (1 + q.v) * TILE2 * 8);
      as.waitcnt_lgkm(0);
      waited = nloads;
      return;
    }
    const_to_s(T_C, q.c);
    for (int e = 0; e < 4; ++e) as.vop1(VOP1_MOV, "v_mov_b32_e32", dst + e, S(T_C + (e & 1)));
  }
  void set_base() {
    as.sop1(SOP1_GETPC, "s_getpc_b64", T_BASE, Src{0, false, 0}, "");
    if (as.want_text) as.lines.back() = "s_getpc_b64 s[" + std::to_string(T_BASE) + ":" + std::to_string(T_BASE + 1) + "]";
    const int64_t rel = (int64_t)(T.rt0 - cur_va());
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_BASE, S(T_BASE), K((uint32_t)(uint64_t)rel));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", T_BASE + 1, S(T_BASE + 1), K((uint32_t)((uint64_t)rel >> 32)));
  }
  void routine(int rid) {
    const uint64_t off = T.rt_va[rid] - T.rt0;
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_TGT, S(T_BASE), K((uint32_t)off));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", T_TGT + 1, S(T_BASE + 1), K((uint32_t)(off >> 32)));
    as.sop1(SOP1_SWAPPC, "s_swappc_b64", T_RR, S(T_TGT), "");
    if (as.want_text)
      as.lines.back() = "s_swappc_b64 s[" + std::to_string(T_RR) + ":" + std::to_string(T_RR + 1) + "], s[" +
                        std::to_string(T_TGT) + ":" + std::to_string(T_TGT + 1) + "]";
  }

  bool emit_inline(int i) {
    const Op64& o = ops[i];
    const int ra = opnd_reg(o.a);
    const int rb = o.un ? 0 : opnd_reg(o.b);
    free_at(i);
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted"; return false; }
    const int d = blk(k);
    for (int e = 0; e < R2; ++e) {
      const Src a = ra < 0 ? S(T_C) : V(ra + 2 * e);
      if (o.un) {
        switch (o.op) {
          case SRHIP_UOP_NEG:
          case SRHIP_UOP_ABS:
            as.vop1(VOP1_MOV, "v_mov_b32_e32", d + 2 * e, V(ra + 2 * e));
            if (o.op == SRHIP_UOP_NEG) as.vop2(VOP2_XOR_B32, "v_xor_b32_e32", d + 2 * e + 1, K(0x80000000u), ra + 2 * e + 1);
            else as.vop2(VOP2_AND_B32, "v_and_b32_e32", d + 2 * e + 1, K(0x7fffffffu), ra + 2 * e + 1);
            break;
          case SRHIP_UOP_SQUARE: vop3d(VOP3_MUL_F64, "v_mul_f64", d + 2 * e, a, a, nullptr, 0); break;
          default: {  // CUBE = (x*x)*x
            const int t = (d == ra) ? GT2 + 2 * e : d + 2 * e;
            vop3d(VOP3_MUL_F64, "v_mul_f64", t, a, a, nullptr, 0);
            vop3d(VOP3_MUL_F64, "v_mul_f64", d + 2 * e, V(t), a, nullptr, 0);
          }
        }
      } else {
        const Src b = rb < 0 ? S(T_C) : V(rb + 2 * e);
        switch (o.op) {
          case SRHIP_BOP_ADD: vop3d(VOP3_ADD_F64, "v_add_f64", d + 2 * e, a, b, nullptr, 0); break;
          case SRHIP_BOP_SUB: vop3d(VOP3_ADD_F64, "v_add_f64", d + 2 * e, a, b, nullptr, 2); break;
          default: vop3d(VOP3_MUL_F64, "v_mul_f64", d + 2 * e, a, b, nullptr, 0);
        }
      }
    }
    owner[k] = i;
    loc[i] = k;
    return true;
  }

  bool emit_call(int i) {
    const Op64& o = ops[i];
    if (o.krid >= 0) {  // one constant operand: in s_k : s_kh
      const bool rc = o.b.k == Q_C;
      operand_to(A2, rc ? o.a : o.b);
      const uint64_t c = rc ? o.b.c : o.a.c;
      as.sop1(SOP1_MOV, "s_mov_b32", T_K, K((uint32_t)c), "s" + std::to_string(T_K));
      as.sop1(SOP1_MOV, "s_mov_b32", T_KH, K((uint32_t)(c >> 32)), "s" + std::to_string(T_KH));
      free_at(i);
      routine(o.krid);
    } else {
      operand_to(A2, o.a);
      if (!o.un) operand_to(B2, o.b);
      free_at(i);
      routine(o.rid);
    }
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted"; return false; }
    mov_block(blk(k), A2);
    owner[k] = i;
    loc[i] = k;
    return true;
  }

  // rows past the last of the last tile: 0 in block `reg`
  void emit_mask(int reg) {
    const int L_nomask = as.label();
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_PE, S(T_TILE), K(1));
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_PE), S(T_NT));
    as.branch(SOPP_SCC0, "s_cbranch_scc0", L_nomask);
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_PARTIAL), K((uint32_t)TILE2));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_nomask);
    for (int e = 0; e < R2; ++e) {
      as.sop2(SOP2_SUB_I32, "s_sub_i32", T_PE, S(T_PARTIAL), K((uint32_t)e));
      as.vopc(VOPC_GT_I32, "v_cmp_gt_i32_e32", S(T_PE), LROW2);
      as.sopp(0x00, "s_nop", 1);  // VALU-written VCC read as a VALU mask
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", reg + 2 * e, K(0), reg + 2 * e, ", vcc");
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", reg + 2 * e + 1, K(0), reg + 2 * e + 1, ", vcc");
    }
    as.bind(L_nomask);
  }

  // L2: residuals r = ŷ - y, masked, squared (weighted) into the lane's sum
  void emit_tail_l2(int rreg) {
    for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", Y2 + 2 * e, V(rreg + 2 * e), V(Y2 + 2 * e), nullptr, 2);
    emit_mask(Y2);
    const int L_unw = as.label(), L_sum = as.label();
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_WOFF), K(0));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", GT2, S(T_WOFF), LANE2);
    as.ds_read_b128(GT2, GT2, 0);
    as.waitcnt_lgkm(0);
    for (int e = 0; e < R2; ++e) {  // Σ w·(r·r)
      const Src r = V(Y2 + 2 * e);
      vop3d(VOP3_MUL_F64, "v_mul_f64", Y2 + 2 * e, r, r, nullptr, 0);
      const Src w = V(GT2 + 2 * e), t = V(Y2 + 2 * e), l = V(LSUM2);
      vop3d(VOP3_FMA_F64, "v_fma_f64", LSUM2, w, t, &l, 0);
    }
    as.branch(SOPP_BRANCH, "s_branch", L_sum);
    as.bind(L_unw);
    for (int e = 0; e < R2; ++e) {
      const Src r = V(Y2 + 2 * e), l = V(LSUM2);
      vop3d(VOP3_FMA_F64, "v_fma_f64", LSUM2, r, r, &l, 0);
    }
    as.bind(L_sum);
  }

  // any other loss: r = ŷ - y into A, ℓ(r) by the loss routine (the Float64
  // interpreter's elem_loss, its parameter in s_k : s_kh), times w when
  // weighted, masked past the last row, summed into the lane's sum
  void emit_tail_loss(int rreg) {
    for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", A2 + 2 * e, V(rreg + 2 * e), V(Y2 + 2 * e), nullptr, 2);
    as.sop1(SOP1_MOV, "s_mov_b32", T_K, K((uint32_t)opt.lparam), "s" + std::to_string(T_K));
    as.sop1(SOP1_MOV, "s_mov_b32", T_KH, K((uint32_t)(opt.lparam >> 32)), "s" + std::to_string(T_KH));
    routine(kLoss64[opt.loss]);
    const int L_unw = as.label();
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_WOFF), K(0));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", GT2, S(T_WOFF), LANE2);
    as.ds_read_b128(GT2, GT2, 0);
    as.waitcnt_lgkm(0);
    for (int e = 0; e < R2; ++e) vop3d(VOP3_MUL_F64, "v_mul_f64", A2 + 2 * e, V(GT2 + 2 * e), V(A2 + 2 * e), nullptr, 0);
    as.bind(L_unw);
    emit_mask(A2);
    for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", LSUM2, V(LSUM2), V(A2 + 2 * e), nullptr, 0);
  }

  // out mode: the tile's root values to the tree's output rows (lane ℓ holds
  // rows 2ℓ, 2ℓ+1: one coalesced 1 KiB global_store_dwordx4 per wave at
  // s[92:93] + 16ℓ), then the next tile's rows. Rows past the last are
  // written too: they lie in the output's padding (stride n_pad).
  void emit_store_out(int rreg) {
    const int voff = Y2;  // no y in out mode: 16ℓ = 8 · (2ℓ)
    as.vop2(VOP2_LSHLREV_B32, "v_lshlrev_b32_e32", voff, K(3), LROW2);
    as.put(0xdc7c8000u);  // global_store_dwordx4 voff, v[rreg:rreg+3], s[T_OUT:T_OUT+1]
    as.put((uint32_t)voff | ((uint32_t)rreg << 8) | ((uint32_t)T_OUT << 16));
    if (as.want_text)
      as.lines.push_back("global_store_dwordx4 v" + std::to_string(voff) + ", v[" + std::to_string(rreg) + ":" +
                         std::to_string(rreg + 3) + "], s[" + std::to_string(T_OUT) + ":" + std::to_string(T_OUT + 1) +
                         "]");
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_OUT, S(T_OUT), K((uint32_t)(TILE2 * 8)));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", T_OUT + 1, S(T_OUT + 1), K(0));
  }

  bool emit_tree() {
    if (!analyze()) return false;
    L_tile = as.label();
    L_done = as.label();
    as.sop1(SOP1_MOV, "s_mov_b32", T_STATUS, K(0), "s" + std::to_string(T_STATUS));
    if (has_call) set_base();
    as.sopc(SOPC_GE_U32, "s_cmp_ge_u32", S(T_TILE), S(T_NT));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_done);
    // ---- tile
    as.bind(L_tile);
    for (int k = 0; k < NPOOL2; ++k) owner[k] = -1;
    nloads = 0;
    waited = 0;
    if (!opt.out) {  // out mode: no y column
      as.ds_read_b128(Y2, LANE2, 0);
      ++nloads;
    }
    for (size_t j = 0; j < feats.size(); ++j) {
      const int f = feats[j];
      xblk[f] = (int)j;
      owner[j] = 1000 + f;
      load_idx[f] = nloads++;
      as.ds_read_b128(blk((int)j), LANE2, (1 + f) * TILE2 * 8);
    }
    std::fill(loc.begin(), loc.end(), -1);
    for (int i = 0; i < n; ++i) {
      if (!(inline64(ops[i]) ? emit_inline(i) : emit_call(i))) return false;
    }
    // root value → rreg
    int rreg;
    if (root.k == Q_VAL) rreg = blk(loc[root.v]);
    else if (root.k == Q_X) { wait_for(root.v); rreg = blk(xblk[root.v]); }
    else {
      const_to_s(T_C, root.c);
      for (int e = 0; e < 4; ++e) as.vop1(VOP1_MOV, "v_mov_b32_e32", GT2 + e, S(T_C + (e & 1)));
      rreg = GT2;
    }
    for (int e = 0; e < R2; ++e) {  // chk = fma(v, 0, chk): NaN for a non-finite root value
      const Src r = V(rreg + 2 * e), z = K(0), c = V(CHK2);
      vop3d(VOP3_FMA_F64, "v_fma_f64", CHK2, r, z, &c, 0);
    }
    wait_all();
    if (opt.out) {
      emit_store_out(rreg);
    } else {
      if (opt.loss == SRHIP_LOSS_L2) emit_tail_l2(rreg);
      else emit_tail_loss(rreg);
      // a failed tile ends the tree (out mode: every tile is evaluated, as MODE_OUT does)
      as.put(0x7c000000u | ((uint32_t)VOPC_U_F64 << 17) | ((uint32_t)CHK2 << 9) | (uint32_t)(256 + CHK2));
      if (as.want_text) as.t("v_cmp_u_f64_e32 vcc, " + pr(CHK2) + ", " + pr(CHK2));
      as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_done);
    }
    // ---- next tile
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", LANE2, S(T_TILEBYTES), LANE2);
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_TILE, S(T_TILE), K(1));
    as.sopc(SOPC_LT_U32, "s_cmp_lt_u32", S(T_TILE), S(T_NT));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_tile);
    as.bind(L_done);
    as.sop1(SOP1_SETPC, "s_setpc_b64", 0, S(T_RT), "");
    if (as.want_text) as.lines.back() = "s_setpc_b64 s[" + std::to_string(T_RT) + ":" + std::to_string(T_RT + 1) + "]";
    return true;
  }
};

bool gen_tree64(const Ins<double>* prog, const Tmpl64& T, const Opts64& opt, bool text, std::vector<uint32_t>& out,
                std::vector<std::string>* lines, int32_t* off, int* max_feat, std::string* why) {
  std::vector<Op64> ir;
  Q root;
  if (!build_ir64(prog, ir, root)) { *why = "program not translatable"; return false; }
  const size_t start = (out.size() + 15) / 16 * 16;  // 64-byte aligned entries
  Asm as;
  as.want_text = text;
  Gen64 g(as, T, T.area_va + start * 4, opt);
  g.ops = ir;
  g.root = root;
  if (!g.emit_tree()) { *why = g.why; return false; }
  as.finish();
  while (out.size() < start) {
    out.push_back(0xbf800000u);
    if (lines) lines->push_back("s_nop 0");
  }
  out.insert(out.end(), as.w.begin(), as.w.end());
  if (lines) {
    lines->push_back("; tree code at " + std::to_string(start * 4));
    lines->insert(lines->end(), as.lines.begin(), as.lines.end());
  }
  *off = (int32_t)(start * 4);
  *max_feat = std::max(*max_feat, g.max_feat);
  return true;
}

// Trees that compile are appended to ok_trees / offs, the others to `rest`; a
// tree that no longer fits in the area ends the call (returns its position).
size_t codegen64(const CompiledBatch<double>& cb, const std::vector<int32_t>& cand, size_t from, const Opts64& opt,
                 bool text,
                 std::vector<uint32_t>& words, std::vector<std::string>* lines, std::vector<int32_t>& offs,
                 std::vector<int32_t>& ok_trees, std::vector<int32_t>& rest, int* max_feat, Stats* st) {
  const Tmpl64& T = tmpl64();
  for (size_t k = from; k < cand.size(); ++k) {
    const int32_t t = cand[k];
    int32_t off = -1;
    std::string why;
    const size_t before = words.size(), lbefore = lines ? lines->size() : 0;
    int mf = *max_feat;
    const bool okc = cb.tree_off[t] >= 0 && gen_tree64(&cb.code[cb.tree_off[t]], T, opt, text, words, lines, &off, &mf, &why);
    if (okc && words.size() * 4 > T.area_bytes) {
      words.resize(before);
      if (lines) lines->resize(lbefore);
      return k;
    }
    if (okc) {
      *max_feat = mf;
      ok_trees.push_back(t);
      offs.push_back(off);
      if (st) st->ntrees++;
    } else {
      words.resize(before);
      if (lines) lines->resize(lbefore);
      rest.push_back(t);
      if (st) st->nrejected++;
      static const bool dbg = std::getenv("SRHIP_JIT_DEBUG") != nullptr;
      if (dbg) std::fprintf(stderr, "jit64: tree %d not compiled: %s\n", t, why.c_str());
    }
  }
  return cand.size();
}

struct Jit64Args {
  EvalArgs<double> e;
  const int32_t* code_off;
  int nraw;
};

// ---- Float64 gradient tree code: reverse-mode ∂L/∂c (jit_grad.cpp's Float64 counterpart)
//
// Tree code of one tree (L2 loss):
//   prologue  the tree's constants (s_load_dwordx16 from s[78:79]) into VGPR
//             pairs C0 + 2j, accumulators ACC + 2j = 0, routine base
//   tile      forward as the Float64 loss tree code (the interpreter's routines,
//             + - * neg abs square cube inline), every value the reverse pass
//             reads kept in its block; the root marked into CHK, a failed tile
//             ends the tree; r = ŷ - y masked past the last row, Σ w·r² into
//             LSUM, the seed 2·w·r;
//             reverse: adjoints in pool blocks (sign carried as a flag), a
//             constant's adjoint summed over the lane's rows into its
//             accumulator; the rules of device_ops.h bop_d / uop_d with the
//             Float64 routines for the quotients (b_div: g/b, g/a, 0.5g/f),
//             pow (b_pow at b - 1), log, sin and cos
//   epilogue  each accumulator summed over the wave (DPP, as the Float64 tree
//             loop's wave sum) and stored to this row group's partials at
//             s[84:85] + 8j; return
constexpr int GP0 = SR_JIT64_G_POOL0, GNP = SR_JIT64_G_NPOOL, GC0 = SR_JIT64_G_C0, GACC2 = SR_JIT64_G_ACC;
constexpr int GNACC = SR_JIT64_G_NACC, GSCPTR = SR_JIT64_G_SCPTR, GSGPTR = SR_JIT64_G_SGPTR;
// scratch VGPRs of the reverse pass (routine temporaries: free between calls)
constexpr int HX0 = 0, HX1 = 4, HTS = 8, HTP = 12, HTR = 16;
enum : int { VOPC_LT_F64 = 0x61, VOPC_NEQ_F64 = 0x6d };

enum { H_VAL = 0, H_X = 1, H_C = 2 };
struct HOpnd {
  int k = H_VAL;
  int v = -1;   // value id or feature
  int ci = -1;  // constant index within the tree
};
enum { HK_UN = 0, HK_BIN = 1, HK_MAT = 2 };  // HK_MAT: a constant broadcast into a block
struct HOp {
  int kind = HK_UN;
  int op = 0;
  HOpnd a, b;
  int rid = -1;
};
constexpr uint32_t kGrad64Uops = (1u << SRHIP_UOP_NEG) | (1u << SRHIP_UOP_ABS) | (1u << SRHIP_UOP_SQUARE) |
                                 (1u << SRHIP_UOP_CUBE) | (1u << SRHIP_UOP_EXP) | (1u << SRHIP_UOP_SIN) |
                                 (1u << SRHIP_UOP_COS) | (1u << SRHIP_UOP_LOG) | (1u << SRHIP_UOP_SQRT);
constexpr uint32_t kGrad64Bops = (1u << SRHIP_BOP_ADD) | (1u << SRHIP_BOP_SUB) | (1u << SRHIP_BOP_MUL) |
                                 (1u << SRHIP_BOP_DIV) | (1u << SRHIP_BOP_POW);

bool h_inline(const HOp& o) {
  if (o.kind == HK_MAT) return true;
  return o.kind == HK_UN ? (o.op == SRHIP_UOP_NEG || o.op == SRHIP_UOP_ABS || o.op == SRHIP_UOP_SQUARE ||
                            o.op == SRHIP_UOP_CUBE)
                         : (o.op == SRHIP_BOP_ADD || o.op == SRHIP_BOP_SUB || o.op == SRHIP_BOP_MUL);
}

bool build_hir(const Ins<double>* p, std::vector<HOp>& ops, HOpnd& root, std::string* why) {
  ops.clear();
  HOpnd acc, tmp, slot[kMaxSlots];
  auto val = [&](const HOp& o) {
    ops.push_back(o);
    HOpnd r;
    r.v = (int)ops.size() - 1;
    return r;
  };
  auto mat = [&](const HOpnd& c) {
    HOp m;
    m.kind = HK_MAT;
    m.a = c;
    return val(m);
  };
  for (int pc = 0;; ++pc) {
    if (pc > 4096) { *why = "program too long"; return false; }
    const uint32_t code = p[pc].code;
    const int opc = (int)(code & 0xffu);
    const int slotf = (int)((code >> 8) & 0xffu);
    const int f = (int)(code >> 16);
    uint64_t bits;
    std::memcpy(&bits, &p[pc].imm, 8);
    auto X = [&](int ff) { HOpnd o; o.k = H_X; o.v = ff; return o; };
    auto C = [&]() { HOpnd o; o.k = H_C; o.ci = slotf; return o; };
    if (opc == OP_END) { root = acc; return true; }
    if (opc == OP_LDX) { acc = X(f); continue; }
    if (opc == OP_LDC) { acc = C(); continue; }
    if (opc >= OP_PUSH0 && opc < OP_PUSH0 + kMaxSlots) { slot[opc - OP_PUSH0] = acc; continue; }
    if (opc >= OP_POP0 && opc < OP_POP0 + kMaxSlots) { tmp = slot[opc - OP_POP0]; continue; }
    if (opc >= OP_UN0 && opc < OP_BIN0) {
      HOp o;
      o.kind = HK_UN;
      o.op = opc - OP_UN0;
      if (!((kGrad64Uops >> o.op) & 1u)) { *why = "unary operator without gradient code"; return false; }
      o.a = acc.k == H_C ? mat(acc) : acc;
      acc = val(o);
      continue;
    }
    const int v = (opc - OP_BIN0) / SRHIP_NUM_BOPS;
    HOp o;
    o.kind = HK_BIN;
    o.op = (opc - OP_BIN0) % SRHIP_NUM_BOPS;
    if (!((kGrad64Bops >> o.op) & 1u)) { *why = "binary operator without gradient code"; return false; }
    switch (v) {
      case V_AX: o.a = acc; o.b = X(f); break;
      case V_XA: o.a = X(f); o.b = acc; break;
      case V_AC: o.a = acc; o.b = C(); break;
      case V_CA: o.a = C(); o.b = acc; break;
      case V_AT: o.a = acc; o.b = tmp; break;
      case V_TA: o.a = tmp; o.b = acc; break;
      case V_XX: o.a = X(f); o.b = X((int)bits); break;
      case V_XC: o.a = X(f); o.b = C(); break;
      case V_CX: o.a = C(); o.b = X(f); break;
      default: *why = "bad variant"; return false;
    }
    if (o.a.k == H_C && o.b.k == H_C) o.a = mat(o.a);
    acc = val(o);
  }
}

struct GradGen64 {
  Asm& as;
  const Tmpl64& T;
  uint64_t base_va;
  std::vector<HOp> ops;
  HOpnd root;
  int nc = 0;
  int loss = SRHIP_LOSS_L2;
  uint64_t lparam = 0;  // bits of the loss's Float64 parameter
  std::string why;
  int n = 0;
  std::vector<uint8_t> hasc;  // the value's subtree holds a constant: it needs an adjoint
  std::vector<int> last;      // last step (forward i, loss n, reverse 2n - i) reading the value
  std::vector<int> loc;       // pool block of each value (-1: none)
  int owner[GNP];             // -1 free, value id, 1000 + feature, 2000 + v adjoint
  int refs[GNP];
  struct Adj { int reg = -1; int blk = -2; bool neg = false; };  // blk -1: the seed block Y
  std::vector<Adj> adj;
  int xblk[64], xlast[64], load_idx[64];
  std::vector<int> feats;  // features inline operators read, preloaded per tile
  int nloads = 0, waited = 0, max_feat = -1;
  bool has_call = false;
  int L_tile = -1, L_done = -1;

  GradGen64(Asm& a, const Tmpl64& t, uint64_t va) : as(a), T(t), base_va(va) {}
  uint64_t cur_va() const { return base_va + as.bytes(); }
  static int blk(int k) { return GP0 + 4 * k; }
  int bstep(int i) const { return 2 * n - i; }
  bool needs_adj(const HOpnd& q) const { return q.k == H_C || (q.k == H_VAL && hasc[q.v]); }

  bool analyze() {
    n = (int)ops.size();
    hasc.assign(n, 0);
    last.assign(n, -1);
    loc.assign(n, -1);
    adj.assign(n, Adj());
    for (int f = 0; f < 64; ++f) { xblk[f] = -1; xlast[f] = -1; load_idx[f] = -1; }
    auto usef = [&](const HOpnd& q, int i, bool inl) {
      if (q.k != H_X) return true;
      if (q.v < 0 || q.v > 62) { why = "feature offset beyond the DS immediate"; return false; }
      max_feat = std::max(max_feat, q.v);
      if (inl) {
        if (xlast[q.v] < 0) feats.push_back(q.v);
        xlast[q.v] = std::max(xlast[q.v], i);
      }
      return true;
    };
    for (int i = 0; i < n; ++i) {
      HOp& o = ops[i];
      auto hc = [&](const HOpnd& q) { return q.k == H_C || (q.k == H_VAL && hasc[q.v]); };
      hasc[i] = o.kind == HK_MAT || hc(o.a) || (o.kind == HK_BIN && hc(o.b));
      if (o.a.k == H_C && o.a.ci >= nc) { why = "constant index out of range"; return false; }
      if (o.kind == HK_BIN && o.b.k == H_C && o.b.ci >= nc) { why = "constant index out of range"; return false; }
      const bool inl = h_inline(o);
      if (!inl) {
        o.rid = o.kind == HK_UN ? kUop64[o.op] : kBop64[o.op];
        if (o.rid < 0) { why = "operator without a Float64 routine"; return false; }
        has_call = true;
      }
      if (o.kind != HK_MAT) {
        if (!usef(o.a, i, inl)) return false;
        if (o.kind == HK_BIN && !usef(o.b, i, inl)) return false;
      }
      if (o.a.k == H_VAL && o.kind != HK_MAT) last[o.a.v] = std::max(last[o.a.v], i);
      if (o.kind == HK_BIN && o.b.k == H_VAL) last[o.b.v] = std::max(last[o.b.v], i);
    }
    if (root.k == H_C && root.ci >= nc) { why = "constant index out of range"; return false; }
    // reverse-pass reads of saved values (operands and own results)
    for (int i = 0; i < n; ++i) {
      const HOp& o = ops[i];
      if (!hasc[i] || o.kind == HK_MAT) continue;
      auto use = [&](const HOpnd& q) {
        if (q.k == H_VAL) last[q.v] = std::max(last[q.v], bstep(i));
      };
      auto own = [&]() { last[i] = std::max(last[i], bstep(i)); };
      if (o.kind == HK_BIN) {
        const bool aa = needs_adj(o.a), ab = needs_adj(o.b);
        if (o.op == SRHIP_BOP_MUL) {
          if (ab) use(o.a);
          if (aa) use(o.b);
        } else if (o.op == SRHIP_BOP_DIV) {
          use(o.b);
          if (ab) own();
        } else if (o.op == SRHIP_BOP_POW) {
          use(o.a);
          use(o.b);
          if (ab) own();
        }
      } else {
        if (o.op == SRHIP_UOP_EXP || o.op == SRHIP_UOP_SQRT) own();
        else if (o.op != SRHIP_UOP_NEG) use(o.a);
      }
    }
    if (!usef(root, n, true)) return false;
    if (root.k == H_VAL) last[root.v] = std::max(last[root.v], n);
    if ((int)feats.size() > GNP) { why = "more features than register blocks"; return false; }
    if (loss != SRHIP_LOSS_L2) {  // the seed by the loss's ℓ and dℓ/dr routines
      if (loss < 0 || loss >= SRHIP_NUM_LOSSES || kLoss64[loss] < 0 || kDLoss64[loss] < 0) {
        why = "no Float64 loss / dℓ/dr routine";
        return false;
      }
      has_call = true;
    }
    return true;
  }

  // ---- pool
  int free_block() const {
    for (int k = 0; k < GNP; ++k)
      if (owner[k] == -1) return k;
    return -1;
  }
  void free_values_at(int step) {
    for (int v = 0; v < n; ++v)
      if (last[v] == step && loc[v] >= 0 && owner[loc[v]] == v) { owner[loc[v]] = -1; loc[v] = -1; }
  }
  void free_feats_at(int step) {
    for (int f : feats)
      if (xlast[f] == step && xblk[f] >= 0 && owner[xblk[f]] == 1000 + f) owner[xblk[f]] = -1;
  }
  int new_adj_block(int v) {
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted (adjoints)"; return -1; }
    owner[k] = 2000 + v;
    refs[k] = 1;
    return k;
  }
  void release_adj(const Adj& a) {
    if (a.blk < 0) return;
    if (--refs[a.blk] == 0) owner[a.blk] = -1;
  }
  void share_adj(int v, const Adj& g, bool flip) {
    Adj a = g;
    a.neg = g.neg != flip;
    if (a.blk >= 0) ++refs[a.blk];
    adj[v] = a;
  }

  // ---- emission helpers (Float64: a register pair per row, 2 rows per block)
  static std::string pr(int r) { return "v[" + std::to_string(r) + ":" + std::to_string(r + 1) + "]"; }
  static std::string pname(const Src& s) {
    if (s.enc >= 256) return pr(s.enc - 256);
    if (s.enc < 102) return "s[" + std::to_string(s.enc) + ":" + std::to_string(s.enc + 1) + "]";
    switch (s.enc) {  // inline constants as Float64 values
      case 240: return "0.5";
      case 242: return "1.0";
      case 243: return "-1.0";
      case 244: return "2.0";
      default: return std::to_string(s.enc - 128);  // 128..192: 0..64
    }
  }
  void vop3d(int op, const char* nm, int vdst, const Src& s0, const Src& s1, const Src* s2, int neg) {
    as.put(0xd0000000u | ((uint32_t)op << 16) | (uint32_t)vdst);
    as.put(((uint32_t)(neg & 7) << 29) | ((uint32_t)(s2 ? s2->enc : 0) << 18) | ((uint32_t)s1.enc << 9) |
           (uint32_t)s0.enc);
    if (!as.want_text) return;
    auto f = [&](const Src& s, int i) { return ((neg >> i) & 1 ? "-" : "") + pname(s); };
    as.t(std::string(nm) + " " + pr(vdst) + ", " + f(s0, 0) + ", " + f(s1, 1) + (s2 ? ", " + f(*s2, 2) : ""));
  }
  void mul(int d, const Src& x, const Src& y, int neg = 0) { vop3d(VOP3_MUL_F64, "v_mul_f64", d, x, y, nullptr, neg); }
  void movd(int dst, const Src& src) {  // one Float64 (a register pair, or a constant's pair)
    as.vop3p(VOP3P_MOV_B32, "v_pk_mov_b32", dst, src, src, nullptr, 2, 7, 0, 0);
  }
  void mov_block(int dst, int src) {
    if (dst == src) return;
    movd(dst, V(src));
    movd(dst + 2, V(src + 2));
  }
  void vopc64(int op, const char* nm, const Src& s0, int vsrc1) {
    as.put(0x7c000000u | ((uint32_t)op << 17) | ((uint32_t)vsrc1 << 9) | (uint32_t)s0.enc);
    if (as.want_text) as.t(std::string(nm) + " vcc, " + pname(s0) + ", " + pr(vsrc1));
  }
  void wait_for(int f) {
    const int li = load_idx[f];
    if (li >= waited) {
      as.waitcnt_lgkm(nloads - 1 - li);
      waited = li + 1;
    }
  }
  void wait_all() {
    if (waited < nloads) { as.waitcnt_lgkm(0); waited = nloads; }
  }
  void set_base() {
    as.sop1(SOP1_GETPC, "s_getpc_b64", T_BASE, Src{0, false, 0}, "");
    if (as.want_text) as.lines.back() = "s_getpc_b64 s[" + std::to_string(T_BASE) + ":" + std::to_string(T_BASE + 1) + "]";
    const int64_t rel = (int64_t)(T.rt0 - cur_va());
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_BASE, S(T_BASE), K((uint32_t)(uint64_t)rel));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", T_BASE + 1, S(T_BASE + 1), K((uint32_t)((uint64_t)rel >> 32)));
  }
  void routine(int rid) {
    const uint64_t off = T.rt_va[rid] - T.rt0;
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_TGT, S(T_BASE), K((uint32_t)off));
    as.sop2(SOP2_ADDC_U32, "s_addc_u32", T_TGT + 1, S(T_BASE + 1), K((uint32_t)(off >> 32)));
    as.sop1(SOP1_SWAPPC, "s_swappc_b64", T_RR, S(T_TGT), "");
    if (as.want_text)
      as.lines.back() = "s_swappc_b64 s[" + std::to_string(T_RR) + ":" + std::to_string(T_RR + 1) + "], s[" +
                        std::to_string(T_TGT) + ":" + std::to_string(T_TGT + 1) + "]";
  }
  Src cpair(int ci) const { return V(GC0 + 2 * ci); }
  // forward operand of row e
  Src fsrc(const HOpnd& q, int e) {
    if (q.k == H_C) return cpair(q.ci);
    if (q.k == H_X) return V(blk(xblk[q.v]) + 2 * e);
    return V(blk(loc[q.v]) + 2 * e);
  }
  void operand_to(int dst, const HOpnd& q) {
    if (q.k == H_VAL) { mov_block(dst, blk(loc[q.v])); return; }
    if (q.k == H_X) {
      as.ds_read_b128(dst, LANE2, (1 + q.v) * TILE2 * 8);
      as.waitcnt_lgkm(0);
      waited = nloads;
      return;
    }
    movd(dst, cpair(q.ci));
    movd(dst + 2, cpair(q.ci));
  }

  // ---- forward
  bool emit_mat(int i) {
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted"; return false; }
    movd(blk(k), cpair(ops[i].a.ci));
    movd(blk(k) + 2, cpair(ops[i].a.ci));
    owner[k] = i;
    loc[i] = k;
    return true;
  }
  bool emit_inline(int i) {
    const HOp& o = ops[i];
    if (o.a.k == H_X) wait_for(o.a.v);
    if (o.kind == HK_BIN && o.b.k == H_X) wait_for(o.b.v);
    Src a[R2], b[R2];
    for (int e = 0; e < R2; ++e) {
      a[e] = fsrc(o.a, e);
      if (o.kind == HK_BIN) b[e] = fsrc(o.b, e);
    }
    free_values_at(i);  // blocks dying here may hold the result (rows are independent)
    free_feats_at(i);
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted"; return false; }
    const int d = blk(k);
    for (int e = 0; e < R2; ++e) {
      const int de = d + 2 * e;
      if (o.kind == HK_UN) {
        const int ar = a[e].enc - 256;
        switch (o.op) {
          case SRHIP_UOP_NEG:
          case SRHIP_UOP_ABS:
            as.vop1(VOP1_MOV, "v_mov_b32_e32", de, V(ar));
            if (o.op == SRHIP_UOP_NEG) as.vop2(VOP2_XOR_B32, "v_xor_b32_e32", de + 1, K(0x80000000u), ar + 1);
            else as.vop2(VOP2_AND_B32, "v_and_b32_e32", de + 1, K(0x7fffffffu), ar + 1);
            break;
          case SRHIP_UOP_SQUARE: mul(de, a[e], a[e]); break;
          default: {  // CUBE = (x*x)*x
            const int t = (de == ar) ? GT2 + 2 * e : de;
            mul(t, a[e], a[e]);
            mul(de, V(t), a[e]);
          }
        }
      } else {
        switch (o.op) {
          case SRHIP_BOP_ADD: vop3d(VOP3_ADD_F64, "v_add_f64", de, a[e], b[e], nullptr, 0); break;
          case SRHIP_BOP_SUB: vop3d(VOP3_ADD_F64, "v_add_f64", de, a[e], b[e], nullptr, 2); break;
          default: mul(de, a[e], b[e]);
        }
      }
    }
    owner[k] = i;
    loc[i] = k;
    return true;
  }
  bool emit_call(int i) {
    const HOp& o = ops[i];
    operand_to(A2, o.a);
    if (o.kind == HK_BIN) operand_to(B2, o.b);
    free_values_at(i);
    free_feats_at(i);
    routine(o.rid);
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted"; return false; }
    mov_block(blk(k), A2);
    owner[k] = i;
    loc[i] = k;
    return true;
  }

  // ---- reverse
  void acc_add(int ci, int reg, bool neg) {  // acc_ci ±= row 0 + row 1
    vop3d(VOP3_ADD_F64, "v_add_f64", HTS, V(reg), V(reg + 2), nullptr, 0);
    const Src acc = V(GACC2 + 2 * ci), t = V(HTS);
    vop3d(VOP3_ADD_F64, "v_add_f64", GACC2 + 2 * ci, acc, t, nullptr, neg ? 2 : 0);
  }
  void acc_fma(int ci, const Src& x, const Src& y, bool neg) {  // acc_ci ±= x·y (one rounding)
    const Src acc = V(GACC2 + 2 * ci);
    vop3d(VOP3_FMA_F64, "v_fma_f64", GACC2 + 2 * ci, x, y, &acc, neg ? 1 : 0);
  }
  void mask_nonpos(int d, const HOpnd& q, int scratch) {  // d = 0 where !(0 < q) (both rows)
    for (int e = 0; e < R2; ++e) {
      int ar;
      if (q.k == H_C) { movd(HTR + 2 * e, cpair(q.ci)); ar = HTR + 2 * e; }
      else ar = (q.k == H_X ? scratch : blk(loc[q.v])) + 2 * e;
      vopc64(VOPC_LT_F64, "v_cmp_lt_f64_e32", K(0), ar);
      as.sopp(0x00, "s_nop", 1);  // VALU-written VCC read as a VALU mask
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", d + 2 * e, K(0), d + 2 * e, ", vcc");
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", d + 2 * e + 1, K(0), d + 2 * e + 1, ", vcc");
    }
  }

  bool emit_reverse(int i) {
    const HOp& o = ops[i];
    const Adj g = adj[i];
    if (g.reg < 0) { why = "internal: adjoint missing"; return false; }
    auto gv = [&](int e) { return V(g.reg + 2 * e); };
    auto rsrc = [&](const HOpnd& q, int scratch, int e) {
      if (q.k == H_C) return cpair(q.ci);
      if (q.k == H_X) return V(scratch + 2 * e);
      return V(blk(loc[q.v]) + 2 * e);
    };
    auto fetch = [&](const HOpnd& q, int scratch) {
      if (q.k == H_X) {
        as.ds_read_b128(scratch, LANE2, (1 + q.v) * TILE2 * 8);
        as.waitcnt_lgkm(0);
      }
    };
    auto give = [&](const HOpnd& q, int reg, bool neg, int b) {
      if (q.k == H_C) { acc_add(q.ci, reg, neg); return; }
      Adj a;
      a.reg = reg;
      a.blk = b;
      a.neg = neg;
      adj[q.v] = a;
    };
    auto dest = [&](const HOpnd& q, int tmp, int* b) {
      *b = -2;
      if (q.k != H_VAL) return tmp;
      const int k = new_adj_block(q.v);
      if (k < 0) return -1;
      *b = k;
      return blk(k);
    };
    const int own = o.kind == HK_MAT ? -1 : (loc[i] >= 0 ? blk(loc[i]) : -1);
    if (o.kind == HK_MAT) {
      acc_add(o.a.ci, g.reg, g.neg);
    } else if (o.kind == HK_BIN) {
      const bool aa = needs_adj(o.a), ab = needs_adj(o.b);
      switch (o.op) {
        case SRHIP_BOP_ADD:
        case SRHIP_BOP_SUB:
          if (aa) {
            if (o.a.k == H_C) acc_add(o.a.ci, g.reg, g.neg);
            else share_adj(o.a.v, g, false);
          }
          if (ab) {
            const bool fl = o.op == SRHIP_BOP_SUB;
            if (o.b.k == H_C) acc_add(o.b.ci, g.reg, g.neg != fl);
            else share_adj(o.b.v, g, fl);
          }
          break;
        case SRHIP_BOP_MUL: {
          fetch(o.a, HX0);
          fetch(o.b, HX1);
          if (aa && o.a.k == H_C) {
            for (int e = 0; e < R2; ++e) acc_fma(o.a.ci, gv(e), rsrc(o.b, HX1, e), g.neg);
          } else if (aa) {
            int b;
            const int d = dest(o.a, HTP, &b);
            if (d < 0) return false;
            for (int e = 0; e < R2; ++e) mul(d + 2 * e, rsrc(o.b, HX1, e), gv(e));
            give(o.a, d, g.neg, b);
          }
          if (ab && o.b.k == H_C) {
            for (int e = 0; e < R2; ++e) acc_fma(o.b.ci, gv(e), rsrc(o.a, HX0, e), g.neg);
          } else if (ab) {
            int b;
            const int d = dest(o.b, HTP, &b);
            if (d < 0) return false;
            for (int e = 0; e < R2; ++e) mul(d + 2 * e, rsrc(o.a, HX0, e), gv(e));
            give(o.b, d, g.neg, b);
          }
          break;
        }
        case SRHIP_BOP_DIV: {  // q = a / b: ∂a = g / b (b_div), ∂b = -(g / b)·q
          mov_block(A2, g.reg);
          operand_to(B2, o.b);
          routine(kBop64[SRHIP_BOP_DIV]);
          if (ab) {
            if (o.b.k == H_C) {
              for (int e = 0; e < R2; ++e) acc_fma(o.b.ci, V(A2 + 2 * e), V(own + 2 * e), !g.neg);
            } else {
              int b;
              const int d = dest(o.b, HTP, &b);
              if (d < 0) return false;
              for (int e = 0; e < R2; ++e) mul(d + 2 * e, V(A2 + 2 * e), V(own + 2 * e));
              give(o.b, d, !g.neg, b);
            }
          }
          if (aa) {
            if (o.a.k == H_C) {
              acc_add(o.a.ci, A2, g.neg);
            } else {
              int b;
              const int d = dest(o.a, HTP, &b);
              if (d < 0) return false;
              mov_block(d, A2);
              give(o.a, d, g.neg, b);
            }
          }
          break;
        }
        default: {  // POW: f = a^b; ∂a = g·b·safe_pow(a, b - 1), ∂b = g·f·log(a) where a > 0, else 0
          if (aa) {
            operand_to(A2, o.a);
            operand_to(B2, o.b);
            for (int e = 0; e < R2; ++e)
              vop3d(VOP3_ADD_F64, "v_add_f64", B2 + 2 * e, V(B2 + 2 * e), K(0xbf800000u), nullptr, 0);  // b - 1
            routine(kBop64[SRHIP_BOP_POW]);
            fetch(o.b, HX1);
            int b;
            const int d = dest(o.a, HTP, &b);
            if (d < 0) return false;
            for (int e = 0; e < R2; ++e) {
              mul(d + 2 * e, rsrc(o.b, HX1, e), V(A2 + 2 * e));
              mul(d + 2 * e, V(d + 2 * e), gv(e));
            }
            give(o.a, d, g.neg, b);
          }
          if (ab) {
            operand_to(A2, o.a);
            routine(kUop64[SRHIP_UOP_LOG]);
            fetch(o.a, HX0);
            int b;
            const int d = dest(o.b, HTP, &b);
            if (d < 0) return false;
            for (int e = 0; e < R2; ++e) {
              mul(d + 2 * e, V(own + 2 * e), V(A2 + 2 * e));
              mul(d + 2 * e, V(d + 2 * e), gv(e));
            }
            mask_nonpos(d, o.a, HX0);
            give(o.b, d, g.neg, b);
          }
        }
      }
    } else {
      // unary: the operand is a value (constants were materialised) or a feature
      if (!needs_adj(o.a)) { release_adj(g); return true; }
      const int ar = blk(loc[o.a.v]);
      int b;
      switch (o.op) {
        case SRHIP_UOP_NEG:
          share_adj(o.a.v, g, true);
          break;
        case SRHIP_UOP_EXP: {
          const int d = dest(o.a, HTP, &b);
          if (d < 0) return false;
          for (int e = 0; e < R2; ++e) mul(d + 2 * e, gv(e), V(own + 2 * e));
          give(o.a, d, g.neg, b);
          break;
        }
        case SRHIP_UOP_SQUARE:
        case SRHIP_UOP_CUBE: {  // 2x; (3x)x
          const int d = dest(o.a, HTP, &b);
          if (d < 0) return false;
          if (o.op == SRHIP_UOP_CUBE) {  // 3.0 in s[20:21] (a routine temporary)
            as.sop1(SOP1_MOV, "s_mov_b32", 20, K(0), "s20");
            as.sop1(SOP1_MOV, "s_mov_b32", 21, K(0x40080000u), "s21");
          }
          for (int e = 0; e < R2; ++e) {
            if (o.op == SRHIP_UOP_SQUARE) {
              mul(d + 2 * e, K(0x40000000u), V(ar + 2 * e));
            } else {
              mul(d + 2 * e, S(20), V(ar + 2 * e));
              mul(d + 2 * e, V(d + 2 * e), V(ar + 2 * e));
            }
            mul(d + 2 * e, gv(e), V(d + 2 * e));
          }
          give(o.a, d, g.neg, b);
          break;
        }
        case SRHIP_UOP_ABS: {  // g with a's sign, 0 where a = 0
          const int d = dest(o.a, HTP, &b);
          if (d < 0) return false;
          for (int e = 0; e < R2; ++e) {
            const int de = d + 2 * e, ae = ar + 2 * e, ge = g.reg + 2 * e;
            as.vop2(VOP2_AND_B32, "v_and_b32_e32", de + 1, K(0x80000000u), ae + 1);
            as.vop2(VOP2_XOR_B32, "v_xor_b32_e32", de + 1, V(ge + 1), de + 1);
            as.vop1(VOP1_MOV, "v_mov_b32_e32", de, V(ge));
            vopc64(VOPC_NEQ_F64, "v_cmp_neq_f64_e32", K(0), ae);
            as.sopp(0x00, "s_nop", 1);
            as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", de, K(0), de, ", vcc");
            as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", de + 1, K(0), de + 1, ", vcc");
          }
          give(o.a, d, g.neg, b);
          break;
        }
        case SRHIP_UOP_LOG:    // g / a
        case SRHIP_UOP_SQRT: {  // (0.5 g) / f
          if (o.op == SRHIP_UOP_LOG) {
            mov_block(A2, g.reg);
            mov_block(B2, ar);
          } else {
            for (int e = 0; e < R2; ++e) mul(A2 + 2 * e, gv(e), K(0x3f000000u));
            mov_block(B2, own);
          }
          routine(kBop64[SRHIP_BOP_DIV]);
          const int d = dest(o.a, HTP, &b);
          if (d < 0) return false;
          mov_block(d, A2);
          give(o.a, d, g.neg, b);
          break;
        }
        default: {  // SIN: g cos(a); COS: -g sin(a)
          const bool is_sin = o.op == SRHIP_UOP_SIN;
          mov_block(A2, ar);
          routine(kUop64[is_sin ? SRHIP_UOP_COS : SRHIP_UOP_SIN]);
          const int d = dest(o.a, HTP, &b);
          if (d < 0) return false;
          for (int e = 0; e < R2; ++e) mul(d + 2 * e, gv(e), V(A2 + 2 * e));
          give(o.a, d, g.neg != !is_sin, b);
        }
      }
    }
    release_adj(g);
    return true;
  }

  void emit_mask(int reg) {  // rows past the last of the last tile: 0 in block `reg`
    const int L_nomask = as.label();
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_PE, S(T_TILE), K(1));
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_PE), S(T_NT));
    as.branch(SOPP_SCC0, "s_cbranch_scc0", L_nomask);
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_PARTIAL), K((uint32_t)TILE2));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_nomask);
    for (int e = 0; e < R2; ++e) {
      as.sop2(SOP2_SUB_I32, "s_sub_i32", T_PE, S(T_PARTIAL), K((uint32_t)e));
      as.vopc(VOPC_GT_I32, "v_cmp_gt_i32_e32", S(T_PE), LROW2);
      as.sopp(0x00, "s_nop", 1);
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", reg + 2 * e, K(0), reg + 2 * e, ", vcc");
      as.vop2(VOP2_CNDMASK, "v_cndmask_b32_e32", reg + 2 * e + 1, K(0), reg + 2 * e + 1, ", vcc");
    }
    as.bind(L_nomask);
  }

  // any other elementwise loss: Σ w·ℓ(r) into LSUM and the seed w·ℓ'(r) into
  // Y (r in Y, 0 past the last row), ℓ and ℓ' by the Float64 loss routines
  // (device_ops.h elem_loss / elem_dloss, the parameter in s_k : s_kh), both
  // masked after the call (ℓ'(0) need not be 0: Quantile's is τ); LSUM in the
  // Float64 loss tree code's order (Gen64::emit_tail_loss)
  bool emit_loss_seed() {
    const int k = free_block();
    if (k < 0) { why = "register pool exhausted (loss)"; return false; }
    const int rb = blk(k);
    mov_block(rb, Y2);
    mov_block(A2, Y2);
    as.sop1(SOP1_MOV, "s_mov_b32", T_K, K((uint32_t)lparam), "s" + std::to_string(T_K));
    as.sop1(SOP1_MOV, "s_mov_b32", T_KH, K((uint32_t)(lparam >> 32)), "s" + std::to_string(T_KH));
    routine(kLoss64[loss]);
    mov_block(Y2, A2);
    mov_block(A2, rb);
    routine(kDLoss64[loss]);
    const int L_unw = as.label();
    as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_WOFF), K(0));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", GT2, S(T_WOFF), LANE2);
    as.ds_read_b128(GT2, GT2, 0);
    as.waitcnt_lgkm(0);
    for (int e = 0; e < R2; ++e) {
      mul(Y2 + 2 * e, V(GT2 + 2 * e), V(Y2 + 2 * e));
      mul(A2 + 2 * e, V(GT2 + 2 * e), V(A2 + 2 * e));
    }
    as.bind(L_unw);
    emit_mask(Y2);
    emit_mask(A2);
    for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", LSUM2, V(LSUM2), V(Y2 + 2 * e), nullptr, 0);
    mov_block(Y2, A2);
    return true;
  }

  void dpp_mov(int vdst, int vsrc, uint32_t ctrl, uint32_t row, const char* txt) {
    as.put(0x7e000000u | ((uint32_t)vdst << 17) | ((uint32_t)VOP1_MOV << 9) | 0xfau);
    as.put((uint32_t)vsrc | (ctrl << 8) | (0xfu << 24) | (row << 28));
    if (as.want_text)
      as.lines.push_back("v_mov_b32_dpp v" + std::to_string(vdst) + ", v" + std::to_string(vsrc) + " " + txt +
                         " bank_mask:0xf");
  }

  bool emit_tree() {
    if (!analyze()) return false;
    for (int k = 0; k < GNP; ++k) { owner[k] = -1; refs[k] = 0; }
    L_tile = as.label();
    L_done = as.label();
    // ---- prologue: constants into VGPR pairs, accumulators 0
    as.sop1(SOP1_MOV, "s_mov_b32", T_STATUS, K(0), "s" + std::to_string(T_STATUS));
    for (int c0 = 0; c0 < nc; c0 += 8) {  // s_load_dwordx16 s[0:15], s[78:79], 64·chunk (routine temporaries)
      as.put(0xc0020000u | (4u << 18) | (0u << 6) | (uint32_t)(GSCPTR >> 1));
      as.put((uint32_t)(c0 * 8));
      if (as.want_text)
        as.lines.push_back("s_load_dwordx16 s[0:15], s[" + std::to_string(GSCPTR) + ":" + std::to_string(GSCPTR + 1) +
                           "], " + detail::hex32((uint32_t)(c0 * 8)));
      as.waitcnt_lgkm(0);
      for (int j = c0; j < std::min(nc, c0 + 8); ++j) {
        as.vop1(VOP1_MOV, "v_mov_b32_e32", GC0 + 2 * j, S(2 * (j - c0)));
        as.vop1(VOP1_MOV, "v_mov_b32_e32", GC0 + 2 * j + 1, S(2 * (j - c0) + 1));
      }
    }
    for (int j = 0; j < 2 * nc; ++j) as.vop1(VOP1_MOV, "v_mov_b32_e32", GACC2 + j, K(0));
    if (has_call) set_base();
    as.sopc(SOPC_GE_U32, "s_cmp_ge_u32", S(T_TILE), S(T_NT));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_done);
    // ---- tile: forward
    as.bind(L_tile);
    nloads = 0;
    waited = 0;
    as.ds_read_b128(Y2, LANE2, 0);
    ++nloads;
    for (size_t j = 0; j < feats.size(); ++j) {
      const int f = feats[j];
      xblk[f] = (int)j;
      owner[j] = 1000 + f;
      load_idx[f] = nloads++;
      as.ds_read_b128(blk((int)j), LANE2, (1 + f) * TILE2 * 8);
    }
    std::fill(loc.begin(), loc.end(), -1);
    for (int i = 0; i < n; ++i) {
      const HOp& o = ops[i];
      const bool ok = o.kind == HK_MAT ? emit_mat(i) : h_inline(o) ? emit_inline(i) : emit_call(i);
      if (!ok) return false;
    }
    int rreg;
    if (root.k == H_VAL) rreg = blk(loc[root.v]);
    else if (root.k == H_X) { wait_for(root.v); rreg = blk(xblk[root.v]); }
    else {
      movd(GT2, cpair(root.ci));
      movd(GT2 + 2, cpair(root.ci));
      rreg = GT2;
    }
    for (int e = 0; e < R2; ++e) {  // chk = fma(v, 0, chk): NaN for a non-finite root value
      const Src r = V(rreg + 2 * e), z = K(0), c = V(CHK2);
      vop3d(VOP3_FMA_F64, "v_fma_f64", CHK2, r, z, &c, 0);
    }
    wait_all();
    // a failed tile ends the tree (no reverse pass)
    as.put(0x7c000000u | ((uint32_t)VOPC_U_F64 << 17) | ((uint32_t)CHK2 << 9) | (uint32_t)(256 + CHK2));
    if (as.want_text) as.t("v_cmp_u_f64_e32 vcc, " + pr(CHK2) + ", " + pr(CHK2));
    as.branch(SOPP_VCCNZ, "s_cbranch_vccnz", L_done);
    // ---- loss of the tile and the seed 2·w·r (masked rows: r = 0)
    for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", Y2 + 2 * e, V(rreg + 2 * e), V(Y2 + 2 * e), nullptr, 2);
    free_values_at(n);
    free_feats_at(n);
    emit_mask(Y2);
    if (loss != SRHIP_LOSS_L2) {
      if (!emit_loss_seed()) return false;
    } else {
      const int L_unw = as.label(), L_seed = as.label();
      as.sopc(SOPC_EQ_U32, "s_cmp_eq_u32", S(T_WOFF), K(0));
      as.branch(SOPP_SCC1, "s_cbranch_scc1", L_unw);
      as.vop2(VOP2_ADD_U32, "v_add_u32_e32", GT2, S(T_WOFF), LANE2);
      as.ds_read_b128(GT2, GT2, 0);
      as.waitcnt_lgkm(0);
      for (int e = 0; e < R2; ++e) {  // Σ w·(r·r), the Float64 loss code's order; seed w·r
        const Src r = V(Y2 + 2 * e);
        mul(HTP + 2 * e, r, r);
        const Src w = V(GT2 + 2 * e), t = V(HTP + 2 * e), l = V(LSUM2);
        vop3d(VOP3_FMA_F64, "v_fma_f64", LSUM2, w, t, &l, 0);
        mul(Y2 + 2 * e, w, r);
      }
      as.branch(SOPP_BRANCH, "s_branch", L_seed);
      as.bind(L_unw);
      for (int e = 0; e < R2; ++e) {
        const Src r = V(Y2 + 2 * e), l = V(LSUM2);
        vop3d(VOP3_FMA_F64, "v_fma_f64", LSUM2, r, r, &l, 0);
      }
      as.bind(L_seed);
      for (int e = 0; e < R2; ++e) vop3d(VOP3_ADD_F64, "v_add_f64", Y2 + 2 * e, V(Y2 + 2 * e), V(Y2 + 2 * e), nullptr, 0);
    }
    // ---- reverse pass
    if (root.k == H_C) acc_add(root.ci, Y2, false);
    else if (root.k == H_VAL && hasc[root.v]) {
      Adj s;
      s.reg = Y2;
      s.blk = -1;
      adj[root.v] = s;
    }
    for (int i = n - 1; i >= 0; --i) {
      if (hasc[i] && !emit_reverse(i)) return false;
      free_values_at(bstep(i));
    }
    for (int k = 0; k < GNP; ++k)
      if (owner[k] != -1) { why = "internal: block live after the reverse pass"; return false; }
    // ---- next tile
    as.vop2(VOP2_ADD_U32, "v_add_u32_e32", LANE2, S(T_TILEBYTES), LANE2);
    as.sop2(SOP2_ADD_U32, "s_add_u32", T_TILE, S(T_TILE), K(1));
    as.sopc(SOPC_LT_U32, "s_cmp_lt_u32", S(T_TILE), S(T_NT));
    as.branch(SOPP_SCC1, "s_cbranch_scc1", L_tile);
    // ---- epilogue: each accumulator summed over the wave (the Float64 tree
    // loop's DPP steps: lane 63 holds the sum), stored to this row group's
    // partial of its constant; return
    as.bind(L_done);
    static const struct { uint32_t ctrl, row; bool zero; const char* txt; } steps[] = {
        {0x0b1, 0xf, false, "quad_perm:[1,0,3,2] row_mask:0xf"}, {0x04e, 0xf, false, "quad_perm:[2,3,0,1] row_mask:0xf"},
        {0x141, 0xf, false, "row_half_mirror row_mask:0xf"},     {0x140, 0xf, false, "row_mirror row_mask:0xf"},
        {0x142, 0xa, true, "row_bcast:15 row_mask:0xa"},         {0x143, 0xc, true, "row_bcast:31 row_mask:0xc"}};
    if (nc > 0) as.vop1(VOP1_MOV, "v_mov_b32_e32", HTS + 2, K(0));  // the store's zero offset
    for (int j = 0; j < nc; ++j) {
      const int a = GACC2 + 2 * j;
      for (const auto& st : steps) {
        if (st.zero) {
          as.vop1(VOP1_MOV, "v_mov_b32_e32", HTS, K(0));
          as.vop1(VOP1_MOV, "v_mov_b32_e32", HTS + 1, K(0));
        }
        as.sopp(0x00, "s_nop", 1);  // a DPP source must not be written by the 2 VALU instructions before
        dpp_mov(HTS, a, st.ctrl, st.row, st.txt);
        dpp_mov(HTS + 1, a + 1, st.ctrl, st.row, st.txt);
        vop3d(VOP3_ADD_F64, "v_add_f64", a, V(a), V(HTS), nullptr, 0);
      }
      as.sopp(0x00, "s_nop", 1);
      for (int h = 0; h < 2; ++h) {  // v_readlane_b32 s(20+h), v(a+h), 63
        as.put(0xd2890000u | (uint32_t)(20 + h));
        as.put((uint32_t)(256 + a + h) | (191u << 9));
        if (as.want_text) as.lines.push_back("v_readlane_b32 s" + std::to_string(20 + h) + ", v" + std::to_string(a + h) + ", 63");
      }
      as.sopp(0x00, "s_nop", 4);
      as.vop1(VOP1_MOV, "v_mov_b32_e32", HTS, S(20));
      as.vop1(VOP1_MOV, "v_mov_b32_e32", HTS + 1, S(21));
      // global_store_dwordx2 v[HTS+2] (= 0), v[HTS:HTS+1], s[SGPTR:SGPTR+1] offset:8j
      as.put(0xdc748000u | (uint32_t)((8 * j) & 0x1fff));
      as.put((uint32_t)(HTS + 2) | ((uint32_t)HTS << 8) | ((uint32_t)GSGPTR << 16));
      if (as.want_text)
        as.lines.push_back("global_store_dwordx2 v" + std::to_string(HTS + 2) + ", " + pr(HTS) + ", s[" +
                           std::to_string(GSGPTR) + ":" + std::to_string(GSGPTR + 1) + "]" +
                           (j ? " offset:" + std::to_string(8 * j) : ""));
    }
    as.sop1(SOP1_SETPC, "s_setpc_b64", 0, S(T_RT), "");
    if (as.want_text) as.lines.back() = "s_setpc_b64 s[" + std::to_string(T_RT) + ":" + std::to_string(T_RT + 1) + "]";
    return true;
  }
};

bool gen_grad_tree64(const Ins<double>* prog, int nc, const Tmpl64& T, bool text, std::vector<uint32_t>& out,
                     std::vector<std::string>* lines, int32_t* off, int* max_feat, std::string* why, int loss,
                     uint64_t lparam) {
  if (nc > GNACC) { *why = "more constants than accumulators"; return false; }
  std::vector<HOp> ir;
  HOpnd root;
  if (!build_hir(prog, ir, root, why)) return false;
  const size_t start = (out.size() + 15) / 16 * 16;
  Asm as;
  as.want_text = text;
  GradGen64 g(as, T, T.area_va + start * 4);
  g.ops = ir;
  g.root = root;
  g.nc = nc;
  g.loss = loss;
  g.lparam = lparam;
  if (!g.emit_tree()) { *why = g.why; return false; }
  as.finish();
  while (out.size() < start) {
    out.push_back(0xbf800000u);
    if (lines) lines->push_back("s_nop 0");
  }
  out.insert(out.end(), as.w.begin(), as.w.end());
  if (lines) {
    lines->push_back("; gradient tree code at " + std::to_string(start * 4));
    lines->insert(lines->end(), as.lines.begin(), as.lines.end());
  }
  *off = (int32_t)(start * 4);
  *max_feat = std::max(*max_feat, g.max_feat);
  return true;
}

size_t grad_codegen64(const CompiledBatch<double>& cb, const std::vector<int32_t>& const_off,
                      const std::vector<int32_t>& cand, size_t from, bool text, std::vector<uint32_t>& words,
                      std::vector<std::string>* lines, std::vector<int32_t>& offs, std::vector<int32_t>& ok_trees,
                      std::vector<int32_t>& rest, int* max_feat, GradStats* st, int loss, uint64_t lparam) {
  const Tmpl64& T = tmpl64();
  for (size_t k = from; k < cand.size(); ++k) {
    const int32_t t = cand[k];
    int32_t off = -1;
    std::string why;
    const size_t before = words.size(), lbefore = lines ? lines->size() : 0;
    int mf = *max_feat;
    const int nc = const_off[t + 1] - const_off[t];
    const bool okc = cb.tree_off[t] >= 0 &&
                     gen_grad_tree64(&cb.code[cb.tree_off[t]], nc, T, text, words, lines, &off, &mf, &why, loss, lparam);
    if (okc && words.size() * 4 > T.area_bytes) {
      words.resize(before);
      if (lines) lines->resize(lbefore);
      return k;
    }
    if (okc) {
      *max_feat = mf;
      ok_trees.push_back(t);
      offs.push_back(off);
      if (st) st->ntrees++;
    } else {
      words.resize(before);
      if (lines) lines->resize(lbefore);
      rest.push_back(t);
      if (st) st->nrejected++;
      static const bool dbg = std::getenv("SRHIP_JIT_DEBUG") != nullptr;
      if (dbg) std::fprintf(stderr, "jit64-grad: tree %d not compiled: %s\n", t, why.c_str());
    }
  }
  return cand.size();
}

struct Jit64GradArgs {
  EvalArgs<double> e;
  const int32_t* code_off;
  const double* consts;
  const int32_t* cbase;
  double* gpart;
  int nconst;
  int nraw;
};

}  // namespace

struct GradPart64 {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr, fn_w = nullptr;
  hipFunction_t fn_dl = nullptr, fn_dlw = nullptr;  // the hand-written tree loop (sr_jit64_grad_dl)
  int32_t* d_off = nullptr;    // [nslots] code offsets
  int32_t* d_cbase = nullptr;  // [nslots] first constant of the slot's tree
  int slot0 = 0, nslots = 0;
};
struct GradModule64 {
  std::vector<GradPart64> parts;
  int nslots = 0;
  int nraw = 0;
};

GradModule64* build_grad64(const CompiledBatch<double>& cb, const std::vector<int32_t>& const_off,
                           const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list, std::vector<int32_t>& rest,
                           GradStats* st, int loss, uint64_t lparam) {
  const Tmpl64& T = tmpl64();
  if (!T.ok) { rest = cand; return nullptr; }
  const auto t0 = std::chrono::steady_clock::now();
  struct Chunk { std::vector<uint32_t> words; std::vector<int32_t> offs, slots; };
  std::vector<Chunk> chunks;
  int max_feat = -1;
  size_t pos = 0, bytes = 0;
  constexpr int kMaxParts = 8;
  while (pos < cand.size()) {
    Chunk ch;
    const size_t next = grad_codegen64(cb, const_off, cand, pos, false, ch.words, nullptr, ch.offs, ch.slots, rest,
                                       &max_feat, st, loss, lparam);
    if (next == pos) { rest.push_back(cand[pos]); if (st) st->nrejected++; pos = next + 1; continue; }
    if ((int)chunks.size() + 1 == kMaxParts && next < cand.size()) {
      for (size_t k = next; k < cand.size(); ++k) rest.push_back(cand[k]);
      if (st) st->nrejected += (int)(cand.size() - next);
      pos = cand.size();
    } else {
      pos = next;
    }
    if (ch.slots.empty()) continue;
    bytes += ch.words.size() * 4;
    chunks.push_back(std::move(ch));
  }
  if (chunks.empty()) return nullptr;
  const auto t1 = std::chrono::steady_clock::now();
  GradModule64* m = new GradModule64();
  m->nraw = max_feat + 1;
  try {
    for (Chunk& ch : chunks) {
      GradPart64 pt;
      pt.slot0 = m->nslots;
      pt.nslots = (int)ch.slots.size();
      m->parts.push_back(pt);
      GradPart64& q = m->parts.back();
      std::vector<uint8_t> img(T.img, T.img + T.size);
      std::memcpy(img.data() + T.area_off, ch.words.data(), ch.words.size() * 4);
      HIP_CHECK(hipModuleLoadData(&q.mod, img.data()));
      HIP_CHECK(hipModuleGetFunction(&q.fn, q.mod, "sr_jit64_grad"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_w, q.mod, "sr_jit64_grad_w"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_dl, q.mod, "sr_jit64_grad_dl"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_dlw, q.mod, "sr_jit64_grad_dlw"));
      for (hipFunction_t f : {q.fn, q.fn_w, q.fn_dl, q.fn_dlw})
        HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
      std::vector<int32_t> cbase(ch.slots.size());
      for (size_t k = 0; k < ch.slots.size(); ++k) cbase[k] = const_off[ch.slots[k]];
      HIP_CHECK(hipMalloc((void**)&q.d_off, ch.offs.size() * sizeof(int32_t)));
      HIP_CHECK(hipMemcpy(q.d_off, ch.offs.data(), ch.offs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      HIP_CHECK(hipMalloc((void**)&q.d_cbase, cbase.size() * sizeof(int32_t)));
      HIP_CHECK(hipMemcpy(q.d_cbase, cbase.data(), cbase.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      m->nslots += pt.nslots;
      jit_list.insert(jit_list.end(), ch.slots.begin(), ch.slots.end());
    }
  } catch (...) {
    destroy_grad64(m);
    throw;
  }
  if (st) {
    st->ms_codegen = std::chrono::duration<double, std::milli>(t1 - t0).count();
    st->ms_load = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    st->code_bytes = bytes;
    st->nparts = (int)chunks.size();
  }
  return m;
}

void destroy_grad64(GradModule64* m) {
  if (!m) return;
  for (GradPart64& q : m->parts) {
    for (void* p : {(void*)q.d_off, (void*)q.d_cbase})
      if (p) (void)hipFree(p);
    if (q.mod) (void)hipModuleUnload(q.mod);
  }
  delete m;
}

int grad64_nslots(const GradModule64* m) { return m ? m->nslots : 0; }
int grad64_nparts(const GradModule64* m) { return m ? (int)m->parts.size() : 0; }
void grad64_part(const GradModule64* m, int k, int* slot0, int* nslots) {
  *slot0 = m->parts[k].slot0;
  *nslots = m->parts[k].nslots;
}
int grad64_nraw(const GradModule64* m) { return m ? m->nraw : 0; }
bool has_loss_routine64(int loss) {
  return loss == SRHIP_LOSS_L2 || (loss >= 0 && loss < SRHIP_NUM_LOSSES && kLoss64[loss] >= 0);
}
bool has_dloss_routine64(int loss) {
  return loss == SRHIP_LOSS_L2 ||
         (loss >= 0 && loss < SRHIP_NUM_LOSSES && kLoss64[loss] >= 0 && kDLoss64[loss] >= 0);
}

hipError_t launch_grad_code64(GradModule64* m, int part, const EvalPlan& plan, const EvalArgs<double>& a,
                              const double* consts, double* gpart, int nconst, hipStream_t stream) {
  const GradPart64& q = m->parts[part];
  if (a.nlist != q.nslots || m->nraw > a.nfeat || plan.tile != TILE2 || plan.threads != 256) return hipErrorInvalidValue;
  Jit64GradArgs ja;
  ja.e = a;
  ja.code_off = q.d_off;
  ja.consts = consts;
  ja.cbase = q.d_cbase;
  ja.gpart = gpart;
  ja.nconst = nconst;
  ja.nraw = m->nraw;
  size_t sz = sizeof(ja);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ja, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const size_t narr = 1 + (size_t)m->nraw + (a.w ? 1 : 0);
  const size_t lds = narr * (size_t)plan.ntiles * (size_t)TILE2 * sizeof(double) + 16;
  // the hand-written tree loop (its counter in the last 16 bytes); SRHIP_JIT_DYNLOOP=0: the compiled one
  const char* dl = std::getenv("SRHIP_JIT_DYNLOOP");
  const bool stl = dl && dl[0] == '0';
  hipFunction_t fn = stl ? (a.w ? q.fn_w : q.fn) : (a.w ? q.fn_dlw : q.fn_dl);
  note_kernel(stl ? (a.w ? "sr_jit64_grad_w" : "sr_jit64_grad") : (a.w ? "sr_jit64_grad_dlw" : "sr_jit64_grad_dl"));
  return hipModuleLaunchKernel(fn, (unsigned)a.nrg * (unsigned)a.ntg, 1, 1, 256, 1, 1, (unsigned)lds, stream, nullptr,
                               cfg);
}

bool compile_grad_only64(const CompiledBatch<double>& cb, const std::vector<int32_t>& const_off,
                         const std::vector<int32_t>& cand, std::vector<uint8_t>* bytes, std::string* text,
                         std::vector<int32_t>* offsets, int loss, uint64_t lparam) {
  const Tmpl64& T = tmpl64();
  if (!T.ok) throw Error(SRHIP_ERR_UNSUPPORTED, std::string("Float64 jit template unavailable: ") + T.why);
  std::vector<uint32_t> words;
  std::vector<std::string> lines;
  std::vector<int32_t> offs, okt, rest;
  int mf = -1;
  grad_codegen64(cb, const_off, cand, 0, text != nullptr, words, text ? &lines : nullptr, offs, okt, rest, &mf, nullptr,
                 loss, lparam);
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


struct Part64 {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr, fn_w = nullptr;
  hipFunction_t fn_dl = nullptr, fn_dlw = nullptr;  // the hand-written tree loop (sr_jit64_eval_dl)
  hipFunction_t fn_out = nullptr;                   // per-row output code (sr_jit64_out)
  int32_t* d_off = nullptr;
  int slot0 = 0, nslots = 0;
};
struct Module64 {
  std::vector<Part64> parts;
  int nslots = 0;
  int nraw = 0;
  bool out = false;
};

bool available64() { return tmpl64().ok; }

Module64* build64(const CompiledBatch<double>& cb, const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list,
                  std::vector<int32_t>& rest, Stats* st, const Opts64& opt) {
  const Tmpl64& T = tmpl64();
  if (!T.ok) { rest = cand; return nullptr; }
  const auto t0 = std::chrono::steady_clock::now();
  struct Chunk { std::vector<uint32_t> words; std::vector<int32_t> offs, slots; };
  std::vector<Chunk> chunks;
  int max_feat = -1;
  size_t pos = 0, bytes = 0;
  constexpr int kMaxParts64 = 8;
  while (pos < cand.size()) {
    Chunk ch;
    const size_t next = codegen64(cb, cand, pos, opt, false, ch.words, nullptr, ch.offs, ch.slots, rest, &max_feat, st);
    if (next == pos) { rest.push_back(cand[pos]); if (st) st->nrejected++; pos = next + 1; continue; }
    if ((int)chunks.size() + 1 == kMaxParts64 && next < cand.size()) {
      for (size_t k = next; k < cand.size(); ++k) rest.push_back(cand[k]);
      if (st) st->nrejected += (int)(cand.size() - next);
      pos = cand.size();
    } else {
      pos = next;
    }
    if (ch.slots.empty()) continue;
    bytes += ch.words.size() * 4;
    chunks.push_back(std::move(ch));
  }
  if (chunks.empty()) return nullptr;
  const auto t1 = std::chrono::steady_clock::now();
  Module64* m = new Module64();
  m->nraw = max_feat + 1;
  m->out = opt.out;
  try {
    for (Chunk& ch : chunks) {
      Part64 pt;
      pt.slot0 = m->nslots;
      pt.nslots = (int)ch.slots.size();
      m->parts.push_back(pt);
      Part64& q = m->parts.back();
      std::vector<uint8_t> img(T.img, T.img + T.size);
      std::memcpy(img.data() + T.area_off, ch.words.data(), ch.words.size() * 4);
      HIP_CHECK(hipModuleLoadData(&q.mod, img.data()));
      HIP_CHECK(hipModuleGetFunction(&q.fn, q.mod, "sr_jit64_eval"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_w, q.mod, "sr_jit64_eval_w"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_dl, q.mod, "sr_jit64_eval_dl"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_dlw, q.mod, "sr_jit64_eval_dlw"));
      HIP_CHECK(hipModuleGetFunction(&q.fn_out, q.mod, "sr_jit64_out"));
      for (hipFunction_t f : {q.fn, q.fn_w, q.fn_dl, q.fn_dlw, q.fn_out})
        HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
      HIP_CHECK(hipMalloc((void**)&q.d_off, ch.offs.size() * sizeof(int32_t)));
      HIP_CHECK(hipMemcpy(q.d_off, ch.offs.data(), ch.offs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      m->nslots += pt.nslots;
      jit_list.insert(jit_list.end(), ch.slots.begin(), ch.slots.end());
    }
  } catch (...) {
    destroy64(m);
    throw;
  }
  if (st) {
    st->ms_codegen = std::chrono::duration<double, std::milli>(t1 - t0).count();
    st->ms_load = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    st->code_bytes = bytes;
    st->nparts = (int)chunks.size();
  }
  return m;
}

void destroy64(Module64* m) {
  if (!m) return;
  for (Part64& q : m->parts) {
    if (q.d_off) (void)hipFree(q.d_off);
    if (q.mod) (void)hipModuleUnload(q.mod);
  }
  delete m;
}

int nparts64(const Module64* m) { return m ? (int)m->parts.size() : 0; }
void part64(const Module64* m, int k, int* slot0, int* nslots) {
  *slot0 = m->parts[k].slot0;
  *nslots = m->parts[k].nslots;
}
int nraw64(const Module64* m) { return m ? m->nraw : 0; }

hipError_t launch64(Module64* m, int k, const EvalPlan& plan, const EvalArgs<double>& a, hipStream_t stream) {
  const Part64& q = m->parts[k];
  if (a.nlist != q.nslots || m->nraw > a.nfeat || plan.tile != TILE2 || plan.threads != 256) return hipErrorInvalidValue;
  if (m->out && (a.w != nullptr || a.out == nullptr || a.out_stride < a.n_pad)) return hipErrorInvalidValue;
  Jit64Args ja;
  ja.e = a;
  ja.code_off = q.d_off;
  ja.nraw = m->nraw;
  size_t sz = sizeof(ja);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ja, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const size_t narr = 1 + (size_t)m->nraw + (a.w ? 1 : 0);
  const size_t lds = narr * (size_t)plan.ntiles * (size_t)TILE2 * sizeof(double) + 16;
  // the hand-written tree loop (its counter in the last 16 bytes); SRHIP_JIT_DYNLOOP=0: the compiled one
  const char* dl = std::getenv("SRHIP_JIT_DYNLOOP");
  const bool st = dl && dl[0] == '0';
  hipFunction_t fn = st ? (a.w ? q.fn_w : q.fn) : (a.w ? q.fn_dlw : q.fn_dl);
  note_kernel(st ? (a.w ? "sr_jit64_eval_w" : "sr_jit64_eval") : (a.w ? "sr_jit64_eval_dlw" : "sr_jit64_eval_dl"));
  if (m->out) {  // per-row outputs: the compiled loop, every tree on every tile
    fn = q.fn_out;
    note_kernel("sr_jit64_out");
  }
  return hipModuleLaunchKernel(fn, (unsigned)a.nrg * (unsigned)a.ntg, 1, 1, 256, 1, 1, (unsigned)lds, stream, nullptr,
                               cfg);
}

bool compile_only64(const CompiledBatch<double>& cb, const std::vector<int32_t>& cand, std::vector<uint8_t>* bytes,
                    std::string* text, std::vector<int32_t>* offsets, const Opts64& opt) {
  const Tmpl64& T = tmpl64();
  if (!T.ok) throw Error(SRHIP_ERR_UNSUPPORTED, std::string("Float64 jit template unavailable: ") + T.why);
  std::vector<uint32_t> words;
  std::vector<std::string> lines;
  std::vector<int32_t> offs, okt, rest;
  int mf = -1;
  codegen64(cb, cand, 0, opt, text != nullptr, words, text ? &lines : nullptr, offs, okt, rest, &mf, nullptr);
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

}  // namespace jit
}  // namespace srhip
