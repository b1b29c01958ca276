// jit_asm.h — shared pieces of the tree compilers (jit.cpp: loss tree code,
// jit_grad.cpp: reverse-mode gradient tree code): the register layout of the
// generated routines, the code-object template and its parser, and the gfx950
// instruction encoder with its assembly-text mirror.
#pragma once
#include <elf.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gen/jit_layout_r4.h"
#include "srhip_internal.h"

// code-object templates (jit_blob.S): 1 MiB and 8 MiB code areas
extern "C" const unsigned char srhip_jit_tmpl_s[];
extern "C" const unsigned char srhip_jit_tmpl_s_end[];
extern "C" const unsigned char srhip_jit_tmpl_l[];
extern "C" const unsigned char srhip_jit_tmpl_l_end[];

namespace srhip {
namespace jit {
namespace detail {

constexpr int R = SR_JIT_R;
static_assert(R == 4, "tree code is laid out for 4 rows per lane");
constexpr int VA = SR_JIT_V_A, VB = SR_JIT_V_B, VCHK = SR_JIT_V_CHK, VLANE = SR_JIT_V_LANE;
constexpr int VLSUM = SR_JIT_V_LSUM, VLANE4 = SR_JIT_V_LANE4, VCHKSAVE = SR_JIT_V_CHKSAVE;
constexpr int VGCAN = SR_JIT_V_GCAN, VGMIN = SR_JIT_V_GMIN, VGEXP = SR_JIT_V_GEXP, VGTRIG = SR_JIT_V_GTRIG;
constexpr int VGT = SR_JIT_V_GT, VY = SR_JIT_V_Y, VPOOL0 = SR_JIT_V_POOL0, NPOOL = SR_JIT_V_NPOOL;
constexpr int S_TILE = SR_JIT_S_TILE, S_NT = SR_JIT_S_NT, S_PARTIAL = SR_JIT_S_PARTIAL;
constexpr int S_TILEBYTES = SR_JIT_S_TILEBYTES, S_WOFF = SR_JIT_S_WOFF, S_STATUS = SR_JIT_S_STATUS;
constexpr int S_FLAG = SR_JIT_S_FLAG, S_RR = SR_JIT_S_RR, S_TGT = SR_JIT_S_TGT, S_RT = SR_JIT_S_RT;
constexpr int S_FASTOK = SR_JIT_S_FASTOK, S_EPS = SR_JIT_S_EPS;
constexpr int S_KH = SR_JIT_S_KH;  // high word of a loss routine's Float64 parameter
constexpr int S_K = SR_JIT_S_K, S_PE = SR_JIT_S_PE, S_MODE = SR_JIT_S_MODE, S_X0 = SR_JIT_S_X0;
constexpr int S_BASE = SR_JIT_S_X2;
// per-row output tree code (Options::out): s[92:93] = this tree's output rows
// of the current tile (set by the driver, advanced a tile per tile); above
// every register of tree-code state and of the routines
constexpr int S_OUT = 92;
constexpr int S_RECIP = SR_JIT_S_X1;  // RN(1/c) of a constant divisor (routine b_div_rk)  // s[86:87]: base of the routine region in use (FAST or PRECISE)
// a routine temporary, free between calls: the constant operand of a packed
// tree-code instruction (low half of s[20:21]; VOP3P takes no literal)
constexpr int S_PKC = 20;
constexpr int TILE = 64 * R;
constexpr int kNumRoutines = SR_JIT_NUM_ROUTINES;
const int kUopRoutine[SRHIP_NUM_UOPS] = SR_JIT_UOP_ROUTINE;
const int kBopRoutine[SRHIP_NUM_BOPS] = SR_JIT_BOP_ROUTINE;
const int kBopRoutineRC[SRHIP_NUM_BOPS] = SR_JIT_BOP_ROUTINE_RC;  // rhs constant in s_k
const int kBopRoutineLC[SRHIP_NUM_BOPS] = SR_JIT_BOP_ROUTINE_LC;  // lhs constant in s_k
const int kLossRoutine[SRHIP_NUM_LOSSES] = SR_JIT_LOSS_ROUTINE;     // -1: L2 (inline)
const int kDLossRoutine[SRHIP_NUM_LOSSES] = SR_JIT_DLOSS_ROUTINE;   // dℓ/dr; -1: L2 (inline)
const int kGradLossRoutine[SRHIP_NUM_LOSSES] = SR_JIT_GRAD_LOSS_ROUTINE;  // ℓ in the gradient code
const char* const kRoutineName[kNumRoutines] = SR_JIT_ROUTINE_NAMES;
const int kRoutineTrig[kNumRoutines] = SR_JIT_ROUTINE_TRIG;
const int kRoutineInline[kNumRoutines] = SR_JIT_ROUTINE_INLINE;        // same FAST / PRECISE code, small
const int kRoutineBodyBytes[kNumRoutines] = SR_JIT_ROUTINE_BODY_BYTES;  // up to the return

// ---- the code-object template ---------------------------------------------------
struct Tmpl {
  const uint8_t* img = nullptr;
  size_t size = 0;
  size_t area_off = 0;     // file offset of sr_jit_code
  size_t area_bytes = 0;   // usable bytes of the area
  uint64_t area_va = 0;    // its address in the image
  uint64_t rt_va[kNumRoutines] = {};  // FAST routine addresses
  uint64_t delta = 0;      // PRECISE - FAST region offset
  uint64_t fast0 = 0;      // FAST region start (sr_rt_fast)
  std::vector<uint32_t> body[kNumRoutines];  // inlinable routine bodies (without the return)
  bool ok = false;
  std::string why;
};

inline bool parse_tmpl(const uint8_t* img, size_t size, Tmpl* t) {
  t->img = img;
  t->size = size;
  if (size < sizeof(Elf64_Ehdr)) { t->why = "template too small"; return false; }
  Elf64_Ehdr eh;
  std::memcpy(&eh, img, sizeof(eh));
  if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_ident[EI_CLASS] != ELFCLASS64 ||
      eh.e_shoff + (size_t)eh.e_shnum * sizeof(Elf64_Shdr) > size) {
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
  const size_t nsym = symtab->sh_size / sizeof(Elf64_Sym);
  uint64_t code_va = 0, area_fn_va = 0, area_fn_size = 0, fast0 = 0, prec0 = 0;
  uint64_t prec_va[kNumRoutines] = {};
  int found = 0;
  for (size_t i = 0; i < nsym; ++i) {
    Elf64_Sym sym;
    std::memcpy(&sym, img + symtab->sh_offset + i * sizeof(Elf64_Sym), sizeof(sym));
    if (sym.st_name >= strtab.sh_size) continue;
    const char* nm = reinterpret_cast<const char*>(img + strtab.sh_offset + sym.st_name);
    const std::string n(nm);
    if (n == "sr_jit_code") { code_va = sym.st_value; found |= 1; }
    else if (n == "sr_jit_area") { area_fn_va = sym.st_value; area_fn_size = sym.st_size; found |= 2; }
    else if (n == "sr_rt_fast") { fast0 = sym.st_value; found |= 4; }
    else if (n == "sr_rt_prec") { prec0 = sym.st_value; found |= 8; }
    else if (n.rfind("sr_rt_fast_", 0) == 0 || n.rfind("sr_rt_prec_", 0) == 0) {
      const std::string rn = n.substr(11);
      for (int k = 0; k < kNumRoutines; ++k)
        if (rn == kRoutineName[k]) (n[6] == 'f' ? t->rt_va : prec_va)[k] = sym.st_value;
    }
  }
  if (found != 15) { t->why = "template symbols missing"; return false; }
  for (int k = 0; k < kNumRoutines; ++k) {
    if (!t->rt_va[k] || !prec_va[k]) { t->why = std::string("routine missing: ") + kRoutineName[k]; return false; }
    if (prec_va[k] - t->rt_va[k] != prec0 - fast0) { t->why = "FAST / PRECISE routine layouts differ"; return false; }
  }
  t->delta = prec0 - fast0;
  t->fast0 = fast0;
  const Elf64_Shdr* text = nullptr;
  for (auto& s : sh)
    if (s.sh_type == SHT_PROGBITS && (s.sh_flags & SHF_EXECINSTR) && code_va >= s.sh_addr &&
        code_va < s.sh_addr + s.sh_size)
      text = &s;
  if (!text) { t->why = "code area outside .text"; return false; }
  t->area_va = code_va;
  for (int k = 0; k < kNumRoutines; ++k) {
    if (!kRoutineInline[k]) continue;
    const uint64_t va = t->rt_va[k];
    const size_t nb = (size_t)kRoutineBodyBytes[k];
    if (va < text->sh_addr || va + nb + 4 > text->sh_addr + text->sh_size || nb % 4) continue;
    const size_t off = (size_t)(va - text->sh_addr + text->sh_offset);
    uint32_t ret;
    std::memcpy(&ret, img + off + nb, 4);
    if (ret != (0xbe801d00u | (uint32_t)S_RR)) { t->why = "routine body does not end in its return"; return false; }
    t->body[k].resize(nb / 4);
    std::memcpy(t->body[k].data(), img + off, nb);
  }
  t->area_off = (size_t)(code_va - text->sh_addr + text->sh_offset);
  // the area function: s_endpgm, the area, the compiler's closing s_endpgm
  const uint64_t end = area_fn_va + area_fn_size;
  if (end <= code_va + 64 || end > text->sh_addr + text->sh_size) { t->why = "bad area size"; return false; }
  t->area_bytes = (size_t)(end - code_va) - 64;
  if (t->area_off + t->area_bytes > size) { t->why = "area beyond the image"; return false; }
  t->ok = true;
  return true;
}

struct Templates {
  Tmpl small, large;
  bool ok = false;
  std::string why;
};

inline const Templates& templates() {
  static Templates T;
  static std::once_flag once;
  std::call_once(once, [] {
    const bool a = parse_tmpl(srhip_jit_tmpl_s, (size_t)(srhip_jit_tmpl_s_end - srhip_jit_tmpl_s), &T.small);
    const bool b = parse_tmpl(srhip_jit_tmpl_l, (size_t)(srhip_jit_tmpl_l_end - srhip_jit_tmpl_l), &T.large);
    T.ok = a && b && T.small.delta == T.large.delta;
    T.why = !a ? T.small.why : !b ? T.large.why : (T.ok ? "" : "templates disagree");
  });
  return T;
}

// ---- instruction encoder (gfx950 formats), with an assembly-text mirror ---------
inline std::string hex32(uint32_t v);

struct Src {
  int enc = 0;        // 9-bit operand field
  bool lit = false;   // a 32-bit literal follows
  uint32_t val = 0;   // constant bits (literal or inline constant)
  // assembly text of the operand (only built when text is wanted)
  std::string name() const {
    if (enc >= 256) return "v" + std::to_string(enc - 256);
    if (enc < 102) return "s" + std::to_string(enc);
    return hex32(val);
  }
};

inline bool inline_const(uint32_t b, int* enc) {
  const int32_t i = (int32_t)b;
  if (i >= 0 && i <= 64) { *enc = 128 + i; return true; }
  if (i >= -16 && i <= -1) { *enc = 192 - i; return true; }
  switch (b) {
    case 0x3f000000u: *enc = 240; return true;  // 0.5
    case 0xbf000000u: *enc = 241; return true;
    case 0x3f800000u: *enc = 242; return true;  // 1.0
    case 0xbf800000u: *enc = 243; return true;
    case 0x40000000u: *enc = 244; return true;  // 2.0
    case 0xc0000000u: *enc = 245; return true;
    case 0x40800000u: *enc = 246; return true;  // 4.0
    case 0xc0800000u: *enc = 247; return true;
    case 0x3e22f983u: *enc = 248; return true;  // 1/(2 pi)
    default: return false;
  }
}

inline std::string hex32(uint32_t v) {
  char b[16];
  std::snprintf(b, sizeof b, "0x%x", v);
  return b;
}

inline Src V(int r) { return Src{256 + r, false, 0}; }
inline Src S(int r) { return Src{r, false, 0}; }
inline Src K(uint32_t bits) {
  Src s;
  int e;
  s.val = bits;
  if (inline_const(bits, &e)) {
    s.enc = e;
  } else {
    s.enc = 255;
    s.lit = true;
  }
  return s;
}

struct Asm {
  std::vector<uint32_t> w;
  bool want_text = false;
  std::vector<std::string> lines;
  std::vector<int> lab;  // word index of each label (-1: unbound)
  struct Fix { size_t word; int label; size_t line; };
  std::vector<Fix> fix;

  size_t bytes() const { return w.size() * 4; }
  void put(uint32_t x) { w.push_back(x); }
  void t(const std::string& s) {
    if (want_text) lines.push_back(s);
  }
  int label() { lab.push_back(-1); return (int)lab.size() - 1; }
  void bind(int l) { lab[l] = (int)w.size(); }

  // SOP1/SOP2/SOPC/VOP1/VOP2/VOPC with an optional literal
  void lit(const Src& a) {
    if (a.lit) put(a.val);
  }
  void sop1(int op, const char* nm, int sdst, const Src& s0, const std::string& dname) {
    put(0xbe800000u | ((uint32_t)sdst << 16) | ((uint32_t)op << 8) | (uint32_t)s0.enc);
    lit(s0);
    if (want_text) t(std::string(nm) + " " + dname + ", " + s0.name());
  }
  void sop2(int op, const char* nm, int sdst, const Src& s0, const Src& s1) {
    put(0x80000000u | ((uint32_t)op << 23) | ((uint32_t)sdst << 16) | ((uint32_t)s1.enc << 8) | (uint32_t)s0.enc);
    lit(s0.lit ? s0 : s1);
    if (want_text) t(std::string(nm) + " s" + std::to_string(sdst) + ", " + s0.name() + ", " + s1.name());
  }
  void sopc(int op, const char* nm, const Src& s0, const Src& s1, const std::string& n0 = "") {
    put(0xbf000000u | ((uint32_t)op << 16) | ((uint32_t)s1.enc << 8) | (uint32_t)s0.enc);
    lit(s0.lit ? s0 : s1);
    if (want_text) t(std::string(nm) + " " + (n0.empty() ? s0.name() : n0) + ", " + s1.name());
  }
  void sopp(int op, const char* nm, int imm, bool show = true) {
    put(0xbf800000u | ((uint32_t)op << 16) | ((uint32_t)imm & 0xffffu));
    if (want_text) t(show ? std::string(nm) + " " + std::to_string(imm) : std::string(nm));
  }
  void raw(uint32_t x) {
    put(x);
    if (want_text) t(".long " + hex32(x));
  }
  void branch(int op, const char* nm, int l) {
    fix.push_back({w.size(), l, want_text ? lines.size() : 0});
    put(0xbf800000u | ((uint32_t)op << 16));
    if (want_text) t(std::string(nm) + " @");
  }
  void vop1(int op, const char* nm, int vdst, const Src& s0) {
    put(0x7e000000u | ((uint32_t)vdst << 17) | ((uint32_t)op << 9) | (uint32_t)s0.enc);
    lit(s0);
    if (want_text) t(std::string(nm) + " v" + std::to_string(vdst) + ", " + s0.name());
  }
  void vop2(int op, const char* nm, int vdst, const Src& s0, int vsrc1, const char* tail = "") {
    put(((uint32_t)op << 25) | ((uint32_t)vdst << 17) | ((uint32_t)vsrc1 << 9) | (uint32_t)s0.enc);
    lit(s0);
    if (want_text) t(std::string(nm) + " v" + std::to_string(vdst) + ", " + s0.name() + ", v" + std::to_string(vsrc1) + tail);
  }
  void vopc(int op, const char* nm, const Src& s0, int vsrc1) {
    put(0x7c000000u | ((uint32_t)op << 17) | ((uint32_t)vsrc1 << 9) | (uint32_t)s0.enc);
    lit(s0);
    if (want_text) t(std::string(nm) + " vcc, " + s0.name() + ", v" + std::to_string(vsrc1));
  }
  // VOP3 (no literals on gfx9): abs / neg bit i applies to source i
  void vop3(int op, const char* nm, int vdst, const Src& s0, const Src& s1, const Src* s2, int abs, int neg) {
    if (s0.lit || s1.lit || (s2 && s2->lit)) throw Error(SRHIP_ERR_INVALID, "jit: literal in a VOP3 operand");
    put(0xd0000000u | ((uint32_t)op << 16) | ((uint32_t)(abs & 7) << 8) | (uint32_t)vdst);
    put(((uint32_t)(neg & 7) << 29) | ((uint32_t)(s2 ? s2->enc : 0) << 18) | ((uint32_t)s1.enc << 9) |
        (uint32_t)s0.enc);
    if (!want_text) return;
    auto f = [&](const Src& s, int i) {
      std::string n = s.name();
      if (abs & (1 << i)) n = "|" + n + "|";
      if (neg & (1 << i)) n = "-" + n;
      return n;
    };
    t(std::string(nm) + " v" + std::to_string(vdst) + ", " + f(s0, 0) + ", " + f(s1, 1) + (s2 ? ", " + f(*s2, 2) : ""));
  }
  // VOP3P (two f32 per lane in a register pair; no literals on gfx9): bit i of
  // opsel / opsel_hi / neg_lo / neg_hi applies to source i. A constant source
  // (an inline constant, or an SGPR pair whose low half holds it) feeds both
  // halves with opsel_hi bit 0.
  void vop3p(int op, const char* nm, int vdst, const Src& s0, const Src& s1, const Src* s2, int opsel, int opsel_hi,
             int neg_lo, int neg_hi) {
    if (s0.lit || s1.lit || (s2 && s2->lit)) throw Error(SRHIP_ERR_INVALID, "jit: literal in a VOP3P operand");
    put(0xd3800000u | ((uint32_t)op << 16) | ((uint32_t)((opsel_hi >> 2) & 1) << 14) | ((uint32_t)(opsel & 7) << 11) |
        ((uint32_t)(neg_hi & 7) << 8) | (uint32_t)vdst);
    put(((uint32_t)(neg_lo & 7) << 29) | ((uint32_t)(opsel_hi & 3) << 27) | ((uint32_t)(s2 ? s2->enc : 0) << 18) |
        ((uint32_t)s1.enc << 9) | (uint32_t)s0.enc);
    if (!want_text) return;
    const int n = s2 ? 3 : 2;
    auto pair = [](const Src& s) -> std::string {
      if (s.enc >= 256) return "v[" + std::to_string(s.enc - 256) + ":" + std::to_string(s.enc - 255) + "]";
      if (s.enc < 102) return "s[" + std::to_string(s.enc) + ":" + std::to_string(s.enc + 1) + "]";
      switch (s.val) {  // inline constants by value (llvm-mc reads hex as a literal here)
        case 0x3f000000u: return "0.5";
        case 0xbf000000u: return "-0.5";
        case 0x3f800000u: return "1.0";
        case 0xbf800000u: return "-1.0";
        case 0x40000000u: return "2.0";
        case 0xc0000000u: return "-2.0";
        case 0x40800000u: return "4.0";
        case 0xc0800000u: return "-4.0";
        default: return std::to_string((int32_t)s.val);
      }
    };
    auto arr = [&](const char* key, int bits, int dflt) -> std::string {
      if (bits == dflt) return "";
      std::string r = std::string(" ") + key + ":[";
      for (int i = 0; i < n; ++i) r += std::string(i ? "," : "") + ((bits >> i) & 1 ? "1" : "0");
      return r + "]";
    };
    const int full = (1 << n) - 1;
    t(std::string(nm) + " v[" + std::to_string(vdst) + ":" + std::to_string(vdst + 1) + "], " + pair(s0) + ", " + pair(s1) +
      (s2 ? ", " + pair(*s2) : "") + arr("op_sel", opsel & full, 0) + arr("op_sel_hi", opsel_hi & full, full) +
      arr("neg_lo", neg_lo & full, 0) + arr("neg_hi", neg_hi & full, 0));
  }
  void ds_read_b128(int vdst, int vaddr, int offset) {
    put(0xd8000000u | (0xffu << 17) | (uint32_t)(offset & 0xffff));
    put(((uint32_t)vdst << 24) | (uint32_t)vaddr);
    if (want_text) t("ds_read_b128 v[" + std::to_string(vdst) + ":" + std::to_string(vdst + 3) + "], v" + std::to_string(vaddr) +
      (offset ? " offset:" + std::to_string(offset) : ""));
  }
  // global_load_dwordx4 v[vdst:vdst+3], v[vaddr], s[saddr:saddr+1] offset:off (13-bit signed)
  void global_load_dwordx4(int vdst, int vaddr, int saddr, int off) {
    put(0xdc5c8000u | ((uint32_t)off & 0x1fffu));
    put((uint32_t)vaddr | ((uint32_t)saddr << 16) | ((uint32_t)vdst << 24));
    if (want_text)
      t("global_load_dwordx4 v[" + std::to_string(vdst) + ":" + std::to_string(vdst + 3) + "], v" + std::to_string(vaddr) +
        ", s[" + std::to_string(saddr) + ":" + std::to_string(saddr + 1) + "]" + (off ? " offset:" + std::to_string(off) : ""));
  }
  void waitcnt_vm(int n) { sopp(0x0c, "s_waitcnt", 0x0f70 | (n & 15), false); if (want_text) lines.back() = "s_waitcnt vmcnt(" + std::to_string(n) + ")"; }
  void waitcnt_lgkm(int n) { sopp(0x0c, "s_waitcnt", 0xc07f | (n << 8), false); if (want_text) lines.back() = "s_waitcnt lgkmcnt(" + std::to_string(n) + ")"; }

  void finish() {
    for (const Fix& f : fix) {
      if (lab[f.label] < 0) throw Error(SRHIP_ERR_INVALID, "jit: unbound label");
      const int d = lab[f.label] - (int)(f.word + 1);
      if (d < -32768 || d > 32767) throw Error(SRHIP_ERR_INVALID, "jit: branch out of range");
      w[f.word] = (w[f.word] & 0xffff0000u) | ((uint32_t)d & 0xffffu);
      if (want_text) {
        std::string& s = lines[f.line];
        s = s.substr(0, s.size() - 1) + std::to_string(d);
      }
    }
    fix.clear();
  }
};

// VALU / SALU opcodes (gfx9 encodings, checked against llvm-mc by tests/test_jit.py)
enum : int {
  VOP2_CNDMASK = 0x00, VOP2_ADD_F32 = 0x01, VOP2_SUB_F32 = 0x02, VOP2_SUBREV_F32 = 0x03, VOP2_MUL_F32 = 0x05,
  VOP2_MIN_F32 = 0x0a, VOP2_MAX_F32 = 0x0b, VOP2_LSHLREV_B32 = 0x12, VOP2_AND_B32 = 0x13, VOP2_XOR_B32 = 0x15,
  VOP2_ADD_U32 = 0x34,
  VOP1_MOV = 0x01,
  VOP3_ADD_F32 = 0x101, VOP3_MIN_F32 = 0x10a, VOP3_MAX_F32 = 0x10b, VOP3_FMA_F32 = 0x1cb,
  VOP3_MIN3_F32 = 0x1d0, VOP3_MAX3_F32 = 0x1d3,
  VOP3P_FMA_F32 = 0x30, VOP3P_MUL_F32 = 0x31, VOP3P_ADD_F32 = 0x32, VOP3P_MOV_B32 = 0x33,
  VOPC_LT_F32 = 0x41, VOPC_LE_F32 = 0x43, VOPC_GT_F32 = 0x44, VOPC_U_F32 = 0x48, VOPC_GT_I32 = 0xc4,
  VOPC_NGE_F32 = 0x49, VOPC_NGT_F32 = 0x4b, VOPC_NLE_F32 = 0x4c,
  SOP1_MOV = 0x00, SOP1_GETPC = 0x1c, SOP1_SETPC = 0x1d, SOP1_SWAPPC = 0x1e,
  SOP2_ADD_U32 = 0x00, SOP2_SUB_U32 = 0x01, SOP2_SUB_I32 = 0x03, SOP2_SUBB_U32 = 0x05, SOP2_ADDC_U32 = 0x04, SOP2_CSELECT = 0x0a,
  SOP2_AND_B32 = 0x0c, SOP2_LSHL_B32 = 0x1c, SOP2_MUL_I32 = 0x24, SOP2_MUL_HI_U32 = 0x2c,
  SOPC_EQ_U32 = 0x06, SOPC_LG_U32 = 0x07, SOPC_GE_U32 = 0x09, SOPC_LT_U32 = 0x0a, SOPC_LG_U64 = 0x13,
  SOPP_BRANCH = 0x02, SOPP_SCC0 = 0x04, SOPP_SCC1 = 0x05, SOPP_VCCNZ = 0x07,
};

}  // namespace detail
}  // namespace jit
}  // namespace srhip
