// srhip_internal.h — device program encoding shared by the host compiler
// (compile.cpp) and the HIP kernels (kernels.hip).
//
// A tree is compiled to an accumulator-machine program. Every instruction is
// wave-uniform: it is fetched with scalar loads and dispatched with a
// uniform branch, so the 64 lanes of a wave never diverge on the program.
// Each instruction operates on R rows per lane at once.
//
// Register model (all per lane, R rows each):
//   acc          the value being computed
//   tmp          the second operand popped from the stack
//   slot[0..D)   spilled partial results (Sethi–Ullman order keeps D small)
// Leaf operands are read directly: X[f] from the LDS row tile, constants
// from the instruction's immediate (an SGPR operand of the VALU op).
#pragma once
#include <stdint.h>

#include "../../include/srhip.h"

namespace srhip {

// ---- opcode layout ---------------------------------------------------------
constexpr int kMaxSlots = 16;
enum : int {
  OP_END = 0,
  OP_LDX = 1,                          // acc = X[f]
  OP_LDC = 2,                          // acc = imm
  OP_PUSH0 = 3,                        // slot[k] = acc
  OP_POP0 = OP_PUSH0 + kMaxSlots,      // tmp = slot[k]
  OP_UN0 = OP_POP0 + kMaxSlots,        // acc = u(acc)
  OP_BIN0 = OP_UN0 + SRHIP_NUM_UOPS,   // acc = b(lhs, rhs), see BinVariant
};

// Operand sources of a binary instruction (lhs, rhs):
enum BinVariant : int {
  V_AX = 0,  // (acc, X[f])
  V_XA,      // (X[f], acc)
  V_AC,      // (acc, imm)
  V_CA,      // (imm, acc)
  V_AT,      // (acc, tmp)
  V_TA,      // (tmp, acc)
  V_XX,      // (X[f], X[g]),  g = integer in imm
  V_XC,      // (X[f], imm)
  V_CX,      // (imm, X[f])
  NUM_VARIANTS
};
constexpr int kNumOpcodes = OP_BIN0 + NUM_VARIANTS * SRHIP_NUM_BOPS;
static_assert(kNumOpcodes <= 256, "opcode must fit in 8 bits");

constexpr int bin_opcode(int variant, int bop) {
  return OP_BIN0 + variant * SRHIP_NUM_BOPS + bop;
}

// code word: [7:0] opcode, [15:8] slot index, [31:16] feature index.
// Evaluation programs set bit 15 (kNeedX) on instructions with an X[f]
// operand (LDX and the AX/XA/XX/XC/CX variants): the kernel reads X[f] from
// LDS ahead of the dispatch. Gradient programs use all 8 slot bits for
// constant indices and never set it.
constexpr uint32_t kNeedX = 1u << 15;
constexpr uint32_t make_code(int opc, int slot, int feat) {
  return (uint32_t)opc | ((uint32_t)slot << 8) | ((uint32_t)feat << 16);
}
constexpr bool variant_needs_x(int v) {
  return v == V_AX || v == V_XA || v == V_XX || v == V_XC || v == V_CX;
}
// Longest program (END included) of the VGPR-resident-program kernel
// variant: one instruction per lane, and the dispatch reads one ahead.
constexpr int kVProgMax = 63;

template <typename T>
struct Ins;
template <>
struct alignas(8) Ins<float> {
  uint32_t code;
  float imm;
};
template <>
struct alignas(16) Ins<double> {
  uint32_t code;
  uint32_t pad;
  double imm;
};

// ---- operator properties ------------------------------------------------------
// "lossy" operators can map a non-finite operand to a finite result
// (exp(-Inf) = 0, x/Inf = 0, greater(NaN, 1) = 0, ...). DynamicExpressions
// fails a tree when ANY node value is non-finite at any row (every child
// array is checked, InterfaceDynamicExpressions.jl:43-48). All other
// operators propagate non-finite values, so it is enough to check the
// computed operands of lossy operators plus the root value.
constexpr bool bop_lossy_lhs(int op) {
  return op == SRHIP_BOP_POW || op == SRHIP_BOP_GREATER ||
         op == SRHIP_BOP_LOGICAL_OR || op == SRHIP_BOP_LOGICAL_AND ||
         op == SRHIP_BOP_MAX || op == SRHIP_BOP_MIN;
}
constexpr bool bop_lossy_rhs(int op) {
  return op == SRHIP_BOP_DIV || op == SRHIP_BOP_POW || op == SRHIP_BOP_GREATER ||
         op == SRHIP_BOP_LOGICAL_OR || op == SRHIP_BOP_LOGICAL_AND ||
         op == SRHIP_BOP_MOD || op == SRHIP_BOP_MAX || op == SRHIP_BOP_MIN;
}
constexpr bool uop_lossy(int op) {
  return op == SRHIP_UOP_EXP || op == SRHIP_UOP_TANH || op == SRHIP_UOP_ATAN ||
         op == SRHIP_UOP_ERF || op == SRHIP_UOP_ERFC || op == SRHIP_UOP_SIGN ||
         op == SRHIP_UOP_INV;
}

// ---- operator sets -------------------------------------------------------------
// A kernel variant compiled only with the dispatch cases of a small operator
// set has a shallower dispatch branch tree. The host picks the smallest set
// that contains every operator of the batch.
enum OpSet : int { OPSET_BASIC = 0, OPSET_FULL = 1 };
constexpr uint32_t kBasicBops = (1u << SRHIP_BOP_ADD) | (1u << SRHIP_BOP_SUB) | (1u << SRHIP_BOP_MUL) |
                                (1u << SRHIP_BOP_DIV);
constexpr uint32_t kBasicUops = (1u << SRHIP_UOP_NEG) | (1u << SRHIP_UOP_SQUARE) | (1u << SRHIP_UOP_CUBE) |
                                (1u << SRHIP_UOP_EXP) | (1u << SRHIP_UOP_ABS) | (1u << SRHIP_UOP_LOG) |
                                (1u << SRHIP_UOP_SQRT) | (1u << SRHIP_UOP_SIN) | (1u << SRHIP_UOP_COS);
constexpr bool opset_has_bop(int set, int op) { return set == OPSET_FULL || ((kBasicBops >> op) & 1u); }
constexpr bool opset_has_uop(int set, int op) { return set == OPSET_FULL || ((kBasicUops >> op) & 1u); }

// Stack slots of the ordinary kernel variant; trees needing more (rare:
// < 0.01 % of random trees at maxsize 30) run in the 16-slot variant.
constexpr int kShallowSlots = 2;

// Rough VALU cost per row of each operator (f32), used to balance trees over
// workgroups. Not a correctness input.
constexpr int bop_cost(int op) {
  return op == SRHIP_BOP_DIV ? 12 : op == SRHIP_BOP_POW ? 60 : op == SRHIP_BOP_MOD ? 30 : 2;
}
constexpr int uop_cost(int op) {
  return (op == SRHIP_UOP_NEG || op == SRHIP_UOP_ABS || op == SRHIP_UOP_SQUARE ||
          op == SRHIP_UOP_CUBE || op == SRHIP_UOP_RELU || op == SRHIP_UOP_ROUND ||
          op == SRHIP_UOP_FLOOR || op == SRHIP_UOP_CEIL || op == SRHIP_UOP_SIGN)
             ? 2
             : (op == SRHIP_UOP_EXP || op == SRHIP_UOP_SQRT || op == SRHIP_UOP_INV) ? 14 : 40;
}

// The name of the main (evaluation) kernel the calling thread launched last:
// set at each launch site, read by srhip_last_kernel_name (bench.py ties a
// rocprofv3 PMC summary to the kernel that ran).
void note_kernel(const char* name);
const char* last_kernel();

}  // namespace srhip
