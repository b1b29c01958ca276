// compile.h — host compiler from postfix node streams (include/srhip.h) to
// the device accumulator-machine programs of srhip_internal.h.
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

#include "srhip_internal.h"

namespace srhip {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// a folded feature-free subtree (CompiledBatch::folds)
// operand stack of eval_fold: a deeper fold is recompiled instead
constexpr int kMaxFoldDepth = 64;

struct FoldRec {
  int32_t node_b, node_e;  // postfix nodes [node_b, node_e) of the batch
  int32_t const_b;         // batch-wide index of its first constant
};

template <typename T>
struct CompiledBatch {
  int ntrees = 0;
  std::vector<Ins<T>> code;          // all programs, each terminated by OP_END
  std::vector<int32_t> tree_off;     // start of each tree's program (-1: not run)
  std::vector<int32_t> nodes;        // count_nodes(tree) (src/Complexity.jl:13-19)
  std::vector<uint8_t> static_fail;  // fails for every row count (constant checks)
  std::vector<uint8_t> fail_if_rows; // root is a non-finite constant: fails iff n > 0
  std::vector<int32_t> need;         // stack slots used
  std::vector<int32_t> len;          // program length in instructions (END included)
  std::vector<int32_t> cost;         // VALU cost estimate per row
  int max_feature = -1;              // largest feature index referenced
  int64_t total_nodes = 0;
  // constant map (srhip_program_set_constants without a recompile): per
  // instruction, what its immediate holds: >= 0 the batch-wide index of a
  // constant, <= -2 the folded value of folds[-2 - m], -1 nothing; per tree,
  // 1 when its program has code and every constant-derived immediate is in
  // the map, so new finite constants only rewrite those immediates
  using Fold = FoldRec;
  std::vector<int32_t> cmap;
  std::vector<uint8_t> direct;
  std::vector<Fold> folds;
};

// The value of a folded subtree for the constants `consts` (batch-wide, as in
// trees): `_eval_constant_tree`'s arithmetic, false when an operator output is
// not finite (the tree then fails statically and needs a recompile).
template <typename T>
bool eval_fold(const FoldRec& f, const srhip_trees& trees, T* out);

// Compile every tree of the batch. Throws srhip::Error on malformed input
// (SRHIP_ERR_INVALID) or on operators outside the table (SRHIP_ERR_UNSUPPORTED).
// grad = true compiles for the constant-gradient kernels: no constant folding,
// every constant operand carries its get_constants index in the slot field,
// and a non-finite constant anywhere fails the tree statically.
// keep_layout = true (programs whose constants change in place): a tree that
// fails statically is compiled anyway (static_fail / fail_if_rows still set),
// so its code keeps its place when later constants make it finite again.
template <typename T>
CompiledBatch<T> compile_batch(const srhip_trees& trees, bool grad = false, bool keep_layout = false);

// compile_batch over contiguous slices of the batch on several host threads
// (large batches: srhip_program_set_constants recompiles every call); the
// result is identical to compile_batch's.
template <typename T>
CompiledBatch<T> compile_batch_par(const srhip_trees& trees, bool grad = false, bool keep_layout = false);

}  // namespace srhip
