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
};

// Compile every tree of the batch. Throws srhip::Error on malformed input
// (SRHIP_ERR_INVALID) or on operators outside the table (SRHIP_ERR_UNSUPPORTED).
// grad = true compiles for the constant-gradient kernels: no constant folding,
// every constant operand carries its get_constants index in the slot field,
// and a non-finite constant anywhere fails the tree statically.
template <typename T>
CompiledBatch<T> compile_batch(const srhip_trees& trees, bool grad = false);

// compile_batch over contiguous slices of the batch on several host threads
// (large batches: srhip_program_set_constants recompiles every call); the
// result is identical to compile_batch's.
template <typename T>
CompiledBatch<T> compile_batch_par(const srhip_trees& trees, bool grad = false);

}  // namespace srhip
