// jit.h — the tree compiler: every tree of a large Float32 batch becomes
// straight-line gfx950 machine code (jit.cpp), loaded as one code object per
// program and run by the driver kernel of jit_template.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "compile.h"
#include "kernels.h"

namespace srhip {
namespace jit {

struct Module;

// Options of one compilation (the defaults are the product path).
struct Options {
  bool fast = true;       // emit the FAST-routine path + guards in eligible trees
  bool text = false;      // also produce the assembly text (tests: checked against llvm-mc)
  bool derive = true;     // derived columns (below); SRHIP_JIT_DERIVE=0 turns them off
  bool memc = false;      // constants read from the program's immediates (set_constants needs no new code)
  // the elementwise loss of the tile tail (SRHIP_LOSS_*) and its parameter
  // (Float64 bits, literals of the code): L2 inline, the others through the
  // loss routine of the PRECISE region (device_ops.h elem_loss, bit for bit
  // the interpreter's); PERIODIC keeps every tree off the FAST path
  int loss = SRHIP_LOSS_L2;
  uint64_t lparam = 0;     // Float64 bits (LossFunctions' field, never rounded to Float32)
  // per-row output tree code (srhip_eval_tree_array): every tile stores its
  // root values to the tree's output rows instead of ending with a loss; the
  // PRECISE routines only (the interpreter's values, bit for bit), every tile
  // evaluated whatever fails (the interpreter's MODE_OUT writes them too)
  bool out = false;
};

// Derived columns: a routine unary operator applied to a dataset feature,
// u(x_f), that several trees of the batch share is evaluated once per row by
// the driver while it stages the row tiles (the PRECISE routine, the value
// the Float64-evaluating reference gives) and read by tree code like a
// feature, instead of once per tree. LDS columns of a tile: y, the raw
// features 0 .. nraw-1, the derived columns, w.
constexpr int kMaxDerived = 48;
// Shared subtrees (round 6): a constant-free subtree that several trees of the
// batch contain (cos(x4), exp(x1), cos(exp(x2)), x1 / x3, ...) is evaluated
// once per row per call by the derive pass (api.cpp derive_shared: the
// interpreter's per-row outputs of the subtrees as a program of their own; a
// subtree non-finite at some node on some row has its whole column set to
// NaN) into a column of device memory, [ngcol][n_pad], and the tree code reads
// it with a global load at the tile start instead of computing it (tree code
// column gbase() + g).
constexpr int kMaxGlobalCols = 128;
struct Columns {
  int nraw = 0;                  // raw feature columns staged (max feature used + 1)
  int nder = 0;                  // derived columns (column nraw + k)
  uint32_t der[kMaxDerived] = {};  // (operator << 16) | feature
  int waves = 4;                 // waves per workgroup of the loss tree code (choose_waves)
  int ngcol = 0;                 // shared-subtree columns in device memory
  std::vector<std::string> gkey;  // [ngcol] canonical text of each subtree (jit.cpp subtree_keys)
  std::vector<uint8_t> gkind;    // postfix node streams of the subtrees (SRHIP_NODE_*, raw features)
  std::vector<uint16_t> garg;
  std::vector<int32_t> goff;     // [ngcol + 1]
  int gbase() const { return nraw + nder; }
};
const Columns& columns(const Module* m);
// the module's tree code reads its constants from the device programs
bool memc(const Module* m);
// waves per workgroup of the loss tree code for a batch whose code reads
// `nraw` raw features: 8 from 10 features on (twice the LDS per workgroup, so
// a wide row tile still fits four times; config #5's shard 20.26 -> 17.10 ms,
// profiles/r03_ab_cfg5.txt), else 4; SRHIP_JIT_WAVES forces a width. And the
// LDS a workgroup of that width may take while the CU holds 5 waves per SIMD.
int choose_waves(int nraw);
// tree code can end its tiles with this elementwise loss (L2 inline, the
// others through a loss routine; gen_jit.py leaves out the ones whose
// registers clash with memory-constant tree code)
bool has_loss_routine(int loss);
// the gradient tree code can seed its reverse pass with this loss (L2 inline,
// the others through their loss and dℓ/dr routines)
bool has_dloss_routine(int loss);
size_t lds_per_workgroup(int waves);
bool part_global();
bool dynamic_trees();

// Statistics of one build.
struct Stats {
  int ntrees = 0;          // trees compiled to code
  int nfast = 0;           // of which have a guarded FAST path
  int nrejected = 0;       // trees left to the interpreter (register pool exhausted, ...)
  int nparts = 0;          // code objects (one launch each)
  size_t code_bytes = 0;
  double ms_codegen = 0.0, ms_load = 0.0;
};

// The embedded template could be parsed (false: no tree compiler, the
// interpreter runs everything).
bool available();
// some routine can hand a tile back to the interpreter (sin/cos built with
// TRIG_BAIL in gen_jit.py); false: the bail flags never need reading
bool can_bail();
// this module's tree code can hand a tree back: can_bail(), or its loss
// routine can (Float32 Periodic beyond the routine's Cody-Waite range)
bool module_bails(const Module* m);
const char* unavailable_reason();

// Compile the trees `cand` (tree ids, in list order) of `cb`. Trees that
// compile are appended to `jit_list` (same order), the others to `rest`.
// Returns the loaded module, or nullptr when no tree compiled. Throws
// srhip::Error on HIP failures.
Module* build(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list,
              std::vector<int32_t>& rest, const Options& opt, Stats* st);
void destroy(Module* m);

// bail flags of all slots + bail count + PRECISE redo count: [nslots + 2]
// uint32 (device), cleared by reset_flags
uint32_t* bail_flags(Module* m);
int nslots(const Module* m);
// the module's code objects: consecutive slot ranges (jit_list order), one launch each
int nparts(const Module* m);
void part(const Module* m, int k, int* slot0, int* nslots);
hipError_t reset_flags(Module* m, hipStream_t stream);
// words at bail_flags(m) that reset_flags clears (per-slot flags + 2 counters)
int64_t flag_words(Module* m);

// Launch part k's driver over its slots (EvalArgs as for eval_kernel: list /
// list_off / fail / partial of the part's slots).
// dcols: the derived columns of this call ([nder][n_pad], launch_derive), or
// null: the driver computes the staged ones itself
// gcols: the shared-subtree columns of this call ([ngcol][n_pad], api.cpp derive_shared), or
// null when the module has none
// whether launch() of part k runs a hand-written loop, which writes 4-byte
// partials (EvalArgs::part4 for the finalize)
bool partials4(Module* m, int k);
hipError_t launch(Module* m, int k, const EvalPlan& plan, const EvalArgs<float>& a, bool fast, const float* dcols,
                  hipStream_t stream, const float* gcols = nullptr);
// out[k][r] = u_k(x_{f_k}[r]) for the module's derived columns (nothing to do when there are none)
hipError_t launch_derive(Module* m, const float* X, int64_t n_pad, float* out, hipStream_t stream);

// Test hook: compile without loading; returns bytes and (opt.text) the
// assembly text of the whole area image.
bool compile_only(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand, const Options& opt,
                  std::vector<uint8_t>* bytes, std::string* text, std::vector<int32_t>* offsets, Stats* st);

// ---- gradient tree code (jit_grad.cpp) ----------------------------------------------
// Reverse-mode ∂L/∂c of every constant of a tree in one pass (any elementwise
// loss has_dloss_routine accepts; lparam: its Float64 parameter's bits), for
// gradient programs (compile_batch(..., grad = true)) of Float32 trees whose
// operators are + - * / neg abs square cube exp sin cos and that have at
// most SR_JIT_G_NGACC constants. Constants are read from a device array at
// run time: new constant sets need no new code.
// Shared subtrees (Columns::gkey) in the gradient code: a constant-free
// subtree needs no adjoint, so the derive pass's column (api.cpp
// derive_shared) stands in for its forward value; the column stays in its
// register block from the tile start to its last forward or reverse use.
// Columns from kGradGbase on (raw features stay below); SRHIP_GJIT_GCOLS caps
// them (default 64, 0: none).
constexpr int kGradGbase = 64;
Columns plan_grad_columns(const CompiledBatch<float>& cb, const std::vector<int32_t>& cand);
struct GradModule;
struct GradStats {
  int ntrees = 0;
  int nrejected = 0;
  int nparts = 0;          // code objects (one launch each)
  size_t code_bytes = 0;
  double ms_codegen = 0.0, ms_load = 0.0;
};
GradModule* build_grad(const CompiledBatch<float>& cb, const std::vector<int32_t>& const_off,
                       const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list, std::vector<int32_t>& rest,
                       GradStats* st, int loss = SRHIP_LOSS_L2, uint64_t lparam = 0);
void destroy_grad(GradModule* m);
int grad_nslots(const GradModule* m);
// the module's code objects: consecutive slot ranges, one launch each
int grad_nparts(const GradModule* m);
void grad_part(const GradModule* m, int k, int* slot0, int* nslots);
// Launch part `part` over its slots (EvalArgs as for launch(): list / fail /
// partial of the slots); consts = the program's constants (+16 readable
// floats of padding), gpart = [nrg][nconst] per-row-group ∂L/∂c partials.
// gcols: the module's shared-subtree columns of this call ([ngcol][n_pad],
// api.cpp derive_shared), or null when grad_columns(m).ngcol == 0
hipError_t launch_grad_code(GradModule* m, int part, const EvalPlan& plan, const EvalArgs<float>& a,
                            const float* consts, float* gpart, int nconst, hipStream_t stream,
                            const float* gcols = nullptr);
const Columns& grad_columns(const GradModule* m);
bool compile_grad_only(const CompiledBatch<float>& cb, const std::vector<int32_t>& const_off,
                       const std::vector<int32_t>& cand, std::vector<uint8_t>* bytes, std::string* text,
                       std::vector<int32_t>* offsets, GradStats* st, int loss = SRHIP_LOSS_L2, uint64_t lparam = 0);

// ---- Float64 tree code (jit64.cpp) ---------------------------------------------------
// The shallow trees of a Float64 program as straight-line code with the
// Float64 interpreter's operator routines (no FAST path), L2 loss; 2 rows per
// lane, 128-row tiles. Constants are literals: a program whose constants are
// set again runs on the interpreter.
struct Module64;
// Options of a Float64 build: per-row output code (srhip_eval_tree_array) or
// the loss of the tile tail (L2 inline, the others by a loss routine, the
// parameter's Float64 bits as literals)
struct Opts64 {
  bool out = false;
  int loss = SRHIP_LOSS_L2;
  uint64_t lparam = 0;
};
bool available64();
Module64* build64(const CompiledBatch<double>& cb, const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list,
                  std::vector<int32_t>& rest, Stats* st, const Opts64& opt = Opts64());
void destroy64(Module64* m);
int nparts64(const Module64* m);
void part64(const Module64* m, int k, int* slot0, int* nslots);
int nraw64(const Module64* m);  // feature columns the code reads (staged per tile)
// plan: tile 128 rows, 256 threads; EvalArgs as for the interpreter (list / fail / partial of the part)
hipError_t launch64(Module64* m, int k, const EvalPlan& plan, const EvalArgs<double>& a, hipStream_t stream);
bool compile_only64(const CompiledBatch<double>& cb, const std::vector<int32_t>& cand, std::vector<uint8_t>* bytes,
                    std::string* text, std::vector<int32_t>* offsets,
                    const Opts64& opt = Opts64());

// ---- Float64 gradient tree code (jit64.cpp GradGen64) --------------------------------
// Reverse-mode ∂L/∂c (L2, or any loss has_dloss_routine64 accepts) of gradient programs of Float64 trees whose
// operators are + - * / ^ neg abs square cube exp log sqrt sin cos, with at
// most SR_JIT64_G_NACC constants, read from a device array at run time; the
// Float64 interpreter's routines (forward values and did_succeed are its own).
struct GradModule64;
GradModule64* build_grad64(const CompiledBatch<double>& cb, const std::vector<int32_t>& const_off,
                           const std::vector<int32_t>& cand, std::vector<int32_t>& jit_list, std::vector<int32_t>& rest,
                           GradStats* st, int loss = SRHIP_LOSS_L2, uint64_t lparam = 0);
// the Float64 loss tree code has this loss's routine
bool has_loss_routine64(int loss);
// the Float64 gradient tree code can seed its reverse pass with this loss
bool has_dloss_routine64(int loss);
void destroy_grad64(GradModule64* m);
int grad64_nslots(const GradModule64* m);
int grad64_nparts(const GradModule64* m);
void grad64_part(const GradModule64* m, int k, int* slot0, int* nslots);
int grad64_nraw(const GradModule64* m);
// plan: tile 128 rows, 256 threads; consts = the program's constants (+16
// readable doubles of padding), gpart = [nrg][nconst] per-row-group ∂L/∂c
hipError_t launch_grad_code64(GradModule64* m, int part, const EvalPlan& plan, const EvalArgs<double>& a,
                              const double* consts, double* gpart, int nconst, hipStream_t stream);
bool compile_grad_only64(const CompiledBatch<double>& cb, const std::vector<int32_t>& const_off,
                         const std::vector<int32_t>& cand, std::vector<uint8_t>* bytes, std::string* text,
                         std::vector<int32_t>* offsets, int loss = SRHIP_LOSS_L2, uint64_t lparam = 0);

}  // namespace jit
}  // namespace srhip
