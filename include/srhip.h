/*
 * srhip.h — C ABI of libsrhip.so, the MI355X-native batched expression
 * evaluation engine behind SymbolicRegression.jl's scoring hot path.
 *
 * Every entry point below replaces (a batched form of) one reference
 * interface; the reference file:line is cited on each declaration
 * (paths relative to the SymbolicRegression.jl v0.15.0 repository).
 *
 * Conventions
 *  - Plain C: pointers + sizes, no C++ exceptions cross this boundary.
 *  - Status codes: SRHIP_OK (0) on success, < 0 on error; the message of the
 *    last error on the calling thread is returned by srhip_last_error().
 *  - SRHIP_ERR_UNSUPPORTED means "this call is outside the engine's
 *    coverage" (unknown operator, unsupported loss / dtype, non-finite X):
 *    the caller is expected to fall back to the reference CPU path.
 *  - All host buffers are owned by the caller. Calls are synchronous: the
 *    results are in the caller's buffers when the call returns.
 *  - A context serialises the calls made through it (one mutex, one stream).
 *    Use one context per host thread for concurrency. A program belongs to
 *    the context that created it, and an evaluation call runs on the
 *    PROGRAM's context: a dataset (read-only device memory once created) is
 *    shared by every context of its device, so threads create their programs
 *    in their own contexts and evaluate them concurrently on one dataset.
 *    A program and a dataset on different devices give SRHIP_ERR_INVALID.
 *    Destroy a dataset only when no call on it is in progress.
 *  - Trees cross the boundary as post-order (postfix) node streams: for a
 *    node, its left subtree, then its right subtree, then the node itself.
 *    Constants are listed separately, in the order of the constant leaves in
 *    that stream, which is DynamicExpressions' get_constants order (leaf
 *    order, left to right; test/test_derivatives.jl:126-150).
 */
#ifndef SRHIP_H
#define SRHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRHIP_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define SRHIP_OK 0
#define SRHIP_ERR_INVALID (-1)     /* malformed arguments / trees           */
#define SRHIP_ERR_UNSUPPORTED (-2) /* fall back to the reference CPU path  */
#define SRHIP_ERR_DEVICE (-3)      /* HIP runtime failure                  */
#define SRHIP_ERR_NOMEM (-4)       /* host or device allocation failed     */

/* ---- element types (Dataset{T}: src/Dataset.jl:24-34) ------------------ */
#define SRHIP_F32 0
#define SRHIP_F64 1

/* ---- X layouts ---------------------------------------------------------- */
/* Julia's Dataset.X is (nfeatures, n) column-major (src/ProgramConstants.jl:3-5):
 * element (f, i) at X[i*nfeat + f]. FEATURE_MAJOR is element (f, i) at X[f*n + i]. */
#define SRHIP_X_JULIA 0
#define SRHIP_X_FEATURE_MAJOR 1

/* ---- node kinds of the postfix stream ----------------------------------- */
#define SRHIP_NODE_CONST 0   /* Node(; val=c)                               */
#define SRHIP_NODE_FEATURE 1 /* Node(; feature=f); arg = f-1 (0-based)      */
#define SRHIP_NODE_UNARY 2   /* degree-1 node; arg = SRHIP_UOP_*            */
#define SRHIP_NODE_BINARY 3  /* degree-2 node; arg = SRHIP_BOP_*            */

/* ---- operator ids --------------------------------------------------------
 * Semantics follow src/Operators.jl:8-111 after the user-op → safe-op mapping
 * of src/Options.jl:86-120 (binopmap / unaopmap). The Julia shim maps
 * options.operators.binops[i] / unaops[i] to these ids once per Options
 * (srhip_op_lookup gives the id for a Julia function name).            */
#define SRHIP_BOP_ADD 0          /* +, plus            Operators.jl:23-25 */
#define SRHIP_BOP_SUB 1          /* -, sub             :26-28             */
#define SRHIP_BOP_MUL 2          /* *, mult            :29-31             */
#define SRHIP_BOP_DIV 3          /* /, div             :47-49             */
#define SRHIP_BOP_POW 4          /* ^, safe_pow        :38-46             */
#define SRHIP_BOP_GREATER 5      /* greater            :94-99             */
#define SRHIP_BOP_LOGICAL_OR 6   /* logical_or         :104-106           */
#define SRHIP_BOP_LOGICAL_AND 7  /* logical_and        :109-111           */
#define SRHIP_BOP_MOD 8          /* Base.mod (float)   :17                */
#define SRHIP_BOP_MAX 9          /* Base.max (float)                      */
#define SRHIP_BOP_MIN 10         /* Base.min (float)                      */
#define SRHIP_NUM_BOPS 11

#define SRHIP_UOP_NEG 0          /* neg                :90-92             */
#define SRHIP_UOP_SQUARE 1       /* square = x*x       :32-34             */
#define SRHIP_UOP_CUBE 2         /* cube = x*x*x       :35-37             */
#define SRHIP_UOP_EXP 3
#define SRHIP_UOP_ABS 4
#define SRHIP_UOP_LOG 5          /* safe_log           :50-53             */
#define SRHIP_UOP_LOG2 6         /* safe_log2          :54-57             */
#define SRHIP_UOP_LOG10 7        /* safe_log10         :58-61             */
#define SRHIP_UOP_LOG1P 8        /* safe_log1p         :62-65             */
#define SRHIP_UOP_SQRT 9         /* safe_sqrt          :70-73             */
#define SRHIP_UOP_SIN 10
#define SRHIP_UOP_COS 11
#define SRHIP_UOP_TAN 12
#define SRHIP_UOP_SINH 13
#define SRHIP_UOP_COSH 14
#define SRHIP_UOP_TANH 15
#define SRHIP_UOP_ATAN 16
#define SRHIP_UOP_ASINH 17
#define SRHIP_UOP_ACOSH 18       /* safe_acosh         :66-69             */
#define SRHIP_UOP_ATANH_CLIP 19  /* atanh_clip         :14                */
#define SRHIP_UOP_ERF 20
#define SRHIP_UOP_ERFC 21
#define SRHIP_UOP_GAMMA 22       /* gamma (Inf → NaN)  :8-12              */
#define SRHIP_UOP_RELU 23        /* (x+abs(x))/2       :100-102           */
#define SRHIP_UOP_ROUND 24       /* round, ties to even                   */
#define SRHIP_UOP_FLOOR 25
#define SRHIP_UOP_CEIL 26
#define SRHIP_UOP_SIGN 27
#define SRHIP_UOP_INV 28         /* inv(x) = 1/x                          */
#define SRHIP_NUM_UOPS 29

/* ---- elementwise losses (LossFunctions.jl distance losses; r = ŷ - y,
 * docs/src/losses.md:16-80; default L2DistLoss, src/Options.jl:429-431) -- */
#define SRHIP_LOSS_L2 0        /* r^2                                       */
#define SRHIP_LOSS_L1 1        /* |r|                                       */
#define SRHIP_LOSS_LP 2        /* |r|^p,        params[0] = p               */
#define SRHIP_LOSS_HUBER 3     /* |r|<=d ? r^2/2 : d(|r|-d/2), params[0]=d  */
#define SRHIP_LOSS_LOGCOSH 4   /* log(cosh(r))                              */
#define SRHIP_LOSS_L1EPSINS 5  /* max(0, |r|-eps),  params[0] = eps         */
#define SRHIP_LOSS_L2EPSINS 6  /* max(0, |r|-eps)^2, params[0] = eps        */
#define SRHIP_LOSS_QUANTILE 7  /* r>=0 ? tau*r : (tau-1)*r,  params[0] = tau */
#define SRHIP_LOSS_PERIODIC 8  /* 1 - cos(2πr/c), params[0] = c             */
#define SRHIP_LOSS_LOGITDIST 9 /* -log(4 e^r / (1+e^r)^2)                   */
/* LPDistLoss{n} with an INTEGER n (LPDistLoss(3), not LPDistLoss(3.0)):
 * |r|^n by Julia's T^Integer — Float32 stays Float32 (|r|*|r|*|r| for n = 3,
 * else Float64 power by squaring rounded once), Float64 by compensated power
 * by squaring; params[0] = n, integral with |n| < 2^31 (else INVALID). */
#define SRHIP_LOSS_LPINT 10
#define SRHIP_NUM_LOSSES 11

typedef struct srhip_ctx srhip_ctx;
typedef struct srhip_dataset srhip_dataset;
typedef struct srhip_program srhip_program;

/* A batch of trees as postfix node streams (see header comment). */
typedef struct srhip_trees {
  int32_t ntrees;
  const int32_t* node_off;  /* [ntrees+1]: nodes of tree t are node_off[t] .. node_off[t+1]-1 */
  const uint8_t* kind;      /* [node_off[ntrees]] SRHIP_NODE_*                                  */
  const uint16_t* arg;      /* [node_off[ntrees]] feature (0-based) or operator id              */
  const int32_t* const_off; /* [ntrees+1]: constants of tree t                                   */
  const void* consts;       /* [const_off[ntrees]] of the program dtype                          */
} srhip_trees;

/* ---- library / context ------------------------------------------------- */
int32_t srhip_version(void);
const char* srhip_last_error(void);
int32_t srhip_device_count(int32_t* out_count);
int32_t srhip_open(int32_t device, srhip_ctx** out_ctx);
int32_t srhip_close(srhip_ctx* ctx);

/* Operator table: id and arity (1 or 2) for a Julia operator name
 * ("+", "*", "safe_log", "log", "cos", "^", ...), applying binopmap/unaopmap
 * (src/Options.jl:86-120). Unknown → SRHIP_ERR_UNSUPPORTED. */
int32_t srhip_op_lookup(const char* name, int32_t* out_arity, int32_t* out_id);

/* One operator on scalars of the program dtype (SRHIP_F32 / SRHIP_F64), with
 * the engine's semantics (the same host routines its compiler folds
 * constant subtrees with: Operators.jl:8-111, Float32 transcendentals
 * evaluated in double and rounded once). For the host callers that fold
 * constants themselves — DynamicExpressions' `simplify_tree` /
 * `combine_operators`, used by optimize_and_simplify_population
 * (src/SingleIteration.jl:73-74) and the :simplify mutation
 * (src/Mutate.jl:107-109). b is ignored for arity 1. No device work. */
int32_t srhip_op_eval(int32_t dtype, int32_t arity, int32_t id, double a, double b,
                      double* out);

/* The symbol name of the main evaluation kernel the calling thread launched
 * last ("sr_jit_eval_dlp", "eval_kernel<float>", "sr_jit_grad_dl", ...), as
 * rocprofv3 reports it: ties a profile to the kernel that ran (bench.py). */
int32_t srhip_last_kernel_name(char* buf, int32_t len);

/* ---- dataset: Dataset(X, y; weights) src/Dataset.jl:43-64 ----------------
 * Uploads rows [row_begin, row_end) of X / y / w once (the row shard of this
 * device); X is transposed to feature-major on the device. w may be NULL
 * (unweighted). The dataset is immutable after creation. */
int32_t srhip_dataset_create(srhip_ctx* ctx, int32_t dtype, int32_t x_layout,
                             const void* X, const void* y, const void* w,
                             int64_t n, int32_t nfeat, int64_t row_begin,
                             int64_t row_end, srhip_dataset** out_ds);
int32_t srhip_dataset_destroy(srhip_dataset* ds);
/* rows of this shard, Σw (or the row count), Σ y·w (or Σ y) over the shard —
 * the pieces of avg_y (src/Dataset.jl:56-60) — and whether X is all-finite. */
int32_t srhip_dataset_info(const srhip_dataset* ds, int64_t* out_rows,
                           int32_t* out_nfeat, double* out_sum_w,
                           double* out_sum_yw, int32_t* out_x_finite);

/* ---- programs: a compiled, device-resident batch of trees ---------------
 * Flattens/compiles the postfix streams (register allocation, leaf fusion,
 * static constant checks) and uploads them once; evaluate any number of
 * times afterwards. */
int32_t srhip_program_create(srhip_ctx* ctx, int32_t dtype,
                             const srhip_trees* trees, srhip_program** out_prog);
/* srhip_program_create with flags. SRHIP_PROGRAM_VARYING_CONSTANTS: the
 * caller will set new constants (srhip_program_set_constants, the candidates
 * of `optimize_constants`, src/ConstantOptimization.jl:12-19): Float32 tree
 * code is built reading its constants from memory from the start, so no
 * constant set ever recompiles it (without the flag the first set does). */
#define SRHIP_PROGRAM_VARYING_CONSTANTS 1u
/* SRHIP_PROGRAM_INTERPRETED: build no loss / output tree code (the program is
 * scored only on per-tree row sets, srhip_eval_loss_rowsets, which run in the
 * interpreter: a large batch then skips the code generation and load). */
#define SRHIP_PROGRAM_INTERPRETED 2u
int32_t srhip_program_create_ex(srhip_ctx* ctx, int32_t dtype, const srhip_trees* trees, uint32_t flags,
                                srhip_program** out_prog);
int32_t srhip_program_destroy(srhip_program* prog);
/* per-tree node counts (count_nodes, = compute_complexity without a custom
 * complexity mapping, src/Complexity.jl:13-19) */
int32_t srhip_program_info(const srhip_program* prog, int32_t* out_ntrees,
                           int64_t* out_total_nodes, int32_t* out_nodes /*[ntrees] or NULL*/);
/* Replace the constants of every tree (set_constants, in get_constants
 * order) without recompiling; used by batched constant optimisation
 * (src/ConstantOptimization.jl:12-19). consts has const_off[ntrees] entries. */
int32_t srhip_program_set_constants(srhip_program* prog, const void* consts);

/* ---- batched loss: eval_loss / _eval_loss src/LossFunctions.jl:34-67 ----
 * For every tree t:
 *   out_loss_sum[t] = Σ_i w_i · ℓ(ŷ_t,i, y_i) over the shard (fp64)
 *   out_ok[t]       = did_succeed of eval_tree_array (1/0)
 *   *out_weight_sum = Σ_i w_i (or the row count when unweighted)
 * The reference loss is out_loss_sum[t] / *out_weight_sum computed in T, and
 * T(Inf) when !out_ok[t] (src/LossFunctions.jl:36-38). row_idx (NULL = all
 * rows) selects rows with repetition, as score_func_batch does
 * (src/LossFunctions.jl:95-115); indices are 0-based within the shard.
 * Trees whose evaluation fails get out_loss_sum = NaN. */
int32_t srhip_eval_loss(srhip_dataset* ds, const srhip_program* prog,
                        int32_t loss_kind, const double* loss_params,
                        const int64_t* row_idx, int64_t nidx,
                        double* out_loss_sum, double* out_weight_sum,
                        uint8_t* out_ok);
/* Row shards (config #5, src/ConstantOptimization.jl:43 with the rows split
 * over GPUs): srhip_eval_loss's per-tree partials written to DEVICE memory
 * for a device-side all-reduce (RCCL), no host round trip:
 *   d_out[2t]      = Σ_i w_i ℓ(ŷ_t,i, y_i) over the shard (0 if t failed)
 *   d_out[2t + 1]  = 1 if t failed on the shard (did_succeed false), else 0
 *   d_out[2·ntrees] = Σ_i w_i (the row count when unweighted)
 * d_out holds 2·ntrees + 1 doubles on the context's device. Asynchronous:
 * enqueued on the context's stream; srhip_sync(ctx) before another stream
 * or the host reads d_out. Summed over shards: loss = ΣΣ/ΣΣw, did_succeed =
 * (Σ failed == 0). */
int32_t srhip_eval_loss_packed(srhip_dataset* ds, srhip_program* prog, int32_t loss_kind,
                               const double* loss_params, double* d_out);

/* Convenience: srhip_program_create + srhip_eval_loss + destroy (the program
 * in the dataset's context). */
int32_t srhip_eval_loss_batch(srhip_dataset* ds, const srhip_trees* trees,
                              int32_t loss_kind, const double* loss_params,
                              const int64_t* row_idx, int64_t nidx,
                              double* out_loss_sum, double* out_weight_sum,
                              uint8_t* out_ok);
/* The same with the program in `ctx` (a context of the dataset's device):
 * one context per host thread scores that thread's candidates concurrently
 * with the others on one shared dataset (SearchUtils.jl:33-45, one
 * Threads.@spawn per island). */
int32_t srhip_eval_loss_batch_ctx(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees,
                                  int32_t loss_kind, const double* loss_params,
                                  const int64_t* row_idx, int64_t nidx,
                                  double* out_loss_sum, double* out_weight_sum,
                                  uint8_t* out_ok);

/* ---- per-tree minibatches: score_func_batch src/LossFunctions.jl:95-115 ----
 * The reference draws a fresh sample of batch_size rows (with replacement,
 * :98) for EVERY call, i.e. for every candidate it scores (src/Mutate.jl:41-47
 * parents, :199-205 babies). This scores every tree of the program on its own
 * sample in ONE launch: row_idx is [ntrees][batch_size] (0-based within the
 * shard, repetition allowed), tree t evaluated on rows row_idx[t][0..bs).
 *   out_loss_sum[t]   = Σ_k w_{idx[t][k]} · ℓ(ŷ_t, y) over tree t's sample
 *   out_weight_sum[t] = Σ_k w_{idx[t][k]} (batch_size when unweighted)
 *   out_ok[t]         = did_succeed on that sample
 * The loss is out_loss_sum[t] / out_weight_sum[t] in T (Inf if !ok), as
 * srhip_eval_loss. Runs in the interpreter (one tree per workgroup over its
 * gathered sample). */
int32_t srhip_eval_loss_rowsets(srhip_dataset* ds, const srhip_program* prog,
                                int32_t loss_kind, const double* loss_params,
                                const int64_t* row_idx, int64_t batch_size,
                                double* out_loss_sum, double* out_weight_sum,
                                uint8_t* out_ok);
/* Convenience: program (SRHIP_PROGRAM_INTERPRETED) in ctx (NULL = the
 * dataset's context) + srhip_eval_loss_rowsets + destroy — Julia's batched
 * score_func_batch over a vector of candidates. */
int32_t srhip_eval_loss_batch_rowsets_ctx(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees,
                                          int32_t loss_kind, const double* loss_params,
                                          const int64_t* row_idx, int64_t batch_size,
                                          double* out_loss_sum, double* out_weight_sum,
                                          uint8_t* out_ok);

/* ---- per-row outputs: eval_tree_array src/InterfaceDynamicExpressions.jl:50-52
 * out is [ntrees][rows] of the dataset dtype (row-major per tree); rows of a
 * failed tree are unspecified (the reference returns an undef array). */
int32_t srhip_eval_tree_array(srhip_dataset* ds, const srhip_program* prog,
                              void* out, uint8_t* out_ok);

/* ---- constant gradients: eval_grad_tree_array(tree, X, options;
 * variable=false) src/InterfaceDynamicExpressions.jl:105-107, fused with the
 * loss: out_dloss[c] = Σ_i w_i ∂ℓ(ŷ_i, y_i)/∂c for every constant c of every
 * tree (laid out like consts, const_off order). Also returns the loss sums
 * and did_succeed like srhip_eval_loss. */
int32_t srhip_eval_loss_grad(srhip_dataset* ds, const srhip_program* prog,
                             int32_t loss_kind, const double* loss_params,
                             double* out_loss_sum, double* out_dloss,
                             double* out_weight_sum, uint8_t* out_ok);

/* Per-row constant gradients for few trees: out_grad is
 * [total consts][rows] (∂ŷ_i/∂c), out_value [ntrees][rows]. */
int32_t srhip_eval_grad_tree_array(srhip_dataset* ds, const srhip_program* prog,
                                   void* out_value, void* out_grad,
                                   uint8_t* out_ok);

/* ---- batched constant optimisation ----------------------------------------
 * optimize_constants (src/ConstantOptimization.jl:22-65) for every tree of a
 * batch at once — the per-member loop of optimize_and_simplify_population
 * (src/SingleIteration.jl:63-82) in one call: every start (x0 and
 * `nrestarts` perturbed copies x0 .* (1 .+ randn/2), :46-54) of every tree
 * is a candidate, all advance in lockstep, and each phase of an iteration is
 * ONE evaluation of all candidates. BFGS (Newton for one constant, :32-33)
 * with LineSearches.BackTracking, or Nelder-Mead for trees of two or more
 * constants (:35-36); `iterations` = optimizer_iterations (Options.jl,
 * default 8). The best start of a tree is kept if it converged, else the
 * tree keeps x0 (:56-63). Gradients are analytic (srhip_eval_loss_grad), not
 * Optim's finite differences. */
#define SRHIP_OPT_BFGS 0
#define SRHIP_OPT_NELDERMEAD 1
typedef struct srhip_constopt_options {
  int32_t algorithm;          /* SRHIP_OPT_*                                              */
  int32_t iterations;         /* optimizer_iterations                                     */
  int32_t nrestarts;          /* optimizer_nrestarts                                      */
  int32_t loss_kind;          /* SRHIP_LOSS_* (srhip_optimize_constants_batch)            */
  const double* loss_params;  /* the loss parameter, or NULL                              */
  /* [nrestarts * const_off[ntrees]]: the standard normal draws of the
   * perturbed starts (Julia: randn(T, size(x0)) per restart), tree by tree,
   * restart by restart; NULL: drawn from an internal generator seeded with
   * `seed` */
  const double* start_noise;
  uint64_t seed;
} srhip_constopt_options;

/* On the engine: loss and ∂L/∂c of all candidates per launch on `ds` (the
 * programs in `ctx`, a context of the dataset's device; NULL = the dataset's
 * own context). Outputs (caller-owned): out_consts [const_off[ntrees]] of
 * the dtype — the constants to set_constants! (x0 where the run did not
 * converge); out_loss [ntrees] the loss at those constants in T (+Inf on
 * failure); out_converged [ntrees]; out_num_evals [ntrees] loss evaluations
 * (a member's num_evals increment). */
int32_t srhip_optimize_constants_batch(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees,
                                       const srhip_constopt_options* opts, void* out_consts, double* out_loss,
                                       uint8_t* out_converged, double* out_num_evals);
/* Where the last srhip_optimize_constants_batch call of this thread spent
 * its time: out[0..8] = total, program builds, set_constants, loss calls,
 * gradient calls, the kernels inside those calls (HIP events) — seconds —
 * then the number of builds, loss calls, gradient calls and full program
 * rebuilds inside set_constants, then the builds' tree-code generation and
 * code-object load times (s) (the first n of these 12 written). The rest of
 * the total is the host optimiser's own algebra. */
int32_t srhip_constopt_profile(double* out, int32_t n);
/* The same optimiser over any evaluator (row-sharded datasets whose partials
 * the caller all-reduces, custom losses on the CPU, tests): fn scores
 * ntasks candidates — tree_idx[k] is the input tree of candidate k, consts
 * their constants concatenated in that order (values of the dtype) —
 * writing out_f[ntasks] (the loss, +Inf on failure) and, when grad != 0,
 * out_g[constants] (∂L/∂c, NaN for failed candidates). A nonzero return
 * aborts the optimisation with SRHIP_ERR_INVALID. No device is used. */
typedef int32_t (*srhip_constopt_eval_fn)(void* user, int64_t ntasks, const int32_t* tree_idx, const double* consts,
                                          int32_t grad, double* out_f, double* out_g);
int32_t srhip_optimize_constants_cb(const srhip_trees* trees, int32_t dtype, const srhip_constopt_options* opts,
                                    srhip_constopt_eval_fn fn, void* user, void* out_consts, double* out_loss,
                                    uint8_t* out_converged, double* out_num_evals);

/* ---- tree compiler ---------------------------------------------------------
 * Large programs are compiled to machine code, one block per tree
 * (symbolicregression.jl_amd/csrc/jit.cpp for Float32, jit64.cpp for
 * Float64; SRHIP_JIT=0 turns it off, =1 on for every size). Tree code
 * computes exactly what the interpreter computes: eval_loss with L2 and with
 * every elementwise loss (Float32 Periodic: a tile whose |r·2π/c| leaves
 * its routine's Cody-Waite range hands the tree back to the interpreter),
 * and the per-row outputs of eval_tree_array. This reports:
 * trees compiled, of which with a guarded Float32-transcendental path, code
 * bytes, host code generation and code-object load times (ms). All zero for
 * an interpreted program. */
int32_t srhip_program_jit_info(const srhip_program* prog, int32_t* out_ntrees, int32_t* out_nfast,
                               int64_t* out_code_bytes, double* out_ms_codegen, double* out_ms_load);
/* How srhip_program_set_constants applied new constants so far: in place
 * (the device programs' immediates overwritten, same buffers; tree code built
 * with its constants in memory reads them from there) or by a full rebuild
 * (folding or a static verdict changed, or the first new constant set of a
 * tree-code program whose constants were compiled into its code: rebuilt once
 * as memory-constant tree code). */
int32_t srhip_program_update_stats(const srhip_program* prog, int64_t* out_inplace, int64_t* out_rebuilt);
/* Gradient tree code of this program (reverse-mode ∂L/∂c for
 * srhip_eval_loss_grad, built on the first gradient call; Float32: L2 and the
 * losses with a dℓ/dr routine — all but Periodic; Float64 (jit64.cpp): all
 * but LP, the non-integer LPDistLoss; LPINT has its routines in both):
 * trees compiled, trees left to the forward-mode interpreter, code bytes,
 * codegen and load times (ms). All zero before the first gradient call. */
int32_t srhip_program_grad_jit_info(const srhip_program* prog, int32_t* out_ntrees, int32_t* out_nrejected,
                                    int64_t* out_code_bytes, double* out_ms_codegen, double* out_ms_load);
/* Trees of the last eval on this context whose tree code handed a tile back
 * (a sin/cos argument beyond the fast reduction) and were re-evaluated, and
 * tiles that tree code redid with the Float64-evaluated routines (a FAST-path
 * guard fired or the tile failed; out_redone may be NULL). */
int32_t srhip_last_bailed(const srhip_ctx* ctx, int32_t* out_ntrees, int64_t* out_redone);
/* Trees the last eval or gradient on this context ran as tree code (0: all
 * interpreted; srhip_eval_loss_grad: L2 and, compiled at their first use,
 * the other losses with a dℓ/dr routine, Float32 and Float64). */
int32_t srhip_last_tree_code(const srhip_ctx* ctx, int32_t* out_ntrees);
/* Testing hook (no device needed): compile Float32 trees with the tree
 * compiler (fast: bit 0 the guarded FAST path, bit 1 memory-constant code,
 * bit 2 the per-row output code of srhip_eval_tree_array; bit 3: the trees
 * are Float64 (consts double) and go through the Float64 tree compiler; bit
 * 4: no assembly text — the multi-threaded code generation of the product
 * path, whose bytes must equal the text path's).
 * Returns the code bytes, their assembly text ('\n'-separated lines)
 * and, per compiled tree, (tree id, byte offset). Each inout_n* holds the
 * capacity on entry and the size on return; SRHIP_ERR_INVALID if too small. */
int32_t srhip_jit_compile(const srhip_trees* trees, int32_t fast, uint8_t* out_bytes, int64_t* inout_nbytes,
                          char* out_text, int64_t* inout_ntext, int32_t* out_offsets,
                          int64_t* inout_noffsets);
/* Testing hook, same contract: the gradient tree code (reverse-mode ∂L/∂c,
 * the fast path of srhip_eval_loss_grad) of Float32 trees. */
int32_t srhip_jit_compile_grad(const srhip_trees* trees, uint8_t* out_bytes, int64_t* inout_nbytes,
                               char* out_text, int64_t* inout_ntext, int32_t* out_offsets,
                               int64_t* inout_noffsets);
/* Testing hook, same contract: the loss tree code (grad = 0; fast: its
 * guarded FAST path) or the gradient tree code (grad = 1) of Float32 trees
 * for the elementwise loss `loss` (SRHIP_LOSS_*) with its parameter; fast
 * bit 3: Float64 trees through the Float64 tree compiler with that loss's
 * routine in the tile tail, or with grad = 1 their gradient tree code. SRHIP_ERR_UNSUPPORTED when Float32 tree code has no routine for that
 * loss (a Float64 tree without one is not compiled). */
int32_t srhip_jit_compile_loss(const srhip_trees* trees, int32_t grad, int32_t fast, int32_t loss, double loss_param,
                               uint8_t* out_bytes, int64_t* inout_nbytes, char* out_text, int64_t* inout_ntext,
                               int32_t* out_offsets, int64_t* inout_noffsets);
/* Testing hook (no device needed): the host side of
 * srhip_program_set_constants. Compiles the trees (dtype F32/F64), writes
 * new_consts through the programs' constant map (loss programs, grad = 0, or
 * gradient programs, grad = 1) and compares every tree with a fresh compile
 * of the new constants: out_mismatch = trees whose instruction stream or
 * static verdict differs (0 is correct), out_recompiled = trees the update
 * compiled again, out_relayout = 1 when it needed a rebuild instead.
 * grad | 2: the images of a program whose constants change (VARYING_CONSTANTS
 * or after its first set: a tree that fails statically keeps its code). */
int32_t srhip_debug_constant_map(const srhip_trees* trees, int32_t dtype, int32_t grad, const void* new_consts,
                                 int64_t* out_mismatch, int64_t* out_recompiled, int32_t* out_relayout);

/* ---- instrumentation ----------------------------------------------------
 * Device time (ms, HIP events on the context's stream) of the evaluation
 * kernel(s) of the last eval call on this context, and the number of kernel
 * launches it made. */
int32_t srhip_last_kernel_time(const srhip_ctx* ctx, double* out_ms,
                               int32_t* out_launches);
/* Synchronise the context's stream. */
int32_t srhip_sync(srhip_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* SRHIP_H */
