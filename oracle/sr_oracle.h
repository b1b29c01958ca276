/*
 * sr_oracle.h — CPU restatement of SymbolicRegression.jl's scoring hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * / the timed CPU baseline. The product (libsrhip.so and the srhip Python
 * package) never links, loads or calls it.
 *
 * Parity status: the evaluator being restated is DynamicExpressions.jl
 * 0.4.x (compat "0.4.2" at Project.toml:23, no Manifest, so the patch version
 * is unpinned; not vendored in the reference). Julia is absent from this
 * image, so the restatement is pinned by the reference's own known-answer
 * tests (test_operators.jl, test_nan_detection.jl, test_turbo_nan.jl,
 * test_evaluation.jl, test_losses.jl, test_tree_construction.jl,
 * test_derivatives.jl — ported in tests/test_oracle_kat.py) rather than by
 * outputs of the reference itself.
 *
 * Trees use the same postfix node streams as include/srhip.h.
 * X is Julia's Dataset.X layout: (nfeat, n) column-major, X[i*nfeat + f].
 */
#ifndef SR_ORACLE_H
#define SR_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* scalar operator semantics (src/Operators.jl:8-111) */
float oracle_binop_f32(int op, float x, float y);
double oracle_binop_f64(int op, double x, double y);
float oracle_unop_f32(int op, float x);
double oracle_unop_f64(int op, double x);

/* eval_tree_array(tree, X, options) for one tree; returns did_succeed (1/0).
 * out[n] receives the prediction (unspecified when the tree fails). */
int oracle_eval_tree_f32(const uint8_t* kind, const uint16_t* arg,
                         const float* consts, int32_t nnodes, const float* X,
                         int64_t n, int32_t nfeat, float* out);
int oracle_eval_tree_f64(const uint8_t* kind, const uint16_t* arg,
                         const double* consts, int32_t nnodes, const double* X,
                         int64_t n, int32_t nfeat, double* out);

/* elementwise loss ℓ(prediction, target) (LossFunctions distance losses) */
double oracle_elem_loss_f64(int loss, const double* params, double yhat, double y);
float oracle_elem_loss_f32(int loss, const double* params, float yhat, float y);

/* Batched eval_loss over many trees (src/LossFunctions.jl:34-67), threaded
 * over trees with OpenMP (nthreads <= 0: all cores). Per tree:
 *   out_sum[t]  = Σ w_i ℓ_i in fp64 (NaN when the tree fails)
 *   out_ok[t]   = did_succeed
 *   out_loss[t] = the reference's eval_loss value in T: Inf on failure,
 *                 else out_sum / Σw rounded to T.
 * w may be NULL. row_idx (NULL = all rows) selects rows with repetition.  */
void oracle_eval_loss_batch_f32(int32_t ntrees, const int32_t* node_off,
                                const uint8_t* kind, const uint16_t* arg,
                                const int32_t* const_off, const float* consts,
                                const float* X, const float* y, const float* w,
                                int64_t n, int32_t nfeat, int loss,
                                const double* params, const int64_t* row_idx,
                                int64_t nidx, int nthreads, double* out_sum,
                                float* out_loss, uint8_t* out_ok);
void oracle_eval_loss_batch_f64(int32_t ntrees, const int32_t* node_off,
                                const uint8_t* kind, const uint16_t* arg,
                                const int32_t* const_off, const double* consts,
                                const double* X, const double* y, const double* w,
                                int64_t n, int32_t nfeat, int loss,
                                const double* params, const int64_t* row_idx,
                                int64_t nidx, int nthreads, double* out_sum,
                                double* out_loss, uint8_t* out_ok);

/* eval_grad_tree_array(tree, X, options; variable=false) restated by
 * forward-mode differentiation (one tangent per constant). grad is
 * [nconst][n]. Returns did_succeed. */
int oracle_eval_grad_consts_f64(const uint8_t* kind, const uint16_t* arg,
                                const double* consts, int32_t nnodes,
                                const double* X, int64_t n, int32_t nfeat,
                                double* out, double* grad);
/* the same in Float32 arithmetic (the reference's own precision for Float32
 * trees; the tests measure how far it strays from the Float64 gradient) */
int oracle_eval_grad_consts_f32(const uint8_t* kind, const uint16_t* arg,
                                const float* consts, int32_t nnodes,
                                const float* X, int64_t n, int32_t nfeat,
                                float* out, float* grad);

int oracle_max_threads(void);
/* test-only rounding-noise model of the float64 evaluator (sr_oracle.c) */
void oracle_set_noise(double eps, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
