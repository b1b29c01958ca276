/*
 * sr_oracle_eval.h — the recursive array evaluator, instantiated for
 * T = float / double by sr_oracle.c (TEST INFRASTRUCTURE ONLY).
 *
 * Restates DynamicExpressions.jl 0.4.x `eval_tree_array` as called from
 * src/InterfaceDynamicExpressions.jl:50-52 (contract :17-49):
 *  - post-order recursion, one length-n array per leaf / fused leaf pair,
 *    reused in place by unary nodes and left children;
 *  - `is_constant(tree)` subtrees (degree >= 1, no feature leaf) are folded
 *    to a scalar: every operator output is checked with isfinite, constant
 *    leaves inside them are not (deg0_eval_constant returns (val, true));
 *  - fused leaf patterns (named in test/test_evaluation.jl:15-23):
 *      deg2_l0_r0_eval   op(leaf, leaf)
 *      deg2_l0_eval      op(leaf, subtree)      deg2_r0_eval op(subtree, leaf)
 *      deg1_l2_ll0_lr0   u(b(leaf, leaf))       deg1_l1_ll0  u(u(leaf))
 *    constant leaves of a fused pattern are checked (`@return_on_check`);
 *    in the two-operator fusions a non-finite inner value is replaced by Inf
 *    before the outer operator is applied;
 *  - every child array is checked for non-finite values before use
 *    (`@return_on_nonfinite_array`), and so is the final result; the first
 *    failure returns (undef, false).
 * Expected macros: T, SFX, CAT and the operator functions of sr_oracle_ops.h.
 */

typedef struct {
  int deg, op, feat, l, r;
  T val;
  int has_feature; /* subtree contains a feature leaf */
} CAT(onode, SFX);

#define ONODE CAT(onode, SFX)

/* Parse a postfix stream into nodes; returns the root index or -1. */
static int CAT(parse, SFX)(const uint8_t* kind, const uint16_t* arg,
                           const T* consts, int nnodes, ONODE* nd) {
  int* stk = (int*)malloc(sizeof(int) * (nnodes + 1));
  int sp = 0, ci = 0;
  for (int i = 0; i < nnodes; ++i) {
    ONODE* x = &nd[i];
    x->l = x->r = -1;
    x->op = 0; x->feat = 0; x->val = 0;
    switch (kind[i]) {
      case SRHIP_NODE_CONST: x->deg = 0; x->feat = -1; x->val = consts[ci++]; x->has_feature = 0; break;
      case SRHIP_NODE_FEATURE: x->deg = 0; x->feat = arg[i]; x->has_feature = 1; break;
      case SRHIP_NODE_UNARY:
        if (sp < 1) { free(stk); return -1; }
        x->deg = 1; x->op = arg[i]; x->l = stk[--sp];
        x->has_feature = nd[x->l].has_feature; break;
      case SRHIP_NODE_BINARY:
        if (sp < 2) { free(stk); return -1; }
        x->deg = 2; x->op = arg[i]; x->r = stk[--sp]; x->l = stk[--sp];
        x->has_feature = nd[x->l].has_feature | nd[x->r].has_feature; break;
      default: free(stk); return -1;
    }
    stk[sp++] = i;
  }
  int root = (sp == 1) ? stk[0] : -1;
  free(stk);
  return root;
}

static inline int CAT(isfin, SFX)(T v) { return ISFINITE(v); }

static inline T CAT(apply_b, SFX)(int op, T x, T y) {
  switch (op) {
    case SRHIP_BOP_ADD: return CAT(b_add, SFX)(x, y);
    case SRHIP_BOP_SUB: return CAT(b_sub, SFX)(x, y);
    case SRHIP_BOP_MUL: return CAT(b_mul, SFX)(x, y);
    case SRHIP_BOP_DIV: return CAT(b_div, SFX)(x, y);
    case SRHIP_BOP_POW: return CAT(b_pow, SFX)(x, y);
    case SRHIP_BOP_GREATER: return CAT(b_greater, SFX)(x, y);
    case SRHIP_BOP_LOGICAL_OR: return CAT(b_or, SFX)(x, y);
    case SRHIP_BOP_LOGICAL_AND: return CAT(b_and, SFX)(x, y);
    case SRHIP_BOP_MOD: return CAT(b_mod, SFX)(x, y);
    case SRHIP_BOP_MAX: return CAT(b_max, SFX)(x, y);
    case SRHIP_BOP_MIN: return CAT(b_min, SFX)(x, y);
  }
  return (T)NAN;
}
static inline T CAT(apply_u, SFX)(int op, T x) {
  switch (op) {
    case SRHIP_UOP_NEG: return CAT(u_neg, SFX)(x);
    case SRHIP_UOP_SQUARE: return CAT(u_square, SFX)(x);
    case SRHIP_UOP_CUBE: return CAT(u_cube, SFX)(x);
    case SRHIP_UOP_EXP: return CAT(u_exp, SFX)(x);
    case SRHIP_UOP_ABS: return CAT(u_abs, SFX)(x);
    case SRHIP_UOP_LOG: return CAT(u_log, SFX)(x);
    case SRHIP_UOP_LOG2: return CAT(u_log2, SFX)(x);
    case SRHIP_UOP_LOG10: return CAT(u_log10, SFX)(x);
    case SRHIP_UOP_LOG1P: return CAT(u_log1p, SFX)(x);
    case SRHIP_UOP_SQRT: return CAT(u_sqrt, SFX)(x);
    case SRHIP_UOP_SIN: return CAT(u_sin, SFX)(x);
    case SRHIP_UOP_COS: return CAT(u_cos, SFX)(x);
    case SRHIP_UOP_TAN: return CAT(u_tan, SFX)(x);
    case SRHIP_UOP_SINH: return CAT(u_sinh, SFX)(x);
    case SRHIP_UOP_COSH: return CAT(u_cosh, SFX)(x);
    case SRHIP_UOP_TANH: return CAT(u_tanh, SFX)(x);
    case SRHIP_UOP_ATAN: return CAT(u_atan, SFX)(x);
    case SRHIP_UOP_ASINH: return CAT(u_asinh, SFX)(x);
    case SRHIP_UOP_ACOSH: return CAT(u_acosh, SFX)(x);
    case SRHIP_UOP_ATANH_CLIP: return CAT(u_atanh_clip, SFX)(x);
    case SRHIP_UOP_ERF: return CAT(u_erf, SFX)(x);
    case SRHIP_UOP_ERFC: return CAT(u_erfc, SFX)(x);
    case SRHIP_UOP_GAMMA: return CAT(u_gamma, SFX)(x);
    case SRHIP_UOP_RELU: return CAT(u_relu, SFX)(x);
    case SRHIP_UOP_ROUND: return CAT(u_round, SFX)(x);
    case SRHIP_UOP_FLOOR: return CAT(u_floor, SFX)(x);
    case SRHIP_UOP_CEIL: return CAT(u_ceil, SFX)(x);
    case SRHIP_UOP_SIGN: return CAT(u_sign, SFX)(x);
    case SRHIP_UOP_INV: return CAT(u_inv, SFX)(x);
  }
  return (T)NAN;
}

/* Row loops specialised per operator: FOR_EACH_BOP(op, BODY) expands BODY(F)
 * with F the operator's inline function, inside a switch on op. */
#define BOP_CASE(ID, NAME, BODY) case ID: { BODY(CAT(NAME, SFX)) } break;
#define FOR_EACH_BOP(OP, BODY) switch (OP) { \
  BOP_CASE(SRHIP_BOP_ADD, b_add, BODY) BOP_CASE(SRHIP_BOP_SUB, b_sub, BODY) \
  BOP_CASE(SRHIP_BOP_MUL, b_mul, BODY) BOP_CASE(SRHIP_BOP_DIV, b_div, BODY) \
  BOP_CASE(SRHIP_BOP_POW, b_pow, BODY) BOP_CASE(SRHIP_BOP_GREATER, b_greater, BODY) \
  BOP_CASE(SRHIP_BOP_LOGICAL_OR, b_or, BODY) BOP_CASE(SRHIP_BOP_LOGICAL_AND, b_and, BODY) \
  BOP_CASE(SRHIP_BOP_MOD, b_mod, BODY) BOP_CASE(SRHIP_BOP_MAX, b_max, BODY) \
  BOP_CASE(SRHIP_BOP_MIN, b_min, BODY) default: break; }
#define UOP_CASE(ID, NAME, BODY) case ID: { BODY(CAT(NAME, SFX)) } break;
#define FOR_EACH_UOP(OP, BODY) switch (OP) { \
  UOP_CASE(SRHIP_UOP_NEG, u_neg, BODY) UOP_CASE(SRHIP_UOP_SQUARE, u_square, BODY) \
  UOP_CASE(SRHIP_UOP_CUBE, u_cube, BODY) UOP_CASE(SRHIP_UOP_EXP, u_exp, BODY) \
  UOP_CASE(SRHIP_UOP_ABS, u_abs, BODY) UOP_CASE(SRHIP_UOP_LOG, u_log, BODY) \
  UOP_CASE(SRHIP_UOP_LOG2, u_log2, BODY) UOP_CASE(SRHIP_UOP_LOG10, u_log10, BODY) \
  UOP_CASE(SRHIP_UOP_LOG1P, u_log1p, BODY) UOP_CASE(SRHIP_UOP_SQRT, u_sqrt, BODY) \
  UOP_CASE(SRHIP_UOP_SIN, u_sin, BODY) UOP_CASE(SRHIP_UOP_COS, u_cos, BODY) \
  UOP_CASE(SRHIP_UOP_TAN, u_tan, BODY) UOP_CASE(SRHIP_UOP_SINH, u_sinh, BODY) \
  UOP_CASE(SRHIP_UOP_COSH, u_cosh, BODY) UOP_CASE(SRHIP_UOP_TANH, u_tanh, BODY) \
  UOP_CASE(SRHIP_UOP_ATAN, u_atan, BODY) UOP_CASE(SRHIP_UOP_ASINH, u_asinh, BODY) \
  UOP_CASE(SRHIP_UOP_ACOSH, u_acosh, BODY) UOP_CASE(SRHIP_UOP_ATANH_CLIP, u_atanh_clip, BODY) \
  UOP_CASE(SRHIP_UOP_ERF, u_erf, BODY) UOP_CASE(SRHIP_UOP_ERFC, u_erfc, BODY) \
  UOP_CASE(SRHIP_UOP_GAMMA, u_gamma, BODY) UOP_CASE(SRHIP_UOP_RELU, u_relu, BODY) \
  UOP_CASE(SRHIP_UOP_ROUND, u_round, BODY) UOP_CASE(SRHIP_UOP_FLOOR, u_floor, BODY) \
  UOP_CASE(SRHIP_UOP_CEIL, u_ceil, BODY) UOP_CASE(SRHIP_UOP_SIGN, u_sign, BODY) \
  UOP_CASE(SRHIP_UOP_INV, u_inv, BODY) default: break; }

typedef struct {
  const ONODE* nd;
  const T* X;
  int64_t n;
  int nfeat;
} CAT(ectx, SFX);
#define ECTX CAT(ectx, SFX)

#define XAT(c, f, j) ((c)->X[(int64_t)(j) * (c)->nfeat + (f)])

/* _eval_constant_tree: scalar evaluation of a feature-free subtree */
static int CAT(eval_const, SFX)(const ONODE* nd, int i, T* out) {
  const ONODE* x = &nd[i];
  if (x->deg == 0) { *out = x->val; return 1; }
  if (x->deg == 1) {
    T a;
    if (!CAT(eval_const, SFX)(nd, x->l, &a)) return 0;
    *out = CAT(apply_u, SFX)(x->op, a);
    return CAT(isfin, SFX)(*out);
  }
  T a, b;
  if (!CAT(eval_const, SFX)(nd, x->l, &a)) return 0;
  if (!CAT(eval_const, SFX)(nd, x->r, &b)) return 0;
  *out = CAT(apply_b, SFX)(x->op, a, b);
  return CAT(isfin, SFX)(*out);
}

static int CAT(all_finite, SFX)(const T* a, int64_t n) {
  for (int64_t j = 0; j < n; ++j)
    if (!CAT(isfin, SFX)(a[j])) return 0;
  return 1;
}

/* Returns 1 on success with *res a fresh length-n array (caller frees);
 * 0 on failure (res freed / NULL). */
static int CAT(eval_rec, SFX)(const ECTX* c, int i, T** res);

static int CAT(deg0_eval, SFX)(const ECTX* c, const ONODE* x, T** res) {
  int64_t n = c->n;
  T* a = (T*)malloc(sizeof(T) * (n > 0 ? n : 1));
  if (x->feat < 0) {
    for (int64_t j = 0; j < n; ++j) a[j] = x->val;
  } else {
    for (int64_t j = 0; j < n; ++j) a[j] = XAT(c, x->feat, j);
  }
  *res = a;
  return 1;
}

static int CAT(eval_rec, SFX)(const ECTX* c, int i, T** res) {
  const ONODE* nd = c->nd;
  const ONODE* x = &nd[i];
  int64_t n = c->n;
  *res = NULL;
  if (x->deg == 0) return CAT(deg0_eval, SFX)(c, x, res);
  if (!x->has_feature) { /* is_constant(tree): constant folding */
    T v;
    if (!CAT(eval_const, SFX)(nd, i, &v)) return 0;
    T* a = (T*)malloc(sizeof(T) * (n > 0 ? n : 1));
    for (int64_t j = 0; j < n; ++j) a[j] = v;
    *res = a;
    return 1;
  }
  if (x->deg == 1) {
    const ONODE* l = &nd[x->l];
    int op = x->op;
    if (l->deg == 2 && nd[l->l].deg == 0 && nd[l->r].deg == 0) {
      /* deg1_l2_ll0_lr0_eval: u(b(leaf, leaf)); not both constants here */
      const ONODE* ll = &nd[l->l];
      const ONODE* lr = &nd[l->r];
      int opl = l->op;
      if (ll->feat < 0 && !CAT(isfin, SFX)(ll->val)) return 0;
      if (lr->feat < 0 && !CAT(isfin, SFX)(lr->val)) return 0;
      T* a = (T*)malloc(sizeof(T) * (n > 0 ? n : 1));
#define L2BODY(FB)                                                              \
      for (int64_t j = 0; j < n; ++j) {                                         \
        T p = ll->feat < 0 ? ll->val : XAT(c, ll->feat, j);                     \
        T q = lr->feat < 0 ? lr->val : XAT(c, lr->feat, j);                     \
        T xl = FB(p, q);                                                        \
        a[j] = CAT(isfin, SFX)(xl) ? CAT(apply_u, SFX)(op, xl) : (T)INFINITY;   \
      }
      FOR_EACH_BOP(opl, L2BODY)
#undef L2BODY
      *res = a;
      return 1;
    }
    if (l->deg == 1 && nd[l->l].deg == 0) {
      /* deg1_l1_ll0_eval: u(u(leaf)); the leaf is a feature here */
      const ONODE* ll = &nd[l->l];
      int opl = l->op;
      T* a = (T*)malloc(sizeof(T) * (n > 0 ? n : 1));
      for (int64_t j = 0; j < n; ++j) {
        T xl = CAT(apply_u, SFX)(opl, XAT(c, ll->feat, j));
        a[j] = CAT(isfin, SFX)(xl) ? CAT(apply_u, SFX)(op, xl) : (T)INFINITY;
      }
      *res = a;
      return 1;
    }
    /* deg1_eval */
    T* a;
    if (!CAT(eval_rec, SFX)(c, x->l, &a)) return 0;
    if (!CAT(all_finite, SFX)(a, n)) { free(a); return 0; }
#define U1BODY(FU) for (int64_t j = 0; j < n; ++j) a[j] = FU(a[j]);
    FOR_EACH_UOP(op, U1BODY)
#undef U1BODY
    *res = a;
    return 1;
  }
  /* degree 2 */
  const ONODE* l = &nd[x->l];
  const ONODE* r = &nd[x->r];
  int op = x->op;
  if (l->deg == 0 && r->deg == 0) {
    /* deg2_l0_r0_eval (not both constants: that is a constant subtree) */
    if (l->feat < 0 && !CAT(isfin, SFX)(l->val)) return 0;
    if (r->feat < 0 && !CAT(isfin, SFX)(r->val)) return 0;
    T* a = (T*)malloc(sizeof(T) * (n > 0 ? n : 1));
#define B00BODY(FB)                                                          \
    if (l->feat < 0) { T cv = l->val;                                        \
      for (int64_t j = 0; j < n; ++j) a[j] = FB(cv, XAT(c, r->feat, j)); }    \
    else if (r->feat < 0) { T cv = r->val;                                   \
      for (int64_t j = 0; j < n; ++j) a[j] = FB(XAT(c, l->feat, j), cv); }    \
    else { for (int64_t j = 0; j < n; ++j)                                   \
      a[j] = FB(XAT(c, l->feat, j), XAT(c, r->feat, j)); }
    FOR_EACH_BOP(op, B00BODY)
#undef B00BODY
    *res = a;
    return 1;
  }
  if (l->deg == 0) {
    /* deg2_l0_eval: op(leaf, subtree) */
    T* a;
    if (!CAT(eval_rec, SFX)(c, x->r, &a)) return 0;
    if (!CAT(all_finite, SFX)(a, n)) { free(a); return 0; }
    if (l->feat < 0) {
      T cv = l->val;
      if (!CAT(isfin, SFX)(cv)) { free(a); return 0; }
#define BL0C(FB) for (int64_t j = 0; j < n; ++j) a[j] = FB(cv, a[j]);
      FOR_EACH_BOP(op, BL0C)
#undef BL0C
    } else {
#define BL0X(FB) for (int64_t j = 0; j < n; ++j) a[j] = FB(XAT(c, l->feat, j), a[j]);
      FOR_EACH_BOP(op, BL0X)
#undef BL0X
    }
    *res = a;
    return 1;
  }
  if (r->deg == 0) {
    /* deg2_r0_eval: op(subtree, leaf) */
    T* a;
    if (!CAT(eval_rec, SFX)(c, x->l, &a)) return 0;
    if (!CAT(all_finite, SFX)(a, n)) { free(a); return 0; }
    if (r->feat < 0) {
      T cv = r->val;
      if (!CAT(isfin, SFX)(cv)) { free(a); return 0; }
#define BR0C(FB) for (int64_t j = 0; j < n; ++j) a[j] = FB(a[j], cv);
      FOR_EACH_BOP(op, BR0C)
#undef BR0C
    } else {
#define BR0X(FB) for (int64_t j = 0; j < n; ++j) a[j] = FB(a[j], XAT(c, r->feat, j));
      FOR_EACH_BOP(op, BR0X)
#undef BR0X
    }
    *res = a;
    return 1;
  }
  /* deg2_eval */
  T* a;
  if (!CAT(eval_rec, SFX)(c, x->l, &a)) return 0;
  if (!CAT(all_finite, SFX)(a, n)) { free(a); return 0; }
  T* b;
  if (!CAT(eval_rec, SFX)(c, x->r, &b)) { free(a); return 0; }
  if (!CAT(all_finite, SFX)(b, n)) { free(a); free(b); return 0; }
#define B2BODY(FB) for (int64_t j = 0; j < n; ++j) a[j] = FB(a[j], b[j]);
  FOR_EACH_BOP(op, B2BODY)
#undef B2BODY
  free(b);
  *res = a;
  return 1;
}

int CAT(oracle_eval_tree, SFX)(const uint8_t* kind, const uint16_t* arg,
                               const T* consts, int32_t nnodes, const T* X,
                               int64_t n, int32_t nfeat, T* out) {
  if (nnodes <= 0) return 0;
  ONODE* nd = (ONODE*)malloc(sizeof(ONODE) * nnodes);
  int root = CAT(parse, SFX)(kind, arg, consts, nnodes, nd);
  if (root < 0) { free(nd); return 0; }
  ECTX c = {nd, X, n, nfeat};
  T* a = NULL;
  int ok = CAT(eval_rec, SFX)(&c, root, &a);
  if (ok) ok = CAT(all_finite, SFX)(a, n);
  if (a) {
    if (out) memcpy(out, a, sizeof(T) * (size_t)n);
    free(a);
  }
  free(nd);
  return ok;
}

/* elementwise distance losses, r = ŷ - y (docs/src/losses.md) */
static inline double CAT(elem_loss_d, SFX)(int loss, const double* p, double r) {
  double ar = fabs(r);
  switch (loss) {
    case SRHIP_LOSS_L2: return r * r;
    case SRHIP_LOSS_L1: return ar;
    case SRHIP_LOSS_LP: return pow(ar, p[0]);
    case SRHIP_LOSS_HUBER: return ar <= p[0] ? 0.5 * r * r : p[0] * (ar - 0.5 * p[0]);
    case SRHIP_LOSS_LOGCOSH: return ar + log1p(exp(-2.0 * ar)) - 0.69314718055994530942;
    case SRHIP_LOSS_L1EPSINS: return ar > p[0] ? ar - p[0] : 0.0;
    case SRHIP_LOSS_L2EPSINS: { double e = ar > p[0] ? ar - p[0] : 0.0; return e * e; }
    case SRHIP_LOSS_QUANTILE: return r >= 0 ? p[0] * r : (p[0] - 1.0) * r;
    case SRHIP_LOSS_PERIODIC: return 1.0 - cos(r * (2.0 * 3.14159265358979323846 / p[0])); /* k = 2π/c stored, 1 - cos(r·k) */
    case SRHIP_LOSS_LOGITDIST: return ar + 2.0 * log1p(exp(-ar)) - 1.38629436111989061883;
  }
  return NAN;
}

/* ℓ in T: the residual is formed in T (ŷ - y), L2 squares in T (abs2 in T),
 * the other losses evaluate in double and round to T. */
static inline T CAT(elem_loss, SFX)(int loss, const double* p, T yhat, T y) {
  T r = yhat - y;
  if (loss == SRHIP_LOSS_L2) return r * r;
  if (loss == SRHIP_LOSS_L1) return FABS(r);
  if (loss == SRHIP_LOSS_LPINT) return CAT(ipow, SFX)(FABS(r), (long long)p[0]); /* T^Integer in T */
  return (T)CAT(elem_loss_d, SFX)(loss, p, (double)r);
}

void CAT(oracle_eval_loss_batch, SFX)(int32_t ntrees, const int32_t* node_off,
                                      const uint8_t* kind, const uint16_t* arg,
                                      const int32_t* const_off, const T* consts,
                                      const T* X, const T* y, const T* w,
                                      int64_t n, int32_t nfeat, int loss,
                                      const double* params, const int64_t* row_idx,
                                      int64_t nidx, int nthreads, double* out_sum,
                                      T* out_loss, uint8_t* out_ok) {
  const T* Xe = X; const T* ye = y; const T* we = w;
  T *Xg = NULL, *yg = NULL, *wg = NULL;
  int64_t ne = n;
  if (row_idx) { /* score_func_batch: view(X, :, idx) */
    ne = nidx;
    Xg = (T*)malloc(sizeof(T) * (size_t)(nidx * nfeat + 1));
    yg = (T*)malloc(sizeof(T) * (size_t)(nidx + 1));
    if (w) wg = (T*)malloc(sizeof(T) * (size_t)(nidx + 1));
    for (int64_t k = 0; k < nidx; ++k) {
      int64_t i = row_idx[k];
      memcpy(Xg + k * nfeat, X + i * nfeat, sizeof(T) * nfeat);
      yg[k] = y[i];
      if (w) wg[k] = w[i];
    }
    Xe = Xg; ye = yg; we = wg;
  }
  double wsum = 0.0;
  if (we) { for (int64_t i = 0; i < ne; ++i) wsum += (double)we[i]; }
  else wsum = (double)ne;
  if (nthreads <= 0) nthreads = oracle_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
  for (int32_t t = 0; t < ntrees; ++t) {
    int32_t b = node_off[t], e = node_off[t + 1];
    T* pred = (T*)malloc(sizeof(T) * (size_t)(ne > 0 ? ne : 1));
    int ok = CAT(oracle_eval_tree, SFX)(kind + b, arg + b, consts + const_off[t],
                                        e - b, Xe, ne, nfeat, pred);
    double s = NAN;
    if (ok) {
      s = 0.0;
      if (we) { for (int64_t i = 0; i < ne; ++i) s += (double)we[i] * (double)CAT(elem_loss, SFX)(loss, params, pred[i], ye[i]); }
      else { for (int64_t i = 0; i < ne; ++i) s += (double)CAT(elem_loss, SFX)(loss, params, pred[i], ye[i]); }
    }
    free(pred);
    out_ok[t] = (uint8_t)ok;
    out_sum[t] = s;
    if (out_loss) out_loss[t] = ok ? (T)(s / wsum) : (T)INFINITY;
  }
  free(Xg); free(yg); free(wg);
}

/* forward-mode constant gradients (one tangent per constant).
 * did_succeed here: every node value (constant leaves included) finite at
 * every row — the eval_tree_array rule without constant folding; identical
 * to it whenever all constants are finite. */
static int CAT(grad_rec, SFX)(const ECTX* c, int i, int nc, int* cidx,
                              T* val, T* tan /*[nc][n]*/) {
  const ONODE* nd = c->nd;
  const ONODE* x = &nd[i];
  int64_t n = c->n;
  if (x->deg == 0) {
    for (int k = 0; k < nc; ++k) memset(tan + (size_t)k * n, 0, sizeof(T) * (size_t)n);
    if (x->feat < 0) {
      int k = (*cidx)++;
      if (!CAT(isfin, SFX)(x->val)) return 0; /* every node finite, constants included */
      for (int64_t j = 0; j < n; ++j) { val[j] = x->val; tan[(size_t)k * n + j] = 1; }
    } else {
      for (int64_t j = 0; j < n; ++j) val[j] = XAT(c, x->feat, j);
    }
    return 1;
  }
  if (x->deg == 1) {
    if (!CAT(grad_rec, SFX)(c, x->l, nc, cidx, val, tan)) return 0;
    for (int64_t j = 0; j < n; ++j) {
      T d = CAT(du, SFX)(x->op, val[j]);
      val[j] = CAT(apply_u, SFX)(x->op, val[j]);
      for (int k = 0; k < nc; ++k) tan[(size_t)k * n + j] *= d;
    }
    return CAT(all_finite, SFX)(val, n);
  }
  T* v2 = (T*)malloc(sizeof(T) * (size_t)(n > 0 ? n : 1));
  T* t2 = (T*)malloc(sizeof(T) * (size_t)(nc > 0 ? nc : 1) * (size_t)(n > 0 ? n : 1));
  int ok = CAT(grad_rec, SFX)(c, x->l, nc, cidx, val, tan) &&
           CAT(grad_rec, SFX)(c, x->r, nc, cidx, v2, t2);
  if (ok) {
    for (int64_t j = 0; j < n; ++j) {
      T dx, dy;
      CAT(db, SFX)(x->op, val[j], v2[j], &dx, &dy);
      for (int k = 0; k < nc; ++k)
        tan[(size_t)k * n + j] = dx * tan[(size_t)k * n + j] + dy * t2[(size_t)k * n + j];
      val[j] = CAT(apply_b, SFX)(x->op, val[j], v2[j]);
    }
    ok = CAT(all_finite, SFX)(val, n);
  }
  free(v2); free(t2);
  return ok;
}
