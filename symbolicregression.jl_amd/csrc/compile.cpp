// compile.cpp — postfix node streams → device accumulator-machine programs.
//
// Per tree:
//  1. parse the post-order stream into nodes (DAG sharing was already
//     expanded by the flattener: a shared child appears once per reference,
//     as DynamicExpressions evaluates it, test_preserve_multiple_parents.jl:9-14);
//  2. fold every maximal feature-free subtree of degree >= 1 into one
//     constant with host_ops.h, reproducing `_eval_constant_tree` (a folded
//     operator output that is non-finite makes the tree fail for every row
//     count, as the reference does before looking at rows);
//  3. static checks of the remaining constant leaves: DynamicExpressions
//     checks every constant leaf that sits next to a feature-bearing subtree
//     (`@return_on_check` in the fused deg2_l0*/deg1_l2* kernels), so a
//     non-finite one fails the tree; a non-finite constant ROOT fails only
//     when there are rows (fill + final array check);
//  4. emit code in Sethi–Ullman order (the operand needing more stack slots
//     first), fusing leaf operands into the consuming instruction.
#include "compile.h"

#include <algorithm>
#include <limits>
#include <exception>
#include <thread>

#include <cmath>
#include <cstring>

#include "host_ops.h"

namespace srhip {
namespace {


struct HNode {
  int deg;       // 0, 1, 2
  int op;        // operator id (deg >= 1)
  int feat;      // feature index (deg 0, -1 for a constant)
  int l, r;      // children
  double val;    // constant value (deg 0 const), held in T precision
  int cidx;      // constant index in get_constants order (deg 0 const); <= -2: folded (cmap fold ref)
  int size;      // nodes in the subtree (postfix: it spans [i - size + 1, i])
  int cpre;      // constants before the subtree's first node (tree-local)
  bool has_feature;
  int need;      // stack slots needed (Sethi–Ullman number for this machine)
};

template <typename T>
struct TreeCompiler {
  std::vector<HNode> nd;
  std::vector<Ins<T>>* out;
  std::vector<int32_t>* cmap;  // parallel to out: batch-wide constant index of each immediate
  std::vector<FoldRec>* folds;
  int cbase = 0;               // batch-wide index of this tree's first constant
  int nbase = 0;               // batch-wide index of this tree's first node
  bool grad = false;  // slot field carries constant indices
  bool fold_fail = false;
  int max_feat = -1;

  static bool is_leaf(const HNode& x) { return x.deg == 0; }

  // Scalar evaluation of a feature-free subtree (`_eval_constant_tree`).
  bool eval_const(int i, T* v) {
    const HNode& x = nd[i];
    if (x.deg == 0) { *v = (T)x.val; return true; }
    if (x.deg == 1) {
      T a;
      if (!eval_const(x.l, &a)) return false;
      *v = host::unop<T>(x.op, a);
      return std::isfinite(*v);
    }
    T a, b;
    if (!eval_const(x.l, &a) || !eval_const(x.r, &b)) return false;
    *v = host::binop<T>(x.op, a, b);
    return std::isfinite(*v);
  }

  void fold(int i) {
    HNode& x = nd[i];
    if (x.deg == 0) return;
    if (!x.has_feature) {
      T v;
      if (!eval_const(i, &v)) {
        fold_fail = true;
        v = std::numeric_limits<T>::quiet_NaN();  // the tree fails statically; a defined immediate (keep_layout)
      }
      const int first = i - x.size + 1;
      folds->push_back({nbase + first, nbase + i + 1, cbase + nd[first].cpre});
      x.deg = 0; x.feat = -1; x.val = (double)v; x.l = x.r = -1;
      x.cidx = -2 - ((int)folds->size() - 1);  // a folded value: its cmap reference
      return;
    }
    fold(x.l);
    if (x.deg == 2) fold(x.r);
  }

  int compute_need(int i) {
    HNode& x = nd[i];
    if (x.deg == 0) return x.need = 0;
    if (x.deg == 1) return x.need = compute_need(x.l);
    int a = compute_need(x.l), b = compute_need(x.r);
    const HNode& L = nd[x.l];
    const HNode& R = nd[x.r];
    if (is_leaf(L) || is_leaf(R)) return x.need = std::max(a, b);
    int hi = std::max(a, b), lo = std::min(a, b);
    return x.need = std::max(hi, lo + 1);
  }

  bool nonroot_const_nonfinite(int i) {
    const HNode& x = nd[i];
    if (x.deg == 0) return x.feat < 0 && !std::isfinite(x.val);
    if (nonroot_const_nonfinite(x.l)) return true;
    return x.deg == 2 && nonroot_const_nonfinite(x.r);
  }

  uint32_t need_x(int opc) const {
    if (grad) return 0;
    const bool nx = opc == OP_LDX || (opc >= OP_BIN0 && variant_needs_x((opc - OP_BIN0) / SRHIP_NUM_BOPS));
    return nx ? kNeedX : 0;
  }
  void put(int opc, int slot, int feat, T imm, int32_t gidx = -1) {
    Ins<T> ins;
    std::memset(&ins, 0, sizeof(ins));
    ins.code = make_code(opc, slot, feat) | need_x(opc);
    ins.imm = imm;
    out->push_back(ins);
    cmap->push_back(gidx);
  }
  // the constant operand x: its immediate and batch-wide index
  void putc(int opc, const HNode& x, int feat) {
    put(opc, ci(x), feat, (T)x.val, x.cidx >= 0 ? cbase + x.cidx : x.cidx <= -2 ? x.cidx : -1);
  }
  void put_feat2(int opc, int f, int g) {
    Ins<T> ins;
    std::memset(&ins, 0, sizeof(ins));
    ins.code = make_code(opc, 0, f) | need_x(opc);
    if constexpr (sizeof(T) == 4) {
      uint32_t gg = (uint32_t)g;
      std::memcpy(&ins.imm, &gg, 4);
    } else {
      uint64_t gg = (uint64_t)g;
      std::memcpy(&ins.imm, &gg, 8);
    }
    out->push_back(ins);
    cmap->push_back(-1);
  }

  // Emit code leaving node i's value in acc; slots [base, ...) are free.
  void emit(int i, int base) {
    const HNode& x = nd[i];
    if (x.deg == 0) {
      if (x.feat >= 0) put(OP_LDX, 0, x.feat, T(0));
      else putc(OP_LDC, x, 0);
      return;
    }
    if (x.deg == 1) {
      emit(x.l, base);
      put(OP_UN0 + x.op, 0, 0, T(0));
      return;
    }
    const HNode& L = nd[x.l];
    const HNode& R = nd[x.r];
    const int op = x.op;
    if (is_leaf(L) && is_leaf(R)) {
      if (L.feat >= 0 && R.feat >= 0) put_feat2(bin_opcode(V_XX, op), L.feat, R.feat);
      else if (L.feat >= 0) putc(bin_opcode(V_XC, op), R, L.feat);
      else if (R.feat >= 0) putc(bin_opcode(V_CX, op), L, R.feat);
      else {  // two constants: only without folding (gradient programs)
        putc(OP_LDC, L, 0);
        putc(bin_opcode(V_AC, op), R, 0);
      }
      return;
    }
    if (is_leaf(R)) {
      emit(x.l, base);
      if (R.feat >= 0) put(bin_opcode(V_AX, op), 0, R.feat, T(0));
      else putc(bin_opcode(V_AC, op), R, 0);
      return;
    }
    if (is_leaf(L)) {
      emit(x.r, base);
      if (L.feat >= 0) put(bin_opcode(V_XA, op), 0, L.feat, T(0));
      else putc(bin_opcode(V_CA, op), L, 0);
      return;
    }
    if (base >= kMaxSlots) throw Error(SRHIP_ERR_UNSUPPORTED, "tree needs more than 16 stack slots");
    if (L.need >= R.need) {
      emit(x.l, base);
      put(OP_PUSH0 + base, base, 0, T(0));
      emit(x.r, base + 1);
      put(OP_POP0 + base, base, 0, T(0));
      put(bin_opcode(V_TA, op), 0, 0, T(0));  // lhs = tmp (left), rhs = acc (right)
    } else {
      emit(x.r, base);
      put(OP_PUSH0 + base, base, 0, T(0));
      emit(x.l, base + 1);
      put(OP_POP0 + base, base, 0, T(0));
      put(bin_opcode(V_AT, op), 0, 0, T(0));  // lhs = acc (left), rhs = tmp (right)
    }
  }

  // slot-field value of a constant operand: its index (gradient programs)
  int ci(const HNode& x) const { return grad ? x.cidx : 0; }

  bool any_const_nonfinite(int i) const {
    const HNode& x = nd[i];
    if (x.deg == 0) return x.feat < 0 && !std::isfinite(x.val);
    if (any_const_nonfinite(x.l)) return true;
    return x.deg == 2 && any_const_nonfinite(x.r);
  }

  int cost(int i) const {
    const HNode& x = nd[i];
    if (x.deg == 0) return 1;
    if (x.deg == 1) return uop_cost(x.op) + cost(x.l);
    return bop_cost(x.op) + cost(x.l) + cost(x.r);
  }
};

}  // namespace

template <typename T>
CompiledBatch<T> compile_batch(const srhip_trees& trees, bool grad, bool keep_layout) {
  if (trees.ntrees < 0) throw Error(SRHIP_ERR_INVALID, "negative tree count");
  if (trees.ntrees > 0 && (!trees.node_off || !trees.kind || !trees.arg || !trees.const_off))
    throw Error(SRHIP_ERR_INVALID, "null tree arrays");
  CompiledBatch<T> cb;
  const int nt = trees.ntrees;
  cb.ntrees = nt;
  cb.tree_off.assign(nt, -1);
  cb.nodes.assign(nt, 0);
  cb.static_fail.assign(nt, 0);
  cb.fail_if_rows.assign(nt, 0);
  cb.need.assign(nt, 0);
  cb.len.assign(nt, 0);
  cb.cost.assign(nt, 0);
  cb.direct.assign(nt, 0);
  const T* consts = static_cast<const T*>(trees.consts);
  TreeCompiler<T> tc;
  tc.out = &cb.code;
  tc.cmap = &cb.cmap;
  tc.folds = &cb.folds;
  tc.grad = grad;
  std::vector<int> stk;
  for (int t = 0; t < nt; ++t) {
    const int b = trees.node_off[t], e = trees.node_off[t + 1];
    const int cb0 = trees.const_off[t], ce = trees.const_off[t + 1];
    if (e <= b) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + " is empty");
    if (ce < cb0) throw Error(SRHIP_ERR_INVALID, "bad const_off");
    tc.nd.assign(e - b, HNode{});
    tc.fold_fail = false;
    tc.cbase = cb0;
    tc.nbase = b;
    stk.clear();
    int ci = cb0;
    for (int i = 0; i < e - b; ++i) {
      HNode& x = tc.nd[i];
      x.l = x.r = -1; x.op = 0; x.feat = -1; x.val = 0; x.need = 0; x.cidx = -1;
      x.cpre = ci - cb0;  // constants before this node (a subtree's first node is a leaf)
      const int kind = trees.kind[b + i];
      const int arg = trees.arg[b + i];
      switch (kind) {
        case SRHIP_NODE_CONST:
          if (ci >= ce) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": more constant leaves than constants");
          x.cidx = ci - cb0;
          x.deg = 0; x.val = (double)consts[ci++]; x.has_feature = false; x.size = 1;
          break;
        case SRHIP_NODE_FEATURE:
          x.deg = 0; x.feat = arg; x.has_feature = true; x.size = 1;
          tc.max_feat = std::max(tc.max_feat, arg);
          break;
        case SRHIP_NODE_UNARY:
          if (arg >= SRHIP_NUM_UOPS) throw Error(SRHIP_ERR_UNSUPPORTED, "unknown unary operator id " + std::to_string(arg));
          if (stk.empty()) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": stack underflow");
          x.deg = 1; x.op = arg; x.l = stk.back(); stk.pop_back();
          x.has_feature = tc.nd[x.l].has_feature;
          x.size = 1 + tc.nd[x.l].size;
          break;
        case SRHIP_NODE_BINARY:
          if (arg >= SRHIP_NUM_BOPS) throw Error(SRHIP_ERR_UNSUPPORTED, "unknown binary operator id " + std::to_string(arg));
          if (stk.size() < 2) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": stack underflow");
          x.deg = 2; x.op = arg;
          x.r = stk.back(); stk.pop_back();
          x.l = stk.back(); stk.pop_back();
          x.has_feature = tc.nd[x.l].has_feature || tc.nd[x.r].has_feature;
          x.size = 1 + tc.nd[x.l].size + tc.nd[x.r].size;
          break;
        default:
          throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": bad node kind " + std::to_string(kind));
      }
      stk.push_back(i);
    }
    if (stk.size() != 1) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": postfix stream does not reduce to one root");
    if (ci != ce) throw Error(SRHIP_ERR_INVALID, "tree " + std::to_string(t) + ": constant count mismatch");
    const int root = stk[0];
    cb.nodes[t] = e - b;
    cb.total_nodes += e - b;
    cb.cost[t] = tc.cost(root);

    if (grad) {
      // gradient programs: no folding; a non-finite constant fails statically
      if (ce - cb0 > 255) throw Error(SRHIP_ERR_UNSUPPORTED, "gradients support at most 255 constants per tree");
      if (tc.any_const_nonfinite(root)) {
        cb.static_fail[t] = 1;
        if (!keep_layout) continue;
      }
      cb.need[t] = tc.compute_need(root);
      if (cb.need[t] > kMaxSlots) throw Error(SRHIP_ERR_UNSUPPORTED, "tree needs more than 16 stack slots");
      cb.tree_off[t] = (int32_t)cb.code.size();
      tc.emit(root, 0);
      tc.put(OP_END, 0, 0, T(0));
      cb.len[t] = (int32_t)cb.code.size() - cb.tree_off[t];
      cb.direct[t] = 1;
      continue;
    }
    const bool root_is_leaf = tc.nd[root].deg == 0;
    tc.fold(root);
    // keep_layout (programs whose constants change: set_constants patches
    // them in place): a tree that fails statically keeps its code too — its
    // verdict decides its result — so that constants that make it finite
    // again are patched into that code instead of rebuilding the program
    if (tc.fold_fail) {
      cb.static_fail[t] = 1;
      if (!keep_layout) continue;
    } else if (root_is_leaf || tc.nd[root].deg == 0) {
      // a leaf (or folded) root: `deg0_eval` fill/copy + the final array check
      const HNode& r = tc.nd[root];
      if (r.feat < 0 && !std::isfinite(r.val)) {
        cb.fail_if_rows[t] = 1;
        if (!keep_layout) continue;
      }
    } else if (tc.nonroot_const_nonfinite(root)) {
      cb.static_fail[t] = 1;
      if (!keep_layout) continue;
    }
    cb.need[t] = tc.compute_need(root);
    if (cb.need[t] > kMaxSlots) throw Error(SRHIP_ERR_UNSUPPORTED, "tree needs more than 16 stack slots");
    cb.tree_off[t] = (int32_t)cb.code.size();
    tc.emit(root, 0);
    tc.put(OP_END, 0, 0, T(0));
    cb.len[t] = (int32_t)cb.code.size() - cb.tree_off[t];
    // folded values are in the map too (folds); set_constants decides the
    // verdict of a keep_layout tree from its patched immediates
    cb.direct[t] = 1;
  }
  cb.max_feature = tc.max_feat;
  // trailing OP_ENDs: the kernels prefetch one instruction past each END and
  // the VGPR-resident-program variant loads kVProgMax + 1 instructions per tree
  for (int i = 0; i <= kVProgMax; ++i) tc.put(OP_END, 0, 0, T(0));
  return cb;
}

template <typename T>
CompiledBatch<T> compile_batch_par(const srhip_trees& trees, bool grad, bool keep_layout) {
  const int nt = trees.ntrees;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nthr = (int)std::min<unsigned>(8u, hw);
  if (nt < 2048 || nthr < 2) return compile_batch<T>(trees, grad, keep_layout);
  const int nchunk = nthr;
  std::vector<CompiledBatch<T>> part(nchunk);
  std::vector<std::exception_ptr> err(nchunk);
  std::vector<std::thread> th;
  for (int k = 0; k < nchunk; ++k) {
    th.emplace_back([&, k] {
      try {
        const int t0 = (int)((int64_t)nt * k / nchunk), t1 = (int)((int64_t)nt * (k + 1) / nchunk);
        srhip_trees v = trees;  // a view of trees [t0, t1): the offsets index the shared arrays
        v.ntrees = t1 - t0;
        v.node_off = trees.node_off + t0;
        v.const_off = trees.const_off + t0;
        part[k] = compile_batch<T>(v, grad, keep_layout);
      } catch (...) {
        err[k] = std::current_exception();
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
  // merge: each part ends in the kVProgMax + 1 trailing OP_ENDs, kept once at the end
  CompiledBatch<T> cb;
  cb.ntrees = nt;
  const size_t tail = (size_t)kVProgMax + 1;
  for (int k = 0; k < nchunk; ++k) {
    CompiledBatch<T>& p = part[k];
    const int32_t base = (int32_t)cb.code.size();
    cb.code.insert(cb.code.end(), p.code.begin(), p.code.end() - (k + 1 < nchunk ? (std::ptrdiff_t)tail : 0));
    const int32_t fbase = (int32_t)cb.folds.size();  // this part's fold references move up by fbase
    for (auto it = p.cmap.begin(); it != p.cmap.end() - (k + 1 < nchunk ? (std::ptrdiff_t)tail : 0); ++it)
      cb.cmap.push_back(*it <= -2 ? *it - fbase : *it);
    cb.folds.insert(cb.folds.end(), p.folds.begin(), p.folds.end());
    cb.direct.insert(cb.direct.end(), p.direct.begin(), p.direct.end());
    for (int32_t o : p.tree_off) cb.tree_off.push_back(o < 0 ? o : o + base);
    cb.nodes.insert(cb.nodes.end(), p.nodes.begin(), p.nodes.end());
    cb.static_fail.insert(cb.static_fail.end(), p.static_fail.begin(), p.static_fail.end());
    cb.fail_if_rows.insert(cb.fail_if_rows.end(), p.fail_if_rows.begin(), p.fail_if_rows.end());
    cb.need.insert(cb.need.end(), p.need.begin(), p.need.end());
    cb.len.insert(cb.len.end(), p.len.begin(), p.len.end());
    cb.cost.insert(cb.cost.end(), p.cost.begin(), p.cost.end());
    cb.max_feature = std::max(cb.max_feature, p.max_feature);
    cb.total_nodes += p.total_nodes;
  }
  return cb;
}

template <typename T>
bool eval_fold(const FoldRec& f, const srhip_trees& trees, T* out) {
  T stk[kMaxFoldDepth];
  int sp = 0;
  const T* c = static_cast<const T*>(trees.consts) + f.const_b;
  for (int i = f.node_b; i < f.node_e; ++i) {
    const int arg = trees.arg[i];
    switch (trees.kind[i]) {
      case SRHIP_NODE_CONST:
        if (sp == kMaxFoldDepth) return false;
        stk[sp++] = *c++;
        break;
      case SRHIP_NODE_UNARY:
        if (sp < 1) return false;
        stk[sp - 1] = host::unop<T>(arg, stk[sp - 1]);
        if (!std::isfinite(stk[sp - 1])) return false;
        break;
      case SRHIP_NODE_BINARY:
        if (sp < 2) return false;
        stk[sp - 2] = host::binop<T>(arg, stk[sp - 2], stk[sp - 1]);
        --sp;
        if (!std::isfinite(stk[sp - 1])) return false;
        break;
      default:
        return false;  // a feature: not a folded subtree
    }
  }
  if (sp != 1) return false;
  *out = stk[0];
  return true;
}

template CompiledBatch<float> compile_batch<float>(const srhip_trees&, bool, bool);
template CompiledBatch<double> compile_batch<double>(const srhip_trees&, bool, bool);
template CompiledBatch<float> compile_batch_par<float>(const srhip_trees&, bool, bool);
template CompiledBatch<double> compile_batch_par<double>(const srhip_trees&, bool, bool);
template bool eval_fold<float>(const FoldRec&, const srhip_trees&, float*);
template bool eval_fold<double>(const FoldRec&, const srhip_trees&, double*);

}  // namespace srhip
