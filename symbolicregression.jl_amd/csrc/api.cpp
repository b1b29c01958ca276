// api.cpp — the C ABI of libsrhip.so (include/srhip.h).
//
// Host runtime: contexts (device + stream + workspace, one mutex), device
// datasets (uploaded once, feature-major, rows padded), compiled programs
// (device resident), evaluation planning and launches, results back to the
// caller's buffers. No C++ exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <limits>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <type_traits>
#include <numeric>
#include <thread>
#include <string>
#include <vector>

#include "../../include/srhip.h"
#include "compile.h"
#include "host_ops.h"
#include "constopt.h"
#include "jit.h"
#include "kernels.h"

namespace srhip {
namespace {
thread_local const char* t_last_kernel = "";
}
void note_kernel(const char* name) { t_last_kernel = name ? name : ""; }
const char* last_kernel() { return t_last_kernel; }
}  // namespace srhip

using namespace srhip;

namespace {

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_CHECK(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      throw Error(SRHIP_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const Error& e) {
    return set_error(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return set_error(SRHIP_ERR_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return set_error(SRHIP_ERR_INVALID, e.what());
  } catch (...) {
    return set_error(SRHIP_ERR_INVALID, "unknown error");
  }
}

// grow-only device buffer
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t n) {
    if (n <= bytes) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) throw Error(SRHIP_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    bytes = n;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// scoped device buffer: freed when it goes out of scope (hipFree waits for
// the device, so an in-flight copy never reads freed memory)
struct ScopedBuf : DevBuf {
  ScopedBuf() = default;
  ScopedBuf(const ScopedBuf&) = delete;
  ScopedBuf& operator=(const ScopedBuf&) = delete;
  ~ScopedBuf() { release(); }
};

constexpr int64_t kRowPad = 8192;  // dataset rows are padded to a multiple of this

int64_t pad_rows(int64_t rows) { return ((std::max<int64_t>(rows, 1) + kRowPad - 1) / kRowPad) * kRowPad; }

size_t dtype_size(int dtype) { return dtype == SRHIP_F32 ? 4 : 8; }

// Persistent host-copy workers of one context (copy_rows_to_host): created
// at the first large per-row output, joined when the context closes. A job is
// one function run by every worker with its index; the caller keeps issuing
// the DMA chunks meanwhile and waits for the job at the end.
class CopyPool {
 public:
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size(); }
  void start(unsigned n, int device) {
    if (!th_.empty()) return;
    for (unsigned j = 0; j < n; ++j)
      th_.emplace_back([this, j, device] {
        const bool dev_ok = hipSetDevice(device) == hipSuccess;
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
          cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
          if (stop_) return;
          seen = gen_;
          std::function<void(unsigned, bool)> f = job_;
          lk.unlock();
          f(j, dev_ok);
          lk.lock();
          if (--busy_ == 0) cv_done_.notify_all();
        }
      });
  }
  void submit(std::function<void(unsigned, bool)> f) {
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = std::move(f);
      busy_ = (unsigned)th_.size();
      ++gen_;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    cv_done_.wait(lk, [&] { return busy_ == 0; });
  }

 private:
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, cv_done_;
  std::function<void(unsigned, bool)> job_;
  uint64_t gen_ = 0;
  unsigned busy_ = 0;
  bool stop_ = false;
};

}  // namespace

struct srhip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // kernel timing of the current call: event pairs recorded around each launch
  // and read after the call's one stream synchronisation (timing_finish)
  std::vector<hipEvent_t> tev;
  int tpairs = 0;
  bool timing_pending = false;
  bool cnt_pending = false;    // tree-code bail / PRECISE-redo counters copied to pin_cnt
  // pinned host copies of the per-tree results 
  double* pin_sum = nullptr;
  uint8_t* pin_ok = nullptr;
  size_t pin_cap = 0;
  // where the finalize of the current evaluation writes the per-tree results:
  // the pinned host buffers themselves (zero copy) or sums / oks on the device
  double* res_sum = nullptr;
  uint8_t* res_ok = nullptr;
  bool res_host = false;
  bool want_device_results = false;  // srhip_eval_loss_packed: per-tree results stay in device buffers
  uint32_t* pin_cnt = nullptr;  // [2]
  // pinned staging of large per-row outputs (srhip_eval_tree_array): two
  // halves, DMA into one while the other is copied to the caller's memory
  unsigned char* pin_stage = nullptr;
  size_t stage_cap = 0;
  std::vector<hipEvent_t> stage_evs;  // one per chunk of a staged copy
  std::unique_ptr<CopyPool> copy_pool;  // its host-copy workers (persistent)
  double last_ms = 0.0;
  int last_launches = 0;
  int last_bailed = 0;  // trees re-evaluated after their tree code handed a tile back
  int last_jit_trees = 0;  // trees the last evaluation ran as tree code
  int64_t last_redone = 0;  // tiles tree code redid with the PRECISE routines
  DevBuf partial, sums, oks, dloss, scratch_idx, gather, derived;
  DevBuf gderived;  // [ngcol][n_pad] shared-subtree columns of the tree code (jit.h Columns)
  DevBuf gpartial, gsum, gok, gti;  // their derive pass's partials, per-column results, threaded records
  DevBuf fail;  // [list slots] early-exit flags of the eval kernel (MODE_LOSS)
  bool fail_clean = false;  // all of `fail` is zero: the finalize kernels clear the flags they read
  DevBuf ti_rec;  // threaded-interpreter records of the shallow f32 list
  DevBuf bail_list, bail_fail;  // trees whose tree code handed a tile back, and their flags
  DevBuf gpart;  // [nrg][nconst] per-row-group ∂L/∂c of the gradient tree code
  std::vector<double> h_sum;
  std::vector<uint8_t> h_ok;
};

struct srhip_dataset {
  srhip_ctx* ctx = nullptr;
  int dtype = SRHIP_F32;
  int64_t rows = 0;
  int nfeat = 0;
  int64_t n_pad = 0;
  void* X = nullptr;
  void* y = nullptr;
  void* w = nullptr;
  double sum_w = 0.0, sum_yw = 0.0;
  bool x_finite = true;
  std::vector<double> h_w;  // host copy of the shard weights (Σw of row samples)
};

struct srhip_program {
  srhip_ctx* ctx = nullptr;
  int dtype = SRHIP_F32;
  int ntrees = 0;
  // host copy of the postfix streams (for set_constants → recompile)
  std::vector<int32_t> node_off, const_off;
  std::vector<uint8_t> kind;
  std::vector<uint16_t> arg;
  std::vector<unsigned char> consts;
  // compiled metadata
  std::vector<int32_t> nodes;
  std::vector<uint8_t> static_fail, fail_if_rows;
  // the static verdicts on the device (srhip_eval_loss_packed), uploaded when stale
  uint8_t* d_verdict = nullptr;
  bool verdict_stale = true;
  int max_feature = -1;
  int64_t total_nodes = 0;
  // device
  void* d_code = nullptr;
  int32_t* d_tree_off = nullptr;
  int32_t* d_list = nullptr;  // [nlist_a + nlist_b]: shallow trees then deep trees
  int nlist_a = 0, nlist_b = 0;
  // tree code (jit.cpp) of the first nlist_j shallow slots, Float32 programs
  jit::Module* jit = nullptr;
  jit::Module64* jit64 = nullptr;  // Float64 programs: the same slots as Float64 tree code (jit64.cpp)
  int nlist_j = 0;
  std::vector<int32_t> h_jit_list;  // the trees of those slots, in slot order
  // the same trees' tree code for other elementwise losses (jit::Options::loss),
  // built at a loss's first evaluation; null m: that loss runs interpreted
  struct LossJit { int kind; uint64_t bits; jit::Module* m; };
  mutable std::vector<LossJit> jit_loss;
  // Float64 programs: the same trees' tree code for the other losses and for
  // per-row outputs (kind -2), built at first use (module64)
  struct LossJit64 { int kind; uint64_t bits; jit::Module64* m; };
  mutable std::vector<LossJit64> jit64_loss;
  // the constants the tree code was built with: the trees of a later loss or
  // output build are compiled with them, so that every tree folds and fails
  // statically as in that build (the slot layouts match); memory-constant code
  // reads the current constants from the programs either way
  std::vector<unsigned char> jit_consts, gjit_consts;
  jit::Stats jit_stats;
  // tree code is compiled for one constant set: a program whose constants are
  // set again (srhip_program_set_constants) runs on the interpreter
  bool jit_allowed = true;
  // tree code whatever the tree count (the shared-subtree derive program: a few dozen subtrees
  // over every row of the call; jit_wanted's 256-tree bar is for the cost of loading a code object
  // per program, which this program pays once and keeps)
  bool jit_forced = false;
  // gradient tree code allowed (the rerun of Periodic's handed-back trees: none)
  bool gjit_allowed = true;
  // tree code reads its constants from the device programs (jit::Options::memc):
  // built at the first new constant set, after which set_constants only
  // updates the programs in place
  bool jit_memc = false;
  // host image of the uploaded programs: set_constants patches the device
  // copies in place when only instruction immediates change
  std::vector<unsigned char> h_code, h_gcode;
  std::vector<int32_t> h_toff, h_gtoff, h_len, h_glen;
  // their constant maps (CompiledBatch::cmap / direct): new constants of a
  // tree whose immediates are its constants are written without a recompile
  std::vector<int32_t> h_cmap, h_gcmap;
  std::vector<uint8_t> h_direct, h_gdirect;
  std::vector<FoldRec> h_folds, h_gfolds;
  // the constants each image was last compiled / patched with: a tree that
  // is recompiled at every set (a failing one) is skipped while they stand
  std::vector<unsigned char> h_cprev, h_gcprev;
  int64_t n_inplace = 0, n_rebuild = 0;
  int opset = OPSET_FULL;      // smallest operator set covering the compiled programs
  // gradient programs (compiled on first use)
  bool grad_built = false;
  bool grad_stale = false;  // constants changed since the gradient programs were patched
  std::vector<uint8_t> g_static_fail;
  void* d_gcode = nullptr;
  int32_t* d_gtree_off = nullptr;
  int32_t* d_gitems = nullptr;  // work items (tree | group << 24): shallow then deep
  int32_t* d_const_off = nullptr;
  // work items by pass: shallow items carrying 1, 2 or kGradG tangents, then deep ones
  int ngitems[4] = {0, 0, 0, 0};
  int g_opset = OPSET_FULL;
  // gradient tree code (jit_grad.cpp) of the Float32 trees it can compile;
  // with it, the interpreter runs the remaining trees' items (ngitems_rest,
  // stored after the ngitems[] items in d_gitems)
  jit::GradModule* gjit = nullptr;
  jit::GradStats gjit_stats;
  // its candidate trees (cost order) and compiled slot list: the gradient tree
  // code of another elementwise loss is built from the same candidates at that
  // loss's first gradient and used only with the same slots (null m: that
  // loss's gradients run interpreted)
  std::vector<int32_t> h_gcand, h_gjl;
  struct GradLossJit { int kind; uint64_t bits; jit::GradModule* m; };
  std::vector<GradLossJit> gjit_loss;
  int ngitems_rest[4] = {0, 0, 0, 0};
  int32_t* d_gjit_list = nullptr;   // [nslots] tree of each gradient-code slot
  int32_t* d_gjit_cidx = nullptr;   // constants of those trees
  int ngjit_cidx = 0;
  float* d_gconsts = nullptr;       // the constants as Float32 (+16 padding)
  // Float64 programs: the gradient tree code of jit64.cpp (L2), its constants (+16 padding)
  jit::GradModule64* gjit64 = nullptr;
  struct GradLossJit64 { int kind; uint64_t bits; jit::GradModule64* m; };
  std::vector<GradLossJit64> gjit64_loss;  // other losses' Float64 gradient tree code (same slots)
  double* d_gconsts64 = nullptr;
  size_t gcs64_cap = 0;
  size_t gjl_cap = 0, gjc_cap = 0, gcs_cap = 0;
  // byte capacities of the device buffers above (kept across rebuilds)
  size_t code_cap = 0, toff_cap = 0, list_cap = 0;
  size_t gcode_cap = 0, gtoff_cap = 0, gitems_cap = 0, gconst_cap = 0;
  // the shared subtrees of the tree code (jit.h Columns) as a program of their
  // own, run by the interpreter's per-row output mode once per call
  // (derive_shared); built at the first call that needs it
  mutable srhip_program* shared = nullptr;
  mutable std::vector<std::string> shared_keys;
  // the same for the gradient tree code's columns (jit::grad_columns)
  mutable srhip_program* gshared = nullptr;
  mutable std::vector<std::string> gshared_keys;
};

namespace {

// Programs are rebuilt by every srhip_program_set_constants (the batched
// constant optimiser does so once per line-search round) and hipFree
// synchronises the device, so rebuilds reuse buffers that are large enough.
void ensure_dev(void** ptr, size_t* cap, size_t bytes) {
  if (*ptr && *cap >= bytes) return;
  if (*ptr) (void)hipFree(*ptr);
  *ptr = nullptr;
  *cap = 0;
  HIP_CHECK(hipMalloc(ptr, bytes));
  *cap = bytes;
}

// ---- per-call kernel timing (no synchronisation per launch) -----------------------
void timing_reset(srhip_ctx* c) {
  c->last_ms = 0.0;
  c->last_launches = 0;
  c->last_bailed = 0;
  c->last_redone = 0;
  c->tpairs = 0;
  c->timing_pending = false;
  c->cnt_pending = false;
}
int timed_begin(srhip_ctx* c, hipStream_t s) {
  while (c->tev.size() < 2 * (size_t)(c->tpairs + 1)) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    c->tev.push_back(e);
  }
  HIP_CHECK(hipEventRecord(c->tev[2 * (size_t)c->tpairs], s));
  return c->tpairs++;
}
void timed_end(srhip_ctx* c, hipStream_t s, int k) {
  HIP_CHECK(hipEventRecord(c->tev[2 * (size_t)k + 1], s));
  c->timing_pending = true;
  c->last_launches += 1;
}
// after the stream is synchronised: kernel times and the copied-back counters
void timing_finish(srhip_ctx* c) {
  if (c->timing_pending) {
    double tot = 0.0;
    for (int k = 0; k < c->tpairs; ++k) {
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, c->tev[2 * (size_t)k], c->tev[2 * (size_t)k + 1]));
      tot += ms;
    }
    c->last_ms = tot;
    c->timing_pending = false;
  }
  if (c->cnt_pending) {
    c->last_redone = c->pin_cnt[1];
    c->cnt_pending = false;
  }
}

void free_grad_device(srhip_program* p) {
  for (void* q : {p->d_gcode, (void*)p->d_gtree_off, (void*)p->d_gitems, (void*)p->d_const_off,
                  (void*)p->d_gjit_list, (void*)p->d_gjit_cidx, (void*)p->d_gconsts})
    if (q) (void)hipFree(q);
  p->d_gcode = nullptr;
  p->d_gtree_off = p->d_gitems = p->d_const_off = nullptr;
  p->d_gjit_list = p->d_gjit_cidx = nullptr;
  p->d_gconsts = nullptr;
  p->gcode_cap = p->gtoff_cap = p->gitems_cap = p->gconst_cap = 0;
  p->gjl_cap = p->gjc_cap = p->gcs_cap = 0;
  jit::destroy_grad(p->gjit);
  p->gjit = nullptr;
  for (auto& l : p->gjit_loss) jit::destroy_grad(l.m);
  p->gjit_loss.clear();
  jit::destroy_grad64(p->gjit64);
  p->gjit64 = nullptr;
  for (auto& l : p->gjit64_loss) jit::destroy_grad64(l.m);
  p->gjit64_loss.clear();
  if (p->d_gconsts64) (void)hipFree(p->d_gconsts64);
  p->d_gconsts64 = nullptr;
  p->gcs64_cap = 0;
  p->grad_built = false;
}

// Gradient tree code on/off: SRHIP_GJIT=0 never, =1 for every Float32
// program, default for programs of at least 256 trees (loading a code object
// costs about a millisecond).
bool gjit_wanted(int ntrees) {
  if (!jit::available() || ntrees == 0) return false;
  const char* e = std::getenv("SRHIP_GJIT");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return ntrees >= 256;
}

// LDS for the row tiles of a gradient tree-code workgroup (SRHIP_GJIT_LDS, KiB:
// experiments); more tiles per workgroup amortise each tree's call over more rows
size_t gjit_tile_budget() {
  static const size_t b = [] {
    const char* e = std::getenv("SRHIP_GJIT_LDS");
    return (size_t)(e ? std::atoi(e) : 52) * 1024;
  }();
  return b;
}

// the constants the gradient tree code reads (s_load), 16 of padding: Float32
// (jit_grad.cpp) or Float64 (jit64.cpp) as the program's
void upload_gconsts(srhip_program* p) {
  const size_t nconst = p->const_off.back();
  if (p->dtype == SRHIP_F64) {
    std::vector<double> h(nconst + 16, 0.0);
    if (nconst) std::memcpy(h.data(), p->consts.data(), nconst * sizeof(double));
    ensure_dev((void**)&p->d_gconsts64, &p->gcs64_cap, h.size() * sizeof(double));
    HIP_CHECK(hipMemcpyAsync(p->d_gconsts64, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, p->ctx->stream));
  } else {
    std::vector<float> h(nconst + 16, 0.0f);
    if (nconst) std::memcpy(h.data(), p->consts.data(), nconst * sizeof(float));
    ensure_dev((void**)&p->d_gconsts, &p->gcs_cap, h.size() * sizeof(float));
    HIP_CHECK(hipMemcpyAsync(p->d_gconsts, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, p->ctx->stream));
  }
  HIP_CHECK(hipStreamSynchronize(p->ctx->stream));
}

void free_loss_jits(const srhip_program* p) {
  for (auto& l : p->jit_loss) jit::destroy(l.m);
  p->jit_loss.clear();
  for (auto& l : p->jit64_loss) jit::destroy64(l.m);
  p->jit64_loss.clear();
}

void free_program_device(srhip_program* p) {
  for (srhip_program** q : {&p->shared, &p->gshared})
    if (*q) {
      free_program_device(*q);
      delete *q;
      *q = nullptr;
    }
  p->shared_keys.clear();
  p->gshared_keys.clear();
  jit::destroy(p->jit);
  p->jit = nullptr;
  jit::destroy64(p->jit64);
  p->jit64 = nullptr;
  free_loss_jits(p);
  p->nlist_j = 0;
  if (p->d_code) (void)hipFree(p->d_code);
  if (p->d_verdict) (void)hipFree(p->d_verdict);
  p->d_verdict = nullptr;
  p->verdict_stale = true;
  if (p->d_tree_off) (void)hipFree(p->d_tree_off);
  if (p->d_list) (void)hipFree(p->d_list);
  p->d_code = nullptr;
  p->d_tree_off = nullptr;
  p->d_list = nullptr;
  p->code_cap = p->toff_cap = p->list_cap = 0;
  free_grad_device(p);
}

// New constants (p->consts) into a built program image, compiling only the
// trees that need it: a tree whose constant-derived immediates are all in the
// constant map (direct) gets the new values written through it — a constant
// as given, a folded subtree evaluated again (eval_fold) — as long as every
// new constant and folded value is finite (the static verdicts then stay
// clear); the others (static failures, non-finite values) are compiled again
// as one small batch and must keep their instruction stream (a tree that
// newly fails statically keeps its old code; its verdict decides its result).
// Returns false when the layout must change (the caller rebuilds: the image
// may then be half patched). *verdicts_changed is set when a static verdict
// moved.
template <typename T>
bool patch_image(srhip_program* p, std::vector<unsigned char>& code, const std::vector<int32_t>& toff,
                 const std::vector<int32_t>& len, std::vector<int32_t>& cmap, std::vector<uint8_t>& direct,
                 std::vector<FoldRec>& folds, std::vector<uint8_t>& sfail, std::vector<uint8_t>* fir, bool grad,
                 bool* verdicts_changed, std::vector<unsigned char>& cprev, int64_t* n_recompiled = nullptr) {
  const int nt = p->ntrees;
  if (cmap.size() * sizeof(Ins<T>) != code.size() || (int)direct.size() != nt || (int)toff.size() != nt ||
      (int)len.size() != nt || (int)sfail.size() != nt)
    return false;
  Ins<T>* ins = reinterpret_cast<Ins<T>*>(code.data());
  const T* c = reinterpret_cast<const T*>(p->consts.data());
  const int32_t* co = p->const_off.data();
  srhip_trees tr;  // the program's own trees with the new constants (eval_fold)
  tr.ntrees = nt;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = co;
  tr.consts = c;
  std::vector<int32_t> redo;
  const bool keep = p->jit_memc;  // compiled with keep_layout: every tree has its code
  const T* cp = cprev.size() == p->consts.size() ? reinterpret_cast<const T*>(cprev.data()) : nullptr;
  for (int t = 0; t < nt; ++t) {
    if (!direct[t] && cp && std::memcmp(cp + co[t], c + co[t], (size_t)(co[t + 1] - co[t]) * sizeof(T)) == 0)
      continue;  // compiled with these very constants: same code, same verdict
    if (direct[t] && keep) {
      // keep_layout: the code stays, the verdict follows from the patched
      // immediates as compile_batch decides it — a folded subtree that is no
      // longer finite fails the tree statically; else a non-finite constant
      // operand does (fail_if_rows for a tree that is one constant)
      bool fold_bad = false, const_bad = false, unsure = false;
      for (int i = toff[t], e = toff[t] + len[t]; i < e; ++i) {
        const int32_t m = cmap[i];
        if (m >= 0) {
          ins[i].imm = c[m];
          const_bad |= !std::isfinite(c[m]);
        } else if (m <= -2) {
          const FoldRec& f = folds[-2 - m];
          if (!eval_fold<T>(f, tr, &ins[i].imm)) {
            ins[i].imm = std::numeric_limits<T>::quiet_NaN();
            if (f.node_e - f.node_b >= kMaxFoldDepth) unsure = true;  // eval_fold's stack, not the value
            else fold_bad = true;
          }
        }
      }
      if (!unsure) {
        const int nb = p->node_off[t], ne = p->node_off[t + 1];
        const bool one_const = ne - nb == 1 && p->kind[nb] == SRHIP_NODE_CONST;
        const uint8_t nsf = (uint8_t)(grad ? const_bad : (fold_bad || (const_bad && !one_const)));
        const uint8_t nfir = (uint8_t)(!grad && !fold_bad && const_bad && one_const);
        if (sfail[t] != nsf || (fir && (*fir)[t] != nfir)) *verdicts_changed = true;
        sfail[t] = nsf;
        if (fir) (*fir)[t] = nfir;
        continue;
      }
    } else if (direct[t]) {
      bool finite = true;
      for (int k = co[t]; k < co[t + 1]; ++k) finite &= std::isfinite(c[k]);
      for (int i = toff[t], e = toff[t] + len[t]; i < e && finite; ++i) {
        const int32_t m = cmap[i];
        if (m >= 0) ins[i].imm = c[m];
        else if (m <= -2) finite = eval_fold<T>(folds[-2 - m], tr, &ins[i].imm);
      }
      if (finite) continue;
    }
    redo.push_back(t);
  }
  if (n_recompiled) *n_recompiled = (int64_t)redo.size();
  if (std::getenv("SRHIP_DEBUG_SETC")) std::fprintf(stderr, "srhip set_constants: %d of %d trees recompiled\n", (int)redo.size(), nt);
  if (redo.empty()) {
    cprev = p->consts;
    return true;
  }
  const int nr = (int)redo.size();
  std::vector<int32_t> s_noff(1, 0), s_coff(1, 0);
  std::vector<uint8_t> s_kind;
  std::vector<uint16_t> s_arg;
  std::vector<T> s_c;
  for (int32_t t : redo) {
    const int b = p->node_off[t], e = p->node_off[t + 1];
    s_kind.insert(s_kind.end(), p->kind.begin() + b, p->kind.begin() + e);
    s_arg.insert(s_arg.end(), p->arg.begin() + b, p->arg.begin() + e);
    s_c.insert(s_c.end(), c + co[t], c + co[t + 1]);
    s_noff.push_back((int32_t)s_kind.size());
    s_coff.push_back((int32_t)s_c.size());
  }
  srhip_trees sub;
  sub.ntrees = nr;
  sub.node_off = s_noff.data();
  sub.kind = s_kind.data();
  sub.arg = s_arg.data();
  sub.const_off = s_coff.data();
  sub.consts = s_c.data();
  CompiledBatch<T> rb = compile_batch_par<T>(sub, grad, p->jit_memc);
  for (int r = 0; r < nr; ++r) {
    const int t = redo[r];
    if (rb.tree_off[r] >= 0) {
      if (toff[t] < 0 || rb.len[r] != len[t]) return false;
      const Ins<T>* src = &rb.code[rb.tree_off[r]];
      for (int j = 0; j < len[t]; ++j)
        if (src[j].code != ins[toff[t] + j].code) return false;
      for (int j = 0; j < len[t]; ++j) {
        ins[toff[t] + j] = src[j];
        const int32_t m = rb.cmap[rb.tree_off[r] + j];
        int32_t& dst = cmap[toff[t] + j];
        if (m >= 0) {
          dst = co[t] + (m - s_coff[r]);
        } else if (m <= -2) {  // the fold, in the program's numbering (reusing the slot it had)
          const FoldRec& f = rb.folds[-2 - m];
          const FoldRec g{p->node_off[t] + (f.node_b - s_noff[r]), p->node_off[t] + (f.node_e - s_noff[r]),
                          co[t] + (f.const_b - s_coff[r])};
          if (dst <= -2) {
            folds[-2 - dst] = g;
          } else {
            folds.push_back(g);
            dst = -2 - ((int32_t)folds.size() - 1);
          }
        } else {
          dst = -1;
        }
      }
      direct[t] = rb.direct[r];
    } else {
      direct[t] = 0;  // keeps its old code: the static verdict decides its result
    }
    if (sfail[t] != rb.static_fail[r] || (fir && (*fir)[t] != rb.fail_if_rows[r])) *verdicts_changed = true;
    sfail[t] = rb.static_fail[r];
    if (fir) (*fir)[t] = rb.fail_if_rows[r];
  }
  cprev = p->consts;
  return true;
}

// New constants for built gradient programs: immediates patched in place when
// the programs keep their shape, else a rebuild. Deferred from set_constants
// to the next gradient call (a line search sets constants many times between
// two gradient calls).
template <typename T>
void patch_grad_constants(srhip_program* p) {
  p->grad_stale = false;
  bool vchg = false;  // the gradient kernels read the verdicts from the programs themselves
  if (patch_image<T>(p, p->h_gcode, p->h_gtoff, p->h_glen, p->h_gcmap, p->h_gdirect, p->h_gfolds, p->g_static_fail,
                     nullptr, /*grad=*/true, &vchg, p->h_gcprev)) {
    hipStream_t s = p->ctx->stream;
    HIP_CHECK(hipMemcpyAsync(p->d_gcode, p->h_gcode.data(), p->h_gcode.size(), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (p->gjit || p->gjit64) upload_gconsts(p);
  } else {
    p->grad_built = false;  // rebuilt below
  }
}

// Gradient programs: compiled without folding, one work item per (tree,
// tangent group of kGradG constants), cost-sorted.
template <typename T>
void build_grad_program(srhip_program* p) {
  if (p->grad_built && p->grad_stale) patch_grad_constants<T>(p);
  if (p->grad_built) return;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->consts.data();
  CompiledBatch<T> cb = compile_batch_par<T>(tr, /*grad=*/true, p->jit_memc);
  if (p->ntrees >= (1 << 24)) throw Error(SRHIP_ERR_UNSUPPORTED, "too many trees for gradient work items");
  p->g_static_fail = cb.static_fail;
  p->g_opset = OPSET_BASIC;
  for (const Ins<T>& ins : cb.code) {
    const int opc = (int)(ins.code & 0xffu);
    if (opc >= OP_BIN0 ? !opset_has_bop(OPSET_BASIC, (opc - OP_BIN0) % SRHIP_NUM_BOPS)
                       : opc >= OP_UN0 && !opset_has_uop(OPSET_BASIC, opc - OP_UN0))
      p->g_opset = OPSET_FULL;
  }
  // gradient tree code for the Float32 trees it can compile (cost-sorted slots)
  jit::destroy_grad(p->gjit);
  p->gjit = nullptr;
  for (auto& l : p->gjit_loss) jit::destroy_grad(l.m);
  p->gjit_loss.clear();
  jit::destroy_grad64(p->gjit64);
  p->gjit64 = nullptr;
  for (auto& l : p->gjit64_loss) jit::destroy_grad64(l.m);
  p->gjit64_loss.clear();
  p->h_gcand.clear();
  p->h_gjl.clear();
  p->gjit_stats = jit::GradStats();
  std::vector<uint8_t> in_jit(p->ntrees, 0);
  std::vector<int32_t> gjl, gcidx;
  if constexpr (std::is_same<T, float>::value) {
    std::vector<int32_t> cand;
    for (int t = 0; t < p->ntrees; ++t)
      if (cb.tree_off[t] >= 0) cand.push_back(t);
    if (p->gjit_allowed && gjit_wanted((int)cand.size())) {
      std::stable_sort(cand.begin(), cand.end(), [&](int32_t x, int32_t y) {
        return cb.cost[x] != cb.cost[y] ? cb.cost[x] > cb.cost[y] : x < y;
      });
      std::vector<int32_t> rest;
      p->gjit = jit::build_grad(cb, p->const_off, cand, gjl, rest, &p->gjit_stats);
      if (p->gjit) {
        p->h_gcand = cand;
        p->h_gjl = gjl;
        p->gjit_consts = p->consts;
      }
      if (p->gjit)
        for (int32_t t : gjl) {
          in_jit[t] = 1;
          for (int k = p->const_off[t]; k < p->const_off[t + 1]; ++k) gcidx.push_back(k);
        }
      else
        gjl.clear();
    }
  } else {  // Float64: the gradient tree code of jit64.cpp (L2)
    std::vector<int32_t> cand;
    for (int t = 0; t < p->ntrees; ++t)
      if (cb.tree_off[t] >= 0) cand.push_back(t);
    if (p->gjit_allowed && gjit_wanted((int)cand.size()) && jit::available64()) {
      std::stable_sort(cand.begin(), cand.end(), [&](int32_t x, int32_t y) {
        return cb.cost[x] != cb.cost[y] ? cb.cost[x] > cb.cost[y] : x < y;
      });
      std::vector<int32_t> rest;
      p->gjit64 = jit::build_grad64(cb, p->const_off, cand, gjl, rest, &p->gjit_stats);
      if (p->gjit64) {
        p->h_gcand = cand;
        p->h_gjl = gjl;
        p->gjit_consts = p->consts;
        for (int32_t t : gjl) {
          in_jit[t] = 1;
          for (int k = p->const_off[t]; k < p->const_off[t + 1]; ++k) gcidx.push_back(k);
        }
      } else {
        gjl.clear();
      }
    }
  }
  // a work item carries the tangents of its group only: groups of 1 and 2
  // constants run in kernels with fewer tangents (and more rows per lane)
  auto by_cost = [](const std::pair<int, int32_t>& x, const std::pair<int, int32_t>& y) {
    return x.first != y.first ? x.first > y.first : x.second < y.second;
  };
  std::vector<int32_t> items;
  for (int rest_only = 0; rest_only < 2; ++rest_only) {
    std::vector<std::pair<int, int32_t>> cls[4];  // (cost, item)
    for (int t = 0; t < p->ntrees; ++t) {
      if (cb.tree_off[t] < 0 || (rest_only && in_jit[t])) continue;
      const int nc = p->const_off[t + 1] - p->const_off[t];
      const int ngroups = std::max(1, (nc + kGradG - 1) / kGradG);
      for (int gi = 0; gi < ngroups; ++gi) {
        const int ntan = std::min(kGradG, nc - gi * kGradG);
        const int k = cb.need[t] > 4 ? 3 : ntan <= 1 ? 0 : ntan <= 2 ? 1 : 2;
        cls[k].push_back({cb.cost[t], (int32_t)(t | (gi << 24))});
      }
    }
    for (int k = 0; k < 4; ++k) {
      std::stable_sort(cls[k].begin(), cls[k].end(), by_cost);
      for (auto& q : cls[k]) items.push_back(q.second);
      (rest_only ? p->ngitems_rest : p->ngitems)[k] = (int)cls[k].size();
    }
  }
  std::vector<int32_t> toff(cb.tree_off);
  for (auto& v : toff) v = std::max(v, 0);
  hipStream_t s = p->ctx->stream;
  ensure_dev(&p->d_gcode, &p->gcode_cap, std::max<size_t>(cb.code.size(), 1) * sizeof(Ins<T>));
  ensure_dev((void**)&p->d_gtree_off, &p->gtoff_cap, std::max<size_t>(toff.size(), 1) * sizeof(int32_t));
  ensure_dev((void**)&p->d_gitems, &p->gitems_cap, std::max<size_t>(items.size(), 1) * sizeof(int32_t));
  ensure_dev((void**)&p->d_const_off, &p->gconst_cap, p->const_off.size() * sizeof(int32_t));
  HIP_CHECK(hipMemcpyAsync(p->d_gcode, cb.code.data(), cb.code.size() * sizeof(Ins<T>), hipMemcpyHostToDevice, s));
  if (!toff.empty())
    HIP_CHECK(hipMemcpyAsync(p->d_gtree_off, toff.data(), toff.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  if (!items.empty())
    HIP_CHECK(hipMemcpyAsync(p->d_gitems, items.data(), items.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(p->d_const_off, p->const_off.data(), p->const_off.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, s));
  p->ngjit_cidx = (int)gcidx.size();
  if (p->gjit || p->gjit64) {
    ensure_dev((void**)&p->d_gjit_list, &p->gjl_cap, gjl.size() * sizeof(int32_t));
    HIP_CHECK(hipMemcpyAsync(p->d_gjit_list, gjl.data(), gjl.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    ensure_dev((void**)&p->d_gjit_cidx, &p->gjc_cap, std::max<size_t>(gcidx.size(), 1) * sizeof(int32_t));
    if (!gcidx.empty())
      HIP_CHECK(hipMemcpyAsync(p->d_gjit_cidx, gcidx.data(), gcidx.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  if (p->gjit || p->gjit64) upload_gconsts(p);
  p->h_gcode.assign(reinterpret_cast<const unsigned char*>(cb.code.data()),
                    reinterpret_cast<const unsigned char*>(cb.code.data() + cb.code.size()));
  p->h_gtoff = cb.tree_off;
  p->h_glen = cb.len;
  p->h_gcmap = cb.cmap;
  p->h_gdirect = cb.direct;
  p->h_gfolds = cb.folds;
  p->h_gcprev = p->consts;
  p->grad_built = true;
  p->grad_stale = false;
}

// Tree code (jit.cpp, jit64.cpp) on/off: SRHIP_JIT=0 never, =1 for every
// program, default for programs of at least 256 shallow trees (code generation
// ~5 µs per tree, loading a code object about a millisecond). The bar was 512
// until round 4: a 512-tree shard of config #2 (bench.py --shard trees, N = 8)
// has 509-512 shallow trees — a tree folds to a constant or fails statically —
// so three of the eight shards ran interpreted at 0.84-0.89 ms against
// 0.55-0.64 ms for the others (profiles/r04_shard_fast.jsonl).
// SRHIP_JIT_FAST=0 keeps the FAST path out.
bool jit_wanted(int nshallow) {
  if (!jit::available() || nshallow == 0) return false;
  const char* e = std::getenv("SRHIP_JIT");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return nshallow >= 256;
}
// Tree code: SRHIP_JIT_CONTIG=1 gives tree group g the contiguous slots
// [g*tpb, (g+1)*tpb) of the cost-sorted list (its code one contiguous range).
// Measured slower than the snake deal (config #2 3.39 -> 3.63 ms, config #5
// gradient 49.6 -> 60.9 ms: the expensive trees end up in a few groups;
// profiles/r02i_evalknobs.txt), so off by default.
bool jit_contig() {
  const char* e = std::getenv("SRHIP_JIT_CONTIG");  // read per launch: A/B measurements
  return e && e[0] == '1';
}

// Tree code: every tree group of a row group on one XCD, so that the row
// group's X tile comes from HBM once and from that XCD's L2 for the other tree
// groups (config #2: 110 -> 32 MB fetched per launch, 3.006 -> 2.982 ms);
// SRHIP_RG_XCD=0: blocks in launch order
bool rg_xcd() {
  const char* e = std::getenv("SRHIP_RG_XCD");  // read per launch: A/B measurements
  return !(e && e[0] == '0');
}
// SRHIP_TG_MAJOR=1 (experiment, read per launch): within an XCD the blocks
// run tree group by tree group (jit_template.hip block_of, rotate 3), so the
// workgroups resident on a CU share their tree code in the instruction cache
int rotate_mode() {
  if (!rg_xcd()) return 0;
  const char* e = std::getenv("SRHIP_TG_MAJOR");
  return (e && e[0] == '1') ? 3 : 2;
}

bool zero_copy_enabled() {
  const char* e = std::getenv("SRHIP_ZERO_COPY");  // read per call: A/B measurements
  return !(e && e[0] == '0');
}
void ensure_pinned(srhip_ctx* c, size_t nt);

// Wait for a call's last launch by polling the stream instead of the runtime's
// blocking wait: hipStreamSynchronize sleeps on a completion interrupt, whose
// wake-up costs tens of microseconds per call on an idle host (more when the
// cores sit in deep C-states), on every synchronous eval_loss. The spin is
// bounded (SRHIP_SPIN_US, default 200 µs: a loss call of a search-sized batch
// ends well within it) and then falls back to the blocking wait, so a long
// kernel (config #5's 48 ms gradients) does not hold a host core that the
// caller's other threads need. SRHIP_SPIN=0: the blocking wait (A/B).
void wait_stream(hipStream_t s) {
  const char* e = std::getenv("SRHIP_SPIN");  // read per call: A/B measurements
  if (e && e[0] == '0') {
    HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  static const double budget_us = [] {
    const char* b = std::getenv("SRHIP_SPIN_US");
    return b ? std::max(0.0, std::atof(b)) : 200.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t r;
  int k = 0;
  while ((r = hipStreamQuery(s)) == hipErrorNotReady) {
    __builtin_ia32_pause();
    if ((++k & 63) == 0 &&
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > budget_us) {
      HIP_CHECK(hipStreamSynchronize(s));
      return;
    }
  }
  HIP_CHECK(r);
}

// LDS for the row tiles of a tree-code workgroup (SRHIP_EVAL_LDS, KiB)
size_t jit_tile_budget() {
  static const size_t b = [] {
    const char* e = std::getenv("SRHIP_EVAL_LDS");
    return (size_t)(e ? std::atoi(e) : 40) * 1024;
  }();
  return b;
}
bool jit_fast_enabled() {
  const char* e = std::getenv("SRHIP_JIT_FAST");
  return !(e && e[0] == '0');
}

template <typename T>
void build_program(srhip_program* p) {
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->consts.data();
  CompiledBatch<T> cb = compile_batch_par<T>(tr, /*grad=*/false, p->jit_memc);
  p->nodes = cb.nodes;
  p->static_fail = cb.static_fail;
  p->fail_if_rows = cb.fail_if_rows;
  p->verdict_stale = true;
  p->max_feature = cb.max_feature;
  p->total_nodes = cb.total_nodes;
  // operator set: every opcode left after folding must be in it
  p->opset = OPSET_BASIC;
  for (const Ins<T>& ins : cb.code) {
    const int opc = (int)(ins.code & 0xffu);
    if (opc >= OP_BIN0 ? !opset_has_bop(OPSET_BASIC, (opc - OP_BIN0) % SRHIP_NUM_BOPS)
                       : opc >= OP_UN0 && !opset_has_uop(OPSET_BASIC, opc - OP_UN0))
      p->opset = OPSET_FULL;
  }
  // trees to run, cost-descending; shallow (<= kShallowSlots) and deep lists
  std::vector<int32_t> a, b;
  for (int t = 0; t < p->ntrees; ++t) {
    if (cb.tree_off[t] < 0) continue;
    (cb.need[t] <= kShallowSlots && cb.len[t] <= kVProgMax ? a : b).push_back(t);
  }
  auto by_cost = [&](int32_t x, int32_t y) {
    return cb.cost[x] != cb.cost[y] ? cb.cost[x] > cb.cost[y] : x < y;
  };
  std::stable_sort(a.begin(), a.end(), by_cost);
  std::stable_sort(b.begin(), b.end(), by_cost);
  // tree code for the shallow Float32 trees of large batches: the compiled
  // trees lead the shallow list, the others follow (interpreter)
  jit::destroy(p->jit);
  p->jit = nullptr;
  jit::destroy64(p->jit64);
  p->jit64 = nullptr;
  free_loss_jits(p);
  p->h_jit_list.clear();
  p->nlist_j = 0;
  p->jit_stats = jit::Stats();
  if constexpr (std::is_same<T, float>::value) {
    if (p->jit_allowed && (jit_wanted((int)a.size()) || (p->jit_forced && jit::available() && !a.empty()))) {
      std::vector<int32_t> jl, rest;
      jit::Options jo;
      jo.fast = jit_fast_enabled();
      const char* me = std::getenv("SRHIP_JIT_MEMC");  // read per build: tests
      jo.memc = p->jit_memc || (me && me[0] == '1');
      p->jit = jit::build(cb, a, jl, rest, jo, &p->jit_stats);
      if (p->jit) {
        p->nlist_j = (int)jl.size();
        p->h_jit_list = jl;
        p->jit_consts = p->consts;
        a = jl;
        a.insert(a.end(), rest.begin(), rest.end());
      }
    }
  } else {
    // Float64 tree code (jit64.cpp) for the shallow trees of large batches;
    // SRHIP_JIT64=0: interpreted
    static const bool on64 = [] { const char* e = std::getenv("SRHIP_JIT64"); return !(e && e[0] == '0'); }();
    // Float64 tree code holds its constants as literals: a VARYING_CONSTANTS program (the
    // optimiser's candidates) would rebuild it interpreted at its first set_constants
    if (on64 && p->jit_allowed && !p->jit_memc && jit_wanted((int)a.size()) && jit::available64()) {
      std::vector<int32_t> jl, rest;
      p->jit64 = jit::build64(cb, a, jl, rest, &p->jit_stats);
      if (p->jit64) {
        p->nlist_j = (int)jl.size();
        p->h_jit_list = jl;
        p->jit_consts = p->consts;
        a = jl;
        a.insert(a.end(), rest.begin(), rest.end());
      }
    }
  }
  p->nlist_a = (int)a.size();
  p->nlist_b = (int)b.size();
  std::vector<int32_t> list(a);
  list.insert(list.end(), b.begin(), b.end());
  std::vector<int32_t> toff(cb.tree_off);
  for (auto& v : toff) v = std::max(v, 0);
  // second half of d_list: program offset of every list slot (one load
  // instead of list -> tree_off when the kernel prefetches the next program)
  const size_t nl = list.size();
  list.resize(2 * nl);
  for (size_t k = 0; k < nl; ++k) list[nl + k] = toff[list[k]];

  p->grad_built = false;  // the gradient programs embed the constants too
  hipStream_t s = p->ctx->stream;
  HIP_CHECK(hipStreamSynchronize(s));  // no launch may still read the old buffers
  // +64 instructions of OP_END padding: the VGPR-resident program load reads
  // 64 instructions from the start of every program
  const size_t ncode_alloc = cb.code.size() + 64;
  ensure_dev(&p->d_code, &p->code_cap, ncode_alloc * sizeof(Ins<T>));
  HIP_CHECK(hipMemsetAsync(p->d_code, 0, ncode_alloc * sizeof(Ins<T>), p->ctx->stream));
  ensure_dev((void**)&p->d_tree_off, &p->toff_cap, std::max<size_t>(toff.size(), 1) * sizeof(int32_t));
  ensure_dev((void**)&p->d_list, &p->list_cap, std::max<size_t>(list.size(), 1) * sizeof(int32_t));
  HIP_CHECK(hipMemcpyAsync(p->d_code, cb.code.data(), cb.code.size() * sizeof(Ins<T>), hipMemcpyHostToDevice, s));
  if (!toff.empty())
    HIP_CHECK(hipMemcpyAsync(p->d_tree_off, toff.data(), toff.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  if (!list.empty())
    HIP_CHECK(hipMemcpyAsync(p->d_list, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
  p->h_code.assign(reinterpret_cast<const unsigned char*>(cb.code.data()),
                   reinterpret_cast<const unsigned char*>(cb.code.data() + cb.code.size()));
  p->h_toff = cb.tree_off;
  p->h_len = cb.len;
  p->h_cmap = cb.cmap;
  p->h_direct = cb.direct;
  p->h_folds = cb.folds;
  p->h_cprev = p->consts;
}

void build_program_f32(srhip_program* p) { build_program<float>(p); }

// srhip_program_set_constants: new immediates written into the host image
// through its constant map (patch_image) and the device programs overwritten
// in place (no reallocation, no list rebuild; the gradient programs are
// patched at the next gradient call); a changed layout rebuilds.
template <typename T>
void update_constants(srhip_program* p) {
  if (p->jit64) {  // Float64 tree code holds its constants as literals: interpreted from now on
    p->jit_allowed = false;
    ++p->n_rebuild;
    const bool had_grad = p->grad_built;
    build_program<T>(p);
    if (had_grad) {
      p->grad_built = true;
      p->grad_stale = true;
    }
    return;
  }
  if (p->jit && !p->jit_memc && !jit::memc(p->jit)) {
    // first new constant set of a tree-code program with constants in its
    // code: rebuilt once as memory-constant tree code (jit.cpp Gen::memc),
    // which later constant sets reach through the in-place program update
    p->jit_memc = true;
    ++p->n_rebuild;
    const bool had_grad = p->grad_built;
    build_program<T>(p);
    if (had_grad) {  // same trees: the gradient programs (and their tree code) only need the constants
      p->grad_built = true;
      p->grad_stale = true;
    }
    return;
  }
  if (!p->jit) p->jit_allowed = false;
  // same layout: the immediates and the host-side static verdicts change in
  // place (the host image is idle: every upload of it ends in a synchronisation,
  // and the copy is ordered after the launches that read the old programs)
  bool vchg = false;
  const auto t0 = std::chrono::steady_clock::now();
  if (!patch_image<T>(p, p->h_code, p->h_toff, p->h_len, p->h_cmap, p->h_direct, p->h_folds, p->static_fail,
                      &p->fail_if_rows, /*grad=*/false, &vchg, p->h_cprev)) {
    ++p->n_rebuild;
    build_program<T>(p);
    if (std::getenv("SRHIP_DEBUG_SETC"))
      std::fprintf(stderr, "srhip set_constants: full rebuild of %d trees %.1f us\n", p->ntrees,
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return;
  }
  if (vchg) p->verdict_stale = true;
  const auto t1 = std::chrono::steady_clock::now();
  hipStream_t s = p->ctx->stream;
  HIP_CHECK(hipMemcpyAsync(p->d_code, p->h_code.data(), p->h_code.size(), hipMemcpyHostToDevice, s));
  if (p->grad_built) p->grad_stale = true;  // patched by the next gradient call (patch_grad_constants)
  HIP_CHECK(hipStreamSynchronize(s));
  if (std::getenv("SRHIP_DEBUG_SETC"))
    std::fprintf(stderr, "srhip set_constants: patch %.1f us, upload of %zu bytes %.1f us\n",
                 std::chrono::duration<double, std::micro>(t1 - t0).count(), p->h_code.size(),
                 std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
  ++p->n_inplace;
}

void check_program_vs_dataset(const srhip_dataset* ds, const srhip_program* p) {
  if (!ds || !p) throw Error(SRHIP_ERR_INVALID, "null dataset or program");
  // a dataset is read-only device memory once created: any context of its
  // device may evaluate a program on it (the program's context runs the call)
  if (ds->ctx->device != p->ctx->device)
    throw Error(SRHIP_ERR_INVALID, "dataset is on device " + std::to_string(ds->ctx->device) + " but the program on device " +
                                       std::to_string(p->ctx->device) +
                                       ": create the program with a context of the dataset's device");
  if (ds->dtype != p->dtype) throw Error(SRHIP_ERR_INVALID, "dataset and program dtypes differ");
  if (p->max_feature >= ds->nfeat)
    throw Error(SRHIP_ERR_INVALID, "tree references feature " + std::to_string(p->max_feature + 1) +
                                       " but the dataset has " + std::to_string(ds->nfeat));
  if (!ds->x_finite)
    throw Error(SRHIP_ERR_UNSUPPORTED,
                "X contains non-finite values: did_succeed of fused leaves differs from the reference; use the CPU path");
}

// Threaded interpreter on/off (SRHIP_TI=0 disables it; built only when the
// kernels were compiled with SR_TI).
static bool ti_enabled() {
  const char* e = std::getenv("SRHIP_TI");  // read per launch: tests compare both paths
  return ti_compiled() && !(e && e[0] == '0');
}

// Row-group rotation of the tree order, off by default (SRHIP_ROT=1 enables
// it): measured 4.09 -> 4.15 ms on config #2.
// The interpreter kernels' waves take their trees from an LDS counter
// (eval_kernel.h, a.rotate & 4): interleaved A/B (tools/interp_dyn_ab.py,
// profiles/r04_interp_dyn_ab.jsonl) config #3 interpreted 0.511 → 0.469 ms,
// a 300-tree batch 0.117 → 0.112, config #2 interpreted 5.95 → 5.90; sums bit
// for bit. SRHIP_INTERP_DYN=0 (read per launch): round-robin.
static bool interp_dyn() {
  const char* e = std::getenv("SRHIP_INTERP_DYN");
  return !(e && e[0] == '0');
}
static bool rotate_enabled() {
  const char* e = std::getenv("SRHIP_ROT");  // read per launch: A/B measurements
  return e && e[0] == '1';
}

// Trees whose tree code handed a tile back (a sin/cos argument beyond the
// fast reduction, jit_template.hip) are evaluated again, whole, by the
// shallow interpreter kernel; finalize overwrites their results.
template <typename T>
void rerun_bailed(srhip_ctx* c, const srhip_program* p, jit::Module* jm, const EvalArgs<T>& ja, const EvalPlan& jplan,
                  int nfeat, int64_t rows, int loss, double lparam) {
  (void)jplan;
  if constexpr (std::is_same<T, float>::value) {
    hipStream_t s = c->stream;
    const int nj = p->nlist_j;
    if (!jit::module_bails(jm)) return;  // no routine hands a tile back: the finalize copied the counters
    std::vector<uint32_t> flags((size_t)nj + 2);
    HIP_CHECK(hipMemcpyAsync(flags.data(), jit::bail_flags(jm), flags.size() * sizeof(uint32_t),
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    c->last_redone = flags[nj + 1];
    if (flags[nj] == 0) return;
    std::vector<int32_t> slots;
    for (int k = 0; k < nj; ++k)
      if (flags[k]) slots.push_back(k);
    if (slots.empty()) return;
    // list = tree ids, list_off = program offsets (copied from the program's list)
    std::vector<int32_t> all((size_t)2 * (p->nlist_a + p->nlist_b));
    HIP_CHECK(hipMemcpyAsync(all.data(), p->d_list, all.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const size_t nl = (size_t)p->nlist_a + p->nlist_b;
    const int nb = (int)slots.size();
    std::vector<int32_t> bl(2 * (size_t)nb);
    for (int k = 0; k < nb; ++k) {
      bl[k] = all[slots[k]];
      bl[nb + k] = all[nl + slots[k]];
    }
    c->bail_list.ensure(bl.size() * sizeof(int32_t));
    c->bail_fail.ensure((size_t)nb * sizeof(uint32_t));
    HIP_CHECK(hipMemcpyAsync(c->bail_list.p, bl.data(), bl.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(c->bail_fail.p, 0, (size_t)nb * sizeof(uint32_t), s));
    EvalPlan plan;
    if (!plan_eval(p->dtype, false, OPSET_FULL, MODE_LOSS, ja.w != nullptr, nfeat, rows, nb, &plan))
      throw Error(SRHIP_ERR_UNSUPPORTED, "row tile does not fit in LDS");
    EvalArgs<T> a = ja;
    a.contig = 0;  // the interpreter kernel deals its slots in snake order
    a.rotate = 0;
    a.list = static_cast<const int32_t*>(c->bail_list.p);
    a.list_off = a.list + nb;
    a.fail = static_cast<uint32_t*>(c->bail_fail.p);
    a.nlist = nb;
    a.ti_rec = nullptr;
    if (ti_enabled()) {
      c->ti_rec.ensure((size_t)nb * 64 * sizeof(uint4));
      HIP_CHECK(launch_ti_records(reinterpret_cast<const Ins<float>*>(a.prog), a.list_off, nb,
                                  (uint32_t)(plan.ntiles * plan.tile * sizeof(T)), static_cast<uint4*>(c->ti_rec.p), s));
      a.ti_rec = static_cast<const uint4*>(c->ti_rec.p);
    }
    a.ntiles = plan.ntiles;
    a.ntg = plan.ntg;
    a.tpb = plan.tpb;
    a.nrg = plan.nrg;
    a.loss = loss;
    a.lparam = lparam;
    c->partial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<T>));
    a.partial = static_cast<Part<T>*>(c->partial.p);
    const int tk = timed_begin(c, s);
    note_kernel(sizeof(T) == 4 ? "eval_kernel<float>" : "eval_kernel<double>");
    HIP_CHECK(launch_eval<T>(plan, a, MODE_LOSS, s));
    timed_end(c, s, tk);
    HIP_CHECK(launch_finalize<T>(a, c->res_sum, c->res_ok, s));
    c->last_bailed = nb;
    if (std::getenv("SRHIP_DEBUG_PASSES")) std::fprintf(stderr, "srhip pass bail-rerun: %d trees\n", nb);
  }
}

// Compute units of the context's device (queried once).
int device_cus(const srhip_ctx* c) {
  // contexts on several threads may ask at once: each entry is written with
  // the same value by whichever thread gets there first
  static std::atomic<int> cus[64];
  const int d = c->device;
  if (d < 0 || d >= 64) return 256;
  int v = cus[d].load(std::memory_order_relaxed);
  if (!v) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0) v = 256;
    cus[d].store(v, std::memory_order_relaxed);
  }
  return v;
}

// Tree-code grids whose workgroups fill a whole number of rounds of the
// device's resident workgroups plus a fraction f of one: the last round
// would run with most of the device idle. The row groups past the whole
// rounds are cut into single tiles instead (a quarter of the work each),
// when their rounds, ceil(f·ntiles)/ntiles, come to less than a full one.
// Rounds are counted at 5 waves per SIMD (the tree code's 94 VGPRs, LDS per
// workgroup sized to match: jit::lds_per_workgroup). SRHIP_JIT_TAIL=0 keeps
// every row group whole.
void tail_split(const srhip_ctx* c, EvalPlan* plan, int64_t rows, int jw) {
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_TAIL"); return !(e && e[0] == '0'); }();
  if (!on || plan->ntiles < 2 || rows <= 0) return;
  const int64_t conc = (int64_t)device_cus(c) * std::max(1, 20 / jw);
  const int64_t W = (int64_t)plan->nrg * plan->ntg;
  const int64_t full = W / conc;
  const int64_t rest = W - full * conc;  // workgroups of the last, partial round
  if (full < 1 || rest == 0) return;
  // row groups in the whole rounds (the remaining ones become single tiles)
  const int64_t nbig = full * conc / plan->ntg;
  const int64_t left_rows = rows - nbig * (int64_t)plan->rows_wg;
  if (nbig < 1 || left_rows <= 0) return;
  const int64_t nsmall = (left_rows + plan->tile - 1) / plan->tile;
  const int64_t small_rounds_x = (nsmall * plan->ntg + conc - 1) / conc;  // rounds of single-tile groups
  if (small_rounds_x >= plan->ntiles) return;  // no shorter than one more round of whole groups
  plan->nbig = (int)nbig;
  plan->ts = 1;
  plan->nrg = (int)(nbig + nsmall);
}

// The tree code of a Float32 program for an elementwise loss: the L2 build
// itself, or (other losses) the same trees compiled with that loss's tile
// tail, built at the loss's first evaluation and kept with the program
// (SRHIP_JIT_LOSSES=0: other losses interpreted). Null: no tree code.
jit::Module* loss_module(const srhip_program* p, int loss, double lparam) {
  if (!p->jit || p->nlist_j == 0) return nullptr;
  if (loss == SRHIP_LOSS_L2) return p->jit;
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_LOSSES"); return !(e && e[0] == '0'); }();
  if (!on || loss < 0 || loss >= SRHIP_NUM_LOSSES || !jit::has_loss_routine(loss)) return nullptr;
  uint64_t bits;
  std::memcpy(&bits, &lparam, 8);
  for (const auto& l : p->jit_loss)
    if (l.kind == loss && l.bits == bits) return l.m;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->jit_consts.data();
  CompiledBatch<float> cb = compile_batch_par<float>(tr);
  jit::Options jo;
  jo.fast = jit_fast_enabled();
  jo.memc = jit::memc(p->jit);
  jo.loss = loss;
  jo.lparam = bits;
  std::vector<int32_t> jl, rest;
  jit::Stats st;
  jit::Module* m = jit::build(cb, p->h_jit_list, jl, rest, jo, &st);
  if (m && (jl != p->h_jit_list || !rest.empty())) {
    jit::destroy(m);  // a different slot layout: this loss runs interpreted
    m = nullptr;
  }
  p->jit_loss.push_back({loss, bits, m});
  return m;
}

// The Float64 tree code of a program for an elementwise loss (L2: the build
// itself; the others: the same trees with that loss's routine in the tile
// tail, jit64.cpp emit_tail_loss) or for per-row outputs (kind -2:
// srhip_eval_tree_array, jit64.cpp emit_store_out), built at its first use
// and kept with the program; null (SRHIP_JIT64_EXTRA=0, a different slot
// layout): interpreted. The constants are literals of the code: new constants
// destroy it with the L2 build (update_constants).
jit::Module64* module64(const srhip_program* p, int kind, double lparam) {
  if (!p->jit64 || p->nlist_j == 0) return nullptr;
  if (kind == SRHIP_LOSS_L2) return p->jit64;
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT64_EXTRA"); return !(e && e[0] == '0'); }();
  if (!on || kind < -2 || kind >= SRHIP_NUM_LOSSES || (kind >= 0 && !jit::has_loss_routine64(kind))) return nullptr;
  uint64_t bits = 0;
  if (kind != -2) std::memcpy(&bits, &lparam, 8);
  for (const auto& l : p->jit64_loss)
    if (l.kind == kind && l.bits == bits) return l.m;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->jit_consts.data();
  CompiledBatch<double> cb = compile_batch_par<double>(tr);
  jit::Opts64 o;
  o.out = kind == -2;
  o.loss = kind == -2 ? SRHIP_LOSS_L2 : kind;
  o.lparam = bits;
  std::vector<int32_t> jl, rest;
  jit::Stats st;
  jit::Module64* m = jit::build64(cb, p->h_jit_list, jl, rest, &st, o);
  if (m && (jl != p->h_jit_list || !rest.empty())) {
    jit::destroy64(m);  // a different slot layout: interpreted
    m = nullptr;
  }
  p->jit64_loss.push_back({kind, bits, m});
  return m;
}

// The per-row output tree code of a Float32 program (srhip_eval_tree_array):
// the same trees compiled with jit::Options::out, PRECISE routines only, built
// at the first per-row evaluation and kept with the program (kind -2 in
// jit_loss); null (SRHIP_JIT_OUT=0, a different slot layout): interpreted.
jit::Module* out_module(const srhip_program* p) {
  if (!p->jit || p->nlist_j == 0) return nullptr;
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_OUT"); return !(e && e[0] == '0'); }();
  if (!on) return nullptr;
  for (const auto& l : p->jit_loss)
    if (l.kind == -2) return l.m;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->jit_consts.data();
  CompiledBatch<float> cb = compile_batch_par<float>(tr);
  jit::Options jo;
  jo.fast = false;
  jo.memc = jit::memc(p->jit);
  jo.out = true;
  std::vector<int32_t> jl, rest;
  jit::Stats st;
  jit::Module* m = jit::build(cb, p->h_jit_list, jl, rest, jo, &st);
  if (m && (jl != p->h_jit_list || !rest.empty())) {
    jit::destroy(m);
    m = nullptr;
  }
  p->jit_loss.push_back({-2, 0, m});
  return m;
}

// The gradient tree code of a Float32 program for an elementwise loss: the
// L2 build, or the same candidates compiled with that loss's seed (jit_grad.cpp
// emit_loss_seed), built at the loss's first gradient and kept with the
// program; null: that loss's gradients run interpreted (SRHIP_JIT_LOSSES=0,
// no dℓ/dr routine, or a different slot layout).
jit::GradModule* grad_module(srhip_program* p, int loss, double lparam) {
  if (!p->gjit) return nullptr;
  if (loss == SRHIP_LOSS_L2) return p->gjit;
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_LOSSES"); return !(e && e[0] == '0'); }();
  if (!on || loss < 0 || loss >= SRHIP_NUM_LOSSES || !jit::has_dloss_routine(loss)) return nullptr;
  uint64_t bits;
  std::memcpy(&bits, &lparam, 8);
  for (const auto& l : p->gjit_loss)
    if (l.kind == loss && l.bits == bits) return l.m;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->gjit_consts.data();
  CompiledBatch<float> cb = compile_batch_par<float>(tr, /*grad=*/true);
  std::vector<int32_t> gjl, rest;
  jit::GradStats st;
  jit::GradModule* m = jit::build_grad(cb, p->const_off, p->h_gcand, gjl, rest, &st, loss, bits);
  if (m && gjl != p->h_gjl) {
    jit::destroy_grad(m);
    m = nullptr;
  }
  p->gjit_loss.push_back({loss, bits, m});
  return m;
}

// The same for a Float64 program (jit64.cpp GradGen64): the L2 build, or the
// same candidates compiled with that loss's seed; null: interpreted.
jit::GradModule64* grad_module64(srhip_program* p, int loss, double lparam) {
  if (!p->gjit64) return nullptr;
  if (loss == SRHIP_LOSS_L2) return p->gjit64;
  static const bool on = [] { const char* e = std::getenv("SRHIP_JIT_LOSSES"); return !(e && e[0] == '0'); }();
  if (!on || loss < 0 || loss >= SRHIP_NUM_LOSSES || !jit::has_dloss_routine64(loss)) return nullptr;
  uint64_t bits;
  std::memcpy(&bits, &lparam, 8);
  for (const auto& l : p->gjit64_loss)
    if (l.kind == loss && l.bits == bits) return l.m;
  srhip_trees tr;
  tr.ntrees = p->ntrees;
  tr.node_off = p->node_off.data();
  tr.kind = p->kind.data();
  tr.arg = p->arg.data();
  tr.const_off = p->const_off.data();
  tr.consts = p->gjit_consts.data();
  CompiledBatch<double> cb = compile_batch_par<double>(tr, /*grad=*/true);
  std::vector<int32_t> gjl, rest;
  jit::GradStats st;
  jit::GradModule64* m = jit::build_grad64(cb, p->const_off, p->h_gcand, gjl, rest, &st, loss, bits);
  if (m && gjl != p->h_gjl) {
    jit::destroy_grad64(m);
    m = nullptr;
  }
  p->gjit64_loss.push_back({loss, bits, m});
  return m;
}

// The shared subtrees of a tree-code module (jit.h Columns), once per row of
// the call, into c->gderived ([ngcol][n_pad]): the subtrees are a program of
// their own (p->shared, interpreted, no tree code) run in the interpreter's
// per-row output mode — the interpreter's values, which the tree code's
// PRECISE routines equal bit for bit — and its finalize gives each subtree's
// did_succeed over the call's rows; a subtree that failed (some node
// non-finite on some row) has its whole column set to NaN, so every tree
// that reads it fails, as DynamicExpressions fails a tree with a non-finite
// node on any row (src/InterfaceDynamicExpressions.jl:17-48).
// slot / keys: the program's cache of the subtree program (p->shared for the
// loss tree code, p->gshared for the gradient tree code).
bool derive_jit_enabled() {
  static const bool on = [] { const char* e = std::getenv("SRHIP_DERIVE_JIT"); return !(e && e[0] == '0'); }();
  return on;
}
void derive_shared(srhip_ctx* c, srhip_program*& slot, std::vector<std::string>& keys, const jit::Columns& jc,
                   const float* X, int64_t rows, int64_t n_pad, int nfeat) {
  hipStream_t s = c->stream;
  if (!slot || keys != jc.gkey) {
    if (slot) {
      free_program_device(slot);
      delete slot;
      slot = nullptr;
    }
    auto* q = new srhip_program();
    q->ctx = c;
    q->dtype = SRHIP_F32;
    q->ntrees = jc.ngcol;
    // per-row output tree code for the subtrees (SRHIP_DERIVE_JIT=0: the interpreter's MODE_OUT)
    q->jit_allowed = derive_jit_enabled();
    q->jit_forced = true;
    q->node_off.assign(jc.goff.begin(), jc.goff.end());
    q->const_off.assign((size_t)jc.ngcol + 1, 0);
    q->kind = jc.gkind;
    q->arg = jc.garg;
    q->consts.resize(1);
    try {
      build_program_f32(q);
    } catch (...) {
      free_program_device(q);
      delete q;
      throw;
    }
    slot = q;
    keys = jc.gkey;
  }
  const srhip_program* q = slot;
  const int ng = jc.ngcol;
  c->gderived.ensure((size_t)ng * (size_t)n_pad * sizeof(float));
  c->gsum.ensure((size_t)ng * sizeof(double));
  c->gok.ensure((size_t)ng);
  float* out = static_cast<float*>(c->gderived.p);
  if (q->nlist_a + q->nlist_b != ng) throw Error(SRHIP_ERR_INVALID, "shared subtree failed statically");
  // every subtree as per-row output tree code (jit_template.hip sr_jit_out_d, PRECISE routines:
  // the interpreter's values bit for bit, test_jit_out_gpu.py): one launch per code object part
  jit::Module* om = (q->jit && q->nlist_j == ng && rows > 0) ? out_module(q) : nullptr;
  if (om && !jit::module_bails(om)) {
    const jit::Columns& jc2 = jit::columns(om);
    if (jc2.nraw > nfeat) throw Error(SRHIP_ERR_INVALID, "dataset has fewer features than the subtrees read");
    const int narr = 1 + jc2.nraw + jc2.nder;
    const int jw = jc2.waves;
    const size_t lds_wg = jit::lds_per_workgroup(jw);
    const size_t budget = std::max(jit_tile_budget() * jw / 4,
                                   lds_wg - (jit::part_global() ? 0 : std::min<size_t>(lds_wg / 4, 8192)));
    for (int k = 0; k < jit::nparts(om); ++k) {
      int s0, nsl;
      jit::part(om, k, &s0, &nsl);
      if (nsl == 0) continue;
      EvalPlan plan;
      if (!plan_geometry(4, 4, kShallowSlots, narr, 1, rows, nsl, &plan, budget, 52 * 1024 * jw / 4,
                         16384 * 4 / jw, 64 * jw / 4))
        throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(nfeat) + " features does not fit in LDS");
      plan.threads = 64 * jw;
      tail_split(c, &plan, rows, jw);
      EvalArgs<float> a;
      a.prog = static_cast<const Ins<float>*>(q->d_code);
      a.tree_off = q->d_tree_off;
      a.list = q->d_list + s0;
      a.list_off = q->d_list + (q->nlist_a + q->nlist_b) + s0;
      a.fail = nullptr;
      a.ti_rec = nullptr;
      a.nlist = nsl;
      a.X = X;
      a.y = nullptr;
      a.w = nullptr;
      a.n = rows;
      a.n_pad = n_pad;
      a.nfeat = nfeat;
      a.ntiles = plan.ntiles;
      a.ntg = plan.ntg;
      a.tpb = plan.tpb;
      a.nrg = plan.nrg;
      a.loss = SRHIP_LOSS_L2;
      a.rotate = rg_xcd() ? rotate_mode() : (rotate_enabled() ? 1 : 0);
      a.contig = 0;
      a.lparam = 0.0;
      c->gpartial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<float>));
      a.partial = static_cast<Part<float>*>(c->gpartial.p);
      a.out = out;
      a.out_stride = n_pad;
      HIP_CHECK(jit::launch(om, k, plan, a, false, nullptr, s, nullptr));
      HIP_CHECK(launch_finalize<float>(a, static_cast<double*>(c->gsum.p), static_cast<uint8_t*>(c->gok.p), s));
    }
    HIP_CHECK(launch_poison_columns(static_cast<const uint8_t*>(c->gok.p), ng, out, n_pad, s));
    return;
  }
  const int lists[2][2] = {{0, q->nlist_a}, {q->nlist_a, q->nlist_b}};
  for (int pass = 0; pass < 2; ++pass) {
    const int s0 = lists[pass][0], nlist = lists[pass][1];
    if (nlist == 0) continue;
    EvalPlan plan;
    if (!plan_eval(SRHIP_F32, pass == 1, q->opset, MODE_OUT, false, nfeat, rows, nlist, &plan))
      throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(nfeat) + " features does not fit in LDS");
    if (plan.tile % 256 != 0)  // the tree code reads whole 256-row tiles of the columns
      throw Error(SRHIP_ERR_INVALID, "shared-subtree derive pass: tile of " + std::to_string(plan.tile) + " rows");
    EvalArgs<float> a;
    a.prog = static_cast<const Ins<float>*>(q->d_code);
    a.tree_off = q->d_tree_off;
    a.list = q->d_list + s0;
    a.list_off = q->d_list + (q->nlist_a + q->nlist_b) + s0;
    a.fail = nullptr;
    a.ti_rec = nullptr;
    if (ti_enabled() && pass == 0) {
      c->gti.ensure((size_t)nlist * 64 * sizeof(uint4));
      HIP_CHECK(launch_ti_records(a.prog, a.list_off, nlist, (uint32_t)(plan.ntiles * plan.tile * sizeof(float)),
                                  static_cast<uint4*>(c->gti.p), s));
      a.ti_rec = static_cast<const uint4*>(c->gti.p);
    }
    a.nlist = nlist;
    a.X = X;
    a.y = nullptr;
    a.w = nullptr;
    a.n = rows;
    a.n_pad = n_pad;
    a.nfeat = nfeat;
    a.ntiles = plan.ntiles;
    a.ntg = plan.ntg;
    a.tpb = plan.tpb;
    a.nrg = plan.nrg;
    a.loss = SRHIP_LOSS_L2;
    a.rotate = interp_dyn() ? 4 : 0;
    a.contig = 0;
    a.lparam = 0.0;
    c->gpartial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<float>));
    a.partial = static_cast<Part<float>*>(c->gpartial.p);
    a.out = out;
    a.out_stride = n_pad;
    HIP_CHECK(launch_eval<float>(plan, a, MODE_OUT, s));
    HIP_CHECK(launch_finalize<float>(a, static_cast<double*>(c->gsum.p), static_cast<uint8_t*>(c->gok.p), s));
  }
  HIP_CHECK(launch_poison_columns(static_cast<const uint8_t*>(c->gok.p), ng, out, n_pad, s));
}

// Run the evaluation kernels for both tree lists. The view (X, y, w, rows,
// n_pad) may be the dataset itself or a gathered row subset.
template <typename T>
void run_eval(srhip_ctx* c, const srhip_program* p, int mode, const T* X, const T* y,
              const T* w, int64_t rows, int64_t n_pad, int nfeat, int loss, double lparam,
              T* out, int64_t out_stride, int64_t seg = 0) {
  hipStream_t s = c->stream;
  timing_reset(c);
  c->sums.ensure(std::max<size_t>(p->ntrees, 1) * sizeof(double));
  c->oks.ensure(std::max<size_t>(p->ntrees, 1));
  // the finalize writes the per-tree results straight into the pinned host
  // buffers (no copy launches; SRHIP_ZERO_COPY=0: device buffers + copies)
  c->res_host = zero_copy_enabled() && !c->want_device_results;
  if (c->res_host) {
    ensure_pinned(c, std::max<size_t>(p->ntrees, 1));
    c->res_sum = c->pin_sum;
    c->res_ok = c->pin_ok;
  } else {
    c->res_sum = static_cast<double*>(c->sums.p);
    c->res_ok = static_cast<uint8_t*>(c->oks.p);
  }
  const size_t nslots = (size_t)p->nlist_a + p->nlist_b;
  // slot ranges: [0, nj) tree code, [nj, nlist_a) shallow interpreter, then deep
  // (per-tree row sets, seg > 0: the interpreter, one tree per workgroup)
  jit::Module* jm = (!std::is_same<T, float>::value || seg > 0) ? nullptr
                    : mode == MODE_LOSS                          ? loss_module(p, loss, lparam)
                                                                 : out_module(p);
  // Float64 programs: their tree code (this loss, or per-row outputs)
  jit::Module64* jm64 = nullptr;
  if constexpr (std::is_same<T, double>::value)
    if (p->jit64 && p->nlist_j > 0 && seg == 0) jm64 = module64(p, mode == MODE_LOSS ? loss : -2, lparam);
  const bool use_jit = jm != nullptr || jm64 != nullptr;
  c->last_jit_trees = (use_jit && rows > 0) ? p->nlist_j : 0;
  const int nj = use_jit ? p->nlist_j : 0;
  // failure flags (and the tree code's bail flags): the finalize kernels of
  // the previous call left them clean; one clearing launch only after a new
  // buffer, an interrupted call or a path that leaves them set (gradients,
  // tree code that can hand tiles back)
  const bool jit_bail = jm != nullptr && jit::module_bails(jm);
  if (mode == MODE_LOSS) {
    const size_t need = std::max<size_t>(nslots, 1) * sizeof(uint32_t);
    if (c->fail.bytes < need) {
      c->fail.ensure(need);
      c->fail_clean = false;
    }
    if (!c->fail_clean || jit_bail)
      HIP_CHECK(launch_zero_words(static_cast<uint32_t*>(c->fail.p), (int64_t)(c->fail.bytes / sizeof(uint32_t)),
                                  jit_bail ? jit::bail_flags(jm) : nullptr, jit_bail ? jit::flag_words(jm) : 0,
                                  s));
    c->fail_clean = false;  // until every finalize of this call is enqueued
  }
  // launches: the tree-code parts (pass -1, one per code object), the shallow
  // interpreter (0), the deep interpreter (1)
  struct Launch { int pass, s0, nlist, part; };
  std::vector<Launch> launches;
  if (nj > 0) {
    if constexpr (std::is_same<T, float>::value) {
      for (int k = 0; k < jit::nparts(jm); ++k) {
        int s0, nsl;
        jit::part(jm, k, &s0, &nsl);
        launches.push_back({-1, s0, nsl, k});
      }
    } else {
      for (int k = 0; k < jit::nparts64(jm64); ++k) {
        int s0, nsl;
        jit::part64(jm64, k, &s0, &nsl);
        launches.push_back({-1, s0, nsl, k});
      }
    }
  }
  launches.push_back({0, nj, p->nlist_a - nj, -1});
  launches.push_back({1, p->nlist_a, p->nlist_b, -1});
  for (size_t li = 0; li < launches.size(); ++li) {
    const int pass = launches[li].pass;
    const int s0 = launches[li].s0;
    const int nlist = launches[li].nlist;
    const bool last_jit = pass == -1 && (li + 1 == launches.size() || launches[li + 1].pass != -1);
    // no rows (an empty row shard): nothing to launch; every tree's result is
    // its static verdict (finish_results, pack_partials_kernel)
    if (rows == 0) continue;
    if (nlist == 0) {
      if (last_jit) throw Error(SRHIP_ERR_INVALID, "empty tree-code part");
      continue;
    }
    EvalPlan plan;
    if (pass == -1 && jm64) {
      // Float64 tree code: 128-row tiles of y, the features it reads, w; 4 waves
      const int narr = 1 + jit::nraw64(jm64) + (w ? 1 : 0);
      if (jit::nraw64(jm64) > nfeat) throw Error(SRHIP_ERR_INVALID, "dataset has fewer features than the program reads");
      if (!plan_geometry(8, 2, kShallowSlots, narr, 1, rows, nlist, &plan, 52 * 1024, 52 * 1024, 16384, 64))
        throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(nfeat) + " features does not fit in LDS");
      plan.threads = 256;
    } else if (pass == -1) {
      // LDS columns: y, the raw features the tree code reads, its derived columns, w
      const jit::Columns& jc = jit::columns(jm);
      if (jc.nraw > nfeat) throw Error(SRHIP_ERR_INVALID, "dataset has fewer features than the program reads");
      const int narr = 1 + jc.nraw + jc.nder + (w ? 1 : 0);
      // partials go to global memory: LDS holds the tiles (1 byte per slot keeps the slot bound away)
      // 16384 workgroups of 4 waves, >= 64 trees per group (16 per wave): config #2 kernel
      // 2.997 -> 2.867 ms at 4096 trees, 0.865 -> 0.828 at 1024, 512 unchanged
      // (profiles/r02n_targetwg.txt); scaled by the waves per workgroup
      const int jw = jc.waves;
      const size_t lds_wg = jit::lds_per_workgroup(jw);
      const size_t budget = std::max(jit_tile_budget() * jw / 4,
                                     lds_wg - (jit::part_global() ? 0 : std::min<size_t>(lds_wg / 4, 8192)));
      if (!plan_geometry(4, 4, kShallowSlots, narr, 1, rows, nlist, &plan, budget, 52 * 1024 * jw / 4,
                         16384 * 4 / jw, 64 * jw / 4))
        throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(nfeat) + " features does not fit in LDS");
      plan.threads = 64 * jw;
      tail_split(c, &plan, rows, jw);
    } else if (!plan_eval(p->dtype, pass == 1, p->opset, mode, w != nullptr, nfeat, rows, nlist, &plan)) {
      throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(nfeat) + " features does not fit in LDS");
    }
    if (seg > 0) {
      // per-tree row sets: one tree per workgroup of one wave, staging its
      // own segment (eval_kernel.h seg0); the segment holds the row groups
      plan.tpb = 1;
      plan.ntg = nlist;
      plan.threads = 64;
      if ((int64_t)plan.nrg * plan.rows_wg > seg) throw Error(SRHIP_ERR_INVALID, "row set segment too short");
    }
    EvalArgs<T> a;
    a.prog = static_cast<const Ins<T>*>(p->d_code);
    a.tree_off = p->d_tree_off;
    a.list = p->d_list + s0;
    a.list_off = p->d_list + (p->nlist_a + p->nlist_b) + s0;
    a.fail = mode == MODE_LOSS ? static_cast<uint32_t*>(c->fail.p) + s0 : nullptr;
    a.ti_rec = nullptr;
    if (ti_enabled() && std::is_same<T, float>::value && pass == 0) {
      c->ti_rec.ensure((size_t)nlist * 64 * sizeof(uint4));
      HIP_CHECK(launch_ti_records(reinterpret_cast<const Ins<float>*>(a.prog), a.list_off, nlist,
                                  (uint32_t)(plan.ntiles * plan.tile * sizeof(T)),
                                  static_cast<uint4*>(c->ti_rec.p), s));
      a.ti_rec = static_cast<const uint4*>(c->ti_rec.p);
    }
    a.nlist = nlist;
    a.X = X;
    a.y = y;
    a.w = w;
    a.n = rows;
    a.n_pad = n_pad;
    a.nfeat = nfeat;
    a.ntiles = plan.ntiles;
    a.ntg = plan.ntg;
    a.tpb = plan.tpb;
    a.nrg = plan.nrg;
    a.loss = loss;
    a.rotate = rotate_enabled() ? 1 : 0;
    a.contig = (pass == -1 && jm && jit_contig()) ? 1 : 0;
    if (pass == -1 && jm && rg_xcd()) a.rotate = rotate_mode();  // tree code: row groups per XCD
    if (pass >= 0 && interp_dyn()) a.rotate |= 4;  // interpreter: trees from an LDS counter
    a.lparam = lparam;
    c->partial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<T>));
    a.partial = static_cast<Part<T>*>(c->partial.p);
    a.out = out;
    a.out_stride = out_stride;
    a.seg = seg;
    const int tk = timed_begin(c, s);
    if (pass == -1) {
      if constexpr (std::is_same<T, float>::value) {
        // the derived columns of this call, once per row, before the first part
        const jit::Columns& jc = jit::columns(jm);
        static const bool precompute = [] { const char* e = std::getenv("SRHIP_JIT_DERIVE_PRE"); return !(e && e[0] == '0'); }();
        const float* dcols = nullptr;
        if (jc.nder > 0 && precompute) {
          c->derived.ensure((size_t)jc.nder * (size_t)n_pad * sizeof(float));
          if (launches[li].part == 0) HIP_CHECK(jit::launch_derive(jm, X, n_pad, static_cast<float*>(c->derived.p), s));
          dcols = static_cast<const float*>(c->derived.p);
        }
        // the shared subtrees of this call, once per row, before the first part
        // (inside the timed region: their cost is the call's)
        const float* gcols = nullptr;
        if (jc.ngcol > 0) {
          if (launches[li].part == 0) derive_shared(c, p->shared, p->shared_keys, jc, X, rows, n_pad, nfeat);
          gcols = static_cast<const float*>(c->gderived.p);
        }
        HIP_CHECK(jit::launch(jm, launches[li].part, plan, a, jit_fast_enabled(), dcols, s, gcols));
      } else {
        HIP_CHECK(jit::launch64(jm64, launches[li].part, plan, a, s));
      }
    } else {
      // the interpreter's pass after a tree-code pass runs the few trees left
      // over: the call's main kernel stays the tree code
      if (nj == 0) note_kernel(sizeof(T) == 4 ? "eval_kernel<float>" : "eval_kernel<double>");
      HIP_CHECK(launch_eval<T>(plan, a, mode, s));
    }
    timed_end(c, s, tk);
    // the last tree-code part's finalize hands over and clears the tree code's counters
    uint32_t* cnt = (last_jit && jm && !jit_bail) ? jit::bail_flags(jm) + nj : nullptr;
    EvalArgs<T> af = a;  // the hand-written tree loops write 4-byte partials
    if constexpr (std::is_same<T, float>::value) af.part4 = (pass == -1 && jit::partials4(jm, launches[li].part)) ? 1 : 0;
    HIP_CHECK(launch_finalize<T>(af, c->res_sum, c->res_ok, s, cnt, cnt ? c->pin_cnt : nullptr));
    if (cnt) c->cnt_pending = true;
    static const bool dbg = std::getenv("SRHIP_DEBUG_PASSES") != nullptr;
    if (dbg) {  // debugging only: wait for the launch to report its time
      HIP_CHECK(hipStreamSynchronize(s));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, c->tev[2 * (size_t)tk], c->tev[2 * (size_t)tk + 1]));
      std::fprintf(stderr, "srhip pass %s: %d trees, %.3f ms (grid %d x %d, %d tiles/wg)\n",
                   pass == -1 ? "tree-code" : pass == 0 ? "shallow" : "deep", nlist, ms, plan.nrg, plan.ntg,
                   plan.ntiles);
    }
    if (last_jit) rerun_bailed<T>(c, p, jm, a, plan, nfeat, rows, loss, lparam);
  }
  if (mode == MODE_LOSS) c->fail_clean = true;
}

// Copy per-tree results to the caller, applying the static verdicts.
void ensure_pinned(srhip_ctx* c, size_t nt) {
  if (nt <= c->pin_cap) return;
  if (c->pin_sum) (void)hipHostFree(c->pin_sum);
  if (c->pin_ok) (void)hipHostFree(c->pin_ok);
  c->pin_sum = nullptr;
  c->pin_ok = nullptr;
  c->pin_cap = 0;
  // coherent: the finalize kernel may write them directly (zero copy)
  HIP_CHECK(hipHostMalloc((void**)&c->pin_sum, nt * sizeof(double), hipHostMallocCoherent));
  HIP_CHECK(hipHostMalloc((void**)&c->pin_ok, nt, hipHostMallocCoherent));
  c->pin_cap = nt;
}

// the per-tree results to pinned host memory (asynchronous; nothing to copy
// when the finalize wrote them there)
bool enqueue_result_copies(srhip_ctx* c, const srhip_program* p, int64_t rows) {
  const int nt = p->ntrees;
  if (!(rows > 0 && nt > 0 && (p->nlist_a + p->nlist_b) > 0)) return false;
  if (c->res_host) return true;
  HIP_CHECK(hipMemcpyAsync(c->pin_sum, c->sums.p, nt * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(hipMemcpyAsync(c->pin_ok, c->oks.p, nt, hipMemcpyDeviceToHost, c->stream));
  return true;
}

// wait for the call, then the per-tree results with the static verdicts applied
void finish_results(srhip_ctx* c, const srhip_program* p, int64_t rows, bool copied, double* out_sum,
                    uint8_t* out_ok) {
  wait_stream(c->stream);
  timing_finish(c);
  const int nt = p->ntrees;
  for (int t = 0; t < nt; ++t) {
    bool ok;
    double sm;
    if (p->static_fail[t]) { ok = false; sm = NAN; }
    else if (p->fail_if_rows[t]) { ok = rows == 0; sm = rows == 0 ? 0.0 : NAN; }
    else if (rows == 0 || !copied) { ok = true; sm = 0.0; }
    else { ok = c->pin_ok[t] != 0; sm = c->pin_sum[t]; }
    if (out_sum) out_sum[t] = sm;
    if (out_ok) out_ok[t] = ok ? 1 : 0;
  }
}

// Copy per-tree results to the caller, applying the static verdicts.
void collect_results(srhip_ctx* c, const srhip_program* p, int64_t rows, double* out_sum,
                     uint8_t* out_ok) {
  ensure_pinned(c, std::max(p->ntrees, 1));
  const bool copied = enqueue_result_copies(c, p, rows);
  finish_results(c, p, rows, copied, out_sum, out_ok);
}

template <typename T>
int eval_loss_impl(srhip_dataset* ds, const srhip_program* p, int loss, const double* params,
                   const int64_t* row_idx, int64_t nidx, double* out_sum, double* out_wsum,
                   uint8_t* out_ok) {
  srhip_ctx* c = p->ctx;  // the program's context runs the call (stream, workspace, results)
  const T* X = static_cast<const T*>(ds->X);
  const T* y = static_cast<const T*>(ds->y);
  const T* w = static_cast<const T*>(ds->w);
  int64_t rows = ds->rows, n_pad = ds->n_pad;
  double wsum = ds->w ? ds->sum_w : (double)ds->rows;
  if (row_idx) {
    if (nidx < 0) throw Error(SRHIP_ERR_INVALID, "negative index count");
    for (int64_t k = 0; k < nidx; ++k)
      if (row_idx[k] < 0 || row_idx[k] >= ds->rows) throw Error(SRHIP_ERR_INVALID, "row index out of range");
    const int64_t gp = pad_rows(nidx);
    const size_t es = sizeof(T);
    c->scratch_idx.ensure(std::max<int64_t>(nidx, 1) * sizeof(int64_t));
    c->gather.ensure((size_t)gp * (ds->nfeat + 2) * es);
    T* Xg = static_cast<T*>(c->gather.p);
    T* yg = Xg + (size_t)gp * ds->nfeat;
    T* wg = yg + gp;
    if (nidx > 0) {
      HIP_CHECK(hipMemcpyAsync(c->scratch_idx.p, row_idx, nidx * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
      HIP_CHECK(launch_gather_rows<T>(X, y, w, ds->nfeat, ds->n_pad,
                                      static_cast<const int64_t*>(c->scratch_idx.p), nidx, 0, gp, Xg,
                                      yg, w ? wg : nullptr, c->stream));
    }
    if (w) {  // Σ w over the (repeated) sample
      wsum = 0.0;
      for (int64_t k = 0; k < nidx; ++k) wsum += ds->h_w[row_idx[k]];
    } else {
      wsum = (double)nidx;
    }
    X = Xg;
    y = yg;
    w = w ? wg : nullptr;
    rows = nidx;
    n_pad = gp;
  }
  run_eval<T>(c, p, MODE_LOSS, X, y, w, rows, n_pad, ds->nfeat, loss, params ? params[0] : 0.0, nullptr, 0);
  collect_results(c, p, rows, out_sum, out_ok);
  if (out_wsum) *out_wsum = wsum;
  return SRHIP_OK;
}

// score_func_batch for every tree of the program on its OWN row sample
// (src/LossFunctions.jl:95-115 draws `batch_size` rows with replacement per
// call): the samples are gathered into one segment per tree — seg rows,
// row set t in [t·seg, t·seg + bs), padded with its last row — and the
// interpreter runs one tree per workgroup over its segment (run_eval seg).
// One gather, one evaluation launch and one finalize for all trees.
template <typename T>
int eval_loss_rowsets_impl(srhip_dataset* ds, const srhip_program* p, int loss, const double* params,
                           const int64_t* row_idx, int64_t bs, double* out_sum, double* out_wsum,
                           uint8_t* out_ok) {
  srhip_ctx* c = p->ctx;
  const int nt = p->ntrees;
  if (bs < 0) throw Error(SRHIP_ERR_INVALID, "negative batch size");
  if (bs > 0 && nt > 0 && !row_idx) throw Error(SRHIP_ERR_INVALID, "row_idx is NULL");
  const int64_t nidx = (int64_t)nt * bs;
  for (int64_t k = 0; k < nidx; ++k)
    if (row_idx[k] < 0 || row_idx[k] >= ds->rows) throw Error(SRHIP_ERR_INVALID, "row index out of range");
  // segment: a power of two >= the row group of any interpreter variant
  // (rows_wg = tiles · 64R is a power of two < 2·bs, or one 512-row tile)
  int64_t seg = 512;
  while (seg < bs && seg < kRowPad) seg *= 2;
  if (seg < bs) seg = pad_rows(bs);
  const T* w = static_cast<const T*>(ds->w);
  const int64_t gp = seg * std::max(nt, 1);
  const size_t es = sizeof(T);
  c->scratch_idx.ensure((size_t)std::max<int64_t>(nidx, 1) * sizeof(int64_t));
  c->gather.ensure((size_t)gp * (ds->nfeat + 2) * es);
  T* Xg = static_cast<T*>(c->gather.p);
  T* yg = Xg + (size_t)gp * ds->nfeat;
  T* wg = yg + gp;
  if (nidx > 0) {
    HIP_CHECK(hipMemcpyAsync(c->scratch_idx.p, row_idx, nidx * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(launch_gather_rows<T>(static_cast<const T*>(ds->X), static_cast<const T*>(ds->y), w, ds->nfeat,
                                    ds->n_pad, static_cast<const int64_t*>(c->scratch_idx.p), bs, seg, gp, Xg, yg,
                                    w ? wg : nullptr, c->stream));
  }
  run_eval<T>(c, p, MODE_LOSS, Xg, yg, w ? wg : nullptr, bs, gp, ds->nfeat, loss, params ? params[0] : 0.0, nullptr,
              0, seg);
  collect_results(c, p, bs, out_sum, out_ok);  // (the copy of row_idx is ordered before these waits)
  if (out_wsum)
    for (int t = 0; t < nt; ++t) {  // Σ w over tree t's (repeated) sample
      double s = 0.0;
      if (w)
        for (int64_t k = 0; k < bs; ++k) s += ds->h_w[row_idx[(size_t)t * bs + k]];
      else
        s = (double)bs;
      out_wsum[t] = s;
    }
  return SRHIP_OK;
}

template <typename T>
int eval_loss_packed_impl(srhip_dataset* ds, srhip_program* p, int loss, const double* params, double* d_out) {
  srhip_ctx* c = p->ctx;
  const int nt = p->ntrees;
  const double wsum = ds->w ? ds->sum_w : (double)ds->rows;
  c->want_device_results = true;
  try {
    run_eval<T>(c, p, MODE_LOSS, static_cast<const T*>(ds->X), static_cast<const T*>(ds->y),
                static_cast<const T*>(ds->w), ds->rows, ds->n_pad, ds->nfeat, loss, params ? params[0] : 0.0, nullptr, 0);
  } catch (...) {
    c->want_device_results = false;
    throw;
  }
  c->want_device_results = false;
  if (p->verdict_stale || !p->d_verdict) {
    std::vector<uint8_t> v((size_t)std::max(nt, 1), 0);
    for (int t = 0; t < nt; ++t) v[t] = p->static_fail[t] ? 1 : p->fail_if_rows[t] ? 2 : 0;
    if (!p->d_verdict) HIP_CHECK(hipMalloc((void**)&p->d_verdict, v.size()));
    HIP_CHECK(hipMemcpyAsync(p->d_verdict, v.data(), v.size(), hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));  // v leaves scope
    p->verdict_stale = false;
  }
  c->sums.ensure(std::max<size_t>(nt, 1) * sizeof(double));
  c->oks.ensure(std::max<size_t>(nt, 1));
  HIP_CHECK(launch_pack_partials(static_cast<const double*>(c->sums.p), static_cast<const uint8_t*>(c->oks.p),
                                 p->d_verdict, nt, ds->rows, wsum, d_out, c->stream));
  return SRHIP_OK;  // timing_finish once the stream is synchronised (srhip_sync / srhip_last_kernel_time)
}

// Device rows (pitch bytes apart) to the caller's contiguous host rows,
// through the pinned staging halves: the DMA of chunk i overlaps the host
// copy of chunk i-1 (spread over persistent threads). A pageable destination
// otherwise goes through the runtime's own staging, one chunk at a time
// (config #3's 0.82 GB output: 94 ms, profiles/r02j_configs.jsonl).
void copy_rows_to_host(srhip_ctx* c, unsigned char* dst, const unsigned char* src, size_t pitch, size_t row_bytes,
                       int64_t nrows) {
  hipStream_t s = c->stream;
  const int64_t k = std::max<int64_t>(1, (int64_t)((48u << 20) / row_bytes));  // rows per chunk
  const size_t half = (size_t)k * row_bytes;
  if (c->stage_cap < 2 * half) {
    if (c->pin_stage) (void)hipHostFree(c->pin_stage);
    c->pin_stage = nullptr;
    c->stage_cap = 0;
    HIP_CHECK(hipHostMalloc((void**)&c->pin_stage, 2 * half, hipHostMallocDefault));
    c->stage_cap = 2 * half;
  }
  const int64_t nch = (nrows + k - 1) / k;
  while ((int64_t)c->stage_evs.size() < nch) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->stage_evs.push_back(e);
  }
  // host copy threads: SRHIP_COPY_THREADS, default 16 (the CPU share of one
  // GPU on the target hosts; first-touch page faults of the caller's fresh
  // buffer are most of the cost: 0.82 GB in 43 ms on 16 threads, 63 ms on 8,
  // profiles/r03_hostcopy.txt)
  static const unsigned nthr = [] {
    const char* e = std::getenv("SRHIP_COPY_THREADS");
    const unsigned want = e ? (unsigned)std::max(1, std::atoi(e)) : 16u;
    return std::max(1u, std::min(want, std::max(1u, std::thread::hardware_concurrency())));
  }();
  if (!c->copy_pool) c->copy_pool.reset(new CopyPool());
  c->copy_pool->start(nthr, c->device);
  // workers copy their stripe of each chunk once its DMA has landed; the DMA of
  // chunk i reuses the half of chunk i-2 after every worker is done with it
  std::atomic<int64_t> recorded{-1};
  std::atomic<bool> failed{false};
  std::unique_ptr<std::atomic<unsigned>[]> done(new std::atomic<unsigned>[(size_t)nch]);
  for (int64_t i = 0; i < nch; ++i) done[i].store(0);
  c->copy_pool->submit([&](unsigned j, bool dev_ok) {
    if (!dev_ok) failed = true;
    for (int64_t i = 0; i < nch; ++i) {
      while (recorded.load(std::memory_order_acquire) < i) {
        if (failed.load()) return;
        std::this_thread::yield();
      }
      if (failed.load() || hipEventSynchronize(c->stage_evs[i]) != hipSuccess) { failed = true; return; }
      const int64_t r0 = i * k, nr = std::min(k, nrows - r0);
      const size_t n = (size_t)nr * row_bytes;
      const size_t per = ((n + nthr - 1) / nthr + 63) / 64 * 64;
      const size_t b0 = std::min(n, (size_t)j * per), e0 = std::min(n, b0 + per);
      if (b0 < e0) std::memcpy(dst + (size_t)r0 * row_bytes + b0, c->pin_stage + (size_t)(i & 1) * half + b0, e0 - b0);
      done[i].fetch_add(1, std::memory_order_release);
    }
  });
  try {
    for (int64_t i = 0; i < nch; ++i) {
      if (i >= 2)
        while (done[i - 2].load(std::memory_order_acquire) < nthr) {
          if (failed.load()) throw Error(SRHIP_ERR_DEVICE, "host copy of the per-row outputs failed");
          std::this_thread::yield();
        }
      const int64_t r0 = i * k, nr = std::min(k, nrows - r0);
      HIP_CHECK(hipMemcpy2DAsync(c->pin_stage + (size_t)(i & 1) * half, row_bytes, src + (size_t)r0 * pitch, pitch,
                                 row_bytes, (size_t)nr, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipEventRecord(c->stage_evs[i], s));
      recorded.store(i, std::memory_order_release);
    }
  } catch (...) {
    failed = true;
    c->copy_pool->wait();
    throw;
  }
  c->copy_pool->wait();
  if (failed.load()) throw Error(SRHIP_ERR_DEVICE, "host copy of the per-row outputs failed");
}

template <typename T>
int eval_tree_array_impl(srhip_dataset* ds, const srhip_program* p, void* out, uint8_t* out_ok) {
  srhip_ctx* c = p->ctx;
  const int nt = p->ntrees;
  const int64_t rows = ds->rows, n_pad = ds->n_pad;
  const size_t es = sizeof(T);
  c->gather.ensure(std::max<size_t>((size_t)nt * n_pad * es, es));
  T* d_out = static_cast<T*>(c->gather.p);
  run_eval<T>(c, p, MODE_OUT, static_cast<const T*>(ds->X), nullptr, nullptr, rows, n_pad,
              ds->nfeat, SRHIP_LOSS_L2, 0.0, d_out, n_pad);
  if (out && rows > 0 && nt > 0) {
    if ((size_t)rows * es * nt < (32u << 20))
      HIP_CHECK(hipMemcpy2DAsync(out, rows * es, d_out, n_pad * es, rows * es, nt, hipMemcpyDeviceToHost, c->stream));
    else
      copy_rows_to_host(c, static_cast<unsigned char*>(out), reinterpret_cast<const unsigned char*>(d_out),
                        (size_t)n_pad * es, (size_t)rows * es, nt);
  }
  collect_results(c, p, rows, nullptr, out_ok);
  if (out) {  // rows of trees that were never run: NaN (reference: undefined)
    T* o = static_cast<T*>(out);
    for (int t = 0; t < nt; ++t)
      if (p->static_fail[t] || p->fail_if_rows[t])
        for (int64_t i = 0; i < rows; ++i) o[(size_t)t * rows + i] = (T)NAN;
  }
  return SRHIP_OK;
}

template <typename T>
void run_grad(srhip_ctx* c, srhip_program* p, int mode, const srhip_dataset* ds, int loss, double lparam,
              T* out_value, T* out_grad, int64_t out_stride) {
  build_grad_program<T>(p);
  hipStream_t s = c->stream;
  timing_reset(c);
  const int nt = p->ntrees;
  const int nconst = p->const_off.back();
  c->sums.ensure(std::max<size_t>(nt, 1) * sizeof(double));
  c->oks.ensure(std::max<size_t>(nt, 1));
  c->dloss.ensure(std::max<size_t>(nconst, 1) * sizeof(double));
  // gradient tree code (∂L/∂c of the loss) for the trees it holds; the
  // interpreter items of the other trees follow
  bool use_gjit = false;
  if constexpr (std::is_same<T, float>::value) {
    jit::GradModule* gm = (p->gjit && mode == GRAD_LOSS && ds->rows > 0) ? grad_module(p, loss, lparam) : nullptr;
    if (gm) {
      const int nparts = jit::grad_nparts(gm);
      const int narr = 1 + ds->nfeat + (ds->w ? 1 : 0);
      std::vector<EvalPlan> plans(nparts);
      use_gjit = true;
      for (int k = 0; k < nparts && use_gjit; ++k) {
        int s0, nsl;
        jit::grad_part(gm, k, &s0, &nsl);
        // partials go straight to global memory: LDS holds the row tiles only (1 byte per slot below
        // keeps plan_geometry's slot bound out of the way)
        use_gjit = plan_geometry(4, 4, kShallowSlots, narr, 1, ds->rows, nsl, &plans[k], gjit_tile_budget()) &&
                   plans[k].nrg == plans[0].nrg;
      }
      if (use_gjit) {
        const int nsl_all = jit::grad_nslots(gm);
        c->fail.ensure((size_t)nsl_all * sizeof(uint32_t));
        c->fail_clean = false;  // the gradient kernels leave their flags set
        HIP_CHECK(hipMemsetAsync(c->fail.p, 0, (size_t)nsl_all * sizeof(uint32_t), s));
        c->gpart.ensure(std::max<size_t>((size_t)plans[0].nrg * nconst, 1) * sizeof(float));
        // the shared subtrees' columns of this call (jit::grad_columns), timed with the call
        const jit::Columns& gcj = jit::grad_columns(gm);
        const float* gcols = nullptr;
        if (gcj.ngcol > 0) {
          const int tk = timed_begin(c, s);
          derive_shared(c, p->gshared, p->gshared_keys, gcj, static_cast<const float*>(ds->X), ds->rows, ds->n_pad,
                        ds->nfeat);
          timed_end(c, s, tk);
          gcols = static_cast<const float*>(c->gderived.p);
        }
        for (int k = 0; k < nparts; ++k) {
          int s0, nsl;
          jit::grad_part(gm, k, &s0, &nsl);
          const EvalPlan& plan = plans[k];
          EvalArgs<float> a;
          std::memset(&a, 0, sizeof(a));
          a.list = p->d_gjit_list + s0;
          a.fail = static_cast<uint32_t*>(c->fail.p) + s0;
          a.nlist = nsl;
          a.X = static_cast<const float*>(ds->X);
          a.y = static_cast<const float*>(ds->y);
          a.w = static_cast<const float*>(ds->w);
          a.n = ds->rows;
          a.n_pad = ds->n_pad;
          a.nfeat = ds->nfeat;
          a.ntiles = plan.ntiles;
          a.ntg = plan.ntg;
          a.tpb = plan.tpb;
          a.nrg = plan.nrg;
          a.loss = loss;
          a.contig = jit_contig() ? 1 : 0;
          a.rotate = rotate_mode();
          c->partial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<float>));
          a.partial = static_cast<Part<float>*>(c->partial.p);
          const int tk = timed_begin(c, s);
          HIP_CHECK(jit::launch_grad_code(gm, k, plan, a, p->d_gconsts, static_cast<float*>(c->gpart.p), nconst,
                                          s, gcols));
          timed_end(c, s, tk);
          HIP_CHECK(launch_finalize<float>(a, static_cast<double*>(c->sums.p), static_cast<uint8_t*>(c->oks.p), s));
          static const bool dbg = std::getenv("SRHIP_DEBUG_PASSES") != nullptr;
          if (dbg) {
            HIP_CHECK(hipStreamSynchronize(s));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, c->tev[2 * (size_t)tk], c->tev[2 * (size_t)tk + 1]));
            std::fprintf(stderr, "srhip grad tree code part %d: %d trees, %.3f ms (grid %d x %d, %d tiles/wg)\n", k,
                         nsl, ms, plan.nrg, plan.ntg, plan.ntiles);
          }
        }
        HIP_CHECK(launch_gconst_finalize(static_cast<const float*>(c->gpart.p), plans[0].nrg, nconst,
                                         p->d_gjit_cidx, p->ngjit_cidx, static_cast<double*>(c->dloss.p), s));
      }
    }
  } else if (jit::GradModule64* gm = (p->gjit64 && mode == GRAD_LOSS && ds->rows > 0) ? grad_module64(p, loss, lparam)
                                                                                      : nullptr) {
    // Float64 gradient tree code: 128-row tiles of y, the features it reads, w
    const int nparts = jit::grad64_nparts(gm);
    const int narr = 1 + jit::grad64_nraw(gm) + (ds->w ? 1 : 0);
    if (jit::grad64_nraw(gm) > ds->nfeat) throw Error(SRHIP_ERR_INVALID, "dataset has fewer features than the program reads");
    std::vector<EvalPlan> plans(nparts);
    use_gjit = true;
    for (int k = 0; k < nparts && use_gjit; ++k) {
      int s0, nsl;
      jit::grad64_part(gm, k, &s0, &nsl);
      use_gjit = plan_geometry(8, 2, kShallowSlots, narr, 1, ds->rows, nsl, &plans[k], gjit_tile_budget()) &&
                 plans[k].nrg == plans[0].nrg;
      plans[k].threads = 256;
    }
    if (use_gjit) {
      c->fail.ensure((size_t)jit::grad64_nslots(gm) * sizeof(uint32_t));
      c->fail_clean = false;
      HIP_CHECK(hipMemsetAsync(c->fail.p, 0, (size_t)jit::grad64_nslots(gm) * sizeof(uint32_t), s));
      c->gpart.ensure(std::max<size_t>((size_t)plans[0].nrg * nconst, 1) * sizeof(double));
      for (int k = 0; k < nparts; ++k) {
        int s0, nsl;
        jit::grad64_part(gm, k, &s0, &nsl);
        const EvalPlan& plan = plans[k];
        EvalArgs<double> a;
        std::memset(&a, 0, sizeof(a));
        a.list = p->d_gjit_list + s0;
        a.fail = static_cast<uint32_t*>(c->fail.p) + s0;
        a.nlist = nsl;
        a.X = static_cast<const double*>(ds->X);
        a.y = static_cast<const double*>(ds->y);
        a.w = static_cast<const double*>(ds->w);
        a.n = ds->rows;
        a.n_pad = ds->n_pad;
        a.nfeat = ds->nfeat;
        a.ntiles = plan.ntiles;
        a.ntg = plan.ntg;
        a.tpb = plan.tpb;
        a.nrg = plan.nrg;
        a.loss = loss;
        c->partial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * sizeof(Part<double>));
        a.partial = static_cast<Part<double>*>(c->partial.p);
        const int tk = timed_begin(c, s);
        HIP_CHECK(jit::launch_grad_code64(gm, k, plan, a, p->d_gconsts64, static_cast<double*>(c->gpart.p), nconst, s));
        timed_end(c, s, tk);
        HIP_CHECK(launch_finalize<double>(a, static_cast<double*>(c->sums.p), static_cast<uint8_t*>(c->oks.p), s));
      }
      // gpart is not cleared: a failed tree's row groups stop writing their partials, so its constants'
      // sums here may hold an earlier call's values; collect_grad_results (the only reader of c->dloss)
      // reports NaN for every constant of a failed tree (test_jit64_grad_gpu.py
      // test_failed_trees_gradients_are_nan_not_stale)
      HIP_CHECK(launch_gconst_finalize(static_cast<const double*>(c->gpart.p), plans[0].nrg, nconst,
                                       p->d_gjit_cidx, p->ngjit_cidx, static_cast<double*>(c->dloss.p), s));
    }
  }
  c->last_jit_trees = use_gjit ? (int)p->h_gjl.size() : 0;
  const int* ngi = use_gjit ? p->ngitems_rest : p->ngitems;
  int first = 0;
  if (use_gjit)
    for (int k = 0; k < 4; ++k) first += p->ngitems[k];
  for (int pass = 0; pass < 4; ++pass) {
    const int nitems = ngi[pass];
    const int item0 = first;
    first += nitems;
    if (nitems == 0 || ds->rows == 0) continue;
    const bool deep = pass == 3;
    const int G = pass == 0 ? 1 : pass == 1 ? 2 : kGradG;
    EvalPlan plan;
    if (!plan_grad(p->dtype, deep, G, mode, ds->w != nullptr, ds->nfeat, ds->rows, nitems, &plan))
      throw Error(SRHIP_ERR_UNSUPPORTED, "row tile of " + std::to_string(ds->nfeat) + " features does not fit in LDS");
    GradArgs<T> a;
    a.prog = static_cast<const Ins<T>*>(p->d_gcode);
    a.tree_off = p->d_gtree_off;
    a.items = p->d_gitems + item0;
    a.nitems = nitems;
    a.dyn = interp_dyn() ? 1 : 0;
    a.const_off = p->d_const_off;
    a.X = static_cast<const T*>(ds->X);
    a.y = static_cast<const T*>(ds->y);
    a.w = static_cast<const T*>(ds->w);
    a.n = ds->rows;
    a.n_pad = ds->n_pad;
    a.nfeat = ds->nfeat;
    a.ntiles = plan.ntiles;
    a.ntg = plan.ntg;
    a.tpb = plan.tpb;
    a.nrg = plan.nrg;
    a.loss = loss;
    a.lparam = lparam;
    a.G = G;
    a.opset = deep ? OPSET_FULL : p->g_opset;
    c->partial.ensure((size_t)plan.nrg * plan.ntg * plan.tpb * (2 + G) * sizeof(T));
    a.partial = static_cast<T*>(c->partial.p);
    a.out_value = out_value;
    a.out_grad = out_grad;
    a.out_stride = out_stride;
    const int tk = timed_begin(c, s);
    note_kernel(sizeof(T) == 4 ? "grad_kernel<float>" : "grad_kernel<double>");
    HIP_CHECK(launch_grad<T>(plan, a, mode, s));
    timed_end(c, s, tk);
    HIP_CHECK(launch_grad_finalize<T>(a, static_cast<double*>(c->sums.p), static_cast<uint8_t*>(c->oks.p),
                                      static_cast<double*>(c->dloss.p), s));
    static const bool dbg = std::getenv("SRHIP_DEBUG_PASSES") != nullptr;
    if (dbg) {
      HIP_CHECK(hipStreamSynchronize(s));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, c->tev[2 * (size_t)tk], c->tev[2 * (size_t)tk + 1]));
      std::fprintf(stderr, "srhip grad pass %d: %d items, G=%d, R=%d, opset %d, %.3f ms (grid %d x %d, %d tiles/wg)\n",
                   pass, nitems, G, plan.R, a.opset, ms, plan.nrg, plan.ntg, plan.ntiles);
    }
  }
}

// per-tree results of a gradient pass: static verdicts applied
void collect_grad_results(srhip_ctx* c, const srhip_program* p, int64_t rows, double* out_sum,
                          double* out_dloss, uint8_t* out_ok) {
  const int nt = p->ntrees;
  const int nconst = p->const_off.back();
  c->h_sum.assign(nt, 0.0);
  c->h_ok.assign(nt, 1);
  std::vector<double> hd(nconst, 0.0);
  if (rows > 0 && nt > 0 && (p->ngitems[0] + p->ngitems[1] + p->ngitems[2] + p->ngitems[3]) > 0) {
    HIP_CHECK(hipMemcpyAsync(c->h_sum.data(), c->sums.p, nt * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipMemcpyAsync(c->h_ok.data(), c->oks.p, nt, hipMemcpyDeviceToHost, c->stream));
    if (nconst > 0)
      HIP_CHECK(hipMemcpyAsync(hd.data(), c->dloss.p, nconst * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_CHECK(hipStreamSynchronize(c->stream));
  timing_finish(c);
  for (int t = 0; t < nt; ++t) {
    const bool fail = p->g_static_fail[t] || (rows > 0 && !c->h_ok[t]);
    if (out_ok) out_ok[t] = fail ? 0 : 1;
    if (out_sum) out_sum[t] = fail ? NAN : (rows > 0 ? c->h_sum[t] : 0.0);
    for (int k = p->const_off[t]; k < p->const_off[t + 1]; ++k)
      if (out_dloss) out_dloss[k] = fail ? NAN : (rows > 0 ? hd[k] : 0.0);
  }
}

template <typename T>
int eval_loss_grad_impl(srhip_dataset* ds, srhip_program* p, int loss, const double* params,
                        double* out_sum, double* out_dloss, double* out_wsum, uint8_t* out_ok) {
  srhip_ctx* c = p->ctx;
  run_grad<T>(c, p, GRAD_LOSS, ds, loss, params ? params[0] : 0.0, nullptr, nullptr, 0);
  if (out_wsum) *out_wsum = ds->w ? ds->sum_w : (double)ds->rows;
  const bool periodic = std::is_same<T, float>::value && loss == SRHIP_LOSS_PERIODIC && c->last_jit_trees > 0;
  if (!periodic) {
    collect_grad_results(c, p, ds->rows, out_sum, out_dloss, out_ok);
    return SRHIP_OK;
  }
  // Float32 Periodic as gradient tree code: a row beyond the Cody-Waite range made its tree fail
  // there (device_ops.h periodic_g_f32); every failed tree of the call is evaluated again in the
  // forward-mode interpreter (a program of those trees, no tree code), whose results replace the
  // tree code's — failing trees fail there too, the others get OCML's full-range sin / cos
  const int nt = p->ntrees, nconst = p->const_off.back();
  std::vector<double> sum(nt), dl(std::max(nconst, 1));
  std::vector<uint8_t> ok(nt);
  collect_grad_results(c, p, ds->rows, sum.data(), dl.data(), ok.data());
  std::vector<int32_t> redo;
  for (int t = 0; t < nt; ++t)
    if (!ok[t] && !p->g_static_fail[t]) redo.push_back(t);
  if (!redo.empty()) {
    const double ms = c->last_ms;
    const int nl = c->last_launches;
    const int ljt = c->last_jit_trees;  // the call's tree code (the rerun below reports none)
    const char* lkn = t_last_kernel;  // string literals only
    std::vector<int32_t> noff{0}, coff{0};
    std::vector<uint8_t> kind;
    std::vector<uint16_t> arg;
    std::vector<T> cs;
    const T* pc = reinterpret_cast<const T*>(p->consts.data());
    for (int32_t t : redo) {
      kind.insert(kind.end(), p->kind.begin() + p->node_off[t], p->kind.begin() + p->node_off[t + 1]);
      arg.insert(arg.end(), p->arg.begin() + p->node_off[t], p->arg.begin() + p->node_off[t + 1]);
      noff.push_back((int32_t)kind.size());
      cs.insert(cs.end(), pc + p->const_off[t], pc + p->const_off[t + 1]);
      coff.push_back((int32_t)cs.size());
    }
    // the program of those trees, built here (the caller holds the context's lock)
    auto* q = new srhip_program();
    q->ctx = c;
    q->dtype = p->dtype;
    q->ntrees = (int)redo.size();
    q->jit_allowed = false;
    q->gjit_allowed = false;
    q->node_off = noff;
    q->const_off = coff;
    q->kind = kind;
    q->arg = arg;
    q->consts.resize(std::max<size_t>(cs.size() * sizeof(T), 1));
    if (!cs.empty()) std::memcpy(q->consts.data(), cs.data(), cs.size() * sizeof(T));
    std::vector<double> s2(redo.size()), d2(std::max<size_t>(cs.size(), 1));
    std::vector<uint8_t> ok2(redo.size());
    try {
      build_program<T>(q);
      eval_loss_grad_impl<T>(ds, q, loss, params, s2.data(), d2.data(), nullptr, ok2.data());
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      free_program_device(q);
      delete q;
      throw;
    }
    HIP_CHECK(hipStreamSynchronize(c->stream));
    free_program_device(q);
    delete q;
    for (size_t i = 0; i < redo.size(); ++i) {
      const int32_t t = redo[i];
      sum[t] = s2[i];
      ok[t] = ok2[i];
      for (int32_t k = p->const_off[t]; k < p->const_off[t + 1]; ++k) dl[k] = d2[coff[i] + (k - p->const_off[t])];
    }
    c->last_ms += ms;  // the call's kernel time: both runs
    c->last_launches += nl;
    c->last_jit_trees = ljt;
    t_last_kernel = lkn;
  }
  if (out_sum) std::copy(sum.begin(), sum.end(), out_sum);
  if (out_dloss && nconst > 0) std::copy(dl.begin(), dl.begin() + nconst, out_dloss);
  if (out_ok) std::copy(ok.begin(), ok.end(), out_ok);
  return SRHIP_OK;
}

template <typename T>
int eval_grad_tree_array_impl(srhip_dataset* ds, srhip_program* p, void* out_value, void* out_grad,
                              uint8_t* out_ok) {
  srhip_ctx* c = p->ctx;
  const int nt = p->ntrees;
  const int nconst = p->const_off.back();
  const int64_t rows = ds->rows, n_pad = ds->n_pad;
  const size_t es = sizeof(T);
  c->gather.ensure(std::max<size_t>((size_t)(nt + nconst) * n_pad * es, es));
  T* d_val = static_cast<T*>(c->gather.p);
  T* d_grad = d_val + (size_t)nt * n_pad;
  run_grad<T>(c, p, GRAD_OUT, ds, SRHIP_LOSS_L2, 0.0, d_val, d_grad, n_pad);
  if (rows > 0) {
    if (out_value && nt > 0)
      HIP_CHECK(hipMemcpy2DAsync(out_value, rows * es, d_val, n_pad * es, rows * es, nt, hipMemcpyDeviceToHost, c->stream));
    if (out_grad && nconst > 0)
      HIP_CHECK(hipMemcpy2DAsync(out_grad, rows * es, d_grad, n_pad * es, rows * es, nconst, hipMemcpyDeviceToHost, c->stream));
  }
  collect_grad_results(c, p, rows, nullptr, nullptr, out_ok);
  return SRHIP_OK;
}

struct OpName {
  const char* name;
  int arity;
  int id;
};
// Julia operator names → ids, including binopmap/unaopmap (src/Options.jl:86-120)
const OpName kOpNames[] = {
    {"+", 2, SRHIP_BOP_ADD}, {"plus", 2, SRHIP_BOP_ADD},
    {"-", 2, SRHIP_BOP_SUB}, {"sub", 2, SRHIP_BOP_SUB},
    {"*", 2, SRHIP_BOP_MUL}, {"mult", 2, SRHIP_BOP_MUL},
    {"/", 2, SRHIP_BOP_DIV}, {"div", 2, SRHIP_BOP_DIV},
    {"^", 2, SRHIP_BOP_POW}, {"pow", 2, SRHIP_BOP_POW}, {"safe_pow", 2, SRHIP_BOP_POW},
    {"greater", 2, SRHIP_BOP_GREATER},
    {"logical_or", 2, SRHIP_BOP_LOGICAL_OR},
    {"logical_and", 2, SRHIP_BOP_LOGICAL_AND},
    {"mod", 2, SRHIP_BOP_MOD},
    {"max", 2, SRHIP_BOP_MAX},
    {"min", 2, SRHIP_BOP_MIN},
    {"neg", 1, SRHIP_UOP_NEG},
    {"square", 1, SRHIP_UOP_SQUARE},
    {"cube", 1, SRHIP_UOP_CUBE},
    {"exp", 1, SRHIP_UOP_EXP},
    {"abs", 1, SRHIP_UOP_ABS},
    {"log", 1, SRHIP_UOP_LOG}, {"safe_log", 1, SRHIP_UOP_LOG},
    {"log2", 1, SRHIP_UOP_LOG2}, {"safe_log2", 1, SRHIP_UOP_LOG2},
    {"log10", 1, SRHIP_UOP_LOG10}, {"safe_log10", 1, SRHIP_UOP_LOG10},
    {"log1p", 1, SRHIP_UOP_LOG1P}, {"safe_log1p", 1, SRHIP_UOP_LOG1P},
    {"sqrt", 1, SRHIP_UOP_SQRT}, {"safe_sqrt", 1, SRHIP_UOP_SQRT},
    {"sin", 1, SRHIP_UOP_SIN},
    {"cos", 1, SRHIP_UOP_COS},
    {"tan", 1, SRHIP_UOP_TAN},
    {"sinh", 1, SRHIP_UOP_SINH},
    {"cosh", 1, SRHIP_UOP_COSH},
    {"tanh", 1, SRHIP_UOP_TANH},
    {"atan", 1, SRHIP_UOP_ATAN},
    {"asinh", 1, SRHIP_UOP_ASINH},
    {"acosh", 1, SRHIP_UOP_ACOSH}, {"safe_acosh", 1, SRHIP_UOP_ACOSH},
    {"atanh", 1, SRHIP_UOP_ATANH_CLIP}, {"atanh_clip", 1, SRHIP_UOP_ATANH_CLIP},
    {"erf", 1, SRHIP_UOP_ERF},
    {"erfc", 1, SRHIP_UOP_ERFC},
    {"gamma", 1, SRHIP_UOP_GAMMA},
    {"relu", 1, SRHIP_UOP_RELU},
    {"round", 1, SRHIP_UOP_ROUND},
    {"floor", 1, SRHIP_UOP_FLOOR},
    {"ceil", 1, SRHIP_UOP_CEIL},
    {"sign", 1, SRHIP_UOP_SIGN},
    {"inv", 1, SRHIP_UOP_INV},
};

}  // namespace

extern "C" {

int32_t srhip_version(void) { return SRHIP_ABI_VERSION; }

const char* srhip_last_error(void) { return g_last_error.c_str(); }

int32_t srhip_device_count(int32_t* out_count) {
  return guarded([&] {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (out_count) *out_count = n;
    return n > 0 ? SRHIP_OK : set_error(SRHIP_ERR_DEVICE, "no HIP device available");
  });
}

int32_t srhip_open(int32_t device, srhip_ctx** out_ctx) {
  return guarded([&] {
    if (!out_ctx) throw Error(SRHIP_ERR_INVALID, "out_ctx is null");
    *out_ctx = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw Error(SRHIP_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n) throw Error(SRHIP_ERR_INVALID, "device index out of range");
    HIP_CHECK(hipSetDevice(device));
    auto* c = new srhip_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreate(&c->ev[i]);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->pin_cnt, 2 * sizeof(uint32_t), hipHostMallocCoherent);
    if (e != hipSuccess) {
      delete c;
      throw Error(SRHIP_ERR_DEVICE, std::string("stream/event creation: ") + hipGetErrorString(e));
    }
    *out_ctx = c;
    return SRHIP_OK;
  });
}

int32_t srhip_close(srhip_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return SRHIP_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->copy_pool.reset();  // joins the host-copy workers
    ctx->partial.release();
    ctx->sums.release();
    ctx->oks.release();
    ctx->dloss.release();
    ctx->scratch_idx.release();
    ctx->gather.release();
    ctx->fail.release();
    ctx->ti_rec.release();
    ctx->bail_list.release();
    ctx->bail_fail.release();
    for (auto& e : ctx->ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->tev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->stage_evs)
      if (e) (void)hipEventDestroy(e);
    for (void* h : {(void*)ctx->pin_sum, (void*)ctx->pin_ok, (void*)ctx->pin_cnt, (void*)ctx->pin_stage})
      if (h) (void)hipHostFree(h);
    ctx->gpart.release();
    ctx->derived.release();
    ctx->gderived.release();
    ctx->gpartial.release();
    ctx->gsum.release();
    ctx->gok.release();
    ctx->gti.release();
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return SRHIP_OK;
  });
}

int32_t srhip_op_lookup(const char* name, int32_t* out_arity, int32_t* out_id) {
  return guarded([&] {
    if (!name) throw Error(SRHIP_ERR_INVALID, "null name");
    for (const auto& o : kOpNames) {
      if (std::strcmp(o.name, name) == 0) {
        if (out_arity) *out_arity = o.arity;
        if (out_id) *out_id = o.id;
        return SRHIP_OK;
      }
    }
    throw Error(SRHIP_ERR_UNSUPPORTED, std::string("operator not supported by the engine: ") + name);
  });
}

int32_t srhip_last_kernel_name(char* buf, int32_t len) {
  return guarded([&] {
    if (!buf || len <= 0) throw Error(SRHIP_ERR_INVALID, "null or empty buffer");
    std::snprintf(buf, (size_t)len, "%s", srhip::last_kernel());
    return SRHIP_OK;
  });
}

int32_t srhip_op_eval(int32_t dtype, int32_t arity, int32_t id, double a, double b, double* out) {
  return guarded([&] {
    if (!out) throw Error(SRHIP_ERR_INVALID, "null out");
    if (dtype != SRHIP_F32 && dtype != SRHIP_F64) throw Error(SRHIP_ERR_UNSUPPORTED, "dtype must be F32 or F64");
    bool known = false;
    for (const auto& o : kOpNames) known = known || (o.arity == arity && o.id == id);
    if (!known) throw Error(SRHIP_ERR_UNSUPPORTED, "unknown operator id for this arity");
    if (dtype == SRHIP_F32) {
      const float x = (float)a, y = (float)b;
      *out = arity == 1 ? (double)host::unop<float>(id, x) : (double)host::binop<float>(id, x, y);
    } else {
      *out = arity == 1 ? host::unop<double>(id, a) : host::binop<double>(id, a, b);
    }
    return SRHIP_OK;
  });
}

int32_t srhip_dataset_create(srhip_ctx* ctx, int32_t dtype, int32_t x_layout, const void* X,
                             const void* y, const void* w, int64_t n, int32_t nfeat,
                             int64_t row_begin, int64_t row_end, srhip_dataset** out_ds) {
  return guarded([&] {
    if (!ctx || !out_ds) throw Error(SRHIP_ERR_INVALID, "null ctx or out_ds");
    *out_ds = nullptr;
    if (dtype != SRHIP_F32 && dtype != SRHIP_F64) throw Error(SRHIP_ERR_UNSUPPORTED, "dtype must be F32 or F64");
    if (x_layout != SRHIP_X_JULIA && x_layout != SRHIP_X_FEATURE_MAJOR) throw Error(SRHIP_ERR_INVALID, "bad X layout");
    if (n < 0 || nfeat <= 0 || nfeat > 65535) throw Error(SRHIP_ERR_INVALID, "bad shape");
    if (row_begin < 0 || row_end < row_begin || row_end > n) throw Error(SRHIP_ERR_INVALID, "bad row range");
    if ((row_end > row_begin) && (!X || !y)) throw Error(SRHIP_ERR_INVALID, "null X or y");
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIP_CHECK(hipSetDevice(ctx->device));
    const size_t es = dtype_size(dtype);
    const int64_t rows = row_end - row_begin;
    const int64_t n_pad = pad_rows(rows);
    auto* ds = new srhip_dataset();
    ds->ctx = ctx;
    ds->dtype = dtype;
    ds->rows = rows;
    ds->nfeat = nfeat;
    ds->n_pad = n_pad;
    try {
      HIP_CHECK(hipMalloc(&ds->X, (size_t)n_pad * nfeat * es));
      HIP_CHECK(hipMalloc(&ds->y, (size_t)n_pad * es));
      if (w) HIP_CHECK(hipMalloc(&ds->w, (size_t)n_pad * es));
      HIP_CHECK(hipMemsetAsync(ds->X, 0, (size_t)n_pad * nfeat * es, ctx->stream));
      HIP_CHECK(hipMemsetAsync(ds->y, 0, (size_t)n_pad * es, ctx->stream));
      if (w) HIP_CHECK(hipMemsetAsync(ds->w, 0, (size_t)n_pad * es, ctx->stream));
      if (rows > 0) {
        // raw shard upload, then pack/transposes on the device; the staging
        // buffers are freed on every path (ScopedBuf), the error path included
        ScopedBuf raw_b, rawv_b, bad_b;
        raw_b.ensure((size_t)rows * nfeat * es);
        rawv_b.ensure((size_t)rows * es);
        bad_b.ensure(sizeof(int));
        void* raw = raw_b.p;
        void* rawv = rawv_b.p;
        int* bad = static_cast<int*>(bad_b.p);
        HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), ctx->stream));
        if (x_layout == SRHIP_X_JULIA) {
          HIP_CHECK(hipMemcpyAsync(raw, static_cast<const char*>(X) + (size_t)row_begin * nfeat * es,
                                   (size_t)rows * nfeat * es, hipMemcpyHostToDevice, ctx->stream));
        } else {
          HIP_CHECK(hipMemcpy2DAsync(raw, rows * es, static_cast<const char*>(X) + row_begin * es, n * es,
                                     rows * es, nfeat, hipMemcpyHostToDevice, ctx->stream));
        }
        const int64_t src_stride = rows;  // packed feature-major shard
        if (dtype == SRHIP_F32)
          HIP_CHECK(launch_pack_x<float>((const float*)raw, x_layout, src_stride, rows, nfeat, n_pad, (float*)ds->X, bad, ctx->stream));
        else
          HIP_CHECK(launch_pack_x<double>((const double*)raw, x_layout, src_stride, rows, nfeat, n_pad, (double*)ds->X, bad, ctx->stream));
        const void* vecs[2] = {y, w};
        void* dsts[2] = {ds->y, ds->w};
        for (int k = 0; k < 2; ++k) {
          if (!vecs[k]) continue;
          HIP_CHECK(hipMemcpyAsync(rawv, static_cast<const char*>(vecs[k]) + (size_t)row_begin * es, (size_t)rows * es,
                                   hipMemcpyHostToDevice, ctx->stream));
          if (dtype == SRHIP_F32)
            HIP_CHECK(launch_pack_vec<float>((const float*)rawv, rows, n_pad, (float*)dsts[k], ctx->stream));
          else
            HIP_CHECK(launch_pack_vec<double>((const double*)rawv, rows, n_pad, (double*)dsts[k], ctx->stream));
        }
        int hbad = 0;
        HIP_CHECK(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        ds->x_finite = hbad == 0;
      }
      HIP_CHECK(hipStreamSynchronize(ctx->stream));
      // Σw and Σ y·w over the shard, in double (src/Dataset.jl:56-60)
      double sw = 0.0, syw = 0.0;
      for (int64_t i = row_begin; i < row_end; ++i) {
        const double yi = dtype == SRHIP_F32 ? (double)static_cast<const float*>(y)[i] : static_cast<const double*>(y)[i];
        double wi = 1.0;
        if (w) {
          wi = dtype == SRHIP_F32 ? (double)static_cast<const float*>(w)[i] : static_cast<const double*>(w)[i];
          ds->h_w.push_back(wi);
        }
        sw += wi;
        syw += yi * wi;
      }
      ds->sum_w = sw;
      ds->sum_yw = syw;
    } catch (...) {
      if (ds->X) (void)hipFree(ds->X);
      if (ds->y) (void)hipFree(ds->y);
      if (ds->w) (void)hipFree(ds->w);
      delete ds;
      throw;
    }
    *out_ds = ds;
    return SRHIP_OK;
  });
}

int32_t srhip_dataset_destroy(srhip_dataset* ds) {
  return guarded([&] {
    if (!ds) return SRHIP_OK;
    std::lock_guard<std::mutex> lk(ds->ctx->mu);
    (void)hipSetDevice(ds->ctx->device);
    (void)hipStreamSynchronize(ds->ctx->stream);
    if (ds->X) (void)hipFree(ds->X);
    if (ds->y) (void)hipFree(ds->y);
    if (ds->w) (void)hipFree(ds->w);
    delete ds;
    return SRHIP_OK;
  });
}

int32_t srhip_dataset_info(const srhip_dataset* ds, int64_t* out_rows, int32_t* out_nfeat,
                           double* out_sum_w, double* out_sum_yw, int32_t* out_x_finite) {
  return guarded([&] {
    if (!ds) throw Error(SRHIP_ERR_INVALID, "null dataset");
    if (out_rows) *out_rows = ds->rows;
    if (out_nfeat) *out_nfeat = ds->nfeat;
    if (out_sum_w) *out_sum_w = ds->sum_w;
    if (out_sum_yw) *out_sum_yw = ds->sum_yw;
    if (out_x_finite) *out_x_finite = ds->x_finite ? 1 : 0;
    return SRHIP_OK;
  });
}

int32_t srhip_program_create(srhip_ctx* ctx, int32_t dtype, const srhip_trees* trees,
                             srhip_program** out_prog) {
  return srhip_program_create_ex(ctx, dtype, trees, 0u, out_prog);
}

int32_t srhip_program_create_ex(srhip_ctx* ctx, int32_t dtype, const srhip_trees* trees, uint32_t flags,
                                srhip_program** out_prog) {
  return guarded([&] {
    if (!ctx || !trees || !out_prog) throw Error(SRHIP_ERR_INVALID, "null argument");
    *out_prog = nullptr;
    if (dtype != SRHIP_F32 && dtype != SRHIP_F64) throw Error(SRHIP_ERR_UNSUPPORTED, "dtype must be F32 or F64");
    if (trees->ntrees < 0) throw Error(SRHIP_ERR_INVALID, "negative tree count");
    if (flags & ~(SRHIP_PROGRAM_VARYING_CONSTANTS | SRHIP_PROGRAM_INTERPRETED))
      throw Error(SRHIP_ERR_INVALID, "unknown program flags");
    const int nt = trees->ntrees;
    auto* p = new srhip_program();
    p->ctx = ctx;
    p->dtype = dtype;
    p->ntrees = nt;
    p->jit_memc = (flags & SRHIP_PROGRAM_VARYING_CONSTANTS) != 0;
    if (flags & SRHIP_PROGRAM_INTERPRETED) p->jit_allowed = false;
    try {
      if (nt > 0) {
        if (!trees->node_off || !trees->const_off) throw Error(SRHIP_ERR_INVALID, "null offsets");
        const int nn = trees->node_off[nt];
        const int nc = trees->const_off[nt];
        if (trees->node_off[0] != 0 || trees->const_off[0] != 0 || nn < 0 || nc < 0)
          throw Error(SRHIP_ERR_INVALID, "offsets must start at 0");
        for (int t = 0; t < nt; ++t)
          if (trees->node_off[t + 1] < trees->node_off[t] || trees->const_off[t + 1] < trees->const_off[t])
            throw Error(SRHIP_ERR_INVALID, "offsets must be non-decreasing");
        if (nn > 0 && (!trees->kind || !trees->arg)) throw Error(SRHIP_ERR_INVALID, "null node arrays");
        if (nc > 0 && !trees->consts) throw Error(SRHIP_ERR_INVALID, "null constants");
        p->node_off.assign(trees->node_off, trees->node_off + nt + 1);
        p->const_off.assign(trees->const_off, trees->const_off + nt + 1);
        p->kind.assign(trees->kind, trees->kind + nn);
        p->arg.assign(trees->arg, trees->arg + nn);
        const size_t cb = (size_t)nc * dtype_size(dtype);
        p->consts.resize(std::max<size_t>(cb, 1));
        if (cb) std::memcpy(p->consts.data(), trees->consts, cb);
      } else {
        p->node_off.assign(1, 0);
        p->const_off.assign(1, 0);
        p->consts.resize(1);
      }
      std::lock_guard<std::mutex> lk(ctx->mu);
      HIP_CHECK(hipSetDevice(ctx->device));
      if (dtype == SRHIP_F32) build_program<float>(p);
      else build_program<double>(p);
    } catch (...) {
      free_program_device(p);
      delete p;
      throw;
    }
    *out_prog = p;
    return SRHIP_OK;
  });
}

int32_t srhip_program_destroy(srhip_program* prog) {
  return guarded([&] {
    if (!prog) return SRHIP_OK;
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    (void)hipSetDevice(prog->ctx->device);
    (void)hipStreamSynchronize(prog->ctx->stream);
    free_program_device(prog);
    delete prog;
    return SRHIP_OK;
  });
}

int32_t srhip_program_info(const srhip_program* prog, int32_t* out_ntrees, int64_t* out_total_nodes,
                           int32_t* out_nodes) {
  return guarded([&] {
    if (!prog) throw Error(SRHIP_ERR_INVALID, "null program");
    if (out_ntrees) *out_ntrees = prog->ntrees;
    if (out_total_nodes) *out_total_nodes = prog->total_nodes;
    if (out_nodes) std::copy(prog->nodes.begin(), prog->nodes.end(), out_nodes);
    return SRHIP_OK;
  });
}

int32_t srhip_program_set_constants(srhip_program* prog, const void* consts) {
  return guarded([&] {
    if (!prog) throw Error(SRHIP_ERR_INVALID, "null program");
    const size_t cb = (size_t)prog->const_off.back() * dtype_size(prog->dtype);
    if (cb && !consts) throw Error(SRHIP_ERR_INVALID, "null constants");
    if (cb) std::memcpy(prog->consts.data(), consts, cb);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    if (prog->dtype == SRHIP_F32) update_constants<float>(prog);
    else update_constants<double>(prog);
    return SRHIP_OK;
  });
}

// A SRHIP_LOSS_* kind and its parameter: UNSUPPORTED beyond the table,
// INVALID without a needed parameter or for LPDistLoss{n} with n not an integer
// of magnitude below 2^31
static void check_loss(int32_t kind, const double* params) {
  if (kind < 0 || kind >= SRHIP_NUM_LOSSES) throw Error(SRHIP_ERR_UNSUPPORTED, "unsupported loss");
  const bool needs = kind != SRHIP_LOSS_L2 && kind != SRHIP_LOSS_L1 && kind != SRHIP_LOSS_LOGCOSH &&
                     kind != SRHIP_LOSS_LOGITDIST;
  if (needs && !params) throw Error(SRHIP_ERR_INVALID, "loss needs a parameter");
  if (kind == SRHIP_LOSS_LPINT && !(params[0] == std::trunc(params[0]) && std::fabs(params[0]) < 2147483648.0))
    throw Error(SRHIP_ERR_INVALID, "LPDistLoss{n} (SRHIP_LOSS_LPINT) needs an integer n");
}

int32_t srhip_eval_loss(srhip_dataset* ds, const srhip_program* prog, int32_t loss_kind,
                        const double* loss_params, const int64_t* row_idx, int64_t nidx,
                        double* out_loss_sum, double* out_weight_sum, uint8_t* out_ok) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    check_loss(loss_kind, loss_params);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    if (ds->dtype == SRHIP_F32)
      return eval_loss_impl<float>(ds, prog, loss_kind, loss_params, row_idx, nidx, out_loss_sum, out_weight_sum, out_ok);
    return eval_loss_impl<double>(ds, prog, loss_kind, loss_params, row_idx, nidx, out_loss_sum, out_weight_sum, out_ok);
  });
}

int32_t srhip_eval_loss_packed(srhip_dataset* ds, srhip_program* prog, int32_t loss_kind, const double* loss_params,
                               double* d_out) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    if (!d_out) throw Error(SRHIP_ERR_INVALID, "null output");
    check_loss(loss_kind, loss_params);
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, d_out) != hipSuccess || at.type != hipMemoryTypeDevice)
      throw Error(SRHIP_ERR_INVALID, "d_out is not device memory");
    if (at.device != prog->ctx->device)
      throw Error(SRHIP_ERR_INVALID, "d_out is on device " + std::to_string(at.device) + ", the program on device " +
                                         std::to_string(prog->ctx->device));
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    if (ds->dtype == SRHIP_F32) return eval_loss_packed_impl<float>(ds, prog, loss_kind, loss_params, d_out);
    return eval_loss_packed_impl<double>(ds, prog, loss_kind, loss_params, d_out);
  });
}

int32_t srhip_eval_loss_batch(srhip_dataset* ds, const srhip_trees* trees, int32_t loss_kind,
                              const double* loss_params, const int64_t* row_idx, int64_t nidx,
                              double* out_loss_sum, double* out_weight_sum, uint8_t* out_ok) {
  if (!ds) return set_error(SRHIP_ERR_INVALID, "null dataset");
  return srhip_eval_loss_batch_ctx(ds->ctx, ds, trees, loss_kind, loss_params, row_idx, nidx, out_loss_sum,
                                   out_weight_sum, out_ok);
}

int32_t srhip_eval_loss_batch_ctx(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees, int32_t loss_kind,
                                  const double* loss_params, const int64_t* row_idx, int64_t nidx,
                                  double* out_loss_sum, double* out_weight_sum, uint8_t* out_ok) {
  if (!ds) return set_error(SRHIP_ERR_INVALID, "null dataset");
  if (!ctx) return set_error(SRHIP_ERR_INVALID, "null ctx");
  srhip_program* p = nullptr;
  int32_t rc = srhip_program_create(ctx, ds->dtype, trees, &p);
  if (rc != SRHIP_OK) return rc;
  rc = srhip_eval_loss(ds, p, loss_kind, loss_params, row_idx, nidx, out_loss_sum, out_weight_sum, out_ok);
  std::string err = g_last_error;
  srhip_program_destroy(p);
  g_last_error = err;
  return rc;
}

int32_t srhip_eval_loss_rowsets(srhip_dataset* ds, const srhip_program* prog, int32_t loss_kind,
                                const double* loss_params, const int64_t* row_idx, int64_t batch_size,
                                double* out_loss_sum, double* out_weight_sum, uint8_t* out_ok) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    check_loss(loss_kind, loss_params);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    if (ds->dtype == SRHIP_F32)
      return eval_loss_rowsets_impl<float>(ds, prog, loss_kind, loss_params, row_idx, batch_size, out_loss_sum,
                                           out_weight_sum, out_ok);
    return eval_loss_rowsets_impl<double>(ds, prog, loss_kind, loss_params, row_idx, batch_size, out_loss_sum,
                                          out_weight_sum, out_ok);
  });
}

int32_t srhip_eval_loss_batch_rowsets_ctx(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees,
                                          int32_t loss_kind, const double* loss_params, const int64_t* row_idx,
                                          int64_t batch_size, double* out_loss_sum, double* out_weight_sum,
                                          uint8_t* out_ok) {
  if (!ds) return set_error(SRHIP_ERR_INVALID, "null dataset");
  if (!ctx) ctx = ds->ctx;
  srhip_program* p = nullptr;
  // row sets run in the interpreter: no tree code to build
  int32_t rc = srhip_program_create_ex(ctx, ds->dtype, trees, SRHIP_PROGRAM_INTERPRETED, &p);
  if (rc != SRHIP_OK) return rc;
  rc = srhip_eval_loss_rowsets(ds, p, loss_kind, loss_params, row_idx, batch_size, out_loss_sum, out_weight_sum,
                               out_ok);
  std::string err = g_last_error;
  srhip_program_destroy(p);
  g_last_error = err;
  return rc;
}

int32_t srhip_eval_tree_array(srhip_dataset* ds, const srhip_program* prog, void* out, uint8_t* out_ok) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    if (ds->dtype == SRHIP_F32) return eval_tree_array_impl<float>(ds, prog, out, out_ok);
    return eval_tree_array_impl<double>(ds, prog, out, out_ok);
  });
}

int32_t srhip_eval_loss_grad(srhip_dataset* ds, const srhip_program* prog, int32_t loss_kind,
                             const double* loss_params, double* out_loss_sum, double* out_dloss,
                             double* out_weight_sum, uint8_t* out_ok) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    check_loss(loss_kind, loss_params);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    auto* p = const_cast<srhip_program*>(prog);  // gradient programs are built lazily
    if (ds->dtype == SRHIP_F32)
      return eval_loss_grad_impl<float>(ds, p, loss_kind, loss_params, out_loss_sum, out_dloss, out_weight_sum, out_ok);
    return eval_loss_grad_impl<double>(ds, p, loss_kind, loss_params, out_loss_sum, out_dloss, out_weight_sum, out_ok);
  });
}

int32_t srhip_eval_grad_tree_array(srhip_dataset* ds, const srhip_program* prog, void* out_value,
                                   void* out_grad, uint8_t* out_ok) {
  return guarded([&] {
    check_program_vs_dataset(ds, prog);
    std::lock_guard<std::mutex> lk(prog->ctx->mu);
    HIP_CHECK(hipSetDevice(prog->ctx->device));
    auto* p = const_cast<srhip_program*>(prog);
    if (ds->dtype == SRHIP_F32) return eval_grad_tree_array_impl<float>(ds, p, out_value, out_grad, out_ok);
    return eval_grad_tree_array_impl<double>(ds, p, out_value, out_grad, out_ok);
  });
}

int32_t srhip_last_kernel_time(const srhip_ctx* ctx, double* out_ms, int32_t* out_launches) {
  return guarded([&] {
    if (!ctx) throw Error(SRHIP_ERR_INVALID, "null ctx");
    auto* c = const_cast<srhip_ctx*>(ctx);
    if (c->timing_pending || c->cnt_pending) {  // a call that returned before its results were read
      std::lock_guard<std::mutex> lk(c->mu);
      HIP_CHECK(hipSetDevice(c->device));
      HIP_CHECK(hipStreamSynchronize(c->stream));
      timing_finish(c);
    }
    if (out_ms) *out_ms = ctx->last_ms;
    if (out_launches) *out_launches = ctx->last_launches;
    return SRHIP_OK;
  });
}

int32_t srhip_sync(srhip_ctx* ctx) {
  return guarded([&] {
    if (!ctx) throw Error(SRHIP_ERR_INVALID, "null ctx");
    HIP_CHECK(hipSetDevice(ctx->device));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return SRHIP_OK;
  });
}

}  // extern "C"

int32_t srhip_program_update_stats(const srhip_program* prog, int64_t* out_inplace, int64_t* out_rebuilt) {
  return guarded([&] {
    if (!prog) throw Error(SRHIP_ERR_INVALID, "null program");
    if (out_inplace) *out_inplace = prog->n_inplace;
    if (out_rebuilt) *out_rebuilt = prog->n_rebuild;
    return SRHIP_OK;
  });
}

int32_t srhip_program_grad_jit_info(const srhip_program* prog, int32_t* out_ntrees, int32_t* out_nrejected,
                                    int64_t* out_code_bytes, double* out_ms_codegen, double* out_ms_load) {
  return guarded([&] {
    if (!prog) throw Error(SRHIP_ERR_INVALID, "null program");
    const bool on = prog->gjit != nullptr || prog->gjit64 != nullptr;
    if (out_ntrees) *out_ntrees = on ? prog->gjit_stats.ntrees : 0;
    if (out_nrejected) *out_nrejected = on ? prog->gjit_stats.nrejected : 0;
    if (out_code_bytes) *out_code_bytes = on ? (int64_t)prog->gjit_stats.code_bytes : 0;
    if (out_ms_codegen) *out_ms_codegen = on ? prog->gjit_stats.ms_codegen : 0.0;
    if (out_ms_load) *out_ms_load = on ? prog->gjit_stats.ms_load : 0.0;
    return SRHIP_OK;
  });
}

int32_t srhip_program_jit_info(const srhip_program* prog, int32_t* out_ntrees, int32_t* out_nfast,
                               int64_t* out_code_bytes, double* out_ms_codegen, double* out_ms_load) {
  return guarded([&] {
    if (!prog) throw Error(SRHIP_ERR_INVALID, "null program");
    const bool on = prog->jit != nullptr || prog->jit64 != nullptr;
    if (out_ntrees) *out_ntrees = on ? prog->nlist_j : 0;
    if (out_nfast) *out_nfast = on ? prog->jit_stats.nfast : 0;
    if (out_code_bytes) *out_code_bytes = on ? (int64_t)prog->jit_stats.code_bytes : 0;
    if (out_ms_codegen) *out_ms_codegen = on ? prog->jit_stats.ms_codegen : 0.0;
    if (out_ms_load) *out_ms_load = on ? prog->jit_stats.ms_load : 0.0;
    return SRHIP_OK;
  });
}

int32_t srhip_last_tree_code(const srhip_ctx* ctx, int32_t* out_ntrees) {
  return guarded([&] {
    if (!ctx || !out_ntrees) throw Error(SRHIP_ERR_INVALID, "null argument");
    *out_ntrees = ctx->last_jit_trees;
    return SRHIP_OK;
  });
}

int32_t srhip_last_bailed(const srhip_ctx* ctx, int32_t* out_ntrees, int64_t* out_redone) {
  return guarded([&] {
    if (!ctx || !out_ntrees) throw Error(SRHIP_ERR_INVALID, "null argument");
    auto* c = const_cast<srhip_ctx*>(ctx);
    if (c->timing_pending || c->cnt_pending) {
      std::lock_guard<std::mutex> lk(c->mu);
      HIP_CHECK(hipSetDevice(c->device));
      HIP_CHECK(hipStreamSynchronize(c->stream));
      timing_finish(c);
    }
    *out_ntrees = ctx->last_bailed;
    if (out_redone) *out_redone = ctx->last_redone;
    return SRHIP_OK;
  });
}

namespace {
int32_t jit_compile_hook(const srhip_trees* trees, int mode, uint8_t* out_bytes, int64_t* inout_nbytes,
                         char* out_text, int64_t* inout_ntext, int32_t* out_offsets, int64_t* inout_noffsets,
                         int loss = SRHIP_LOSS_L2, double lparam = 0.0, bool out_mode = false, bool notext = false) {
  return guarded([&] {
    if (!trees || !inout_nbytes || !inout_ntext || !inout_noffsets) throw Error(SRHIP_ERR_INVALID, "null argument");
    if (!jit::available()) throw Error(SRHIP_ERR_UNSUPPORTED, std::string("tree compiler: ") + jit::unavailable_reason());
    std::vector<uint8_t> bytes;
    std::string text;
    std::vector<int32_t> offs;
    if (loss < 0 || loss >= SRHIP_NUM_LOSSES) throw Error(SRHIP_ERR_INVALID, "unknown loss");
    uint64_t lbits;
    std::memcpy(&lbits, &lparam, 8);
    if (mode == 2 && !jit::has_dloss_routine(loss))
      throw Error(SRHIP_ERR_UNSUPPORTED, "no gradient tree code for this loss");
    if (mode != 2 && mode != 5 && mode != 6 && !jit::has_loss_routine(loss))
      throw Error(SRHIP_ERR_UNSUPPORTED, "no tree code for this loss");
    if (mode == 6) {  // Float64 gradient tree code (jit64.cpp GradGen64)
      if (!jit::has_dloss_routine64(loss)) throw Error(SRHIP_ERR_UNSUPPORTED, "no Float64 gradient tree code for this loss");
      CompiledBatch<double> cb = compile_batch<double>(*trees, /*grad=*/true);
      std::vector<int32_t> cand, coff(trees->const_off, trees->const_off + trees->ntrees + 1);
      for (int t = 0; t < cb.ntrees; ++t)
        if (cb.tree_off[t] >= 0) cand.push_back(t);
      jit::compile_grad_only64(cb, coff, cand, &bytes, &text, &offs, loss, lbits);
    } else if (mode == 5) {  // Float64 tree code (jit64.cpp): L2, another loss's tail, or per-row outputs
      CompiledBatch<double> cb = compile_batch<double>(*trees);
      std::vector<int32_t> cand;
      for (int t = 0; t < cb.ntrees; ++t)
        if (cb.tree_off[t] >= 0 && cb.need[t] <= kShallowSlots) cand.push_back(t);
      jit::Opts64 o;
      o.out = out_mode;
      o.loss = out_mode ? SRHIP_LOSS_L2 : loss;
      o.lparam = lbits;
      jit::compile_only64(cb, cand, &bytes, &text, &offs, o);
    } else if (mode == 2) {  // gradient tree code
      CompiledBatch<float> cb = compile_batch<float>(*trees, /*grad=*/true);
      std::vector<int32_t> cand, coff(trees->const_off, trees->const_off + trees->ntrees + 1);
      for (int t = 0; t < cb.ntrees; ++t)
        if (cb.tree_off[t] >= 0) cand.push_back(t);
      jit::compile_grad_only(cb, coff, cand, &bytes, &text, &offs, nullptr, loss, lbits);
    } else {
      CompiledBatch<float> cb = compile_batch<float>(*trees);
      std::vector<int32_t> cand;
      for (int t = 0; t < cb.ntrees; ++t)
        if (cb.tree_off[t] >= 0 && cb.need[t] <= kShallowSlots) cand.push_back(t);
      jit::Options jo;
      jo.fast = mode == 1 || mode == 4;
      jo.memc = mode == 3 || mode == 4;
      jo.text = !notext;  // no text: the parallel code generation of build()
      jo.loss = loss;
      jo.lparam = lbits;
      jo.out = out_mode;
      jit::compile_only(cb, cand, jo, &bytes, &text, &offs, nullptr);
    }
    if ((int64_t)bytes.size() > *inout_nbytes || (int64_t)text.size() + 1 > *inout_ntext ||
        (int64_t)offs.size() > *inout_noffsets) {
      *inout_nbytes = (int64_t)bytes.size();
      *inout_ntext = (int64_t)text.size() + 1;
      *inout_noffsets = (int64_t)offs.size();
      throw Error(SRHIP_ERR_INVALID, "output buffers too small");
    }
    if (out_bytes && !bytes.empty()) std::memcpy(out_bytes, bytes.data(), bytes.size());
    if (out_text) std::memcpy(out_text, text.c_str(), text.size() + 1);
    if (out_offsets && !offs.empty()) std::memcpy(out_offsets, offs.data(), offs.size() * sizeof(int32_t));
    *inout_nbytes = (int64_t)bytes.size();
    *inout_ntext = (int64_t)text.size() + 1;
    *inout_noffsets = (int64_t)offs.size();
    return SRHIP_OK;
  });
}
}  // namespace

int32_t srhip_jit_compile(const srhip_trees* trees, int32_t fast, uint8_t* out_bytes, int64_t* inout_nbytes,
                          char* out_text, int64_t* inout_ntext, int32_t* out_offsets,
                          int64_t* inout_noffsets) {
  // fast: bit 0 the FAST path, bit 1 memory-constant code (mode 3 / 4 below),
  // bit 2 per-row output code, bit 3 Float64 trees (jit64.cpp; the other bits ignored)
  if (fast & 8)  // Float64 trees (bit 2: their per-row output code)
    return jit_compile_hook(trees, 5, out_bytes, inout_nbytes, out_text, inout_ntext, out_offsets, inout_noffsets,
                            SRHIP_LOSS_L2, 0.0, (fast & 4) != 0);
  return jit_compile_hook(trees, (fast & 2) ? ((fast & 1) ? 4 : 3) : ((fast & 1) ? 1 : 0), out_bytes, inout_nbytes,
                          out_text, inout_ntext, out_offsets, inout_noffsets, SRHIP_LOSS_L2, 0.0, (fast & 4) != 0,
                          (fast & 16) != 0);
}

int32_t srhip_jit_compile_grad(const srhip_trees* trees, uint8_t* out_bytes, int64_t* inout_nbytes,
                               char* out_text, int64_t* inout_ntext, int32_t* out_offsets,
                               int64_t* inout_noffsets) {
  return jit_compile_hook(trees, 2, out_bytes, inout_nbytes, out_text, inout_ntext, out_offsets, inout_noffsets);
}

int32_t srhip_jit_compile_loss(const srhip_trees* trees, int32_t grad, int32_t fast, int32_t loss, double loss_param,
                               uint8_t* out_bytes, int64_t* inout_nbytes, char* out_text, int64_t* inout_ntext,
                               int32_t* out_offsets, int64_t* inout_noffsets) {
  // fast bit 3: the Float64 tree compiler (jit64.cpp) with this loss's tail, or with grad its gradient code
  return jit_compile_hook(trees, (fast & 8) ? (grad ? 6 : 5) : grad ? 2 : ((fast & 1) ? 1 : 0), out_bytes, inout_nbytes, out_text,
                          inout_ntext, out_offsets, inout_noffsets, loss, loss_param);
}

namespace {
template <typename T>
void constant_map_check(const srhip_trees* trees, bool grad, bool keep, const void* new_consts, int64_t* mismatch,
                        int64_t* recompiled, int32_t* relayout) {
  srhip_program p;  // host state only: patch_image reads the trees and writes the images
  p.ntrees = trees->ntrees;
  p.jit_memc = keep;  // patch_image recompiles with keep_layout for such programs
  const int nt = trees->ntrees;
  p.node_off.assign(trees->node_off, trees->node_off + nt + 1);
  p.const_off.assign(trees->const_off, trees->const_off + nt + 1);
  p.kind.assign(trees->kind, trees->kind + p.node_off[nt]);
  p.arg.assign(trees->arg, trees->arg + p.node_off[nt]);
  const size_t cbytes = (size_t)p.const_off[nt] * sizeof(T);
  p.consts.resize(std::max<size_t>(cbytes, 1));
  if (cbytes) std::memcpy(p.consts.data(), trees->consts, cbytes);
  CompiledBatch<T> cb = compile_batch_par<T>(*trees, grad, keep);
  std::vector<unsigned char> code(reinterpret_cast<const unsigned char*>(cb.code.data()),
                                  reinterpret_cast<const unsigned char*>(cb.code.data() + cb.code.size()));
  std::vector<uint8_t> sfail = cb.static_fail, fir = cb.fail_if_rows;
  std::vector<unsigned char> cprev = p.consts;  // the constants the image was compiled with
  if (cbytes) std::memcpy(p.consts.data(), new_consts, cbytes);
  bool vchg = false;
  *relayout = patch_image<T>(&p, code, cb.tree_off, cb.len, cb.cmap, cb.direct, cb.folds, sfail, grad ? nullptr : &fir,
                             grad, &vchg, cprev, recompiled) ? 0 : 1;
  if (*relayout) return;
  srhip_trees fresh_trees = *trees;
  fresh_trees.consts = new_consts;
  const CompiledBatch<T> fresh = compile_batch_par<T>(fresh_trees, grad, keep);
  const Ins<T>* ins = reinterpret_cast<const Ins<T>*>(code.data());
  *mismatch = 0;
  for (int t = 0; t < nt; ++t) {
    bool bad = sfail[t] != fresh.static_fail[t] || (!grad && fir[t] != fresh.fail_if_rows[t]);
    // a tree that fails statically is never evaluated: its immediates are free
    if (!bad && fresh.tree_off[t] >= 0 && !fresh.static_fail[t] && !fresh.fail_if_rows[t]) {
      bad = cb.tree_off[t] < 0 || cb.len[t] != fresh.len[t] ||
            std::memcmp(ins + cb.tree_off[t], &fresh.code[fresh.tree_off[t]], sizeof(Ins<T>) * fresh.len[t]) != 0;
    }
    if (bad && std::getenv("SRHIP_DEBUG_CMAP"))
      std::fprintf(stderr, "cmap mismatch tree %d: sfail %d/%d fir %d/%d toff %d/%d len %d/%d\n", t, sfail[t],
                   fresh.static_fail[t], fir[t], fresh.fail_if_rows[t], cb.tree_off[t], fresh.tree_off[t], cb.len[t],
                   fresh.len[t]);
    *mismatch += bad ? 1 : 0;
  }
}
}  // namespace

int32_t srhip_debug_constant_map(const srhip_trees* trees, int32_t dtype, int32_t grad, const void* new_consts,
                                 int64_t* out_mismatch, int64_t* out_recompiled, int32_t* out_relayout) {
  return guarded([&] {
    if (!trees || !out_mismatch || !out_recompiled || !out_relayout) throw Error(SRHIP_ERR_INVALID, "null argument");
    if (trees->ntrees < 0 || (trees->ntrees > 0 && (!trees->node_off || !trees->const_off)))
      throw Error(SRHIP_ERR_INVALID, "bad trees");
    if (trees->ntrees > 0 && trees->const_off[trees->ntrees] > 0 && !new_consts) throw Error(SRHIP_ERR_INVALID, "null constants");
    *out_mismatch = 0;
    *out_recompiled = 0;
    *out_relayout = 0;
    const bool g = (grad & 1) != 0, keep = (grad & 2) != 0;
    if (dtype == SRHIP_F32) constant_map_check<float>(trees, g, keep, new_consts, out_mismatch, out_recompiled, out_relayout);
    else if (dtype == SRHIP_F64) constant_map_check<double>(trees, g, keep, new_consts, out_mismatch, out_recompiled, out_relayout);
    else throw Error(SRHIP_ERR_UNSUPPORTED, "dtype must be F32 or F64");
    return SRHIP_OK;
  });
}

// ---- batched constant optimisation (constopt.cpp) ------------------------------
namespace {

void check_rc(int32_t rc) {
  if (rc != SRHIP_OK) throw Error(rc, g_last_error);
}

copt::Problem make_problem(const srhip_trees* trees, int dtype) {
  if (!trees || trees->ntrees < 0 || !trees->const_off || (trees->ntrees > 0 && !trees->node_off))
    throw Error(SRHIP_ERR_INVALID, "null or malformed trees");
  if (dtype != SRHIP_F32 && dtype != SRHIP_F64) throw Error(SRHIP_ERR_UNSUPPORTED, "dtype must be F32 or F64");
  copt::Problem pb;
  pb.dtype = dtype;
  pb.const_off.assign(trees->const_off, trees->const_off + trees->ntrees + 1);
  if (pb.const_off[0] != 0) throw Error(SRHIP_ERR_INVALID, "const_off[0] must be 0");
  for (int t = 0; t < trees->ntrees; ++t)
    if (pb.const_off[t + 1] < pb.const_off[t]) throw Error(SRHIP_ERR_INVALID, "const_off must be non-decreasing");
  const size_t nc = (size_t)pb.const_off.back();
  if (nc && !trees->consts) throw Error(SRHIP_ERR_INVALID, "null consts");
  pb.consts.resize(nc);
  for (size_t j = 0; j < nc; ++j)
    pb.consts[j] = dtype == SRHIP_F32 ? (double)static_cast<const float*>(trees->consts)[j]
                                      : static_cast<const double*>(trees->consts)[j];
  return pb;
}

copt::Options make_copt_options(const srhip_constopt_options* o) {
  if (!o) throw Error(SRHIP_ERR_INVALID, "null options");
  copt::Options r;
  r.algorithm = o->algorithm;
  r.iterations = o->iterations;
  r.nrestarts = o->nrestarts;
  r.noise = o->start_noise;
  r.seed = o->seed;
  return r;
}

void write_result(const copt::Result& r, int dtype, void* out_consts, double* out_loss, uint8_t* out_conv,
                  double* out_nev, bool loss_in_t) {
  const size_t nc = r.consts.size(), nt = r.loss.size();
  if (out_consts)
    for (size_t j = 0; j < nc; ++j) {
      if (dtype == SRHIP_F32) static_cast<float*>(out_consts)[j] = (float)r.consts[j];
      else static_cast<double*>(out_consts)[j] = r.consts[j];
    }
  for (size_t t = 0; t < nt; ++t) {
    if (out_loss) {
      double v = r.loss[t];
      if (loss_in_t && dtype == SRHIP_F32) v = (double)(float)v;
      out_loss[t] = v;
    }
    if (out_conv) out_conv[t] = r.converged[t];
    if (out_nev) out_nev[t] = r.num_evals[t];
  }
}

// Where the time of the last srhip_optimize_constants_batch call on this
// thread went (srhip_constopt_profile): program builds, constant uploads,
// loss and gradient calls (wall), the kernels inside them (HIP events).
struct CoptProfile {
  double total = 0, create = 0, set = 0, loss = 0, grad = 0, kernel_ms = 0;
  int64_t ncreate = 0, nloss = 0, ngrad = 0, nrebuilt = 0;
  double jit_codegen_ms = 0, jit_load_ms = 0;  // of the builds (tree code)
};
thread_local CoptProfile t_copt;
double secs_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// The candidates of one evaluation set as a program on the engine (memory-
// constant tree code: constant updates never recompile); loss and ∂L/∂c of
// every member in one call each, finished as the reference's loss (:12-19).
struct EngineSet : copt::Set {
  srhip_ctx* ctx;
  srhip_dataset* ds;
  int dtype, loss;
  const double* params;
  srhip_program* prog = nullptr;
  std::vector<int32_t> coff;  // members' constant offsets
  EngineSet(srhip_ctx* c, srhip_dataset* d, const srhip_trees* trees, int dt, int ls, const double* pr,
            const std::vector<int32_t>& members)
      : ctx(c), ds(d), dtype(dt), loss(ls), params(pr) {
    const size_t es = dt == SRHIP_F32 ? 4 : 8;
    std::vector<int32_t> noff{0};
    std::vector<uint8_t> kind;
    std::vector<uint16_t> arg;
    std::vector<unsigned char> cst;
    coff.push_back(0);
    for (int32_t t : members) {
      if (t < 0 || t >= trees->ntrees) throw Error(SRHIP_ERR_INVALID, "member out of range");
      const int32_t a = trees->node_off[t], b = trees->node_off[t + 1];
      kind.insert(kind.end(), trees->kind + a, trees->kind + b);
      arg.insert(arg.end(), trees->arg + a, trees->arg + b);
      noff.push_back((int32_t)kind.size());
      const int32_t ca = trees->const_off[t], cb = trees->const_off[t + 1];
      const unsigned char* src = static_cast<const unsigned char*>(trees->consts);
      cst.insert(cst.end(), src + (size_t)ca * es, src + (size_t)cb * es);
      coff.push_back(coff.back() + (cb - ca));
    }
    srhip_trees tr;
    tr.ntrees = (int32_t)members.size();
    tr.node_off = noff.data();
    tr.kind = kind.data();
    tr.arg = arg.data();
    tr.const_off = coff.data();
    tr.consts = cst.data();
    const auto t0 = std::chrono::steady_clock::now();
    check_rc(srhip_program_create_ex(ctx, dtype, &tr, SRHIP_PROGRAM_VARYING_CONSTANTS, &prog));
    t_copt.create += secs_since(t0);
    t_copt.ncreate += 1;
    {
      int32_t nt = 0, nf = 0;
      int64_t nb = 0;
      double mc = 0, ml = 0;
      if (srhip_program_jit_info(prog, &nt, &nf, &nb, &mc, &ml) == SRHIP_OK) {
        t_copt.jit_codegen_ms += mc;
        t_copt.jit_load_ms += ml;
      }
    }
  }
  ~EngineSet() override {
    int64_t inplace = 0, rebuilt = 0;
    if (prog && srhip_program_update_stats(prog, &inplace, &rebuilt) == SRHIP_OK) t_copt.nrebuilt += rebuilt;
    if (prog) (void)srhip_program_destroy(prog);
  }
  void eval(const std::vector<double>& X, bool grad, std::vector<double>& f, std::vector<double>& g) override {
    const int n = (int)coff.size() - 1;
    const size_t nc = (size_t)coff.back();
    if (X.size() != nc) throw Error(SRHIP_ERR_INVALID, "constant count mismatch");
    auto t0 = std::chrono::steady_clock::now();
    if (dtype == SRHIP_F32) {
      std::vector<float> c(nc);
      for (size_t j = 0; j < nc; ++j) c[j] = (float)X[j];
      check_rc(srhip_program_set_constants(prog, c.data()));
    } else {
      check_rc(srhip_program_set_constants(prog, X.data()));
    }
    t_copt.set += secs_since(t0);
    std::vector<double> sums(std::max(n, 1)), dl(std::max<size_t>(nc, 1));
    std::vector<uint8_t> ok(std::max(n, 1));
    double wsum = 0.0;
    t0 = std::chrono::steady_clock::now();
    if (grad) check_rc(srhip_eval_loss_grad(ds, prog, loss, params, sums.data(), dl.data(), &wsum, ok.data()));
    else check_rc(srhip_eval_loss(ds, prog, loss, params, nullptr, 0, sums.data(), &wsum, ok.data()));
    (grad ? t_copt.grad : t_copt.loss) += secs_since(t0);
    (grad ? t_copt.ngrad : t_copt.nloss) += 1;
    {
      double ms = 0.0;
      if (srhip_last_kernel_time(ctx, &ms, nullptr) == SRHIP_OK) t_copt.kernel_ms += ms;
    }
    f.assign(n, 0.0);
    for (int t = 0; t < n; ++t) {
      const double v = sums[t] / wsum;
      f[t] = (ok[t] && std::isfinite(v)) ? v : INFINITY;
    }
    if (grad) {
      g.assign(nc, 0.0);
      for (int t = 0; t < n; ++t)
        for (int32_t j = coff[t]; j < coff[t + 1]; ++j) g[j] = ok[t] ? dl[j] / wsum : NAN;
    }
  }
};
struct EngineFactory : copt::Factory {
  srhip_ctx* ctx;
  srhip_dataset* ds;
  const srhip_trees* trees;
  int dtype, loss;
  const double* params;
  std::unique_ptr<copt::Set> make(const std::vector<int32_t>& members) override {
    return std::unique_ptr<copt::Set>(new EngineSet(ctx, ds, trees, dtype, loss, params, members));
  }
};

// the caller's evaluator
struct CallbackSet : copt::Set {
  srhip_constopt_eval_fn fn;
  void* user;
  std::vector<int32_t> members;
  size_t nconst;
  void eval(const std::vector<double>& X, bool grad, std::vector<double>& f, std::vector<double>& g) override {
    if (X.size() != nconst) throw Error(SRHIP_ERR_INVALID, "constant count mismatch");
    f.assign(members.size(), 0.0);
    g.assign(grad ? nconst : 0, 0.0);
    const int32_t rc = fn(user, (int64_t)members.size(), members.data(), X.data(), grad ? 1 : 0, f.data(),
                          grad ? g.data() : nullptr);
    if (rc != 0) throw Error(SRHIP_ERR_INVALID, "constant optimisation: the evaluator callback failed");
  }
};
struct CallbackFactory : copt::Factory {
  srhip_constopt_eval_fn fn;
  void* user;
  const std::vector<int32_t>* const_off;
  std::unique_ptr<copt::Set> make(const std::vector<int32_t>& members) override {
    std::unique_ptr<CallbackSet> s(new CallbackSet());
    s->fn = fn;
    s->user = user;
    s->members = members;
    s->nconst = 0;
    const int nt = (int)const_off->size() - 1;
    for (int32_t t : members) {
      if (t < 0 || t >= nt) throw Error(SRHIP_ERR_INVALID, "member out of range");
      s->nconst += (size_t)((*const_off)[t + 1] - (*const_off)[t]);
    }
    return s;
  }
};

}  // namespace

int32_t srhip_optimize_constants_batch(srhip_ctx* ctx, srhip_dataset* ds, const srhip_trees* trees,
                                       const srhip_constopt_options* opts, void* out_consts, double* out_loss,
                                       uint8_t* out_converged, double* out_num_evals) {
  return guarded([&] {
    if (!ds) throw Error(SRHIP_ERR_INVALID, "null dataset");
    if (!opts) throw Error(SRHIP_ERR_INVALID, "null options");
    check_loss(opts->loss_kind, opts->loss_params);
    t_copt = CoptProfile();
    const auto t0 = std::chrono::steady_clock::now();
    copt::Problem pb = make_problem(trees, ds->dtype);
    EngineFactory fac;
    fac.ctx = ctx ? ctx : ds->ctx;
    fac.ds = ds;
    fac.trees = trees;
    fac.dtype = ds->dtype;
    fac.loss = opts->loss_kind;
    fac.params = opts->loss_params;
    const copt::Result r = copt::optimize(pb, make_copt_options(opts), fac);
    write_result(r, ds->dtype, out_consts, out_loss, out_converged, out_num_evals, true);
    t_copt.total = secs_since(t0);
    return SRHIP_OK;
  });
}

int32_t srhip_constopt_profile(double* out, int32_t n) {
  return guarded([&] {
    if (!out || n < 0) throw Error(SRHIP_ERR_INVALID, "null output");
    const CoptProfile& q = t_copt;
    const double v[12] = {q.total, q.create, q.set, q.loss, q.grad, q.kernel_ms * 1e-3,
                          (double)q.ncreate, (double)q.nloss, (double)q.ngrad, (double)q.nrebuilt,
                          q.jit_codegen_ms * 1e-3, q.jit_load_ms * 1e-3};
    for (int32_t i = 0; i < n && i < 12; ++i) out[i] = v[i];
    return SRHIP_OK;
  });
}

int32_t srhip_optimize_constants_cb(const srhip_trees* trees, int32_t dtype, const srhip_constopt_options* opts,
                                    srhip_constopt_eval_fn fn, void* user, void* out_consts, double* out_loss,
                                    uint8_t* out_converged, double* out_num_evals) {
  return guarded([&] {
    if (!fn) throw Error(SRHIP_ERR_INVALID, "null evaluator");
    copt::Problem pb = make_problem(trees, dtype);
    CallbackFactory fac;
    fac.fn = fn;
    fac.user = user;
    fac.const_off = &pb.const_off;
    const copt::Result r = copt::optimize(pb, make_copt_options(opts), fac);
    write_result(r, dtype, out_consts, out_loss, out_converged, out_num_evals, false);
    return SRHIP_OK;
  });
}
