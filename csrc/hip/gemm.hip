// Plain bf16 GEMMs of the training step on hipBLASLt, with per-shape
// algorithm selection that is MEASURED on the MI355X instead of taken from
// the library's heuristic.
//
// The Llama-3-8B step issues ~15 distinct GEMM forms (5 projections x
// forward / dgrad / wgrad-accumulate); hipBLASLt's default pick for them runs
// at 1.0-1.6 PF/s (scripts/gemm_bench.py).  toa_gemm_tune() times every
// solution hipBLASLt has for a form (getAllAlgos, two passes: 1 rep each,
// then the best 8 at 10 reps) and records the winner's solution index;
// tf_operator_amd/ops/gemm.py persists the table (ops/gemm_tuning_gfx950.json)
// and re-installs it at start-up with toa_gemm_set_algo(), so training never
// tunes.  Forms without an entry use the library heuristic.
//
// Column-major BLAS convention (D = alpha op(A) op(B) + beta C, D m x n).
// The row-major wrappers in ops/gemm.py map
//   Y = X W^T  -> D^T = op_T(W) op_N(X)     (m=N, n=M, k=K)
//   dX = dY W  -> D^T = op_N(W) op_N(dY)    (m=K, n=M, k=N)
//   dW += dY^T X -> D^T = op_N(X) op_T(dY)  (m=K, n=N, k=M, beta=1)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

typedef std::tuple<int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int> Key;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool has_algo = false;
  bool ran = false;
  int index = -1;
};

struct Ctx {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  size_t ws_size = 0;
  int device = -1;
  std::map<Key, Plan> plans;
  std::map<Key, int> wanted;  // installed tuned indices, resolved lazily
  // solution index -> algo, filled by ONE getAlgosFromIndex call for every
  // installed index (a call per form cost ~30 ms each in the first step)
  std::map<int, hipblasLtMatmulAlgo_t> by_index;
  bool by_index_built = false;
  std::mutex mu;
};

Ctx& ctx() {
  static Ctx c;
  return c;
}

// TOA_GEMM_TRACE=1: host time of each first-use phase on stderr (the GEMM
// layer's share of a job's submit -> first step)
bool trace_on() {
  static const bool on = [] {
    const char* e = std::getenv("TOA_GEMM_TRACE");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

struct PhaseTimer {
  const char* what;
  std::chrono::steady_clock::time_point t0;
  explicit PhaseTimer(const char* w) : what(w), t0(std::chrono::steady_clock::now()) {}
  ~PhaseTimer() {
    if (what != nullptr && trace_on())
      std::fprintf(stderr, "[toa_gemm] %s %.2f ms\n", what,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};

hipblasOperation_t op_of(int t) { return t ? HIPBLAS_OP_T : HIPBLAS_OP_N; }

int ensure_handle(Ctx& c) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (c.h != nullptr && c.device == dev) return 0;
  PhaseTimer t("hipblasLtCreate+workspace");
  if (hipblasLtCreate(&c.h) != HIPBLAS_STATUS_SUCCESS) return 1;
  c.ws_size = 256ull << 20;  // 256 MB: stream-K / split-K solutions need room
  if (hipMalloc(&c.ws, c.ws_size) != hipSuccess) {
    c.ws = nullptr;
    c.ws_size = 0;
  }
  c.device = dev;
  return 0;
}

// out_bf16: D type bf16 (else fp32)
Plan& plan_for(Ctx& c, const Key& k) {
  auto it = c.plans.find(k);
  if (it != c.plans.end()) return it->second;
  Plan p;
  const int ta = std::get<0>(k), tb = std::get<1>(k), out_f32 = std::get<9>(k);
  const int64_t m = std::get<2>(k), n = std::get<3>(k), kk = std::get<4>(k);
  const int64_t lda = std::get<5>(k), ldb = std::get<6>(k), ldc = std::get<7>(k);
  hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  hipblasOperation_t oa = op_of(ta), ob = op_of(tb);
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ta ? kk : m, ta ? m : kk, lda);
  hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, tb ? n : kk, tb ? kk : n, ldb);
  hipblasLtMatrixLayoutCreate(&p.c, out_f32 ? HIP_R_32F : HIP_R_16BF, m, n, ldc);
  return c.plans.emplace(k, p).first->second;
}

bool supported(Ctx& c, Plan& p, hipblasLtMatmulAlgo_t& algo, float beta) {
  const float alpha = 1.f;
  size_t ws = 0;
  if (hipblaslt_ext::matmulIsAlgoSupported(c.h, p.desc, &alpha, p.a, p.b, &beta, p.c, p.c, algo, ws) !=
      HIPBLAS_STATUS_SUCCESS)
    return false;
  return ws <= c.ws_size;
}

// Stream-K solutions (kernel names with _SK<n>, n > 0) run a persistent grid
// of one workgroup per CU holding the whole register file, so a collective
// kernel on another stream gets no CU until the GEMM ends -- or, once
// resident, delays one of the GEMM's workgroups by the collective's whole
// duration (profiles/r2_sk_contention, profiles/r3_overlap).
bool is_streamk(const std::string& kname) {
  for (size_t p = kname.find("_SK"); p != std::string::npos; p = kname.find("_SK", p + 1))
    if (p + 3 < kname.size() && kname[p + 3] >= '1' && kname[p + 3] <= '9') return true;
  return false;
}

// policy: untuned forms take the heuristic's best NON-stream-K solution
bool g_no_streamk = false;

int resolve(Ctx& c, const Key& k, Plan& p, float beta) {
  if (p.has_algo) return 0;
  auto w = c.wanted.find(k);
  if (w != c.wanted.end()) {
    if (!c.by_index_built || c.by_index.find(w->second) == c.by_index.end()) {
      std::vector<int> idx;
      for (const auto& kv : c.wanted)
        if (c.by_index.find(kv.second) == c.by_index.end()) idx.push_back(kv.second);
      std::sort(idx.begin(), idx.end());
      idx.erase(std::unique(idx.begin(), idx.end()), idx.end());
      // Most of this call's ~0.47 s is loading the chosen solutions' code
      // objects; a typed getAllAlgos lookup only moves that into
      // matmulIsAlgoSupported (0.27 + 0.36 s, profiles/r3_first), so
      // toa_gemm_prewarm() takes it off the first step instead.
      std::vector<hipblasLtMatmulHeuristicResult_t> res;
      PhaseTimer t(idx.empty() ? nullptr : "getAlgosFromIndex");
      if (!idx.empty() && hipblaslt_ext::getAlgosFromIndex(c.h, idx, res) == HIPBLAS_STATUS_SUCCESS)
        for (const auto& r : res) c.by_index[hipblaslt_ext::getIndexFromAlgo(const_cast<hipblasLtMatmulAlgo_t&>(r.algo))] = r.algo;
      c.by_index_built = true;
    }
    auto a = c.by_index.find(w->second);
    PhaseTimer t("matmulIsAlgoSupported");
    if (a != c.by_index.end() && supported(c, p, a->second, beta)) {
      p.algo = a->second;
      p.has_algo = true;
      p.index = w->second;
      return 0;
    }
  }
  PhaseTimer t("heuristic");
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsz = c.ws_size;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
  hipblasLtMatmulHeuristicResult_t r[16];
  int got = 0;
  hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(c.h, p.desc, p.a, p.b, p.c, p.c, pref, g_no_streamk ? 16 : 1, r, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || got == 0) return 2;
  int pick = 0;
  if (g_no_streamk)
    for (int i = 0; i < got; ++i)
      if (!is_streamk(hipblaslt_ext::getKernelNameFromAlgo(c.h, r[i].algo))) {
        pick = i;
        break;
      }
  p.algo = r[pick].algo;
  p.has_algo = true;
  p.index = hipblaslt_ext::getIndexFromAlgo(p.algo);
  return 0;
}

int run(Ctx& c, Plan& p, hipblasLtMatmulAlgo_t& algo, const void* A, const void* B, void* C, float beta,
        hipStream_t s) {
  const float alpha = 1.f;
  PhaseTimer t(p.ran ? nullptr : "first hipblasLtMatmul");
  p.ran = true;
  return hipblasLtMatmul(c.h, p.desc, &alpha, A, p.a, B, p.b, &beta, C, p.c, C, p.c, &algo, c.ws, c.ws_size, s) ==
                 HIPBLAS_STATUS_SUCCESS
             ? 0
             : 3;
}

}  // namespace

// D (= C) = op(A) op(B) + beta C ; bf16 A/B, bf16 or fp32 C/D, fp32 accumulate.
extern "C" int toa_gemm(int ta, int tb, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda, const void* B,
                        int64_t ldb, void* C, int64_t ldc, float beta, int out_f32, hipStream_t stream) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  if (ensure_handle(c)) return 1;
  const Key key{ta, tb, m, n, k, lda, ldb, ldc, beta != 0.f, out_f32};
  Plan& p = plan_for(c, key);
  if (int e = resolve(c, key, p, beta)) return e;
  return run(c, p, p.algo, A, B, C, beta, stream);
}

// Install a tuned solution index for a form (from the persisted table).
extern "C" int toa_gemm_set_algo(int ta, int tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                                 int64_t ldc, int beta_nz, int out_f32, int index) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  const Key key{ta, tb, m, n, k, lda, ldb, ldc, beta_nz, out_f32};
  c.wanted[key] = index;
  auto it = c.plans.find(key);
  if (it != c.plans.end()) it->second.has_algo = false;
  return 0;
}

// Index of the solution a form currently runs (-1 if not resolved yet).
extern "C" int toa_gemm_current_algo(int ta, int tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                                     int64_t ldc, int beta_nz, int out_f32) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  auto it = c.plans.find(Key{ta, tb, m, n, k, lda, ldb, ldc, beta_nz, out_f32});
  return (it == c.plans.end() || !it->second.has_algo) ? -1 : it->second.index;
}

// Time every hipBLASLt solution for a form on the given (scratch) buffers and
// keep the fastest.  Returns 0 and writes the winner's index / ms, the
// heuristic default's ms, and the number of candidates timed.
//
// exclude_streamk: skip stream-K solutions (is_streamk above); the
// data-parallel (world > 1) policy tunes without them.
extern "C" int toa_gemm_tune(int ta, int tb, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                             const void* B, int64_t ldb, void* C, int64_t ldc, float beta, int out_f32,
                             hipStream_t stream, int* best_index, float* best_ms, float* default_ms,
                             int* n_timed, int exclude_streamk) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  if (ensure_handle(c)) return 1;
  const Key key{ta, tb, m, n, k, lda, ldb, ldc, beta != 0.f, out_f32};
  Plan& p = plan_for(c, key);
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  if (hipblaslt_ext::getAllAlgos(c.h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, op_of(ta), op_of(tb), HIP_R_16BF,
                                 HIP_R_16BF, out_f32 ? HIP_R_32F : HIP_R_16BF, out_f32 ? HIP_R_32F : HIP_R_16BF,
                                 HIPBLAS_COMPUTE_32F, all) != HIPBLAS_STATUS_SUCCESS)
    return 4;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // Cold-cache timing: in the training step every GEMM streams operands that
  // the previous kernels evicted from L2 and the 256 MB Infinity Cache, so
  // each timed rep is preceded by a 512 MB write that flushes both (timing
  // back-to-back reps on hot buffers picked solutions that lost in-model).
  static void* flush = nullptr;
  const size_t flush_bytes = 512ull << 20;
  if (flush == nullptr && hipMalloc(&flush, flush_bytes) != hipSuccess) flush = nullptr;
  auto time_it = [&](hipblasLtMatmulAlgo_t& algo, int reps) -> float {
    if (run(c, p, algo, A, B, C, beta, stream)) return 1e30f;  // warm-up / launch check
    float total = 0.f;
    for (int i = 0; i < reps; ++i) {
      if (flush != nullptr) (void)hipMemsetAsync(flush, i & 0xff, flush_bytes, stream);
      (void)hipEventRecord(e0, stream);
      run(c, p, algo, A, B, C, beta, stream);
      (void)hipEventRecord(e1, stream);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      total += ms;
    }
    return total / reps;
  };
  // the heuristic default, for the report
  Plan dflt = p;
  dflt.has_algo = false;
  c.wanted.erase(key);
  float dms = 1e30f;
  if (resolve(c, key, dflt, beta) == 0) dms = time_it(dflt.algo, 10);
  std::vector<std::pair<float, size_t>> first;
  for (size_t i = 0; i < all.size(); ++i) {
    if (!supported(c, p, all[i].algo, beta)) continue;
    if (exclude_streamk && is_streamk(hipblaslt_ext::getKernelNameFromAlgo(c.h, all[i].algo))) continue;
    first.emplace_back(time_it(all[i].algo, 2), i);
  }
  std::sort(first.begin(), first.end());
  const bool dflt_ok = dflt.has_algo && !(exclude_streamk && is_streamk(hipblaslt_ext::getKernelNameFromAlgo(c.h, dflt.algo)));
  float bms = dflt_ok ? dms : 1e30f;
  int bidx = dflt_ok ? dflt.index : -1;
  hipblasLtMatmulAlgo_t balgo = dflt.algo;
  for (size_t j = 0; j < first.size() && j < 8; ++j) {
    const float ms = time_it(all[first[j].second].algo, 10);
    if (ms < bms) {
      bms = ms;
      balgo = all[first[j].second].algo;
      bidx = hipblaslt_ext::getIndexFromAlgo(balgo);
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  p.algo = balgo;
  p.has_algo = bidx >= 0;
  p.index = bidx;
  if (bidx >= 0) c.wanted[key] = bidx;
  *best_index = bidx;
  *best_ms = bms;
  *default_ms = dms;
  *n_timed = (int)first.size();
  return 0;
}

// Kernel name of the solution a form runs (resolved on first use); "" if
// the form was never run.  Returns the name's length.
extern "C" int toa_gemm_kernel_name(int ta, int tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                                    int64_t ldc, int beta_nz, int out_f32, char* buf, int buflen) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  auto it = c.plans.find(Key{ta, tb, m, n, k, lda, ldb, ldc, beta_nz, out_f32});
  std::string name;
  if (it != c.plans.end() && it->second.has_algo && c.h != nullptr)
    name = hipblaslt_ext::getKernelNameFromAlgo(c.h, it->second.algo);
  if (buf != nullptr && buflen > 0) {
    const size_t nn = std::min((size_t)buflen - 1, name.size());
    std::memcpy(buf, name.data(), nn);
    buf[nn] = 0;
  }
  return (int)name.size();
}

// Policy for forms without a tuned entry: 1 = the heuristic's best
// non-stream-K solution (forms already resolved keep theirs).
extern "C" int toa_gemm_set_no_streamk(int on) {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  g_no_streamk = on != 0;
  return 0;
}

// Resolve every installed form's plan now (handle + workspace, ONE batched
// index lookup, per-form support checks) instead of inside the first step.
// Host-side work only -- no kernel runs -- so ops/gemm.py calls it from a
// helper thread while the model's weights are being initialised.  Returns
// the number of installed forms that resolved.
extern "C" int toa_gemm_prewarm() {
  Ctx& c = ctx();
  std::lock_guard<std::mutex> g(c.mu);
  if (ensure_handle(c)) return -1;
  PhaseTimer t("prewarm");
  int ok = 0;
  for (const auto& kv : c.wanted) {
    Plan& p = plan_for(c, kv.first);
    if (resolve(c, kv.first, p, std::get<8>(kv.first) ? 1.f : 0.f) == 0) ++ok;
  }
  return ok;
}
