#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

namespace gk {

namespace {

constexpr size_t kWorkspace = 64ull << 20;
// one workspace per stream that calls the library: the trainer's overlapped schedule records
// library GEMMs on two streams that run concurrently inside one graph
constexpr int kSlots = 4;

struct Plan {
  bool ok = false;
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
};

struct State {
  std::mutex mu;
  int device = -1;
  hipblasLtHandle_t h = nullptr;
  void* ws[kSlots] = {};
  hipStream_t ws_stream[kSlots] = {};
  unsigned long ws_used[kSlots] = {};   // 0 = free, else last-use tick
  unsigned long tick = 0;
  std::map<std::tuple<int, int, int, int, int, int, int>, Plan> plans;
};

State& st() {
  static State s;
  return s;
}

void check(hipblasStatus_t e, const char* what) {
  if (e != HIPBLAS_STATUS_SUCCESS)
    throw std::runtime_error(std::string("hipBLASLt ") + what + " failed: status " + std::to_string((int)e));
}

void init_locked(State& s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("blaslt_init: hipGetDevice failed");
  if (s.h && s.device == dev) return;
  if (s.h) throw std::runtime_error("blaslt: one device per process (got a second device)");
  check(hipblasLtCreate(&s.h), "create");
  for (int i = 0; i < kSlots; ++i)
    if (hipMalloc(&s.ws[i], kWorkspace) != hipSuccess) throw std::runtime_error("blaslt: workspace hipMalloc failed");
  s.device = dev;
}

// Row-major C = A . B^T is column-major C^T = B . A^T: the library's matrix A is our B (K x N,
// ld ldb, transposed), its matrix B is our A (K x M, ld lda, not transposed) -- the TN layout.
Plan make_plan(State& s, int M, int N, int K, int lda, int ldb, int ldc) {
  Plan p;
  check(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F), "desc");
  hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
  check(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA)), "transA");
  check(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB)), "transB");
  check(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, ldb), "layout A");
  check(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, lda), "layout B");
  check(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_32F, N, M, ldc), "layout C");
  hipblasLtMatmulPreference_t pref;
  check(hipblasLtMatmulPreferenceCreate(&pref), "pref");
  uint64_t w = kWorkspace;
  check(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w, sizeof(w)),
        "pref workspace");
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t e = hipblasLtMatmulAlgoGetHeuristic(s.h, p.op, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (e == HIPBLAS_STATUS_SUCCESS && n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS) {
    p.ok = true;
    p.algo = res[0].algo;
  }
  return p;
}

void* workspace_for(State& s, hipStream_t stream) {
  // least-recently-used slot when a new stream shows up (engines come and go in one process;
  // at most two of their streams run library GEMMs at the same time)
  ++s.tick;
  int lru = 0;
  for (int i = 0; i < kSlots; ++i) {
    if (s.ws_used[i] && s.ws_stream[i] == stream) { s.ws_used[i] = s.tick; return s.ws[i]; }
    if (s.ws_used[i] < s.ws_used[lru]) lru = i;
  }
  s.ws_stream[lru] = stream;
  s.ws_used[lru] = s.tick;
  return s.ws[lru];
}

}  // namespace

void blaslt_init(bool force) {
  if (!force && !blaslt_enabled()) return;
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  init_locked(s);
}

// GK_BLASLT=1 sends the plain (non-weight-gradient) GEMMs gemm_library_wanted() picks of >= 60 GFLOP
// to the library, GK_BLASLT=all every eligible one; off by default (the hand-written gemm256 takes
// them).  Separately, GK_WGRAD_GEMM=lib
// routes the largest weight-gradient products (>= 8 M outputs and >= 60 GFLOP: dW_hh at H = 2048) to
// the library (trainer_seq.cpp wgrad_engine); by default gemm256 takes those too.
bool blaslt_enabled() {
  const char* e = std::getenv("GK_BLASLT");
  return e && (e[0] == '1' || std::strcmp(e, "all") == 0);
}

double blaslt_min_gflop() {
  const char* e = std::getenv("GK_BLASLT");
  return e && std::strcmp(e, "all") == 0 ? 0.0 : 60.0;
}

bool blaslt_gemm_nt(const u16* A, int lda, const u16* B, int ldb, float* C, int ldc, int M, int N, int K,
                    bool accumulate, hipStream_t stream) {
  // (the policy -- blaslt_enabled / gemm_library_wanted -- is the caller's; algo 4 forces a call)
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  init_locked(s);   // no-op after blaslt_init(); never allocates inside a capture then
  auto key = std::make_tuple(M, N, K, lda, ldb, ldc, 0);
  auto it = s.plans.find(key);
  if (it == s.plans.end()) it = s.plans.emplace(key, make_plan(s, M, N, K, lda, ldb, ldc)).first;
  const Plan& p = it->second;
  if (!p.ok) return false;
  const float alpha = 1.f, beta = accumulate ? 1.f : 0.f;
  check(hipblasLtMatmul(s.h, p.op, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo, workspace_for(s, stream), kWorkspace,
                        stream),
        "matmul");
  return true;
}

}  // namespace gk
