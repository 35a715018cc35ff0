// Probe: hipBLASLt (bf16 x bf16 -> fp32, TN) on the engine's large plain GEMMs, with and without
// the BGRADB (row-sum) epilogue, against sampled fp64 host dot products.  Decides whether the
// large weight-gradient GEMMs go to the library (csrc/runtime/blaslt.cpp).
//   hipcc --offload-arch=gfx950 -O2 scripts/probe_blaslt.cpp -lhipblaslt -o probe_blaslt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define BK(x) do { auto e_ = (x); if (e_ != HIPBLAS_STATUS_SUCCESS) { printf("BLAS %d @%d\n", (int)e_, __LINE__); return -1.0;} } while (0)

static unsigned short f2bf(float f) { unsigned u; memcpy(&u, &f, 4); return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
static float bf2f(unsigned short h) { unsigned u = (unsigned)h << 16; float f; memcpy(&f, &u, 4); return f; }

// C[M][N] (row-major, ldc=N) = A[M][K] . B[N][K]^T ; returns us per call or <0 if no algo
static double run(hipblasLtHandle_t h, int M, int N, int K, bool rowsum, int* nalgo, double* err, double* rserr) {
  std::vector<unsigned short> hA((size_t)M * K), hB((size_t)N * K);
  unsigned s = 12345;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 32768.f - 1.f; };
  for (auto& x : hA) x = f2bf(rnd());
  for (auto& x : hB) x = f2bf(rnd());
  void *dA, *dB, *dC, *ws, *dR;
  const size_t wsz = 64ull << 20;
  CK(hipMalloc(&dA, hA.size() * 2)); CK(hipMalloc(&dB, hB.size() * 2));
  CK(hipMalloc(&dC, (size_t)M * N * 4)); CK(hipMalloc(&ws, wsz)); CK(hipMalloc(&dR, (size_t)M * 4));
  CK(hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
  hipblasLtMatmulDesc_t op;
  BK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
  BK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA)));
  BK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB)));
  if (rowsum) {
    hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BGRADB;
    int32_t bt = HIP_R_32F;
    BK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    BK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dR, sizeof(dR)));
    BK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  hipblasLtMatrixLayout_t la, lb, lc;
  BK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K));   // our B as column-major K x N
  BK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K));   // our A as column-major K x M
  BK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, N, M, N));    // our C as column-major N x M
  hipblasLtMatmulPreference_t pref;
  BK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t w64 = wsz;
  BK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w64, sizeof(w64)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  hipblasLtMatmulAlgoGetHeuristic(h, op, la, lb, lc, lc, pref, 8, res, &n);
  *nalgo = n;
  if (n == 0) return -1.0;
  const float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  double best = 1e30;
  for (int a = 0; a < n && a < 4; ++a) {
    for (int w = 0; w < 3; ++w)
      BK(hipblasLtMatmul(h, op, &alpha, dB, la, dA, lb, &beta, dC, lc, dC, lc, &res[a].algo, ws, wsz, 0));
    CK(hipEventRecord(e0, 0));
    const int it = 10;
    for (int i = 0; i < it; ++i)
      BK(hipblasLtMatmul(h, op, &alpha, dB, la, dA, lb, &beta, dC, lc, dC, lc, &res[a].algo, ws, wsz, 0));
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms * 1e3 / it < best) best = ms * 1e3 / it;
  }
  std::vector<float> hC((size_t)M * N), hR(M);
  CK(hipMemcpy(hC.data(), dC, hC.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hR.data(), dR, hR.size() * 4, hipMemcpyDeviceToHost));
  double me = 0, mr = 0;
  for (int t = 0; t < 64; ++t) {
    const int i = (t * 7919) % M, j = (t * 104729) % N;
    double ref = 0;
    for (int k = 0; k < K; ++k) ref += (double)bf2f(hA[(size_t)i * K + k]) * bf2f(hB[(size_t)j * K + k]);
    me = fmax(me, fabs(ref - hC[(size_t)i * N + j]) / sqrt((double)K));
    if (rowsum) {
      double rs = 0;
      for (int k = 0; k < K; ++k) rs += bf2f(hA[(size_t)i * K + k]);
      mr = fmax(mr, fabs(rs - hR[i]) / sqrt((double)K));
    }
  }
  *err = me; *rserr = mr;
  hipFree(dA); hipFree(dB); hipFree(dC); hipFree(ws); hipFree(dR);
  return best;
}

int main(int argc, char** argv) {
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) { printf("create failed\n"); return 1; }
  struct S { const char* name; int M, N, K; } shapes[] = {
      {"h2048.dW_hh", 6144, 2048, 65536}, {"h2048.dW_ih", 6144, 512, 65536}, {"h2048.dH", 65536, 2048, 256},
      {"h1024.dWhh", 3072, 1024, 8192}, {"h1024.Gi", 8192, 3072, 1024}, {"sq4096", 4096, 4096, 4096}};
  // optional: M N K triples on the command line (no row-sum variant)
  std::vector<S> custom;
  for (int i = 1; i + 2 < argc; i += 3) custom.push_back({"custom", atoi(argv[i]), atoi(argv[i + 1]), atoi(argv[i + 2])});
  std::vector<S> list = custom.empty() ? std::vector<S>(std::begin(shapes), std::end(shapes)) : custom;
  for (auto& sh : list)
    for (int rs = 0; rs < (custom.empty() ? 2 : 1); ++rs) {
      int na = 0; double err = 0, rserr = 0;
      const double us = run(h, sh.M, sh.N, sh.K, rs, &na, &err, &rserr);
      const double tf = us > 0 ? 2.0 * sh.M * sh.N * (double)sh.K / us / 1e6 : 0;
      printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"rowsum\": %d, \"algos\": %d, \"us\": %.1f, "
             "\"tflops\": %.1f, \"err_per_sqrtK\": %.2e, \"rowsum_err\": %.2e}\n",
             sh.name, sh.M, sh.N, sh.K, rs, na, us, tf, err, rserr);
      fflush(stdout);
    }
  hipblasLtDestroy(h);
  return 0;
}
