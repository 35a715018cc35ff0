// Generic bf16 "NT" MFMA GEMM  C[M][N] = A[M][K] · B[N][K]^T  with fp32 accumulate.
//
// Used for every non-recurrent product of the engine:
//   * P = Emb·W_ih0^T + b_ih0        (the layer-0 input projection folded into a V x 3H table)
//   * Gi = H_below·W_ih^T + b_ih      (hoisted input projection, layers >= 1)
//   * dH = dlogits·W_fc,  dX = dGi·W_ih
//   * weight gradients  dW = dG^T·H  over all B·T tokens (split-K partial slabs, one slab per
//     time chunk so they run on a side stream while the serial recurrence continues), with the
//     bias gradient as the fused row sum of A, and the one-hot A of the embedding gradient
//     generated from the char ids on the fly (no gather/scatter, no float atomics:
//     bitwise-deterministic).
// Tile 64x64 per 4-wave workgroup (2x2 waves of 32x32 = 2x2 MFMA 16x16x32 tiles), operands
// straight to VGPRs with a two-batch software pipeline (mma_tile.h), XCD-aware bijective
// block remap so tiles sharing an operand panel share an L2 (cdna_hip_programming.md T1).
#include <stdexcept>
#include "kernels.h"
#include "mma_tile.h"
#include "../runtime/blaslt.h"

namespace gk {

[[noreturn]] static void throw_gemm_shape() {
  throw std::runtime_error("gemm_nt: LDS kernel requested for an unsupported shape/alignment");
}

DEV int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int KB, bool ONEHOT, bool ROWSUM>
__global__ void __launch_bounds__(256) gemm_nt_kernel(GemmArgs a, int ntn, int ntm, int kper) {
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tn = id % ntn;
  const int tm = (id / ntn) % ntm;
  const int sp = id / (ntn * ntm);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  const int m0 = tm * 64 + wm * 32, n0 = tn * 64 + wn * 32;
  const int kbeg = sp * kper;
  const int nks = kper / 32;

  f32x4 acc[2][2];
  zero_acc(acc);
  float rs[2] = {0.f, 0.f};
  const u16* B = a.B + (size_t)(n0 + lr) * a.ldb + kbeg + lk;
  if constexpr (ONEHOT) {
    // A[m][k] = (ids[k] == m): 8 ids per lane per k-step compared against the lane's two rows.
    // ids and B fragments for k-step ks+1 are in flight while k-step ks computes.
    const int* ids = a.onehot_ids + kbeg + lk;
    auto ldids = [&](int ks, int4& i0, int4& i1) {
      i0 = *reinterpret_cast<const int4*>(ids + ks * 32);
      i1 = *reinterpret_cast<const int4*>(ids + ks * 32 + 4);
    };
    auto ldb = [&](int ks, bf16x8 (&bf)[2]) {
#pragma unroll
      for (int c = 0; c < 2; ++c) bf[c] = ld8(B + (size_t)c * 16 * a.ldb + ks * 32);
    };
    auto step = [&](const int4& i0, const int4& i1, const bf16x8 (&bf)[2]) {
      const int idv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int row = m0 + r * 16 + lr;
        bf16x8 af;
#pragma unroll
        for (int e = 0; e < 8; ++e) af[e] = (__bf16)(idv[e] == row ? 1.0f : 0.0f);
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[r][c] = mfma16(af, bf[c], acc[r][c]);
      }
    };
    int4 x0, x1, y0, y1;
    bf16x8 b0[2], b1[2];
    ldids(0, x0, x1); ldb(0, b0);
    int ks = 0;
    for (; ks + 2 <= nks; ks += 2) {
      ldids(ks + 1, y0, y1); ldb(ks + 1, b1);
      step(x0, x1, b0);
      if (ks + 2 < nks) { ldids(ks + 2, x0, x1); ldb(ks + 2, b0); }
      step(y0, y1, b1);
    }
    if (ks < nks) step(x0, x1, b0);
  } else {
    const u16* A = a.A + (size_t)(m0 + lr) * a.lda + kbeg + lk;
    // bias gradient = row sums of A, from the fragments already loaded (tn == 0 tiles, wave column 0)
    const bool do_rs = ROWSUM && tn == 0 && wn == 0;
    MmaLoop<2, 2, KB>::run(acc, A, a.lda, B, 16 * a.ldb, nks, rs, do_rs);
  }

  // epilogue: lane (l&15) = column, rows (l>>4)*4 + i
  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = n0 + c * 16 + lr;
      const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + r * 16 + (lane >> 4) * 4 + i;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[r][c][i] + bb;
        if (a.accumulate) *dst += v; else *dst = v;
      }
    }
  if constexpr (ROWSUM && !ONEHOT) {
    if (tn == 0 && wn == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        float v = rs[r];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) a.rowsumA[(size_t)sp * a.M + m0 + r * 16 + lane] = v;
      }
    }
  }
}

// Row sums of a bf16 [M][K] matrix (the bias gradient that rides along a library GEMM): one
// 256-thread workgroup per row, 16-B loads four deep, fixed-order wave + LDS reduction
// (deterministic).  Needs K % 8 == 0, lda % 8 == 0 and a 16-B aligned A.
__global__ void __launch_bounds__(256) rowsum_bf16_kernel(const u16* __restrict__ A, int lda, int K,
                                                          float* __restrict__ out) {
  const uint4* row = reinterpret_cast<const uint4*>(A + (size_t)blockIdx.x * lda);
  const int n8 = K / 8;
  float acc = 0.f;
  int i = threadIdx.x;
  auto add8 = [&](uint4 q) {
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += __uint_as_float(w[e] << 16) + __uint_as_float(w[e] & 0xffff0000u);
  };
  for (; i + 3 * 256 < n8; i += 4 * 256) {
    const uint4 q0 = row[i], q1 = row[i + 256], q2 = row[i + 512], q3 = row[i + 768];
    add8(q0); add8(q1); add8(q2); add8(q3);
  }
  for (; i < n8; i += 256) add8(row[i]);
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

bool gemm_library_ok(const GemmArgs& a) {
  if (a.onehot_ids || a.bias || a.splits != 1 || !a.A || !a.B || !a.C) return false;
  if (a.rowsumA && (a.K % 8 || a.lda % 8 || reinterpret_cast<uintptr_t>(a.A) % 16)) return false;
  return a.M > 0 && a.N > 0 && a.K > 0;
}

bool gemm_library_wanted(const GemmArgs& a) {
  if (a.algo == 4) return true;
  if (a.algo != 0 || !blaslt_enabled() || 2.0 * a.M * a.N * (double)a.K < blaslt_min_gflop() * 1e9) return false;
  // with the bias row sum the library pays a second pass over A (5.5 TB/s): worth it only where
  // the LDS kernel's split-K slabs get big -- dW_hh at H = 2048 (6144 x 2048: 1.90 -> 1.25 + 0.15 ms);
  // at H = 1024 (3072 x 1024, K = 65536) the two GEMMs tie and the row sum is pure loss
  // (profiles/r1_blaslt_ab.jsonl).  GK_BLASLT=all lifts this too (tests).
  if (a.rowsumA && (double)a.M * a.N < 8e6 && blaslt_min_gflop() > 0) return false;
  return true;
}

void rowsum_bf16(const u16* A, int lda, int M, int K, float* out, hipStream_t s) {
  hipLaunchKernelGGL(rowsum_bf16_kernel, dim3(M), dim3(256), 0, s, A, lda, K, out);
}

bool gemm_library(const GemmArgs& a, hipStream_t s) {
  if (!gemm_library_ok(a)) return false;
  if (!blaslt_gemm_nt(a.A, a.lda, a.B, a.ldb, a.C, a.ldc, a.M, a.N, a.K, a.accumulate != 0, s)) return false;
  if (a.rowsumA) hipLaunchKernelGGL(rowsum_bf16_kernel, dim3(a.M), dim3(256), 0, s, a.A, a.lda, a.K, a.rowsumA);
  return true;
}

void gemm_nt(const GemmArgs& a, hipStream_t s) {
  if (a.B2 && !gemm_lds_ok(a) && !(gemm_variants().onehot && onehot_dp_ok(a)))
    throw std::runtime_error("gemm_nt: a split B operand (B2) needs a one-hot LDS / streaming kernel");
  // large plain products: hipBLASLt (bf16 in, fp32 out), when it has an algorithm for the shape
  if (gemm_library_wanted(a) && gemm_library(a, s)) return;
  if (a.algo == 4) throw std::runtime_error("gemm_nt: library GEMM requested but not available for this shape");
  if (a.algo == 5) {
    if (!gemm256_ok(a)) throw_gemm_shape();
    gemm256(a, s);
    return;
  }
  if (a.algo == 3) {
    if (!gemm_small_kblocks(a)) throw_gemm_shape();
    gemm_small(a, s);
    return;
  }
  // large plain products (a full wave of 256 x 256 tiles): the 256 x 256 LDS kernel
  if (a.algo == 0 && a.splits == 1 && gemm256_ok(a) && (a.M / 256) * (a.N / 256) >= 256 && a.K >= 256) {
    gemm256(a, s);
    return;
  }
  // one-hot dP over the whole vocabulary (V = 256): the streaming kernel reads G once
  if ((a.algo == 0 || a.algo == 2) && a.onehot_ids && gemm_variants().onehot && onehot_dp_ok(a)) {
    onehot_dp(a, s);
    return;
  }
  // latency-bound regime (fewer than one 128 x 128 workgroup per CU): the one-shot small kernel
  if (a.algo == 0 && gemm_small_kblocks(a) &&
      (a.M % 128 || a.N % 128 || (a.M / 128) * (a.N / 128) * a.splits < 256)) {
    gemm_small(a, s);
    return;
  }
  // the LDS-staged kernel measured faster on every engine shape it supports (scripts/bench_gemm.py)
  if (a.algo == 2 || (a.algo == 0 && gemm_lds_ok(a))) {
    if (!gemm_lds_ok(a)) throw_gemm_shape();
    gemm_lds(a, s);
    return;
  }
  const int ntn = a.N / 64, ntm = a.M / 64;
  const int kper = a.K / a.splits;
  const int nks = kper / 32;
  const int nwg = ntn * ntm * a.splits;
  const bool rsum = a.rowsumA != nullptr;
  dim3 grid(nwg), block(256);
#define GL(KBV, OH, RS) hipLaunchKernelGGL((gemm_nt_kernel<KBV, OH, RS>), grid, block, 0, s, a, ntn, ntm, kper)
  if (a.onehot_ids) { GL(1, true, false); return; }
  if (nks % 4 == 0) { if (rsum) GL(4, false, true); else GL(4, false, false); }
  else if (nks % 2 == 0) { if (rsum) GL(2, false, true); else GL(2, false, false); }
  else { if (rsum) GL(1, false, true); else GL(1, false, false); }
#undef GL
}

}  // namespace gk
