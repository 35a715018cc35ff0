// fp32-faithful generation kernels (Generator precision "fp32", the C API's default).
//
// The reference computes every generation step in fp32: the matvecs (/root/reference/namegensf.cu:
// 233-242), sigmoid / tanh / Hadamard gates (:676-854), softmax (:294-300, intended semantics
// :302-313) and the inverse-CDF sampler over fp32 probabilities (:322-333).  The bf16 fast mode
// rounds the weights and hidden states to bf16, which moves CDF boundaries by ~1e-3 and flips a
// few percent of names; this path keeps fp32 end to end on the master weights (no copies):
//   * gemm_f32_nt: C = A · B^T (+ bias) on v_mfma_f32_16x16x4_f32 (true fp32 products, fp32
//     accumulate), 64 x 64 tiles of 4 waves, 16-deep k-tiles double-buffered through LDS;
//   * gru_gates_f32: r, z, n gates and h' = (1 - z) n + z h with IEEE expf / tanhf (not the fast
//     intrinsics), layer 0's input projection gathered from the fp32 table P = Emb W_ih0^T + b_ih0;
//   * sample_f32: max-subtracted fp32 softmax and the `psum > r` rule (first index whose running
//     sum exceeds r, else V - 1), EOS written then the name stops (namegensf.cu:877-882).
#include <algorithm>
#include <cstdlib>
#include "kernels.h"
#include "common.h"
#include "gen_sample.h"

namespace gk {

typedef float f32x4v __attribute__((ext_vector_type(4)));

namespace {
constexpr int kT = 64, kBK = 16, kLd = kBK + 4;   // tile, k-tile, padded LDS row (16-B aligned rows)
}

__global__ void __launch_bounds__(256) gemm_f32_nt_kernel(GemmF32Args g) {
  __shared__ __attribute__((aligned(16))) float As[2][kT][kLd];
  __shared__ __attribute__((aligned(16))) float Bs[2][kT][kLd];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * kT, n0 = blockIdx.x * kT, sp = blockIdx.z;
  const int kper = g.K / g.splits;
  const int lrow = t >> 2, lk = (t & 3) * 4;          // this thread's 16 B of each operand k-tile
  const float* pa = g.A + (size_t)(m0 + lrow) * g.lda + (size_t)sp * kper + lk;
  const float* pb = g.B + (size_t)(n0 + lrow) * g.ldb + (size_t)sp * kper + lk;
  float4 ra = *reinterpret_cast<const float4*>(pa);
  float4 rb = *reinterpret_cast<const float4*>(pb);
  *reinterpret_cast<float4*>(&As[0][lrow][lk]) = ra;
  *reinterpret_cast<float4*>(&Bs[0][lrow][lk]) = rb;
  __syncthreads();
  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;           // MFMA operand: row / column, k within 4
  const int nk = kper / kBK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {                                 // next k-tile in flight during the MFMAs
      ra = *reinterpret_cast<const float4*>(pa + (kt + 1) * kBK);
      rb = *reinterpret_cast<const float4*>(pb + (kt + 1) * kBK);
    }
#pragma unroll
    for (int kk = 0; kk < kBK / 4; ++kk) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][wm * 32 + i * 16 + fr][kk * 4 + fk];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[cur][wn * 32 + j * 16 + fr][kk * 4 + fk];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      *reinterpret_cast<float4*>(&As[cur ^ 1][lrow][lk]) = ra;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][lrow][lk]) = rb;
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 32 + j * 16 + fr;
    const float bias = (g.bias && sp == 0) ? g.bias[col] : 0.f;
    float* C = g.C + (size_t)sp * g.slab;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + fk * 4 + r;
        C[(size_t)row * g.ldc + col] = acc[i][j][r] + bias;
      }
  }
}

// Big products (batched generation: 4096 names x 3H x H per layer and char): 128 x 128 tiles, each
// wave 64 x 64 = 4 x 4 MFMA tiles (16 independent accumulator chains), half the LDS reads and
// operand traffic per MFMA of the 64 x 64 kernel; next k-tile's global loads issued before the MFMAs.
constexpr int kT2 = 128;
__global__ void __launch_bounds__(256) gemm_f32_nt128_kernel(GemmF32Args g) {
  __shared__ __attribute__((aligned(16))) float As[2][kT2][kLd];
  __shared__ __attribute__((aligned(16))) float Bs[2][kT2][kLd];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * kT2, n0 = blockIdx.x * kT2;
  const int lrow = t >> 2, lk = (t & 3) * 4;          // rows lrow and lrow + 64, 16 B each
  const float* pa = g.A + (size_t)(m0 + lrow) * g.lda + lk;
  const float* pb = g.B + (size_t)(n0 + lrow) * g.ldb + lk;
  const size_t a64 = (size_t)64 * g.lda, b64 = (size_t)64 * g.ldb;
  float4 ra0 = *reinterpret_cast<const float4*>(pa), ra1 = *reinterpret_cast<const float4*>(pa + a64);
  float4 rb0 = *reinterpret_cast<const float4*>(pb), rb1 = *reinterpret_cast<const float4*>(pb + b64);
  *reinterpret_cast<float4*>(&As[0][lrow][lk]) = ra0;
  *reinterpret_cast<float4*>(&As[0][lrow + 64][lk]) = ra1;
  *reinterpret_cast<float4*>(&Bs[0][lrow][lk]) = rb0;
  *reinterpret_cast<float4*>(&Bs[0][lrow + 64][lk]) = rb1;
  __syncthreads();
  f32x4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;
  const int nk = g.K / kBK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      const int o = (kt + 1) * kBK;
      ra0 = *reinterpret_cast<const float4*>(pa + o); ra1 = *reinterpret_cast<const float4*>(pa + a64 + o);
      rb0 = *reinterpret_cast<const float4*>(pb + o); rb1 = *reinterpret_cast<const float4*>(pb + b64 + o);
    }
#pragma unroll
    for (int kk = 0; kk < kBK / 4; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[cur][wm * 64 + i * 16 + fr][kk * 4 + fk];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[cur][wn * 64 + j * 16 + fr][kk * 4 + fk];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      *reinterpret_cast<float4*>(&As[cur ^ 1][lrow][lk]) = ra0;
      *reinterpret_cast<float4*>(&As[cur ^ 1][lrow + 64][lk]) = ra1;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][lrow][lk]) = rb0;
      *reinterpret_cast<float4*>(&Bs[cur ^ 1][lrow + 64][lk]) = rb1;
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + fr;
    const float bias = g.bias ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + fk * 4 + r;
        g.C[(size_t)row * g.ldc + col] = acc[i][j][r] + bias;
      }
  }
}

void gemm_f32_nt(const GemmF32Args& g, hipStream_t s) {
  if (g.M % kT || g.N % kT || g.splits < 1 || g.K % g.splits || (g.K / g.splits) % kBK || g.lda % 4 || g.ldb % 4 ||
      (g.splits > 1 && g.slab < (long)g.M * g.ldc))
    throw std::runtime_error("gemm_f32_nt: needs M, N % 64 == 0, (K / splits) % 16 == 0 and 16-B aligned rows");
  if (g.splits == 1 && g.M % kT2 == 0 && g.N % kT2 == 0 && (g.M / kT2) * (g.N / kT2) >= 256) {
    hipLaunchKernelGGL(gemm_f32_nt128_kernel, dim3(g.N / kT2, g.M / kT2), dim3(256), 0, s, g);
    return;
  }
  hipLaunchKernelGGL(gemm_f32_nt_kernel, dim3(g.N / kT, g.M / kT, g.splits), dim3(256), 0, s, g);
}

DEV float sigmoid_ieee(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void gru_gates_f32_kernel(GruGatesF32Args a) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)a.Bp * a.H) return;
  const int b = (int)(i / a.H), j = (int)(i % a.H), H = a.H;
  const float* gi = a.Gi + (size_t)b * 3 * H;
  if (a.P) {
    int id = a.ids[b];
    if (id < 0 || id >= a.V) {   // never expected: flag it instead of reading outside the table
      if (a.err && j == 0) {
        atomicOr(a.err, 16u);
        a.err[1] = (unsigned)id;   // diagnostics: the offending value and row
        a.err[2] = (unsigned)b;
      }
      id = 0;
    }
    gi = a.P + (size_t)id * 3 * H;
  }
  const float* gh = a.Gh + (size_t)b * 3 * H;
  float xi[3], xh[3];   // pre-activations: split-K slabs summed in slab order (deterministic)
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    xh[q] = gh[q * H + j];
    for (int s2 = 1; s2 < a.gh_splits; ++s2) xh[q] += gh[s2 * a.gh_slab + q * H + j];
    xi[q] = gi[q * H + j];
    if (!a.P)
      for (int s2 = 1; s2 < a.gi_splits; ++s2) xi[q] += gi[s2 * a.gi_slab + q * H + j];
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (a.bgh) xh[q] += a.bgh[q * H + j];
    if (a.bgi && !a.P) xi[q] += a.bgi[q * H + j];
  }
  const float r = sigmoid_ieee(xi[0] + xh[0]);
  const float z = sigmoid_ieee(xi[1] + xh[1]);
  const float n = tanhf(xi[2] + r * xh[2]);
  const float h = (1.f - z) * n + z * a.hprev[i];
  a.hout[i] = h;
  if (a.hsplit) {
    const u16 hi = f2bf(h), lo = f2bf(h - bf2f(hi));
    u16* d = a.hsplit + (size_t)b * 3 * H + j;
    d[0] = hi; d[H] = hi; d[2 * H] = lo;
  }
}

// fp32 [R][K] -> bf16 [R][3K] = [hi | lo | hi] (the weight side of a bf16x3 product)
__global__ void split_bf16x3_kernel(const float* __restrict__ src, int R, int K, u16* __restrict__ dst) {
  const long n = (long)R * K, stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const long r = i / K, k = i - r * K;
    const float x = src[i];
    const u16 hi = f2bf(x), lo = f2bf(x - bf2f(hi));
    u16* d = dst + r * 3 * K + k;
    d[0] = hi; d[K] = lo; d[2 * K] = hi;
  }
}
void split_bf16x3(const float* src, int R, int K, u16* dst, hipStream_t s) {
  const long n = (long)R * K;
  hipLaunchKernelGGL(split_bf16x3_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0, s, src, R, K, dst);
}

void gru_gates_f32(const GruGatesF32Args& a, hipStream_t s) {
  const long n = (long)a.Bp * a.H;
  hipLaunchKernelGGL(gru_gates_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

// One wave per row: lane owns V/64 consecutive logits (softmax + CDF search: gen_sample.h),
// instantiated for the exact count when V = 256 (a wider instance computes every slot)
template <int MAXPER>
__global__ void __launch_bounds__(64) sample_f32_kernel(SampleF32Args a) {
  const int b = blockIdx.x, lane = threadIdx.x, per = a.V / 64;
  if (b >= a.N) return;
  const float* x = a.logits + (size_t)b * a.V + lane * per;
  // (fixed-bound loops guarded by `per`: the arrays stay in registers)
  float xv[MAXPER];
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    if (e < per) {
      float v = x[e];
      for (int s2 = 1; s2 < a.splits; ++s2) v += x[s2 * a.slab + e];   // split-K slabs, fixed order
      if (a.bias) v += a.bias[lane * per + e];
      xv[e] = v;
    } else {
      xv[e] = -INFINITY;
    }
  }
  const float rnd = a.rf[(size_t)b * a.max_len + a.step];
  const int sel = softmax_sample_wave(xv, per, a.V, rnd, a.probs ? a.probs + (size_t)b * a.V : nullptr);
  if (lane == 0) {
    if (a.alive[b]) {
      a.out[(size_t)b * (a.max_len + 1) + a.step] = (unsigned char)sel;
      if (sel == a.eos) a.alive[b] = 0;
    }
    a.ids[b] = sel;
  }
}

__global__ void gen_reset_kernel(GenResetArgs a) {
  const long n = (long)a.Bp * a.H, stride = (long)gridDim.x * blockDim.x;
  const int hbm = a.hb_cols ? a.hb_cols / a.H : 1;   // bf16 copies per row: 1, or 3 (bf16x3 split)
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (l < a.L) {
        a.hf[l][i] = 0.f;
        if (a.hb[l])
          for (int c = 0; c < hbm; ++c) a.hb[l][(i / a.H) * (long)hbm * a.H + c * a.H + i % a.H] = 0;
      }
    }
    if (i < a.Bp) { a.ids[i] = a.sos; a.alive[i] = 1; }
    if (i < (long)a.Bp * (a.ML + 1)) a.out[i] = 0;
  }
}
void gen_reset(const GenResetArgs& a, hipStream_t s) {
  if (a.L > 4 || a.H < a.ML + 1) throw std::runtime_error("gen_reset: at most 4 layers, H > max_len");
  if (a.hb_cols && a.hb_cols != a.H && a.hb_cols != 3 * a.H) throw std::runtime_error("gen_reset: hb_cols must be H or 3H");
  hipLaunchKernelGGL(gen_reset_kernel, dim3(256), dim3(256), 0, s, a);
}

void sample_f32(const SampleF32Args& a, hipStream_t s) {
  if (a.V % 64 || a.V > 512) throw std::runtime_error("sample_f32: needs V % 64 == 0 and V <= 512");
  if (a.N <= 0) return;
  if (a.V == 256) hipLaunchKernelGGL(sample_f32_kernel<4>, dim3(a.N), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(sample_f32_kernel<8>, dim3(a.N), dim3(64), 0, s, a);
}

}  // namespace gk
