// One-shot small GEMM for the latency-bound products of the h512 step: the layer-0 P table
// (256 x 1536 x 512), dW_ih0 / dEmb (1536 x 512 x 256, 256 x 512 x 1536) and the split-K dW_fc
// (256 x 512 x 8192).  With 128 x 128 tiles these give 24-256 workgroups that each walk 3-8
// dependent 64-deep k-tiles, every one a full memory round trip (profiles: 7-10 us per launch).
// Here a 64 x 64 tile stages its WHOLE K-slice (<= 512) into LDS with one burst of LDS-DMA
// (global_load_lds_dwordx4, the XOR-swizzled image of gemm_lds.hip per 64-deep block), waits once,
// then runs all its MFMAs: one memory latency per workgroup instead of one per k-tile, and 4x the
// workgroups of the 128 x 128 kernel.
//   * 256 threads = 2 x 2 waves of 32 x 32 (2 x 2 MFMA 16x16x32 tiles);
//   * LDS: NKB x (64 + 64) rows x 128 B = NKB x 16 KiB (NKB <= 8: two workgroups per CU up to 4);
//   * split-K slabs, fused bias (unsplit) and fused row sums of A as in gemm_lds;
//   * grouped launch for several independent products (dW_ih0 and dEmb share one).
#include <algorithm>
#include <stdexcept>
#include <string>
#include "kernels.h"
#include "common.h"

namespace gk {

typedef __attribute__((address_space(3))) void lds_void_s;

DEV int xcd_remap_s(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// NCH > 1 (K-slices of NCH x 512): the slice is streamed as NCH bursts of 8 blocks through the same
// LDS (one memory latency per 512-deep chunk instead of one per 64-deep k-tile).
template <int NKB, bool BIAS, bool ROWSUM>
DEV void gemm_small_body(const GemmArgs& a, int id, int ntn, int ntm, u16 (*lds)[2][64 * 64], int nch = 1) {
  const int tn = id % ntn, tm = (id / ntn) % ntm, sp = id / (ntn * ntm);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int row0 = tm * 64, col0 = tn * 64;
  const int srow = lane >> 3, sslot = lane & 7;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_rs = ROWSUM && a.rowsumA && tn == 0 && wn == 0;
  float rs[2] = {0.f, 0.f};
  for (int ch = 0; ch < nch; ++ch) {
  const int kbeg = (sp * nch + ch) * NKB * 64;
  if (ch) __syncthreads();   // every wave is done reading the previous chunk
  // the whole chunk in one burst: per 64-deep block, wave w stages rows 16w .. 16w+15 of A and B
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = w * 16 + q * 8 + srow;
      const int c = sslot ^ ((r >> 1) & 7);
      const size_t ko = (size_t)kbeg + kb * 64 + c * 8;
      if (!a.A32)
        __builtin_amdgcn_global_load_lds(a.A + (size_t)(row0 + r) * a.lda + ko,
                                         (lds_void_s*)(&lds[kb][0][(w * 16 + q * 8) * 64]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(a.B + (size_t)(col0 + r) * a.ldb + ko,
                                       (lds_void_s*)(&lds[kb][1][(w * 16 + q * 8) * 64]), 16, 0, 0);
    }
  if (a.A32) {
    // fp32 A: float4 loads, rounded to bf16 into the same swizzled image (chunk c of row r in slot
    // c ^ ((r >> 1) & 7)); per 64 x 64 block 1024 float4, 4 per thread
    const int tid = threadIdx.x;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int q = tid + 256 * p;
        if (!a.a32_trans) {   // row r, k 4q4 .. +3 of the block (8-B LDS writes)
          const int r = q >> 4, k4 = (q & 15) * 4;
          const float4 v = *reinterpret_cast<const float4*>(a.A32 + (size_t)(row0 + r) * a.lda + kbeg + kb * 64 + k4);
          const int c = (k4 >> 3) ^ ((r >> 1) & 7);
          uint2 u;
          u.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
          u.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
          *reinterpret_cast<uint2*>(&lds[kb][0][r * 64 + c * 8 + (k4 & 7)]) = u;
        } else {              // A32[k][m]: k = q / 16 of the block, rows m 4(q % 16) .. +3
          const int k = q >> 4, m4 = (q & 15) * 4;
          const float4 v = *reinterpret_cast<const float4*>(a.A32 + (size_t)(kbeg + kb * 64 + k) * a.lda + row0 + m4);
          const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = m4 + i, c = (k >> 3) ^ ((r >> 1) & 7);
            lds[kb][0][r * 64 + c * 8 + (k & 7)] = f2bf(e[i]);
          }
        }
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + lq;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ra = wm * 32 + t * 16 + lr, rb = wn * 32 + t * 16 + lr;
        af[t] = *reinterpret_cast<const bf16x8*>(&lds[kb][0][ra * 64 + ((c ^ ((ra >> 1) & 7)) * 8)]);
        bfr[t] = *reinterpret_cast<const bf16x8*>(&lds[kb][1][rb * 64 + ((c ^ ((rb >> 1) & 7)) * 8)]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      if (do_rs) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 8; ++e) rs[t] += (float)af[t][e];
      }
    }
  }

  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = col0 + wn * 32 + j * 16 + lr;
    const float bb = BIAS ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + wm * 32 + i * 16 + lq * 4 + e;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[i][j][e] + bb;
        if (a.accumulate) *dst += v; else *dst = v;
      }
  }
  if (do_rs) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float v = rs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) a.rowsumA[(size_t)sp * a.M + row0 + wm * 32 + t * 16 + lane] = v;
    }
  }
}

template <int NKB, bool BIAS, bool ROWSUM>
__global__ void __launch_bounds__(256, NKB <= 4 ? 2 : 1) gemm_small_kernel(GemmArgs a, int ntn, int ntm, int nch) {
  __shared__ __attribute__((aligned(16))) u16 lds[NKB][2][64 * 64];
  gemm_small_body<NKB, BIAS, ROWSUM>(a, xcd_remap_s(blockIdx.x, gridDim.x), ntn, ntm, lds, nch);
}

// Jobs share the chunk depth NKB; each streams its K-slice as nch[k] chunks.  per_xcd: every job's
// tile count is a multiple of 8, and each XCD runs 1/8 of EVERY job (job k's blocks occupy local
// slots [xs[k], xs[k+1]) of each XCD, job 0 first in dispatch order, consecutive job ids on one XCD as
// in xcd_remap_s) -- a long job (a 4-chunk dW_fc K-slice) is spread over the chip instead of
// filling the first XCDs; else ids are dealt as one range (xcd_remap_s) and cut at start[k].
struct SmallGroup { GemmArgs job[4]; int start[5], xs[5]; int ntn[4], ntm[4], nch[4]; int n, per_xcd; };

template <int NKB, bool BIAS, bool ROWSUM>
__global__ void __launch_bounds__(256, NKB <= 4 ? 2 : 1) gemm_small_group_kernel(SmallGroup g) {
  __shared__ __attribute__((aligned(16))) u16 lds[NKB][2][64 * 64];
  int k = 0, id;
  if (g.per_xcd) {
    const int x = blockIdx.x % 8, loc = blockIdx.x / 8;
    while (k + 1 < g.n && loc >= g.xs[k + 1]) ++k;
    id = x * (g.xs[k + 1] - g.xs[k]) + (loc - g.xs[k]);
  } else {
    const int gid = xcd_remap_s(blockIdx.x, gridDim.x);
    while (k + 1 < g.n && gid >= g.start[k + 1]) ++k;
    id = gid - g.start[k];
  }
  gemm_small_body<NKB, BIAS, ROWSUM>(g.job[k], id, g.ntn[k], g.ntm[k], lds, g.nch[k]);
}

// + trailing blocks running the batch transpose (gemm_with_prep in gemm_lds.hip)
template <int NKB, bool BIAS>
__global__ void __launch_bounds__(256, NKB <= 4 ? 2 : 1) gemm_small_prep_kernel(GemmArgs a, int ntn, int ntm,
                                                                                   PrepJob pj, int nprep, int nch) {
  __shared__ __attribute__((aligned(16))) u16 lds[NKB][2][64 * 64];
  const int ng = ntn * ntm * a.splits;
  if ((int)blockIdx.x >= ng) {
    prep_batch_body(pj, (int)blockIdx.x - ng, nprep);
    return;
  }
  gemm_small_body<NKB, BIAS, false>(a, xcd_remap_s(blockIdx.x, ng), ntn, ntm, lds, nch);
}

// 64-deep blocks per chunk (0 = unsupported); *nch = chunks per K-slice (slices of n x 512 stream)
static int small_blocks(const GemmArgs& a, int* nch) {
  *nch = 1;
  if (a.onehot_ids || a.M % 64 || a.N % 64 || a.K % a.splits) return 0;
  const int kper = a.K / a.splits;
  if (kper % 64) return 0;
  int nkb = kper / 64;
  if (nkb > 8 && nkb % 8 == 0 && nkb <= 32) { *nch = nkb / 8; nkb = 8; }
  if (nkb != 2 && nkb != 3 && nkb != 4 && nkb != 8) return 0;
  if ((a.lda % 8) || (a.ldb % 8)) return 0;
  if ((reinterpret_cast<uintptr_t>(a.A32 ? (const void*)a.A32 : (const void*)a.A) |
       reinterpret_cast<uintptr_t>(a.B)) & 15) return 0;
  return nkb;
}
int gemm_small_kblocks(const GemmArgs& a) {
  int nch = 1;
  const int nkb = small_blocks(a, &nch);
  return nkb * nch;
}

template <class Launch>
static void dispatch_nkb(int nkb, bool bias, bool rs, const Launch& L) {
#define GS_CASE(N)                                                      \
  case N:                                                               \
    if (rs) { if (bias) L.template go<N, true, true>(); else L.template go<N, false, true>(); } \
    else { if (bias) L.template go<N, true, false>(); else L.template go<N, false, false>(); } \
    return;
  switch (nkb) { GS_CASE(2) GS_CASE(3) GS_CASE(4) GS_CASE(8) default: break; }
#undef GS_CASE
  throw std::runtime_error("gemm_small: unsupported K-slice");
}

struct SmallLaunch {
  const GemmArgs& a; int ntn, ntm, nch; hipStream_t s;
  template <int N, bool B, bool R> void go() const {
    hipLaunchKernelGGL((gemm_small_kernel<N, B, R>), dim3(ntn * ntm * a.splits), dim3(256), 0, s, a, ntn, ntm, nch);
  }
};
struct SmallGroupLaunch {
  const SmallGroup& g; int tot; hipStream_t s;
  template <int N, bool B, bool R> void go() const {
    hipLaunchKernelGGL((gemm_small_group_kernel<N, B, R>), dim3(tot), dim3(256), 0, s, g);
  }
};

void gemm_small(const GemmArgs& a, hipStream_t s) {
  int nch = 1;
  const int nkb = small_blocks(a, &nch);
  if (!nkb) throw std::runtime_error("gemm_small: unsupported shape");
  dispatch_nkb(nkb, a.bias && a.splits == 1, a.rowsumA != nullptr, SmallLaunch{a, a.N / 64, a.M / 64, nch, s});
}

void gemm_small_with_prep(const GemmArgs& a, const PrepJob& p, hipStream_t s) {
  int nch = 1;
  const int nkb = small_blocks(a, &nch);
  if (!nkb || a.rowsumA) throw std::runtime_error("gemm_small_with_prep: unsupported shape");
  const int ntn = a.N / 64, ntm = a.M / 64, nprep = prep_batch_blocks(p.T, p.Bp);
  // past one round of workgroups at one per CU (the 128 KiB 8-block image): 4-block chunks, two per CU
  // (config 5's 256 x 6144 table, 384 tiles: 41.5 -> 29.9 us, step 7.938-7.963 -> 7.920-7.928 ms,
  // profiles/r6_prep4_c5_ab.jsonl); the same k order, so the same table
  int nkb2 = nkb;
  if (nkb == 8 && ntn * ntm * a.splits > 256) { nkb2 = 4; nch *= 2; }
  const dim3 grid(ntn * ntm * a.splits + nprep), block(256);
  const bool bias = a.bias && a.splits == 1;
#define GP_CASE(N)                                                                                        \
  case N:                                                                                                 \
    if (bias) hipLaunchKernelGGL((gemm_small_prep_kernel<N, true>), grid, block, 0, s, a, ntn, ntm, p, nprep, nch); \
    else hipLaunchKernelGGL((gemm_small_prep_kernel<N, false>), grid, block, 0, s, a, ntn, ntm, p, nprep, nch);     \
    return;
  switch (nkb2) { GP_CASE(2) GP_CASE(3) GP_CASE(4) GP_CASE(8) default: break; }
#undef GP_CASE
}

int gemm_small_group_depth(const GemmArgs* jobs, int n) {
  int nkb = 0;
  for (int k = 0; k < n; ++k) {
    const int kb = gemm_small_kblocks(jobs[k]);
    if (!kb) return 0;
    nkb = k ? std::min(nkb, kb) : kb;
  }
  while (nkb > 8) nkb = nkb % 8 ? 0 : 8;   // chunks of <= 8 blocks (gemm_small's K-slice rule)
  if (nkb != 2 && nkb != 3 && nkb != 4 && nkb != 8) return 0;
  for (int k = 0; k < n; ++k)
    if (gemm_small_kblocks(jobs[k]) % nkb) return 0;
  return nkb;
}

void gemm_small_group(const GemmArgs* jobs, int n, hipStream_t s) {
  if (n < 1 || n > 4) throw std::runtime_error("gemm_small_group: 1..4 jobs");
  SmallGroup g;
  g.n = n;
  int tot = 0;
  const int nkb = gemm_small_group_depth(jobs, n);
  const bool bias = jobs[0].bias && jobs[0].splits == 1;
  bool rs = false;
  g.per_xcd = 1;
  g.xs[0] = 0;
  for (int k = 0; k < n; ++k) {
    const GemmArgs& a = jobs[k];
    if (!nkb || (a.bias && a.splits == 1) != bias)
      throw std::runtime_error("gemm_small_group: job " + std::to_string(k) + " incompatible");
    rs = rs || a.rowsumA != nullptr;
    g.job[k] = a;
    g.ntn[k] = a.N / 64; g.ntm[k] = a.M / 64;
    g.nch[k] = gemm_small_kblocks(a) / nkb;
    g.start[k] = tot;
    const int nt = g.ntn[k] * g.ntm[k] * a.splits;
    tot += nt;
    if (nt % 8) g.per_xcd = 0;
    g.xs[k + 1] = g.xs[k] + nt / 8;
  }
  g.start[n] = tot;
  dispatch_nkb(nkb, bias, rs, SmallGroupLaunch{g, tot, s});
}

}  // namespace gk
