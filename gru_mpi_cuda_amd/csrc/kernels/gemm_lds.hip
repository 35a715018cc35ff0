// LDS-staged bf16 MFMA GEMM for the large products (weight gradients over B*T tokens, hoisted
// input projections, dH at large H):  C[M][N] (+)= A[M][K] · B[N][K]^T, fp32 accumulate.
//
// gfx950 structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop", 2-buffer form):
//   * 128 x 128 x 64 tiles, 256 threads = 2 x 2 waves, each wave 64 x 64 = 4 x 4 MFMA 16x16x32;
//   * global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR round trip); one
//     wave-instruction writes 1 KiB = 8 rows x 128 B of the tile, so the LDS image is lane-linear
//     and the bank swizzle goes on the per-lane SOURCE address (rule 21);
//   * swizzle: logical 16-B chunk c of row r lives in slot c ^ ((r >> 1) & 7).  For the
//     ds_read_b128 fragment reads (16 rows x one chunk per lane quarter) every 16-lane group then
//     touches 16 distinct 16-B bank slots -> conflict-free (derivation in docs/DESIGN.md);
//   * double-buffered: tile k+1's LDS-DMA is in flight while tile k's 32 MFMAs run, one
//     vmcnt(0) + barrier per tile;
//   * XCD-aware bijective block remap (T1) so neighbouring tiles share an L2;
//   * split-K slabs for the K = B*T weight-gradient products.
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "kernels.h"
#include "common.h"

namespace gk {

typedef __attribute__((address_space(3))) void lds_void;

DEV int xcd_remap2(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// OH: one-hot A (dP = onehot(ids)^T · B, the embedding-table gradient): A[m][k] = (ids[k] == m) is
// synthesised into the same swizzled LDS image the LDS-DMA would have written, from char ids
// prefetched one k-tile ahead -- no A operand in memory at all.
template <bool BIAS, bool ROWSUM, bool OH = false>
DEV void gemm_lds_body(const GemmArgs& a, int id, int ntn, int ntm, int kper, u16 (&lds)[2][2][128 * 64]) {
  // the shorter tile dimension is the fast block index, so the workgroups sharing the long
  // operand's panel are neighbours on one XCD and stream it through its L2 together (one-hot dP at
  // h2048, 2 x 48 tiles: B is the only operand in memory, and column-fast order read it once per
  // row tile from HBM: 380 -> 341 us).  a.raster: 0 auto, 1 column-fast (GemmArgs::raster)
  const bool mfast = OH ? a.raster != 1 : (a.raster == 0 && ntm < ntn);
  const int tn = mfast ? (id / ntm) % ntn : id % ntn;
  const int tm = mfast ? id % ntm : (id / ntn) % ntm;
  const int sp = id / (ntn * ntm);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int row0 = tm * 128, col0 = tn * 128;
  const int kbeg = sp * kper, nk = kper / 64;

  // staging geometry: wave w, instruction q covers tile rows (4w+q)*8 .. +7
  const int srow = lane >> 3, sslot = lane & 7;
  const u16* srcA[4];
  const u16* srcB[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = (4 * w + q) * 8 + srow;
    const int c = sslot ^ ((r >> 1) & 7);
    srcA[q] = OH ? nullptr : a.A + (size_t)(row0 + r) * a.lda + kbeg + c * 8;
    srcB[q] = (a.B2 && col0 >= a.b2_row ? a.B2 : a.B) + (size_t)(col0 + r) * a.ldb + kbeg + c * 8;
  }
  // one-hot: row r = (4w+q)*8 + srow keeps logical chunk c = sslot ^ (4(q&1) + (srow>>1)) in this
  // lane's slot, so a lane needs the 8 ids of two chunks per k-tile
  int4 idn[2][2];
  auto load_ids = [&](int kt) {
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int c = sslot ^ (4 * v + (srow >> 1));
      const int4* p = reinterpret_cast<const int4*>(a.onehot_ids + kbeg + kt * 64 + c * 8);
      idn[v][0] = p[0];
      idn[v][1] = p[1];
    }
  };
  if constexpr (OH) load_ids(0);
  auto stage = [&](int buf, int kt) {
    if constexpr (OH) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = (4 * w + q) * 8 + srow, m = row0 + r;
        const int4 i0 = idn[q & 1][0], i1 = idn[q & 1][1];
        const int iv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
        unsigned wv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          wv[e] = (iv[2 * e] == m ? 0x3F80u : 0u) | ((iv[2 * e + 1] == m ? 0x3F80u : 0u) << 16);
        *reinterpret_cast<uint4*>(&lds[buf][0][r * 64 + sslot * 8]) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
      if (kt + 1 < nk) load_ids(kt + 1);   // lands by the vmcnt(0) that ends this k-tile
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(srcB[q] + kt * 64, (lds_void*)(&lds[buf][1][(4 * w + q) * 8 * 64]), 16, 0, 0);
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int base = (4 * w + q) * 8 * 64;
      __builtin_amdgcn_global_load_lds(srcA[q] + kt * 64, (lds_void*)(&lds[buf][0][base]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(srcB[q] + kt * 64, (lds_void*)(&lds[buf][1][base]), 16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias gradients: row sums of A from the A fragments already in registers (one wave column
  // of the first column tile does it; wave-uniform branch)
  const bool do_rs = ROWSUM && tn == 0 && wn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + lq;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ra = wm * 64 + t * 16 + lr;
        const int rb = wn * 64 + t * 16 + lr;
        af[t] = *reinterpret_cast<const bf16x8*>(&lds[cur][0][ra * 64 + ((c ^ ((ra >> 1) & 7)) * 8)]);
        bfr[t] = *reinterpret_cast<const bf16x8*>(&lds[cur][1][rb * 64 + ((c ^ ((rb >> 1) & 7)) * 8)]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      if (do_rs) {
#pragma unroll
        for (int t = 0; t < 4; ++t) rs[t] = add_sum8(af[t], rs[t]);   // four v_dot2 (common.h)
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + wn * 64 + j * 16 + lr;
    const float bb = BIAS ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + wm * 64 + i * 16 + lq * 4 + e;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[i][j][e] + bb;
        if (a.accumulate) *dst += v; else *dst = v;
      }
  }
  if (do_rs) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = rs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) a.rowsumA[(size_t)sp * a.M + row0 + wm * 64 + t * 16 + lane] = v;
    }
  }
}

template <bool BIAS, bool ROWSUM, bool OH = false>
__global__ void __launch_bounds__(256, 2) gemm_lds_kernel(GemmArgs a, int ntn, int ntm, int kper) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][128 * 64];
  gemm_lds_body<BIAS, ROWSUM, OH>(a, xcd_remap2(blockIdx.x, gridDim.x), ntn, ntm, kper, lds);
}

// grouped launch: block range [start[k], start[k+1]) serves job k (after the XCD remap, so each
// job's neighbouring tiles still share an L2)
struct GemmGroup { GemmArgs job[4]; int start[5]; int ntn[4], ntm[4], kper[4]; int n; };

template <bool BIAS, bool ROWSUM>
__global__ void __launch_bounds__(256, 2) gemm_lds_group_kernel(GemmGroup g) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][128 * 64];
  const int id = xcd_remap2(blockIdx.x, gridDim.x);
  int k = 0;
  while (k + 1 < g.n && id >= g.start[k + 1]) ++k;
  gemm_lds_body<BIAS, ROWSUM>(g.job[k], id - g.start[k], g.ntn[k], g.ntm[k], g.kper[k], lds);
}

template <bool BIAS>
__global__ void __launch_bounds__(256, 2) gemm_lds_prep_kernel(GemmArgs a, int ntn, int ntm, int kper, PrepJob pj,
                                                                int nprep) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][128 * 64];
  const int ng = ntn * ntm * a.splits;
  if ((int)blockIdx.x >= ng) {   // trailing blocks: batch transpose (block-uniform branch)
    prep_batch_body(pj, (int)blockIdx.x - ng, nprep);
    return;
  }
  gemm_lds_body<BIAS, false>(a, xcd_remap2(blockIdx.x, ng), ntn, ntm, kper, lds);
}

void gemm_with_prep(const GemmArgs& a, const PrepJob& p, hipStream_t s) {
  if (gemm_small_kblocks(a) && !a.rowsumA && (a.M % 128 || a.N % 128 || (a.M / 128) * (a.N / 128) * a.splits < 256)) {
    gemm_small_with_prep(a, p, s);
    return;
  }
  if (!gemm_lds_ok(a) || a.rowsumA || a.accumulate) {
    prep_batch(p.in, p.Bmax, p.T, p.Bp, p.ids, p.labels, p.inv_count, s);
    gemm_nt(a, s);
    return;
  }
  const int ntn = a.N / 128, ntm = a.M / 128, kper = a.K / a.splits;
  const int nprep = prep_batch_blocks(p.T, p.Bp);
  dim3 grid(ntn * ntm * a.splits + nprep), block(256);
  if (a.bias && a.splits == 1)
    hipLaunchKernelGGL((gemm_lds_prep_kernel<true>), grid, block, 0, s, a, ntn, ntm, kper, p, nprep);
  else
    hipLaunchKernelGGL((gemm_lds_prep_kernel<false>), grid, block, 0, s, a, ntn, ntm, kper, p, nprep);
}

bool gemm_lds_ok(const GemmArgs& a) {
  if (a.M % 128 || a.N % 128 || a.K % a.splits) return false;
  const int kper = a.K / a.splits;
  if (kper % 64 || kper < 128) return false;
  if (a.B2 && (!a.onehot_ids || a.b2_row % 128 || (reinterpret_cast<uintptr_t>(a.B2) & 15))) return false;
  if (a.onehot_ids) {   // synthesised A: 16-B aligned id chunks, no bias / row sums
    return !a.rowsumA && !a.bias && !(a.ldb % 8) && !(reinterpret_cast<uintptr_t>(a.B) & 15) &&
           !(reinterpret_cast<uintptr_t>(a.onehot_ids) & 15);
  }
  // 16-B aligned rows for the LDS-DMA loads
  if ((a.lda % 8) || (a.ldb % 8)) return false;
  if ((reinterpret_cast<uintptr_t>(a.A) | reinterpret_cast<uintptr_t>(a.B)) & 15) return false;
  return true;
}

void gemm_lds_group(const GemmArgs* jobs, int n, hipStream_t s) {
  if (n < 1 || n > 4) throw std::runtime_error("gemm_lds_group: 1..4 jobs");
  GemmGroup g;
  g.n = n;
  int tot = 0;
  const bool bias = jobs[0].bias && jobs[0].splits == 1, rs = jobs[0].rowsumA != nullptr;
  for (int k = 0; k < n; ++k) {
    const GemmArgs& a = jobs[k];
    if (!gemm_lds_ok(a) || (a.bias && a.splits == 1) != bias || (a.rowsumA != nullptr) != rs)
      throw std::runtime_error("gemm_lds_group: job " + std::to_string(k) + " incompatible");
    g.job[k] = a;
    g.ntn[k] = a.N / 128; g.ntm[k] = a.M / 128; g.kper[k] = a.K / a.splits;
    g.start[k] = tot;
    tot += g.ntn[k] * g.ntm[k] * a.splits;
  }
  g.start[n] = tot;
  dim3 grid(tot), block(256);
  if (rs) {
    if (bias) hipLaunchKernelGGL((gemm_lds_group_kernel<true, true>), grid, block, 0, s, g);
    else hipLaunchKernelGGL((gemm_lds_group_kernel<false, true>), grid, block, 0, s, g);
  } else {
    if (bias) hipLaunchKernelGGL((gemm_lds_group_kernel<true, false>), grid, block, 0, s, g);
    else hipLaunchKernelGGL((gemm_lds_group_kernel<false, false>), grid, block, 0, s, g);
  }
}

void gemm_lds(const GemmArgs& a0, hipStream_t s) {
  const GemmArgs& a = a0;
  const int ntn = a.N / 128, ntm = a.M / 128, kper = a.K / a.splits;
  dim3 grid(ntn * ntm * a.splits), block(256);
  if (a.onehot_ids) {
    hipLaunchKernelGGL((gemm_lds_kernel<false, false, true>), grid, block, 0, s, a, ntn, ntm, kper);
    return;
  }
  const bool bias = a.bias && a.splits == 1;
  if (a.rowsumA) {
    if (bias) hipLaunchKernelGGL((gemm_lds_kernel<true, true>), grid, block, 0, s, a, ntn, ntm, kper);
    else hipLaunchKernelGGL((gemm_lds_kernel<false, true>), grid, block, 0, s, a, ntn, ntm, kper);
  } else {
    if (bias) hipLaunchKernelGGL((gemm_lds_kernel<true, false>), grid, block, 0, s, a, ntn, ntm, kper);
    else hipLaunchKernelGGL((gemm_lds_kernel<false, false>), grid, block, 0, s, a, ntn, ntm, kper);
  }
}

}  // namespace gk
