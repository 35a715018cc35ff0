// Fused step tail for gfx950: everything between the backward sequence kernel and the next step
// as ONE launch (SURVEY §3.5 train_step, its last rows; the reference has no training at all,
// namegensf.cu is inference only).
//
// The phased tail is three dependent launches -- reduce_multi (the layer-0 table gradient dP from
// its per-row-block partials + the loss), gemm_small_group (dW_ih0 = dP^T Emb, dEmb = dP W_ih0)
// and adam_cast (Adam + bf16 refresh of every tensor): 5.6 + 5.6 + 20.2 us at the headline, each
// with its own grid fill / drain and a dependent-kernel boundary (profiles/r3_base_step_summary.txt).
// Only the embedding side depends on the dP chain; the bulk of the Adam bytes (W_hh, W_fc, the
// biases) does not.  Here every piece is a block of one grid:
//
//   blocks  [dW_fc K-slices] [dP tiles] [loss] [Adam: the other tensors] [dW_ih0 tiles] [dEmb K-slices]
//                                                                          wait: their dP column blocks
//
// * A dW_fc block computes one 64 x 64 tile of dW_fc = dl^T H (+ the b_fc row sums) over one token
//   slice into a partial slab; the tile's last slice to arrive sums the slabs and runs the Adam of
//   that W_fc tile (and b_fc).  These replace the separate dW_fc launch before the backward.
//
// * A dW_ih0 block computes one 64 x 64 output tile (K = V, unsplit) and then runs the Adam +
//   refresh of exactly that tile of W_ih0 from the gradient it holds in LDS (no hand-off) -- once
//   the dEmb blocks that read the same W_ih^T tile (its bf16 B operand, which that refresh
//   overwrites) have signalled their reads done.
// * A dEmb block computes one 64 x 64 tile over one K-slice of 3H into a partial slab; the LAST of
//   the tile's slices to arrive (its atomic add returns the epoch's last count) sums the slabs in
//   fixed order and runs the Adam + refresh of that tile of Emb, after the dW_ih0 blocks that read
//   the same Emb^T rows have signalled.  Every product block signals its reads before it waits.
// * Waits are bounded by wall clock (error bit 8).  Only the product blocks wait, on points other
//   blocks reach without waiting first, and there are fewer product blocks than resident slots
//   (checked on the host): the launch drains whatever the dispatch order.
// * Counters are monotonic per epoch (the fused-tail launch count, bumped together with the step
//   counter by the backward kernel before this launch): a column block is complete at
//   (V / 32) * epoch arrivals, a dEmb tile's last slice sees se * epoch - 1.  Nothing is reset.
//
// Hand-offs follow MI355X_MICROARCH.md 'Valid forms' row 1: sc1 (write-through) stores, every
// storing wave drains (vmcnt(0)), a workgroup barrier, one agent-scope atomic add per block; the
// consumer polls (or learns from its own add) and then reads those bytes with sc1 loads only.
//
// Same partials, same orders and same MFMA k-sequences as the phased tail: the fused step is
// bitwise equal to forward_backward + optimizer_step (tests/test_engine_gpu.py).
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "kernels.h"
#include "common.h"
#include "optim_dev.h"

namespace gk {

static constexpr unsigned kTailErr = 8u;                          // error bit: an in-launch wait timed out
static constexpr unsigned long long kTailWaitTicks = 20000000ull;   // 0.2 s of the 100 MHz wall clock

DEV unsigned* tail_ctr(unsigned* s, int k) { return s + 16 * k; }   // one 64-B line each

// one lane polls counter c until >= target (sc1 loads, bounded); the caller joins at a barrier
DEV void tail_wait(const unsigned* c, unsigned target, unsigned* err) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(4);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kTailWaitTicks) {
        if (err) __hip_atomic_fetch_or(err, kTailErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
}
// every storing wave drains its write-through stores, a barrier, then one lane adds; returns the
// counter's previous value to every thread (through LDS)
DEV unsigned tail_arrive(unsigned* c, unsigned* shared_word) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) *shared_word = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return *shared_word;
}

// a block's reads are done (its MFMAs consumed them): one lane adds after a barrier
DEV void tail_reads_done(unsigned* c) {
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- dP tile: 32 rows x 64 columns of the [V][H3] table gradient, summed over the row-block
// partials in fixed order (as reduce_multi), stored bf16 row-major and, through LDS, transposed
DEV void tail_dp_tile(const TailArgs& t, int id, u16 (*tile)[kAdamTileP]) {
  const int tiles_c = t.H3 / 64;
  const int r0 = (id / tiles_c) * 32, c0 = (id % tiles_c) * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const long n = (long)t.V * t.H3;
  const brsrc_t rb = brsrc(t.dP_bf, (unsigned)(n * 2)), rt = brsrc(t.dPT_bf, (unsigned)(n * 2));
  float4 acc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
    acc[q] = sum_slabs4<false>(t.dP_part, n, t.nslP, (size_t)(r0 + ty + 16 * q) * t.H3 + c0 + 4 * tx);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = r0 + ty + 16 * q;
    u32x2_t w;
    w.x = (unsigned)f2bf(acc[q].x) | ((unsigned)f2bf(acc[q].y) << 16);
    w.y = (unsigned)f2bf(acc[q].z) | ((unsigned)f2bf(acc[q].w) << 16);
    bst8_sc1(rb, (unsigned)(((size_t)r * t.H3 + c0 + 4 * tx) * 2), w);
    unsigned* tw = reinterpret_cast<unsigned*>(&tile[ty + 16 * q][4 * tx]);
    tw[0] = w.x;
    tw[1] = w.y;
  }
  __syncthreads();
  {   // 64 columns x 4 pieces of 8 rows: dP^T[c0 + col][r0 + 8 seg ..]
    const int col = threadIdx.x >> 2, seg = threadIdx.x & 3;
    u16 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[seg * 8 + e][col];
    bst16_sc1(rt, (unsigned)(((size_t)(c0 + col) * t.V + r0 + seg * 8) * 2), *reinterpret_cast<const u32x4_t*>(v));
  }
}

// ---- one 64 x 64 tile of an NT product over a K-slice of 8 k-steps (256): 4 waves as 2 x 2 of
// 32 x 32, register-direct MFMA 16x16x32 bf16, k-steps in increasing order (the MFMA sequence of
// gemm_small).  Every operand load of the slice is in flight at once: B (written by an earlier
// launch) is issued by tail_loadB BEFORE the block waits for A (written in this launch, sc1 loads),
// so only A's latency follows the wait -- one round trip instead of one per k-step pair.
struct TailFrags { bf16x8 a[8][2], b[8][2]; };
DEV void tail_loadB(const u16* B, int ldb, int col0, int k0, TailFrags& f) {
  const int lane = threadIdx.x & 63, wn = (threadIdx.x >> 6) & 1;
  const u16* p = B + (size_t)(col0 + wn * 32 + (lane & 15)) * ldb + k0 + 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int c = 0; c < 2; ++c) f.b[ks][c] = ld8(p + (size_t)16 * c * ldb + ks * 32);
}
DEV void tail_loadA_sc1(const u16* A, int lda, long a_bytes, int row0, int k0, TailFrags& f) {
  const int lane = threadIdx.x & 63, wm = (threadIdx.x >> 6) >> 1;
  const brsrc_t rA = brsrc(A, (unsigned)a_bytes);
  const unsigned base = (unsigned)(((size_t)(row0 + wm * 32 + (lane & 15)) * lda + k0 + 8 * (lane >> 4)) * 2);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int r = 0; r < 2; ++r) f.a[ks][r] = bld8_sc1(rA, base + (unsigned)((16 * r * lda + ks * 32) * 2));
}
// both operands written in this launch (the next step's P table): sc1 loads of rows row0 + wsel*32..
DEV void tail_load_sc1(const u16* A, int lda, long a_bytes, int row0, int k0, int wsel, bf16x8 (&fr)[8][2]) {
  const int lane = threadIdx.x & 63;
  const brsrc_t rA = brsrc(A, (unsigned)a_bytes);
  const unsigned base = (unsigned)(((size_t)(row0 + wsel * 32 + (lane & 15)) * lda + k0 + 8 * (lane >> 4)) * 2);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int r = 0; r < 2; ++r) fr[ks][r] = bld8_sc1(rA, base + (unsigned)((16 * r * lda + ks * 32) * 2));
}
DEV void tail_mma(const TailFrags& f, f32x4 (&acc)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(f.a[ks][i], f.b[ks][j], acc[i][j]);
}
// the whole product tile: K-slices of 256 in order, each slice's B loads issued before `wait`
// (called once, before the first slice's A loads)
// rs (do_rs): this lane's partial row sums of its two A fragments, in the order of gemm_small's
template <class Wait>
DEV void tail_product(const u16* A, int lda, long a_bytes, const u16* B, int ldb, int row0, int col0, int k0, int kl,
                      f32x4 (&acc)[2][2], Wait&& wait, float* rs = nullptr) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  TailFrags f;
  for (int kc = 0; kc < kl; kc += 256) {
    tail_loadB(B, ldb, col0, k0 + kc, f);
    if (kc == 0) wait();
    tail_loadA_sc1(A, lda, a_bytes, row0, k0 + kc, f);
    tail_mma(f, acc);
    if (rs)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) rs[i] += (float)f.a[ks][i][e];
  }
}
// row / column within the 64 x 64 tile of this lane's acc[i][j][e]
DEV int acc_row(int i, int e) { return ((threadIdx.x >> 6) >> 1) * 32 + i * 16 + ((threadIdx.x & 63) >> 4) * 4 + e; }
DEV int acc_col(int j) { return ((threadIdx.x >> 6) & 1) * 32 + j * 16 + (threadIdx.x & 15); }

template <int MINW>   // minimum waves per SIMD (= resident 256-thread workgroups per CU)
__global__ void __launch_bounds__(256, MINW) tail_kernel(OptimArgs a, OptCastJobs j, TailArgs t) {
  __shared__ __attribute__((aligned(16))) u16 tile[64][kAdamTileP];
  __shared__ __attribute__((aligned(16))) float gt[64][68];   // a product tile's fp32 gradient
  __shared__ __attribute__((aligned(16))) float gb[64];       // b_fc gradients of a dW_fc row tile
  __shared__ unsigned s_prev;
  const int gi = blockIdx.x;   // grid index (stamps); item index below it (after the batch-prep blocks)
  if (t.dbg && threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    t.dbg[(size_t)gi * 4 + 0] = __builtin_amdgcn_s_memrealtime();
    t.dbg[(size_t)gi * 4 + 3] = (unsigned long long)gi | ((unsigned long long)xcc << 16);
  }
  if (gi < t.nB) {   // the next step's batch preparation (its slot's pinned host reads), waits for nothing
    prep_batch_body(t.prep, gi, t.nB);
    if (t.dbg && threadIdx.x == 0) t.dbg[(size_t)gi * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  const int it = gi - t.nB;
  const bool failed = step_failed(a);         // a persistent kernel of this step gave up: no update
  const AdamCoef co = adam_coef(a);           // the step counter was bumped before this launch
  unsigned* err = const_cast<unsigned*>(a.err);
  const unsigned ep = *t.epoch;
  const int ntE = t.E / 64;
  const unsigned colTarget = (unsigned)(t.V / 32) * ep;
  const int eP = t.nF, eL = eP + t.nP, eA0 = eL + 1, eW = eA0 + t.nA0, eE = eW + t.nW, eQ = eE + t.nE;
  unsigned* rdW = tail_ctr(t.sync, t.H3 / 64 + (t.V / 64) * ntE);   // [E/64]: dW_ih0 blocks done reading Emb^T
  unsigned* rdE = rdW + 16 * ntE;                                     // [E/64][8]: dEmb blocks done reading W_ih^T
  unsigned* cFc = rdE + 16 * 8 * ntE;                                 // [V/64][H/64]: dW_fc slices arrived
  unsigned* cEmb = cFc + 16 * (t.V / 64) * (t.H / 64);                // [V/64]: Emb row block tiles refreshed
  unsigned* cWih = cEmb + 16 * (t.V / 64);                            // [H3/64]: W_ih0 row block tiles refreshed
  unsigned* cBi = cWih + 16 * (t.H3 / 64);                            // b_ih0 blocks refreshed
  if (it < eP) {           // dW_fc tile (tm, tn) over token slice sp; the tile's last slice runs its Adam
    const int ntH = t.H / 64, ntV = t.V / 64;
    const int tn = it % ntH, tm = (it / ntH) % ntV, sp = it / (ntH * ntV);
    const int kl = t.tok / t.nfc;
    const bool do_rs = tn == 0 && ((threadIdx.x >> 6) & 1) == 0;
    float rs[2] = {0.f, 0.f};
    f32x4 acc[2][2];
    tail_product(t.dlT, t.ldl, (long)t.V * t.ldl * 2, t.HTop, t.ldh, tm * 64, tn * 64, sp * kl, kl, acc, [&] {
      if (t.fc_after_dp) {   // let the dP chain have the memory system first
        tail_wait(tail_ctr(t.sync, it % (t.H3 / 64)), colTarget, err);
        __syncthreads();
      }
    }, do_rs ? rs : nullptr);
    const long n = (long)t.V * t.H;
    const brsrc_t rS = brsrc(t.slab_fc, (unsigned)(t.nfc * n * 4));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const size_t o = (size_t)sp * n + (size_t)(tm * 64 + acc_row(i, e)) * t.H + tn * 64 + acc_col(jj);
          bst1_sc1(rS, (unsigned)(o * 4), acc[i][jj][e]);
        }
    if (do_rs) {   // as gemm_small: lane partials over lane >> 4, then lanes 0..15 hold the 16 rows
      const int lane = threadIdx.x & 63;
      const brsrc_t rR = brsrc(t.rs_fc, (unsigned)(t.nfc * t.V * 4));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v = rs[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16)
          bst1_sc1(rR, (unsigned)(((size_t)sp * t.V + tm * 64 + ((threadIdx.x >> 6) >> 1) * 32 + i * 16 + lane) * 4), v);
      }
    }
    const unsigned prev = tail_arrive(cFc + 16 * (tm * ntH + tn), &s_prev);
    if (prev == (unsigned)t.nfc * ep - 1u) {   // last slice of this tile: every slab is published
      const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t o = (size_t)(tm * 64 + ty + 16 * q) * t.H + tn * 64 + 4 * tx;
        *reinterpret_cast<float4*>(&gt[ty + 16 * q][4 * tx]) = sum_slabs4<true>(t.slab_fc, n, t.nfc, o);
      }
      if (tn == 0 && threadIdx.x < 16)   // this row tile's 64 b_fc gradients (row 0 of the tile holds them)
        *reinterpret_cast<float4*>(&gb[4 * threadIdx.x]) =
            sum_slabs4<true>(t.rs_fc, t.V, t.nfc, (size_t)tm * 64 + 4 * threadIdx.x);
      __syncthreads();
      if (!failed) {
        adam_cast_unit<false, false>(a, j.job[t.jf], tm * ntH + tn, co, tile, gt);
        if (tn == 0 && threadIdx.x < 16) {   // b_fc elements tm*64 .. +63: one float4 per thread
          const OptCastJob& J = j.job[t.jb];
          const long i4 = (J.off >> 2) + tm * 16 + threadIdx.x;
          float4 p = reinterpret_cast<float4*>(a.p)[i4];
          const float4 g = *reinterpret_cast<const float4*>(&gb[4 * threadIdx.x]);
          float4 m = make_float4(0.f, 0.f, 0.f, 0.f), v = m;
          if (!a.sgd) { m = reinterpret_cast<float4*>(a.m)[i4]; v = reinterpret_cast<float4*>(a.v)[i4]; }
          adam_update4(a, co, p, g, m, v);
          if (!a.sgd) { reinterpret_cast<float4*>(a.m)[i4] = m; reinterpret_cast<float4*>(a.v)[i4] = v; }
          reinterpret_cast<float4*>(a.p)[i4] = p;
          reinterpret_cast<float4*>(const_cast<float*>(a.g))[i4] = g;
        }
      }
    }
  } else if (it < eL) {
    const int id = it - eP;
    tail_dp_tile(t, id, tile);
    (void)tail_arrive(tail_ctr(t.sync, id % (t.H3 / 64)), &s_prev);   // its column block
  } else if (it < eA0) {   // loss = sum of the per-block partials, fixed order (one wave)
    if (threadIdx.x < 64) {
      float acc = 0.f;
      for (int i = threadIdx.x; i < t.nloss; i += 64) acc += t.loss_part[i];
      acc = wave_sum(acc);
      if (threadIdx.x == 0) *t.loss = acc;
    }
  } else if (it < eW) {    // Adam + bf16 refresh (every tensor but W_ih0 / Emb: blk_start skips them)
    const int b = it - eA0;
    if (t.adam_after_dp) {   // let the dP tiles have the memory system first (spread over the column counters)
      tail_wait(tail_ctr(t.sync, b % (t.H3 / 64)), colTarget, err);
      __syncthreads();
    }
    int k = 0;
    while (k + 1 < j.n && b >= j.blk_start[k + 1]) ++k;
    if (t.P && k == t.jbi) {   // b_ih0: read by the P items of this launch
      if (!failed) adam_cast_unit<false, true>(a, j.job[k], b - j.blk_start[k], co, tile);
      (void)tail_arrive(cBi, &s_prev);
    } else if (!failed) {
      adam_cast_unit<false, false>(a, j.job[k], b - j.blk_start[k], co, tile);
    }
  } else if (it < eE) {    // dW_ih0 tile (tm, tn) = dP[:, tm]^T · Emb[:, tn] (K = V), then its Adam
    const int id = it - eW, tm = id / ntE, tn = id % ntE;
    f32x4 acc[2][2];
    tail_product(t.dPT_bf, t.V, (long)t.V * t.H3 * 2, t.EmbT, t.V, tm * 64, tn * 64, 0, t.V, acc, [&] {
      tail_wait(tail_ctr(t.sync, tm), colTarget, err);
      if (t.dbg && threadIdx.x == 0) t.dbg[(size_t)gi * 4 + 1] = __builtin_amdgcn_s_memrealtime();
      __syncthreads();
    });
    tail_reads_done(rdW + 16 * tn);
    // this tile's refresh rewrites W_ih^T rows tn*64.., columns tm*64..: K-slice tm*64 / kl of the
    // dEmb blocks of E-tile tn, all V/64 of them, must have read it
    tail_wait(rdE + 16 * (tn * 8 + tm * 64 / (t.H3 / t.se)), (unsigned)(t.V / 64) * ep, err);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) gt[acc_row(i, e)][acc_col(jj)] = acc[i][jj][e];
    __syncthreads();
    if (t.P) {   // the refreshed rows feed the P items: write-through row-major copy, then count the tile
      if (!failed) adam_cast_unit<false, true>(a, j.job[t.jw], tm * ntE + tn, co, tile, gt, !t.dP_alias);
      (void)tail_arrive(cWih + 16 * tm, &s_prev);
    } else if (!failed) {
      adam_cast_unit<false, false>(a, j.job[t.jw], tm * ntE + tn, co, tile, gt, !t.dP_alias);
    }
  } else if (it < eQ) {    // dEmb tile (vm, tn) over K-slice ks; the tile's last slice runs its Adam
    const int id = it - eE, ks = id % t.se, tl = id / t.se, vm = tl / ntE, tn = tl % ntE;
    const int kl = t.H3 / t.se;
    f32x4 acc[2][2];
    tail_product(t.dP_bf, t.H3, (long)t.V * t.H3 * 2, t.WihT, t.H3, vm * 64, tn * 64, ks * kl, kl, acc, [&] {
      for (int c = ks * kl / 64; c < (ks + 1) * kl / 64; ++c) tail_wait(tail_ctr(t.sync, c), colTarget, err);
      if (t.dbg && threadIdx.x == 0) t.dbg[(size_t)gi * 4 + 1] = __builtin_amdgcn_s_memrealtime();
      __syncthreads();
    });
    tail_reads_done(rdE + 16 * (tn * 8 + ks));
    const long n = (long)t.V * t.E;
    const brsrc_t rS = brsrc(t.slab_e, (unsigned)(t.se * n * 4));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const size_t o = (size_t)ks * n + (size_t)(vm * 64 + acc_row(i, e)) * t.E + tn * 64 + acc_col(jj);
          bst1_sc1(rS, (unsigned)(o * 4), acc[i][jj][e]);
        }
    const unsigned prev = tail_arrive(tail_ctr(t.sync, t.H3 / 64 + tl), &s_prev);
    if (prev == (unsigned)t.se * ep - 1u) {   // last slice of this tile: every slab is published
      // the refresh rewrites Emb^T rows tn*64..: every dW_ih0 block of E-tile tn must have read them
      tail_wait(rdW + 16 * tn, (unsigned)(t.H3 / 64) * ep, err);
      __syncthreads();
      const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t o = (size_t)(vm * 64 + ty + 16 * q) * t.E + tn * 64 + 4 * tx;
        *reinterpret_cast<float4*>(&gt[ty + 16 * q][4 * tx]) = sum_slabs4<true>(t.slab_e, n, t.se, o);
      }
      __syncthreads();
      if (t.P) {
        if (!failed) adam_cast_unit<false, true>(a, j.job[t.je], vm * ntE + tn, co, tile, gt);
        (void)tail_arrive(cEmb + 16 * vm, &s_prev);
      } else if (!failed) {
        adam_cast_unit<false, false>(a, j.job[t.je], vm * ntE + tn, co, tile, gt);
      }
    }
  } else {                 // the next step's P tile (tv, tn) = Emb[tv] · W_ih0[tn]^T + b_ih0[tn] (K = E)
    const int id = it - eQ, tv = id / (t.H3 / 64), tn = id % (t.H3 / 64);
    const int nbi = (t.H3 + 1023) / 1024;   // blocks of the flat b_ih0 job
    tail_wait(cEmb + 16 * tv, (unsigned)ntE * ep, err);
    tail_wait(cWih + 16 * tn, (unsigned)ntE * ep, err);
    tail_wait(cBi, (unsigned)nbi * ep, err);
    if (t.dbg && threadIdx.x == 0) t.dbg[(size_t)gi * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    const int wm = (threadIdx.x >> 6) >> 1, wn = (threadIdx.x >> 6) & 1;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    TailFrags f;
    for (int kc = 0; kc < t.E; kc += 256) {   // the k-step sequence of the prologue's P GEMM (gemm_small)
      tail_load_sc1(t.EmbR, t.E, (long)t.V * t.E * 2, tv * 64, kc, wm, f.a);
      tail_load_sc1(t.WihR, t.E, (long)t.H3 * t.E * 2, tn * 64, kc, wn, f.b);
      tail_mma(f, acc);
    }
    const brsrc_t rb = brsrc(t.bih, (unsigned)(t.H3 * 4));
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int c = tn * 64 + acc_col(jj);
      const float bias = bld1_sc1(rb, (unsigned)(c * 4));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) t.P[(size_t)(tv * 64 + acc_row(i, e)) * t.H3 + c] = acc[i][jj][e] + bias;
    }
  }
  if (t.dbg && threadIdx.x == 0) t.dbg[(size_t)gi * 4 + 2] = __builtin_amdgcn_s_memrealtime();
}

static int tail_occ() {   // GK_TAIL_OCC: 3 (default) or 4 resident workgroups per CU
  static const int v = [] {
    const char* e = std::getenv("GK_TAIL_OCC");
    return (e && std::atoi(e) == 4) ? 4 : 3;
  }();
  return v;
}
template <class K>
static int resident_wgs(K kernel) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess) return 0;
  return ncu * per;
}

int tail_resident_slots() {
  static const int cap3 = resident_wgs(tail_kernel<3>), cap4 = resident_wgs(tail_kernel<4>);
  return tail_occ() == 4 ? cap4 : cap3;
}

bool tail_step(const OptimArgs& a, OptCastJobs& j, TailArgs& t, hipStream_t s) {
  if (!t.sync || !t.epoch || !t.dP_part || !t.dP_bf || !t.dPT_bf || !t.EmbT || !t.WihT || !t.slab_e || !t.loss ||
      !t.loss_part || t.V % 64 || t.H3 % 64 || t.E % 64 || t.nslP < 1 || t.se < 1 || t.H3 % t.se ||
      (t.H3 / t.se) % 64 || t.jw < 0 || t.je < 0 || t.jw >= j.n || t.je >= j.n)
    throw std::runtime_error("tail_step: incomplete arguments");
  const OptCastJob &W = j.job[t.jw], &Em = j.job[t.je];
  if (W.R != t.H3 || W.C != t.E || Em.R != t.V || Em.C != t.E)
    throw std::runtime_error("tail_step: W_ih0 / embedding jobs do not match the products");
  if (t.nfc) {
    if (!t.dlT || !t.HTop || !t.slab_fc || !t.rs_fc || t.tok % t.nfc || (t.tok / t.nfc) % 256 || t.H % 64 ||
        t.jf < 0 || t.jb < 0 || t.jf >= j.n || t.jb >= j.n || j.job[t.jf].R != t.V || j.job[t.jf].C != t.H ||
        j.job[t.jb].R != 0 || j.job[t.jb].C != t.V || t.ldl % 8 || t.ldh % 8)
      throw std::runtime_error("tail_step: inconsistent dW_fc arguments");
  }
  int tot = 0;
  for (int k = 0; k < j.n; ++k) {
    const OptCastJob& J = j.job[k];
    if (J.R && (J.R % 64 || J.C % 64)) throw std::runtime_error("tail_step: matrix job needs R, C % 64 == 0");
    if (!J.R && J.C % 4) throw std::runtime_error("tail_step: flat job needs C % 4 == 0");
    j.blk_start[k] = tot;
    const bool in_products = k == t.jw || k == t.je || (t.nfc && (k == t.jf || k == t.jb));
    if (!in_products) tot += J.R == 0 ? (J.C + 1023) / 1024 : (J.R / 64) * (J.C / 64);
  }
  j.blk_start[j.n] = tot;
  t.nF = t.nfc ? (t.V / 64) * (t.H / 64) * t.nfc : 0;
  t.nP = (t.V / 32) * (t.H3 / 64);
  t.nA0 = tot;
  t.nW = (t.H3 / 64) * (t.E / 64);
  t.nE = (t.V / 64) * (t.E / 64) * t.se;
  if (t.P) {
    if (!t.EmbR || !t.WihR || !t.bih || t.E % 256 || t.jbi < 0 || t.jbi >= j.n || j.job[t.jbi].R != 0 ||
        j.job[t.jbi].C != t.H3 || t.jbi == t.jw || t.jbi == t.je)
      throw std::runtime_error("tail_step: inconsistent P-table arguments");
    t.nPt = (t.V / 64) * (t.H3 / 64);
  } else {
    t.nPt = 0;
  }
  t.nB = t.prep.in ? prep_batch_blocks(t.prep.T, t.prep.Bp) : 0;
  t.nItems = t.nB + t.nF + t.nP + 1 + t.nA0 + t.nW + t.nE + t.nPt;
  const int occ = tail_occ();
  const int cap = tail_resident_slots();
  // A product block waits only for points that other blocks reach without waiting first (dP tiles;
  // product blocks signal their reads before they wait).  With fewer product blocks than resident
  // slots, a block they wait for always gets a slot: the launch drains whatever the dispatch order.
  // The P items wait for product blocks (which wait only for dP tiles): still a bounded chain, and
  // all waiting blocks together stay below the resident slots.
  const int waiting = t.nW + t.nE + t.nPt + (t.fc_after_dp ? t.nF : 0) + (t.adam_after_dp ? t.nA0 : 0);
  if (cap <= 0 || waiting >= cap || t.se > 8 || (t.H3 / t.se) % 256 || t.V % 256) return false;
  if (t.dbg && t.nItems > 65536) t.dbg = nullptr;
  if (occ == 4) hipLaunchKernelGGL(tail_kernel<4>, dim3(t.nItems), dim3(256), 0, s, a, j, t);
  else hipLaunchKernelGGL(tail_kernel<3>, dim3(t.nItems), dim3(256), 0, s, a, j, t);
  return true;
}

}  // namespace gk
