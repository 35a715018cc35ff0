// Large-H timestep kernels (H >= 1024 with a batch too big for the persistent kernels):
// the per-step recurrent GEMM is a real GEMM here (B = 512, H = 2048: 12.9 GFLOP per step),
// so it runs on the LDS-staged MFMA structure of gemm_lds.hip with the GRU math fused into the
// epilogue.
//
//   forward : tile = 128 batch rows x 32 units x 3 gates.  The B tile's 96 rows are gathered
//             from the three gate blocks of W_hh (row g*H + j0 + u), so wave (wm, wn) holds
//             r/z/n pre-activations of the same (row, unit) in acc[i][0..2] -> gates, blend and
//             all stores straight from registers.
//   backward: tile = 64 rows x 64 units, K = 3H (dh = dGh_{t+1} · W_hh), then the gate-gradient
//             epilogue; transposed copies (dGh^T, dGi^T for the weight-gradient GEMMs) go
//             through the then-idle LDS.
// Staging: global_load_lds_dwordx4 into a lane-linear LDS image, XOR swizzle on the source
// address (conflict-free ds_read_b128), 2 buffers, one vmcnt(0) + barrier per 64-deep k-tile.
#include <cstdlib>
#include <type_traits>
#include "kernels.h"
#include "common.h"

namespace gk {

typedef __attribute__((address_space(3))) void lds_void_t;

DEV int swz(int r, int c) { return c ^ ((r >> 1) & 7); }


// Wait until k-tile kt has landed while `ahead` later k-tiles (PER LDS-DMA instructions each,
// per wave) stay in flight.  vmcnt retires in issue order, so loads the compiler issues after
// ours only make the wait more conservative.
template <int N> DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int PER, int A> DEV void wait_ahead(int ahead) {
  if (ahead >= A) { vm_wait<A * PER>(); return; }
  if constexpr (A > 0) wait_ahead<PER, A - 1>(ahead);
}
// lds_barrier (common.h): LDS-DMA completion is covered by the explicit vm_wait before it.
// NS-deep LDS ring: NS-1 k-tiles in flight.  One barrier per k-tile: it publishes tile kt and
// proves every wave is done with the slot tile kt+NS-1 is about to overwrite.
template <int NS, int PER, class Stage, class Compute>
DEV void ring_loop(int nk, Stage&& stage, Compute&& compute) {
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    wait_ahead<PER, NS - 2>(min(NS - 2, nk - 1 - kt));
    lds_barrier();
    if (kt + NS - 1 < nk) stage((kt + NS - 1) % NS, kt + NS - 1);
    compute(kt % NS);
  }
  __syncthreads();
}

// ==================================================================== forward
// LDS: [FNS slots] x (A 128x64 + B 96x64) bf16 = FNS x 28 KiB
// FUSED: the layer's input projection runs in the same tile as a first K phase (A = x rows,
// B = W_ih gate rows, K = Kin) ahead of the recurrent phase (A = h_{t-1}, B = W_hh, K = H): the
// r/z pre-activations of both phases share accumulators, the n gate keeps its input part apart
// (n = tanh(gi_n + r * gh_n)).  Used for layers >= 1 of batched generation, where Gi cannot be
// hoisted out of the time loop (the input is the layer below at the same step).
constexpr int FNS = 4, BNS = 6;
// NS: LDS ring depth.  4 (112 KiB, one workgroup per CU) when the grid is about one wave of
// workgroups (training at H = 2048: 256 tiles); 2 (56 KiB, two per CU) for big-batch generation,
// where several rounds of tiles per CU need the second workgroup to hide latency.
// (A 5-deep ring and nontemporal saves measured slower and were removed in round 4:
// profiles/r2_h2048_skns3_ab.jsonl.)
template <bool FUSED, int NS>
__global__ void __launch_bounds__(256, NS == 2 ? 2 : 1) gru_fwd_step_lds_kernel(FwdStepArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[NS][(128 + 96) * 64];
  const int H = a.H;
  const int j0 = blockIdx.x * 32, b0 = blockIdx.y * 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;

  // ---- epilogue operands first (latency hides under the K loop)
  constexpr int NGI = FUSED ? 1 : 4;
  float gi[NGI][4][3], bh[3], bi[3], hp[4][4];
  const int u = j0 + wn * 16 + lr;
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    bh[g] = a.bhh[g * H + u];
    bi[g] = FUSED ? a.bih[g * H + u] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) hp[i][e] = a.hprev_f[(size_t)(b0 + wm * 64 + i * 16 + lq * 4 + e) * H + u];
  if constexpr (!FUSED) {
    // source rows first (all 16 ids in one round trip), then the 48 gathers
    const float* src[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) src[i][e] = a.Gi + (size_t)(b0 + wm * 64 + i * 16 + lq * 4 + e) * 3 * H;
    if (a.ids) {
      const int4* id4 = reinterpret_cast<const int4*>(a.ids + b0 + wm * 64 + lq * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int4 v = id4[i * 4];
        src[i][0] = a.P + (size_t)v.x * 3 * H; src[i][1] = a.P + (size_t)v.y * 3 * H;
        src[i][2] = a.P + (size_t)v.z * 3 * H; src[i][3] = a.P + (size_t)v.w * 3 * H;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int g = 0; g < 3; ++g) gi[i][e][g] = src[i][e][g * H + u];
  }

  f32x4 acc[4][3];
  f32x4 accN[FUSED ? 4 : 1];   // input part of the n gate (FUSED)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FUSED) accN[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // one K phase: A rows b0.. of Am [.][K], B rows (gate, unit) -> Bm row g*H + j0 + unit; the n
  // gate accumulates into acc[.][2] or (input phase) accN
  auto phase = [&](const u16* Am, const u16* Bm, int K, auto input_tag) {
    constexpr bool input = decltype(input_tag)::value;
    const u16* srcA[4];
    const u16* srcB[3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (4 * w + q) * 8 + srow;
      srcA[q] = Am + (size_t)(b0 + r) * K + swz(r, sslot) * 8;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int r = (3 * w + q) * 8 + srow;       // 0..95
      srcB[q] = Bm + (size_t)((r >> 5) * H + j0 + (r & 31)) * K + swz(r, sslot) * 8;
    }
    auto stage = [&](int buf, int kt) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(srcA[q] + kt * 64, (lds_void_t*)(&lds[buf][(4 * w + q) * 8 * 64]), 16, 0, 0);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        __builtin_amdgcn_global_load_lds(srcB[q] + kt * 64, (lds_void_t*)(&lds[buf][(128 + (3 * w + q) * 8) * 64]), 16, 0, 0);
    };
    ring_loop<NS, 7>(K / 64, stage, [&](int cur) {
      const u16* LA = lds[cur];
      const u16* LB = lds[cur] + 128 * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + lq;
        bf16x8 af[4], bfr[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + lr;
          af[i] = *reinterpret_cast<const bf16x8*>(&LA[r * 64 + swz(r, c) * 8]);
        }
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const int r = g * 32 + wn * 16 + lr;
          bfr[g] = *reinterpret_cast<const bf16x8*>(&LB[r * 64 + swz(r, c) * 8]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i][0] = mfma16(af[i], bfr[0], acc[i][0]);
          acc[i][1] = mfma16(af[i], bfr[1], acc[i][1]);
          if constexpr (FUSED && input) accN[FUSED ? i : 0] = mfma16(af[i], bfr[2], accN[FUSED ? i : 0]);
          else acc[i][2] = mfma16(af[i], bfr[2], acc[i][2]);
        }
      }
    });
  };
  if constexpr (FUSED) phase(a.x_bf, a.Wih, a.Kin, std::true_type{});
  phase(a.hprev_bf, a.Whh, H, std::false_type{});

  // ---- fused GRU epilogue from registers; bf16 h tile staged in LDS for the transposed copy
  u16* st = lds[0];     // [128 rows][32 units]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rr = wm * 64 + i * 16 + lq * 4 + e;
      const int b = b0 + rr;
      const float ghr = acc[i][0][e] + bh[0], ghz = acc[i][1][e] + bh[1], ghn = acc[i][2][e] + bh[2];
      float gir, giz, gin;
      if constexpr (FUSED) { gir = bi[0]; giz = bi[1]; gin = accN[FUSED ? i : 0][e] + bi[2]; }
      else { gir = gi[FUSED ? 0 : i][e][0]; giz = gi[FUSED ? 0 : i][e][1]; gin = gi[FUSED ? 0 : i][e][2]; }
      const float r = sigmoidf_(gir + ghr);
      const float z = sigmoidf_(giz + ghz);
      const float n = tanhf_(gin + r * ghn);
      const float h = n + z * (hp[i][e] - n);
      const size_t o = (size_t)b * H + u;
      a.h_f[o] = h;
      const u16 hb = f2bf(h);
      a.h_bf[o] = hb;
      if (a.s16) st_save16(a.s16 + o * 4, r, z, n, ghn);
      else if (a.sr) { a.sr[o] = r; a.sz[o] = z; a.sn[o] = n; a.sghn[o] = ghn; }
      st[rr * 32 + wn * 16 + lr] = hb;
    }
  if (a.hT) {
    __syncthreads();
    // 32 units x 128 rows: 512 x 16-B pieces, 2 per thread
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int q = threadIdx.x + p * 256;
      const int unit = q >> 4, seg = q & 15;          // 16 segments of 8 rows
      u16 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = st[(seg * 8 + k) * 32 + unit];
      *reinterpret_cast<uint4*>(a.hT + (size_t)(j0 + unit) * a.ldT + a.colT + b0 + seg * 8) =
          *reinterpret_cast<const uint4*>(v);
    }
  }
}

// 64-row forward (default where the 128-row tile would give one workgroup per CU; StepLdsVariants::fwd64 = 0
// reverts, 2 = 4-deep ring): tile 64 rows x 32 units x 3 gates, 4 waves of 32 rows x 16 units, a
// 3-deep ring of 20 KiB slots, two workgroups per CU.  At B = 512, H = 2048 that is 512 workgroups:
// twice the k-tile streams in flight per CU of the 128-row tile, for 1.4x its L2 bytes per FLOP
// (the W_hh tile is shared by 64 rows instead of 128): h2048 step 9.72-9.74 -> 9.43-9.47 ms
// (profiles/r2_h2048_fwd64_ab.jsonl).  Training path only (no fused input phase).
// FUSED: layers >= 1 of batched generation -- the input projection as a first K phase (A = x rows,
// B = W_ih gate rows) ahead of the recurrent one, as in the 128-row kernel.
template <int NS, bool FUSED = false>
__global__ void __launch_bounds__(256, 2) gru_fwd_step_lds64_kernel(FwdStepArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[NS][(64 + 96) * 64];
  const int H = a.H;
  const int j0 = blockIdx.x * 32, b0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;
  const int u = j0 + wn * 16 + lr;

  constexpr int NGI = FUSED ? 1 : 2;
  float gi[NGI][4][3], bh[3], bi[3], hp[2][4];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    bh[g] = a.bhh[g * H + u];
    bi[g] = FUSED ? a.bih[g * H + u] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) hp[i][e] = a.hprev_f[(size_t)(b0 + wm * 32 + i * 16 + lq * 4 + e) * H + u];
  if constexpr (!FUSED) {
    const float* src[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) src[i][e] = a.Gi + (size_t)(b0 + wm * 32 + i * 16 + lq * 4 + e) * 3 * H;
    if (a.ids) {
      const int4* id4 = reinterpret_cast<const int4*>(a.ids + b0 + wm * 32 + lq * 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int4 v = id4[i * 4];
        src[i][0] = a.P + (size_t)v.x * 3 * H; src[i][1] = a.P + (size_t)v.y * 3 * H;
        src[i][2] = a.P + (size_t)v.z * 3 * H; src[i][3] = a.P + (size_t)v.w * 3 * H;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int g = 0; g < 3; ++g) gi[FUSED ? 0 : i][e][g] = src[i][e][g * H + u];
  }

  f32x4 acc[2][3];
  f32x4 accN[FUSED ? 2 : 1];   // input part of the n gate (FUSED)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FUSED) accN[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // one K phase: A rows b0.. of Am [.][K], B rows (gate, unit) -> Bm row g*H + j0 + unit.
  // 20 DMA pieces per k-tile, 5 per wave: piece p = 5w + q, image rows 8p..8p+7 (A for p < 8)
  auto phase = [&](const u16* Am, const u16* Bm, int K, auto input_tag) {
    constexpr bool input = decltype(input_tag)::value;
    const u16* src[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int p = 5 * w + q, r = p * 8 + srow;
      if (p < 8) {
        src[q] = Am + (size_t)(b0 + r) * K + swz(r, sslot) * 8;
      } else {
        const int rb = r - 64;
        src[q] = Bm + (size_t)((rb >> 5) * H + j0 + (rb & 31)) * K + swz(rb, sslot) * 8;
      }
    }
    auto stage = [&](int buf, int kt) {
#pragma unroll
      for (int q = 0; q < 5; ++q)
        __builtin_amdgcn_global_load_lds(src[q] + kt * 64, (lds_void_t*)(&lds[buf][(5 * w + q) * 8 * 64]), 16, 0, 0);
    };
    ring_loop<NS, 5>(K / 64, stage, [&](int cur) {
      const u16* LA = lds[cur];
      const u16* LB = lds[cur] + 64 * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + lq;
        bf16x8 af[2], bfr[3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = wm * 32 + i * 16 + lr;
          af[i] = *reinterpret_cast<const bf16x8*>(&LA[r * 64 + swz(r, c) * 8]);
        }
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const int r = g * 32 + wn * 16 + lr;
          bfr[g] = *reinterpret_cast<const bf16x8*>(&LB[r * 64 + swz(r, c) * 8]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc[i][0] = mfma16(af[i], bfr[0], acc[i][0]);
          acc[i][1] = mfma16(af[i], bfr[1], acc[i][1]);
          if constexpr (FUSED && input) accN[FUSED ? i : 0] = mfma16(af[i], bfr[2], accN[FUSED ? i : 0]);
          else acc[i][2] = mfma16(af[i], bfr[2], acc[i][2]);
        }
      }
    });
  };
  if constexpr (FUSED) phase(a.x_bf, a.Wih, a.Kin, std::true_type{});
  phase(a.hprev_bf, a.Whh, H, std::false_type{});

  u16* st = lds[0];     // [64 rows][32 units]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rr = wm * 32 + i * 16 + lq * 4 + e;
      const int b = b0 + rr;
      const float ghr = acc[i][0][e] + bh[0], ghz = acc[i][1][e] + bh[1], ghn = acc[i][2][e] + bh[2];
      float gir, giz, gin;
      if constexpr (FUSED) { gir = bi[0]; giz = bi[1]; gin = accN[FUSED ? i : 0][e] + bi[2]; }
      else { gir = gi[FUSED ? 0 : i][e][0]; giz = gi[FUSED ? 0 : i][e][1]; gin = gi[FUSED ? 0 : i][e][2]; }
      const float r = sigmoidf_(gir + ghr);
      const float z = sigmoidf_(giz + ghz);
      const float n = tanhf_(gin + r * ghn);
      const float h = n + z * (hp[i][e] - n);
      const size_t o = (size_t)b * H + u;
      a.h_f[o] = h;
      const u16 hb = f2bf(h);
      a.h_bf[o] = hb;
      if (a.s16) st_save16(a.s16 + o * 4, r, z, n, ghn);
      else if (a.sr) { a.sr[o] = r; a.sz[o] = z; a.sn[o] = n; a.sghn[o] = ghn; }
      st[rr * 32 + wn * 16 + lr] = hb;
    }
  if (a.hT) {
    __syncthreads();
    // 32 units x 64 rows: 256 x 16-B pieces, 1 per thread
    const int q = threadIdx.x;
    const int unit = q >> 3, seg = q & 7;
    u16 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = st[(seg * 8 + k) * 32 + unit];
    *reinterpret_cast<uint4*>(a.hT + (size_t)(j0 + unit) * a.ldT + a.colT + b0 + seg * 8) =
        *reinterpret_cast<const uint4*>(v);
  }
}

// (Round 2's 8-wave variant of the 128 x 96 forward tile -- two wave groups splitting each k-tile,
// h2048 9.84 -> 9.71 ms, profiles/r2_h2048_fwd8_ab.jsonl -- was removed in round 5: the 64-row tile
// below took every grid it served, so no default plan launched it.)

// ==================================================================== forward, big batch
// Tile 256 rows x 64 units x 3 gates for big-batch steps (batched generation: 4096+ names): 8 waves
// of 64 rows x 32 units, each holding the r/z/n pre-activations of its items in acc[4][2][3]
// (+ the input part of n in accN when FUSED).  Per 64-deep k-tile a wave issues 7 LDS-DMA pieces
// for 48 MFMAs -- twice the MFMA work per DMA piece of the 128 x 96 tile, whose issue cost bounds
// it.  2-deep ring of 56 KiB slots; epilogue operands are gathered after the K loop (the
// accumulators take the register file).
template <bool FUSED>
__global__ void __launch_bounds__(512, 1) gru_fwd_step_big_kernel(FwdStepArgs a) {
  constexpr int NS = 2, RA = 256, RB = 192, NP = (RA + RB) / 8 / 8;   // pieces per wave per k-tile
  __shared__ __attribute__((aligned(16))) u16 lds[NS][(RA + RB) * 64];
  const int H = a.H;
  const int j0 = blockIdx.x * 64, b0 = blockIdx.y * RA;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;

  f32x4 acc[4][2][3];
  f32x4 accN[FUSED ? 4 : 1][FUSED ? 2 : 1];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
#pragma unroll
      for (int g = 0; g < 3; ++g) acc[i][jt][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (FUSED) accN[i][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  auto phase = [&](const u16* Am, const u16* Bm, int K, auto input_tag) {
    constexpr bool input = decltype(input_tag)::value;
    // piece p = w*NP + q covers image rows 8p..8p+7: A rows (batch) below RA, then B rows
    // (gate g = rb / 64, unit rb % 64 -> W row g*H + j0 + unit)
    const u16* src[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int r = (w * NP + q) * 8 + srow;
      if (r < RA) {
        src[q] = Am + (size_t)(b0 + r) * K + swz(r, sslot) * 8;
      } else {
        const int rb = r - RA;
        src[q] = Bm + (size_t)((rb >> 6) * H + j0 + (rb & 63)) * K + swz(rb, sslot) * 8;
      }
    }
    auto stage = [&](int buf, int kt) {
#pragma unroll
      for (int q = 0; q < NP; ++q)
        __builtin_amdgcn_global_load_lds(src[q] + kt * 64, (lds_void_t*)(&lds[buf][(w * NP + q) * 8 * 64]), 16, 0, 0);
    };
    ring_loop<NS, NP>(K / 64, stage, [&](int cur) {
      const u16* LA = lds[cur];
      const u16* LB = lds[cur] + RA * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + lq;
        bf16x8 af[4], bfr[2][3];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm * 64 + i * 16 + lr;
          af[i] = *reinterpret_cast<const bf16x8*>(&LA[r * 64 + swz(r, c) * 8]);
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            const int r = g * 64 + wn * 32 + jt * 16 + lr;
            bfr[jt][g] = *reinterpret_cast<const bf16x8*>(&LB[r * 64 + swz(r, c) * 8]);
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) {
            acc[i][jt][0] = mfma16(af[i], bfr[jt][0], acc[i][jt][0]);
            acc[i][jt][1] = mfma16(af[i], bfr[jt][1], acc[i][jt][1]);
            if constexpr (FUSED && input) accN[FUSED ? i : 0][FUSED ? jt : 0] = mfma16(af[i], bfr[jt][2], accN[FUSED ? i : 0][FUSED ? jt : 0]);
            else acc[i][jt][2] = mfma16(af[i], bfr[jt][2], acc[i][jt][2]);
          }
      }
    });
  };
  if constexpr (FUSED) phase(a.x_bf, a.Wih, a.Kin, std::true_type{});
  phase(a.hprev_bf, a.Whh, H, std::false_type{});

  // ---- epilogue: per unit tile, gather this lane's operands, then the GRU math; bf16 h tile
  // staged in LDS [256 rows][64 units] for the transposed copy
  u16* st = lds[0];
  const int* idp = a.ids ? a.ids + b0 + wm * 64 + lq * 4 : nullptr;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int uu = wn * 32 + jt * 16 + lr, u = j0 + uu;
    float bh[3], bi[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      bh[g] = a.bhh[g * H + u];
      bi[g] = FUSED ? a.bih[g * H + u] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float gi[4][3], hp[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int b = b0 + wm * 64 + i * 16 + lq * 4 + e;
        hp[e] = a.hprev_f[(size_t)b * H + u];
        if constexpr (!FUSED) {
          const float* src = idp ? a.P + (size_t)idp[i * 16 + e] * 3 * H : a.Gi + (size_t)b * 3 * H;
#pragma unroll
          for (int g = 0; g < 3; ++g) gi[e][g] = src[g * H + u];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = wm * 64 + i * 16 + lq * 4 + e, b = b0 + rr;
        const float ghr = acc[i][jt][0][e] + bh[0], ghz = acc[i][jt][1][e] + bh[1], ghn = acc[i][jt][2][e] + bh[2];
        float gir, giz, gin;
        if constexpr (FUSED) { gir = bi[0]; giz = bi[1]; gin = accN[FUSED ? i : 0][FUSED ? jt : 0][e] + bi[2]; }
        else { gir = gi[e][0]; giz = gi[e][1]; gin = gi[e][2]; }
        const float r = sigmoidf_(gir + ghr);
        const float z = sigmoidf_(giz + ghz);
        const float n = tanhf_(gin + r * ghn);
        const float h = n + z * (hp[e] - n);
        const size_t o = (size_t)b * H + u;
        a.h_f[o] = h;
        const u16 hb = f2bf(h);
        a.h_bf[o] = hb;
        if (a.s16) st_save16(a.s16 + o * 4, r, z, n, ghn);
      else if (a.sr) { a.sr[o] = r; a.sz[o] = z; a.sn[o] = n; a.sghn[o] = ghn; }
        st[rr * 64 + uu] = hb;
      }
    }
  }
  if (a.hT) {
    __syncthreads();
    // 64 units x 256 rows: 2048 x 16-B pieces, 4 per thread
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = threadIdx.x + p * 512;
      const int unit = q >> 5, seg = q & 31;          // 32 segments of 8 rows
      u16 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = st[(seg * 8 + k) * 64 + unit];
      *reinterpret_cast<uint4*>(a.hT + (size_t)(j0 + unit) * a.ldT + a.colT + b0 + seg * 8) =
          *reinterpret_cast<const uint4*>(v);
    }
  }
}

// ==================================================================== backward
// tile 64 rows x 64 units over K = 3H (the 4-wave version of this kernel lost to the 8-wave one
// below: r1_bwd_lds8_ab.json, removed in round 4).
// 8 waves: two wave groups split every 64-deep k-tile by its two
// 32-deep k-steps (group g does k-step g), so each wave issues half the LDS-DMA pieces and half the
// MFMAs of a 4-wave kernel and two waves share each SIMD (one's DMA issue and LDS latency hide
// under the other's MFMAs).  Group 1's partial dh tile is added to group 0's through LDS before the
// epilogue.
__global__ void __launch_bounds__(512, 1) gru_bwd_step_lds8_kernel(BwdStepArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[BNS][(64 + 64) * 64];
  const int H = a.H, H3 = 3 * a.H;
  const int j0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, grp = w >> 2, wl = w & 3;
  const int wm = wl >> 1, wn = wl & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;

  // epilogue operands (group 0), loaded ahead of the K loop so their latency hides under it:
  // element (i, jt, e) -> row b0 + wm*32 + i*16 + lq*4 + e, unit j0 + wn*32 + jt*16 + lr
  float dy[2][2][4], cin[2][2][4], sr_[2][2][4], sz_[2][2][4], sn_[2][2][4], sg_[2][2][4], hpv[2][2][4];
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const size_t o = (size_t)(b0 + wm * 32 + i * 16 + lq * 4 + e) * H + j0 + wn * 32 + jt * 16 + lr;
          dy[i][jt][e] = a.dy[o];
          cin[i][jt][e] = a.carry_in ? a.carry_in[o] : 0.f;
          sr_[i][jt][e] = a.r[o]; sz_[i][jt][e] = a.z[o]; sn_[i][jt][e] = a.n[o];
          sg_[i][jt][e] = a.ghn[o]; hpv[i][jt][e] = a.hprev[o];
        }
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.dgh_next) {
    // 16 DMA pieces (8 rows x 128 B) per k-tile: piece p = 2w + q covers image rows 8p..8p+7,
    // the A rows (dGh_{t+1}) for p < 8, the B rows (W_hh^T) after
    const u16* src[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = (2 * w + q) * 8 + srow, rr = r & 63;
      const u16* base = r < 64 ? a.dgh_next + (size_t)(b0 + rr) * H3 : a.WhhT + (size_t)(j0 + rr) * H3;
      src[q] = base + swz(rr, sslot) * 8;
    }
    auto stage = [&](int buf, int kt) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds(src[q] + kt * 64, (lds_void_t*)(&lds[buf][(2 * w + q) * 8 * 64]), 16, 0, 0);
    };
    ring_loop<BNS, 2>(H3 / 64, stage, [&](int cur) {
      const u16* LA = lds[cur];
      const u16* LB = lds[cur] + 64 * 64;
      const int c = grp * 4 + lq;   // this group's 32-deep k-step
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ra = wm * 32 + t * 16 + lr, rb = wn * 32 + t * 16 + lr;
        af[t] = *reinterpret_cast<const bf16x8*>(&LA[ra * 64 + swz(ra, c) * 8]);
        bfr[t] = *reinterpret_cast<const bf16x8*>(&LB[rb * 64 + swz(rb, c) * 8]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    });
    // group 1 -> LDS -> group 0 (ring_loop ended with a barrier: the ring is free)
    f32x4* red = reinterpret_cast<f32x4*>(&lds[0][0]);   // [4 waves][4 tiles][64 lanes]
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) red[(wl * 4 + i * 2 + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] += red[(wl * 4 + i * 2 + j) * 64 + lane];
    }
    __syncthreads();
  }

  // ---- gate-gradient epilogue (group 0); transposed staging [4 kinds][64 units][64 rows] bf16
  u16* st = lds[0];
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = wm * 32 + i * 16 + lq * 4 + e, uu = wn * 32 + jt * 16 + lr;
          const int b = b0 + rr, j = j0 + uu;
          const size_t o = (size_t)b * H + j;
          const float dh = dy[i][jt][e] + cin[i][jt][e] + acc[i][jt][e];
          const float r = sr_[i][jt][e], z = sz_[i][jt][e], n = sn_[i][jt][e];
          const float dn = dh * (1.f - z);
          const float dz = dh * (hpv[i][jt][e] - n);
          const float dan = dn * (1.f - n * n);
          const float dar = dan * sg_[i][jt][e] * r * (1.f - r);
          const float daz = dz * z * (1.f - z);
          a.carry_out[o] = z * dh;
          const u16 br = f2bf(dar), bz = f2bf(daz), bn = f2bf(dan * r), bi = f2bf(dan);
          const size_t og = (size_t)b * H3 + j;
          a.dgh[og] = br; a.dgh[og + H] = bz; a.dgh[og + 2 * H] = bn;
          if (a.dgi) { a.dgi[og] = br; a.dgi[og + H] = bz; a.dgi[og + 2 * H] = bi; }
          st[(0 * 64 + uu) * 64 + rr] = br;
          st[(1 * 64 + uu) * 64 + rr] = bz;
          st[(2 * 64 + uu) * 64 + rr] = bn;
          st[(3 * 64 + uu) * 64 + rr] = bi;
        }
  }
  __syncthreads();
  // 4 kinds x 64 units x 64 rows = 2048 pieces of 8 rows (16 B), 4 per thread
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int q = threadIdx.x + p * 512;
    const int kind = q >> 9, rem = q & 511, unit = rem >> 3, seg = rem & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(&st[(kind * 64 + unit) * 64 + seg * 8]);
    const int g = kind < 3 ? kind : 2;
    const size_t off = (size_t)(g * H + j0 + unit) * a.ldT + a.colT + b0 + seg * 8;
    if (kind < 3 && a.dghT) *reinterpret_cast<uint4*>(a.dghT + off) = v;
    if (a.dgiT && (kind == 3 || (kind < 2 && !a.dgiT_n_only))) *reinterpret_cast<uint4*>(a.dgiT + off) = v;
  }
}

// ==================================================================== backward, split-K
// Large-batch backward step (B = 512, H = 2048: dh = dGh_{t+1} · W_hh is 512 x 2048 x 6144).  The
// 64 x 64 kernel above streams (64 + 64) x 3H operands per workgroup: 1.5 MB at H = 2048, bound
// by the per-CU L2 read rate.  Here a workgroup owns a 128 x 128 tile over a 1/S slice of K (half
// the operand bytes per output), S workgroups per tile fill the chip, and they meet through
// global memory: each writes its fp32 partial tile write-through (sc1), drains, bumps the tile's
// arrival counter, and waits until all S have arrived; then workgroup s sums the S partials in
// slab order 0, 1, ... (deterministic, whoever runs it) for its share of the tile's rows and runs
// the gate-gradient epilogue there.  All workgroups are co-resident (the host checks occupancy),
// other kernels' workgroups never wait, so every spin ends; it is bounded anyway (error word).
// Counters are monotonic: launch k of a tile leaves them at k*S, so no reset node is needed.
namespace {
typedef unsigned int sk_u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t sk_rsrc_t;
DEV sk_rsrc_t sk_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
constexpr int SKNS = 4;                       // LDS ring: 4 x 32 KiB
constexpr unsigned kSkSpinLimit = 1u << 21;   // x s_sleep(1): far beyond any real wait
}

// NS: LDS ring depth (4 x 32 KiB; 3 and 5 measured equal / slower: profiles/r2_h2048_skns3_ab.jsonl).
// PF (default): the epilogue's fp32 operands (dy, carry, saves, h_{t-1}) are loaded before the K
// loop, so their latency hides under it instead of following the split-K exchange (h2048 step
// 10.36-10.50 -> 9.82-9.85 ms, profiles/r2_h2048_step_variants_ab.jsonl); always on at S = 4.
template <int S, int NS = SKNS, bool PF = false>
__global__ void __launch_bounds__(512, 1) gru_bwd_step_sk_kernel(BwdStepArgs a) {
  static_assert(!PF || S == 4, "prefetch holds one epilogue quarter");
  __shared__ __attribute__((aligned(16))) u16 lds[NS][256 * 64];
  const int H = a.H, H3 = 3 * a.H;
  // block -> (tile, split), a speed choice only (the exchange does not depend on placement):
  //  sk_map 0: the S splits of a tile are 8 blocks apart (one XCD under the dispatcher's round-robin
  //            placement): an XCD streams 2 unit tiles x every row tile over ALL of K (9 MB at B = 512,
  //            H = 2048 -- more than its 4 MB L2);
  //  sk_map 1: XCD x (= bid % 8) takes split x % S of every row tile of 1/(8/S) of the unit tiles:
  //            one K-slice of the operands (4.5 MB), the S partners of a tile on S different XCDs.
  const int bid = blockIdx.x;
  const int ntu = H / 128;
  int split, tile;
  if (a.sk_map == 1) {
    const int ntr = a.Bp / 128, x = bid & 7, i = bid >> 3, G = 8 / S;
    split = x % S;
    const int ut = i / ntr + (ntu / G) * (x / S), rt = i % ntr;
    tile = rt * ntu + ut;
  } else {
    split = (bid >> 3) % S;
    tile = (bid / (8 * S)) * 8 + (bid & 7);
  }
  const int j0 = (tile % ntu) * 128, b0 = (tile / ntu) * 128;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;             // K loop: wave = 64 rows x 32 units
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;
  constexpr int NQ = 4 / S;                       // epilogue quarters (32 rows) per workgroup
  constexpr int PIECE = 8 * 4 * 2 * 64;           // f32x4 per partial tile: [wave][i][jn][lane]
  const bool kloop = a.dgh_next != nullptr;

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // epilogue element (quarter qq, piece pp, row e) -> offset into the [Bp][H] operands
  auto epi_off = [&](int qq, int pp, int e) {
    const int sq = split + S * qq, P = w + 8 * pp;
    const int wnp = P >> 2, ii = (P >> 1) & 1, jn = P & 1;
    const int b = b0 + 32 * sq + ii * 16 + lq * 4 + e;
    return (size_t)b * H + j0 + wnp * 32 + jn * 16 + lr;
  };
  float pre[PF ? 2 : 1][4][6];
  if constexpr (PF) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t o = epi_off(0, pp, e);
        pre[pp][e][0] = a.dy[o] + (a.carry_in ? a.carry_in[o] : 0.f);
        pre[pp][e][1] = a.r[o]; pre[pp][e][2] = a.z[o]; pre[pp][e][3] = a.n[o];
        pre[pp][e][4] = a.hprev[o]; pre[pp][e][5] = a.ghn[o];
      }
  }
  const sk_rsrc_t rP = sk_rsrc(a.sk_part, (unsigned)(a.sk_part_floats * 4));
  const size_t tile_base = (size_t)tile * S * PIECE;   // f32x4 units
  if (kloop) {
    const int nk = H3 / 64 / S, kt0 = split * nk;
    // 32 DMA pieces (8 rows x 128 B) per k-tile, 4 per wave: image rows 0..127 = A (dGh_{t+1}),
    // 128..255 = B (W_hh^T)
    const u16* src[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (4 * w + q) * 8 + srow, rr = r & 127;
      const u16* base = r < 128 ? a.dgh_next + (size_t)(b0 + rr) * H3 : a.WhhT + (size_t)(j0 + rr) * H3;
      src[q] = base + swz(rr, sslot) * 8 + (size_t)kt0 * 64;
    }
    auto stage = [&](int buf, int kt) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(src[q] + kt * 64, (lds_void_t*)(&lds[buf][(4 * w + q) * 8 * 64]), 16, 0, 0);
    };
    ring_loop<NS, 4>(nk, stage, [&](int cur) {
      const u16* LA = lds[cur];
      const u16* LB = lds[cur] + 128 * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + lq;
        bf16x8 af[4], bfr[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ra = wm * 64 + i * 16 + lr;
          af[i] = *reinterpret_cast<const bf16x8*>(&LA[ra * 64 + swz(ra, c) * 8]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int rb = wn * 32 + j * 16 + lr;
          bfr[j] = *reinterpret_cast<const bf16x8*>(&LB[rb * 64 + swz(rb, c) * 8]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
    });
    // publish this split's partial tile (write-through), drain, arrive, wait for all S
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const size_t o = tile_base + (size_t)split * PIECE + ((w * 4 + i) * 2 + j) * 64 + lane;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u32x4, acc[i][j]), rP, (unsigned)(o * 16), 0, 16);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned* cnt = a.sk_cnt + (size_t)tile * 16;
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (old / S + 1) * S;
      unsigned spins = 0;
      while ((int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSkSpinLimit) {
          if (a.err) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
  }

  // ---- epilogue: quarter sq = rows 32 sq .. 32 sq + 31 of the tile; thread piece P = w + 8 pp
  // covers partial fragment (wave wm_q*4 + P/4, i = 2(sq&1) + (P/2)&1, jn = P&1) of every slab:
  // 4 rows x 1 unit per piece, 8 items per thread.  Transposed staging [4 kinds][128 units][40].
  u16* st = lds[0];
#pragma unroll
  for (int qq = 0; qq < NQ; ++qq) {
    const int sq = split + S * qq;
    const int wmq = sq >> 1, ib = 2 * (sq & 1);
    if (qq) __syncthreads();   // the previous quarter's transposed reads are done with st
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int P = w + 8 * pp;
      const int wnp = P >> 2, ii = (P >> 1) & 1, jn = P & 1, i = ib + ii;
      f32x4 ps = f32x4{0.f, 0.f, 0.f, 0.f};
      if (kloop) {
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) {
          const size_t o = tile_base + (size_t)s2 * PIECE + (((wmq * 4 + wnp) * 4 + i) * 2 + jn) * 64 + lane;
          ps += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rP, (unsigned)(o * 16), 0, 16));
        }
      }
      const int ut = wnp * 32 + jn * 16 + lr;   // unit within the tile
      const int j = j0 + ut;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rq = ii * 16 + lq * 4 + e;    // row within the quarter
        const int b = b0 + 32 * sq + rq;
        const size_t o = (size_t)b * H + j;
        float dh, r, z, n, hp, ghn;
        if constexpr (PF) {
          dh = pre[pp][e][0] + ps[e]; r = pre[pp][e][1]; z = pre[pp][e][2]; n = pre[pp][e][3];
          hp = pre[pp][e][4]; ghn = pre[pp][e][5];
        } else {
          dh = a.dy[o] + (a.carry_in ? a.carry_in[o] : 0.f) + ps[e];
          r = a.r[o]; z = a.z[o]; n = a.n[o]; hp = a.hprev[o]; ghn = a.ghn[o];
        }
        const float dn = dh * (1.f - z);
        const float dz = dh * (hp - n);
        const float dan = dn * (1.f - n * n);
        const float dar = dan * ghn * r * (1.f - r);
        const float daz = dz * z * (1.f - z);
        a.carry_out[o] = z * dh;
        const u16 br = f2bf(dar), bz = f2bf(daz), bn = f2bf(dan * r), bi = f2bf(dan);
        const size_t og = (size_t)b * H3 + j;
        a.dgh[og] = br; a.dgh[og + H] = bz; a.dgh[og + 2 * H] = bn;
        if (a.dgi) { a.dgi[og] = br; a.dgi[og + H] = bz; a.dgi[og + 2 * H] = bi; }
        st[(0 * 128 + ut) * 40 + rq] = br;
        st[(1 * 128 + ut) * 40 + rq] = bz;
        st[(2 * 128 + ut) * 40 + rq] = bn;
        st[(3 * 128 + ut) * 40 + rq] = bi;
      }
    }
    __syncthreads();
    // 4 kinds x 128 units x 32 rows = 2048 pieces of 8 rows (16 B), 4 per thread
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = tid + p * 512;
      const int kind = q >> 9, rem = q & 511, unit = rem >> 2, seg = rem & 3;
      const uint4 v = *reinterpret_cast<const uint4*>(&st[(kind * 128 + unit) * 40 + seg * 8]);
      const int g = kind < 3 ? kind : 2;
      const size_t off = (size_t)(g * H + j0 + unit) * a.ldT + a.colT + b0 + 32 * sq + seg * 8;
      if (kind < 3 && a.dghT) *reinterpret_cast<uint4*>(a.dghT + off) = v;
      if (a.dgiT && (kind == 3 || (kind < 2 && !a.dgiT_n_only))) *reinterpret_cast<uint4*>(a.dgiT + off) = v;
    }
  }
}

// (A 64-row split-K backward with two workgroups per CU lost to this one: h2048 step 9.37-9.41 ->
// 10.04-10.05 ms, profiles/r2_h2048_bwd_sk64_ab.jsonl; removed in round 4.)

static int sk_capacity(const void* kernel, int threads = 512) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess) return 0;
  return per * cus;
}

int gru_bwd_step_sk_splits(int H, int Bp) {
  if (H % 128 || Bp % 128) return 0;
  const int tiles = (H / 128) * (Bp / 128);
  if (tiles % 8) return 0;
  static const int cap4 = sk_capacity((const void*)gru_bwd_step_sk_kernel<4>);
  static const int cap2 = sk_capacity((const void*)gru_bwd_step_sk_kernel<2>);
  // H = 2048 (K = 6144): 40.3 -> 35.4 us per step (profiles/r1_bwd_step_sk_ab.jsonl).  H = 1024 was
  // a loss before the epilogue operands moved ahead of the K loop (9.50 -> 9.62 ms per h1024_l2 step
  // at B = 1024); with them it gains: 8.67 -> 8.17-8.19 ms (profiles/r2_h1024l2_b1024_sk_ab.jsonl).
  if (H < step_lds_variants().bwd_sk_min_h) return 0;
  if ((3 * H / 64) % 4 == 0 && tiles * 4 <= cap4 && tiles * 4 >= 192) return 4;
  if ((3 * H / 64) % 2 == 0 && tiles * 2 <= cap2 && tiles * 2 >= 192) return 2;
  return 0;
}

StepLdsVariants& step_lds_variants() {
  static StepLdsVariants v;   // measured-best defaults; tests switch them at run time
  return v;
}

bool gru_step_lds_ok(int H, int Bp) { return H >= 256 && H % 64 == 0 && Bp % 128 == 0; }

void gru_fwd_step_lds(const FwdStepArgs& a, hipStream_t s) {
  // big tile: only with the fused input phase on a full round of tiles (without it, the P-table
  // gather moves behind the K loop and it measured slower: profiles/r1_generate_step_kernel_ab.json)
  if (a.x_bf && a.Kin % 64 == 0 && a.Bp % 256 == 0 && a.H % 64 == 0 && (a.H / 64) * (a.Bp / 256) >= 256) {
    hipLaunchKernelGGL(gru_fwd_step_big_kernel<true>, dim3(a.H / 64, a.Bp / 256), dim3(512), 0, s, a);
    return;
  }
  const dim3 grid(a.H / 32, a.Bp / 128), block(256);
  // grids of >= 512 128-row tiles: the 2-deep 128-row kernel, two workgroups per CU (the 64-row tile
  // there measured 74-75 -> 88 us per char at 2048 names, profiles/r2_generate_fwd64_all_ab.txt).
  // Smaller grids: the 64-row tile, two workgroups per CU, 3-deep ring (h2048 9.72 -> 9.43-9.47 ms,
  // profiles/r2_h2048_fwd64_ab.jsonl; fused input phase 55.8 -> 54.3-54.9 us per char at 1024 names,
  // r2_generate_fwd64_fused_ab.txt).  StepLdsVariants::fwd64 = 0 keeps the 128-row kernel everywhere.
  const bool small_grid = grid.x * grid.y < 512;
  if (small_grid && step_lds_variants().fwd64 && a.Bp % 64 == 0 && (!a.x_bf || a.Kin % 64 == 0)) {
    if (a.x_bf) hipLaunchKernelGGL((gru_fwd_step_lds64_kernel<3, true>), dim3(a.H / 32, a.Bp / 64), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(gru_fwd_step_lds64_kernel<3>, dim3(a.H / 32, a.Bp / 64), dim3(256), 0, s, a);
    return;
  }
  if (a.x_bf) hipLaunchKernelGGL((gru_fwd_step_lds_kernel<true, 2>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((gru_fwd_step_lds_kernel<false, 2>), grid, block, 0, s, a);
}
void gru_bwd_step_lds(const BwdStepArgs& a, hipStream_t s) {
  if (const int S = gru_bwd_step_sk_splits(a.H, a.Bp)) {
    const int tiles = (a.H / 128) * (a.Bp / 128);
    if (a.sk_part && a.sk_cnt && a.sk_part_floats >= (long)a.H * a.Bp * S && a.sk_cnt_words >= (long)tiles * 16) {
      BwdStepArgs b = a;
      // splits across XCDs where whole unit-tile groups fit per XCD (h2048 9.46-9.47 vs 9.49 ms,
      // profiles/r4_h2048_skmap.jsonl), else the splits of a tile 8 blocks apart
      b.sk_map = (a.H / 128) % (8 / S) == 0 ? 1 : 0;
      if (S == 4) hipLaunchKernelGGL((gru_bwd_step_sk_kernel<4, SKNS, true>), dim3(tiles * 4), dim3(512), 0, s, b);
      else hipLaunchKernelGGL(gru_bwd_step_sk_kernel<2>, dim3(tiles * 2), dim3(512), 0, s, b);
      return;
    }
  }
  hipLaunchKernelGGL(gru_bwd_step_lds8_kernel, dim3(a.H / 64, a.Bp / 64), dim3(512), 0, s, a);
}

}  // namespace gk
