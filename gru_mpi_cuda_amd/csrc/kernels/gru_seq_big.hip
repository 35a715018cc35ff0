// Persistent large-H backward recurrence: ONE launch runs all T backward steps
// of a layer whose per-step GEMM is a real GEMM (B = 512 rows, H = 2048: dh = dGh . W_hh is 12.9
// GFLOP per step), where the register-resident persistent kernels of gru_seq.hip do not fit and the
// per-step kernels of gru_step_lds.hip pay a launch, a grid ramp and a drain per timestep.
//
// (Round 4 also built the forward twin -- 256 workgroups of 128 rows x 32 units x 3 gates, W_hh
// streamed through a 4-deep LDS ring, T-deep per-producer h tiles with epoch flags.  Correct, and
// slower than the 64-row step kernels: h2048 forward 3.04-3.34 ms vs 2.89-2.97, step 9.24 vs 8.69-8.72
// ms, profiles/r4_h2048_big_v1_ab.jsonl, r4_h2048_big_acq_ab.jsonl, r4_h2048_h1024_big_ab.jsonl; removed.)
#include <stdexcept>
#include <type_traits>
#include <string>
#include "kernels.h"
#include "common.h"

namespace gk {

namespace {
typedef __attribute__((address_space(3))) void lds_void_g;
typedef __amdgpu_buffer_rsrc_t rsrc_g;
typedef unsigned int u32x4_g __attribute__((ext_vector_type(4)));
constexpr unsigned long long kSpinTicks = 500000000ull;   // 5 s of s_memrealtime (100 MHz)

DEV int swz(int r, int c) { return c ^ ((r >> 1) & 7); }
DEV rsrc_g mk_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
template <int N> DEV void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
}  // namespace

// ==================================================================== persistent large-H forward, 64-row tiles
// The 64-row forward step kernel's tile (gru_step_lds.hip gru_fwd_step_lds64_kernel: 64 rows x 32
// units x 3 gates, 4 waves of 32 x 16, a 3-deep ring of 20 KiB, two workgroups per CU -- one's
// epilogue under the other's K loop) with all T steps in one launch: (H/32) x (Bp/64) = 512
// workgroups at h2048 / h1024_l2 x 1024, all co-resident.  The unit group is the fast block index,
// so an XCD streams the W_hh slices of 1/8 of the unit groups (3.1 MB at H = 2048).  Per step:
// wave 0 polls the epoch flags of the row group's H/32 producers (sc1), then (xch_acquire) one agent
// acquire, a barrier, the K loop streams A = h_{t-1} of the 64 rows from the producers' [64][32]
// exchange tiles (T-deep) and B = W_hh; the bf16 h tile is staged in LDS and published (256 x 16-B
// sc1 stores, drain, barrier, one flag), and only then go the saves the backward reads (h fp32 and
// bf16, h^T, r / z / n / gh_n recomputed from the live accumulators) and the next step's inputs.
namespace {
constexpr int kF64NS = 3;   // LDS ring: 3 x (64 + 96) rows x 128 B = 60 KiB
}

__global__ void __launch_bounds__(256, 2) gru_fwd_seq64_kernel(SeqFwdArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[kF64NS][(64 + 96) * 64];   // one object: st aliases slot 0
  const int H = a.H, Bp = a.Bp, T = a.T;
  const int nrg = Bp / 64, ncg = H / 32;
  const int cg = blockIdx.x % ncg, rg = blockIdx.x / ncg;
  const int j0 = cg * 32, b0 = rg * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;
  const int u = j0 + wn * 16 + lr;
  const bool acq = a.xch_acquire != 0;
  auto row_of = [&](int i, int e) { return b0 + wm * 32 + i * 16 + lq * 4 + e; };
  float bh[3], hp[2][4], gi[2][4][3];
#pragma unroll
  for (int g = 0; g < 3; ++g) bh[g] = a.bhh[g * H + u];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) hp[i][e] = a.h0 ? a.h0[(size_t)row_of(i, e) * H + u] : 0.f;
  auto load_gi = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int b = row_of(i, e);
        const float* src = a.ids ? a.P + (size_t)a.ids[(size_t)t * Bp + b] * 3 * H : a.Gi + ((size_t)t * Bp + b) * 3 * H;
#pragma unroll
        for (int g = 0; g < 3; ++g) gi[i][e][g] = src[g * H + u];
      }
  };
  const size_t xstep = (size_t)nrg * ncg * 2048;   // exchange elements per step: [nrg][ncg][64][32]
  const rsrc_g rX = mk_rsrc(a.xch, (unsigned)((size_t)T * xstep * 2));
  const rsrc_g rH0 = mk_rsrc(a.HSb, (unsigned)((size_t)Bp * H * 2));   // HS[0] = h_init, row-major bf16
  unsigned* const flags = a.cnt + (size_t)rg * ncg * 16;
  // 20 LDS-DMA pieces (8 image rows) per k-tile, 5 per wave: image rows 0..63 = A, 64..159 = W_hh
  auto stage = [&](int buf, int kt, int t) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int p = 5 * w + q, r = p * 8 + srow;
      lds_void_g* dst = (lds_void_g*)(&lds[buf][p * 8 * 64]);
      if (p < 8) {
        const int c = swz(r, sslot);   // the logical 16-B chunk this lane's slot holds
        if (t > 0) {   // producer 2 kt + c / 4 of the row group, its tile row r, units 8 (c % 4) ..
          const unsigned off = (unsigned)(((((size_t)(t - 1) * nrg + rg) * ncg + 2 * kt + (c >> 2)) * 2048 + r * 32 + (c & 3) * 8) * 2);
          if (acq) __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, dst, 16, off, 0, 0, 0);
          else __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, dst, 16, off, 0, 0, 16);   // aux 16 = sc1
        } else {
          const unsigned off = (unsigned)(((size_t)(b0 + r) * H + kt * 64 + c * 8) * 2);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rH0, dst, 16, off, 0, 0, 0);
        }
      } else {
        const int rb = r - 64;
        const u16* src = a.Whh + (size_t)((rb >> 5) * H + j0 + (rb & 31)) * H + kt * 64 + swz(rb, sslot) * 8;
        __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
      }
    }
  };
  const int nk = H / 64;
  if (a.ids || a.Gi) load_gi(0);

  for (int t = 0; t < T; ++t) {
    f32x4 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 3; ++g) acc[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t > 0) {   // h_{t-1} of the row group: every producer's flag at epoch >= t
      if (w == 0) {
        unsigned long long t0 = 0;
        unsigned n = 0;
        for (;;) {
          bool ok = true;
          if (lane < ncg) ok = __hip_atomic_load(flags + lane * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)t;
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if ((n++ & 63u) == 0u) {   // (first check: the clock only, as gru_seq.hip SpinBudget)
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (!t0) t0 = now;
            else if (a.err && (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u)) break;
            else if (now - t0 > kSpinTicks) {
              if (lane == 0 && a.err) __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
        }
        if (acq) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
    }
    if (t > 0 || a.h0) {
      // 3-deep ring: 2 k-tiles in flight, one barrier per k-tile (5 pieces per wave per k-tile)
#pragma unroll
      for (int s2 = 0; s2 < kF64NS - 1; ++s2) stage(s2, s2, t);
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) vmwait<5>(); else vmwait<0>();
        lds_barrier();
        if (kt + kF64NS - 1 < nk) stage((kt + kF64NS - 1) % kF64NS, kt + kF64NS - 1, t);
        const u16* LA = lds[kt % kF64NS];
        const u16* LB = LA + 64 * 64;
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
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int g = 0; g < 3; ++g) acc[i][g] = mfma16(af[i], bfr[g], acc[i][g]);
        }
      }
      __syncthreads();   // every wave is done with the ring: slot 0 becomes the h staging tile
    }
    u16* st = lds[0];   // [64 rows][32 units] bf16
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float ghr = acc[i][0][e] + bh[0], ghz = acc[i][1][e] + bh[1], ghn = acc[i][2][e] + bh[2];
        const float r = sigmoidf_(gi[i][e][0] + ghr);
        const float z = sigmoidf_(gi[i][e][1] + ghz);
        const float n = tanhf_(gi[i][e][2] + r * ghn);
        const float h = n + z * (hp[i][e] - n);
        hp[i][e] = h;
        st[(wm * 32 + i * 16 + lq * 4 + e) * 32 + wn * 16 + lr] = f2bf(h);
      }
    __syncthreads();
    // publish: this producer's [64][32] tile, 16 B per thread, write-through; drain; one flag
    const u32x4_g hv4 = *reinterpret_cast<const u32x4_g*>(&st[tid * 8]);
    {
      const unsigned off = (unsigned)(((((size_t)t * nrg + rg) * ncg + cg) * 2048 + tid * 8) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(hv4, rX, off, 0, 16);   // aux 16 = sc1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flags + cg * 16, (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // after the signal: the saves of the backward (gates recomputed from the live accumulators)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t o = (size_t)row_of(i, e) * H + u;
        a.HSf[(size_t)(t + 1) * Bp * H + o] = hp[i][e];
        if (a.sr) {
          const float ghn = acc[i][2][e] + bh[2];
          const float r = sigmoidf_(gi[i][e][0] + acc[i][0][e] + bh[0]);
          const float z = sigmoidf_(gi[i][e][1] + acc[i][1][e] + bh[1]);
          const float n = tanhf_(gi[i][e][2] + r * ghn);
          const size_t so = (size_t)t * Bp * H + o;
          a.sr[so] = r; a.sz[so] = z; a.sn[so] = n; a.sghn[so] = ghn;
        }
      }
    // row-major bf16 h: row tid / 4, units 8 (tid % 4) ..
    *reinterpret_cast<u32x4_g*>(a.HSb + ((size_t)(t + 1) * Bp + b0 + (tid >> 2)) * H + j0 + (tid & 3) * 8) = hv4;
    if (a.HT) {   // transposed: unit tid / 8, rows 8 (tid % 8) ..
      const int unit = tid >> 3, seg = tid & 7;
      u16 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = st[(seg * 8 + k) * 32 + unit];
      *reinterpret_cast<uint4*>(a.HT + (size_t)(j0 + unit) * a.ldT + (size_t)(t + 1) * Bp + b0 + seg * 8) =
          *reinterpret_cast<const uint4*>(v);
    }
    if (t + 1 < T && (a.ids || a.Gi)) load_gi(t + 1);
    __syncthreads();   // st (ring slot 0) is refilled by the next step's K loop
  }
}

bool gru_fwd_seq64_supported(int H, int Bp) {
  if (H % 64 || Bp % 64 || H < 1024 || H / 32 > 64) return false;
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gru_fwd_seq64_kernel, 256, 0) != hipSuccess) return false;
  return (long)ncu * per >= (long)(H / 32) * (Bp / 64);
}

void gru_fwd_seq64(const SeqFwdArgs& a, hipStream_t s) {
  if (!gru_fwd_seq64_supported(a.H, a.Bp) || !a.xch || !a.cnt || !a.HSb || !a.HSf || !a.Whh || !a.bhh ||
      (!a.ids == !a.Gi) || (a.ids && !a.P))
    throw std::runtime_error("gru_fwd_seq64: unsupported shape or incomplete arguments");
  if ((size_t)a.T * a.Bp * a.H * 2 >= (1ull << 32))
    throw std::runtime_error("gru_fwd_seq64: exchange exceeds the 4 GB buffer range");
  hipLaunchKernelGGL(gru_fwd_seq64_kernel, dim3((a.H / 32) * (a.Bp / 64)), dim3(256), 0, s, a);
}

// ==================================================================== persistent large-H backward
// ONE launch runs all T backward steps of a layer at large H with a large batch (B = 512, H = 2048:
// dh = dGh_{t+1} . W_hh is 512 x 2048 x 6144 per step), replacing T launches of the split-K step
// kernel (gru_step_lds.hip gru_bwd_step_sk_kernel, whose tiling and epilogue it keeps):
//   * 256 workgroups = 64 tiles of 128 rows x 128 units, each over S = 4 K-slices; the block order of
//     sk_map 1 (XCD x takes split x % 4 of every row tile of half the unit tiles);
//   * per step t (descending): wave 0 polls the epoch flags of the dGh_{t+1} producers of this
//     workgroup's A operand (its 128 rows x K-slice: 4 row-quarter producers of each of the slice's
//     128-column blocks), then (xch_acquire) one agent acquire; the K loop streams A (T-deep
//     exchange: plain loads behind the acquire, or sc1) and W_hh^T (plain, its first ring slots issued
//     before the wait) through a 4-deep LDS ring; the fp32 partial tile goes out write-through (parity-double-buffered), one
//     flag per (tile, split), and the S partners wait for each other;
//   * the epilogue runs on row quarter `split` of the tile: partials summed in split order (the same
//     sum whoever runs it), the gate gradients, carry = z * dh kept in REGISTERS across steps (the
//     same thread owns the same elements every step), dGh_t staged row-major in LDS and published as
//     whole 256-B row segments (sc1) + drain + barrier + one flag -- only then dGi_t and the
//     transposed dGh^T / dGi^T (weight-gradient operands), which nobody in this launch reads.
// Flags (zeroed before the launch): dGh producers at cnt[(tile * 4 + split) * 16] = steps
// published, partial tiles at cnt[4096 + (tile * 4 + split) * 16] = the same count.
namespace {
constexpr int kBS = 4;                      // split-K partners per tile
constexpr int kBNS = 4;                     // LDS ring: 4 x (128 + 128) rows x 128 B = 128 KiB
constexpr int kPiece = 8 * 4 * 2 * 64;      // f32x4 per partial tile: [wave][i][jn][lane]
constexpr int kRowPad = 136;                // row-major staging pitch (u16): 272-B rows
DEV int big_bwd_ntu(int H) { return H / 128; }
}  // namespace

__global__ void __launch_bounds__(512, 1) gru_bwd_seq_big_kernel(SeqBwdArgs a) {
  // ONE __shared__ object (ring + bias accumulators): see the forward
  __shared__ __attribute__((aligned(16))) u16 lds_all[kBNS * 256 * 64 + 2 * 4 * 128 * 2];
  u16 (*lds)[256 * 64] = reinterpret_cast<u16 (*)[256 * 64]>(lds_all);
  const int H = a.H, H3 = 3 * H, Bp = a.Bp, T = a.T;
  const int ntu = big_bwd_ntu(H), ntr = Bp / 128;
  const int bid = blockIdx.x, x = bid & 7, ib = bid >> 3;
  const int split = x % kBS;
  const int ut = ib / ntr + (ntu / 2) * (x / kBS), rt = ib % ntr;
  const int tile = rt * ntu + ut;
  const int j0 = ut * 128, b0 = rt * 128;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int lr = lane & 15, lq = lane >> 4;
  const int srow = lane >> 3, sslot = lane & 7;
  const int nk = H3 / 64 / kBS, kt0 = split * nk;   // k-tiles per slice
  const int ncb = H3 / kBS / 128;                    // 128-column blocks per slice
  const size_t slot = (size_t)Bp * H3;               // exchange elements per step
  const rsrc_g rX = mk_rsrc(a.xbuf, (unsigned)((size_t)T * slot * 2));
  const rsrc_g rP = mk_rsrc(a.part, (unsigned)((size_t)2 * 64 * kBS * kPiece * 16));
  unsigned* const gflag = a.cnt;
  unsigned* const pflag = a.cnt + 4096;
  const bool acq = a.xch_acquire != 0;
  // epilogue items: row quarter `split`, piece P = w + 8 pp -> (wnp, ii, jn), 4 rows e each
  const int sq = split, wmq = sq >> 1, ibq = 2 * (sq & 1);
  float carry[2][4];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp)
#pragma unroll
    for (int e = 0; e < 4; ++e) carry[pp][e] = 0.f;
  // bias gradients of the quarter's 32 rows, summed over all steps: [16-row half ii][dar, daz,
  // dan * r, dan][128 units] in LDS beside the ring, each slot owned by one lane (no atomics: the
  // sums are deterministic)
  float (*bacc)[4][128] = reinterpret_cast<float (*)[4][128]>(lds_all + kBNS * 256 * 64);
  for (int i = tid; i < 2 * 4 * 128; i += 512) (&bacc[0][0][0])[i] = 0.f;
  auto item_off = [&](int pp, int e) {
    const int P = w + 8 * pp, wnp = P >> 2, ii = (P >> 1) & 1, jn = P & 1;
    return (size_t)(b0 + 32 * sq + ii * 16 + lq * 4 + e) * H + j0 + wnp * 32 + jn * 16 + lr;
  };
  // K-loop staging: piece q of wave w = image rows (4w + q) * 8 .. +8; waves 0-3 stage A, 4-7 W_hh^T
  auto stage = [&](int buf, int kt, int t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (4 * w + q) * 8 + srow, rr = r & 127;
      lds_void_g* dst = (lds_void_g*)(&lds[buf][(4 * w + q) * 8 * 64]);
      const int col = (kt0 + kt) * 64 + swz(rr, sslot) * 8;
      if (w < 4) {
        const unsigned off = (unsigned)((((size_t)(t + 1) * Bp + b0 + rr) * H3 + col) * 2);
        if (acq) __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, dst, 16, off, 0, 0, 0);   // behind the acquire
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, dst, 16, off, 0, 0, 16);     // aux 16 = sc1
      } else {
        __builtin_amdgcn_global_load_lds(a.WhhT + (size_t)(j0 + rr) * H3 + col, dst, 16, 0, 0);
      }
    }
  };
  auto spin_until = [&](const unsigned* f, int nflags, int stride, unsigned target, auto flag_of) {
    unsigned long long t0 = 0;
    unsigned n = 0;
    for (;;) {
      bool ok = true;
      if (lane < nflags) ok = __hip_atomic_load(f + (size_t)flag_of(lane) * stride, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if ((n++ & 63u) == 0u) {   // (first check: the clock only)
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (!t0) t0 = now;
        else if (a.err && (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u)) break;
        else if (now - t0 > kSpinTicks) {
          if (lane == 0 && a.err) __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  };

  for (int t = T - 1; t >= 0; --t) {
    const unsigned ep = (unsigned)(T - 1 - t);   // steps this launch has published before this one
    // the epilogue's operands first: their latency hides under the wait and the K loop
    float pre[2][4][6];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t o = (size_t)t * Bp * H + item_off(pp, e);
        pre[pp][e][0] = a.dy[o];
        pre[pp][e][1] = a.sr[o]; pre[pp][e][2] = a.sz[o]; pre[pp][e][3] = a.sn[o];
        pre[pp][e][4] = a.HSf[o]; pre[pp][e][5] = a.sghn[o];   // HSf + t*Bp*H = h_{t-1}
      }
    float ps[2][4];    // dh = (dy + carry) + partial sum: the step kernel's rounding order
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int e = 0; e < 4; ++e) ps[pp][e] = 0.f;
    __syncthreads();   // the previous step's LDS staging reads are done before the ring refills
    const bool kloop = t < T - 1;
    if (kloop) {
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // W_hh^T rows of the first ring slots do not depend on the exchange: waves 4-7 put them in flight
      // before the wait (each wave's vmcnt counts only its own pieces, so the ring's waits still hold)
      if (w >= 4) {
#pragma unroll
        for (int s2 = 0; s2 < kBNS - 1; ++s2) stage(s2, s2, t);
      }
      // dGh_{t+1}: column block cb of this slice (gate cb / ntu, unit tile cb % ntu) x 4 row quarters
      if (w == 0) {
        spin_until(gflag, 4 * ncb, 16, ep, [&](int l) {
          const int cb = split * ncb + (l >> 2);
          return (rt * ntu + cb % ntu) * kBS + (l & 3);
        });
        if (acq) {   // as the forward: plain A loads behind one wave's agent acquire, shared in L2
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
      if (w < 4) {
#pragma unroll
        for (int s2 = 0; s2 < kBNS - 1; ++s2) stage(s2, s2, t);
      }
      for (int kt = 0; kt < nk; ++kt) {
        const int ahead = min(kBNS - 2, nk - 1 - kt);
        if (ahead >= 2) vmwait<8>(); else if (ahead == 1) vmwait<4>(); else vmwait<0>();
        lds_barrier();
        if (kt + kBNS - 1 < nk) stage((kt + kBNS - 1) % kBNS, kt + kBNS - 1, t);
        const u16* LA = lds[kt % kBNS];
        const u16* LB = LA + 128 * 64;
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
      }
      // this split's partial tile, write-through; drain; one flag; wait for the S partners
      const size_t pbase = ((size_t)(ep & 1) * 64 + tile) * kBS * kPiece;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const size_t o = pbase + (size_t)split * kPiece + ((w * 4 + i) * 2 + j) * 64 + lane;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g, acc[i][j]), rP, (unsigned)(o * 16), 0, 16);
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(pflag + (size_t)(tile * kBS + split) * 16, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0)
        spin_until(pflag, kBS, 16, ep, [&](int l) { return tile * kBS + l; });
      __syncthreads();
      // partial sums of the epilogue items, split order 0..S-1
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int P = w + 8 * pp, wnp = P >> 2, ii = (P >> 1) & 1, jn = P & 1, i = ibq + ii;
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < kBS; ++s2) {
          const size_t o = pbase + (size_t)s2 * kPiece + (((wmq * 4 + wnp) * 4 + i) * 2 + jn) * 64 + lane;
          sum += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rP, (unsigned)(o * 16), 0, 16));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) ps[pp][e] = sum[e];
      }
    }
    // ---- gate gradients; row-major staging [4 kinds][32 rows][kRowPad] + transposed [4][128][40]
    u16* stR = &lds[0][0];
    u16* stT = &lds[0][0] + 4 * 32 * kRowPad;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int P = w + 8 * pp, wnp = P >> 2, ii = (P >> 1) & 1, jn = P & 1;
      const int uu = wnp * 32 + jn * 16 + lr;
      float bs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rq = ii * 16 + lq * 4 + e;
        const float dh = (pre[pp][e][0] + carry[pp][e]) + ps[pp][e];
        const float r = pre[pp][e][1], z = pre[pp][e][2], n = pre[pp][e][3];
        const float hp = pre[pp][e][4], ghn = pre[pp][e][5];
        const float dn = dh * (1.f - z);
        const float dz = dh * (hp - n);
        const float dan = dn * (1.f - n * n);
        const float dar = dan * ghn * r * (1.f - r);
        const float daz = dz * z * (1.f - z);
        carry[pp][e] = z * dh;
        bs[0] += dar; bs[1] += daz; bs[2] += dan * r; bs[3] += dan;
        const u16 br = f2bf(dar), bz = f2bf(daz), bn = f2bf(dan * r), bi = f2bf(dan);
        stR[(0 * 32 + rq) * kRowPad + uu] = br;
        stR[(1 * 32 + rq) * kRowPad + uu] = bz;
        stR[(2 * 32 + rq) * kRowPad + uu] = bn;
        stR[(3 * 32 + rq) * kRowPad + uu] = bi;
        stT[(0 * 128 + uu) * 40 + rq] = br;
        stT[(1 * 128 + uu) * 40 + rq] = bz;
        stT[(2 * 128 + uu) * 40 + rq] = bn;
        stT[(3 * 128 + uu) * 40 + rq] = bi;
      }
      if (a.dbhh_part || a.dbih_part) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = bs[q];
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          if (lq == 0) bacc[ii][q][uu] += v;
        }
      }
    }
    __syncthreads();
    // publish dGh_t: 3 gates x 32 rows x 256 B (whole lines of this producer), write-through
    if (t > 0) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int q = tid + 512 * p, g = q >> 9, rq = (q >> 4) & 31, seg = q & 15;
        const u32x4_g v = *reinterpret_cast<const u32x4_g*>(&stR[(g * 32 + rq) * kRowPad + seg * 8]);
        const unsigned off = (unsigned)((((size_t)t * Bp + b0 + 32 * sq + rq) * H3 + g * H + j0 + seg * 8) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, rX, off, 0, 16);   // aux 16 = sc1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(gflag + (size_t)(tile * kBS + split) * 16, ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // after the signal: row-major dGi_t (the dX GEMM's operand) and the transposed copies
    if (a.dgi) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int q = tid + 512 * p, g = q >> 9, rq = (q >> 4) & 31, seg = q & 15;
        const int kind = g < 2 ? g : 3;
        *reinterpret_cast<u32x4_g*>(a.dgi + ((size_t)t * Bp + b0 + 32 * sq + rq) * H3 + g * H + j0 + seg * 8) =
            *reinterpret_cast<const u32x4_g*>(&stR[(kind * 32 + rq) * kRowPad + seg * 8]);
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = tid + p * 512;
      const int kind = q >> 9, rem = q & 511, unit = rem >> 2, seg = rem & 3;
      const uint4 v = *reinterpret_cast<const uint4*>(&stT[(kind * 128 + unit) * 40 + seg * 8]);
      const int g = kind < 3 ? kind : 2;
      const size_t off = (size_t)(g * H + j0 + unit) * a.ldG + (size_t)t * Bp + b0 + 32 * sq + seg * 8;
      if (kind < 3 && a.dghT) *reinterpret_cast<uint4*>(a.dghT + off) = v;
      if (a.dgiT && (kind == 3 || (kind < 2 && !a.dgiT_n_only))) *reinterpret_cast<uint4*>(a.dgiT + off) = v;
    }
  }
  // ---- bias-gradient partials of this workgroup's 32 rows ("row block" rt * 4 + split of
  // dbhh_part / dbih_part [Bp/32][3H]): the two 16-row halves' LDS sums
  if (a.dbhh_part || a.dbih_part) {
    __syncthreads();
    const int q = tid >> 7, u = tid & 127;
    const float v = bacc[0][q][u] + bacc[1][q][u];
    const size_t rb = (size_t)(b0 / 32 + sq) * H3;
    if (a.dbhh_part && q < 3) a.dbhh_part[rb + q * H + j0 + u] = v;
    if (a.dbih_part && q != 2) a.dbih_part[rb + (q == 3 ? 2 : q) * H + j0 + u] = v;
  }
}

bool gru_bwd_seq_big_supported(int H, int Bp) {
  if (H % 256 || Bp % 128 || H < 1024) return false;
  const int ntu = H / 128, ntr = Bp / 128;
  if (ntu * ntr != 64 || ntu % 2) return false;   // 256 workgroups = 64 tiles x 4 splits, sk_map 1 order
  if (3 * H / kBS / 128 * 4 > 64) return false;    // <= 64 dGh producers per slice (one lane each)
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gru_bwd_seq_big_kernel, 512, 0) != hipSuccess) return false;
  return ncu * per >= 256;
}

long gru_bwd_seq_big_part_floats(int H, int Bp) { return 2L * Bp * H * kBS; }

void gru_bwd_seq_big(const SeqBwdArgs& a, hipStream_t s) {
  if (!gru_bwd_seq_big_supported(a.H, a.Bp) || !a.xbuf || !a.cnt || !a.part || !a.dy || !a.sr || !a.sz ||
      !a.sn || !a.sghn || !a.HSf || !a.WhhT || a.ldG < a.T * a.Bp)
    throw std::runtime_error("gru_bwd_seq_big: unsupported shape or incomplete arguments");
  if ((size_t)a.T * a.Bp * 3 * a.H * 2 >= (1ull << 32))
    throw std::runtime_error("gru_bwd_seq_big: exchange exceeds the 4 GB buffer range");
  hipLaunchKernelGGL(gru_bwd_seq_big_kernel, dim3(256), dim3(512), 0, s, a);
}

}  // namespace gk
