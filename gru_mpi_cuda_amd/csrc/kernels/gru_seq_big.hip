// Persistent large-H backward recurrence: ONE launch runs all T backward steps
// of a layer whose per-step GEMM is a real GEMM (B = 512 rows, H = 2048: dh = dGh . W_hh is 12.9
// GFLOP per step), where the register-resident persistent kernels of gru_seq.hip do not fit and the
// per-step kernels of gru_step_lds.hip pay a launch, a grid ramp and a drain per timestep.
//
// (Round 4 also built the forward twin -- 256 workgroups of 128 rows x 32 units x 3 gates, W_hh
// streamed through a 4-deep LDS ring, T-deep per-producer h tiles with epoch flags.  Correct, and
// slower than the 64-row step kernels: h2048 forward 3.04-3.34 ms vs 2.89-2.97, step 9.24 vs 8.69-8.72
// ms, profiles/r4_h2048_big_v1_ab.jsonl, r4_h2048_big_acq_ab.jsonl, r4_h2048_h1024_big_ab.jsonl; removed.
// A second try on the 64-row step kernel's tile -- two workgroups per CU, 512 co-resident, the same
// k order and epilogue -- was correct and slower still: h2048 9.37-9.40 vs 8.77-8.81 ms, h1024_l2 x
// 1024 equal, profiles/r4_h2048_h1024_fwd64_ab.jsonl; removed.)
#include <algorithm>
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

// ==================================================================== persistent large-H backward
// ONE launch runs all T backward steps of a layer at large H with a large batch (B = 512, H = 2048:
// dh = dGh_{t+1} . W_hh is 512 x 2048 x 6144 per step), replacing T launches of the split-K step
// kernel (gru_step_lds.hip gru_bwd_step_sk_kernel, whose tiling and epilogue it keeps):
//   * 256 workgroups = 64 tiles of 128 rows x 128 units, each over S = 4 K-slices; the block order of
//     sk_map 1 (XCD x takes split x % 4 of every row tile of half the unit tiles);
//   * per step t (descending): wave 0 polls the epoch flags of the dGh_{t+1} producers of this
//     workgroup's A operand (its 128 rows x K-slice: 4 row-quarter producers of each of the slice's
//     128-column blocks), then one agent acquire; the K loop streams A (the exchange ring: plain
//     loads behind the acquire) and W_hh^T (plain, its first ring slots issued
//     before the wait) through a 4-deep LDS ring; the fp32 partial tile goes out write-through (parity-double-buffered), one
//     flag per (tile, split), and the S partners wait for each other;
//   * fused dy (SeqBwdArgs::dl, the top layer): dy_t = dl_t . W_fc is not read from memory; each split
//     adds vocabulary quarter `split` (64 deep) of it to its partial tile, from one extra k-tile
//     (A = dl_t rows, B = W_fc^T rows) staged in ring slot 3 at the top of the step (waves 1-7 wait
//     for it while wave 0 polls) and multiplied under the latency of the first exchange k-tiles.  This removes the dH GEMM
//     (65536 x 2048 x 256 at config 5: 173 us) and its 537 MB fp32 dy, written once and read back by
//     this kernel.  At t = T - 1 (no exchange yet) the splits still trade partials: the partial flags
//     count ep + 1;
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

// FDY: the fused dy (SeqBwdArgs::dl), compile-time and only with the packed bf16 saves (s16): the
// register file is full, and dy / the four fp32 save slots of the epilogue prefetch pay for its staging
template <bool FDY>
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
  const int nslot = a.xring >= 2 && a.xring < T ? a.xring : T;   // slots addressed (ring or T-deep)
  const rsrc_g rX = mk_rsrc(a.xbuf, (unsigned)((size_t)nslot * slot * 2));
  // exchange ring (SeqBwdArgs::xring): dGh_t in slot t % xr.  A workgroup publishes dGh_t only after
  // its S partners' step-t partials, whose K-slices together need dGh_{t+1} from every workgroup of
  // the row tile, each of which published it after its own step-(t+1) reads of dGh_{t+2}: the slot
  // being rewritten (t + 2 for xr = 2) has no reader left.
  const int xr = a.xring >= 2 ? a.xring : T;
  // (fused dy: dl [T * Bp][256] and W_fc^T [H][256] bf16)
  const rsrc_g rL = mk_rsrc(a.dl, FDY ? (unsigned)((size_t)T * Bp * 256 * 2) : 0u);
  const rsrc_g rF = mk_rsrc(a.WfcT, FDY ? (unsigned)((size_t)H * 256 * 2) : 0u);
  const rsrc_g rP = mk_rsrc(a.part, (unsigned)((size_t)2 * 64 * kBS * kPiece * 16));
  unsigned* const gflag = a.cnt;
  unsigned* const pflag = a.cnt + 4096;
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
        const unsigned off = (unsigned)((((size_t)((t + 1) % xr) * Bp + b0 + rr) * H3 + col) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, dst, 16, off, 0, 0, 0);   // behind the acquire
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
        pre[pp][e][0] = FDY ? 0.f : a.dy[o];
        if (FDY || a.s16) ld_save16_raw(a.s16 + o * 4, pre[pp][e][1], pre[pp][e][2]);   // unpacked at use
        else { pre[pp][e][1] = a.sr[o]; pre[pp][e][2] = a.sz[o]; pre[pp][e][3] = a.sn[o]; pre[pp][e][5] = a.sghn[o]; }
        pre[pp][e][4] = a.HSf[o];   // HSf + t*Bp*H = h_{t-1}
      }
    float ps[2][4];    // dh = (dy + carry) + partial sum: the step kernel's rounding order
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int e = 0; e < 4; ++e) ps[pp][e] = 0.f;
    __syncthreads();   // the previous step's LDS staging reads are done before the ring refills
    const bool xloop = t < T - 1;          // dGh_{t+1} . W_hh (nothing to exchange at the last step)
    constexpr bool fdy = FDY;              // + this split's quarter of dl_t . W_fc
    if (xloop || fdy) {
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto mma_tile = [&](const u16* LA) {
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
      };
      if constexpr (FDY) {
        // the dy k-tile into ring slot 3 (first refilled at k-tile 3, after this tile's MFMAs):
        // A = dl_t rows b0.. x vocabulary quarter `split` (waves 0-3), B = W_fc^T rows j0.. (waves 4-7)
        // buffer loads: the lane part is one of two offsets (row srow, swizzled chunk for even / odd q),
        // everything else a scalar offset -- the 64-bit addresses, and then 4 lane offsets, spilled
        const int wu = __builtin_amdgcn_readfirstlane(w);
        const unsigned lo[2] = {(unsigned)((srow * 256 + (sslot ^ ((srow >> 1) & 7)) * 8) * 2),
                                (unsigned)((srow * 256 + (sslot ^ ((4 + (srow >> 1)) & 7)) * 8) * 2)};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          lds_void_g* dst = (lds_void_g*)(&lds[kBNS - 1][(4 * w + q) * 8 * 64]);
          const int rowq = ((4 * wu + q) * 8) & 127;   // first tile row of this piece
          if (wu < 4)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rL, dst, 16, lo[q & 1], ((t * Bp + b0 + rowq) * 256 + split * 64) * 2, 0, 0);
          else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rF, dst, 16, lo[q & 1], ((j0 + rowq) * 256 + split * 64) * 2, 0, 0);
        }
      }
      // W_hh^T rows of the first ring slots do not depend on the exchange: waves 4-7 put them in flight
      // before the wait (each wave's vmcnt counts only its own pieces, so the ring's waits still hold)
      if (xloop && w >= 4) {
#pragma unroll
        for (int s2 = 0; s2 < kBNS - 1; ++s2) stage(s2, s2, t);
      }
      // dGh_{t+1}: column block cb of this slice (gate cb / ntu, unit tile cb % ntu) x 4 row quarters
      if (xloop && w == 0) {
        spin_until(gflag, 4 * ncb, 16, ep, [&](int l) {
          const int cb = split * ncb + (l >> 2);
          return (rt * ntu + cb % ntu) * kBS + (l & 3);
        });
        // plain A loads behind one wave's agent acquire, shared in the XCD's L2 (sc1 loads instead --
        // one fetch per workgroup from the memory side -- measured equal, r4_h2048_big_acq_ab.jsonl;
        // that switch was removed in round 5)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if constexpr (FDY) {
        // the dy tile's share of each wave has landed -- waves 1-7 wait while wave 0 polls (waves 4-7
        // keep their 3 W_hh^T slots, issued behind it, in flight)
        if (xloop && w >= 4) vmwait<12>(); else vmwait<0>();
      }
      if (xloop || FDY) __syncthreads();   // the flags are seen (xloop) and the dy tile is published (FDY)
      if (xloop && w < 4) {
#pragma unroll
        for (int s2 = 0; s2 < kBNS - 1; ++s2) stage(s2, s2, t);
      }
      // the dy tile's MFMAs under the latency of the first exchange k-tiles just issued
      if constexpr (FDY) mma_tile(lds[kBNS - 1]);
      if (xloop) {
        for (int kt = 0; kt < nk; ++kt) {
          const int ahead = min(kBNS - 2, nk - 1 - kt);
          if (ahead >= 2) vmwait<8>(); else if (ahead == 1) vmwait<4>(); else vmwait<0>();
          lds_barrier();   // (at kt = 0 also: every wave is done with the dy tile in slot 3)
          if (kt + kBNS - 1 < nk) stage((kt + kBNS - 1) % kBNS, kt + kBNS - 1, t);
          mma_tile(lds[kt % kBNS]);
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
      // (partial flags count ep + 1: with the fused dy the partners also trade at t = T - 1, ep = 0)
      if (tid == 0)
        __hip_atomic_store(pflag + (size_t)(tile * kBS + split) * 16, ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0)
        spin_until(pflag, kBS, 16, ep + 1, [&](int l) { return tile * kBS + l; });
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
        float r = pre[pp][e][1], z = pre[pp][e][2], n = pre[pp][e][3], ghn = pre[pp][e][5];
        if (FDY || a.s16) unpack_save16(pre[pp][e][1], pre[pp][e][2], r, z, n, ghn);
        const float hp = pre[pp][e][4];
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
        const unsigned off = (unsigned)((((size_t)(t % xr) * Bp + b0 + 32 * sq + rq) * H3 + g * H + j0 + seg * 8) * 2);
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
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gru_bwd_seq_big_kernel<false>, 512, 0) != hipSuccess) return false;
  int per2 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, gru_bwd_seq_big_kernel<true>, 512, 0) != hipSuccess) return false;
  per = std::min(per, per2);
  return ncu * per >= 256;
}

long gru_bwd_seq_big_part_floats(int H, int Bp) { return 2L * Bp * H * kBS; }

void gru_bwd_seq_big(const SeqBwdArgs& a, hipStream_t s) {
  if (!gru_bwd_seq_big_supported(a.H, a.Bp) || !a.xbuf || !a.cnt || !a.part || (!a.dy && !a.dl) || ((!a.sr || !a.sz ||
      !a.sn || !a.sghn) && !a.s16) || !a.HSf || !a.WhhT || a.ldG < a.T * a.Bp)
    throw std::runtime_error("gru_bwd_seq_big: unsupported shape or incomplete arguments");
  if (a.dl && (!a.WfcT || a.V != 64 * kBS || !a.s16))
    throw std::runtime_error("gru_bwd_seq_big: the fused dy needs W_fc^T, V = 256 and the packed saves");
  // only min(T, xring) slots of the exchange are addressed when a ring is active
  const size_t slots = a.xring >= 2 && a.xring < a.T ? (size_t)a.xring : (size_t)a.T;
  if (slots * a.Bp * 3 * a.H * 2 >= (1ull << 32))
    throw std::runtime_error("gru_bwd_seq_big: exchange exceeds the 4 GB buffer range");
  if ((size_t)a.T * a.Bp * 256 * 2 >= (1ull << 31)) throw std::runtime_error("gru_bwd_seq_big: dl exceeds the buffer range");
  if (a.dl) hipLaunchKernelGGL(gru_bwd_seq_big_kernel<true>, dim3(256), dim3(512), 0, s, a);
  else hipLaunchKernelGGL(gru_bwd_seq_big_kernel<false>, dim3(256), dim3(512), 0, s, a);
}

}  // namespace gk
