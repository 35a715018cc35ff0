// Persistent (whole-sequence) GRU recurrence kernels for gfx950: ONE launch runs all T
// timesteps of one layer, forward or backward.
//
// Why: at the headline shape (B = 256 per GPU, H = 512) one timestep's recurrent GEMM is
// 0.4 GFLOP -- a few hundred ns of MFMA work spread over 256 CUs -- so a per-step launch is
// dominated by the launch/drain floor (profiles/: ~1.6 us graph node + ~1 us store drain +
// ~1 us of load latency).  Here:
//   * grid = (H/16 unit tiles) x (Bp/32 row blocks), one 512-thread workgroup per CU, all
//     co-resident (checked on the host against the occupancy query);
//   * each wave keeps its K-slice of the recurrent weights in VGPRs for the whole sequence
//     (W_hh never re-read from memory);
//   * step t+1 of row block rb needs h_t of those 32 rows from all H/16 unit-tile workgroups:
//     the 1 KB tile each workgroup produces is stored write-through (sc1) by one wave, that
//     wave drains (s_waitcnt vmcnt(0)) and bumps the row block's counter (agent-scope atomic);
//     consumers poll the counter with sc1 loads and read the tiles with sc1 buffer loads
//     (cdna_hip_programming.md §6 Guideline 16, MI355X_MICROARCH.md 'Valid forms' row 1).
//     Every spin is bounded: on timeout an error word is set and the kernel runs to completion.
//   * backward additionally accumulates the weight gradients dW_hh = Σ_t dGh_t^T h_{t-1} and
//     the embedding-side dP = Σ_t onehot(x_t)^T dGi_t (layer 0) plus both bias gradients in
//     registers, using the MFMA pipe that the latency-bound recurrence leaves idle; partial
//     sums per row block are reduced by one small kernel afterwards (no float atomics).
// Reference mapping: this is the whole per-char hot loop of /root/reference/namegensf.cu:661-872
// (for all names at once), plus the BPTT half the reference does not have.
#include "kernels.h"
#include "mma_tile.h"
#include "seq_sync.h"

namespace gk {

// ==================================================================== forward
// RS = 1: every wave covers both 16-row tiles of the row block over a K/8 slice (NKW = H/256
//         k-steps); the 8 partial sums of each output meet in LDS.
// RS = 2: waves 0-3 own row tile 0, waves 4-7 row tile 1, each over a K/4 slice (NKW = H/128):
//         the same MFMAs and exchange loads per wave, half the LDS partial traffic (4 partials of
//         3 gates per output instead of 8, read by the epilogue thread of the same row tile).
// (Rejected and removed in round 4, history in docs/DESIGN.md §6.3: a table-free layer 0 computing
// its P-table columns in every workgroup, layer 0's input projection in the post-publish slack, the
// FC / softmax-xent pipeline inside the forward, and the saves issued inside the publish drain.)
// FC = true (gru_fwd_seq_fc): the same recurrence in blocks [0, H/16 * Bp/32), plus kFcCons FC
// consumer workgroups per row block behind them in the same grid (fwd_fc_consumer below); the
// recurrence then also drains its h copies before each step's first barrier and signals T + 1
// after the last step, so a consumer that saw epoch t + 2 may read HSb / HF of step t.
static constexpr size_t kFwdRecLds = sizeof(float) * 8 * 6 * 256 + sizeof(u16) * 32 * 24 + sizeof(u16) * 16 * 40;
static constexpr size_t kFwdFcLds = sizeof(u16) * 32 * (512 + 8) + sizeof(u16) * 32 * (256 + 8) +
                                    sizeof(float) * (2 * 8 * 32 + 3 * 32);

// ---------------------------------------------------------------------------- FC consumers
// Workgroup ci of the consumer part of gru_fwd_seq_fc's grid serves row block rbk = ci % nrb as its
// consumer c = ci / nrb (placed on rbk's XCD by the dispatcher's round-robin; the placement census
// covers producers and consumers, so a row block whose members are not all on one XCD takes the
// write-through protocol for every hand-off).  Two phases, both behind the recurrence:
//  1. items: step t = c, c + kFcCons, ... of the row block -- the 32 x V logits of h_t (X tile read
//     from HSb once the row block's producers signalled t + 2, W_fc fragments already in flight),
//     softmax-xent, the loss partial, dl as bf16 fragment blocks (dlF), dy_t = dl · W_fc (fp32); then
//     the consumer's own flag line carries "items done".
//  2. dW_fc: consumer c owns the 64 x 64 tile c of the row block's V x H partial and accumulates
//     dl_t^T h_t over t = 0 .. T-1 in order (one flag check per step: the item of step t done), from
//     dlF and the backward's fragment-tiled HF copy -- K = 32 rows per step, one MFMA per 16 x 16
//     tile; the tiles of unit column 0 also take db_fc (row sums of dl^T, an MFMA against ones).
//     The row block's partial lands in slab rbk (the trainer's dW_fc / db_fc slabs, summed in Adam).
// The recurrence never waits on a consumer.  This is the FC / softmax-xent / dH work of fc_xent and
// the dW_fc K-slices of the post-backward group, off the step's serial tail (VERDICT r5 item 1;
// reference: the per-char FC + softmax of /root/reference/namegensf.cu:856-873).
template <int H>
DEV void fwd_fc_consumer(const SeqFwdArgs& a, const SeqFcArgs& f, unsigned char* smem, int ci) {
  constexpr int V = 256, NW = 8, LDX = H + 8, LDR = V + 8, NKS = H / 32, NKC = 4;
  static_assert((V / 64) * (H / 64) == kFcCons, "one 64 x 64 dW_fc tile per consumer");
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // scalar: fragment offsets go to soffset
  const int T = a.T, Bp = a.Bp, nrb = Bp / 32;
  constexpr int nunit = H / 16;
  const int rbk = ci % nrb, c = ci / nrb, b0 = rbk * 32;
  unsigned* const fl = a.cnt + (size_t)rbk * (nunit + kFcCons) * kFlagStride;   // producers' lines
  unsigned* const cfl = fl + (size_t)nunit * kFlagStride;                       // consumers' lines
  const int probe = f.probe & 7;
  if (probe == 3) return;
  const bool loc = a.allow_local && row_block_local(fl, nunit + c, nunit + kFcCons, a.err);
  if (probe == 1) return;
  u16* xs = reinterpret_cast<u16*>(smem);              // [32][H + 8] X tile
  u16* dlr = xs + 32 * LDX;                            // [32][V + 8] dl row-major (dH A operand)
  float* red = reinterpret_cast<float*>(dlr + 32 * LDR);   // [2][8][32] row max / sum-exp partials
  float* lab = red + 2 * NW * 32;                      // [32] label logit
  float* lrow = lab + 32;                              // [32] row loss
  int* ys = reinterpret_cast<int*>(lrow + 32);         // [32] labels
  const rsrc_t rH = make_rsrc(a.HSb, (unsigned)((size_t)(T + 1) * Bp * H * 2));
  const rsrc_t rD = make_rsrc(f.dlF, (unsigned)((size_t)T * Bp * V * 2));
  const int v0 = w * 32;
  float bias[2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) bias[cc] = f.b[v0 + cc * 16 + lr];
  // W_fc fragments (FT layout, 1 KB per load instruction): wave w's 2 vocab tiles, k-steps ks..ks+NKC;
  // buffer loads with the lane's 16 B in the VGPR offset and the block in the scalar offset (64-bit
  // VGPR addresses per fragment pushed the consumer past its 128-register budget)
  const rsrc_t rWf = make_rsrc(f.Wf, (unsigned)(V * H * 2)), rWt = make_rsrc(f.WTf, (unsigned)(V * H * 2));
  const unsigned l16 = (unsigned)lane * 16u;
  auto load_w = [&](bf16x8 (&b)[NKC][2], int ks) {
    if (probe == 4) {   // diagnostic: the items without their weight stream
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) b[kk][0] = b[kk][1] = zero8();
      return;
    }
#pragma unroll
    for (int kk = 0; kk < NKC; ++kk)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) b[kk][cc] = ld8_plain_s(rWf, l16, ((v0 / 16 + cc) * NKS + ks + kk) * 1024);
  };
  auto mma_w = [&](f32x4 (&acc)[2][2], const bf16x8 (&b)[NKC][2], int ks) {
#pragma unroll
    for (int kk = 0; kk < NKC; ++kk) {
      bf16x8 af[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) af[r] = *reinterpret_cast<const bf16x8*>(xs + (r * 16 + lr) * LDX + (ks + kk) * 32 + 8 * lq);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) acc[r][cc] = mfma16(af[r], b[kk][cc], acc[r][cc]);
    }
  };
  // W_fc^T fragments of wave w's 64 dH columns, two k-steps of V
  auto load_wt = [&](bf16x8 (&b)[2][4], int kk0) {
    if (probe == 4) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) b[kk][cc] = zero8();
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) b[kk][cc] = ld8_plain_s(rWt, l16, ((w * 4 + cc) * (V / 32) + kk0 + kk) * 1024);
  };
  auto mma_t = [&](f32x4 (&acc)[2][4], const bf16x8 (&b)[2][4], int kk0) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) af[r] = *reinterpret_cast<const bf16x8*>(dlr + (r * 16 + lr) * LDR + (kk0 + kk) * 32 + 8 * lq);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) acc[r][cc] = mfma16(af[r], b[kk][cc], acc[r][cc]);
    }
  };

  // ---- phase 1: the FC items of this consumer
  for (int t = c; t < T; t += kFcCons) {
    const int m0 = t * Bp + b0;
    bf16x8 wa[NKC][2], wb[NKC][2];
    load_w(wa, 0);
    load_w(wb, NKC);
    const int ylab = tid < 32 ? f.labels[m0 + tid] : 0;
    const float inv = f.inv_count[0];
    // h_t of the whole row block is in HSb once every producer signalled t + 2 (T + 1: the final signal).
    // The producers' flag lines are the recurrence's own hot lines: until this item is near, one lane
    // polls one of them with a long back-off (a full 32-lane sweep every ~100 clocks by each waiting
    // consumer measured +0.7 us per recurrence step), then the sweep of all producers.
    if (tid < 64) {
      SpinBudget spin(a.err);
      for (;;) {
        unsigned v = 0;
        if (lane == 0) v = __hip_atomic_load(fl + (size_t)(c % nunit) * kFlagStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = __builtin_amdgcn_readfirstlane(v);
        if (v + 1u >= (unsigned)(t + 2)) break;
        __builtin_amdgcn_s_sleep(16);
        if (spin.expired()) break;   // the full wait below reports it
      }
    }
    wait_flags(fl, nunit, (unsigned)(t + 2), a.err);
    stamp(a.dbg, t, 0);
    constexpr int NXP = 32 * H / 8 / 512;
    u32x4 xv[NXP];
#pragma unroll
    for (int e = 0; e < NXP; ++e) {
      const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
      xv[e] = __builtin_amdgcn_raw_buffer_load_b128(rH, (unsigned)((((size_t)(t + 1) * Bp + b0 + row) * H + c8 * 8) * 2), 0, 16);
    }
#pragma unroll
    for (int e = 0; e < NXP; ++e) {
      const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
      *reinterpret_cast<u32x4*>(xs + row * LDX + c8 * 8) = xv[e];
    }
    if (tid < 32) ys[tid] = ylab;
    lds_barrier();
    stamp(a.dbg, t, 1);
    f32x4 acc[2][2];
    zero_acc(acc);
#pragma unroll
    for (int ks = 0; ks < NKS; ks += 2 * NKC) {
      mma_w(acc, wa, ks);
      if (ks + 2 * NKC < NKS) load_w(wa, ks + 2 * NKC);
      mma_w(acc, wb, ks + NKC);
      if (ks + 3 * NKC < NKS) load_w(wb, ks + 3 * NKC);
    }
    bf16x8 ta[2][4], tb[2][4];   // the dH pass's first W_fc^T fragments, under the softmax
    load_wt(ta, 0);
    load_wt(tb, 2);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[r][cc][i] += bias[cc];
    // softmax statistics across the 8 waves' columns
    float mx[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float m = max16(fmaxf(acc[r][0][i], acc[r][1][i]));
        if (lr == 0) red[w * 32 + r * 16 + lq * 4 + i] = m;
      }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r * 16 + lq * 4 + i;
        float m = red[row];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
        mx[r][i] = m;
        const float e = sum16(__expf(acc[r][0][i] - m) + __expf(acc[r][1][i] - m));
        if (lr == 0) red[NW * 32 + w * 32 + row] = e;
      }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      u16 dv[2][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r * 16 + lq * 4 + i;
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sum += red[NW * 32 + ww * 32 + row];
        const int y = ys[row];
        const float scale = (y >= 0) ? inv : 0.f;
        const float rs = __builtin_amdgcn_rcpf(sum);
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          const int col = v0 + cc * 16 + lr;
          const float x = acc[r][cc][i];
          if (col == y) lab[row] = x;
          const float d = (__expf(x - mx[r][i]) * rs - (col == y ? 1.f : 0.f)) * scale;
          dv[cc][i] = f2bf(d);
          dlr[row * LDR + col] = dv[cc][i];
        }
      }
      // dlF block (t, rbk, vocab tile): lane L holds rows 8(L >> 4) .. +8 of vocab column L & 15; this
      // lane's 4 rows r*16 + 4lq .. +4 are half of lane (2r + lq/2)*16 + lr's slot
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const unsigned lo = (unsigned)dv[cc][0] | ((unsigned)dv[cc][1] << 16);
        const unsigned hi = (unsigned)dv[cc][2] | ((unsigned)dv[cc][3] << 16);
        const unsigned off = (unsigned)(((((size_t)(t * nrb + rbk) * (V / 16) + v0 / 16 + cc) * 64 +
                                          (2 * r + (lq >> 1)) * 16 + lr) * 8 + (lq & 1) * 4) * 2);
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 pv = {lo, hi};
        if (loc) __builtin_amdgcn_raw_buffer_store_b64(pv, rD, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(pv, rD, off, 0, 16);
      }
    }
    lds_barrier();   // dl row-major and the label logits in LDS
    stamp(a.dbg, t, 2);
    if (tid < 32) {
      const int row = tid, y = ys[row];
      float m = red[row], sum = 0.f;
      for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
      for (int ww = 0; ww < NW; ++ww) sum += red[NW * 32 + ww * 32 + row];
      lrow[row] = (y >= 0) ? (logf(sum) + m - lab[row]) * inv : 0.f;
    }
    // dy_t = dl · W_fc: wave w's 64 columns, K = V
    f32x4 dacc[2][4];
    zero_acc(dacc);
#pragma unroll
    for (int kk0 = 0; kk0 < V / 32; kk0 += 4) {
      mma_t(dacc, ta, kk0);
      if (kk0 + 4 < V / 32) load_wt(ta, kk0 + 4);
      mma_t(dacc, tb, kk0 + 2);
      if (kk0 + 6 < V / 32) load_wt(tb, kk0 + 6);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          f.dy[(size_t)(m0 + r * 16 + lq * 4 + i) * H + w * 64 + cc * 16 + lr] = dacc[r][cc][i];
    lds_barrier();   // lrow complete
    if (tid == 0) {
      float s = 0.f;
      for (int i = 0; i < 32; ++i) s += lrow[i];
      f.loss_part[m0 / 32] = s;
    }
    // item done: every wave's dlF stores complete, then one flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(a.dbg, t, 3);
    if (tid == 0) {
      if (loc) signal_flag_local(cfl + (size_t)c * kFlagStride, (unsigned)(t / kFcCons + 1));
      else signal_flag(cfl + (size_t)c * kFlagStride, (unsigned)(t / kFcCons + 1));
    }
  }

  if (probe == 2 || probe == 4) return;
  // ---- phase 2: this consumer's 64 x 64 tile of the row block's dW_fc partial, t = 0 .. T-1 in order
  constexpr int TPH = H / 64;
  const int tv = (c / TPH) * 4 + (w >> 1);          // 16-row vocab tile
  const int th = (c % TPH) * 4 + 2 * (w & 1);       // first of two 16-column unit tiles
  const bool rs_on = (c % TPH) == 0 && (w & 1) == 0;
  const rsrc_t rF = make_rsrc(a.HF, (unsigned)((size_t)(T + 1) * Bp * H * 2));
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  f32x4 aw[2], ab;
  aw[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  aw[1] = aw[0];
  ab = aw[0];
  // steps in groups of DG: one poll covers the group's items (lane i: step t0 + i), then all of its
  // fragments are loaded at once and accumulated in step order (deterministic)
  constexpr int DG = 4;
  for (int t0 = 0; t0 < T; t0 += DG) {
    const int n = T - t0 < DG ? T - t0 : DG;
    {
      SpinBudget spin(a.err);
      for (;;) {
        bool ok = true;
        if (lane < n)
          ok = __hip_atomic_load(cfl + (size_t)((t0 + lane) % kFcCons) * kFlagStride, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)((t0 + lane) / kFcCons + 1);
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(8);
        if (spin.expired()) {
          if (lane == 0) __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    bf16x8 A[DG], Bf[DG][2];
#pragma unroll
    for (int i = 0; i < DG; ++i) {
      if (i < n) {
        const int t = t0 + i;
        A[i] = ld8_sc1(rD, (unsigned)((((size_t)(t * nrb + rbk) * (V / 16) + tv) * 512 + lane * 8) * 2));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          Bf[i][j] = ld8_sc1(rF, (unsigned)(((((size_t)(t + 1) * nunit + th + j) * nrb + rbk) * 512 + lane * 8) * 2));
      }
    }
#pragma unroll
    for (int i = 0; i < DG; ++i) {
      if (i < n) {
#pragma unroll
        for (int j = 0; j < 2; ++j) aw[j] = mfma16(A[i], Bf[i][j], aw[j]);
        if (rs_on) ab = mfma16(A[i], ones, ab);
      }
    }
  }
  float* W = f.dW + (size_t)rbk * V * H;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) W[(size_t)(tv * 16 + lq * 4 + i) * H + (th + j) * 16 + lr] = aw[j][i];
  if (rs_on && lr == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f.db[(size_t)rbk * V + tv * 16 + lq * 4 + i] = ab[i];
  }
}


template <int NKW, int RS, bool FC, int WPE = FC ? 4 : 1>
__global__ void __launch_bounds__(512, WPE) gru_fwd_seq_kernel(SeqFwdArgs a, SeqFcArgs fc) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[FC ? (kFwdFcLds > kFwdRecLds ? kFwdFcLds : kFwdRecLds) : kFwdRecLds];
  auto& part = *reinterpret_cast<float(*)[8][6][256]>(smem);
  // padded rows (48 B / 80 B, still 16-B aligned for the vector reads): the epilogue's per-item
  // u16 writes -- rows 4 apart within a wave -- land in distinct banks (unpadded: 2-way / 4-way)
  auto& stg = *reinterpret_cast<u16(*)[32][24]>(smem + sizeof(float) * 8 * 6 * 256);
  auto& stgT = *reinterpret_cast<u16(*)[16][40]>(smem + sizeof(float) * 8 * 6 * 256 + sizeof(u16) * 32 * 24);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int H = a.H, Bp = a.Bp, T = a.T;
  const int nrb = Bp / 32;
  const unsigned nunit = (unsigned)(H / 16);
  if constexpr (FC) {
    const int nrec = (int)nunit * nrb;
    if ((int)blockIdx.x >= nrec) {
      zero_next_flags(a.zero_next, a.zero_words);
      if constexpr (NKW * 128 == 512 && RS == 2) fwd_fc_consumer<512>(a, fc, smem, (int)blockIdx.x - nrec);
      return;
    }
  }
  // flag lines per row block: its H/16 producers (+ its FC consumers)
  const size_t rb_lines = nunit + (FC ? kFcCons : 0);
  // (FC: the grid also holds the consumers, so the block -> tile map takes the recurrence's own count)
  const int ut = FC ? seq_unit_tile_n(nrb, (int)nunit * nrb) : seq_unit_tile(nrb);
  const int j0 = ut * 16, rbk = FC ? seq_row_block_n(nrb, (int)nunit * nrb) : seq_row_block(nrb), b0 = rbk * 32;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  constexpr int NR = RS == 2 ? 1 : 2;           // row tiles per wave
  const int rt = RS == 2 ? (w >> 2) : 0;        // first row tile of this wave
  const int k0 = (RS == 2 ? (w & 3) : w) * NKW * 32;

  bf16x8 bw[NKW][3];   // this wave's K-slice of W_h{r,z,n} for the 16 units, resident all sequence
#pragma unroll
  for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
    for (int g = 0; g < 3; ++g) bw[kk][g] = ld8(a.Whh + (size_t)(g * H + j0 + lr) * H + k0 + kk * 32 + lk);

  // this thread's epilogue item (row, unit) -- one per thread with 512 threads
  const int rb = tid >> 8, reg = (tid >> 6) & 3, ln = tid & 63;
  const int row = rb * 16 + (ln >> 4) * 4 + reg, col = ln & 15;
  const int b = b0 + row, j = j0 + col;
  float bh[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) bh[g] = a.bhh[g * H + j];
  float hp = a.h0 ? a.h0[(size_t)b * H + j] : 0.f;
  const rsrc_t rH = make_rsrc(a.HSb, (unsigned)((size_t)(T + 1) * Bp * H * 2));
  const rsrc_t rX = make_rsrc(a.xch, (unsigned)((size_t)T * Bp * H * 2));
  // exchange ring: the slot of step t is reused at step t + xr.  Safe for xr >= 2: a producer writes
  // step t only after every producer of its row block published step t - 1, i.e. finished reading
  // the tiles of step t - 2 -- the ones the write replaces when xr = 2.
  const int xr = a.xring >= 2 ? a.xring : T;
  const unsigned sv_bytes = (unsigned)((size_t)T * Bp * H * 4);   // < 4 GB: checked on the host
  const rsrc_t rHSf = make_rsrc(a.HSf, sv_bytes + (unsigned)(Bp * H * 4));
  const rsrc_t rSr = make_rsrc(a.sr, a.sr ? sv_bytes : 0u), rSz = make_rsrc(a.sz, a.sz ? sv_bytes : 0u);
  const rsrc_t rSn = make_rsrc(a.sn, a.sn ? sv_bytes : 0u), rSg = make_rsrc(a.sghn, a.sghn ? sv_bytes : 0u);
  const rsrc_t rS16 = make_rsrc(a.s16, a.s16 ? 2u * sv_bytes : 0u);   // < 4 GB: checked on the host
  const unsigned sv_lane = (unsigned)((b * H + j) * 4);
  stamp(a.dbg, T + 1, 0);   // prologue stamps in the (unused) step slot T + 1
  zero_next_flags(a.zero_next, a.zero_words);
  // (probe 3: consumers leave before the census, which then covers the producers only)
  const int cens = FC && (fc.probe & 7) == 3 ? (int)nunit : (int)rb_lines;
  if (FC && (fc.probe & 8)) __builtin_amdgcn_s_setprio(2);
  const bool loc = a.allow_local && row_block_local(a.cnt + (size_t)rbk * rb_lines * kFlagStride, ut, cens, a.err);
  stamp(a.dbg, T + 1, 4);

  // the input projection of step t, gathered one step ahead, after the publish (its latency off
  // the critical path; issued before wave 0's drain it would be part of it: vmcnt retires in order).
  // The char id it needs is loaded one step earlier still, so the gather never waits on an id load.
  int idn = a.ids ? a.ids[b] : 0;   // id of the step whose row load_gi gathers next
  auto load_gi = [&](int t, float (&gi)[3]) {
    if (t >= T) return;
    const float* src = a.ids ? a.P + (size_t)idn * 3 * H : a.Gi + ((size_t)t * Bp + b) * 3 * H;
#pragma unroll
    for (int g = 0; g < 3; ++g) gi[g] = src[g * H + j];
    if (a.ids && t + 1 < T) idn = a.ids[(size_t)(t + 1) * Bp + b];
  };
  float gin[3] = {0.f, 0.f, 0.f};
  load_gi(0, gin);
  for (int t = 0; t < T; ++t) {
    stamp(a.dbg, t, 0);
    const float gi[3] = {gin[0], gin[1], gin[2]};
    f32x4 acc[NR][3];
    zero_acc(acc);
    if (t > 0 || a.h0) {
      // wave w's K-slice [k0, k0 + 32*NKW) is produced by unit tiles k0/16 .. k0/16 + 2*NKW - 1
      bf16x8 af[NKW][NR];
      if (t > 0) {
        // h_t from the producers' exchange tiles (written at step t-1); unit u = k0 + 32kk + lk
        // lives in tile u/16 at column u%16
        const size_t slot = ((size_t)((t - 1) % xr) * nrb + rbk) * nunit;
        wave_wait_load<NKW>(a.cnt + (size_t)rbk * rb_lines * kFlagStride, lane < 2 * NKW, k0 / 16 + lane,
                            (unsigned)t, a.err, [&](int kk) {
          const int u = k0 + kk * 32 + lk;
          const unsigned tb = (unsigned)(((slot + u / 16) * 32 + lr) * 16 + (u & 15)) * 2;
#pragma unroll
          for (int r = 0; r < NR; ++r) af[kk][r] = ld8_sc1(rX, tb + (unsigned)((rt + r) * 16 * 16 * 2));
        });
      } else {   // h_init, row-major HS[0] (written before the launch)
        const unsigned base = (unsigned)((((size_t)b0 + rt * 16 + lr) * H + k0 + lk) * 2);
#pragma unroll
        for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
          for (int r = 0; r < NR; ++r) af[kk][r] = ld8_sc1(rH, base + (unsigned)(r * 16 * H * 2 + kk * 64));
      }
      stamp(a.dbg, t, 1);
#pragma unroll
      for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int g = 0; g < 3; ++g) acc[r][g] = mfma16(af[kk][r], bw[kk][g], acc[r][g]);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[w][r * 3 + g][i * 64 + lane] = acc[r][g][i];
    // FC consumers read wave 2's HF block of step t - 1 once wave 0 signals t + 1: drain it before
    // the barrier wave 0 passes first (its exchange loads retired, so this waits on nothing else)
    if constexpr (FC) {
      if (w == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    stamp(a.dbg, t, 2);
    float gh[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      float s = 0.f;
      if constexpr (RS == 2) {
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) s += part[rb * 4 + ww][g][reg * 64 + ln];
      } else {
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) s += part[ww][rb * 3 + g][reg * 64 + ln];
      }
      gh[g] = s + bh[g];
    }
    const float r = sigmoidf_(gi[0] + gh[0]);
    const float z = sigmoidf_(gi[1] + gh[1]);
    const float n = tanhf_(gi[2] + r * gh[2]);
    const float h = n + z * (hp - n);
    hp = h;
    const u16 hb = f2bf(h);
    stg[row][col] = hb;
    stgT[col][row] = hb;
    __syncthreads();
    stamp(a.dbg, t, 3);
    if (w == 0) {
      // publish: the 32x16 bf16 tile (1 KB, whole lines of its own), 16 B per lane, write-through;
      // drain; one signal.  Then the row-major copy for the GEMMs that read HS later.
      const u32x4 v = *reinterpret_cast<const u32x4*>(&stg[lane >> 1][(lane & 1) * 8]);
      const unsigned xo = (unsigned)((((size_t)(t % xr) * nrb + rbk) * nunit + ut) * 512 + lane * 8) * 2;
      unsigned* fl = a.cnt + ((size_t)rbk * rb_lines + ut) * kFlagStride;
      if (loc) {
        st16_plain(rX, xo, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) signal_flag_local(fl, (unsigned)(t + 1));
      } else {
        st16_sc1(rX, xo, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) signal_flag(fl, (unsigned)(t + 1));
      }
      stamp(a.dbg, t, 4);
      const size_t hs = ((size_t)(t + 1) * Bp + b0 + (lane >> 1)) * H + j0 + (lane & 1) * 8;
      if (FC && !loc) st16_sc1(rH, (unsigned)(hs * 2), v);   // write-through: FC consumers on other XCDs
      else *reinterpret_cast<u32x4*>(a.HSb + hs) = v;
      stamp(a.dbg, t, 5);
    } else if (w == 1 && a.HT) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(&stgT[lane >> 2][(lane & 3) * 8]);
      *reinterpret_cast<u32x4*>(a.HT + (size_t)(j0 + (lane >> 2)) * a.ldT + (size_t)(t + 1) * Bp + b0 + (lane & 3) * 8) = v;
    } else if (w == 2 && a.HF) {   // the backward's dW_hh operand: one whole 1-KB block
      const u32x4 v = *reinterpret_cast<const u32x4*>(&stgT[lane & 15][8 * (lane >> 4)]);
      const size_t hf = (((size_t)(t + 1) * nunit + ut) * nrb + rbk) * 512 + lane * 8;
      if (FC && !loc) st16_sc1(make_rsrc(a.HF, (unsigned)((size_t)(T + 1) * Bp * H * 2)), (unsigned)(hf * 2), v);
      else *reinterpret_cast<u32x4*>(a.HF + hf) = v;
    }
    // the next gather, then the saves for the backward pass, AFTER the publish (not part of wave
    // 0's drain).  Saves as buffer stores: one per-lane offset for the launch, the step in the
    // scalar offset -- with 64-bit VGPR address math the compiler reused the in-flight gather's
    // destination as a temporary and waited for it (+0.3 us per step at H = 512).
    load_gi(t + 1, gin);
    const int sstep = __builtin_amdgcn_readfirstlane(t * Bp * H * 4);   // uniform: no waterfall loop
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(h), rHSf, sv_lane, sstep + Bp * H * 4, 0);
    if (a.s16) {   // packed bf16 (r, z, n, gh_n): one 8-B store at twice the fp32 offsets
      typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
      const u32x2_ pv = {(unsigned)f2bf(r) | ((unsigned)f2bf(z) << 16), (unsigned)f2bf(n) | ((unsigned)f2bf(gh[2]) << 16)};
      __builtin_amdgcn_raw_buffer_store_b64(pv, rS16, sv_lane * 2u, sstep * 2, 0);
    } else if (a.sr) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r), rSr, sv_lane, sstep, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(z), rSz, sv_lane, sstep, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(n), rSn, sv_lane, sstep, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gh[2]), rSg, sv_lane, sstep, 0);
    }
    stamp(a.dbg, t, 6);
  }
  if constexpr (FC) {   // h of the last step complete in HSb / HF -> epoch T + 1 for the consumers
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned* fl = a.cnt + ((size_t)rbk * rb_lines + ut) * kFlagStride;
      if (loc) signal_flag_local(fl, (unsigned)(T + 1));
      else signal_flag(fl, (unsigned)(T + 1));
    }
  }
}

// ==================================================================== two-layer wavefront forward
// Layer hi at step t depends on layer lo only through h_lo(t) (/root/reference/namegensf.cu:773-854:
// layer 1's input is layer 0's output for the same char), so one launch runs lo's step s and hi's
// step s-1 in iteration s = 0..T.  Both operands -- h_lo(s-1) and h_hi(s-2) -- were published by
// the previous iteration, so one poll loop waits for both (lanes 0-31 poll lo's producers, 32-63
// hi's).  The h_lo(s-1) K-slice feeds BOTH lo's recurrent product (W_hh,lo) and hi's input product
// (W_ih,hi): hi needs no Gi GEMM and no Gi buffer.  hi's r/z gates accumulate W_ih x + W_hh h in
// one MFMA chain; its n gate keeps the two apart (n = tanh(gi_n + r gh_n)).
//
// Register/LDS budget (H = 1024, 8 waves, 256 registers each): the three resident weight K-slices
// (W_hh,lo, W_ih,hi, W_hh,hi over K/8) take 36 * NKW = 144.  The exchange operands are loaded
// straight into LDS (buffer_load ... lds, 16 B per lane in MFMA fragment order, 16 KB per wave for
// both streams) and read back per k-step, so they hold no registers across the poll loop.  After
// its MFMAs a wave writes its 14 K-partial tiles over its own staging area (nothing else reads it
// by then); the epilogue sums the eight waves' partials.  (A transposed product -- weights as the
// A operand -- scattered each save store over 16 rows: 1.5 us more per iteration.)  The wave index is read as a scalar so everything derived from it stays in SGPRs.  (Builds that
// kept the operands in registers spilled 51-110 VGPRs; a 4-wave build fit but ran one wave per
// SIMD and exposed every LDS and memory latency: 8.9 us per iteration.)
// Exchange layout, flags, saves and the L2-local hand-off are gru_fwd_seq_kernel's, per layer;
// lo's tile publishes from wave 0 and hi's from wave 1, so the two drains overlap.
template <int NKW>   // k-steps per wave: H / 256
__global__ void __launch_bounds__(512, 1) gru_fwd_seq2_kernel(SeqFwd2Args a) {
  constexpr int NKS = NKW < 4 ? 4 : NKW;   // staging k-steps (>= 4: the area also holds 14 x 256 floats)
  // [wave][stream lo/hi][k-step][row tile][lane] MFMA B fragments; reused as float partials
  // [wave][14][256] (lo r,z,n x 2 row tiles | hi r, z (input + recurrent), gi_n, gh_n x 2)
  __shared__ __attribute__((aligned(16))) bf16x8 stage[8][2][NKS][2][64];
  __shared__ __attribute__((aligned(16))) u16 stg[2][32][24];
  __shared__ __attribute__((aligned(16))) u16 stgT[2][16][40];
  typedef __attribute__((address_space(3))) void lds_void;
  const SeqFwdArgs& L0 = a.lo;
  const SeqFwdArgs& L1 = a.hi;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = L0.H, Bp = L0.Bp, T = L0.T;
  const int nrb = Bp / 32, ut = seq_unit_tile(nrb);
  const int j0 = ut * 16, rbk = seq_row_block(nrb), b0 = rbk * 32;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  const int k0 = w * NKW * 32;
  const unsigned nunit = (unsigned)(H / 16);

  bf16x8 wh0[NKW][3], wi1[NKW][3], wh1[NKW][3];
#pragma unroll
  for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      const size_t o = (size_t)(g * H + j0 + lr) * H + k0 + kk * 32 + lk;
      wh0[kk][g] = ld8(L0.Whh + o);
      wi1[kk][g] = ld8(a.Wih + o);
      wh1[kk][g] = ld8(L1.Whh + o);
    }

  // this thread's epilogue item: row tile q = w / 4, element e = w % 4 of lane `lane`'s accumulator
  // -> (batch row 16 q + 4 (lane >> 4) + e, unit lane & 15), partial index e * 64 + lane; a wave's
  // 64 items are 4 rows x 16 consecutive units, so every save store is 4 whole 64-B segments
  const int q = w >> 2, e = w & 3;
  const int row = q * 16 + 4 * (lane >> 4) + e, col = lane & 15;
  const int b = b0 + row, j = j0 + col, pidx = e * 64 + lane;
  float bh0[3], bh1[3], bi1[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    bh0[g] = L0.bhh[g * H + j];
    bh1[g] = L1.bhh[g * H + j];
    bi1[g] = a.bih[g * H + j];
  }
  float hp0 = L0.h0 ? L0.h0[(size_t)b * H + j] : 0.f;
  float hp1 = L1.h0 ? L1.h0[(size_t)b * H + j] : 0.f;
  const unsigned hs_bytes = (unsigned)((size_t)(T + 1) * Bp * H * 2), x_bytes = (unsigned)((size_t)T * Bp * H * 2);
  const rsrc_t rH0 = make_rsrc(L0.HSb, hs_bytes), rX0 = make_rsrc(L0.xch, x_bytes);
  const rsrc_t rH1 = make_rsrc(L1.HSb, hs_bytes), rX1 = make_rsrc(L1.xch, x_bytes);
  // exchange rings as gru_fwd_seq_kernel's (L0.xring for both layers): lo's tile of step t is read in
  // iteration t + 1, hi's in t + 2; a slot is rewritten xr steps later, after every producer of the
  // row block published the iteration in which it was last read
  const int xr = L0.xring >= 2 ? L0.xring : T;
  zero_next_flags(L0.zero_next, L0.zero_words);
  zero_next_flags(L1.zero_next, L1.zero_words);
  unsigned* const fl0 = L0.cnt + (size_t)rbk * nunit * kFlagStride;
  unsigned* const fl1 = L1.cnt + (size_t)rbk * nunit * kFlagStride;
  const bool loc = L0.allow_local && row_block_local(fl0, ut, (int)nunit, L0.err);

  // k-step kk of stream st (both row tiles) into this wave's staging area, from exchange slot ts
  // (sc1, after a poll saw the producers) or from the row-major HS[0] (the carried state).  Byte
  // offsets: one per-lane VGPR for the launch, the rest (slot, k-step, row tile) in the scalar offset.
  const unsigned xl = (unsigned)((((lk >> 4) * 32 + lr) * 16 + (lk & 15)) * 2);
  const unsigned hl = (unsigned)((lr * H + lk) * 2);
  auto stage_x = [&](int st, int kk, int ts) {
    const rsrc_t rX = st == 0 ? rX0 : rX1;
    const int so = (int)((((size_t)(ts % xr) * nrb + rbk) * nunit + (k0 + kk * 32) / 16) * 1024);
#pragma unroll
    for (int r = 0; r < 2; ++r)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(&stage[w][st][kk][r][0]), 16, xl, so + r * 512, 0, 16);
  };
  auto stage_h0 = [&](int st) {
    const rsrc_t rH = st == 0 ? rH0 : rH1;
#pragma unroll
    for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
      for (int r = 0; r < 2; ++r)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rH, (lds_void*)(&stage[w][st][kk][r][0]), 16, hl,
                                                 (int)((((size_t)b0 + r * 16) * H + k0 + kk * 32) * 2), 0, 16);
  };
  float* const mypart = reinterpret_cast<float*>(&stage[w][0][0][0][0]);
  auto partial = [&](int ww, int set) -> float {
    return reinterpret_cast<const float*>(&stage[ww][0][0][0][0])[set * 256 + pidx];
  };

  // lo's input projection for step t, gathered one iteration ahead (off the critical path), from
  // a char id loaded one iteration before that (the gather never waits on an id load)
  int idn = L0.ids ? L0.ids[b] : 0;
  auto load_gi0 = [&](int t, float (&gi)[3]) {
    if (t >= T) return;
    const float* src = L0.ids ? L0.P + (size_t)idn * 3 * H : L0.Gi + ((size_t)t * Bp + b) * 3 * H;
#pragma unroll
    for (int g = 0; g < 3; ++g) gi[g] = src[g * H + j];
    if (L0.ids && t + 1 < T) idn = L0.ids[(size_t)(t + 1) * Bp + b];
  };
  float gin[3] = {0.f, 0.f, 0.f};
  load_gi0(0, gin);
  for (int s = 0; s <= T; ++s) {
    const bool do0 = s < T, do1 = s > 0;   // lo's step s, hi's step s - 1
    stamp(L0.dbg, s, 0);
    float gi0[3] = {gin[0], gin[1], gin[2]};
    const bool hasA = s > 0 || L0.h0, hasB = do1 && (s > 1 || L1.h0);   // h_lo(s-1), h_hi(s-2)
    if (s >= 2) {
      wave_wait_load2<NKW>(fl0, fl1, k0 / 16, (unsigned)s, (unsigned)(s - 1), L0.err,
                           [&](int kk) { stage_x(0, kk, s - 1); }, [&](int kk) { stage_x(1, kk, s - 2); });
    } else {
      if (s == 1) wave_wait_load<NKW>(fl0, lane < 2 * NKW, k0 / 16 + lane, 1u, L0.err, [&](int kk) { stage_x(0, kk, 0); });
      else if (hasA) stage_h0(0);
      if (hasB) stage_h0(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's staged operands are in LDS
    stamp(L0.dbg, s, 5);
    f32x4 acc0[2][3], acc1[2][4];   // acc1: hi's r, z (input + recurrent), gi_n, gh_n
    zero_acc(acc0);
    zero_acc(acc1);
    if (hasA && hasB) {   // the steady state: every product, no branches between the MFMAs
#pragma unroll
      for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const bf16x8 x = stage[w][0][kk][r][lane], y = stage[w][1][kk][r][lane];
#pragma unroll
          for (int g = 0; g < 3; ++g) acc0[r][g] = mfma16(x, wh0[kk][g], acc0[r][g]);
#pragma unroll
          for (int g = 0; g < 3; ++g) acc1[r][g] = mfma16(x, wi1[kk][g], acc1[r][g]);
          acc1[r][0] = mfma16(y, wh1[kk][0], acc1[r][0]);
          acc1[r][1] = mfma16(y, wh1[kk][1], acc1[r][1]);
          acc1[r][3] = mfma16(y, wh1[kk][2], acc1[r][3]);
        }
    } else {
#pragma unroll
      for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          if (hasA) {
            const bf16x8 x = stage[w][0][kk][r][lane];
#pragma unroll
            for (int g = 0; g < 3; ++g) acc0[r][g] = mfma16(x, wh0[kk][g], acc0[r][g]);
#pragma unroll
            for (int g = 0; g < 3; ++g) acc1[r][g] = mfma16(x, wi1[kk][g], acc1[r][g]);
          }
          if (hasB) {
            const bf16x8 y = stage[w][1][kk][r][lane];
            acc1[r][0] = mfma16(y, wh1[kk][0], acc1[r][0]);
            acc1[r][1] = mfma16(y, wh1[kk][1], acc1[r][1]);
            acc1[r][3] = mfma16(y, wh1[kk][2], acc1[r][3]);
          }
        }
    }
    stamp(L0.dbg, s, 1);
    // partials over this wave's own staging area (its reads above precede these writes in the
    // wave's in-order LDS queue; no other wave reads it before the barrier)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int g = 0; g < 3; ++g) mypart[(r * 3 + g) * 256 + i * 64 + lane] = acc0[r][g][i];
#pragma unroll
        for (int g = 0; g < 4; ++g) mypart[(6 + r * 4 + g) * 256 + i * 64 + lane] = acc1[r][g][i];
      }
    __syncthreads();
    stamp(L0.dbg, s, 2);
    float h0v = 0.f, r0 = 0.f, z0 = 0.f, n0 = 0.f, ghn0 = 0.f;
    float h1v = 0.f, r1 = 0.f, z1 = 0.f, n1 = 0.f, ghn1 = 0.f;
    if (do0) {
      float gh[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) sum += partial(ww, q * 3 + g);
        gh[g] = sum + bh0[g];
      }
      r0 = sigmoidf_(gi0[0] + gh[0]);
      z0 = sigmoidf_(gi0[1] + gh[1]);
      n0 = tanhf_(gi0[2] + r0 * gh[2]);
      ghn0 = gh[2];
      h0v = n0 + z0 * (hp0 - n0);
      hp0 = h0v;
      const u16 hb = f2bf(h0v);
      stg[0][row][col] = hb;
      stgT[0][col][row] = hb;
    }
    if (do1) {
      float v[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) sum += partial(ww, 6 + q * 4 + g);
        v[g] = sum;
      }
      r1 = sigmoidf_(v[0] + bi1[0] + bh1[0]);
      z1 = sigmoidf_(v[1] + bi1[1] + bh1[1]);
      ghn1 = v[3] + bh1[2];
      n1 = tanhf_(v[2] + bi1[2] + r1 * ghn1);
      h1v = n1 + z1 * (hp1 - n1);
      hp1 = h1v;
      const u16 hb = f2bf(h1v);
      stg[1][row][col] = hb;
      stgT[1][col][row] = hb;
    }
    __syncthreads();   // also: every partial read before the next iteration's staging overwrites it
    stamp(L0.dbg, s, 3);
    if (w < 2) {
      // publish (lo from wave 0, hi from wave 1): the 32x16 bf16 tile, write-through unless the row
      // block is XCD-local; drain; one signal.  Then the row-major copy for the later GEMMs.
      const int ly = w, t = s - ly;
      if (ly == 0 ? do0 : do1) {
        const SeqFwdArgs& Y = ly == 0 ? L0 : L1;
        const u32x4 v = *reinterpret_cast<const u32x4*>(&stg[ly][lane >> 1][(lane & 1) * 8]);
        const unsigned xo = (unsigned)((((size_t)(t % xr) * nrb + rbk) * nunit + ut) * 512 + lane * 8) * 2;
        unsigned* fl = (ly == 0 ? fl0 : fl1) + (size_t)ut * kFlagStride;
        const rsrc_t rX = ly == 0 ? rX0 : rX1;
        if (loc) {
          st16_plain(rX, xo, v);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) signal_flag_local(fl, (unsigned)(t + 1));
        } else {
          st16_sc1(rX, xo, v);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) signal_flag(fl, (unsigned)(t + 1));
        }
        if (ly == 0) stamp(L0.dbg, s, 4);
        *reinterpret_cast<u32x4*>(Y.HSb + ((size_t)(t + 1) * Bp + b0 + (lane >> 1)) * H + j0 + (lane & 1) * 8) = v;
      }
    } else if (w < 6) {
      // waves 2, 3: lo's transposed and fragment-tiled copies; waves 4, 5: hi's
      const int ly = (w - 2) >> 1, t = s - ly;
      const SeqFwdArgs& Y = ly == 0 ? L0 : L1;
      if (ly == 0 ? do0 : do1) {
        if (((w - 2) & 1) == 0) {
          if (Y.HT) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(&stgT[ly][lane >> 2][(lane & 3) * 8]);
            *reinterpret_cast<u32x4*>(Y.HT + (size_t)(j0 + (lane >> 2)) * Y.ldT + (size_t)(t + 1) * Bp + b0 + (lane & 3) * 8) = v;
          }
        } else if (Y.HF) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(&stgT[ly][lane & 15][8 * (lane >> 4)]);
          *reinterpret_cast<u32x4*>(Y.HF + (((size_t)(t + 1) * nunit + ut) * nrb + rbk) * 512 + lane * 8) = v;
        }
      }
    }
    // next step's input gather and the saves for the backward pass after the publishes (a load
    // issued before wave 0's drain would be part of it: vmcnt retires in order)
    load_gi0(s + 1, gin);
    if (do0) {
      L0.HSf[((size_t)(s + 1) * Bp + b) * H + j] = h0v;
      const size_t so = ((size_t)s * Bp + b) * H + j;
      if (L0.s16) st_save16(L0.s16 + so * 4, r0, z0, n0, ghn0);
      else if (L0.sr) { L0.sr[so] = r0; L0.sz[so] = z0; L0.sn[so] = n0; L0.sghn[so] = ghn0; }
    }
    if (do1) {
      L1.HSf[((size_t)s * Bp + b) * H + j] = h1v;
      const size_t so = ((size_t)(s - 1) * Bp + b) * H + j;
      if (L1.s16) st_save16(L1.s16 + so * 4, r1, z1, n1, ghn1);
      else if (L1.sr) { L1.sr[so] = r1; L1.sz[so] = z1; L1.sn[so] = n1; L1.sghn[so] = ghn1; }
    }
  }
}

// ==================================================================== backward
// NKW3: k-steps per wave of the dh GEMM (K = 3H split over 8 waves)
// NTW : 16-col tiles per wave of the fused dW_hh accumulator (H / 128); 0 = not fused
// NTP : 16-col tiles per wave of the fused dP accumulator (V / 128); 0 = not fused
// (Rejected and removed in round 4: dy = dl · W_fc inside this kernel, and the fused weight-gradient
// MFMAs inside the publish drain; docs/DESIGN.md §3.4, §6.3.)
template <int NKW3, int NTW, int NTP>
__global__ void __launch_bounds__(512, 1) gru_bwd_seq_kernel(SeqBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float part[8][2][256];      // 16 KB
  __shared__ __attribute__((aligned(16))) u16 srow[3][32][24];        // dGh tile, gate-major (exchange; 48-B rows)
  __shared__ __attribute__((aligned(16))) u16 sgT[4][16][40];         // dGh^T gates r,z,n + dGi_n^T (padded rows)
  __shared__ __attribute__((aligned(16))) float red[6][16][33];
  // H = 1024 (NKW3 = 12): scalar wave index and scalar-offset exchange loads (below); the smaller
  // variants measured slower with them (h512 step 0.2257 -> 0.2327 ms, profiles/r2_bwd_soffset_ab.json)
  constexpr bool kScalarX = NKW3 >= 12;
  const int tid = threadIdx.x, lane = tid & 63, w = kScalarX ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int H = a.H, H3 = 3 * a.H, Bp = a.Bp, T = a.T;
  const int nrb = Bp / 32, ut = seq_unit_tile(nrb);
  const int j0 = ut * 16, rbk = seq_row_block(nrb), b0 = rbk * 32;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  const int k0 = w * NKW3 * 32;
  const unsigned nunit = (unsigned)(H / 16);

  // this wave's K-slice of W_hh^T rows j0..j0+15 (dh = dGh · W_hh), resident all sequence: in
  // VGPRs, or -- for the variants with fused weight gradients, whose accumulators take the
  // register file -- lane-linear in LDS (each lane re-reads only its own 16-B slots: conflict-free,
  // and program order suffices, no barrier)
  // (also at H = 1024, NKW3 = 12, where the 48-VGPR slice measured 342 -> 327 us per layer in LDS)
  constexpr bool kBwLds = NTW > 0 || NTP > 0 || NKW3 >= 12;
  __shared__ __attribute__((aligned(16))) bf16x8 bwL[kBwLds ? NKW3 : 1][kBwLds ? 512 : 1];
  bf16x8 bw[kBwLds ? 1 : NKW3];
#pragma unroll
  for (int kk = 0; kk < NKW3; ++kk) {
    const bf16x8 v = ld8(a.WhhT + (size_t)(j0 + lr) * H3 + k0 + kk * 32 + lk);
    if constexpr (kBwLds) bwL[kk][tid] = v; else bw[kk] = v;
  }

  const int rb = tid >> 8, reg = (tid >> 6) & 3, ln = tid & 63;
  const int row = rb * 16 + (ln >> 4) * 4 + reg, col = ln & 15;
  const int b = b0 + row, j = j0 + col;
  float carry = 0.f;
  float dbh[3] = {0.f, 0.f, 0.f}, dbi = 0.f;   // dbi: only the n gate differs from dbh
  f32x4 accW[3][NTW > 0 ? NTW : 1];
  f32x4 accP[3][NTP > 0 ? NTP : 1];
  zero_acc(accW);
  zero_acc(accP);
  // exchange ring (SeqBwdArgs::xring, gru_seq16.hip): the slot of step t is reused at step t - xr
  const int xr = a.xring >= 2 ? a.xring : T;
  const rsrc_t rX = make_rsrc(a.xbuf, (unsigned)((size_t)T * Bp * H3 * 2));
  const unsigned xlane = (unsigned)(((lk >> 4) * 3 * 512 + lr * 16 + (lk & 15)) * 2);   // exchange lane offset
  zero_next_flags(a.zero_next, a.zero_words);
  const bool loc = a.allow_local && row_block_local(a.cnt + (size_t)rbk * nunit * kFlagStride, ut, (int)nunit, a.err);
  // the saves of step t-1 are loaded during step t, right after its hand-off: in front of the
  // next poll they would delay it (vmcnt retires in order), and they have a whole step to land
  float sv[6];
  int svid = 0;
  // the step's 32 row ids for the fused dP one-hot: staged through LDS by the epilogue threads of
  // unit column 0 and read back right before use (8 ids held in registers across the barriers and
  // the publish pushed the register file over the limit)
  __shared__ __attribute__((aligned(16))) int idsL[NTP > 0 ? 32 : 1];
  auto load_saves = [&](int t) {
    const size_t o = ((size_t)t * Bp + b) * H + j;
    sv[0] = a.dy[o];
    if (a.s16) ld_save16_raw(a.s16 + o * 4, sv[1], sv[2]);   // unpacked at use
    else { sv[1] = a.sr[o]; sv[2] = a.sz[o]; sv[3] = a.sn[o]; sv[4] = a.sghn[o]; }
    sv[5] = a.HSf[o];   // HS[t] = h_{t-1}
    if constexpr (NTP > 0) svid = a.ids[(size_t)t * Bp + b];   // this thread's row id (fused dP)
  };
  load_saves(T - 1);

  for (int t = T - 1; t >= 0; --t) {
    const int s = T - 1 - t;
    stamp(a.dbg, s, 0);
    f32x4 acc[2];
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1] = acc[0];
    if (s > 0) {
      // wave w's columns [k0, k0 + 32*NKW3) of dGh (3 gates x H) come from unit tiles ((k0+16p) mod H)/16
      bf16x8 af[NKW3][2];
      // dGh_{t+1} column c = k0 + 32kk + lk (gate c/H, unit c%H) lives in producer tile (c%H)/16 of
      // slot t+1 at column (c/H)*16 + c%16
      // 32-column k-steps never straddle a gate (H % 32 == 0): gate c0 / H and producer tile
      // (c0 % H) / 16 are wave-uniform (scalar offset); the lane part is fixed for the launch
      const size_t slot = ((size_t)((t + 1) % xr) * nrb + rbk) * nunit;
      wave_wait_load<NKW3>(a.cnt + (size_t)rbk * nunit * kFlagStride, lane < 2 * NKW3,
                           ((k0 + 16 * lane) % H) / 16, (unsigned)s, a.err, [&](int kk) {
        if constexpr (kScalarX) {
          const int c0 = k0 + kk * 32;
          const int so = (int)((((slot + (size_t)((c0 % H) / 16)) * 3 + (size_t)(c0 / H)) * 512) * 2);
#pragma unroll
          for (int r = 0; r < 2; ++r) af[kk][r] = ld8_sc1s(rX, xlane + (unsigned)(r * 16 * 16 * 2), so);
        } else {
          const int c = k0 + kk * 32 + lk, u = c % H;
          const unsigned tb = (unsigned)(((slot + u / 16) * 3 + c / H) * 512 + lr * 16 + (u & 15)) * 2;
#pragma unroll
          for (int r = 0; r < 2; ++r) af[kk][r] = ld8_sc1(rX, tb + (unsigned)(r * 16 * 16 * 2));
        }
      });
      stamp(a.dbg, s, 1);
#pragma unroll
      for (int kk = 0; kk < NKW3; ++kk) {
        bf16x8 bk;
        if constexpr (kBwLds) bk = bwL[kk][tid]; else bk = bw[kk];
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = mfma16(af[kk][r], bk, acc[r]);
      }
    }
    const int idc = svid;
    float sr = sv[1], sz = sv[2], sn = sv[3], sghn = sv[4];
    const float dy = sv[0], hprev = sv[5];
    if (t > 0) load_saves(t - 1);
    if (a.s16) unpack_save16(sr, sz, sr, sz, sn, sghn);
    // operands of the fused weight-gradient MFMAs (independent of other workgroups): issued after
    // the hand-off so the poll above does not wait behind them; first used after the publish
    bf16x8 hB[NTW > 0 ? NTW : 1];
    if constexpr (NTW > 0) {
      if (a.HF) {   // whole 1-KB fragment blocks (8 lines each) instead of 16 rows x 64 B
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
          hB[nt] = ld8(a.HF + (((size_t)t * nunit + w * NTW + nt) * nrb + rbk) * 512 + lane * 8);
      } else {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
          hB[nt] = ld8(a.HT + (size_t)(w * NTW * 16 + nt * 16 + lr) * a.ldT + (size_t)t * Bp + b0 + lk);
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][r][i * 64 + lane] = acc[r][i];
    __syncthreads();
    stamp(a.dbg, s, 2);
    float dh = dy + carry;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) dh += part[ww][rb][reg * 64 + ln];
    const float dn = dh * (1.f - sz);
    const float dz = dh * (hprev - sn);
    const float dan = dn * (1.f - sn * sn);
    const float dar = dan * sghn * sr * (1.f - sr);
    const float daz = dz * sz * (1.f - sz);
    const float dhn = dan * sr;
    carry = sz * dh;
    dbh[0] += dar; dbh[1] += daz; dbh[2] += dhn; dbi += dan;
    const u16 br = f2bf(dar), bz = f2bf(daz), bn = f2bf(dhn), bi = f2bf(dan);
    srow[0][row][col] = br; srow[1][row][col] = bz; srow[2][row][col] = bn;
    sgT[0][col][row] = br; sgT[1][col][row] = bz; sgT[2][col][row] = bn; sgT[3][col][row] = bi;
    if constexpr (NTP > 0) {
      if (col == 0) idsL[row] = idc;
    }
    __syncthreads();
    stamp(a.dbg, s, 3);
    // fused weight-gradient MFMAs (A = this step's dG^T tile from LDS), off the exchange: every wave
    // runs them after the publish / transposed copies.  (Deferred into the next step's exchange-load window they delayed its
    // recurrent MFMAs: 0.2199 -> 0.2291 ms, profiles/r2_rejected_ab.jsonl)
    auto fused_mma = [&]() {
      if constexpr (NTW > 0 || NTP > 0) {
        bf16x8 ga[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) ga[g] = *reinterpret_cast<const bf16x8*>(&sgT[g][lr][lk]);
        if constexpr (NTW > 0) {
#pragma unroll
          for (int g = 0; g < 3; ++g)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) accW[g][nt] = mfma16(ga[g], hB[nt], accW[g][nt]);
        }
        if constexpr (NTP > 0) {
          ga[2] = *reinterpret_cast<const bf16x8*>(&sgT[3][lr][lk]);   // dGi: n gate without r
          int idv[8];
          const int4 i0 = *reinterpret_cast<const int4*>(&idsL[lk]), i1 = *reinterpret_cast<const int4*>(&idsL[lk + 4]);
          idv[0] = i0.x; idv[1] = i0.y; idv[2] = i0.z; idv[3] = i0.w;
          idv[4] = i1.x; idv[5] = i1.y; idv[6] = i1.z; idv[7] = i1.w;
#pragma unroll
          for (int nt = 0; nt < NTP; ++nt) {
            const int v = (w * NTP + nt) * 16 + lr;
            bf16x8 oh;
#pragma unroll
            for (int e = 0; e < 8; ++e) oh[e] = (__bf16)(idv[e] == v ? 1.0f : 0.0f);
#pragma unroll
            for (int g = 0; g < 3; ++g) accP[g][nt] = mfma16(ga[g], oh, accP[g][nt]);
          }
        }
      }
    };
    if (w == 0) {
      // publish the dGh_t tile as 3 gate blocks of [32 rows][16 units] (1 KB each, whole lines of its
      // own): a consumer's 16-row fragment of one gate is then 512 contiguous bytes per producer
      // (8 full lines per load instruction instead of 16-row x 96-B strided pieces)
      const size_t tile = (((size_t)(t % xr) * nrb + rbk) * nunit + ut) * (3 * 32 * 16);
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(&srow[g][lane >> 1][(lane & 1) * 8]);
        if (loc) st16_plain(rX, (unsigned)((tile + g * 512 + lane * 8) * 2), v);
        else st16_sc1(rX, (unsigned)((tile + g * 512 + lane * 8) * 2), v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned* fl = a.cnt + ((size_t)rbk * nunit + ut) * kFlagStride;
      if (lane == 0) {
        if (loc) signal_flag_local(fl, (unsigned)(s + 1));
        else signal_flag(fl, (unsigned)(s + 1));
      }
      stamp(a.dbg, s, 4);
    } else if (w <= 4 && a.dghT) {
      // transposed copies for the (non-fused) weight-gradient GEMMs: 16 units x 32 rows per gate
      const int g = w - 1;          // 0..3 : dGh r, z, n and dGi n
      const u32x4 v = *reinterpret_cast<const u32x4*>(&sgT[g][lane >> 2][(lane & 3) * 8]);
      const size_t c0 = (size_t)t * Bp + b0 + (lane & 3) * 8;
      const int gg = g < 3 ? g : 2;
      const size_t rowsel = (size_t)(gg * H + j0 + (lane >> 2)) * a.ldG + c0;
      if (g < 3) *reinterpret_cast<u32x4*>(a.dghT + rowsel) = v;
      if (g != 2) *reinterpret_cast<u32x4*>(a.dgiT + rowsel) = v;
    }
    if (a.dgi) {   // row-major dGi for the layer below, after the publish (not in wave 0's drain)
      const size_t og = ((size_t)t * Bp + b) * H3 + j;
      a.dgi[og] = br; a.dgi[og + H] = bz; a.dgi[og + 2 * H] = bi;
    }
    stamp(a.dbg, s, 5);
    fused_mma();
    stamp(a.dbg, s, 6);
  }

  // ---- partial weight gradients of this row block
  if constexpr (NTW > 0) {
    float* W = a.dWhh_part + (size_t)rbk * H3 * H;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          W[(size_t)(g * H + j0 + (lane >> 4) * 4 + i) * H + (w * NTW + nt) * 16 + lr] = accW[g][nt][i];
  }
  if constexpr (NTP > 0) {
    float* Pp = a.dP_part + (size_t)rbk * a.V * H3;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int nt = 0; nt < NTP; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          Pp[(size_t)((w * NTP + nt) * 16 + lr) * H3 + g * H + j0 + (lane >> 4) * 4 + i] = accP[g][nt][i];
  }
  // ---- bias gradients: reduce the per-thread sums over the 32 rows of the block
  red[0][col][row] = dbh[0]; red[1][col][row] = dbh[1]; red[2][col][row] = dbh[2];
  red[3][col][row] = dbh[0]; red[4][col][row] = dbh[1]; red[5][col][row] = dbi;
  __syncthreads();
  if (tid < 96) {
    const int k = tid >> 4, c = tid & 15;
    float sum = 0.f;
    for (int rr = 0; rr < 32; ++rr) sum += red[k][c][rr];
    float* dst = (k < 3 ? a.dbhh_part : a.dbih_part);
    if (dst) dst[(size_t)rbk * H3 + (k % 3) * H + j0 + c] = sum;
  }
}

// ==================================================================== host side
template <class K>
static int resident_blocks(K kernel, int block = 512) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess) return 0;
  return ncu * per;
}

// row-tile split: RS = 2 up to H = 512 (H=512 forward kernel 77.5 -> 72.5 us, per step 2.16 ->
// 2.00 us); RS = 1 at H = 1024, where the K/4 slice's 16 producers per wave measured no better
// (profiles/r1_fwd_row_split_ab.json).
static int fwd_rs(int H) { return H <= 512 ? 2 : 1; }

#define FWD_VARIANTS(X) X(256, 1, 1) X(256, 2, 2) X(512, 2, 1) X(512, 4, 2) X(1024, 4, 1) X(1024, 8, 2)

bool gru_fwd_seq_supported(int H, int Bp) {
  if (Bp % 32) return false;
  const int rs = fwd_rs(H);
  int cap = -1;
#define X(HH, NK, RS) if (H == HH && rs == RS) cap = resident_blocks(gru_fwd_seq_kernel<NK, RS, false>);
  FWD_VARIANTS(X)
#undef X
  return cap >= (H / 16) * (Bp / 32);
}

void gru_fwd_seq(const SeqFwdArgs& a, hipStream_t s) {
  if ((size_t)(a.T + 1) * a.Bp * a.H * (a.s16 ? 8 : 4) >= (1ull << 31))
    throw std::runtime_error("gru_fwd_seq: saves exceed the 2 GB buffer-offset range");
  dim3 grid((a.H / 16) * (a.Bp / 32)), block(512);
  const int rs = fwd_rs(a.H);
#define X(HH, NK, RS)                                                          \
  if (a.H == HH && rs == RS) {                                                \
    hipLaunchKernelGGL((gru_fwd_seq_kernel<NK, RS, false>), grid, block, 0, s, a, SeqFcArgs{});   \
    return;                                                                    \
  }
  FWD_VARIANTS(X)
#undef X
  throw std::runtime_error("gru_fwd_seq: no kernel variant for this shape");
}

// The one-layer forward with the FC consumers in the same grid (H = 512, V = 256): co-residency of
// the H/16 x Bp/32 recurrence blocks AND nrb x kFcCons consumers (two 512-thread workgroups per CU at
// <= 128 VGPRs and ~52 KB of LDS each), and room for both in one 64-lane placement census.
bool gru_fwd_seq_fc_supported(int H, int Bp, int V) {
  if (H != 512 || V != 256 || Bp % 32 || fwd_rs(H) != 2) return false;
  if (H / 16 + kFcCons > 64) return false;
  const int cap = resident_blocks(gru_fwd_seq_kernel<4, 2, true>);
  return cap >= (H / 16 + kFcCons) * (Bp / 32);
}

void gru_fwd_seq_fc(const SeqFwdArgs& a, const SeqFcArgs& f, hipStream_t s) {
  if (a.H != 512 || f.V != 256 || !a.HF || !f.Wf || !f.WTf || !f.dlF || !f.dy || !f.dW || !f.db || !f.loss_part ||
      !f.labels || !f.inv_count || !f.b)
    throw std::runtime_error("gru_fwd_seq_fc: needs H = 512, V = 256, the HF copy and every FC buffer");
  if ((size_t)(a.T + 1) * a.Bp * a.H * (a.s16 ? 8 : 4) >= (1ull << 31))
    throw std::runtime_error("gru_fwd_seq_fc: saves exceed the 2 GB buffer-offset range");
  const int nrb = a.Bp / 32;
  dim3 grid((a.H / 16) * nrb + kFcCons * nrb), block(512);
  if (f.probe & 16)   // diagnostic: the FC build without the 128-VGPR cap (cannot host consumers)
    hipLaunchKernelGGL((gru_fwd_seq_kernel<4, 2, true, 1>), grid, block, 0, s, a, f);
  else
    hipLaunchKernelGGL((gru_fwd_seq_kernel<4, 2, true>), grid, block, 0, s, a, f);
}

#define FWD2_VARIANTS(X) X(256, 1) X(512, 2) X(1024, 4)

bool gru_fwd_seq2_supported(int H, int Bp) {
  if (Bp % 32) return false;
  int cap = -1;
#define X(HH, NK) if (H == HH) cap = resident_blocks(gru_fwd_seq2_kernel<NK>);
  FWD2_VARIANTS(X)
#undef X
  return cap >= (H / 16) * (Bp / 32);
}

void gru_fwd_seq2(const SeqFwd2Args& a, hipStream_t s) {
  const SeqFwdArgs& l0 = a.lo;
  const SeqFwdArgs& l1 = a.hi;
  if (l1.H != l0.H || l1.Bp != l0.Bp || l1.T != l0.T || !a.Wih || !a.bih || !l1.HSf || !l1.HSb || !l1.xch ||
      !l1.cnt || l1.xch == l0.xch || l1.cnt == l0.cnt)
    throw std::runtime_error("gru_fwd_seq2: inconsistent layer arguments");
  dim3 grid((l0.H / 16) * (l0.Bp / 32)), block(512);
#define X(HH, NK)                                                           \
  if (l0.H == HH) {                                                         \
    hipLaunchKernelGGL((gru_fwd_seq2_kernel<NK>), grid, block, 0, s, a);    \
    return;                                                                 \
  }
  FWD2_VARIANTS(X)
#undef X
  throw std::runtime_error("gru_fwd_seq2: no kernel variant for H=" + std::to_string(l0.H));
}

// fused-variant table: (H, fuse dW_hh, fuse dP) -> kernel
#define BWD_VARIANTS(X)               \
  X(256, 3, 2, 2) X(256, 3, 2, 0) X(256, 3, 0, 0) \
  X(512, 6, 4, 2) X(512, 6, 4, 0) X(512, 6, 0, 0) \
  X(1024, 12, 0, 2) X(1024, 12, 0, 0)

bool gru_bwd_seq_supported(int H, int Bp, bool fuse_w, bool fuse_p) {
  if (Bp % 32) return false;
  int cap = -1;
#define X(HH, NK, NW, NP) \
  if (H == HH && (NW > 0) == fuse_w && (NP > 0) == fuse_p) cap = resident_blocks(gru_bwd_seq_kernel<NK, NW, NP>);
  BWD_VARIANTS(X)
#undef X
  return cap >= (H / 16) * (Bp / 32);
}

void gru_bwd_seq(const SeqBwdArgs& a, hipStream_t s) {
  dim3 grid((a.H / 16) * (a.Bp / 32)), block(512);
  const bool fw = a.dWhh_part != nullptr, fp = a.dP_part != nullptr;
#define X(HH, NK, NW, NP)                                                              \
  if (a.H == HH && (NW > 0) == fw && (NP > 0) == fp) {                                \
    hipLaunchKernelGGL((gru_bwd_seq_kernel<NK, NW, NP>), grid, block, 0, s, a);       \
    return;                                                                            \
  }
  BWD_VARIANTS(X)
#undef X
  // an unmatched (H, fuse dW_hh, fuse dP) must not silently leave the gradients untouched
  throw std::runtime_error("gru_bwd_seq: no kernel variant for H=" + std::to_string(a.H) +
                           " fuse_w=" + std::to_string(fw) + " fuse_p=" + std::to_string(fp));
}

}  // namespace gk
