// Fused FC head: logits = X·W_fc^T + b_fc on MFMA, then in the same launch either
//   * fc_xent  : max-subtracted softmax + cross-entropy + dL/dlogits (training), or
//   * fc_sample: softmax + on-device inverse-CDF sampling (generation).
//
// Replaces the reference's FC matvec + add + set_zero + racy atomic softmax and the
// per-char D2H copy + host `random_select` (/root/reference/namegensf.cu:861-876,
// kernels K7/K2/K8/K9 of SURVEY §2.2, sampler H7 at namegensf.cu:322-333).
// A workgroup owns 32 full rows (all V columns) so the row reductions stay on chip:
// each of the V/64 waves holds a 32x64 slab in 8 MFMA accumulators, rows are reduced
// across the 16 column lanes with DPP-able xor shuffles and across waves through LDS.
#include <cstdlib>
#include <stdexcept>
#include "kernels.h"
#include "mma_tile.h"

namespace gk {

static constexpr int FROWS = 32;

// Computes the wave's 32x64 logits slab (bias added) into acc.
template <int KB>
DEV void fc_logits(f32x4 (&acc)[2][4], const u16* X, const u16* W, const float* bias, int H, int m0,
                   int lane, int w) {
  zero_acc(acc);
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  const u16* A = X + (size_t)(m0 + lr) * H + lk;
  const u16* B = W + (size_t)(w * 64 + lr) * H + lk;
  MmaLoop<2, 4, KB>::run(acc, A, H, B, 16 * H, H / 32);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float bb = bias[w * 64 + c * 16 + lr];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[r][c][i] += bb;
  }
}

// Row max and sum-of-exp over all V columns; results broadcast per (rb, reg) to every lane.
DEV void row_stats(const f32x4 (&acc)[2][4], float* red /*[2][NW][32]*/, int NW, int lane, int w,
                   float (&mx)[2][4], float (&se)[2][4]) {
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float m = fmaxf(fmaxf(acc[r][0][i], acc[r][1][i]), fmaxf(acc[r][2][i], acc[r][3][i]));
      m = max16(m);
      if ((lane & 15) == 0) red[w * 32 + r * 16 + (lane >> 4) * 4 + i] = m;
    }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + (lane >> 4) * 4 + i;
      float m = red[row];
      for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
      mx[r][i] = m;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) s += __expf(acc[r][c][i] - m);
      s = sum16(s);
      if ((lane & 15) == 0) red[NW * 32 + w * 32 + row] = s;
    }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + (lane >> 4) * 4 + i;
      float s = 0.f;
      for (int ww = 0; ww < NW; ++ww) s += red[NW * 32 + ww * 32 + row];
      se[r][i] = s;
    }
}

// dH tile: rows m0..m0+31 x CT*16 columns from n0, K = V, A = dl from LDS (row-major, padded
// stride ldr), B = W_fc^T rows from global (all V/32 k-steps of B issued up front).
template <int CT>
DEV void fc_dh_tile(const u16* dlr, int ldr, const u16* WT, int V, int H, float* dy, int m0, int n0,
                    int lane) {
  const int lr = lane & 15, lq = lane >> 4;
  f32x4 acc[2][CT];
  zero_acc(acc);
  const u16* B = WT + (size_t)(n0 + lr) * V + 8 * lq;
  for (int k0 = 0; k0 < V; k0 += 128) {       // 4 k-steps of B in flight per round
    bf16x8 bf[4][CT];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int c = 0; c < CT; ++c) bf[kk][c] = ld8(B + (size_t)c * 16 * V + k0 + kk * 32);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 af[2];
#pragma unroll
      for (int r = 0; r < 2; ++r)
        af[r] = *reinterpret_cast<const bf16x8*>(dlr + (r * 16 + lr) * ldr + k0 + kk * 32 + 8 * lq);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[r][c] = mfma16(af[r], bf[kk][c], acc[r][c]);
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dy[(size_t)(m0 + r * 16 + lq * 4 + i) * H + n0 + c * 16 + lr] = acc[r][c][i];
}

template <int KB>
__global__ void __launch_bounds__(512) fc_xent_kernel(FcXentArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int m0 = blockIdx.x * FROWS;
  const int V = a.V, ldr = V + 8;
  f32x4 acc[2][4];
  fc_logits<KB>(acc, a.X, a.W, a.b, a.H, m0, lane, w);

  float* red = smem;                               // [2][NW][32]
  float* lab = smem + 2 * NW * 32;                 // [32] label logit
  float* lrow = lab + 32;                          // [32] per-row loss
  u16* st = reinterpret_cast<u16*>(lrow + 32);     // [V][40] bf16 dl^T staging (80-B column stride:
                                                   // the 16 column lanes of a write hit distinct banks)
  u16* dlr = st + (size_t)V * 40;                  // [32][V+8] bf16 dl row-major (dH A operand)
  float mx[2][4], se[2][4];
  row_stats(acc, red, NW, lane, w, mx, se);
  const float inv = a.inv_count[0];
  const int lr = lane & 15;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + (lane >> 4) * 4 + i;
      const int y = a.labels[m0 + row];
      const float scale = (y >= 0) ? inv : 0.f;
      const float rs = __builtin_amdgcn_rcpf(se[r][i]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = w * 64 + c * 16 + lr;
        const float x = acc[r][c][i];
        if (col == y) lab[row] = x;
        const float p = __expf(x - mx[r][i]) * rs;
        const float d = (p - (col == y ? 1.f : 0.f)) * scale;
        const u16 db = f2bf(d);
        if (a.dl) a.dl[(size_t)(m0 + row) * V + col] = db;
        st[col * 40 + row] = db;
        dlr[row * ldr + col] = db;
      }
    }
  __syncthreads();
  // per-row nll (one thread per row), then the block partial
  if (threadIdx.x < FROWS) {
    const int row = threadIdx.x;
    const int y = a.labels[m0 + row];
    float m = red[row];
    for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
    float s = 0.f;
    for (int ww = 0; ww < NW; ++ww) s += red[NW * 32 + ww * 32 + row];
    lrow[row] = (y >= 0) ? (logf(s) + m - lab[row]) * inv : 0.f;
  }
  // dl^T: each column's 32 rows are 64 contiguous bytes -> four 16-B stores
  for (int q = threadIdx.x; q < V * 4; q += blockDim.x) {
    const int col = q >> 2, seg = q & 3;
    *reinterpret_cast<uint4*>(a.dlT + (size_t)col * a.ldT + a.colT + m0 + seg * 8) =
        *reinterpret_cast<const uint4*>(st + col * 40 + seg * 8);
  }
  if (a.dy) {   // fused dH = dl · W_fc; each wave owns H/NW columns
    const int per = a.H / NW, n0 = w * per;
    int c = 0;
    for (; c + 64 <= per; c += 64) fc_dh_tile<4>(dlr, ldr, a.WT, V, a.H, a.dy, m0, n0 + c, lane);
    for (; c < per; c += 16) fc_dh_tile<1>(dlr, ldr, a.WT, V, a.H, a.dy, m0, n0 + c, lane);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < FROWS; ++i) t += lrow[i];
    a.loss_part[blockIdx.x] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// fc_xent for V = 256 with fused dH (the training path at every H % 512 == 0): 8 waves per 32-row
// block, so each SIMD has two waves to overlap latency with, and every weight fragment a wave
// needs is in flight at once instead of a few k-steps at a time:
//   * X [32][H] staged once in LDS (rows padded by 16 B: the 16 rows of a fragment read land in
//     distinct 16-B slots), read as MFMA A operand by all waves;
//   * wave w owns logits columns [32w, 32w+32): its W_fc slab (H/16 fragments) streams in chunks
//     of 8 k-steps, two chunks in flight;
//   * softmax row statistics across the 8 waves through LDS (two barriers);
//   * dlogits (bf16) to LDS as the A operand of dH and as the dl^T staging tile;
//   * wave w owns dH columns [w H/8, (w+1) H/8): its W_fc^T fragments (64 columns x K = 256 per
//     pass) are loaded before the softmax, while the row statistics are being reduced.
// profiles/: 34.5 us -> see r1 notes for the measured time of this variant.
namespace {
constexpr int kX2Pad = 8;   // bf16 of padding per staged X row
}

// fragments from the FT layout (kernels.h ft_offset): one whole 1-KB block per load instruction
template <int NKC>
DEV void fc2_load_w(bf16x8 (&b)[NKC][2], const u16* Wf, int H, int v0, int ks, int lane) {
#pragma unroll
  for (int kk = 0; kk < NKC; ++kk)
#pragma unroll
    for (int c = 0; c < 2; ++c) b[kk][c] = ld8(Wf + ((size_t)((v0 / 16 + c) * (H / 32) + ks + kk) * 64 + lane) * 8);
}
template <int NKC>
DEV void fc2_mma(f32x4 (&acc)[2][2], const bf16x8 (&b)[NKC][2], const u16* xs, int ldx, int ks, int lane) {
  const int lr = lane & 15, lk = 8 * (lane >> 4);
#pragma unroll
  for (int kk = 0; kk < NKC; ++kk) {
    bf16x8 af[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) af[r] = *reinterpret_cast<const bf16x8*>(xs + (r * 16 + lr) * ldx + (ks + kk) * 32 + lk);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[r][c] = mfma16(af[r], b[kk][c], acc[r][c]);
  }
}
// W_fc^T fragments of one 64-column dH pass: [8 k-steps of V=256][4 column tiles]
DEV void fc2_load_wt(bf16x8 (&bt)[8][4], const u16* WTf, int n0, int lane) {
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
#pragma unroll
    for (int c = 0; c < 4; ++c) bt[kk][c] = ld8(WTf + ((size_t)((n0 / 16 + c) * 8 + kk) * 64 + lane) * 8);
}

// DH = true (every default plan): dH = dl · W_fc fused, the dlogits never leave LDS.  DH = false
// writes the row-major bf16 dl instead and leaves dH to a GEMM (a round-2 plan computed dy inside
// the backward sequence kernel from it: fc_xent 16.3 -> 11.4 us but the backward +7-10 us,
// profiles/r2_bwd_dh_ab.jsonl; that consumer was removed in round 4).
template <int HH, bool DH>
__global__ void __launch_bounds__(512, 1) fc_xent_v256_kernel(FcXentArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int nst = 0;
  auto STAMP = [&]() {
    if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[nst] = __builtin_amdgcn_s_memrealtime();
    ++nst;
  };
  STAMP();
  constexpr int V = 256, NW = 8, NKC = 8, LDR = V + 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  constexpr int H = HH;
  const int ldx = H + kX2Pad, m0 = blockIdx.x * FROWS;
  u16* xs = reinterpret_cast<u16*>(smem);                         // [32][H + 8]
  float* red = reinterpret_cast<float*>(xs + FROWS * ldx);         // [2][8][32]
  float* lab = red + 2 * NW * 32;                                  // [32]
  float* lrow = lab + 32;                                          // [32]
  u16* st = reinterpret_cast<u16*>(lrow + 32);                     // [V][40]   dl^T staging
  u16* dlr = st + V * 40;                                          // [32][V+8] dl row-major

  // ---- scalars first (a global load issued behind the weight stream would wait for all of it:
  // vmcnt retires in order), then stage X, and put the first two chunks of this wave's W_fc
  // slab in flight
  const int v0 = w * 32, nks = H / 32;
  const float inv = a.inv_count[0];
  float bias[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) bias[c] = a.b[v0 + c * 16 + lr];
  bf16x8 b0[NKC][2], b1[NKC][2];
  // X: H/128 16-B pieces per thread, loaded ahead of the weight stream
  constexpr int nxp = FROWS * H / 8 / 512;
  uint4 xv[nxp];
#pragma unroll
  for (int e = 0; e < nxp; ++e) {
    const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
    xv[e] = *reinterpret_cast<const uint4*>(a.X + (size_t)(m0 + row) * H + c8 * 8);
  }
  const int ylab = tid < FROWS ? a.labels[m0 + tid] : 0;
  fc2_load_w<NKC>(b0, a.Wf, H, v0, 0, lane);
  if (nks > NKC) fc2_load_w<NKC>(b1, a.Wf, H, v0, NKC, lane);
#pragma unroll
  for (int e = 0; e < nxp; ++e) {
    const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
    *reinterpret_cast<uint4*>(xs + row * ldx + c8 * 8) = xv[e];
  }
  int* ys = reinterpret_cast<int*>(dlr + FROWS * LDR);           // [32] labels of the block
  if (tid < FROWS) ys[tid] = ylab;
  lds_barrier();   // LDS hand-off only: the weight loads stay in flight
  STAMP();

  // ---- logits: 32 rows x this wave's 32 columns, K = H in chunks of 8 k-steps (2 in flight)
  f32x4 acc[2][2];
  zero_acc(acc);
  for (int ks = 0; ks < nks; ks += 2 * NKC) {
    fc2_mma<NKC>(acc, b0, xs, ldx, ks, lane);
    if (ks + 2 * NKC < nks) fc2_load_w<NKC>(b0, a.Wf, H, v0, ks + 2 * NKC, lane);
    if (ks + NKC < nks) {
      fc2_mma<NKC>(acc, b1, xs, ldx, ks + NKC, lane);
      if (ks + 3 * NKC < nks) fc2_load_w<NKC>(b1, a.Wf, H, v0, ks + 3 * NKC, lane);
    }
  }
  // the first dH pass's W_fc^T fragments go out now, under the softmax reductions (not earlier:
  // the scheduler barrier keeps them from overlapping the W_fc slab's registers)
  __builtin_amdgcn_sched_barrier(0);
  STAMP();
  const int per = H / NW;                 // dH columns of this wave (a multiple of 64)
  bf16x8 bt[8][4];
  if constexpr (DH) fc2_load_wt(bt, a.WTf, w * per, lane);
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[r][c][i] += bias[c];

  // ---- softmax statistics over the 8 waves' columns
  float mx[2][4], se[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float m = max16(fmaxf(acc[r][0][i], acc[r][1][i]));
      if (lr == 0) red[w * 32 + r * 16 + lq * 4 + i] = m;
    }
  lds_barrier();   // LDS hand-off only: the weight loads stay in flight
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
  lds_barrier();   // LDS hand-off only: the weight loads stay in flight
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + lq * 4 + i;
      float sum = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sum += red[NW * 32 + ww * 32 + row];
      se[r][i] = sum;
      const int y = ys[row];
      const float scale = (y >= 0) ? inv : 0.f;
      const float rs = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = v0 + c * 16 + lr;
        const float x = acc[r][c][i];
        if (col == y) lab[row] = x;
        const float d = (__expf(x - mx[r][i]) * rs - (col == y ? 1.f : 0.f)) * scale;
        const u16 db = f2bf(d);
        // dl^T staging: row r of column col at r ^ 2 ((col >> 3) & 1) -- with the plain index, columns
        // col and col + 8 of a 32-lane write half met in one bank (40-u16 pitch: 20 dwords, period 8)
        st[col * 40 + (row ^ (((col >> 3) & 1) << 1))] = db;
        dlr[row * LDR + col] = db;
      }
    }
  lds_barrier();   // LDS hand-off only: the weight loads stay in flight
  STAMP();
  // per-row nll (one thread per row; the statistics are still in LDS)
  if (tid < FROWS) {
    const int row = tid, y = ys[row];
    float m = red[row], sum = 0.f;
    for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
    for (int ww = 0; ww < NW; ++ww) sum += red[NW * 32 + ww * 32 + row];
    lrow[row] = (y >= 0) ? (logf(sum) + m - lab[row]) * inv : 0.f;
  }
  // dl^T: each column's 32 rows are 64 contiguous bytes -> four 16-B stores (rows XOR 2 undone by
  // swapping the dword pairs)
  for (int q = tid; q < V * 4; q += 512) {
    const int col = q >> 2, seg = q & 3;
    uint4 v = *reinterpret_cast<const uint4*>(st + col * 40 + seg * 8);
    if ((col >> 3) & 1) v = make_uint4(v.y, v.x, v.w, v.z);
    *reinterpret_cast<uint4*>(a.dlT + (size_t)col * a.ldT + a.colT + m0 + seg * 8) = v;
  }
  STAMP();
  if constexpr (!DH) {   // row-major dl: 32 rows x 512 B, whole 16-B pieces
    for (int q = tid; q < FROWS * V / 8; q += 512) {
      const int r2 = q / (V / 8), c8 = q % (V / 8);
      *reinterpret_cast<uint4*>(a.dl + (size_t)(m0 + r2) * V + c8 * 8) =
          *reinterpret_cast<const uint4*>(dlr + r2 * LDR + c8 * 8);
    }
  }
  // ---- dH = dl · W_fc: 32 rows x this wave's columns, 64 per pass, K = V = 256
  if constexpr (DH) for (int n0 = w * per; n0 < (w + 1) * per; n0 += 64) {
    if (n0 != w * per) fc2_load_wt(bt, a.WTf, n0, lane);
    f32x4 dacc[2][4];
    zero_acc(dacc);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      bf16x8 af[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) af[r] = *reinterpret_cast<const bf16x8*>(dlr + (r * 16 + lr) * LDR + kk * 32 + 8 * lq);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) dacc[r][c] = mfma16(af[r], bt[kk][c], dacc[r][c]);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a.dy[(size_t)(m0 + r * 16 + lq * 4 + i) * H + n0 + c * 16 + lr] = dacc[r][c][i];
  }
  STAMP();
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int i = 0; i < FROWS; ++i) t += lrow[i];
    a.loss_part[blockIdx.x] = t;
  }
  STAMP();
}

// ---------------------------------------------------------------------------------------------
// fc_xent_fl: the V = 256, H = 512 training FC head with W_fc read ONCE per 32-row block (the 8-wave
// kernel above streams it twice, 512 KB per CU: W_fc for the logits, W_fc^T for dH -- the arrival of
// those fragments is most of its 15 us, docs/DESIGN.md §3.4).  The vocabulary is walked in 4 chunks
// of 64 columns; chunk c's 64 x 512 slab of W_fc lands in LDS by DMA (double-buffered, chunk c + 1 in
// flight) and is read twice from the one image:
//   * row reads (ds_read_b128) as the B operand of the chunk's logits  S_c = X · W_c^T  (K = H), X's
//     fragments held in VGPRs for the whole launch;
//   * transposed reads (ds_read_b64_tr_b16) as the B operand of  U = alpha U + e_c · W_c  (K = the
//     chunk's 64 vocabulary columns),
// with an online softmax across chunks (running row max m, alpha = exp(m_old - m_new), e_c = exp(S_c -
// m_new) in bf16).  At the end  dy = scale (U / s - W_fc[y])  = scale (softmax - onehot) · W_fc, the same
// quantity fc_xent computes as dl · W_fc; dl itself (for dW_fc) comes from the logits kept in
// registers, exactly as fc_xent forms it.  W_fc is read from its FT copy (the LDS-DMA source address
// of each lane is the FT position of the 8 elements it places).
// LDS image of a chunk: 4 quarters (128 columns each) of [64 rows][256 B], chunk ch of row r at
// 16 (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))): the row reads of the 16x16x32 operand are 2-way, the
// transposed reads conflict-free (cdna_hip_programming.md T10, image (b)).
namespace {
constexpr int kFlVC = 64;                 // vocabulary columns per chunk
constexpr int kFlQB = 64 * 256;           // one quarter image [64 rows][256 B]
constexpr int kFlCB = 4 * kFlQB;          // one chunk buffer (64 KB)
constexpr int kFlELD = 72;                // e tile row pitch (u16)
}
DEV int fl_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
typedef short fl_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fl_v4s fl_lds_v4s;
typedef __attribute__((address_space(3))) void fl_lds_void;

__global__ void __launch_bounds__(512, 1) fc_xent_fl_kernel(FcXentArgs a) {
  constexpr int H = 512, V = 256, NKS = H / 32, NCH = V / kFlVC;
  // Separate LDS objects on purpose: the compiler's wait insertion treats an LDS-DMA in flight as a
  // possible writer of every LDS read of the SAME object, so one shared buffer would put a vmcnt(0)
  // (the next chunk's DMA) in front of every read of the current chunk
  __shared__ __attribute__((aligned(16))) unsigned char wb0[kFlCB];   // chunk buffers: [4][64][256 B]
  __shared__ __attribute__((aligned(16))) unsigned char wb1[kFlCB];
  __shared__ __attribute__((aligned(16))) u16 et[32 * kFlELD];        // e tile (bf16)
  __shared__ __attribute__((aligned(16))) float red[8 * 32];          // [4][32] max | [4][32] sum partials
  __shared__ float mrow[2 * 32];                                      // running max (by chunk parity)
  __shared__ float alpha[32], srow[32];                               // rescale factors, final sums
  __shared__ int ys[32];                                              // labels
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * FROWS;
  const int r = w & 1, vt = w >> 1;   // this wave's logits tile of a chunk: row tile r, vocab tile vt
  int nst = 0;   // diagnostic phase stamps of workgroup 0 (scripts/probe_fc.py)
  auto STAMP = [&]() {
    if (a.dbg && blockIdx.x == 0 && tid == 0) a.dbg[nst] = __builtin_amdgcn_s_memrealtime();
    ++nst;
  };
  STAMP();
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(a.Wf), (short)0, V * H * 2, 0x00020000);
  // chunk c -> buffer b: wave w places 1-KB pieces n = 8w .. 8w+7 (quarter n / 16, rows 4 (n % 16) .. +3;
  // lane L: row + L / 16, physical 16-B chunk L % 16, i.e. logical chunk (L % 16) ^ swz(row))
  auto dma = [&](int c, int b) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = w * 8 + i, hq = n >> 4, vr = 4 * (n & 15) + (lane >> 4);
      const int h0 = hq * 128 + (((lane & 15) ^ fl_swz(vr)) << 3), v = c * kFlVC + vr;
      const unsigned src = (unsigned)(((((v >> 4) * NKS + (h0 >> 5)) * 64 + (v & 15) + 16 * ((h0 >> 3) & 3)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (fl_lds_void*)((b ? wb1 : wb0) + hq * kFlQB + (n & 15) * 1024),
                                                16, src, 0, 0, 0);
    }
  };
  dma(0, 0);
  // X fragments of row tile r (all K), resident for the launch
  bf16x8 xa[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) xa[ks] = ld8(a.X + (size_t)(m0 + r * 16 + lr) * H + ks * 32 + 8 * lq);
  const float inv = a.inv_count[0];
  if (tid < FROWS) {
    ys[tid] = a.labels[m0 + tid];
    mrow[tid] = -INFINITY;
  }
  // (no global load may follow a DMA inside the chunk loop: waiting for its value would drain the DMA)
  float bvs[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) bvs[c] = a.b[c * kFlVC + vt * 16 + lr];
  dma(1, 1);   // last in the prologue: the first chunk's wait (vmcnt(8)) leaves exactly it in flight
  float s_run = 0.f;   // thread tid < 32: running sum of exp of row tid
  f32x4 lg[NCH], U[2][4];
  zero_acc(U);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int b = c & 1;
    const unsigned char* wb = b ? wb1 : wb0;
    // B1: chunk c in LDS (own pieces: vmcnt -- chunk c + 1's 8 pieces may stay in flight; all: barrier)
    if (c == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    STAMP();
    if (c >= 1 && c + 1 < NCH) dma(c + 1, (c + 1) & 1);   // into chunk c - 1's buffer, read by all waves by now
    // logits tile: rows 16 r + (lane & 15) x vocab columns 64 c + 16 vt + ..., K = H
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    {
      const int vr = vt * 16 + lr, sw = fl_swz(vr);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int ch = ((ks & 3) * 4 + lq) ^ sw;
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wb + (ks >> 2) * kFlQB + vr * 256 + ch * 16);
        acc = mfma16(xa[ks], bfr, acc);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += bvs[c];
    lg[c] = acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float m = max16(acc[i]);
      if (lr == 0) red[vt * 32 + r * 16 + lq * 4 + i] = m;
    }
    lds_barrier();   // B2: the chunk's per-tile row maxima
    STAMP();
    const float* mo = mrow + (c & 1) * 32;
    float* mn_out = mrow + ((c + 1) & 1) * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + lq * 4 + i;
      const float mc = fmaxf(fmaxf(red[row], red[32 + row]), fmaxf(red[64 + row], red[96 + row]));
      const float mn = fmaxf(mo[row], mc);
      const float e = __expf(acc[i] - mn);
      et[row * kFlELD + vt * 16 + lr] = f2bf(e);
      const float se = sum16(e);
      if (lr == 0) red[128 + vt * 32 + row] = se;
    }
    if (tid < FROWS) {
      const float mc = fmaxf(fmaxf(red[tid], red[32 + tid]), fmaxf(red[64 + tid], red[96 + tid]));
      const float mn = fmaxf(mo[tid], mc);
      alpha[tid] = __expf(mo[tid] - mn);   // 0 on the first chunk (m = -inf)
      mn_out[tid] = mn;
    }
    lds_barrier();   // B3: e tile, alpha, the chunk's row sums
    STAMP();
    if (tid < FROWS) s_run = alpha[tid] * s_run + ((red[128 + tid] + red[160 + tid]) + (red[192 + tid] + red[224 + tid]));
    // U = alpha U + e_c · W_c: wave w owns dH columns 64 w .. 64 w + 63
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float al = alpha[rt * 16 + lq * 4 + i];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) U[rt][nt][i] *= al;
      }
#pragma unroll
    for (int ks2 = 0; ks2 < kFlVC / 32; ++ks2) {
      bf16x8 ae[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        ae[rt] = *reinterpret_cast<const bf16x8*>(et + (rt * 16 + lr) * kFlELD + ks2 * 32 + 8 * lq);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        // B[k = v][n = h]: lane 4q + p of each 16-lane group addresses row 32 ks2 + 8 (lane >> 4) + q (+ 4),
        // columns 64 w + 16 nt + 4 p .. +3; lane i of the group receives column i of the 4 rows
        const int q = (lane & 15) >> 2, p = lane & 3;
        const int hin = 64 * (w & 1) + 16 * nt + 4 * p, hq = w >> 1;
        // (assembled as whole 64-bit halves: per-element bf16 inserts were miscompiled into
        // duplicated halves)
        typedef unsigned fl_u32x2 __attribute__((ext_vector_type(2)));
        typedef unsigned fl_u32x4 __attribute__((ext_vector_type(4)));
        fl_u32x2 half[2];
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) {
          const int vr = ks2 * 32 + 8 * lq + 4 * hr + q;
          const unsigned char* ad = wb + hq * kFlQB + vr * 256 + (((hin >> 3) ^ fl_swz(vr)) << 4) + 8 * ((hin >> 2) & 1);
          half[hr] = __builtin_bit_cast(fl_u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((fl_lds_v4s*)(ad)));
        }
        const fl_u32x4 raw = {half[0].x, half[0].y, half[1].x, half[1].y};
        const bf16x8 bt = __builtin_bit_cast(bf16x8, raw);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) U[rt][nt] = mfma16(ae[rt], bt, U[rt][nt]);
      }
    }
  }
  // ---- final row statistics; dl (for dW_fc), the loss, dy
  // the label rows W_fc[y][.] at this lane's dy positions (rows 16 rt + 4 lq + i, columns 64 w + 16 nt +
  // lane & 15), gathered from the FT copy (their latency under the dl pass): dy = scale (U / s - W_fc[y])
  u16 wy[2][4][4];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = max(ys[rt * 16 + lq * 4 + i], 0);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int h = 64 * w + 16 * nt + lr;
        wy[rt][i][nt] = a.Wf[((((v >> 4) * NKS + (h >> 5)) * 64 + (v & 15) + 16 * ((h >> 3) & 3)) * 8) + (h & 7)];
      }
    }
  const float* mfin = mrow + (NCH & 1) * 32;
  if (tid < FROWS) srow[tid] = s_run;
  lds_barrier();
  STAMP();
  float* lab = red;   // [32] label logits (the partial arrays are free now)
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    u16 dv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + lq * 4 + i, col = c * kFlVC + vt * 16 + lr, y = ys[row];
      const float x = lg[c][i];
      if (col == y) lab[row] = x;
      const float scale = y >= 0 ? inv : 0.f;
      const float d = (__expf(x - mfin[row]) * __builtin_amdgcn_rcpf(srow[row]) - (col == y ? 1.f : 0.f)) * scale;
      dv[i] = f2bf(d);
    }
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 pv = {(unsigned)dv[0] | ((unsigned)dv[1] << 16), (unsigned)dv[2] | ((unsigned)dv[3] << 16)};
    *reinterpret_cast<u32x2*>(a.dlT + (size_t)(c * kFlVC + vt * 16 + lr) * a.ldT + a.colT + m0 + r * 16 + lq * 4) = pv;
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rt * 16 + lq * 4 + i, y = ys[row];
      const float scale = y >= 0 ? inv : 0.f, rs = __builtin_amdgcn_rcpf(srow[row]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        a.dy[(size_t)(m0 + row) * H + 64 * w + 16 * nt + lr] = (U[rt][nt][i] * rs - bf2f(wy[rt][i][nt])) * scale;
    }
  lds_barrier();   // label logits
  STAMP();
  if (w == 0) {
    float l = 0.f;
    if (lane < FROWS) {
      const int y = ys[lane];
      l = y >= 0 ? (logf(srow[lane]) + mfin[lane] - lab[lane]) * inv : 0.f;
    }
    l = wave_sum(l);
    if (lane == 0) a.loss_part[blockIdx.x] = l;
  }
  STAMP();
}

bool fc_xent_fl_ok(const FcXentArgs& a) {
  return step_lds_variants().fc_flash && a.V == 256 && a.H == 512 && a.Wf && a.dy && !a.dl && a.M % FROWS == 0 &&
         a.ldT % 4 == 0 && a.colT % 4 == 0;
}

template <int KB>
__global__ void __launch_bounds__(512) fc_sample_kernel(FcSampleArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int m0 = blockIdx.x * FROWS;
  const int V = a.V;
  f32x4 acc[2][4];
  fc_logits<KB>(acc, a.X, a.W, a.b, a.H, m0, lane, w);
  float* red = smem;                   // [2][NW][32]
  float* prob = smem + 2 * NW * 32;    // [32][V]
  float mx[2][4], se[2][4];
  row_stats(acc, red, NW, lane, w, mx, se);
  const int lr = lane & 15;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + (lane >> 4) * 4 + i;
      const float rs = 1.f / se[r][i];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = w * 64 + c * 16 + lr;
        const float p = __expf(acc[r][c][i] - mx[r][i]) * rs;
        prob[row * V + col] = p;
        if (a.probs) a.probs[(size_t)(m0 + row) * V + col] = p;
      }
    }
  __syncthreads();
  // inverse CDF: first index with running fp32 sum > r (namegensf.cu:326-331), else V-1.
  // One wave per row: lane holds V/64 consecutive probabilities, sums them in index order,
  // an exclusive wave scan gives its prefix, and the lowest hitting index wins.
  const int per = V / 64;
  for (int row = w; row < FROWS; row += NW) {
    const int b = m0 + row;
    if (b >= a.N) continue;                              // padding rows (wave-uniform)
    const float rnd = a.rf[(size_t)b * a.max_len + a.step];
    float loc = 0.f;
    for (int e = 0; e < per; ++e) loc += prob[row * V + lane * per + e];
    float inc = loc;                                     // inclusive scan of lane totals
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    float psum = inc - loc;
    int hit = V;                                         // V = "no hit in this lane"
    for (int e = 0; e < per; ++e) {
      psum += prob[row * V + lane * per + e];
      if (psum > rnd) { hit = lane * per + e; break; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hit = min(hit, __shfl_xor(hit, o, 64));
    if (lane == 0) {
      const int sel = (hit >= V) ? V - 1 : hit;
      if (a.alive[b]) {
        a.out[(size_t)b * (a.max_len + 1) + a.step] = (unsigned char)sel;
        if (sel == a.eos) a.alive[b] = 0;
      }
      a.ids[b] = sel;
    }
  }
}

// Generation at V = 256: the 8-wave logits structure of fc_xent_v256 (X tile staged in LDS, each
// wave streaming a 32-column W_fc slab from the fragment-tiled copy, whole lines per load), then
// softmax into an LDS probability tile and the same inverse-CDF scan as fc_sample_kernel.
template <int HH>
__global__ void __launch_bounds__(512, 1) fc_sample_v256_kernel(FcSampleArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int V = 256, NW = 8, NKC = 8, H = HH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int ldx = H + kX2Pad, m0 = blockIdx.x * FROWS;
  u16* xs = reinterpret_cast<u16*>(smem);                         // [32][H + 8]
  float* red = reinterpret_cast<float*>(xs + FROWS * ldx);         // [2][8][32]
  float* prob = red + 2 * NW * 32;                                 // [32][V]
  const int v0 = w * 32, nks = H / 32;
  float bias[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) bias[c] = a.b[v0 + c * 16 + lr];
  bf16x8 b0[NKC][2], b1[NKC][2];
  constexpr int nxp = FROWS * H / 8 / 512;
  uint4 xv[nxp];
#pragma unroll
  for (int e = 0; e < nxp; ++e) {
    const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
    xv[e] = *reinterpret_cast<const uint4*>(a.X + (size_t)(m0 + row) * H + c8 * 8);
  }
  fc2_load_w<NKC>(b0, a.Wf, H, v0, 0, lane);
  if (nks > NKC) fc2_load_w<NKC>(b1, a.Wf, H, v0, NKC, lane);
#pragma unroll
  for (int e = 0; e < nxp; ++e) {
    const int q = tid + e * 512, row = q / (H / 8), c8 = q % (H / 8);
    *reinterpret_cast<uint4*>(xs + row * ldx + c8 * 8) = xv[e];
  }
  __syncthreads();
  f32x4 acc[2][2];
  zero_acc(acc);
  for (int ks = 0; ks < nks; ks += 2 * NKC) {
    fc2_mma<NKC>(acc, b0, xs, ldx, ks, lane);
    if (ks + 2 * NKC < nks) fc2_load_w<NKC>(b0, a.Wf, H, v0, ks + 2 * NKC, lane);
    if (ks + NKC < nks) {
      fc2_mma<NKC>(acc, b1, xs, ldx, ks + NKC, lane);
      if (ks + 3 * NKC < nks) fc2_load_w<NKC>(b1, a.Wf, H, v0, ks + 3 * NKC, lane);
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[r][c][i] += bias[c];
  // softmax over the 8 waves' columns: row max, then row sum of exp
  float mx[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float m = max16(fmaxf(acc[r][0][i], acc[r][1][i]));
      if (lr == 0) red[w * 32 + r * 16 + lq * 4 + i] = m;
    }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + lq * 4 + i;
      float m = red[row];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) m = fmaxf(m, red[ww * 32 + row]);
      mx[r][i] = m;
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[r][c][i] = __expf(acc[r][c][i] - m);
      const float e = sum16(acc[r][0][i] + acc[r][1][i]);
      if (lr == 0) red[NW * 32 + w * 32 + row] = e;
    }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r * 16 + lq * 4 + i;
      float sum = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sum += red[NW * 32 + ww * 32 + row];
      const float rs = 1.f / sum;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int col = v0 + c * 16 + lr;
        const float p = acc[r][c][i] * rs;
        prob[row * V + col] = p;
        if (a.probs) a.probs[(size_t)(m0 + row) * V + col] = p;
      }
    }
  __syncthreads();
  // inverse CDF (namegensf.cu:326-331): one wave per row, 4 consecutive probabilities per lane
  for (int row = w; row < FROWS; row += NW) {
    const int b = m0 + row;
    if (b >= a.N) continue;                              // padding rows (wave-uniform)
    const float rnd = a.rf[(size_t)b * a.max_len + a.step];
    const float4 pv = *reinterpret_cast<const float4*>(prob + row * V + lane * 4);
    const float loc = ((pv.x + pv.y) + pv.z) + pv.w;     // index order, as the reference's loop
    float inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    float psum = inc - loc;
    int hit = V;
    const float pe[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      psum += pe[e];
      if (hit == V && psum > rnd) hit = lane * 4 + e;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hit = min(hit, __shfl_xor(hit, o, 64));
    if (lane == 0) {
      const int sel = (hit >= V) ? V - 1 : hit;
      if (a.alive[b]) {
        a.out[(size_t)b * (a.max_len + 1) + a.step] = (unsigned char)sel;
        if (sel == a.eos) a.alive[b] = 0;
      }
      a.ids[b] = sel;
    }
  }
}

// Row-wise softmax cross-entropy on precomputed logits: one 256-thread block per 32 rows, one wave
// per row at a time (V/64 consecutive logits per lane), fp32 statistics, deterministic loss
// partial (fixed-order sum of the block's rows).
__global__ void __launch_bounds__(256) softmax_xent_kernel(const float* __restrict__ logits, FcXentArgs a) {
  __shared__ u16 st[512][34];        // dl^T staging [V][32 rows] (+2 pad)
  __shared__ float nll[32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, V = a.V, per = V / 64;
  const int m0 = blockIdx.x * 32;
  const float inv = a.inv_count[0];
  // V = 256 (4 logits per lane): one 16-B load per row, all 8 rows of the wave issued up front (one
  // memory latency per block instead of one per row), 8-B dl stores
  if (per == 4) {
    float4 xv[8];
    int yv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int row = m0 + w + 4 * k;
      xv[k] = *reinterpret_cast<const float4*>(logits + (size_t)row * V + lane * 4);
      yv[k] = a.labels[row];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int rr = w + 4 * k, row = m0 + rr, y = yv[k];
      const float x[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
      const float mx = wave_max(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
      float ex[4], se = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) { ex[e] = __expf(x[e] - mx); se += ex[e]; }
      se = wave_sum(se);
      const float rs = 1.f / se, scale = (y >= 0) ? inv : 0.f;
      float ly = 0.f;
      u16 d[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = lane * 4 + e;
        if (col == y) ly = x[e];
        d[e] = f2bf((ex[e] * rs - (col == y ? 1.f : 0.f)) * scale);
        st[col][rr] = d[e];
      }
      if (a.dl)
        *reinterpret_cast<uint2*>(a.dl + (size_t)row * V + lane * 4) =
            make_uint2((unsigned)d[0] | ((unsigned)d[1] << 16), (unsigned)d[2] | ((unsigned)d[3] << 16));
      ly = wave_sum(ly);   // only the label's lane contributes
      if (lane == 0) nll[rr] = (y >= 0) ? (logf(se) + mx - ly) * inv : 0.f;
    }
  } else
  for (int rr = w; rr < 32; rr += 4) {
    const int row = m0 + rr, y = a.labels[row];
    const float* L = logits + (size_t)row * V + lane * per;
    float x[8];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e < per) { x[e] = L[e]; mx = fmaxf(mx, x[e]); }
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e < per) se += __expf(x[e] - mx);
    se = wave_sum(se);
    const float rs = 1.f / se, scale = (y >= 0) ? inv : 0.f;
    float ly = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e < per) {
        const int col = lane * per + e;
        if (col == y) ly = x[e];
        const u16 d = f2bf((__expf(x[e] - mx) * rs - (col == y ? 1.f : 0.f)) * scale);
        if (a.dl) a.dl[(size_t)row * V + col] = d;
        st[col][rr] = d;
      }
    ly = wave_sum(ly);   // only the label's lane contributes
    if (lane == 0) nll[rr] = (y >= 0) ? (logf(se) + mx - ly) * inv : 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (int r = 0; r < 32; ++r) acc += nll[r];
    a.loss_part[blockIdx.x] = acc;
  }
  // dl^T: each vocab column's 32 rows are 64 contiguous bytes -> four 16-B stores
  for (int q = threadIdx.x; q < V * 4; q += 256) {
    const int col = q >> 2, seg = q & 3;
    u16 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = st[col][seg * 8 + e];
    *reinterpret_cast<uint4*>(a.dlT + (size_t)col * a.ldT + a.colT + m0 + seg * 8) = *reinterpret_cast<const uint4*>(v);
  }
}

void softmax_xent(const float* logits, const FcXentArgs& a, hipStream_t s) {
  if (a.V % 64 || a.V > 512 || a.M % 32 || (a.ldT % 8) || (a.colT % 8))
    throw std::runtime_error("softmax_xent: needs V % 64 == 0, V <= 512, M % 32 == 0, 16-B aligned dl^T columns");
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(a.M / 32), dim3(256), 0, s, logits, a);
}

bool fc_xent_fused_ok(int V, int H, int M) { return V == 256 && (H == 512 || H == 1024) && M % FROWS == 0; }

// the 8-wave V = 256 kernel: fused dH (dy + W_fc^T FT copy, no row-major dl), or dl only (no dy)
static bool fc_xent_v256_ok(const FcXentArgs& a) {
  const bool dh = a.dy && a.WTf && !a.dl, dl_only = !a.dy && a.dl;
  return a.V == 256 && a.Wf && (dh || dl_only) && (a.H == 512 || a.H == 1024) && a.M % FROWS == 0;
}

void fc_xent(const FcXentArgs& a, hipStream_t s) {
  if (fc_xent_fl_ok(a)) {
    hipLaunchKernelGGL(fc_xent_fl_kernel, dim3(a.M / FROWS), dim3(512), 0, s, a);
    return;
  }
  if (fc_xent_v256_ok(a)) {
    const size_t shm = (size_t)FROWS * (a.H + kX2Pad) * 2 + (2 * 8 * 32 + 64) * 4 + 256 * 40 * 2 +
                       (size_t)FROWS * (256 + 8) * 2 + FROWS * 4;
    static bool attr = false;
    if (!attr) {
      for (const void* k : {(const void*)fc_xent_v256_kernel<512, true>, (const void*)fc_xent_v256_kernel<1024, true>,
                            (const void*)fc_xent_v256_kernel<512, false>, (const void*)fc_xent_v256_kernel<1024, false>})
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    const dim3 g(a.M / FROWS), blk(512);
    if (a.dy) {
      if (a.H == 512) hipLaunchKernelGGL((fc_xent_v256_kernel<512, true>), g, blk, shm, s, a);
      else hipLaunchKernelGGL((fc_xent_v256_kernel<1024, true>), g, blk, shm, s, a);
    } else {
      if (a.H == 512) hipLaunchKernelGGL((fc_xent_v256_kernel<512, false>), g, blk, shm, s, a);
      else hipLaunchKernelGGL((fc_xent_v256_kernel<1024, false>), g, blk, shm, s, a);
    }
    return;
  }
  const int NW = a.V / 64;
  if (a.dy && (a.H % (16 * NW) || a.V % 128 || !a.WT))
    throw std::runtime_error("fc_xent: fused dH needs H % (V/4) == 0, V % 128 == 0 and W_fc^T");
  const size_t shm = (2 * NW * 32 + 64) * 4 + (size_t)a.V * 40 * 2 + (size_t)FROWS * (a.V + 8) * 2;
  const int nks = a.H / 32;
  dim3 grid(a.M / FROWS), block(64 * NW);
  if (nks % 8 == 0) hipLaunchKernelGGL(fc_xent_kernel<4>, grid, block, shm, s, a);
  else if (nks % 2 == 0) hipLaunchKernelGGL(fc_xent_kernel<2>, grid, block, shm, s, a);
  else hipLaunchKernelGGL(fc_xent_kernel<1>, grid, block, shm, s, a);
}

void fc_sample(const FcSampleArgs& a, hipStream_t s) {
  if (a.Wf && a.V == 256 && (a.H == 512 || a.H == 1024) && a.Bp % FROWS == 0) {
    const size_t shm = (size_t)FROWS * (a.H + kX2Pad) * 2 + (2 * 8 * 32) * 4 + (size_t)FROWS * 256 * 4;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fc_sample_v256_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)fc_sample_v256_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    if (a.H == 512) hipLaunchKernelGGL(fc_sample_v256_kernel<512>, dim3(a.Bp / FROWS), dim3(512), shm, s, a);
    else hipLaunchKernelGGL(fc_sample_v256_kernel<1024>, dim3(a.Bp / FROWS), dim3(512), shm, s, a);
    return;
  }
  const int NW = a.V / 64;
  const size_t shm = (2 * NW * 32) * 4 + (size_t)a.V * FROWS * 4;
  const int nks = a.H / 32;
  dim3 grid(a.Bp / FROWS), block(64 * NW);
  if (nks % 2 == 0) hipLaunchKernelGGL(fc_sample_kernel<2>, grid, block, shm, s, a);
  else hipLaunchKernelGGL(fc_sample_kernel<1>, grid, block, shm, s, a);
}

}  // namespace gk
