// 256 x 256 x 64 bf16 MFMA GEMM for the large plain products (the weight gradients over B*T tokens
// at H >= 1024, the hoisted input projections, FC dH at large H):
//     C[M][N] (+)= A[M][K] · B[N][K]^T (+ bias[N]),  fp32 accumulate, optional split-K slabs.
//
// gfx950 structure (cdna_hip_programming.md §5, the 256² geometry):
//   * one 512-thread workgroup per CU (128 KiB LDS), 8 waves as 2 (M) x 4 (N), each wave a 128 x 64
//     output of 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 VGPRs), 64 MFMAs per wave per
//     64-deep k-tile -- 4x the MFMA work per staged byte of the 128² kernel (gemm_lds.hip);
//   * staging global -> LDS with global_load_lds_dwordx4 only (no VGPR round trip): a k-tile is four
//     16 KiB half-tiles (A rows 0-127 / 128-255, B rows 0-127 / 128-255), each a lane-linear
//     [128][64] image filled by 2 wave-instructions per wave; the bank swizzle (16-B chunk c of row
//     r in slot c ^ ((r >> 1) & 7), conflict-free ds_read_b128 fragment reads, docs/DESIGN.md) is
//     applied on the per-lane SOURCE address and on the read;
//   * two k-tile buffers: tile t+1 is issued at the top of tile t and lands under its 64 MFMAs per
//     wave (~2k cycles per SIMD); one vmcnt(0) + barrier per k-tile;
//   * per k-tile the wave runs four groups of 16 MFMAs (k-step x row half) with the fragments of
//     the next group read under the current one (register double buffer, order pinned);
//   * bijective XCD-aware block remap, then a grouped raster (4 tile-rows x all columns) so an
//     XCD's resident workgroups share A and B panels in its L2.
// Measured (scripts/bench_gemm.py, random operands, profiles/r2_gemm256.jsonl): 4096^3 1172 TF,
// 8192^3 1287 TF (hipBLASLt on the same box 1190 / 1441); the 128^2 kernel 906 / 893.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "kernels.h"
#include "common.h"

namespace gk {

typedef __attribute__((address_space(3))) void lds256_t;

namespace {
constexpr int kBM = 256, kBN = 256, kBK = 64;
}

DEV int xcd_remap256(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// RS: also the row sums of A (the bias gradient of a weight-gradient product) into
// rowsumA[split][M], from the A fragments already in registers -- by the waves of the first column
// tile that read each row (wave column 0 of tile column 0), instead of a second pass over A
template <bool BIAS, bool ACC, bool RS>
__global__ void __launch_bounds__(512, 1) gemm256_kernel(GemmArgs a, int ntn, int ntm, int kper) {
  // [buffer][A | B][half][128 rows x 64 bf16]: one array (a second __shared__ object can make
  // hipcc drain vmcnt before every ds_read, cdna_hip_programming.md §5 item 4a)
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][2][128 * 64];
  const int id = xcd_remap256(blockIdx.x, gridDim.x);
  // grouped raster inside each split: runs of kGroupM tile-rows, column-major within the run, so an
  // XCD's ~32 resident workgroups cover a 4 x 8 block of tiles (4 A panels + 8 B panels in its L2)
  // instead of 1 x 32 (1 + 32 panels)
  constexpr int kGroupM = 4;
  const int sp = id / (ntn * ntm), pid = id % (ntn * ntm);
  const int per_group = kGroupM * ntn, first_m = (pid / per_group) * kGroupM;
  const int gm = min(ntm - first_m, kGroupM);
  const int tm = first_m + (pid % per_group) % gm, tn = (pid % per_group) / gm;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, lq = lane >> 4;
  const int row0 = tm * kBM, col0 = tn * kBN;
  const int kbeg = sp * kper, nk = kper / kBK;

  // staging: wave w's instruction q of a half-tile covers rows (2w + q) * 8 .. + 7
  const int srow = lane >> 3, sslot = lane & 7;
  const u16* src[2][2][2];   // [A | B][half][q]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = (2 * w + q) * 8 + srow;
      const int c = sslot ^ ((r >> 1) & 7);
      src[0][h][q] = a.A + (size_t)(row0 + h * 128 + r) * a.lda + kbeg + c * 8;
      src[1][h][q] = a.B + (size_t)(col0 + h * 128 + r) * a.ldb + kbeg + c * 8;
    }
  auto stage = [&](int buf, int kt) {
#pragma unroll
    for (int op = 0; op < 2; ++op)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          __builtin_amdgcn_global_load_lds(src[op][h][q] + kt * kBK, (lds256_t*)(&lds[buf][op][h][(2 * w + q) * 8 * 64]),
                                           16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int bh = wc >> 1, bo = (wc & 1) * 64;   // this wave's B half and row offset inside it
  // fragment reads: A row tile i (0..7) / B column tile j (0..3) at k-step ks of buffer buf
  auto rdA = [&](int buf, int i, int ks) {
    const int r = i * 16 + lr, c = ks * 4 + lq;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][0][wr][r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  auto rdB = [&](int buf, int j, int ks) {
    const int r = bo + j * 16 + lr, c = ks * 4 + lq;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][1][bh][r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  // A k-tile is 4 groups g = (k-step g >> 1, row half g & 1) of 16 MFMAs; the fragments of group
  // g + 1 are read BEFORE the MFMAs of group g (register double buffer), so every LDS read has a
  // 16-MFMA group (~256 cycles) to land instead of stalling the next MFMA.
  bf16x8 a0[4], a1[4], b0[4], b1[4];
  const bool do_rs = RS && tn == 0 && wc == 0;   // wave-uniform
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#define GK_RDA(dst, buf, g) { for (int i = 0; i < 4; ++i) dst[i] = rdA(buf, ((g) & 1) * 4 + i, (g) >> 1); }
#define GK_RDB(dst, buf, g) { for (int j = 0; j < 4; ++j) dst[j] = rdB(buf, j, (g) >> 1); }
#define GK_MMA(ga, gb, g) { for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) \
    acc[((g) & 1) * 4 + i][j] = mfma16(ga[i], gb[j], acc[((g) & 1) * 4 + i][j]); \
    if (do_rs) for (int i = 0; i < 4; ++i) rs[((g) & 1) * 4 + i] = add_sum8(ga[i], rs[((g) & 1) * 4 + i]); }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    // (sched_barrier pins the block order: left alone, hipcc sinks each read to just before its
    // first use and waits lgkmcnt(0) there.  Measured and not kept: a third A set + setprio(1)
    // around each MFMA group, within noise of this order -- profiles/r2_gemm256.jsonl)
    GK_RDA(a0, cur, 0); GK_RDB(b0, cur, 0);
    GK_RDA(a1, cur, 1);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(a0, b0, 0);
    __builtin_amdgcn_sched_barrier(0);
    GK_RDA(a0, cur, 2); GK_RDB(b1, cur, 2);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(a1, b0, 1);
    __builtin_amdgcn_sched_barrier(0);
    GK_RDA(a1, cur, 3);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(a0, b1, 2);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(a1, b1, 3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#undef GK_RDA
#undef GK_RDB
#undef GK_MMA

  if (do_rs) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float v = rs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) a.rowsumA[(size_t)sp * a.M + row0 + wr * 128 + t * 16 + lane] = v;
    }
  }
  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + wc * 64 + j * 16 + lr;
    const float bb = BIAS ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + wr * 128 + i * 16 + lq * 4 + e;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[i][j][e] + bb;
        if (ACC) *dst += v; else *dst = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// The same 256 x 256 x 64 pipeline on v_mfma_f32_32x32x16_bf16: a wave's
// 128 x 64 output is 4 x 2 accumulators of 32 x 32 (f32x16, 128 VGPRs as before), a 64-deep k-tile
// four 16-deep k-steps of 8 MFMAs, each MFMA twice the FLOPs per operand VGPR read of 16x16x32.
// Operand lane map (cdna_hip_programming.md): lane l holds row / column l & 31, k = 8 (l >> 5) + j,
// i.e. 16-B chunk 2 ks + (l >> 5) of the LDS row -- the same XOR swizzle keeps the ds_read_b128
// conflict-free (16 lanes = 16 rows, pairs of rows on the two bank halves, 8 distinct slots).
// Accumulator: col = l & 31, row = (q & 3) + 8 (q >> 2) + 4 (l >> 5) for register q.
typedef float f32x16 __attribute__((ext_vector_type(16)));
DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <bool BIAS, bool ACC, bool RS>
__global__ void __launch_bounds__(512, 1) gemm256m32_kernel(GemmArgs a, int ntn, int ntm, int kper) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][2][128 * 64];
  const int id = xcd_remap256(blockIdx.x, gridDim.x);
  constexpr int kGroupM = 4;
  const int sp = id / (ntn * ntm), pid = id % (ntn * ntm);
  const int per_group = kGroupM * ntn, first_m = (pid / per_group) * kGroupM;
  const int gm = min(ntm - first_m, kGroupM);
  const int tm = first_m + (pid % per_group) % gm, tn = (pid % per_group) / gm;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int l32 = lane & 31, lh = lane >> 5;
  const int row0 = tm * kBM, col0 = tn * kBN;
  const int kbeg = sp * kper, nk = kper / kBK;

  const int srow = lane >> 3, sslot = lane & 7;
  const u16* src[2][2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = (2 * w + q) * 8 + srow;
      const int c = sslot ^ ((r >> 1) & 7);
      src[0][h][q] = a.A + (size_t)(row0 + h * 128 + r) * a.lda + kbeg + c * 8;
      src[1][h][q] = a.B + (size_t)(col0 + h * 128 + r) * a.ldb + kbeg + c * 8;
    }
  auto stage = [&](int buf, int kt) {
#pragma unroll
    for (int op = 0; op < 2; ++op)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          __builtin_amdgcn_global_load_lds(src[op][h][q] + kt * kBK, (lds256_t*)(&lds[buf][op][h][(2 * w + q) * 8 * 64]),
                                           16, 0, 0);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int bh = wc >> 1, bo = (wc & 1) * 64;
  auto rdA = [&](int buf, int i, int ks) {
    const int r = i * 32 + l32, c = ks * 2 + lh;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][0][wr][r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  auto rdB = [&](int buf, int j, int ks) {
    const int r = bo + j * 32 + l32, c = ks * 2 + lh;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][1][bh][r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  bf16x8 fa[2][4], fb[2][2];   // register double buffer over k-steps
  const bool do_rs = RS && tn == 0 && wc == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#define GK_RD(set, buf, ks) { for (int i = 0; i < 4; ++i) fa[set][i] = rdA(buf, i, ks); \
                              for (int j = 0; j < 2; ++j) fb[set][j] = rdB(buf, j, ks); }
#define GK_MMA(set) { for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) \
    acc[i][j] = mfma32(fa[set][i], fb[set][j], acc[i][j]); \
    if (do_rs) for (int i = 0; i < 4; ++i) rs[i] = add_sum8(fa[set][i], rs[i]); }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    GK_RD(0, cur, 0);
    GK_RD(1, cur, 1);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(0);
    __builtin_amdgcn_sched_barrier(0);
    GK_RD(0, cur, 2);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(1);
    __builtin_amdgcn_sched_barrier(0);
    GK_RD(1, cur, 3);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(0);
    __builtin_amdgcn_sched_barrier(0);
    GK_MMA(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#undef GK_RD
#undef GK_MMA

  if (do_rs) {   // lanes l and l + 32 hold the two k-halves of row l & 31
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = rs[i] + __shfl_xor(rs[i], 32, 64);
      if (lane < 32) a.rowsumA[(size_t)sp * a.M + row0 + wr * 128 + i * 32 + lane] = v;
    }
  }
  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = col0 + wc * 64 + j * 32 + l32;
    const float bb = BIAS ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = row0 + wr * 128 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[i][j][q] + bb;
        if (ACC) *dst += v; else *dst = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Phased, staggered form (round 5, cdna_hip_programming.md §5 "The 256² 8-phase template",
// T3+T4+T5): the same 256 x 256 x 64 tile, 2 (M) x 4 (N) waves of 128 x 64, two 64 KiB k-tile
// buffers -- but the k-tile is four PHASES, each {fragment reads + LDS-DMA staging (segment R) -> raw
// s_barrier -> lgkmcnt(0) -> setprio(1) 16 MFMAs setprio(0) (segment M) -> raw s_barrier}, the
// staging runs ahead with a COUNTED vmcnt (never vmcnt(0) in the loop), and the two wave rows run one
// barrier apart, so on each SIMD (one wave of each row) one wave's M segment overlaps the other's R
// segment and the MFMA pipe does not idle while fragments are read.
//
// A wave's output is 4 quadrants of 64 x 32 (A sub-tile sa = rows 64 sa.. of its row's half, B
// sub-tile sb = cols 32 sb..); phases (A0,F) (A0,S) (A1,S) (A1,F) with F = B sub-tile 0, S = 1, so
// every fragment is read once per k-tile (A in one 32-VGPR set, F / S 16 each).  Buffer kt & 1 holds
// k-tile kt.  Ordering: LDS-DMA data is visible to a ds_read only after the issuing wave's counted
// vmcnt and then a barrier the reader has passed; a buffer region is restaged only after its readers
// retired their reads (lgkmcnt(0)) and then a barrier the stager has passed.  With the rows one
// barrier apart, a program barrier of the lagging row is the NEXT hardware barrier of the leading
// one, so everything shared by both rows needs one program barrier more: a B half (staged by one row,
// read by both) is read two barriers after its wait and restaged two barriers after its last read;
// an A half is staged and read by the same row only and keeps the plain distances.  Per k-tile kt
// (buffer C):
//   R1: read F (4) + A0 (8) of C
//   R2: read S (4) of C; stage B(kt+1) pieces 2, 3 into the other buffer
//   R3: read A1 (8) of C
//   R4: stage A(kt+2) (C's A last read in R3 by this row; SC 1: pieces 0, 1 here, the rest in
//       R1(kt+1)) and B(kt+2) pieces 0, 1 (C's B last read in R2) into C; counted vmcnt -- k-tile
//       kt+1 landed, first read in R1(kt+1) two barriers on
// so most of a k-tile is in flight for four phases before its wait.
// Measured (random operands, same box, profiles/r5_gemm_stagger_sched_ab.jsonl, plain form; the
// unstaggered schedule it replaced and gemm256_kernel -- one vmcnt(0) + __syncthreads per k-tile --
// in r5_gemm_stagger_v2.jsonl): 8192^3 1449 TF (unstaggered 1230, gemm256_kernel 1278, hipBLASLt
// 1613), 4096^3 1316 (1088 / 1187, hipBLASLt 1308), h2048 dW_hh (6144 x 2048 x 65536, 192-row tiles,
// one round) 1384 unsplit (1174 / 975, hipBLASLt 1329), h1024 dW_ih 4-way 1056 (965 / 889).  The R
// segments set the pace: with B(kt+1) pieces 2, 3 in R1 beside its 12 fragment reads instead of R2,
// 1357 / 1234 / 1340 / 1004 TF; with all four B(kt+1) pieces in R1 / R2 (R4 only the A pieces)
// 1456 / 1326 but 1281 on the long-K dW_hh (B then lands two phases after its issue).  The first
// staggered version staged A(kt+1) in R1 / R2 of k-tile kt: h2048 dW_hh unsplit 1093
// (r5_gemm_stagger_v1.jsonl) -- the long-K products need the depth.  Issuing A pieces 2.. of k-tile
// kt+2 in R1(kt+1) instead (at most 4 LDS-DMA pieces in any R segment, three phases of slack for
// them): 8192^3 1398 -> 1475, 4096^3 1241 -> 1291, h1024 dW_ih 4-way 995 -> 1063, but h2048 dW_hh
// unsplit 1336 -> 1307 (r5_gemm_stagger_sc_ab.jsonl), so it is taken up to 128 k-tiles per workgroup.
template <int N> DEV void vmwait256() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// BM = 256 or 192 rows of A per tile (192: M = 3H products at 3H % 256 != 0 or whose 256-row grid
// leaves part of a round idle -- dW_hh at H = 2048 is 32 x 8 = 256 tiles of 192 rows, one full round,
// against 24 x 8 = 192 of 256; gemm256_tile_rows picks by fill).  Waves are 2 (M) x 4 (N) with a
// (BM / 2) x 64 output: RT = BM / 32 row tiles of 16, a quadrant is RT / 2 of them x 2 column tiles.
// LDS per buffer: A [BM][64] + B [256][64] bf16, staged in 1-KiB pieces of 8 rows (one wave
// instruction each): A BM / 64 pieces per wave, B 4.
template <int BM, bool BIAS, bool ACC, bool RS, int SC>
__global__ void __launch_bounds__(512, 1) gemm256p_kernel(GemmArgs a, int ntn, int ntm, int kper, int kGroupM) {
  constexpr int RT = BM / 32, QR = RT / 2;          // row tiles per wave / per quadrant
  constexpr int NA = BM / 64, NB = 4;                // staging pieces per wave: A, B
  static_assert(NB == 4, "the schedule stages B pieces 0, 1 in R4 and 2, 3 in R1");
  constexpr int AOFF = 0, BOFF = BM * 64;            // element offsets inside a buffer
  __shared__ __attribute__((aligned(16))) u16 lds[2][(BM + 256) * 64];   // ONE array (§5 item 4a)
  const int id = xcd_remap256(blockIdx.x, gridDim.x);
  const int sp = id / (ntn * ntm), pid = id % (ntn * ntm);
  const int per_group = kGroupM * ntn, first_m = (pid / per_group) * kGroupM;
  const int gm = min(ntm - first_m, kGroupM);
  const int tm = first_m + (pid % per_group) % gm, tn = (pid % per_group) / gm;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, lq = lane >> 4;
  const int row0 = tm * BM, col0 = tn * kBN;
  const int kbeg = sp * kper, nk = kper / kBK;

  // staging: piece q of wave w covers image rows (NA w + q) * 8 .. + 7 of A, (NB w + q) * 8 .. of B
  const int srow = lane >> 3, sslot = lane & 7;
  // (fixed-size arrays: a local array whose bound depends on BM, captured by the staging lambdas,
  // made ROCm 7.2's host pass drop the kernel's launch stub without a diagnostic)
  static_assert(NA <= 4, "A pieces per wave");
  const u16* srcA[4];
  const u16* srcB[4];
#pragma unroll
  for (int q = 0; q < NA; ++q) {
    const int r = (NA * w + q) * 8 + srow;
    srcA[q] = a.A + (size_t)(row0 + r) * a.lda + kbeg + (sslot ^ ((r >> 1) & 7)) * 8;
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int r = (NB * w + q) * 8 + srow;
    srcB[q] = a.B + (size_t)(col0 + r) * a.ldb + kbeg + (sslot ^ ((r >> 1) & 7)) * 8;
  }
  auto stA = [&](int kt, int q) {
    __builtin_amdgcn_global_load_lds(srcA[q] + kt * kBK, (lds256_t*)(&lds[kt & 1][AOFF + (NA * w + q) * 8 * 64]), 16, 0, 0);
  };
  auto stB = [&](int kt, int q) {
    __builtin_amdgcn_global_load_lds(srcB[q] + kt * kBK, (lds256_t*)(&lds[kt & 1][BOFF + (NB * w + q) * 8 * 64]), 16, 0, 0);
  };

  f32x4 acc[RT][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow = wr * (BM / 2), brow = (wc >> 1) * 128 + (wc & 1) * 64;
  // fragment reads: A sub-tile sa (rows arow + 16 (QR sa + i) + lr), B sub-tile sb (rows
  // brow + 32 sb + 16 j + lr), k-step ks (chunk 4 ks + lq), swizzled as staged
  auto rdA = [&](int buf, int sa, int i, int ks) {
    const int r = arow + (QR * sa + i) * 16 + lr, c = ks * 4 + lq;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][AOFF + r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  auto rdB = [&](int buf, int sb, int j, int ks) {
    const int r = brow + sb * 32 + j * 16 + lr, c = ks * 4 + lq;
    return *reinterpret_cast<const bf16x8*>(&lds[buf][BOFF + r * 64 + ((c ^ ((r >> 1) & 7)) * 8)]);
  };
  bf16x8 fa[2][QR], fb0[2][2], fb1[2][2];   // [k-step][tile]
  // row sums (the workgroups of tile column 0): row tile t of a wave row by its wave column t % 4
  // (spread over the four SIMDs), four v_dot2 per A fragment after the MFMAs that read it.  Measured
  // on the single-round grid of 192-row tiles (6144 x 2048 x 65536; plain 1274 TF): 1183 TF this
  // way, 1092 on the MFMA pipe (A times a fragment of ones), 1047 with the v_dot2 moved into the next
  // R segment -- the R segments, not the MFMAs, set the pace there (profiles/r5_s20_gemm.jsonl,
  // r5_s21_gemm.jsonl, r5_s22_gemm.jsonl).
  const bool do_rs = RS && tn == 0;   // wave-uniform
  float rs[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) rs[i] = 0.f;
#define GK_RA(buf, sa) { _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < QR; ++i) fa[ks][i] = rdA(buf, sa, i, ks); }
#define GK_RB(dst, buf, sb) { _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int j = 0; j < 2; ++j) dst[ks][j] = rdB(buf, sb, j, ks); }
#define GK_MMA(sa, fb, sb) { \
    __builtin_amdgcn_s_setprio(1); \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < QR; ++i) \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) \
        acc[(sa) * QR + i][(sb) * 2 + j] = mfma16(fa[ks][i], fb[ks][j], acc[(sa) * QR + i][(sb) * 2 + j]); \
    __builtin_amdgcn_s_setprio(0); }
#define GK_RS(sa) { if (do_rs) { _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < QR; ++i) \
      if ((((sa) * QR + i) & 3) == wc) rs[(sa) * QR + i] = add_sum8(fa[ks][i], rs[(sa) * QR + i]); } }
#define GK_SYNC() { __builtin_amdgcn_s_barrier(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
                    __builtin_amdgcn_sched_barrier(0); }
#define GK_END() { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); __builtin_amdgcn_sched_barrier(0); }

  // prologue: k-tile 0, then A(1) and B(1) pieces 0, 1; wave row 1 takes one extra barrier
#pragma unroll
  for (int q = 0; q < NB; ++q) stB(0, q);
#pragma unroll
  for (int q = 0; q < NA; ++q) stA(0, q);
  // SC 1: A pieces 2.. of k-tile kt+2 are issued in R1(kt+1) instead of R4(kt) (see gemm256())
  constexpr int NAE = SC == 1 ? 2 : NA;   // A pieces staged in R4
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < NA; ++q) stA(1, q);
    stB(1, 0); stB(1, 1);
    vmwait256<NA + 2>();
  } else {
    vmwait256<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < nk; ++kt) {
    const int C = kt & 1;
    GK_RB(fb0, C, 0);
    __builtin_amdgcn_sched_barrier(0);
    GK_RA(C, 0);
    if constexpr (SC == 1) {
      if (kt >= 1 && kt + 1 < nk) {
#pragma unroll
        for (int q = NAE; q < NA; ++q) stA(kt + 1, q);
      }
    }
    GK_SYNC(); GK_MMA(0, fb0, 0); GK_RS(0); GK_END();
    GK_RB(fb1, C, 1);
    if (kt + 1 < nk) { stB(kt + 1, 2); stB(kt + 1, 3); }
    GK_SYNC(); GK_MMA(0, fb1, 1); GK_END();
    GK_RA(C, 1);
    GK_SYNC(); GK_MMA(1, fb1, 1); GK_RS(1); GK_END();
    if (kt + 2 < nk) {
#pragma unroll
      for (int q = 0; q < NAE; ++q) stA(kt + 2, q);
      stB(kt + 2, 0); stB(kt + 2, 1);
      vmwait256<NAE + 2>();
    } else {
      vmwait256<0>();
    }
    GK_SYNC(); GK_MMA(1, fb0, 0); GK_END();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();

#undef GK_RA
#undef GK_RB
#undef GK_MMA
#undef GK_RS
#undef GK_SYNC
#undef GK_END

  if (do_rs) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      if ((t & 3) != wc) continue;
      float v = rs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) a.rowsumA[(size_t)sp * a.M + row0 + arow + t * 16 + lane] = v;
    }
  }
  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + wc * 64 + j * 16 + lr;
    const float bb = BIAS ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + arow + i * 16 + lq * 4 + e;
        float* dst = C + (size_t)row * a.ldc + col;
        const float v = acc[i][j][e] + bb;
        if (ACC) *dst += v; else *dst = v;
      }
  }
}

// (Round 4: the same tile on a 4-deep ring of 32-deep k-tiles -- three 32 KiB tiles in flight
// instead of one 64 KiB tile, conflict-free 64-B-row swizzle c ^ 2((r >> 3) & 1) -- measured slower on
// every shape: h2048 dW_hh 1032 vs 1122 TF at split 4, sq8192 1190 vs 1254 TF
// (profiles/r4_gemm256_ring.jsonl); removed.  Twice the barriers per MFMA cost more than the deeper
// prefetch gained.)

// Which form (gemm_variants().mfma = 16 / 32 forces one; read per launch so tests and benches switch
// it in-process).  Default: 32x32x16 only for short K-slices (<= 256), where it measured faster --
// h2048 dH 65536 x 2048 x 256: 438 vs 360 TF -- and 16x16x32 elsewhere (sq8192 1284 vs 1203 TF,
// h2048 dW_hh 4-way split 1139 vs 1073 TF; profiles/r3_gemm256_m32.jsonl)
GemmVariants& gemm_variants() {
  static GemmVariants v;
  return v;
}
static int gemm256_mfma(int kper) {
  const int m = gemm_variants().mfma;
  if (m == 16 || m == 32) return m;
  return kper <= 256 ? 32 : 16;
}
// The phased, staggered pipeline (gemm256p_kernel) for the 16x16x32 form: gemm_variants().phased = 1
// always, = 0 never; unset: the split-K / row-sum weight-gradient products, the 192-row shapes and
// K-slices >= 4096, gemm256_kernel (one vmcnt(0) + barrier per k-tile) for the shorter unsplit plain
// products.  In microbenchmarks the staggered kernel led there too (h1024 Gi 795 vs 755 TF, h2048
// logits 770 vs 758, profiles/r5_gemm_plain_shapes_ab.jsonl), but in the h2048 step the logits GEMM
// (with its bias) took 140.7 us on it against 122.6 on gemm256_kernel (r5_c5_step_summary_final.txt,
// r5_c5_step_summary_dp256.txt), so the plain products stay where they were
static int gemm256_phased_mode() {
  const int p = gemm_variants().phased;
  return p == 0 || p == 1 ? p : -1;
}
static bool gemm256_phased() { return gemm256_phased_mode() != 0; }

int gemm256_tile_rows(int M, int N, int K, int splits) {
  if (N % kBN || splits < 1 || K % splits) return 0;
  auto fill = [&](int bm) {
    if (M % bm) return -1.0;
    const long wg = (long)(M / bm) * (N / kBN) * splits, rounds = (wg + 255) / 256;
    return (double)wg / (rounds * 256);
  };
  const double f256 = fill(256), f192 = gemm256_phased() && gemm256_mfma(K / splits) != 32 ? fill(192) : -1.0;
  if (f256 < 0 && f192 < 0) return 0;
  return f192 > f256 + 1e-9 ? 192 : 256;
}

bool gemm256_ok(const GemmArgs& a) {
  if (a.onehot_ids || !a.A) return false;
  if (a.N % kBN || a.splits < 1 || a.K % a.splits) return false;
  const int kper = a.K / a.splits;
  if (kper % kBK || a.lda % 8 || a.ldb % 8) return false;
  if (a.splits > 1 && (a.bias || a.accumulate || a.ldc != a.N)) return false;
  if (a.rowsumA && (a.bias || a.accumulate)) return false;
  return gemm256_tile_rows(a.M, a.N, a.K, a.splits) != 0;
}

void gemm256(const GemmArgs& a, hipStream_t s) {
  if (!gemm256_ok(a)) throw std::runtime_error("gemm256: unsupported shape");
  const int kper = a.K / a.splits;
  const int form = gemm256_mfma(kper);
  const int mode = gemm256_phased_mode();
  const int bm_best = gemm256_tile_rows(a.M, a.N, a.K, a.splits);
  const bool phased = mode == 1 || (mode == -1 && (a.splits > 1 || a.rowsumA || bm_best == 192 || kper >= 4096));
  // where the A pieces of k-tile kt+2 are issued: SC 1 (two in R4(kt), the rest in R1(kt+1), no
  // segment with more than 4 LDS-DMA pieces) up to 128 k-tiles per workgroup, SC 0 (all in R4(kt),
  // four phases of slack) for the long-K products that stream their operands from memory
  // (profiles/r5_gemm_stagger_sc_ab.jsonl); GemmVariants::sched = 0 / 1 forces one
  const int scv = gemm_variants().sched;
  const int sc = scv == 0 || scv == 1 ? scv : (kper / kBK <= 128 ? 1 : 0);
  // raster run length of the staggered kernel: 4 tile-rows; 2 / 8 / 16 measured, none better across
  // shapes (profiles/r5_gemm_groupm_ab.jsonl); GemmVariants::groupm for A/B runs only
  const int gmr = std::max(1, gemm_variants().groupm);
  // the 32x32 form and the unphased 16x16 kernel have 256-row tiles only
  const int bm = (form == 32 || !phased) ? 256 : bm_best;
  if (a.M % bm) throw std::runtime_error("gemm256: M not a multiple of the tile rows");
  const int ntn = a.N / kBN, ntm = a.M / bm;
  const dim3 grid(ntn * ntm * a.splits), block(512);
#define GK_L(B_, A_, R_)                                                                                          \
  do {                                                                                                            \
    if (form == 32) hipLaunchKernelGGL((gemm256m32_kernel<B_, A_, R_>), grid, block, 0, s, a, ntn, ntm, kper);    \
    else if (phased && bm == 192 && sc == 1) hipLaunchKernelGGL((gemm256p_kernel<192, B_, A_, R_, 1>), grid, block, 0, s, a, ntn, ntm, kper, gmr); \
    else if (phased && bm == 192) hipLaunchKernelGGL((gemm256p_kernel<192, B_, A_, R_, 0>), grid, block, 0, s, a, ntn, ntm, kper, gmr); \
    else if (phased && sc == 1) hipLaunchKernelGGL((gemm256p_kernel<256, B_, A_, R_, 1>), grid, block, 0, s, a, ntn, ntm, kper, gmr); \
    else if (phased) hipLaunchKernelGGL((gemm256p_kernel<256, B_, A_, R_, 0>), grid, block, 0, s, a, ntn, ntm, kper, gmr); \
    else hipLaunchKernelGGL((gemm256_kernel<B_, A_, R_>), grid, block, 0, s, a, ntn, ntm, kper);                  \
  } while (0)
  if (a.rowsumA) {   // weight-gradient form: no bias, no accumulate
    if (a.bias || a.accumulate) throw std::runtime_error("gemm256: row sums only without bias / accumulate");
    GK_L(false, false, true);
  } else if (a.bias) {
    if (a.accumulate) GK_L(true, true, false); else GK_L(true, false, false);
  } else {
    if (a.accumulate) GK_L(false, true, false); else GK_L(false, false, false);
  }
#undef GK_L
}

}  // namespace gk
