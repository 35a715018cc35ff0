// Register-direct MFMA main loop shared by the recurrent-step, FC and generic GEMM kernels.
//
// One wave accumulates an (RB*16) x (CT*16) tile of  C += A[rows][k] * B[cols][k]^T  over
// `nks` 32-deep k-steps.  Both operands are K-contiguous, so each fragment is one 16-byte
// load per lane (common.h).  Loads go straight to VGPRs (no LDS round trip: the
// recurrent GEMMs are latency-bound at M = batch, SURVEY §7.4 hard part 1) and are
// software-pipelined two batches deep with *named* register sets (runtime-indexed
// fragment arrays would spill to scratch: cdna_hip_programming.md §5.4 rule 20).
#pragma once
#include "common.h"

namespace gk {

DEV float sum8(const bf16x8& v) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (float)v[i];
  return s;
}

// A: pointer at (row0 + (lane&15)) * lda + k0 + 8*(lane>>4); row-block stride 16*lda.
// B: pointer at (col0 + (lane&15)) * ldb + k0 + 8*(lane>>4); col-tile c starts at B + c*bts.
// With `rs` non-null the row sums of A are accumulated from the fragments already in registers
// (lane partials; reduce over lane>>4 afterwards) -- no second pass over A.
template <int RB, int CT, int KB>
struct MmaLoop {
  static DEV void load(bf16x8 (&a)[KB][RB], bf16x8 (&b)[KB][CT], const u16* A, int lda,
                       const u16* B, int bts, int kstep) {
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int ko = (kstep + kk) * 32;
#pragma unroll
      for (int r = 0; r < RB; ++r) a[kk][r] = ld8(A + (size_t)r * 16 * lda + ko);
#pragma unroll
      for (int c = 0; c < CT; ++c) b[kk][c] = ld8(B + (size_t)c * bts + ko);
    }
  }
  static DEV void mma(f32x4 (&acc)[RB][CT], const bf16x8 (&a)[KB][RB], const bf16x8 (&b)[KB][CT],
                      float (&rs)[RB], bool do_rs) {
#pragma unroll
    for (int kk = 0; kk < KB; ++kk)
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[r][c] = mfma16(a[kk][r], b[kk][c], acc[r][c]);
    if (do_rs) {
#pragma unroll
      for (int kk = 0; kk < KB; ++kk)
#pragma unroll
        for (int r = 0; r < RB; ++r) rs[r] += sum8(a[kk][r]);
    }
  }
  // nks must be a multiple of KB
  static DEV void run(f32x4 (&acc)[RB][CT], const u16* A, int lda, const u16* B, int bts, int nks,
                      float (&rs)[RB], bool do_rs) {
    const int nb = nks / KB;
    if (nb <= 0) return;
    bf16x8 a0[KB][RB], b0[KB][CT], a1[KB][RB], b1[KB][CT];
    load(a0, b0, A, lda, B, bts, 0);
    int bt = 0;
    for (; bt + 2 <= nb; bt += 2) {
      load(a1, b1, A, lda, B, bts, (bt + 1) * KB);
      mma(acc, a0, b0, rs, do_rs);
      if (bt + 2 < nb) load(a0, b0, A, lda, B, bts, (bt + 2) * KB);
      mma(acc, a1, b1, rs, do_rs);
    }
    if (bt < nb) mma(acc, a0, b0, rs, do_rs);
  }
  static DEV void run(f32x4 (&acc)[RB][CT], const u16* A, int lda, const u16* B, int bts, int nks) {
    float rs[RB];
    run(acc, A, lda, B, bts, nks, rs, false);
  }
};

template <int RB, int CT>
DEV void zero_acc(f32x4 (&acc)[RB][CT]) {
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
}

}  // namespace gk
