// hipBLASLt for the large *plain* GEMMs (no one-hot A operand, no fused bias): the weight-gradient
// products over B*T tokens at H >= 2048 and the FC backward dH.  Measured on MI355X
// (scripts/probe_blaslt.cpp, profiles/r1_blaslt_probe.jsonl): 1.38 PFLOP/s on dW_hh at H = 2048
// against 0.89 for the engine's LDS kernel.  Everything fused (persistent recurrence, GRU
// epilogues, one-hot dP, FC + softmax-xent) stays on the hand-written kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace gk {

using u16 = unsigned short;

// Create the handle and the workspace (call before any stream capture; idempotent).
// force: create the handle and workspace even when GK_BLASLT is off (a caller that routes some of its
// own products to the library, e.g. the trainer's weight-gradient engine)
void blaslt_init(bool force = false);
// Smallest GEMM (2*M*N*K, in GFLOP) routed to the library under algo 0: 60, or 0 with GK_BLASLT=all.
// The library is OFF by default (gemm256 took the weight gradients in round 2); GK_BLASLT=1 / all
// enables it.
double blaslt_min_gflop();
bool blaslt_enabled();
// C[M][N] (ldc) = A[M][K] (lda) . B[N][K]^T (ldb), fp32 out, fp32 accumulation (C += with
// accumulate).  Returns false (and launches nothing) when the library has no algorithm for it.
bool blaslt_gemm_nt(const u16* A, int lda, const u16* B, int ldb, float* C, int ldc, int M, int N, int K,
                    bool accumulate, hipStream_t s);

}  // namespace gk
