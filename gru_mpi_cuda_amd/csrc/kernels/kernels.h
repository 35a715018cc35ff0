// Host-side launch API of every HIP kernel in the engine (gfx950 only).
//
// Reference mapping: the reference's nine kernels K1..K9
// (/root/reference/namegensf.cu:112-300) -- embedding, five element-wise ops, matvec,
// set_zero, softmax -- are replaced by *fused* kernels: one launch per GRU timestep
// (all three gate GEMMs + sigmoid/tanh/Hadamard epilogue), one fused FC+softmax(+xent or
// +sampling) launch, and MFMA GEMMs for the hoisted / weight-gradient products.
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short u16;
#define DEV_HOST_INLINE __host__ __device__ __forceinline__

namespace gk {

// ------------------------------------------------------------------ recurrent steps
struct FwdStepArgs {
  const u16* hprev_bf = nullptr;   // [Bp][H]   h_{t-1} (bf16 MFMA operand)
  const float* hprev_f = nullptr;  // [Bp][H]   h_{t-1} fp32 (blend operand)
  const u16* Whh = nullptr;        // [3H][H]
  const float* bhh = nullptr;      // [3H]
  // input projection source (exactly one):
  const float* P = nullptr;        //   [V][3H] table  Emb·W_ih^T + b_ih, gathered by ids
  const int* ids = nullptr;        //   [Bp]
  const float* Gi = nullptr;       //   [Bp][3H] precomputed (incl. b_ih)
  const u16* x_bf = nullptr;       //   fused: Gi = x_bf[Bp][Kin] · Wih[3H][Kin]^T + bih
  const u16* Wih = nullptr;
  const float* bih = nullptr;
  int Kin = 0;
  // outputs
  float* h_f = nullptr;            // [Bp][H]
  u16* h_bf = nullptr;             // [Bp][H]
  u16* hT = nullptr;               // transposed copy: hT[j*ldT + colT + b]  (nullable)
  int ldT = 0, colT = 0;
  float* sr = nullptr; float* sz = nullptr; float* sn = nullptr; float* sghn = nullptr;  // saves (nullable)
  u16* s16 = nullptr;              // packed bf16 saves [Bp][H][4] (r, z, n, gh_n) instead of sr..sghn
                                   // (LDS-staged kernels only, common.h st_save16)
  int Bp = 0, H = 0;
  int algo = 0;                    // 0 auto, 1 register-direct tile, 2 LDS-staged big tile (gru_step_lds.hip)
};
void gru_fwd_step(const FwdStepArgs& a, hipStream_t s);

struct BwdStepArgs {
  int dgiT_n_only = 0;             // write only the n-gate rows of dgiT (its r/z rows equal dghT's)
  const u16* dgh_next = nullptr;   // [Bp][3H] dGh_{t+1} (null at t = T-1)
  const u16* WhhT = nullptr;       // [H][3H]
  const float* carry_in = nullptr; // [Bp][H]  z_{t+1} ⊙ dh_{t+1}    (null at t = T-1)
  const float* dy = nullptr;       // [Bp][H]  dL/dh_t from above (FC or next layer)
  const float *r = nullptr, *z = nullptr, *n = nullptr, *ghn = nullptr;  // saves at t
  const float* hprev = nullptr;    // [Bp][H]  h_{t-1}
  float* carry_out = nullptr;      // [Bp][H]
  u16* dgh = nullptr;              // [Bp][3H]
  u16* dghT = nullptr;             // [3H][ldT] at column colT + b
  u16* dgiT = nullptr;             // [3H][ldT]
  u16* dgi = nullptr;              // [Bp][3H] row-major dGi (nullable; needed below layer 0 only)
  int ldT = 0, colT = 0, Bp = 0, H = 0;
  int algo = 0;                    // as FwdStepArgs::algo
  // split-K LDS kernel (gru_step_lds.hip): fp32 partial tiles, per-tile arrival counters (64-B
  // lines, zeroed once, monotonic across launches) and the error word of its bounded spin
  float* sk_part = nullptr;
  long sk_part_floats = 0;
  unsigned* sk_cnt = nullptr;
  long sk_cnt_words = 0;
  int sk_map = 0;                  // block -> (tile, split) order (gru_bwd_step_sk_kernel)
  unsigned* err = nullptr;
};
void gru_bwd_step(const BwdStepArgs& a, hipStream_t s);
// split-K count the backward LDS step kernel would use for (H, Bp): 0 = the 64 x 64 kernel;
// workspace: H * Bp * splits fp32 partials, (H/128)(Bp/128) * 16 counter words
int gru_bwd_step_sk_splits(int H, int Bp);
// Run-time kernel / step-plan variants: the measured-best defaults, settable at run time
// (set_step_lds_variants, bench.py --variant) so one process can test or A/B every variant.  The
// large-H step-kernel fields are read per launch (gru_step_lds.hip), the plan fields when a step
// graph is recorded.  0 fields mean "automatic" where noted.
struct StepLdsVariants {
  int fwd64 = 1;         // large-H forward step kernel: the 64-row tile (two workgroups per CU) on grids
                         // of < 512 128-row tiles; 0 = the 128-row 2-deep kernel everywhere
  int bwd_sk_min_h = 1024;  // smallest H that takes the split-K backward step kernel (read per call)
  int dwfc_group = 1;    // single-GPU step: the dW_fc K-slices run after the backward sweep inside the
                         // dW_ih0 / dEmb launch (one launch fewer; 0.2183-0.2226 vs 0.2255-0.2274 ms,
                         // profiles/r4_dwfc_group_ab.jsonl), 0: their own launch before the backward.
  int bwd_big = 1;       // large H x large batch: the persistent split-K backward (0: T step kernels)
  int bwd16 = 1;         // persistent backward on 16-row blocks where 32-row blocks are not XCD-local
                         // (H = 1024, Bp = 128: the config-4 shard)
  int bwd_xring = 2;     // persistent backward (32- and 16-row, large-H): dGh exchange as a ring of this
                         // many slots instead of one per step (0); docs/DESIGN.md §3.1d.  2 since round 6:
                         // headline -0.6 us, config-4 shard -7 us against 4 (profiles/r6_bxr2_*.jsonl)
  int fwd_xring = 4;     // one-layer persistent forward: the same for the h exchange (the two-layer
                         // wavefront keeps one slot per step: measured equal, r4_fwd_xring_ab.jsonl)
  int save16 = 1;        // layers whose forward AND backward kernels take them (LDS-staged step kernels or
                         // the two-layer wavefront; the large-H or 16-row persistent backward): packed
                         // bf16 (r, z, n, gh_n) saves instead of four fp32 arrays (SeqPlan::s16)
  int fc_flash = 0;      // V = 256, H = 512 training FC head: fc_xent_fl (W_fc read once per block, online
                         // softmax over 4 vocabulary chunks, fc.hip); 0: the 8-wave two-stream kernel
  int fwd_fc = 0;        // one-layer H = 512, V = 256: the FC head (fc_xent + dW_fc) as consumer
                         // workgroups inside the persistent forward launch (gru_fwd_seq_fc); 0: after it
  int big_dy = 1;        // top layer on the persistent large-H backward, V = 256: dy = dl · W_fc inside it
                         // (SeqBwdArgs::dl) instead of the dH GEMM + an fp32 dy in memory
  int ld_pad = -1;       // padding of the dGh^T / dGi^T / dl^T leading dimension: -1 = 64 elements where
                         // its rows would be >= 64 KiB apart (trainer.cpp), else this many (tests)
};
// (Round 5 removed the measured-equal / marginal switches fwd_ns, fwd8, fwd64 = 2, fwd64_fused,
// fwd64_all, bwd_sk_pf, bwd_sk_map and big_acq with the code only they reached; docs/DESIGN.md §7.)
StepLdsVariants& step_lds_variants();
// gemm256 (algo 5) forms for A/B runs and tests, set at run time (bindings set_gemm_variants); every
// default is the measured-best rule of gemm256.hip
struct GemmVariants {
  int mfma = 0;     // 16 / 32: force v_mfma_f32_16x16x32 / 32x32x16; 0: by K-slice (32 up to 256 deep)
  int phased = -1;  // 1 / 0: always / never the staggered phased pipeline; -1: by shape
  int sched = -1;   // staggered pipeline staging schedule 0 / 1; -1: by k-tiles per workgroup
  int groupm = 4;   // grouped raster run length (tile-rows)
  int onehot = 1;   // one-hot dP products with V = 256 on the streaming kernel (onehot.hip), 1: 128-column x
                    // 64-token k-tiles, 2: 64 x 128, 3: 32 x 256; 0: the one-hot gemm_lds kernel
};
GemmVariants& gemm_variants();
// LDS-staged large-H step kernels: H % 64 == 0, Bp % 128 == 0, no fused input projection
bool gru_step_lds_ok(int H, int Bp);
// which per-step kernel gru_fwd_step/gru_bwd_step pick for (algo, H, Bp) without fused input
bool gru_step_picks_lds(int algo, int H, int Bp);
void gru_fwd_step_lds(const FwdStepArgs& a, hipStream_t s);
void gru_bwd_step_lds(const BwdStepArgs& a, hipStream_t s);

// ------------------------------------------------------------------ persistent sequence kernels
// One launch per layer runs all T steps (gru_seq.hip).  Requires 512-thread co-residency of
// (H/16) x (Bp/32) workgroups; callers check *_supported() and fall back to per-step kernels.
// Batch preparation: a pinned staging slot (in[0] = rows, in[1] = 1/valid labels as float bits,
// x [Bmax][T] at in + 16, y after it) transposed into ids / labels [T][Bp] (rows >= in[0]: id 0, label -1)
struct PrepJob { const int* in = nullptr; int Bmax = 0, T = 0, Bp = 0; int* ids = nullptr; int* labels = nullptr; float* inv_count = nullptr; };
struct SeqFwdArgs {
  u16* HSb = nullptr;              // [T+1][Bp][H] bf16; HS[0] = h_init, step t writes HS[t+1]
  // exchange copy of h_{t+1}, tiled per producer: [T][Bp/32][H/16][32 rows][16] bf16 -- every
  // 128-B line belongs to ONE producer, so a consumer never loads a line part of which is unpublished
  u16* xch = nullptr;
  float* HSf = nullptr;            // [T+1][Bp][H] fp32
  u16* HT = nullptr; int ldT = 0;  // [H][ldT] bf16, h_t at column (t+1)*Bp + b (nullable)
  // fragment-tiled copy of h for the backward's fused dW_hh (nullable): block (t, unit tile u,
  // row block rb) at ((t * H/16 + u) * Bp/32 + rb) * 512 holds HS[t] units 16u + (l & 15), rows
  // 32rb + 8(l >> 4) .. +8 in lane l's 16 bytes; step t writes block t+1, HF[0] = h_init is the
  // caller's
  u16* HF = nullptr;
  float *sr = nullptr, *sz = nullptr, *sn = nullptr, *sghn = nullptr;   // [T][Bp][H] (nullable)
  u16* s16 = nullptr;              // packed bf16 saves [T][Bp][H][4] instead (two-layer wavefront only)
  const u16* Whh = nullptr; const float* bhh = nullptr;
  const float* P = nullptr; const int* ids = nullptr;   // layer 0: table + ids [T][Bp]
  const float* Gi = nullptr;                            // layers >= 1: [T][Bp][3H]
  const float* h0 = nullptr;       // optional fp32 initial state (HSb[0] must hold its bf16)
  unsigned* cnt = nullptr;         // [Bp/32][H/16][16] epoch flags, zero at launch
  unsigned* zero_next = nullptr;   // flag block of the NEXT sequence kernel, zeroed here (nullable)
  long zero_words = 0;
  unsigned* err = nullptr;
  unsigned long long* dbg = nullptr;   // diagnostic: [2 wgs][T][8] s_memrealtime stamps (nullable)
  int allow_local = 1;             // 0: never the L2-local hand-off (gru_seq.hip row_block_local)
  int xring = 0;                   // h exchange as a ring of xring slots (>= 2; 0 = one per step)
  int T = 0, Bp = 0, H = 0;
};
// FC consumer workgroups per row block of the one-layer forward with the FC head inside (gru_fwd_seq_fc)
static constexpr int kFcCons = 32;
// flag words a sequence kernel needs in `cnt` ([Bp/32] row blocks x (H/16 producers + kFcCons FC
// consumers) x 16-word lines; the consumer lines are used by gru_fwd_seq_fc only); zero per launch
inline long seq_flag_words(int H, int Bp) { return (long)(Bp / 32) * (H / 16 + kFcCons) * 16; }
bool gru_fwd_seq_supported(int H, int Bp);
void gru_fwd_seq(const SeqFwdArgs& a, hipStream_t s);
// The FC head inside the one-layer persistent forward (gru_seq.hip fwd_fc_consumer): kFcCons extra
// workgroups per row block, co-resident with the recurrence, compute each finished step's logits,
// softmax-xent, loss partial, dl and dy = dl · W_fc (fc_xent's work), then the row block's dW_fc /
// db_fc partial (the dW_fc K-slices' work) -- nothing of the FC head is left for after the forward.
struct SeqFcArgs {
  const u16* Wf = nullptr;          // W_fc [V][H] in the FT fragment layout (ft_offset)
  const u16* WTf = nullptr;         // W_fc^T [H][V] in the FT fragment layout
  const float* b = nullptr;         // b_fc [V]
  const int* labels = nullptr;      // [T][Bp], -1 = ignore
  const float* inv_count = nullptr; // device scalar 1 / #valid tokens
  float* dy = nullptr;              // [T*Bp][H] fp32 dL/dh of the top layer
  u16* dlF = nullptr;               // [T][Bp/32][V/16] 1-KB blocks of dl^T fragments (T*Bp*V bf16)
  float* loss_part = nullptr;       // [T*Bp/32] per-32-row loss partials (fc_xent's order)
  float* dW = nullptr;              // [Bp/32][V][H] dW_fc partial per row block
  float* db = nullptr;              // [Bp/32][V] db_fc partial per row block
  int V = 0;
  int probe = 0;                    // diagnostic (scripts/probe_fwd_fc.py): 1 consumers stop after the
                                    // census, 2 after their items (no dW_fc); 0 = everything
};
bool gru_fwd_seq_fc_supported(int H, int Bp, int V);
void gru_fwd_seq_fc(const SeqFwdArgs& a, const SeqFcArgs& f, hipStream_t s);


// Two-layer wavefront forward (gru_seq.hip gru_fwd_seq2_kernel): ONE persistent launch runs layer
// `lo` at step s and layer `hi` at step s-1 in iteration s = 0..T.  hi's input projection
// W_ih · h_lo(t) + b_ih is computed in the kernel from the same exchange tiles lo's next step reads
// (no Gi GEMM, no Gi buffer); lo takes its input projection as SeqFwdArgs does (P table or Gi).
// hi.Gi is unused; hi.xch and hi.cnt must not alias lo's.
struct SeqFwd2Args {
  SeqFwdArgs lo, hi;
  const u16* Wih = nullptr;     // hi's W_ih [3H][H] bf16
  const float* bih = nullptr;   // hi's b_ih [3H]
};
bool gru_fwd_seq2_supported(int H, int Bp);
void gru_fwd_seq2(const SeqFwd2Args& a, hipStream_t s);

struct SeqBwdArgs {
  const float* dy = nullptr;       // [T][Bp][H]
  const float *sr = nullptr, *sz = nullptr, *sn = nullptr, *sghn = nullptr;   // [T][Bp][H]
  const u16* s16 = nullptr;        // packed bf16 saves [T][Bp][H][4] instead (16-row and large-H kernels)
  const float* HSf = nullptr;      // [T+1][Bp][H]
  const u16* HT = nullptr; int ldT = 0;     // h_{t-1} at column t*Bp + b (fused dW_hh)
  const u16* HF = nullptr;         // SeqFwdArgs::HF of the same layer: preferred over HT when set
  const u16* WhhT = nullptr;       // [H][3H]
  u16* xbuf = nullptr;             // dGh exchange, tiled per producer, one slot per step or a ring of
                                   // xring slots: [T or xring][Bp/32][H/16][3 gates][32 rows][16 units] bf16
  u16* dghT = nullptr; u16* dgiT = nullptr; int ldG = 0;   // [3H][ldG] transposed copies (nullable)
  u16* dgi = nullptr;              // [T][Bp][3H] row-major dGi (nullable)
  float* dWhh_part = nullptr;      // [Bp/32][3H][H] fused dW_hh partials (nullable = not fused)
  float* dbhh_part = nullptr;      // [Bp/32][3H]
  float* dbih_part = nullptr;      // [Bp/32][3H]
  const int* ids = nullptr;        // [T][Bp] (fused dP)
  float* dP_part = nullptr; int V = 0;   // [Bp/32][V][3H] (nullable = not fused)
  unsigned* cnt = nullptr;
  unsigned* zero_next = nullptr;   // as SeqFwdArgs
  long zero_words = 0;
  unsigned* err = nullptr;
  unsigned long long* dbg = nullptr;   // diagnostic stamps, as SeqFwdArgs::dbg
  int allow_local = 1;             // as SeqFwdArgs::allow_local
  float* part = nullptr;           // large-H kernel: split-K partial tiles (gru_bwd_seq_big_part_floats)
                                   // (one fetch per XCD, shared in its L2) instead of sc1 loads
  int dgiT_n_only = 0;             // large-H kernel: dGi^T gets only the n-gate rows (r / z = dGh^T's)
  // large-H kernel, top layer: dy = dl · W_fc computed inside (one extra 64-deep k-tile per K-slice,
  // run while the exchange flags are awaited) instead of read from `dy`: dl [T*Bp][V] bf16 row-major
  // (softmax_xent's), W_fc^T [H][V] bf16, V = 4 x 64
  const u16* dl = nullptr;
  const u16* WfcT = nullptr;
  int xring = 0;                   // step / 16-row kernels: exchange slots reused every xring steps
                                   // (>= 2; 0 = one per step; StepLdsVariants::bwd_xring)
  int T = 0, Bp = 0, H = 0;
};
bool gru_bwd_seq_supported(int H, int Bp, bool fuse_w, bool fuse_p);
void gru_bwd_seq(const SeqBwdArgs& a, hipStream_t s);
// The same backward on 16-row row blocks x 32 units (gru_seq16.hip): 8 XCD-local row blocks at
// Bp = 128, half the streamed dGh per workgroup; H = 1024, no fused dW_hh.  Bias / dP partials are
// per 16-row block: dbhh_part / dbih_part [Bp/16][3H], dP_part [Bp/16][V][3H].
bool gru_bwd_seq16_supported(int H, int Bp, bool fuse_p);
void gru_bwd_seq16(const SeqBwdArgs& a, hipStream_t s);
// Persistent backward for large H with a large batch (gru_seq_big.hip): 64 tiles of 128 rows x 128
// units x 4 K-slices = 256 workgroups, dGh exchanged through the T-deep `xbuf` ([T][Bp][3H] bf16),
// split-K partials through `part`, epoch flags in cnt[0, 8192) (zeroed before the launch); writes
// dghT / dgiT (ldG >= T * Bp, column t * Bp + b) and the optional row-major dgi.  (H/128)(Bp/128) = 64.
bool gru_bwd_seq_big_supported(int H, int Bp);
long gru_bwd_seq_big_part_floats(int H, int Bp);
void gru_bwd_seq_big(const SeqBwdArgs& a, hipStream_t s);

// ------------------------------------------------------------------ FC + softmax
struct FcXentArgs {
  const u16* X = nullptr;          // [M][H] top-layer hidden states (bf16)
  const u16* W = nullptr;          // [V][H]
  const float* b = nullptr;        // [V]
  const int* labels = nullptr;     // [M], -1 = ignore
  const float* inv_count = nullptr;// device scalar 1 / #valid tokens
  u16* dl = nullptr;               // [M][V] bf16 dL/dlogits
  u16* dlT = nullptr;              // [V][ldT] at column colT + row
  float* loss_part = nullptr;      // [M/32] per-block partial (already scaled)
  // fused dH = dlogits · W_fc (nullable): dy [M][H] fp32 from WT = W_fc^T [H][V] bf16
  const u16* WT = nullptr;
  float* dy = nullptr;
  int M = 0, H = 0, V = 0, ldT = 0, colT = 0;
  // FT-layout copies of W [V][H] and W^T [H][V] (ft_offset): required by the 8-wave V = 256 kernel
  const u16* Wf = nullptr;
  const u16* WTf = nullptr;
  unsigned long long* dbg = nullptr;   // diagnostic phase stamps of workgroup 0 (nullable)
};
void fc_xent(const FcXentArgs& a, hipStream_t s);
// Softmax-xent over precomputed fp32 logits [M][V] (V % 64 == 0, V <= 512, M % 32 == 0): the large-H
// path, where the logits and dH are LDS GEMMs and only this row-wise part stays fused.  Writes dl
// (row-major, nullable), dlT (transposed) and the per-32-row loss partials like fc_xent.
void softmax_xent(const float* logits, const FcXentArgs& a, hipStream_t s);
// the 8-wave fused kernel covers this shape (else the trainer takes the GEMM + softmax_xent path)
bool fc_xent_fused_ok(int V, int H, int M);

struct FcSampleArgs {              // generation: logits -> softmax -> inverse-CDF sample
  const u16* X = nullptr;          // [Bp][H]
  const u16* W = nullptr;          // [V][H]
  const u16* Wf = nullptr;         // FT copy of W (nullable; V = 256, H in {512, 1024}: 8-wave kernel)
  const float* b = nullptr;        // [V]
  const float* rf = nullptr;       // [N][max_len] uniforms (global name index)
  int* ids = nullptr;              // [Bp] in: unused / out: sampled char (next input)
  unsigned char* out = nullptr;    // [N][max_len+1]
  int* alive = nullptr;            // [Bp]
  float* probs = nullptr;          // optional [Bp][V] softmax output (debug / tests)
  int N = 0, Bp = 0, H = 0, V = 0, step = 0, max_len = 0, eos = 0;
};
void fc_sample(const FcSampleArgs& a, hipStream_t s);

// ------------------------------------------------------------------ fp32-faithful generation (gen_f32.hip)
struct GemmF32Args {               // C[M][N] = A[M][K] · B[N][K]^T (+ bias[N]), fp32 MFMA
  const float* A = nullptr; int lda = 0;
  const float* B = nullptr; int ldb = 0;
  float* C = nullptr; int ldc = 0;
  const float* bias = nullptr;
  int M = 0, N = 0, K = 0;         // M, N % 64 == 0, K % 16 == 0
  int splits = 1;                  // split-K: slab s (K range s*K/splits ..) at C + s*slab; bias in slab 0
  long slab = 0;
};
void gemm_f32_nt(const GemmF32Args& g, hipStream_t s);
struct GruGatesF32Args {           // h' = GRU gates from gi (or P[ids]) and gh = h W_hh^T + b_hh
  const float* P = nullptr; const int* ids = nullptr;   // layer 0: gi row = P[ids[b]] ([V][3H])
  const float* Gi = nullptr;       // layers >= 1: [Bp][3H] (with b_ih)
  const float* Gh = nullptr;       // [Bp][3H] (with b_hh)
  int gi_splits = 1, gh_splits = 1;   // split-K slabs of Gi / Gh, summed here in fixed order
  long gi_slab = 0, gh_slab = 0;
  const float* hprev = nullptr; float* hout = nullptr;   // [Bp][H]
  int Bp = 0, H = 0, V = 0;
  unsigned* err = nullptr;         // layer 0: bit 4 set (and the row clamped) on a char id outside [0, V)
  // bf16x3 mode: biases not folded into split-K slabs (nullable), and the bf16 split copy of h'
  // written as the next products' A operand: hsplit[b] = [hi | hi | lo] of h'[b] ([Bp][3H])
  const float* bgh = nullptr; const float* bgi = nullptr;
  unsigned short* hsplit = nullptr;
};
void gru_gates_f32(const GruGatesF32Args& a, hipStream_t s);
struct SampleF32Args {             // softmax of fp32 logits + inverse-CDF sample (same I/O as fc_sample)
  const float* logits = nullptr;   // [Bp][V]
  int splits = 1; long slab = 0;   // split-K slabs of the logits, summed in fixed order
  const float* rf = nullptr;
  int* ids = nullptr; unsigned char* out = nullptr; int* alive = nullptr;
  float* probs = nullptr;
  int N = 0, V = 0, step = 0, max_len = 0, eos = 0;
  const float* bias = nullptr;     // nullable: added after the slab sum (bf16x3 split-K logits)
};
void sample_f32(const SampleF32Args& a, hipStream_t s);
// bf16x3 operands: an fp32 value x = hi + lo with hi = bf16(x), lo = bf16(x - hi).  Weights become
// [R][3K] = [hi | lo | hi] rows and activations [hi | hi | lo] rows, so ONE bf16 MFMA GEMM over 3K
// accumulates hi*hi + hi*lo + lo*hi in fp32 (the lo*lo term, ~2^-16 relative, is dropped).
void split_bf16x3(const float* src, int R, int K, unsigned short* dst, hipStream_t s);
// per-batch generation reset as ONE kernel node (instead of memset nodes): h slot 0 of every layer
// (fp32 and, if given, bf16) = 0, ids = sos, alive = 1, output rows = NUL
struct GenResetArgs {
  float* hf[4] = {nullptr, nullptr, nullptr, nullptr};
  unsigned short* hb[4] = {nullptr, nullptr, nullptr, nullptr};
  int hb_cols = 0;                 // columns of hb rows: H (bf16 copy) or 3H (bf16x3 split copy); 0 = H
  int* ids = nullptr; int* alive = nullptr; unsigned char* out = nullptr;
  int L = 0, Bp = 0, H = 0, ML = 0, sos = 0;
};
void gen_reset(const GenResetArgs& a, hipStream_t s);
// Persistent fp32 generation for small batches (gen_persist.hip): ONE launch runs every char of up to
// 64 names with the fp32 recurrent weights resident in VGPRs across 256 workgroups (exchange
// buffers in `ws`).
struct GenPersistArgs {
  const float* Whh[4] = {}; const float* Wih[4] = {};   // [3H][H] (Wih[0] unused: folded into P)
  const float* bhh[4] = {}; const float* bih[4] = {};   // [3H]
  const float* Wfc = nullptr; const float* bfc = nullptr;   // [V][H], [V]
  const float* P = nullptr;        // [V][3H] layer-0 table Emb W_ih0^T + b_ih0
  const float* rf = nullptr;       // [N][ML] uniforms
  unsigned char* out = nullptr;    // [N][ML + 1]
  float* probs = nullptr;          // nullable [Npad][V]: softmax of the last step (tests)
  float* ws = nullptr;             // gen_persist_ws_floats(): two exchange-buffer sets (launch parity)
  int par = 0;                     // this launch's set; it refills the other set's tagged slots
  unsigned* sync = nullptr;        // gen_persist_sync_words(): epoch flags + arrival count (zeroed once, self-cleaning)
  unsigned* err = nullptr;         // bit 32: a cross-workgroup wait hit its spin limit
  unsigned long long* dbg = nullptr;   // diagnostic (nullable): [2 wgs][ML + 1][16] s_memrealtime stamps
  int N = 0, H = 0, L = 0, V = 0, ML = 0, sos = 0, eos = 0;
};
bool gen_persist_supported(int H, int L, int V, int N, int ML);
long gen_persist_ws_floats(int H, int L, int V, int ML);
void gen_persist_fill_ws(float* ws, int H, int L, int V, int ML, hipStream_t s);   // both sets -> kEmpty
long gen_persist_sync_words(int L);
void gen_persist_f32(const GenPersistArgs& a, hipStream_t s);

// ------------------------------------------------------------------ generic GEMM
// C[M][N] (+)= A[M][K] · B[N][K]^T  (bf16 in, fp32 accumulate), both operands K-contiguous.
struct GemmArgs {
  const u16* A = nullptr; int lda = 0;
  const int* onehot_ids = nullptr; // if set, A[m][k] = (ids[k] == m) generated on the fly
  const u16* B = nullptr; int ldb = 0;
  float* C = nullptr; int ldc = 0;
  const float* bias = nullptr;     // [N] added in the epilogue (non-split only)
  float* rowsumA = nullptr;        // [splits][M] partial row sums of A (nullable)
  int M = 0, N = 0, K = 0;
  int splits = 1;                  // split-K: slab s written at C + s*M*ldc (ldc == N)
  int accumulate = 0;              // C += result instead of C = result
  // B rows >= b2_row are read from B2 (same row indexing; one-hot LDS kernel only, b2_row % 128 == 0):
  // layer 0's dP reads the r/z gate rows of dGi^T from dGh^T, where they are identical
  const u16* B2 = nullptr; int b2_row = 0;
  int raster = 0;                  // LDS 128x128 kernel tile order: 0 auto (shorter dimension fast), 1 column-fast
  // gemm_small / gemm_small_group only: A taken from an fp32 matrix, rounded to bf16 while staging
  // (no separate cast pass): A[m][k] = A32[m * lda + k], or with a32_trans A32[k * lda + m]
  const float* A32 = nullptr; int a32_trans = 0;
  int algo = 0;                    // 0 auto, 1 register-direct 64x64 tiles, 2 LDS-staged 128x128,
                                   // 3 one-shot 64x64 (gemm_small), 4 hipBLASLt (+ row-sum kernel),
                                   // 5 LDS-staged 256x256 (gemm256.hip)
};
// algo 0 sends plain (no one-hot, no bias, unsplit) products of >= blaslt_min_gflop() to hipBLASLt
bool gemm_library_ok(const GemmArgs& a);
bool gemm_library_wanted(const GemmArgs& a);
// the product on hipBLASLt (+ the row-sum pass when rowsumA): false, with nothing launched, when the
// library has no algorithm for the shape
bool gemm_library(const GemmArgs& a, hipStream_t s);
void gemm_nt(const GemmArgs& a, hipStream_t s);
bool gemm_lds_ok(const GemmArgs& a);
// dP = onehot(ids)^T · G^T with V = 256 (onehot.hip): G streamed once, all-zero one-hot tiles skipped
bool onehot_dp_ok(const GemmArgs& a);
int onehot_dp_splits(int N, int K);   // its K-slice count for an N-column product (about 384 workgroups)
void onehot_dp(const GemmArgs& a, hipStream_t s);
bool gemm256_ok(const GemmArgs& a);
// rows of A per gemm256 tile for (M, N, splits): 256 or 192 (the phased kernel), 0 = no fit
int gemm256_tile_rows(int M, int N, int K, int splits);
void gemm256(const GemmArgs& a, hipStream_t s);
// out[m] = sum_k A[m][k] (bf16 A, fp32 sums; the bias gradient beside a GEMM without row sums)
void rowsum_bf16(const u16* A, int lda, int M, int K, float* out, hipStream_t s);
// several independent LDS-GEMM problems in ONE launch (fills the chip with small products);
// all jobs gemm_lds_ok, with the same bias / row-sum flags; n <= 4
void gemm_lds_group(const GemmArgs* jobs, int n, hipStream_t s);
void gemm_lds(const GemmArgs& a, hipStream_t s);
// one-shot 64 x 64 small GEMM (gemm_small.hip): the whole K-slice (128, 192, 256 or 512 deep) staged
// at once; for the latency-bound small products.  kblocks = 64-deep blocks per K-slice, 0 = unsupported
int gemm_small_kblocks(const GemmArgs& a);
void gemm_small(const GemmArgs& a, hipStream_t s);
// up to 4 independent small GEMMs in one launch: the jobs' K-slices must be multiples of one chunk
// depth (gemm_small_group_depth != 0; longer slices stream as several chunks), same bias mode
int gemm_small_group_depth(const GemmArgs* jobs, int n);
void gemm_small_group(const GemmArgs* jobs, int n, hipStream_t s);

// sum `splits` slabs [splits][n] -> dst[n] (optionally also as bf16 and/or accumulate)
void reduce_slabs(const float* src, int splits, long n, float* dst, hipStream_t s);

// out = bf16 of in [R][C] (row-major) and/or its transpose [C][R]
void cast_bf16(const float* in, long n, u16* out, hipStream_t s);
void transpose_bf16(const float* in, int R, int C, u16* outT, hipStream_t s);
// column sums of a [R][C] fp32 matrix -> out[C]
void colsum(const float* in, int R, int C, float* out, hipStream_t s);

// ------------------------------------------------------------------ optimiser / misc
struct OptimArgs {
  float* p = nullptr; const float* g = nullptr; float* m = nullptr; float* v = nullptr;
  long n = 0;
  int* step = nullptr;             // device step counter (graph-replay safe), incremented by caller kernel
  const float* gscale = nullptr;   // device scalar gradient scale (clip); nullable = 1
  // step error word (cross-workgroup spin limit in the persistent / split-K kernels): when set,
  // the update is skipped (no garbage gradient reaches the weights) and the word is mirrored to
  // host-mapped memory (err_host) where the host watchdog sees it without a device sync
  const unsigned* err = nullptr;
  unsigned* err_host = nullptr;
  float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.f;
  int sgd = 0;
  // learning-rate schedule, evaluated on the device from the step counter (graph-replay safe):
  // linear warm-up over `warmup` steps, then 0 = constant, 1 = cosine, 2 = linear decay to lr_min
  // at step `total` (models/cpu_ref.py lr_at is the host twin)
  int sched = 0, warmup = 0, total = 0;
  float lr_min = 0.f;
  // 1: a gradient summed from slabs (OptCastJob::gsl) is also written to g (observable); 0: it stays
  // in registers (the one-graph step without GRUConfig.keep_grads)
  int keep_g = 1;
};
void adam_step(const OptimArgs& a, hipStream_t s);
void bump_step(int* step, hipStream_t s);
// sum of squares of x[n] -> partials; finalize computes clip scale = min(1, clip/(sqrt(sum)+1e-6))
void sumsq_partials(const float* x, long n, float* partials, int nparts, hipStream_t s);
void clip_scale_finalize(const float* partials, int nparts, float clip, float* scale, hipStream_t s);
// deterministic sum of partials -> out[0]; optionally also ++(*bump) (the optimiser step counter)
void sum_partials(const float* partials, int n, float* out, hipStream_t s, int* bump = nullptr);

// multi-tensor launches (one kernel for the whole list)
// job: dst = sum of `splits` consecutive slabs of n floats.  Cast jobs (bf and/or bfT set) see the
// slab as [R][C] (R, C multiples of 64) and also write bf16 [R][C] / bf16 [C][R] (dst nullable).
// `bump` (nullable): the launch also increments the device step counter once.
struct SlabJob { const float* src; float* dst; long n; int splits; u16* bf; u16* bfT; int R, C; };
struct SlabJobs { SlabJob job[24]; int blk_start[25]; int n = 0; int* bump = nullptr;
  void add(const float* s, int splits, long n_, float* d) {
    job[n++] = SlabJob{s, d, n_, splits, nullptr, nullptr, 0, 0}; }
  void add_cast(const float* s, int splits, int R, int C, float* d, u16* bf, u16* bfT) {
    job[n++] = SlabJob{s, d, (long)R * C, splits, bf, bfT, R, C}; } };
void reduce_slabs_multi(SlabJobs& j, hipStream_t s);
int reduce_slabs_blocks(SlabJobs& j);   // fills j.blk_start, returns the launch's block count
// "FT" (fragment-tiled) bf16 layout of a K-contiguous [R][K] matrix: element (r, k) at
//   ((r/16 * K/32 + k/32) * 64 + (r%16) + 16*((k%32)/8)) * 8 + k%8
// i.e. every 16x32 MFMA operand fragment is 1 KB contiguous in lane order, so a fragment load is
// 8 whole 128-B lines instead of 16 rows x 64-B pieces (per-CU load throughput is bound by line
// requests: profiles/r1_fc_xent_notes).  ft_offset() gives the element index.
DEV_HOST_INLINE long ft_offset(int r, int k, int K) {
  return ((long)((r >> 4) * (K >> 5) + (k >> 5)) * 64 + (r & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
}
// src16 (instead of src): a bf16 source -- the layouts re-derived from gathered bf16 working copies
// (sharded optimiser, Trainer::record_sharded_opt mode 2); bf16 -> fp32 -> bf16 is exact
struct CastJob { const float* src; u16* dst; u16* dstT; int R, C; u16* dstF = nullptr; u16* dstTF = nullptr;
                 const u16* src16 = nullptr; };
struct CastJobs { CastJob job[24]; int blk_start[25]; int n = 0;
  void add(const float* s, int R, int C, u16* d, u16* dT, u16* dF = nullptr, u16* dTF = nullptr) {
    job[n++] = CastJob{s, d, dT, R, C, dF, dTF}; }
  void add16(const u16* s, int R, int C, u16* d, u16* dT, u16* dF = nullptr, u16* dTF = nullptr) {
    job[n++] = CastJob{nullptr, d, dT, R, C, dF, dTF, s}; } };
void cast_multi(CastJobs& j, hipStream_t s);
// Fused optimiser + weight refresh, one launch over every parameter tensor: Adam/SGD on the fp32
// master slice [off, off+R*C) of the flat buffers, then (matrix jobs) its bf16 copy and/or bf16
// transpose.  Matrix jobs need R % 64 == 0 and C % 64 == 0; R == 0 marks a flat (bias) job of C
// elements, C % 4 == 0.
// dstF / dstTF (nullable): FT-layout copies of the matrix / its transpose (see ft_offset)
// Flat job with dst: the updated values' bf16 also go to dst[i - off] (the flat bf16 working copy of
// the sharded optimiser's mode 2)
// gsl (nullable): the job's gradient is the fixed-order sum of nsl slabs gsl[s * R*C + i] (split-K /
// per-row-block partials), summed here instead of by a separate reduce launch; the sum is also
// written to the gradient buffer (it stays observable).
struct OptCastJob { long off; int R, C; u16* dst; u16* dstT; u16* dstF = nullptr; u16* dstTF = nullptr;
                    const float* gsl = nullptr; int nsl = 0; };
struct OptCastJobs { OptCastJob job[32]; int blk_start[33]; int n = 0;
  void add(long off, int R, int C, u16* d, u16* dT, u16* dF = nullptr, u16* dTF = nullptr) {
    job[n++] = OptCastJob{off, R, C, d, dT, dF, dTF}; } };
void adam_cast_multi(const OptimArgs& a, OptCastJobs& j, hipStream_t s);

void fill_f32(float* p, long n, float v, hipStream_t s);
// Exact exchange of the fp32 entries of up to 16 flat ranges (the biases, which kernels read in fp32)
// between ranks of a sharded optimiser: pack (unpack = 0): pack[k] = bits of p[f] if f is in the
// owned chunk [lo, hi), else 0; unpack (1): p[f] = bits of pack[k] for f < tail (the replicated tail,
// updated identically on every rank, is left alone).  k enumerates the ranges in order.
struct FlatRanges { long off[16]; int n[16]; int cnt = 0; __host__ __device__ long total() const { long t = 0; for (int i = 0; i < cnt; ++i) t += n[i]; return t; } };
void flat_pack_u32(float* p, unsigned* pack, const FlatRanges& r, long lo, long hi, long tail, int unpack, hipStream_t s);
// placement census: out[b] = HW_REG_XCC_ID of the CU that ran block b
void xcc_census(unsigned* out, int nblocks, int threads, hipStream_t s);
// fault injection for watchdog tests: one wave busy-waits `us` microseconds (capped at 5 s)
void spin_delay(int us, hipStream_t s);
// graph-replay probe: a memset (mode 0), memcpy (1), 2-D memcpy (2), 32-bit pattern memset (3), five
// memset nodes in a row (4) or an odd-sized byte memset (5) captured before a checking kernel on one stream, replayed `reps` times (host sync every `sync_every` replays, 0 = never);
// returns how many words the kernel found not yet written by the node, summed over the replays
long graph_node_probe(long words, int reps, int sync_every, int mode);
std::vector<long> graph_node_probe_detail();
// fault injection: nblocks blocks each holding a whole CU's LDS for `us` microseconds (capped at 5 s)
void block_cus(int nblocks, int us, hipStream_t s);

// Batch preparation on device: in = [hdr 16 ints: B, float-bits of 1/#valid][x Bmax*T][y Bmax*T]
// batch-major int32 (may be pinned host memory, read zero-copy); out ids/labels time-major [T][Bp]
// (pad rows: id 0, label -1) and inv_count.
void prep_batch(const int* in, int Bmax, int T, int Bp, int* ids, int* labels, float* inv_count, hipStream_t s);
inline int prep_batch_blocks(int T, int Bp) {
  const int n = (T * Bp + 255) / 256;
  return n < 64 ? n : 64;
}
// The layer-0 P-table GEMM (P = Emb·W_ih0^T + b_ih0, only V/128 x 3H/128 tiles) and the batch
// preparation in ONE launch: the transpose's latency-bound zero-copy reads of the pinned slot run
// on blocks beside the GEMM tiles instead of as a kernel of their own (a forked graph branch for
// it measured +95 us per step: profiles/r1_sched_fork_fence_ab.jsonl).  Falls back to two launches
// when the GEMM shape is not LDS-kernel compatible.
void gemm_with_prep(const GemmArgs& g, const PrepJob& p, hipStream_t s);
void gemm_small_with_prep(const GemmArgs& g, const PrepJob& p, hipStream_t s);

}  // namespace gk
