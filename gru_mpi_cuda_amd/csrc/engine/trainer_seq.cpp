// Single-stream training step built around the persistent sequence kernels (gru_seq.hip):
//
//   P-table GEMM -> [per layer: Gi GEMM (l>0) -> forward sequence kernel]
//   -> fused FC + softmax-xent over all B*T tokens -> dH GEMM -> dW_fc split-K GEMM
//   -> [per layer, top-down: backward sequence kernel with fused dW_hh / dP / bias partials
//       -> (l>0) dW_ih GEMM + dX GEMM]
//   -> one multi-tensor reduction of all partial slabs (+ loss) -> dW_ih0 / dEmb GEMMs (single GPU:
//      with the dW_fc K-slices in the same launch).
//
// Every layer falls back to the per-timestep kernels when its shape cannot be made
// co-resident (gru_*_seq_supported), so any config still runs -- just slower.
#include "trainer.h"
#include <algorithm>
#include <string>

namespace gk {

// data-parallel: a layer group's collective stays open across the next persistent backward kernel
// (span mode; joining it before that kernel measured the same at one rank, docs/DESIGN.md §6.2)
static bool ar_span() { return true; }

// Weight-gradient product engine choice: "256" the 256 x 256 LDS kernel (gemm256.hip) with a
// split-K depth picked for whole waves of workgroups, "lib" hipBLASLt for the products with >= 8 M
// outputs and >= 60 GFLOP (dW_hh at H = 2048: one unsplit library GEMM), "128" the 128 x 128 split-K
// path only; default (0) "auto" = gemm256 everywhere.  Round 4 sent dW_hh at H = 2048 to the library
// by default (1.37 vs 1.12 PF); the staggered phased gemm256p takes that product unsplit on 192-row
// tiles at 1.35-1.38 PF against the library's 1.33-1.42 on the same boxes, and the h2048 step runs
// 8.62-8.64 ms against 8.62 with the library (profiles/r5_s24_gemm.jsonl, r5_s24_benches.jsonl), so
// no library kernel is on the default path.
static int wgrad_engine() {   // read at record time (tests switch it per trainer)
  const char* v = std::getenv("GK_WGRAD_GEMM");
  if (!v || !*v) return 0;
  if (std::string(v) == "lib") return 1;
  if (std::string(v) == "128") return 128;
  return 256;
}

// split-K depth for gemm256: the one that fills whole waves of 256 workgroups best with the tile
// gemm256 picks for it (256 or 192 rows, gemm256_tile_rows; ties: the shallower, fewer slabs),
// K-slices at least 2048 deep
static int gemm256_splits(int M, int N, int K) {
  int best = 0;
  double best_fill = 0.0;
  for (int sp = 1; sp <= 8; sp *= 2) {
    if (K % sp || (K / sp) % 64 || (sp > 1 && K / sp < 2048)) continue;
    const int bm = gemm256_tile_rows(M, N, K, sp);
    if (!bm) continue;
    const int wg = (M / bm) * (N / 256) * sp, rounds = (wg + 255) / 256;
    const double fill = (double)wg / (rounds * 256);
    if (fill > best_fill + 1e-9) { best_fill = fill; best = sp; }
  }
  return best_fill >= 0.7 ? best : 0;
}

void Trainer::wgrad_gemm(const u16* A, int lda, const u16* Bm, int ldb, int M, int N, int K, float* dst,
                         float* rowsum_dst, hipStream_t s) {
  const int eng = wgrad_engine();
  if (eng == 1 && wgrad_prefers_library(M, N, K)) {
    GemmArgs w;   // one unsplit library GEMM straight into the gradient (+ a row-sum pass for the bias)
    w.A = A; w.lda = lda; w.B = Bm; w.ldb = ldb; w.C = dst; w.ldc = N; w.rowsumA = rowsum_dst;
    w.M = M; w.N = N; w.K = K;
    if (gemm_library(w, s)) return;
  }
  if (eng == 256 || eng == 0) {
    GemmArgs w;
    w.A = A; w.lda = lda; w.B = Bm; w.ldb = ldb; w.M = M; w.N = N; w.K = K;
    const int sp = gemm256_splits(M, N, K);
    w.splits = std::max(sp, 1);
    w.C = sp == 1 ? dst : slab_w_; w.ldc = N;
    if (rowsum_dst) w.rowsumA = sp == 1 ? rowsum_dst : rs_w_;   // bias gradient fused (row sums of A)
    if (sp && sp <= splits_ && gemm256_ok(w)) {
      // (slabs of their own summed inside the Adam launch instead of this reduce measured equal in the
      // config-4 shard: the three 11-us reduces gone, Adam 75 -> 103 us, step 1.3139 vs 1.3132 ms in
      // the trace, profiles/r6_c4_wgrad_defer_step_summary.txt; not kept)
      w.algo = 5;
      gemm_nt(w, s);
      if (sp > 1) {
        SlabJobs j;
        j.add(slab_w_, sp, (long)M * N, dst);
        if (rowsum_dst) j.add(rs_w_, sp, M, rowsum_dst);
        reduce_slabs_multi(j, s);
      }
      return;
    }
  }
  // split K only as deep as it takes to give the chip ~256 workgroups: every extra split costs a
  // full M x N fp32 slab written and read again (8 slabs of dW_hh at H=1024 = 100 MB).  With no
  // split the GEMM writes the gradient (and the bias row sums) directly.
  {
    // large products (H >= 2048 over B*T tokens): one unsplit hipBLASLt GEMM straight into the
    // gradient (+ a row-sum kernel for the bias) -- no slabs to write and reduce
    GemmArgs w;
    w.A = A; w.lda = lda; w.B = Bm; w.ldb = ldb; w.C = dst; w.ldc = N; w.rowsumA = rowsum_dst;
    w.M = M; w.N = N; w.K = K;
    if (wgrad_engine() != 128 && gemm_library_wanted(w) && gemm_library_ok(w)) {
      gemm_nt(w, s);
      return;
    }
  }
  const int tiles = std::max(1, (M / 128) * (N / 128));
  auto can_split = [&](int s2) { return s2 <= splits_ && K % s2 == 0 && (K / s2) % 128 == 0; };
  int sp = 1;
  while (can_split(sp * 2) && tiles * sp < 256) sp *= 2;
  // a ragged last round of workgroups (two resident per CU: 512 slots) idles part of the chip for a
  // whole K-slice; one more split evens it out (H = 2048: 768 tiles -> 1536 = 3 full rounds)
  const int slots = 512, wg = tiles * sp;
  if (wg > slots && wg % slots && (double)wg / slots / ((wg + slots - 1) / slots) < 0.85 && can_split(sp * 2)) sp *= 2;
  GemmArgs w;
  w.A = A; w.lda = lda; w.B = Bm; w.ldb = ldb;
  w.M = M; w.N = N; w.K = K; w.splits = sp;
  if (sp == 1 && gemm_lds_ok(w)) {
    w.C = dst; w.ldc = N; w.rowsumA = rowsum_dst;
    gemm_nt(w, s);
    return;
  }
  w.C = slab_w_; w.ldc = N; w.rowsumA = rowsum_dst ? rs_w_ : nullptr;
  gemm_nt(w, s);
  SlabJobs j;
  j.add(slab_w_, sp, (long)M * N, dst);
  if (rowsum_dst) j.add(rs_w_, sp, M, rowsum_dst);
  reduce_slabs_multi(j, s);
}

void Trainer::slab_job(SlabJobs& j, const float* src, int splits, long n, float* dst) {
  // deep split-K slabs (32) stay with the reduce kernel: summed inside the Adam launch they serialise
  // 32 loads per element on its few tile blocks (16: two batches of 8 in flight)
  constexpr int max_splits = 16;
  SlabJobs& t = (defer_slabs_ && splits <= max_splits) ? deferred_ : j;
  if (t.n >= 24) throw std::runtime_error("slab job list full");
  t.add(src, splits, n, dst);
}

void Trainer::record_fb_seq(hipStream_t s, bool dp) {
  const int V = d_.V, E = d_.E, H = d_.H, T = d_.T, L = d_.L, B = Bp_;
  const int H3 = 3 * H;
  const long tok = (long)T * B;
  const long fw = seq_flag_words(H, B);
  ev_next_ = 0;
  fc_held_on_ = false;
  if (dp) { ar_ready_ = ar_launched_ = 0; ar_busy_ = false; ar_log_.clear(); }
  dp_tail_rec_ = false;
  // Flag blocks: forward(l) at cnt_ + l*fw, backward(l) at cnt_ + (L+l)*fw.  Each persistent
  // kernel zeroes the block of the kernel that follows it (forward(l) -> backward(l) ->
  // next step's forward(l)), so no memset node is needed; a block whose partner runs per-step
  // is zeroed by a memset instead.  The arena starts zeroed for the first step.
  nloss_ = (int)(tok / 32);
  {
    // layer-0 input projection folded into a [V][3H] table: Gi(t,b) = P[x(t,b)], launched together
    // with the batch preparation (independent work, one graph node)
    GemmArgs g;
    g.A = Emb; g.lda = E; g.B = Ls_[0].Wih; g.ldb = E; g.C = Ptab_; g.ldc = H3;
    g.bias = P("bias_ih_l0"); g.M = V; g.N = H3; g.K = E;
    gemm_with_prep(g, PrepJob{stage_src_, Bp_, T, Bp_, ids_, labels_, inv_count_}, s);
  }
  if (carry_) record_carry(s);
  // ------------------------------------------------------------------ forward
  auto fwd_args = [&](int l) {
    Layer& y = Ls_[l];
    SeqFwdArgs a;
    a.HSb = y.HSb; a.HSf = y.HSf; a.HT = y.HT; a.ldT = (T + 1) * B; a.HF = seq_[l].HF;
    a.xch = xbuf_;   // shared with the backward exchange: the kernels never overlap
    if (y.s16) a.s16 = y.s16;   // (SeqPlan::s16)
    else { a.sr = y.sr; a.sz = y.sz; a.sn = y.sn; a.sghn = y.sghn; }
    a.Whh = y.Whh; a.bhh = P("bias_hh_l" + std::to_string(l));
    if (l == 0) { a.P = Ptab_; a.ids = ids_; }
    else a.Gi = y.Gi;
    a.cnt = cnt_ + (size_t)l * fw; a.err = err_; a.allow_local = xcd_local_;
    a.xring = step_lds_variants().fwd_xring;
    if (seq_[l].bwd) { a.zero_next = cnt_ + (size_t)(L + l) * fw; a.zero_words = fw; }
    a.T = T; a.Bp = B; a.H = H;
    if (carry_) a.h0 = y.HSf;   // carried state: HS[0] (bf16 copy read as the first MFMA operand)
    // (zeroed by a kernel node, not a memset node: memset nodes misbehaved on graph replay in
    // the generator, see Generator::reset_batch)
    if (!seq_[l].bwd) fill_f32(reinterpret_cast<float*>(a.cnt), fw, 0.f, s);
    return a;
  };
  for (int l = 0; l < L; ++l) {
    Layer& y = Ls_[l];
    if (l > 0) {
      GemmArgs g;   // hoisted input projection over all B*T tokens
      g.A = Ls_[l - 1].HSb + (size_t)B * H; g.lda = H; g.B = y.Wih; g.ldb = H;
      g.C = y.Gi; g.ldc = H3; g.bias = P("bias_ih_l" + std::to_string(l));
      g.M = (int)tok; g.N = H3; g.K = H;
      gemm_nt(g, s);
    }
    if (persist_fwd_ && fwd_wave_ && l + 1 < L) {
      // layers l and l+1 as one wavefront launch: l+1's input projection runs inside it
      SeqFwd2Args w2;
      w2.lo = fwd_args(l);
      w2.hi = fwd_args(l + 1);
      w2.hi.Gi = nullptr;
      w2.hi.xch = xbuf_ + (size_t)T * B * H;   // xbuf_ holds 3 layers' worth of exchange tiles
      w2.lo.xring = w2.hi.xring = 0;   // (a ring measured equal here: profiles/r4_fwd_xring_ab.jsonl)
      w2.Wih = Ls_[l + 1].Wih; w2.bih = P("bias_ih_l" + std::to_string(l + 1));
      gru_fwd_seq2(w2, s);
      ++l;
    } else if (persist_fwd_ && fc_in_fwd_) {
      // the FC head's consumer workgroups in the same launch (fc_xent + dW_fc K-slices' work)
      SeqFwdArgs a = fwd_args(l);
      a.HT = nullptr;   // its only reader at L = 1 was the dW_fc GEMM
      SeqFcArgs f;
      f.Wf = WfcF; f.WTf = WfcTF; f.b = P("fc.bias"); f.labels = labels_; f.inv_count = inv_count_;
      f.dy = y.dy; f.dlF = dlT_; f.loss_part = loss_part_; f.dW = slab_fc2_; f.db = rs_fc2_; f.V = V;
      gru_fwd_seq_fc(a, f, s);
    } else if (persist_fwd_) {
      gru_fwd_seq(fwd_args(l), s);
    } else {
      for (int t = 0; t < T; ++t) fwd_step(l, t, s);
    }
  }
  // ------------------------------------------------------------------ FC + loss + dH
  Layer& top = Ls_[L - 1];
  SlabJobs tail;   // reductions deferred to the last multi-tensor reduce (layer 0's)
  if (fc_in_fwd_) {
    // done inside the forward launch: loss partials, dy, and one dW_fc / db_fc partial per row block
    tail.add(slab_fc2_, B / 32, (long)V * H, G("fc.weight"));
    tail.add(rs_fc2_, B / 32, V, G("fc.bias"));
  } else {
    FcXentArgs f;
    f.X = top.HSb + (size_t)B * H; f.W = Wfc; f.b = P("fc.bias");
    f.labels = labels_; f.inv_count = inv_count_;
    f.dl = dl_; f.dlT = dlT_; f.ldT = (int)ldG_; f.colT = 0;
    f.loss_part = loss_part_; f.M = (int)tok; f.H = H; f.V = V;
    if (fc_split_) {
      // large H: logits and dH as LDS GEMMs around a row-wise softmax-xent (the fused FC kernel
      // stages a 32 x H tile of X per workgroup; at H = 2048 that leaves it at ~0.2 PF)
      GemmArgs lg;   // logits = X · W_fc^T + b_fc
      lg.A = f.X; lg.lda = H; lg.B = Wfc; lg.ldb = H; lg.C = logits_; lg.ldc = V; lg.bias = f.b;
      lg.M = (int)tok; lg.N = V; lg.K = H;
      gemm_nt(lg, s);
      softmax_xent(logits_, f, s);
      if (!dy_in_bwd_) {   // (else the top layer's large-H backward forms dy from dl itself)
        GemmArgs g;   // dy_top = dlogits · W_fc
        g.A = dl_; g.lda = V; g.B = WfcT; g.ldb = V; g.C = top.dy; g.ldc = H;
        g.M = (int)tok; g.N = H; g.K = V;
        gemm_nt(g, s);
      }
    } else if (V % 128 == 0 && H % (16 * (V / 64)) == 0) {
      // dy_top = dlogits · W_fc fused into the softmax-xent kernel (dlogits never leave LDS)
      f.dl = nullptr; f.WT = WfcT; f.dy = top.dy; f.Wf = WfcF; f.WTf = WfcTF;
      fc_xent(f, s);
    } else {
      fc_xent(f, s);
      GemmArgs g;   // dy_top = dlogits · W_fc
      g.A = dl_; g.lda = V; g.B = WfcT; g.ldb = V; g.C = top.dy; g.ldc = H;
      g.M = (int)tok; g.N = H; g.K = V;
      gemm_nt(g, s);
    }
    // dW_fc = dlogits^T · H_top, db_fc = row sums of dlogits^T: split-K into dedicated slabs whose
    // reduce joins the multi-tensor reduce after the backward sweep (one launch fewer)
    // few output tiles (V x H): split K until ~256 workgroups fill the chip
    const int tiles = std::max(1, (V / 128) * (H / 128));
    int sp = 1;
    while (sp * 2 <= kFcSplitsMax && tiles * sp < 256 && tok % (sp * 2) == 0 && (tok / (sp * 2)) % 128 == 0)
      sp *= 2;
    // ... and at deep K (>= 4096 per slice after that) one more, for a whole round at two per CU (h2048,
    // 2 x 16 tiles over 65536 tokens: 8 / 16 / 32 / 64 K-slices 138 / 107 / 122 / 129 us standalone,
    // profiles/r6_gemm_dwfc.jsonl)
    if (sp * 2 <= kFcSplitsMax && tiles * sp < 512 && tok % (sp * 2) == 0 && tok / (sp * 2) >= 4096) sp *= 2;
    GemmArgs w;
    w.A = dlT_; w.lda = (int)ldG_; w.B = top.HT + B; w.ldb = (T + 1) * B;
    w.C = slab_fc2_; w.ldc = H; w.rowsumA = rs_fc2_;
    w.M = V; w.N = H; w.K = (int)tok; w.splits = sp;
    // one-shot small GEMM over 512-deep K-slices when that fits the slab budget: one memory
    // latency per workgroup and half the slabs of the 32-way 128 x 128 split
    // 1024: 8 slabs, summed inside the Adam launch (0.2362 -> 0.2338 ms at h512,
    // profiles/r1_fc_kslice_ab.jsonl; 512 measured equal to 128x128 split-K, r1_small_gemm_ab.jsonl)
    // (only while its 64 x 64 tiles x K-slices fit one round at one workgroup per CU: at H = 1024 the
    // 512 workgroups took 22.4 us in the config-4 shard, the 128^2 kernel 14.5 at 16 K-slices standalone,
    // profiles/r6_gemm_c4_shapes.jsonl)
    constexpr int kslice = 1024;
    if (kslice > 0 && tok % kslice == 0 && tok / kslice <= kFcSplitsMax && (V / 64) * (H / 64) * (tok / kslice) <= 256) {
      GemmArgs ws = w;
      ws.splits = (int)(tok / kslice); ws.algo = 3;
      if (gemm_small_kblocks(ws)) { w = ws; sp = ws.splits; }
    }
    // (gemm256 on 2048-deep K-slices at h2048 -- 8 tiles x 32 splits -- measured equal: the GEMM
    // 194 -> 173 us, its 32 slabs given back in the reduce; profiles/r4_h2048_dwfc256_ab.jsonl.  Again
    // with the staggered gemm256p in round 5: 192 -> 163 us, the reduce 14 -> 27 us, step 8.92 / 8.91
    // vs 8.93 / 8.90 ms; profiles/r5_dwfc256_ab.jsonl)
    // single GPU, slabs summed inside Adam: nothing reads dW_fc before the optimiser, so its
    // K-slices can join the dW_ih0 / dEmb launch after the backward sweep (one launch fewer; its
    // latency-bound tiles run beside theirs)
    // pipelined data-parallel tail (dp_pipe_on): the K-slices run after the backward too, beside the
    // first collective (record_dp_tail_l1)
    fc_held_on_ = (dp && dp_pipe_on()) ||
                  (!dp && defer_slabs_ && sp <= 8 && w.algo == 3 && step_lds_variants().dwfc_group);
    if (fc_held_on_) fc_held_ = w;
    else gemm_nt(w, s);
    tail.add(slab_fc2_, sp, (long)V * H, G("fc.weight"));
    tail.add(rs_fc2_, sp, V, G("fc.bias"));
  }
  // ------------------------------------------------------------------ backward (BPTT)
  for (int l = L - 1; l >= 0; --l) {
    Layer& y = Ls_[l];
    const SeqPlan& q = seq_[l];
    const std::string k = std::to_string(l);
    if (q.bwd) {
      SeqBwdArgs a;
      a.dy = y.dy;
      if (q.s16) a.s16 = y.s16;   // (SeqPlan::s16)
      else { a.sr = y.sr; a.sz = y.sz; a.sn = y.sn; a.sghn = y.sghn; }
      a.HSf = y.HSf; a.HT = y.HT; a.ldT = (T + 1) * B; a.HF = q.HF; a.WhhT = y.WhhT; a.xbuf = xbuf_;
      const bool need_T = !q.fuse_w || (l == 0 ? !q.fuse_p : true);
      a.dghT = need_T ? y.dghT : nullptr; a.dgiT = need_T ? y.dgiT : nullptr; a.ldG = (int)ldG_;
      a.dgi = y.dgi;
      a.dWhh_part = q.dWhh_part; a.dbhh_part = q.dbhh_part; a.dbih_part = q.dbih_part;
      if (q.fuse_p) { a.ids = ids_; a.dP_part = dP_part_; a.V = V; }
      a.cnt = cnt_ + (size_t)(L + l) * fw; a.err = err_; a.allow_local = xcd_local_;
      if (persist_fwd_) { a.zero_next = cnt_ + (size_t)l * fw; a.zero_words = fw; }
      a.T = T; a.Bp = B; a.H = H;
      if (!persist_fwd_) fill_f32(reinterpret_cast<float*>(a.cnt), fw, 0.f, s);
      a.xring = step_lds_variants().bwd_xring;
      if (q.rows16) gru_bwd_seq16(a, s); else gru_bwd_seq(a, s);
    } else if (q.big) {
      SeqBwdArgs a;
      a.dy = y.dy; a.HSf = y.HSf;
      if (q.s16) a.s16 = y.s16;
      else { a.sr = y.sr; a.sz = y.sz; a.sn = y.sn; a.sghn = y.sghn; }
      a.WhhT = y.WhhT; a.xbuf = xbuf_; a.part = bpart_;
      a.dghT = y.dghT; a.dgiT = y.dgiT; a.ldG = (int)ldG_; a.dgi = y.dgi;
      a.dgiT_n_only = l == 0 && dgiT_share_;
      a.dbhh_part = q.dbhh_part; a.dbih_part = l == 0 ? q.dbih_part : nullptr;   // (l > 0: from the dW_ih GEMM)
      if (dy_in_bwd_ && l == L - 1) { a.dl = dl_; a.WfcT = WfcT; a.V = V; a.dy = nullptr; }
      a.cnt = cnt_ + (size_t)(L + l) * fw; a.err = err_;
      a.T = T; a.Bp = B; a.H = H;
      a.xring = step_lds_variants().bwd_xring;
      fill_f32(reinterpret_cast<float*>(a.cnt), 8192, 0.f, s);
      gru_bwd_seq_big(a, s);
    } else {
      for (int t = T - 1; t >= 0; --t) bwd_step(l, t, s);
    }
    // data-parallel: groups that became ready before this kernel go out now (they cannot overlap it)
    if (dp && q.bwd) ar_flush(s, false);
    // weight gradients not accumulated inside the sequence kernel
    SlabJobs j;
    if (q.fuse_w) slab_job(j, q.dWhh_part, q.nrb, (long)H3 * H, G("weight_hh_l" + k));
    if (q.bwd || q.big) slab_job(j, q.dbhh_part, q.nrb, H3, G("bias_hh_l" + k));
    // layer 0's dP goes straight to the bf16 (+ transposed) GEMM operands of the tail -- or, when the
    // tail runs after the data-parallel all-reduce, to fp32 dP (the tensor that is all-reduced)
    if (l == 0 && q.fuse_p) {
      if (dp) j.add(dP_part_, q.nrb, (long)V * H3, dP_target());
      else j.add_cast(dP_part_, q.nrb, V, H3, nullptr, dP_bf_, dPT_bf_);
    }
    if (l == 0 && (q.bwd || q.big)) slab_job(j, q.dbih_part, q.nrb, H3, G("bias_ih_l0"));
    // dW_fc / db_fc slabs: with the top layer's group when data-parallel (the FC group is
    // all-reduced with it), else with layer 0's reduce; the pipelined tail reduces them on their own
    const bool pipe = dp && l == 0 && dp_pipe_on();
    if ((dp ? l == L - 1 : l == 0) && !pipe)
      for (int k2 = 0; k2 < tail.n; ++k2)
        slab_job(j, tail.job[k2].src, tail.job[k2].splits, tail.job[k2].n, tail.job[k2].dst);
    if (l == 0) {   // + the loss partials and the optimiser step counter
      j.add(loss_part_, nloss_, 1, loss_);
      j.bump = step_;
    }
    if (pipe) {   // one-layer data-parallel: the bucketed, pipelined tail records the rest of the step
      if (!q.fuse_p || !q.fuse_w) throw std::runtime_error("pipelined data-parallel tail: needs the fused dW_hh / dP backward");
      record_dp_tail_l1(s, j, tail);
      HIP_LAUNCH_CHECK();
      return;
    }
    if (j.n) reduce_slabs_multi(j, s);
    if (!q.fuse_w)
      wgrad_gemm(y.dghT, (int)ldG_, y.HT, (T + 1) * B, H3, H, (int)tok, G("weight_hh_l" + k),
                 (q.bwd || q.big) ? nullptr : G("bias_hh_l" + k), s);
    if (l == 0) {
      if (!q.fuse_p) {
        GemmArgs p;   // dP = onehot(x)^T · dGi, split-K then reduce
        int sp = splits_;
        while (sp > 1 && (tok % sp || (tok / sp) % 128)) sp >>= 1;
        p.onehot_ids = ids_; p.B = y.dgiT; p.ldb = (int)ldG_;
        if (dgiT_share_) { p.B = y.dghT; p.B2 = y.dgiT; p.b2_row = H3 - H; }
        p.C = slab_w_; p.ldc = H3; p.M = V; p.N = H3; p.K = (int)tok; p.splits = sp;
        {   // the streaming one-hot kernel (G read once) picks its own K-slices (<= the slab's splits_)
          GemmArgs q = p;
          q.splits = std::min(splits_, onehot_dp_splits(H3, (int)tok));
          if (gemm_variants().onehot && onehot_dp_ok(q)) { p = q; sp = q.splits; }
        }
        gemm_nt(p, s);
        float* dPd = dp ? dP_target() : dP_;
        reduce_slabs(slab_w_, sp, (long)V * H3, dPd, s);
        if (!q.bwd && !q.big) colsum(dPd, V, H3, G("bias_ih_l0"), s);
      }
      if (dp) {   // layer 0's group [W_hh0, b_hh0, b_ih0, dP] closes the step's collectives
        ar_ready_ = group_end(0);
        // collectives still open across the backward (upper layers' groups) end here; nothing is left to overlap with, so the last collectives go on the step
        // stream itself (a fork + join around them only adds graph edges -- measured: a forked
        // branch in the step graph slowed the kernels beside it).  The step's LAST collective
        // carries the error word along (max over ranks, same launch): a persistent kernel that
        // gave up on ANY rank makes every rank skip the update.
        ar_join(s);
        const long n = ar_ready_ - ar_launched_;
        if (n > 0) {
          if (dP_inplace_) comm_->allreduce_avg_f32_err(grads_ + ar_launched_, n, err_, s);
          else comm_->allreduce_avg_f32(grads_ + ar_launched_, n, s);
          ar_log_.push_back({ar_launched_, n});
          ar_launched_ = ar_ready_;
        }
        if (!dP_inplace_) {
          comm_->allreduce_avg_f32_err(dP_, (long)V * H3, err_, s);
          ar_log_.push_back({-1, (long)V * H3});
        } else if (n <= 0) {
          comm_->allreduce_max_u32(err_, 1, s);
        }
      }
    } else {
      const int K = in_dim(l);
      // dW_ih = dGi^T · h_below, db_ih = row sums of dGi^T
      wgrad_gemm(y.dgiT, (int)ldG_, Ls_[l - 1].HT + B, (T + 1) * B, H3, K, (int)tok, G("weight_ih_l" + k),
                 G("bias_ih_l" + k), s);
      if (dp) {
        ar_ready_ = group_end(l);   // FC (if l is the top layer) + this layer's four gradients
        // span (default): the group goes out now and its collective stays open across the next
        // persistent backward kernel (joined before the embedding tail).  Neither waits on the
        // other -- the RCCL kernel only on its peers, the sequence kernel only on its own
        // workgroups -- so if the collective's workgroups cannot co-reside they run after it
        // (no overlap, no deadlock).  (Joined before the persistent kernel instead: equal at one rank.)
        // The fork comes after the dX GEMM below, so the collective starts beside the sequence
        // kernel rather than beside that bandwidth-bound GEMM.
        if (!seq_[l - 1].bwd) ar_flush(s, false);
        else if (!ar_span()) ar_join(s);   // (no-op unless an earlier flush is still open)
      }
      GemmArgs dx;  // dy of the layer below = dGi · W_ih
      dx.A = y.dgi; dx.lda = H3; dx.B = y.WihT; dx.ldb = H3;
      dx.C = Ls_[l - 1].dy; dx.ldc = H; dx.M = (int)tok; dx.N = H; dx.K = H3;
      gemm_nt(dx, s);
      if (dp && seq_[l - 1].bwd && ar_span()) ar_flush(s, false);
    }
  }
  // ------------------------------------------------------------------ embedding-side gradients
  if (dp) {
    // from the averaged dP; its dEmb slabs are already global (after the collective), so like the
    // single-GPU step they are summed inside the Adam launch (one reduce launch fewer)
    defer_slabs_ = o_.clip <= 0.f;
    record_emb_tail(s, dP_target());
    defer_slabs_ = false;
  } else {
    record_emb_tail(s, seq_[0].fuse_p ? nullptr : dP_);
  }
  HIP_LAUNCH_CHECK();
}

// The pipelined one-layer data-parallel tail (Trainer::dp_pipe_).  j holds the
// backward's slab jobs (W_hh0, b_hh0, b_ih0 partials, dP -> the W_ih0 slot, loss); fc_tail the dW_fc /
// db_fc K-slice slabs of the held FC GEMM.  Three readiness buckets of the flat gradient (layout:
// fc.weight, fc.bias | weight_hh_l0, bias_hh_l0, bias_ih_l0 | dP in the weight_ih_l0 slot):
//   s : reduce(j)                         c : AR1 = [W_hh0 .. dP] + error word (max over ranks)
//   s : dW_fc K-slices -> reduce(fc)      c : AR2 = [fc.weight, fc.bias]
//   s : join AR1 -> dW_ih0 / dEmb (one grouped launch on the averaged fp32 dP) -> Adam(all but FC)
//   s : join AR2 -> Adam(FC)
// At world W, AR1 (4.6 MB at the headline) runs beside the dW_fc GEMM and its reduce, AR2 beside the
// embedding GEMMs and the first Adam launch, instead of one 5.25 MB collective with nothing beside
// it.  Every per-element sum is the single-bucket step's (same reduce kernel and order, the same GEMM
// k order, Adam per element), so at one rank the result is bitwise that step's
// (tests/test_engine_gpu.py::test_dp_pipelined_tail_world1).  Reference: the reference's only
// parallel layer is scatter -> compute -> gather around the name loop (namegensf.cu:628-636, 889).
void Trainer::record_dp_tail_l1(hipStream_t s, SlabJobs& j, const SlabJobs& fc_tail) {
  const long r0 = off_.at("weight_hh_l0"), r1 = group_end(0);
  if (j.n) reduce_slabs_multi(j, s);
  hipEvent_t e = ev();
  HIP_CHECK(hipEventRecord(e, s));          // fork AR1 after the reduce
  HIP_CHECK(hipStreamWaitEvent(sc_, e, 0));
  comm_->allreduce_avg_f32_err(grads_ + r0, r1 - r0, err_, sc_);
  ar_log_.push_back({r0, r1 - r0});
  hipEvent_t ar1 = ev();
  HIP_CHECK(hipEventRecord(ar1, sc_));
  // beside AR1: the dW_fc K-slices (held back from before the backward) and their slab reduce
  if (fc_held_on_) gemm_nt(fc_held_, s);
  else if (!fc_in_fwd_) throw std::runtime_error("pipelined data-parallel tail: the dW_fc GEMM was not held");
  fc_held_on_ = false;
  if (fc_tail.n) {
    SlabJobs f;
    for (int k = 0; k < fc_tail.n; ++k) f.job[f.n++] = fc_tail.job[k];
    reduce_slabs_multi(f, s);
  }
  hipEvent_t e2 = ev();
  HIP_CHECK(hipEventRecord(e2, s));
  HIP_CHECK(hipStreamWaitEvent(sc_, e2, 0));
  comm_->allreduce_avg_f32(grads_, r0, sc_);   // [fc.weight, fc.bias] (offset 0: readiness order)
  ar_log_.push_back({0, r0});
  hipEvent_t ar2 = ev();
  HIP_CHECK(hipEventRecord(ar2, sc_));
  // join AR1: the embedding-side GEMMs from the averaged dP, then Adam on everything but the FC pair
  HIP_CHECK(hipStreamWaitEvent(s, ar1, 0));
  defer_slabs_ = true;
  record_emb_tail(s, dP_target());
  record_opt(s, 1);
  defer_slabs_ = false;
  // join AR2: Adam on the FC pair
  HIP_CHECK(hipStreamWaitEvent(s, ar2, 0));
  record_opt(s, 2);
  ar_busy_ = false;
  opt_in_fb_ = true;
  dp_tail_rec_ = true;
}

// dEmb = dP · W_ih0 and dW_ih0 = dP^T · Emb from the layer-0 table gradient dP.  dP_fp32 may
// alias the W_ih0 gradient slot (data-parallel): it is fully read by the cast before the GEMM
// below overwrites that slot (same stream).
void Trainer::record_emb_tail(hipStream_t s, const float* dP_fp32) {
  const int V = d_.V, E = d_.E, H3 = 3 * d_.H;
  // data-parallel, slab sums deferred into Adam: the one-shot GEMMs stage the all-reduced fp32 dP
  // themselves (no cast launch), and dW_ih0 goes to a one-slab buffer that Adam reads -- dP lives in
  // the W_ih0 gradient slot, so the GEMM must not write there while its other blocks read dP
  if (dP_fp32 && defer_slabs_ && H3 % V == 0 && H3 / V <= splits_) {
    GemmArgs g;   // dW_ih0 = dP^T · Emb
    g.A32 = dP_fp32; g.a32_trans = 1; g.lda = H3; g.B = EmbT; g.ldb = V; g.C = slab_w_; g.ldc = E;
    g.M = H3; g.N = E; g.K = V;
    GemmArgs es;  // dEmb = dP · W_ih0, K-slices of V into slab_e_
    es.A32 = dP_fp32; es.lda = H3; es.B = Ls_[0].WihT; es.ldb = H3; es.C = slab_e_; es.ldc = E;
    es.M = V; es.N = E; es.K = H3; es.splits = H3 / V;
    const int nkb = gemm_small_kblocks(g);
    if (nkb && nkb == gemm_small_kblocks(es)) {
      const GemmArgs pair[2] = {g, es};
      gemm_small_group(pair, 2, s);
      slab_job(deferred_, slab_w_, 1, (long)H3 * E, G("weight_ih_l0"));
      slab_job(deferred_, slab_e_, es.splits, (long)V * E, G("embedding"));
      HIP_LAUNCH_CHECK();
      return;
    }
  }
  if (dP_fp32) {
    CastJobs j;
    j.add(dP_fp32, V, H3, dP_bf_, dPT_bf_);
    cast_multi(j, s);
  }
  GemmArgs g;   // dW_ih0 = dP^T · Emb
  g.A = dPT_bf_; g.lda = V; g.B = EmbT; g.ldb = V; g.C = G("weight_ih_l0"); g.ldc = E;
  g.M = H3; g.N = E; g.K = V;
  GemmArgs e;   // dEmb = dP · W_ih0, split-K (K = 3H on only V x E outputs) into slab_e_
  int se = splits_;
  while (se > 1 && (H3 % se || (H3 / se) % 64 || H3 / se < 128)) se >>= 1;
  e.A = dP_bf_; e.lda = H3; e.B = Ls_[0].WihT; e.ldb = H3; e.C = slab_e_; e.ldc = E;
  e.M = V; e.N = E; e.K = H3; e.splits = se;
  // one-shot small GEMMs when dEmb's K-slice can match dW_ih0's (K = V): one grouped launch
  if (H3 % V == 0 && H3 / V <= splits_) {
    GemmArgs es = e;
    es.splits = H3 / V;
    // the held dW_fc K-slices (4-chunk tiles) first: they are the long ones
    const GemmArgs three[3] = {fc_held_, g, es};
    const bool with_fc = fc_held_on_ && gemm_small_group_depth(three, 3) == gemm_small_kblocks(g);
    const int nkb = gemm_small_kblocks(g);
    if (nkb && nkb == gemm_small_kblocks(es)) {
      const GemmArgs pair[2] = {g, es};
      if (fc_held_on_ && !with_fc) gemm_nt(fc_held_, s);
      if (with_fc) gemm_small_group(three, 3, s);
      else gemm_small_group(pair, 2, s);
      fc_held_on_ = false;
      SlabJobs r;
      slab_job(r, slab_e_, es.splits, (long)V * E, G("embedding"));
      if (r.n) reduce_slabs_multi(r, s);
      HIP_LAUNCH_CHECK();
      return;
    }
  }
  if (fc_held_on_) gemm_nt(fc_held_, s);
  fc_held_on_ = false;
  const GemmArgs both[2] = {g, e};
  // one launch for both products while they fit one round of 128^2 workgroups at two per CU; past that
  // (h2048: 768 + 256 tiles) each on its own launch
  const long wg = (long)(g.M / 128) * (g.N / 128) * g.splits + (long)(e.M / 128) * (e.N / 128) * e.splits;
  if (gemm_lds_ok(g) && gemm_lds_ok(e) && wg <= 512) {
    gemm_lds_group(both, 2, s);
  } else {
    gemm_nt(g, s);
    gemm_nt(e, s);
  }
  SlabJobs r;
  slab_job(r, slab_e_, se, (long)V * E, G("embedding"));
  if (r.n) reduce_slabs_multi(r, s);
  HIP_LAUNCH_CHECK();
}

std::string Trainer::plan() const {
  std::string p = std::string("fwd=") +
                  (persist_fwd_ ? (fwd_wave_ ? "persistent+wave" : fc_in_fwd_ ? "persistent+fc" : "persistent") : "per-step");
  for (size_t l = 0; l < seq_.size(); ++l) {
    p += " bwd" + std::to_string(l) + "=" +
         (seq_[l].bwd ? (seq_[l].rows16 ? "persistent16" : "persistent") : seq_[l].big ? "persistent-big" : "per-step");
    if (seq_[l].fuse_w) p += "+dWhh";
    if (seq_[l].fuse_p) p += "+dP";
    if (dy_in_bwd_ && l + 1 == seq_.size()) p += "+dy";
  }
  bool any_step = !persist_fwd_;
  for (const SeqPlan& q : seq_) any_step |= !q.bwd;
  if (any_step) p += std::string(" step=") + (gru_step_picks_lds(step_algo_, d_.H, Bp_) ? "lds" : "reg");
  p += overlap_ ? " overlap(chunks=" + std::to_string(C_) + ")" : " serial";
  return p;
}

unsigned Trainer::read_error() {
  unsigned e = 0;
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(&e, err_, 4, hipMemcpyDeviceToHost));
  return e;
}

}  // namespace gk
