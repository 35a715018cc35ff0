#include "trainer.h"
#include "../runtime/trace.h"
#include "../runtime/blaslt.h"

#include <cstring>
#include <algorithm>

namespace gk {

static int round_up(int x, int m) { return (x + m - 1) / m * m; }


Trainer::Trainer(const Dims& d, const OptCfg& o, float* params, float* grads, float* m, float* v, long nflat,
                 const std::map<std::string, long>& offsets)
    : d_(d), o_(o), params_(params), grads_(grads), m_(m), v_(v), nflat_(nflat), off_(offsets) {
  if (d_.V % 64 || d_.E % 64 || d_.H % 64)
    throw std::runtime_error("HIP engine needs vocab, embed and hidden to be multiples of 64");
  Bp_ = round_up(std::max(d_.B, 1), 64);
  // library handle + workspace now, never inside the step-graph capture (also where the weight-
  // gradient engine will route dW_hh to the library)
  blaslt_init(wgrad_prefers_library(3 * d_.H, d_.H, (long)d_.T * Bp_));
  C_ = std::max(1, d_.chunks);
  while (C_ > 1 && d_.T % C_) --C_;
  Tc_ = d_.T / C_;
  const int V = d_.V, E = d_.E, H = d_.H, T = d_.T, L = d_.L, B = Bp_;
  const size_t tok = (size_t)T * B;
  // leading dimension of the token-major transposed operands (dGh^T / dGi^T, dl^T): rows 64 KiB or
  // more apart (tok = T * B, usually a power of two) get 64 elements of padding -- config 5 (128 KiB
  // rows): one-hot dP 226 -> 198 us, dW_hh 1224 -> 1187, backward 3191 -> 3148, step 8.005-8.049 ->
  // 7.966-7.974 ms; at the headline's 16 KiB rows it measured 1-2 us slower, so those stay dense
  // (profiles/r6_ldpad_*.jsonl, r6_ldpad_traces.txt)
  const int pad = step_lds_variants().ld_pad;
  ldG_ = (long)tok + (pad >= 0 ? pad : tok >= 32768 ? 64 : 0);

  // ---- size the arena
  struct Pend { size_t off; };
  std::vector<size_t> lo;
  auto R = [&](size_t bytes) { return arena_.reserve(bytes); };
  size_t o_ids = R(tok * 4), o_lab = R(tok * 4), o_inv = R(16), o_P = R((size_t)V * 3 * H * 4);
  size_t o_lp = R(tok / 32 * 4 + 16), o_loss = R(16), o_sfc = R((size_t)C_ * V * H * 4), o_rfc = R((size_t)C_ * V * 4);
  size_t o_sP = R((size_t)C_ * V * 3 * H * 4), o_dP = R((size_t)V * 3 * H * 4);
  size_t o_np = R(256 * 4), o_gs = R(16), o_step = R(16);
  size_t o_Emb = R((size_t)V * E * 2), o_EmbT = R((size_t)V * E * 2), o_Wfc = R((size_t)V * H * 2), o_WfcT = R((size_t)V * H * 2);
  size_t o_WfcF = R((size_t)V * H * 2), o_WfcTF = R((size_t)V * H * 2);
  size_t o_dl = R(tok * V * 2), o_dlT = R((size_t)ldG_ * V * 2), o_dPb = R((size_t)V * 3 * H * 2), o_dPTb = R((size_t)V * 3 * H * 2);
  // fp32 logits of the GEMM + row-softmax FC path (shapes the fused 8-wave kernel does not cover)
  fc_split_ = !fc_xent_fused_ok(V, H, (int)tok) && tok % 128 == 0 && V % 128 == 0 && V <= 512 && H % 64 == 0 &&
              H >= 128;
  size_t o_lg = fc_split_ ? R(tok * V * 4) : 0;
  struct LO { size_t HSf, sr, sz, sn, sghn, dy, Gi, c0, c1, HSb, HT, g0, g1, dghT, dgiT, dgi, Whh, WhhT, Wih, WihT, shh, rhh, sih, rih; };
  std::vector<LO> los(L);
  for (int l = 0; l < L; ++l) {
    const int K = in_dim(l);
    LO& x = los[l];
    x.HSf = R((tok + B) * H * 4);
    x.sr = R(tok * H * 4); x.sz = R(tok * H * 4); x.sn = R(tok * H * 4); x.sghn = R(tok * H * 4);
    x.dy = R(tok * H * 4);
    x.Gi = l > 0 ? R(tok * 3 * H * 4) : 0;
    x.c0 = R((size_t)B * H * 4); x.c1 = R((size_t)B * H * 4);
    x.HSb = R((tok + B) * H * 2); x.HT = R((tok + B) * H * 2);
    x.g0 = R((size_t)B * 3 * H * 2); x.g1 = R((size_t)B * 3 * H * 2);
    x.dghT = R((size_t)ldG_ * 3 * H * 2); x.dgiT = R((size_t)ldG_ * 3 * H * 2);
    x.dgi = l > 0 ? R(tok * 3 * H * 2) : 0;
    x.Whh = R((size_t)3 * H * H * 2); x.WhhT = R((size_t)3 * H * H * 2);
    x.Wih = R((size_t)3 * H * K * 2); x.WihT = R((size_t)3 * H * K * 2);
    x.shh = R((size_t)C_ * 3 * H * H * 4); x.rhh = R((size_t)C_ * 3 * H * 4);
    x.sih = l > 0 ? R((size_t)C_ * 3 * H * K * 4) : 0; x.rih = l > 0 ? R((size_t)C_ * 3 * H * 4) : 0;
  }
  // ---- persistent-sequence path (gru_seq.hip): decided per layer from the occupancy query
  const char* pe = std::getenv("GK_PERSIST");
  const bool allow = !(pe && pe[0] == '0');
  persist_fwd_ = allow && gru_fwd_seq_supported(H, B);
  {
    const char* fw = std::getenv("GK_FWD_WAVE");
    fwd_wave_ = persist_fwd_ && L >= 2 && !(fw && fw[0] == '0') && gru_fwd_seq2_supported(H, B);
  }
  if (const char* sa = std::getenv("GK_STEP_ALGO")) step_algo_ = std::atoi(sa);
  if (const char* xl = std::getenv("GK_XCD_LOCAL")) xcd_local_ = std::atoi(xl) != 0;
  if (step_algo_ == 2 && !gru_step_lds_ok(H, B)) step_algo_ = 0;
  {
    // shapes where both one-hot dP call sites (whole sequence, and per time chunk in the overlapped
    // schedule) are LDS-kernel shapes with 128-aligned gate blocks (gemm_lds_ok with B2)
    const long tok = (long)d_.T * B, ctok = (long)Tc_ * B;
    dgiT_share_ = V % 128 == 0 && H % 128 == 0 && B % 8 == 0 && tok % 128 == 0 &&
                  ctok % 128 == 0;
  }
  seq_.resize(L);
  bool any_bwd = false;
  for (int l = 0; l < L; ++l) {
    SeqPlan& q = seq_[l];
    q.fuse_p = (l == 0) && V == 256 && allow && gru_bwd_seq_supported(H, B, H <= 512, true);
    q.fuse_w = allow && H <= 512 && gru_bwd_seq_supported(H, B, true, q.fuse_p);
    q.bwd = allow && gru_bwd_seq_supported(H, B, q.fuse_w, q.fuse_p);
    if (!q.bwd) q.fuse_w = q.fuse_p = false;
    q.big = allow && !q.bwd && step_lds_variants().bwd_big && gru_bwd_seq_big_supported(H, B) &&
            seq_flag_words(H, B) >= 8192;
    // 32-row blocks that cannot be XCD-local (Bp/32 not a multiple of 8) but 16-row ones can
    q.rows16 = q.bwd && !q.fuse_w && (B / 32) % 8 != 0 && (B / 16) % 8 == 0 && step_lds_variants().bwd16 &&
               gru_bwd_seq16_supported(H, B, q.fuse_p);
    q.nrb = q.rows16 ? B / 16 : B / 32;
    any_bwd |= q.bwd;
  }
  // packed bf16 saves where the layer's forward (persistent, or the LDS-staged step kernels) and
  // backward (any persistent kernel) both read / write them
  for (int l = 0; l < L; ++l) {
    SeqPlan& q = seq_[l];
    const bool fwd16 = persist_fwd_ || gru_step_picks_lds(step_algo_, H, B);
    q.s16 = step_lds_variants().save16 && d_.overlap == 0 && (q.big || q.bwd) && fwd16;
  }
  splits_ = 8;
  size_t o_cnt = R((size_t)2 * L * seq_flag_words(H, B) * 4 + 64), o_err = R(64), o_x = R((size_t)T * B * 3 * H * 2);
  // split-K slab: large enough for every weight-gradient product it serves
  constexpr int kSlots = 2 + 2 * kMaxGroup;   // per-step pair + two multi-step groups
  size_t o_dst = R((size_t)kSlots * slot_ints() * 4);
  const size_t wmax = std::max({(size_t)V * H, (size_t)3 * H * H, (size_t)V * 3 * H, (size_t)3 * H * E});
  size_t o_sw = R((size_t)splits_ * wmax * 4);
  size_t o_rw = R((size_t)splits_ * std::max(V, 3 * H) * 4);
  size_t o_sfc2 = R((size_t)kFcSplitsMax * V * H * 4), o_rfc2 = R((size_t)kFcSplitsMax * V * 4);
  size_t o_se = R((size_t)splits_ * V * E * 4);
  std::vector<size_t> o_pw(L, 0), o_pbh(L, 0), o_pbi(L, 0), o_hf(L, 0), o_s16(L, 0);
  for (int l = 0; l < L; ++l) {
    if (seq_[l].s16) o_s16[l] = R(tok * H * 8);
    if (seq_[l].fuse_w) o_pw[l] = R((size_t)seq_[l].nrb * 3 * H * H * 4);
    if (seq_[l].fuse_w && persist_fwd_) o_hf[l] = R((tok + B) * H * 2);
    if (seq_[l].bwd || seq_[l].big) {
      o_pbh[l] = R((size_t)seq_[l].nrb * 3 * H * 4);
      o_pbi[l] = R((size_t)seq_[l].nrb * 3 * H * 4);
    }
  }
  size_t o_pP = seq_[0].fuse_p ? R((size_t)seq_[0].nrb * V * 3 * H * 4) : 0;
  // per-step backward on the split-K LDS kernel: partial tiles + monotonic arrival counters
  // (shared by all layers: their step kernels run one after another on one stream)
  int sk = 0;
  bool any_big = false;
  for (int l = 0; l < L; ++l) {
    if (!seq_[l].bwd && !seq_[l].big) sk = gru_bwd_step_sk_splits(H, B);
    any_big |= seq_[l].big;
  }
  size_t o_bp = any_big ? R((size_t)gru_bwd_seq_big_part_floats(H, B) * 4) : 0;
  sk_part_floats_ = sk ? (long)H * B * sk : 0;
  sk_cnt_words_ = sk ? (long)(H / 128) * (B / 64) * 16 : 0;   // 64-row tiles (gru_bwd_step_sk64) need twice the 128-row count
  size_t o_skp = sk ? R((size_t)sk_part_floats_ * 4) : 0, o_skc = sk ? R((size_t)sk_cnt_words_ * 4) : 0;
  (void)any_bwd;
  arena_.commit();   // zero-filled: HS[0] = h_init = 0, HT columns [0,Bp) = 0
  d_stage_ = arena_.get<int>(o_dst);
  cnt_ = arena_.get<unsigned>(o_cnt); err_ = arena_.get<unsigned>(o_err); xbuf_ = arena_.get<u16>(o_x);
  slab_w_ = arena_.get<float>(o_sw); rs_w_ = arena_.get<float>(o_rw);
  slab_fc2_ = arena_.get<float>(o_sfc2); rs_fc2_ = arena_.get<float>(o_rfc2); slab_e_ = arena_.get<float>(o_se);
  for (int l = 0; l < L; ++l) {
    seq_[l].dWhh_part = seq_[l].fuse_w ? arena_.get<float>(o_pw[l]) : nullptr;
    seq_[l].HF = o_hf[l] ? arena_.get<u16>(o_hf[l]) : nullptr;   // zero-filled: HF[0] = h_init
    seq_[l].dbhh_part = (seq_[l].bwd || seq_[l].big) ? arena_.get<float>(o_pbh[l]) : nullptr;
    seq_[l].dbih_part = (seq_[l].bwd || seq_[l].big) ? arena_.get<float>(o_pbi[l]) : nullptr;
  }
  dP_part_ = seq_[0].fuse_p ? arena_.get<float>(o_pP) : nullptr;
  bpart_ = any_big ? arena_.get<float>(o_bp) : nullptr;
  sk_part_ = sk ? arena_.get<float>(o_skp) : nullptr;
  sk_cnt_ = sk ? arena_.get<unsigned>(o_skc) : nullptr;

  ids_ = arena_.get<int>(o_ids); labels_ = arena_.get<int>(o_lab); inv_count_ = arena_.get<float>(o_inv);
  Ptab_ = arena_.get<float>(o_P); loss_part_ = arena_.get<float>(o_lp); loss_ = arena_.get<float>(o_loss);
  slab_fc_ = arena_.get<float>(o_sfc); rs_fc_ = arena_.get<float>(o_rfc); slab_P_ = arena_.get<float>(o_sP);
  dP_ = arena_.get<float>(o_dP); norm_parts_ = arena_.get<float>(o_np); gscale_ = arena_.get<float>(o_gs);
  step_ = arena_.get<int>(o_step);
  Emb = arena_.get<u16>(o_Emb); EmbT = arena_.get<u16>(o_EmbT); Wfc = arena_.get<u16>(o_Wfc); WfcT = arena_.get<u16>(o_WfcT);
  WfcF = arena_.get<u16>(o_WfcF); WfcTF = arena_.get<u16>(o_WfcTF);
  logits_ = fc_split_ ? arena_.get<float>(o_lg) : nullptr;
  dl_ = arena_.get<u16>(o_dl); dlT_ = arena_.get<u16>(o_dlT); dP_bf_ = arena_.get<u16>(o_dPb); dPT_bf_ = arena_.get<u16>(o_dPTb);
  Ls_.resize(L);
  for (int l = 0; l < L; ++l) {
    const LO& x = los[l];
    Layer& y = Ls_[l];
    y.HSf = arena_.get<float>(x.HSf); y.sr = arena_.get<float>(x.sr); y.sz = arena_.get<float>(x.sz);
    y.sn = arena_.get<float>(x.sn); y.sghn = arena_.get<float>(x.sghn); y.dy = arena_.get<float>(x.dy);
    y.Gi = l > 0 ? arena_.get<float>(x.Gi) : nullptr;
    y.carry[0] = arena_.get<float>(x.c0); y.carry[1] = arena_.get<float>(x.c1);
    y.HSb = arena_.get<u16>(x.HSb); y.HT = arena_.get<u16>(x.HT);
    y.dgh[0] = arena_.get<u16>(x.g0); y.dgh[1] = arena_.get<u16>(x.g1);
    y.dghT = arena_.get<u16>(x.dghT); y.dgiT = arena_.get<u16>(x.dgiT);
    y.dgi = l > 0 ? arena_.get<u16>(x.dgi) : nullptr;
    y.Whh = arena_.get<u16>(x.Whh); y.WhhT = arena_.get<u16>(x.WhhT);
    y.Wih = arena_.get<u16>(x.Wih); y.WihT = arena_.get<u16>(x.WihT);
    y.slab_hh = arena_.get<float>(x.shh); y.rs_hh = arena_.get<float>(x.rhh);
    y.slab_ih = l > 0 ? arena_.get<float>(x.sih) : nullptr; y.rs_ih = l > 0 ? arena_.get<float>(x.rih) : nullptr;
    y.s16 = o_s16[l] ? arena_.get<u16>(o_s16[l]) : nullptr;
  }

  HIP_CHECK(hipStreamCreateWithFlags(&s0_, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&s1_, hipStreamNonBlocking));
  {   // gradient collectives: highest-priority stream so their kernels dispatch ahead of compute
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamCreateWithPriority(&sc_, hipStreamNonBlocking, hi));
  }
  events_.resize(64 + 8 * C_ * L);
  for (auto& e : events_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_CHECK(hipStreamCreateWithFlags(&sx_, hipStreamNonBlocking));
  HIP_CHECK(hipHostMalloc(&h_stage_, kSlots * (2 * tok + 16) * sizeof(int)));
  std::memset(h_stage_, 0, kSlots * (2 * tok + 16) * sizeof(int));
  // The staging events only tell the host that the graph which read a pinned slot has finished;
  // the host never reads device results through them, so they skip the system-scope release
  // (an end-of-step L2 writeback to host-coherent memory between consecutive step graphs).
  const unsigned stage_flags = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
  for (auto& e : stage_done_) {
    HIP_CHECK(hipEventCreateWithFlags(&e, stage_flags));
    HIP_CHECK(hipEventRecord(e, s0_));
  }
  for (auto& e : group_done_) {
    HIP_CHECK(hipEventCreateWithFlags(&e, stage_flags));
    HIP_CHECK(hipEventRecord(e, s0_));
  }
  for (auto* ev : {&copy_done_[0], &copy_done_[1], &group_copy_done_[0], &group_copy_done_[1]}) {
    HIP_CHECK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(*ev, sx_));
  }
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 64, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(err_host_, 0, 64);
  HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_host_dev_), err_host_, 0));
  const char* ng = std::getenv("GK_NO_GRAPH");
  if (ng && ng[0] == '1') use_graph_ = false;
  overlap_ = d_.overlap != 0;
  dy_in_bwd_ = fc_split_ && !overlap_ && !seq_.empty() && seq_.back().big && seq_.back().s16 && d_.V == 256 &&
               step_lds_variants().big_dy;
  fc_in_fwd_ = persist_fwd_ && !fwd_wave_ && d_.L == 1 && !overlap_ && !fc_split_ && !seq_.empty() &&
               seq_[0].bwd && seq_[0].fuse_w && seq_[0].HF && step_lds_variants().fwd_fc &&
               Bp_ / 32 <= kFcSplitsMax && gru_fwd_seq_fc_supported(d_.H, Bp_, d_.V);
}

Trainer::~Trainer() {
  if (pbf_) (void)hipFree(pbf_);
  if (bpack_) (void)hipFree(bpack_);
  for (auto& g : g_fb_) g.reset();
  for (auto& g : g_step_) g.reset();
  for (auto& g : g_group_) g.reset();
  g_opt_.reset();
  for (auto& e : events_) (void)hipEventDestroy(e);
  for (auto& g : g_group_) g.reset();
  for (auto& e : stage_done_) if (e) (void)hipEventDestroy(e);
  for (auto& e : group_done_) if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {copy_done_[0], copy_done_[1], group_copy_done_[0], group_copy_done_[1]})
    if (e) (void)hipEventDestroy(e);
  wd_.reset();   // the watchdog thread reads err_host_
  if (h_stage_) (void)hipHostFree(h_stage_);
  if (err_host_) (void)hipHostFree(err_host_);
  if (s0_) (void)hipStreamDestroy(s0_);
  if (s1_) (void)hipStreamDestroy(s1_);
  if (sx_) (void)hipStreamDestroy(sx_);
  if (sc_) (void)hipStreamDestroy(sc_);
}

hipEvent_t Trainer::ev() {
  if (ev_next_ >= events_.size()) throw std::runtime_error("trainer: event pool exhausted");
  return events_[ev_next_++];
}


void Trainer::set_carry(bool on) {
  if (on == carry_) return;
  carry_ = on;
  for (auto& g : g_fb_) g.reset();   // the copies and the kernels' h0 argument are captured
  for (auto& g : g_step_) g.reset();
  for (auto& g : g_group_) g.reset();
}

// Every copy of h kept per step: fp32 and bf16 row-major [T+1][Bp][H], the transposed bf16
// [H][(T+1)Bp] (columns t*Bp..) and, for fused backward layers, the fragment-tiled HF (slot t
// contiguous, Bp*H elements).  HS[0] is h_init for the forward and h_{-1} for the backward.
void Trainer::record_carry(hipStream_t s) {
  const int H = d_.H, T = d_.T, B = Bp_;
  const size_t n = (size_t)B * H, ldT = (size_t)(T + 1) * B;
  for (int l = 0; l < d_.L; ++l) {
    Layer& y = Ls_[l];
    HIP_CHECK(hipMemcpyAsync(y.HSf, y.HSf + (size_t)T * n, n * 4, hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipMemcpyAsync(y.HSb, y.HSb + (size_t)T * n, n * 2, hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipMemcpy2DAsync(y.HT, ldT * 2, y.HT + (size_t)T * B, ldT * 2, (size_t)B * 2, H,
                               hipMemcpyDeviceToDevice, s));
    if (seq_[l].HF)
      HIP_CHECK(hipMemcpyAsync(seq_[l].HF, seq_[l].HF + (size_t)T * n, n * 2, hipMemcpyDeviceToDevice, s));
  }
}

void Trainer::reset_hidden(hipStream_t s) {
  const int H = d_.H, T = d_.T, B = Bp_;
  const size_t n = (size_t)B * H, ldT = (size_t)(T + 1) * B;
  for (int l = 0; l < d_.L; ++l) {
    Layer& y = Ls_[l];
    for (int t : {0, T}) {
      HIP_CHECK(hipMemsetAsync(y.HSf + (size_t)t * n, 0, n * 4, s));
      HIP_CHECK(hipMemsetAsync(y.HSb + (size_t)t * n, 0, n * 2, s));
      HIP_CHECK(hipMemset2DAsync(y.HT + (size_t)t * B, ldT * 2, 0, (size_t)B * 2, H, s));
      if (seq_[l].HF) HIP_CHECK(hipMemsetAsync(seq_[l].HF + (size_t)t * n, 0, n * 2, s));
    }
  }
}

void Trainer::set_lr(float lr) {
  o_.lr = lr;
  g_opt_.reset();   // lr is a kernel argument frozen into the captured graphs
  for (auto& g : g_step_) g.reset();
  for (auto& g : g_group_) g.reset();
}

void Trainer::refresh_weights(hipStream_t s) {
  // one launch: every master weight -> bf16 copy (+ transposed bf16 copy where a kernel needs it)
  const int V = d_.V, E = d_.E, H = d_.H;
  CastJobs j;
  j.add(P("embedding"), V, E, Emb, EmbT);
  for (int l = 0; l < d_.L; ++l) {
    const std::string k = std::to_string(l);
    j.add(P("weight_hh_l" + k), 3 * H, H, Ls_[l].Whh, Ls_[l].WhhT);
    j.add(P("weight_ih_l" + k), 3 * H, in_dim(l), Ls_[l].Wih, Ls_[l].WihT);
  }
  j.add(P("fc.weight"), V, H, Wfc, WfcT, WfcF, WfcTF);
  cast_multi(j, s);
  HIP_LAUNCH_CHECK();
}

void Trainer::set_batch(const int* x, const int* y, int B, hipStream_t s) {
  if (B > Bp_ || B <= 0) throw std::runtime_error("set_batch: batch larger than the trainer was built for");
  (void)s;
  // Batch-major ids/labels are written into a pinned staging slot and copied to the device slot by
  // one DMA on the copy stream, off the step's critical path; the step graph captured against that
  // slot reads the device copy in its first kernel (prep_batch: transpose + pad).  The slot pair is
  // reused only after the graph that last read it has completed (stage_done_, recorded after each
  // launch), which also means its copy is done.
  const int slot = (stage_slot_ ^= 1);
  HIP_CHECK(hipEventSynchronize(stage_done_[slot]));
  fill_slot(slot, x, y, B);
  copy_slots(slot, 1, copy_done_[slot]);
}

void Trainer::copy_slots(int first, int n, hipEvent_t done) {
  const size_t off = (size_t)first * slot_ints();
  HIP_CHECK(hipMemcpyAsync(d_stage_ + off, h_stage_ + off, (size_t)n * slot_ints() * sizeof(int),
                           hipMemcpyHostToDevice, sx_));
  HIP_CHECK(hipEventRecord(done, sx_));
}

void Trainer::fill_slot(int slot, const int* x, const int* y, int B) {
  const int T = d_.T;
  const size_t n = (size_t)Bp_ * T;
  int* h = h_stage_ + (size_t)slot * slot_ints();
  long valid = 0;
  for (size_t i = 0; i < (size_t)B * T; ++i) valid += y[i] >= 0;
  const float inv = 1.0f / (float)std::max(1L, valid);
  h[0] = B;
  std::memcpy(h + 1, &inv, 4);
  std::memcpy(h + 16, x, (size_t)B * T * 4);
  std::memcpy(h + 16 + n, y, (size_t)B * T * 4);
}

void Trainer::set_batch_device(const int* x, const int* y, int B, hipStream_t s) {
  // device-resident batch: bring it through host memory once (not a hot path)
  if (B > Bp_ || B <= 0) throw std::runtime_error("set_batch_device: bad batch size");
  const size_t cnt = (size_t)B * d_.T;
  std::vector<int> hx(cnt), hy(cnt);
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipMemcpy(hx.data(), x, cnt * 4, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(hy.data(), y, cnt * 4, hipMemcpyDeviceToHost));
  set_batch(hx.data(), hy.data(), B, s);
}

void Trainer::fwd_step(int l, int t, hipStream_t s) {
  const int H = d_.H, B = Bp_;
  Layer& y = Ls_[l];
  FwdStepArgs a;
  a.hprev_bf = y.HSb + (size_t)t * B * H;
  a.hprev_f = y.HSf + (size_t)t * B * H;
  a.Whh = y.Whh;
  a.bhh = P("bias_hh_l" + std::to_string(l));
  if (l == 0) { a.P = Ptab_; a.ids = ids_ + (size_t)t * B; }
  else a.Gi = y.Gi + (size_t)t * B * 3 * H;
  a.h_f = y.HSf + (size_t)(t + 1) * B * H;
  a.h_bf = y.HSb + (size_t)(t + 1) * B * H;
  a.hT = y.HT; a.ldT = (d_.T + 1) * B; a.colT = (t + 1) * B;
  const size_t so = (size_t)t * B * H;
  if (y.s16 && !overlap_) a.s16 = y.s16 + so * 4;
  else { a.sr = y.sr + so; a.sz = y.sz + so; a.sn = y.sn + so; a.sghn = y.sghn + so; }
  a.Bp = B; a.H = H; a.algo = step_algo_;
  gru_fwd_step(a, s);
}

void Trainer::bwd_step(int l, int t, hipStream_t s) {
  const int H = d_.H, B = Bp_, T = d_.T;
  Layer& y = Ls_[l];
  BwdStepArgs a;
  const bool last = (t == T - 1);
  a.dgh_next = last ? nullptr : y.dgh[(t + 1) & 1];
  a.WhhT = y.WhhT;
  a.carry_in = last ? nullptr : y.carry[(t + 1) & 1];
  const size_t so = (size_t)t * B * H;
  a.dy = y.dy + so;
  a.r = y.sr + so; a.z = y.sz + so; a.n = y.sn + so; a.ghn = y.sghn + so;
  a.hprev = y.HSf + so;
  a.carry_out = y.carry[t & 1];
  a.dgh = y.dgh[t & 1];
  a.dghT = y.dghT; a.dgiT = y.dgiT; a.ldT = (int)ldG_; a.colT = t * B;
  a.dgi = y.dgi ? y.dgi + (size_t)t * B * 3 * H : nullptr;
  a.dgiT_n_only = l == 0 && dgiT_share_;
  a.Bp = B; a.H = H; a.algo = step_algo_;
  a.sk_part = sk_part_; a.sk_part_floats = sk_part_floats_; a.sk_cnt = sk_cnt_; a.sk_cnt_words = sk_cnt_words_;
  a.err = err_;
  gru_bwd_step(a, s);
}

void Trainer::record_fb(hipStream_t s0) {
  const int V = d_.V, E = d_.E, H = d_.H, T = d_.T, L = d_.L, B = Bp_, C = C_, Tc = Tc_;
  const int H3 = 3 * H;
  hipStream_t s1 = overlap_ ? s1_ : s0;   // serial mode: one stream, edges become no-ops
  ev_next_ = 0;
  std::vector<std::vector<hipEvent_t>> evDy(L, std::vector<hipEvent_t>(C, nullptr));
  auto edge = [&](hipStream_t from, hipStream_t to) {
    if (from == to) return;
    hipEvent_t e = ev();
    HIP_CHECK(hipEventRecord(e, from));
    HIP_CHECK(hipStreamWaitEvent(to, e, 0));
  };
  prep_batch(stage_src_, Bp_, T, Bp_, ids_, labels_, inv_count_, s0);
  if (carry_) record_carry(s0);
  edge(s0, s1);   // fork

  // layer-0 input projection folded into a [V][3H] table: Gi(t,b) = P[x(t,b)]  (exact: Emb[x]·W^T)
  {
    GemmArgs g;
    g.A = Emb; g.lda = E; g.B = Ls_[0].Wih; g.ldb = E; g.C = Ptab_; g.ldc = H3;
    g.bias = P("bias_ih_l0"); g.M = V; g.N = H3; g.K = E;
    gemm_nt(g, s0);
  }
  // ------------------------------------------------------------------ forward
  for (int l = 0; l < L; ++l) {
    Layer& y = Ls_[l];
    std::vector<hipEvent_t> evF(C);
    for (int c = 0; c < C; ++c) {
      if (l > 0) {
        // Gi for this chunk from the layer below (already complete: layers run in order on s0)
        GemmArgs g;
        g.A = Ls_[l - 1].HSb + (size_t)(1 + c * Tc) * B * H; g.lda = H;
        g.B = y.Wih; g.ldb = H;
        g.C = y.Gi + (size_t)c * Tc * B * H3; g.ldc = H3;
        g.bias = P("bias_ih_l" + std::to_string(l));
        g.M = Tc * B; g.N = H3; g.K = H;
        gemm_nt(g, s0);
      }
      for (int t = c * Tc; t < (c + 1) * Tc; ++t) fwd_step(l, t, s0);
      if (l == L - 1) {
        edge(s0, s1);
        const size_t t0 = (size_t)c * Tc * B;   // first token of the chunk
        FcXentArgs f;
        f.X = y.HSb + (t0 + B) * H; f.W = Wfc; f.b = P("fc.bias");
        f.labels = labels_ + t0; f.inv_count = inv_count_;
        f.dl = dl_ + t0 * V; f.dlT = dlT_; f.ldT = (int)ldG_; f.colT = (int)t0;
        f.loss_part = loss_part_ + t0 / 32;
        f.M = Tc * B; f.H = H; f.V = V;
        fc_xent(f, s1);
        GemmArgs g;   // dy_top = dlogits · W_fc
        g.A = dl_ + t0 * V; g.lda = V; g.B = WfcT; g.ldb = V;
        g.C = y.dy + t0 * H; g.ldc = H; g.M = Tc * B; g.N = H; g.K = V;
        gemm_nt(g, s1);
        GemmArgs w;   // dW_fc slab c (+ db_fc as row sums of dlogits^T)
        w.A = dlT_ + t0; w.lda = (int)ldG_; w.B = y.HT + t0 + B; w.ldb = (T + 1) * B;
        w.C = slab_fc_ + (size_t)c * V * H; w.ldc = H; w.rowsumA = rs_fc_ + (size_t)c * V;
        w.M = V; w.N = H; w.K = Tc * B;
        gemm_nt(w, s1);
        hipEvent_t e = ev();
        HIP_CHECK(hipEventRecord(e, s1));
        evDy[l][c] = e;   // (serial mode: recorded on s0 itself, the wait is a no-op)
      }
    }
  }
  // ------------------------------------------------------------------ backward (BPTT)
  for (int l = L - 1; l >= 0; --l) {
    Layer& y = Ls_[l];
    const int K = in_dim(l);
    for (int c = C - 1; c >= 0; --c) {
      HIP_CHECK(hipStreamWaitEvent(s0, evDy[l][c], 0));
      for (int t = (c + 1) * Tc - 1; t >= c * Tc; --t) bwd_step(l, t, s0);
      edge(s0, s1);
      const size_t t0 = (size_t)c * Tc * B;
      GemmArgs w;   // dW_hh slab c = dGh^T · h_{t-1}, db_hh = row sums of dGh^T
      w.A = y.dghT + t0; w.lda = (int)ldG_; w.B = y.HT + t0; w.ldb = (T + 1) * B;
      w.C = y.slab_hh + (size_t)c * H3 * H; w.ldc = H; w.rowsumA = y.rs_hh + (size_t)c * H3;
      w.M = H3; w.N = H; w.K = Tc * B;
      gemm_nt(w, s1);
      if (l == 0) {
        GemmArgs p;   // dP slab c = onehot(x)^T · dGi   ([V][3H]; gives dEmb, dW_ih0, db_ih0)
        p.onehot_ids = ids_ + t0; p.B = y.dgiT + t0; p.ldb = (int)ldG_;
        if (dgiT_share_) { p.B = y.dghT + t0; p.B2 = y.dgiT + t0; p.b2_row = 2 * H; }
        p.C = slab_P_ + (size_t)c * V * H3; p.ldc = H3; p.M = V; p.N = H3; p.K = Tc * B;
        gemm_nt(p, s1);
      } else {
        GemmArgs wi;  // dW_ih slab c = dGi^T · h_below
        wi.A = y.dgiT + t0; wi.lda = (int)ldG_; wi.B = Ls_[l - 1].HT + t0 + B; wi.ldb = (T + 1) * B;
        wi.C = y.slab_ih + (size_t)c * H3 * K; wi.ldc = K; wi.rowsumA = y.rs_ih + (size_t)c * H3;
        wi.M = H3; wi.N = K; wi.K = Tc * B;
        gemm_nt(wi, s1);
        GemmArgs dx;  // dy of the layer below = dGi · W_ih
        dx.A = y.dgi + t0 * H3; dx.lda = H3; dx.B = y.WihT; dx.ldb = H3;
        dx.C = Ls_[l - 1].dy + t0 * H; dx.ldc = H; dx.M = Tc * B; dx.N = H; dx.K = H3;
        gemm_nt(dx, s1);
        hipEvent_t e = ev();
        HIP_CHECK(hipEventRecord(e, s1));
        evDy[l - 1][c] = e;
      }
    }
  }
  // ------------------------------------------------------------------ finalize gradients (s1)
  {
    SlabJobs j;   // every split-K slab set -> its gradient segment, one launch
    j.add(slab_fc_, C, (long)V * H, G("fc.weight"));
    j.add(rs_fc_, C, V, G("fc.bias"));
    for (int l = 0; l < L; ++l) {
      const std::string k = std::to_string(l);
      j.add(Ls_[l].slab_hh, C, (long)H3 * H, G("weight_hh_l" + k));
      j.add(Ls_[l].rs_hh, C, H3, G("bias_hh_l" + k));
      if (l > 0) {
        j.add(Ls_[l].slab_ih, C, (long)H3 * in_dim(l), G("weight_ih_l" + k));
        j.add(Ls_[l].rs_ih, C, H3, G("bias_ih_l" + k));
      }
    }
    j.add(slab_P_, C, (long)V * H3, dP_);
    reduce_slabs_multi(j, s1);
  }
  {
    CastJobs j;
    j.add(dP_, V, H3, dP_bf_, dPT_bf_);
    cast_multi(j, s1);
  }
  colsum(dP_, V, H3, G("bias_ih_l0"), s1);
  {
    GemmArgs g;   // dW_ih0 = dP^T · Emb
    g.A = dPT_bf_; g.lda = V; g.B = EmbT; g.ldb = V; g.C = G("weight_ih_l0"); g.ldc = E;
    g.M = H3; g.N = E; g.K = V;
    gemm_nt(g, s1);
    GemmArgs e;   // dEmb = dP · W_ih0
    e.A = dP_bf_; e.lda = H3; e.B = Ls_[0].WihT; e.ldb = H3; e.C = G("embedding"); e.ldc = E;
    e.M = V; e.N = E; e.K = H3;
    gemm_nt(e, s1);
  }
  // loss = Σ partials (fixed order); also advances the optimiser's device step counter
  sum_partials(loss_part_, (int)((size_t)T * B / 32), loss_, s1, step_);
  edge(s1, s0);   // join
  HIP_LAUNCH_CHECK();
}

OptimArgs Trainer::optim_args() const {
  OptimArgs a;
  a.p = params_; a.g = grads_; a.m = m_; a.v = v_; a.n = nflat_; a.step = step_;
  a.gscale = o_.clip > 0.f ? gscale_ : nullptr;
  a.err = err_; a.err_host = err_host_dev_;
  a.lr = o_.lr; a.b1 = o_.b1; a.b2 = o_.b2; a.eps = o_.eps; a.wd = o_.wd; a.sgd = o_.sgd;
  a.sched = o_.sched; a.warmup = o_.warmup; a.total = o_.total; a.lr_min = o_.lr_min;
  a.keep_g = o_.keep_grads;
  return a;
}

void Trainer::set_shard_optim(int mode) {
  const bool on = mode != 0;
  if (mode < 0 || mode > 2) throw std::runtime_error("set_shard_optim: mode 0 (off), 1 (fp32 gather) or 2 (bf16 gather)");
  if (on && !comm_) throw std::runtime_error("set_shard_optim: needs a communicator (call set_comm first)");
  if (on && o_.clip > 0.f)
    throw std::runtime_error("set_shard_optim: gradient clipping needs the global norm; not supported sharded");
  if (on && nflat_ % 4) throw std::runtime_error("set_shard_optim: flat parameter count must be a multiple of 4");
  shard_opt_ = on;
  shard_mode_ = mode;
  if (on) {
    const int W = comm_->world();
    shard_chunk_ = nflat_ / (4L * W) * 4;
    if ((long)W * shard_chunk_ > 0 && shard_chunk_ > (1L << 30))
      throw std::runtime_error("set_shard_optim: shard too large for one optimiser job");
  }
  if (mode == 2) {
    if (d_.V % 64 || d_.E % 64 || d_.H % 64)
      throw std::runtime_error("set_shard_optim(2): the bf16 re-layout needs V, E, H % 64 == 0");
    branges_ = FlatRanges{};
    auto addr = [&](const std::string& k, int n) {
      if (branges_.cnt >= 16) throw std::runtime_error("set_shard_optim(2): too many bias tensors");
      branges_.off[branges_.cnt] = off_.at(k);
      branges_.n[branges_.cnt++] = n;
    };
    for (int l = 0; l < d_.L; ++l) {
      addr("bias_ih_l" + std::to_string(l), 3 * d_.H);
      addr("bias_hh_l" + std::to_string(l), 3 * d_.H);
    }
    addr("fc.bias", d_.V);
    if (!pbf_) HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&pbf_), (size_t)nflat_ * 2));
    if (!bpack_) HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&bpack_), (size_t)branges_.total() * 4));
  }
  g_step_[0].reset();
  g_step_[1].reset();
  g_group_[0].reset();
  g_group_[1].reset();
}

void Trainer::record_sharded_opt(hipStream_t s) {
  const int r = comm_->rank(), W = comm_->world();
  const long c = shard_chunk_, tail = nflat_ - (long)W * c;
  ar_log_.clear();
  // in-place reduce-scatter: the owned slice's mean lands at grads_ + r*c, where Adam reads it
  if (c > 0) comm_->reduce_scatter_avg_f32(grads_, grads_ + (long)r * c, c, s);
  if (tail > 0) {
    comm_->allreduce_avg_f32_err(grads_ + (long)W * c, tail, err_, s);
    ar_log_.push_back({(long)W * c, tail});
  } else {
    comm_->allreduce_max_u32(err_, 1, s);   // every rank skips a step that failed anywhere
  }
  // the fused optimiser launch's flat path (same update code as the replicated step), no casts:
  // the bf16 copies are refreshed from the gathered masters below
  OptCastJobs j;
  if (shard_mode_ == 2) {
    // mode 2: the owned slice's (and the tail's) bf16 working copy straight from Adam's registers;
    // all-gather those (half the bytes of the fp32 masters) with the owned fp32 biases packed beside
    // them, then re-derive every bf16 layout locally
    if (c > 0) j.add((long)r * c, 0, (int)c, pbf_ + (long)r * c, nullptr);
    if (tail > 0) j.add((long)W * c, 0, (int)tail, pbf_ + (long)W * c, nullptr);
    if (j.n) adam_cast_multi(optim_args(), j, s);
    const long nb = branges_.total();
    flat_pack_u32(params_, bpack_, branges_, (long)r * c, (long)(r + 1) * c, (long)W * c, 0, s);
    comm_->allgather_u16_sum_u32(pbf_ + (long)r * c, pbf_, c, bpack_, nb, s);   // one group launch
    flat_pack_u32(params_, bpack_, branges_, 0, 0, (long)W * c, 1, s);
    refresh_from_bf16(s);
    HIP_LAUNCH_CHECK();
    return;
  }
  if (c > 0) j.add((long)r * c, 0, (int)c, nullptr, nullptr);
  if (tail > 0) j.add((long)W * c, 0, (int)tail, nullptr, nullptr);   // every rank: the same tail
  if (j.n) adam_cast_multi(optim_args(), j, s);
  if (c > 0 && W > 1) comm_->allgather_f32(params_ + (long)r * c, params_, c, s);   // in place
  refresh_weights(s);
  HIP_LAUNCH_CHECK();
}

void Trainer::refresh_from_bf16(hipStream_t s) {
  // the refresh_weights layouts, from the gathered flat bf16 working copy (bitwise what the casts of
  // the fp32 masters give: rounding is per element)
  const int V = d_.V, E = d_.E, H = d_.H;
  auto B16 = [&](const std::string& k) { return pbf_ + off_.at(k); };
  CastJobs j;
  j.add16(B16("embedding"), V, E, Emb, EmbT);
  for (int l = 0; l < d_.L; ++l) {
    const std::string k = std::to_string(l);
    j.add16(B16("weight_hh_l" + k), 3 * H, H, Ls_[l].Whh, Ls_[l].WhhT);
    j.add16(B16("weight_ih_l" + k), 3 * H, in_dim(l), Ls_[l].Wih, Ls_[l].WihT);
  }
  j.add16(B16("fc.weight"), V, H, Wfc, WfcT, WfcF, WfcTF);
  cast_multi(j, s);
  HIP_LAUNCH_CHECK();
}

void Trainer::gather_params(hipStream_t s) {
  if (shard_mode_ != 2 || !comm_ || comm_->world() == 1 || shard_chunk_ == 0) return;
  const long c = shard_chunk_;
  comm_->allgather_f32(params_ + (long)comm_->rank() * c, params_, c, s);   // in place
}

void Trainer::gather_opt_state(hipStream_t s) {
  if (!shard_opt_ || !comm_ || comm_->world() == 1 || shard_chunk_ == 0) return;
  const long c = shard_chunk_, o = (long)comm_->rank() * c;
  comm_->allgather_f32(m_ + o, m_, c, s);
  comm_->allgather_f32(v_ + o, v_, c, s);
}

void Trainer::record_opt(hipStream_t s, int part) {
  if (part != 0 && o_.clip > 0.f)
    throw std::runtime_error("record_opt: a split optimiser launch cannot clip (needs the global norm)");
  if (o_.clip > 0.f) {
    sumsq_partials(grads_, nflat_, norm_parts_, 256, s);
    clip_scale_finalize(norm_parts_, 256, o_.clip, gscale_, s);
  }
  OptimArgs a = optim_args();
  const int V = d_.V, E = d_.E, H = d_.H;
  if (V % 64 == 0 && E % 64 == 0 && H % 64 == 0) {
    // one launch: update every tensor and write its bf16 (+ transposed) MFMA copies from the
    // freshly updated registers (no second pass over the fp32 master weights)
    OptCastJobs j;
    if (part != 2) {
      j.add(off_.at("embedding"), V, E, Emb, EmbT);
      for (int l = 0; l < d_.L; ++l) {
        const std::string k = std::to_string(l);
        j.add(off_.at("weight_hh_l" + k), 3 * H, H, Ls_[l].Whh, Ls_[l].WhhT);
        j.add(off_.at("weight_ih_l" + k), 3 * H, in_dim(l), Ls_[l].Wih, Ls_[l].WihT);
        j.add(off_.at("bias_ih_l" + k), 0, 3 * H, nullptr, nullptr);
        j.add(off_.at("bias_hh_l" + k), 0, 3 * H, nullptr, nullptr);
      }
    }
    if (part != 1) {
      // the plain W_fc / W_fc^T copies only where a kernel reads them: the fused V = 256 FC kernel of
      // the sequence step reads the fragment-tiled copies only
      const bool plain = overlap_ || fc_split_ || !(V == 256 && (H == 512 || H == 1024));
      j.add(off_.at("fc.weight"), V, H, plain ? Wfc : nullptr, plain ? WfcT : nullptr, WfcF, WfcTF);
      j.add(off_.at("fc.bias"), 0, V, nullptr, nullptr);
    }
    // deferred slab reductions: summed inside the Adam launch where a job covers exactly the
    // gradient segment; anything else is reduced first
    SlabJobs rest;
    for (int d = 0; d < deferred_.n; ++d) {
      const SlabJob& D = deferred_.job[d];
      bool used = false;
      for (int k = 0; k < j.n && !used; ++k) {
        OptCastJob& J = j.job[k];
        const long n = J.R ? (long)J.R * J.C : (long)J.C;
        if (!J.gsl && D.dst == grads_ + J.off && D.n == n && !D.bf && !D.bfT) {
          J.gsl = D.src; J.nsl = D.splits; used = true;
        }
      }
      if (!used) rest.job[rest.n++] = D;
    }
    if (rest.n) reduce_slabs_multi(rest, s);
    adam_cast_multi(a, j, s);
  } else {
    if (part != 0) throw std::runtime_error("record_opt: split optimiser launches need V, E, H % 64 == 0");
    if (deferred_.n) reduce_slabs_multi(deferred_, s);
    adam_step(a, s);
    refresh_weights(s);
  }
  deferred_.n = 0;
  HIP_LAUNCH_CHECK();
}

void Trainer::forward_backward(hipStream_t s) {
  GK_TRACE("gk.forward_backward");
  const int slot = stage_slot_;
  stage_src_ = dev_slot(slot);
  HIP_CHECK(hipStreamWaitEvent(s, copy_done_[slot], 0));
  if (!use_graph_) {
    // eager: run on the internal streams, ordered after / before the caller's stream
    hipEvent_t a = events_.back();
    HIP_CHECK(hipEventRecord(a, s));
    HIP_CHECK(hipStreamWaitEvent(s0_, a, 0));
    if (overlap_) record_fb(s0_); else record_fb_seq(s0_);
    HIP_CHECK(hipEventRecord(a, s0_));
    HIP_CHECK(hipStreamWaitEvent(s, a, 0));
  } else {
    if (!g_fb_[slot].ready()) {
      g_fb_[slot].begin(s0_);
      if (overlap_) record_fb(s0_); else record_fb_seq(s0_);
      g_fb_[slot].end(s0_);
    }
    g_fb_[slot].launch(s);
  }
  HIP_CHECK(hipEventRecord(stage_done_[slot], s));
}

void Trainer::optimizer_step(hipStream_t s) {
  GK_TRACE("gk.optimizer_step");
  if (!use_graph_) { record_opt(s); return; }
  if (!g_opt_.ready()) {
    g_opt_.begin(s0_);
    record_opt(s0_);
    g_opt_.end(s0_);
  }
  g_opt_.launch(s);
}

void Trainer::set_comm(RcclComm* c, const std::vector<std::pair<long, long>>& buckets, long min_bucket_floats) {
  comm_ = c;
  if (!c) shard_opt_ = false;
  buckets_ = buckets;
  min_bucket_ = std::max(1L, min_bucket_floats);
  // the overlapped path relies on the readiness order of the flat layout (models/params.py)
  const int L = d_.L;
  long prev = off_.at("fc.weight");
  bool ok = prev == 0 && off_.at("fc.bias") > prev;
  prev = off_.at("fc.bias");
  for (int l = L - 1; l >= 0; --l) {
    const std::string k = std::to_string(l);
    for (const char* n : {"weight_hh_l", "bias_hh_l", "bias_ih_l", "weight_ih_l"}) {
      const long o = off_.at(n + k);
      ok = ok && o > prev;
      prev = o;
    }
  }
  ok = ok && off_.at("embedding") > prev;
  if (!ok) throw std::runtime_error("set_comm: flat gradient layout is not in readiness order");
  // dP [V][3H] goes into the W_ih0 gradient slot when it fits (one contiguous collective)
  dP_inplace_ = (long)d_.V * 3 * d_.H <= 3L * d_.H * d_.E;
  g_step_[0].reset();
  g_step_[1].reset();
  g_group_[0].reset();
  g_group_[1].reset();
}

void Trainer::set_dp_pipeline(int mode) {
  if (mode < -1 || mode > 1) throw std::runtime_error("set_dp_pipeline: -1 (auto), 0 or 1");
  dp_pipe_ = mode;
  g_step_[0].reset();
  g_step_[1].reset();
  g_group_[0].reset();
  g_group_[1].reset();
}

bool Trainer::dp_pipe_on() const {
  if (!comm_ || overlap_ || shard_opt_ || d_.L != 1 || o_.clip > 0.f) return false;
  const int V = d_.V, E = d_.E, H = d_.H;
  if (V % 64 || E % 64 || H % 64 || !dP_inplace_) return false;
  // auto (-1) is OFF: on a 1-rank communicator the pipelined tail measured 0.2524 against 0.2215 ms per
  // step -- every cross-stream edge of the captured graph opened a 5-10 us gap and the dW_fc K-slices
  // did not start before AR1 had ended (profiles/r5_rccl_self_dp_pipeline{1,0}_timeline.txt)
  return dp_pipe_ == 1;
}

long Trainer::group_end(int l) const {
  if (l >= d_.L) return off_.at("weight_hh_l" + std::to_string(d_.L - 1));   // FC group
  if (l > 0) return off_.at("weight_hh_l" + std::to_string(l - 1));
  return off_.at("weight_ih_l0") + (dP_inplace_ ? (long)d_.V * 3 * d_.H : 0L);
}

bool Trainer::ar_flush(hipStream_t s, bool force, bool with_err) {
  const long n = ar_ready_ - ar_launched_;
  if (n <= 0 || (!force && n < min_bucket_)) return false;
  auto reduce = [&](hipStream_t st) {
    if (with_err) comm_->allreduce_avg_f32_err(grads_ + ar_launched_, n, err_, st);
    else comm_->allreduce_avg_f32(grads_ + ar_launched_, n, st);
  };
  hipEvent_t e = ev();
  HIP_CHECK(hipEventRecord(e, s));          // fork: everything recorded on s so far
  HIP_CHECK(hipStreamWaitEvent(sc_, e, 0));
  reduce(sc_);
  ar_log_.push_back({ar_launched_, n});
  ar_launched_ = ar_ready_;
  ar_busy_ = true;
  return true;
}

void Trainer::ar_join(hipStream_t s) {
  if (!ar_busy_) return;
  hipEvent_t e = ev();
  HIP_CHECK(hipEventRecord(e, sc_));
  HIP_CHECK(hipStreamWaitEvent(s, e, 0));
  ar_busy_ = false;
}

void Trainer::record_allreduce(hipStream_t s) {
  // plain bucketed mean all-reduce of the whole flat fp32 gradient after the backward; the last
  // bucket carries the error word (max over ranks) so every rank skips a failed step together
  if (!comm_) return;
  for (size_t i = 0; i < buckets_.size(); ++i) {
    const auto& b = buckets_[i];
    if (i + 1 == buckets_.size()) comm_->allreduce_avg_f32_err(grads_ + b.first, b.second, err_, s);
    else comm_->allreduce_avg_f32(grads_ + b.first, b.second, s);
  }
  if (buckets_.empty()) comm_->allreduce_max_u32(err_, 1, s);
}

void Trainer::enable_watchdog(int timeout_ms) {
  wd_.reset();
  if (timeout_ms >= 0) {   // 0: no step deadline, still the communicator and the step error word
    wd_ = std::make_unique<Watchdog>(comm_, timeout_ms);
    wd_->set_error_word(err_host_);
  }
}

void Trainer::step(hipStream_t s) {
  GK_TRACE("gk.train_step");
  if (!use_graph_) {
    forward_backward(s);
    record_allreduce(s);
    optimizer_step(s);
    if (wd_) { HIP_CHECK(hipEventRecord(stage_done_[stage_slot_], s)); wd_->watch(stage_done_[stage_slot_]); }
    return;
  }
  const int slot = stage_slot_;
  stage_src_ = dev_slot(slot);
  HIP_CHECK(hipStreamWaitEvent(s, copy_done_[slot], 0));
  Graph& g = g_step_[slot];
  if (!g.ready()) {
    GK_TRACE("gk.capture_step_graph");
    g.begin(s0_);
    try {
      record_step_body();
    } catch (...) {
      defer_slabs_ = false;
      deferred_.n = 0;
      hipGraph_t broken = nullptr;          // leave the stream out of capture mode, then rethrow
      (void)hipStreamEndCapture(s0_, &broken);
      if (broken) (void)hipGraphDestroy(broken);
      (void)hipGetLastError();
      throw;
    }
    g.end(s0_);
  }
  g.launch(s);
  HIP_CHECK(hipEventRecord(stage_done_[slot], s));
  if (wd_) wd_->watch(stage_done_[slot]);
}

void Trainer::set_graph_steps(int G) {
  if (G < 1 || G > kMaxGroup) throw std::runtime_error("set_graph_steps: 1.." + std::to_string(kMaxGroup));
  group_ = G;
  g_group_[0].reset();
  g_group_[1].reset();
}

void Trainer::set_batches(const int* x, const int* y, int B, int n) {
  if (n != group_) throw std::runtime_error("set_batches: expected " + std::to_string(group_) + " batches");
  if (B > Bp_ || B <= 0) throw std::runtime_error("set_batches: batch larger than the trainer was built for");
  const int gp = (group_parity_ ^= 1);
  HIP_CHECK(hipEventSynchronize(group_done_[gp]));   // the group graph that last read these slots is done
  const size_t per = (size_t)B * d_.T;
  for (int j = 0; j < n; ++j) fill_slot(group_slot(gp, j), x + j * per, y + j * per, B);
  copy_slots(group_slot(gp, 0), n, group_copy_done_[gp]);   // the group's slots are contiguous
}

void Trainer::step_group(hipStream_t s) {
  GK_TRACE("gk.train_step_group");
  if (!use_graph_) throw std::runtime_error("step_group: needs graph mode");
  const int gp = group_parity_;
  Graph& g = g_group_[gp];
  if (!g.ready()) {
    GK_TRACE("gk.capture_group_graph");
    g.begin(s0_);
    try {
      for (int j = 0; j < group_; ++j) {
        stage_src_ = dev_slot(group_slot(gp, j));
        record_step_body();
      }
    } catch (...) {
      defer_slabs_ = false;
      deferred_.n = 0;
      hipGraph_t broken = nullptr;
      (void)hipStreamEndCapture(s0_, &broken);
      if (broken) (void)hipGraphDestroy(broken);
      (void)hipGetLastError();
      throw;
    }
    g.end(s0_);
  }
  HIP_CHECK(hipStreamWaitEvent(s, group_copy_done_[gp], 0));
  g.launch(s);
  HIP_CHECK(hipEventRecord(group_done_[gp], s));
  if (wd_) wd_->watch(group_done_[gp]);
}

void Trainer::record_step_body() {
  if (shard_opt_) {
    // sharded optimiser: whole backward first (slab sums into the flat gradient), then
    // reduce-scatter -> Adam on the owned slice -> all-gather -> bf16 refresh
    deferred_.n = 0;
    if (overlap_) record_fb(s0_); else record_fb_seq(s0_);
    record_sharded_opt(s0_);
    return;
  }
  deferred_.n = 0;
  opt_in_fb_ = false;
  if (dp_overlap()) {
    // readiness-ordered collectives on the comm stream, overlapped with the rest of the
    // backward; joined before the optimiser (the embedding-side tail runs after the join)
    record_fb_seq(s0_, /*dp=*/true);
    if (opt_in_fb_) { opt_in_fb_ = false; return; }   // the pipelined tail recorded its own Adam launches
  } else {
    defer_slabs_ = !overlap_ && !comm_ && o_.clip <= 0.f;
    if (overlap_) record_fb(s0_); else record_fb_seq(s0_);
    defer_slabs_ = false;
    record_allreduce(s0_);
  }
  record_opt(s0_);
}

float Trainer::read_loss() {
  float v = 0.f;
  if (read_error())
    throw std::runtime_error("[rank " + std::to_string(global_rank()) +
                             "] a cross-workgroup wait hit its spin limit (persistent sequence kernel: error bit 1, "
                             "split-K backward step kernel: bit 2; workgroups not co-resident?)");
  HIP_CHECK(hipMemcpy(&v, loss_, 4, hipMemcpyDeviceToHost));
  return v;
}

int Trainer::get_step() {
  int v = 0;
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(&v, step_, 4, hipMemcpyDeviceToHost));
  return v;
}

void Trainer::set_step(int v) {
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(step_, &v, 4, hipMemcpyHostToDevice));
}

float Trainer::read_grad_norm() {
  float v[2] = {0.f, 0.f};
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(v, gscale_, 8, hipMemcpyDeviceToHost));
  return v[1];
}

uintptr_t Trainer::buffer(const std::string& n) const {
  auto u = [](const void* p) { return reinterpret_cast<uintptr_t>(p); };
  if (n == "ids") return u(ids_);
  if (n == "labels") return u(labels_);
  if (n == "P") return u(Ptab_);
  if (n == "loss") return u(loss_);
  if (n == "dl") return u(dl_);
  if (n == "step") return u(step_);
  if (n == "err") return u(err_);
  if (n.rfind("HSf", 0) == 0) return u(Ls_.at(std::stoi(n.substr(3))).HSf);
  if (n.rfind("dy", 0) == 0) return u(Ls_.at(std::stoi(n.substr(2))).dy);
  throw std::runtime_error("unknown buffer " + n);
}

}  // namespace gk
