#include "generator.h"
#include "../runtime/trace.h"
#include "../runtime/blaslt.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace gk {

static int rup(int x, int m) { return (x + m - 1) / m * m; }

Generator::Generator(const GenDims& d, const float* params, const std::map<std::string, long>& offsets)
    : d_(d), params_(params), off_(offsets) {
  if (d_.V % 64 || d_.E % 64 || d_.H % 64)
    throw std::runtime_error("HIP generator needs vocab, embed and hidden to be multiples of 64");
  blaslt_init();   // before any graph capture (large prep GEMMs may go to the library)
  Bmax_ = rup(std::max(32, d_.max_batch), 64);
  const int V = d_.V, E = d_.E, H = d_.H, L = d_.L, B = Bmax_;
  std::vector<size_t> ohf, ohb, oWhh, oWih;
  // bf16x3: the bf16 weight / state copies hold split rows ([hi | lo | hi] / [hi | hi | lo], 3x wide)
  const size_t xw = d_.fp32 == 2 ? 3 : 1;
  for (int i = 0; i < 2 * L; ++i) { ohf.push_back(arena_.reserve((size_t)B * H * 4)); ohb.push_back(arena_.reserve((size_t)B * H * 2 * xw)); }
  for (int l = 0; l < L; ++l) {
    oWhh.push_back(arena_.reserve((size_t)3 * H * H * 2 * xw));
    oWih.push_back(arena_.reserve((size_t)3 * H * (l == 0 ? E : H) * 2 * xw));
  }
  size_t oEmb = arena_.reserve((size_t)V * E * 2), oWfc = arena_.reserve((size_t)V * H * 2 * xw);
  size_t oWfcF = arena_.reserve((size_t)V * H * 2);   // fragment-tiled copy for the 8-wave sampler
  size_t oP = arena_.reserve((size_t)V * 3 * H * 4), orf = arena_.reserve((size_t)B * d_.max_len * 4);
  size_t oids = arena_.reserve((size_t)B * 4), oal = arena_.reserve((size_t)B * 4);
  size_t oout = arena_.reserve((size_t)B * (d_.max_len + 1));
  size_t ogh = 0, ogi = 0, olg = 0, oerr = arena_.reserve(256), opws = 0, opsync = 0;
  // persistent small-batch path (every mode): exchange buffers, flags, and in bf16 mode an fp32
  // layer-0 table of its own (Ptab_ holds the bf16-product one there)
  opws = arena_.reserve((size_t)gen_persist_ws_floats(H, L, V, d_.max_len) * 4);
  opsync = arena_.reserve((size_t)gen_persist_sync_words(L) * 4);
  const size_t oP32 = d_.fp32 ? 0 : arena_.reserve((size_t)V * 3 * H * 4);
  if (d_.fp32) {
    // room for split-K slabs of small batches (f32_splits / split3_splits): kF32SlabRows rows
    const size_t rows = std::max<size_t>(B, kF32SlabRows);
    ogh = arena_.reserve(rows * 3 * H * 4);
    ogi = arena_.reserve(rows * 3 * H * 4);
    olg = arena_.reserve(rows * V * 4);
  }
  arena_.commit();
  err_ = arena_.get<unsigned>(oerr);
  pws_ = arena_.get<float>(opws); psync_ = arena_.get<unsigned>(opsync);
  if (d_.fp32) { gh_ = arena_.get<float>(ogh); gi_ = arena_.get<float>(ogi); logits_ = arena_.get<float>(olg); }
  for (int i = 0; i < 2 * L; ++i) { hf_.push_back(arena_.get<float>(ohf[i])); hb_.push_back(arena_.get<u16>(ohb[i])); }
  for (int l = 0; l < L; ++l) { Whh_.push_back(arena_.get<u16>(oWhh[l])); Wih_.push_back(arena_.get<u16>(oWih[l])); }
  Emb_ = arena_.get<u16>(oEmb); Wfc_ = arena_.get<u16>(oWfc); WfcF_ = arena_.get<u16>(oWfcF);
  Ptab_ = arena_.get<float>(oP);
  Ptab32_ = d_.fp32 ? Ptab_ : arena_.get<float>(oP32);
  rf_ = arena_.get<float>(orf); ids_ = arena_.get<int>(oids); alive_ = arena_.get<int>(oal);
  out_ = arena_.get<unsigned char>(oout);
  HIP_CHECK(hipStreamCreateWithFlags(&cap_, hipStreamNonBlocking));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_pin_), 64, hipHostMallocDefault));
  const char* ng = std::getenv("GK_NO_GRAPH");
  if (ng && ng[0] == '1') use_graph_ = false;
  if (const char* sa = std::getenv("GK_STEP_ALGO")) step_algo_ = std::atoi(sa);   // 0 auto, 1 reg, 2 LDS
  const char* gp = std::getenv("GK_GEN_PERSIST");
  if (gp && gp[0] == '0') persist_ = false;
}

bool Generator::uses_persist(int n) const {
  // bf16 mode: only where the persistent fp32 launch is faster than the bf16 per-char graph (up to
  // 40 names: 29.0 vs 33.2 us per char at 32, 33.7 vs 34.0 at 40, 34.8 vs 34.6 at 48 on the
  // reference model, launches included, profiles/r5_gen_persist_vs_bf16_graph.jsonl)
  // The bf16 mode's choice is PRECISION-visible (the persistent launch runs exact fp32), so it follows
  // the job's global name count when the caller gave one (set_global_names): a data-parallel call
  // then picks the same arithmetic on every world size.  fp32 mode: both paths are fp32.
  if (!d_.fp32 && std::max(n, global_n_) > persist_max_bf16_) return false;
  return persist_ && n <= persist_max_ && gen_persist_supported(d_.H, d_.L, d_.V, n, d_.max_len);
}

Generator::~Generator() {
  graphs_.clear();
  if (cap_) (void)hipStreamDestroy(cap_);
  if (err_pin_) (void)hipHostFree(err_pin_);
}

void Generator::refresh_weights(hipStream_t s) {
  const int V = d_.V, E = d_.E, H = d_.H;
  if (d_.fp32) {   // fp32 layer-0 table P = Emb · W_ih0^T + b_ih0 from the master weights
    GemmF32Args g;
    g.A = P("embedding"); g.lda = E; g.B = P("weight_ih_l0"); g.ldb = E; g.C = Ptab_; g.ldc = 3 * H;
    g.bias = P("bias_ih_l0"); g.M = V; g.N = 3 * H; g.K = E;
    gemm_f32_nt(g, s);
    if (split3()) {   // the products' weight operands: [hi | lo | hi] rows
      for (int l = 0; l < d_.L; ++l) {
        const std::string k = std::to_string(l);
        split_bf16x3(P("weight_hh_l" + k), 3 * H, H, Whh_[l], s);
        if (l > 0) split_bf16x3(P("weight_ih_l" + k), 3 * H, H, Wih_[l], s);
      }
      split_bf16x3(P("fc.weight"), V, H, Wfc_, s);
    }
    HIP_LAUNCH_CHECK();
    return;
  }
  CastJobs j;
  j.add(P("embedding"), V, E, Emb_, nullptr);
  for (int l = 0; l < d_.L; ++l) {
    const std::string k = std::to_string(l);
    j.add(P("weight_hh_l" + k), 3 * H, H, Whh_[l], nullptr);
    j.add(P("weight_ih_l" + k), 3 * H, l == 0 ? E : H, Wih_[l], nullptr);
  }
  j.add(P("fc.weight"), V, H, Wfc_, nullptr, (V % 64 || H % 64) ? nullptr : WfcF_);
  cast_multi(j, s);
  {   // fp32 table for the persistent small-batch launch (exact fp32 there)
    GemmF32Args g;
    g.A = P("embedding"); g.lda = E; g.B = P("weight_ih_l0"); g.ldb = E; g.C = Ptab32_; g.ldc = 3 * H;
    g.bias = P("bias_ih_l0"); g.M = V; g.N = 3 * H; g.K = E;
    gemm_f32_nt(g, s);
  }
  GemmArgs g;   // layer-0 input projection table P = Emb · W_ih0^T + b_ih0  ([V][3H])
  g.A = Emb_; g.lda = E; g.B = Wih_[0]; g.ldb = E; g.C = Ptab_; g.ldc = 3 * H;
  g.bias = P("bias_ih_l0"); g.M = V; g.N = 3 * H; g.K = E;
  gemm_nt(g, s);
  HIP_LAUNCH_CHECK();
}

// Per-batch state reset as one kernel node.  Replays of a graph whose reset was five memset
// nodes (h, ids, alive, out) left stale and garbage ids in the padded rows of the fp32 path and
// made replays disagree (scripts/repro_gen_fp32.py with SYNC_FIRST=1: error word 16, replays not
// identical); a kernel node is ordered like every other node of the chain.
void Generator::reset_batch(int Bp, bool bf16, hipStream_t s) {
  // (round 3's memset-node diagnostics, scripts/gpu_graph_fault3.sh, profiles/r3_graph_replay.md)
  GenResetArgs r;
  r.L = d_.L; r.Bp = Bp; r.H = d_.H; r.ML = d_.max_len; r.sos = d_.sos;
  r.hb_cols = split3() ? 3 * d_.H : d_.H;
  for (int l = 0; l < d_.L; ++l) {
    r.hf[l] = hf_[2 * l];
    r.hb[l] = (bf16 || split3()) ? hb_[2 * l] : nullptr;
  }
  r.ids = ids_; r.alive = alive_; r.out = out_;
  gen_reset(r, s);
}

void Generator::record_steps(int n, hipStream_t s) {
  const int H = d_.H, L = d_.L, V = d_.V, ML = d_.max_len;
  const int Bp = rup(n, 32);
  // per-batch init (part of the graph): h = 0, input = SOS, alive = 1, output rows = NUL
  reset_batch(Bp, true, s);
  for (int st = 0; st < ML; ++st) {
    const int cur = st & 1, nxt = cur ^ 1;
    for (int l = 0; l < L; ++l) {
      const std::string k = std::to_string(l);
      FwdStepArgs a;
      a.hprev_bf = hb_[2 * l + cur]; a.hprev_f = hf_[2 * l + cur];
      a.Whh = Whh_[l]; a.bhh = P("bias_hh_l" + k);
      if (l == 0) { a.P = Ptab_; a.ids = ids_; }
      else { a.x_bf = hb_[2 * (l - 1) + nxt]; a.Wih = Wih_[l]; a.bih = P("bias_ih_l" + k); a.Kin = H; }
      a.h_f = hf_[2 * l + nxt]; a.h_bf = hb_[2 * l + nxt];
      a.Bp = Bp; a.H = H; a.algo = step_algo_;
      gru_fwd_step(a, s);
    }
    FcSampleArgs f;
    f.X = hb_[2 * (L - 1) + nxt]; f.W = Wfc_; f.Wf = WfcF_; f.b = P("fc.bias"); f.rf = rf_;
    f.ids = ids_; f.out = out_; f.alive = alive_; f.probs = (st == ML - 1) ? probe_ : nullptr;
    f.N = n; f.Bp = Bp; f.H = H; f.V = V; f.step = st; f.max_len = ML; f.eos = d_.eos;
    fc_sample(f, s);
  }
  HIP_LAUNCH_CHECK();
}

// fp32-faithful step: per layer gh = h W_hh^T + b_hh (and gi = x W_ih^T + b_ih above layer 0) as
// fp32 MFMA GEMMs on the master weights, the gates in IEEE fp32, then logits = h W_fc^T + b_fc and
// the fp32 softmax sampler -- the reference's per-char arithmetic (namegensf.cu:669-876) batched
// Split-K depth of a small-batch fp32 GEMM: enough 64 x 64 tiles x slabs to fill the chip
// (<= 512 workgroups), K-slices >= 64 deep, slabs within the buffer; 1 for big batches.
static int f32_splits(int M, int N, int K, int rows_cap) {
  const int tiles = (M / 64) * (N / 64);
  int sp = 1;
  while (sp < 32 && tiles * sp * 2 <= 512 && K % (sp * 2) == 0 && (K / (sp * 2)) % 16 == 0 &&
         K / (sp * 2) >= 64 && M * sp * 2 <= rows_cap)
    sp *= 2;
  return sp;
}

// bf16x3 split-K depth: unsplit when the LDS-staged kernels get a grid (>= 128 tiles of 128 x 128),
// else the one-shot small GEMM over the smallest K-slice count that gives ~256 workgroups (slices
// it supports: 2-4 or 8 k-blocks of 64, or whole multiples of 8 up to 32); slabs within rows_cap
static int split3_splits(int M, int N, int K3, int rows_cap) {
  if (M % 128 == 0 && N % 128 == 0 && (M / 128) * (N / 128) >= 128) return 1;
  const int tiles = (M / 64) * (N / 64);
  int last = 1;
  for (int sp = 2; sp <= 32; ++sp) {
    if (K3 % sp || (K3 / sp) % 64 || M * sp > rows_cap) continue;
    const int nkb = K3 / sp / 64;
    if (!(nkb == 2 || nkb == 3 || nkb == 4 || nkb == 8 || (nkb % 8 == 0 && nkb <= 32))) continue;
    last = sp;
    if (tiles * sp >= 256) return sp;
  }
  return last;
}

int Generator::product_f32(const float* A32, const u16* A3, const float* W32, const u16* W3, const float* bias, int M,
                           int N, float* C, hipStream_t s) {
  const int H = d_.H;
  const int cap = std::max(Bmax_, kF32SlabRows);
  if (!split3()) {
    GemmF32Args g;
    g.A = A32; g.lda = H; g.B = W32; g.ldb = H; g.C = C; g.ldc = N;
    g.bias = bias; g.M = M; g.N = N; g.K = H;
    g.splits = f32_splits(M, N, H, cap); g.slab = (long)M * N;
    gemm_f32_nt(g, s);
    return g.splits;
  }
  GemmArgs g;
  g.A = A3; g.lda = 3 * H; g.B = W3; g.ldb = 3 * H; g.C = C; g.ldc = N;
  g.M = M; g.N = N; g.K = 3 * H;
  g.splits = split3_splits(M, N, 3 * H, cap);
  if (g.splits == 1) {
    g.bias = bias;   // split: the consumer adds the bias after the slab sum
    // the 256 x 256 kernel from 3/4 of a wave of its tiles (4096 names x 3H: 192 tiles), where the
    // 128 x 128 kernel's 1.5 rounds of 512 slots leave as much idle
    if (M % 256 == 0 && N % 256 == 0 && (M / 256) * (N / 256) >= 192) g.algo = 5;
  } else {
    g.algo = 3;
  }
  gemm_nt(g, s);
  return g.splits;
}

void Generator::record_steps_f32(int n, hipStream_t s) {
  const int H = d_.H, L = d_.L, V = d_.V, ML = d_.max_len;
  const int Bp = rup(n, 64);
  const bool x3 = split3();
  reset_batch(Bp, false, s);
  for (int st = 0; st < ML; ++st) {
    const int cur = st & 1, nxt = cur ^ 1;
    for (int l = 0; l < L; ++l) {
      const std::string k = std::to_string(l);
      const float* bh = P("bias_hh_l" + k);
      const int sh = product_f32(hf_[2 * l + cur], hb_[2 * l + cur], P("weight_hh_l" + k), Whh_[l], bh, Bp, 3 * H, gh_, s);
      GruGatesF32Args a;
      if (l == 0) {
        a.P = Ptab_; a.ids = ids_;
      } else {
        const float* bi = P("bias_ih_l" + k);
        const int si = product_f32(hf_[2 * (l - 1) + nxt], hb_[2 * (l - 1) + nxt], P("weight_ih_l" + k), Wih_[l], bi,
                                   Bp, 3 * H, gi_, s);
        a.Gi = gi_; a.gi_splits = si; a.gi_slab = (long)Bp * 3 * H;
        if (x3 && si > 1) a.bgi = bi;
      }
      a.Gh = gh_; a.gh_splits = sh; a.gh_slab = (long)Bp * 3 * H; a.hprev = hf_[2 * l + cur]; a.hout = hf_[2 * l + nxt];
      if (x3 && sh > 1) a.bgh = bh;
      if (x3) a.hsplit = hb_[2 * l + nxt];
      a.Bp = Bp; a.H = H; a.V = V; a.err = err_;
      gru_gates_f32(a, s);
    }
    const float* bf = P("fc.bias");
    const int sf = product_f32(hf_[2 * (L - 1) + nxt], hb_[2 * (L - 1) + nxt], P("fc.weight"), Wfc_, bf, Bp, V, logits_, s);
    SampleF32Args q;
    q.logits = logits_; q.splits = sf; q.slab = (long)Bp * V; q.rf = rf_; q.ids = ids_; q.out = out_; q.alive = alive_;
    if (x3 && sf > 1) q.bias = bf;
    q.probs = (st == ML - 1) ? probe_ : nullptr;
    q.N = n; q.V = V; q.step = st; q.max_len = ML; q.eos = d_.eos;
    sample_f32(q, s);
  }
  HIP_LAUNCH_CHECK();
}

void Generator::generate(const float* rf, int N, unsigned char* out, hipStream_t s) {
  GK_TRACE("gk.generate");
  const int ML = d_.max_len;
  // the error word covers the whole call: every batch ORs its bits in, read_error() reports them all
  // (a persistent launch's spin-limit bit 32 is taken out again below once its batch is regenerated)
  if (!err_clean_) HIP_CHECK(hipMemsetAsync(err_, 0, 16, s));
  err_clean_ = false;
  for (int start = 0; start < N; start += Bmax_) {
    const int n = std::min(Bmax_, N - start);
    bool persist_done = false;
    if (uses_persist(n)) {   // one launch for the whole batch: no graph needed
      GenPersistArgs a;
      for (int l = 0; l < d_.L; ++l) {
        const std::string k = std::to_string(l);
        a.Whh[l] = P("weight_hh_l" + k); a.bhh[l] = P("bias_hh_l" + k);
        if (l > 0) { a.Wih[l] = P("weight_ih_l" + k); a.bih[l] = P("bias_ih_l" + k); }
      }
      // the caller's uniforms and output rows directly (no staging copies: two fewer stream
      // operations per call on the latency-bound small-batch path)
      a.Wfc = P("fc.weight"); a.bfc = P("fc.bias"); a.P = Ptab32_; a.probs = probe_;
      a.rf = rf + (size_t)start * ML; a.out = out + (size_t)start * (ML + 1);
      a.ws = pws_; a.sync = psync_; a.err = err_; a.dbg = persist_dbg_;
      if (ppar_ < 0) {   // first launch: both sets' tagged slots -> kEmpty; later launches refill in-kernel
        gen_persist_fill_ws(pws_, d_.H, d_.L, d_.V, ML, s);
        ppar_ = 0;
      }
      a.par = ppar_;
      ppar_ ^= 1;
      a.N = n; a.H = d_.H; a.L = d_.L; a.V = d_.V; a.ML = ML; a.sos = d_.sos; a.eos = d_.eos;
      if (inject_) {   // test hook: OR the spin-limit bit into the word (earlier batches' bits stay)
        unsigned cur = 0;
        HIP_CHECK(hipMemcpyAsync(&cur, err_, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        cur |= 32u;
        HIP_CHECK(hipMemcpyAsync(err_, &cur, 4, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
        inject_ = false;
      }
      gen_persist_f32(a, s);
      // small batch, latency-bound launch: check its error word now.  A spin timeout means the
      // workgroups were not co-resident (something else held CUs): the batch's output is garbage,
      // so say so, stop using the persistent path and regenerate the batch on the per-char graph.
      // (pinned host word: 138 vs 146-150 us per 1-name call against a pageable one; skipping the
      // next call's memset after a clean call another ~2 us: profiles/r5_gen_err_readback_ab.txt)
      HIP_CHECK(hipMemcpyAsync(err_pin_, err_, 4, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      const unsigned e = *reinterpret_cast<volatile unsigned*>(err_pin_);
      if (e == 0 && start + n >= N) err_clean_ = true;   // the call ends here, word still 0
      persist_done = !(e & 32u);
      if (!persist_done) {
        std::fprintf(stderr, "[generator] persistent launch hit its spin limit (error word %u): "
                             "disabling it, regenerating %d names on the per-char graph\n", e, n);
        persist_ = false;
        const unsigned keep = e & ~32u;   // the other bits stay (earlier batches' errors)
        HIP_CHECK(hipMemcpy(err_, &keep, 4, hipMemcpyHostToDevice));
      }
    }
    if (persist_done) continue;   // rows already in `out`
    HIP_CHECK(hipMemcpyAsync(rf_, rf + (size_t)start * ML, (size_t)n * ML * 4, hipMemcpyDeviceToDevice, s));
    if (use_graph_) {
      auto& g = graphs_[n];
      if (!g) {
        g.reset(new Graph());
        g->begin(cap_);
        if (d_.fp32) record_steps_f32(n, cap_); else record_steps(n, cap_);
        g->end(cap_);
      }
      g->launch(s);
    } else {
      if (d_.fp32) record_steps_f32(n, s); else record_steps(n, s);
    }
    HIP_CHECK(hipMemcpyAsync(out + (size_t)start * (ML + 1), out_, (size_t)n * (ML + 1), hipMemcpyDeviceToDevice, s));
  }
}

unsigned Generator::read_error() {
  unsigned e[4] = {0, 0, 0, 0};
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(e, err_, 16, hipMemcpyDeviceToHost));
  // reporting is the caller's (HipGenerator / the C API raise or print it); the detail line is a debug aid
  const char* dbg = std::getenv("GK_GEN_DEBUG");
  if (e[0] && dbg && dbg[0] && dbg[0] != '0')
    std::fprintf(stderr, "[generator] error word %u: id %d (0x%08x) at row %u\n", e[0], (int)e[1], e[1], e[2]);
  return e[0];
}

}  // namespace gk
