// Native training-step executor (SURVEY §3.5 train_step, §7.1 engine/trainer).
//
// One Trainer per process/GPU.  It owns the whole BPTT working set in one device arena and
// records a full forward + loss + backward + weight-gradient step as ONE hipGraph over two
// HIP streams:
//   s0  the serial critical path: per-timestep recurrent kernels, forward then backward;
//   s1  everything that only *consumes* a finished time chunk: FC + softmax-xent + dH for
//       chunk c while s0 is still stepping chunk c+1 forward, and the split-K weight-gradient
//       GEMMs of chunk c while s0 steps chunk c-1 backward.
// The latency-bound recurrence leaves most of the chip idle; the side stream fills it.
// Parameters / gradients / Adam moments live in caller-owned flat fp32 buffers (the Python
// side keeps them as torch tensors so RCCL all-reduce and checkpointing work on them directly).
#pragma once
#include <map>
#include <cstdlib>
#include <string>
#include <vector>
#include "../runtime/runtime.h"
#include "../kernels/kernels.h"
#include "../comm/rccl_comm.h"
#include "../comm/watchdog.h"
#include <memory>

namespace gk {

struct Dims {
  int V = 256, E = 512, H = 512, L = 1, B = 256, T = 32, chunks = 4;
  int overlap = 1;   // side stream for chunk-consumers (0 = everything on one stream)
};
struct OptCfg {
  float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.f, clip = 0.f;
  int sgd = 0;
  int sched = 0, warmup = 0, total = 0;   // OptimArgs::sched / warmup / total
  float lr_min = 0.f;
  int keep_grads = 1;   // OptimArgs::keep_g
};

class Trainer {
 public:
  Trainer(const Dims& d, const OptCfg& o, float* params, float* grads, float* m, float* v, long nflat,
          const std::map<std::string, long>& offsets);
  ~Trainer();

  void refresh_weights(hipStream_t s);                  // bf16 / transposed copies of the master weights
  void set_batch(const int* x_bt, const int* y_bt, int B, hipStream_t s);  // host [B][T] ids/labels
  void forward_backward(hipStream_t s);                 // graph replay (captured on first call)
  void optimizer_step(hipStream_t s);                   // clip + Adam/SGD + refresh (graph)
  float read_loss();                                    // blocking
  float read_grad_norm();                               // blocking (valid when clip > 0)
  int get_step();                                       // optimiser step counter (device)
  void set_step(int v);                                 // for resume
  void set_lr(float lr);
  void set_use_graph(bool g) { use_graph_ = g; }
  // Truncated BPTT over a continuous stream: with carry on, each step starts from
  // the previous step's final hidden state (HS[T] -> HS[0] copies at the head of the step graph;
  // no gradient flows into it).  reset_hidden zeroes the carried state.
  void set_carry(bool on);
  bool carry() const { return carry_; }
  void reset_hidden(hipStream_t s);
  int padded_batch() const { return Bp_; }
  long workspace_bytes() const { return (long)arena_.bytes(); }
  // test/debug access to internal buffers by name
  uintptr_t buffer(const std::string& name) const;

 private:
  void record_fb(hipStream_t s0);
  // Slab reductions whose only consumer is the optimiser (single GPU, no clipping, one-graph step):
  // handed to the fused Adam/cast launch, which sums the partials itself (one launch and one pass
  // over the gradients fewer).  slab_job() routes a job to `j` or, when deferring, to deferred_.
  bool defer_slabs_ = false;
  SlabJobs deferred_;
  void slab_job(SlabJobs& j, const float* src, int splits, long n, float* dst);
  void record_carry(hipStream_t s);     // HS[T] -> HS[0] of every layer and copy (carry_ only)
  bool carry_ = false;
  // part: 0 every tensor, 1 every tensor but the FC pair, 2 the FC pair only (pipelined DP tail)
  void record_opt(hipStream_t s0, int part = 0);
  void fwd_step(int l, int t, hipStream_t s);
  void bwd_step(int l, int t, hipStream_t s);
  hipEvent_t ev();
  float* P(const std::string& name) const { return params_ + off_.at(name); }
  float* G(const std::string& name) const { return grads_ + off_.at(name); }
  int in_dim(int l) const { return l == 0 ? d_.E : d_.H; }

  Dims d_;
  OptCfg o_;
  int Bp_ = 0, Tc_ = 0, C_ = 1;
  float* params_; float* grads_; float* m_; float* v_;
  long nflat_;
  std::map<std::string, long> off_;

  Arena arena_;
  hipStream_t s0_ = nullptr, s1_ = nullptr;
  std::vector<hipEvent_t> events_;
  size_t ev_next_ = 0;
  Graph g_fb_[2], g_opt_;          // one forward/backward graph per staging slot
  bool use_graph_ = true;
  bool overlap_ = true;
  // batch staging, slots of [16 hdr][Bp*T x][Bp*T y] (batch-major): the host fills a pinned slot,
  // one DMA on the copy stream sx_ moves it to the same slot of the device staging d_stage_ while the
  // previous graph still runs, and the step graph's first kernel reads the DEVICE slot (no pinned
  // host memory read inside a step).  Graph k is captured against slot k.
  int* h_stage_ = nullptr;
  int* d_stage_ = nullptr;
  hipStream_t sx_ = nullptr;
  hipEvent_t stage_done_[2] = {nullptr, nullptr};
  hipEvent_t copy_done_[2] = {nullptr, nullptr};       // per-step slots 0, 1 reached the device
  hipEvent_t group_copy_done_[2] = {nullptr, nullptr}; // a multi-step slot group reached the device
  int stage_slot_ = 0;
  const int* stage_src_ = nullptr;   // device slot the graph being recorded reads
  size_t slot_ints() const { return 16 + 2 * (size_t)Bp_ * d_.T; }
  const int* dev_slot(int slot) const { return d_stage_ + (size_t)slot * slot_ints(); }
  void fill_slot(int slot, const int* x, const int* y, int B);
  void copy_slots(int first, int n, hipEvent_t done);   // pinned -> device, on sx_
  // single-graph step (prep + fwd/bwd + in-graph RCCL all-reduce + optimiser)
  Graph g_step_[2];
  Graph g_group_[2];
  hipEvent_t group_done_[2] = {nullptr, nullptr};
  int group_ = 1, group_parity_ = 0;
  int group_slot(int parity, int j) const { return 2 + parity * kMaxGroup + j; }
  void record_step_body();       // one step's capture body (shared by step() and step_group())
  RcclComm* comm_ = nullptr;
  std::vector<std::pair<long, long>> buckets_;   // plain buckets (eager / chunked-overlap paths)
  void record_allreduce(hipStream_t s);
  // ---- readiness-ordered, overlapped all-reduce (persistent single-graph path)
  // The flat gradient is laid out in readiness order (FC, layer L-1 ... layer 0: W_hh, b_hh, b_ih,
  // W_ih).  Layer 0's group ends inside the W_ih0 segment: instead of dEmb + dW_ih0 the engine
  // all-reduces dP = dL/d(Emb·W_ih0^T) [V][3H] written there (both are linear in dP with
  // replicated Emb / W_ih0; 5.25 vs 7.35 MB at H=512) and derives them after the collective.
  // While recording, the ready prefix [0, ar_ready_) grows as groups finish; ar_flush() hands
  // [ar_launched_, ar_ready_) to RCCL on the comm stream sc_ once it reaches min_bucket_ floats
  // (or at the end).  Collectives never run concurrently with a persistent sequence kernel
  // (its workgroups must all be co-resident, and an RCCL kernel holding CUs while waiting on a
  // peer could starve it): flushes happen right after a persistent kernel, and the step stream
  // joins the comm stream before launching the next one.
  bool dp_overlap() const { return comm_ != nullptr && !overlap_; }
  long group_end(int l) const;       // end of layer l's readiness group (l == L: the FC group)
  // returns true when a collective was recorded; with_err: it also max-reduces the error word
  bool ar_flush(hipStream_t s, bool force, bool with_err = false);
  void ar_join(hipStream_t s);
  float* dP_target() { return dP_inplace_ ? G("weight_ih_l0") : dP_; }
  // Pipelined data-parallel tail (one-layer models, where every gradient but FC's is ready only when
  // the persistent backward ends): three readiness buckets instead of one exposed collective --
  //   reduce [W_hh0, b_hh0, b_ih0, dP] slabs -> AR1 (+ error word) on the comm stream
  //   | beside it: dW_fc K-slices -> reduce -> AR2 (FC pair) on the comm stream
  //   join AR1 -> dW_ih0 / dEmb from the averaged dP -> Adam (all but FC) | beside it: AR2
  //   join AR2 -> Adam (FC pair).
  // dp_pipe_: -1 auto (= off: measured slower, dp_pipe_on), 0 one collective (the single-bucket
  // step), 1 on.
  int dp_pipe_ = -1;
  bool dp_tail_rec_ = false;
  bool dp_pipe_on() const;
  bool opt_in_fb_ = false;   // record_fb_seq recorded the optimiser itself (pipelined tail)
  void record_dp_tail_l1(hipStream_t s, SlabJobs& j, const SlabJobs& fc_tail);
  hipStream_t sc_ = nullptr;
  long min_bucket_ = 0, ar_ready_ = 0, ar_launched_ = 0;
  bool ar_busy_ = false, dP_inplace_ = false;
  std::vector<std::pair<long, long>> ar_log_;   // (offset, floats) of every recorded collective
  // sharded optimiser (set_shard_optim): mode 1 all-gathers the fp32 masters, mode 2 the bf16 working
  // copies (flat mirror pbf_; the fp32 biases ride along as an exact integer-sum exchange, bpack_) and
  // re-derives every bf16 layout locally -- the fp32 masters of other ranks' slices then go stale on this
  // rank (gather_params() for checkpoints)
  bool shard_opt_ = false;
  int shard_mode_ = 0;
  long shard_chunk_ = 0;
  u16* pbf_ = nullptr;
  unsigned* bpack_ = nullptr;
  FlatRanges branges_;
  void record_sharded_opt(hipStream_t s);
  void refresh_from_bf16(hipStream_t s);
  OptimArgs optim_args() const;
 public:
  void set_batch_device(const int* x, const int* y, int B, hipStream_t s);
  // buckets: plain bucket list; min_bucket_floats: smallest collective of the overlapped path
  void set_comm(RcclComm* c, const std::vector<std::pair<long, long>>& buckets, long min_bucket_floats);
  // collectives recorded into the last captured step graph (tests / plan printing)
  const std::vector<std::pair<long, long>>& allreduce_log() const { return ar_log_; }
  // pipelined data-parallel tail (see dp_pipe_): -1 auto, 0 off, 1 on; takes effect at the next capture
  void set_dp_pipeline(int mode);
  int dp_pipeline() const { return dp_pipe_on() ? 1 : 0; }
  // whether the last recorded step actually contains the pipelined tail (a capture fallback or an
  // eager step records the single-collective structure whatever dp_pipeline() says)
  bool dp_tail_recorded() const { return dp_tail_rec_; }
  // Sharded optimiser step (ZeRO-1 style, data-parallel only; call after set_comm).  The step graph
  // reduce-scatters the flat fp32 gradient in place (rank r owns floats [r*c, (r+1)*c), c a multiple
  // of 4; the < 4*world-float tail is all-reduced), runs Adam on the owned slice of the masters and
  // moments, all-gathers the updated masters in place and refreshes the bf16 MFMA copies.  Moments
  // outside the owned slice go stale: gather_opt_state() all-gathers them (checkpoints).
  void set_shard_optim(int mode);   // 0 off, 1 fp32 masters gathered, 2 bf16 working copies gathered
  bool shard_optim() const { return shard_opt_; }
  int shard_mode() const { return shard_mode_; }
  // mode 2: all-gather the fp32 masters (every rank's slice current again; checkpoints, state_dict)
  void gather_params(hipStream_t s);
  long shard_chunk() const { return shard_chunk_; }
  void gather_opt_state(hipStream_t s);
  void step(hipStream_t s);      // whole training step as one graph replay
  // Multi-step graphs: G consecutive steps (G = 1..kMaxGroup) captured into ONE graph, each reading
  // its own staging slot -- one graph boundary (~13 us at the headline) per G steps.  set_batches()
  // stages G batches ([G][B][T] each), step_group() launches them; two slot groups alternate so the
  // host fills one while the other runs.
  static constexpr int kMaxGroup = 32;
  void set_graph_steps(int G);
  int graph_steps() const { return group_; }
  void set_batches(const int* x, const int* y, int B, int n);
  void step_group(hipStream_t s);
  // test hook: set the device step error word (fault injection)
  void inject_error(unsigned bits) { HIP_CHECK(hipMemcpy(err_, &bits, 4, hipMemcpyHostToDevice)); }
  // watchdog over the launched steps (call after set_comm): timeout_ms > 0 aborts a step that
  // is not done in time, 0 only watches the communicator and the step error word, < 0 disables
  void enable_watchdog(int timeout_ms);
  int watchdog_status() const { return wd_ ? wd_->status() : 0; }
  std::string watchdog_message() { return wd_ ? wd_->message() : std::string(); }
 private:
  std::unique_ptr<Watchdog> wd_;

  struct Layer {
    float *HSf, *sr, *sz, *sn, *sghn, *dy, *Gi, *carry[2];
    u16* s16 = nullptr;   // packed bf16 saves [T][Bp][H][4] when SeqPlan::s16 (then sr..sghn are unused)
    u16 *HSb, *HT, *dgh[2], *dghT, *dgiT, *dgi;
    u16 *Whh, *WhhT, *Wih, *WihT;
    float *slab_hh, *rs_hh, *slab_ih, *rs_ih;
  };
  std::vector<Layer> Ls_;
  // persistent-sequence path
  struct SeqPlan {
    bool bwd = false, fuse_w = false, fuse_p = false;
    bool big = false;    // large H: the persistent split-K backward (gru_seq_big.hip) instead of T step kernels
    bool rows16 = false; // the persistent backward on 16-row blocks (gru_seq16.hip)
    bool s16 = false;    // packed bf16 (r, z, n, gh_n) saves: its forward and backward kernels both take them
    int nrb = 0;         // row blocks of the backward's bias / dP / dW_hh partials
    float *dWhh_part = nullptr, *dbhh_part = nullptr, *dbih_part = nullptr;
    u16* HF = nullptr;   // fragment-tiled h for the fused dW_hh (SeqFwdArgs::HF)
  };
  // dp: data-parallel recording (overlapped readiness-ordered all-reduce, dP in place, tail after)
  void record_fb_seq(hipStream_t s0, bool dp = false);
  void record_emb_tail(hipStream_t s, const float* dP_fp32);   // dP_fp32 null: bf16 copies already made
  // GK_WGRAD_GEMM=lib: the products the library takes (trainer_seq.cpp wgrad_gemm); by default none
  static bool wgrad_prefers_library(int M, int N, long K) {
    const char* v = std::getenv("GK_WGRAD_GEMM");
    return v && std::string(v) == "lib" && (double)M * N >= 8e6 && 2.0 * M * N * (double)K >= 60e9;
  }
  void wgrad_gemm(const u16* A, int lda, const u16* Bm, int ldb, int M, int N, int K, float* slab,
                  float* rowsum, hipStream_t s);
  bool persist_fwd_ = false;
  // one-layer H = 512, V = 256: the FC head runs as consumer workgroups of the persistent forward
  // (gru_fwd_seq_fc): no fc_xent launch, no dW_fc GEMM; decided per trainer (StepLdsVariants::fwd_fc)
  bool fc_in_fwd_ = false;
  bool dy_in_bwd_ = false;     // the top layer's large-H backward computes dy = dl · W_fc itself (big_dy)
  bool fwd_wave_ = false;      // layer pairs (0,1), (2,3).. forward as one wavefront launch (gru_fwd_seq2)
  float* bpart_ = nullptr;     // split-K partial tiles of the persistent large-H backward
  int step_algo_ = 0;          // per-step kernel choice (GK_STEP_ALGO: 0 auto, 1 register tile, 2 LDS tile)
  std::vector<SeqPlan> seq_;
  int splits_ = 8;
  unsigned *cnt_ = nullptr, *err_ = nullptr;
  unsigned *err_host_ = nullptr, *err_host_dev_ = nullptr;   // host-mapped mirror of *err_ (watchdog)
  float* sk_part_ = nullptr;         // split-K backward step kernel workspace (gru_step_lds.hip)
  unsigned* sk_cnt_ = nullptr;
  long sk_part_floats_ = 0, sk_cnt_words_ = 0;
  int xcd_local_ = 1;          // persistent kernels may use the L2-local hand-off (GK_XCD_LOCAL=0: never)
  // layer 0's per-step backward writes only the n-gate rows of dGi^T; the one-hot dP GEMM reads the
  // r/z rows from dGh^T, where they are identical (measured: profiles/r2_h2048_dgit_share_ab.jsonl)
  bool dgiT_share_ = false;
  u16* xbuf_ = nullptr;
  float *slab_w_ = nullptr, *rs_w_ = nullptr, *dP_part_ = nullptr;
  // dedicated split-K slabs whose reduce is deferred into the final multi-tensor reduce
  float *slab_fc2_ = nullptr, *rs_fc2_ = nullptr, *slab_e_ = nullptr;
  // the dW_fc GEMM held back to run inside the embedding-side launch (StepLdsVariants::dwfc_group)
  GemmArgs fc_held_;
  bool fc_held_on_ = false;
  int nloss_ = 0;                // loss partials of the recorded step (fc_xent blocks)
  long ldG_ = 0;   // leading dimension of dGh^T / dGi^T / dl^T (tokens + padding)
  static constexpr int kFcSplitsMax = 32;   // dW_fc: only (V/128)(H/128) output tiles -> deep split-K
 public:
  bool uses_persistent() const { return persist_fwd_ || (!seq_.empty() && seq_[0].bwd); }
  std::string plan() const;
  unsigned read_error();
 private:
  int *ids_, *labels_;
  float *inv_count_, *Ptab_, *loss_part_, *loss_, *slab_fc_, *rs_fc_, *slab_P_, *dP_;
  float *norm_parts_, *gscale_;
  int* step_;
  u16 *Emb, *EmbT, *Wfc, *WfcT, *dl_, *dlT_, *dP_bf_, *dPT_bf_;
  bool fc_split_ = false;        // FC as LDS GEMM (logits) + softmax_xent + LDS GEMM (dH)
  float* logits_ = nullptr;
  u16 *WfcF, *WfcTF;   // fragment-tiled (kernels.h ft_offset) copies of W_fc and W_fc^T for fc_xent
};

}  // namespace gk
