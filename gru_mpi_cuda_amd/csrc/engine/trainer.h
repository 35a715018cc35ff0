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
  int padded_batch() const { return Bp_; }
  long workspace_bytes() const { return (long)arena_.bytes(); }
  // test/debug access to internal buffers by name
  uintptr_t buffer(const std::string& name) const;

 private:
  void record_fb(hipStream_t s0);
  void record_opt(hipStream_t s0);
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
  // pinned host staging, 2 slots of [16 hdr][Bp*T x][Bp*T y] (batch-major); the step graph's
  // first kernel reads its slot zero-copy.  Graph k is captured against slot k.
  int* h_stage_ = nullptr;
  hipEvent_t stage_done_[2] = {nullptr, nullptr};
  int stage_slot_ = 0;
  const int* stage_src_ = nullptr;   // slot the graph being recorded reads
  size_t slot_ints() const { return 16 + 2 * (size_t)Bp_ * d_.T; }
  void fill_slot(int slot, const int* x, const int* y, int B);
  // single-graph step (prep + fwd/bwd + in-graph RCCL all-reduce + optimiser)
  Graph g_step_[2];
  RcclComm* comm_ = nullptr;
  std::vector<std::pair<long, long>> buckets_;
  // data-parallel: all-reduce dP = dL/d(Emb·W_ih0^T) [V][3H] instead of dEmb + dW_ih0 (both are
  // linear in dP with replicated Emb / W_ih0): buckets_dp_ = buckets_ minus those two segments
  std::vector<std::pair<long, long>> buckets_dp_;
  bool dp_trick() const { return comm_ != nullptr && !overlap_; }
  void record_allreduce(hipStream_t s, bool dp_trick = false);
 public:
  void set_batch_device(const int* x, const int* y, int B, hipStream_t s);
  void set_comm(RcclComm* c, const std::vector<std::pair<long, long>>& buckets);
  void step(hipStream_t s);      // whole training step as one graph replay
  // collective watchdog over the launched steps (needs set_comm first; 0 disables)
  void enable_watchdog(int timeout_ms);
  int watchdog_status() const { return wd_ ? wd_->status() : 0; }
  std::string watchdog_message() { return wd_ ? wd_->message() : std::string(); }
 private:
  std::unique_ptr<Watchdog> wd_;

  struct Layer {
    float *HSf, *sr, *sz, *sn, *sghn, *dy, *Gi, *carry[2];
    u16 *HSb, *HT, *dgh[2], *dghT, *dgiT, *dgi;
    u16 *Whh, *WhhT, *Wih, *WihT;
    float *slab_hh, *rs_hh, *slab_ih, *rs_ih;
  };
  std::vector<Layer> Ls_;
  // persistent-sequence path
  struct SeqPlan {
    bool bwd = false, fuse_w = false, fuse_p = false;
    float *dWhh_part = nullptr, *dbhh_part = nullptr, *dbih_part = nullptr;
  };
  void record_fb_seq(hipStream_t s0, bool defer_tail = false);
  void record_emb_tail(hipStream_t s, bool from_fp32);
  void wgrad_gemm(const u16* A, int lda, const u16* Bm, int ldb, int M, int N, int K, float* slab,
                  float* rowsum, hipStream_t s);
  bool persist_fwd_ = false;
  int step_algo_ = 0;          // per-step kernel choice (GK_STEP_ALGO: 0 auto, 1 register tile, 2 LDS tile)
  std::vector<SeqPlan> seq_;
  int splits_ = 8;
  unsigned *cnt_ = nullptr, *err_ = nullptr;
  u16* xbuf_ = nullptr;
  float *slab_w_ = nullptr, *rs_w_ = nullptr, *dP_part_ = nullptr;
  // dedicated split-K slabs whose reduce is deferred into the final multi-tensor reduce
  float *slab_fc2_ = nullptr, *rs_fc2_ = nullptr, *slab_e_ = nullptr;
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
};

}  // namespace gk
