// Device-resident batched name generator (reference parity half).
//
// The reference generates ONE name at a time with 51 launches + 2 blocking memcpys +
// host sampling per character (/root/reference/namegensf.cu:649-884).  Here all local
// names advance together: per character, one fused step launch per layer (layer >= 1 fuses
// its input projection W_ih·h_below as a second MFMA product) and one FC+softmax+sample
// launch that writes the chosen char straight into the next step's input ids and into the
// output rows.  The MAX_LEN loop is captured once into a hipGraph; the host touches the
// device only to upload the uniforms and to read the finished names.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>
#include "../runtime/runtime.h"
#include "../kernels/kernels.h"

namespace gk {

struct GenDims {
  int V = 256, E = 512, H = 1024, L = 2, max_len = 10, sos = 0, eos = 0, max_batch = 4096;
  // 1: fp32-faithful (the reference's arithmetic: fp32 MFMA GEMMs on the fp32 master weights, IEEE
  // gates and softmax, gen_f32.hip); 0: bf16 MFMA fast mode; 2: bf16x3 -- the fp32 path with its
  // products as bf16 MFMA GEMMs over split operands (hi*hi + hi*lo + lo*hi, ~2^-16 relative error)
  int fp32 = 0;
};

class Generator {
 public:
  Generator(const GenDims& d, const float* params, const std::map<std::string, long>& offsets);
  ~Generator();
  void refresh_weights(hipStream_t s);   // bf16 weights + layer-0 table (call after params change)
  // rf: device [N][max_len] uniforms of THIS rank's names; out: device [N][max_len+1]
  void generate(const float* rf, int N, unsigned char* out, hipStream_t s);
  void set_use_graph(bool g) { use_graph_ = g; }
  // optional: device [Bp][V] softmax of the last generated step (tests)
  void set_probe(float* probs) { probe_ = probs; graphs_.clear(); }
  // Small batches (fp32 modes: <= GK_GEN_PERSIST_MAX names, default and at most 64; bf16 mode: <= 24):
  // one persistent launch per batch (gen_persist.hip, exact fp32) instead of the per-char graph.
  // On by default; GK_GEN_PERSIST=0 or set_persist(false) turns it off.
  void set_persist(bool on) { persist_ = on; }
  void set_persist_max(int n) { persist_max_ = n; }
  void set_persist_dbg(unsigned long long* p) { persist_dbg_ = p; }   // diagnostic stamps (nullable)
  bool uses_persist(int n) const;
  // names in the whole (data-parallel) job; 0 = unknown (then the per-call count decides)
  void set_global_names(int n) { global_n_ = n > 0 ? n : 0; }
  unsigned read_error();   // blocking: device error word (fp32 path: bit 4 = char id out of range)
  // fault injection (tests): the next persistent launch starts with its spin-timeout bit set, as if
  // an earlier wait had given up -- generate() must notice and regenerate the batch
  void inject_persist_error() { inject_ = true; }
  // diagnostic: DOT dump of the per-char graph captured for batches of n names (false: none yet)
  bool dump_graph(int n, const std::string& path) const {
    auto it = graphs_.find(n);
    if (it == graphs_.end() || !it->second) return false;
    it->second->dot(path.c_str());
    return true;
  }

 private:
  void record_steps(int n_active, hipStream_t s);
  void record_steps_f32(int n_active, hipStream_t s);
  // one product of the fp32 / bf16x3 path: C = h W^T (+ bias) -> splits (slabs of M x N at C).  fp32
  // reads A32 / W32; bf16x3 the split copies A3 ([hi|hi|lo] rows) / W3 ([hi|lo|hi] rows)
  int product_f32(const float* A32, const u16* A3, const float* W32, const u16* W3, const float* bias, int M, int N,
                  float* C, hipStream_t s);
  bool split3() const { return d_.fp32 == 2; }
  void reset_batch(int Bp, bool bf16, hipStream_t s);
  const float* P(const std::string& n) const { return params_ + off_.at(n); }

  GenDims d_;
  int Bmax_;
  const float* params_;
  std::map<std::string, long> off_;
  Arena arena_;
  hipStream_t cap_ = nullptr;
  bool use_graph_ = true;
  float* probe_ = nullptr;
  std::map<int, std::unique_ptr<Graph>> graphs_;   // keyed by active-name count
  // buffers
  std::vector<float*> hf_;             // [L*2][Bmax][H]
  std::vector<u16*> hb_;
  std::vector<u16*> Whh_, Wih_;
  u16 *Emb_, *Wfc_, *WfcF_;
  int step_algo_ = 0;
  float *Ptab_, *rf_;
  float* Ptab32_ = nullptr;     // fp32 layer-0 table of the persistent launch (= Ptab_ in the fp32 modes)
  int *ids_, *alive_;
  unsigned char* out_;
  float *gh_ = nullptr, *gi_ = nullptr, *logits_ = nullptr;   // fp32 mode: [Bmax][3H] x2, [Bmax][V]
  unsigned* err_ = nullptr;
  unsigned* err_pin_ = nullptr;   // pinned host word: the persistent launch's error-word read-back
  // the device error word is known to be zero (the last call ended on a persistent launch that read
  // it back as 0, nothing queued since): the next call skips its clearing memset
  bool err_clean_ = false;
  bool persist_ = true;
  bool inject_ = false;
  int global_n_ = 0;            // set_global_names
  int persist_max_ = 64;        // names per batch up to which the persistent launch is used
  int persist_max_bf16_ = 40;   // ... in the bf16 mode (it runs exact fp32, faster up to ~40 names:
                                // profiles/r5_gen_persist_vs_bf16_graph_final.jsonl)
  unsigned long long* persist_dbg_ = nullptr;
  float* pws_ = nullptr;        // persistent path: exchange buffers (two sets, by launch parity)
  int ppar_ = -1;               // the next persistent launch's set; -1: workspace not filled yet
  unsigned* psync_ = nullptr;   // persistent path: flags + done counter (self-cleaning, arena-zeroed)
  static constexpr int kF32SlabRows = 2048;   // fp32 split-K slab capacity (rows x 3H)
};

}  // namespace gk
