// Native runtime pieces: rank-tagged HIP error checking, a bump-pointer device arena,
// and a small RAII wrapper for a captured hipGraph.
//
// The reference's only error handling is CUDA_CALL -> exit(1) and it never checks kernel
// launches (/root/reference/namegensf.cu:11-19).  Here every API call
// and every launch sequence is checked, and failures raise (to Python) with the rank in
// the message instead of killing the process.
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <vector>
#include <cstdlib>

namespace gk {

inline int& global_rank() { static int r = -1; return r; }

[[noreturn]] inline void hip_fail(hipError_t e, const char* what, const char* file, int line) {
  std::string msg = "[rank " + std::to_string(global_rank()) + "] HIP error '" + hipGetErrorString(e) +
                    "' (" + std::to_string((int)e) + ") at " + file + ":" + std::to_string(line) + ": " + what;
  throw std::runtime_error(msg);
}

#define HIP_CHECK(x)                                              \
  do {                                                            \
    hipError_t _e = (x);                                          \
    if (_e != hipSuccess) ::gk::hip_fail(_e, #x, __FILE__, __LINE__); \
  } while (0)

#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

// One hipMalloc, carved into 256-byte aligned pieces.  Everything the engine needs per
// step is allocated once up front (no allocation inside a captured graph; 288 GB HBM makes
// "allocate the whole BPTT working set" the right trade-off).
class Arena {
 public:
  Arena() = default;
  ~Arena() { release(); }
  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;

  // two-phase: reserve() sizes everything, commit() allocates, then get() returns pointers
  size_t reserve(size_t bytes) {
    size_t off = size_;
    size_ += (bytes + 255) / 256 * 256;
    return off;
  }
  void commit() {
    if (base_) return;
    HIP_CHECK(hipMalloc(&base_, size_ ? size_ : 256));
    HIP_CHECK(hipMemset(base_, 0, size_ ? size_ : 256));
    // hipMemset is asynchronous on the null stream, and the engines' non-blocking streams do not
    // wait for it: without this a first batch copied on the trainer's copy stream could land before
    // the zero-fill and be wiped (a loss of 0 in one GPU-suite run)
    HIP_CHECK(hipDeviceSynchronize());
  }
  template <class T> T* get(size_t off) const { return reinterpret_cast<T*>(static_cast<char*>(base_) + off); }
  size_t bytes() const { return size_; }
  void release() {
    if (base_) { (void)hipFree(base_); base_ = nullptr; }
  }

 private:
  void* base_ = nullptr;
  size_t size_ = 0;
};

class Graph {
 public:
  ~Graph() { reset(); }
  void reset() {
    if (exec_) { (void)hipGraphExecDestroy(exec_); exec_ = nullptr; }
    if (graph_) { (void)hipGraphDestroy(graph_); graph_ = nullptr; }
  }
  bool ready() const { return exec_ != nullptr; }
  void begin(hipStream_t s) { reset(); HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)); }
  void end(hipStream_t s) {
    HIP_CHECK(hipStreamEndCapture(s, &graph_));
    HIP_CHECK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
  }
  void launch(hipStream_t s) { HIP_CHECK(hipGraphLaunch(exec_, s)); }
  // diagnostic: the captured graph as Graphviz DOT (nodes, their kinds and dependency edges)
  void dot(const char* path) const { if (graph_) HIP_CHECK(hipGraphDebugDotPrint(graph_, path, 0)); }

 private:
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace gk
