// Collective watchdog: a host thread that watches the last launched training
// step.  If its completion event has not fired within `timeout_ms`, or the communicator
// reports an asynchronous error, it aborts the RCCL communicator (ncclCommAbort), which
// unblocks every collective stuck in a kernel on this rank, and records why.  The training
// loop then sees a failed sync / non-zero status and can exit or restart from the last
// checkpoint instead of hanging the node.  The reference's failure handling is
// CUDA_CALL -> exit(1) only (/root/reference/namegensf.cu:11-19).
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <hip/hip_runtime.h>
#include "rccl_comm.h"

namespace gk {

class Watchdog {
 public:
  enum Status { kOk = 0, kTimeout = 1, kCommError = 2, kStepError = 3 };
  // timeout_ms 0: no step deadline (still watches the communicator and the step error word)
  Watchdog(RcclComm* comm, int timeout_ms, int poll_ms = 20);
  // host-mapped mirror of the device step error word (written by the optimiser kernel)
  void set_error_word(const volatile unsigned* w) {
    std::lock_guard<std::mutex> g(mu_);
    err_word_ = w;
  }
  ~Watchdog();
  // arm: the work recorded before `ev` must complete within the timeout from now
  void watch(hipEvent_t ev);
  int status() const { return status_.load(); }
  std::string message();

 private:
  void run();
  RcclComm* comm_;
  const volatile unsigned* err_word_ = nullptr;
  int timeout_ms_, poll_ms_, device_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  hipEvent_t ev_ = nullptr;
  std::chrono::steady_clock::time_point armed_at_;
  bool stop_ = false;
  std::atomic<int> status_{kOk};
  std::string msg_;
  std::thread th_;
};

}  // namespace gk
