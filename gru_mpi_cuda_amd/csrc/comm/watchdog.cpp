#include "watchdog.h"

#include <cstdio>
#include "../runtime/runtime.h"
#include "../runtime/trace.h"

namespace gk {

Watchdog::Watchdog(RcclComm* comm, int timeout_ms, int poll_ms)
    : comm_(comm), timeout_ms_(timeout_ms), poll_ms_(poll_ms) {
  HIP_CHECK(hipGetDevice(&device_));
  th_ = std::thread([this] { run(); });
}

Watchdog::~Watchdog() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void Watchdog::watch(hipEvent_t ev) {
  std::lock_guard<std::mutex> g(mu_);
  ev_ = ev;
  armed_at_ = std::chrono::steady_clock::now();
}

std::string Watchdog::message() {
  std::lock_guard<std::mutex> g(mu_);
  return msg_;
}

void Watchdog::run() {
  (void)hipSetDevice(device_);
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::milliseconds(poll_ms_));
    if (stop_ || status_.load() != kOk) continue;
    // asynchronous communicator errors (peer died, transport failure)
    if (comm_) {
      try {
        comm_->check_async_error();
      } catch (const std::exception& e) {
        msg_ = e.what();
        status_ = kCommError;
        trace_mark("watchdog: comm error, aborting communicator");
        comm_->abort();
        std::fprintf(stderr, "[gk watchdog] %s -> communicator aborted\n", msg_.c_str());
        continue;
      }
    }
    // a persistent / split-K kernel hit its cross-workgroup spin limit: the step was not applied
    // (OptimArgs::err); stop the job before the other ranks wait on this one forever
    if (err_word_ && *err_word_) {
      msg_ = "[rank " + std::to_string(comm_ ? comm_->rank() : global_rank()) +
             "] a cross-workgroup wait hit its spin limit (error word " + std::to_string(*err_word_) +
             "); the step's update was skipped";
      status_ = kStepError;
      ev_ = nullptr;
      trace_mark("watchdog: step error word set");
      if (comm_) comm_->abort();
      std::fprintf(stderr, "[gk watchdog] %s\n", msg_.c_str());
      continue;
    }
    if (!ev_) continue;
    const hipError_t q = hipEventQuery(ev_);
    if (q == hipSuccess) { ev_ = nullptr; continue; }
    if (q != hipErrorNotReady) {
      msg_ = std::string("step event query failed: ") + hipGetErrorString(q);
      status_ = kCommError;
      continue;
    }
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - armed_at_).count();
    if (timeout_ms_ > 0 && ms > timeout_ms_) {
      msg_ = "[rank " + std::to_string(comm_ ? comm_->rank() : global_rank()) + "] training step not done after " +
             std::to_string(ms) + " ms (timeout " + std::to_string(timeout_ms_) + " ms)";
      status_ = kTimeout;
      ev_ = nullptr;
      trace_mark("watchdog: step timeout, aborting communicator");
      if (comm_) comm_->abort();
      std::fprintf(stderr, "[gk watchdog] %s -> communicator aborted\n", msg_.c_str());
    }
  }
}

}  // namespace gk
