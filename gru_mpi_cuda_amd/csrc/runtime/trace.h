// roctx ranges around host-side phases: visible in `rocprofv3 --marker-trace`
// timelines next to the kernels they launch.  The reference has no tracing at all.
// Compiled in unconditionally; a push/pop pair costs ~100 ns when no profiler is attached.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace gk {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* msg) { roctxMarkA(msg); }

}  // namespace gk

#define GK_TRACE_CAT2(a, b) a##b
#define GK_TRACE_CAT(a, b) GK_TRACE_CAT2(a, b)
#define GK_TRACE(name) ::gk::TraceRange GK_TRACE_CAT(_gk_trace_, __LINE__)(name)
