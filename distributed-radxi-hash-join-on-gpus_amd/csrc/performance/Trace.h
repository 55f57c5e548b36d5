// roctx ranges around every join phase (SURVEY §5 "tracing": the reference has
// gettimeofday timers only).  Visible in `rocprofv3 --marker-trace` timelines
// next to the kernels; a no-op when no profiler is attached.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace hpcjoin {
namespace performance {

class TraceRange {
 public:
  explicit TraceRange(const char *name) { roctxRangePush(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange &) = delete;
  TraceRange &operator=(const TraceRange &) = delete;
};

}  // namespace performance
}  // namespace hpcjoin
