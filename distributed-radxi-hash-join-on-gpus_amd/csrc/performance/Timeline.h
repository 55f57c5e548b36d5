// Per-join sub-phase timer behind the reference's detailed .perf keys
// (/root/reference/performance/Measurements.cpp:272-542: MIMAINPART,
// MWINPUT, LPHISTCOMP, LPPART, BPBUILD, ...).  The reference brackets CPU
// loops with gettimeofday; here most of that work is kernels and RCCL calls
// enqueued on HIP streams, so a span is a pair of timing events on the
// stream that does the work (begin and end may sit on different streams:
// e.g. "last scatter done" -> "last exchange chunk landed").  resolve(),
// after the join's final synchronisation, adds every span's length to the
// Measurements table under its key (µs).  On the host path the same calls
// time the host work directly.  Events come from a pool reused across joins.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace hpcjoin {
namespace performance {

class Timeline {
 public:
  explicit Timeline(bool device) : device_(device) {}
  ~Timeline();
  Timeline(const Timeline &) = delete;
  Timeline &operator=(const Timeline &) = delete;

  void reset();                                   // start of a join
  // Create n timing events up front (engine start): a first join would
  // otherwise pay each hipEventCreate inside its span.
  void reserveEvents(size_t n);
  void begin(const char *key, hipStream_t s = nullptr);
  void end(const char *key, hipStream_t s = nullptr);  // closes the key's open span
  // One span charged to two keys in proportion wa : wb (a fused kernel doing
  // two reference phases, e.g. build + probe of one LDS table).
  void beginSplit(const char *key, const char *a, double wa, const char *b, double wb, hipStream_t s = nullptr);
  // Shared time points (device): mark() records one event on s; spans can
  // begin / end at an existing event, so back-to-back spans (one phase ends
  // where the next begins) cost one event instead of two.  Every timing event
  // is a packet the stream waits on (~4-5 us each: 17 per bitmap join were
  // 50 us of a 1.4 ms join at 125M, profiles/r2s).  Host path: mark() returns
  // nullptr and the *At calls take the host clock.
  hipEvent_t mark(hipStream_t s = nullptr);
  void beginAt(const char *key, hipEvent_t at);
  void endAt(const char *key, hipEvent_t at);
  void beginSplitAt(const char *key, const char *a, double wa, const char *b, double wb, hipEvent_t at);
  void resolve();                                 // after the final sync: spans -> Measurements (µs, summed)

 private:
  struct Span {
    std::string key;
    hipEvent_t b = nullptr, e = nullptr;
    uint64_t hb = 0, he = 0;
    bool closed = false;
    std::string ka, kb;  // split spans: charged to ka and kb
    double wa = 0, wb = 0;
  };
  hipEvent_t event();
  bool device_;
  std::vector<Span> spans_;
  std::vector<hipEvent_t> pool_;
  size_t used_ = 0;
};

}  // namespace performance
}  // namespace hpcjoin
