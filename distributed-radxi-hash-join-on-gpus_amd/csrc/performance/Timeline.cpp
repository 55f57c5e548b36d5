#include "Timeline.h"

#include <cstdlib>
#include <map>

#include "../utils/Hip.h"
#include "Clock.h"
#include "Measurements.h"

namespace hpcjoin {
namespace performance {

Timeline::~Timeline() {
  for (hipEvent_t e : pool_) (void)hipEventDestroy(e);
}

hipEvent_t Timeline::event() {
  if (used_ == pool_.size()) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));  // timing enabled
    pool_.push_back(e);
  }
  return pool_[used_++];
}

void Timeline::reserveEvents(size_t n) {
  while (pool_.size() < n) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    pool_.push_back(e);
  }
}

void Timeline::reset() {
  spans_.clear();
  used_ = 0;
}

// HPCJOIN_TIMELINE=0: no device sub-phase events (their keys stay 0); for
// measuring what the timing events cost inside a join.
static bool timelineOff() {
  static const bool off = [] {
    const char *e = std::getenv("HPCJOIN_TIMELINE");
    return e && std::atoi(e) == 0;
  }();
  return off;
}

void Timeline::begin(const char *key, hipStream_t s) {
  if (device_ && timelineOff()) return;
  Span sp;
  sp.key = key;
  if (device_) {
    sp.b = event();
    HIP_CHECK(hipEventRecord(sp.b, s));
  } else {
    sp.hb = nowUs();
  }
  spans_.push_back(sp);
}

void Timeline::beginSplit(const char *key, const char *a, double wa, const char *b, double wb, hipStream_t s) {
  begin(key, s);
  if (device_ && timelineOff()) return;
  spans_.back().ka = a;
  spans_.back().kb = b;
  spans_.back().wa = wa;
  spans_.back().wb = wb;
}

void Timeline::end(const char *key, hipStream_t s) {
  if (device_ && timelineOff()) return;
  for (auto it = spans_.rbegin(); it != spans_.rend(); ++it) {
    if (it->closed || it->key != key) continue;
    if (device_) {
      it->e = event();
      HIP_CHECK(hipEventRecord(it->e, s));
    } else {
      it->he = nowUs();
    }
    it->closed = true;
    return;
  }
  JOIN_ASSERT(false, "Timeline", "end(%s) without begin", key);
}

hipEvent_t Timeline::mark(hipStream_t s) {
  if (!device_ || timelineOff()) return nullptr;
  hipEvent_t e = event();
  HIP_CHECK(hipEventRecord(e, s));
  return e;
}

void Timeline::beginAt(const char *key, hipEvent_t at) {
  if (device_ && timelineOff()) return;
  Span sp;
  sp.key = key;
  if (device_)
    sp.b = at;
  else
    sp.hb = nowUs();
  spans_.push_back(sp);
}

void Timeline::beginSplitAt(const char *key, const char *a, double wa, const char *b, double wb, hipEvent_t at) {
  beginAt(key, at);
  if (device_ && timelineOff()) return;
  spans_.back().ka = a;
  spans_.back().kb = b;
  spans_.back().wa = wa;
  spans_.back().wb = wb;
}

void Timeline::endAt(const char *key, hipEvent_t at) {
  if (device_ && timelineOff()) return;
  for (auto it = spans_.rbegin(); it != spans_.rend(); ++it) {
    if (it->closed || it->key != key) continue;
    if (device_)
      it->e = at;
    else
      it->he = nowUs();
    it->closed = true;
    return;
  }
  JOIN_ASSERT(false, "Timeline", "endAt(%s) without begin", key);
}

void Timeline::resolve() {
  std::map<std::string, double> us;
  for (const Span &sp : spans_) {
    if (!sp.closed) continue;
    double t = 0;
    if (device_) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, sp.b, sp.e));
      t = ms > 0 ? ms * 1000.0 : 0.0;
    } else {
      t = (double)(sp.he - sp.hb);
    }
    if (sp.ka.empty()) {
      us[sp.key] += t;
    } else {
      const double w = sp.wa + sp.wb;
      us[sp.ka] += w > 0 ? t * sp.wa / w : t / 2;
      us[sp.kb] += w > 0 ? t * sp.wb / w : t / 2;
    }
  }
  for (auto &kv : us) Measurements::add(kv.first, kv.second, "us");
  reset();
}

}  // namespace performance
}  // namespace hpcjoin
