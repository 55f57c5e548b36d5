#include "Timeline.h"

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

void Timeline::reset() {
  spans_.clear();
  used_ = 0;
}

void Timeline::begin(const char *key, hipStream_t s) {
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
  spans_.back().ka = a;
  spans_.back().kb = b;
  spans_.back().wa = wa;
  spans_.back().wb = wb;
}

void Timeline::end(const char *key, hipStream_t s) {
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
