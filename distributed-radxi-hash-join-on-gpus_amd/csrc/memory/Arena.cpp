#include "Arena.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>

#include "../utils/Hip.h"

namespace hpcjoin {
namespace memory {

// HPCJOIN_TRACE_ALLOC=1: one stderr line per raw allocation (arena growth or
// fallback) with its duration -- steady-state joins should print none.
static bool traceAlloc() {
  static const bool on = [] {
    const char *e = std::getenv("HPCJOIN_TRACE_ALLOC");
    return e && e[0] == '1';
  }();
  return on;
}

// HPCJOIN_ARENA_SKIP_MB=n (experiments): every rewind leaves the first n MiB
// of the first chunk unused, shifting where a join's buffers land.
static uint64_t skipBytes() {
  static const uint64_t b = [] {
    const char *e = std::getenv("HPCJOIN_ARENA_SKIP_MB");
    return e && e[0] ? (uint64_t)std::atoll(e) << 20 : 0ull;
  }();
  return b;
}

// HPCJOIN_POISON_ARENA=1: fill every raw allocation with 0xA5 bytes, so code
// that silently relies on zeroed workspace memory fails loudly (debugging).
static bool poisonAlloc() {
  static const bool on = [] {
    const char *e = std::getenv("HPCJOIN_POISON_ARENA");
    return e && e[0] == '1';
  }();
  return on;
}

void *Arena::rawAlloc(Location loc, uint64_t bytes, int device) {
  if (bytes == 0) bytes = ALIGNMENT;
  void *p = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  struct Trace {
    Location loc;
    uint64_t bytes;
    std::chrono::steady_clock::time_point t0;
    ~Trace() {
      if (traceAlloc())
        std::fprintf(stderr, "[arena] alloc %s %.3f MB in %.3f ms\n",
                     loc == Location::Device ? "device" : (loc == Location::Pinned ? "pinned" : "host"), bytes / 1e6,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
  } trace{loc, bytes, t0};
  if (loc == Location::Device) {
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipMalloc(&p, bytes));
    if (poisonAlloc()) {
      // On a private non-blocking stream: the synchronous hipMemset runs on
      // the null stream, which waits for every blocking stream of the device
      // -- with in-process ranks sharing one device, another rank's stream
      // (and the barrier it is heading for) -- and deadlocked the ranks.
      hipStream_t ps;
      HIP_CHECK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
      HIP_CHECK(hipMemsetAsync(p, 0xA5, bytes, ps));
      HIP_CHECK(hipStreamSynchronize(ps));
      HIP_CHECK(hipStreamDestroy(ps));
    }
  } else if (loc == Location::Pinned) {
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable));
  } else {
    int r = posix_memalign(&p, ALIGNMENT, bytes);
    JOIN_ASSERT(r == 0 && p, "Arena", "posix_memalign(%lu) failed", (unsigned long)bytes);
    if (poisonAlloc()) std::memset(p, 0xA5, bytes);
  }
  return p;
}

void Arena::rawFree(Location loc, void *p) {
  if (!p) return;
  if (loc == Location::Device)
    (void)hipFree(p);  // never throw from a destructor path
  else if (loc == Location::Pinned)
    (void)hipHostFree(p);
  else
    std::free(p);
}

Arena::~Arena() { releaseAll(); }

void Arena::releaseAll() {
  ++epoch_;
  if (!fallbacks_.empty() || !chunks_.empty()) ++generation_;
  for (auto &f : fallbacks_) rawFree(loc_, f.p);
  fallbacks_.clear();
  fallbackBytes_ = 0;
  for (auto &c : chunks_) rawFree(loc_, c.base);
  chunks_.clear();
}

uint64_t Arena::capacity() const {
  uint64_t s = 0;
  for (const auto &c : chunks_) s += c.cap;
  return s;
}

uint64_t Arena::used() const {
  uint64_t s = 0;
  for (const auto &c : chunks_) s += c.used;
  return s;
}

void Arena::addChunk(uint64_t bytes, bool touch, void *stream) {
  bytes = ceilDiv(std::max<uint64_t>(bytes, ALIGNMENT), BIG_ALIGNMENT) * BIG_ALIGNMENT;
  uint8_t *p = static_cast<uint8_t *>(rawAlloc(loc_, bytes + TAG_BYTES, device_));  // + the allocation's tag
  if (touch) {
    if (loc_ == Location::Device) {
      HIP_CHECK(hipSetDevice(device_));
      const hipStream_t s = static_cast<hipStream_t>(stream);
      HIP_CHECK(hipMemsetAsync(p, poisonAlloc() ? 0xA5 : 0, bytes, s));
      HIP_CHECK(hipStreamSynchronize(s));
    } else {
      std::memset(p, poisonAlloc() ? 0xA5 : 0, bytes);
    }
  }
  chunks_.push_back(Chunk{p, bytes, 0});  // growth: existing allocations (and peers' mappings) stay valid
}

void Arena::reserve(uint64_t bytes) {
  releaseAll();
  if (bytes) addChunk(bytes, false);
}

uint64_t Arena::ensure(uint64_t bytes, bool touch, void *stream) {
  bytes += skipBytes();
  const uint64_t have = capacity();
  if (have >= bytes) return 0;
  if (used() <= skipBytes() && fallbacks_.empty()) {
    // Between joins nothing lives in the chunks: re-lay them out as ONE chunk
    // of the request (first fit over several smaller chunks could leave a big
    // buffer without a chunk that holds it), so the total is the request,
    // not the old chunks plus the request.
    releaseAll();
    addChunk(bytes, touch, stream);
    return capacity() > have ? capacity() - have : 0;
  }
  addChunk(bytes - have, touch, stream);  // mid-join: the shortfall (get() falls back for what misfits)
  return capacity() - have;
}

uint64_t Arena::ensureParts(const std::vector<uint64_t> &parts, bool touch, void *stream) {
  uint64_t want = skipBytes();
  for (uint64_t p : parts) want += p;
  const uint64_t have = capacity();
  if (have >= want) return 0;
  if (used() <= skipBytes() && fallbacks_.empty()) {
    releaseAll();
    for (size_t i = 0; i < parts.size(); ++i) addChunk(parts[i] + (i == 0 ? skipBytes() : 0), touch, stream);
    return capacity() > have ? capacity() - have : 0;
  }
  addChunk(want - have, touch, stream);  // mid-join: the shortfall
  return capacity() - have;
}

uint64_t Arena::trim(uint64_t keep) {
  const uint64_t have = capacity() + fallbackBytes_;
  if (have <= keep && fallbacks_.empty()) return 0;
  releaseAll();
  peakFallback_ = 0;
  if (keep) addChunk(keep, false);
  return have > capacity() ? have - capacity() : 0;
}

void *Arena::get(uint64_t bytes) {
  const uint64_t sz = ceilDiv(bytes ? bytes : 1, ALIGNMENT) * ALIGNMENT;
  // Big buffers start on 2 MiB boundaries (fragment / TLB granularity), as a
  // fresh hipMalloc would: sub-allocating them at 256-B offsets measurably
  // slowed the build/probe reads of the partitioned relations.
  const uint64_t align = sz >= BIG_BYTES ? BIG_ALIGNMENT : ALIGNMENT;
  for (auto &c : chunks_) {  // first fit, in chunk order (deterministic per allocation sequence)
    const uint64_t start = ceilDiv(c.used, align) * align;
    if (start + sz <= c.cap) {
      c.used = start + sz;
      const uint64_t u = used() + fallbackBytes_;
      if (u > peak_) peak_ = u;
      return c.base + start;
    }
  }
  void *p = rawAlloc(loc_, sz + TAG_BYTES, device_);
  const uint64_t accounted = sz + (align > ALIGNMENT ? align : 0);  // room for the padding once sub-allocated
  fallbacks_.push_back(Fallback{p, sz, accounted});
  fallbackBytes_ += accounted;
  peakFallback_ = std::max(peakFallback_, fallbackBytes_);
  const uint64_t u = used() + fallbackBytes_;
  if (u > peak_) peak_ = u;
  return p;  // a new allocation frees nothing: generation() unchanged
}

void Arena::reset() {
  // The last join's fallback allocations become chunks: a join that repeats
  // the allocation sequence fits them again (first fit, in order), and
  // nothing is freed, so generation() -- and every peer's IPC mapping of
  // them -- stays valid.  (Freeing them and adding one consolidated chunk
  // meant a peer re-imported a new allocation at the address range it had
  // just unmapped; at 8 ranks on one GPU that second join's one-sided puts
  // missed the windows.)  Consolidation happens where a join is planned:
  // ensure() with nothing handed out re-lays everything out as one chunk.
  ++epoch_;
  for (auto &f : fallbacks_) chunks_.push_back(Chunk{static_cast<uint8_t *>(f.p), f.bytes, 0});
  fallbacks_.clear();
  fallbackBytes_ = 0;
  peakFallback_ = 0;
  for (auto &c : chunks_) c.used = 0;
  if (!chunks_.empty() && skipBytes() < chunks_[0].cap) chunks_[0].used = skipBytes();
}

bool Arena::owns(const void *p) const {
  const uint8_t *q = static_cast<const uint8_t *>(p);
  for (const auto &c : chunks_)
    if (q >= c.base && q < c.base + c.cap) return true;
  return false;
}

void *Arena::allocationOf(const void *p) const {
  const uint8_t *q = static_cast<const uint8_t *>(p);
  for (const auto &c : chunks_)
    if (q >= c.base && q < c.base + c.cap) return c.base;
  for (const auto &f : fallbacks_) {
    const uint8_t *b = static_cast<const uint8_t *>(f.p);
    if (q >= b && q < b + f.bytes) return f.p;
  }
  return nullptr;
}

void *Arena::tagOf(const void *base) const {
  for (const auto &c : chunks_)
    if (c.base == base) return c.base + c.cap;
  for (const auto &f : fallbacks_)
    if (f.p == base) return static_cast<uint8_t *>(f.p) + f.bytes;
  return nullptr;
}

void Arena::freeFallback(void *p) {
  for (size_t i = 0; i < fallbacks_.size(); ++i)
    if (fallbacks_[i].p == p) {
      rawFree(loc_, p);
      fallbackBytes_ -= fallbacks_[i].accounted;
      fallbacks_.erase(fallbacks_.begin() + i);
      ++generation_;
      ++epoch_;
      return;
    }
}

}  // namespace memory
}  // namespace hpcjoin
