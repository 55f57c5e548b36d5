// Bump allocator over one big HBM (hipMalloc) or host (posix_memalign) block.
//
// The reference's memory::Pool (/root/reference/memory/Pool.cpp:25-79) is a
// process-global host bump allocator with a posix_memalign fallback.  On
// MI355X the same idea is what keeps hipMalloc/hipFree (which synchronise the
// device) out of the timed join: a join's windows, send buffers and
// workspaces are carved from a per-engine Arena that is rewound with reset()
// at the start of every join.  When a join needs more than the arena holds,
// the overflow is served by individual allocations and the arena grows to the
// observed peak at the next reset(), so steady-state joins never allocate.
#pragma once

#include <cstdint>
#include <vector>

#include "../core/Types.h"

namespace hpcjoin {
namespace memory {

class Arena {
 public:
  static constexpr uint64_t ALIGNMENT = 256;  // >= a 128-B L2 line, 16-B LDS-DMA friendly
  static constexpr uint64_t BIG_BYTES = 4ull << 20;
  static constexpr uint64_t BIG_ALIGNMENT = 2ull << 20;

  Arena(Location loc, int device = 0) : loc_(loc), device_(device) {}
  ~Arena();
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;

  void reserve(uint64_t bytes);       // (re)allocate the main block (frees everything)
  void *get(uint64_t bytes);          // bump-allocate (fallback allocation when exhausted)
  template <typename T>
  T *getArray(uint64_t count) { return reinterpret_cast<T *>(get(count * sizeof(T))); }
  void reset();                       // rewind; grow to the last peak if it overflowed
  void releaseAll();

  Location location() const { return loc_; }
  int device() const { return device_; }
  uint64_t capacity() const { return capacity_; }
  uint64_t used() const { return used_; }
  uint64_t peak() const { return peak_; }
  uint64_t fallbackBytes() const { return fallbackBytes_; }
  bool owns(const void *p) const;
  // Start of the raw allocation (main block or fallback) holding p; null if none.
  void *allocationOf(const void *p) const;
  void freeFallback(void *p);         // frees one fallback allocation (no-op for arena memory)

  static void *rawAlloc(Location loc, uint64_t bytes, int device);
  static void rawFree(Location loc, void *p);

 private:
  Location loc_;
  int device_;
  uint8_t *base_ = nullptr;
  uint64_t capacity_ = 0;
  uint64_t used_ = 0;
  uint64_t peak_ = 0;
  uint64_t fallbackBytes_ = 0;
  std::vector<std::pair<void *, uint64_t>> fallbacks_;
};

}  // namespace memory
}  // namespace hpcjoin
