// Bump allocator over a few big HBM (hipMalloc) or host (posix_memalign) chunks.
//
// The reference's memory::Pool (/root/reference/memory/Pool.cpp:25-79) is a
// process-global host bump allocator with a posix_memalign fallback.  On
// MI355X the same idea is what keeps hipMalloc/hipFree (which synchronise the
// device, and on a fresh box can take seconds when the driver has to clear
// the pages: profiles/r3a) out of the timed join: a join's windows, send
// buffers and workspaces are carved from a per-engine Arena that is rewound
// with reset() at the start of every join.
//
// Growth never moves or frees memory a previous join used: when a join needs
// more than the chunks hold, the overflow is served by individual
// allocations, which reset() keeps as chunks, so the next join with the same
// allocation sequence fits (first fit over the chunks in order) and
// steady-state joins never allocate.  ensure() grows ahead of
// time (HashJoin reserves its plan's estimate at construction) and can touch
// the new pages once, so a first join does not pay the first-touch cost;
// between joins it re-lays the chunks out as one chunk of the request (the
// total never ratchets to old chunks + request), and trim() gives memory back.
// generation() counts FREES only (releaseAll, freeFallback, trim): an address a peer mapped (one-sided windows) stays
// valid until then, and frees happen only between joins, so a peer's
// mappings of one join all carry one generation and an import never has to
// close a mapping the same join still uses (core/ExecContext::ipcImport).
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
  // Every raw allocation (chunk or fallback) ends in TAG_BYTES the arena
  // never hands out: the one-sided exchange stamps an exported allocation
  // there, so a peer can prove its IPC mapping names that allocation and not
  // a freed one at the same address (core/ExecContext::ipcImport).
  static constexpr uint64_t TAG_BYTES = 256;

  Arena(Location loc, int device = 0) : loc_(loc), device_(device) {}
  ~Arena();
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;

  void reserve(uint64_t bytes);       // one chunk of `bytes` (frees everything first)
  // Grow so that the chunks hold >= bytes in all: with nothing handed out,
  // by re-laying them out as one chunk of `bytes`; otherwise by the shortfall;
  // touch = write the new chunk once (device: a memset ordered on `stream`,
  // then waited for -- the engine's streams are non-blocking, so a null-stream
  // memset could land after a join's first writes) so its pages are mapped
  // before the first join uses them.  Returns the bytes added.
  uint64_t ensure(uint64_t bytes, bool touch = false, void *stream = nullptr);
  // As ensure(sum of parts), laid out as one chunk per part (in order) when
  // the arena must be re-laid out: a join's big buffers then each start at an
  // allocation of their own.  Returns the bytes added.
  uint64_t ensureParts(const std::vector<uint64_t> &parts, bool touch = false, void *stream = nullptr);
  // Between joins: drop everything handed out (previous joins' outputs
  // included) and shrink to one chunk of `keep` bytes (0 = none) if the
  // arena holds more.  Returns the bytes freed.
  uint64_t trim(uint64_t keep = 0);
  void *get(uint64_t bytes);          // bump-allocate (fallback allocation when exhausted)
  template <typename T>
  T *getArray(uint64_t count) { return reinterpret_cast<T *>(get(count * sizeof(T))); }
  void reset();                       // rewind; the last join's fallback allocations become chunks
  void releaseAll();

  Location location() const { return loc_; }
  int device() const { return device_; }
  uint64_t capacity() const;          // bytes over all chunks
  uint64_t used() const;              // bytes handed out from the chunks since the last reset
  uint64_t peak() const { return peak_; }
  uint64_t fallbackBytes() const { return fallbackBytes_; }
  size_t chunkCount() const { return chunks_.size(); }
  uint64_t generation() const { return generation_; }
  // Counts rewinds and frees: memory handed out before an epoch change may
  // be handed out again (or be gone), so a result left in the workspace
  // (HashJoin::getOutput) is valid only while the epoch is unchanged.
  uint64_t epoch() const { return epoch_; }
  bool owns(const void *p) const;
  // Start of the raw allocation (chunk or fallback) holding p; null if none.
  void *allocationOf(const void *p) const;
  // The TAG_BYTES tail of the allocation starting at `base`; null if none.
  void *tagOf(const void *base) const;
  void freeFallback(void *p);         // frees one fallback allocation (no-op for arena memory)

  static void *rawAlloc(Location loc, uint64_t bytes, int device);
  static void rawFree(Location loc, void *p);

 private:
  struct Chunk {
    uint8_t *base;
    uint64_t cap;
    uint64_t used;
  };
  void addChunk(uint64_t bytes, bool touch, void *stream = nullptr);
  Location loc_;
  int device_;
  std::vector<Chunk> chunks_;
  uint64_t peak_ = 0;
  uint64_t fallbackBytes_ = 0;
  uint64_t peakFallback_ = 0;  // largest fallbackBytes_ since the last reset
  uint64_t generation_ = 0;
  uint64_t epoch_ = 0;
  struct Fallback {
    void *p;
    uint64_t bytes;      // allocated
    uint64_t accounted;  // + the big-buffer alignment it would need inside a chunk
  };
  std::vector<Fallback> fallbacks_;
};

}  // namespace memory
}  // namespace hpcjoin
