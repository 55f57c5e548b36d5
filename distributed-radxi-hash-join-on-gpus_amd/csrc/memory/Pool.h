// Process-global pool with the reference API (/root/reference/memory/Pool.h:19-27):
// allocate / getMemory / free / freeAll / reset.  The pool can live in HBM
// (device relations, the default on MI355X) or in host memory (reference
// path).  Fixes the reference's Pool::free self-recursion:
// free() releases fallback allocations and is a no-op for pool memory.
#pragma once

#include <cstdint>

#include "../core/Types.h"

namespace hpcjoin {
namespace memory {

class Arena;

class Pool {
 public:
  static void allocate(uint64_t size);                                  // host pool (reference)
  static void allocate(uint64_t size, Location loc, int device = 0);    // HBM or host pool
  static void *getMemory(uint64_t size);
  static void free(void *memory);
  static void freeAll();
  static void reset();

  static Location location();
  static uint64_t capacity();
  static uint64_t used();
  static bool contains(const void *p);
  static Arena *arena();

 protected:
  static Arena *instance;
};

}  // namespace memory
}  // namespace hpcjoin
