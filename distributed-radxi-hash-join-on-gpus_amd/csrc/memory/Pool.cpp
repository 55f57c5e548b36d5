#include "Pool.h"

#include "../utils/Debug.h"
#include "Arena.h"

namespace hpcjoin {
namespace memory {

Arena *Pool::instance = nullptr;

void Pool::allocate(uint64_t size) { allocate(size, Location::Host, 0); }

void Pool::allocate(uint64_t size, Location loc, int device) {
  freeAll();
  instance = new Arena(loc, device);
  instance->reserve(size);
  JOIN_DEBUG("Pool", "allocated %lu bytes of %s memory", (unsigned long)size, locationName(loc));
}

void *Pool::getMemory(uint64_t size) {
  if (!instance) allocate(0);
  return instance->get(size);
}

void Pool::free(void *memory) {
  if (instance && memory && !instance->owns(memory)) instance->freeFallback(memory);
}

void Pool::freeAll() {
  delete instance;
  instance = nullptr;
}

void Pool::reset() {
  if (instance) instance->reset();
}

Location Pool::location() { return instance ? instance->location() : Location::Host; }
uint64_t Pool::capacity() { return instance ? instance->capacity() : 0; }
uint64_t Pool::used() { return instance ? instance->used() : 0; }
bool Pool::contains(const void *p) { return instance && instance->owns(p); }
Arena *Pool::arena() { return instance; }

}  // namespace memory
}  // namespace hpcjoin
