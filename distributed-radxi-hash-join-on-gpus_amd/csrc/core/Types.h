// Common low-level types and portability-free macros for the MI355X join engine.
#pragma once

#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HJ_HD __host__ __device__ __forceinline__
#else
#define HJ_HD inline
#endif

namespace hpcjoin {

// Where a buffer lives.  The engine has exactly two execution targets: the
// MI355X (HBM, HIP kernels) and the single-thread host reference path that
// mirrors the reference's CPU semantics (plumbing config 1 / test oracle).
// Host: pageable host memory (host engine).  Device: HBM.  Pinned: page-locked
// host memory mapped into the GPU address space -- relations larger than HBM
// stay there and the device kernels read them over the host link (the
// reference's dormant UVA / out-of-GPU-memory path).
enum class Location : int { Host = 0, Device = 1, Pinned = 2 };

inline const char *locationName(Location l) {
  return l == Location::Device ? "device" : (l == Location::Pinned ? "pinned" : "host");
}
// Can device kernels dereference memory at this location?
inline bool deviceAccessible(Location l) { return l != Location::Host; }

HJ_HD uint32_t ceilLog2(uint64_t x) {
  uint32_t b = 0;
  while ((uint64_t(1) << b) < x) ++b;
  return b;
}

HJ_HD uint64_t ceilDiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

}  // namespace hpcjoin
