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
enum class Location : int { Host = 0, Device = 1 };

inline const char *locationName(Location l) { return l == Location::Device ? "device" : "host"; }

HJ_HD uint32_t ceilLog2(uint64_t x) {
  uint32_t b = 0;
  while ((uint64_t(1) << b) < x) ++b;
  return b;
}

HJ_HD uint64_t ceilDiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

}  // namespace hpcjoin
