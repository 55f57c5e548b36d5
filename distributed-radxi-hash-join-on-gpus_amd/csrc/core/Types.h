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

// Kernel-shape variants kept for sweeps and A/B tests (defaults = the
// measured best).  They live in the JoinConfig, are copied into the JoinPlan
// once, and reach the launchers through their argument structs: no kernel
// launcher reads the environment (Python: HPCJOIN_<FIELD> is resolved once by
// utils.config.config_from_dict).
struct KernelVariants {
  uint32_t netIpt = 0;        // claim-scatter tile: 0 = 8 x 1024, 16 = 16 x 1024 (u32 words only), 15 = 15K tiles at 2048-way
  uint32_t netThreads = 0;    // claim-scatter workgroup width: 0 = 1024, 512 = half-width (2-3 per CU)
  uint32_t bmThreads = 0;     // bitmap kernels' workgroup size: 0 = auto (256 for <= 32 KiB bitmaps, else 1024)
  int32_t bmFlat = -1;        // bitmap slice walk: -1 = auto, 0 = per claim slice, 1 = one flat walk per partition
  uint32_t reduceChunks = 0;  // replicated bitmap plan: all-reduce ranges (0 = auto: one per 32 MiB, <= 4)
  uint32_t keyCount = 8;      // key-only count kernel: 8 = span work queue with the quotient table (bpKeyQuotientKernel;
                              // counted tables for heavy partitions and 45-48-bit fragments, v2 for unsplit words),
                              // 9 = every partition on counted tables (bpKeyCountedSpansKernel; set after repeated
                              // keys), 7 = the v2 bucket table (bpKeySpanKernel) everywhere
  uint32_t rowsLds = 1;       // fused row output with the inner rows cached in LDS (0 = staged kernel)
  uint32_t matVariant = 1;    // late-materialization store/load flavour (materialize.hip)
};

}  // namespace hpcjoin
