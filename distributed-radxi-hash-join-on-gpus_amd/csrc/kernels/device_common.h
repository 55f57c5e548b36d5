// Device-side building blocks shared by the gfx950 kernels: wave64 scans and
// reductions and LDS block scans.  Wave width is hard-coded to 64 (CDNA).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../utils/Hip.h"

namespace hpcjoin {
namespace kernels {

constexpr int WAVE = 64;

template <typename T>
__device__ __forceinline__ T waveInclusiveScan(T x) {
  const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    T y = __shfl_up(x, o, WAVE);
    if (lane >= o) x += y;
  }
  return x;
}

// A wave-uniform 64-bit value moved to scalar registers.  readfirstlane
// returns int: each half goes through uint32_t, or a low half with bit 31 set
// would sign-extend over the high half (a silent wrong address past 2^31
// elements, not a fault).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

template <typename T>
__device__ __forceinline__ T waveReduceSum(T x) {
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, WAVE);
  return x;
}

// Workgroup barrier that orders LDS accesses only.  __syncthreads() is a
// workgroup-scope release/acquire for every address space, so the compiler
// puts s_waitcnt vmcnt(0) in front of it: all of the wave's global loads in
// flight (a prefetched tile) must land first.  Kernels whose waves hand each
// other data through LDS alone use this one and keep their loads in flight.
__device__ __forceinline__ void ldsBarrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <bool LDS_ONLY>
__device__ __forceinline__ void blockBarrier() {
  if constexpr (LDS_ONLY)
    ldsBarrier();
  else
    __syncthreads();
}

// Exclusive scan of an LDS array data[0..n) into out[0..n) (may alias) by a
// workgroup of NT threads; each thread owns a contiguous run of entries.
// waveTot must hold NT/64 entries of T.  Contains the barriers it needs; all
// threads of the block must call it.  LDS_ONLY: its barriers order LDS only
// (ldsBarrier), for callers with global loads in flight across the scan.
template <int NT, typename T, typename U, bool LDS_ONLY = false>
__device__ __forceinline__ T blockExclusiveScanLds(const U *data, T *out, int n, T *waveTot) {
  const int t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
  const int per = (n + NT - 1) / NT;
  const int b = t * per;
  T local = 0;
  for (int i = 0; i < per; ++i)
    if (b + i < n) local += T(data[b + i]);
  T incl = waveInclusiveScan<T>(local);
  if (lane == WAVE - 1) waveTot[wid] = incl;
  blockBarrier<LDS_ONLY>();
  T prefix = 0, total = 0;
#pragma unroll
  for (int w = 0; w < NT / WAVE; ++w) {
    T v = waveTot[w];
    if (w < wid) prefix += v;
    total += v;
  }
  T run = prefix + incl - local;
  for (int i = 0; i < per; ++i)
    if (b + i < n) {
      T v = T(data[b + i]);
      out[b + i] = run;
      run += v;
    }
  blockBarrier<LDS_ONLY>();
  return total;
}

template <int NT, typename T>
__device__ __forceinline__ T blockReduceSum(T x, T *waveTot) {
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
  x = waveReduceSum<T>(x);
  __syncthreads();
  if (lane == 0) waveTot[wid] = x;
  __syncthreads();
  T total = 0;
#pragma unroll
  for (int w = 0; w < NT / WAVE; ++w) total += waveTot[w];
  return total;
}

}  // namespace kernels
}  // namespace hpcjoin
