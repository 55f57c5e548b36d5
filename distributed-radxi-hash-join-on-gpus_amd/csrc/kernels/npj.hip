// No-partitioning hash join (NPJ) baseline: one global open-addressing table
// in HBM, 64-bit CAS inserts, linear probing.  Counterpart of the reference's
// dormant build_kernel / probe_kernel / simple_hash_join* family
// (/root/reference/operators/gpu/kernels_optimized.cu:1250-1377,
// small_data_optimized.cu:1731-2087).  Used by the micro-benchmarks to show
// what the radix-partitioned join buys over random HBM accesses.
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

constexpr int NPJ_T = 256;

uint64_t npjTableSlots(uint64_t innerSize) { return uint64_t(1) << ceilLog2(2 * (innerSize ? innerSize : 1)); }

__device__ __forceinline__ uint64_t npjHash(uint64_t k, uint64_t mask) {
  return ((k * 0x9E3779B97F4A7C15ull) >> 17) & mask;
}

__global__ __launch_bounds__(NPJ_T) void npjBuildKernel(const ulonglong2 *__restrict__ R, uint64_t n,
                                                        unsigned long long *table, uint64_t mask) {
  const uint64_t stride = (uint64_t)gridDim.x * NPJ_T;
  for (uint64_t i = (uint64_t)blockIdx.x * NPJ_T + threadIdx.x; i < n; i += stride) {
    const unsigned long long k = R[i].x;
    uint64_t h = npjHash(k, mask);
    while (atomicCAS(&table[h], ~0ull, k) != ~0ull) h = (h + 1) & mask;
  }
}

__global__ __launch_bounds__(NPJ_T) void npjProbeKernel(const ulonglong2 *__restrict__ S, uint64_t n,
                                                        const unsigned long long *__restrict__ table, uint64_t mask,
                                                        unsigned long long *result) {
  __shared__ unsigned long long wt[NPJ_T / WAVE];
  const uint64_t stride = (uint64_t)gridDim.x * NPJ_T;
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * NPJ_T + threadIdx.x; i < n; i += stride) {
    const unsigned long long k = S[i].x;
    uint64_t h = npjHash(k, mask);
    unsigned long long e;
    while ((e = table[h]) != ~0ull) {
      c += (e == k);
      h = (h + 1) & mask;
    }
  }
  c = blockReduceSum<NPJ_T, unsigned long long>(c, wt);
  if (threadIdx.x == 0 && c) atomicAdd(result, c);
}

__global__ __launch_bounds__(NPJ_T) void npjBuildRidsKernel(const ulonglong2 *__restrict__ R, uint64_t n,
                                                            unsigned long long *table, unsigned long long *rids,
                                                            uint64_t mask) {
  const uint64_t stride = (uint64_t)gridDim.x * NPJ_T;
  for (uint64_t i = (uint64_t)blockIdx.x * NPJ_T + threadIdx.x; i < n; i += stride) {
    const ulonglong2 t = R[i];
    uint64_t h = npjHash(t.x, mask);
    while (atomicCAS(&table[h], ~0ull, t.x) != ~0ull) h = (h + 1) & mask;
    rids[h] = t.y;  // the slot is this tuple's alone once claimed
  }
}

// Two walks of the probe chain per outer tuple: count its matches, claim
// that many output slots with one atomic, then write them.
__global__ __launch_bounds__(NPJ_T) void npjProbePairsKernel(const ulonglong2 *__restrict__ S, uint64_t n,
                                                             const unsigned long long *__restrict__ table,
                                                             const unsigned long long *__restrict__ rids,
                                                             uint64_t mask, ulonglong2 *__restrict__ out,
                                                             uint64_t capacity, unsigned long long *cursor) {
  const uint64_t stride = (uint64_t)gridDim.x * NPJ_T;
  for (uint64_t i = (uint64_t)blockIdx.x * NPJ_T + threadIdx.x; i < n; i += stride) {
    const ulonglong2 t = S[i];
    const uint64_t h0 = npjHash(t.x, mask);
    unsigned long long m = 0, e;
    for (uint64_t h = h0; (e = table[h]) != ~0ull; h = (h + 1) & mask) m += (e == t.x);
    if (m == 0) continue;
    unsigned long long at = atomicAdd(cursor, m);
    for (uint64_t h = h0; at < capacity && (e = table[h]) != ~0ull; h = (h + 1) & mask)
      if (e == t.x) out[at++] = make_ulonglong2(rids[h], t.y);
  }
}

void npjBuildRids(const data::Tuple *R, uint64_t nR, unsigned long long *table, unsigned long long *rids,
                  uint64_t slots, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(table, 0xFF, slots * sizeof(unsigned long long), s));
  if (nR == 0) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceilDiv(nR, NPJ_T), 8192);
  hipLaunchKernelGGL(npjBuildRidsKernel, dim3(blocks), dim3(NPJ_T), 0, s, reinterpret_cast<const ulonglong2 *>(R), nR,
                     table, rids, slots - 1);
  HIP_CHECK_LAUNCH();
}

void npjProbePairs(const data::Tuple *S, uint64_t nS, const unsigned long long *table,
                   const unsigned long long *rids, uint64_t slots, ulonglong2 *out, uint64_t capacity,
                   unsigned long long *cursor, hipStream_t s) {
  if (nS == 0) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceilDiv(nS, NPJ_T), 8192);
  hipLaunchKernelGGL(npjProbePairsKernel, dim3(blocks), dim3(NPJ_T), 0, s, reinterpret_cast<const ulonglong2 *>(S),
                     nS, table, rids, slots - 1, out, capacity, cursor);
  HIP_CHECK_LAUNCH();
}

void npjBuild(const data::Tuple *R, uint64_t nR, unsigned long long *table, uint64_t slots, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(table, 0xFF, slots * sizeof(unsigned long long), s));
  if (nR == 0) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceilDiv(nR, NPJ_T), 8192);
  hipLaunchKernelGGL(npjBuildKernel, dim3(blocks), dim3(NPJ_T), 0, s, reinterpret_cast<const ulonglong2 *>(R), nR,
                     table, slots - 1);
  HIP_CHECK_LAUNCH();
}

void npjProbe(const data::Tuple *S, uint64_t nS, const unsigned long long *table, uint64_t slots,
              unsigned long long *result, hipStream_t s) {
  if (nS == 0) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceilDiv(nS, NPJ_T), 8192);
  hipLaunchKernelGGL(npjProbeKernel, dim3(blocks), dim3(NPJ_T), 0, s, reinterpret_cast<const ulonglong2 *>(S), nS,
                     table, slots - 1, result);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
