// Device relation generators (replace the sequential generators and the MPI
// pairwise shuffle of /root/reference/data/Relation.cpp:63-141).
//
// Every element is a pure function of (params, global index), so each rank
// writes its slice of one global relation straight into HBM with 16-byte
// stores and no communication.  Bit-identical host versions live in
// host/HostOps.cpp (used by the CPU reference path and the tests).
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

__device__ __forceinline__ uint64_t zipfRank(const ZipfParams &z, double u) {
  double uz = u * z.zetan;
  if (uz < 1.0) return 0;
  if (uz < 1.0 + z.half_pow_theta) return 1;
  uint64_t r = (uint64_t)((double)z.n * pow(z.eta * u - z.eta + 1.0, z.alpha));
  return r >= z.n ? z.n - 1 : r;
}

__device__ __forceinline__ uint64_t genKey(const GenParams &p, uint64_t gi) {
  switch (p.dist) {
    case KeyDistribution::Unique:
      return p.keyOffset + p.perm(gi);
    case KeyDistribution::Dense:
      return p.keyOffset + gi;
    case KeyDistribution::Modulo:
      return p.keyOffset + p.perm(gi % p.modulo);
    case KeyDistribution::Uniform:
      return p.keyOffset + (uint64_t)(uniform01(p.seed, gi) * (double)p.domain) % p.domain;
    case KeyDistribution::Zipf:
    default:
      return p.keyOffset + p.perm(zipfRank(p.zipf, uniform01(p.seed, gi)));
  }
}

__global__ __launch_bounds__(256) void generateKernel(ulonglong2 *__restrict__ out, uint64_t n, GenParams p) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t gi = p.globalOffset + i;
    ulonglong2 t;
    t.x = genKey(p, gi);
    if (p.tpchSparse) t.x = tpchSparseKey(t.x);
    if (p.sparse64) t.x = sparseKey(t.x);
    t.y = p.ridOffset + i;
    out[i] = t;
  }
}

// Oracle support for skewed joins (no closed form for Zipf x Zipf):
// counts[key - lo] += 1 for keys in [lo, lo + domain), *outside += the rest.
// Global atomics (u32 counts, memory-side adds); the match count is then
// sum_k countsR[k] * countsS[k], computed independently of the join.
__global__ __launch_bounds__(256) void countKeysKernel(const ulonglong2 *__restrict__ in, uint64_t n, uint64_t lo,
                                                       uint64_t domain, uint32_t *__restrict__ counts,
                                                       unsigned long long *__restrict__ outside) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t miss = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t k = in[i].x - lo;
    if (k < domain)
      atomicAdd(&counts[k], 1u);
    else
      ++miss;
  }
  if (miss) atomicAdd(outside, (unsigned long long)miss);
}

void countKeys(const data::Tuple *in, uint64_t n, uint64_t lo, uint64_t domain, uint32_t *counts,
               unsigned long long *outside, hipStream_t s) {
  if (n == 0) return;
  const uint64_t want = ceilDiv(n, 256);
  hipLaunchKernelGGL(countKeysKernel, dim3((uint32_t)(want < 16384 ? want : 16384)), dim3(256), 0, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, lo, domain, counts, outside);
  HIP_CHECK_LAUNCH();
}

void generate(data::Tuple *out, uint64_t n, const GenParams &p, hipStream_t s) {
  if (n == 0) return;
  const uint32_t threads = 256;
  const uint64_t want = ceilDiv(n, threads);
  const uint32_t blocks = (uint32_t)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(generateKernel, dim3(blocks), dim3(threads), 0, s, reinterpret_cast<ulonglong2 *>(out), n, p);
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadDatagen() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&generateKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
