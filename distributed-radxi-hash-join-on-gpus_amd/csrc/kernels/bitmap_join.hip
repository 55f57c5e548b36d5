// Single-level counting join for unique inner keys: one LDS bitmap per network
// partition.
//
// After the network pass every partition holds the key fragments above the
// network digit (CompressedTuple: value >> keyShift).  With dense keys the
// fragment range of one partition is 2^(keyBits - networkBits); when that fits
// an LDS bitmap (<= 2^20 bits = 128 KiB) the partition is joined in place, as
// the reference's default single-level plan does
// (core/Configuration.h:28 ENABLE_TWO_LEVEL_PARTITIONING=false; build/probe per
// network partition, tasks/BuildProbe.cpp:47-121), without the second radix
// pass.  Build: atomicOr of the fragment's bit; a bit that was already set is
// a duplicate inner key, which the bitmap cannot count -- the kernel raises
// `dup` and the caller redoes the join with the two-level pass.  Probe: one
// LDS bit test per outer tuple.  Partitions arrive as the sampled network
// pass's claim slices (up to `groups` segments per partition, gaps between).
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

constexpr int BM_NTH = 1024;
constexpr int BM_U = 8;  // loads in flight per lane

__device__ __forceinline__ uint64_t bmLoad(const uint64_t *p) { return __builtin_nontemporal_load(p); }

__global__ __launch_bounds__(BM_NTH) void bitmapJoinKernel(
    const uint64_t *__restrict__ r, const uint64_t *__restrict__ s, const uint64_t *__restrict__ rStart,
    const uint32_t *__restrict__ rLen, const uint64_t *__restrict__ sStart, const uint32_t *__restrict__ sLen,
    uint32_t groups, uint32_t keyShift, uint32_t words, unsigned long long *__restrict__ matches,
    uint32_t *__restrict__ dup) {
  extern __shared__ uint32_t bm[];
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  for (uint32_t w = t; w < words; w += BM_NTH) bm[w] = 0;
  __syncthreads();
  const uint64_t limit = (uint64_t)words * 32;
  uint32_t dupv = 0;
  for (uint32_t g = 0; g < groups; ++g) {
    const uint64_t *src = r + rStart[(size_t)d * groups + g];
    const uint32_t n = rLen[(size_t)d * groups + g];
    for (uint32_t i0 = 0; i0 < n; i0 += BM_NTH * BM_U) {
      uint64_t v[BM_U];
#pragma unroll
      for (int k = 0; k < BM_U; ++k) {
        const uint32_t i = i0 + k * BM_NTH + t;
        v[k] = i < n ? bmLoad(src + i) : ~0ull;
      }
#pragma unroll
      for (int k = 0; k < BM_U; ++k) {
        if (i0 + k * BM_NTH + t >= n) continue;
        const uint64_t f = v[k] >> keyShift;
        if (f >= limit) {  // outside the planned range: let the caller fall back
          dupv = 1;
          continue;
        }
        const uint32_t bit = 1u << (f & 31);
        dupv |= (atomicOr(&bm[f >> 5], bit) & bit) ? 1u : 0u;
      }
    }
  }
  __syncthreads();
  uint32_t cnt = 0;
  for (uint32_t g = 0; g < groups; ++g) {
    const uint64_t *src = s + sStart[(size_t)d * groups + g];
    const uint32_t n = sLen[(size_t)d * groups + g];
    for (uint32_t i0 = 0; i0 < n; i0 += BM_NTH * BM_U) {
      uint64_t v[BM_U];
#pragma unroll
      for (int k = 0; k < BM_U; ++k) {
        const uint32_t i = i0 + k * BM_NTH + t;
        v[k] = i < n ? bmLoad(src + i) : ~0ull;
      }
#pragma unroll
      for (int k = 0; k < BM_U; ++k) {
        const uint64_t f = v[k] >> keyShift;  // padding lanes carry ~0 >> keyShift >= limit
        if (f < limit) cnt += (bm[f >> 5] >> (f & 31)) & 1u;
      }
    }
  }
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((t & (WAVE - 1)) == 0 && cnt) atomicAdd(matches, (unsigned long long)cnt);
  if (dupv) atomicOr(dup, 1u);
}

void bitmapJoin(const uint64_t *r, const uint64_t *s, const uint64_t *rStart, const uint32_t *rLen,
                const uint64_t *sStart, const uint32_t *sLen, uint32_t partitions, uint32_t groups,
                uint32_t keyShift, uint32_t bits, unsigned long long *matches, uint32_t *dup, hipStream_t st) {
  HJ_CHECK(bits <= BITMAP_MAX_BITS, "bitmapJoin: %u fragment bits exceed the %u-bit LDS bitmap", bits,
           BITMAP_MAX_BITS);
  HJ_CHECK(keyShift < 64, "bitmapJoin: keyShift=%u", keyShift);
  if (partitions == 0) return;
  const uint32_t words = bits > 5 ? 1u << (bits - 5) : 1u;
  hipLaunchKernelGGL(bitmapJoinKernel, dim3(partitions), dim3(BM_NTH), (size_t)words * 4, st, r, s, rStart, rLen,
                     sStart, sLen, groups, keyShift, words, matches, dup);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
