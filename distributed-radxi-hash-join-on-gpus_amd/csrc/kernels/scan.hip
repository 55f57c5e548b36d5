// Device exclusive scan (u32) built from wave64 shuffles and LDS block scans.
// Replaces the thrust::exclusive_scan calls of the reference GPU drivers
// (/root/reference/operators/gpu/small_data.cu:95-155).  Three launches:
// per-block reduce -> single-block scan of block sums -> per-block downsweep.
#include "kernels.h"

#include <algorithm>
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

constexpr int SCAN_T = 256;
constexpr int SCAN_PER = 8;
constexpr uint32_t SCAN_TILE = SCAN_T * SCAN_PER;

size_t scanWorkspaceBytes(uint64_t n) { return (ceilDiv(n, SCAN_TILE) + 16) * sizeof(uint64_t); }

template <typename T>
__global__ __launch_bounds__(SCAN_T) void scanReduceKernel(const uint32_t *__restrict__ in, uint64_t n,
                                                           T *__restrict__ sums) {
  __shared__ T wt[SCAN_T / WAVE];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  T s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    const uint64_t idx = base + (uint64_t)i * SCAN_T + threadIdx.x;
    if (idx < n) s += in[idx];
  }
  s = blockReduceSum<SCAN_T, T>(s, wt);
  if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

template <typename T>
__global__ __launch_bounds__(SCAN_T) void scanSumsKernel(T *sums, uint32_t nb, T *total) {
  __shared__ T wt[SCAN_T / WAVE];
  const T t = blockExclusiveScanLds<SCAN_T, T, T>(sums, sums, (int)nb, wt);
  if (threadIdx.x == 0 && total) *total = t;
}

template <typename T>
__global__ __launch_bounds__(SCAN_T) void scanDownKernel(const uint32_t *__restrict__ in, uint64_t n,
                                                         const T *__restrict__ sums, T *__restrict__ out) {
  __shared__ T tile[SCAN_TILE];
  __shared__ T wt[SCAN_T / WAVE];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  const uint32_t cnt = (uint32_t)min((uint64_t)SCAN_TILE, n - base);
  for (uint32_t i = threadIdx.x; i < SCAN_TILE; i += SCAN_T) tile[i] = i < cnt ? in[base + i] : 0;
  __syncthreads();
  blockExclusiveScanLds<SCAN_T, T, T>(tile, tile, (int)SCAN_TILE, wt);
  const T off = sums[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < cnt; i += SCAN_T) out[base + i] = tile[i] + off;
}

template <typename T>
static void scanExclusive(const uint32_t *in, T *out, uint64_t n, T *total, void *workspace, hipStream_t s) {
  if (n == 0) {
    if (total) HIP_CHECK(hipMemsetAsync(total, 0, sizeof(T), s));
    return;
  }
  const uint32_t nb = (uint32_t)ceilDiv(n, SCAN_TILE);
  T *sums = reinterpret_cast<T *>(workspace);
  hipLaunchKernelGGL(scanReduceKernel<T>, dim3(nb), dim3(SCAN_T), 0, s, in, n, sums);
  HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(scanSumsKernel<T>, dim3(1), dim3(SCAN_T), 0, s, sums, nb, total);
  HIP_CHECK_LAUNCH();
  hipLaunchKernelGGL(scanDownKernel<T>, dim3(nb), dim3(SCAN_T), 0, s, in, n, sums, out);
  HIP_CHECK_LAUNCH();
}

void scanExclusiveU32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *workspace,
                      hipStream_t s) {
  scanExclusive<uint32_t>(in, out, n, total, workspace, s);
}

void scanExclusiveU32to64(const uint32_t *in, unsigned long long *out, uint64_t n, unsigned long long *total,
                          void *workspace, hipStream_t s) {
  scanExclusive<unsigned long long>(in, out, n, total, workspace, s);
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
// Zero fill with the engine's own kernel (no runtime fill kernel: those are
// loaded lazily by the runtime on first use).
__global__ __launch_bounds__(SCAN_T) void zeroWordsKernel(unsigned long long *p, uint64_t words) {
  for (uint64_t i = (uint64_t)blockIdx.x * SCAN_T + threadIdx.x; i < words; i += (uint64_t)gridDim.x * SCAN_T)
    p[i] = 0;
}

void zeroWords(void *p, uint64_t words, hipStream_t s) {
  if (words == 0) return;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (words + SCAN_T - 1) / SCAN_T);
  hipLaunchKernelGGL(zeroWordsKernel, dim3(grid), dim3(SCAN_T), 0, s, static_cast<unsigned long long *>(p), words);
  HIP_CHECK_LAUNCH();
}

// dst (pinned, device-mapped host memory) = src, by the engine's own kernel:
// a join's small read-backs need no copy engine (SDMA: the first copy of a
// process stalled its join by ~12-17 ms, profiles/r1_sdma_outlier.md) and no
// runtime blit kernel.  System-scope stores: visible to the host once the
// kernel (and the event behind it) completes.
template <typename W>
__global__ __launch_bounds__(SCAN_T) void copyToHostKernel(W *dst, const W *__restrict__ src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * SCAN_T + threadIdx.x; i < n; i += (uint64_t)gridDim.x * SCAN_T)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void copyFromHost(void *dst, const void *src, uint64_t bytes, hipStream_t s) { copyToHost(dst, src, bytes, s); }

void copyToHost(void *dst, const void *src, uint64_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes;
  auto go = [&](auto w) {
    using W = decltype(w);
    const uint64_t n = bytes / sizeof(W);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(256, (n + SCAN_T - 1) / SCAN_T);
    hipLaunchKernelGGL(copyToHostKernel<W>, dim3(grid), dim3(SCAN_T), 0, s, static_cast<W *>(dst),
                       static_cast<const W *>(src), n);
  };
  if ((a & 7) == 0)
    go((unsigned long long)0);
  else if ((a & 3) == 0)
    go(0u);
  else
    go((unsigned char)0);
  HIP_CHECK_LAUNCH();
}

void preloadScan() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&scanSumsKernel<uint32_t>)));
}

}  // namespace kernels
}  // namespace hpcjoin
