// Device-side reduction for ranks that share one process and one device
// (comm/InProcessCommunicator): rank r sums slice r of every rank's buffer and
// writes the sum back into all of them.  Only rank r touches slice r, so the
// ranks need one barrier before (every buffer final) and one after (every
// slice written) -- no staging through the host.  RCCL does the same job
// with ncclAllReduce across processes (comm/RcclCommunicator).
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

constexpr int AR_NT = 256;
constexpr uint32_t AR_MAX_RANKS = 64;

__global__ __launch_bounds__(AR_NT) void sumSlicesKernel(uint64_t *const *__restrict__ bufs, uint32_t n,
                                                         uint64_t lo, uint64_t hi) {
  const uint64_t stride = (uint64_t)gridDim.x * AR_NT;
  for (uint64_t i = lo + (uint64_t)blockIdx.x * AR_NT + threadIdx.x; i < hi; i += stride) {
    uint64_t s = 0;
    for (uint32_t r = 0; r < n; ++r) s += bufs[r][i];
    for (uint32_t r = 0; r < n; ++r) bufs[r][i] = s;
  }
}

void sumSlices(uint64_t *const *devBufs, uint32_t n, uint64_t lo, uint64_t hi, hipStream_t s) {
  HJ_CHECK(n >= 1 && n <= AR_MAX_RANKS, "sumSlices: %u ranks", n);
  if (hi <= lo) return;
  const uint64_t want = ceilDiv(hi - lo, (uint64_t)AR_NT);
  const uint32_t grid = (uint32_t)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(sumSlicesKernel, dim3(grid), dim3(AR_NT), 0, s, devBufs, n, lo, hi);
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadCollectives() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sumSlicesKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
