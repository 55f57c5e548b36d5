// Capacity spill: joins whose relations plus workspace exceed HBM run in K
// passes (operators/HashJoin::runPasses).  Pass k joins only the tuples whose
// key hashes to k (kernels::passOf) on both sides -- equal keys always meet in
// the same pass -- so every pass needs ~1/K of the windows, partition buffers
// and tables, and the match counts of the passes add up.
//
// Reference: the dormant large-data machinery runs a join chunk by chunk with
// histograms accumulated across iterations (operators/gpu/kernels.cu:563-857,
// data/data.hpp:12-20,67-83) and reads managed / host memory in place
// (operators/gpu/small_data_optimized.cu:848-1041).  Here the split is by key
// hash instead of input position, so a pass is a complete join of its own.
#include "kernels.h"
#include "device_common.h"

#include <algorithm>

namespace hpcjoin {
namespace kernels {

constexpr int PT = 256;

// counts[p] += tuples of in[0, n) in pass p (K <= MAX_SPILL_PASSES).
__global__ __launch_bounds__(PT) void passCountsKernel(const ulonglong2 *__restrict__ in, uint64_t n, uint32_t K,
                                                        unsigned long long *__restrict__ counts) {
  __shared__ unsigned int c[MAX_SPILL_PASSES];
  for (uint32_t p = threadIdx.x; p < K; p += PT) c[p] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * PT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * PT)
    atomicAdd(&c[passOf(in[i].x, K)], 1u);
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < K; p += PT)
    if (c[p]) atomicAdd(&counts[p], (unsigned long long)c[p]);
}

void passCounts(const data::Tuple *in, uint64_t n, uint32_t K, unsigned long long *counts, hipStream_t s) {
  HJ_CHECK(K >= 1 && K <= MAX_SPILL_PASSES, "passCounts: %u passes", K);
  if (n == 0) return;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (n + PT - 1) / PT);
  hipLaunchKernelGGL(passCountsKernel, dim3(grid), dim3(PT), 0, s, reinterpret_cast<const ulonglong2 *>(in), n, K,
                     counts);
  HIP_CHECK_LAUNCH();
}

// out[...] = the tuples of in[0, n) in pass k (any order).  A workgroup
// takes 4096-tuple tiles (16 per thread), ranks the tile's pass-k tuples with
// a block scan and reserves their run with ONE device atomic per tile: the
// per-wave version (one atomic per 64 tuples on a single counter) serialised
// on that counter at ~0.36 s per pass of 1B x 1B.
constexpr int CI = 16;
__global__ __launch_bounds__(PT) void passCompactKernel(const ulonglong2 *__restrict__ in, uint64_t n, uint32_t K,
                                                         uint32_t k, ulonglong2 *__restrict__ out,
                                                         unsigned long long *__restrict__ cursor,
                                                         unsigned long long capacity) {
  __shared__ uint32_t waveTot[PT / WAVE];
  __shared__ unsigned long long base;
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wid = t / WAVE;
  constexpr uint64_t TILE = (uint64_t)PT * CI;
  const uint64_t tiles = (n + TILE - 1) / TILE;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {  // block-uniform
    const uint64_t t0 = tile * TILE;
    ulonglong2 v[CI];
    uint32_t take = 0;  // bit i: element i of this thread is in pass k
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const uint64_t idx = t0 + (uint64_t)i * PT + t;  // coalesced; output order within a pass is free
      if (idx < n) {
        v[i] = in[idx];
        if (passOf(v[i].x, K) == k) take |= 1u << i;
      }
    }
    const uint32_t mine = (uint32_t)__popc(take);
    const uint32_t incl = waveInclusiveScan<uint32_t>(mine);
    if (lane == WAVE - 1) waveTot[wid] = incl;
    __syncthreads();
    uint32_t prefix = incl - mine, total = 0;
#pragma unroll
    for (int w = 0; w < PT / WAVE; ++w) {
      const uint32_t x = waveTot[w];
      if (w < (int)wid) prefix += x;
      total += x;
    }
    if (t == 0) base = total ? atomicAdd(cursor, (unsigned long long)total) : 0ull;
    __syncthreads();
    const unsigned long long at = base + prefix;
    uint32_t j = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i)
      if (take & (1u << i)) {
        // Never past the pass buffer: a count that drifted from the plan's
        // (relation changed after planning) shows as cursor != count on the host.
        if (at + j < capacity) out[at + j] = v[i];
        ++j;
      }
    __syncthreads();  // waveTot / base reused by the next tile
  }
}

void passCompact(const data::Tuple *in, uint64_t n, uint32_t K, uint32_t k, data::Tuple *out,
                 unsigned long long *cursor, hipStream_t s, uint64_t capacity) {
  HJ_CHECK(K >= 1 && K <= MAX_SPILL_PASSES && k < K, "passCompact: pass %u of %u", k, K);
  if (n == 0) return;
  const uint64_t tiles = (n + (uint64_t)PT * CI - 1) / ((uint64_t)PT * CI);
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, tiles);
  hipLaunchKernelGGL(passCompactKernel, dim3(grid), dim3(PT), 0, s, reinterpret_cast<const ulonglong2 *>(in), n, K,
                     k, reinterpret_cast<ulonglong2 *>(out), cursor, (unsigned long long)capacity);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
