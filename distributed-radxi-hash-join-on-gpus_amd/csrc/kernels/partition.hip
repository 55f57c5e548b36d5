// Radix partitioning kernels for MI355X (gfx950): both passes of the join.
//
// Pass 1 (network partitioning) replaces the CPU software-write-combining loop
// of /root/reference/tasks/NetworkPartitioning.cpp:74-222 and the LocalHistogram
// pass of /root/reference/histograms/LocalHistogram.cpp:35-53.  Pass 2 (local
// partitioning) replaces /root/reference/tasks/LocalPartitioning.cpp:138-250.
//
// Design (CDNA4-first, not a translation):
//  * Histogram: one workgroup (4 wave64s) owns a contiguous run of 4096-tuple
//    tiles; each wave counts into its own LDS sub-histogram (4 x F u32), which
//    cuts LDS atomic contention 4x, then the block writes a digit-major
//    [F][blocks] histogram so ONE exclusive scan per digit yields every
//    block's private output cursor (no global atomics, no inter-WG hand-off).
//  * Scatter = LDS write-combining: each tile is ranked per digit with LDS
//    atomics, block-scanned, reordered through LDS so that consecutive lanes
//    hold consecutive tuples of the same digit, then streamed out.  Because a
//    workgroup's tiles are contiguous and its cursors persist in LDS, a
//    digit's output run continues across tiles and the L2 / Infinity Cache
//    merge the partial lines (the GPU analog of the reference's 64-byte
//    cache-line buffers + non-temporal flushes).
//  * The packed CompressedTuple (8 B) halves everything written after pass 1.
#include "kernels.h"
#include "device_common.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <type_traits>

namespace hpcjoin {
namespace kernels {

constexpr int NT = PART_THREADS;
constexpr uint32_t NGROUPS = 8;  // XCDs on MI355X

PartitionGeometry partitionGeometry(uint64_t n, uint32_t maxBlocks) {
  PartitionGeometry g;
  const uint64_t tiles = ceilDiv(n, PART_TILE);
  if (tiles == 0) {
    g.blocks = 1;
    g.tilesPerBlock = 1;
    return g;
  }
  g.tilesPerBlock = (uint32_t)ceilDiv(tiles, maxBlocks);
  g.blocks = (uint32_t)ceilDiv(tiles, g.tilesPerBlock);
  return g;
}


// ------------------------------------------------------------------ loads
// Input streams are read exactly once: non-temporal loads keep them from
// evicting the partially filled output lines the L2 is write-combining.
using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));
template <typename InT>
struct Loader;
template <>
struct Loader<ulonglong2> {
  static __device__ __forceinline__ ulonglong2 load(const ulonglong2 *p) {
    const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    return make_ulonglong2(v.x, v.y);
  }
};
template <>
struct Loader<uint64_t> {
  static __device__ __forceinline__ uint64_t load(const uint64_t *p) { return __builtin_nontemporal_load(p); }
};
template <>
struct Loader<uint32_t> {
  static __device__ __forceinline__ uint32_t load(const uint32_t *p) { return __builtin_nontemporal_load(p); }
};

// What a scatter policy loads per element.  PlainLoad: the whole input
// element.  KeyLoad: only the key of a 16-byte tuple, for policies whose
// output never carries the rid (count-only fragments, key-only words): half
// the VGPRs per element in flight.  With whole tuples the frag scatter sat at
// 121 VGPRs and the compiler reused the dead rid halves of pending loads for
// address arithmetic, which put an s_waitcnt vmcnt(0) after every second
// load of the next tile's prefetch (three serial HBM round trips per tile).
template <typename In>
struct PlainLoad {
  using LoadT = In;
  static __device__ __forceinline__ LoadT load(const In *p) { return Loader<In>::load(p); }
};
struct KeyLoad {
  using LoadT = uint64_t;
  static __device__ __forceinline__ LoadT load(const ulonglong2 *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(p));
  }
};

// ------------------------------------------------------- histogram (pass 1)
__device__ __forceinline__ void netHistogramBody(const ulonglong2 *__restrict__ in, uint64_t n, uint32_t tpb,
                                                 uint32_t bits, uint32_t *__restrict__ blockHist, KeyMix mix,
                                                 uint32_t stride, uint32_t *hsh) {
  const uint32_t F = 1u << bits, mask = F - 1;
  const int wid = threadIdx.x / WAVE;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  uint32_t *wh = hsh + wid * F;
  const uint64_t begin = (uint64_t)blockIdx.x * tpb * PART_TILE;
  const uint64_t end = min(n, begin + (uint64_t)tpb * PART_TILE);
  for (uint64_t base = begin; base < end; base += (uint64_t)PART_TILE * stride) {
    uint64_t k[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint64_t idx = base + (uint64_t)i * NT + threadIdx.x;
      k[i] = idx < end ? mix.apply(in[idx].x) : 0;
    }
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint64_t idx = base + (uint64_t)i * NT + threadIdx.x;
      if (idx < end) atomicAdd(&wh[k[i] & mask], 1u);
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < F; d += NT)
    blockHist[(uint64_t)d * gridDim.x + blockIdx.x] = hsh[d] + hsh[F + d] + hsh[2 * F + d] + hsh[3 * F + d];
}

// Exact (every tile) and sampled (1 tile in `stride`) launches are separate
// kernels so that a trace tells a full pre-read from a sample.
__global__ __launch_bounds__(NT) void netHistogramKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                         uint32_t tpb, uint32_t bits,
                                                         uint32_t *__restrict__ blockHist, KeyMix mix) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  netHistogramBody(in, n, tpb, bits, blockHist, mix, 1, hsh);
}

__global__ __launch_bounds__(NT) void netSampledHistogramKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                                uint32_t tpb, uint32_t bits,
                                                                uint32_t *__restrict__ blockHist, KeyMix mix,
                                                                uint32_t stride) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  netHistogramBody(in, n, tpb, bits, blockHist, mix, stride, hsh);
}

void netHistogram(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                  uint32_t *blockHist, hipStream_t s, KeyMix mix, uint32_t sampleStride) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netHistogram: bits=%u out of range", bits);
  HJ_CHECK(sampleStride >= 1, "netHistogram: sampleStride must be >= 1");
  const size_t lds = size_t(4) << bits << 2;
  if (sampleStride > 1)
    hipLaunchKernelGGL(netSampledHistogramKernel, dim3(g.blocks), dim3(NT), lds, s,
                       reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock, bits, blockHist, mix,
                       sampleStride);
  else
    hipLaunchKernelGGL(netHistogramKernel, dim3(g.blocks), dim3(NT), lds, s, reinterpret_cast<const ulonglong2 *>(in),
                       n, g.tilesPerBlock, bits, blockHist, mix);
  HIP_CHECK_LAUNCH();
}

// ---------------------------------------- sampled per-(group, digit) totals
// A sampled pass only needs per-(XCD group, digit) totals.  Group g's tiles
// (those of blocks b = g mod NGROUPS, block by block) are numbered 0, 1, ...;
// every stride-th of them is sampled, one workgroup per sampled tile, and its
// LDS histogram is added into totals[g][d] with one device atomic per
// non-empty digit.  Against netHistogram + netGroupTotals (every block of the
// geometry runs, samples its own tiles and writes F block counts) this reads
// 1/stride of the input at every size -- a block range shorter than stride
// tiles still sampled one full tile, 1/15 of a 125M-tuple input -- and writes
// no per-block array (47-57 us -> see profiles at 125M).  sampleScale()
// computes the same tile set on the host.
__host__ __device__ inline uint64_t sampledTile(uint64_t local, uint32_t g, uint32_t tpb) {
  return ((local / tpb) * NGROUPS + g) * tpb + local % tpb;
}

struct SampledSideArgs {
  const ulonglong2 *in;
  uint64_t n;
  uint32_t tpb, blocks, stride;
  unsigned long long *totals;  // [NGROUPS][F]
};

// Workgroups [0, wgA) sample side a, the rest side b (both sides of a join
// in one launch).
__global__ __launch_bounds__(NT) void netSampledTotalsKernel(SampledSideArgs a, SampledSideArgs b, uint32_t wgA,
                                                             uint32_t bits, KeyMix mix) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  const bool onB = blockIdx.x >= wgA;
  const SampledSideArgs &sd = onB ? b : a;
  const uint32_t w = onB ? blockIdx.x - wgA : blockIdx.x;
  const uint32_t g = w % NGROUPS;
  const uint64_t local = (uint64_t)(w / NGROUPS) * sd.stride;
  const uint64_t tile = sampledTile(local, g, sd.tpb);
  const uint64_t begin = tile * PART_TILE, n = sd.n;
  if (tile / sd.tpb >= sd.blocks || begin >= n) return;  // uniform over the workgroup
  const uint64_t end = min(n, begin + PART_TILE);
  const ulonglong2 *__restrict__ in = sd.in;
  const uint32_t F = 1u << bits, mask = F - 1;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  uint32_t *wh = hsh + (threadIdx.x / WAVE) * F;
  uint64_t k[PART_ITEMS];
#pragma unroll
  for (int i = 0; i < (int)PART_ITEMS; ++i) {
    const uint64_t idx = begin + (uint64_t)i * NT + threadIdx.x;
    k[i] = idx < end ? mix.apply(in[idx].x) : 0;
  }
#pragma unroll
  for (int i = 0; i < (int)PART_ITEMS; ++i) {
    const uint64_t idx = begin + (uint64_t)i * NT + threadIdx.x;
    if (idx < end) atomicAdd(&wh[k[i] & mask], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < F; d += NT) {
    const uint32_t c = hsh[d] + hsh[F + d] + hsh[2 * F + d] + hsh[3 * F + d];
    if (c) atomicAdd(&sd.totals[(uint64_t)g * F + d], (unsigned long long)c);
  }
}

// Tiles of XCD group g in geometry gm (blocks b = g mod NGROUPS).
static uint64_t groupTiles(const PartitionGeometry &gm, uint64_t n, uint32_t g) {
  const uint64_t tiles = ceilDiv(n, PART_TILE);
  uint64_t t = 0;
  for (uint32_t b = g; b < gm.blocks; b += NGROUPS) {
    const uint64_t b0 = (uint64_t)b * gm.tilesPerBlock;
    if (b0 < tiles) t += std::min<uint64_t>(gm.tilesPerBlock, tiles - b0);
  }
  return t;
}

uint32_t sampleStrideFor(const PartitionGeometry &g, uint64_t n, uint32_t F, uint32_t stride) {
  uint64_t minTiles = UINT64_MAX;
  for (uint32_t gr = 0; gr < NGROUPS; ++gr) {
    const uint64_t t = groupTiles(g, n, gr);
    if (t) minTiles = std::min(minTiles, t);
  }
  if (minTiles == UINT64_MAX || stride <= 1) return 1;
  const uint64_t most = minTiles * PART_TILE / (32ull * std::max<uint32_t>(F, 1));
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(stride, most));
}

// Workgroups one side needs (sampled tiles of its largest XCD group x groups).
static uint32_t sampledWorkgroups(const PartitionGeometry &g, uint64_t n, uint32_t stride) {
  uint64_t perGroup = 0;
  for (uint32_t gr = 0; gr < NGROUPS; ++gr) perGroup = std::max(perGroup, ceilDiv(groupTiles(g, n, gr), stride));
  HJ_CHECK(perGroup * NGROUPS < (1ull << 30), "netSampledTotals: %llu sampled tiles", (unsigned long long)perGroup);
  return (uint32_t)(perGroup * NGROUPS);
}

static SampledSideArgs sampledSide(const SampledInput &x) {
  HJ_CHECK(x.stride >= 1, "netSampledTotals: sampleStride must be >= 1");
  return SampledSideArgs{reinterpret_cast<const ulonglong2 *>(x.data), x.n, x.geom.tilesPerBlock, x.geom.blocks,
                         x.stride, reinterpret_cast<unsigned long long *>(x.totals)};
}

void netSampledTotals(const SampledInput *sides, uint32_t count, uint32_t bits, hipStream_t s, KeyMix mix,
                      bool preZeroed) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netSampledTotals: bits=%u out of range", bits);
  HJ_CHECK(count == 1 || count == 2, "netSampledTotals: %u sides", count);
  const uint32_t F = 1u << bits;
  const size_t bytes = (size_t)NGROUPS * F * sizeof(uint64_t);
  // Both sides' totals adjacent: one clear.
  if (preZeroed) {
    // DeviceControl totals: the layout kernel that read them last cleared them.
  } else if (count == 2 && sides[1].totals == sides[0].totals + (size_t)NGROUPS * F) {
    HIP_CHECK(hipMemsetAsync(sides[0].totals, 0, 2 * bytes, s));
  } else {
    for (uint32_t i = 0; i < count; ++i) HIP_CHECK(hipMemsetAsync(sides[i].totals, 0, bytes, s));
  }
  const SampledSideArgs a = sampledSide(sides[0]), b = count == 2 ? sampledSide(sides[1]) : a;
  const uint32_t wgA = sampledWorkgroups(sides[0].geom, sides[0].n, sides[0].stride);
  const uint32_t wgB = count == 2 ? sampledWorkgroups(sides[1].geom, sides[1].n, sides[1].stride) : 0;
  if (wgA + wgB == 0) return;
  const size_t lds = size_t(4) << bits << 2;
  hipLaunchKernelGGL(netSampledTotalsKernel, dim3(wgA + wgB), dim3(NT), lds, s, a, b, wgA, bits, mix);
  HIP_CHECK_LAUNCH();
}

void netSampledTotals(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                      uint64_t *totals, hipStream_t s, KeyMix mix, uint32_t sampleStride) {
  const SampledInput one{in, n, g, sampleStride, totals};
  netSampledTotals(&one, 1, bits, s, mix);
}

// --------------------------------------------------- digit totals / cursors
__global__ __launch_bounds__(NT) void digitTotalsKernel(const uint32_t *__restrict__ blockHist, uint32_t F,
                                                        uint32_t blocks, uint32_t bpc, uint64_t *totals) {
  __shared__ uint64_t wt[NT / WAVE];
  const uint32_t d = blockIdx.x, c = blockIdx.y;
  const uint32_t b0 = c * bpc, b1 = min(blocks, b0 + bpc);
  uint64_t s = 0;
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += NT) s += blockHist[(uint64_t)d * blocks + b];
  s = blockReduceSum<NT, uint64_t>(s, wt);
  if (threadIdx.x == 0) totals[(uint64_t)c * F + d] = s;
}

void digitTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                 uint32_t chunks, uint64_t *totals, hipStream_t s) {
  hipLaunchKernelGGL(digitTotalsKernel, dim3(F, chunks), dim3(NT), 0, s, blockHist, F, blocks, blocksPerChunk,
                     totals);
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(NT) void netCursorsKernel(const uint32_t *__restrict__ blockHist, uint32_t F,
                                                       uint32_t blocks, uint32_t bpc, const uint64_t *base,
                                                       uint64_t *cursors) {
  __shared__ uint64_t wt[NT / WAVE];
  const uint32_t d = blockIdx.x;
  const uint32_t chunks = (blocks + bpc - 1) / bpc;
  for (uint32_t c = 0; c < chunks; ++c) {
    const uint32_t b0 = c * bpc, nb = min(blocks, b0 + bpc) - b0;
    const uint64_t off = (uint64_t)d * blocks + b0;
    const uint64_t bse = base[(uint64_t)c * F + d];
    // exclusive scan of blockHist[d][b0..b0+nb) (global) -> cursors (global)
    const int per = (nb + NT - 1) / NT;
    const int b = threadIdx.x * per;
    uint64_t local = 0;
    for (int i = 0; i < per; ++i)
      if (b + i < (int)nb) local += blockHist[off + b + i];
    const uint64_t incl = waveInclusiveScan<uint64_t>(local);
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    __syncthreads();
    if (lane == WAVE - 1) wt[wid] = incl;
    __syncthreads();
    uint64_t prefix = 0;
    for (int w = 0; w < wid; ++w) prefix += wt[w];
    uint64_t run = bse + prefix + incl - local;
    for (int i = 0; i < per; ++i)
      if (b + i < (int)nb) {
        const uint64_t v = blockHist[off + b + i];
        cursors[off + b + i] = run;
        run += v;
      }
  }
}

void netCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                const uint64_t *base, uint64_t *cursors, hipStream_t s) {
  hipLaunchKernelGGL(netCursorsKernel, dim3(F), dim3(NT), 0, s, blockHist, F, blocks, blocksPerChunk, base,
                     cursors);
  HIP_CHECK_LAUNCH();
}

// Group cursors for claim-mode scatter: the workgroups of a chunk are split
// into NGROUPS groups by (block - chunkBegin) % NGROUPS, which is the XCD
// round-robin of the dispatcher (a speed assumption only).  Each group owns a
// contiguous slice of every digit's region, sized by the group's histogram,
// and its workgroups claim space from the slice with one device atomic per
// digit per tile.  gcur[c][g][d] = base[c][d] + sum of the earlier groups.
template <typename CurT>
__global__ __launch_bounds__(NT) void netGroupCursorsKernel(const uint32_t *__restrict__ blockHist, uint32_t F,
                                                            uint32_t blocks, uint32_t bpc, const uint64_t *base,
                                                            CurT *gcur) {
  __shared__ unsigned long long gs[NGROUPS];
  const uint32_t d = blockIdx.x;
  const uint32_t chunks = (blocks + bpc - 1) / bpc;
  for (uint32_t c = 0; c < chunks; ++c) {
    if (threadIdx.x < NGROUPS) gs[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b0 = c * bpc, b1 = min(blocks, b0 + bpc);
    unsigned long long mine = 0;  // NT % NGROUPS == 0: thread t only sees group t % NGROUPS
    for (uint32_t b = b0 + threadIdx.x; b < b1; b += NT) mine += blockHist[(uint64_t)d * blocks + b];
    atomicAdd(&gs[threadIdx.x % NGROUPS], mine);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long run = base[(uint64_t)c * F + d];
      for (uint32_t g = 0; g < NGROUPS; ++g) {
        gcur[((uint64_t)c * NGROUPS + g) * F + d] = (CurT)run;
        run += gs[g];
      }
    }
    __syncthreads();
  }
}

void netGroupCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                     const uint64_t *base, void *gcur, bool narrow, hipStream_t s) {
  if (narrow)
    hipLaunchKernelGGL(netGroupCursorsKernel<uint32_t>, dim3(F), dim3(NT), 0, s, blockHist, F, blocks, blocksPerChunk,
                       base, reinterpret_cast<uint32_t *>(gcur));
  else
    hipLaunchKernelGGL(netGroupCursorsKernel<unsigned long long>, dim3(F), dim3(NT), 0, s, blockHist, F, blocks,
                       blocksPerChunk, base, reinterpret_cast<unsigned long long *>(gcur));
  HIP_CHECK_LAUNCH();
}

// totals[c][g][d]: one workgroup per (digit, chunk); thread t only sees
// blocks of group t % NGROUPS (NT % NGROUPS == 0, b0 is where the groups start).
__global__ __launch_bounds__(NT) void netChunkGroupTotalsKernel(const uint32_t *__restrict__ blockHist, uint32_t F,
                                                                uint32_t blocks, uint32_t bpc,
                                                                unsigned long long *totals) {
  __shared__ unsigned long long gs[NGROUPS];
  const uint32_t d = blockIdx.x, c = blockIdx.y;
  const uint32_t b0 = c * bpc, b1 = min(blocks, b0 + bpc);
  if (threadIdx.x < NGROUPS) gs[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long mine = 0;
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += NT) mine += blockHist[(uint64_t)d * blocks + b];
  atomicAdd(&gs[threadIdx.x % NGROUPS], mine);
  __syncthreads();
  if (threadIdx.x < NGROUPS) totals[((uint64_t)c * NGROUPS + threadIdx.x) * F + d] = gs[threadIdx.x];
}

void netChunkGroupTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                         uint32_t chunks, uint64_t *totals, hipStream_t s) {
  HJ_CHECK(blocksPerChunk >= 1 && (uint64_t)chunks * blocksPerChunk >= blocks, "netChunkGroupTotals: %u x %u < %u",
           chunks, blocksPerChunk, blocks);
  hipLaunchKernelGGL(netChunkGroupTotalsKernel, dim3(F, chunks), dim3(NT), 0, s, blockHist, F, blocks,
                     blocksPerChunk, reinterpret_cast<unsigned long long *>(totals));
  HIP_CHECK_LAUNCH();
}

// totals[g][d] = sum of blockHist[d][b] over the blocks b of XCD group g (b % NGROUPS == g).
__global__ __launch_bounds__(NT) void netGroupTotalsKernel(const uint32_t *__restrict__ blockHist, uint32_t F,
                                                           uint32_t blocks, unsigned long long *totals) {
  __shared__ unsigned long long gs[NGROUPS];
  const uint32_t d = blockIdx.x;
  if (threadIdx.x < NGROUPS) gs[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long mine = 0;  // NT % NGROUPS == 0: thread t only sees group t % NGROUPS
  for (uint32_t b = threadIdx.x; b < blocks; b += NT) mine += blockHist[(uint64_t)d * blocks + b];
  atomicAdd(&gs[threadIdx.x % NGROUPS], mine);
  __syncthreads();
  if (threadIdx.x < NGROUPS) totals[(uint64_t)threadIdx.x * F + d] = gs[threadIdx.x];
}

void netGroupTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint64_t *totals, hipStream_t s) {
  hipLaunchKernelGGL(netGroupTotalsKernel, dim3(F), dim3(NT), 0, s, blockHist, F, blocks,
                     reinterpret_cast<unsigned long long *>(totals));
  HIP_CHECK_LAUNCH();
}

// -------------------------------------------------- LDS write-combining scatter
// A scatter policy says how a tuple is ranked (digit), what is staged in LDS
// (the packed output word, possibly carrying its digit in spare top bits),
// how the digit is recovered from the staged word and what is finally
// written.  Only the compressed network pass may need a separate LDS digit
// array: the local pass and wide tuples recompute the digit from the staged
// word, and compressed words carry it in their top bits whenever the key
// range leaves `bits` spare bits (JoinPlan knows; the 1B config does).
struct NetCompressedPol : PlainLoad<ulonglong2> {  // 16 B tuple -> 8 B CompressedTuple, digit in the top bits
  using InT = ulonglong2;
  using StageT = uint64_t;
  using OutT = uint64_t;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  uint32_t bits, keyShift;
  KeyMix mix;
  // ~0 = keep the rid below keyShift; 0 = key-only words (count-only joins of
  // keys too wide for a CompressedTuple: value = key >> bits, keyShift = 0).
  uint64_t ridMask = ~0ull;
  __device__ __forceinline__ uint32_t digit(const InT &x) const { return (uint32_t)(mix.apply(x.x) & mask); }
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t d) const {
    return (x.y & ridMask) | ((mix.apply(x.x) >> bits) << keyShift) | ((uint64_t)d << (64 - bits));
  }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return (uint32_t)(v >> (64 - bits)); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v & (~0ull >> bits); }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
struct NetCompressedDigPol : NetCompressedPol {  // no spare bits: digits staged separately
  static constexpr bool kDigArray = true;
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t) const {
    return (x.y & ridMask) | ((mix.apply(x.x) >> bits) << keyShift);
  }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v; }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
// Key-only words (count-only joins of keys too wide for a CompressedTuple,
// JoinPlan::keyOnly): value = mixed key >> bits, digit in the top bits (the
// word has `bits` spare bits by construction); only keys are loaded.  MIX is
// the plan's key mixing as a compile-time choice (no branch per element).
template <bool MIX>
__device__ __forceinline__ uint64_t mixKey(const KeyMix &m, uint64_t k) {
  if constexpr (MIX)
    return KeyMix{1u, m.bits}.apply(k);
  else
    return k;
}
template <bool MIX>
struct NetKeyPol : KeyLoad {
  using InT = ulonglong2;
  using StageT = uint64_t;
  using OutT = uint64_t;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  uint32_t bits;
  KeyMix mix;
  __device__ __forceinline__ uint32_t digit(const LoadT &k) const { return (uint32_t)(mixKey<MIX>(mix, k) & mask); }
  __device__ __forceinline__ StageT stage(const LoadT &k, uint32_t d) const {
    return (mixKey<MIX>(mix, k) >> bits) | ((uint64_t)d << (64 - bits));
  }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return (uint32_t)(v >> (64 - bits)); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v & (~0ull >> bits); }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
// Count-only projection: a counting join never reads a rid, so the network
// pass keeps only the key fragment above the network digit (4 bytes instead
// of the 8-byte CompressedTuple; the reference compares key bits only,
// tasks/BuildProbe.cpp:101-102, and reports only the count, :115).  The
// digit rides in the staged word's top bits (fragBits + bits <= 32, checked
// by the launcher).
//
// FILT (partition-group passes, kernels.h netScatterFragRange): only digits
// [dLo, dLo + range) are written, renumbered 0..range-1; every other tuple
// gets the sentinel digit `range`, is ranked and staged behind the kept ones
// and never stored (scatterTile: FilterOf).
template <bool FILT>
__device__ __forceinline__ uint32_t rangeDigit(uint32_t d, uint32_t dLo, uint32_t range) {
  if constexpr (FILT) {
    d -= dLo;  // wraps below dLo
    return d < range ? d : range;
  } else {
    return d;
  }
}
template <bool MIX, bool FILT = false>
struct NetFragPolT : KeyLoad {
  using InT = ulonglong2;
  using StageT = uint32_t;
  using OutT = uint32_t;
  static constexpr bool kDigArray = false;
  static constexpr bool kEarly = true;  // earlyPrefetch
  static constexpr bool kFilter = FILT;
  uint64_t mask;
  uint32_t bits;
  KeyMix mix;
  uint32_t dLo = 0, range = 0;
  __device__ __forceinline__ uint32_t digit(const LoadT &k) const {
    return rangeDigit<FILT>((uint32_t)(mixKey<MIX>(mix, k) & mask), dLo, range);
  }
  __device__ __forceinline__ StageT stage(const LoadT &k, uint32_t d) const {
    return (uint32_t)(mixKey<MIX>(mix, k) >> bits) | (d << (32 - bits));
  }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return v >> (32 - bits); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v & (0xFFFFFFFFu >> bits); }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
using NetFragPol = NetFragPolT<false>;  // ablation entry (no key mixing)
// Fragments of keys wider than 32 bits (fragWordFits: keyBits <= 32 + bits,
// e.g. 6B dense keys = 33 bits): the staged u32 word is the whole fragment
// and the digit goes to the tile's u16 digit array (no early prefetch).
template <bool MIX, bool FILT = false>
struct NetFragDigPolT : KeyLoad {
  using InT = ulonglong2;
  using StageT = uint32_t;
  using OutT = uint32_t;
  static constexpr bool kDigArray = true;
  static constexpr bool kFilter = FILT;
  uint64_t mask;
  uint32_t bits;
  KeyMix mix;
  uint32_t dLo = 0, range = 0;
  __device__ __forceinline__ uint32_t digit(const LoadT &k) const {
    return rangeDigit<FILT>((uint32_t)(mixKey<MIX>(mix, k) & mask), dLo, range);
  }
  __device__ __forceinline__ StageT stage(const LoadT &k, uint32_t) const {
    return (uint32_t)(mixKey<MIX>(mix, k) >> bits);
  }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &) const { return 0; }  // digits: LDS array
  __device__ __forceinline__ OutT out(const StageT &v) const { return v; }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = v; }
};
struct NetWidePol : PlainLoad<ulonglong2> {  // 16 B tuple -> 16 B tuple (full-range keys)
  using InT = ulonglong2;
  using StageT = ulonglong2;
  using OutT = ulonglong2;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  KeyMix mix;
  __device__ __forceinline__ uint32_t digit(const InT &x) const { return (uint32_t)(mix.apply(x.x) & mask); }
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t) const {
    return make_ulonglong2(mix.apply(x.x), x.y);
  }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return (uint32_t)(v.x & mask); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v; }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
struct LocalCompressedPol : PlainLoad<uint64_t> {  // 8 B -> 8 B, digit = (value >> shift) & mask
  using InT = uint64_t;
  using StageT = uint64_t;
  using OutT = uint64_t;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  uint32_t shift;
  __device__ __forceinline__ uint32_t digit(const InT &x) const { return (uint32_t)((x >> shift) & mask); }
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t) const { return x; }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return digit(v); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v; }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
struct LocalWidePol : PlainLoad<ulonglong2> {  // 16 B -> 16 B, digit = (key >> shift) & mask
  using InT = ulonglong2;
  using StageT = ulonglong2;
  using OutT = ulonglong2;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  uint32_t shift;
  __device__ __forceinline__ uint32_t digit(const InT &x) const { return (uint32_t)((x.x >> shift) & mask); }
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t) const { return x; }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return digit(v); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return v; }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
// u32 key fragment -> u16 of the bits above the local digit (count-only
// two-level pass, JoinPlan::fragments): 2 bytes written per tuple.
struct LocalFragPol : PlainLoad<uint32_t> {
  using InT = uint32_t;
  using StageT = uint32_t;
  using OutT = uint16_t;
  static constexpr bool kDigArray = false;
  uint64_t mask;
  uint32_t shift;
  uint32_t fragShift;
  __device__ __forceinline__ uint32_t digit(const InT &x) const { return (uint32_t)((x >> shift) & mask); }
  __device__ __forceinline__ StageT stage(const InT &x, uint32_t) const { return x; }
  __device__ __forceinline__ uint32_t stagedDigit(const StageT &v) const { return digit(v); }
  __device__ __forceinline__ OutT out(const StageT &v) const { return (uint16_t)(v >> fragShift); }
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const { o[pos] = out(v); }
};
struct LocalSplitPol : LocalCompressedPol {  // 8 B -> u32 rid / key low word + u16 fragment (kernels.h, SplitLayout)
  using OutT = uint32_t;
  uint16_t *hi;
  uint32_t fragShift;
  uint32_t loShift = 0;
  __device__ __forceinline__ void store(OutT *o, uint64_t pos, const StageT &v) const {
    o[pos] = (uint32_t)(v >> loShift);
    hi[pos] = (uint16_t)(v >> fragShift);
  }
};

// Digit arrays in LDS are padded to at least 1024 entries (the widest
// workgroup): every thread of the claim loop then owns whole, existing
// entries, and the loop needs no per-thread bound check (see scatterTile).
HJ_HD uint32_t padDigits(uint32_t F) { return F > 1024u ? F : 1024u; }

// LDS per workgroup: cursor and wbase (FP x CurT), cnt and off (FP x u32)
// with FP = padDigits(F), scan scratch, the reordered tile (TILE x StageT)
// and, only for NetCompressedDigPol, the tile's digits (TILE x u16).
template <class Pol, typename CurT, int TILE>
struct ScatterLayout {
  static __host__ __device__ constexpr size_t valOffset(uint32_t F) {
    return ((size_t)padDigits(F) * (2 * sizeof(CurT) + 8) + 64 + 15) & ~size_t(15);
  }
  static __host__ __device__ constexpr size_t bytes(uint32_t F) {
    return valOffset(F) + (size_t)TILE * sizeof(typename Pol::StageT) + (Pol::kDigArray ? (size_t)TILE * 2 : 0);
  }
};

// Per-workgroup LDS carve of the scatter (see ScatterLayout).
template <class Pol, typename CurT, int TILE>
struct ScatterSmem {
  CurT *cursor, *wbase;
  uint32_t *cnt, *off, *wave;
  typename Pol::StageT *val;
  uint16_t *dig;
  __device__ __forceinline__ ScatterSmem(unsigned char *smem, uint32_t F) {
    const uint32_t FP = padDigits(F);
    cursor = reinterpret_cast<CurT *>(smem);
    wbase = cursor + FP;
    cnt = reinterpret_cast<uint32_t *>(wbase + FP);
    off = cnt + FP;
    wave = off + FP;
    val = reinterpret_cast<typename Pol::StageT *>(smem + ScatterLayout<Pol, CurT, TILE>::valOffset(F));
    dig = reinterpret_cast<uint16_t *>(val + TILE);
  }
};

// Where the branch-free scatter sends what must not land in the output:
// stores of lanes without an element (a range's tail tile) or past a bounded
// slice, and the claim atomics of padding digits (adding 0).  Writing these
// to scratch instead of branching around them keeps the tile loop free of
// divergent control flow: after a store or atomic under an exec mask the
// compiler's wait-count pass can no longer count the wave's memory operations
// and falls back to vmcnt(0) -- every load and store of the wave in flight
// must land -- and it serialises the write-out's LDS reads element by element.
__device__ ulonglong2 g_scatterTrash[1024];

// Per-phase shader-clock breakdown of the claim scatter's tile loop, built
// only with -DHPCJOIN_SCATTER_PROF (HPCJOIN_EXTRA_HIPFLAGS at build time;
// tools/scatter_phases.py reads it through ops.scatter_profile()).  Wave 0
// of every workgroup stamps s_memtime at the phase boundaries; the sums of
// the per-phase deltas (scalar registers) are added to g_scatterProf once per
// range, by lane 0, with vector atomics.
//   0 rank (includes waiting for the tile's loads)  1 barrier A
//   2 claims + prefetch issue  3 scan  4 staging  5 write bases (claims land)
//   6 barrier B  7 write-out issue
__device__ unsigned long long g_scatterProf[10];
struct ScatterProf {
#ifdef HPCJOIN_SCATTER_PROF
  uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t last = 0, tiles = 0;
  __device__ __forceinline__ void start() { last = __builtin_readcyclecounter(); }
  __device__ __forceinline__ void mark(int i) {
    const uint64_t now = __builtin_readcyclecounter();
    acc[i] += now - last;
    last = now;
  }
  __device__ __forceinline__ void flush() {
    if (threadIdx.x != 0) return;
    for (int i = 0; i < 8; ++i) atomicAdd(&g_scatterProf[i], (unsigned long long)acc[i]);
    atomicAdd(&g_scatterProf[8], (unsigned long long)tiles);
    atomicAdd(&g_scatterProf[9], 1ull);
  }
#else
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush() {}
#endif
};

template <class P, class = void>
struct TwoArrayStore : std::false_type {};
template <class P>
struct TwoArrayStore<P, std::void_t<decltype(&P::hi)>> : std::true_type {};

// Stores x at out[pos] when ok, else into the trash line of thread t.
template <class Pol>
__device__ __forceinline__ void storeSel(const Pol &pol, typename Pol::OutT *out, uint64_t pos,
                                         const typename Pol::StageT &x, bool ok, uint32_t t) {
  using OutT = typename Pol::OutT;
  OutT *trash = reinterpret_cast<OutT *>(g_scatterTrash);
  if constexpr (TwoArrayStore<Pol>::value) {
    uint16_t *hi = ok ? pol.hi + pos : reinterpret_cast<uint16_t *>(g_scatterTrash + 512) + t;
    OutT *lo = ok ? out + pos : trash + t;
    *lo = (OutT)(x >> pol.loShift);
    *hi = (uint16_t)(x >> pol.fragShift);
  } else {
    OutT *p = ok ? out + pos : trash + t;
    *p = pol.out(x);
  }
}

template <class Pol, int NTH, int IPT, bool FULL>
__device__ __forceinline__ void loadTile(const typename Pol::InT *__restrict__ src, uint32_t count,
                                         typename Pol::LoadT (&v)[IPT]) {
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const uint32_t idx = i * NTH + threadIdx.x;
    if (FULL || idx < count) v[i] = Pol::load(src + idx);
  }
}

// Next tile into registers, branch-free: indices past the range end read its
// last element (loaded, never ranked), so every tile issues exactly IPT loads.
// im: slot map of the input (RoundMap; identity unless the local pass reads a
// round-interleaved network window).
template <class Pol, int NTH, int IPT>
__device__ __forceinline__ void prefetchTile(const typename Pol::InT *__restrict__ in, uint64_t nbase, uint64_t last,
                                             typename Pol::LoadT (&v)[IPT], const RoundMap &im = RoundMap()) {
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const uint64_t idx = nbase + (uint64_t)(i * NTH + threadIdx.x);
    v[i] = Pol::load(in + im(idx < last ? idx : last));
  }
}

// Early prefetch: when the staged word is no wider than the loaded one and
// carries its digit (no separate digit array), the rank phase turns every
// loaded element into its staged word right away, so the registers of the
// loaded tile are free again before the scan -- the next tile's loads are
// issued after the claims (so the claim atomics, issued first, can be waited
// for without waiting for the loads) and overlap the scan, the staging and
// the write-out instead of only the write-out.  Only where the tile's loads
// take at most 16 VGPRs per thread: with wider tiles the staged words, ranks
// and next tile no longer fit 128 VGPRs (1024-thread groups) and spill.  And
// only for policies that opt in (kEarly): measured on MI355X, same box, the
// count-only fragment scatter gains (1.90 -> 1.80 ms per call, 1B x 1B join
// 10.16 -> 9.62 ms) while the key-only scatter is unchanged (2.28 / 2.31) and
// the local split scatter loses (1.45 -> 1.54).
template <class P, class = void>
struct FilterOf : std::false_type {};
template <class P>
struct FilterOf<P, std::void_t<decltype(P::kFilter)>> : std::integral_constant<bool, P::kFilter> {};

template <class P, class = void>
struct EarlyOptIn : std::false_type {};
template <class P>
struct EarlyOptIn<P, std::void_t<decltype(P::kEarly)>> : std::integral_constant<bool, P::kEarly> {};
template <class Pol, int IPT>
constexpr bool earlyPrefetch() {
  return EarlyOptIn<Pol>::value && !Pol::kDigArray && sizeof(typename Pol::StageT) <= sizeof(typename Pol::LoadT) &&
         IPT * sizeof(typename Pol::LoadT) <= 64;
}

// One tile.  The next tile's loads ([nbase, nbase + TILE), clamped to nlast)
// are issued into v while this one is staged or written out: the caller's
// next tile of the same range, or the first tile of its next range.
// FULL tiles (every tile but a range's tail) have no divergent
// control flow at all, so hipcc keeps the IPT LDS atomics, loads and stores
// in flight with counted waits; the tail tile predicates its LDS work only.
// BOUNDED (claim mode with estimated slices): l.cursor[d] holds the end of the
// group's slice of digit d; claimed positions past it are not written (the
// caller detects the overflow from the final claim cursors and re-runs).
// MAXD = padDigits(F) / NTH claim entries per thread.
template <class Pol, typename CurT, int NTH, int IPT, int MODE, bool FULL, bool CLAIM, bool BOUNDED, int MAXD>
__device__ __forceinline__ void scatterTile(const typename Pol::InT *__restrict__ in, uint64_t base, uint64_t end,
                                            uint32_t count, uint32_t F, const ScatterSmem<Pol, CurT, NTH * IPT> &l,
                                            const Pol &pol, typename Pol::OutT *__restrict__ out,
                                            typename Pol::LoadT (&v)[IPT], CurT *__restrict__ gcur,
                                            ScatterProf &pf, uint64_t nbase, uint64_t nlast,
                                            const RoundMap &im = RoundMap(), const RoundMap &om = RoundMap()) {
  constexpr uint32_t TILE = NTH * IPT;
  pf.start();
  constexpr bool EARLY = earlyPrefetch<Pol, IPT>();
  const uint32_t t = threadIdx.x;
  // EARLY: sw = staged words, dr = ranks (then positions); else dr = digit << 16 | rank.
  uint32_t dr[IPT];
  typename Pol::StageT sw[EARLY ? IPT : 1];
  // FILT: tuples outside the pass's digit range (sentinel digit F) are neither
  // ranked nor staged -- a pass over a quarter of the digits does a quarter of
  // the LDS work; the scan's entry F then stays 0 and off[F] = kept.
  constexpr bool FILT = FilterOf<Pol>::value;
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const uint32_t idx = i * NTH + t;
    if (FULL || idx < count) {
      const uint32_t d = pol.digit(v[i]);
      const bool keep = !FILT || d < F;
      if constexpr (EARLY) {
        if (keep) dr[i] = atomicAdd(&l.cnt[d], 1u);
        sw[i] = pol.stage(v[i], d);
      } else {
        dr[i] = (d << 16) | (keep ? atomicAdd(&l.cnt[d], 1u) : 0u);
      }
    }
  }
  pf.mark(0);
  // Barriers of the tile loop order LDS only (ldsBarrier): the waves share
  // nothing through global memory here, and a full __syncthreads() would make
  // every wave wait for its prefetch of the next tile (vmcnt(0)) before the
  // write-out, so loads and stores of a workgroup would never overlap.
  ldsBarrier();  // A: counts final; previous tile's write-out done
  pf.mark(1);
  CurT claim[MAXD];
  if constexpr (CLAIM) {
    // One device atomic per digit claims this tile's run in the group's slice,
    // issued before the scan so its round trip overlaps the scan.  Waves whose
    // digits are all padding (d >= F: F < NTH) skip it on a scalar branch (no
    // exec mask); a wave straddling F (only F < 64) sends its padding lanes'
    // zero adds to the trash.
    CurT *trash = reinterpret_cast<CurT *>(g_scatterTrash);
    const uint32_t wave0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t & ~(uint32_t)(WAVE - 1)));
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
      const uint32_t d = t + k * NTH;
      if (wave0 + k * NTH < F) claim[k] = atomicAdd(d < F ? gcur + d : trash + t, (CurT)l.cnt[d]);
    }
  }
  if constexpr (EARLY) prefetchTile<Pol, NTH, IPT>(in, nbase, nlast, v, im);
  pf.mark(2);
  // FILT: entry F (never counted) is scanned too: off[F] = kept tuples, and
  // the write-out stops there.
  blockExclusiveScanLds<NTH, uint32_t, uint32_t, true>(l.cnt, l.off, (int)F + (FILT ? 1 : 0), l.wave);
  uint32_t kept = count;
  if constexpr (FILT) kept = (uint32_t)__builtin_amdgcn_readfirstlane((int)l.off[F]);
  pf.mark(3);
  if constexpr (!CLAIM) {
    for (uint32_t d = t; d < F; d += NTH) {
      const CurT c = l.cursor[d];
      l.wbase[d] = c - (CurT)l.off[d];  // wraps; wbase + idx lands back in range
      l.cursor[d] = c + (CurT)l.cnt[d];
      l.cnt[d] = 0;
    }
  }
  // Staging: every position first, then every write (one batch of LDS reads
  // and one of writes; interleaved, each write waited for its own read).
  if constexpr (EARLY) {
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t idx = i * NTH + t;
      if ((FULL || idx < count) && (!FILT || pol.stagedDigit(sw[i]) < F)) dr[i] += l.off[pol.stagedDigit(sw[i])];
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t idx = i * NTH + t;
      if ((FULL || idx < count) && (!FILT || pol.stagedDigit(sw[i]) < F)) l.val[dr[i]] = sw[i];
    }
  } else {
    uint32_t pos[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t idx = i * NTH + t;
      if (FULL || idx < count) pos[i] = l.off[dr[i] >> 16] + (dr[i] & 0xFFFFu);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t idx = i * NTH + t;
      if ((FULL || idx < count) && (!FILT || (dr[i] >> 16) < F)) {
        const uint32_t d = dr[i] >> 16;
        l.val[pos[i]] = pol.stage(v[i], d);
        if constexpr (Pol::kDigArray) l.dig[pos[i]] = (uint16_t)d;
      }
    }
    // Prefetch the next tile while this one is streamed out.
    prefetchTile<Pol, NTH, IPT>(in, nbase, nlast, v, im);
  }
  pf.mark(4);
  if constexpr (CLAIM) {
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {  // padding entries get garbage bases nobody reads
      const uint32_t d = t + k * NTH;
      l.wbase[d] = claim[k] - (CurT)l.off[d];
      l.cnt[d] = 0;
    }
  }
  pf.mark(5);
  ldsBarrier();  // B: staged tile and write bases visible
  pf.mark(6);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const uint32_t idx = i * NTH + t;
    if constexpr (FILT) {  // whole waves past the kept tuples skip on a scalar branch
      if ((uint32_t)i * NTH + (t & ~(uint32_t)(WAVE - 1)) >= kept) continue;
    }
    const bool have = FILT ? idx < kept : (FULL || idx < count);
    const uint32_t at = have ? idx : 0;  // the tail tile's element 0 exists
    const typename Pol::StageT x = l.val[at];
    uint32_t d;
    if constexpr (Pol::kDigArray)
      d = l.dig[at];
    else
      d = pol.stagedDigit(x);
    if constexpr (MODE == 0) {
      const CurT pos = (CurT)(l.wbase[d] + (CurT)idx);
      bool ok = have;
      if constexpr (BOUNDED) ok = ok && pos < l.cursor[d];
      storeSel(pol, out, om((uint64_t)pos), x, ok, t);
    } else if constexpr (MODE == 1) {
      if (have) out[base + idx] = pol.out(x);
      asm volatile("" ::"v"(l.wbase[d]));
    } else {
      const auto y = pol.out(x);
      asm volatile("" ::"v"(y), "v"(l.wbase[d]));
    }
  }
  pf.mark(7);
#ifdef HPCJOIN_SCATTER_PROF
  ++pf.tiles;
#endif
}

// Scatter [begin, end) of `in` into `out` at the cursors held in LDS
// (initialised by the caller, advanced here).  Per tile:
//   rank (LDS atomics) | A | claim + scan + per-digit write base | stage into
//   LDS, prefetch next tile into registers | B | stream the reordered tile out.
// MODE (ablation only): 0 = real scatter, 1 = coalesced write-out, 2 = none.
template <class Pol, typename CurT, int NTH, int IPT, int MODE, bool CLAIM = false, bool BOUNDED = false,
          int MAXD = 1>
__device__ __forceinline__ void scatterRange(const typename Pol::InT *__restrict__ in, uint64_t begin, uint64_t end,
                                             uint32_t F, unsigned char *smem, const Pol &pol,
                                             typename Pol::OutT *__restrict__ out, CurT *gcur = nullptr,
                                             const RoundMap &im = RoundMap(), const RoundMap &om = RoundMap()) {
  constexpr uint32_t TILE = NTH * IPT;
  const ScatterSmem<Pol, CurT, TILE> l(smem, F);
  typename Pol::LoadT v[IPT];
  ScatterProf pf;
  if (begin < end) prefetchTile<Pol, NTH, IPT>(in, begin, end - 1, v, im);
  for (uint64_t base = begin; base < end; base += TILE) {
    if (base + TILE <= end)
      scatterTile<Pol, CurT, NTH, IPT, MODE, true, CLAIM, BOUNDED, MAXD>(in, base, end, TILE, F, l, pol, out, v,
                                                                         gcur, pf, base + TILE, end - 1, im, om);
    else
      scatterTile<Pol, CurT, NTH, IPT, MODE, false, CLAIM, BOUNDED, MAXD>(in, base, end, (uint32_t)(end - base), F, l,
                                                                          pol, out, v, gcur, pf, base + TILE, end - 1,
                                                                          im, om);
  }
  pf.flush();
  __syncthreads();
}

// Occupancy target per geometry: 256-thread groups aim at 3 per CU (LDS-bound),
// 512 at 2, 1024 at 1 (second launch-bounds argument = waves per SIMD).
template <int NTH>
struct ScatterOcc {
  static constexpr int value = NTH == 256 ? 3 : (NTH == 512 ? 4 : 4);
};

// Per-workgroup cursors (ablation baseline): F <= NTH * MAXD digits, no claims.
template <class Pol, typename CurT, int NTH, int IPT, int MODE>
__global__ __launch_bounds__(NTH, ScatterOcc<NTH>::value) void netScatterKernel(
    const typename Pol::InT *__restrict__ in, uint64_t n, uint32_t tpb, uint32_t F, Pol pol, uint32_t totalBlocks,
    uint32_t blockBegin, const uint64_t *__restrict__ cursors, typename Pol::OutT *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t blk = blockBegin + blockIdx.x;
  const uint32_t FP = padDigits(F);
  CurT *cursor = reinterpret_cast<CurT *>(smem);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(cursor + 2 * FP);
  for (uint32_t d = threadIdx.x; d < FP; d += NTH) {
    if (d < F) cursor[d] = (CurT)cursors[(uint64_t)d * totalBlocks + blk];
    cnt[d] = 0;
  }
  __syncthreads();
  const uint64_t begin = (uint64_t)blk * tpb * PART_TILE;  // geometry is in PART_TILE units
  const uint64_t end = min(n, begin + (uint64_t)tpb * PART_TILE);
  scatterRange<Pol, CurT, NTH, IPT, MODE>(in, begin, end, F, smem, pol, out);
}

// Claim-mode network scatter: cursors come from the group slices (gcur is
// [NGROUPS][F] for this chunk), so no per-workgroup cursor array is loaded.
// MAXD = padDigits(F) / NTH (scatterLaunchMaxd).
template <class Pol, typename CurT, int NTH, int IPT, int MODE, bool BOUNDED, int MAXD>
__global__ __launch_bounds__(NTH, ScatterOcc<NTH>::value) void netScatterClaimKernel(
    const typename Pol::InT *__restrict__ in, uint64_t n, uint32_t tpb, uint32_t F, Pol pol, uint32_t blockBegin,
    CurT *__restrict__ gcur, typename Pol::OutT *out, const CurT *__restrict__ gend = nullptr,
    const uint32_t *__restrict__ roundMeta = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t blk = blockBegin + blockIdx.x;
  RoundMap om;  // output slot map, decided by the layout kernel (RoundMap)
  if (roundMeta) {
    om.lp = roundMeta[0];
    om.lv = roundMeta[1];
    om.lns = roundMeta[2];
  }
  const uint32_t FP = padDigits(F);
  CurT *sliceEnd = reinterpret_cast<CurT *>(smem);  // the per-workgroup cursor array is unused in claim mode
  uint32_t *cnt = reinterpret_cast<uint32_t *>(reinterpret_cast<CurT *>(smem) + 2 * FP);
  const size_t grp = (size_t)(blockIdx.x % NGROUPS) * F;
  for (uint32_t d = threadIdx.x; d < FP; d += NTH) {
    cnt[d] = 0;
    if constexpr (BOUNDED)
      if (d < F) sliceEnd[d] = gend[grp + d];
  }
  __syncthreads();
  const uint64_t begin = (uint64_t)blk * tpb * PART_TILE;
  const uint64_t end = min(n, begin + (uint64_t)tpb * PART_TILE);
  scatterRange<Pol, CurT, NTH, IPT, MODE, true, BOUNDED, MAXD>(in, begin, end, F, smem, pol, out, gcur + grp,
                                                               RoundMap(), om);
}

// Calls fn(std::integral_constant<int, MAXD>) with MAXD = padDigits(F) / NTH:
// one of two values per workgroup width (F <= 1024 or F = 2048).
template <int NTH, class Fn>
static void withMaxd(uint32_t F, Fn &&fn) {
  constexpr int LO = 1024 / NTH, HI = (1 << MAX_PART_BITS) / NTH;
  static_assert(HI == 2 * LO, "withMaxd: two digit-array sizes");
  if (padDigits(F) / NTH == (uint32_t)LO)
    fn(std::integral_constant<int, LO>());
  else
    fn(std::integral_constant<int, HI>());
}

// Default geometry (measured on MI355X, tools/microbench.py ablation).
constexpr int SC_NTH = 256;
constexpr int SC_IPT = 16;

template <class Pol, typename CurT, int NTH = SC_NTH, int IPT = SC_IPT, int MODE = 0>
static void launchNet(const Pol &pol, const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                      uint32_t blockBegin, uint32_t blockEnd, const uint64_t *cursors, void *out, hipStream_t s) {
  const uint32_t F = 1u << bits;
  const size_t lds = ScatterLayout<Pol, CurT, NTH * IPT>::bytes(F);
  HJ_CHECK(lds <= 160 * 1024, "scatter LDS %zu too large", lds);
  hipLaunchKernelGGL((netScatterKernel<Pol, CurT, NTH, IPT, MODE>), dim3(blockEnd - blockBegin), dim3(NTH), lds, s,
                     reinterpret_cast<const typename Pol::InT *>(in), n, g.tilesPerBlock, F, pol, g.blocks,
                     blockBegin, cursors, reinterpret_cast<typename Pol::OutT *>(out));
  HIP_CHECK_LAUNCH();
}

// True when key >> bits, shifted to keyShift, leaves `bits` spare top bits.
static bool digitFitsOnTop(uint32_t bits, uint32_t keyShift, uint32_t keyBits) {
  const uint32_t high = keyBits > bits ? keyBits - bits : 0;
  return keyShift + high + bits <= 64;
}

// Production geometry of the claim-mode scatter (tools/microbench.py
// ablation on MI355X: 1024 threads x 8 tuples per LDS tile = 8192-tuple
// tiles, one workgroup per CU).
constexpr int CL_NTH = 1024;  // production width (the local pass and the default network pass)
constexpr int CL_IPT_DEFAULT = 8;
constexpr int CL_IPT = CL_IPT_DEFAULT;

template <class Pol, int CL_IPT, int CL_NTH = 1024>
static void launchNetClaimIpt(const Pol &pol, const data::Tuple *in, uint64_t n, uint32_t bits,
                              const PartitionGeometry &g, uint32_t blockBegin, uint32_t blockEnd, void *gcur,
                              void *out, hipStream_t s, const void *gend, bool narrow, uint32_t digits = 0,
                              const uint32_t *roundMeta = nullptr) {
  // digits: claim slices per group (filtered range passes); else 2^bits.
  const uint32_t F = digits ? digits : 1u << bits;
  const auto *src = reinterpret_cast<const typename Pol::InT *>(in);
  auto *dst = reinterpret_cast<typename Pol::OutT *>(out);
  const dim3 grid(blockEnd - blockBegin);
  auto go = [&](auto cur, auto maxd) {
    using C = decltype(cur);
    constexpr int M = decltype(maxd)::value;
    const size_t lds = ScatterLayout<Pol, C, CL_NTH * CL_IPT>::bytes(F);
    HJ_CHECK(lds <= 160 * 1024, "scatter LDS %zu too large", lds);
    auto *gc = reinterpret_cast<C *>(gcur);
    if (gend)
      hipLaunchKernelGGL((netScatterClaimKernel<Pol, C, CL_NTH, CL_IPT, 0, true, M>), grid, dim3(CL_NTH), lds, s, src,
                         n, g.tilesPerBlock, F, pol, blockBegin, gc, dst, reinterpret_cast<const C *>(gend),
                         roundMeta);
    else
      hipLaunchKernelGGL((netScatterClaimKernel<Pol, C, CL_NTH, CL_IPT, 0, false, M>), grid, dim3(CL_NTH), lds, s,
                         src, n, g.tilesPerBlock, F, pol, blockBegin, gc, dst, nullptr, roundMeta);
  };
  withMaxd<CL_NTH>(F, [&](auto maxd) {
    if (narrow)
      go(uint32_t(), maxd);
    else
      go((unsigned long long)0, maxd);
  });
  HIP_CHECK_LAUNCH();
}

// Tile of the claim scatter (PartitionGeometry::ipt = KernelVariants::netIpt):
// 8192 tuples by default, with the early prefetch (earlyPrefetch: the next
// tile's loads overlap the scan and staging).  ipt 16 = 16384-tuple tiles of
// 4-byte staged words (longer runs per partition and tile, but too many
// registers for the early prefetch: 1B x 1B 10.08 ms vs 9.56 with 8192 +
// early prefetch, same box, profiles/r5/README.md); ipt 15 = 15360 at
// 2048-way.
template <class Pol>
static void launchNetClaim(const Pol &pol, const data::Tuple *in, uint64_t n, uint32_t bits,
                           const PartitionGeometry &g, uint32_t blockBegin, uint32_t blockEnd, void *gcur,
                           void *out, hipStream_t s, const void *gend, bool narrow,
                           const uint32_t *roundMeta = nullptr) {
  // PartitionGeometry::nth = 512 (KernelVariants::netThreads): half-width
  // workgroups with the same per-thread tile, so two or three share a CU and
  // one's rank/scan/claim phases overlap another's loads and stores.
  if (g.nth == 512) {
    if constexpr (sizeof(typename Pol::StageT) == 4) {
      if (g.ipt == 16) {
        launchNetClaimIpt<Pol, 16, 512>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, 0, roundMeta);
        return;
      }
    }
    launchNetClaimIpt<Pol, CL_IPT_DEFAULT, 512>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend,
                                                narrow, 0, roundMeta);
    return;
  }
  if constexpr (sizeof(typename Pol::StageT) == 4) {
    if (g.ipt == 16) {
      launchNetClaimIpt<Pol, 16>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, 0, roundMeta);
      return;
    }
  }
  if (g.ipt == 15 && narrow && bits == MAX_PART_BITS)
    launchNetClaimIpt<Pol, 15>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, 0, roundMeta);
  else if (g.ipt == 12)  // 12288-tuple tiles (sweep: longer runs per digit and tile)
    launchNetClaimIpt<Pol, 12>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, 0, roundMeta);
  else
    launchNetClaimIpt<Pol, CL_IPT_DEFAULT>(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, 0, roundMeta);
}

void scatterProfile(unsigned long long out[10], bool reset) {
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_scatterProf), 10 * sizeof(unsigned long long)));
  if (reset) {
    const unsigned long long z[10] = {};
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_scatterProf), z, sizeof(z)));
  }
}

bool scatterProfileBuilt() {
#ifdef HPCJOIN_SCATTER_PROF
  return true;
#else
  return false;
#endif
}

void netScatter(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift, const PartitionGeometry &g,
                uint32_t blockBegin, uint32_t blockEnd, void *gcur, uint64_t *out, hipStream_t s, uint32_t keyBits,
                KeyMix mix, const void *gend, int narrowMode, bool withRids, const uint32_t *roundMeta) {
  const bool narrow = narrowMode < 0 ? cursorsNarrow(n) : narrowMode != 0;
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatter: bits=%u out of range", bits);
  HJ_CHECK(blockBegin <= blockEnd && blockEnd <= g.blocks, "netScatter: block range [%u,%u) of %u", blockBegin,
           blockEnd, g.blocks);
  if (n == 0 || blockEnd == blockBegin) return;
  HJ_CHECK(withRids || keyShift == 0, "netScatter: key-only words need keyShift 0 (got %u)", keyShift);
  if (!withRids) {  // key >> bits always leaves `bits` spare top bits
    auto go = [&](auto kpol) {
      kpol.mask = (1ull << bits) - 1;
      kpol.bits = bits;
      kpol.mix = mix;
      launchNetClaim(kpol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, roundMeta);
    };
    if (mix.on)
      go(NetKeyPol<true>());
    else
      go(NetKeyPol<false>());
    return;
  }
  NetCompressedPol pol;
  pol.mask = (1ull << bits) - 1;
  pol.bits = bits;
  pol.keyShift = keyShift;
  pol.mix = mix;
  if (digitFitsOnTop(bits, keyShift, mix.on ? std::max(keyBits, mix.bits) : keyBits)) {
    launchNetClaim(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, roundMeta);
  } else {
    NetCompressedDigPol dpol;
    static_cast<NetCompressedPol &>(dpol) = pol;
    launchNetClaim(dpol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, roundMeta);
  }
}

void netScatterWide(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                    uint32_t blockBegin, uint32_t blockEnd, void *gcur, data::Tuple *out, hipStream_t s,
                    KeyMix mix, const void *gend, int narrowMode) {
  const bool narrow = narrowMode < 0 ? cursorsNarrow(n) : narrowMode != 0;
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatterWide: bits=%u out of range", bits);
  HJ_CHECK(blockBegin <= blockEnd && blockEnd <= g.blocks, "netScatterWide: block range [%u,%u) of %u",
           blockBegin, blockEnd, g.blocks);
  if (n == 0 || blockEnd == blockBegin) return;
  NetWidePol pol;
  pol.mask = (1ull << bits) - 1;
  pol.mix = mix;
  launchNetClaim(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow);
}

void netScatterFrag(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g, uint32_t blockBegin,
                    uint32_t blockEnd, void *gcur, uint32_t *out, hipStream_t s, uint32_t keyBits, KeyMix mix,
                    const void *gend, int narrowMode, const uint32_t *roundMeta) {
  const bool narrow = narrowMode < 0 ? cursorsNarrow(n) : narrowMode != 0;
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatterFrag: bits=%u out of range", bits);
  const uint32_t kb = mix.on ? std::max(keyBits, mix.bits) : keyBits;
  HJ_CHECK(fragWordFits(kb, bits), "netScatterFrag: %u-bit keys leave a fragment wider than %u bits above %u radix bits",
           kb, 32 - bits, bits);
  HJ_CHECK(blockBegin <= blockEnd && blockEnd <= g.blocks, "netScatterFrag: block range [%u,%u) of %u", blockBegin,
           blockEnd, g.blocks);
  if (n == 0 || blockEnd == blockBegin) return;
  auto go = [&](auto pol) {
    pol.mask = (1ull << bits) - 1;
    pol.bits = bits;
    pol.mix = mix;
    launchNetClaim(pol, in, n, bits, g, blockBegin, blockEnd, gcur, out, s, gend, narrow, roundMeta);
  };
  const bool digitOnTop = kb <= 32;  // fragment + digit fit the staged u32
  if (mix.on && digitOnTop)
    go(NetFragPolT<true>());
  else if (digitOnTop)
    go(NetFragPolT<false>());
  else if (mix.on)
    go(NetFragDigPolT<true>());
  else
    go(NetFragDigPolT<false>());
}

void netScatterFragRange(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g, void *gcur,
                         uint32_t *out, hipStream_t s, uint32_t keyBits, KeyMix mix, const void *gend, bool narrow,
                         uint32_t dLo, uint32_t range) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatterFragRange: bits=%u out of range", bits);
  const uint32_t kb = mix.on ? std::max(keyBits, mix.bits) : keyBits;
  HJ_CHECK(fragWordFits(kb, bits), "netScatterFragRange: %u-bit keys above %u radix bits", kb, bits);
  // The sentinel digit `range` needs an LDS counter of its own: range < padDigits(range).
  HJ_CHECK(range >= 1 && range < padDigits(range) && dLo + range <= (1u << bits) && gend,
           "netScatterFragRange: digits [%u, %u) of %u (at most %u per pass, bounded slices)", dLo, dLo + range,
           1u << bits, padDigits(1) - 1);
  if (n == 0) return;
  auto go = [&](auto pol) {
    pol.mask = (1ull << bits) - 1;
    pol.bits = bits;
    pol.mix = mix;
    pol.dLo = dLo;
    pol.range = range;
    launchNetClaimIpt<decltype(pol), CL_IPT_DEFAULT>(pol, in, n, bits, g, 0, g.blocks, gcur, out, s, gend, narrow,
                                                     range);
  };
  const bool digitOnTop = kb <= 32;
  if (mix.on && digitOnTop)
    go(NetFragPolT<true, true>());
  else if (digitOnTop)
    go(NetFragPolT<false, true>());
  else if (mix.on)
    go(NetFragDigPolT<true, true>());
  else
    go(NetFragDigPolT<false, true>());
}

// ------------------------------------------------ device-side sampled layout
// Turns the sampled per-(XCD group, digit) counts into bounded claim slices
// on the device, so a sampled network pass needs no host round trip between
// its histogram and its scatter (the whole count-only join is then one
// stream of kernels with a single synchronisation at the end).  Entry
// j = d * G + g (partition-major, groups inside) is stored at i = g * F + d,
// the claim-cursor layout.  cap = roundup16(min(est + margin, total_g)),
// est = sampled * total_g / seen_g, margin = sigmas * sqrt(max(est, 1) *
// total_g / seen_g) + frac * est + floor (sigmas = frac = floor = 0 with an
// exact histogram: the slices are then exactly the counts, rounded to lines).
constexpr int LAY_NT = 1024;
template <typename CurT>
struct LayoutSideArgs {
  const unsigned long long *sampled;
  SampleScale sc;
  CurT *gstart, *gcur, *gend;
  unsigned long long *capacityUsed;
  unsigned long long *clear;  // = sampled when it is DeviceControl scratch, else nullptr
  uint32_t *roundMeta;        // LayoutInput::roundMeta
  uint32_t roundLp, roundMaxLv;
  unsigned long long roundCapacity;
};

// Workgroup i lays out side i (one or two sides per launch).
// Digits [dLo, dLo + F) of totals laid out as [G][Fsrc] (a partition-group
// pass lays out its range only; F = Fsrc, dLo = 0 otherwise).
template <typename CurT>
__global__ __launch_bounds__(LAY_NT) void netSampledLayoutKernel(LayoutSideArgs<CurT> s0, LayoutSideArgs<CurT> s1,
                                                                  uint32_t F, uint32_t Fsrc, uint32_t dLo) {
  const LayoutSideArgs<CurT> &ls = blockIdx.x ? s1 : s0;
  const unsigned long long *__restrict__ sampled = ls.sampled;
  const SampleScale &sc = ls.sc;
  CurT *__restrict__ gstart = ls.gstart;
  CurT *__restrict__ gcur = ls.gcur;
  CurT *__restrict__ gend = ls.gend;
  unsigned long long *__restrict__ capacityUsed = ls.capacityUsed;
  __shared__ unsigned long long wt[LAY_NT / WAVE];
  __shared__ unsigned long long maxCapS;
  constexpr uint32_t G = NGROUPS;
  const uint32_t n = F * G;
  const uint32_t per = (n + LAY_NT - 1) / LAY_NT, t = threadIdx.x;
  const uint32_t j0 = t * per;
  constexpr int MAXPER = ((1u << MAX_PART_BITS) * NGROUPS + LAY_NT - 1) / LAY_NT;
  unsigned long long cap[MAXPER];
  unsigned long long local = 0;
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    cap[k] = 0;
    const uint32_t j = j0 + k;
    if (k < (int)per && j < n) {
      const uint32_t d = j / G, g = j % G;
      const double seen = sc.seen[g], total = sc.total[g];
      double c = 0;
      if (seen > 0) {
        const double scale = total / seen;
        const double est = (double)sampled[(size_t)g * Fsrc + dLo + d] * scale;
        // sigma of a count scaled by `scale` from k samples: scale * sqrt(k);
        // at least one sample's worth (k = 0 says little about a cell).
        const double margin = sc.sigmas * sqrt(fmax(est, scale) * scale) + sc.frac * est + sc.floor;
        c = fmin(ceil(est + margin), total);
      }
      if (ls.clear) ls.clear[(size_t)g * Fsrc + dLo + d] = 0;  // read once (above), by this thread
      cap[k] = ((unsigned long long)c + 15ull) & ~15ull;
      local += cap[k];
    }
  }
  // Round-interleaved slices (RoundMap) when the largest slice allows them.
  uint32_t lv = 0, lns = 0;
  unsigned long long roundUsed = 0;
  if (ls.roundMeta) {  // uniform per workgroup
    if (t == 0) maxCapS = 0;
    __syncthreads();
    unsigned long long m = 0;
#pragma unroll
    for (int k = 0; k < MAXPER; ++k) m = cap[k] > m ? cap[k] : m;
    atomicMax(&maxCapS, m);
    __syncthreads();
    const unsigned long long maxCap = maxCapS;
    while ((1u << lns) < n) ++lns;
    uint32_t v = ls.roundLp;
    while ((1ull << v) < maxCap) ++v;
    roundUsed = roundSlots(maxCap, ls.roundLp, lns);
    if ((1u << lns) == n && v <= ls.roundMaxLv && roundUsed <= ls.roundCapacity) lv = v;
    if (t == 0) {
      ls.roundMeta[0] = lv ? ls.roundLp : 0;
      ls.roundMeta[1] = lv;
      ls.roundMeta[2] = lv ? lns : 0;
      ls.roundMeta[3] = 0;
    }
  }
  const unsigned long long incl = waveInclusiveScan<unsigned long long>(local);
  const int lane = t & (WAVE - 1), wid = t / WAVE;
  if (lane == WAVE - 1) wt[wid] = incl;
  __syncthreads();
  unsigned long long run = incl - local;
  for (int w = 0; w < wid; ++w) run += wt[w];
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    const uint32_t j = j0 + k;
    if (k < (int)per && j < n) {
      const uint32_t i = (j % G) * F + j / G;
      const unsigned long long b = lv ? (unsigned long long)i << lv : run;
      gstart[i] = (CurT)b;
      gcur[i] = (CurT)b;
      gend[i] = (CurT)(b + cap[k]);
      run += cap[k];
    }
  }
  if (t == LAY_NT - 1) *capacityUsed = lv ? roundUsed : run;
}

template <typename CurT>
static LayoutSideArgs<CurT> layoutSide(const LayoutInput &x) {
  auto *sampled = reinterpret_cast<const unsigned long long *>(x.sampled);
  return LayoutSideArgs<CurT>{sampled, x.sc,
                              static_cast<CurT *>(x.gstart), static_cast<CurT *>(x.gcur), static_cast<CurT *>(x.gend),
                              x.capacityUsed,
                              x.clearSampled ? const_cast<unsigned long long *>(sampled) : nullptr,
                              x.roundMeta, x.roundLp, x.roundMaxLv, (unsigned long long)x.roundCapacity};
}

void netSampledLayout(const LayoutInput *sides, uint32_t count, uint32_t F, bool narrow, hipStream_t s, uint32_t dLo,
                      uint32_t range) {
  HJ_CHECK(F >= 1 && F <= (1u << MAX_PART_BITS), "netSampledLayout: F=%u", F);
  HJ_CHECK(count == 1 || count == 2, "netSampledLayout: %u sides", count);
  const uint32_t R = range ? range : F;
  HJ_CHECK(dLo + R <= F, "netSampledLayout: digits [%u, %u) of %u", dLo, dLo + R, F);
  for (uint32_t k = 0; k < count; ++k)
    HJ_CHECK(!sides[k].roundMeta || (range == 0 && sides[k].roundLp >= 1 && sides[k].roundLp <= 16),
             "netSampledLayout: round slices need a whole-range layout and 1 <= lp <= 16 (lp %u, range %u)",
             sides[k].roundLp, range);
  const LayoutInput &b = sides[count - 1];
  if (narrow)
    hipLaunchKernelGGL(netSampledLayoutKernel<uint32_t>, dim3(count), dim3(LAY_NT), 0, s,
                       layoutSide<uint32_t>(sides[0]), layoutSide<uint32_t>(b), R, F, dLo);
  else
    hipLaunchKernelGGL(netSampledLayoutKernel<unsigned long long>, dim3(count), dim3(LAY_NT), 0, s,
                       layoutSide<unsigned long long>(sides[0]), layoutSide<unsigned long long>(b), R, F, dLo);
  HIP_CHECK_LAUNCH();
}

void netSampledLayout(const uint64_t *sampled, uint32_t F, const SampleScale &sc, void *gstart, void *gcur, void *gend,
                      bool narrow, unsigned long long *capacityUsed, hipStream_t s) {
  const LayoutInput one{sampled, sc, gstart, gcur, gend, capacityUsed};
  netSampledLayout(&one, 1, F, narrow, s);
}

SampleScale sampleScale(const PartitionGeometry &g, uint64_t n, uint32_t sampleStride, bool exact) {
  SampleScale sc{};
  const uint64_t span = (uint64_t)g.tilesPerBlock * PART_TILE;
  for (uint32_t b = 0; b < g.blocks; ++b) {
    const uint64_t begin = (uint64_t)b * span, end = std::min(n, begin + span);
    if (begin < end) sc.total[b % NGROUPS] += (double)(end - begin);
  }
  // The tiles netSampledTotals reads (every tile when sampleStride == 1).
  for (uint32_t gr = 0; gr < NGROUPS; ++gr) {
    const uint64_t tiles = groupTiles(g, n, gr);
    for (uint64_t local = 0; local < tiles; local += sampleStride) {
      const uint64_t begin = sampledTile(local, gr, g.tilesPerBlock) * PART_TILE;
      if (begin < n) sc.seen[gr] += (double)std::min<uint64_t>(PART_TILE, n - begin);
    }
  }
  if (exact) {
    sc.sigmas = sc.frac = sc.floor = 0;
  } else {  // 6 sigma + 2% + 256 (tasks/SampledNetworkPartitioning.cpp, same statistics)
    sc.sigmas = 6.0;
    sc.frac = 0.02;
    sc.floor = 256.0;
  }
  return sc;
}

uint64_t sampledWindowCapacity(const SampleScale &sc, uint32_t F, uint32_t roundLp) {
  const uint64_t bound = sampledLayoutCapacityBound(sc, F);
  if (!roundLp) return bound;
  double maxCap = 0;
  for (uint32_t g = 0; g < NGROUPS; ++g) {
    if (sc.total[g] <= 0) continue;
    const double scale = sc.seen[g] > 0 ? sc.total[g] / sc.seen[g] : 1.0;
    // The largest slice: its sampled estimate up to 5 sigma above the mean,
    // plus the layout kernel's margin taken at that estimate.
    const double mean = sc.total[g] / F;
    const double hi = mean + 5.0 * std::sqrt(std::max(mean, scale) * scale);
    maxCap = std::max(maxCap, hi + sc.sigmas * std::sqrt(std::max(hi, scale) * scale) + sc.frac * hi + sc.floor + 16.0);
  }
  uint32_t lns = 0;
  while ((1u << lns) < NGROUPS * F) ++lns;
  return std::max<uint64_t>(bound, roundSlots((uint64_t)std::ceil(maxCap), roundLp, lns));
}

uint64_t sampledLayoutCapacityBound(const SampleScale &sc, uint32_t F) {
  // Per group: sum_d est_d = total_g; sum_d sqrt(max(est_d,scale) * scale) <=
  // sqrt(F * scale * (total_g + F * scale)) (Cauchy-Schwarz); + ceil and the 16-tuple
  // line rounding per slice.
  double b = 0;
  for (uint32_t g = 0; g < NGROUPS; ++g) {
    if (sc.total[g] <= 0) continue;
    const double scale = sc.seen[g] > 0 ? sc.total[g] / sc.seen[g] : 1.0;
    b += (1.0 + sc.frac) * sc.total[g] + sc.sigmas * std::sqrt((double)F * scale * (sc.total[g] + F * scale)) +
         (sc.floor + 17.0) * F;
  }
  return (uint64_t)(b * 1.0001) + 4096;
}

void scatterAblation(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift, const PartitionGeometry &g,
                     const uint64_t *cursors, uint64_t *out, int mode, int geometry, hipStream_t s, void *gcur,
                     const uint32_t *roundMeta) {
  NetCompressedPol pol;
  pol.mask = (1ull << bits) - 1;
  pol.bits = bits;
  pol.keyShift = keyShift;
  NetCompressedDigPol dpol;
  static_cast<NetCompressedPol &>(dpol) = pol;
#define HJ_CLAIM(NTH, IPT)                                                                                        \
  withMaxd<NTH>(1u << bits, [&](auto maxd) {                                                                      \
    constexpr int M = decltype(maxd)::value;                                                                      \
    const size_t lds = ScatterLayout<NetCompressedPol, uint32_t, NTH * IPT>::bytes(1u << bits);                  \
    auto *gc = reinterpret_cast<uint32_t *>(gcur);                                                                \
    if (mode == 1)                                                                                                \
      hipLaunchKernelGGL((netScatterClaimKernel<NetCompressedPol, uint32_t, NTH, IPT, 1, false, M>), dim3(g.blocks), \
                         dim3(NTH), lds, s, reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock,         \
                         1u << bits, pol, 0u, gc, out);                                                           \
    else if (mode == 3)                                                                                           \
      hipLaunchKernelGGL((netScatterClaimKernel<NetCompressedPol, uint32_t, NTH, IPT, 0, false, M>), dim3(g.blocks), \
                         dim3(NTH), lds, s, reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock,         \
                         1u << bits, pol, 0u, gc, out, nullptr, roundMeta);                                       \
    else                                                                                                          \
      hipLaunchKernelGGL((netScatterClaimKernel<NetCompressedPol, uint32_t, NTH, IPT, 0, false, M>), dim3(g.blocks), \
                         dim3(NTH), lds, s, reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock,         \
                         1u << bits, pol, 0u, gc, out);                                                           \
  })
#define HJ_ABL(P, p, NTH, IPT)                                                                                    \
  do {                                                                                                            \
    if (mode == 1) launchNet<P, uint32_t, NTH, IPT, 1>(p, in, n, bits, g, 0, g.blocks, cursors, out, s);          \
    else if (mode == 2) launchNet<P, uint32_t, NTH, IPT, 2>(p, in, n, bits, g, 0, g.blocks, cursors, out, s);     \
    else launchNet<P, uint32_t, NTH, IPT, 0>(p, in, n, bits, g, 0, g.blocks, cursors, out, s);                    \
  } while (0)
  // 10: the count-only fragment scatter of the bitmap plan (4-byte output,
  // 1024 x 16 tiles): mode 0 real, 1 coalesced write-out, 2 no write-out.
  // Measured at 1B tuples, bits 8/9/10/11: 4.18/4.30/4.45/4.70 ms real against
  // ~3.87 coalesced and ~2.6 without writes (streaming ceiling of the byte mix
  // 3.47 ms, tools/stream_mix_bench.py): the scatter pays for runs of ~16
  // fragments per partition and tile.  Key-only loads with 24-key tiles
  // (longer runs) spilled and ran 4.56 ms at bits 10; key-only loads through a
  // buffer resource with two register tiles (the next tile's loads issued
  // before this one is ranked) ran 2 % slower in the 1B join (network pass
  // 8.78 vs 8.60 ms): the pass is bound by the scattered writes, not by load
  // latency.
  HJ_CHECK(mode != 3 || (geometry >= 6 && geometry <= 9 && roundMeta), "scatterAblation: mode 3 needs a claim geometry");
  NetFragPol fpol;
  fpol.mask = (1ull << bits) - 1;
  fpol.bits = bits;
  using FragLayout = ScatterLayout<NetFragPol, uint32_t, 1024 * 16>;
  const size_t fragLds = FragLayout::bytes(1u << bits);
#define HJ_FRAG(M)                                                                                                \
  withMaxd<1024>(1u << bits, [&](auto maxd) {                                                                     \
    hipLaunchKernelGGL((netScatterClaimKernel<NetFragPol, uint32_t, 1024, 16, M, false, decltype(maxd)::value>),  \
                       dim3(g.blocks), dim3(1024), fragLds, s, reinterpret_cast<const ulonglong2 *>(in), n,      \
                       g.tilesPerBlock, 1u << bits, fpol, 0u, reinterpret_cast<uint32_t *>(gcur),                 \
                       reinterpret_cast<uint32_t *>(out));                                                        \
  })
  if (geometry == 10) {
    if (mode == 1) HJ_FRAG(1);
    else if (mode == 2) HJ_FRAG(2);
    else HJ_FRAG(0);
    HIP_CHECK_LAUNCH();
    return;
  }
#undef HJ_FRAG
  switch (geometry) {
    case 1: HJ_ABL(NetCompressedPol, pol, 512, 16); break;
    case 2: HJ_ABL(NetCompressedPol, pol, 1024, 8); break;
    case 3: HJ_ABL(NetCompressedPol, pol, 1024, 16); break;
    case 4: HJ_ABL(NetCompressedDigPol, dpol, 256, 16); break;
    case 5: HJ_ABL(NetCompressedPol, pol, 256, 8); break;
    case 6: HJ_CLAIM(256, 16); break;
    case 7: HJ_CLAIM(512, 16); break;
    case 8: HJ_CLAIM(1024, 16); break;
    case 9: HJ_CLAIM(1024, 8); break;
    default: HJ_ABL(NetCompressedPol, pol, 256, 16); break;
  }
#undef HJ_ABL
#undef HJ_CLAIM
}

// Ablation: per-tuple global atomics on a per-digit cursor (no LDS staging).
__global__ __launch_bounds__(NT) void netScatterGlobalAtomicKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                                   uint32_t bits, uint32_t keyShift,
                                                                   unsigned long long *cursor, uint64_t *out) {
  const uint64_t mask = (1ull << bits) - 1;
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += stride) {
    const ulonglong2 x = in[i];
    const unsigned long long pos = atomicAdd(&cursor[x.x & mask], 1ull);
    out[pos] = x.y | ((x.x >> bits) << keyShift);
  }
}

void netScatterGlobalAtomic(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift,
                            uint64_t *digitCursor, uint64_t *out, hipStream_t s) {
  if (n == 0) return;
  const uint64_t want = ceilDiv(n, NT);
  const uint32_t blocks = (uint32_t)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(netScatterGlobalAtomicKernel, dim3(blocks), dim3(NT), 0, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, bits, keyShift,
                     reinterpret_cast<unsigned long long *>(digitCursor), out);
  HIP_CHECK_LAUNCH();
}

// ------------------------------------------------------ pass 2 (local) kernels
// KIND: 0 = 8-byte CompressedTuple / key-only word, 1 = 16-byte tuple (its
// key), 2 = u32 key fragment (JoinPlan::fragments).
template <int KIND>
__device__ __forceinline__ uint64_t localWord(const void *in, uint64_t i) {
  if constexpr (KIND == 1)
    return reinterpret_cast<const ulonglong2 *>(in)[i].x;
  else if constexpr (KIND == 2)
    return reinterpret_cast<const uint32_t *>(in)[i];
  else
    return reinterpret_cast<const uint64_t *>(in)[i];
}

template <int WIDE>
__global__ __launch_bounds__(NT) void localHistogramKernel(const void *__restrict__ in,
                                                           const LocalItem *__restrict__ items, uint32_t shift,
                                                           uint32_t bits, uint32_t *__restrict__ itemHist,
                                                           uint32_t stride, RoundMap rm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  const int wid = threadIdx.x / WAVE;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  const LocalItem it = items[blockIdx.x];
  uint32_t *wh = hsh + wid * F;
  for (uint32_t base = 0; base < it.len; base += PART_TILE * stride) {
    uint64_t w[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = base + i * NT + threadIdx.x;
      w[i] = idx < it.len ? localWord<WIDE>(in, rm(it.begin + idx)) : 0;
    }
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = base + i * NT + threadIdx.x;
      if (idx < it.len) atomicAdd(&wh[(w[i] >> shift) & mask], 1u);
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < F; d += NT)
    itemHist[(uint64_t)blockIdx.x * F + d] = hsh[d] + hsh[F + d] + hsh[2 * F + d] + hsh[3 * F + d];
}

// 8-byte words whose digit lies inside one 32-bit half (HALF 0 = low word,
// 1 = high word; shift is then relative to that half): every thread loads
// only that half, and both of a batch's two sampled tiles are in flight
// before the first is counted (an item of the 1B x 1B general path holds two
// sampled tiles: one HBM round trip instead of two).
template <int HALF>
__global__ __launch_bounds__(NT) void localHistogramHalfKernel(const uint32_t *__restrict__ in,
                                                               const LocalItem *__restrict__ items, uint32_t shift,
                                                               uint32_t bits, uint32_t *__restrict__ itemHist,
                                                               uint32_t stride, RoundMap rm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  const uint32_t F = 1u << bits, mask = F - 1;
  const int wid = threadIdx.x / WAVE;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  const LocalItem it = items[blockIdx.x];
  uint32_t *wh = hsh + wid * F;
  const uint32_t step = PART_TILE * stride;
  for (uint32_t base = 0; base < it.len; base += 2 * step) {
    uint32_t w[2][PART_ITEMS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < (int)PART_ITEMS; ++i) {
        const uint32_t idx = base + t * step + i * NT + threadIdx.x;
        w[t][i] = idx < it.len ? __builtin_nontemporal_load(in + 2 * rm(it.begin + idx) + HALF) : 0u;
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < (int)PART_ITEMS; ++i) {
        const uint32_t idx = base + t * step + i * NT + threadIdx.x;
        if (idx < it.len) atomicAdd(&wh[(w[t][i] >> shift) & mask], 1u);
      }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < F; d += NT)
    itemHist[(uint64_t)blockIdx.x * F + d] = hsh[d] + hsh[F + d] + hsh[2 * F + d] + hsh[3 * F + d];
}

void localHistogram(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift,
                    uint32_t bits, uint32_t *itemHist, hipStream_t s, uint32_t sampleStride, bool frag, RoundMap rm) {
  HJ_CHECK(bits <= MAX_PART_BITS, "localHistogram: bits=%u out of range", bits);
  HJ_CHECK(sampleStride >= 1, "localHistogram: sampleStride must be >= 1");
  HJ_CHECK(!(wide && frag), "localHistogram: fragments are not wide tuples");
  if (nItems == 0) return;
  const size_t lds = size_t(4) << bits << 2;
  const char *hv = std::getenv("HPCJOIN_LH_HALF");  // "0": the whole-word kernel (A/B)
  if (!wide && !frag && (shift + bits <= 32 || shift >= 32) && !(hv && hv[0] == '0')) {
    const auto *w = static_cast<const uint32_t *>(in);
    if (shift >= 32)
      hipLaunchKernelGGL(localHistogramHalfKernel<1>, dim3(nItems), dim3(NT), lds, s, w, items, shift - 32, bits,
                         itemHist, sampleStride, rm);
    else
      hipLaunchKernelGGL(localHistogramHalfKernel<0>, dim3(nItems), dim3(NT), lds, s, w, items, shift, bits,
                         itemHist, sampleStride, rm);
  } else if (frag)
    hipLaunchKernelGGL(localHistogramKernel<2>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits, itemHist,
                       sampleStride, rm);
  else if (wide)
    hipLaunchKernelGGL(localHistogramKernel<1>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits, itemHist,
                       sampleStride, rm);
  else
    hipLaunchKernelGGL(localHistogramKernel<0>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits, itemHist,
                       sampleStride, rm);
  HIP_CHECK_LAUNCH();
}

uint32_t assignLocalStreams(LocalItem *items, uint32_t nItems) {
  // Block b of the local scatter runs item (b % NGROUPS) * q + b / NGROUPS, so
  // the items of group g = item / q are one contiguous run of the (lp-sorted)
  // list and share an XCD; a stream = one (lp, group) run.
  const uint32_t q = (nItems + NGROUPS - 1) / NGROUPS;
  uint32_t streams = 0, prevLp = ~0u, prevG = ~0u;
  for (uint32_t i = 0; i < nItems; ++i) {
    const uint32_t g = i / (q ? q : 1);
    if (items[i].lp != prevLp || g != prevG) {
      ++streams;
      prevLp = items[i].lp;
      prevG = g;
    }
    items[i].stream = streams - 1;
  }
  return streams;
}

// One workgroup per owned partition lp: turns the [item][F] histograms of its
// items into the start of every (stream, sub-partition) claim slice and the
// final partition begin offsets partBegin[lp*F + q].
template <typename CurT>
__global__ __launch_bounds__(NT) void localCursorsKernel(const uint32_t *__restrict__ itemHist,
                                                         const uint32_t *__restrict__ lpItemBegin, uint32_t owned,
                                                         uint32_t bits, const uint64_t *__restrict__ lpBase,
                                                         const LocalItem *__restrict__ items, CurT *__restrict__ gcur,
                                                         uint64_t *__restrict__ partBegin) {
  extern __shared__ __attribute__((aligned(16))) uint64_t csh[];
  const uint32_t F = 1u << bits;
  uint64_t *tot = csh;     // [F]
  uint64_t *wt = csh + F;  // [NT/64]
  const uint32_t lp = blockIdx.x;
  const uint32_t ib = lpItemBegin[lp], ie = lpItemBegin[lp + 1];
  for (uint32_t q = threadIdx.x; q < F; q += NT) {
    uint64_t s = 0;
    for (uint32_t it = ib; it < ie; ++it) s += itemHist[(uint64_t)it * F + q];
    tot[q] = s;
  }
  __syncthreads();
  blockExclusiveScanLds<NT, uint64_t, uint64_t>(tot, tot, (int)F, wt);
  const uint64_t base = lpBase[lp];
  for (uint32_t q = threadIdx.x; q < F; q += NT) {
    uint64_t run = base + tot[q];
    partBegin[(uint64_t)lp * F + q] = run;
    uint32_t prev = ~0u;
    for (uint32_t it = ib; it < ie; ++it) {
      const uint32_t st = items[it].stream;
      if (st != prev) {
        gcur[(uint64_t)st * F + q] = (CurT)run;
        prev = st;
      }
      run += itemHist[(uint64_t)it * F + q];
    }
  }
  if (lp == owned - 1 && threadIdx.x == 0) partBegin[(uint64_t)owned * F] = lpBase[owned];
}

void localCursors(const uint32_t *itemHist, const uint32_t *lpItemBegin, uint32_t owned, uint32_t bits,
                  const uint64_t *lpBase, const LocalItem *items, void *gcur, bool narrow, uint64_t *partBegin,
                  hipStream_t s) {
  if (owned == 0) return;
  const size_t lds = (size_t(1) << bits) * 8 + 64;
  if (narrow)
    hipLaunchKernelGGL(localCursorsKernel<uint32_t>, dim3(owned), dim3(NT), lds, s, itemHist, lpItemBegin, owned, bits,
                       lpBase, items, reinterpret_cast<uint32_t *>(gcur), partBegin);
  else
    hipLaunchKernelGGL(localCursorsKernel<unsigned long long>, dim3(owned), dim3(NT), lds, s, itemHist, lpItemBegin,
                       owned, bits, lpBase, items, reinterpret_cast<unsigned long long *>(gcur), partBegin);
  HIP_CHECK_LAUNCH();
}

// Sampled local pass: tuples of item it the histogram read (tiles 0, S, 2S...).
__device__ __forceinline__ uint32_t sampledLen(uint32_t len, uint32_t stride) {
  uint32_t seen = 0;
  for (uint32_t b = 0; b < len; b += PART_TILE * stride) seen += min((uint32_t)PART_TILE, len - b);
  return seen;
}

// One workgroup per owned partition lp: capacity of each final partition
// (lp, q) = sampled estimate + LOCAL_SIGMAS sigma of the sampling error + 2% + 64.
// With ~240 sampled tuples per final partition (1 tile in 16), a low sample
// shrinks both the estimate and its margin: at 6 sigma a slot overflows with
// probability ~1e-7 (Poisson lower tail), i.e. a few percent of 1B x 1B joins
// (2^19 slots) would take the exact re-run; at 8 sigma ~1e-11.  The price is
// memory only (gaps are never read): ~+15% of the local output allocation.
constexpr double LOCAL_SIGMAS = 8.0;
__global__ __launch_bounds__(NT) void localCapacityKernel(const uint32_t *__restrict__ itemHist,
                                                          const uint32_t *__restrict__ lpItemBegin,
                                                          const LocalItem *__restrict__ items, uint32_t bits,
                                                          uint32_t stride, uint32_t align, uint32_t *__restrict__ caps) {
  const uint32_t F = 1u << bits, lp = blockIdx.x;
  const uint32_t ib = lpItemBegin[lp], ie = lpItemBegin[lp + 1];
  double len = 0, seen = 0;
  for (uint32_t it = ib; it < ie; ++it) {
    len += items[it].len;
    seen += sampledLen(items[it].len, stride);
  }
  const double scale = seen > 0 ? len / seen : 1.0;
  for (uint32_t q = threadIdx.x; q < F; q += NT) {
    double est = 0;
    for (uint32_t it = ib; it < ie; ++it) {
      const uint32_t s = sampledLen(items[it].len, stride);
      if (s) est += (double)itemHist[(uint64_t)it * F + q] * ((double)items[it].len / s);
    }
    const double cap = est + LOCAL_SIGMAS * sqrt(fmax(est, 1.0) * scale) + 0.02 * est + 64.0;
    // Whole 128-byte lines per slot (align = 16 tuples of 8 bytes, or 64 of
    // 6 bytes): partitions never share a cache line, so the scatter's partial
    // lines at slot edges are not split across XCDs and every build/probe read
    // starts line-aligned.
    const uint32_t c = (uint32_t)min(ceil(cap), 4294967040.0);
    caps[(uint64_t)lp * F + q] = (c + align - 1) / align * align;
  }
}

// gcur = partBegin = exclusive prefix of caps; gend = start + cap.  Both are
// clamped to the allocated capacity, so no write or later read can leave the
// buffer even if the host-side bound were ever too small (the slot would
// just overflow and trigger the exact re-run).
__global__ __launch_bounds__(NT) void localSampledCursorsKernel(const uint32_t *__restrict__ caps,
                                                                const unsigned long long *__restrict__ starts,
                                                                uint64_t P, unsigned long long capacity,
                                                                unsigned long long *__restrict__ gcur,
                                                                unsigned long long *__restrict__ gend,
                                                                uint64_t *__restrict__ partBegin) {
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < P; i += stride) {
    const unsigned long long s = min(starts[i], capacity);
    gcur[i] = s;
    gend[i] = min(s + (unsigned long long)caps[i], capacity);
    partBegin[i] = s;
  }
}

// flag |= some final claim cursor passed its slice end (the run is redone
// exactly); gcur is clamped to the slice end so that, used as partition ends,
// it never points past what was written.
__global__ __launch_bounds__(NT) void claimOverflowKernel(unsigned long long *__restrict__ gcur,
                                                          const unsigned long long *__restrict__ gend, uint64_t P,
                                                          unsigned int *flag) {
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  bool over = false;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < P; i += stride) {
    const unsigned long long g = gcur[i], e = gend[i];
    if (g > e) {
      over = true;
      gcur[i] = e;
    }
  }
  if (__any(over) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(flag, 1u);
}

void localSampledLayout(const uint32_t *itemHist, const uint32_t *lpItemBegin, const LocalItem *items,
                        uint32_t owned, uint32_t bits, uint32_t sampleStride, uint32_t *caps,
                        unsigned long long *starts, void *scanWorkspace, unsigned long long *gcur,
                        unsigned long long *gend, uint64_t *partBegin, uint64_t capacity, hipStream_t s,
                        uint32_t align) {
  if (owned == 0) return;
  HJ_CHECK(align >= 1 && align <= 256, "localSampledLayout: align=%u", align);
  const uint64_t P = (uint64_t)owned << bits;
  hipLaunchKernelGGL(localCapacityKernel, dim3(owned), dim3(NT), 0, s, itemHist, lpItemBegin, items, bits,
                     sampleStride, align, caps);
  HIP_CHECK_LAUNCH();
  scanExclusiveU32to64(caps, starts, P, nullptr, scanWorkspace, s);
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ceilDiv(P, NT), 4096);
  hipLaunchKernelGGL(localSampledCursorsKernel, dim3(grid), dim3(NT), 0, s, caps, starts, P,
                     (unsigned long long)capacity, gcur, gend, partBegin);
  HIP_CHECK_LAUNCH();
}

uint64_t localSampledCapacityBound(uint64_t n, uint64_t partitions, uint32_t sampleStride, uint32_t align) {
  // Sum of the per-partition capacities: estimates sum to n; by Cauchy-Schwarz
  // the sigma terms sum to at most LOCAL_SIGMAS sqrt(n * S * P); + per partition for
  // the constant, the ceil and float rounding.
  // (an item's len/seen ratio is at most ~sampleStride; +1 covers the rounding)
  const double bound = 1.02 * (double)n +
                       LOCAL_SIGMAS * std::sqrt(((double)n + (double)partitions) * (sampleStride + 1.0) * (double)partitions) +
                       (66.0 + align) * (double)partitions;  // 64 + ceil + line rounding + float slack
  return (uint64_t)(bound * 1.001) + 1024;
}

void claimOverflow(unsigned long long *gcur, const unsigned long long *gend, uint64_t P, unsigned int *flag,
                   hipStream_t s) {
  if (P == 0) return;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ceilDiv(P, NT), 4096);
  hipLaunchKernelGGL(claimOverflowKernel, dim3(grid), dim3(NT), 0, s, gcur, gend, P, flag);
  HIP_CHECK_LAUNCH();
}

template <class Pol, typename CurT, int NTH, int IPT, bool BOUNDED, int MAXD>
__global__ __launch_bounds__(NTH, ScatterOcc<NTH>::value) void localScatterClaimKernel(
    const typename Pol::InT *__restrict__ in, const LocalItem *__restrict__ items, uint32_t nItems, uint32_t F,
    Pol pol, CurT *__restrict__ gcur, typename Pol::OutT *out, const CurT *__restrict__ gend, RoundMap im) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t q = (nItems + NGROUPS - 1) / NGROUPS;
  const uint32_t item = (blockIdx.x % NGROUPS) * q + blockIdx.x / NGROUPS;  // XCD-contiguous items
  if (item >= nItems) return;  // uniform per workgroup
  const uint32_t FP = padDigits(F);
  CurT *sliceEnd = reinterpret_cast<CurT *>(smem);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(reinterpret_cast<CurT *>(smem) + 2 * FP);
  const LocalItem it = items[item];
  for (uint32_t d = threadIdx.x; d < FP; d += NTH) {
    cnt[d] = 0;
    if constexpr (BOUNDED)
      if (d < F) sliceEnd[d] = gend[(uint64_t)it.stream * F + d];
  }
  __syncthreads();
  scatterRange<Pol, CurT, NTH, IPT, 0, true, BOUNDED, MAXD>(in, it.begin, it.begin + it.len, F, smem, pol, out,
                                                            gcur + (uint64_t)it.stream * F, im);
}

// Persistent local claim scatter.  Work items are short (1B x 1B: a network
// partition's slice of one claim group, ~120K tuples = 15 tiles) and the
// production workgroup owns its CU (1024 threads, ~90 KB of LDS), so a
// workgroup per item drained the tile pipeline at every item end (the last
// tile's write-out overlapped nothing) and refilled it at the next item's
// start (workgroup launch, LDS init, first tile's loads exposed).  Here a
// workgroup walks the items of its XCD's contiguous run with a stride of the
// workgroups on that XCD, and the prefetch issued while an item's last tile
// is staged already loads the next item's first tile.  Between items only
// the bounded slot ends are swapped (after an LDS barrier: the last
// write-out read them).
template <class Pol, typename CurT, int NTH, int IPT, bool BOUNDED, int MAXD>
__global__ __launch_bounds__(NTH, ScatterOcc<NTH>::value) void localScatterPersistKernel(
    const typename Pol::InT *__restrict__ in, const LocalItem *__restrict__ items, uint32_t nItems, uint32_t F,
    Pol pol, CurT *__restrict__ gcur, typename Pol::OutT *out, const CurT *__restrict__ gend, uint32_t perXcd,
    RoundMap im) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr uint32_t TILE = NTH * IPT;
  const uint32_t q = (nItems + NGROUPS - 1) / NGROUPS;
  const uint32_t first = (blockIdx.x % NGROUPS) * q, last = min(nItems, first + q);  // this XCD's items
  uint32_t cur = first + blockIdx.x / NGROUPS;
  if (cur >= last) return;  // uniform per workgroup
  const uint32_t FP = padDigits(F);
  const ScatterSmem<Pol, CurT, TILE> l(smem, F);
  LocalItem it = items[cur];
  for (uint32_t d = threadIdx.x; d < FP; d += NTH) {
    l.cnt[d] = 0;
    if constexpr (BOUNDED)
      if (d < F) l.cursor[d] = gend[(uint64_t)it.stream * F + d];
  }
  __syncthreads();
  typename Pol::LoadT v[IPT];
  ScatterProf pf;
  prefetchTile<Pol, NTH, IPT>(in, it.begin, it.begin + it.len - 1, v, im);
  for (;;) {
    const uint32_t nxt = cur + perXcd;
    const bool more = nxt < last;
    const LocalItem nit = more ? items[nxt] : it;
    const uint64_t end = it.begin + it.len;
    CurT *gc = gcur + (uint64_t)it.stream * F;
    for (uint64_t base = it.begin; base < end; base += TILE) {
      const bool lastTile = base + TILE >= end;
      const uint64_t nb = lastTile ? nit.begin : base + TILE;
      const uint64_t nl = lastTile ? nit.begin + nit.len - 1 : end - 1;
      if (base + TILE <= end)
        scatterTile<Pol, CurT, NTH, IPT, 0, true, true, BOUNDED, MAXD>(in, base, end, TILE, F, l, pol, out, v, gc,
                                                                       pf, nb, nl, im);
      else
        scatterTile<Pol, CurT, NTH, IPT, 0, false, true, BOUNDED, MAXD>(in, base, end, (uint32_t)(end - base), F, l,
                                                                        pol, out, v, gc, pf, nb, nl, im);
    }
    if (!more) break;
    if constexpr (BOUNDED) {
      CurT e[MAXD];
#pragma unroll
      for (int k = 0; k < MAXD; ++k) {
        const uint32_t d = threadIdx.x + k * NTH;
        e[k] = d < F ? gend[(uint64_t)nit.stream * F + d] : (CurT)0;
      }
      ldsBarrier();  // every wave's last write-out has read the old slot ends
#pragma unroll
      for (int k = 0; k < MAXD; ++k) {
        const uint32_t d = threadIdx.x + k * NTH;
        if (d < F) l.cursor[d] = e[k];
      }
      // visible to the next tile's write-out through its barriers A and B
    }
    it = nit;
    cur = nxt;
  }
  pf.flush();
}

// Workgroups per XCD of the persistent local scatter: what stays resident.
template <class K>
static uint32_t persistPerXcd(K kernel, uint32_t nth, size_t lds, uint32_t nItems) {
  static thread_local int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  int per = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void *>(kernel), (int)nth, lds));
  const uint32_t q = (nItems + NGROUPS - 1) / NGROUPS;
  const uint32_t want = (uint32_t)std::max(1, per) * (uint32_t)std::max(1, cus / (int)NGROUPS);
  return std::max<uint32_t>(1, std::min<uint32_t>(want, q));
}

template <class P, typename C, int NTH, int IPT>
static void launchLocalClaimPersist(const void *in, const LocalItem *items, uint32_t nItems, uint32_t F, const P &pol,
                                    void *gcur, void *out, const void *gend, hipStream_t s, RoundMap rm) {
  const size_t lds = ScatterLayout<P, C, NTH * IPT>::bytes(F);
  HJ_CHECK(lds <= 160 * 1024, "local scatter LDS %zu too large", lds);
  withMaxd<NTH>(F, [&](auto maxd) {
    constexpr int M = decltype(maxd)::value;
    auto go = [&](auto kernel, const C *ge) {
      const uint32_t per = persistPerXcd(kernel, NTH, lds, nItems);
      hipLaunchKernelGGL(kernel, dim3(per * NGROUPS), dim3(NTH), lds, s, reinterpret_cast<const typename P::InT *>(in),
                         items, nItems, F, pol, reinterpret_cast<C *>(gcur), reinterpret_cast<typename P::OutT *>(out),
                         ge, per, rm);
    };
    if (gend)
      go(localScatterPersistKernel<P, C, NTH, IPT, true, M>, reinterpret_cast<const C *>(gend));
    else
      go(localScatterPersistKernel<P, C, NTH, IPT, false, M>, nullptr);
  });
}

// One local claim-scatter launch (MAXD from F, bounded when gend is given).
template <class P, typename C, int NTH, int IPT>
static void launchLocalClaim(const void *in, const LocalItem *items, uint32_t nItems, uint32_t F, const P &pol,
                             void *gcur, void *out, const void *gend, hipStream_t s, RoundMap rm) {
  const size_t lds = ScatterLayout<P, C, NTH * IPT>::bytes(F);
  HJ_CHECK(lds <= 160 * 1024, "local scatter LDS %zu too large", lds);
  const uint32_t grid = ((nItems + NGROUPS - 1) / NGROUPS) * NGROUPS;
  withMaxd<NTH>(F, [&](auto maxd) {
    constexpr int M = decltype(maxd)::value;
    if (gend)
      hipLaunchKernelGGL((localScatterClaimKernel<P, C, NTH, IPT, true, M>), dim3(grid), dim3(NTH), lds, s,
                         reinterpret_cast<const typename P::InT *>(in), items, nItems, F, pol,
                         reinterpret_cast<C *>(gcur), reinterpret_cast<typename P::OutT *>(out),
                         reinterpret_cast<const C *>(gend), rm);
    else
      hipLaunchKernelGGL((localScatterClaimKernel<P, C, NTH, IPT, false, M>), dim3(grid), dim3(NTH), lds, s,
                         reinterpret_cast<const typename P::InT *>(in), items, nItems, F, pol,
                         reinterpret_cast<C *>(gcur), reinterpret_cast<typename P::OutT *>(out), nullptr, rm);
  });
}

template <class P>
static void setSplit(P &, const SplitLayout &) {}
static void setSplit(LocalFragPol &p, const SplitLayout &sl) { p.fragShift = sl.fragShift; }
static void setSplit(LocalSplitPol &p, const SplitLayout &sl) {
  p.hi = sl.hi;
  p.fragShift = sl.fragShift;
  p.loShift = sl.loShift;
}

// Alternative workgroup geometries of the production local scatter (split
// output, 64-bit cursors, bounded slots) for the geometry sweep.
template <int NTH, int IPT>
static void launchLocalSplitGeom(const void *in, const LocalItem *items, uint32_t nItems, uint32_t F,
                                 const LocalSplitPol &pol, void *gcur, void *out, const void *gend, hipStream_t s,
                                 RoundMap rm) {
  launchLocalClaim<LocalSplitPol, unsigned long long, NTH, IPT>(in, items, nItems, F, pol, gcur, out, gend, s, rm);
}

void localScatter(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift, uint32_t bits,
                  void *gcur, bool narrow, void *out, hipStream_t s, const void *gend, SplitLayout split,
                  uint32_t geometry, bool frag, RoundMap rm) {
  HJ_CHECK(!(wide && split.on), "localScatter: the split layout needs compressed input");
  HJ_CHECK(!split.on || frag || split.hi, "localScatter: split layout without a fragment column");
  HJ_CHECK(!(frag && wide), "localScatter: fragments are not wide tuples");
  HJ_CHECK(bits <= MAX_PART_BITS, "localScatter: bits=%u out of range", bits);
  if (nItems == 0) return;
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  const uint32_t grid = ((nItems + NGROUPS - 1) / NGROUPS) * NGROUPS;
  // geometry 5: the default 1024 x 8 shape as one workgroup per item (the
  // round-5 kernel, kept for A/B); 0: persistent workgroups over the items;
  // 6 / 7: persistent with 12 / 10 tuples per thread (longer runs per digit
  // and tile, split layout only).
  const bool persist = geometry == 0;
  if ((geometry == 6 || geometry == 7) && split.on && !wide && !frag && gend) {
    LocalSplitPol pol;
    pol.mask = mask;
    pol.shift = shift;
    setSplit(pol, split);
    auto go = [&](auto cur, auto ipt) {
      using C = decltype(cur);
      launchLocalClaimPersist<LocalSplitPol, C, CL_NTH, decltype(ipt)::value>(in, items, nItems, F, pol, gcur, out,
                                                                               gend, s, rm);
    };
    if (geometry == 6) {
      if (narrow) go(uint32_t(), std::integral_constant<int, 12>());
      else go((unsigned long long)0, std::integral_constant<int, 12>());
    } else {
      if (narrow) go(uint32_t(), std::integral_constant<int, 10>());
      else go((unsigned long long)0, std::integral_constant<int, 10>());
    }
    HIP_CHECK_LAUNCH();
    return;
  }
  if (geometry != 0 && geometry != 5 && split.on && !wide && !frag && !narrow && gend) {
    LocalSplitPol pol;
    pol.mask = mask;
    pol.shift = shift;
    setSplit(pol, split);
    switch (geometry) {
      case 1: launchLocalSplitGeom<512, 8>(in, items, nItems, F, pol, gcur, out, gend, s, rm); break;
      case 2: launchLocalSplitGeom<512, 16>(in, items, nItems, F, pol, gcur, out, gend, s, rm); break;
      case 3: launchLocalSplitGeom<256, 16>(in, items, nItems, F, pol, gcur, out, gend, s, rm); break;
      default: launchLocalSplitGeom<1024, 16>(in, items, nItems, F, pol, gcur, out, gend, s, rm); break;
    }
    HIP_CHECK_LAUNCH();
    return;
  }
#define HJ_LOCAL(P, C)                                                                                      \
  do {                                                                                                      \
    P pol;                                                                                                  \
    pol.mask = mask;                                                                                        \
    pol.shift = shift;                                                                                      \
    setSplit(pol, split);                                                                                   \
    if (persist)                                                                                            \
      launchLocalClaimPersist<P, C, CL_NTH, CL_IPT>(in, items, nItems, F, pol, gcur, out, gend, s, rm);     \
    else                                                                                                    \
      launchLocalClaim<P, C, CL_NTH, CL_IPT>(in, items, nItems, F, pol, gcur, out, gend, s, rm);            \
  } while (0)
  if (frag && narrow) HJ_LOCAL(LocalFragPol, uint32_t);
  else if (frag) HJ_LOCAL(LocalFragPol, unsigned long long);
  else if (wide && narrow) HJ_LOCAL(LocalWidePol, uint32_t);
  else if (wide) HJ_LOCAL(LocalWidePol, unsigned long long);
  else if (split.on && narrow) HJ_LOCAL(LocalSplitPol, uint32_t);
  else if (split.on) HJ_LOCAL(LocalSplitPol, unsigned long long);
  else if (narrow) HJ_LOCAL(LocalCompressedPol, uint32_t);
  else HJ_LOCAL(LocalCompressedPol, unsigned long long);
#undef HJ_LOCAL
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadPartition() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&netHistogramKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
