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

#include <type_traits>

namespace hpcjoin {
namespace kernels {

constexpr int NT = PART_THREADS;

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

static size_t scatterLds(uint32_t F, size_t outBytes) {
  return size_t(F) * 16 + 64 + size_t(PART_TILE) * outBytes + size_t(PART_TILE) * 2;
}

size_t netScatterLdsBytes(uint32_t bits, bool wide) { return scatterLds(1u << bits, wide ? 16 : 8); }

// ------------------------------------------------------------------ loads
template <typename InT>
struct Loader;
template <>
struct Loader<ulonglong2> {
  static __device__ __forceinline__ ulonglong2 load(const ulonglong2 *p) { return *p; }
};
template <>
struct Loader<uint64_t> {
  static __device__ __forceinline__ uint64_t load(const uint64_t *p) { return *p; }
};

// ------------------------------------------------------- histogram (pass 1)
__global__ __launch_bounds__(NT) void netHistogramKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                         uint32_t tpb, uint32_t bits,
                                                         uint32_t *__restrict__ blockHist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  const uint32_t F = 1u << bits, mask = F - 1;
  const int wid = threadIdx.x / WAVE;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  uint32_t *wh = hsh + wid * F;
  const uint64_t begin = (uint64_t)blockIdx.x * tpb * PART_TILE;
  const uint64_t end = min(n, begin + (uint64_t)tpb * PART_TILE);
  for (uint64_t base = begin; base < end; base += PART_TILE) {
    uint64_t k[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint64_t idx = base + (uint64_t)i * NT + threadIdx.x;
      k[i] = idx < end ? in[idx].x : 0;
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

void netHistogram(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                  uint32_t *blockHist, hipStream_t s) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netHistogram: bits=%u out of range", bits);
  const size_t lds = size_t(4) << bits << 2;
  hipLaunchKernelGGL(netHistogramKernel, dim3(g.blocks), dim3(NT), lds, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock, bits, blockHist);
  HIP_CHECK_LAUNCH();
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

// -------------------------------------------------- LDS write-combining scatter
struct ScatterLds {
  uint64_t *cursor;  // [F]
  uint32_t *cnt;     // [F]
  uint32_t *off;     // [F]
  uint32_t *wave;    // [16]
  void *val;         // [TILE] of OutT
  uint16_t *dig;     // [TILE]
};

template <typename OutT>
__device__ __forceinline__ ScatterLds carveScatterLds(unsigned char *smem, uint32_t F) {
  ScatterLds l;
  l.cursor = reinterpret_cast<uint64_t *>(smem);
  l.cnt = reinterpret_cast<uint32_t *>(l.cursor + F);
  l.off = l.cnt + F;
  l.wave = l.off + F;
  l.val = reinterpret_cast<void *>(l.wave + 16);
  l.dig = reinterpret_cast<uint16_t *>(reinterpret_cast<OutT *>(l.val) + PART_TILE);
  return l;
}

// Scatter [begin, end) of `in` into `out` at the cursors held in l.cursor
// (initialised by the caller, advanced here).  DigitFn(InT) -> digit,
// PackFn(InT) -> OutT.
template <typename InT, typename OutT, typename DigitFn, typename PackFn>
__device__ __forceinline__ void scatterRange(const InT *__restrict__ in, uint64_t begin, uint64_t end, uint32_t F,
                                             const ScatterLds &l, OutT *__restrict__ out, DigitFn digitOf,
                                             PackFn pack) {
  OutT *sVal = reinterpret_cast<OutT *>(l.val);
  const uint32_t t = threadIdx.x;
  for (uint64_t base = begin; base < end; base += PART_TILE) {
    const uint32_t cnt = (uint32_t)min((uint64_t)PART_TILE, end - base);
    InT v[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = i * NT + t;
      if (idx < cnt) v[i] = Loader<InT>::load(in + base + idx);
    }
    uint32_t dr[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = i * NT + t;
      if (idx < cnt) {
        const uint32_t d = digitOf(v[i]);
        const uint32_t r = atomicAdd(&l.cnt[d], 1u);
        dr[i] = (d << 16) | r;
      }
    }
    __syncthreads();
    blockExclusiveScanLds<NT, uint32_t, uint32_t>(l.cnt, l.off, (int)F, l.wave);
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = i * NT + t;
      if (idx < cnt) {
        const uint32_t d = dr[i] >> 16;
        const uint32_t pos = l.off[d] + (dr[i] & 0xFFFFu);
        sVal[pos] = pack(v[i]);
        l.dig[pos] = (uint16_t)d;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = i * NT + t;
      if (idx < cnt) {
        const uint32_t d = l.dig[idx];
        out[l.cursor[d] + (idx - l.off[d])] = sVal[idx];
      }
    }
    __syncthreads();
    for (uint32_t d = t; d < F; d += NT) {
      l.cursor[d] += l.cnt[d];
      l.cnt[d] = 0;
    }
    __syncthreads();
  }
}

template <bool WIDE>
__global__ __launch_bounds__(NT) void netScatterKernel(const ulonglong2 *__restrict__ in, uint64_t n, uint32_t tpb,
                                                       uint32_t bits, uint32_t keyShift, uint32_t totalBlocks,
                                                       uint32_t blockBegin, const uint64_t *__restrict__ cursors,
                                                       void *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using OutT = typename std::conditional<WIDE, ulonglong2, uint64_t>::type;
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  const uint32_t blk = blockBegin + blockIdx.x;
  ScatterLds l = carveScatterLds<OutT>(smem, F);
  for (uint32_t d = threadIdx.x; d < F; d += NT) {
    l.cursor[d] = cursors[(uint64_t)d * totalBlocks + blk];
    l.cnt[d] = 0;
  }
  __syncthreads();
  const uint64_t begin = (uint64_t)blk * tpb * PART_TILE;
  const uint64_t end = min(n, begin + (uint64_t)tpb * PART_TILE);
  auto digitOf = [mask](const ulonglong2 &x) -> uint32_t { return (uint32_t)(x.x & mask); };
  if constexpr (WIDE) {
    auto pack = [](const ulonglong2 &x) -> ulonglong2 { return x; };
    scatterRange<ulonglong2, ulonglong2>(in, begin, end, F, l, reinterpret_cast<ulonglong2 *>(out), digitOf, pack);
  } else {
    auto pack = [bits, keyShift](const ulonglong2 &x) -> uint64_t { return x.y | ((x.x >> bits) << keyShift); };
    scatterRange<ulonglong2, uint64_t>(in, begin, end, F, l, reinterpret_cast<uint64_t *>(out), digitOf, pack);
  }
}

void netScatter(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift, const PartitionGeometry &g,
                uint32_t blockBegin, uint32_t blockEnd, const uint64_t *cursors, uint64_t *out, hipStream_t s) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatter: bits=%u out of range", bits);
  HJ_CHECK(blockBegin <= blockEnd && blockEnd <= g.blocks, "netScatter: block range [%u,%u) of %u", blockBegin,
           blockEnd, g.blocks);
  if (n == 0 || blockEnd == blockBegin) return;
  const size_t lds = netScatterLdsBytes(bits, false);
  hipLaunchKernelGGL(netScatterKernel<false>, dim3(blockEnd - blockBegin), dim3(NT), lds, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock, bits, keyShift, g.blocks,
                     blockBegin, cursors, (void *)out);
  HIP_CHECK_LAUNCH();
}

void netScatterWide(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                    uint32_t blockBegin, uint32_t blockEnd, const uint64_t *cursors, data::Tuple *out,
                    hipStream_t s) {
  HJ_CHECK(bits >= 1 && bits <= MAX_PART_BITS, "netScatterWide: bits=%u out of range", bits);
  HJ_CHECK(blockBegin <= blockEnd && blockEnd <= g.blocks, "netScatterWide: block range [%u,%u) of %u",
           blockBegin, blockEnd, g.blocks);
  if (n == 0 || blockEnd == blockBegin) return;
  const size_t lds = netScatterLdsBytes(bits, true);
  hipLaunchKernelGGL(netScatterKernel<true>, dim3(blockEnd - blockBegin), dim3(NT), lds, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, g.tilesPerBlock, bits, 0u, g.blocks, blockBegin,
                     cursors, (void *)out);
  HIP_CHECK_LAUNCH();
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
template <bool WIDE>
__device__ __forceinline__ uint64_t localWord(const void *in, uint64_t i) {
  if constexpr (WIDE)
    return reinterpret_cast<const ulonglong2 *>(in)[i].x;
  else
    return reinterpret_cast<const uint64_t *>(in)[i];
}

template <bool WIDE>
__global__ __launch_bounds__(NT) void localHistogramKernel(const void *__restrict__ in,
                                                           const LocalItem *__restrict__ items, uint32_t shift,
                                                           uint32_t bits, uint32_t *__restrict__ itemHist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hsh[];
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  const int wid = threadIdx.x / WAVE;
  for (uint32_t i = threadIdx.x; i < 4 * F; i += NT) hsh[i] = 0;
  __syncthreads();
  const LocalItem it = items[blockIdx.x];
  uint32_t *wh = hsh + wid * F;
  for (uint32_t base = 0; base < it.len; base += PART_TILE) {
    uint64_t w[PART_ITEMS];
#pragma unroll
    for (int i = 0; i < (int)PART_ITEMS; ++i) {
      const uint32_t idx = base + i * NT + threadIdx.x;
      w[i] = idx < it.len ? localWord<WIDE>(in, it.begin + idx) : 0;
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

void localHistogram(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift,
                    uint32_t bits, uint32_t *itemHist, hipStream_t s) {
  HJ_CHECK(bits <= MAX_PART_BITS, "localHistogram: bits=%u out of range", bits);
  if (nItems == 0) return;
  const size_t lds = size_t(4) << bits << 2;
  if (wide)
    hipLaunchKernelGGL(localHistogramKernel<true>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits, itemHist);
  else
    hipLaunchKernelGGL(localHistogramKernel<false>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits, itemHist);
  HIP_CHECK_LAUNCH();
}

// One workgroup per owned partition lp: turns the [item][F] histograms of its
// items into per-item cursors (sub-partition major) and the final partition
// begin offsets partBegin[lp*F + q].
__global__ __launch_bounds__(NT) void localCursorsKernel(const uint32_t *__restrict__ itemHist,
                                                         const uint32_t *__restrict__ lpItemBegin, uint32_t owned,
                                                         uint32_t bits, const uint64_t *__restrict__ lpBase,
                                                         uint64_t *__restrict__ itemCursors,
                                                         uint64_t *__restrict__ partBegin) {
  extern __shared__ __attribute__((aligned(16))) uint64_t csh[];
  const uint32_t F = 1u << bits;
  uint64_t *tot = csh;           // [F]
  uint64_t *wt = csh + F;        // [NT/64]
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
    for (uint32_t it = ib; it < ie; ++it) {
      itemCursors[(uint64_t)it * F + q] = run;
      run += itemHist[(uint64_t)it * F + q];
    }
  }
  if (lp == owned - 1 && threadIdx.x == 0) partBegin[(uint64_t)owned * F] = lpBase[owned];
}

void localCursors(const uint32_t *itemHist, const uint32_t *lpItemBegin, uint32_t owned, uint32_t bits,
                  const uint64_t *lpBase, uint64_t *itemCursors, uint64_t *partBegin, hipStream_t s) {
  if (owned == 0) return;
  const size_t lds = (size_t(1) << bits) * 8 + 64;
  hipLaunchKernelGGL(localCursorsKernel, dim3(owned), dim3(NT), lds, s, itemHist, lpItemBegin, owned, bits, lpBase,
                     itemCursors, partBegin);
  HIP_CHECK_LAUNCH();
}

template <bool WIDE>
__global__ __launch_bounds__(NT) void localScatterKernel(const void *__restrict__ in,
                                                         const LocalItem *__restrict__ items, uint32_t shift,
                                                         uint32_t bits, const uint64_t *__restrict__ itemCursors,
                                                         void *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using T = typename std::conditional<WIDE, ulonglong2, uint64_t>::type;
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  ScatterLds l = carveScatterLds<T>(smem, F);
  for (uint32_t d = threadIdx.x; d < F; d += NT) {
    l.cursor[d] = itemCursors[(uint64_t)blockIdx.x * F + d];
    l.cnt[d] = 0;
  }
  __syncthreads();
  const LocalItem it = items[blockIdx.x];
  const T *src = reinterpret_cast<const T *>(in);
  auto pack = [](const T &x) -> T { return x; };
  if constexpr (WIDE) {
    auto digitOf = [shift, mask](const ulonglong2 &x) -> uint32_t { return (uint32_t)((x.x >> shift) & mask); };
    scatterRange<T, T>(src, it.begin, it.begin + it.len, F, l, reinterpret_cast<T *>(out), digitOf, pack);
  } else {
    auto digitOf = [shift, mask](const uint64_t &x) -> uint32_t { return (uint32_t)((x >> shift) & mask); };
    scatterRange<T, T>(src, it.begin, it.begin + it.len, F, l, reinterpret_cast<T *>(out), digitOf, pack);
  }
}

void localScatter(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift, uint32_t bits,
                  const uint64_t *itemCursors, void *out, hipStream_t s) {
  HJ_CHECK(bits <= MAX_PART_BITS, "localScatter: bits=%u out of range", bits);
  if (nItems == 0) return;
  const size_t lds = scatterLds(1u << bits, wide ? 16 : 8);
  if (wide)
    hipLaunchKernelGGL(localScatterKernel<true>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits,
                       itemCursors, out);
  else
    hipLaunchKernelGGL(localScatterKernel<false>, dim3(nItems), dim3(NT), lds, s, in, items, shift, bits,
                       itemCursors, out);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
