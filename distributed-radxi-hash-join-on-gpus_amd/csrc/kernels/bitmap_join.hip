// Single-level counting join for unique inner keys: one LDS bitmap per network
// partition.
//
// After the network pass every partition holds the key fragments above the
// network digit.  With dense keys the fragment range of one partition is
// 2^(keyBits - networkBits); when that fits an LDS bitmap (<= 2^20 bits =
// 128 KiB) the partition is joined in place, as the reference's default
// single-level plan does (core/Configuration.h:28 ENABLE_TWO_LEVEL_PARTITIONING
// = false; build/probe per network partition, tasks/BuildProbe.cpp:47-121),
// without the second radix pass.  Build: atomicOr of the fragment's bit; a bit
// that was already set is a duplicate inner key, which a bitmap cannot count
// -- the kernel raises BM_FLAG_DUP and the caller redoes the join on the
// two-level pass.  Probe: one LDS bit test per outer tuple.
//
// Three launch shapes (kernels.h):
//   bitmapJoin   build + probe of partition d in one workgroup (one rank)
//   bitmapBuild  the partition's bitmap is written to HBM (replicated plan:
//                every rank's bitmaps are summed by an RCCL all-reduce)
//   bitmapProbe  the (all-reduced) bitmap is loaded into LDS, its bits are
//                counted (cross-rank duplicate check), the outer side probed
// Elements are u32 key fragments of the count-only network pass (claim
// slices of a sampled pass, read as 16-byte vectors: slices start on 16-
// element boundaries) or 8-byte CompressedTuples (value >> keyShift) of an
// exchanged window (host-built segment table).
#include "kernels.h"
#include "device_common.h"

#include <algorithm>
#include <cstdlib>

namespace hpcjoin {
namespace kernels {

// 16-byte loads in flight per lane.  (HPCJOIN_BM_U=8 was a sweep variant:
// 2.71 -> 2.66 ms on the pre-pipelined kernel; with the pipelined walks it
// needs 128 VGPRs and spills, so only 4 is built.)
constexpr int BM_U = 4;

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

// Claim slices [CLAIM_GROUPS][F] of a sampled network pass: slice (g, d) is
// [start, min(cur, end)); cur > end means it overflowed (flagged, the caller
// redoes the join with exact slices).
template <typename CurT>
struct ClaimSrc {
  const CurT *start, *cur, *end;
  uint32_t F;
  const uint32_t *roundMeta;  // BitmapSlices::roundMeta
  __device__ __forceinline__ uint32_t groups() const { return CLAIM_GROUPS; }
  // Slot map of the fragment window (RoundMap), decided by the layout kernel.
  __device__ __forceinline__ RoundMap roundMap() const {
    RoundMap m;
    if (roundMeta) {
      m.lp = roundMeta[0];
      m.lv = roundMeta[1];
      m.lns = roundMeta[2];
    }
    return m;
  }
  __device__ __forceinline__ void get(uint32_t d, uint32_t g, uint64_t &b, uint64_t &len, uint32_t &flags) const {
    const size_t i = (size_t)g * F + d;
    const uint64_t s0 = start[i], c = cur[i], e = end[i];
    if (c > e) flags |= BM_FLAG_OVERFLOW;
    b = s0;
    len = (c < e ? c : e) - s0;
  }
};

// Host-built segment table [F][groups] (exchanged windows: one segment per
// (source rank, exchange chunk) of every owned partition).
struct TableSrc {
  const uint64_t *start;
  const uint64_t *len;
  uint32_t G;
  __device__ __forceinline__ uint32_t groups() const { return G; }
  __device__ __forceinline__ RoundMap roundMap() const { return RoundMap(); }
  __device__ __forceinline__ void get(uint32_t d, uint32_t g, uint64_t &b, uint64_t &n, uint32_t &) const {
    const size_t i = (size_t)d * G + g;
    b = start[i];
    n = len[i];
  }
};

// fn(fragment) for every element of src[0, len): 8-byte CompressedTuples of an
// exchanged window (value >> shift), NTH threads x 2U loads per batch.
template <int NTH, int U, typename Fn>
__device__ __forceinline__ void visitSlice64(const uint64_t *__restrict__ src, uint64_t len, uint32_t shift, Fn &&fn) {
  const uint32_t t = threadIdx.x;
  constexpr int U8 = 2 * U;
  for (uint64_t i0 = 0; i0 < len; i0 += (uint64_t)NTH * U8) {
    uint64_t x[U8];
#pragma unroll
    for (int k = 0; k < U8; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < len) x[k] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int k = 0; k < U8; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < len) fn(x[k] >> shift);  // only lanes holding an element (no padding values)
    }
  }
}

// fn(fragment) for every u32 fragment of src[0, len): 16-byte vector loads,
// software-pipelined -- batch k+1 is in flight while batch k is consumed.
// The walk of long slices (N = 1 at 1B: 1.40 ms for the join kernel vs 1.49
// with the flat walk below, whose address select costs more than the two
// latencies per slice start it saves when slices are long).
// src[b, b + len) in logical positions (b a multiple of 4), at rm's slots.
template <int NTH, int U, typename Fn>
__device__ __forceinline__ void visitSlice32(const uint32_t *__restrict__ src, uint64_t b, uint64_t len,
                                             const RoundMap &rm, Fn &&fn) {
  const uint32_t t = threadIdx.x;
  const uint64_t nv = len >> 2;
  constexpr uint64_t STEP = (uint64_t)NTH * U;
  u32x4 cur[U], nxt[U];
  auto load = [&](u32x4(&x)[U], uint64_t i0) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < nv) x[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + rm(b + (i << 2))));
    }
  };
  if (nv) load(cur, 0);
  for (uint64_t i0 = 0; i0 < nv; i0 += STEP) {
    if (i0 + STEP < nv) load(nxt, i0 + STEP);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < nv) {
        fn((uint64_t)cur[k].x);
        fn((uint64_t)cur[k].y);
        fn((uint64_t)cur[k].z);
        fn((uint64_t)cur[k].w);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) cur[k] = nxt[k];
  }
  const uint32_t rem = (uint32_t)(len & 3);
  if (t < rem) fn((uint64_t)src[rm(b + (nv << 2) + t)]);
}

// fn(fragment) for every u32 fragment of partition d: its
// CLAIM_GROUPS claim slices walked as ONE stream of 16-byte vectors (slices
// start on 16-element boundaries).  The slice table is read once per
// workgroup (one round trip) and kept in scalar registers; batch k+1 is in
// flight while batch k is consumed, across slice boundaries.  Walking the
// slices one after another instead drains the pipeline at each of the 2 x 8
// slice starts (a table read plus a first load: two HBM latencies each),
// which dominates when slices are short (one N = 8 rank's share of 1B keys:
// 15K fragments per slice, one batch).  Each slice's last len % 4 elements
// are visited at the end.
template <int NTH, int U, class Src, typename Fn>
__device__ __forceinline__ void visitClaim(const uint32_t *__restrict__ src, const Src &cs, uint32_t d, uint32_t &flags,
                                           Fn &&fn) {
  constexpr uint32_t G = CLAIM_GROUPS;
  __shared__ uint64_t sBase[G], sLen[G], sPre[G], sAdj[G];
  const uint32_t t = threadIdx.x;
  __syncthreads();  // an earlier walk's readers of the slice table are done
  if (t < G) {
    uint64_t b, len;
    cs.get(d, t, b, len, flags);
    sBase[t] = b;
    sLen[t] = len;
  }
  __syncthreads();
  // Vector index i of the stream lies in slice g = max{g : pre[g] <= i}; its
  // address is v + i + adj[g], adj[g] = base[g] / 4 - pre[g] (mod 2^64),
  // accumulated as adj[0] + sum over the passed slice starts of adj[j] -
  // adj[j-1].  Prefixes and deltas are workgroup-uniform (scalar registers):
  // no LDS read on the load's address path.
  if (t < G) {
    uint64_t pre = 0;
    for (uint32_t j = 0; j < t; ++j) pre += sLen[j] >> 2;
    sPre[t] = pre;
    sAdj[t] = (sBase[t] >> 2) - pre;
  }
  __syncthreads();
  const RoundMap rm = cs.roundMap();  // vector i of the stream: slot rm(4 (i + a)) / 4
  static_assert(G == 8, "visitClaim: the slice map is written out for 8 XCD groups");
  const uint64_t p1 = uniform64(sPre[1]), p2 = uniform64(sPre[2]), p3 = uniform64(sPre[3]),
                 p4 = uniform64(sPre[4]), p5 = uniform64(sPre[5]), p6 = uniform64(sPre[6]),
                 p7 = uniform64(sPre[7]);
  const uint64_t total = p7 + (uniform64(sLen[7]) >> 2);
  const uint64_t a0 = uniform64(sAdj[0]), d1 = uniform64(sAdj[1] - sAdj[0]), d2 = uniform64(sAdj[2] - sAdj[1]),
                 d3 = uniform64(sAdj[3] - sAdj[2]), d4 = uniform64(sAdj[4] - sAdj[3]),
                 d5 = uniform64(sAdj[5] - sAdj[4]), d6 = uniform64(sAdj[6] - sAdj[5]),
                 d7 = uniform64(sAdj[7] - sAdj[6]);
  const u32x4 *v = reinterpret_cast<const u32x4 *>(src);
  auto at = [&](uint64_t i) {
    uint64_t a = a0;
    a += i >= p1 ? d1 : 0;
    a += i >= p2 ? d2 : 0;
    a += i >= p3 ? d3 : 0;
    a += i >= p4 ? d4 : 0;
    a += i >= p5 ? d5 : 0;
    a += i >= p6 ? d6 : 0;
    a += i >= p7 ? d7 : 0;
    return v + (rm((i + a) << 2) >> 2);
  };
  constexpr uint64_t STEP = (uint64_t)NTH * U;
  u32x4 cur[U], nxt[U];
  auto load = [&](u32x4(&x)[U], uint64_t i0) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < total) x[k] = __builtin_nontemporal_load(at(i));
    }
  };
  if (total) load(cur, 0);
  for (uint64_t i0 = 0; i0 < total; i0 += STEP) {
    if (i0 + STEP < total) load(nxt, i0 + STEP);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = i0 + (uint64_t)k * NTH + t;
      if (i < total) {
        fn((uint64_t)cur[k].x);
        fn((uint64_t)cur[k].y);
        fn((uint64_t)cur[k].z);
        fn((uint64_t)cur[k].w);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) cur[k] = nxt[k];
  }
  if (t < 4 * G) {
    const uint32_t g = t >> 2, j = t & 3;
    const uint64_t len = sLen[g];
    if (j < (uint32_t)(len & 3)) fn((uint64_t)src[rm(sBase[g] + (len & ~3ull) + j)]);
  }
}

// Every element of partition d of one side.  u32 fragments: one
// flat walk over all claim slices (flat != 0: short partitions) or one
// pipelined walk per slice (long partitions).
template <int NTH, typename E, int U, class Src, typename Fn>
__device__ __forceinline__ void visitPartition(const E *__restrict__ src, const Src &ss, uint32_t d, uint32_t shift,
                                               uint32_t flat, uint32_t &flags, Fn &&fn) {
  if constexpr (sizeof(E) == 4) {
    if (flat) {
      visitClaim<NTH, U>(src, ss, d, flags, fn);
      return;
    }
    const RoundMap rm = ss.roundMap();
    for (uint32_t g = 0; g < ss.groups(); ++g) {
      uint64_t b, len;
      ss.get(d, g, b, len, flags);
      visitSlice32<NTH, U>(src, b, len, rm, fn);
    }
  } else {
    for (uint32_t g = 0; g < ss.groups(); ++g) {
      uint64_t b, len;
      ss.get(d, g, b, len, flags);
      visitSlice64<NTH, U>(src + b, len, shift, fn);
    }
  }
}

// Build: fire-and-forget LDS ORs (no returned value to wait for); a repeated
// fragment is found afterwards as fewer set bits than inserted fragments
// (bmCheckDup).  Returns this thread's inserted count.
template <int NTH, typename E, int U, class Src>
// This workgroup's bitmap covers fragments [base, base + limit) of the
// partition's range [0, limit << split).
__device__ __forceinline__ uint64_t bmBuild(uint32_t *bm, const E *__restrict__ r, const Src &rs, uint32_t d,
                                            uint32_t shift, uint32_t flat, uint64_t limit, uint32_t &flags,
                                            uint64_t base = 0, uint32_t split = 0) {
  uint32_t inserted = 0;
  const uint64_t range = limit << split;
  visitPartition<NTH, E, U>(r, rs, d, shift, flat, flags, [&](uint64_t f) {
    const uint64_t g = f - base;
    if (g >= limit) {
      if (f >= range) flags |= BM_FLAG_DUP;  // outside the planned fragment range: the caller falls back
      return;                                // else: another workgroup's piece
    }
    __hip_atomic_fetch_or(&bm[g >> 5], 1u << (g & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    ++inserted;
  });
  return inserted;
}

// After the build's barrier: set bits of the bitmap vs fragments inserted by
// the whole workgroup; fewer bits = a repeated inner key.  Returns the bits.
template <int NTH>
__device__ __forceinline__ uint64_t bmCheckDup(const uint32_t *bm, uint32_t words, uint64_t inserted, uint32_t &flags,
                                               uint64_t *wt) {
  uint64_t bits = 0;
  for (uint32_t w = threadIdx.x; w < words; w += NTH) bits += __popc(bm[w]);
  const uint64_t setBits = blockReduceSum<NTH, uint64_t>(bits, wt);
  const uint64_t total = blockReduceSum<NTH, uint64_t>(inserted, wt);
  if (setBits != total) flags |= BM_FLAG_DUP;
  return setBits;
}

template <int NTH, typename E, int U, class Src>
__device__ __forceinline__ uint64_t bmProbe(const uint32_t *bm, const E *__restrict__ s, const Src &ss, uint32_t d,
                                            uint32_t shift, uint32_t flat, uint64_t limit, uint32_t &flags,
                                            uint64_t base = 0) {
  uint32_t cnt = 0;
  visitPartition<NTH, E, U>(s, ss, d, shift, flat, flags, [&](uint64_t f) {
    const uint64_t g = f - base;
    if (g < limit) cnt += (bm[g >> 5] >> (g & 31)) & 1u;
  });
  return cnt;
}

__device__ __forceinline__ void bmFinish(BitmapCounters *out, uint64_t matches, uint64_t bits, uint32_t flags) {
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) {
    matches += __shfl_xor(matches, o);
    bits += __shfl_xor(bits, o);
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    if (matches) atomicAdd(&out->matches, (unsigned long long)matches);
    if (bits) atomicAdd(&out->popcount, (unsigned long long)bits);
  }
  const bool dup = __ballot(flags & BM_FLAG_DUP) != 0, ovf = __ballot(flags & BM_FLAG_OVERFLOW) != 0;
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    if (dup) atomicAdd(&out->dup, 1ull);
    if (ovf) atomicAdd(&out->overflow, 1ull);
  }
}

// Mailbox delivery (MailboxArgs::box set): once every wave of the workgroup
// has added its counters (barrier), one thread counts the workgroup in with
// an agent-scope release; the workgroup that arrives last acquires, so it sees
// every workgroup's sums, copies them into the host-mapped mailbox with
// system-scope stores, publishes seq (release: the sums are visible to the
// host first) and returns the counters and the arrival count to zero for the
// next join.  One fenced atomic per workgroup: a fenced arrival per wave (an
// L2 write-back and invalidate each) made the 1B join kernel 0.64 ms slower.
// Vector stores only.
__device__ __forceinline__ void bmPublish(BitmapCounters *out, const MailboxArgs &mb) {
  __syncthreads();  // every wave's counter atomics are done
  if (threadIdx.x != 0) return;
  const unsigned int prev = __hip_atomic_fetch_add(mb.arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (prev + 1 != gridDim.x) return;
  unsigned long long v[4];
  unsigned long long *src = &out->matches;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long *dst = &mb.box->matches;
#pragma unroll
  for (int i = 0; i < 4; ++i) __hip_atomic_store(dst + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&mb.box->seq, mb.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
  for (int i = 0; i < 4; ++i) __hip_atomic_store(src + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(mb.arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename E, int U, class Src, int NTH>
__global__ __launch_bounds__(NTH) void bitmapJoinKernel(const E *__restrict__ r, const E *__restrict__ s, Src rs,
                                                        Src ss, uint32_t shift, uint32_t words, uint32_t flat,
                                                        uint32_t split, BitmapCounters *__restrict__ out,
                                                        MailboxArgs mb) {
  extern __shared__ uint32_t bm[];
  __shared__ uint64_t wt[NTH / WAVE];
  for (uint32_t w = threadIdx.x; w < words; w += NTH) bm[w] = 0;
  __syncthreads();
  // Workgroup = (partition d, piece h of its fragment range); split = 0: one piece.
  const uint32_t d = blockIdx.x >> split;
  const uint64_t limit = (uint64_t)words * 32, base = (uint64_t)(blockIdx.x & ((1u << split) - 1)) * limit;
  uint32_t flags = 0;
  const uint64_t inserted = bmBuild<NTH, E, U>(bm, r, rs, d, shift, flat, limit, flags, base, split);
  __syncthreads();
  bmCheckDup<NTH>(bm, words, inserted, flags, wt);
  const uint64_t cnt = bmProbe<NTH, E, U>(bm, s, ss, d, shift, flat, limit, flags, base);
  bmFinish(out, cnt, 0, flags);
  if (mb.box) bmPublish(out, mb);
}

template <typename E, int U, class Src, int NTH>
__global__ __launch_bounds__(NTH) void bitmapBuildKernel(const E *__restrict__ r, Src rs, uint32_t shift,
                                                         uint32_t words, uint32_t flat, uint32_t pieceBase,
                                                         uint32_t split, uint32_t *__restrict__ bitmaps,
                                                         BitmapCounters *__restrict__ out) {
  extern __shared__ uint32_t bm[];
  __shared__ uint64_t wt[NTH / WAVE];
  for (uint32_t w = threadIdx.x; w < words; w += NTH) bm[w] = 0;
  __syncthreads();
  // Piece q = (partition d, h-th 2^-split of its fragment range); pieces of a
  // partition are adjacent in `bitmaps`, so the array is the partitions' full
  // bitmaps in order whatever the split.
  const uint32_t q = pieceBase + blockIdx.x, d = q >> split;
  const uint64_t limit = (uint64_t)words * 32, base = (uint64_t)(q & ((1u << split) - 1)) * limit;
  uint32_t flags = 0;
  const uint64_t inserted = bmBuild<NTH, E, U>(bm, r, rs, d, shift, flat, limit, flags, base, split);
  __syncthreads();
  bmCheckDup<NTH>(bm, words, inserted, flags, wt);
  uint32_t *dst = bitmaps + (size_t)q * words;
  for (uint32_t w = threadIdx.x; w < words; w += NTH) dst[w] = bm[w];
  bmFinish(out, 0, 0, flags);
}

template <typename E, int U, class Src, int NTH>
__global__ __launch_bounds__(NTH) void bitmapProbeKernel(const E *__restrict__ s, Src ss, uint32_t shift,
                                                         uint32_t words, uint32_t flat, uint32_t pieceBase,
                                                         uint32_t split, const uint32_t *__restrict__ bitmaps,
                                                         BitmapCounters *__restrict__ out) {
  extern __shared__ uint32_t bm[];
  const uint32_t q = pieceBase + blockIdx.x, d = q >> split;
  const uint64_t limit = (uint64_t)words * 32, base = (uint64_t)(q & ((1u << split) - 1)) * limit;
  const u32x4 *src = reinterpret_cast<const u32x4 *>(bitmaps + (size_t)q * words);
  uint64_t bits = 0;
  for (uint32_t w = threadIdx.x; w < words / 4; w += NTH) {  // words is a power of two >= 32
    const u32x4 x = __builtin_nontemporal_load(src + w);
    bm[4 * w] = x.x;
    bm[4 * w + 1] = x.y;
    bm[4 * w + 2] = x.z;
    bm[4 * w + 3] = x.w;
    bits += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
  }
  __syncthreads();
  uint32_t flags = 0;
  const uint64_t cnt = bmProbe<NTH, E, U>(bm, s, ss, d, shift, flat, limit, flags, base);
  bmFinish(out, cnt, bits, flags);
}

uint32_t bitmapWords(uint32_t bits) { return bits > 7 ? 1u << (bits - 5) : 4u; }

static void checkBits(uint32_t bits, uint32_t keyShift, uint32_t elemBytes, uint32_t maxSplit = 0) {
  HJ_CHECK(bits <= BITMAP_MAX_BITS + maxSplit, "bitmap join: %u fragment bits exceed the %u-bit LDS bitmap", bits,
           BITMAP_MAX_BITS + maxSplit);
  HJ_CHECK(elemBytes == 4 || elemBytes == 8, "bitmap join: %u-byte elements", elemBytes);
  HJ_CHECK(elemBytes == 8 ? keyShift < 64 : keyShift == 0, "bitmap join: keyShift=%u for %u-byte elements", keyShift,
           elemBytes);
}

// Threads per workgroup: 1024 for the large bitmaps (one workgroup per CU
// holds the LDS; 16 waves keep the loads in flight), 256 when the bitmap is
// at most 32 KiB (bits <= 18: several workgroups per CU, so short partitions
// -- one rank's share at N = 8 -- overlap each other's latencies).
// BitmapSlices::threads = 256|1024 forces one (KernelVariants::bmThreads).
static int bmThreads(uint32_t bits, uint32_t forced) {
  return forced == 256 || forced == 1024 ? (int)forced : bits <= 18 ? 256 : 1024;
}

// Flat walk over a partition's claim slices when the average partition is
// short (< 2^18 elements; BitmapSlices::flat = 0|1 forces it).  Measured 1024-
// thread join kernel: 1B (977K per partition) per-slice 1.40 ms vs flat 1.49;
// 125M (122K per partition) per-slice 0.358 ms vs flat 0.33.
static uint32_t bmFlat(const BitmapSlices &a, const BitmapSlices *b, uint32_t partitions) {
  if (a.flat >= 0) return a.flat ? 1u : 0u;
  const uint64_t n = std::max<uint64_t>(a.count, b ? b->count : 0);
  return n > 0 && n / std::max<uint32_t>(partitions, 1) < (1ull << 18) ? 1u : 0u;
}

// Dispatch on (element, slice source, threads): u32 fragments come with claim
// slices, 8-byte CompressedTuples with a segment table.
#define HJ_BM_NTH(...)           \
  do {                           \
    if (nth == 256) {            \
      constexpr int NTH = 256;   \
      __VA_ARGS__;               \
    } else {                     \
      constexpr int NTH = 1024;  \
      __VA_ARGS__;               \
    }                            \
  } while (0)

#define HJ_BM_DISPATCH(...)                                                                                      \
  do {                                                                                                           \
    const int nth = bmThreads(bits, src.threads);                                                                             \
    if (elemBytes == 4) {                                                                                        \
      HJ_CHECK(src.kind == BitmapSlices::Claim, "bitmap join: u32 fragments need claim slices");                \
      using E = uint32_t;                                                                                        \
      if (src.narrow) {                                                                                          \
        using S = ClaimSrc<uint32_t>;                                                                            \
        constexpr int U = BM_U;                                                                                  \
        HJ_BM_NTH(__VA_ARGS__);                                                                                  \
      } else {                                                                                                   \
        using S = ClaimSrc<unsigned long long>;                                                                  \
        constexpr int U = BM_U;                                                                                  \
        HJ_BM_NTH(__VA_ARGS__);                                                                                     \
      }                                                                                                          \
    } else {                                                                                                     \
      HJ_CHECK(src.kind == BitmapSlices::Table, "bitmap join: 8-byte tuples need a segment table");             \
      using E = uint64_t;                                                                                        \
      using S = TableSrc;                                                                                        \
      constexpr int U = BM_U;                                                                                    \
      HJ_BM_NTH(__VA_ARGS__);                                                                                       \
    }                                                                                                            \
  } while (0)

template <class S>
static S makeSrc(const BitmapSlices &b, uint32_t F);
template <>
ClaimSrc<uint32_t> makeSrc(const BitmapSlices &b, uint32_t F) {
  return ClaimSrc<uint32_t>{static_cast<const uint32_t *>(b.start), static_cast<const uint32_t *>(b.cur),
                            static_cast<const uint32_t *>(b.end), F, b.roundMeta};
}
template <>
ClaimSrc<unsigned long long> makeSrc(const BitmapSlices &b, uint32_t F) {
  return ClaimSrc<unsigned long long>{static_cast<const unsigned long long *>(b.start),
                                      static_cast<const unsigned long long *>(b.cur),
                                      static_cast<const unsigned long long *>(b.end), F, b.roundMeta};
}
template <>
TableSrc makeSrc(const BitmapSlices &b, uint32_t) {
  return TableSrc{b.segStart, b.segLen, b.groups};
}

void bitmapJoin(uint32_t elemBytes, const void *r, const void *s, const BitmapSlices &rsl, const BitmapSlices &ssl,
                uint32_t partitions, uint32_t keyShift, uint32_t bits, BitmapCounters *out, hipStream_t st,
                const MailboxArgs &mb) {
  checkBits(bits, keyShift, elemBytes, BITMAP_MAX_SPLIT);
  HJ_CHECK(rsl.kind == ssl.kind && rsl.narrow == ssl.narrow, "bitmap join: inner and outer slices differ in kind");
  HJ_CHECK(!mb.box || mb.arrivals, "bitmap join: a mailbox needs an arrival counter");
  HJ_CHECK(partitions > 0 || !mb.box, "bitmap join: no partitions to publish a mailbox result");
  if (partitions == 0) return;
  const uint32_t split = bits > BITMAP_MAX_BITS ? bits - BITMAP_MAX_BITS : 0;
  const uint32_t words = bitmapWords(bits - split);
  const uint32_t flat = bmFlat(rsl, &ssl, partitions);
  const BitmapSlices &src = rsl;
  HJ_BM_DISPATCH(hipLaunchKernelGGL((bitmapJoinKernel<E, U, S, NTH>), dim3(partitions << split), dim3(NTH),
                                    (size_t)words * 4, st,
                                    static_cast<const E *>(r), static_cast<const E *>(s), makeSrc<S>(rsl, partitions),
                                    makeSrc<S>(ssl, partitions), keyShift, words, flat, split, out, mb));
  HIP_CHECK_LAUNCH();
}

void bitmapBuild(uint32_t elemBytes, const void *r, const BitmapSlices &src, uint32_t partitions, uint32_t keyShift,
                 uint32_t bits, uint32_t *bitmaps, BitmapCounters *out, hipStream_t st, uint32_t first,
                 uint32_t count) {
  checkBits(bits, keyShift, elemBytes, BITMAP_MAX_SPLIT);
  if (count == UINT32_MAX) count = partitions - std::min(first, partitions);
  HJ_CHECK(first <= partitions && count <= partitions - first, "bitmapBuild: partitions [%u, +%u) of %u", first, count,
           partitions);
  if (partitions == 0 || count == 0) return;
  const uint32_t split = bits > BITMAP_MAX_BITS ? bits - BITMAP_MAX_BITS : 0;
  const uint32_t words = bitmapWords(bits - split);
  const uint32_t flat = bmFlat(src, nullptr, partitions);
  HJ_BM_DISPATCH(hipLaunchKernelGGL((bitmapBuildKernel<E, U, S, NTH>), dim3(count << split), dim3(NTH),
                                    (size_t)words * 4, st, static_cast<const E *>(r), makeSrc<S>(src, partitions),
                                    keyShift, words, flat, first << split, split, bitmaps, out));
  HIP_CHECK_LAUNCH();
}

void bitmapProbe(uint32_t elemBytes, const void *s, const BitmapSlices &src, uint32_t partitions, uint32_t keyShift,
                 uint32_t bits, const uint32_t *bitmaps, BitmapCounters *out, hipStream_t st, uint32_t first,
                 uint32_t count) {
  checkBits(bits, keyShift, elemBytes, BITMAP_MAX_SPLIT);
  if (count == UINT32_MAX) count = partitions - std::min(first, partitions);
  HJ_CHECK(first <= partitions && count <= partitions - first, "bitmapProbe: partitions [%u, +%u) of %u", first, count,
           partitions);
  if (partitions == 0 || count == 0) return;
  const uint32_t split = bits > BITMAP_MAX_BITS ? bits - BITMAP_MAX_BITS : 0;
  const uint32_t words = bitmapWords(bits - split);
  const uint32_t flat = bmFlat(src, nullptr, partitions);
  HJ_BM_DISPATCH(hipLaunchKernelGGL((bitmapProbeKernel<E, U, S, NTH>), dim3(count << split), dim3(NTH),
                                    (size_t)words * 4, st, static_cast<const E *>(s), makeSrc<S>(src, partitions),
                                    keyShift, words, flat, first << split, split, bitmaps, out));
  HIP_CHECK_LAUNCH();
}
#undef HJ_BM_DISPATCH
#undef HJ_BM_NTH

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadBitmapJoin() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(
      &a, reinterpret_cast<const void *>(&bitmapJoinKernel<uint32_t, BM_U, ClaimSrc<uint32_t>, 1024>)));
}

}  // namespace kernels
}  // namespace hpcjoin
