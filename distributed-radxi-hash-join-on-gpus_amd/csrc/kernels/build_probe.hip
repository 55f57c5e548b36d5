// LDS hash build/probe over (partition, R-chunk, S-chunk) work items.
//
// Replaces the reference's CPU bucket-chained build/probe
// (/root/reference/tasks/BuildProbe.cpp:47-121) and its GPU offload
// (/root/reference/operators/gpu/eth.cu:25-109, which only had 16 buckets per
// partition and a build/probe stride mismatch), plus the
// dormant probe / probe_skew / probe_count / probe_match_rate kernels
// (kernels_optimized.cu:127-848).
//
// MI355X design:
//  * After two radix passes a final partition's inner side fits an LDS open
//    addressing table (load factor <= 0.5, linear probing, LDS CAS inserts).
//  * Skew: a partition whose inner side exceeds rChunk, or whose outer side
//    exceeds sChunk, is expanded into several work items (the
//    skew_detect -> generate_block_mapping idea of kernels_optimized.cu:301-457,
//    without CUDA dynamic parallelism, which HIP does not have).  Items are
//    materialised by a count -> scan -> emit sequence on the device.
//  * Persistent-style grid: a fixed grid (<= 8 WGs/CU) grid-strides over the
//    item list so the LDS table is carved once per workgroup.
//  * Counting: per-lane counters -> wave64 reduction -> one 64-bit global
//    atomic per workgroup.  Materialisation: per-lane register slots, one
//    wave-aggregated reservation per 64 probes (not one atomic per match).
#include "kernels.h"
#include "device_common.h"

#include <cstdlib>
#include <type_traits>

namespace hpcjoin {
namespace kernels {

constexpr int BPT = 256;
constexpr uint32_t EMPTY32 = 0xFFFFFFFFu;
constexpr unsigned long long EMPTY64 = ~0ull;
constexpr int MAT_SLOTS = 2;  // register-held matches per probe before the overflow path

enum BPMode : int { BP_CCOUNT = 0, BP_CMAT = 1, BP_WCOUNT = 2, BP_WMAT = 3 };

static int bpMode(const BPArgs &a) {
  return (a.wide ? 2 : 0) + (a.materialize ? 1 : 0);
}

static size_t bpEntryBytes(int mode) {
  switch (mode) {
    case BP_CCOUNT: return 4;
    case BP_CMAT: return 8;
    case BP_WCOUNT: return 8;
    default: return 16;
  }
}

// Direct-addressed counting: a final partition's fragments span at most
// 2^fragBits values, so with fragBits <= 13 (8192 x 4 B = 32 KiB, the hash
// table's own budget) counts[fragment] replaces hashing: one LDS atomic add
// per inner tuple, one LDS read per outer tuple, no probe chains, duplicates
// on either side counted exactly.  1B unique keys after 9 + 9 radix bits
// leave 12 fragment bits.
constexpr uint32_t BP_DIRECT_MAX_BITS = 13;
static bool bpDirect(const BPArgs &a) {
  return bpMode(a) == BP_CCOUNT && a.fragBits > 0 && a.fragBits <= BP_DIRECT_MAX_BITS;
}

bool bpDirectSplit(const BPArgs &a) { return bpDirect(a) && a.split && !a.itemCounts; }

size_t bpLdsBytes(const BPArgs &a) {
  if (bpDirect(a)) return (size_t(4) << a.fragBits) + 64;
  const uint64_t slots = uint64_t(1) << ceilLog2(2ull * a.rChunk);
  return slots * bpEntryBytes(bpMode(a)) + 64;
}

__device__ __forceinline__ uint32_t hash32(uint32_t frag, uint32_t tbits) {
  return (frag * 2654435761u) >> (32 - tbits);
}
__device__ __forceinline__ uint32_t hash64(uint64_t key, uint32_t tbits) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tbits));
}

// dedupParts (optional, key-only words with repeated keys): partitions with
// more than rChunk inner tuples are listed there (appended at *dedupCount)
// for bpKeyDedup, which compacts them and emits their spans itself; those of
// more than BP_DEDUP_SEG_MIN are also listed in dedupBig (their later
// segments get workgroups of their own).
// heavySpans (optional): partitions with more than heavyMin inner tuples
// (rChunk: more than one table; 0 once repeated keys were seen) get no work
// items here; their spans go to heavySpans instead (appended at *heavyCount,
// at most heavyCapacity written) for bpKeyCountedSpans.
__global__ __launch_bounds__(BPT) void bpPlanCountsKernel(const uint64_t *__restrict__ partR,
                                                          const uint64_t *__restrict__ partS,
                                                          const uint64_t *__restrict__ partREnd,
                                                          const uint64_t *__restrict__ partSEnd, uint32_t P, uint32_t rc,
                                                          uint32_t sc, uint32_t *counts, BPSpan *__restrict__ heavySpans,
                                                          uint32_t *__restrict__ heavyCount, uint32_t heavyCapacity,
                                                          uint32_t heavyMin, uint32_t *__restrict__ dedupParts,
                                                          uint32_t *__restrict__ dedupCount,
                                                          uint32_t *__restrict__ dedupBig,
                                                          uint32_t *__restrict__ dedupBigCount) {
  const uint32_t p = blockIdx.x * BPT + threadIdx.x;
  if (p >= P) return;
  const uint64_t nr = partREnd[p] - partR[p], ns = partSEnd[p] - partS[p];
  const uint32_t c = (nr == 0 || ns == 0) ? 0u : (uint32_t)(ceilDiv(nr, rc) * ceilDiv(ns, sc));
  if (dedupParts && nr > rc && c) {  // more than one inner chunk: compacted first (bpKeyDedup), spans after
    dedupParts[atomicAdd(dedupCount, 1u)] = p;
    if (nr > BP_DEDUP_SEG_MIN) dedupBig[atomicAdd(dedupBigCount, 1u)] = p;
    counts[p] = 0;
    return;
  }
  if (heavySpans && nr > heavyMin && c) {
    const uint32_t nsChunks = (uint32_t)ceilDiv(ns, sc);
    const uint32_t o = atomicAdd(heavyCount, c);
    for (uint32_t i = 0; i < c && o + i < heavyCapacity; ++i) {
      BPSpan sp;
      sp.rb = partR[p] + (uint64_t)(i / nsChunks) * rc;
      sp.sb = partS[p] + (uint64_t)(i % nsChunks) * sc;
      sp.nr = (uint32_t)(min(nr - (uint64_t)(i / nsChunks) * rc, (uint64_t)rc));
      sp.ns = (uint32_t)(min(ns - (uint64_t)(i % nsChunks) * sc, (uint64_t)sc));
      sp.flags = sp.pad1 = 0;
      heavySpans[o + i] = sp;
    }
    counts[p] = 0;
    return;
  }
  counts[p] = c;
}

void bpPlanCounts(const BPArgs &a, uint32_t *counts, hipStream_t s) {
  if (a.P == 0) return;
  HJ_CHECK(!a.heavySpans || a.heavyCount, "bpPlanCounts: heavy spans without their counter");
  HJ_CHECK(!a.dedupParts || (a.dedupBig && a.dedupBigCount), "bpPlanCounts: compaction list without the big list");
  hipLaunchKernelGGL(bpPlanCountsKernel, dim3(ceilDiv(a.P, BPT)), dim3(BPT), 0, s, a.partR, a.partS,
                     a.partREnd ? a.partREnd : a.partR + 1, a.partSEnd ? a.partSEnd : a.partS + 1, a.P, a.rChunk,
                     a.sChunk, counts, a.heavySpans, a.heavyCount, a.heavyCapacity,
                     a.heavyMin, a.dedupParts, a.dedupCount, a.dedupBig, a.dedupBigCount);
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(BPT) void bpEmitKernel(const uint64_t *__restrict__ partS,
                                                    const uint64_t *__restrict__ partSEnd, uint32_t P, uint32_t sc,
                                                    const uint32_t *__restrict__ counts,
                                                    const uint32_t *__restrict__ offsets, BPItem *items,
                                                    uint32_t capacity) {
  const uint32_t p = blockIdx.x * BPT + threadIdx.x;
  if (p >= P) return;
  const uint32_t c = counts[p];
  if (c == 0) return;
  const uint32_t nsChunks = (uint32_t)ceilDiv(partSEnd[p] - partS[p], sc);
  const uint32_t o = offsets[p];
  for (uint32_t i = 0; i < c && o + i < capacity; ++i) {
    BPItem it;
    it.part = p;
    it.rChunk = i / nsChunks;
    it.sChunk = i % nsChunks;
    it.pad = 0;
    items[o + i] = it;
  }
}

void bpEmit(const BPArgs &a, const uint32_t *counts, const uint32_t *offsets, BPItem *items, uint32_t capacity,
            hipStream_t s) {
  if (a.P == 0) return;
  hipLaunchKernelGGL(bpEmitKernel, dim3(ceilDiv(a.P, BPT)), dim3(BPT), 0, s, a.partS,
                     a.partSEnd ? a.partSEnd : a.partS + 1, a.P, a.sChunk, counts, offsets,
                     items, capacity);
  HIP_CHECK_LAUNCH();
}

// Wave-aggregated output reservation: every lane of the (converged) wave calls
// this with its number of register-held matches; returns the lane's slot.
// With item offsets (two-pass materialization) the wave claims from the
// item's LDS cursor; otherwise from the global cursor (single pass).
__device__ __forceinline__ unsigned long long reserveOutput(uint32_t mine, unsigned long long *cursor,
                                                            uint32_t *itemCursor, unsigned long long itemBase) {
  const uint32_t incl = waveInclusiveScan<uint32_t>(mine);
  const uint32_t total = __shfl(incl, WAVE - 1, WAVE);
  unsigned long long base = 0;
  if ((threadIdx.x & (WAVE - 1)) == WAVE - 1 && total)
    base = itemCursor ? itemBase + atomicAdd(itemCursor, total) : atomicAdd(cursor, (unsigned long long)total);
  base = __shfl(base, WAVE - 1, WAVE);
  return base + (incl - mine);
}

__device__ __forceinline__ unsigned long long reserveOne(unsigned long long *cursor, uint32_t *itemCursor,
                                                         unsigned long long itemBase) {
  return itemCursor ? itemBase + atomicAdd(itemCursor, 1u) : atomicAdd(cursor, 1ull);
}

__device__ __forceinline__ void emitPair(const BPArgs &a, unsigned long long pos, uint64_t ridR, uint64_t ridS) {
  if (pos < a.outCapacity) a.outPairs[pos] = make_ulonglong2(ridR, ridS);
}

// Tuples per thread per batch: a whole 4096-tuple inner chunk is loaded with
// one round of independent loads (16 per lane) before any LDS insert, instead
// of one dependent HBM round trip per insert.
constexpr int BP_K = 16;

template <typename V, bool FULL>
__device__ __forceinline__ void bpLoad(const V *__restrict__ src, uint32_t n, uint32_t b0, V (&v)[BP_K]) {
#pragma unroll
  for (int k = 0; k < BP_K; ++k) {
    const uint32_t idx = b0 + k * BPT + threadIdx.x;
    if (FULL || idx < n) v[k] = src[idx];
  }
}

// One batch of an item's side into registers.  Counting keeps only the 32-bit
// key fragment per tuple (half the registers of the 8-byte value, so 16
// loads per lane stay in flight without scratch spills); materializing keeps
// the whole tuple.  Sources: 8-byte / 16-byte tuples, or the local pass's
// split columns (kernels.h, SplitLayout), where counting reads only the
// 2-byte fragment column.
template <int MODE, bool SPLIT, typename L, bool FULL>
__device__ __forceinline__ void bpLoadSide(const void *__restrict__ src, const uint16_t *__restrict__ hi,
                                           uint64_t off, uint32_t n, uint32_t b0, const BPArgs &a, L (&v)[BP_K]) {
#pragma unroll
  for (int k = 0; k < BP_K; ++k) {
    const uint32_t idx = b0 + k * BPT + threadIdx.x;
    if (FULL || idx < n) {
      if constexpr (MODE == BP_CCOUNT) {
        if constexpr (SPLIT)
          v[k] = hi[off + idx];
        else  // fragShift >= keyShift >= 32: the fragment lies in the tuple's high dword
          v[k] = reinterpret_cast<const uint32_t *>(src)[2 * (off + idx) + 1] >> (a.fragShift - 32);
      } else if constexpr (SPLIT) {
        v[k] = (uint64_t)reinterpret_cast<const uint32_t *>(src)[off + idx] | ((uint64_t)hi[off + idx] << a.fragShift);
      } else {
        v[k] = reinterpret_cast<const L *>(src)[off + idx];
      }
    }
  }
}

// Production count kernel of the split layout with direct-addressed tables:
// the fragment column is read as aligned 8-byte words (4 fragments each, one
// 512-byte request per wave instruction instead of 128 bytes), elements
// outside [begin, end) of a word are masked, and only a 32-bit fragment
// array lives in registers.  4 words per lane per batch (4096 fragments per
// workgroup, one final partition's side) keep it at 50 VGPRs, so 8
// workgroups (32 wave64s, 8 x 16 KiB of LDS) share a CU: 0.81 ms per 1B x 1B
// join against 1.04 ms with 8 words per lane at 5 per CU (81 VGPRs).
constexpr int BPD_T = 256;
constexpr int BPD_K = 4;     // words per lane per batch: 4096 fragments per workgroup batch
constexpr int BPD_MINB = 8;  // workgroups per CU

template <int K, bool FULL>
__device__ __forceinline__ void bpdLoad(const uint64_t *__restrict__ w, uint32_t nw, uint32_t b0, uint64_t (&v)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t idx = b0 + k * BPD_T + threadIdx.x;
    if (FULL || idx < nw) v[k] = w[idx];
  }
}

template <int K, int MINB>
__global__ __launch_bounds__(BPD_T, MINB) void bpDirectSplitKernel(BPArgs a, const BPItem *__restrict__ items,
                                                                 const uint32_t *__restrict__ nItemsPtr,
                                                                 uint32_t capacity) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *cnt = reinterpret_cast<uint32_t *>(smem);
  const uint32_t slots = 1u << a.fragBits;
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(smem + ((size_t)slots * 4 + 15) / 16 * 16);
  const uint64_t *R64 = reinterpret_cast<const uint64_t *>(a.Rhi);
  const uint64_t *S64 = reinterpret_cast<const uint64_t *>(a.Shi);
  constexpr uint32_t WB = BPD_T * K;  // words per batch
  const uint32_t t = threadIdx.x;
  const uint32_t nItems = min(*nItemsPtr, capacity);
  uint64_t matches = 0;
  for (uint32_t w = blockIdx.x; w < nItems; w += gridDim.x) {
    const BPItem it = items[w];
    const uint64_t rb = a.partR[it.part] + (uint64_t)it.rChunk * a.rChunk;
    const uint64_t re = min(a.partREnd[it.part], rb + a.rChunk);
    const uint64_t sb = a.partS[it.part] + (uint64_t)it.sChunk * a.sChunk;
    const uint64_t se = min(a.partSEnd[it.part], sb + a.sChunk);
    // Aligned word ranges covering [rb, re) and [sb, se).
    const uint64_t rw0 = rb >> 2, sw0 = sb >> 2;
    const uint32_t rnw = re > rb ? (uint32_t)(((re + 3) >> 2) - rw0) : 0;
    const uint32_t snw = se > sb ? (uint32_t)(((se + 3) >> 2) - sw0) : 0;
    uint64_t rv[K], sv[K];
    if (rnw >= WB) bpdLoad<K, true>(R64 + rw0, rnw, 0, rv);
    else bpdLoad<K, false>(R64 + rw0, rnw, 0, rv);
    if (snw >= WB) bpdLoad<K, true>(S64 + sw0, snw, 0, sv);
    else bpdLoad<K, false>(S64 + sw0, snw, 0, sv);
    for (uint32_t i = t; i < slots; i += BPD_T) cnt[i] = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < rnw; b0 += WB) {
      if (b0) bpdLoad<K, false>(R64 + rw0, rnw, b0, rv);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t idx = b0 + k * BPD_T + t;
        if (idx < rnw) {
          const uint64_t e0 = (rw0 + idx) << 2;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (e0 + j >= rb && e0 + j < re) atomicAdd(&cnt[(uint32_t)(rv[k] >> (16 * j)) & 0xFFFFu], 1u);
        }
      }
    }
    __syncthreads();
    for (uint32_t b0 = 0; b0 < snw; b0 += WB) {
      if (b0) {
        if (b0 + WB <= snw) bpdLoad<K, true>(S64 + sw0, snw, b0, sv);
        else bpdLoad<K, false>(S64 + sw0, snw, b0, sv);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t idx = b0 + k * BPD_T + t;
        if (idx < snw) {
          const uint64_t e0 = (sw0 + idx) << 2;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (e0 + j >= sb && e0 + j < se) matches += cnt[(uint32_t)(sv[k] >> (16 * j)) & 0xFFFFu];
        }
      }
    }
    __syncthreads();  // the next item clears the table
  }
  const unsigned long long total = blockReduceSum<BPD_T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(a.result, total);
}

// Materializing build/probe of the split layout (u32 rid column + u16
// fragment column).  The LDS table is two u32 arrays (fragment, rid) of
// nextpow2(2 * rChunk) slots; with the planner's 2048-tuple inner chunks that
// is 32 KiB, and at 117 VGPRs (no scratch; a 5-per-CU budget spilled 68 B per
// lane) 4 workgroups share a CU (the generic 8-byte-entry kernel held 176
// VGPRs and 64 KiB: 2 per CU).  Per outer batch
// every lane first probes all its tuples (first match + match count per
// tuple), then the wave reserves its output once: per-batch wave scans give
// each (tuple, lane) a slot, one LDS atomic per wave claims the range, and
// every store instruction writes lane-consecutive pairs.  Tuples with more
// than one match walk their chain again to emit the rest.
constexpr int BPM_T = 256;
constexpr int BPM_K = 8;

template <bool FULL, int K>
__device__ __forceinline__ void bpmLoad(const uint32_t *__restrict__ rid, const uint16_t *__restrict__ hi, uint64_t off,
                                        uint32_t n, uint32_t b0, uint32_t (&r)[K], uint32_t (&f)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t idx = b0 + k * BPM_T + threadIdx.x;
    if (FULL || idx < n) {
      r[k] = rid[off + idx];
      f[k] = hi[off + idx];
    }
  }
}

__device__ __forceinline__ void waveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));

// Fused row output (ROWS): a wave's matches of one probe batch occupy output
// rows [base, base + T).  Per window of BPM_LIST (= 128) rows their
// (inner, outer) rid pairs are listed at the head of the wave's 5 KiB LDS
// stage; lane pair (2j, 2j + 1) takes list entries j, j + 32, j + 64, j + 96
// and issues the eight 16-byte half-row loads of their payloads at once
// (inner rows plain: each is re-read ~4x while its work item is hot; outer
// rows, each read once, non-temporal so they do not push the inner rows out
// of L2).  The rows are then assembled 64 at a time in the stage (over the
// consumed list) and written by 5 store instructions of 64 consecutive
// 16-byte pieces (per-lane 80-byte row stores measured 2x slower).  Same
// layout as operators/LateMaterialization, whose separate pass this replaces
// at N = 1: no pair array is written and read back.
constexpr uint32_t BPM_LIST = 128;

__device__ __forceinline__ void bpmLoadRow(const BPArgs &a, const uint2 *list, uint32_t j, uint32_t m, uint32_t half,
                                           uint2 &p, ulonglong2 &va, ulonglong2 &vb) {
  p = list[j < m ? j : 0];
  va = a.rowsA[2 * ((uint64_t)p.x - a.offA) + half];
  const u64x2 v =
      __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a.rowsB + 2 * ((uint64_t)p.y - a.offB) + half));
  vb = make_ulonglong2(v.x, v.y);
}

__device__ __forceinline__ void bpmStageRow(ulonglong2 *stage, uint32_t j, uint32_t mh, uint32_t half, uint2 p,
                                            ulonglong2 va, ulonglong2 vb) {
  if (j < mh) {
    if (half == 0) stage[5 * j] = make_ulonglong2(p.x, p.y);
    stage[5 * j + 1 + half] = va;
    stage[5 * j + 3 + half] = vb;
  }
}

__device__ __forceinline__ void bpmStoreRows(const BPArgs &a, const ulonglong2 *stage, uint32_t mh,
                                             unsigned long long r0, uint32_t lane) {
  ulonglong2 *o = a.outRows + 5 * r0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t q = WAVE * k + lane;
    if (q < 5 * mh && r0 + q / 5 < a.outCapacity) {
      const ulonglong2 v = stage[q];
      const u64x2 vv = {v.x, v.y};
      __builtin_nontemporal_store(vv, reinterpret_cast<u64x2 *>(o + q));
    }
  }
}

__device__ __forceinline__ void bpmGatherRows(const BPArgs &a, ulonglong2 *stage, uint32_t m,
                                              unsigned long long row0, uint32_t lane) {
  const uint32_t half = lane & 1, j0 = lane >> 1;
  const uint2 *list = reinterpret_cast<const uint2 *>(stage);
  uint2 p0, p1, p2, p3;
  ulonglong2 a0, a1, a2, a3, b0, b1, b2, b3;
  bpmLoadRow(a, list, j0, m, half, p0, a0, b0);
  bpmLoadRow(a, list, j0 + 32, m, half, p1, a1, b1);
  bpmLoadRow(a, list, j0 + 64, m, half, p2, a2, b2);
  bpmLoadRow(a, list, j0 + 96, m, half, p3, a3, b3);
  waveSync();  // the list is consumed: the stage is reused for the rows
  const uint32_t m0 = min(64u, m);
  bpmStageRow(stage, j0, m0, half, p0, a0, b0);
  bpmStageRow(stage, j0 + 32, m0, half, p1, a1, b1);
  waveSync();
  bpmStoreRows(a, stage, m0, row0, lane);
  waveSync();
  if (m > 64) {  // wave-uniform
    const uint32_t m1 = m - 64;
    bpmStageRow(stage, j0, m1, half, p2, a2, b2);
    bpmStageRow(stage, j0 + 32, m1, half, p3, a3, b3);
    waveSync();
    bpmStoreRows(a, stage, m1, row0 + 64, lane);
    waveSync();
  }
}

template <bool ROWS>
__global__ __launch_bounds__(BPM_T, ROWS ? 3 : 4) void bpMatSplitKernel(BPArgs a, const BPItem *__restrict__ items,
                                                              const uint32_t *__restrict__ nItemsPtr,
                                                              uint32_t capacity) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ ulonglong2 rowStage[ROWS ? BPM_T / WAVE : 1][ROWS ? 5 * WAVE : 1];
  const uint32_t maxSlots = 1u << ceilLog2(2ull * a.rChunk);
  uint32_t *fragT = reinterpret_cast<uint32_t *>(smem);
  uint32_t *ridT = fragT + maxSlots;
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(ridT + maxSlots);
  __shared__ uint32_t itemCursor;
  const uint32_t *Rr = reinterpret_cast<const uint32_t *>(a.R);
  const uint32_t *Sr = reinterpret_cast<const uint32_t *>(a.S);
  // Rows: 4 outer tuples per thread per batch (the gather state needs the registers).
  constexpr int K = ROWS ? 4 : BPM_K;
  constexpr uint32_t BATCH = BPM_T * K;
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1);
  const bool perItem = a.itemOffsets != nullptr;
  const uint32_t nItems = min(*nItemsPtr, capacity);
  uint64_t matches = 0;
  for (uint32_t w = blockIdx.x; w < nItems; w += gridDim.x) {
    const BPItem it = items[w];
    const uint64_t rb = a.partR[it.part] + (uint64_t)it.rChunk * a.rChunk;
    const uint64_t re = min(a.partREnd[it.part], rb + a.rChunk);
    const uint64_t sb = a.partS[it.part] + (uint64_t)it.sChunk * a.sChunk;
    const uint64_t se = min(a.partSEnd[it.part], sb + a.sChunk);
    const uint32_t nr = (uint32_t)(re - rb), ns = (uint32_t)(se - sb);
    uint32_t tbits = ceilLog2(2ull * nr);
    if (tbits < 6) tbits = 6;
    const uint32_t slots = 1u << tbits, mask = slots - 1;
    const unsigned long long itemBase = perItem ? a.itemOffsets[w] : 0ull;
    uint32_t rr[K], rf[K], sr[K], sf[K];
    if (nr >= BATCH) bpmLoad<true>(Rr, a.Rhi, rb, nr, 0, rr, rf);
    else bpmLoad<false>(Rr, a.Rhi, rb, nr, 0, rr, rf);
    if (ns >= BATCH) bpmLoad<true>(Sr, a.Shi, sb, ns, 0, sr, sf);
    else bpmLoad<false>(Sr, a.Shi, sb, ns, 0, sr, sf);
    for (uint32_t i = t; i < slots; i += BPM_T) fragT[i] = EMPTY32;
    if (t == 0) itemCursor = 0;
    __syncthreads();

    // ---- build
    for (uint32_t b0 = 0; b0 < nr; b0 += BATCH) {
      if (b0) bpmLoad<false>(Rr, a.Rhi, rb, nr, b0, rr, rf);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (b0 + k * BPM_T + t < nr) {
          uint32_t h = hash32(rf[k], tbits);
          while (atomicCAS(&fragT[h], EMPTY32, rf[k]) != EMPTY32) h = (h + 1) & mask;
          ridT[h] = rr[k];
        }
      }
    }
    __syncthreads();

    // ---- probe
    for (uint32_t b0 = 0; b0 < ns; b0 += BATCH) {
      if (b0) {
        if (b0 + BATCH <= ns) bpmLoad<true>(Sr, a.Shi, sb, ns, b0, sr, sf);
        else bpmLoad<false>(Sr, a.Shi, sb, ns, b0, sr, sf);
      }
      const uint32_t kmax = min((uint32_t)K, (uint32_t)ceilDiv(ns - b0, BPM_T));  // block-uniform
      uint32_t found[K], first[K], incl[K];
      uint32_t waveTotal = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        found[k] = 0;
        first[k] = 0;
        incl[k] = 0;
        if ((uint32_t)k >= kmax) continue;
        if (b0 + k * BPM_T + t < ns) {
          const uint32_t frag = sf[k];
          uint32_t h = hash32(frag, tbits), e;
          while ((e = fragT[h]) != EMPTY32) {
            if (e == frag) {
              if (found[k] == 0) first[k] = ridT[h];
              ++found[k];
            }
            h = (h + 1) & mask;
          }
        }
        incl[k] = waveInclusiveScan<uint32_t>(found[k]);
        waveTotal += __shfl(incl[k], WAVE - 1, WAVE);
        matches += found[k];
      }
      unsigned long long base = 0;
      if (lane == WAVE - 1 && waveTotal)
        base = perItem ? itemBase + atomicAdd(&itemCursor, waveTotal)
                       : atomicAdd(a.outCursor, (unsigned long long)waveTotal);
      base = __shfl(base, WAVE - 1, WAVE);
      if constexpr (ROWS) {
        ulonglong2 *stg = rowStage[t / WAVE];
        uint2 *list = reinterpret_cast<uint2 *>(stg);
        for (uint32_t w0 = 0; w0 < waveTotal; w0 += BPM_LIST) {  // wave-uniform; > 1 window only with duplicates
          uint32_t kb = 0;  // rows of columns < k
#pragma unroll
          for (int k = 0; k < K; ++k) {
            if ((uint32_t)k >= kmax) break;
            const uint32_t r0 = kb + incl[k] - found[k];
            if (found[k] && r0 < w0 + BPM_LIST && r0 + found[k] > w0) {
              if (r0 >= w0) list[r0 - w0] = make_uint2(first[k], sr[k]);
              if (found[k] > 1) {  // duplicate inner keys: the chain's other matches
                const uint32_t frag = sf[k];
                uint32_t h = hash32(frag, tbits), e, j = 0;
                while ((e = fragT[h]) != EMPTY32) {
                  if (e == frag) {
                    if (j && r0 + j >= w0 && r0 + j < w0 + BPM_LIST) list[r0 + j - w0] = make_uint2(ridT[h], sr[k]);
                    ++j;
                  }
                  h = (h + 1) & mask;
                }
              }
            }
            kb += __shfl(incl[k], WAVE - 1, WAVE);
          }
          waveSync();
          bpmGatherRows(a, stg, min(BPM_LIST, waveTotal - w0), base + w0, lane);
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if ((uint32_t)k >= kmax) break;
        const unsigned long long pos = base + incl[k] - found[k];
        if (found[k]) emitPair(a, pos, first[k], sr[k]);
        if (found[k] > 1) {  // duplicate inner keys: emit the chain's other matches
          const uint32_t frag = sf[k];
          uint32_t h = hash32(frag, tbits), e, j = 0;
          while ((e = fragT[h]) != EMPTY32) {
            if (e == frag) {
              if (j) emitPair(a, pos + j, ridT[h], sr[k]);
              ++j;
            }
            h = (h + 1) & mask;
          }
        }
        base += __shfl(incl[k], WAVE - 1, WAVE);
      }
    }
    __syncthreads();  // the next item clears the table and the cursor
  }
  const unsigned long long total = blockReduceSum<BPM_T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(a.result, total);
}

// Fused row output with the inner payload rows in LDS (split layout, inner
// chunks of <= BPR_MAX_R tuples).  The build also gathers the chunk's inner
// rows once into LDS (each random 32-byte row costs one 64-byte line fetch;
// re-reading them from L2 per match lost all reuse with ~1500 items in flight:
// the inner side then fetched 37 GB for SF100 instead of 9.6).  Per probe batch
// a wave reserves one contiguous output range, lists its matches (inner index,
// outer rid) in LDS, and writes each window of <= 128 rows in 16-byte pieces
// q = 64 i + lane of the window's 5 m pieces: piece q is field q % 5 of row
// q / 5 -- rid pair and inner halves from LDS, outer halves loaded from
// global memory (non-temporal, each outer row is read once).  All loads of a
// window are issued before its stores, and every store instruction writes
// 1 KiB of contiguous output: no staging buffer, no partial lines inside a
// window.  LDS for 1024-tuple chunks: 52 KiB (3 blocks of 4 waves per CU).
// (Measured and dropped: 512-tuple chunks at 5 blocks per CU, the window in
// two rounds of 5 pieces to fit 96 VGPRs: SF100 build/probe 38.2 vs 28.0 ms.)
constexpr int BPR_T = 256;
constexpr int BPR_K = 2;  // outer tuples per thread per batch: ~128 matches per wave (one window)
constexpr uint32_t BPR_MAX_R = 1024;
constexpr uint32_t BPR_LIST = 128;

static size_t bpMatRowsLds(uint32_t rChunk) {
  const size_t slots = size_t(1) << ceilLog2(2ull * rChunk);
  return (size_t)rChunk * 32 + (BPR_T / WAVE) * BPR_LIST * 8 + slots * 4 + (size_t)rChunk * 4 + slots * 2 + 64;
}

__device__ __forceinline__ void bprEmitWindow(const BPArgs &a, const uint2 *list, const ulonglong2 *rowsL,
                                              const uint32_t *ridL, uint32_t m, unsigned long long row0,
                                              uint32_t lane) {
  const uint32_t P = 5 * m;
  ulonglong2 v0, v1, v2, v3, v4, v5, v6, v7, v8, v9;
#define BPR_FETCH(I, V)                                                                                       \
  {                                                                                                           \
    const uint32_t q = WAVE * (I) + lane;                                                                     \
    if (q < P) {                                                                                              \
      const uint32_t row = q / 5, f = q - 5 * row;                                                            \
      const uint2 e = list[row];                                                                              \
      if (f >= 3) {                                                                                           \
        const u64x2 x = __builtin_nontemporal_load(                                                           \
            reinterpret_cast<const u64x2 *>(a.rowsB + 2 * ((uint64_t)e.y - a.offB) + (f - 3)));               \
        V = make_ulonglong2(x.x, x.y);                                                                        \
      } else if (f == 0) {                                                                                    \
        V = make_ulonglong2(ridL[e.x], e.y);                                                                  \
      } else {                                                                                                \
        V = rowsL[2 * e.x + (f - 1)];                                                                         \
      }                                                                                                       \
    }                                                                                                         \
  }
  BPR_FETCH(0, v0) BPR_FETCH(1, v1) BPR_FETCH(2, v2) BPR_FETCH(3, v3) BPR_FETCH(4, v4)
  BPR_FETCH(5, v5) BPR_FETCH(6, v6) BPR_FETCH(7, v7) BPR_FETCH(8, v8) BPR_FETCH(9, v9)
#undef BPR_FETCH
  ulonglong2 *o = a.outRows + 5 * row0;
  const unsigned long long lim = a.outCapacity > row0 ? 5 * (a.outCapacity - row0) : 0;  // pieces below capacity
#define BPR_STORE(I, V)                                                                                       \
  {                                                                                                           \
    const uint32_t q = WAVE * (I) + lane;                                                                     \
    if (q < P && q < lim) {                                                                                   \
      const u64x2 x = {V.x, V.y};                                                                             \
      __builtin_nontemporal_store(x, reinterpret_cast<u64x2 *>(o + q));                                       \
    }                                                                                                         \
  }
  BPR_STORE(0, v0) BPR_STORE(1, v1) BPR_STORE(2, v2) BPR_STORE(3, v3) BPR_STORE(4, v4)
  BPR_STORE(5, v5) BPR_STORE(6, v6) BPR_STORE(7, v7) BPR_STORE(8, v8) BPR_STORE(9, v9)
#undef BPR_STORE
}

// (HIP launch bounds: the second value is waves per SIMD: 3 blocks of 4 waves per CU.)
__global__ __launch_bounds__(BPR_T, 3) void bpMatRowsKernel(BPArgs a, const BPItem *__restrict__ items,
                                                            const uint32_t *__restrict__ nItemsPtr,
                                                            uint32_t capacity) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t maxSlots = 1u << ceilLog2(2ull * a.rChunk);
  ulonglong2 *rowsL = reinterpret_cast<ulonglong2 *>(smem);                        // [rChunk][2]
  uint2 *lists = reinterpret_cast<uint2 *>(rowsL + 2 * (size_t)a.rChunk);          // [waves][BPR_LIST]
  uint32_t *fragT = reinterpret_cast<uint32_t *>(lists + (BPR_T / WAVE) * BPR_LIST);  // [slots]
  uint32_t *ridL = fragT + maxSlots;                                               // [rChunk]
  uint16_t *idxT = reinterpret_cast<uint16_t *>(ridL + a.rChunk);                  // [slots]
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(
      reinterpret_cast<uintptr_t>(idxT + maxSlots + 3) & ~uintptr_t(7));
  __shared__ uint32_t itemCursor;
  const uint32_t *Rr = reinterpret_cast<const uint32_t *>(a.R);
  const uint32_t *Sr = reinterpret_cast<const uint32_t *>(a.S);
  constexpr uint32_t BATCH = BPR_T * BPR_K;
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1);
  uint2 *list = lists + (t / WAVE) * BPR_LIST;
  const uint32_t nItems = min(*nItemsPtr, capacity);
  uint64_t matches = 0;
  for (uint32_t w = blockIdx.x; w < nItems; w += gridDim.x) {
    const BPItem it = items[w];
    const uint64_t rb = a.partR[it.part] + (uint64_t)it.rChunk * a.rChunk;
    const uint64_t re = min(a.partREnd[it.part], rb + a.rChunk);
    const uint64_t sb = a.partS[it.part] + (uint64_t)it.sChunk * a.sChunk;
    const uint64_t se = min(a.partSEnd[it.part], sb + a.sChunk);
    const uint32_t nr = (uint32_t)(re - rb), ns = (uint32_t)(se - sb);
    uint32_t tbits = ceilLog2(2ull * nr);
    if (tbits < 6) tbits = 6;
    const uint32_t slots = 1u << tbits, mask = slots - 1;
    const unsigned long long itemBase = a.itemOffsets[w];
    uint32_t sr[BPR_K], sf[BPR_K];  // first outer batch: in flight during the build
#pragma unroll
    for (int k = 0; k < BPR_K; ++k) {
      const uint32_t i = k * BPR_T + t;
      sr[k] = i < ns ? Sr[sb + i] : 0u;
      sf[k] = i < ns ? (uint32_t)a.Shi[sb + i] : 0u;
    }
    for (uint32_t i = t; i < slots; i += BPR_T) fragT[i] = EMPTY32;
    if (t == 0) itemCursor = 0;
    __syncthreads();

    // ---- build: table (fragment -> chunk index), rids, then the inner rows
    for (uint32_t i = t; i < nr; i += BPR_T) {
      const uint32_t r = Rr[rb + i], f = a.Rhi[rb + i];
      ridL[i] = r;
      uint32_t h = hash32(f, tbits);
      while (atomicCAS(&fragT[h], EMPTY32, f) != EMPTY32) h = (h + 1) & mask;
      idxT[h] = (uint16_t)i;
    }
    __syncthreads();
    for (uint32_t i0 = t; i0 < 2 * nr; i0 += 4 * BPR_T) {  // 4 independent 16-byte loads per thread
      const uint32_t i1 = i0 + BPR_T, i2 = i0 + 2 * BPR_T, i3 = i0 + 3 * BPR_T;
      ulonglong2 x0, x1, x2, x3;
      x0 = a.rowsA[2 * ((uint64_t)ridL[i0 >> 1] - a.offA) + (i0 & 1)];
      if (i1 < 2 * nr) x1 = a.rowsA[2 * ((uint64_t)ridL[i1 >> 1] - a.offA) + (i1 & 1)];
      if (i2 < 2 * nr) x2 = a.rowsA[2 * ((uint64_t)ridL[i2 >> 1] - a.offA) + (i2 & 1)];
      if (i3 < 2 * nr) x3 = a.rowsA[2 * ((uint64_t)ridL[i3 >> 1] - a.offA) + (i3 & 1)];
      rowsL[i0] = x0;
      if (i1 < 2 * nr) rowsL[i1] = x1;
      if (i2 < 2 * nr) rowsL[i2] = x2;
      if (i3 < 2 * nr) rowsL[i3] = x3;
    }
    __syncthreads();

    // ---- probe + rows (the next batch's outer tuples are loaded while this
    // batch's rows are gathered and written)
    for (uint32_t b0 = 0; b0 < ns; b0 += BATCH) {
      uint32_t found[BPR_K], first[BPR_K], incl[BPR_K];
      uint32_t waveTotal = 0;
#pragma unroll
      for (int k = 0; k < BPR_K; ++k) {
        const uint32_t i = b0 + k * BPR_T + t;
        found[k] = 0;
        first[k] = 0;
        if (i < ns) {
          uint32_t h = hash32(sf[k], tbits), e;
          while ((e = fragT[h]) != EMPTY32) {
            if (e == sf[k]) {
              if (found[k] == 0) first[k] = idxT[h];
              ++found[k];
            }
            h = (h + 1) & mask;
          }
        }
        incl[k] = waveInclusiveScan<uint32_t>(found[k]);
        waveTotal += __shfl(incl[k], WAVE - 1, WAVE);
        matches += found[k];
      }
      uint32_t nsr[BPR_K], nsf[BPR_K];
#pragma unroll
      for (int k = 0; k < BPR_K; ++k) {
        const uint32_t i = b0 + BATCH + k * BPR_T + t;
        nsr[k] = i < ns ? Sr[sb + i] : 0u;
        nsf[k] = i < ns ? (uint32_t)a.Shi[sb + i] : 0u;
      }
      unsigned long long base = 0;
      if (lane == WAVE - 1 && waveTotal) base = itemBase + atomicAdd(&itemCursor, waveTotal);
      base = __shfl(base, WAVE - 1, WAVE);
      for (uint32_t w0 = 0; w0 < waveTotal; w0 += BPR_LIST) {  // wave-uniform; > 1 window only with duplicates
        uint32_t kb = 0;
#pragma unroll
        for (int k = 0; k < BPR_K; ++k) {
          const uint32_t r0 = kb + incl[k] - found[k];
          if (found[k] && r0 < w0 + BPR_LIST && r0 + found[k] > w0) {
            if (r0 >= w0) list[r0 - w0] = make_uint2(first[k], sr[k]);
            if (found[k] > 1) {  // duplicate inner keys: the chain's other matches
              uint32_t h = hash32(sf[k], tbits), e, j = 0;
              while ((e = fragT[h]) != EMPTY32) {
                if (e == sf[k]) {
                  if (j && r0 + j >= w0 && r0 + j < w0 + BPR_LIST) list[r0 + j - w0] = make_uint2(idxT[h], sr[k]);
                  ++j;
                }
                h = (h + 1) & mask;
              }
            }
          }
          kb += __shfl(incl[k], WAVE - 1, WAVE);
        }
        waveSync();
        bprEmitWindow(a, list, rowsL, ridL, min(BPR_LIST, waveTotal - w0), base + w0, lane);
        waveSync();
      }
#pragma unroll
      for (int k = 0; k < BPR_K; ++k) {
        sr[k] = nsr[k];
        sf[k] = nsf[k];
      }
    }
    __syncthreads();  // the next item rebuilds the table, rows and cursor
  }
  const unsigned long long total = blockReduceSum<BPR_T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(a.result, total);
}

static size_t bpMatSplitLds(const BPArgs &a) { return (size_t(8) << ceilLog2(2ull * a.rChunk)) + 64; }

// ITEMS: count pre-pass of a two-pass materialization (per-item match counts);
// a separate instantiation so the count-only production kernel is unchanged.
// Occupancy is LDS-bound: 4-byte count tables (32 KiB) fit 4 workgroups per
// CU, 8-byte tables (64 KiB) only 2 -- so the 8-byte modes get the 256-VGPR
// budget of 2 workgroups per CU instead of spilling to scratch at 128.
// (The per-item count variant keeps 3: its extra reduction would spill at 128.)
template <int MODE, bool ITEMS>
constexpr int bpMinBlocks() { return MODE == 0 ? (ITEMS ? 3 : 4) : 2; }

// Counting modes with a hash table (CCOUNT without direct addressing,
// WCOUNT): the table key and its hash for a register-held element.
template <int MODE, typename L>
__device__ __forceinline__ auto bpKey(const L &v) {
  if constexpr (MODE == BP_CCOUNT) return (uint32_t)v;
  else return (unsigned long long)v.x;  // BP_WCOUNT: ulonglong2 {key, rid}
}
template <int MODE, typename K>
__device__ __forceinline__ uint32_t bpHash(K key, uint32_t tbits) {
  if constexpr (MODE == BP_CCOUNT) return hash32((uint32_t)key, tbits);
  else return hash64((uint64_t)key, tbits);
}

template <int MODE, bool ITEMS = false, bool SPLIT = false, bool DIRECT = false>
__global__ __launch_bounds__(BPT, (bpMinBlocks<MODE, ITEMS>())) void buildProbeKernel(BPArgs a, const BPItem *__restrict__ items,
                                                        const uint32_t *__restrict__ nItemsPtr, uint32_t capacity) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool WIDE = (MODE == BP_WCOUNT || MODE == BP_WMAT);
  constexpr bool MAT = (MODE == BP_CMAT || MODE == BP_WMAT);
  using Entry = typename std::conditional<MODE == BP_CCOUNT, uint32_t, unsigned long long>::type;
  using V = typename std::conditional<WIDE, ulonglong2, uint64_t>::type;
  constexpr uint32_t BATCH = BPT * BP_K;
  const uint64_t maxSlots = DIRECT ? (uint64_t(1) << a.fragBits) : (uint64_t(1) << ceilLog2(2ull * a.rChunk));
  Entry *table = reinterpret_cast<Entry *>(smem);
  unsigned long long *ridTable = reinterpret_cast<unsigned long long *>(smem) + maxSlots;  // WMAT only
  constexpr size_t EB = MODE == BP_CCOUNT ? 4 : (MODE == BP_WMAT ? 16 : 8);
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(smem + maxSlots * EB);
  const uint32_t t = threadIdx.x;
  const uint64_t ridMask = a.keyShift >= 64 ? ~0ull : ((1ull << a.keyShift) - 1);
  static_assert(!(SPLIT && WIDE), "the split layout holds compressed tuples");
  static_assert(!DIRECT || MODE == BP_CCOUNT, "direct-addressed tables count only");
  using L = typename std::conditional<MODE == BP_CCOUNT, uint32_t, V>::type;  // register-held element
  uint64_t matches = 0;
  const uint32_t nItems = min(*nItemsPtr, capacity);
  __shared__ uint32_t itemCursorLds;
  uint32_t *itemCursor = nullptr;
  if constexpr (MAT) itemCursor = a.itemOffsets ? &itemCursorLds : nullptr;

  for (uint32_t w = blockIdx.x; w < nItems; w += gridDim.x) {
    const BPItem it = items[w];
    const uint64_t rb = a.partR[it.part] + (uint64_t)it.rChunk * a.rChunk;
    const uint64_t re = min(a.partREnd[it.part], rb + a.rChunk);
    const uint64_t sb = a.partS[it.part] + (uint64_t)it.sChunk * a.sChunk;
    const uint64_t se = min(a.partSEnd[it.part], sb + a.sChunk);
    const uint32_t nr = (uint32_t)(re - rb), ns = (uint32_t)(se - sb);
    uint32_t tbits = DIRECT ? a.fragBits : ceilLog2(2ull * nr);
    if (!DIRECT && tbits < 6) tbits = 6;
    const uint32_t slots = 1u << tbits, mask = slots - 1;
    unsigned long long itemBase = 0;
    if constexpr (MAT) {
      if (itemCursor) {
        itemBase = a.itemOffsets[w];
        if (t == 0) itemCursorLds = 0;
      }
    }
    const uint64_t matchesBefore = matches;

    // First inner batch and first outer batch are in flight while the table is cleared.
    L rv[BP_K], sv[BP_K];
    if (nr >= BATCH) bpLoadSide<MODE, SPLIT, L, true>(a.R, a.Rhi, rb, nr, 0, a, rv);
    else bpLoadSide<MODE, SPLIT, L, false>(a.R, a.Rhi, rb, nr, 0, a, rv);
    if (ns >= BATCH) bpLoadSide<MODE, SPLIT, L, true>(a.S, a.Shi, sb, ns, 0, a, sv);
    else bpLoadSide<MODE, SPLIT, L, false>(a.S, a.Shi, sb, ns, 0, a, sv);
    for (uint32_t i = t; i < slots; i += BPT) table[i] = DIRECT ? (Entry)0 : (Entry)(MODE == BP_CCOUNT ? EMPTY32 : EMPTY64);
    __syncthreads();

    // Counting hash tables: the BP_K elements of a lane walk their probe
    // sequences together -- each round issues one LDS access per pending
    // element back to back, so a round costs one LDS latency instead of BP_K
    // (a lane otherwise waits out every element's chain one after another).
    // Measured on MI355X (sparse 63-bit keys, 1B x 1B, KCOUNT): 23 ms with
    // interleaved rounds vs 14 ms walking the elements one after another --
    // a round re-issues the LDS access of every element until the longest
    // chain of the wave ends, and 64-bit LDS CAS throughput is what binds.
    // Kept for experiments: compile with -DHPCJOIN_BP_INTERLEAVE.
#ifdef HPCJOIN_BP_INTERLEAVE
    constexpr bool INTERLEAVED = !MAT && !DIRECT;
#else
    constexpr bool INTERLEAVED = false;
#endif
    // ---- build
    for (uint32_t b0 = 0; b0 < nr; b0 += BATCH) {
      if (b0) bpLoadSide<MODE, SPLIT, L, false>(a.R, a.Rhi, rb, nr, b0, a, rv);
      if constexpr (INTERLEAVED) {
        using K = decltype(bpKey<MODE, L>(rv[0]));
        const K empty = (K)(MODE == BP_CCOUNT ? EMPTY32 : EMPTY64);
        uint32_t hh[BP_K], pend = 0;
#pragma unroll
        for (int k = 0; k < BP_K; ++k) {
          hh[k] = bpHash<MODE>(bpKey<MODE, L>(rv[k]), tbits);
          if (b0 + k * BPT + t < nr) pend |= 1u << k;
        }
        while (pend) {
          // Every CAS of the round is issued before any result is used, and
          // without branches: an element that is not pending (already placed,
          // or a lane past the batch end) swaps its key for itself, which
          // never changes the table.
          K old[BP_K];
#pragma unroll
          for (int k = 0; k < BP_K; ++k) {
            const K key = bpKey<MODE, L>(rv[k]);
            old[k] = atomicCAS(reinterpret_cast<K *>(&table[hh[k]]), (pend & (1u << k)) ? empty : key, key);
          }
#pragma unroll
          for (int k = 0; k < BP_K; ++k)
            if (pend & (1u << k)) {
              if (old[k] == empty)
                pend &= ~(1u << k);
              else
                hh[k] = (hh[k] + 1) & mask;
            }
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < BP_K; ++k) {
        const uint32_t idx = b0 + k * BPT + t;
        if (idx < nr) {
          if constexpr (DIRECT) {
            atomicAdd(&table[rv[k]], 1u);
          } else if constexpr (MODE == BP_CCOUNT) {
            const uint32_t frag = rv[k];
            uint32_t h = hash32(frag, tbits);
            while (atomicCAS(&table[h], EMPTY32, frag) != EMPTY32) h = (h + 1) & mask;
          } else if constexpr (!WIDE) {
            const uint64_t v = rv[k];
            const uint32_t frag = (uint32_t)(v >> a.fragShift);
            uint32_t h = hash32(frag, tbits);
            while (atomicCAS(&table[h], EMPTY64, (unsigned long long)v) != EMPTY64) h = (h + 1) & mask;
          } else {
            const ulonglong2 v = rv[k];
            uint32_t h = hash64(v.x, tbits);
            while (atomicCAS(&table[h], EMPTY64, (unsigned long long)v.x) != EMPTY64) h = (h + 1) & mask;
            if constexpr (MAT) ridTable[h] = v.y;
          }
        }
      }
    }
    __syncthreads();

    // ---- probe
    for (uint32_t b0 = 0; b0 < ns; b0 += BATCH) {
      if (b0) {
        if (b0 + BATCH <= ns) bpLoadSide<MODE, SPLIT, L, true>(a.S, a.Shi, sb, ns, b0, a, sv);
        else bpLoadSide<MODE, SPLIT, L, false>(a.S, a.Shi, sb, ns, b0, a, sv);
      }
      if constexpr (INTERLEAVED) {
        using K = decltype(bpKey<MODE, L>(sv[0]));
        const K empty = (K)(MODE == BP_CCOUNT ? EMPTY32 : EMPTY64);
        uint32_t hh[BP_K], live = 0, found = 0;
#pragma unroll
        for (int k = 0; k < BP_K; ++k) {
          hh[k] = bpHash<MODE>(bpKey<MODE, L>(sv[k]), tbits);
          if (b0 + k * BPT + t < ns) live |= 1u << k;
        }
        while (live) {
          K e[BP_K];  // every pending read of the round is issued before any is compared
#pragma unroll
          for (int k = 0; k < BP_K; ++k) e[k] = reinterpret_cast<const K *>(table)[hh[k]];
#pragma unroll
          for (int k = 0; k < BP_K; ++k)
            if (live & (1u << k)) {
              if (e[k] == empty) {
                live &= ~(1u << k);
              } else {
                found += (e[k] == bpKey<MODE, L>(sv[k]));
                hh[k] = (hh[k] + 1) & mask;
              }
            }
        }
        matches += found;
        continue;
      }
#pragma unroll
      for (int k = 0; k < BP_K; ++k) {
        const uint32_t idx = b0 + k * BPT + t;
        const bool active = idx < ns;
        uint32_t found = 0;
        uint64_t m0 = 0, m1 = 0, sRid = 0;
        if (active) {
          if constexpr (DIRECT) {
            found = table[sv[k]];
          } else if constexpr (MODE == BP_CCOUNT) {
            const uint32_t frag = sv[k];
            uint32_t h = hash32(frag, tbits);
            uint32_t e;
            while ((e = table[h]) != EMPTY32) {
              found += (e == frag);
              h = (h + 1) & mask;
            }
          } else if constexpr (!WIDE) {
            const uint64_t v = sv[k];
            const uint32_t frag = (uint32_t)(v >> a.fragShift);
            uint32_t h = hash32(frag, tbits);
            {
              sRid = v & ridMask;
              unsigned long long e;
              while ((e = table[h]) != EMPTY64) {
                if ((uint32_t)(e >> a.fragShift) == frag) {
                  const uint64_t rr = e & ridMask;
                  if (found == 0) m0 = rr;
                  else if (found == 1) m1 = rr;
                  else emitPair(a, reserveOne(a.outCursor, itemCursor, itemBase), rr, sRid);  // overflow path
                  ++found;
                }
                h = (h + 1) & mask;
              }
            }
          } else {
            const ulonglong2 v = sv[k];
            uint32_t h = hash64(v.x, tbits);
            sRid = v.y;
            unsigned long long e;
            while ((e = table[h]) != EMPTY64) {
              if (e == v.x) {
                if constexpr (MAT) {
                  const uint64_t rr = ridTable[h];
                  if (found == 0) m0 = rr;
                  else if (found == 1) m1 = rr;
                  else emitPair(a, reserveOne(a.outCursor, itemCursor, itemBase), rr, sRid);
                }
                ++found;
              }
              h = (h + 1) & mask;
            }
          }
        }
        matches += found;
        if constexpr (MAT) {
          const uint32_t mine = found < MAT_SLOTS ? found : MAT_SLOTS;
          const unsigned long long pos = reserveOutput(mine, a.outCursor, itemCursor, itemBase);
          if (mine > 0) emitPair(a, pos, m0, sRid);
          if (mine > 1) emitPair(a, pos + 1, m1, sRid);
        }
      }
    }
    if constexpr (ITEMS) {
      const unsigned long long im =
          blockReduceSum<BPT, unsigned long long>((unsigned long long)(matches - matchesBefore), wsum);
      if (t == 0) a.itemCounts[w] = (uint32_t)im;
    }
    __syncthreads();
  }
  const unsigned long long total = blockReduceSum<BPT, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(a.result, total);
}

// Key-only words (JoinPlan::keyOnly) are counted over spans in key_tables.hip.
void buildProbe(const BPArgs &args, const BPItem *items, const uint32_t *nItems, uint32_t capacity, hipStream_t s) {
  if (capacity == 0) return;
  BPArgs a = args;
  if (!a.partREnd) a.partREnd = a.partR + 1;
  if (!a.partSEnd) a.partSEnd = a.partS + 1;
  const size_t lds = bpLdsBytes(a);
  HJ_CHECK(lds <= 160 * 1024, "buildProbe: LDS request %zu exceeds 160 KiB (rChunk=%u)", lds, a.rChunk);
  const uint32_t perCu = (uint32_t)((160 * 1024) / lds);
  const uint32_t maxBlocks = 256 * (perCu < 8 ? (perCu ? perCu : 1) : 8);
  const uint32_t blocks = capacity < maxBlocks ? capacity : maxBlocks;
  HJ_CHECK(!(a.split && a.wide), "buildProbe: the split layout holds compressed tuples");
  HJ_CHECK(!a.split || (a.Rhi && a.Shi), "buildProbe: split layout without fragment columns");
  HJ_CHECK(a.wide || a.keyOnly || a.fragShift >= 32,
           "buildProbe: fragShift=%u < 32 (the rid field of a CompressedTuple is >= 32 bits)", a.fragShift);
  HJ_CHECK(!a.keyOnly, "buildProbe: key-only words are counted over spans (buildProbeKeySpans)");
  if (bpMode(a) == BP_CCOUNT && a.split && bpDirect(a) && !a.itemCounts) {
    const size_t ldsD = ((size_t(4) << a.fragBits) + 15) / 16 * 16 + 64;
    const uint32_t perCuD = (uint32_t)std::min<size_t>(BPD_MINB, (160 * 1024) / ldsD);  // occupancy target
    const uint32_t blocksD = std::min<uint32_t>(capacity, 256 * std::max<uint32_t>(perCuD, 1));
    hipLaunchKernelGGL((bpDirectSplitKernel<BPD_K, BPD_MINB>), dim3(blocksD), dim3(BPD_T), ldsD, s, a, items, nItems,
                       capacity);
    HIP_CHECK_LAUNCH();
    return;
  }
  if (bpMode(a) == BP_CCOUNT) {
    // Count-only instantiations: per-item counts (two-pass materialization's
    // count pass) x split columns x direct-addressed table.
#define HJ_BP_COUNT(ITEMS, SPLIT, DIRECT)                                                                         \
  hipLaunchKernelGGL((buildProbeKernel<BP_CCOUNT, ITEMS, SPLIT, DIRECT>), dim3(blocks), dim3(BPT), lds, s, a, items, \
                     nItems, capacity)
    const bool direct = bpDirect(a), it = a.itemCounts != nullptr, sp = a.split != 0;
    if (it) {
      if (sp) { if (direct) HJ_BP_COUNT(true, true, true); else HJ_BP_COUNT(true, true, false); }
      else { if (direct) HJ_BP_COUNT(true, false, true); else HJ_BP_COUNT(true, false, false); }
    } else {
      if (sp) { if (direct) HJ_BP_COUNT(false, true, true); else HJ_BP_COUNT(false, true, false); }
      else { if (direct) HJ_BP_COUNT(false, false, true); else HJ_BP_COUNT(false, false, false); }
    }
#undef HJ_BP_COUNT
    HIP_CHECK_LAUNCH();
    return;
  }
  if (a.split) {  // materialize
    const size_t ldsM = bpMatSplitLds(a);
    const bool rows = a.outRows != nullptr;
    const size_t stageBytes = rows ? (BPM_T / WAVE) * 5 * WAVE * sizeof(ulonglong2) : 0;  // 20 KiB
    HJ_CHECK(ldsM + stageBytes <= 160 * 1024, "buildProbe: LDS request %zu exceeds 160 KiB (rChunk=%u)",
             ldsM + stageBytes, a.rChunk);
    const uint32_t perCuM = (uint32_t)std::min<size_t>(4, (160 * 1024) / (ldsM + stageBytes + 64));
    const uint32_t blocksM = std::min<uint32_t>(capacity, 256 * std::max<uint32_t>(perCuM, 1));
    if (rows) HJ_CHECK(a.rowsA && a.rowsB && a.itemOffsets, "buildProbe: row output needs payload columns and item offsets");
    if (rows && a.rowsLds && a.rChunk <= BPR_MAX_R) {
      const size_t ldsR = bpMatRowsLds(a.rChunk);
      const uint32_t perCuR = (uint32_t)std::max<size_t>(1, std::min<size_t>(3, (160 * 1024) / (ldsR + 16)));
      const uint32_t blocksR = std::min<uint32_t>(capacity, 256 * perCuR);
      hipLaunchKernelGGL(bpMatRowsKernel, dim3(blocksR), dim3(BPR_T), ldsR, s, a, items, nItems, capacity);
    } else if (rows) {
      hipLaunchKernelGGL(bpMatSplitKernel<true>, dim3(blocksM), dim3(BPM_T), ldsM, s, a, items, nItems, capacity);
    } else {
      hipLaunchKernelGGL(bpMatSplitKernel<false>, dim3(blocksM), dim3(BPM_T), ldsM, s, a, items, nItems, capacity);
    }
    HIP_CHECK_LAUNCH();
    return;
  }
  switch (bpMode(a)) {
    case BP_CMAT:
      hipLaunchKernelGGL(buildProbeKernel<BP_CMAT>, dim3(blocks), dim3(BPT), lds, s, a, items, nItems, capacity);
      break;
    case BP_WCOUNT:
      if (a.itemCounts)
        hipLaunchKernelGGL((buildProbeKernel<BP_WCOUNT, true>), dim3(blocks), dim3(BPT), lds, s, a, items, nItems,
                           capacity);
      else
        hipLaunchKernelGGL(buildProbeKernel<BP_WCOUNT>, dim3(blocks), dim3(BPT), lds, s, a, items, nItems, capacity);
      break;
    default:
      hipLaunchKernelGGL(buildProbeKernel<BP_WMAT>, dim3(blocks), dim3(BPT), lds, s, a, items, nItems, capacity);
      break;
  }
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadBuildProbe() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&bpPlanCountsKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
