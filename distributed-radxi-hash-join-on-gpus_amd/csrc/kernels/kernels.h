// Host-side launch API of every hand-written CDNA4 (gfx950) kernel.
//
// Kernel map vs the reference GPU library:
//   datagen.hip      device relation generators (replace Relation.cpp:63-141)
//   partition.hip    LDS radix histogram + LDS write-combining scatter, both
//                    radix passes (network pass = NetworkPartitioning.cpp:74-222,
//                    local pass = LocalPartitioning.cpp:138-250; supersede the
//                    dormant histogram_build_L1/L2 + reorder_L1/L2 families of
//                    kernels.cu / kernels_optimized.cu / kernels_tile.cu)
//   build_probe.hip  LDS hash build/probe over (partition, R-chunk, S-chunk)
//                    work items (BuildProbe.cpp:47-121, eth.cu:25-109, and the
//                    probe / probe_skew / probe_count / probe_match_rate family)
//   scan.hip         wave64 LDS exclusive scans (replaces thrust::exclusive_scan)
//   npj.hip          no-partitioning join baseline (build_kernel/probe_kernel)
//   microbench.hip   bandwidth / ablation micro-benchmarks
#pragma once

#include <hip/hip_runtime.h>

#include "../core/Types.h"
#include "../data/Tuple.h"
#include "Random.h"

namespace hpcjoin {
namespace kernels {

// ---------------------------------------------------------------- geometry
constexpr uint32_t PART_THREADS = 256;   // 4 wave64s per partitioning workgroup
constexpr uint32_t PART_ITEMS = 16;      // tuples per thread per tile
constexpr uint32_t PART_TILE = PART_THREADS * PART_ITEMS;  // 4096 tuples per LDS tile
constexpr uint32_t MAX_PART_BITS = 11;   // LDS cursor/count arrays sized for 2048 digits

struct PartitionGeometry {
  uint32_t blocks = 0;         // workgroups of the pass (each owns a contiguous tile range)
  uint32_t tilesPerBlock = 0;  // tiles per workgroup
  uint32_t ipt = 0;            // claim-scatter tile variant (KernelVariants::netIpt; 0 = auto)
  uint32_t nth = 0;            // claim-scatter workgroup width (KernelVariants::netThreads; 0 = 1024)
  uint64_t tuplesPerBlock() const { return uint64_t(tilesPerBlock) * PART_TILE; }
};
// Cap the grid at ~8 workgroups per CU (2048) and give each workgroup a
// contiguous run of tiles so its per-digit output runs stay contiguous.
PartitionGeometry partitionGeometry(uint64_t n, uint32_t maxBlocks = 2048);


// ----------------------------------------------------------------- datagen
enum class KeyDistribution : int { Unique = 0, Modulo = 1, Uniform = 2, Zipf = 3, Dense = 4 };

struct GenParams {
  KeyDistribution dist = KeyDistribution::Unique;
  uint64_t globalOffset = 0;  // global index of local element 0
  uint64_t ridOffset = 0;     // rid of local element 0
  uint64_t domain = 0;        // key domain: keys in [keyOffset, keyOffset + domain)
  uint64_t keyOffset = 0;
  uint64_t modulo = 0;        // Modulo: key = perm(gi % modulo)
  FeistelPermutation perm{};  // Unique/Modulo/Zipf rank -> key bijection
  uint64_t seed = 0;
  ZipfParams zipf{};
  bool tpchSparse = false;    // TPC-H O_ORDERKEY layout: k -> (k / 8) * 32 + k % 8 + 1
  bool sparse64 = false;      // sparse random 63-bit keys: k -> sparseKey(k) (after tpchSparse)
};
HJ_HD uint64_t tpchSparseKey(uint64_t k) { return (k >> 3) * 32 + (k & 7) + 1; }
void generate(data::Tuple *out, uint64_t n, const GenParams &p, hipStream_t s);
// Oracle of skewed joins: counts[key - lo] += 1 for keys in [lo, lo + domain)
// (u32 counts, zeroed by the caller); *outside += keys outside that range.
void countKeys(const data::Tuple *in, uint64_t n, uint64_t lo, uint64_t domain, uint32_t *counts,
               unsigned long long *outside, hipStream_t s);

// ------------------------------------------------- pass 1: network partition
// Hash partitioning for keys whose low bits are structured (sparse TPC-H
// order keys, multiples of a stride): radix digits are taken from a bijection
// of the key on [0, 2^bits) instead of the raw key, and the mixed key is what
// the network pass stores, so every later pass and the build/probe compare
// mixed keys (equality is preserved by the bijection).  Off = identity, which
// is optimal for dense keys (perfectly balanced partitions).
struct KeyMix {
  uint32_t on = 0;
  uint32_t bits = 64;
  HJ_HD uint64_t apply(uint64_t k) const {
    if (!on) return k;
    const uint64_t m = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    const uint32_t h = (bits + 1) / 2;
    k = (k * 0x9E3779B97F4A7C15ull) & m;  // odd multiplier: bijective mod 2^bits
    k ^= k >> h;                           // xor-shift: bijective on [0, 2^bits)
    k = (k * 0xC2B2AE3D27D4EB4Full) & m;
    k ^= k >> h;
    return k;
  }
};

// Sparse random int64 keys (BASELINE: "random int64 keys"): a fixed bijection
// of [0, 2^63) applied to the generated dense key, so unique / foreign-key
// structure (and the exact oracle) is preserved while the keys spread over
// the whole non-negative int64 range -- a 1B-key relation then needs all 63
// key bits, so only the wide / key-only paths can join it.
constexpr uint64_t SPARSE_KEY_MAX = (1ull << 63) - 1;
HJ_HD uint64_t sparseKey(uint64_t k) {
  const KeyMix m{1u, 63u};
  return m.apply((k ^ 0x2545F4914F6CDD1DULL) & SPARSE_KEY_MAX);
}

// blockHist is digit-major [F][blocks] (u32).
void netHistogram(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                  uint32_t *blockHist, hipStream_t s, KeyMix mix = KeyMix(), uint32_t sampleStride = 1);
// Sampled variant (sampleStride > 1): every workgroup counts only tiles 0, S,
// 2S, ... of its own range (estimates for the single-rank sampled network pass).
// totals[g][d] (u64): blockHist summed over the workgroups of XCD group g.
void netGroupTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint64_t *totals, hipStream_t s);
// Tile stride of a sampled pass over n tuples into F digits: the requested
// stride, lowered so that every (XCD group, digit) cell gets >= 32 sampled
// tuples on average (small inputs; a cell sampled 0 times is the usual
// overflow cause).
uint32_t sampleStrideFor(const PartitionGeometry &g, uint64_t n, uint32_t F, uint32_t stride);
// Sampled [NGROUPS][F] totals: every sampleStride-th tile of each XCD group
// (the tile set sampleScale() counts as seen); totals are cleared first.
void netSampledTotals(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                      uint64_t *totals, hipStream_t s, KeyMix mix, uint32_t sampleStride);
// Both sides of a join in one launch (one clear when the totals are adjacent).
struct SampledInput {
  const data::Tuple *data;
  uint64_t n;
  PartitionGeometry geom;
  uint32_t stride;
  uint64_t *totals;  // [NGROUPS][F]
};
// preZeroed: the totals are already zero (DeviceControl), no clear is issued.
void netSampledTotals(const SampledInput *sides, uint32_t count, uint32_t bits, hipStream_t s, KeyMix mix,
                      bool preZeroed = false);
// totals[c][g][d] (u64) = sum of blockHist[d][b] over the blocks b of chunk c
// (blocksPerChunk each) with (b - first block of c) % NGROUPS == g: the claim
// groups of chunk c's scatter launch (sampled N > 1 network pass).
void netChunkGroupTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                         uint32_t chunks, uint64_t *totals, hipStream_t s);
// totals[c][F] = sum of blockHist over the blocks of chunk c (blocksPerChunk each).
void digitTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                 uint32_t chunks, uint64_t *totals, hipStream_t s);
// cursors[d][b] = base[chunk(b)][d] + sum_{b' in chunk(b), b' < b} blockHist[d][b'].
void netCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                const uint64_t *base, uint64_t *cursors, hipStream_t s);
// Compressed (8 B) and wide (16 B, full-range keys) scatter into the send buffer.
// Group ("claim") cursors: workgroups are split into NGROUPS groups by
// blockIdx % NGROUPS (the XCD round-robin: a speed assumption only); every
// group owns a slice of every digit's region and claims runs from it with
// one device atomic per digit per tile, so the workgroups of an XCD append to
// ONE stream per digit and output lines fill inside that XCD's L2.
constexpr uint32_t CLAIM_GROUPS = 8;
// Round-interleaved claim slices (single-rank network windows).  A linear
// window puts every slice's run contiguously, so a tile's write-out -- runs
// for all G x F slices -- lands on G x F different pages spread over the whole
// window and the scatter's translation misses run at ~0.1 per tuple
// (rocprofv3 TCP_UTCL1_TRANSLATION_MISS, 8.9e7 per 1e9-tuple call).  Here
// slice i (= g * F + d, the claim-cursor index) owns logical positions
// L = i << lv | k, and L lives at physical slot
//   (k >> lp) << (lns + lp) | i << lp | (k & (2^lp - 1))   (lns = log2(G * F)):
// round j holds the j-th 2^lp-slot piece of every slice, so writers that
// advance through their slices at similar rates all write inside one or two
// rounds (a few MB) at any moment.  lp = lv = 0 is the identity (linear).
// Physical slots used: ceil(max slice capacity / 2^lp) rounds of 2^(lns + lp).
struct RoundMap {
  uint32_t lp = 0, lv = 0, lns = 0, pad = 0;
  HJ_HD uint64_t operator()(uint64_t L) const {
    const uint64_t k = L & ((1ull << lv) - 1);
    return ((k >> lp) << (lns + lp)) | ((L >> lv) << lp) | (k & ((1ull << lp) - 1));
  }
  HJ_HD bool on() const { return lv != 0; }
};
// 32-bit cursors whenever every output position fits (half the atomics' bytes).
inline bool cursorsNarrow(uint64_t outSize) { return outSize < (1ull << 32); }
// gcur[c][g][d] (u32 if narrow else u64): start of group g's slice of digit d in chunk c.
void netGroupCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                     const uint64_t *base, void *gcur, bool narrow, hipStream_t s);
// Scatters the tiles of workgroups [blockBegin, blockEnd) (one exchange chunk)
// claiming from that chunk's gcur[g][d] (narrow = cursorsNarrow(n)).
// keyBits: bits of the largest key (lets the kernel carry the digit in the
// packed word's spare top bits instead of a separate LDS array).
// withRids = false: key-only words (value = mixed key >> bits, keyShift 0) for
// counting joins whose keys do not fit a CompressedTuple (JoinPlan::keyOnly).
void netScatter(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift, const PartitionGeometry &g,
                uint32_t blockBegin, uint32_t blockEnd, void *gcur, uint64_t *out, hipStream_t s,
                uint32_t keyBits = 64, KeyMix mix = KeyMix(), const void *gend = nullptr, int narrowMode = -1,
                bool withRids = true, const uint32_t *roundMeta = nullptr);
void netScatterWide(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g,
                    uint32_t blockBegin, uint32_t blockEnd, void *gcur, data::Tuple *out, hipStream_t s,
                    KeyMix mix = KeyMix(), const void *gend = nullptr, int narrowMode = -1);
// Count-only projection (JoinPlan::fragments): the scatter writes only the
// u32 key fragment (mixed key >> bits) -- 4 bytes per tuple instead of 8.
// Needs a fragment of at most 32 bits above the digit (fragWordFits); with
// keyBits <= 32 the digit rides in the staged word, above that (e.g. 6B dense
// keys, 33 bits) the tile keeps a separate digit array.
HJ_HD bool fragWordFits(uint32_t keyBits, uint32_t bits) { return keyBits <= 32 + bits; }
void netScatterFrag(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g, uint32_t blockBegin,
                    uint32_t blockEnd, void *gcur, uint32_t *out, hipStream_t s, uint32_t keyBits,
                    KeyMix mix = KeyMix(), const void *gend = nullptr, int narrowMode = -1,
                    const uint32_t *roundMeta = nullptr);
// Partition-group pass of the same scatter: only tuples whose digit is in
// [dLo, dLo + range) are written, into [G][range] bounded claim slices (gcur /
// gend laid out by netSampledLayout with the same range); the others are read
// and dropped.  range < 1024 (one sentinel counter in the tile's LDS arrays).
// The final claim cursors count every kept tuple (overflow check as usual).
void netScatterFragRange(const data::Tuple *in, uint64_t n, uint32_t bits, const PartitionGeometry &g, void *gcur,
                         uint32_t *out, hipStream_t s, uint32_t keyBits, KeyMix mix, const void *gend, bool narrow,
                         uint32_t dLo, uint32_t range);
// Sampled network pass sized on the device (no host round trip): from the
// sampled [G][F] group totals (netGroupTotals) to bounded claim slices
// gstart/gcur/gend ([G][F], u32 if narrow else u64) and *capacityUsed = the
// sum of the slice capacities.  The host sizes the output buffer with
// sampledLayoutCapacityBound() beforehand.
struct SampleScale {
  double total[CLAIM_GROUPS];  // tuples each XCD group scatters
  double seen[CLAIM_GROUPS];   // of those, read by the sampled histogram
  double sigmas, frac, floor;  // margin = sigmas * sigma + frac * est + floor (0, 0, 0 = exact histogram)
};
SampleScale sampleScale(const PartitionGeometry &g, uint64_t n, uint32_t sampleStride, bool exact);
uint64_t sampledLayoutCapacityBound(const SampleScale &sc, uint32_t F);
void netSampledLayout(const uint64_t *sampled, uint32_t F, const SampleScale &sc, void *gstart, void *gcur, void *gend,
                      bool narrow, unsigned long long *capacityUsed, hipStream_t s);
// One or two sides per launch (same cursor width).
struct LayoutInput {
  const uint64_t *sampled;
  SampleScale sc;
  void *gstart, *gcur, *gend;
  unsigned long long *capacityUsed;
  bool clearSampled = false;  // zero `sampled` after reading it (DeviceControl totals)
  // Round-interleaved slices (RoundMap), decided on the device: with
  // roundMeta set, slices of 2^roundLp-slot pieces are used when the largest
  // slice needs lv <= roundMaxLv bits and the rounds fit roundCapacity slots;
  // roundMeta[0..2] = {lp, lv, lns} then (else zeros: linear slices).  Both
  // the scatter (netScatter / netScatterFrag roundMeta) and the read-back
  // take the map from there.  Needs G * F a power of two.
  uint32_t *roundMeta = nullptr;
  uint32_t roundLp = 0, roundMaxLv = 0;
  uint64_t roundCapacity = 0;
};
// Piece size (log2 slots) of a round-interleaved window of elemBytes-wide
// words: JoinConfig::roundLp is given for 8-byte words; 4-byte fragment
// windows use pieces of the same bytes.  0 = linear slices.
inline uint32_t roundLpFor(uint32_t roundLp, uint32_t elemBytes) {
  return roundLp ? roundLp + (elemBytes == 4 ? 1 : 0) : 0;
}
// Slots a round-interleaved window needs for slices of at most maxCap tuples.
HJ_HD uint64_t roundSlots(uint64_t maxCap, uint32_t lp, uint32_t lns) {
  return ((maxCap + (1ull << lp) - 1) >> lp) << (lns + lp);
}
// Window slots of a sampled single-rank pass: the linear bound, or (roundLp >
// 0) at least what round-interleaved slices need when every slice's sampled
// estimate lands within 5 sigma of its group's mean (even data; skewed data
// then gets linear slices inside the same window).
uint64_t sampledWindowCapacity(const SampleScale &sc, uint32_t F, uint32_t roundLp);
// range > 0: lay out only digits [dLo, dLo + range) of the [G][F] totals, as
// [G][range] slices (a partition-group pass, netScatterFragRange).
void netSampledLayout(const LayoutInput *sides, uint32_t count, uint32_t F, bool narrow, hipStream_t s,
                      uint32_t dLo = 0, uint32_t range = 0);
// gend (optional, same layout and width as gcur): end of every group slice.
// Positions claimed past a slice end are not written; the final gcur values
// tell the caller each slice's demand (the sampled pass re-runs exactly on
// overflow).  narrowMode: 1/0 = 32/64-bit cursors, -1 = cursorsNarrow(n).
// Ablation entry (micro-benchmarks): mode 0 = real scatter, 1 = coalesced
// write-out, 2 = no write-out; 32-bit cursors, compressed output.
// geometry: 0 = 256x16 (default), 1 = 512x16, 2 = 1024x8, 3 = 1024x16,
// 4 = 256x16 with a separate LDS digit array, 5 = 256x8.
// geometries 6..9 = claim mode (256x16, 512x16, 1024x16, 1024x8) using gcur
// (u32 group cursors [8][F], re-initialised by the caller before each call);
// mode 3 = the real scatter into round-interleaved slices (device roundMeta,
// RoundMap; gcur then holds logical slice starts).
void scatterAblation(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift, const PartitionGeometry &g,
                     const uint64_t *cursors, uint64_t *out, int mode, int geometry, hipStream_t s,
                     void *gcur = nullptr, const uint32_t *roundMeta = nullptr);

// Ablation baseline: one global atomic per tuple, no LDS staging
// (reference histogram_build_global / reorder_global, kernels.cu:256-298).
void netScatterGlobalAtomic(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift,
                            uint64_t *digitCursor, uint64_t *out, hipStream_t s);

// --------------------------------------------------- pass 2: local partition
// One work item = a contiguous run (<= LOCAL_ITEM_MAX tuples) of one received
// segment that belongs to owned partition `lp`.  Items are sorted by lp.
struct LocalItem {
  uint64_t begin;
  uint32_t len;
  uint32_t lp;
  uint32_t stream;  // claim stream (assignLocalStreams), device path only
  uint32_t pad;
};
// Assigns claim streams (one per (lp, XCD group) run of the lp-sorted items);
// returns the number of streams.
uint32_t assignLocalStreams(LocalItem *items, uint32_t nItems);
constexpr uint32_t LOCAL_ITEM_TILES = 16;
constexpr uint32_t LOCAL_ITEM_MAX = LOCAL_ITEM_TILES * PART_TILE;  // 65536

// digit = (word >> shift) & (2^bits - 1).  For compressed tuples word = value,
// shift = keyShift; for wide tuples word = key, shift = networkBits; for u32
// key fragments (frag) word = fragment, shift = 0.
// rm: the network window's slot map (RoundMap; items are logical positions).
void localHistogram(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift,
                    uint32_t bits, uint32_t *itemHist, hipStream_t s, uint32_t sampleStride = 1, bool frag = false,
                    RoundMap rm = RoundMap());
// gcur[stream][F] (u32 if narrow else u64) claim slices + partBegin[owned*F+1].
void localCursors(const uint32_t *itemHist, const uint32_t *lpItemBegin, uint32_t owned, uint32_t bits,
                  const uint64_t *lpBase, const LocalItem *items, void *gcur, bool narrow, uint64_t *partBegin,
                  hipStream_t s);
// Split (SoA) tuples of the local pass output (device, compressed format),
// the columnar layout of the reference's dormant GPU library (relation_t
// {key*, id*}, /root/reference/data/data.hpp:57-62): after both radix passes
// a final partition implies networkBits + localBits key bits, so a tuple is
// its rid (u32 column) plus the key fragment above fragShift (u16 column) --
// 6 bytes instead of 8, and a count-only build/probe reads just the 2-byte
// fragment column.  Both columns are unit-stride in every scatter run and
// every build/probe batch.
struct SplitLayout {
  uint32_t on = 0;
  uint32_t fragShift = 32;   // CompressedTuple fragment position (value >> fragShift)
  // Low column = (u32)(value >> loShift): 0 for CompressedTuples (the rid);
  // localBits for key-only words (JoinPlan::keyOnly), whose 6-byte split is
  // the key fragment above both radix digits (lo = its low 32 bits, hi = the
  // next 16: fragShift = localBits + 32), 2 bytes less per tuple than the
  // 8-byte word in the local pass output and the count kernel's reads.
  uint32_t loShift = 0;
  uint16_t *hi = nullptr;    // fragment column (element i <-> lo[i])
  HJ_HD uint64_t value(uint32_t rid, uint16_t frag) const { return (uint64_t)rid | ((uint64_t)frag << fragShift); }
};
constexpr uint32_t SPLIT_BYTES = 6;

// split.on (compressed input only): out is the u32 rid column, split.hi the
// u16 fragment column (kernels.h, SplitLayout).
// frag: the input is u32 key fragments (JoinPlan::fragments) and the output
// the u16 column of fragment >> bits alone (out; split.hi unused).
void localScatter(const void *in, bool wide, const LocalItem *items, uint32_t nItems, uint32_t shift,
                  uint32_t bits, void *gcur, bool narrow, void *out, hipStream_t s, const void *gend = nullptr,
                  SplitLayout split = SplitLayout(), uint32_t geometry = 0, bool frag = false,
                  RoundMap rm = RoundMap());
// Sampled local pass (no exact local histogram): itemHist from
// localHistogram(sampleStride) -> per-final-partition capacities (estimate +
// 8 sigma + 2% + 64) -> gapped partition-major layout: gcur = partBegin =
// starts, gend = starts + caps (64-bit cursors; one claim stream per lp).
// After the bounded localScatter the final gcur values are the partition ends.
void localSampledLayout(const uint32_t *itemHist, const uint32_t *lpItemBegin, const LocalItem *items,
                        uint32_t owned, uint32_t bits, uint32_t sampleStride, uint32_t *caps,
                        unsigned long long *starts, void *scanWorkspace, unsigned long long *gcur,
                        unsigned long long *gend, uint64_t *partBegin, uint64_t capacity, hipStream_t s,
                        uint32_t align = 16);
// Upper bound of the layout's total capacity (host-side sizing of the output).
// align: slot granularity in tuples (16 = 128-byte lines of 8-byte tuples,
// 64 = whole lines of both split columns).
uint64_t localSampledCapacityBound(uint64_t n, uint64_t partitions, uint32_t sampleStride, uint32_t align = 16);
// *flag |= 1 if any gcur[i] > gend[i] (a bounded claim slice overflowed);
// gcur is clamped to gend, so it is always safe to use as partition ends.
void claimOverflow(unsigned long long *gcur, const unsigned long long *gend, uint64_t P, unsigned int *flag,
                   hipStream_t s);

// A resolved work item of key-only counting: one inner chunk against one
// outer chunk of a final partition.
struct BPSpan {
  unsigned long long rb, sb;  // first inner / outer word of the span
  uint32_t nr, ns;            // inner (<= rChunk) / outer (<= sChunk) words
  uint32_t flags;             // bit 0: the inner words are compacted (distinct words, counts in BPArgs::dedupCounts)
  uint32_t pad1;
};
// --------------------------------------------------------------- build/probe
struct BPItem {
  uint32_t part;
  uint32_t rChunk;
  uint32_t sChunk;
  uint32_t pad;
};
struct BPArgs {
  const void *R = nullptr;        // partitioned inner (u64 compressed or Tuple)
  const void *S = nullptr;        // partitioned outer
  const uint64_t *partR = nullptr;  // [P+1] partition begin offsets
  const uint64_t *partS = nullptr;
  // Partition ends (gapped layouts of the sampled local pass); null = partR + 1 / partS + 1.
  const uint64_t *partREnd = nullptr;
  const uint64_t *partSEnd = nullptr;
  uint32_t P = 0;
  uint32_t rChunk = 4096;   // max inner tuples per LDS table
  uint32_t sChunk = 65536;  // max outer tuples per work item
  uint32_t fragShift = 0;   // compressed: key fragment = value >> fragShift
  uint32_t keyShift = 32;   // compressed: rid = value & (2^keyShift - 1)
  // Compressed: fragments are < 2^fragBits (0 = unknown).  Counting with
  // fragBits <= BP_DIRECT_MAX_BITS uses a direct-addressed LDS count array
  // (counts[fragment]) instead of a hash table.
  uint32_t fragBits = 0;
  bool wide = false;
  bool materialize = false;
  // Key-only words (JoinPlan::keyOnly, counting): R and S hold 8-byte
  // key >> networkBits values; the table compares whole values.
  bool keyOnly = false;
  // Split layout (on = 1): R and S are u32 rid columns, Rhi / Shi the u16
  // fragment columns (kernels.h, SplitLayout).
  uint32_t split = 0;
  const uint16_t *Rhi = nullptr;
  const uint16_t *Shi = nullptr;
  unsigned long long *result = nullptr;     // match counter (device)
  unsigned long long *outCursor = nullptr;  // materialize: pair cursor (device)
  ulonglong2 *outPairs = nullptr;           // materialize: (rid_inner, rid_outer)
  uint64_t outCapacity = 0;
  // Exact materialization in two passes: a count pass writes the matches of
  // every work item (itemCounts), an exclusive scan turns them into output
  // offsets (itemOffsets), and the materialize pass places each item's pairs
  // from its offset with LDS-atomic cursors -- no contended device-wide
  // atomic per wave (measured 9.4M of them at 600M pairs).
  uint32_t *itemCounts = nullptr;
  const unsigned long long *itemOffsets = nullptr;
  // Fused row output (materialize pass of the split layout, both payload
  // columns local): whole 80-byte rows [rid_inner, rid_outer, inner row,
  // outer row] go to outRows (outCapacity rows) instead of pairs to outPairs.
  const ulonglong2 *rowsA = nullptr;  // inner payload rows, 2 x 16 B each
  const ulonglong2 *rowsB = nullptr;  // outer payload rows
  uint64_t offA = 0, offB = 0;        // rid of row 0 of each column
  ulonglong2 *outRows = nullptr;
  // Key-only words: bits of the fragment above both radix digits (0 =
  // unknown); the quotient-table kernel (keyCount 8) needs <= 44, the
  // counted-table kernel <= 48.
  uint32_t keyFragBits = 0;
  // Flags of the quotient-table kernel (build_probe.hip, KQF_*): bit 1 a
  // key's copies chained (count exact; keyCount 9 from then on); bit 3 a span
  // filled its overflow table (count void: re-run on counted tables, which
  // have no capacity limit).
  unsigned long long *sideOverflow = nullptr;
  // Optional (key-only spans with the quotient table): bpPlanCounts writes
  // the spans of partitions with more than rChunk inner tuples here (at most
  // heavyCapacity; heavyCount: u32 total, zeroed by the caller) instead of
  // giving them work items.
  BPSpan *heavySpans = nullptr;
  uint32_t *heavyCount = nullptr;
  uint32_t heavyCapacity = 0;
  uint32_t heavyMin = 0xFFFFFFFFu;  // inner tuples above which a partition is heavy
  // Optional (counted tables, repeated keys): partitions of more than rChunk
  // inner tuples go to dedupParts (u32 count at dedupCount, zeroed by the
  // caller); bpKeyDedup compacts each one's inner words in place to
  // (distinct word, count) -- the count in dedupCounts, indexed like R -- and
  // appends its spans, flagged as compacted, to heavySpans.
  uint32_t *dedupParts = nullptr;
  uint32_t *dedupCount = nullptr;
  uint32_t *dedupCounts = nullptr;
  uint64_t *dedupLen = nullptr;  // [P][BP_DEDUP_SEGS] compacted words per segment (kept for span re-emits)
  uint32_t *dedupBig = nullptr;       // listed partitions of more than one segment (u32 count at dedupBigCount)
  uint32_t *dedupBigCount = nullptr;
  // Kernel variants (KernelVariants::keyCount / rowsLds).
  uint32_t keyCount = 8;
  uint32_t rowsLds = 1;
};
// Payload columns + output of a fused materializing join (HashJoin::setRowSink).
struct RowSink {
  const uint64_t *rowsA = nullptr;
  uint64_t offA = 0;
  uint64_t rowsAN = 0;      // rows in rowsA: rids [offA, offA + rowsAN)
  const uint64_t *rowsB = nullptr;
  uint64_t offB = 0;
  uint64_t rowsBN = 0;
  uint64_t *out = nullptr;  // [capacity][10] u64
  uint64_t capacity = 0;
};
size_t bpLdsBytes(const BPArgs &a);
// True when a count over the split layout uses the direct-addressed count
// table (fragments <= 13 bits): its LDS table does not grow with the inner
// side, so a work item may take any number of inner tuples.
bool bpDirectSplit(const BPArgs &a);
constexpr uint32_t BP_DIRECT_R_CHUNK = 1u << 18;
void bpPlanCounts(const BPArgs &a, uint32_t *counts, hipStream_t s);
void bpEmit(const BPArgs &a, const uint32_t *counts, const uint32_t *offsets, BPItem *items,
            uint32_t capacity, hipStream_t s);
// Grid-strides over min(*nItems, capacity) items; nItems is a device word
// written by the scan, so no host round trip sits between plan and probe.
void buildProbe(const BPArgs &a, const BPItem *items, const uint32_t *nItems, uint32_t capacity, hipStream_t s);
// Key-only counting (BPArgs::keyOnly) over resolved spans: the item list with
// every item's bounds looked up once (bpEmitSpans), consumed through a device
// work queue (queue: one u32, cleared by the launcher) with the next span's
// words prefetched during the current probe.
void bpEmitSpans(const BPArgs &a, const uint32_t *counts, const uint32_t *offsets, BPSpan *spans, uint32_t capacity,
                 hipStream_t s);
void buildProbeKeySpans(const BPArgs &a, const BPSpan *spans, const uint32_t *nSpans, uint32_t capacity,
                        uint32_t *queue, hipStream_t s);
// keyCount 8 (quotient table, build_probe.hip) applies: split key-only words
// of <= 44 fragment bits, rChunk <= 2048.
bool bpKeyQuotientFits(const BPArgs &a);
// Counted tables (bpKeyCountedSpans) apply: split key-only words of <= 48
// fragment bits, rChunk <= 2048.
bool bpKeyCountedFits(const BPArgs &a);
// The spans bpPlanCounts wrote to a.heavySpans (partitions of repeated inner
// keys): counted tables (build_probe.hip, bpKeyCountedSpansKernel); adds to
// a.result.
void bpKeyCountedSpans(const BPArgs &a, uint32_t *queue, hipStream_t s);
// Compacts the partitions bpPlanCounts listed in a.dedupParts (see BPArgs)
// and appends their counted spans; run before bpKeyCountedSpans.
void bpKeyDedup(const BPArgs &a, uint32_t maxParts, bool emitOnly, hipStream_t s);
// After bpKeyDedup (not on an emitOnly re-run): one workgroup per partition
// of several segments moves the segments' compacted lists together (in
// place, in segment order) and emits the partition's counted spans over the
// merged list -- ceil(distinct / rChunk) passes over its outer side instead
// of one per segment.
void bpKeyDedupMerge(const BPArgs &a, uint32_t maxParts, hipStream_t s);
// Segments per compacted partition (bpKeyDedup): BPArgs::dedupLen has P of
// them; a partition of n words has min(16, ceil(n / BP_DEDUP_SEG_MIN)).
constexpr uint32_t BP_DEDUP_SEGS = 16;
constexpr uint64_t BP_DEDUP_SEG_MIN = 32768;

// Single-level counting join of unique inner keys (bitmap_join.hip): one
// workgroup per network partition sets a 2^bits LDS bitmap from the inner
// fragments and tests the outer ones.
//   elemBytes 4: u32 key fragments (count-only network pass), keyShift 0,
//                partitions given as the claim slices of a sampled pass
//   elemBytes 8: CompressedTuples (fragment = value >> keyShift), partitions
//                given as a segment table [F][groups] (exchanged windows)
constexpr uint32_t BITMAP_MAX_BITS = 20;  // 128 KiB of LDS
// The bitmap kernels may split a partition's fragment range over 2^split
// workgroups (each holds one 128 KiB piece and reads all of the partition's
// fragments): 21 fragment bits, e.g. 3B dense keys over a 2048-way digit.
constexpr uint32_t BITMAP_MAX_SPLIT = 1;
constexpr uint32_t BM_FLAG_DUP = 1;       // an inner fragment repeats or leaves the range: fall back
constexpr uint32_t BM_FLAG_OVERFLOW = 2;  // a sampled claim slice overflowed: redo with exact slices
// Four u64 sums, so that one all-reduce of the struct combines every rank's
// outcome on the device (dup / overflow: waves that raised the flag).
struct BitmapCounters {
  unsigned long long matches;
  unsigned long long popcount;  // bitmapProbe: set bits of the probed bitmaps
  unsigned long long dup;       // BM_FLAG_DUP raised
  unsigned long long overflow;  // BM_FLAG_OVERFLOW raised
};
// Result delivery without a device->host copy.  A ResultMailbox lives in
// host-mapped pinned memory; the last wave of a join's final kernel writes the
// join's counters into it with system-scope stores and then publishes `seq`
// (release), so the host spins on one word instead of waiting for a copy
// engine or a blit kernel (BENCH_r04: two joins stalled 6-8 ms after their
// last kernel, in the D2H copy + stream synchronisation).
struct ResultMailbox {
  unsigned long long seq;  // written last
  unsigned long long matches, popcount, dup, overflow;
  unsigned long long pad[3];
};
// Per-engine persistent device scratch that the kernels consuming it restore
// to zero, so a join issues no memset (no runtime fill kernel, no first-use
// load of the runtime's blit code): sampled totals of both sides (cleared by
// netSampledLayout after it reads them) and the bitmap join's counters plus
// the arrival count of its final kernel (cleared by that kernel's last wave).
struct DeviceControl {
  unsigned long long totals[2 * CLAIM_GROUPS * (1u << MAX_PART_BITS)];
  BitmapCounters counters;
  unsigned int arrivals;
  unsigned int pad[15];
};
// Passed to the final kernel of a mailbox join (box == nullptr: plain counters).
struct MailboxArgs {
  ResultMailbox *box = nullptr;  // device alias of the host-mapped mailbox
  unsigned int *arrivals = nullptr;
  unsigned long long seq = 0;
};
// ------------------------------------------------- exchange verification
// Content checksum of exchanged tuples (JoinConfig::verifyExchange,
// kernels/verify.hip): each tuple adds exchangeHash(mixed key, rid) to the sum
// of its (source, chunk, partition) run, on the sender from its input and on
// the receiver from its window; the sums must agree.
HJ_HD uint64_t exchangeHash(uint64_t mk, uint64_t rid) {
  uint64_t x = mk * 0x9E3779B97F4A7C15ull ^ (rid + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  return x;
}
// How a window word holds (mixed key, rid): Compressed value = rid |
// (mk >> bits) << keyShift (keyShift 0: key-only words, no rid); Wide 16-B
// tuples (mk, rid).  withRid = 0 when the rid did not travel (count-only wire).
struct ChecksumFormat {
  enum Kind : uint32_t { Compressed = 0, Wide = 1 };
  uint32_t kind = Compressed;
  uint32_t bits = 0, keyShift = 0, withRid = 0;
};
struct ChecksumSeg {
  uint64_t begin, len;  // window tuple range
  uint32_t partition;   // global partition id (the digit the window word omits)
  uint32_t slot;        // index of the (source, chunk, partition) sum
};
// sums[d] += hashes of in[begin, end) by digit (mk & (2^bits - 1)); sums zeroed by the caller.
void exchangeChecksumSend(const data::Tuple *in, uint64_t begin, uint64_t end, uint32_t bits, KeyMix mix,
                          bool withRid, unsigned long long *sums, hipStream_t s);
// sums[seg.slot] += hashes of the window run of every segment (segs: device array).
void exchangeChecksumRecv(const void *window, const ChecksumFormat &fmt, const ChecksumSeg *segs, uint32_t nSegs,
                          unsigned long long *sums, hipStream_t s);
void flipWindowWord(void *window, uint64_t word, hipStream_t s);

// ------------------------------------------------------- capacity spill
// Pass of a key when a join runs in K passes (kernels/spill.hip): a hash of
// the whole key, independent of the radix digits (its low bits), so every
// pass spreads over all partitions.
constexpr uint32_t MAX_SPILL_PASSES = 256;
HJ_HD uint32_t passOf(uint64_t key, uint32_t K) {
  uint64_t x = key ^ 0x5851F42D4C957F2Dull;
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return (uint32_t)(((x >> 32) * (uint64_t)K) >> 32);
}
// counts[p] += tuples of pass p (counts zeroed by the caller).
void passCounts(const data::Tuple *in, uint64_t n, uint32_t K, unsigned long long *counts, hipStream_t s);
// out = the tuples of pass k (any order); *cursor (zeroed by the caller) ends at their count.
// Writes stop at `capacity` tuples (the cursor still counts every one).
void passCompact(const data::Tuple *in, uint64_t n, uint32_t K, uint32_t k, data::Tuple *out,
                 unsigned long long *cursor, hipStream_t s, uint64_t capacity);

// p[0, words) = 0 (u64 words) with the engine's own kernel.
void zeroWords(void *p, uint64_t words, hipStream_t s);
// dst (pinned, device-mapped host memory) = src (device), by the engine's own kernel.
void copyToHost(void *dst, const void *src, uint64_t bytes, hipStream_t s);
// dst (device) = src (pinned, device-mapped host memory): the same kernel the other way round.
void copyFromHost(void *dst, const void *src, uint64_t bytes, hipStream_t s);
struct BitmapSlices {
  enum Kind : int { Claim = 0, Table = 1 };
  int kind = Claim;
  // Claim: [CLAIM_GROUPS][F] slice starts, final claim cursors, slice ends (u32 if narrow).
  const void *start = nullptr, *cur = nullptr, *end = nullptr;
  bool narrow = true;
  // Table: [F][groups] segment starts and lengths (device arrays).
  const uint64_t *segStart = nullptr, *segLen = nullptr;
  uint32_t groups = 0;
  // Elements over all partitions (0 = unknown): picks the slice walk of the
  // u32 kernels (one flat walk per partition when partitions are short).
  uint64_t count = 0;
  // Forced kernel shape (KernelVariants::bmThreads / bmFlat; read from the
  // inner side's slices): 0 / -1 = auto.
  uint32_t threads = 0;
  int32_t flat = -1;
  // Claim: device {lp, lv, lns, 0} of a round-interleaved fragment window
  // (RoundMap, LayoutInput::roundMeta); null = linear slices.
  const uint32_t *roundMeta = nullptr;
};
// u32 words of one partition's bitmap (a power of two >= 4).
uint32_t bitmapWords(uint32_t bits);
// bits may exceed BITMAP_MAX_BITS by up to BITMAP_MAX_SPLIT: each partition
// is then joined by 2^(bits - BITMAP_MAX_BITS) workgroups.
// mb.box != nullptr: the kernel's last wave publishes *out into the mailbox
// (seq mb.seq) and resets *out and *mb.arrivals to zero.
void bitmapJoin(uint32_t elemBytes, const void *r, const void *s, const BitmapSlices &rs, const BitmapSlices &ss,
                uint32_t partitions, uint32_t keyShift, uint32_t bits, BitmapCounters *out, hipStream_t st,
                const MailboxArgs &mb = MailboxArgs());
// bitmaps[d * bitmapWords(bits) ...] = partition d's bitmap of r.
// Partitions [first, first + count) only (count = UINT32_MAX: to the end).
void bitmapBuild(uint32_t elemBytes, const void *r, const BitmapSlices &rs, uint32_t partitions, uint32_t keyShift,
                 uint32_t bits, uint32_t *bitmaps, BitmapCounters *out, hipStream_t st, uint32_t first = 0,
                 uint32_t count = UINT32_MAX);
// Probes s against bitmaps (e.g. all-reduced over ranks); out->popcount += set bits.
// Partitions [first, first + count) only (count = UINT32_MAX: to the end);
// slices and bitmaps are indexed by the global partition number.
void bitmapProbe(uint32_t elemBytes, const void *s, const BitmapSlices &ss, uint32_t partitions, uint32_t keyShift,
                 uint32_t bits, const uint32_t *bitmaps, BitmapCounters *out, hipStream_t st, uint32_t first = 0,
                 uint32_t count = UINT32_MAX);

// ------------------------------------------------------------ wire codec
// Exchange wire format for 8-byte CompressedTuples (N > 1).  On the wire a
// tuple needs only its key fragment above the network digit (the receiver
// knows the partition) and its rid relative to the sending rank's smallest
// rid (frame of reference): w = ridBits + keyFragmentBits bits, e.g. 48 for
// 1B unique keys on 8 ranks (21 + 25 with one rid base per rank and
// exchange chunk) instead of 64.  Tuples are bit-packed
// in groups of 64: a group of a segment occupies w u64 words, lane j of a
// wave64 writing word j.  The xGMI links are the bottleneck of the
// distributed join, so this cuts the exchange time by (64 - w) / 64.
struct WireCodec {
  uint32_t w = 0;         // bits per tuple on the wire (0 = codec off)
  uint32_t ridBits = 0;   // low bits of a wire value: rid - base
  uint32_t keyShift = 32; // CompressedTuple: value = rid | fragment << keyShift
  // ridBits == 0 (count-only joins: no rid is ever read): only the key
  // fragment travels; decoded tuples carry the sender's base as their rid.
  HJ_HD uint64_t encode(uint64_t v, uint64_t base) const {
    const uint64_t rid = v & ((1ull << keyShift) - 1);
    return ((rid - base) & ((1ull << ridBits) - 1)) | ((v >> keyShift) << ridBits);
  }
  HJ_HD uint64_t decode(uint64_t e, uint64_t base) const {
    const uint64_t rid = (e & ((1ull << ridBits) - 1)) + base;
    return rid | ((e >> ridBits) << keyShift);
  }
  HJ_HD uint64_t words(uint64_t n) const { return (n + 63) / 64 * w; }
};
// One contiguous run of tuples <-> one packed run of words.
struct WireSeg {
  uint64_t raw;     // tuple offset in the raw (8-byte) buffer
  uint64_t wire;    // word offset in the wire buffer
  uint64_t n;       // tuples
  uint64_t base;    // rid base of the sending rank
  uint64_t group0;  // first global group index of this segment (prefix of ceil(n/64))
};
// segs is a device array (nSegs entries, ascending group0); totalGroups = sum ceil(n/64).
// rm: slot map of `raw` (RoundMap of a round-interleaved send buffer; seg.raw
// is then a logical position).
void wirePack(const uint64_t *raw, uint64_t *wire, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
              const WireCodec &c, hipStream_t s, RoundMap rm = RoundMap());
void wireUnpack(const uint64_t *wire, uint64_t *raw, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
                const WireCodec &c, hipStream_t s);
// Raw segmented gather: dst[seg.wire + t] = src[seg.raw + t] for t < seg.n
// (same segment list format; offsets in 8-byte words, nothing past seg.n written).
void segCopy(const uint64_t *src, uint64_t *dst, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
             hipStream_t s, RoundMap rm = RoundMap());

// ------------------------------------------------------------------- scans
size_t scanWorkspaceBytes(uint64_t n);
// out[i] = sum_{j<i} in[j]; *total = sum of all (device pointer, may be null).
void scanExclusiveU32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *workspace,
                      hipStream_t s);
// Same with 64-bit prefix sums (per-item match counts -> output offsets).
void scanExclusiveU32to64(const uint32_t *in, unsigned long long *out, uint64_t n, unsigned long long *total,
                          void *workspace, hipStream_t s);

// Claim-scatter phase profile (partition.hip, built with
// -DHPCJOIN_SCATTER_PROF): shader-clock sums per tile phase [8], tiles [8],
// ranges [9]; all zero in a normal build.
void scatterProfile(unsigned long long out[10], bool reset);
bool scatterProfileBuilt();

// --------------------------------------------------- no-partitioning join
uint64_t npjTableSlots(uint64_t innerSize);
void npjBuild(const data::Tuple *R, uint64_t nR, unsigned long long *table, uint64_t slots, hipStream_t s);
void npjProbe(const data::Tuple *S, uint64_t nS, const unsigned long long *table, uint64_t slots,
              unsigned long long *result, hipStream_t s);
// Materializing NPJ (the reference's simple_hash_join writes (rid, rid)
// pairs through a global cursor, small_data_optimized.cu:1731-1823): the
// build also stores each inner tuple's rid next to its key slot (rids[slots]);
// the probe gives every outer tuple with m matches one cursor claim of m
// and writes (inner rid, outer rid) pairs at out[claim..) while they fit
// `capacity` (the cursor still counts all matches: a caller that sized out
// from npjProbe's count never overflows).
void npjBuildRids(const data::Tuple *R, uint64_t nR, unsigned long long *table, unsigned long long *rids,
                  uint64_t slots, hipStream_t s);
void npjProbePairs(const data::Tuple *S, uint64_t nS, const unsigned long long *table,
                   const unsigned long long *rids, uint64_t slots, ulonglong2 *out, uint64_t capacity,
                   unsigned long long *cursor, hipStream_t s);

// ---------------------------------------------------------- micro-benchmarks
// Plan-time repeated-key probe (microbench.hip): S evenly spaced keys of
// in[0, n) into a set in ws (sampleRepeatsBytes(S)); *repeats = sampled keys
// that were already in it.
size_t sampleRepeatsBytes(uint32_t S);
void sampleRepeats(const data::Tuple *in, uint64_t n, uint32_t S, void *ws, unsigned int *repeats, hipStream_t s);
// Stream-mix ceiling (microbench.hip): n elements, read streams of ra / rb
// bytes, write streams of wa / wb bytes per element (0 = none), in order.
void streamMix(int ra, int rb, int wa, int wb, const void *a, const void *b, void *oa, void *ob, uint64_t n,
               unsigned long long *sink, hipStream_t s);
void copyKernel(const ulonglong2 *in, ulonglong2 *out, uint64_t n16, hipStream_t s);
void readKernel(const ulonglong2 *in, uint64_t n16, unsigned long long *sink, hipStream_t s);
void projectKeys(const ulonglong2 *in, uint64_t n, uint32_t shift, uint32_t *out, int ipt, hipStream_t s);
void probeBitmapGlobal(const ulonglong2 *in, uint64_t n, const uint32_t *bm, uint64_t keyMask,
                       unsigned long long *count, int ipt, hipStream_t s);
// In-process all-reduce step (comm/InProcessCommunicator): devBufs is a device
// array of the n ranks' buffers; element i in [lo, hi) of every buffer becomes
// the sum over ranks.
void sumSlices(uint64_t *const *devBufs, uint32_t n, uint64_t lo, uint64_t hi, hipStream_t s);
void gatherVariant(int mode, const uint64_t *rids, uint64_t n, const ulonglong2 *rows, ulonglong2 *out,
                   hipStream_t s);

}  // namespace kernels
}  // namespace hpcjoin

namespace hpcjoin {
namespace kernels {
// out[0] = max key, out[1] = max rid, out[2] = min rid over n tuples (device);
// out[0..1] must be zeroed and out[2] set to ~0.
void keyRidMax(const data::Tuple *in, uint64_t n, unsigned long long *out, hipStream_t s);
}  // namespace kernels
}  // namespace hpcjoin

namespace hpcjoin {
namespace kernels {
// ------------------------------------------------ late materialization
// Payload rows are ROW_WORDS x u64 (32 bytes), a pure function of (seed, rid).
constexpr uint32_t ROW_WORDS = 4;
HJ_HD uint64_t payloadWord(uint64_t seed, uint64_t rid, uint32_t w) {
  return mix64(seed * 0x9E3779B97F4A7C15ULL + rid * ROW_WORDS + w);
}
void generatePayload(uint64_t *rows, uint64_t n, uint64_t ridOffset, uint64_t seed, hipStream_t s);
// Requests for one side of the materialized pairs: x = owner | (pair index << 8), y = rid.
void makeRequests(const ulonglong2 *pairs, uint64_t n, int side, uint64_t ridsPerRank, uint32_t nodes,
                  ulonglong2 *req, hipStream_t s);
// After partitioning requests by owner: rids[j] = req[j].y, idx[j] = req[j].x >> 8.
void splitRequests(const ulonglong2 *req, uint64_t n, uint64_t *rids, uint64_t *idx, hipStream_t s);
// rowsOut[j] = payload[rids[j] - ridOffset]
void gatherRows(const uint64_t *rids, uint64_t n, uint64_t ridOffset, const uint64_t *payload, uint64_t *rowsOut,
                hipStream_t s);
// out[idx[j] * stride + col .. + ROW_WORDS) = rows[j]
// Single rank: out[i] = {pair, rowsA[pair.x - offA], rowsB[pair.y - offB]} (10 words).
void materializeLocal(const ulonglong2 *pairs, uint64_t n, const uint64_t *rowsA, uint64_t offA,
                      const uint64_t *rowsB, uint64_t offB, uint64_t *out, hipStream_t s, uint32_t variant = 1);
void placeRows(const uint64_t *rows, const uint64_t *idx, uint64_t n, uint64_t *out, uint32_t strideWords,
               uint32_t colWord, hipStream_t s);
// Every HIP source file is its own code object, loaded by the runtime at the
// first use of one of its kernels -- 1-2 ms each, which landed inside the
// first join.  ExecContext calls this once per process and device: one
// hipFuncGetAttributes per file loads them all up front.
void preloadPartition();
void preloadBuildProbe();
void preloadKeyTables();
void preloadBitmapJoin();
void preloadScan();
void preloadWire();
void preloadCollectives();
void preloadMaterialize();
void preloadDatagen();
inline void preloadCodeObjects() {
  preloadPartition();
  preloadBuildProbe();
  preloadKeyTables();
  preloadBitmapJoin();
  preloadScan();
  preloadWire();
  preloadCollectives();
  preloadMaterialize();
  preloadDatagen();
}

}  // namespace kernels
}  // namespace hpcjoin
