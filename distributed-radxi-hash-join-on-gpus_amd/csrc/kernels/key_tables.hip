// Key-only counting joins (JoinPlan::keyOnly: 63-bit keys, no rids) over
// resolved spans of the split local output: the v2 bucket table, the
// quotient table and counted tables.  Split out of build_probe.hip (the
// rid-carrying build/probe kernels); reference semantics as there
// (/root/reference/tasks/BuildProbe.cpp:81-106: exact key compare, every
// copy counted).
#include "kernels.h"
#include "device_common.h"

#include <algorithm>

namespace hpcjoin {
namespace kernels {

constexpr int KT_EMIT_T = 256;

// ---------------------------------------------------------------- key-only
// Key-only 8-byte words (JoinPlan::keyOnly: wide keys, no rids) are counted
// over resolved spans below: the v2 bucket table (keyCount 7), the quotient
// table (8) and counted tables (9).  Round 2's per-item kernels (variants
// 0-6) were pruned in round 4; measurements in profiles/r2v, profiles/r3k.
constexpr uint32_t BPK_SLOTS = 4;

// ------------------------------------------------------- key-only spans (v2)
// The key-only count as a work queue of resolved spans.  Measured on the
// item kernel above (1B x 1B sparse keys, 4.93 ms, 3.3 TB/s, 63 % wait):
// every item started with a chain of dependent scalar loads (item -> four
// partition bounds) and only then issued its data loads, so each workgroup
// paid ~3 memory latencies per ~30 KB item.  Here
//  * spans carry their resolved bounds (bpEmitSpans), 32 B each;
//  * a workgroup grabs KS_CHUNK consecutive spans from a device counter
//    (dynamic: hot partitions' spans spread over workgroups), stages their
//    descriptors in LDS with one load, and walks them in order;
//  * the next span's inner and outer words are loaded into registers while
//    the current span probes, so its latency hides behind the LDS work;
//  * loads are unpredicated (indices clamped into the span) and the bucket
//    hash is one 32-bit multiply of the folded word (the 64-bit product of
//    hash64 is three quarter-rate multiplies).
// Table: the same 4-slot buckets + fill counters as bpKeyCountKernel.
constexpr uint32_t KS_CHUNK = 32;
// Spans a counted-table workgroup takes from its queue at a time.  Counted
// spans are few on unique keys (the partitions just above rChunk: ~360 at
// 1B x 1B) and each costs ~4 us: grabbing 32 at a time left 12 workgroups
// working through them one after another (0.124 ms per join).
constexpr uint32_t KC_GRAB = 4;

__global__ __launch_bounds__(KT_EMIT_T) void bpEmitSpansKernel(const uint64_t *__restrict__ partR,
                                                         const uint64_t *__restrict__ partREnd,
                                                         const uint64_t *__restrict__ partS,
                                                         const uint64_t *__restrict__ partSEnd, uint32_t P,
                                                         uint32_t rc, uint32_t sc, const uint32_t *__restrict__ counts,
                                                         const uint32_t *__restrict__ offsets, BPSpan *spans,
                                                         uint32_t capacity) {
  const uint32_t p = blockIdx.x * KT_EMIT_T + threadIdx.x;
  if (p >= P) return;
  const uint32_t c = counts[p];
  if (c == 0) return;
  const uint64_t r0 = partR[p], r1 = partREnd[p], s0 = partS[p], s1 = partSEnd[p];
  const uint32_t nsChunks = (uint32_t)ceilDiv(s1 - s0, sc);
  const uint32_t o = offsets[p];
  for (uint32_t i = 0; i < c && o + i < capacity; ++i) {
    const uint64_t rb = r0 + (uint64_t)(i / nsChunks) * rc, sb = s0 + (uint64_t)(i % nsChunks) * sc;
    BPSpan sp;
    sp.rb = rb;
    sp.sb = sb;
    sp.nr = (uint32_t)(min(r1, rb + rc) - rb);
    sp.ns = (uint32_t)(min(s1, sb + sc) - sb);
    sp.flags = sp.pad1 = 0;
    spans[o + i] = sp;
  }
}

void bpEmitSpans(const BPArgs &a, const uint32_t *counts, const uint32_t *offsets, BPSpan *spans, uint32_t capacity,
                 hipStream_t s) {
  if (a.P == 0) return;
  hipLaunchKernelGGL(bpEmitSpansKernel, dim3(ceilDiv(a.P, KT_EMIT_T)), dim3(KT_EMIT_T), 0, s, a.partR,
                     a.partREnd ? a.partREnd : a.partR + 1, a.partS, a.partSEnd ? a.partSEnd : a.partS + 1, a.P,
                     a.rChunk, a.sChunk, counts, offsets, spans, capacity);
  HIP_CHECK_LAUNCH();
}

// Bucket of a key-only word: fold the high half in with a 24-bit multiply
// (full rate), one 32-bit multiplicative hash of the result.  Within a final
// partition the word's low localBits bits are equal: they only offset the
// product, whose top bits still come from the varying bits above them.
__device__ __forceinline__ uint32_t ksBucket(uint64_t w, uint32_t bbits) {
  const uint32_t x = (uint32_t)w ^ __umul24((uint32_t)(w >> 32), 0x2C1B3Cu);
  return (x * 0x9E3779B1u) >> (32 - bbits);
}

// K words of a span per lane (indices clamped into the span: no predication).
// Split layout (SplitLayout::loShift = localBits): the u32 low column and the
// u16 high column compose the key fragment lo | hi << 32.
template <int T, int K, bool SPLIT>
struct KsSrc {
  const void *lo;
  const uint16_t *hi;
  __device__ __forceinline__ void load(uint64_t base, uint32_t n, uint64_t (&v)[K]) const {
    const uint32_t last = n ? n - 1 : 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t i = base + min((uint32_t)(k * T) + threadIdx.x, last);
      if constexpr (SPLIT)
        v[k] = (uint64_t)__builtin_nontemporal_load(static_cast<const uint32_t *>(lo) + i) |
               ((uint64_t)__builtin_nontemporal_load(hi + i) << 32);
      else
        v[k] = __builtin_nontemporal_load(static_cast<const uint64_t *>(lo) + i);
    }
  }
};

// The bucket table: 4 slots (32 B) per bucket, stored SoA: all first 16-byte
// halves, then all second halves, so a random ds_read_b128 starts at one of
// 16 bank quads instead of 8 (32-byte AoS buckets, round 3's variant 6):
// half the expected lane collisions per 16-lane group.
struct KsTable {
  unsigned long long *t;
  uint32_t maxBuckets;
  __device__ __forceinline__ const ulonglong2 *half(uint32_t b, int h) const {
    return reinterpret_cast<const ulonglong2 *>(t + (h ? 2 * maxBuckets : 0)) + b;
  }
  __device__ __forceinline__ unsigned long long &slot(uint32_t b, uint32_t p) const {
    return t[(p >> 1) * 2 * maxBuckets + 2 * b + (p & 1)];
  }
};

// One batch of T x K outer words (the first `valid` of them counted) against
// the bucketized table; returns this lane's matches.
template <int T, int K, int H>
__device__ __forceinline__ uint32_t ksProbeBatch(const uint64_t (&sv)[K], uint32_t valid, const KsTable &table,
                                                 const uint32_t *fill, uint32_t bbits, uint32_t bmask) {
  uint32_t matches = 0;
#pragma unroll
  for (int h = 0; h < K / H; ++h) {
    uint32_t bk[H], f[H];
    ulonglong2 e0[H], e1[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
      bk[j] = ksBucket(sv[h * H + j], bbits);
      f[j] = fill[bk[j]];
      e0[j] = *table.half(bk[j], 0);
      e1[j] = *table.half(bk[j], 1);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const int k = h * H + j;
      const uint64_t v = sv[k];
      const uint32_t m = f[j];  // slots in use (> 4: passed through)
      // Non-short-circuit tests: the whole 32-byte bucket is read up front.
      uint32_t c = (uint32_t)((m > 0) & (e0[j].x == v)) + (uint32_t)((m > 1) & (e0[j].y == v)) +
                   (uint32_t)((m > 2) & (e1[j].x == v)) + (uint32_t)((m > 3) & (e1[j].y == v));
      // Elements passed through (~4 % of buckets at load 1/2, so most waves
      // have a lane here): continue bucket by bucket, each step one round
      // trip (counter and both halves of the bucket read together).
      uint32_t b = bk[j], fb = m;
      while (fb > BPK_SLOTS) {
        b = (b + 1) & bmask;
        fb = fill[b];
        const ulonglong2 x0 = *table.half(b, 0), x1 = *table.half(b, 1);
        c += (uint32_t)((fb > 0) & (x0.x == v)) + (uint32_t)((fb > 1) & (x0.y == v)) +
             (uint32_t)((fb > 2) & (x1.x == v)) + (uint32_t)((fb > 3) & (x1.y == v));
      }
      matches += (uint32_t)(k * T) + threadIdx.x < valid ? c : 0u;
    }
  }
  return matches;
}

template <int T, int K, int H, int MINW, bool SPLIT>
__global__ __launch_bounds__(T, MINW) void bpKeySpanKernel(KsSrc<T, K, SPLIT> R, KsSrc<T, K, SPLIT> S,
                                                           const BPSpan *__restrict__ spans,
                                                           const uint32_t *__restrict__ nSpansPtr, uint32_t capacity,
                                                           uint32_t *__restrict__ queue, uint32_t maxR,
                                                           unsigned long long *__restrict__ result) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t maxSlots = 1u << ceilLog2(2ull * maxR);
  const KsTable table{reinterpret_cast<unsigned long long *>(smem), maxSlots / BPK_SLOTS};
  uint32_t *fill = reinterpret_cast<uint32_t *>(table.t + maxSlots);
  BPSpan *desc = reinterpret_cast<BPSpan *>(fill + maxSlots / BPK_SLOTS);
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(desc + KS_CHUNK);
  uint32_t *qbase = reinterpret_cast<uint32_t *>(wsum + T / WAVE);
  constexpr uint32_t BATCH = T * K;
  const uint32_t t = threadIdx.x;
  const uint32_t n = min(*nSpansPtr, capacity);
  uint64_t matches = 0;
  uint64_t rv[K], sv[K], nrv[K], nsv[K];
  for (;;) {
    if (t == 0) *qbase = atomicAdd(queue, KS_CHUNK);
    __syncthreads();
    const uint32_t base = __builtin_amdgcn_readfirstlane(*qbase);
    if (base >= n) break;
    const uint32_t cnt = min(KS_CHUNK, n - base);
    if (t < cnt) desc[t] = spans[base + t];
    __syncthreads();
    {
      const BPSpan d = desc[0];
      R.load(d.rb, d.nr, rv);
      S.load(d.sb, d.ns, sv);
    }
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint64_t rb = uniform64(desc[i].rb);
      const uint64_t sb = uniform64(desc[i].sb);
      const uint32_t nr = __builtin_amdgcn_readfirstlane(desc[i].nr);
      const uint32_t ns = __builtin_amdgcn_readfirstlane(desc[i].ns);
      uint32_t tbits = nr > 1 ? 32 - __clz(2 * nr - 1) : 1;
      if (tbits < 6) tbits = 6;
      const uint32_t bbits = tbits - 2, bmask = (1u << bbits) - 1;
      for (uint32_t j = t; j <= bmask; j += T) fill[j] = 0;
      __syncthreads();
      // ---- build (nr <= maxR <= BATCH: one batch, from registers)
      {
        uint32_t bk[K], pos[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool valid = (uint32_t)(k * T) + t < nr;
          bk[k] = ksBucket(rv[k], bbits);
          pos[k] = atomicAdd(&fill[bk[k]], valid ? 1u : 0u);
          pos[k] = valid ? pos[k] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (pos[k] == 0xFFFFFFFFu) continue;
          uint32_t b = bk[k], p = pos[k];
          while (p >= BPK_SLOTS) {  // home bucket full: the next one (its counter marks the pass)
            b = (b + 1) & bmask;
            p = atomicAdd(&fill[b], 1u);
          }
          table.slot(b, p) = rv[k];
        }
      }
      __syncthreads();
      // ---- the next span's words stream in while this one probes
      if (i + 1 < cnt) {
        const BPSpan d = desc[i + 1];
        R.load(d.rb, d.nr, nrv);
        S.load(d.sb, d.ns, nsv);
      }
      // ---- probe: the first batch from registers (no wait on the prefetch
      // above: vmcnt is in order, so a load issued here would make the first
      // use wait for the next span's words too), later batches loaded inline.
      matches += ksProbeBatch<T, K, H>(sv, ns, table, fill, bbits, bmask);
      for (uint32_t b0 = BATCH; b0 < ns; b0 += BATCH) {
        uint64_t xv[K];
        S.load(sb + b0, ns - b0, xv);
        matches += ksProbeBatch<T, K, H>(xv, ns - b0, table, fill, bbits, bmask);
      }
      __syncthreads();  // the next span clears the counters
#pragma unroll
      for (int k = 0; k < K; ++k) {
        rv[k] = nrv[k];
        sv[k] = nsv[k];
      }
    }
  }
  const unsigned long long total = blockReduceSum<T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(result, total);
}

// ------------------------------------------- key-only spans, quotient table (v4)
// KernelVariants::keyCount 8.  A key fragment of f <= 32 + KQ_BITS bits
// (63-bit keys after 10 + 9 radix bits: f = 44) is split into
//   v = frag >> s (32 bits, s = f - 32)   and   lo = frag's low s bits;
//   home bucket b = (lo ^ h(v)) mod 2^KQ_BITS   (h: multiplicative hash of v),
// and the bucket stores only v: (b, v) determines the fragment (lo = b ^ h(v)
// on its low s bits), so a slot is 4 bytes.
//
// Layout (round 4): 4096 buckets x 4 u32 slots, stored as two 8-byte halves
// (slots 0-1 of every bucket, then slots 2-3: a random ds_read_b64 starts at
// one of 32 bank pairs), plus a u16 fill count per bucket.  A build is one
// LDS atomic add on the bucket's count (its old value is the slot) and one
// store; a probe reads the count and both halves (three LDS reads, no loop)
// and compares the first `fill` slots.  Slots are never cleared -- the count
// says which hold keys -- so there is no empty marker and no escape value:
// every 32-bit v is a key.  (Round 3's two-slot buckets at ~1/2 load sent
// ~37 % of probes, so nearly every wave, into an overflow walk: PMC showed the
// kernel VALU-bound at 43 VALU instructions per word.)
//
// Exactness: (b, v) names a key only in its home bucket, and a key never
// leaves it: the fifth and later keys of a bucket (~0.2 % of probes at 2048
// keys per span) go to a small overflow table of full 48-bit fragments
// (KQ_OV entries, linear probing, compared whole), read only when the home
// bucket's count exceeds 4.  More than KQ_OV_CAP overflow keys in one span --
// a key with hundreds of copies in a light partition -- stops inserting and
// sets KQF_COUNTED: the count is void and the join's build/probe re-runs on
// counted tables.  (Round 3 let keys spill into the next bucket, where a
// stored v of another home could equal the probe's.)
//
// Counted tables (bpKeyCountedSpansKernel) keep a salted stored value with an
// empty marker: kqSalt / kqKey below.
constexpr uint32_t KQ_BITS = 12;
constexpr uint32_t KQ_BUCKETS = 1u << KQ_BITS;
constexpr uint32_t KQ_SLOTS = 4;
constexpr uint32_t KQ_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t KQ_OV_BITS = 9;
constexpr uint32_t KQ_OV = 1u << KQ_OV_BITS;  // overflow entries (4 KiB)
constexpr uint32_t KQ_OV_CAP = 3 * KQ_OV / 4;  // at most this many inserted: probes always find an empty entry
constexpr unsigned long long KQ_OV_EMPTY = ~0ull;  // fragments are < 2^48
// A placement that walked past this many overflow entries saw one key's
// copies chained (unique keys at <= 25 % overflow load never do): KQF_CHAINS,
// and later joins put every partition on counted spans (keyCount 9).
constexpr uint32_t KQ_LONG_CHAIN = 64;
// BPArgs::sideOverflow bits.
constexpr unsigned long long KQF_CHAINS = 2;   // copies of a key chained (count exact)
constexpr unsigned long long KQF_COUNTED = 8;  // quotient overflow table full: count void, re-run counted

// Quotient-table key of a fragment: (home bucket, stored value).  v is bits
// [s, s + 32) of the fragment: one v_alignbit of its two halves.
__device__ __forceinline__ void kq4Key(uint64_t frag, uint32_t s, uint32_t &b, uint32_t &v) {
  v = __builtin_amdgcn_alignbit((uint32_t)(frag >> 32), (uint32_t)frag, s);
  const uint32_t lo = (uint32_t)frag & ((1u << s) - 1u);
  b = (lo ^ ((v * 0x9E3779B1u) >> (32 - KQ_BITS))) & (KQ_BUCKETS - 1);
}

__device__ __forceinline__ uint32_t kqSalt(uint32_t b) { return (b + 1u) * 0x85EBCA77u; }

// (bucket, stored value, tag) of a fragment of f <= 48 bits; s = f - 32
// (0 when f <= 32).  The bucket absorbs the low KQ_BITS of lo, the tag holds
// the rest of lo (f > 44 only: counted tables keep it next to the count).
__device__ __forceinline__ void kqKey(uint64_t frag, uint32_t s, uint32_t &b, uint32_t &v, uint32_t &tag) {
  const uint32_t e = (uint32_t)(frag >> s);
  const uint32_t lo = (uint32_t)frag & ((1u << s) - 1u);
  b = (lo ^ ((e * 0x9E3779B1u) >> (32 - KQ_BITS))) & (KQ_BUCKETS - 1);
  tag = lo >> KQ_BITS;
  v = e ^ kqSalt(b);
}

// Overflow-table home of a key from its (bucket, stored value): (b, v) is a
// bijection of the fragment, so one 32-bit multiply spreads keys as well as
// hashing the whole fragment would.
__device__ __forceinline__ uint32_t kqOvHash(uint32_t b, uint32_t v) {
  return ((v ^ (b << 20)) * 0x9E3779B1u) >> (32 - KQ_OV_BITS);
}

// Copies of `frag` (home h) in the overflow table (it holds < KQ_OV entries).
__device__ __forceinline__ uint32_t kqOvCount(const unsigned long long *ov, uint32_t h, uint64_t frag) {
  uint32_t c = 0;
  for (uint32_t w = 0; w < KQ_OV; ++w) {
    const unsigned long long y = ov[h];
    if (y == KQ_OV_EMPTY) break;
    c += y == frag;
    h = (h + 1) & (KQ_OV - 1);
  }
  return c;
}

// Overflow placement; at the table's cap nothing is placed and full = true
// (the span's count is void).
__device__ __forceinline__ void kqOvInsert(unsigned long long *ov, uint32_t *ovN, uint32_t h, uint64_t frag,
                                           bool &chained, bool &full) {
  if (atomicAdd(ovN, 1u) >= KQ_OV_CAP) {
    full = true;
    return;
  }
  for (uint32_t w = 0;; ++w) {  // < KQ_OV_CAP entries taken: an empty one exists
    if (atomicCAS(&ov[h], KQ_OV_EMPTY, (unsigned long long)frag) == KQ_OV_EMPTY) {
      chained |= w > KQ_LONG_CHAIN;
      return;
    }
    h = (h + 1) & (KQ_OV - 1);
  }
}

// One batch of T x K outer fragments (the first `valid` counted) against the
// four-slot table: the count and slots 0-1 for every probe; slots 2-3 only
// in lanes whose bucket holds more than two keys (~8 % at 2048 keys per
// span: an exec-masked read costs the LDS pipe a few lanes, not 64 -- the
// kernel is LDS-pipe bound, PMC profiles/r4p); the overflow table past four.
template <int T, int K>
__device__ __forceinline__ uint32_t kq4ProbeBatch(const uint64_t (&pv)[K], uint32_t valid, uint32_t s,
                                                  const uint2 *h0, const uint2 *h1, const uint16_t *fill,
                                                  const unsigned long long *ov) {
  uint32_t bk[K], v[K], f[K];
  uint2 x[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    kq4Key(pv[k], s, bk[k], v[k]);
    f[k] = fill[bk[k]];
    x[k] = h0[bk[k]];
  }
  uint32_t matches = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint32_t c = (uint32_t)(f[k] > 0 && x[k].x == v[k]) + (uint32_t)(f[k] > 1 && x[k].y == v[k]);
    if (f[k] > 2) {
      const uint2 y = h1[bk[k]];
      c += (uint32_t)(y.x == v[k]) + (uint32_t)(f[k] > 3 && y.y == v[k]);
      if (f[k] > KQ_SLOTS) c += kqOvCount(ov, kqOvHash(bk[k], v[k]), pv[k]);
    }
    matches += (uint32_t)(k * T) + threadIdx.x < valid ? c : 0u;
  }
  return matches;
}

// Counted table (bpKeyCountedSpansKernel): 3072 buckets of two 8-byte
// entries (one 16-byte ds_read_b128 reads a bucket) and a u32 count per entry
// apart (one ds_read_b64 per bucket).  Entry = one distinct key:
//   lo = stored value v, hi = b << 20 | tag << 16 | ovf,
// (b, v, tag) from kqKey, a bijection of the fragment, so an entry names its
// key wherever it sits and never equals the empty word ~0 (hi bits 1-15 are
// zero).  A key claims the first empty entry of its home bucket (64-bit CAS),
// then walks the following buckets (linear probing over entries); a key that
// leaves its home sets the home's ovf bit (entry 0 of a full bucket).  A probe
// reads the home bucket and its counts together: a hit in either entry adds
// the count; only lanes whose home bucket overflowed walk, behind a scalar
// any().  At 2048 keys in 3072 buckets ~5 % of keys leave their home (the
// round-5 layout, one entry per home at 4096 homes in 6144 entries, displaced
// ~21 %, and every probe walk re-read one 8-byte entry per step).
constexpr uint32_t KC_B = 3072;
constexpr uint32_t KC_E = 2 * KC_B;
__device__ __forceinline__ uint32_t kcBucket(uint64_t frag, uint32_t s) {
  const uint32_t h = (uint32_t)(frag >> s) * 0x9E3779B1u ^ ((uint32_t)frag & ((1u << s) - 1u)) * 0x85EBCA77u;
  return __umulhi(h ^ (h >> 15), KC_B);
}
__device__ __forceinline__ uint32_t kcHi(uint32_t b, uint32_t tag) { return (b << 20) | (tag << 16); }
constexpr uint32_t KC_EMPTY_HI = 0xFFFFFFFFu;

template <int T, int K>
__device__ __forceinline__ uint64_t kqProbeCounted(const uint64_t (&pv)[K], uint32_t valid, uint32_t s,
                                                   const uint4 *tab4, const uint2 *cnt2) {
  uint32_t hb[K], v[K], hk[K];
  uint4 x[K];
  uint2 c[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint32_t b, tg;
    kqKey(pv[k], s, b, v[k], tg);
    hk[k] = kcHi(b, tg);
    hb[k] = kcBucket(pv[k], s);
    x[k] = tab4[hb[k]];
    c[k] = cnt2[hb[k]];
  }
  uint64_t matches = 0;
  bool walk[K];
  bool any = false;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const bool h0 = x[k].x == v[k] && (x[k].y & ~1u) == hk[k];
    const bool h1 = x[k].z == v[k] && x[k].w == hk[k];
    const bool counted = (uint32_t)(k * T) + threadIdx.x < valid;
    matches += counted ? (h0 ? c[k].x : h1 ? c[k].y : 0u) : 0u;
    walk[k] = !h0 && !h1 && counted && (x[k].y & 1u) != 0 && x[k].y != KC_EMPTY_HI;
    any |= walk[k];
  }
  if (__any(any)) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      uint32_t b = hb[k];
      bool w = walk[k];
      for (uint32_t step = 1; w && step < KC_B; ++step) {
        b = b + 1 == KC_B ? 0u : b + 1;
        const uint4 y = tab4[b];
        if (y.x == v[k] && (y.y & ~1u) == hk[k]) {
          matches += cnt2[b].x;
          break;
        }
        if (y.z == v[k] && y.w == hk[k]) {
          matches += cnt2[b].y;
          break;
        }
        w = y.y != KC_EMPTY_HI && y.w != KC_EMPTY_HI;
      }
    }
  }
  return matches;
}

size_t bpKeyQuotientLdsBytes() {
  return KQ_BUCKETS * KQ_SLOTS * 4 + KQ_BUCKETS * 2 + KQ_OV * 8 + 16 + KS_CHUNK * sizeof(BPSpan) + 16 * 8 + 16;
}

// T = 1024, K = 2: a span's <= 2048 inner words are one register batch.  The
// ~77 KiB table admits two workgroups per CU: 32 waves, as the round-3
// 512-thread kernel had at 4 workgroups.
template <int T, int K, int MINW>
__global__ __launch_bounds__(T, MINW) void bpKeyQuotientKernel(KsSrc<T, K, true> R, KsSrc<T, K, true> S,
                                                               const BPSpan *__restrict__ spans,
                                                               const uint32_t *__restrict__ nSpansPtr,
                                                               uint32_t capacity, uint32_t *__restrict__ queue,
                                                               uint32_t s, unsigned long long *__restrict__ result,
                                                               unsigned long long *__restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *slots = reinterpret_cast<uint32_t *>(smem);  // [half][bucket][2]
  const uint2 *h0 = reinterpret_cast<const uint2 *>(smem);
  const uint2 *h1 = h0 + KQ_BUCKETS;
  uint16_t *fill = reinterpret_cast<uint16_t *>(slots + KQ_BUCKETS * KQ_SLOTS);
  uint32_t *fill2 = reinterpret_cast<uint32_t *>(fill);  // two counts per word (atomics)
  unsigned long long *ov = reinterpret_cast<unsigned long long *>(fill + KQ_BUCKETS);
  uint32_t *ovN = reinterpret_cast<uint32_t *>(ov + KQ_OV);
  BPSpan *desc = reinterpret_cast<BPSpan *>(ovN + 4);
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(desc + KS_CHUNK);
  uint32_t *qbase = reinterpret_cast<uint32_t *>(wsum + T / WAVE);
  constexpr uint32_t BATCH = T * K;
  const uint32_t t = threadIdx.x;
  const uint32_t n = min(*nSpansPtr, capacity);
  auto clearFill = [&]() {
    for (uint32_t i = t; i < KQ_BUCKETS / 4; i += T) reinterpret_cast<uint2 *>(fill2)[i] = make_uint2(0u, 0u);
  };
  clearFill();
  for (uint32_t i = t; i < KQ_OV; i += T) ov[i] = KQ_OV_EMPTY;
  if (t == 0) *ovN = 0;
  uint64_t matches = 0;
  bool full = false, chained = false;
  // Spans i + 1 and i + 2 are in flight while span i builds and probes (a
  // span is ~2.6 us of a workgroup's time at two workgroups per CU; the loads
  // of the next span alone, issued after the build, did not cover HBM latency
  // under load).  Three register sets in fixed roles (the span loop unrolled
  // by three): a copy between sets would make the compiler wait for the
  // copied loads (vmcnt(0)) at the end of every span.  Every load is issued
  // unconditionally -- past the chunk's end it re-reads its last span -- so
  // the waits stay counted.
  uint64_t ra[K], sa[K], rb[K], sb[K], rc[K], sc[K];
  auto loadSpan = [&](const BPSpan &d, uint64_t (&rr)[K], uint64_t (&ss)[K]) {
    R.load(d.rb, d.nr, rr);
    S.load(d.sb, d.ns, ss);
  };
  // Span i from (rv, sv); span i + 2 loads into (rn, sn), the set span i - 1 used.
  auto span = [&](uint32_t i, uint32_t cnt, const uint64_t (&rv)[K], const uint64_t (&sv)[K], uint64_t (&rn)[K],
                  uint64_t (&sn)[K]) {
    const uint64_t s0 = uniform64(desc[i].sb);
    const uint32_t nr = __builtin_amdgcn_readfirstlane(desc[i].nr);
    const uint32_t ns = __builtin_amdgcn_readfirstlane(desc[i].ns);
    // ---- build (nr <= BATCH: one batch, from registers): the old count is the slot
#pragma unroll
    for (int k = 0; k < K; ++k) {
      uint32_t b, v;
      kq4Key(rv[k], s, b, v);
      if ((uint32_t)(k * T) + t >= nr) continue;
      const uint32_t sh = (b & 1u) * 16u;
      const uint32_t slot = (atomicAdd(&fill2[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
      if (slot < KQ_SLOTS)
        slots[(slot >> 1) * (2 * KQ_BUCKETS) + 2 * b + (slot & 1u)] = v;
      else
        kqOvInsert(ov, ovN, kqOvHash(b, v), rv[k], chained, full);
    }
    __syncthreads();
    const bool ovUsed = __builtin_amdgcn_readfirstlane(*ovN) != 0;  // no insert until the next build
    loadSpan(desc[min(i + 2, cnt - 1)], rn, sn);
    // ---- probe: first batch from registers, later batches loaded inline
    matches += kq4ProbeBatch<T, K>(sv, ns, s, h0, h1, fill, ov);
    for (uint32_t b0 = BATCH; b0 < ns; b0 += BATCH) {
      uint64_t xv[K];
      S.load(s0 + b0, ns - b0, xv);
      matches += kq4ProbeBatch<T, K>(xv, ns - b0, s, h0, h1, fill, ov);
    }
    __syncthreads();  // every probe of this span is done
    clearFill();      // (slots keep stale keys: the counts hide them)
    if (ovUsed) {
      for (uint32_t j = t; j < KQ_OV; j += T) ov[j] = KQ_OV_EMPTY;
      if (t == 0) *ovN = 0;
    }
    __syncthreads();  // table empty again before the next build
  };
  for (;;) {
    if (t == 0) *qbase = atomicAdd(queue, KS_CHUNK);
    __syncthreads();  // (first round: also orders the table clear before any build)
    const uint32_t base = __builtin_amdgcn_readfirstlane(*qbase);
    if (base >= n) break;
    const uint32_t cnt = min(KS_CHUNK, n - base);
    if (t < cnt) desc[t] = spans[base + t];
    __syncthreads();
    loadSpan(desc[0], ra, sa);
    loadSpan(desc[min(1u, cnt - 1)], rb, sb);
    for (uint32_t i = 0; i < cnt; i += 3) {
      span(i, cnt, ra, sa, rc, sc);
      if (i + 1 < cnt) span(i + 1, cnt, rb, sb, ra, sa);
      if (i + 2 < cnt) span(i + 2, cnt, rc, sc, rb, sb);
    }
  }
  const unsigned long long total = blockReduceSum<T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(result, total);
  if (__any(full) && (t & (WAVE - 1)) == 0) atomicOr(flags, KQF_COUNTED);
  if (__any(chained) && (t & (WAVE - 1)) == 0) atomicOr(flags, KQF_CHAINS);
}

bool bpKeyQuotientFits(const BPArgs &a) {
  return bpKeyCountedFits(a) && a.keyFragBits <= 32 + KQ_BITS;
}

bool bpKeyCountedFits(const BPArgs &a) {
  return a.keyOnly && a.split && !a.materialize && !a.wide && a.keyFragBits >= 1 && a.keyFragBits <= 48 &&
         a.rChunk <= 2048;
}

static void launchKeyQuotient(const BPArgs &a, const BPSpan *spans, const uint32_t *nSpans, uint32_t capacity,
                              uint32_t *queue, hipStream_t st) {
  constexpr int T = 1024, K = 2;
  HJ_CHECK(bpKeyQuotientFits(a), "buildProbeKeySpans: quotient table needs split key-only words of <= %u bits "
           "(got %u) and rChunk <= 2048 (got %u)", 32 + KQ_BITS, a.keyFragBits, a.rChunk);
  HJ_CHECK(a.sideOverflow, "buildProbeKeySpans: quotient table needs a flag word");
  const uint32_t s = a.keyFragBits > 32 ? a.keyFragBits - 32 : 0;
  const size_t lds = bpKeyQuotientLdsBytes();
  const uint32_t perCu = (uint32_t)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
  const dim3 grid(std::min<uint32_t>(ceilDiv(capacity, KS_CHUNK), 256 * perCu));
  HIP_CHECK(hipMemsetAsync(queue, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL((bpKeyQuotientKernel<T, K, 8>), grid, dim3(T), lds, st, KsSrc<T, K, true>{a.R, a.Rhi},
                     KsSrc<T, K, true>{a.S, a.Shi}, spans, nSpans, capacity, queue, s, a.result, a.sideOverflow);
  HIP_CHECK_LAUNCH();
}

// ------------------------------------- key-only: partitions with repeated keys
// Partitions with more than rChunk inner tuples (with unique keys a few in a
// thousand, just above the mean; with repeated keys the hot ones) skip the
// span work queue, whose one-slot-per-tuple quotient table holds every copy
// of a key.  Their spans (bpPlanCounts -> heavySpans, same rChunk x sChunk
// tiling) are counted here on a *counted* table (see kqProbeCounted): one
// entry per distinct key, so copies only add to a count.  A span's <= 2048
// inner words fill at most a third of the 6144 entries.  The table also
// carries 45-48-bit fragments (the tag in the entry) and every 32-bit stored
// value (the empty word is not a key's), so it never needs a fallback: plans whose fragments the quotient table cannot
// hold, and quotient spans that filled their overflow table, count here.  A
// hot partition's spans spread over workgroups like any others.
//
// Compacted spans (BPSpan::flags bit 0, from bpKeyDedup): the inner words are
// distinct keys with a count each in BPArgs::dedupCounts, added whole.  A hot
// key's million copies then cost one table entry instead of ~500 inner
// chunks each re-reading the partition's outer side.
// Structure as bpKeyQuotientKernel (T = 1024, K = 2): spans from a work queue
// in chunks of KS_CHUNK, spans i + 1 and i + 2 in flight while span i builds
// and probes, the span loop unrolled by three over fixed register sets.  The
// table is 72 KiB with the counts; 1024-thread workgroups at <= 64 VGPRs put
// two on a CU.
template <int T, int K, int MINW>
__global__ __launch_bounds__(T, MINW) void bpKeyCountedSpansKernel(KsSrc<T, K, true> R, KsSrc<T, K, true> S,
                                                                    const uint32_t *__restrict__ rCounts,
                                                                    const BPSpan *__restrict__ spans,
                                                                    const uint32_t *__restrict__ nSpansPtr,
                                                                    uint32_t capacity, uint32_t *__restrict__ queue,
                                                                    uint32_t s, unsigned long long *__restrict__ result) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long *tab64 = reinterpret_cast<unsigned long long *>(smem);  // [entry] value | hi << 32
  const uint4 *tab4 = reinterpret_cast<const uint4 *>(smem);                 // [bucket]
  uint32_t *cnt = reinterpret_cast<uint32_t *>(tab64 + KC_E);                // [entry] count
  const uint2 *cnt2 = reinterpret_cast<const uint2 *>(cnt);                 // [bucket]
  BPSpan *desc = reinterpret_cast<BPSpan *>(cnt + KC_E);
  unsigned long long *wsum = reinterpret_cast<unsigned long long *>(desc + KS_CHUNK);
  uint32_t *qbase = reinterpret_cast<uint32_t *>(wsum + T / WAVE);
  constexpr uint32_t BATCH = T * K;
  const uint32_t t = threadIdx.x;
  const uint32_t n = __builtin_amdgcn_readfirstlane(min(*nSpansPtr, capacity));
  // Workgroups past the spans' chunk count have nothing to take from the
  // queue: they leave before clearing a 72 KiB table (with no heavy spans --
  // unique keys -- the whole launch of 512 groups cost ~0.12 ms per join).
  // The remaining groups drain the queue (a group may take several chunks).
  if (blockIdx.x >= (n + KC_GRAB - 1) / KC_GRAB) return;  // uniform per workgroup
  {
    uint4 *t4 = reinterpret_cast<uint4 *>(smem);  // entries (all ones) then counts (zero)
    for (uint32_t i = t; i < KC_E * 12 / 16; i += T)
      t4[i] = i < KC_E / 2 ? make_uint4(KQ_EMPTY, KQ_EMPTY, KQ_EMPTY, KQ_EMPTY) : make_uint4(0, 0, 0, 0);
  }
  uint64_t matches = 0;
  uint64_t ra[K], sa[K], rb[K], sb[K], rc[K], sc[K];
  auto loadSpan = [&](const BPSpan &d, uint64_t (&rr)[K], uint64_t (&ss)[K]) {
    R.load(d.rb, d.nr, rr);
    S.load(d.sb, d.ns, ss);
  };
  auto span = [&](uint32_t i, uint32_t nc, const uint64_t (&rv)[K], const uint64_t (&sv)[K], uint64_t (&rn)[K],
                  uint64_t (&sn)[K]) {
    const uint64_t r0 = uniform64(desc[i].rb), s0 = uniform64(desc[i].sb);
    const uint32_t nr = __builtin_amdgcn_readfirstlane(desc[i].nr);
    const uint32_t ns = __builtin_amdgcn_readfirstlane(desc[i].ns);
    const bool compacted = __builtin_amdgcn_readfirstlane(desc[i].flags) & 1u;
    // ---- build: nr <= rChunk <= BATCH, one pass
    uint32_t used[K];  // the entry each lane claimed or added to: cleared after the probe
#pragma unroll
    for (int k = 0; k < K; ++k) {
      used[k] = KC_E;
      if ((uint32_t)(k * T) + t >= nr) continue;
      uint32_t add = 1;
      if (compacted) add = rCounts[r0 + (uint32_t)(k * T) + t];
      uint32_t b, v, tg;
      kqKey(rv[k], s, b, v, tg);
      const uint32_t hi = kcHi(b, tg);
      const unsigned long long mine = ((unsigned long long)hi << 32) | v;
      // <= 2048 distinct keys in 6144 entries: an empty entry is always
      // reached.  The home bucket's two entries first, straight-line (~95 % of
      // keys end there); a lane whose home is full walks on and marks it.
      const uint32_t e0 = 2 * kcBucket(rv[k], s);
      auto mineOrClaimed = [&](unsigned long long o) {
        return o == ~0ull || ((uint32_t)o == v && ((uint32_t)(o >> 32) & ~1u) == hi);
      };
      uint32_t e = e0;
      bool placed = mineOrClaimed(atomicCAS(&tab64[e], ~0ull, mine));
      if (!placed) {
        e = e0 + 1;
        placed = mineOrClaimed(atomicCAS(&tab64[e], ~0ull, mine));
      }
      if (!placed) {
        atomicOr(&tab64[e0], 1ull << 32);  // the home bucket is full: mark it overflowed
        for (uint32_t step = 2; step < KC_E && !placed; ++step) {
          e = e + 1 == KC_E ? 0u : e + 1;
          placed = mineOrClaimed(atomicCAS(&tab64[e], ~0ull, mine));
        }
      }
      atomicAdd(&cnt[e], add);
      used[k] = e;
    }
    __syncthreads();
    loadSpan(desc[min(i + 2, nc - 1)], rn, sn);
    // ---- probe: first batch from registers, later batches loaded inline
    matches += kqProbeCounted<T, K>(sv, ns, s, tab4, cnt2);
    for (uint32_t b0 = BATCH; b0 < ns; b0 += BATCH) {
      uint64_t xv[K];
      S.load(s0 + b0, ns - b0, xv);
      matches += kqProbeCounted<T, K>(xv, ns - b0, s, tab4, cnt2);
    }
    __syncthreads();
    // Only the entries this span used (a few per lane instead of the whole
    // 72 KiB table); copies of a key clear the same entry.
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (used[k] >= KC_E) continue;
      tab64[used[k]] = ~0ull;
      cnt[used[k]] = 0;
    }
    __syncthreads();
  };
  for (;;) {
    if (t == 0) *qbase = atomicAdd(queue, KC_GRAB);
    __syncthreads();  // (first round: also orders the table clear before any build)
    const uint32_t base = __builtin_amdgcn_readfirstlane(*qbase);
    if (base >= n) break;
    const uint32_t nc = min(KC_GRAB, n - base);
    if (t < nc) desc[t] = spans[base + t];
    __syncthreads();
    loadSpan(desc[0], ra, sa);
    loadSpan(desc[min(1u, nc - 1)], rb, sb);
    for (uint32_t i = 0; i < nc; i += 3) {
      span(i, nc, ra, sa, rc, sc);
      if (i + 1 < nc) span(i + 1, nc, rb, sb, ra, sa);
      if (i + 2 < nc) span(i + 2, nc, rc, sc, rb, sb);
    }
  }
  const unsigned long long total = blockReduceSum<T, unsigned long long>((unsigned long long)matches, wsum);
  if (t == 0 && total) atomicAdd(result, total);
}

size_t bpKeyCountedLdsBytes() { return KC_E * 12 + KS_CHUNK * sizeof(BPSpan) + 16 * 8 + 16; }

void bpKeyCountedSpans(const BPArgs &a, uint32_t *queue, hipStream_t st) {
  constexpr int T = 1024, K = 2;
  HJ_CHECK(bpKeyCountedFits(a) && a.rChunk <= (uint32_t)(T * K) && a.heavySpans && a.heavyCount && queue,
           "bpKeyCountedSpans: needs split key-only words of <= 48 fragment bits, the heavy span list and a queue");
  const uint32_t s = a.keyFragBits > 32 ? a.keyFragBits - 32 : 0;
  const size_t lds = bpKeyCountedLdsBytes();
  const dim3 grid(std::min<uint32_t>(std::max<uint32_t>(ceilDiv(a.heavyCapacity, KS_CHUNK), 1), 256 * 2));
  HIP_CHECK(hipMemsetAsync(queue, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL((bpKeyCountedSpansKernel<T, K, 8>), grid, dim3(T), lds, st, KsSrc<T, K, true>{a.R, a.Rhi},
                     KsSrc<T, K, true>{a.S, a.Shi}, a.dedupCounts, a.heavySpans, a.heavyCount, a.heavyCapacity, queue,
                     s, a.result);
  HIP_CHECK_LAUNCH();
}

// ------------------------------------------------ in-place inner compaction
// bpKeyDedup: one workgroup per segment of a listed partition (more than
// rChunk inner words, repeated keys known; a partition of n words has
// min(BP_DEDUP_SEGS, ceil(n / 32K)) equal segments, so a hot key's million
// copies are compacted by up to 16 workgroups instead of one: the largest
// partition set the kernel's time).  Work items: segment 0 of every listed
// partition, then segments 1-15 of the partitions bpPlanCounts also listed
// as big (an item per possible segment of every partition cost ~0.6 ms of
// empty items at 1e8 x 4e8).  It streams the segment's inner words in
// 2048-word batches into an LDS table of (full fragment, count) -- 4096
// entries, 64-bit CAS claims, count adds -- and whenever more than 1024
// distinct keys are held (so the next batch still fits at load <= 3/4),
// flushes them back over the segment's own words: word i of the compacted
// list overwrites inner word i, which was already read (a flush writes at most
// as many entries as words consumed since the last one), with its count at
// dedupCounts[i].  A key may appear in several flushes and segments; counts
// then add up in the counted table.  Finally the workgroup emits the
// segment's counted spans over its compacted words (flags bit 0):
// ceil(distinct / rChunk) inner chunks, each against the partition's whole
// outer side.  The inner words are overwritten, so the caller runs this once
// per join (not with per-chunk rebuilds); the compacted lengths are kept per
// segment, and a re-run of the build/probe (span list overflow) only re-emits
// the spans (emitOnly).
constexpr uint32_t KD_ENTRIES = 4096;
constexpr uint32_t KD_FLUSH = 1024;
constexpr uint64_t KD_SEG_MIN = BP_DEDUP_SEG_MIN;

template <int T, int K>
__global__ __launch_bounds__(T) void bpKeyDedupKernel(KsSrc<T, K, true> R, uint32_t *__restrict__ rlo,
                                                       uint16_t *__restrict__ rhi, uint32_t *__restrict__ rCounts,
                                                       const uint32_t *__restrict__ parts,
                                                       const uint32_t *__restrict__ nPartsPtr, uint32_t maxParts,
                                                       const uint32_t *__restrict__ big,
                                                       const uint32_t *__restrict__ nBigPtr,
                                                       const uint64_t *__restrict__ partR,
                                                       const uint64_t *__restrict__ partREnd,
                                                       const uint64_t *__restrict__ partS,
                                                       const uint64_t *__restrict__ partSEnd, uint32_t rc, uint32_t sc,
                                                       BPSpan *__restrict__ spans, uint32_t *__restrict__ spanCount,
                                                       uint32_t spanCapacity, uint64_t *__restrict__ lenBySeg,
                                                       bool emitOnly) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long *key = reinterpret_cast<unsigned long long *>(smem);  // [entry] fragment (~0 = empty)
  uint32_t *cnt = reinterpret_cast<uint32_t *>(key + KD_ENTRIES);         // [entry] count
  uint32_t *ctl = cnt + KD_ENTRIES;                                       // [0] distinct held, [1] out, [2] span base
  constexpr uint32_t BATCH = T * K;
  const uint32_t t = threadIdx.x;
  const uint32_t np = min(*nPartsPtr, maxParts);
  for (uint32_t i = t; i < KD_ENTRIES; i += T) {
    key[i] = ~0ull;
    cnt[i] = 0;
  }
  // Items: segment 0 of every listed partition, then segments 1-15 of the
  // partitions listed as big (empty past a partition's segment count).
  const uint32_t nb = min(*nBigPtr, maxParts);
  for (uint32_t w = blockIdx.x; w < np + nb * (BP_DEDUP_SEGS - 1); w += gridDim.x) {
    const uint32_t p = w < np ? parts[w] : big[(w - np) / (BP_DEDUP_SEGS - 1)];
    const uint32_t sg = w < np ? 0u : 1u + (w - np) % (BP_DEDUP_SEGS - 1);
    const uint64_t pb = uniform64(partR[p]);
    const uint64_t pn = uniform64(partREnd[p]) - pb;
    const uint64_t nseg = min<uint64_t>(BP_DEDUP_SEGS, ceilDiv(pn, KD_SEG_MIN));
    if (sg >= nseg) continue;  // (uniform: no barrier skipped by part of the workgroup)
    const uint64_t len = ceilDiv(pn, nseg);
    const uint64_t rb = pb + sg * len;
    const uint64_t nr = min<uint64_t>(len, pn - sg * len);
    const size_t li = (size_t)p * BP_DEDUP_SEGS + sg;
    if (t == 0) {
      ctl[0] = 0;
      ctl[1] = emitOnly ? (uint32_t)lenBySeg[li] : 0u;
    }
    __syncthreads();
    auto flush = [&]() {
      for (uint32_t i = t; i < KD_ENTRIES; i += T) {
        const unsigned long long f = key[i];
        if (f == ~0ull) continue;
        const uint64_t at = rb + atomicAdd(&ctl[1], 1u);
        rlo[at] = (uint32_t)f;
        rhi[at] = (uint16_t)(f >> 32);
        rCounts[at] = cnt[i];
        key[i] = ~0ull;
        cnt[i] = 0;
      }
      __syncthreads();
      if (t == 0) ctl[0] = 0;
      __syncthreads();
    };
    for (uint64_t b0 = 0; b0 < (emitOnly ? 0 : nr); b0 += BATCH) {
      const uint32_t nb = (uint32_t)min<uint64_t>(nr - b0, BATCH);
      uint64_t v[K];
      R.load(rb + b0, nb, v);  // used (so landed) before the barrier that precedes any flush over them
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const bool valid = (uint32_t)(k * T) + t < nb;
        const unsigned long long f = v[k];
        // Hot partitions are mostly copies of one or two keys: a wave first
        // folds the lanes that hold the key of its first (then second)
        // pending lane into one insert of their popcount, so same-address
        // LDS atomics do not serialise 64 deep.
        uint32_t add = 1;
        bool lead = valid, pending = valid;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const uint64_t pm = __ballot(pending);
          if (!pm) break;
          const int l0 = __ffsll((unsigned long long)pm) - 1;
          const unsigned long long fr = __shfl(f, l0);
          const bool g = pending && f == fr;
          const uint64_t gm = __ballot(g);
          if (g) {
            add = (uint32_t)__popcll(gm);
            lead = (int)(t & (WAVE - 1)) == l0;
            pending = false;
          }
        }
        if (!lead) continue;
        uint32_t h = (uint32_t)((f * 0x9E3779B97F4A7C15ull) >> (64 - 12));
        for (;;) {  // <= KD_FLUSH + BATCH distinct keys in 4096 entries: an empty entry is reached
          const unsigned long long o = atomicCAS(&key[h], ~0ull, f);
          if (o == ~0ull) atomicAdd(&ctl[0], 1u);
          if (o == ~0ull || o == f) {
            atomicAdd(&cnt[h], add);
            break;
          }
          h = (h + 1) & (KD_ENTRIES - 1);
        }
      }
      __syncthreads();
      if (ctl[0] > KD_FLUSH || b0 + BATCH >= nr) flush();
    }
    // ---- the segment's counted spans over its compacted words (a partition
    // of several segments: bpKeyDedupMergeKernel merges the lists and emits;
    // on a re-emit its merged list is segment 0's, the others are empty)
    const uint64_t nd = ctl[1];
    if (t == 0 && !emitOnly) lenBySeg[li] = nd;
    const uint64_t ns = uniform64(partSEnd[p]) - uniform64(partS[p]);
    const uint32_t nsc = (uint32_t)ceilDiv(ns, sc);
    const uint32_t c = (nseg > 1 && !emitOnly) ? 0u : (uint32_t)(ceilDiv(nd, rc) * nsc);
    if (t == 0) ctl[2] = c ? atomicAdd(spanCount, c) : 0u;
    __syncthreads();
    const uint32_t o = ctl[2];
    for (uint32_t i = t; i < c; i += T) {
      if (o + i >= spanCapacity) break;
      BPSpan sp;
      sp.rb = rb + (uint64_t)(i / nsc) * rc;
      sp.sb = partS[p] + (uint64_t)(i % nsc) * sc;
      sp.nr = (uint32_t)min(nd - (uint64_t)(i / nsc) * rc, (uint64_t)rc);
      sp.ns = (uint32_t)min(ns - (uint64_t)(i % nsc) * sc, (uint64_t)sc);
      sp.flags = 1;
      sp.pad1 = 0;
      spans[o + i] = sp;
    }
    __syncthreads();
  }
}

void bpKeyDedup(const BPArgs &a, uint32_t maxParts, bool emitOnly, hipStream_t st) {
  constexpr int T = 512, K = 4;
  if (maxParts == 0) return;
  HJ_CHECK(a.split && a.dedupParts && a.dedupCount && a.dedupCounts && a.dedupLen && a.heavySpans && a.heavyCount &&
               a.rChunk <= (uint32_t)(T * K),
           "bpKeyDedup: needs split key-only words, the partition list, the count column and the span list");
  const size_t lds = KD_ENTRIES * 12 + 16;
  HJ_CHECK(a.dedupBig && a.dedupBigCount, "bpKeyDedup: needs the big-partition list");
  const dim3 grid(std::min<uint32_t>(maxParts, 256 * 3));
  hipLaunchKernelGGL((bpKeyDedupKernel<T, K>), grid, dim3(T), lds, st, KsSrc<T, K, true>{a.R, a.Rhi},
                     static_cast<uint32_t *>(const_cast<void *>(a.R)), const_cast<uint16_t *>(a.Rhi), a.dedupCounts,
                     a.dedupParts, a.dedupCount, maxParts, a.dedupBig, a.dedupBigCount, a.partR, a.partREnd ? a.partREnd : a.partR + 1, a.partS,
                     a.partSEnd ? a.partSEnd : a.partS + 1, a.rChunk, a.sChunk, a.heavySpans, a.heavyCount,
                     a.heavyCapacity, a.dedupLen, emitOnly);
  HIP_CHECK_LAUNCH();
}

// Merge of a multi-segment partition's compacted lists (see bpKeyDedupMerge
// in kernels.h).  Segment g's list (lenBySeg words at the segment's start)
// moves to the end of the lists before it; a destination never reaches past
// its own source (a list is no longer than its segment), so copying the
// segments in order, each in register-staged batches with a barrier between
// the batch's loads and stores, never overwrites a word still to be read.
template <int T, int K>
__global__ __launch_bounds__(T) void bpKeyDedupMergeKernel(
    uint32_t *__restrict__ rlo, uint16_t *__restrict__ rhi, uint32_t *__restrict__ rCounts,
    const uint32_t *__restrict__ big, const uint32_t *__restrict__ nBigPtr, uint32_t maxParts,
    const uint64_t *__restrict__ partR, const uint64_t *__restrict__ partREnd, const uint64_t *__restrict__ partS,
    const uint64_t *__restrict__ partSEnd, uint32_t rc, uint32_t sc, BPSpan *__restrict__ spans,
    uint32_t *__restrict__ spanCount, uint32_t spanCapacity, uint64_t *__restrict__ lenBySeg) {
  __shared__ uint32_t spanBase;
  constexpr uint32_t BATCH = T * K;
  const uint32_t t = threadIdx.x;
  const uint32_t nb = min(*nBigPtr, maxParts);
  for (uint32_t w = blockIdx.x; w < nb; w += gridDim.x) {
    const uint32_t p = big[w];
    const uint64_t pb = uniform64(partR[p]);
    const uint64_t pn = uniform64(partREnd[p]) - pb;
    const uint64_t nseg = min<uint64_t>(BP_DEDUP_SEGS, ceilDiv(pn, KD_SEG_MIN));
    const uint64_t len = ceilDiv(pn, nseg);
    uint64_t out = uniform64(lenBySeg[(size_t)p * BP_DEDUP_SEGS]);  // segment 0 stays where it is
    for (uint32_t g = 1; g < nseg; ++g) {
      const uint64_t L = uniform64(lenBySeg[(size_t)p * BP_DEDUP_SEGS + g]);
      const uint64_t src = pb + g * len, dst = pb + out;
      for (uint64_t i0 = 0; i0 < L; i0 += BATCH) {
        uint32_t lo[K], ct[K];
        uint16_t hi[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint64_t i = i0 + (uint64_t)(k * T + t);
          if (i < L) {
            lo[k] = rlo[src + i];
            hi[k] = rhi[src + i];
            ct[k] = rCounts[src + i];
          }
        }
        __syncthreads();  // the batch is read before any of it is overwritten
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint64_t i = i0 + (uint64_t)(k * T + t);
          if (i < L) {
            rlo[dst + i] = lo[k];
            rhi[dst + i] = hi[k];
            rCounts[dst + i] = ct[k];
          }
        }
        __syncthreads();
      }
      out += L;
    }
    if (t == 0) {  // a re-emit (bpKeyDedup emitOnly) then emits the merged list as segment 0's
      lenBySeg[(size_t)p * BP_DEDUP_SEGS] = out;
      for (uint32_t g = 1; g < BP_DEDUP_SEGS; ++g) lenBySeg[(size_t)p * BP_DEDUP_SEGS + g] = 0;
    }
    const uint64_t ns = uniform64(partSEnd[p]) - uniform64(partS[p]);
    const uint32_t nsc = (uint32_t)ceilDiv(ns, sc);
    const uint32_t c = (uint32_t)(ceilDiv(out, rc) * nsc);
    if (t == 0) spanBase = c ? atomicAdd(spanCount, c) : 0u;
    __syncthreads();
    const uint32_t o = spanBase;
    for (uint32_t i = t; i < c; i += T) {
      if (o + i >= spanCapacity) break;
      BPSpan sp;
      sp.rb = pb + (uint64_t)(i / nsc) * rc;
      sp.sb = partS[p] + (uint64_t)(i % nsc) * sc;
      sp.nr = (uint32_t)min(out - (uint64_t)(i / nsc) * rc, (uint64_t)rc);
      sp.ns = (uint32_t)min(ns - (uint64_t)(i % nsc) * sc, (uint64_t)sc);
      sp.flags = 1;
      sp.pad1 = 0;
      spans[o + i] = sp;
    }
    __syncthreads();
  }
}

void bpKeyDedupMerge(const BPArgs &a, uint32_t maxParts, hipStream_t st) {
  constexpr int T = 512, K = 4;
  if (maxParts == 0) return;
  HJ_CHECK(a.split && a.dedupCounts && a.dedupLen && a.dedupBig && a.dedupBigCount && a.heavySpans && a.heavyCount,
           "bpKeyDedupMerge: needs split key-only words, the big-partition list, the count column and the span list");
  const dim3 grid(std::min<uint32_t>(maxParts, 256 * 4));
  hipLaunchKernelGGL((bpKeyDedupMergeKernel<T, K>), grid, dim3(T), 0, st,
                     static_cast<uint32_t *>(const_cast<void *>(a.R)), const_cast<uint16_t *>(a.Rhi), a.dedupCounts,
                     a.dedupBig, a.dedupBigCount, maxParts, a.partR, a.partREnd ? a.partREnd : a.partR + 1, a.partS,
                     a.partSEnd ? a.partSEnd : a.partS + 1, a.rChunk, a.sChunk, a.heavySpans, a.heavyCount,
                     a.heavyCapacity, a.dedupLen);
  HIP_CHECK_LAUNCH();
}

size_t bpKeySpanLdsBytes(uint32_t maxR) {
  const uint64_t slots = uint64_t(1) << ceilLog2(2ull * maxR);
  return slots * 8 + (slots / BPK_SLOTS) * 4 + KS_CHUNK * sizeof(BPSpan) + 16 * 8 + 16;
}

void buildProbeKeySpans(const BPArgs &a, const BPSpan *spans, const uint32_t *nSpans, uint32_t capacity,
                        uint32_t *queue, hipStream_t s) {
  if (capacity == 0) return;
  constexpr int T = 512, K = 4, H = 2;
  HJ_CHECK(a.keyOnly && !a.materialize && !a.wide, "buildProbeKeySpans: key-only counting joins only");
  HJ_CHECK(!a.split || (a.Rhi && a.Shi), "buildProbeKeySpans: split layout without high columns");
  HJ_CHECK(a.rChunk <= (uint32_t)(T * K), "buildProbeKeySpans: rChunk %u above one %d-word batch", a.rChunk, T * K);
  if ((a.keyCount == 8 || a.keyCount == 9) && bpKeyQuotientFits(a)) {
    launchKeyQuotient(a, spans, nSpans, capacity, queue, s);
    return;
  }
  const size_t lds = bpKeySpanLdsBytes(a.rChunk);
  HJ_CHECK(lds <= 160 * 1024, "buildProbeKeySpans: LDS %zu B exceeds 160 KiB (rChunk=%u)", lds, a.rChunk);
  const uint32_t perCu = (uint32_t)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
  const dim3 grid(std::min<uint32_t>(ceilDiv(capacity, KS_CHUNK), 256 * perCu));
  HIP_CHECK(hipMemsetAsync(queue, 0, sizeof(uint32_t), s));
#define HJ_KS(SPLIT)                                                                                             \
  hipLaunchKernelGGL((bpKeySpanKernel<T, K, H, 8, SPLIT>), grid, dim3(T), lds, s,                                 \
                     KsSrc<T, K, SPLIT>{a.R, SPLIT ? a.Rhi : nullptr}, KsSrc<T, K, SPLIT>{a.S, SPLIT ? a.Shi : nullptr}, \
                     spans, nSpans, capacity, queue, a.rChunk, a.result)
  if (a.split)
    HJ_KS(true);
  else
    HJ_KS(false);
#undef HJ_KS
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadKeyTables() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&bpEmitSpansKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
