#include "HostOps.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "../utils/Debug.h"

namespace hpcjoin {
namespace host {

using kernels::KeyDistribution;

// ------------------------------------------------------------------ datagen
static double zeta(uint64_t n, double theta) {
  // Exact for small n, Euler-Maclaurin tail beyond 2^20 terms.
  const uint64_t m = std::min<uint64_t>(n, 1u << 20);
  double s = 0;
  for (uint64_t i = 1; i <= m; ++i) s += std::pow((double)i, -theta);
  if (n > m) {
    const double a = (double)m, b = (double)n;
    // integral_a^b x^-t dx + (f(b) - f(a))/2 - (f'(b) - f'(a))/12
    s += (std::pow(b, 1 - theta) - std::pow(a, 1 - theta)) / (1 - theta);
    s += (std::pow(b, -theta) - std::pow(a, -theta)) / 2;
    s += (-theta * std::pow(b, -theta - 1) + theta * std::pow(a, -theta - 1)) / 12;
  }
  return s;
}

kernels::ZipfParams makeZipf(uint64_t n, double theta) {
  JOIN_ASSERT(n >= 2, "Zipf", "domain must be >= 2");
  // Gray et al.'s closed-form inverse is the continuous approximation of
  // sum_{i<=r} i^-theta, valid on both sides of 1 (alpha = 1/(1-theta) < 0
  // above it): ranks 0 and 1 are exact, the rest within ~1% of the mass
  // (tests/test_package.py checks theta 0.99 and 1.1).  theta = 1 has no alpha.
  JOIN_ASSERT(theta > 0 && theta <= 4 && std::fabs(theta - 1.0) >= 1e-3, "Zipf",
              "theta must be in (0,4] and not 1, got %f", theta);
  kernels::ZipfParams z;
  z.n = n;
  z.theta = theta;
  z.alpha = 1.0 / (1.0 - theta);
  z.zetan = zeta(n, theta);
  const double zeta2 = 1.0 + std::pow(2.0, -theta);
  z.eta = (1.0 - std::pow(2.0 / (double)n, 1.0 - theta)) / (1.0 - zeta2 / z.zetan);
  z.half_pow_theta = std::pow(0.5, theta);
  return z;
}

static inline uint64_t zipfRank(const kernels::ZipfParams &z, double u) {
  const double uz = u * z.zetan;
  if (uz < 1.0) return 0;
  if (uz < 1.0 + z.half_pow_theta) return 1;
  uint64_t r = (uint64_t)((double)z.n * std::pow(z.eta * u - z.eta + 1.0, z.alpha));
  return r >= z.n ? z.n - 1 : r;
}

void generate(data::Tuple *out, uint64_t n, const kernels::GenParams &p) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t gi = p.globalOffset + i;
    uint64_t k;
    switch (p.dist) {
      case KeyDistribution::Unique: k = p.keyOffset + p.perm(gi); break;
      case KeyDistribution::Dense: k = p.keyOffset + gi; break;
      case KeyDistribution::Modulo: k = p.keyOffset + p.perm(gi % p.modulo); break;
      case KeyDistribution::Uniform:
        k = p.keyOffset + (uint64_t)(kernels::uniform01(p.seed, gi) * (double)p.domain) % p.domain;
        break;
      default: k = p.keyOffset + p.perm(zipfRank(p.zipf, kernels::uniform01(p.seed, gi))); break;
    }
    if (p.tpchSparse) k = kernels::tpchSparseKey(k);
    out[i].key = p.sparse64 ? kernels::sparseKey(k) : k;
    out[i].rid = p.ridOffset + i;
  }
}

// ------------------------------------------------------------ pass 1 (host)
void netHistogram(const data::Tuple *in, uint64_t n, uint32_t bits, const kernels::PartitionGeometry &g,
                  uint32_t *blockHist, kernels::KeyMix mix) {
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  std::memset(blockHist, 0, sizeof(uint32_t) * F * g.blocks);
  for (uint32_t b = 0; b < g.blocks; ++b) {
    const uint64_t begin = (uint64_t)b * g.tuplesPerBlock(), end = std::min(n, begin + g.tuplesPerBlock());
    for (uint64_t i = begin; i < end; ++i) blockHist[(mix.apply(in[i].key) & mask) * g.blocks + b]++;
  }
}

void digitTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t bpc, uint32_t chunks,
                 uint64_t *totals) {
  for (uint32_t c = 0; c < chunks; ++c)
    for (uint32_t d = 0; d < F; ++d) {
      uint64_t s = 0;
      for (uint32_t b = c * bpc; b < std::min(blocks, (c + 1) * bpc); ++b) s += blockHist[(uint64_t)d * blocks + b];
      totals[(uint64_t)c * F + d] = s;
    }
}

void netCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t bpc, const uint64_t *base,
                uint64_t *cursors) {
  const uint32_t chunks = (blocks + bpc - 1) / bpc;
  for (uint32_t d = 0; d < F; ++d)
    for (uint32_t c = 0; c < chunks; ++c) {
      uint64_t run = base[(uint64_t)c * F + d];
      for (uint32_t b = c * bpc; b < std::min(blocks, (c + 1) * bpc); ++b) {
        cursors[(uint64_t)d * blocks + b] = run;
        run += blockHist[(uint64_t)d * blocks + b];
      }
    }
}

void netScatter(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift,
                const kernels::PartitionGeometry &g, uint32_t blockBegin, uint32_t blockEnd, const uint64_t *cursors,
                void *out, bool wide, kernels::KeyMix mix, bool withRids) {
  const uint32_t F = 1u << bits;
  const uint64_t ridMask = withRids ? ~0ull : 0ull;
  const uint64_t mask = F - 1;
  std::vector<uint64_t> cur(F);
  for (uint32_t b = blockBegin; b < blockEnd; ++b) {
    for (uint32_t d = 0; d < F; ++d) cur[d] = cursors[(uint64_t)d * g.blocks + b];
    const uint64_t begin = (uint64_t)b * g.tuplesPerBlock(), end = std::min(n, begin + g.tuplesPerBlock());
    for (uint64_t i = begin; i < end; ++i) {
      const uint64_t key = mix.apply(in[i].key);
      const uint64_t d = key & mask;
      if (wide)
        static_cast<data::Tuple *>(out)[cur[d]++] = data::Tuple{key, in[i].rid};
      else
        static_cast<uint64_t *>(out)[cur[d]++] = (in[i].rid & ridMask) | ((key >> bits) << keyShift);
    }
  }
}

// ------------------------------------------------------------ pass 2 (host)
static inline uint64_t word(const void *in, bool wide, uint64_t i) {
  return wide ? static_cast<const data::Tuple *>(in)[i].key : static_cast<const uint64_t *>(in)[i];
}

void localHistogram(const void *in, bool wide, const kernels::LocalItem *items, uint32_t nItems, uint32_t shift,
                    uint32_t bits, uint32_t *itemHist) {
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  std::memset(itemHist, 0, sizeof(uint32_t) * (uint64_t)F * nItems);
  for (uint32_t it = 0; it < nItems; ++it)
    for (uint64_t i = items[it].begin; i < items[it].begin + items[it].len; ++i)
      itemHist[(uint64_t)it * F + ((word(in, wide, i) >> shift) & mask)]++;
}

void localCursors(const uint32_t *itemHist, const uint32_t *lpItemBegin, uint32_t owned, uint32_t bits,
                  const uint64_t *lpBase, uint64_t *itemCursors, uint64_t *partBegin) {
  const uint32_t F = 1u << bits;
  for (uint32_t lp = 0; lp < owned; ++lp) {
    uint64_t run = lpBase[lp];
    for (uint32_t q = 0; q < F; ++q) {
      partBegin[(uint64_t)lp * F + q] = run;
      for (uint32_t it = lpItemBegin[lp]; it < lpItemBegin[lp + 1]; ++it) {
        itemCursors[(uint64_t)it * F + q] = run;
        run += itemHist[(uint64_t)it * F + q];
      }
    }
  }
  if (owned) partBegin[(uint64_t)owned * F] = lpBase[owned];
}

void localScatter(const void *in, bool wide, const kernels::LocalItem *items, uint32_t nItems, uint32_t shift,
                  uint32_t bits, const uint64_t *itemCursors, void *out) {
  const uint32_t F = 1u << bits;
  const uint64_t mask = F - 1;
  std::vector<uint64_t> cur(F);
  for (uint32_t it = 0; it < nItems; ++it) {
    for (uint32_t q = 0; q < F; ++q) cur[q] = itemCursors[(uint64_t)it * F + q];
    for (uint64_t i = items[it].begin; i < items[it].begin + items[it].len; ++i) {
      const uint64_t q = (word(in, wide, i) >> shift) & mask;
      if (wide)
        static_cast<data::Tuple *>(out)[cur[q]++] = static_cast<const data::Tuple *>(in)[i];
      else
        static_cast<uint64_t *>(out)[cur[q]++] = static_cast<const uint64_t *>(in)[i];
    }
  }
}

// --------------------------------------------------------------- build/probe
static inline uint64_t nextPow2(uint64_t x) {  // 64-bit (reference NEXT_POW_2 was 32-bit only)
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

uint64_t buildProbe(const kernels::BPArgs &a) {
  uint64_t matches = 0;
  const uint64_t ridMask = a.keyShift >= 64 ? ~0ull : ((1ull << a.keyShift) - 1);
  std::vector<uint64_t> bucket, next;
  for (uint32_t p = 0; p < a.P; ++p) {
    const uint64_t rb = a.partR[p], re = a.partREnd ? a.partREnd[p] : a.partR[p + 1], sb = a.partS[p],
                   se = a.partSEnd ? a.partSEnd[p] : a.partS[p + 1];
    const uint64_t nr = re - rb;
    if (nr == 0 || se == sb) continue;
    const uint64_t N = nextPow2(nr);
    bucket.assign(N, 0);
    next.assign(nr, 0);
    if (!a.wide) {
      const uint64_t *R = static_cast<const uint64_t *>(a.R) + rb;
      const uint64_t *S = static_cast<const uint64_t *>(a.S);
      const uint64_t mask = (N - 1) << a.fragShift;
      for (uint64_t t = 0; t < nr; ++t) {
        const uint64_t idx = (a.fragShift >= 64) ? 0 : ((R[t] & mask) >> a.fragShift);
        next[t] = bucket[idx];
        bucket[idx] = t + 1;
      }
      for (uint64_t s = sb; s < se; ++s) {
        const uint64_t v = S[s];
        const uint64_t idx = (a.fragShift >= 64) ? 0 : ((v & mask) >> a.fragShift);
        for (uint64_t hit = bucket[idx]; hit > 0; hit = next[hit - 1]) {
          if ((R[hit - 1] >> a.keyShift) == (v >> a.keyShift)) {
            ++matches;
            if (a.materialize) {
              const unsigned long long pos = (*a.outCursor)++;
              if (pos < a.outCapacity) a.outPairs[pos] = make_ulonglong2(R[hit - 1] & ridMask, v & ridMask);
            }
          }
        }
      }
    } else {
      const data::Tuple *R = static_cast<const data::Tuple *>(a.R) + rb;
      const data::Tuple *S = static_cast<const data::Tuple *>(a.S);
      for (uint64_t t = 0; t < nr; ++t) {
        const uint64_t idx = kernels::mix64(R[t].key) & (N - 1);
        next[t] = bucket[idx];
        bucket[idx] = t + 1;
      }
      for (uint64_t s = sb; s < se; ++s) {
        const uint64_t idx = kernels::mix64(S[s].key) & (N - 1);
        for (uint64_t hit = bucket[idx]; hit > 0; hit = next[hit - 1])
          if (R[hit - 1].key == S[s].key) {
            ++matches;
            if (a.materialize) {
              const unsigned long long pos = (*a.outCursor)++;
              if (pos < a.outCapacity) a.outPairs[pos] = make_ulonglong2(R[hit - 1].rid, S[s].rid);
            }
          }
      }
    }
  }
  return matches;
}

uint64_t npjJoin(const data::Tuple *R, uint64_t nR, const data::Tuple *S, uint64_t nS) {
  std::unordered_map<uint64_t, uint64_t> counts;
  counts.reserve(nR * 2);
  for (uint64_t i = 0; i < nR; ++i) counts[R[i].key]++;
  uint64_t m = 0;
  for (uint64_t i = 0; i < nS; ++i) {
    auto it = counts.find(S[i].key);
    if (it != counts.end()) m += it->second;
  }
  return m;
}

std::vector<std::pair<uint64_t, uint64_t>> npjPairs(const data::Tuple *R, uint64_t nR, const data::Tuple *S,
                                                    uint64_t nS) {
  std::unordered_map<uint64_t, std::vector<uint64_t>> rids;
  rids.reserve(nR * 2);
  for (uint64_t i = 0; i < nR; ++i) rids[R[i].key].push_back(R[i].rid);
  std::vector<std::pair<uint64_t, uint64_t>> out;
  for (uint64_t i = 0; i < nS; ++i) {
    auto it = rids.find(S[i].key);
    if (it == rids.end()) continue;
    for (uint64_t r : it->second) out.emplace_back(r, S[i].rid);
  }
  return out;
}

// Wire codec twins: a plain bit-stream writer/reader over each segment's
// groups of 64 (independent of the device's per-lane word assembly).
void wirePack(const uint64_t *raw, uint64_t *wire, const kernels::WireSeg *segs, uint32_t nSegs,
              const kernels::WireCodec &c) {
  const uint64_t wmask = c.w >= 64 ? ~0ull : ((1ull << c.w) - 1);
  for (uint32_t s = 0; s < nSegs; ++s) {
    const kernels::WireSeg &sg = segs[s];
    uint64_t *out = wire + sg.wire;
    std::fill(out, out + c.words(sg.n), 0ull);
    for (uint64_t t = 0; t < sg.n; ++t) {
      const uint64_t e = c.encode(raw[sg.raw + t], sg.base) & wmask;
      const uint64_t bit = (t / 64) * 64 * c.w + (t % 64) * c.w;
      const uint64_t j = bit / 64, o = bit % 64;
      out[j] |= e << o;
      if (o + c.w > 64) out[j + 1] |= e >> (64 - o);
    }
  }
}

void wireUnpack(const uint64_t *wire, uint64_t *raw, const kernels::WireSeg *segs, uint32_t nSegs,
                const kernels::WireCodec &c) {
  const uint64_t wmask = c.w >= 64 ? ~0ull : ((1ull << c.w) - 1);
  for (uint32_t s = 0; s < nSegs; ++s) {
    const kernels::WireSeg &sg = segs[s];
    const uint64_t *in = wire + sg.wire;
    for (uint64_t t = 0; t < sg.n; ++t) {
      const uint64_t bit = (t / 64) * 64 * c.w + (t % 64) * c.w;
      const uint64_t j = bit / 64, o = bit % 64;
      uint64_t e = in[j] >> o;
      if (o + c.w > 64) e |= in[j + 1] << (64 - o);
      raw[sg.raw + t] = c.decode(e & wmask, sg.base);
    }
  }
}

}  // namespace host
}  // namespace hpcjoin
