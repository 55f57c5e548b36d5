#include "SampledNetworkPartitioning.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <tuple>

#include "../memory/Arena.h"
#include "../performance/Timeline.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

using kernels::CLAIM_GROUPS;

SampledNetworkPartitioning::SampledNetworkPartitioning(data::Relation *innerRelation, data::Relation *outerRelation,
                                                       core::ExecContext *ctx, const core::JoinPlan &plan,
                                                       uint32_t maxBlocks, uint32_t sampleStride)
    : ctx(ctx), plan(plan), maxBlocks(maxBlocks), sampleStride(std::max<uint32_t>(1, sampleStride)) {
  JOIN_ASSERT(ctx->onDevice() && ctx->numberOfNodes() == 1, "SampledNetwork", "single-rank device path only");
  sides[0].relation = innerRelation;
  sides[1].relation = outerRelation;
}

SampledNetworkPartitioning::~SampledNetworkPartitioning() = default;  // events belong to the context pool

// Geometry, sample stride, scale and capacity bound of one side: pure
// functions of the size (host loops over every block and sampled tile, ~20 us),
// computed once per thread and size.
const SampledNetworkPartitioning::SidePlan &SampledNetworkPartitioning::sidePlan(uint64_t n) const {
  struct Key {
    uint64_t n;
    uint32_t maxBlocks, bits, stride, ipt, nth, lp;
    bool operator<(const Key &o) const {
      return std::tie(n, maxBlocks, bits, stride, ipt, nth, lp) <
             std::tie(o.n, o.maxBlocks, o.bits, o.stride, o.ipt, o.nth, o.lp);
    }
  };
  thread_local std::map<Key, SidePlan> cache;
  const uint32_t F = 1u << plan.networkBits;
  const Key k{n, maxBlocks, plan.networkBits, sampleStride, plan.variants.netIpt, plan.variants.netThreads, roundLp()};
  auto it = cache.find(k);
  if (it != cache.end()) return it->second;
  if (cache.size() > 64) cache.clear();
  SidePlan sp;
  sp.geom = kernels::partitionGeometry(n, maxBlocks);
  sp.geom.ipt = plan.variants.netIpt;
  sp.geom.nth = plan.variants.netThreads;
  sp.stride = kernels::sampleStrideFor(sp.geom, n, F, sampleStride);
  sp.sc = kernels::sampleScale(sp.geom, n, sp.stride, sp.stride == 1);
  sp.bound = kernels::sampledWindowCapacity(sp.sc, F, roundLp());
  return cache.emplace(k, sp).first->second;
}

// Sampled totals of both sides (one launch when both are sampled; a side too
// small to sample gets an exact histogram), then each side's bounded claim
// slices are laid out on the device: nothing here waits for the GPU.
void SampledNetworkPartitioning::sample() {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  const hipStream_t st = ctx->stream();
  uint64_t *totals = ctx->workspace().getArray<uint64_t>((uint64_t)2 * G * F);  // adjacent: one clear
  kernels::SampledInput in[2];
  bool bothSampled = true;
  for (int k = 0; k < 2; ++k) {
    Side &s = sides[k];
    const uint64_t n = s.relation->getLocalSize();
    const SidePlan &sp = sidePlan(n);
    s.geom = sp.geom;
    s.stride = sp.stride;
    s.sc = sp.sc;
    s.capacityTotal = sp.bound;
    s.groupTotalsDev = totals + (size_t)k * G * F;
    in[k] = kernels::SampledInput{s.relation->getData(), n, s.geom, s.stride, s.groupTotalsDev};
    bothSampled = bothSampled && s.stride > 1;
  }
  // One span for both histograms, charged to HILOCAL / HOLOCAL by tuples.
  ctx->timeline().beginSplit("HLOCAL", "HILOCAL", (double)in[0].n, "HOLOCAL", (double)in[1].n, st);
  if (bothSampled) {
    kernels::netSampledTotals(in, 2, plan.networkBits, st, mix);
  } else {
    for (int k = 0; k < 2; ++k) {
      if (in[k].stride > 1) {
        kernels::netSampledTotals(&in[k], 1, plan.networkBits, st, mix);
        continue;
      }
      uint32_t *blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * in[k].geom.blocks);
      kernels::netHistogram(in[k].data, in[k].n, plan.networkBits, in[k].geom, blockHist, st, mix, 1);
      kernels::netGroupTotals(blockHist, F, in[k].geom.blocks, in[k].totals, st);
    }
  }
  ctx->timeline().end("HLOCAL", st);
}

// Round-interleaved slices (kernels::RoundMap) for windows the local pass
// reads (two-level plans; the wide scatter keeps linear slices).
uint32_t SampledNetworkPartitioning::roundLp() const {
  return plan.twoLevel && !plan.wide ? kernels::roundLpFor(plan.roundLp, plan.fragments ? 4 : 8) : 0;
}

void SampledNetworkPartitioning::layout() {
  layoutSide(0);
  layoutSide(1);
}

void SampledNetworkPartitioning::layoutSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  Side &s = sides[k];
  const uint64_t n = s.relation->getLocalSize();
  // Claims may run past a slice end by up to n before the overflow is seen:
  // 32-bit cursors only if even that cannot wrap.
  s.narrow = kernels::cursorsNarrow(s.capacityTotal + n);
  // Plan skeleton (filled after the scatter); the window is sized by the
  // layout's capacity bound.
  histograms::ExchangePlan &x = s.xp;
  x = histograms::ExchangePlan();
  x.numberOfNodes = 1;
  x.nodeId = 0;
  x.partitions = F;
  x.chunks = 1;
  x.gapped = true;
  x.owned.resize(F);
  x.localIndex.resize(F);
  for (uint32_t p = 0; p < F; ++p) {
    x.owned[p] = p;
    x.localIndex[p] = (int32_t)p;
  }
  x.sendTotal = n;
  x.scatterTotal = n;
  x.recvTotal = 0;
  s.window.reset(new data::Window(x, s.capacityTotal, ctx, plan.wide, plan.fragments ? 4u : 0u));
  // Slice starts, claim cursors and slice ends ([G][F] each, adjacent: one
  // read-back after the scatter), laid out on the device from the totals.
  // The round map's 4 words follow (read back with them).
  const size_t cb = s.narrow ? 4 : 8, per = (size_t)G * F * cb;
  s.gstart = ctx->workspace().get(3 * per + 16);
  s.gcur = static_cast<uint8_t *>(s.gstart) + per;
  s.gend = static_cast<uint8_t *>(s.gstart) + 2 * per;
  s.roundMeta = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(s.gstart) + 3 * per);
  kernels::LayoutInput in{s.groupTotalsDev, s.sc, s.gstart, s.gcur, s.gend,
                          ctx->workspace().getArray<unsigned long long>(1)};
  if (const uint32_t lp = roundLp()) {
    // Logical positions reach (G * F << lv) + n (claims past a slice end).
    uint32_t lns = 0;
    while ((1u << lns) < G * F) ++lns;
    const uint64_t limit = s.narrow ? (1ull << 32) : (1ull << 62);
    uint32_t maxLv = 0;
    while (maxLv < 40 && ((uint64_t)G * F << (maxLv + 1)) + n < limit) ++maxLv;
    in.roundMeta = s.roundMeta;
    in.roundLp = lp;
    in.roundMaxLv = maxLv;
    in.roundCapacity = s.capacityTotal;
  } else {
    ctx->zero(s.roundMeta, 16);
  }
  kernels::netSampledLayout(&in, 1, F, s.narrow, ctx->stream());
}

bool SampledNetworkPartitioning::scatter() {
  scatterSide(0);
  scatterSide(1);
  const bool ok0 = finishSide(0);
  const bool ok1 = finishSide(1);
  return ok0 && ok1;
}

void SampledNetworkPartitioning::scatterSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  Side &s = sides[k];
  const uint64_t n = s.relation->getLocalSize();
  s.window->start();
  const int nm = s.narrow ? 1 : 0;
  const char *key = k == 0 ? "MIMAINPART" : "MOMAINPART";
  ctx->timeline().begin(key, ctx->stream());
  if (plan.fragments)  // count-only: u32 key fragments (key >> networkBits), no rid
    kernels::netScatterFrag(s.relation->getData(), n, plan.networkBits, s.geom, 0, s.geom.blocks, s.gcur,
                            static_cast<uint32_t *>(s.window->getData()), ctx->stream(), plan.keyBits, mix, s.gend, nm,
                            s.roundMeta);
  else if (plan.wide)
    kernels::netScatterWide(s.relation->getData(), n, plan.networkBits, s.geom, 0, s.geom.blocks, s.gcur,
                            static_cast<data::Tuple *>(s.window->getData()), ctx->stream(), mix, s.gend, nm);
  else
    kernels::netScatter(s.relation->getData(), n, plan.networkBits, plan.keyShift, s.geom, 0, s.geom.blocks, s.gcur,
                        static_cast<uint64_t *>(s.window->getData()), ctx->stream(), plan.keyBits, mix, s.gend, nm,
                        !plan.keyOnly, s.roundMeta);
  ctx->timeline().end(key, ctx->stream());
  const size_t bytes = 3 * (size_t)G * F * (s.narrow ? 4 : 8) + 16;  // starts, final cursors, ends, round map
  s.cursorsBack = ctx->staging().get(bytes);
  ctx->readBack(s.cursorsBack, s.gstart, bytes);
  if (!s.cursorsReady) s.cursorsReady = ctx->acquireEvent();
  HIP_CHECK(hipEventRecord(s.cursorsReady, ctx->stream()));
  s.window->setDataReady(s.cursorsReady);
}

bool SampledNetworkPartitioning::finishSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  Side &s = sides[k];
  utils::waitEvent(s.cursorsReady, ctx->comm(), "sampled network cursors");  // polls: no interrupt wake-up
  const size_t m = (size_t)G * F;
  s.start.resize(m);
  s.fill.assign(m, 0);
  const uint32_t *c32 = static_cast<const uint32_t *>(s.cursorsBack);
  const uint64_t *c64 = static_cast<const uint64_t *>(s.cursorsBack);
  auto at = [&](size_t i) -> uint64_t { return s.narrow ? c32[i] : c64[i]; };
  bool ok = true;
  uint64_t sum = 0, maxEnd = 0, maxCap = 0;
  for (size_t i = 0; i < m; ++i) {
    s.start[i] = at(i);
    s.fill[i] = at(m + i) - s.start[i];  // final claim cursor - slice start
    sum += s.fill[i];
    maxEnd = std::max<uint64_t>(maxEnd, at(2 * m + i));
    maxCap = std::max<uint64_t>(maxCap, at(2 * m + i) - s.start[i]);
    if (s.fill[i] > at(2 * m + i) - s.start[i]) ok = false;
  }
  const uint32_t *meta = reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(s.cursorsBack) +
                                                            3 * m * (s.narrow ? 4 : 8));
  kernels::RoundMap rm;
  rm.lp = meta[0];
  rm.lv = meta[1];
  rm.lns = meta[2];
  if (rm.on()) {
    HJ_CHECK(rm.lv >= rm.lp && maxCap <= (1ull << rm.lv) && (1ull << rm.lns) == m,
             "sampled network layout: round map lp=%u lv=%u lns=%u for slices of %lu over %zu slices", rm.lp, rm.lv,
             rm.lns, (unsigned long)maxCap, m);
    maxEnd = kernels::roundSlots(maxCap, rm.lp, rm.lns);
  }
  HJ_CHECK(maxEnd <= s.capacityTotal, "sampled network layout: slices end at %lu, window holds %lu",
           (unsigned long)maxEnd, (unsigned long)s.capacityTotal);
  s.window->setRoundMap(rm);
  HJ_CHECK(sum == s.relation->getLocalSize(), "sampled network pass claimed %lu of %lu tuples", (unsigned long)sum,
           (unsigned long)s.relation->getLocalSize());
  if (!ok) return false;
  finishPlan(s);
  return true;
}

void SampledNetworkPartitioning::finishPlan(Side &s) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  histograms::ExchangePlan &x = s.xp;
  x.partSize.assign(F, 0);
  x.lpBase.assign(F + 1, 0);
  x.segments.clear();
  for (uint32_t d = 0; d < F; ++d) {
    for (uint32_t g = 0; g < G; ++g) {
      const size_t i = (size_t)g * F + d;
      if (s.fill[i]) x.segments.push_back(histograms::Segment{s.start[i], s.fill[i], d, 0, g});
      x.partSize[d] += s.fill[i];
    }
    x.lpBase[d + 1] = x.lpBase[d] + x.partSize[d];
  }
  x.recvTotal = x.lpBase[F];
  x.sendCounts.assign(1, x.recvTotal);
  x.sendDispls.assign(1, 0);
  x.recvCounts.assign(1, x.recvTotal);
  x.recvDispls.assign(1, 0);
}

}  // namespace tasks
}  // namespace hpcjoin
