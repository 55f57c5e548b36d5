#include "SampledNetworkPartitioning.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../memory/Arena.h"
#include "../performance/Timeline.h"
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

void SampledNetworkPartitioning::sample() {
  const uint32_t F = 1u << plan.networkBits;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  for (Side &s : sides) {
    const char *key = &s == &sides[0] ? "HILOCAL" : "HOLOCAL";
    ctx->timeline().begin(key, ctx->stream());
    const uint64_t n = s.relation->getLocalSize();
    s.geom = kernels::partitionGeometry(n, maxBlocks);
    s.geom.ipt = plan.variants.netIpt;
    s.geom.nth = plan.variants.netThreads;
    s.stride = kernels::sampleStrideFor(s.geom, n, F, sampleStride);
    s.groupTotalsDev = ctx->workspace().getArray<uint64_t>((uint64_t)CLAIM_GROUPS * F);
    if (s.stride > 1) {
      kernels::netSampledTotals(s.relation->getData(), n, plan.networkBits, s.geom, s.groupTotalsDev, ctx->stream(),
                                mix, s.stride);
    } else {
      uint32_t *blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * s.geom.blocks);
      kernels::netHistogram(s.relation->getData(), n, plan.networkBits, s.geom, blockHist, ctx->stream(), mix, 1);
      kernels::netGroupTotals(blockHist, F, s.geom.blocks, s.groupTotalsDev, ctx->stream());
    }
    ctx->timeline().end(key, ctx->stream());
    s.sampled = ctx->staging().getArray<uint64_t>((uint64_t)CLAIM_GROUPS * F);
    HIP_CHECK(hipMemcpyAsync(s.sampled, s.groupTotalsDev, (size_t)CLAIM_GROUPS * F * 8, hipMemcpyDeviceToHost,
                             ctx->stream()));
    if (!s.sampledReady) s.sampledReady = ctx->acquireEvent();
    HIP_CHECK(hipEventRecord(s.sampledReady, ctx->stream()));
  }
}

void SampledNetworkPartitioning::layout() {
  layoutSide(0);
  layoutSide(1);
}

void SampledNetworkPartitioning::layoutSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  {
    Side &s = sides[k];
    HIP_CHECK(hipEventSynchronize(s.sampledReady));
    const uint64_t n = s.relation->getLocalSize();
    // Tuples each group scatters, and how many of them the sample read.
    const kernels::SampleScale sc = kernels::sampleScale(s.geom, n, s.stride, false);
    s.start.assign((size_t)G * F, 0);
    s.cap.assign((size_t)G * F, 0);
    uint64_t cur = 0;
    for (uint32_t d = 0; d < F; ++d)
      for (uint32_t g = 0; g < G; ++g) {
        const size_t i = (size_t)g * F + d;
        double est = 0;
        if (sc.seen[g] > 0) est = (double)s.sampled[i] * sc.total[g] / sc.seen[g];
        // Sampling error of a count scaled by total/seen is ~sqrt(est * total/seen)
        // (at least one sample's worth); 6 sigma + 2% + a fixed floor keeps
        // overflows (and their exact re-run) rare.
        const double scale = sc.seen[g] > 0 ? sc.total[g] / sc.seen[g] : 1.0;
        const double margin = sc.sigmas * std::sqrt(std::max(est, scale) * scale) + sc.frac * est + sc.floor;
        // whole 128-byte lines per slice (16 tuples): slices never share a line
        const uint64_t cap = (std::min<uint64_t>((uint64_t)std::ceil(est + margin), (uint64_t)sc.total[g]) + 15) & ~15ull;
        s.start[i] = cur;
        s.cap[i] = cap;
        cur += cap;
      }
    s.capacityTotal = cur;
    // Claims may run past a slice end by up to n before the overflow is seen:
    // 32-bit cursors only if even that cannot wrap.
    s.narrow = kernels::cursorsNarrow(cur + n);
    // Plan skeleton (filled after the scatter); the window is sized by capacity.
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
    s.window.reset(new data::Window(x, cur, ctx, plan.wide, plan.fragments ? 4u : 0u));
    // Claim cursors (slice starts) and slice ends, in the scatter's cursor width.
    const size_t cb = s.narrow ? 4 : 8;
    s.gcur = ctx->workspace().get((size_t)G * F * cb);
    s.gend = ctx->workspace().get((size_t)G * F * cb);
    // Asynchronous uploads from member vectors (no host round trip before the scatter).
    if (s.narrow) {
      s.cur32.resize((size_t)G * F);
      s.end32.resize((size_t)G * F);
      for (size_t i = 0; i < s.cur32.size(); ++i) {
        s.cur32[i] = (uint32_t)s.start[i];
        s.end32[i] = (uint32_t)(s.start[i] + s.cap[i]);
      }
      ctx->copy(s.gcur, s.cur32.data(), s.cur32.size() * 4, true, false);
      ctx->copy(s.gend, s.end32.data(), s.end32.size() * 4, true, false);
    } else {
      s.end64.resize((size_t)G * F);
      for (size_t i = 0; i < s.end64.size(); ++i) s.end64[i] = s.start[i] + s.cap[i];
      ctx->copy(s.gcur, s.start.data(), s.end64.size() * 8, true, false);
      ctx->copy(s.gend, s.end64.data(), s.end64.size() * 8, true, false);
    }
  }
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
                            static_cast<uint32_t *>(s.window->getData()), ctx->stream(), plan.keyBits, mix, s.gend, nm);
  else if (plan.wide)
    kernels::netScatterWide(s.relation->getData(), n, plan.networkBits, s.geom, 0, s.geom.blocks, s.gcur,
                            static_cast<data::Tuple *>(s.window->getData()), ctx->stream(), mix, s.gend, nm);
  else
    kernels::netScatter(s.relation->getData(), n, plan.networkBits, plan.keyShift, s.geom, 0, s.geom.blocks, s.gcur,
                        static_cast<uint64_t *>(s.window->getData()), ctx->stream(), plan.keyBits, mix, s.gend, nm, !plan.keyOnly);
  ctx->timeline().end(key, ctx->stream());
  const size_t bytes = (size_t)G * F * (s.narrow ? 4 : 8);
  s.cursorsBack = ctx->staging().get(bytes);
  HIP_CHECK(hipMemcpyAsync(s.cursorsBack, s.gcur, bytes, hipMemcpyDeviceToHost, ctx->stream()));
  if (!s.cursorsReady) s.cursorsReady = ctx->acquireEvent();
  HIP_CHECK(hipEventRecord(s.cursorsReady, ctx->stream()));
}

bool SampledNetworkPartitioning::finishSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  Side &s = sides[k];
  HIP_CHECK(hipEventSynchronize(s.cursorsReady));
  s.fill.assign((size_t)G * F, 0);
  const uint32_t *c32 = static_cast<const uint32_t *>(s.cursorsBack);
  const uint64_t *c64 = static_cast<const uint64_t *>(s.cursorsBack);
  bool ok = true;
  uint64_t sum = 0;
  for (size_t i = 0; i < s.fill.size(); ++i) {
    const uint64_t end = s.narrow ? c32[i] : c64[i];  // final claim cursor
    s.fill[i] = end - s.start[i];
    sum += s.fill[i];
    if (s.fill[i] > s.cap[i]) ok = false;
  }
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
