#include "NetworkPartitioning.h"

#include <algorithm>
#include <cstring>

#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

NetworkPartitioning::NetworkPartitioning(uint32_t nodeId, data::Relation *innerRelation,
                                         data::Relation *outerRelation, data::Window *innerWindow,
                                         data::Window *outerWindow, HistogramComputation *histograms,
                                         core::ExecContext *ctx, const core::JoinPlan &plan)
    : nodeId(nodeId), innerRelation(innerRelation), outerRelation(outerRelation), innerWindow(innerWindow),
      outerWindow(outerWindow), histograms(histograms), ctx(ctx), plan(plan) {}

NetworkPartitioning::~NetworkPartitioning() {}

void NetworkPartitioning::execute() {
  partition(innerRelation, innerWindow, histograms->innerLocal(), histograms->innerOffsetMap()->getExchangePlan());
  partition(outerRelation, outerWindow, histograms->outerLocal(), histograms->outerOffsetMap()->getExchangePlan());
}

void NetworkPartitioning::partitionInner(const std::function<void(uint32_t)> &afterChunk) {
  partition(innerRelation, innerWindow, histograms->innerLocal(), histograms->innerOffsetMap()->getExchangePlan(),
            afterChunk);
}

void NetworkPartitioning::partitionOuter(data::Window *window) {
  outerWindow = window;
  partition(outerRelation, outerWindow, histograms->outerLocal(), histograms->outerOffsetMap()->getExchangePlan());
}

void NetworkPartitioning::partition(data::Relation *relation, data::Window *window,
                                    histograms::LocalHistogram *local, const histograms::ExchangePlan &xp,
                                    const std::function<void(uint32_t)> &afterChunk) {
  const uint64_t n = relation->getLocalSize();
  JOIN_ASSERT(xp.scatterTotal == n, "NetworkPartitioning", "plan scatters %lu of %lu tuples",
              (unsigned long)xp.scatterTotal, (unsigned long)n);
  const uint32_t bits = plan.networkBits, F = 1u << bits;
  kernels::PartitionGeometry g = local->geometry();
  g.ipt = plan.variants.netIpt;
  g.nth = plan.variants.netThreads;
  const uint32_t bpc = local->blocksPerChunk(), chunks = local->getChunkCount();
  const bool single = xp.numberOfNodes == 1;
  const uint32_t tb = window->tupleBytes();
  const bool isInner = relation == innerRelation;
  const char *kMain = isInner ? "MIMAINPART" : "MOMAINPART";
  const char *kFlush = isInner ? "MIFLUSHPART" : "MOFLUSHPART";
  const uint64_t tAlloc = performance::nowUs();
  // One-sided device windows take the scatter's stores directly: no send buffer.
  // Replicated runs (split hot partitions) are copied inside a send buffer.
  const bool direct = !single && window->directScatter();
  void *send = single ? window->getData() : direct ? nullptr : ctx->workspace().get(std::max<uint64_t>(xp.sendTotal, 1) * tb);
  // Copies of chunk c's replicated runs, once its scatter is done.
  auto replicate = [&](uint32_t c) {
    for (const histograms::Replica &r : xp.replicas) {
      if (r.chunk != c) continue;
      uint8_t *b = static_cast<uint8_t *>(send);
      if (ctx->onDevice())
        HIP_CHECK(hipMemcpyAsync(b + r.dst * tb, b + r.src * tb, r.len * tb, hipMemcpyDeviceToDevice, ctx->stream()));
      else
        std::memcpy(b + r.dst * tb, b + r.src * tb, r.len * tb);
    }
  };
  performance::Measurements::add(isInner ? "MIMEMALLOC" : "MOMEMALLOC", (double)(performance::nowUs() - tAlloc), "us");
  window->start();
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  performance::Timeline &tl = ctx->timeline();
  tl.begin(kMain, ctx->stream());
  if (ctx->onDevice()) {
    // Claim-mode scatter: per-(chunk, XCD group, digit) slices, one device
    // atomic per digit per 8192-tuple tile (kernels.h, CLAIM_GROUPS).
    // Direct scatter: cursors are absolute tuple indices (8 bytes wide).
    const bool narrow = !direct && kernels::cursorsNarrow(n);
    const uint64_t cb = narrow ? 4 : 8, perChunk = (uint64_t)kernels::CLAIM_GROUPS * F * cb;
    uint8_t *gcur = static_cast<uint8_t *>(ctx->workspace().get(chunks * perChunk));
    uint64_t *base = ctx->workspace().getArray<uint64_t>((uint64_t)chunks * F);
    if (direct) {
      const std::vector<uint64_t> db = window->directDigitBase();
      ctx->copy(base, db.data(), db.size() * 8, true, false);
    } else {
      ctx->copy(base, xp.digitBase.data(), xp.digitBase.size() * 8, true, false);
    }
    kernels::netGroupCursors(local->blockHistogram(), F, g.blocks, bpc, base, gcur, narrow, ctx->stream());
    for (uint32_t c = 0; c < chunks; ++c) {
      const uint32_t b0 = c * bpc, b1 = std::min(g.blocks, b0 + bpc);
      const int narrowMode = narrow ? 1 : 0;
      if (plan.wide)
        kernels::netScatterWide(relation->getData(), n, bits, g, b0, b1, gcur + c * perChunk,
                                static_cast<data::Tuple *>(send), ctx->stream(), mix, nullptr, narrowMode);
      else
        kernels::netScatter(relation->getData(), n, bits, plan.keyShift, g, b0, b1, gcur + c * perChunk,
                            static_cast<uint64_t *>(send), ctx->stream(), plan.keyBits, mix, nullptr, narrowMode,
                            !plan.keyOnly);
      replicate(c);
      if (!single) window->exchange(send, c);
      if (afterChunk) afterChunk(c);
    }
  } else {
    uint64_t *cursors = ctx->workspace().getArray<uint64_t>((uint64_t)F * g.blocks);
    host::netCursors(local->blockHistogram(), F, g.blocks, bpc, xp.digitBase.data(), cursors);
    for (uint32_t c = 0; c < chunks; ++c) {
      const uint32_t b0 = c * bpc, b1 = std::min(g.blocks, b0 + bpc);
      host::netScatter(relation->getData(), n, bits, plan.keyShift, g, b0, b1, cursors, send, plan.wide, mix,
                       !plan.keyOnly);
      replicate(c);
      if (!single) window->exchange(send, c);
      if (afterChunk) afterChunk(c);
    }
  }
  // The reference's MxFLUSHPART is its tail flush + flush_local_all: here the
  // time from the last scatter to the last exchange chunk having landed.
  tl.end(kMain, ctx->stream());
  tl.begin(kFlush, ctx->stream());
  tl.end(kFlush, window->completionStream());
}

}  // namespace tasks
}  // namespace hpcjoin
