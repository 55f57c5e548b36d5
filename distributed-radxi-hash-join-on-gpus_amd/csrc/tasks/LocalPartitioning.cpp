#include "LocalPartitioning.h"

#include <cstdlib>
#include <cstring>

#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

LocalPartitioning::LocalPartitioning(data::Window *innerWindow, data::Window *outerWindow, core::ExecContext *ctx,
                                     const core::JoinPlan &plan, bool forceExact)
    : ctx(ctx), plan(plan), forceExact(forceExact) {
  windows[0] = innerWindow;
  windows[1] = outerWindow;
}

LocalPartitioning::~LocalPartitioning() {}

void LocalPartitioning::execute() {
  if (!innerDone) partition(windows[0], 0);
  innerDone = true;
  partition(windows[1], 1);
}

bool LocalPartitioning::overflowed() const {
  if (overflowFlag.empty()) return false;
  ctx->synchronize();  // no-op after the caller's sync
  for (unsigned int *b : overflowBack)
    if (b && *b != 0) return true;
  return false;
}

void LocalPartitioning::partition(data::Window *w, int which) {
  w->stop();  // compute stream now waits for this window's exchanges
  performance::Timeline &tl = ctx->timeline();
  tl.begin("LPTASKTIME", ctx->stream());
  partitionImpl(w, which);
  tl.end("LPTASKTIME", ctx->stream());
}

// Bytes and host time of this pass's workspace carve-outs (LPMEMSIZE / LPMEMALLOC).
void *LocalPartitioning::alloc(uint64_t bytes) {
  const uint64_t t0 = performance::nowUs();
  void *p = ctx->workspace().get(bytes);
  performance::Measurements::add("LPMEMALLOC", (double)(performance::nowUs() - t0), "us");
  performance::Measurements::add("LPMEMSIZE", (double)bytes, "bytes");
  return p;
}

void LocalPartitioning::partitionImpl(data::Window *w, int which) {
  performance::Timeline &tl = ctx->timeline();
  const histograms::ExchangePlan &xp = w->getPlan();
  const uint32_t owned = (uint32_t)xp.owned.size();
  const bool wide = w->isWide();
  const uint32_t tb = w->tupleBytes();
  elements += xp.recvTotal;

  JOIN_ASSERT(!w->roundMap().on() || (ctx->onDevice() && plan.twoLevel), "LocalPartitioning",
              "round-interleaved windows are read by the device two-level pass only");
  if (!plan.twoLevel && xp.windowIsPartitionMajor()) {
    uint64_t *pb = ctx->workspace().getArray<uint64_t>(owned + 1);
    ctx->copy(pb, xp.lpBase.data(), (owned + 1) * 8, ctx->onDevice(), false);
    w->setPartitioned(w->getData(), pb, 0);
    return;
  }
  const uint32_t bits = plan.twoLevel ? plan.localBits : 0, F = 1u << bits;
  if ((size_t)which >= items.size()) {
    items.resize(which + 1);
    lpItemBegin.resize(which + 1);
  }
  std::vector<kernels::LocalItem> &it = items[which];
  std::vector<uint32_t> &lb = lpItemBegin[which];
  it.clear();
  lb.assign(owned + 1, 0);
  size_t seg = 0;
  const uint64_t itemMax = (uint64_t)plan.localItemTiles * kernels::PART_TILE;
  for (uint32_t lp = 0; lp < owned; ++lp) {
    lb[lp] = (uint32_t)it.size();
    for (; seg < xp.segments.size() && xp.segments[seg].lp == lp; ++seg)
      for (uint64_t off = 0; off < xp.segments[seg].len; off += itemMax) {
        const uint64_t len = std::min<uint64_t>(itemMax, xp.segments[seg].len - off);
        it.push_back(kernels::LocalItem{xp.segments[seg].begin + off, (uint32_t)len, lp, 0, 0});
      }
  }
  lb[owned] = (uint32_t)it.size();
  const uint32_t nItems = (uint32_t)it.size();
  itemTotal += nItems;
  // Count-only fragments (JoinPlan::fragments): the window holds u32 words
  // key >> networkBits; the local digit is their low bits and the output is
  // only the u16 fragment column (no rid column exists).
  const bool frag = w->holdsFragments();
  const uint32_t shift = frag ? 0 : wide ? plan.networkBits : plan.keyShift;
  // Split output columns (kernels.h, SplitLayout): device, compressed, planned to fit.
  kernels::SplitLayout split;
  split.on = ctx->onDevice() && !wide && (plan.splitLocal || frag) ? 1u : 0u;
  split.fragShift = frag ? bits : plan.fragShift;
  if (plan.keyOnly) {  // key fragment above both digits: low 32 bits + next 16 (makePlan checked it fits)
    split.loShift = bits;
    split.fragShift = bits + 32;
  }
  JOIN_ASSERT(!frag || (ctx->onDevice() && plan.twoLevel), "LocalPartitioning", "fragments need the device two-level path");
  const uint32_t ob = frag ? 2 : split.on ? 4 : tb;  // bytes per tuple of the main output column
  const uint32_t align = split.on ? 64 : 16;   // slot granularity: whole 128-byte lines of every column

  uint32_t *itemHist = ctx->workspace().getArray<uint32_t>(std::max<uint64_t>(1, (uint64_t)nItems * F));

  const bool sampledMode =
      ctx->onDevice() && !forceExact && plan.twoLevel && bits > 0 &&
      (plan.localHistogram == core::HistogramMode::Sampled ||
       (plan.localHistogram == core::HistogramMode::Auto && xp.recvTotal >= (16ull << 20)));
  if (sampledMode) {
    anySampled = true;
    // One claim stream per network partition (its items are XCD-contiguous
    // except at group boundaries), so every final partition is one slot.
    for (auto &x : it) x.stream = x.lp;
    const uint64_t P = (uint64_t)owned * F;
    const uint32_t S = plan.localSampleStride;
    const uint64_t cap = kernels::localSampledCapacityBound(xp.recvTotal, P, S, align);
    // HPCJOIN_LP_SKEW="lo:hi" (bytes, experiments only): start the output
    // columns that far into their allocations (HBM channel placement A/B).
    uint64_t skewLo = 0, skewHi = 0;
    if (const char *e = std::getenv("HPCJOIN_LP_SKEW")) {
      skewLo = std::strtoull(e, nullptr, 0);
      if (const char *c = std::strchr(e, ':')) skewHi = std::strtoull(c + 1, nullptr, 0);
    }
    void *sout = static_cast<uint8_t *>(alloc(std::max<uint64_t>(cap, 1) * ob + skewLo)) + skewLo;
    if (frag) split.hi = static_cast<uint16_t *>(sout);
    else if (split.on)
      split.hi = reinterpret_cast<uint16_t *>(static_cast<uint8_t *>(alloc(std::max<uint64_t>(cap, 1) * 2 + skewHi)) +
                                              skewHi);
    uint32_t *caps = ctx->workspace().getArray<uint32_t>(std::max<uint64_t>(P, 1));
    auto *starts = ctx->workspace().getArray<unsigned long long>(std::max<uint64_t>(P, 1));
    void *scanWs = ctx->workspace().get(kernels::scanWorkspaceBytes(std::max<uint64_t>(P, 1)));
    auto *gcur = ctx->workspace().getArray<unsigned long long>(std::max<uint64_t>(P, 1));
    auto *gend = ctx->workspace().getArray<unsigned long long>(std::max<uint64_t>(P, 1));
    uint64_t *pbeg = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(P, 1));
    kernels::LocalItem *dItems = ctx->workspace().getArray<kernels::LocalItem>(std::max<uint32_t>(nItems, 1));
    uint32_t *dLb = ctx->workspace().getArray<uint32_t>(owned + 1);
    if (overflowFlag.size() <= (size_t)which) {
      overflowFlag.resize(which + 1, nullptr);
      overflowBack.resize(which + 1, nullptr);
    }
    if (!overflowFlag[which]) overflowFlag[which] = ctx->workspace().getArray<unsigned int>(1);
    // HPCJOIN_LP_PREP=1 (A/B only): the sampled histogram and the slot
    // layout, which read only this window, run on the decode stream (idle at
    // N = 1) next to whatever the compute stream still does -- the outer
    // network scatter for the inner side, the inner local scatter for the
    // outer side -- once the window's data is complete (Window::dataReady).
    // Measured neutral (18.97 vs 18.93 ms per 1B x 1B general join: the
    // overlapped histograms slow the scatters beside them by as much as they
    // hide, profiles/r6/ab/lp_prep_stream_r7q.jsonl), so off by default.
    const char *pe = std::getenv("HPCJOIN_LP_PREP");
    const bool prep = w->dataReady() && ctx->numberOfNodes() == 1 && pe && pe[0] == '1';
    const hipStream_t ps = prep ? ctx->decodeStream() : ctx->stream();
    if (prep) HIP_CHECK(hipStreamWaitEvent(ps, w->dataReady(), 0));
    ctx->copy(dItems, it.data(), (uint64_t)nItems * sizeof(kernels::LocalItem), true, false, ps);
    ctx->copy(dLb, lb.data(), (owned + 1) * 4ull, true, false, ps);
    ctx->zero(overflowFlag[which], sizeof(unsigned int), ps);
    performance::Measurements::add("LPHISTELEM", (double)(xp.recvTotal / S), "tuples");
    // Back-to-back spans on one stream share their boundary events.
    hipEvent_t p0 = tl.mark(ps);
    tl.beginAt("LPHISTCOMP", p0);
    kernels::localHistogram(w->getData(), wide, dItems, nItems, shift, bits, itemHist, ps, S, frag, w->roundMap());
    hipEvent_t p1 = tl.mark(ps);
    tl.endAt("LPHISTCOMP", p1);
    tl.beginAt("LPOFFSET", p1);
    kernels::localSampledLayout(itemHist, dLb, dItems, owned, bits, S, caps, starts, scanWs, gcur, gend, pbeg, cap,
                                ps, align);
    hipEvent_t p2 = tl.mark(ps);
    tl.endAt("LPOFFSET", p2);
    if (prep) {
      hipEvent_t done = ctx->acquireEvent();
      HIP_CHECK(hipEventRecord(done, ps));
      HIP_CHECK(hipStreamWaitEvent(ctx->stream(), done, 0));
      p2 = tl.mark(ctx->stream());
    }
    tl.beginAt("LPPART", p2);
    kernels::localScatter(w->getData(), wide, dItems, nItems, shift, bits, gcur, false, sout, ctx->stream(), gend,
                          split, plan.localGeometry, frag, w->roundMap());
    tl.endAt("LPPART", tl.mark(ctx->stream()));
    kernels::claimOverflow(gcur, gend, P, overflowFlag[which], ctx->stream());
    // Read back with the join's final synchronisation (one flag per side).
    if (!overflowBack[which]) overflowBack[which] = ctx->staging().getArray<unsigned int>(1);
    ctx->readBack(overflowBack[which], overflowFlag[which], sizeof(unsigned int));
    // Final claim cursors are the partition ends (valid when no slot overflowed).
    w->setPartitioned(sout, pbeg, bits, reinterpret_cast<const uint64_t *>(gcur), split.hi, std::max<uint64_t>(cap, 1));
    return;
  }
  void *out = alloc(std::max<uint64_t>(xp.recvTotal, 1) * ob);
  if (frag) split.hi = static_cast<uint16_t *>(out);
  else if (split.on) split.hi = static_cast<uint16_t *>(alloc(std::max<uint64_t>(xp.recvTotal, 1) * 2));
  uint64_t *partBegin = ctx->workspace().getArray<uint64_t>((uint64_t)owned * F + 1);
  if (ctx->onDevice()) {
    const uint32_t streams = kernels::assignLocalStreams(it.data(), nItems);
    const bool narrow = kernels::cursorsNarrow(xp.recvTotal);
    void *gcur = ctx->workspace().get(std::max<uint64_t>(1, (uint64_t)streams * F) * (narrow ? 4 : 8));
    kernels::LocalItem *dItems = ctx->workspace().getArray<kernels::LocalItem>(std::max<uint32_t>(nItems, 1));
    uint32_t *dLb = ctx->workspace().getArray<uint32_t>(owned + 1);
    uint64_t *dBase = ctx->workspace().getArray<uint64_t>(owned + 1);
    ctx->copy(dItems, it.data(), (uint64_t)nItems * sizeof(kernels::LocalItem), true, false);
    ctx->copy(dLb, lb.data(), (owned + 1) * 4ull, true, false);
    ctx->copy(dBase, xp.lpBase.data(), (owned + 1) * 8ull, true, false);
    if (owned == 0) {
      zero.assign(1, 0);
      ctx->copy(partBegin, zero.data(), 8, true, false);
    }
    performance::Measurements::add("LPHISTELEM", (double)xp.recvTotal, "tuples");
    hipEvent_t p0 = tl.mark(ctx->stream());
    tl.beginAt("LPHISTCOMP", p0);
    kernels::localHistogram(w->getData(), wide, dItems, nItems, shift, bits, itemHist, ctx->stream(), 1, frag,
                            w->roundMap());
    hipEvent_t p1 = tl.mark(ctx->stream());
    tl.endAt("LPHISTCOMP", p1);
    tl.beginAt("LPOFFSET", p1);
    kernels::localCursors(itemHist, dLb, owned, bits, dBase, dItems, gcur, narrow, partBegin, ctx->stream());
    hipEvent_t p2 = tl.mark(ctx->stream());
    tl.endAt("LPOFFSET", p2);
    tl.beginAt("LPPART", p2);
    kernels::localScatter(w->getData(), wide, dItems, nItems, shift, bits, gcur, narrow, out, ctx->stream(), nullptr,
                          split, 0, frag, w->roundMap());
    tl.endAt("LPPART", tl.mark(ctx->stream()));
  } else {
    uint64_t *itemCursors = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(1, (uint64_t)nItems * F));
    if (owned == 0) partBegin[0] = 0;
    performance::Measurements::add("LPHISTELEM", (double)xp.recvTotal, "tuples");
    tl.begin("LPHISTCOMP");
    host::localHistogram(w->getData(), wide, it.data(), nItems, shift, bits, itemHist);
    tl.end("LPHISTCOMP");
    tl.begin("LPOFFSET");
    host::localCursors(itemHist, lb.data(), owned, bits, xp.lpBase.data(), itemCursors, partBegin);
    tl.end("LPOFFSET");
    tl.begin("LPPART");
    host::localScatter(w->getData(), wide, it.data(), nItems, shift, bits, itemCursors, out);
    tl.end("LPPART");
  }
  w->setPartitioned(out, partBegin, bits, nullptr, split.hi, std::max<uint64_t>(xp.recvTotal, 1));
}

}  // namespace tasks
}  // namespace hpcjoin
