#include "BitmapJoin.h"

#include <algorithm>
#include <cmath>
#include <map>
#include <tuple>
#include <cstdlib>
#include <vector>

#include "../comm/Communicator.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../performance/Trace.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

using kernels::BitmapCounters;
using kernels::BitmapSlices;
using kernels::CLAIM_GROUPS;

BitmapJoin::BitmapJoin(data::Relation *innerRelation, data::Relation *outerRelation, core::ExecContext *ctx,
                       const core::JoinPlan &plan, uint32_t maxBlocks, uint32_t sampleStride, hipEvent_t *ev)
    : inner(innerRelation), outer(outerRelation), ctx(ctx), plan(plan), maxBlocks(maxBlocks),
      sampleStride(std::max<uint32_t>(1, sampleStride)), ev(ev) {
  JOIN_ASSERT(plan.bitmapJoin && !plan.materialize && !plan.wide, "BitmapJoin", "needs a counting bitmap plan");
  JOIN_ASSERT(plan.bitmapBits <= kernels::BITMAP_MAX_BITS + kernels::BITMAP_MAX_SPLIT, "BitmapJoin",
              "%u fragment bits do not fit a bitmap", plan.bitmapBits);
  JOIN_ASSERT(kernels::fragWordFits(plan.keyBits, plan.networkBits), "BitmapJoin",
              "%u-bit keys do not leave a u32 fragment above %u radix bits", plan.keyBits, plan.networkBits);
}

BitmapJoin::Outcome BitmapJoin::run(bool exact) { return ctx->onDevice() ? runDevice(exact) : runHost(); }

// Geometry, sample stride, scale and capacity bound of one side: pure
// functions of the sizes, but their host loops (every block and sampled tile)
// took ~20 us per join in front of the first kernel, so they are computed
// once per thread (in-process ranks are threads) and size.
const BitmapJoin::SidePlan &BitmapJoin::sidePlan(uint64_t n, bool exact, uint32_t stride) const {
  struct Key {
    uint64_t n;
    uint32_t maxBlocks, bits, stride, ipt, nth, lp;
    bool exact;
    bool operator<(const Key &o) const {
      return std::tie(n, maxBlocks, bits, stride, ipt, nth, lp, exact) <
             std::tie(o.n, o.maxBlocks, o.bits, o.stride, o.ipt, o.nth, o.lp, o.exact);
    }
  };
  thread_local std::map<Key, SidePlan> cache;
  const uint32_t F = 1u << plan.networkBits;
  const Key k{n, maxBlocks, plan.networkBits, stride, plan.variants.netIpt, plan.variants.netThreads, plan.roundLp,
              exact};
  auto it = cache.find(k);
  if (it != cache.end()) return it->second;
  if (cache.size() > 64) cache.clear();
  SidePlan sp;
  sp.geom = kernels::partitionGeometry(n, maxBlocks);
  sp.geom.ipt = plan.variants.netIpt;
  sp.geom.nth = plan.variants.netThreads;
  sp.stride = exact ? 1 : kernels::sampleStrideFor(sp.geom, n, F, stride);
  sp.sc = kernels::sampleScale(sp.geom, n, sp.stride, exact);
  sp.cap = kernels::sampledWindowCapacity(sp.sc, F, kernels::roundLpFor(plan.roundLp, 4));
  return cache.emplace(k, sp).first->second;
}

// Sampled (or exact) histogram -> device layout of bounded claim slices ->
// bounded claim scatter of u32 fragments.  Nothing here waits for the device.
bool BitmapJoin::sideNarrow(data::Relation *r, bool exact) const {
  const uint64_t n = r->getLocalSize();
  return kernels::cursorsNarrow(sidePlan(n, exact, sampleStride).cap + n);
}

// Sampled (or exact) totals and the device layout of the bounded claim
// slices of one or both sides: one totals launch and one layout launch for
// both (every kernel boundary is ~5 us of idle GPU).
void BitmapJoin::layoutSides(Side *sides, uint32_t count, bool exact, bool narrowOk) {
  const uint32_t bits = plan.networkBits, F = 1u << bits, G = CLAIM_GROUPS;
  memory::Arena &ws = ctx->workspace();
  const hipStream_t st = ctx->stream();
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  // Adjacent: one clear -- or none, in the engine's control block (N = 1),
  // which the layout kernel returns to zero after reading.
  uint64_t *totals = useControl ? reinterpret_cast<uint64_t *>(ctx->control()->totals)
                                : ws.getArray<uint64_t>((uint64_t)count * G * F);
  kernels::SampledInput in[2];
  kernels::LayoutInput lay[2];
  bool sampled = !exact;
  bool narrow = narrowOk;
  for (uint32_t i = 0; i < count; ++i) {
    Side &s = sides[i];
    const uint64_t n = s.relation->getLocalSize();
    const SidePlan &sp = sidePlan(n, exact, sampleStride);
    s.geom = sp.geom;
    const uint32_t stride = sp.stride;
    sampled = sampled && stride > 1;
    in[i] = kernels::SampledInput{s.relation->getData(), n, s.geom, stride, totals + (size_t)i * G * F};
    const kernels::SampleScale &sc = sp.sc;
    s.cap = sp.cap;
    // Claims may run past a slice end by up to n before the overflow is seen.
    narrow = narrow && kernels::cursorsNarrow(s.cap + n);
    lay[i].sampled = in[i].totals;
    lay[i].sc = sc;
    lay[i].clearSampled = useControl;
  }
  if (sampled) {
    kernels::netSampledTotals(in, count, bits, st, mix, useControl);
  } else {  // exact histograms (or an input too small to sample): every tile, per block
    for (uint32_t i = 0; i < count; ++i) {
      uint32_t *blockHist = ws.getArray<uint32_t>((uint64_t)F * in[i].geom.blocks);
      kernels::netHistogram(in[i].data, in[i].n, bits, in[i].geom, blockHist, st, mix, 1);
      kernels::netGroupTotals(blockHist, F, in[i].geom.blocks, in[i].totals, st);
      if (in[i].stride > 1) {  // sampled side next to an exact one: its scale counts every tile now
        const SidePlan &one = sidePlan(in[i].n, exact, 1);
        lay[i].sc = one.sc;
        sides[i].cap = one.cap;
      }
    }
  }
  const size_t cb = narrow ? 4 : 8;
  // Round-interleaved fragment windows (kernels::RoundMap): the slots follow
  // from the layout kernel's map, which every reader takes from roundMeta.
  const uint32_t lp = kernels::roundLpFor(plan.roundLp, 4);
  uint32_t lns = 0;
  while ((1u << lns) < G * F) ++lns;
  for (uint32_t i = 0; i < count; ++i) {
    lay[i].gstart = ws.get((size_t)G * F * cb);
    lay[i].gcur = ws.get((size_t)G * F * cb);
    lay[i].gend = ws.get((size_t)G * F * cb);
    lay[i].capacityUsed = ws.getArray<unsigned long long>(1);
    if (lp) {
      // Logical positions reach (G * F << lv) + n (claims past a slice end).
      const uint64_t n = sides[i].relation->getLocalSize(), limit = narrow ? (1ull << 32) : (1ull << 62);
      uint32_t maxLv = 0;
      while (maxLv < 40 && ((uint64_t)G * F << (maxLv + 1)) + n < limit) ++maxLv;
      lay[i].roundMeta = ws.getArray<uint32_t>(4);
      lay[i].roundLp = lp;
      lay[i].roundMaxLv = maxLv;
      lay[i].roundCapacity = sides[i].cap;
    }
    Side &s = sides[i];
    s.slices = BitmapSlices();
    s.slices.kind = BitmapSlices::Claim;
    s.slices.start = lay[i].gstart;
    s.slices.cur = lay[i].gcur;
    s.slices.end = lay[i].gend;
    s.slices.narrow = narrow;
    s.slices.count = s.relation->getLocalSize();
    s.slices.threads = plan.variants.bmThreads;
    s.slices.flat = plan.variants.bmFlat;
    s.slices.roundMeta = lay[i].roundMeta;
    s.frags = ws.getArray<uint32_t>(std::max<uint64_t>(s.cap, 16));
  }
  kernels::netSampledLayout(lay, count, F, narrow, st);
}

// The bounded claim scatter of one side's u32 fragments into its slices.
void BitmapJoin::scatterSide(Side &s) {
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  kernels::netScatterFrag(s.relation->getData(), s.relation->getLocalSize(), plan.networkBits, s.geom, 0,
                          s.geom.blocks, const_cast<void *>(s.slices.cur), s.frags, ctx->stream(), plan.keyBits, mix,
                          s.slices.end, s.slices.narrow ? 1 : 0, s.slices.roundMeta);
}

// Partition ranges of the replicated plan's all-reduce: one per 32 MiB of
// bitmaps, at most 4 (1B dense keys: 4 x 32 MiB).  Each range is one more
// collective (~10-30 us of launch and handshake over xGMI), against the probe
// of all but the last range moving behind the all-reduce.
// KernelVariants::reduceChunks = k forces k.
static uint32_t reduceChunks(uint64_t bitmapBytes, uint32_t forced) {
  if (forced) return std::max<uint32_t>(1, std::min<uint32_t>(forced, 64));
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4, bitmapBytes >> 25));
}

BitmapJoin::Outcome BitmapJoin::runDeviceGroups(bool exact) {
  const uint32_t nb = plan.networkBits, F = 1u << nb, G = CLAIM_GROUPS, bits = plan.bitmapBits;
  const hipStream_t st = ctx->stream();
  memory::Arena &ws = ctx->workspace();
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  performance::Timeline &tl = ctx->timeline();
  useControl = false;
  auto *cnt = ws.getArray<BitmapCounters>(1);
  ctx->zero(cnt, sizeof(BitmapCounters));
  Side both[2] = {Side{inner, {}, nullptr, {}}, Side{outer, {}, nullptr, {}}};
  // 1. Totals of every digit of both sides (sampled, or exact), read back once.
  uint64_t *totals = ws.getArray<uint64_t>((uint64_t)2 * G * F);
  kernels::SampleScale sc[2];
  {
    kernels::SampledInput in[2];
    bool sampled = !exact;
    for (int i = 0; i < 2; ++i) {
      const uint64_t n = both[i].relation->getLocalSize();
      const SidePlan &sp = sidePlan(n, exact, sampleStride);
      both[i].geom = sp.geom;
      sc[i] = sp.sc;
      sampled = sampled && sp.stride > 1;
      in[i] = kernels::SampledInput{both[i].relation->getData(), n, sp.geom, sp.stride, totals + (size_t)i * G * F};
    }
    utils::faultPoint("network");
    tl.beginSplitAt("HLOCAL", "HILOCAL", (double)inner->getLocalSize(), "HOLOCAL", (double)outer->getLocalSize(),
                    ev[0]);
    if (sampled) {
      kernels::netSampledTotals(in, 2, nb, st, mix, false);
    } else {
      for (int i = 0; i < 2; ++i) {
        uint32_t *blockHist = ws.getArray<uint32_t>((uint64_t)F * in[i].geom.blocks);
        kernels::netHistogram(in[i].data, in[i].n, nb, in[i].geom, blockHist, st, mix, 1);
        kernels::netGroupTotals(blockHist, F, in[i].geom.blocks, in[i].totals, st);
        if (in[i].stride > 1) sc[i] = sidePlan(in[i].n, exact, 1).sc;  // every tile counted now
      }
    }
  }
  uint64_t *back = ctx->staging().getArray<uint64_t>((uint64_t)2 * G * F);
  ctx->readBack(back, totals, (size_t)2 * G * F * 8);
  HIP_CHECK(hipEventRecord(ev[1], st));
  tl.endAt("HLOCAL", ev[1]);
  utils::waitEvent(ev[1], ctx->comm(), "bitmap group totals");
  // 2. Slice capacities per digit (netSampledLayoutKernel's formula, plus one
  // line per slice against rounding differences), then groups of consecutive
  // digits whose two windows fit the budget.  A group has fewer than 1024
  // digits (netScatterFragRange keeps one sentinel counter in LDS).
  std::vector<uint64_t> digitCap[2];
  for (int i = 0; i < 2; ++i) {
    digitCap[i].assign(F, 0);
    for (uint32_t g = 0; g < G; ++g) {
      const double seen = sc[i].seen[g], total = sc[i].total[g];
      if (!(seen > 0)) continue;
      const double scale = total / seen;
      for (uint32_t d = 0; d < F; ++d) {
        const double est = (double)back[((size_t)i * G + g) * F + d] * scale;
        const double margin = sc[i].sigmas * std::sqrt(std::max(est, scale) * scale) + sc[i].frac * est + sc[i].floor;
        const uint64_t c = (uint64_t)std::min(std::ceil(est + margin), total);
        digitCap[i][d] += ((c + 15) & ~15ull) + 16;
      }
    }
  }
  struct Group {
    uint32_t lo = 0, n = 0;
    uint64_t cap[2] = {0, 0};
  };
  std::vector<Group> groups;
  const uint64_t budget = std::max<uint64_t>(plan.groupBudget / 4, 1);  // u32 fragments
  const uint32_t maxRange = 512;
  Group cur;
  for (uint32_t d = 0; d < F; ++d) {
    const uint64_t add = digitCap[0][d] + digitCap[1][d];
    HJ_CHECK(add <= budget, "capacity spill: network partition %u needs %lu fragment slots, the budget holds %lu", d,
             (unsigned long)add, (unsigned long)budget);
    if (cur.n && (cur.cap[0] + cur.cap[1] + add > budget || cur.n == maxRange)) {
      groups.push_back(cur);
      cur = Group();
      cur.lo = d;
    }
    ++cur.n;
    cur.cap[0] += digitCap[0][d];
    cur.cap[1] += digitCap[1][d];
  }
  groups.push_back(cur);
  uint64_t maxCap[2] = {0, 0};
  for (const Group &g : groups)
    for (int i = 0; i < 2; ++i) maxCap[i] = std::max(maxCap[i], g.cap[i]);
  // One cursor width for both sides (claims may run past a slice end by up to n).
  const bool narrow = kernels::cursorsNarrow(maxCap[0] + inner->getLocalSize()) &&
                      kernels::cursorsNarrow(maxCap[1] + outer->getLocalSize());
  const size_t cb = narrow ? 4 : 8;
  kernels::LayoutInput lay[2];
  for (int i = 0; i < 2; ++i) {
    Side &sd = both[i];
    sd.frags = ws.getArray<uint32_t>(maxCap[i] + 4096);
    lay[i].sampled = totals + (size_t)i * G * F;
    lay[i].sc = sc[i];
    lay[i].gstart = ws.get((size_t)G * maxRange * cb);
    lay[i].gcur = ws.get((size_t)G * maxRange * cb);
    lay[i].gend = ws.get((size_t)G * maxRange * cb);
    lay[i].capacityUsed = ws.getArray<unsigned long long>(1);
    lay[i].clearSampled = false;
    sd.slices = BitmapSlices();
    sd.slices.kind = BitmapSlices::Claim;
    sd.slices.start = lay[i].gstart;
    sd.slices.cur = lay[i].gcur;
    sd.slices.end = lay[i].gend;
    sd.slices.narrow = narrow;
    sd.slices.threads = plan.variants.bmThreads;
    sd.slices.flat = plan.variants.bmFlat;
  }
  // 3. One pass per group: lay out its slices, scatter its digits of both
  // relations, join its bitmaps (the counters accumulate).
  tl.beginAt("MIMAINPART", ev[1]);
  for (size_t k = 0; k < groups.size(); ++k) {
    const Group &g = groups[k];
    kernels::netSampledLayout(lay, 2, F, narrow, st, g.lo, g.n);
    for (int i = 0; i < 2; ++i) {
      Side &sd = both[i];
      sd.slices.count = g.cap[i];  // the bitmap kernels' flat-walk choice: tuples per partition
      kernels::netScatterFragRange(sd.relation->getData(), sd.relation->getLocalSize(), nb, sd.geom,
                                   const_cast<void *>(sd.slices.cur), sd.frags, st, plan.keyBits, mix, sd.slices.end,
                                   narrow, g.lo, g.n);
    }
    if (k + 1 == groups.size()) {
      HIP_CHECK(hipEventRecord(ev[2], st));
      tl.endAt("MIMAINPART", ev[2]);
      utils::faultPoint("local");
      utils::faultPoint("build_probe");
    }
    kernels::bitmapJoin(4, both[0].frags, both[1].frags, both[0].slices, both[1].slices, g.n, 0, bits, cnt, st);
  }
  HIP_CHECK(hipEventRecord(ev[4], st));
  tl.beginAt("BPTASKTIME", ev[2]);
  tl.endAt("BPTASKTIME", ev[4]);
  performance::Measurements::add("BPBUILDELEM", (double)inner->getLocalSize(), "tuples");
  performance::Measurements::add("BPPROBEELEM", (double)outer->getLocalSize(), "tuples");
  BitmapCounters *res = ctx->staging().getArray<BitmapCounters>(1);
  const uint64_t tEnqueued = performance::nowUs();
  ctx->readBack(res, cnt, sizeof(BitmapCounters));
  ctx->synchronize();
  Outcome o;
  o.hostWaitMs = (performance::nowUs() - tEnqueued) / 1000.0;
  o.enqueueUs = tEnqueued;
  o.groupPasses = (uint32_t)groups.size();
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
  o.devSampleMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[1], ev[2]));
  o.devScatterMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[2], ev[4]));
  o.devJoinMs = ms;
  o.localMatches = res->matches;
  o.popcount = res->popcount;
  agree(o, (res->dup ? kernels::BM_FLAG_DUP : 0u) | (res->overflow ? kernels::BM_FLAG_OVERFLOW : 0u));
  return o;
}

BitmapJoin::Outcome BitmapJoin::runDevice(bool exact) {
  if (plan.groupBudget && ctx->numberOfNodes() == 1) return runDeviceGroups(exact);
  const uint32_t F = 1u << plan.networkBits, N = ctx->numberOfNodes(), bits = plan.bitmapBits;
  const hipStream_t st = ctx->stream();
  memory::Arena &ws = ctx->workspace();
  // One rank: counters and sampled totals in the engine's control block
  // (no memset) and the result delivered through the host-mapped mailbox (no
  // copy): the join is its kernels plus one spin on a host word.
  useControl = N == 1 && ctx->control() != nullptr;
  BitmapCounters *cnt;
  if (useControl) {
    ctx->beginControl();
    cnt = &ctx->control()->counters;
  } else {
    cnt = ws.getArray<BitmapCounters>(1);
    ctx->zero(cnt, sizeof(BitmapCounters));
  }
  Outcome o;
  // One cursor width for both sides (the fused N = 1 kernel reads both with
  // one slice type; e.g. 1B inner x 4B outer needs 8-byte cursors on both).
  const bool narrowOk = sideNarrow(inner, exact) && sideNarrow(outer, exact);
  // Time points (one event each, shared by the spans that meet there):
  // ev[0] join start, ev[1] inner side partitioned, ev[2] outer side
  // partitioned, ev[3] probe start (N > 1: after the all-reduce), ev[4] end.
  performance::Timeline &tl = ctx->timeline();
  Side both[2] = {Side{inner, {}, nullptr, {}}, Side{outer, {}, nullptr, {}}};
  {
    performance::TraceRange tr("bitmap_network_inner");
    utils::faultPoint("network");
    // Both sides' histograms and layouts first (one launch each), charged to
    // HILOCAL / HOLOCAL by tuples; then the scatters.
    tl.beginSplitAt("HLOCAL", "HILOCAL", (double)inner->getLocalSize(), "HOLOCAL", (double)outer->getLocalSize(),
                    ev[0]);
    layoutSides(both, 2, exact, narrowOk);
    hipEvent_t mid = tl.mark(st);
    tl.endAt("HLOCAL", mid);
    tl.beginAt("MIMAINPART", mid);
    scatterSide(both[0]);
    HIP_CHECK(hipEventRecord(ev[1], st));
    tl.endAt("MIMAINPART", ev[1]);
  }
  Side &ri = both[0], &ro = both[1];
  hipEvent_t joinStart = ev[2];
  if (N == 1) {
    tl.beginAt("MOMAINPART", ev[1]);
    scatterSide(ro);
    HIP_CHECK(hipEventRecord(ev[2], st));
    tl.endAt("MOMAINPART", ev[2]);
    utils::faultPoint("local");
    utils::faultPoint("build_probe");
    // One kernel builds and probes: charged to BPBUILD / BPPROBE by tuples read.
    tl.beginAt("BPTASKTIME", ev[2]);
    tl.beginSplitAt("BPKERNEL", "BPBUILD", (double)inner->getLocalSize(), "BPPROBE", (double)outer->getLocalSize(),
                    ev[2]);
    kernels::MailboxArgs mb;
    mb.box = ctx->mailboxDevice();
    mb.arrivals = &ctx->control()->arrivals;
    mb.seq = ctx->nextMailboxSeq();
    mailboxSeq = mb.seq;
    kernels::bitmapJoin(4, ri.frags, ro.frags, ri.slices, ro.slices, F, 0, bits, cnt, st, mb);
    HIP_CHECK(hipEventRecord(ev[4], st));
    tl.endAt("BPKERNEL", ev[4]);
    tl.endAt("BPTASKTIME", ev[4]);
  } else {
    const uint32_t words = kernels::bitmapWords(bits);
    uint32_t *bm = ws.getArray<uint32_t>((size_t)F * words);
    utils::faultPoint("local");
    tl.beginAt("BPTASKTIME", ev[1]);
    tl.beginAt("BPBUILD", ev[1]);
    // A time point the streams also synchronise on (a timing event when the
    // timeline is on, a pooled sync-only event otherwise).
    auto point = [&](hipStream_t s) {
      hipEvent_t e = tl.mark(s);
      if (!e) {
        e = ctx->acquireEvent();
        HIP_CHECK(hipEventRecord(e, s));
      }
      return e;
    };
    // The all-reduce (exchange stream) overlaps the outer side's network pass:
    // the plan's one link transfer (the reference's puts, MWINPUT).  Build and
    // all-reduce run in K partition ranges: range c's all-reduce starts when
    // its bitmaps are built (while range c + 1 builds), and the probe of a
    // range starts as soon as it is reduced, so after the last range lands
    // only its probe is left.
    const uint32_t K = std::min<uint32_t>(reduceChunks((uint64_t)F * words * 4, plan.variants.reduceChunks), F);
    std::vector<hipEvent_t> built(K), reduced(K);
    for (uint32_t c = 0; c < K; ++c) {
      const uint32_t p0 = (uint32_t)((uint64_t)F * c / K), p1 = (uint32_t)((uint64_t)F * (c + 1) / K);
      kernels::bitmapBuild(4, ri.frags, ri.slices, F, 0, bits, bm, cnt, st, p0, p1 - p0);
      built[c] = point(st);
      if (c == 0) tl.beginAt("MWINPUT", built[0]);
      HIP_CHECK(hipStreamWaitEvent(ctx->commStream(), built[c], 0));
      performance::Measurements::add("MWINPUTCNT", 1, "calls");
      ctx->comm()->allReduceSumDevice(reinterpret_cast<uint64_t *>(bm + (size_t)p0 * words),
                                      (size_t)(p1 - p0) * words / 2, ctx->commStream());
      reduced[c] = point(ctx->commStream());
    }
    tl.endAt("BPBUILD", built[K - 1]);
    tl.endAt("MWINPUT", reduced[K - 1]);
    o.linkBytes = (uint64_t)(2.0 * (N - 1) / N * (double)F * words * 4);
    tl.beginAt("MOMAINPART", built[K - 1]);
    scatterSide(ro);
    HIP_CHECK(hipEventRecord(ev[2], st));
    tl.endAt("MOMAINPART", ev[2]);
    HIP_CHECK(hipStreamWaitEvent(st, reduced[0], 0));
    HIP_CHECK(hipEventRecord(ev[3], st));
    joinStart = ev[3];
    utils::faultPoint("build_probe");
    tl.beginAt("BPPROBE", ev[3]);
    for (uint32_t c = 0; c < K; ++c) {
      const uint32_t p0 = (uint32_t)((uint64_t)F * c / K), p1 = (uint32_t)((uint64_t)F * (c + 1) / K);
      if (c) HIP_CHECK(hipStreamWaitEvent(st, reduced[c], 0));
      kernels::bitmapProbe(4, ro.frags, ro.slices, F, 0, bits, bm, cnt, st, p0, p1 - p0);
    }
    HIP_CHECK(hipEventRecord(ev[4], st));
    tl.endAt("BPPROBE", ev[4]);
    tl.endAt("BPTASKTIME", ev[4]);
  }
  performance::Measurements::add("BPBUILDELEM", (double)inner->getLocalSize(), "tuples");
  performance::Measurements::add("BPPROBEELEM", (double)outer->getLocalSize(), "tuples");
  performance::Measurements::add("BPMEMSIZE", (double)(N > 1 ? (uint64_t)F * kernels::bitmapWords(bits) * 4 : 0),
                                 "bytes");
  // back[0]: this rank's counters; back[1] (N > 1): all ranks' sums, combined
  // on the device behind the probe (one synchronisation per join).
  BitmapCounters *back = ctx->staging().getArray<BitmapCounters>(2);
  const uint64_t tEnqueued = performance::nowUs();
  if (useControl) {
    // The kernel's last wave published the counters: spin on the mailbox,
    // then the streams (their last kernel ends microseconds later).
    const bool arrived = ctx->waitMailbox(mailboxSeq);
    // Polls the end event's signal (no blocking wait on an interrupt).
    if (arrived) utils::waitEvent(ev[4], nullptr, "bitmap join");
    o.hostWaitMs = (performance::nowUs() - tEnqueued) / 1000.0;
    ctx->synchronize();
    JOIN_ASSERT(arrived || ctx->mailbox().seq >= mailboxSeq, "BitmapJoin",
                "the join's final kernel completed without publishing its result (mailbox seq %llu < %llu)",
                (unsigned long long)ctx->mailbox().seq, (unsigned long long)mailboxSeq);
    const kernels::ResultMailbox &m = ctx->mailbox();
    back[0] = BitmapCounters{m.matches, m.popcount, m.dup, m.overflow};
    ctx->endControl();
  } else {
    ctx->readBack(back, cnt, sizeof(BitmapCounters));
    if (N > 1) {
      static_assert(sizeof(BitmapCounters) == 4 * sizeof(uint64_t), "BitmapCounters: four u64 sums");
      ctx->comm()->allReduceSumDevice(reinterpret_cast<uint64_t *>(cnt), 4, st);
      ctx->readBack(back + 1, cnt, sizeof(BitmapCounters));
    }
    ctx->synchronize();
    o.hostWaitMs = (performance::nowUs() - tEnqueued) / 1000.0;
  }
  o.enqueueUs = tEnqueued;
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
  o.devSampleMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[1], ev[2]));
  o.devScatterMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, joinStart, ev[4]));
  o.devJoinMs = ms;
  o.localMatches = back[0].matches;
  o.popcount = back[0].popcount;
  if (N > 1) {
    o.globalMatches = back[1].matches;
    o.dup = back[1].dup > 0;
    o.overflow = back[1].overflow > 0;
    if (!o.overflow && o.popcount != inner->getGlobalSize()) o.dup = true;
  } else {
    agree(o, (back[0].dup ? kernels::BM_FLAG_DUP : 0u) | (back[0].overflow ? kernels::BM_FLAG_OVERFLOW : 0u));
  }
  return o;
}

// Host reference of the same plan (CPU tests of the N-rank logic): exact
// partitioning into u32 fragments, bitmaps as u64 words so the all-reduce
// runs on the host communicator.
BitmapJoin::Outcome BitmapJoin::runHost() {
  const uint32_t nb = plan.networkBits, F = 1u << nb, N = ctx->numberOfNodes();
  const uint32_t words = kernels::bitmapWords(plan.bitmapBits);
  const uint64_t limit = (uint64_t)words * 32;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  auto partition = [&](data::Relation *r, std::vector<uint32_t> &frags, std::vector<uint64_t> &begin) {
    const data::Tuple *t = r->getData();
    const uint64_t n = r->getLocalSize();
    begin.assign(F + 1, 0);
    for (uint64_t i = 0; i < n; ++i) ++begin[(mix.apply(t[i].key) & (F - 1)) + 1];
    for (uint32_t p = 0; p < F; ++p) begin[p + 1] += begin[p];
    std::vector<uint64_t> cur(begin.begin(), begin.end() - 1);
    frags.resize(n);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t k = mix.apply(t[i].key);
      frags[cur[k & (F - 1)]++] = (uint32_t)(k >> nb);
    }
  };
  std::vector<uint32_t> rf, sf;
  std::vector<uint64_t> rb, sb;
  performance::Timeline &tl = ctx->timeline();
  utils::faultPoint("network");
  tl.begin("MIMAINPART");
  partition(inner, rf, rb);
  tl.end("MIMAINPART");
  tl.begin("MOMAINPART");
  partition(outer, sf, sb);
  tl.end("MOMAINPART");
  utils::faultPoint("local");
  tl.begin("BPTASKTIME");
  tl.begin("BPBUILD");
  std::vector<uint64_t> bm64((size_t)F * words / 2, 0);
  uint32_t *bm = reinterpret_cast<uint32_t *>(bm64.data());
  uint32_t flags = 0;
  for (uint32_t p = 0; p < F; ++p)
    for (uint64_t i = rb[p]; i < rb[p + 1]; ++i) {
      const uint64_t f = rf[i];
      if (f >= limit) {
        flags |= kernels::BM_FLAG_DUP;
        continue;
      }
      uint32_t &w = bm[(size_t)p * words + (f >> 5)];
      const uint32_t bit = 1u << (f & 31);
      if (w & bit) flags |= kernels::BM_FLAG_DUP;
      w |= bit;
    }
  tl.end("BPBUILD");
  Outcome o;
  if (N > 1) {
    performance::Measurements::add("MWINPUTCNT", 1, "calls");
    tl.begin("MWINPUT");
    ctx->comm()->allReduceSumHost(bm64.data(), bm64.size());
    tl.end("MWINPUT");
    o.linkBytes = (uint64_t)(2.0 * (N - 1) / N * (double)bm64.size() * 8);
    for (uint64_t w : bm64) o.popcount += (uint64_t)__builtin_popcountll(w);
  }
  utils::faultPoint("build_probe");
  tl.begin("BPPROBE");
  for (uint32_t p = 0; p < F; ++p)
    for (uint64_t i = sb[p]; i < sb[p + 1]; ++i) {
      const uint64_t f = sf[i];
      if (f < limit) o.localMatches += (bm[(size_t)p * words + (f >> 5)] >> (f & 31)) & 1u;
    }
  tl.end("BPPROBE");
  tl.end("BPTASKTIME");
  performance::Measurements::add("BPMEMSIZE", (double)(bm64.size() * 8), "bytes");
  agree(o, flags);
  return o;
}

// One all-reduce decides for every rank: matches, and whether any rank saw a
// duplicate or an overflowed slice.  Replicated plans also compare the set
// bits of the combined bitmaps (identical on every rank) with |R|.
void BitmapJoin::agree(Outcome &o, uint64_t localFlags) {
  uint64_t v[3] = {o.localMatches, (localFlags & kernels::BM_FLAG_DUP) ? 1ull : 0ull,
                   (localFlags & kernels::BM_FLAG_OVERFLOW) ? 1ull : 0ull};
  ctx->comm()->allReduceSumHost(v, 3);
  o.globalMatches = v[0];
  o.dup = v[1] > 0;
  o.overflow = v[2] > 0;
  if (ctx->numberOfNodes() > 1 && !o.overflow && o.popcount != inner->getGlobalSize()) o.dup = true;
}

}  // namespace tasks
}  // namespace hpcjoin
