#include "HashJoin.h"

#include <algorithm>
#include <unordered_set>
#include <cmath>
#include <vector>

#include "../comm/Communicator.h"
#include "../comm/World.h"
#include "../host/HostOps.h"
#include "../data/Window.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../performance/Trace.h"
#include "../tasks/BitmapJoin.h"
#include "ExchangeVerify.h"
#include "JoinStrategies.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace operators {

thread_local uint64_t HashJoin::RESULT_COUNTER = 0;
thread_local std::queue<tasks::Task *> HashJoin::TASK_QUEUE;

using performance::Measurements;
using performance::nowUs;

HashJoin::HashJoin(uint32_t numberOfNodes, uint32_t nodeId, data::Relation *innerRelation,
                   data::Relation *outerRelation)
    : numberOfNodes(numberOfNodes), nodeId(nodeId), innerRelation(innerRelation), outerRelation(outerRelation) {
  comm::Communicator *c = comm::world();
  JOIN_ASSERT(c->size() == numberOfNodes && c->rank() == nodeId, "HashJoin",
              "world communicator is rank %u of %u, caller says %u of %u", c->rank(), c->size(), nodeId,
              numberOfNodes);
  ownedCtx.reset(new core::ExecContext(innerRelation->location(), innerRelation->device(), c));
  ctx = ownedCtx.get();
  makeJoinPlan();
}

HashJoin::HashJoin(data::Relation *innerRelation, data::Relation *outerRelation, core::ExecContext *ctx,
                   const core::JoinConfig &config)
    : numberOfNodes(ctx->numberOfNodes()), nodeId(ctx->nodeId()), innerRelation(innerRelation),
      outerRelation(outerRelation), ctx(ctx), config(config) {
  makeJoinPlan();
}

HashJoin::~HashJoin() {
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
  for (data::Tuple *&b : passBuf) {
    memory::Arena::rawFree(ctx->location(), b);
    b = nullptr;
  }
}

// Per-pass bytes outside the estimate's scaling (plans, histograms, cursors):
// 256 MB, or a quarter of small budgets.
static double spillFixedBytes(uint64_t avail) { return std::min<double>(256.0 * (1 << 20), avail / 4.0); }

// Capacity spill.  A join whose workspace estimate exceeds what HBM has free
// (or config.workspaceBudget) runs in K passes over the key-hash classes
// kernels::passOf: pass k holds ~1/K of both relations (compacted into pass
// buffers) and needs ~1/K of the workspace.  K is the smallest count for
// which one pass's buffers and workspace fit, agreed by all ranks (max).
// The pass sizes are counted once here (one read of each relation), the
// pass buffers allocated once for the largest pass.
void HashJoin::planPasses() {
  uint32_t K = config.passes;
  const uint64_t n[2] = {innerRelation->getLocalSize(), outerRelation->getLocalSize()};
  if (K == 0) {
    K = 1;
    // Materializing joins spill only into a host output buffer (the pairs of
    // all passes together may exceed HBM).
    if (ctx->onDevice() && config.reserveWorkspace && (!plan.materialize || config.outputHost)) {
      // One pass holds its pass buffers (~1/K of both relations) and its
      // join's workspace (~1/K of the estimate, with a margin: a pass join's
      // sampled local pass that overflows re-runs exactly beside its sampled
      // buffers -- 6B x 6B in 6 passes peaked at 1.55x its estimate and ran
      // out of HBM).  workspaceBudget caps both together.
      size_t freeB = 0, totalB = 0;
      HIP_CHECK(hipMemGetInfo(&freeB, &totalB));
      uint64_t avail = (uint64_t)(freeB * 0.85);
      if (config.workspaceBudget) avail = std::min<uint64_t>(avail, config.workspaceBudget);
      const uint64_t est = workspaceEstimate(), tuplesB = (n[0] + n[1]) * sizeof(data::Tuple);
      spill.estimate = est;
      spill.available = avail;
      if (est > avail && plan.bitmapJoin && numberOfNodes == 1) {
        // The bitmap plan spills by partition groups instead (tasks/BitmapJoin):
        // each group pass reads both relations once and writes only the
        // fragments of its network partitions -- no pass buffers, no
        // compaction, and the group count follows from the sampled totals.
        const uint64_t fixed = 96ull << 20;  // plans, cursors, counters (the estimate's first part)
        plan.groupBudget = avail > 2 * fixed ? avail - fixed : avail / 2;
        spill.groupBudget = plan.groupBudget;
      } else if (est > avail) {
        K = 2;
        while (K < kernels::MAX_SPILL_PASSES &&
               (double)est / K * 1.6 + (double)tuplesB / K * 1.05 + spillFixedBytes(avail) > (double)avail)
          ++K;
      }
    }
  }
  K = std::max<uint32_t>(1, std::min<uint32_t>(K, kernels::MAX_SPILL_PASSES));
  auto agreeMax = [&](uint32_t mine) {  // every rank runs the same number of passes
    std::vector<uint64_t> all(numberOfNodes);
    const uint64_t m = mine;
    ctx->comm()->allGatherHost(&m, all.data(), 1);
    for (uint64_t k : all) mine = std::max<uint32_t>(mine, (uint32_t)k);
    return mine;
  };
  K = agreeMax(K);
  passes = K;
  if (K == 1) return;
  JOIN_ASSERT(!plan.materialize || config.outputHost, "HashJoin",
              "capacity spill (%u passes) of a materializing join needs JoinConfig.outputHost: the pairs of every "
              "pass go to one pinned host buffer",
              K);
  data::Relation *rel[2] = {innerRelation, outerRelation};
  std::vector<uint64_t> counts, global;
  auto countPasses = [&](uint32_t k) {
    counts.assign(2 * (size_t)k, 0);
    if (ctx->onDevice()) {
      auto *d = ctx->workspace().getArray<unsigned long long>(2 * (size_t)k);
      ctx->zero(d, 2 * (size_t)k * 8);
      for (int r = 0; r < 2; ++r) kernels::passCounts(rel[r]->getData(), n[r], k, d + (size_t)r * k, ctx->stream());
      HIP_CHECK(hipMemcpyAsync(counts.data(), d, 2 * (size_t)k * 8, hipMemcpyDeviceToHost, ctx->stream()));
      utils::waitStream(ctx->stream(), ctx->comm(), "pass counts");
      ctx->workspace().reset();
    } else {
      for (int r = 0; r < 2; ++r) {
        const data::Tuple *t = rel[r]->getData();
        for (uint64_t i = 0; i < n[r]; ++i) ++counts[(size_t)r * k + kernels::passOf(t[i].key, k)];
      }
    }
    global = counts;
    ctx->comm()->allReduceSumHost(global.data(), global.size());
  };
  countPasses(K);
  // Key-hash classes are balanced only for spread keys: every copy of a hot
  // key lands in one pass (Zipf, repeated inner keys).  The largest pass's
  // buffers and its share of the workspace must fit what the planner assumed
  // for 1/K of the data; otherwise K grows (recount) until it does.  A single
  // key class too big for memory on its own is refused here, not by a failed
  // allocation inside the join.
  if (config.passes == 0 && spill.available) {
    const double total = (double)(n[0] + n[1]) + 1.0;
    for (;;) {
      uint64_t worst = 0;
      for (uint32_t k = 0; k < K; ++k) worst = std::max<uint64_t>(worst, counts[k] + counts[K + k]);
      const double share = (double)worst / total;  // of this rank's tuples
      const double need = (double)spill.estimate * share * 1.6 + (double)worst * sizeof(data::Tuple) * 1.05 +
                          spillFixedBytes(spill.available);
      const bool fits = need <= (double)spill.available;
      // Every rank decides the same next K (the max over ranks).
      uint32_t next = fits ? K : std::min<uint32_t>(kernels::MAX_SPILL_PASSES, K + std::max<uint32_t>(1, K / 2));
      next = agreeMax(next);
      if (next == K) {
        // At the pass limit a balanced class is run anyway (best effort, the
        // estimate's margins); a class far above 1/K is one hot key: refused.
        HJ_CHECK(fits || share < 4.0 / kernels::MAX_SPILL_PASSES,
                 "capacity spill: the largest key-hash class holds %lu of %lu tuples and needs %.1f GB, more than "
                 "the %.1f GB available to one pass even at %u passes (one key too frequent to spill)",
                 (unsigned long)worst, (unsigned long)(n[0] + n[1]), need / 1e9, spill.available / 1e9, K);
        break;
      }
      K = next;
      countPasses(K);
    }
    passes = K;
  }
  for (int r = 0; r < 2; ++r) {
    passCount[r].assign(counts.begin() + (size_t)r * K, counts.begin() + (size_t)(r + 1) * K);
    passGlobal[r].assign(global.begin() + (size_t)r * K, global.begin() + (size_t)(r + 1) * K);
    const uint64_t cap = *std::max_element(passCount[r].begin(), passCount[r].end());
    if (passBuf[r]) memory::Arena::rawFree(ctx->location(), passBuf[r]);
    passBuf[r] = static_cast<data::Tuple *>(
        memory::Arena::rawAlloc(ctx->location(), std::max<uint64_t>(cap, 1) * sizeof(data::Tuple), ctx->device()));
    passCap[r] = std::max<uint64_t>(cap, 1);
    spill.passBuffers += passCap[r] * sizeof(data::Tuple);
  }
  JOIN_DEBUG("HashJoin", "capacity spill: %u passes", K);
}

// One pass per key-hash class: compact both relations' tuples of the class
// into the pass buffers, join them with a plan of their own (bounds
// inherited, no re-scan), add the counts.
JoinResult HashJoin::runPasses() {
  performance::TraceRange traceJoin("hpcjoin::join_passes");
  const uint64_t t0 = nowUs();
  JoinResult total;
  total.innerLocal = innerRelation->getLocalSize();
  total.outerLocal = outerRelation->getLocalSize();
  total.passes = passes;
  data::Relation *rel[2] = {innerRelation, outerRelation};
  core::JoinConfig sub = config;
  sub.passes = 1;
  sub.keyHashing = plan.keyMix ? core::KeyHashing::On : core::KeyHashing::Off;
  uint64_t written = 0;  // pairs appended to config.outputHost so far (materializing spill)
  for (uint32_t k = 0; k < passes; ++k) {
    if (plan.materialize) {
      sub.outputHost = static_cast<ulonglong2 *>(config.outputHost) + written;
      sub.outputCapacity = config.outputCapacity > written ? config.outputCapacity - written : 0;
      JOIN_ASSERT(sub.outputCapacity > 0, "HashJoin", "capacity spill: the host output buffer (%lu pairs) is full "
                  "after pass %u of %u", (unsigned long)config.outputCapacity, k, passes);
    }
    const uint64_t tc = nowUs();
    if (ctx->onDevice()) {
      ctx->resetScratch();
      auto *cur = ctx->workspace().getArray<unsigned long long>(2);
      ctx->zero(cur, 16);
      for (int r = 0; r < 2; ++r)
        kernels::passCompact(rel[r]->getData(), rel[r]->getLocalSize(), passes, k, passBuf[r], cur + r, ctx->stream(),
                             passCap[r]);
      auto *curBack = ctx->staging().getArray<unsigned long long>(2);
      ctx->readBack(curBack, cur, 16);
      utils::waitStream(ctx->stream(), ctx->comm(), "pass compaction");
      for (int r = 0; r < 2; ++r)
        JOIN_ASSERT(curBack[r] == passCount[r][k], "HashJoin",
                    "capacity spill: pass %u compacted %lu %s tuples, the plan counted %lu (relation changed since "
                    "planning?)",
                    k, (unsigned long)curBack[r], r ? "outer" : "inner", (unsigned long)passCount[r][k]);
    } else {
      for (int r = 0; r < 2; ++r) {
        const data::Tuple *t = rel[r]->getData();
        uint64_t at = 0;
        for (uint64_t i = 0; i < rel[r]->getLocalSize(); ++i)
          if (kernels::passOf(t[i].key, passes) == k) passBuf[r][at++] = t[i];
      }
    }
    total.compactMs += (nowUs() - tc) / 1000.0;
    data::Relation Rk(passBuf[0], passCount[0][k], passGlobal[0][k], ctx->location(), ctx->device());
    data::Relation Sk(passBuf[1], passCount[1][k], passGlobal[1][k], ctx->location(), ctx->device());
    Rk.inheritBounds(*innerRelation, planMaxKey, planMaxRid);
    Sk.inheritBounds(*outerRelation, planMaxKey, planMaxRid);
    HashJoin pass(&Rk, &Sk, ctx, sub);
    spill.passEstimate = std::max<uint64_t>(spill.passEstimate, pass.workspaceEstimate());
    spill.passReserved = std::max<uint64_t>(spill.passReserved, ctx->workspace().capacity());
    const JoinResult r = pass.run();
    spill.passPeak = std::max<uint64_t>(spill.passPeak, ctx->workspace().peak());
    if (plan.materialize) {
      JOIN_ASSERT(!r.outputOverflow, "HashJoin",
                  "capacity spill: pass %u of %u produced %lu pairs, the host output buffer has room for %lu", k,
                  passes, (unsigned long)r.outputPairs, (unsigned long)sub.outputCapacity);
      written += r.outputPairs;
      total.outputPairs += r.outputPairs;
    }
    total.localMatches += r.localMatches;
    total.globalMatches += r.globalMatches;
    total.innerReceived += r.innerReceived;
    total.outerReceived += r.outerReceived;
    total.wireBytes += r.wireBytes;
    total.localItems += r.localItems;
    total.buildProbeItems += r.buildProbeItems;
    total.networkFallbacks += r.networkFallbacks;
    total.roundWindows += r.roundWindows;
    total.localFallbacks += r.localFallbacks;
    total.reruns += r.reruns;
    total.devNetworkMs += r.devNetworkMs;
    total.devLocalPartitionMs += r.devLocalPartitionMs;
    total.devBuildProbeMs += r.devBuildProbeMs;
    total.devSpanMs += r.devSpanMs;
    total.bitmapJoin = r.bitmapJoin;
    total.sampledNetwork = r.sampledNetwork;
  }
  total.joinMs = (nowUs() - t0) / 1000.0;
  total.networkMs = total.joinMs;
  result = total;
  if (plan.materialize) {  // every pass appended to the caller's host buffer
    output = static_cast<const ulonglong2 *>(config.outputHost);
    outputEpoch = ctx->workspace().epoch();
  }
  RESULT_COUNTER = result.localMatches;
  return result;
}

void HashJoin::makeJoinPlan() {
  // A device engine also reads pinned host relations in place (zero-copy over
  // the host link: joins whose inputs exceed HBM).
  auto usable = [&](data::Relation *r) {
    return r->location() == ctx->location() || (ctx->onDevice() && r->location() == Location::Pinned);
  };
  JOIN_ASSERT(usable(innerRelation) && usable(outerRelation), "HashJoin",
              "relations must live where the engine runs (%s) or in pinned host memory", locationName(ctx->location()));
  // Max key / rid over both relations and all ranks (the plan must be identical
  // everywhere), plus each rank's rid range per relation and exchange chunk
  // (wire codec bases).  Per rank: {max key, max rid, then for inner and outer
  // and every chunk c: min rid, max rid, and last whether the inner keys' low
  // bits are known to be uniform}.  Generated relations know these bounds
  // (Relation::keyBoundKnown / ridsPositional): no pass over the data; others
  // are scanned once here (kernels::keyRidMax).
  const uint64_t tPlan = nowUs();
  const uint32_t C = std::max<uint32_t>(1, config.chunks);
  ridLo[0] = ridLo[1] = ~0ull;
  ridHi[0] = ridHi[1] = 0;
  const size_t STATS = 4 + 4 * (size_t)C;
  std::vector<uint64_t> st(STATS, 0);
  int which = 0;
  for (data::Relation *r : {innerRelation, outerRelation}) {
    const bool known = r->keyBoundKnown() && r->ridsPositional();
    for (uint32_t c = 0; c < C; ++c) {
      uint64_t b, e;
      histograms::LocalHistogram::chunkRange(r->getLocalSize(), C, config.maxPartitionBlocks, c, &b, &e);
      uint64_t h[3] = {0, 0, ~0ull};
      if (known) {
        h[0] = r->maxKey();
        if (e > b) {
          h[1] = r->ridBase() + e - 1;
          h[2] = r->ridBase() + b;
        }
      } else if (r->keyBoundKnown() && r->ridBoundKnown()) {  // a pass view: the parent join's bounds
        h[0] = r->maxKey();
        if (e > b) {
          h[1] = r->ridMax();
          h[2] = 0;
        }
      } else if (ctx->onDevice() && e > b) {
        unsigned long long *d = ctx->workspace().getArray<unsigned long long>(3);
        HIP_CHECK(hipMemcpyAsync(d, h, 24, hipMemcpyHostToDevice, ctx->stream()));
        kernels::keyRidMax(r->getData() + b, e - b, d, ctx->stream());
        HIP_CHECK(hipMemcpyAsync(h, d, 24, hipMemcpyDeviceToHost, ctx->stream()));
        HIP_CHECK(hipStreamSynchronize(ctx->stream()));
      } else if (!ctx->onDevice()) {
        const data::Tuple *t = r->getData();
        for (uint64_t i = b; i < e; ++i) {
          h[0] = std::max<uint64_t>(h[0], t[i].key);
          h[1] = std::max<uint64_t>(h[1], t[i].rid);
          h[2] = std::min<uint64_t>(h[2], t[i].rid);
        }
      }
      st[0] = std::max(st[0], h[0]);
      st[1] = std::max(st[1], h[1]);
      if (h[2] <= h[1]) {
        ridLo[which] = std::min(ridLo[which], h[2]);
        ridHi[which] = std::max(ridHi[which], h[1]);
      }
      st[2 + ((size_t)which * C + c) * 2] = h[2];
      st[3 + ((size_t)which * C + c) * 2] = h[1];
    }
    ++which;
  }
  st[STATS - 1] = innerRelation->lowBitsUniform() ? 1 : 0;
  st[STATS - 2] = (uint64_t)innerKeyRepeats();
  ctx->workspace().reset();
  std::vector<uint64_t> all(STATS * numberOfNodes);
  ctx->comm()->allGatherHost(st.data(), all.data(), STATS);
  uint64_t mx[2] = {0, 0};
  bool lowBitsUniform = true, repeats = false;
  for (uint32_t r = 0; r < numberOfNodes; ++r) {
    mx[0] = std::max(mx[0], all[STATS * r]);
    mx[1] = std::max(mx[1], all[STATS * r + 1]);
    lowBitsUniform = lowBitsUniform && all[STATS * r + STATS - 1] == 1;
    repeats = repeats || all[STATS * r + STATS - 2] == 2;
  }
  plan = core::makePlan(config, numberOfNodes, innerRelation->getGlobalSize(), outerRelation->getGlobalSize(), mx[0],
                        mx[1]);
  planMaxKey = mx[0];
  planMaxRid = mx[1];
  // Repeated inner keys are known before the first join (generator metadata
  // or the sample above): no bitmap plan to attempt and throw away, and
  // key-only words go on counted tables from the first join instead of
  // switching after a quotient table chained the copies.
  plan.innerRepeats = repeats;
  if (repeats && plan.keyOnly && plan.variants.keyCount == 8) plan.variants.keyCount = 9;
  planWireCodec(all, STATS, C);
  // Key mixing only when the inner keys' low bits are not known to be uniform
  // and a histogram of them says they are skewed (a collective: every rank
  // takes the same branch, lowBitsUniform is all-gathered).
  if (config.keyHashing == core::KeyHashing::Auto && plan.keyBits < 64)
    plan.keyMix = lowBitsUniform ? false : lowKeyBitsSkewed();
  if (!ctx->onDevice()) {
    plan.localHistogram = core::HistogramMode::Exact;  // sampling pays on HBM only
    plan.splitLocal = false;                           // split columns are a device layout
  }
  const uint64_t small = std::min(innerRelation->getGlobalSize(), outerRelation->getGlobalSize());
  const bool sampleable =
      config.networkHistogram == core::HistogramMode::Sampled ||
      (config.networkHistogram == core::HistogramMode::Auto && small >= (16ull << 20));
  plan.sampledNetwork = numberOfNodes == 1 && ctx->onDevice() && plan.chunks == 1 && sampleable;
  // Counting on the split layout reads only the u16 fragment column: the
  // sampled network pass can then write u32 fragments and the local pass the
  // fragment column alone (4 + 2 bytes per tuple instead of 8 + 6).
  // No rid travels, so the rid width (which decides splitLocal) does not
  // matter: only that the u16 column holds the fragment above both digits.
  plan.fragments = plan.sampledNetwork && !plan.materialize && !plan.wide && !plan.keyOnly && plan.twoLevel &&
                   plan.keyBits <= plan.networkBits + plan.localBits + 16 &&
                   kernels::fragWordFits(plan.keyBits, plan.networkBits);
  // N > 1 pipelines (also on the host path, where they run in place: same
  // logic, covered by the CPU tests).
  plan.splitHistogram = config.splitHistogram && numberOfNodes > 1;
  plan.pipelineOuter = config.pipelineOuter && numberOfNodes > 1 && !plan.materialize && plan.twoLevel;
  // One-sided windows: device engines (IPC-mapped peers) or in-process ranks.
  // Puts move raw tuples and complete at a barrier, so neither the wire codec
  // nor per-chunk pipelining of the outer relation applies.
  plan.oneSided = config.exchange == core::ExchangeMode::OneSided && numberOfNodes > 1 &&
                  (ctx->onDevice() || ctx->comm()->sharesAddressSpace());
  if (plan.oneSided) {
    plan.wireBits[0] = plan.wireBits[1] = 0;
    plan.wireRidBits[0] = plan.wireRidBits[1] = 0;
    plan.pipelineOuter = false;
  }
  // N > 1 (tasks/SampledShuffle): two-sided windows; the claim slices' gaps
  // stay off the links either through the codec's pack or, with raw words,
  // through a gather of the filled runs (received straight into the window).
  if (numberOfNodes > 1)
    plan.sampledNetwork = ctx->onDevice() && sampleable && !plan.wide && !plan.oneSided;
  basePlan = plan;  // the two-level plan: what a bitmap plan falls back to
  bitmapExact = !(ctx->onDevice() && sampleable);
  planBitmap();
  JOIN_DEBUG("HashJoin", "%s", plan.describe().c_str());
  planMs = (nowUs() - tPlan) / 1000.0;
  const uint64_t tReserve = nowUs();
  if (ctx->onDevice())
    for (auto &e : ev)
      if (!e) HIP_CHECK(hipEventCreate(&e));
  planPasses();
  if (ctx->onDevice() && config.reserveWorkspace && passes == 1) {
    // Capped by what HBM has free (the estimate is generous for N > 1, where
    // received sizes are only known after the histogram): a short estimate
    // only means the first join falls back to hipMalloc, as without it.
    size_t freeB = 0, totalB = 0;
    HIP_CHECK(hipMemGetInfo(&freeB, &totalB));
    const std::vector<uint64_t> parts = workspaceParts();
    const uint64_t est = workspaceEstimate();
    uint64_t want = std::min<uint64_t>(est, (uint64_t)(freeB * 0.85));
    if (config.workspaceBudget) want = std::min<uint64_t>(want, config.workspaceBudget);
    // Rewound first: a previous join's buffers are dead once a new join is
    // planned on this context, so the chunks are re-laid out instead of
    // growing on top of them.  With the whole estimate: one chunk per part;
    // otherwise one chunk (capped: of what the cap allows).
    // N > 1: re-laying out frees chunks that peers may still have IPC-mapped
    // (one-sided windows of an earlier join).  The free is made a collective
    // step: every rank finishes its device work, closes its mappings of peers'
    // memory, and waits until all peers have closed theirs before any rank
    // frees (the uncoordinated free was a suspected cause of the
    // hangs and failed IPC opens of the 4/8-process test).
    if (numberOfNodes > 1) {
      ctx->synchronize();
      ctx->releaseImports();
      ctx->comm()->barrier();
    }
    ctx->workspace().reset();
    reserved = want == est ? ctx->workspace().ensureParts(parts, true, ctx->stream())
                           : ctx->workspace().ensure(want, true, ctx->stream());
    JOIN_DEBUG("HashJoin", "workspace: estimate %.2f GB, added %.2f GB", want / 1e9, reserved / 1e9);
  }
  reserveMs = (nowUs() - tReserve) / 1000.0;
}

// 1 = this rank's inner keys look unique, 2 = they repeat: from the
// generator when it knows (Relation::keyRepeats), else from 64K evenly
// spaced keys (kernels::sampleRepeats; any repeat in the sample decides).
// A sample can miss rare repeats; the plans stay exact either way (the bitmap
// plan's duplicate check and the quotient table's chain flag still fall back).
int HashJoin::innerKeyRepeats() {
  if (innerRelation->keyRepeats()) return innerRelation->keyRepeats();
  const uint64_t n = innerRelation->getLocalSize();
  const uint32_t S = (uint32_t)std::min<uint64_t>(n, 65536);
  if (S < 2) return 1;
  const data::Tuple *t = innerRelation->getData();
  if (ctx->onDevice()) {
    void *ws = ctx->workspace().get(kernels::sampleRepeatsBytes(S));
    auto *cnt = ctx->workspace().getArray<unsigned int>(1);
    kernels::sampleRepeats(t, n, S, ws, cnt, ctx->stream());
    unsigned int h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, ctx->stream()));
    HIP_CHECK(hipStreamSynchronize(ctx->stream()));
    return h ? 2 : 1;
  }
  std::unordered_set<uint64_t> seen;
  seen.reserve(2 * S);
  for (uint32_t i = 0; i < S; ++i)
    if (!seen.insert(t[(uint64_t)((unsigned __int128)i * n / S)].key).second) return 2;
  return 1;
}

uint64_t HashJoin::workspaceEstimate() const {
  uint64_t b = 0;
  for (uint64_t x : workspaceParts()) b += x;
  return b;
}

// The estimate as the join's big buffers in allocation order, after one part
// for everything small (plans, histograms, cursors, counters, scan scratch,
// build/probe work lists).  Reserved as one chunk per part: a buffer then
// starts at an allocation of its own, as a fallback hipMalloc would put it.
// Sub-allocated from one 40 GiB chunk the same scatters ran 0.3-0.4 ms
// slower each (1B x 1B general path 20.59 vs 19.28 ms same box; which
// kernels were slow moved with the buffers' offsets, profiles/r4sk).
std::vector<uint64_t> HashJoin::workspaceParts() const {
  const uint32_t N = numberOfNodes, F = 1u << plan.networkBits;
  const uint64_t n[2] = {innerRelation->getLocalSize(), outerRelation->getLocalSize()};
  const uint64_t g[2] = {innerRelation->getGlobalSize(), outerRelation->getGlobalSize()};
  std::vector<uint64_t> parts(1, 64ull << 20);
  // Round-interleaved network windows (SampledNetworkPartitioning::roundLp) need a little more room.
  const uint32_t roundLp =
      plan.twoLevel && !plan.wide ? kernels::roundLpFor(plan.roundLp, plan.fragments ? 4 : 8) : 0;
  auto sampledCap = [&](uint64_t m, uint32_t lp = 0) {
    const kernels::PartitionGeometry geom = kernels::partitionGeometry(m, config.maxPartitionBlocks);
    const uint32_t stride = kernels::sampleStrideFor(geom, m, F, std::max<uint32_t>(1, config.sampleStride));
    return kernels::sampledWindowCapacity(kernels::sampleScale(geom, m, stride, false), F, lp);
  };
  if (plan.bitmapJoin) {
    // u32 fragments in claim slices (round-interleaved unless a partition-group pass)
    const uint32_t lp = plan.groupBudget ? 0 : kernels::roundLpFor(plan.roundLp, 4);
    for (int r = 0; r < 2; ++r) parts.push_back((sampledCap(n[r], lp) + 64) * 4);
    if (plan.bitmapReplicated) parts.push_back(2ull * F * kernels::bitmapWords(plan.bitmapBits) * 4);
    return parts;
  }
  const uint64_t wordB = plan.fragments ? 4 : plan.wide ? 16 : 8;
  const uint64_t owned = N == 1 ? F : ceilDiv(F, N) + 1;
  const uint64_t P = plan.twoLevel ? owned << plan.localBits : owned;
  uint64_t recvTotal[2], local[2][2] = {{0, 0}, {0, 0}}, dedup = 0;
  for (int r = 0; r < 2; ++r) {
    // N > 1: the fair share plus a quarter (LPT balances partitions; skew
    // beyond that falls back to allocation inside the first join).
    const uint64_t recv =
        N == 1 ? (plan.sampledNetwork ? sampledCap(n[r], roundLp) : n[r]) : g[r] / N + g[r] / (4 * N) + (1 << 20);
    recvTotal[r] = recv;
    // send buffer (sampled: slice margins; round-interleaved slices up to half again, SampledShuffle)
    if (N > 1 && !plan.oneSided)
      parts.push_back((plan.sampledNetwork ? n[r] + (plan.roundLp ? n[r] / 2 : n[r] / 8) : n[r]) * wordB);
    if (plan.wireBits[r]) parts.push_back((n[r] + recv) * ((plan.wireBits[r] + 7) / 8) + (64ull << 10));  // wire buffers
    else if (N > 1 && plan.sampledNetwork && !plan.oneSided) parts.push_back(n[r] * 8 + (64ull << 10));  // gathered runs
    parts.push_back(recv * wordB);  // window
    if (plan.twoLevel) {
      const uint64_t ob = plan.fragments ? 2 : plan.splitLocal ? kernels::SPLIT_BYTES : (plan.wide ? 16 : 8);
      const uint64_t slots = kernels::localSampledCapacityBound(recv, P, std::max<uint32_t>(1, plan.localSampleStride), 64);
      // Split columns are two allocations (u32, then u16): a part each.
      const bool split = plan.splitLocal && !plan.fragments && !plan.wide;
      local[r][0] = slots * (split ? ob - 2 : ob);
      local[r][1] = split ? slots * 2 : 0;
      // Repeated keys on counted tables: the inner side's compaction counts
      // (u32 per slot) and per-segment lengths / lists (BuildProbe, bpKeyDedup).
      if (r == 0 && plan.keyOnly && plan.variants.keyCount == 9) dedup = slots * 4 + P * (8 + 8 * kernels::BP_DEDUP_SEGS);
    }
  }
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 2; ++c)
      if (local[r][c]) parts.push_back(local[r][c]);
  if (dedup) parts.push_back(dedup);
  // Build/probe work lists (items or spans, 32 B) and materialized pairs.
  parts[0] += (2 * P + recvTotal[1] / std::max<uint32_t>(plan.sChunk, 1) +
               recvTotal[0] / std::max<uint32_t>(plan.rChunk, 1) + 2048) * 48;
  if (plan.materialize && !config.outputHost)
    parts.push_back((config.outputCapacity ? config.outputCapacity : recvTotal[1] + 1024) * 16);
  return parts;
}

// Count-only single-level bitmap plans (tasks/BitmapJoin) and the N > 1 cost
// model.  The network pass runs at 10 bits (1024 partitions, 128 KiB bitmaps
// for 1B dense keys: measured 13.5 ms per 1B x 1B join vs 14.1 ms at 11 bits
// with 64 KiB bitmaps -- the 2048-way scatter writes shorter runs), or 11 when
// the key range needs it.
//   N == 1: on a device engine whenever the fragments fit (host path: only
//           when replicateBitmap = On; it is the reference CPU path there).
//   N > 1:  replicated bitmaps (no tuple shuffle) when they put fewer bytes on
//           the links than the shuffle would (Auto, device), or when forced.
// Link bytes per rank and join:
//   replicated  2 (N-1)/N * 2^(networkBits + bitmapBits) / 8   (ring all-reduce)
//   shuffle     (N-1)/N * (|R| w_R + |S| w_S) / 8 / N          (w = wire bits per tuple)
void HashJoin::planBitmap() {
  const uint32_t N = numberOfNodes;
  plan.bitmapJoin = false;
  plan.bitmapReplicated = false;
  const double perPeer = config.linkGBpsPerPeer > 0 ? config.linkGBpsPerPeer : kDefaultLinkGBpsPerPeer;
  plan.linkGBps = N > 1 ? perPeer * (double)std::min<uint32_t>(N - 1, 7) : 0.0;
  {
    const double share = N > 1 ? (double)(N - 1) / N : 0.0;
    const double wR = plan.wide ? 128 : (plan.wireBits[0] ? plan.wireBits[0] : 64);
    const double wS = plan.wide ? 128 : (plan.wireBits[1] ? plan.wireBits[1] : 64);
    plan.shuffleLinkBytes = share *
                            ((double)innerRelation->getGlobalSize() * wR + (double)outerRelation->getGlobalSize() * wS) /
                            8.0 / std::max<uint32_t>(N, 1);
  }
  if (!config.bitmapJoin || plan.materialize || plan.wide || plan.keyOnly || plan.keyBits >= 64) return;
  // Repeated inner keys would only make the bitmap plan fall back after a
  // whole failed join; replicateBitmap = On still forces it (tests of that
  // fallback path).
  if (plan.innerRepeats && config.replicateBitmap != core::PlanChoice::On) return;
  const uint32_t want = plan.keyBits > kernels::BITMAP_MAX_BITS ? plan.keyBits - kernels::BITMAP_MAX_BITS : 0;
  const uint32_t nb =
      config.networkBits ? config.networkBits : std::min<uint32_t>(kernels::MAX_PART_BITS, std::max<uint32_t>(10, want));
  const uint32_t bits = plan.keyBits > nb ? plan.keyBits - nb : 0;
  // A partition's fragment range may be split over two workgroups of the
  // bitmap kernels (21 bits: e.g. 3B dense keys; the replicated bitmaps
  // travel whole, 256 KiB per partition).
  const uint32_t maxBits = kernels::BITMAP_MAX_BITS + kernels::BITMAP_MAX_SPLIT;
  if (bits > maxBits || !kernels::fragWordFits(plan.keyBits, nb)) return;
  const double bitmapBytes = (double)(1ull << nb) * kernels::bitmapWords(bits) * 4;
  plan.replicatedLinkBytes = N > 1 ? 2.0 * (N - 1) / N * bitmapBytes : 0.0;
  bool use;
  if (N == 1)
    use = ctx->onDevice() || config.replicateBitmap == core::PlanChoice::On;
  else if (config.replicateBitmap == core::PlanChoice::On)
    use = true;
  else if (config.replicateBitmap == core::PlanChoice::Off)
    use = false;
  else
    use = ctx->onDevice() && plan.replicatedLinkBytes <= plan.shuffleLinkBytes;
  if (!use) return;
  plan.networkBits = nb;
  plan.bitmapJoin = true;
  plan.bitmapBits = bits;
  plan.bitmapReplicated = N > 1;
  plan.sampledNetwork = !bitmapExact;
}

// Wire codec per relation (kernels.h, WireCodec): frame-of-reference rids
// (base = the smallest rid of the sending rank's exchange chunk: a chunk is a
// contiguous quarter of the rank's input, so positional rids need 2 bits less
// than with one base per rank) plus the key fragment above the network digit.
// Auto decides by cost on a device engine with N > 1 (codecPays): packing
// saves (64 - w) / 8 bytes per tuple that leaves the rank, at the calibrated
// link rate of min(N - 1, 7) peers; it costs a pack and an unpack pass in HBM
// where raw words need only the gather of the filled runs (SampledShuffle:
// received straight into the window).  On forces it (also on the host path).
// The reference compresses inside its scatter at every N
// (tasks/NetworkPartitioning.cpp:128-129); here the choice follows the links.
bool HashJoin::codecPays(uint32_t w, uint32_t nodes, double perPeerGBps, double extraPsPerTuple) {
  if (w == 0 || w >= 64 || nodes < 2) return false;
  const double linkGBps = perPeerGBps * (double)std::min<uint32_t>(nodes - 1, 7);
  const double savedPs = (64.0 - w) / 8.0 / linkGBps * 1000.0;  // bytes / (GB/s) = ns; x 1000 = ps
  return savedPs > extraPsPerTuple;
}

void HashJoin::planWireCodec(const std::vector<uint64_t> &all, size_t stride, uint32_t chunks) {
  for (int r = 0; r < 2; ++r) {
    plan.wireBits[r] = 0;
    plan.wireRidBits[r] = 0;
    plan.ridBase[r].assign((size_t)numberOfNodes * chunks, 0);
  }
  if (plan.wide || numberOfNodes == 1 || config.wireCodec == core::WireCodecMode::Off) return;
  const double perPeer = config.linkGBpsPerPeer > 0 ? config.linkGBpsPerPeer : kDefaultLinkGBpsPerPeer;
  auto wants = [&](uint32_t w) {
    if (config.wireCodec == core::WireCodecMode::On) return w < 64;
    return ctx->onDevice() && codecPays(w, numberOfNodes, perPeer, config.codecExtraPsPerTuple);
  };
  const uint32_t keyW = plan.keyBits > plan.networkBits ? plan.keyBits - plan.networkBits : 0;
  if (plan.keyOnly) {
    // Key-only words (keyShift 0) are the key above the network digit: only
    // those keyBits - networkBits bits travel (53 of 64 for 63-bit keys), no
    // rid and no rid base (decode then returns the word itself).
    if (keyW >= 1 && wants(keyW))
      for (int r = 0; r < 2; ++r) plan.wireBits[r] = keyW;
    return;
  }
  for (int r = 0; r < 2; ++r) {
    uint64_t span = 1;
    for (uint32_t n = 0; n < numberOfNodes; ++n)
      for (uint32_t c = 0; c < chunks; ++c) {
        const size_t at = stride * n + 2 + ((size_t)r * chunks + c) * 2;
        const uint64_t lo = all[at], hi = all[at + 1];
        if (lo > hi) continue;  // empty chunk
        plan.ridBase[r][(size_t)n * chunks + c] = lo;
        span = std::max<uint64_t>(span, hi - lo + 1);
      }
    // Counting joins never read a rid after the network pass (every count
    // kernel compares key fragments only): the wire carries the fragment alone.
    const uint32_t ridBits = plan.materialize ? std::max<uint32_t>(1, ceilLog2(span)) : 0;
    const uint32_t w = ridBits + keyW;
    if (w >= 1 && wants(w) && ridBits <= plan.keyShift) {
      plan.wireBits[r] = w;
      plan.wireRidBits[r] = ridBits;
    }
  }
  JOIN_DEBUG("HashJoin", "wire codec: inner %u bits, outer %u bits per tuple", plan.wireBits[0], plan.wireBits[1]);
}

// KeyHashing::Auto: histogram the inner keys' low networkBits bits (all ranks)
// once at plan time.  Dense keys give a flat histogram; keys with structured
// low bits (sparse TPC-H order keys, strides) leave digits empty and overfill
// others, which radix partitioning would carry into every later pass.
bool HashJoin::lowKeyBitsSkewed() {
  const uint32_t bits = std::min<uint32_t>(plan.networkBits, kernels::MAX_PART_BITS);
  const uint32_t F = 1u << bits;
  const uint64_t G = innerRelation->getGlobalSize();
  if (G < 64ull * F) return false;  // too few keys to judge (and too small to matter)
  const uint64_t n = innerRelation->getLocalSize();
  const kernels::PartitionGeometry g = kernels::partitionGeometry(n);
  std::vector<uint64_t> totals(F, 0);
  uint32_t *blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * g.blocks);
  if (ctx->onDevice()) {
    uint64_t *d = ctx->workspace().getArray<uint64_t>(F);
    kernels::netHistogram(innerRelation->getData(), n, bits, g, blockHist, ctx->stream());
    kernels::digitTotals(blockHist, F, g.blocks, g.blocks, 1, d, ctx->stream());
    HIP_CHECK(hipMemcpyAsync(totals.data(), d, F * 8, hipMemcpyDeviceToHost, ctx->stream()));
    HIP_CHECK(hipStreamSynchronize(ctx->stream()));
  } else {
    host::netHistogram(innerRelation->getData(), n, bits, g, blockHist);
    host::digitTotals(blockHist, F, g.blocks, g.blocks, 1, totals.data());
  }
  ctx->workspace().reset();
  ctx->comm()->allReduceSumHost(totals.data(), F);
  const double mean = (double)G / F;
  const double mx = (double)*std::max_element(totals.begin(), totals.end());
  const bool skewed = 2.0 * mx > 3.0 * mean + 16.0 * std::sqrt(mean) + 128.0;
  JOIN_DEBUG("HashJoin", "inner low-bit histogram: max %.0f vs mean %.1f -> key mixing %s", mx, mean,
             skewed ? "on" : "off");
  return skewed;
}

bool HashJoin::outputValid() const { return output && ctx->workspace().epoch() == outputEpoch; }

void HashJoin::join() {
  run();
  RESULT_COUNTER = result.localMatches;
}

void HashJoin::setRowSink(const kernels::RowSink &s) {
  const uint64_t off[2] = {s.offA, s.offB}, rows[2] = {s.rowsAN, s.rowsBN};
  for (int r = 0; r < 2; ++r)
    JOIN_ASSERT(ridLo[r] > ridHi[r] || (ridLo[r] >= off[r] && ridHi[r] - off[r] < rows[r]), "HashJoin",
                "row sink: %s payload rows [%lu, %lu) do not cover this rank's rids [%lu, %lu]",
                r ? "outer" : "inner", (unsigned long)off[r], (unsigned long)(off[r] + rows[r]),
                (unsigned long)ridLo[r], (unsigned long)ridHi[r]);
  sink = s;
  hasSink = true;
}

bool HashJoin::canFuseRows() const {
  return ctx->onDevice() && ctx->comm()->size() == 1 && plan.materialize && plan.splitLocal && !plan.wide;
}

JoinResult HashJoin::run() {
  // Watchdog context: an injected stall (HPCJOIN_STALL) waits on this join's
  // communicator, and a timed-out wait names the phase the join was in.
  struct WatchScope {
    explicit WatchScope(comm::Communicator *c) { utils::setWatchComm(c); }
    ~WatchScope() {
      utils::setWatchComm(nullptr);
      utils::setPhase("between joins");
    }
  } watch(ctx->comm());
  utils::setPhase("plan");
  try {
    if (passes > 1) return runPasses();
    return runImpl();
  } catch (const std::exception &e) {
    while (!TASK_QUEUE.empty()) TASK_QUEUE.pop();  // tasks are owned (and freed) by runImpl
    ctx->comm()->abort(e.what());
    throw;
  }
}

JoinResult HashJoin::runImpl() {
  performance::TraceRange traceJoin("hpcjoin::join");
  result = JoinResult();
  result.innerLocal = innerRelation->getLocalSize();
  result.outerLocal = outerRelation->getLocalSize();
  const uint64_t tSetup = nowUs();
  ctx->resetScratch();
  result.setupMs = (nowUs() - tSetup) / 1000.0;
  const bool dev = ctx->onDevice();
  if (dev) HIP_CHECK(hipSetDevice(ctx->device()));
  JoinEnv env{ctx, config, plan, innerRelation, outerRelation, ev, numberOfNodes, nodeId};

  Measurements::startJoin();
  ctx->timeline().reset();
  JoinRun run;
  run.t0 = nowUs();
  if (dev) HIP_CHECK(hipEventRecord(ev[0], ctx->stream()));
  if (plan.bitmapJoin) {
    if (BitmapPlan(env, bitmapExact).run(run.t0, result)) {
      RESULT_COUNTER = result.localMatches;
      return result;
    }
    plan = basePlan;  // a repeated inner key: this and every later join on the two-level plan
    ++result.localFallbacks;
    JOIN_DEBUG("HashJoin", "bitmap join: repeated inner key -> %s", plan.describe().c_str());
  }

  // ----------------------------------------------- histogram, windows, network
  Measurements::startHistogramComputation();
  utils::faultPoint("histogram");
  run.trace.reset(new performance::TraceRange("histogram"));
  const bool sampled = plan.sampledNetwork && !sampledOverflowed;
  bool done = false;
  if (sampled) {
    if (numberOfNodes == 1)
      done = SampledSingleRankExchange(env, localOverflowed).exchange(run);
    else
      done = SampledShuffleExchange(env).exchange(run);
    if (!done) {  // a slice overflowed (skew the sample missed): exact from now on
      sampledOverflowed = true;
      ++result.networkFallbacks;
    }
  }
  if (!done && plan.splitHistogram && !sampled) done = SplitHistogramExchange(env).exchange(run);
  if (!done) ExactExchange(env, sampled).exchange(run);
  Measurements::stopNetworkPartitioning();
  Measurements::storeNetworkDetails(innerRelation->getLocalSize(), outerRelation->getLocalSize(),
                                    run.hc ? run.hc->innerLocal()->getChunkCount() : 1);
  Measurements::startWaitingForNetworkCompletion();
  // Only the inner window is awaited here (a stream wait, no host sync): the
  // outer relation's all-to-all keeps running on the exchange stream while the
  // inner relation's local radix pass runs; LocalPartitioning waits for the
  // outer window right before its own pass.
  run.inner->stop();
  if (config.checks && run.hc) {
    run.inner->assertAllTuplesWritten();
    run.outer->assertAllTuplesWritten();
  }
  const bool verify = numberOfNodes > 1 && run.hc &&
                      (config.verifyExchange == core::PlanChoice::On ||
                       (config.verifyExchange == core::PlanChoice::Auto && plan.oneSided));
  if (verify) {  // both windows complete first (the outer one may still be on the links)
    // Its own phase (verifyMs), kept out of joinMs: hashing the input and both
    // windows again plus two collectives is a check, not join work.
    const uint64_t tv = nowUs();
    run.outer->stop();
    result.exchangeChecked = verifyExchange(env, run).cells;
    result.verifyMs = (nowUs() - tv) / 1000.0;
  }
  if (dev && !run.networkEventRecorded) HIP_CHECK(hipEventRecord(ev[2], ctx->stream()));
  Measurements::stopWaitingForNetworkCompletion();
  run.t3 = nowUs();

  // --------------------------------------------- local pass and build/probe
  LocalPhase local(env, localOverflowed, hasSink && canFuseRows() ? &sink : nullptr);
  local.run(run, result);
  const uint64_t t4 = nowUs();
  ctx->timeline().resolve();  // every stream was synchronised above
  output = local.buildProbes().empty() ? nullptr : local.buildProbes().front()->getOutput();
  outputEpoch = ctx->workspace().epoch();
  local.release();
  result.wireBytes = run.inner->wireBytesSent() + run.outer->wireBytesSent();
  result.innerReceived = run.inner->computeLocalWindowSize();
  result.outerReceived = run.outer->computeLocalWindowSize();
  result.sampledNetwork = run.sampled;
  result.roundWindows = (run.inner->roundMap().on() || run.inner->sendRounded() ? 1u : 0u) +
                        (run.outer->roundMap().on() || run.outer->sendRounded() ? 1u : 0u);
  result.directScatter = run.inner->directScatter() || run.outer->directScatter();
  Measurements::storeLocalPartitioningDetails(result.innerReceived + result.outerReceived, result.localItems);
  Measurements::storeBuildProbeDetails(result.innerReceived, result.outerReceived, result.buildProbeItems);
  Measurements::storeResultTuples(result.localMatches);
  Measurements::stopJoin();
  recordTimes(run, t4);

  uint64_t g = result.localMatches;
  ctx->comm()->allReduceSumHost(&g, 1);
  result.globalMatches = g;
  result.teardownMs = (nowUs() - t4) / 1000.0;
  RESULT_COUNTER = result.localMatches;
  return result;
}

// Host phase spans and the device spans between the join's five events.
void HashJoin::recordTimes(const JoinRun &run, uint64_t t4) {
  result.joinMs = (t4 - run.t0) / 1000.0 - result.verifyMs;
  result.histogramMs = (run.t1 - run.t0) / 1000.0;
  result.windowMs = (run.t2 - run.t1) / 1000.0;
  result.networkMs = (run.t3 - run.t2) / 1000.0 - result.verifyMs;
  result.localMs = (t4 - run.t3) / 1000.0;
  if (!ctx->onDevice()) return;
  float ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
  result.devHistogramMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[1], ev[2]));
  result.devNetworkMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[2], ev[3]));
  result.devLocalPartitionMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[3], ev[4]));
  result.devBuildProbeMs = ms;
  HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[4]));
  result.devSpanMs = ms;
  Measurements::storeDevicePhase("DHIST", result.devHistogramMs);
  Measurements::storeDevicePhase("DNET", result.devNetworkMs);
  Measurements::storeDevicePhase("DLOCPART", result.devLocalPartitionMs);
  Measurements::storeDevicePhase("DBP", result.devBuildProbeMs);
}

}  // namespace operators
}  // namespace hpcjoin
