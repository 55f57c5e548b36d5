#include "JoinStrategies.h"

#include "HashJoin.h"
#include "../comm/Communicator.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../tasks/BitmapJoin.h"
#include "../tasks/NetworkPartitioning.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace operators {

using performance::Measurements;
using performance::nowUs;

void JoinRun::phase(const char *name) {
  trace.reset();  // roctx ranges nest: pop before the next push
  trace.reset(new performance::TraceRange(name));
}

std::unique_ptr<data::Window> ExchangeStrategy::makeWindow(tasks::HistogramComputation &hc, int side) const {
  const core::JoinPlan &plan = env.plan;
  std::unique_ptr<data::Window> w(new data::Window(
      (side == 0 ? hc.innerOffsetMap() : hc.outerOffsetMap())->getExchangePlan(),
      side == 0 ? hc.innerGlobal() : hc.outerGlobal(), hc.assignmentMap(), env.ctx, plan.wide,
      plan.oneSided && env.ctx->onDevice() && !env.ctx->comm()->sharesAddressSpace()));
  if (plan.oneSided) w->enableOneSided();
  if (plan.wireBits[side]) {
    kernels::WireCodec c;
    c.w = plan.wireBits[side];
    c.ridBits = plan.wireRidBits[side];
    c.keyShift = plan.keyShift;
    w->setWireCodec(c, plan.ridBase[side]);
  }
  return w;
}

// ----------------------------------------------------------- N == 1, sampled
bool SampledSingleRankExchange::exchange(JoinRun &run) {
  core::ExecContext *ctx = env.ctx;
  run.sp.reset(new tasks::SampledNetworkPartitioning(env.inner, env.outer, ctx, env.plan,
                                                     env.config.maxPartitionBlocks, env.config.sampleStride));
  tasks::SampledNetworkPartitioning &sp = *run.sp;
  const uint64_t h0 = nowUs();
  sp.sample();
  HIP_CHECK(hipEventRecord(env.ev[1], ctx->stream()));
  Measurements::stopHistogramComputation();
  Measurements::storeHistogramDetails(nowUs() - h0, env.inner->getLocalSize(), env.outer->getLocalSize(), 0, 0, 0);
  run.t1 = nowUs();
  Measurements::startWindowAllocation();
  sp.layoutSide(0);
  Measurements::stopWindowAllocation();
  run.t2 = nowUs();
  Measurements::startNetworkPartitioning();
  run.trace.reset();
  utils::faultPoint("network");
  run.phase("network_partitioning");
  // Host work of each side runs while the GPU works on the other: the outer
  // layout during the inner scatter, the inner plan and local-pass setup
  // during the outer scatter, the outer plan during the inner local pass.
  sp.scatterSide(0);
  sp.layoutSide(1);
  sp.scatterSide(1);
  HIP_CHECK(hipEventRecord(env.ev[2], ctx->stream()));
  run.networkEventRecorded = true;
  bool ok = sp.finishSide(0);
  if (ok) {
    run.lp.reset(new tasks::LocalPartitioning(sp.innerWindow(), sp.outerWindow(), ctx, env.plan, localExact));
    // (Running this pass on a stream of its own, next to the outer network
    // scatter, was measured slower: 18.90 -> 19.11 ms per 1B x 1B general
    // join, the two scatters contending; profiles/r6/README.md.)
    run.lp->partitionSide(sp.innerWindow(), 0);
    ok = sp.finishSide(1);
  }
  if (!ok) {
    run.lp.reset();  // an inner local pass may be queued: harmless, its output is dropped
    run.networkEventRecorded = false;
    return false;
  }
  run.inner = sp.innerWindow();
  run.outer = sp.outerWindow();
  run.sampled = true;
  return true;
}

// ----------------------------------------------------------- N > 1, sampled
bool SampledShuffleExchange::exchange(JoinRun &run) {
  core::ExecContext *ctx = env.ctx;
  run.hc.reset(new tasks::HistogramComputation(env.nodes, env.nodeId, env.inner, env.outer, ctx, env.plan,
                                               env.config.maxPartitionBlocks));
  run.ss.reset(new tasks::SampledShuffle(env.nodes, env.nodeId, run.hc.get(), ctx, env.plan, env.config.sampleStride));
  tasks::SampledShuffle &ss = *run.ss;
  const uint64_t h0 = nowUs();
  ss.sampleAndAssign();
  HIP_CHECK(hipEventRecord(env.ev[1], ctx->stream()));
  Measurements::stopHistogramComputation();
  Measurements::storeHistogramDetails(nowUs() - h0, env.inner->getLocalSize(), env.outer->getLocalSize(),
                                      run.hc->globalUs, run.hc->assignUs, 0);
  run.t1 = nowUs();
  Measurements::startWindowAllocation();
  ss.layoutSide(0);
  ss.layoutSide(1);
  Measurements::stopWindowAllocation();
  run.t2 = nowUs();
  Measurements::startNetworkPartitioning();
  run.trace.reset();
  utils::faultPoint("network");
  run.phase("network_partitioning");
  // Both scatters are enqueued before the first wait: the host gathers the
  // inner chunks' fills (and enqueues their exchanges) while the outer
  // relation is still being scattered.
  ss.scatterSide(0);
  ss.scatterSide(1);
  const bool ok = ss.exchangeSide(0) && ss.exchangeSide(1);
  if (!ok) {
    ctx->synchronize();  // drain what was enqueued; the exact re-run uses fresh buffers
    return false;
  }
  run.inner = ss.window(0);
  run.outer = ss.window(1);
  run.sampled = true;
  return true;
}

// --------------------------------------------------- N > 1, split histogram
bool SplitHistogramExchange::exchange(JoinRun &run) {
  core::ExecContext *ctx = env.ctx;
  run.hc.reset(new tasks::HistogramComputation(env.nodes, env.nodeId, env.inner, env.outer, ctx, env.plan,
                                               env.config.maxPartitionBlocks));
  tasks::HistogramComputation &hc = *run.hc;
  hc.executeInner(env.config.sampleStride);
  if (ctx->onDevice()) HIP_CHECK(hipEventRecord(env.ev[1], ctx->stream()));
  Measurements::stopHistogramComputation();
  Measurements::storeHistogramDetails(hc.localUs, env.inner->getLocalSize(), env.outer->getLocalSize(), hc.globalUs,
                                      hc.assignUs, hc.offsetUs);
  // The head all-gather is the inner relation's; the outer exact histogram's
  // all-gather runs later on the exchange stream (HOGLOBAL Timeline span).
  Measurements::put("HIGLOBAL", (double)hc.globalUs, "us");
  Measurements::put("HOGLOBAL", 0, "us");
  run.t1 = nowUs();
  Measurements::startWindowAllocation();
  run.innerOwned = makeWindow(hc, 0);
  run.inner = run.innerOwned.get();
  Measurements::stopWindowAllocation();
  run.t2 = nowUs();
  Measurements::startNetworkPartitioning();
  run.trace.reset();
  utils::faultPoint("network");
  run.phase("network_partitioning");
  tasks::NetworkPartitioning np(env.nodeId, env.inner, env.outer, run.inner, nullptr, &hc, ctx, env.plan);
  np.partitionInner([&](uint32_t c) {
    if (c == 0) hc.launchOuter(ctx->commStream());
  });
  hc.finishOuter();
  run.outerOwned = makeWindow(hc, 1);
  run.outer = run.outerOwned.get();
  np.partitionOuter(run.outer);
  return true;
}

// ------------------------------------------------------------------- exact
bool ExactExchange::exchange(JoinRun &run) {
  core::ExecContext *ctx = env.ctx;
  run.hc.reset(new tasks::HistogramComputation(env.nodes, env.nodeId, env.inner, env.outer, ctx, env.plan,
                                               env.config.maxPartitionBlocks));
  tasks::HistogramComputation &hc = *run.hc;
  hc.execute();
  if (!retry) {
    if (ctx->onDevice()) HIP_CHECK(hipEventRecord(env.ev[1], ctx->stream()));
    Measurements::stopHistogramComputation();
    Measurements::storeHistogramDetails(hc.localUs, env.inner->getLocalSize(), env.outer->getLocalSize(), hc.globalUs,
                                        hc.assignUs, hc.offsetUs);
    run.t1 = nowUs();
    Measurements::startWindowAllocation();
  }
  run.innerOwned = makeWindow(hc, 0);
  run.outerOwned = makeWindow(hc, 1);
  run.inner = run.innerOwned.get();
  run.outer = run.outerOwned.get();
  if (!retry) {
    Measurements::stopWindowAllocation();
    run.t2 = nowUs();
    Measurements::startNetworkPartitioning();
    run.trace.reset();
    utils::faultPoint("network");
    run.phase("network_partitioning");
  }
  tasks::NetworkPartitioning np(env.nodeId, env.inner, env.outer, run.inner, run.outer, &hc, ctx, env.plan);
  np.execute();
  return true;
}

// -------------------------------------------------------------- local phase
tasks::BuildProbe *LocalPhase::addBuildProbe(data::Window *inner, data::Window *outer) {
  bps.emplace_back(new tasks::BuildProbe(inner, outer, env.ctx, env.plan, env.config.outputCapacity));
  if (sink) bps.back()->setRowSink(sink);
  if (env.config.outputHost && env.plan.materialize) {
    JOIN_ASSERT(env.config.outputCapacity > 0, "HashJoin", "outputHost needs outputCapacity (pairs it holds)");
    bps.back()->setHostOutput(env.config.outputHost);
  }
  return bps.back().get();
}

void LocalPhase::run(JoinRun &run, JoinResult &r) {
  core::ExecContext *ctx = env.ctx;
  const bool dev = ctx->onDevice();
  hipEvent_t *ev = env.ev;
  Measurements::startLocalProcessingPreparations();
  run.trace.reset();
  r.splitPartitions = run.hc ? run.hc->assignmentMap()->splitPartitions() : 0;
  utils::faultPoint("local");
  run.phase("local_processing");
  if (!run.lp) run.lp.reset(new tasks::LocalPartitioning(run.inner, run.outer, ctx, env.plan, localOverflowed));
  tasks::LocalPartitioning *lp = run.lp.get();
  Measurements::stopLocalProcessingPreparations();
  Measurements::startLocalProcessing();
  const uint32_t outerChunks = run.outer->getPlan().chunks;
  if (env.plan.pipelineOuter && !localOverflowed && outerChunks > 1) {
    // N > 1, counting: the outer relation is local-partitioned and probed
    // chunk by chunk as its exchange chunks land (chunk views of the window),
    // so after the last chunk arrives only its own share is left to do.  The
    // inner tables are rebuilt per chunk (off the critical path while later
    // chunks are on the links).
    lp->partitionSide(run.inner, 0);
    for (uint32_t c = 0; c < outerChunks; ++c) {
      outerViews.push_back(run.outer->chunkView(c));
      lp->partitionSide(outerViews.back().get(), 1 + (int)c);
      if (c + 1 == outerChunks && dev) HIP_CHECK(hipEventRecord(ev[3], ctx->stream()));
      if (c == 0) utils::faultPoint("build_probe");
      addBuildProbe(run.inner, outerViews.back().get())->execute();
    }
    r.localItems = lp->workItems();
  } else {
    // The reference's task queue (operators/HashJoin.cpp:187-204): the local
    // pass enqueues the build/probe of its partitions when it is done.
    std::queue<tasks::Task *> &queue = HashJoin::TASK_QUEUE;
    queue.push(lp);
    while (!queue.empty()) {
      tasks::Task *t = queue.front();
      queue.pop();
      if (t->getType() == TASK_BUILD_PROBE) utils::faultPoint("build_probe");
      t->execute();
      if (t->getType() == TASK_PARTITION) {
        if (dev) HIP_CHECK(hipEventRecord(ev[3], ctx->stream()));
        r.localItems = lp->workItems();
        queue.push(addBuildProbe(run.inner, run.outer));
      }
    }
  }
  run.trace.reset();
  if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
  ctx->synchronize();
  r.sampledLocal = lp->sampled();
  if (lp->sampled() && lp->overflowed()) {
    // A sampled slot overflowed (skew the sample missed): the build/probe ran
    // on incomplete partitions.  Redo the local pass exactly over the whole
    // windows, then the build/probe; later joins stay exact.
    localOverflowed = true;
    ++r.localFallbacks;
    r.sampledLocal = false;
    release();
    run.lp.reset(new tasks::LocalPartitioning(run.inner, run.outer, ctx, env.plan, true));
    run.lp->execute();
    r.localItems = run.lp->workItems();
    addBuildProbe(run.inner, run.outer)->execute();
    if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
    ctx->synchronize();
  }
  for (auto &bp : bps)
    while (bp->collect()) {  // rare: item list or output buffer overflowed -> exact re-run
      ++r.reruns;
      bp->execute();
      if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
      ctx->synchronize();
    }
  // Repeated inner keys chained in (or overflowed) the quotient table: later
  // joins count every partition on counted tables (keyCount 9).
  for (auto &bp : bps)
    if (bp->sawDuplicateChains() && env.plan.variants.keyCount == 8) env.plan.variants.keyCount = 9;
  r.localMatches = 0;
  r.buildProbeItems = 0;
  for (auto &bp : bps) {
    r.localMatches += bp->getMatches();
    r.buildProbeItems += bp->getWorkItems();
  }
  // Materializing joins have exactly one build/probe (never pipelined).
  r.outputPairs = env.plan.materialize && !bps.empty() ? bps.front()->getOutputCount() : 0;
  r.outputOverflow = !bps.empty() && bps.front()->outputOverflowed();
  r.rowsFused = !bps.empty() && bps.front()->rowsFused();
  Measurements::stopLocalProcessing();
}

// ---------------------------------------------------------------- bitmaps
bool BitmapPlan::run(uint64_t t0, JoinResult &r) {
  core::ExecContext *ctx = env.ctx;
  const core::JoinPlan &plan = env.plan;
  performance::TraceRange trace("bitmap_join");
  Measurements::startHistogramComputation();
  utils::faultPoint("histogram");
  Measurements::stopHistogramComputation();
  Measurements::startNetworkPartitioning();
  tasks::BitmapJoin bj(env.inner, env.outer, ctx, plan, env.config.maxPartitionBlocks, env.config.sampleStride,
                       env.ev);
  tasks::BitmapJoin::Outcome o = bj.run(exact);
  if (o.overflow) {
    // A sampled slice overflowed on some rank (skew the sample missed): every
    // rank redoes the join with exact histograms, as do later joins.
    exact = true;
    env.plan.sampledNetwork = false;
    env.plan.fragments = false;
    ++r.networkFallbacks;
    if (ctx->onDevice()) HIP_CHECK(hipEventRecord(env.ev[0], ctx->stream()));
    o = bj.run(true);
    JOIN_ASSERT(!o.overflow, "HashJoin", "exact bitmap pass overflowed");
  }
  Measurements::stopNetworkPartitioning();
  if (o.dup) return false;
  Measurements::startLocalProcessing();
  Measurements::stopLocalProcessing();
  const uint64_t t4 = nowUs();
  ctx->timeline().resolve();  // BitmapJoin synchronised all streams
  r.bitmapJoin = true;
  r.groupPasses = o.groupPasses;
  r.sampledNetwork = !exact;
  r.localMatches = o.localMatches;
  r.globalMatches = o.globalMatches;
  r.buildProbeItems = 1ull << plan.networkBits;
  r.innerReceived = env.inner->getLocalSize();
  r.outerReceived = env.outer->getLocalSize();
  r.wireBytes = o.linkBytes;
  r.joinMs = (t4 - t0) / 1000.0;
  r.networkMs = r.joinMs;
  r.devNetworkMs = o.devSampleMs + o.devScatterMs;
  r.devBuildProbeMs = o.devJoinMs;
  r.enqueueMs = o.enqueueUs > t0 ? (o.enqueueUs - t0) / 1000.0 : 0.0;
  r.hostWaitMs = o.hostWaitMs;
  if (ctx->onDevice()) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, env.ev[0], env.ev[4]));
    r.devSpanMs = ms;
  }
  Measurements::storeNetworkDetails(env.inner->getLocalSize(), env.outer->getLocalSize(), 1);
  Measurements::storeBuildProbeDetails(r.innerReceived, r.outerReceived, r.buildProbeItems);
  Measurements::storeResultTuples(r.localMatches);
  Measurements::storeDevicePhase("DNET", r.devNetworkMs);
  Measurements::storeDevicePhase("DBP", r.devBuildProbeMs);
  Measurements::stopJoin();
  return true;
}

}  // namespace operators
}  // namespace hpcjoin
