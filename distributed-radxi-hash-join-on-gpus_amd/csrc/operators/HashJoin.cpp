#include "HashJoin.h"

#include <algorithm>
#include <cmath>
#include <vector>

#include "../comm/Communicator.h"
#include "../comm/World.h"
#include "../host/HostOps.h"
#include "../data/Window.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Trace.h"
#include "../tasks/BuildProbe.h"
#include "../tasks/HistogramComputation.h"
#include "../tasks/LocalPartitioning.h"
#include "../tasks/NetworkPartitioning.h"
#include "../tasks/SampledNetworkPartitioning.h"
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
  // and every chunk c: min rid, max rid}.
  const uint32_t C = std::max<uint32_t>(1, config.chunks);
  const size_t STATS = 2 + 4 * (size_t)C;
  std::vector<uint64_t> st(STATS, 0);
  int which = 0;
  for (data::Relation *r : {innerRelation, outerRelation}) {
    for (uint32_t c = 0; c < C; ++c) {
      uint64_t b, e;
      histograms::LocalHistogram::chunkRange(r->getLocalSize(), C, config.maxPartitionBlocks, c, &b, &e);
      uint64_t h[3] = {0, 0, ~0ull};
      if (ctx->onDevice() && e > b) {
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
      st[2 + ((size_t)which * C + c) * 2] = h[2];
      st[3 + ((size_t)which * C + c) * 2] = h[1];
    }
    ++which;
  }
  ctx->workspace().reset();
  std::vector<uint64_t> all(STATS * numberOfNodes);
  ctx->comm()->allGatherHost(st.data(), all.data(), STATS);
  uint64_t mx[2] = {0, 0};
  for (uint32_t r = 0; r < numberOfNodes; ++r) {
    mx[0] = std::max(mx[0], all[STATS * r]);
    mx[1] = std::max(mx[1], all[STATS * r + 1]);
  }
  plan = core::makePlan(config, numberOfNodes, innerRelation->getGlobalSize(), outerRelation->getGlobalSize(), mx[0],
                        mx[1]);
  planWireCodec(all, STATS, C);
  if (config.keyHashing == core::KeyHashing::Auto && plan.keyBits < 64) plan.keyMix = lowKeyBitsSkewed();
  if (!ctx->onDevice()) {
    plan.localHistogram = core::HistogramMode::Exact;  // sampling pays on HBM only
    plan.splitLocal = false;                           // split columns are a device layout
  }
  {
    const bool eligible = numberOfNodes == 1 && ctx->onDevice() && plan.chunks == 1;
    const uint64_t small = std::min(innerRelation->getGlobalSize(), outerRelation->getGlobalSize());
    if (config.networkHistogram == core::HistogramMode::Sampled)
      plan.sampledNetwork = eligible;
    else if (config.networkHistogram == core::HistogramMode::Auto)
      plan.sampledNetwork = eligible && small >= (16ull << 20);
  }
  // N == 1 counting joins: the single-level bitmap join replaces the local
  // pass when the key fragment above the network digit fits an LDS bitmap.
  // The network pass then runs at 10 bits (1024 partitions, 128 KiB bitmaps
  // for 1B dense keys: measured 13.5 ms per 1B x 1B join vs 14.1 ms at 11 bits
  // with 64 KiB bitmaps -- the 2048-way scatter writes shorter runs), or 11
  // bits when the key range needs it.  The plan keeps a two-level split of the
  // same total for the duplicate-key fallback.
  if (config.bitmapJoin && plan.sampledNetwork && !plan.materialize && !plan.wide && !plan.keyMix) {
    const uint32_t want = plan.keyBits > kernels::BITMAP_MAX_BITS ? plan.keyBits - kernels::BITMAP_MAX_BITS : 0;
    const uint32_t nb = config.networkBits ? config.networkBits
                                           : std::min<uint32_t>(kernels::MAX_PART_BITS, std::max<uint32_t>(10, want));
    const uint32_t bits = plan.keyBits > nb ? plan.keyBits - nb : 0;
    if (plan.keyBits < 64 && bits <= kernels::BITMAP_MAX_BITS && plan.keyShift + bits <= 64) {
      if (nb != plan.networkBits) {
        core::JoinConfig c2 = config;
        const uint32_t total = plan.networkBits + plan.localBits;
        c2.networkBits = nb;
        c2.localBits = total > nb ? std::min<uint32_t>(total - nb, kernels::MAX_PART_BITS) : 1;
        core::JoinPlan p2 = core::makePlan(c2, numberOfNodes, innerRelation->getGlobalSize(),
                                           outerRelation->getGlobalSize(), mx[0], mx[1]);
        p2.keyMix = plan.keyMix;
        p2.sampledNetwork = plan.sampledNetwork;
        p2.localHistogram = plan.localHistogram;
        plan = p2;
        planWireCodec(all, STATS, C);
      }
      plan.bitmapJoin = true;
      plan.bitmapBits = bits;
    }
  }
  // N > 1 pipelines (also on the host path, where they run in place: same
  // logic, covered by the CPU tests).
  plan.splitHistogram = config.splitHistogram && numberOfNodes > 1;
  plan.pipelineOuter = config.pipelineOuter && numberOfNodes > 1 && !plan.materialize && plan.twoLevel;
  JOIN_DEBUG("HashJoin", "%s", plan.describe().c_str());
  if (ctx->onDevice())
    for (auto &e : ev) HIP_CHECK(hipEventCreate(&e));
}

// Wire codec per relation (kernels.h, WireCodec): frame-of-reference rids
// (base = the smallest rid of the sending rank's exchange chunk: a chunk is a
// contiguous quarter of the rank's input, so positional rids need 2 bits less
// than with one base per rank) plus the key fragment above the network digit.
// Auto packs on a device engine with N > 1 when it saves at least 1/8 of the
// wire bytes (w <= 56); On forces it (also on the host path).
void HashJoin::planWireCodec(const std::vector<uint64_t> &all, size_t stride, uint32_t chunks) {
  for (int r = 0; r < 2; ++r) {
    plan.wireBits[r] = 0;
    plan.wireRidBits[r] = 0;
    plan.ridBase[r].assign((size_t)numberOfNodes * chunks, 0);
  }
  if (plan.wide || numberOfNodes == 1 || config.wireCodec == core::WireCodecMode::Off) return;
  const uint32_t keyW = plan.keyBits > plan.networkBits ? plan.keyBits - plan.networkBits : 0;
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
    const uint32_t ridBits = std::max<uint32_t>(1, ceilLog2(span));
    const uint32_t w = ridBits + keyW;
    const bool on = config.wireCodec == core::WireCodecMode::On ? w < 64 : (ctx->onDevice() && w <= 56);
    if (on && ridBits <= plan.keyShift) {
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

void HashJoin::launchBitmapJoin(data::Window *inner, data::Window *outer) {
  const uint32_t F = 1u << plan.networkBits, G = kernels::CLAIM_GROUPS;
  const size_t n = (size_t)F * G;
  // One upload: [inner starts | outer starts] (u64), [inner lens | outer lens]
  // (u32), then the zeroed {matches, dup} words.
  const size_t words = 2 * n + n + 2;  // u64 words: 2n starts, 2n u32 lens = n words, 2 counters
  bmUpload.assign(words, 0);
  uint64_t *starts = bmUpload.data();
  uint32_t *lens = reinterpret_cast<uint32_t *>(bmUpload.data() + 2 * n);
  data::Window *w[2] = {inner, outer};
  for (int k = 0; k < 2; ++k)
    for (const histograms::Segment &sg : w[k]->getPlan().segments) {
      HJ_CHECK(sg.lp < F && sg.source < G && sg.len < (1ull << 32), "bitmap join: segment (%u, %u) of %lu tuples",
               sg.lp, sg.source, (unsigned long)sg.len);
      const size_t i = k * n + (size_t)sg.lp * G + sg.source;
      HJ_CHECK(lens[i] == 0, "bitmap join: two segments for partition %u, group %u", sg.lp, sg.source);
      starts[i] = sg.begin;
      lens[i] = (uint32_t)sg.len;
    }
  uint64_t *dev = ctx->workspace().getArray<uint64_t>(words);
  ctx->copy(dev, bmUpload.data(), words * 8, true, false);
  const uint32_t *dLens = reinterpret_cast<const uint32_t *>(dev + 2 * n);
  unsigned long long *dOut = reinterpret_cast<unsigned long long *>(dev + 3 * n);
  HIP_CHECK(hipEventRecord(ev[3], ctx->stream()));
  utils::faultPoint("build_probe");
  kernels::bitmapJoin(static_cast<const uint64_t *>(inner->getData()), static_cast<const uint64_t *>(outer->getData()),
                      dev, dLens, dev + n, dLens + n, F, G, plan.keyShift, plan.bitmapBits, dOut,
                      reinterpret_cast<uint32_t *>(dOut + 1), ctx->stream());
  HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
  bmBack = ctx->staging().getArray<unsigned long long>(2);
  HIP_CHECK(hipMemcpyAsync(bmBack, dOut, 16, hipMemcpyDeviceToHost, ctx->stream()));
}

void HashJoin::join() {
  run();
  RESULT_COUNTER = result.localMatches;
}

JoinResult HashJoin::run() {
  try {
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

  Measurements::startJoin();
  const uint64_t t0 = nowUs();
  if (dev) HIP_CHECK(hipEventRecord(ev[0], ctx->stream()));

  // ---------------------------------------------------------------- histogram
  Measurements::startHistogramComputation();
  utils::faultPoint("histogram");
  std::unique_ptr<performance::TraceRange> trace(new performance::TraceRange("histogram"));
  std::unique_ptr<tasks::HistogramComputation> hc;
  std::unique_ptr<tasks::SampledNetworkPartitioning> sp;
  std::unique_ptr<data::Window> innerOwned, outerOwned;
  data::Window *innerWindow = nullptr, *outerWindow = nullptr;
  const bool sampled = plan.sampledNetwork && !sampledOverflowed;
  uint64_t t1, t2;
  // Local pass (created early on the single-rank sampled path, which starts
  // the inner relation's local pass while the outer scatter still runs).
  std::unique_ptr<tasks::LocalPartitioning> lp;
  bool networkEventRecorded = false;
  bool bitmapLaunched = false, bitmapDone = false;
  if (sampled) {
    // ---------------------------------------- single-rank sampled network pass
    sp.reset(new tasks::SampledNetworkPartitioning(innerRelation, outerRelation, ctx, plan,
                                                   config.maxPartitionBlocks, config.sampleStride));
    const uint64_t h0 = nowUs();
    sp->sample();
    if (dev) HIP_CHECK(hipEventRecord(ev[1], ctx->stream()));
    Measurements::stopHistogramComputation();
    Measurements::storeHistogramDetails(nowUs() - h0, innerRelation->getLocalSize(), outerRelation->getLocalSize(),
                                        0, 0, 0);
    t1 = nowUs();
    Measurements::startWindowAllocation();
    sp->layoutSide(0);
    Measurements::stopWindowAllocation();
    t2 = nowUs();
    Measurements::startNetworkPartitioning();
    trace.reset();  // roctx ranges nest: pop before the next push
    utils::faultPoint("network");
    trace.reset(new performance::TraceRange("network_partitioning"));
    // Host work of each side runs while the GPU works on the other: the
    // outer layout during the inner scatter, the inner plan and local-pass
    // setup during the outer scatter, the outer plan during the inner local
    // pass.
    sp->scatterSide(0);
    sp->layoutSide(1);
    sp->scatterSide(1);
    if (dev) HIP_CHECK(hipEventRecord(ev[2], ctx->stream()));
    networkEventRecorded = true;
    bool ok = sp->finishSide(0);
    if (ok && plan.bitmapJoin) {
      ok = sp->finishSide(1);
      if (ok) {
        launchBitmapJoin(sp->innerWindow(), sp->outerWindow());
        bitmapLaunched = true;
      }
    } else if (ok) {
      lp.reset(new tasks::LocalPartitioning(sp->innerWindow(), sp->outerWindow(), ctx, plan, localOverflowed));
      lp->partitionSide(sp->innerWindow(), 0);
      ok = sp->finishSide(1);
    }
    if (ok) {
      innerWindow = sp->innerWindow();
      outerWindow = sp->outerWindow();
    } else {
      lp.reset();  // an inner local pass may be queued: harmless, its output is dropped
      networkEventRecorded = false;
      // A slice overflowed: the sample missed skew.  Redo this join (and all
      // later ones) with the exact histogram path.
      sampledOverflowed = true;
      ++result.networkFallbacks;
    }
  }
  if (!innerWindow && plan.splitHistogram && !sampled) {
    // ------------------------ N > 1: outer histogram overlaps the inner exchange
    hc.reset(new tasks::HistogramComputation(numberOfNodes, nodeId, innerRelation, outerRelation, ctx, plan,
                                             config.maxPartitionBlocks));
    hc->executeInner(config.sampleStride);
    if (dev) HIP_CHECK(hipEventRecord(ev[1], ctx->stream()));
    Measurements::stopHistogramComputation();
    Measurements::storeHistogramDetails(hc->localUs, innerRelation->getLocalSize(), outerRelation->getLocalSize(),
                                        hc->globalUs, hc->assignUs, hc->offsetUs);
    t1 = nowUs();
    Measurements::startWindowAllocation();
    auto makeWindow = [&](int r) {
      std::unique_ptr<data::Window> w(new data::Window(
          (r == 0 ? hc->innerOffsetMap() : hc->outerOffsetMap())->getExchangePlan(),
          r == 0 ? hc->innerGlobal() : hc->outerGlobal(), hc->assignmentMap(), ctx, plan.wide));
      if (plan.wireBits[r]) {
        kernels::WireCodec c;
        c.w = plan.wireBits[r];
        c.ridBits = plan.wireRidBits[r];
        c.keyShift = plan.keyShift;
        w->setWireCodec(c, plan.ridBase[r]);
      }
      return w;
    };
    innerOwned = makeWindow(0);
    innerWindow = innerOwned.get();
    Measurements::stopWindowAllocation();
    t2 = nowUs();
    Measurements::startNetworkPartitioning();
    trace.reset();  // roctx ranges nest: pop before the next push
    utils::faultPoint("network");
    trace.reset(new performance::TraceRange("network_partitioning"));
    tasks::NetworkPartitioning np(nodeId, innerRelation, outerRelation, innerWindow, nullptr, hc.get(), ctx, plan);
    np.partitionInner([&](uint32_t c) {
      if (c == 0) hc->launchOuter(ctx->commStream());
    });
    hc->finishOuter();
    outerOwned = makeWindow(1);
    outerWindow = outerOwned.get();
    np.partitionOuter(outerWindow);
  }
  if (!innerWindow) {
    if (!sampled) {
      hc.reset(new tasks::HistogramComputation(numberOfNodes, nodeId, innerRelation, outerRelation, ctx, plan,
                                               config.maxPartitionBlocks));
      hc->execute();
      if (dev) HIP_CHECK(hipEventRecord(ev[1], ctx->stream()));
      Measurements::stopHistogramComputation();
      Measurements::storeHistogramDetails(hc->localUs, innerRelation->getLocalSize(), outerRelation->getLocalSize(),
                                          hc->globalUs, hc->assignUs, hc->offsetUs);
      t1 = nowUs();
      Measurements::startWindowAllocation();
    } else {
      hc.reset(new tasks::HistogramComputation(numberOfNodes, nodeId, innerRelation, outerRelation, ctx, plan,
                                               config.maxPartitionBlocks));
      hc->execute();
    }
    innerOwned.reset(new data::Window(hc->innerOffsetMap()->getExchangePlan(), hc->innerGlobal(),
                                      hc->assignmentMap(), ctx, plan.wide));
    outerOwned.reset(new data::Window(hc->outerOffsetMap()->getExchangePlan(), hc->outerGlobal(),
                                      hc->assignmentMap(), ctx, plan.wide));
    innerWindow = innerOwned.get();
    outerWindow = outerOwned.get();
    for (int r = 0; r < 2; ++r)
      if (plan.wireBits[r]) {
        kernels::WireCodec c;
        c.w = plan.wireBits[r];
        c.ridBits = plan.wireRidBits[r];
        c.keyShift = plan.keyShift;
        (r == 0 ? innerWindow : outerWindow)->setWireCodec(c, plan.ridBase[r]);
      }
    if (!sampled) {
      Measurements::stopWindowAllocation();
      t2 = nowUs();
      // ---------------------------------------------------------------- network
      Measurements::startNetworkPartitioning();
      trace.reset();  // roctx ranges nest: pop before the next push
      utils::faultPoint("network");
      trace.reset(new performance::TraceRange("network_partitioning"));
    }
    tasks::NetworkPartitioning np(nodeId, innerRelation, outerRelation, innerWindow, outerWindow, hc.get(), ctx,
                                  plan);
    np.execute();
  }
  Measurements::stopNetworkPartitioning();
  Measurements::storeNetworkDetails(innerRelation->getLocalSize(), outerRelation->getLocalSize(),
                                    hc ? hc->innerLocal()->getChunkCount() : 1);
  Measurements::startWaitingForNetworkCompletion();
  // Only the inner window is awaited here (a stream wait, no host sync): the
  // outer relation's all-to-all keeps running on the exchange stream while the
  // inner relation's local radix pass runs; LocalPartitioning waits for the
  // outer window right before its own pass.
  innerWindow->stop();
  if (config.checks && hc) {
    innerWindow->assertAllTuplesWritten();
    outerWindow->assertAllTuplesWritten();
  }
  if (dev && !networkEventRecorded) HIP_CHECK(hipEventRecord(ev[2], ctx->stream()));
  Measurements::stopWaitingForNetworkCompletion();
  const uint64_t t3 = nowUs();

  // -------------------------------------------------------------------- local
  Measurements::startLocalProcessingPreparations();
  trace.reset();  // roctx ranges nest: pop before the next push
  utils::faultPoint("local");
  trace.reset(new performance::TraceRange("local_processing"));
  // Every build/probe of this join (one, or one per outer chunk when pipelined).
  std::vector<std::unique_ptr<tasks::BuildProbe>> bps;
  std::vector<std::unique_ptr<data::Window>> outerViews;
  uint64_t bitmapMatches = 0;
  if (bitmapLaunched) {
    Measurements::stopLocalProcessingPreparations();
    Measurements::startLocalProcessing();
    ctx->synchronize();
    if (bmBack[1] == 0) {
      bitmapMatches = bmBack[0];
      bitmapDone = true;
    } else {
      // A repeated (or out-of-range) inner key fragment: the bitmap cannot
      // count it.  Run the two-level pass on the same windows; later joins
      // skip the bitmap.
      plan.bitmapJoin = false;
      ++result.localFallbacks;
    }
  }
  if (!bitmapDone) {
    if (!lp) lp.reset(new tasks::LocalPartitioning(innerWindow, outerWindow, ctx, plan, localOverflowed));
    if (!bitmapLaunched) {
      Measurements::stopLocalProcessingPreparations();
      Measurements::startLocalProcessing();
    }
    const uint32_t outerChunks = outerWindow->getPlan().chunks;
    if (plan.pipelineOuter && !localOverflowed && outerChunks > 1) {
      // ---- N > 1, counting: the outer relation is local-partitioned and probed
      // chunk by chunk as its exchange chunks land (chunk views of the window),
      // so after the last chunk arrives only its own share is left to do.  The
      // inner tables are rebuilt per chunk (2-byte fragments, off the critical
      // path while later chunks are on the links).
      lp->partitionSide(innerWindow, 0);
      for (uint32_t c = 0; c < outerChunks; ++c) {
        outerViews.push_back(outerWindow->chunkView(c));
        lp->partitionSide(outerViews.back().get(), 1 + (int)c);
        if (c + 1 == outerChunks && dev) HIP_CHECK(hipEventRecord(ev[3], ctx->stream()));
        if (c == 0) utils::faultPoint("build_probe");
        bps.emplace_back(new tasks::BuildProbe(innerWindow, outerViews.back().get(), ctx, plan, config.outputCapacity));
        bps.back()->execute();
      }
      result.localItems = lp->workItems();
    } else {
      TASK_QUEUE.push(lp.get());
      // Both tasks are owned here (lp is re-created if its sampled layout overflows).
      while (!TASK_QUEUE.empty()) {
        tasks::Task *t = TASK_QUEUE.front();
        TASK_QUEUE.pop();
        if (t->getType() == TASK_BUILD_PROBE) {
          utils::faultPoint("build_probe");
          t->execute();
          continue;
        }
        t->execute();
        if (t->getType() == TASK_PARTITION) {
          if (dev) HIP_CHECK(hipEventRecord(ev[3], ctx->stream()));
          result.localItems = lp->workItems();
          bps.emplace_back(new tasks::BuildProbe(innerWindow, outerWindow, ctx, plan, config.outputCapacity));
          TASK_QUEUE.push(bps.back().get());
        }
      }
    }
    trace.reset();  // roctx ranges nest: pop before the next push
    if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
    ctx->synchronize();
    result.sampledLocal = lp->sampled();
    if (lp->sampled() && lp->overflowed()) {
      // A sampled slot overflowed (skew the sample missed): the build/probe ran
      // on incomplete partitions.  Redo the local pass exactly over the whole
      // windows, then the build/probe; later joins stay exact.
      localOverflowed = true;
      ++result.localFallbacks;
      result.sampledLocal = false;
      bps.clear();
      outerViews.clear();
      lp.reset(new tasks::LocalPartitioning(innerWindow, outerWindow, ctx, plan, true));
      lp->execute();
      result.localItems = lp->workItems();
      bps.emplace_back(new tasks::BuildProbe(innerWindow, outerWindow, ctx, plan, config.outputCapacity));
      bps.back()->execute();
      if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
      ctx->synchronize();
    }
    for (auto &bp : bps)
      while (bp->collect()) {  // rare: item list or output buffer overflowed -> exact re-run
        ++result.reruns;
        bp->execute();
        if (dev) HIP_CHECK(hipEventRecord(ev[4], ctx->stream()));
        ctx->synchronize();
      }
  }  // !bitmapDone
  Measurements::stopLocalProcessing();
  const uint64_t t4 = nowUs();

  result.localMatches = bitmapMatches;
  result.buildProbeItems = bitmapDone ? (1ull << plan.networkBits) : 0;
  result.bitmapJoin = bitmapDone;
  for (auto &bp : bps) {
    result.localMatches += bp->getMatches();
    result.buildProbeItems += bp->getWorkItems();
  }
  // Materializing joins have exactly one build/probe (never pipelined).
  result.outputPairs =
      plan.materialize && !bps.empty() ? std::min<uint64_t>(bps.front()->getOutputCount(), UINT64_MAX) : 0;
  result.outputOverflow = !bps.empty() && bps.front()->outputOverflowed();
  output = bps.empty() ? nullptr : bps.front()->getOutput();
  bps.clear();
  outerViews.clear();
  result.wireBytes = innerWindow->wireBytesSent() + outerWindow->wireBytesSent();
  result.innerReceived = innerWindow->computeLocalWindowSize();
  result.outerReceived = outerWindow->computeLocalWindowSize();
  result.sampledNetwork = sampled && !sampledOverflowed;
  Measurements::storeLocalPartitioningDetails(result.innerReceived + result.outerReceived, result.localItems);
  Measurements::storeBuildProbeDetails(result.innerReceived, result.outerReceived, result.buildProbeItems);
  Measurements::storeResultTuples(result.localMatches);
  Measurements::stopJoin();

  result.joinMs = (t4 - t0) / 1000.0;
  result.histogramMs = (t1 - t0) / 1000.0;
  result.windowMs = (t2 - t1) / 1000.0;
  result.networkMs = (t3 - t2) / 1000.0;
  result.localMs = (t4 - t3) / 1000.0;
  if (dev) {
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    result.devHistogramMs = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev[1], ev[2]));
    result.devNetworkMs = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev[2], ev[3]));
    result.devLocalPartitionMs = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev[3], ev[4]));
    result.devBuildProbeMs = ms;
    Measurements::storeDevicePhase("DHIST", result.devHistogramMs);
    Measurements::storeDevicePhase("DNET", result.devNetworkMs);
    Measurements::storeDevicePhase("DLOCPART", result.devLocalPartitionMs);
    Measurements::storeDevicePhase("DBP", result.devBuildProbeMs);
  }

  uint64_t g = result.localMatches;
  ctx->comm()->allReduceSumHost(&g, 1);
  result.globalMatches = g;
  result.teardownMs = (nowUs() - t4) / 1000.0;
  RESULT_COUNTER = result.localMatches;
  return result;
}

}  // namespace operators
}  // namespace hpcjoin
