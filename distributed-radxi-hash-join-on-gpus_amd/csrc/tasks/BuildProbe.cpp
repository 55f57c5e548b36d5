#include "BuildProbe.h"

#include <algorithm>
#include <cstring>

#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../operators/HashJoin.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

BuildProbe::BuildProbe(uint64_t innerPartitionSize, data::CompressedTuple *innerPartition,
                       uint64_t outerPartitionSize, data::CompressedTuple *outerPartition)
    : innerPartitionSize(innerPartitionSize), innerPartition(innerPartition), outerPartitionSize(outerPartitionSize),
      outerPartition(outerPartition), reference(true) {
  refBounds = {0, innerPartitionSize, 0, outerPartitionSize};
  args.R = innerPartition;
  args.S = outerPartition;
  args.partR = &refBounds[0];
  args.partS = &refBounds[2];
  args.P = 1;
  args.keyShift = core::Configuration::NETWORK_PARTITIONING_FANOUT + core::Configuration::PAYLOAD_BITS;  // 32
  args.fragShift = args.keyShift + core::Configuration::LOCAL_PARTITIONING_FANOUT;                      // 37
}

BuildProbe::BuildProbe(data::Window *innerWindow, data::Window *outerWindow, core::ExecContext *ctx,
                       const core::JoinPlan &plan, uint64_t outputCapacity)
    : innerPartitionSize(innerWindow->computeLocalWindowSize()), innerPartition(nullptr),
      outerPartitionSize(outerWindow->computeLocalWindowSize()), outerPartition(nullptr), ctx(ctx), plan(plan),
      outputCapacity(outputCapacity) {
  windows[0] = innerWindow;
  windows[1] = outerWindow;
}

BuildProbe::~BuildProbe() {}

void BuildProbe::configure() {
  data::Window *wi = windows[0], *wo = windows[1];
  const uint32_t owned = (uint32_t)wi->getPlan().owned.size();
  args = kernels::BPArgs();
  args.R = wi->getPartitionedData();
  args.S = wo->getPartitionedData();
  args.partR = wi->getPartitionBegin();
  args.partS = wo->getPartitionBegin();
  args.partREnd = wi->getPartitionEnd();
  args.partSEnd = wo->getPartitionEnd();
  args.P = owned << wi->getLocalBits();
  args.rChunk = plan.rChunk;
  args.sChunk = plan.sChunk;
  args.fragShift = plan.wide ? 64 : plan.keyShift + wi->getLocalBits();
  args.keyShift = plan.keyShift;
  if (!plan.wide && !plan.keyOnly && plan.directCount) {  // fragments are < 2^fragBits (direct-addressed counting when small)
    const uint32_t passBits = plan.networkBits + wi->getLocalBits();
    args.fragBits = plan.keyBits > passBits ? std::min<uint32_t>(32, plan.keyBits - passBits) : 1;
  }
  args.wide = plan.wide;
  args.keyOnly = plan.keyOnly;
  args.materialize = plan.materialize;
  args.keyCount = plan.variants.keyCount >= 8 && countedAll ? 9 : plan.variants.keyCount;
  if (plan.keyOnly) {
    const uint32_t passBits = plan.networkBits + wi->getLocalBits();
    args.keyFragBits = plan.keyBits > passBits ? plan.keyBits - passBits : 1;
  }
  args.rowsLds = plan.variants.rowsLds;
  if (wi->getPartitionedHi()) {
    JOIN_ASSERT(wo->getPartitionedHi(), "BuildProbe", "one side split, the other not");
    args.split = 1;
    args.Rhi = wi->getPartitionedHi();
    args.Shi = wo->getPartitionedHi();
  }
  // Direct-addressed counting: duplicate-heavy inner partitions (Zipf) need
  // no inner chunking into rChunk-sized tables -- each work item counts up to
  // 2^18 inner tuples into its count table and probes its outer chunk, so a
  // hot partition costs (inner / 2^18) passes over its outer side instead of
  // (inner / rChunk).
  if (ctx && ctx->onDevice() && kernels::bpDirectSplit(args))
    args.rChunk = std::max<uint32_t>(args.rChunk, kernels::BP_DIRECT_R_CHUNK);
  if (capacity == 0)
    capacity = (uint32_t)std::min<uint64_t>(
        0xFFFFFFF0ull, 2ull * args.P + outerPartitionSize / args.sChunk + innerPartitionSize / args.rChunk + 1024);
}

void BuildProbe::execute() {
  if (reference) {
    args.result = nullptr;
    matches = host::buildProbe(args);
    operators::HashJoin::RESULT_COUNTER += matches;
    return;
  }
  configure();
  const bool dev = ctx->onDevice();
  memory::Arena &ws = ctx->workspace();
  fused = plan.materialize && sink && dev && args.split;
  if (fused) {
    outputCapacity = sink->capacity;
    outPairs = nullptr;
    args.outRows = reinterpret_cast<ulonglong2 *>(sink->out);
    args.rowsA = reinterpret_cast<const ulonglong2 *>(sink->rowsA);
    args.rowsB = reinterpret_cast<const ulonglong2 *>(sink->rowsB);
    args.offA = sink->offA;
    args.offB = sink->offB;
    args.outCapacity = outputCapacity;
  } else if (plan.materialize && hostOut) {
    outPairs = hostOut;  // pinned host memory, written by the place kernel over the host link
    args.outPairs = outPairs;
    args.outCapacity = outputCapacity;
  } else if (plan.materialize) {
    if (outputCapacity == 0) outputCapacity = outerPartitionSize + 1024;
    outPairs = static_cast<ulonglong2 *>(ws.get(outputCapacity * sizeof(ulonglong2)));
    args.outPairs = outPairs;
    args.outCapacity = outputCapacity;
  }
  performance::Timeline &tl = ctx->timeline();
  // The build and the probe of one LDS table run in one kernel (one work
  // item = build + probe): its time is charged to BPBUILD / BPPROBE in
  // proportion to the tuples each reads.
  const double wb = (double)innerPartitionSize, wp = (double)outerPartitionSize;
  performance::Measurements::add("BPBUILDELEM", wb, "tuples");
  performance::Measurements::add("BPPROBEELEM", wp, "tuples");
  if (!dev) {
    hostCursor = 0;
    args.outCursor = reinterpret_cast<unsigned long long *>(&hostCursor);
    tl.begin("BPTASKTIME");
    tl.beginSplit("BPKERNEL", "BPBUILD", wb, "BPPROBE", wp);
    matches = host::buildProbe(args);
    tl.end("BPKERNEL");
    tl.end("BPTASKTIME");
    outputCount = hostCursor;
    workItems = args.P;
    return;
  }
  tl.begin("BPTASKTIME", ctx->stream());
  const uint64_t tAlloc = performance::nowUs();
  counters = ws.getArray<unsigned long long>(4);
  ctx->zero(counters, 4 * sizeof(unsigned long long));
  args.result = counters;
  args.outCursor = counters + 1;
  uint32_t *nItems = reinterpret_cast<uint32_t *>(counters + 2);
  uint32_t *counts = ws.getArray<uint32_t>(std::max<uint32_t>(args.P, 1));
  uint32_t *offsets = ws.getArray<uint32_t>(std::max<uint32_t>(args.P, 1));
  void *scanWs = ws.get(kernels::scanWorkspaceBytes(args.P));
  kernels::BPItem *items = ws.getArray<kernels::BPItem>(capacity);
  performance::Measurements::add("BPMEMALLOC", (double)(performance::nowUs() - tAlloc), "us");
  performance::Measurements::add("BPMEMSIZE",
                                 (double)(2ull * std::max<uint32_t>(args.P, 1) * 4 + kernels::scanWorkspaceBytes(args.P) +
                                          (uint64_t)capacity * sizeof(kernels::BPItem) + kernels::bpLdsBytes(args)),
                                 "bytes");
  // Key-only counting on the quotient table: partitions of repeated keys go
  // to the counted-table kernel instead of the span work queue.  Fragments
  // of 45-48 bits (inputs below ~500M tuples) do not fit the quotient table:
  // every partition is counted there.
  const bool keySpans = args.keyOnly;
  const bool counted = keySpans && args.keyCount >= 8 && kernels::bpKeyCountedFits(args);
  const bool quotient = counted && kernels::bpKeyQuotientFits(args);
  // keyCount 9 (repeated inner keys): partitions of more than one inner chunk
  // are first compacted to (distinct word, count) (kernels::bpKeyDedup), once
  // per join -- not with per-chunk rebuilds of a pipelined outer side, which
  // re-read the inner words.
  // (Leaving partitions of at most one inner chunk on the quotient table
  // instead -- heavy ones compacted and counted -- was exact but took 119 ms
  // of build/probe for Zipf-both sparse 1e9 x 4e9 instead of 13.8: keys with
  // hundreds of copies in light partitions walk the overflow table.)
  const bool dedup = counted && args.keyCount == 9 && args.split && !plan.pipelineOuter;
  if (counted) {
    args.heavySpans = ws.getArray<kernels::BPSpan>(capacity);
    args.heavyCapacity = capacity;
    // keyCount 9 (repeated keys seen): every partition on counted tables.
    args.heavyMin = (args.keyCount == 9 || !quotient) ? 0 : args.rChunk;
    args.heavyCount = nItems + 1;  // high half of counters[2]: read back with the rest
  }
  if (dedup) {
    if (!dedupCounts) {  // kept for the join: a re-run only re-emits the compacted spans
      dedupCounts = ws.getArray<uint32_t>(std::max<uint64_t>(windows[0]->getPartitionedCapacity(), 1));
      dedupLen = ws.getArray<uint64_t>((uint64_t)std::max<uint32_t>(args.P, 1) * kernels::BP_DEDUP_SEGS);
    }
    args.dedupParts = ws.getArray<uint32_t>(std::max<uint32_t>(args.P, 1));
    args.dedupCount = reinterpret_cast<uint32_t *>(counters + 1);  // the pair cursor is unused by a count
    args.dedupBig = ws.getArray<uint32_t>(std::max<uint32_t>(args.P, 1));
    args.dedupBigCount = reinterpret_cast<uint32_t *>(counters + 1) + 1;  // (zeroed with the counters)
    args.dedupCounts = dedupCounts;
    args.dedupLen = dedupLen;
  }
  kernels::bpPlanCounts(args, counts, ctx->stream());
  kernels::scanExclusiveU32(counts, offsets, args.P, nItems, scanWs, ctx->stream());
  if (keySpans) {
    // Key-only counting: resolved spans through a device work queue.
    auto *spans = ws.getArray<kernels::BPSpan>(capacity);
    uint32_t *queue = ws.getArray<uint32_t>(1);
    kernels::bpEmitSpans(args, counts, offsets, spans, capacity, ctx->stream());
    args.sideOverflow = counters + 3;  // quotient table flags (kernels.h, BPArgs::sideOverflow)
    tl.beginSplit("BPKERNEL", "BPBUILD", wb, "BPPROBE", wp, ctx->stream());
    if (dedup) {
      kernels::bpKeyDedup(args, args.P, deduped, ctx->stream());
      if (!deduped) kernels::bpKeyDedupMerge(args, args.P, ctx->stream());
      deduped = true;
    }
    if (!counted || args.heavyMin != 0)  // otherwise every span is on the heavy list
      kernels::buildProbeKeySpans(args, spans, nItems, capacity, queue, ctx->stream());
    if (counted) kernels::bpKeyCountedSpans(args, queue, ctx->stream());  // (the queue word is re-zeroed)
    hipEvent_t done = tl.mark(ctx->stream());
    tl.endAt("BPKERNEL", done);
    tl.endAt("BPTASKTIME", done);
    readBackCounters();
    return;
  }
  kernels::bpEmit(args, counts, offsets, items, capacity, ctx->stream());
  if (!plan.materialize) {
    tl.beginSplit("BPKERNEL", "BPBUILD", wb, "BPPROBE", wp, ctx->stream());
    kernels::buildProbe(args, items, nItems, capacity, ctx->stream());
    hipEvent_t done = tl.mark(ctx->stream());  // one event ends both spans
    tl.endAt("BPKERNEL", done);
    tl.endAt("BPTASKTIME", done);
    readBackCounters();
    return;
  }
  // Two-pass exact materialization: count per item -> 64-bit offsets -> place.
  // (A single pass with one device atomic per wave and batch on a shared
  // output cursor measured 65 ms instead of 29 for the SF100 row output: 4.7M
  // atomics on one address serialize.)
  uint32_t *itemCounts = ws.getArray<uint32_t>(capacity);
  unsigned long long *itemOffsets = ws.getArray<unsigned long long>(capacity);
  void *scanWs64 = ws.get(kernels::scanWorkspaceBytes(capacity));
  ctx->zero(itemCounts, (size_t)capacity * sizeof(uint32_t));
  kernels::BPArgs countArgs = args;
  countArgs.materialize = false;
  countArgs.itemCounts = itemCounts;
  tl.beginSplit("BPKERNEL", "BPBUILD", wb, "BPPROBE", wp, ctx->stream());
  kernels::buildProbe(countArgs, items, nItems, capacity, ctx->stream());  // -> counters[0] = matches
  kernels::scanExclusiveU32to64(itemCounts, itemOffsets, capacity, args.outCursor, scanWs64, ctx->stream());
  args.itemOffsets = itemOffsets;
  args.result = counters + 3;  // the count pass already counted
  kernels::buildProbe(args, items, nItems, capacity, ctx->stream());
  hipEvent_t done = tl.mark(ctx->stream());
  tl.endAt("BPKERNEL", done);
  tl.endAt("BPTASKTIME", done);
  readBackCounters();
}

// Enqueued behind the build/probe, so the join's final synchronisation also
// completes the read-back (no separate blocking copy afterwards).
void BuildProbe::readBackCounters() {
  countersBack = ctx->staging().getArray<unsigned long long>(4);
  ctx->readBack(countersBack, counters, 4 * sizeof(unsigned long long));
}

bool BuildProbe::collect() {
  if (reference || !ctx->onDevice()) {
    overflowOut = plan.materialize && outputCount > outputCapacity;
    return false;
  }
  unsigned long long h[4];
  HIP_CHECK(hipStreamSynchronize(ctx->stream()));  // no-op after the caller's sync
  std::memcpy(h, countersBack, sizeof(h));
  matches = h[0];
  outputCount = h[1];
  uint32_t items, heavy;
  std::memcpy(&items, &h[2], sizeof(items));
  std::memcpy(&heavy, reinterpret_cast<const char *>(&h[2]) + sizeof(items), sizeof(heavy));
  workItems = items + heavy;
  bool again = false;
  if (h[3] & 2) duplicateChains = true;  // exact count; later joins use counted tables throughout
  if (args.sideOverflow && (h[3] & 8)) {  // a quotient span's overflow table filled: count void, counted tables
    countedAll = duplicateChains = true;
    again = true;
  }
  if (items > capacity || heavy > capacity) {
    capacity = std::max(items, heavy);
    again = true;
  }
  if (plan.materialize && outputCount > outputCapacity) {
    if (fused || hostOut) {
      overflowOut = true;  // the buffer is the caller's: it re-runs with a larger one
    } else {
      outputCapacity = outputCount;
      again = true;
    }
  }
  return again;
}

}  // namespace tasks
}  // namespace hpcjoin
