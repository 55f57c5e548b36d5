// The distributed radix hash join operator.  Same entry points as
// /root/reference/operators/HashJoin.h:19-45 (constructor(numberOfNodes,
// nodeId, inner, outer), join(), RESULT_COUNTER, TASK_QUEUE), plus the
// MI355X-native constructor that takes an execution context and a runtime
// JoinConfig, and run() which returns a JoinResult.
//
// Phase structure (reference HashJoin.cpp:45-220):
//   histogram   LocalHistogram kernels -> fused all-gather -> AssignmentMap -> OffsetMap
//   windows     exact-size receive buffers from the engine arena (no hipMalloc in steady state)
//   network     cursor + LDS scatter kernels per chunk, RCCL all-to-allv per chunk on the exchange stream
//   local       TASK_QUEUE: LocalPartitioning (second radix pass), BuildProbe (LDS hash join)
//   result      one sync, counters read back, all-reduce of the match count
#pragma once

#include <cstdint>
#include <memory>
#include <queue>
#include <vector>

#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../tasks/Task.h"

namespace hpcjoin {
namespace data {
class Window;
}
namespace operators {
struct JoinRun;

struct JoinResult {
  uint64_t localMatches = 0;
  uint64_t globalMatches = 0;
  uint64_t outputPairs = 0;        // materialize: pairs written on this rank
  bool outputOverflow = false;
  bool rowsFused = false;          // materialize: whole rows went to the RowSink (no pair array)
  uint32_t reruns = 0;             // build/probe re-launches after an item/output overflow
  double joinMs = 0;               // host wall: histogram start -> local result available
  double histogramMs = 0, windowMs = 0, networkMs = 0, localMs = 0;  // host phases
  double devHistogramMs = 0, devNetworkMs = 0, devLocalPartitionMs = 0, devBuildProbeMs = 0;  // hipEvents
  double setupMs = 0, teardownMs = 0;  // outside the join span: scratch reset / result reduction
  // Host side of the join span: enqueue (join start -> last kernel enqueued)
  // and the wait for the result after it; devSpanMs = first -> last event.
  // joinMs - devSpanMs is what the host added around the device work.
  double enqueueMs = 0, hostWaitMs = 0, devSpanMs = 0;
  uint64_t exchangeChecked = 0;    // (source, chunk, partition) runs whose content was verified (verifyExchange)
  double verifyMs = 0;             // host wall of that verification (excluded from joinMs / networkMs; the
                                   // device spans devNetworkMs / devSpanMs still contain its kernels)
  uint32_t passes = 1;             // capacity spill: key-hash passes the join ran in (JoinConfig::passes)
  double compactMs = 0;            // capacity spill: host wall of the per-pass compaction (in joinMs)
  // Capacity spill of the bitmap plan: partition-group passes of the last
  // join (each reads both relations once and writes only its digit range).
  uint32_t groupPasses = 0;
  uint64_t innerReceived = 0, outerReceived = 0;
  uint64_t wireBytes = 0;          // bytes this rank sent to peers (after the wire codec)
  uint64_t localItems = 0, buildProbeItems = 0;
  uint64_t innerLocal = 0, outerLocal = 0;
  bool sampledNetwork = false;     // network pass sized from a sampled histogram (N == 1)
  uint32_t networkFallbacks = 0;   // sampled pass overflowed -> exact re-run inside this join
  uint32_t roundWindows = 0;       // network windows (N > 1: send buffers) with round-interleaved slices (kernels::RoundMap)
  bool sampledLocal = false;       // local pass sized from a sampled histogram
  bool bitmapJoin = false;         // single-level bitmap join counted the matches (no local pass)
  uint32_t localFallbacks = 0;     // sampled local pass overflowed -> exact re-run
  uint32_t splitPartitions = 0;    // hot network partitions joined by several ranks (AssignmentMap)
  bool directScatter = false;      // one-sided windows: the scatter kernel wrote into the owners' windows
                                   // (false with ExchangeMode::OneSided = staged send buffer + peer copies,
                                   // e.g. when a split hot partition adds replicas)
};

// Achievable one-way bandwidth of one xGMI peer link (MI355X: 7 links of
// ~153 GB/s bidirectional, ~77 GB/s each way; ~64 GB/s is what a grouped
// RCCL send/recv reaches per peer).  Only the planner's cost model uses it.
constexpr double kDefaultLinkGBpsPerPeer = 64.0;

class HashJoin {
 public:
  // Reference constructor: world communicator, default JoinConfig, relation location.
  HashJoin(uint32_t numberOfNodes, uint32_t nodeId, data::Relation *innerRelation, data::Relation *outerRelation);
  HashJoin(data::Relation *innerRelation, data::Relation *outerRelation, core::ExecContext *ctx,
           const core::JoinConfig &config);
  ~HashJoin();

  void join();        // reference API: runs, updates RESULT_COUNTER (local matches)
  // One full join.  If any phase throws on this rank (HIP/RCCL error,
  // failed invariant, injected fault, watchdog timeout), the pending tasks are
  // dropped and the communicator is aborted so peers fail instead of hanging.
  JoinResult run();
  const JoinResult &lastResult() const { return result; }
  const core::JoinPlan &getPlan() const { return plan; }
  const core::JoinConfig &getConfig() const { return config; }
  core::ExecContext *context() const { return ctx; }
  // Materialized (rid_inner, rid_outer) pairs of the last run(), in the engine's workspace: valid
  // until the workspace is rewound or freed (the next join on the context,
  // a new HashJoin planned on it, trim_workspace).  outputValid() says whether
  // it still is.
  const ulonglong2 *getOutput() const { return output; }
  bool outputValid() const;
  // Fused materialization: while a sink is set, a device join at N = 1 over
  // the split layout writes whole output rows (LateMaterialization's layout)
  // from its materialize pass instead of pairs.  canFuseRows() says whether
  // this plan does; the caller keeps the sink's buffers alive over run().
  bool canFuseRows() const;
  // Throws unless the sink's payload columns cover this rank's rids of both
  // relations (the fused kernel indexes rows by rid - offset on the device).
  void setRowSink(const kernels::RowSink &s);
  // Smallest / largest rid of this rank's slice of relation 0 (inner) or 1
  // (outer); lo > hi for an empty slice.
  uint64_t ridMin(int which) const { return ridLo[which]; }
  uint64_t ridMax(int which) const { return ridHi[which]; }
  void clearRowSink() { hasSink = false; }

 protected:
  uint32_t numberOfNodes;
  uint32_t nodeId;
  data::Relation *innerRelation;
  data::Relation *outerRelation;

 public:
  // thread_local: in-process ranks (InProcessCommunicator) each run on their own thread.
  static thread_local uint64_t RESULT_COUNTER;
  static thread_local std::queue<tasks::Task *> TASK_QUEUE;

 private:
  void makeJoinPlan();
  void planPasses();
  JoinResult runPasses();
  void planBitmap();
  void recordTimes(const JoinRun &run, uint64_t t4);
  bool lowKeyBitsSkewed();
 public:
  // Upper estimate of the workspace bytes one run() of this plan carves from
  // the arena (windows, send/wire buffers, local pass output, work lists).
  uint64_t workspaceEstimate() const;
  std::vector<uint64_t> workspaceParts() const;  // the estimate as one chunk per big buffer
  // Bytes the constructor added to the arena (0 if it already held the estimate).
  uint64_t reservedBytes() const { return reserved; }
  uint32_t spillPasses() const { return passes; }
  // Construction cost: planning (key / rid bounds, repeated-key and low-bit
  // scans when the generator did not record them, the all-gather) and the
  // workspace reservation (allocation + first touch).  Host wall time, ms.
  double planMilliseconds() const { return planMs; }
  double reserveMilliseconds() const { return reserveMs; }

 private:
  uint64_t reserved = 0;
  double planMs = 0, reserveMs = 0;
  int innerKeyRepeats();
  void planWireCodec(const std::vector<uint64_t> &rankStats, size_t stride, uint32_t chunks);

 public:
  // The wire codec's cost model (planWireCodec): true when packing w-bit
  // tuples saves more link time per tuple than its extra HBM passes cost.
  static bool codecPays(uint32_t w, uint32_t nodes, double perPeerGBps, double extraPsPerTuple);

 private:
  JoinResult runImpl();
  core::ExecContext *ctx;
  std::unique_ptr<core::ExecContext> ownedCtx;
  core::JoinConfig config;
  core::JoinPlan plan;
  JoinResult result;
  bool sampledOverflowed = false;  // sticky: exact histograms after a sampled pass overflowed
  bool localOverflowed = false;    // sticky: exact local pass after a sampled one overflowed
  core::JoinPlan basePlan;         // two-level plan (what a bitmap plan falls back to)
  bool bitmapExact = false;        // bitmap plan: exact histograms (small inputs, or after an overflow)
  const ulonglong2 *output = nullptr;
  // Capacity spill (planPasses / runPasses): pass count, this rank's and the
  // global tuple counts per pass, the pass buffers (one inner and one outer
  // pass at a time) and the plan's global key / rid bounds.
  uint32_t passes = 1;
  std::vector<uint64_t> passCount[2], passGlobal[2];
  data::Tuple *passBuf[2] = {nullptr, nullptr};
  uint64_t passCap[2] = {0, 0};  // tuples each pass buffer holds
  uint64_t planMaxKey = 0, planMaxRid = 0;
 public:
  // The capacity planner's inputs and outcome (bytes): single-pass workspace
  // estimate, memory available to one pass (free HBM x 0.85, capped by
  // workspaceBudget), the pass buffers, and the largest pass join's estimate
  // and reservation (filled in by runPasses).
  struct SpillInfo {
    uint64_t estimate = 0, available = 0, passBuffers = 0, passEstimate = 0, passReserved = 0, passPeak = 0;
    uint64_t groupBudget = 0;  // bitmap plan: fragment-window bytes of one partition-group pass (0 = none)
  } spill;
 private:
  uint64_t outputEpoch = 0;  // workspace epoch when `output` was written
  kernels::RowSink sink;
  bool hasSink = false;
  uint64_t ridLo[2] = {~0ull, ~0ull}, ridHi[2] = {0, 0};
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};

}  // namespace operators
}  // namespace hpcjoin
