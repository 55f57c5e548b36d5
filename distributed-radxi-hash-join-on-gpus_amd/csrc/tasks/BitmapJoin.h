// Count-only single-level bitmap join (JoinPlan::bitmapJoin).
//
// The reference's default plan joins every network partition directly, with
// no second radix pass (core/Configuration.h:28, operators/HashJoin.cpp:138-166,
// tasks/BuildProbe.cpp:47-121), and a counting join only ever compares key
// bits and reports a count (tasks/BuildProbe.cpp:101-102,115).  For unique
// inner keys whose range fits 2^20 bits per network partition that join is a
// bitmap: this task runs it end to end as one stream of kernels with a single
// synchronisation at the end.
//
// Per relation side (local to the rank, no exchange):
//   sampled LDS histogram (1 tile in sampleStride) -> per-(XCD group, digit)
//   claim slices laid out ON THE DEVICE (kernels::netSampledLayout) ->
//   bounded claim scatter writing u32 key fragments (kernels::netScatterFrag,
//   4 bytes per tuple: the count-only projection).
// Then
//   N == 1  kernels::bitmapJoin: one workgroup per partition builds a 128 KiB
//           LDS bitmap from the inner fragments and probes the outer ones.
//   N > 1   replicated plan: kernels::bitmapBuild writes every partition's
//           bitmap of this rank's inner keys to HBM; ONE RCCL all-reduce (sum)
//           over the exchange stream combines them (unique keys set disjoint
//           bits, so the sum is the OR) while the outer side is partitioned on
//           the compute stream; kernels::bitmapProbe loads each combined
//           bitmap into LDS and probes this rank's own outer tuples.  No tuple
//           crosses a link: the links carry 2 (N-1)/N * 2^keyBits / 8 bytes
//           per rank instead of (N-1)/N of every tuple (HashJoin's cost model
//           picks the cheaper).  A key held by two ranks turns into a carry of
//           the sum; every rank counts the set bits of the whole combined
//           bitmap while probing, and popcount != |R| (global) flags it.
// Outcomes (agreed by all ranks through the result all-reduce):
//   overflow  a sampled slice overflowed: rerun with exact histograms
//   dup       a repeated inner key (or a fragment out of range): the caller
//             redoes the join on the two-level pass
// The host path (CPU, tests) runs the same plan with exact partitioning.
//
// Capacity spill (N = 1, JoinPlan::groupBudget): when both sides' fragment
// windows exceed the memory budget, the sampled totals are read back once and
// the network partitions cut into groups whose windows fit it; each group is
// one pass: both relations are read and only the group's digits are scattered
// (kernels::netScatterFragRange), then the group's bitmaps join.  Reference:
// the large-data drivers process the input per iteration with one histogram
// for all of them (operators/gpu/kernels.cu:563-857, data/data.hpp:67-83);
// here an iteration is a range of network partitions, so no pass buffer or
// compaction pass exists and equal keys always meet in the same pass.
#pragma once

#include <cstdint>

#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../kernels/kernels.h"

namespace hpcjoin {
namespace tasks {

class BitmapJoin {
 public:
  struct Outcome {
    uint64_t localMatches = 0;
    uint64_t globalMatches = 0;
    uint64_t popcount = 0;     // replicated: set bits of the combined bitmaps
    bool dup = false;          // some rank saw a repeated/out-of-range inner fragment, or a cross-rank carry
    bool overflow = false;     // some rank's sampled slice overflowed
    uint64_t linkBytes = 0;    // this rank's share of the all-reduce traffic (ring estimate)
    double devSampleMs = 0, devScatterMs = 0, devJoinMs = 0;  // hipEvents (device engine)
    uint64_t enqueueUs = 0;    // host clock when the last kernel of the join was enqueued
    double hostWaitMs = 0;     // host wait from there to the result (mailbox spin + stream sync)
    uint32_t groupPasses = 0;  // partition-group passes (JoinPlan::groupBudget), 0 = one pass
  };

  // ev: 5 timing events of the caller (ev[0] already recorded at join start).
  BitmapJoin(data::Relation *innerRelation, data::Relation *outerRelation, core::ExecContext *ctx,
             const core::JoinPlan &plan, uint32_t maxBlocks, uint32_t sampleStride, hipEvent_t *ev);
  // exact: full histograms (no overflow possible).  Collective for N > 1.
  Outcome run(bool exact);

 private:
  struct Side {
    data::Relation *relation;
    kernels::PartitionGeometry geom;
    uint32_t *frags = nullptr;
    kernels::BitmapSlices slices;
    uint64_t cap = 0;  // fragment capacity of all slices
  };
  // narrowOk: 4-byte claim cursors are allowed (both sides of a fused bitmap
  // join must use the same cursor width; sideNarrow() says what one side needs).
  struct SidePlan {
    kernels::PartitionGeometry geom;
    uint32_t stride = 1;
    kernels::SampleScale sc{};
    uint64_t cap = 0;
  };
  const SidePlan &sidePlan(uint64_t n, bool exact, uint32_t stride) const;
  void layoutSides(Side *sides, uint32_t count, bool exact, bool narrowOk);
  void scatterSide(Side &s);
  bool sideNarrow(data::Relation *r, bool exact) const;
  Outcome runDevice(bool exact);
  // Capacity spill (JoinPlan::groupBudget, N = 1): the network partitions in
  // groups whose fragment windows fit the budget, one pass per group.
  Outcome runDeviceGroups(bool exact);
  Outcome runHost();
  void agree(Outcome &o, uint64_t localFlags);

  data::Relation *inner, *outer;
  core::ExecContext *ctx;
  const core::JoinPlan &plan;
  uint32_t maxBlocks, sampleStride;
  hipEvent_t *ev;
  bool useControl = false;   // N = 1 device engine: control-block scratch + mailbox result
  uint64_t mailboxSeq = 0;
};

}  // namespace tasks
}  // namespace hpcjoin
