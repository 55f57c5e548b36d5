// Multi-rank network pass without the exact histogram read (the N > 1 form
// of SampledNetworkPartitioning).
//
// The exact exchange reads both relations once just to count them
// (histograms/LocalHistogram, 16 B per tuple) before the scatter can place a
// single tuple -- about a third of the network pass's HBM bytes.  Here:
//   sample    every workgroup histograms 1 tile in `stride` of its own range
//             (kernels::netHistogram), folded into per (exchange chunk, XCD
//             claim group, digit) counts (kernels::netChunkGroupTotals); one
//             copy to the host.
//   assign    per (chunk, digit) estimates of both relations go through the
//             usual fused all-gather and AssignmentMap (LPT, hot-partition
//             split).  The assignment is a pure function of the gathered
//             table, so every rank derives the same one.
//   scatter   the bounded claim-mode scatter fills per (chunk, group, digit)
//             slices sized estimate + margin (6 sigma of the sampling error +
//             2%); each chunk's final claim cursors come back to the host.
//   exchange  one all-gather per relation of every rank's exact slice fills
//             (C x G x F u32 + an overflow flag) gives every rank the exact
//             receive layout; the wire codec's pack kernel gathers the filled
//             runs of each peer (no slice gap crosses a link), one all-to-allv
//             moves them and the unpack writes them at exact window offsets
//             (data::Window::exchangeSegmented).  Own runs are copied.
// A slice that overflowed on any rank (the flag rides in the gather, so every
// rank sees it) -- or a window that the exact fills would overrun -- ends the
// pass before that relation is exchanged: the caller re-runs the join with exact
// histograms (operators::ExactExchange) and stays on them.
//
// Needs a device engine and the wire codec on both relations (packing is what
// removes the slice gaps); HashJoin only plans it then.
// Reference: histograms/LocalHistogram.cpp:35-53 (the pre-read removed here)
// and tasks/NetworkPartitioning.cpp:74-222 (the scatter + MPI_Put exchange).
#pragma once

#include <memory>
#include <vector>

#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../data/Window.h"
#include "../histograms/ExchangePlan.h"
#include "../kernels/kernels.h"
#include "HistogramComputation.h"

namespace hpcjoin {
namespace tasks {

class SampledShuffle {
 public:
  // hc: the join's histogram state (local-histogram geometry per relation,
  // global tables, assignment), owned by the caller and outliving this pass.
  SampledShuffle(uint32_t numberOfNodes, uint32_t nodeId, HistogramComputation *hc, core::ExecContext *ctx,
                 const core::JoinPlan &plan, uint32_t sampleStride);
  ~SampledShuffle();
  SampledShuffle(const SampledShuffle &) = delete;
  SampledShuffle &operator=(const SampledShuffle &) = delete;

  // Both sampled histograms (one wait), the estimates' all-gather and the
  // assignment (collective).
  void sampleAndAssign();
  // Slices, cursor uploads and the (capacity-sized) window of side k.
  void layoutSide(int k);
  // Enqueues side k's bounded scatter, chunk by chunk, with the read-back of
  // every chunk's final claim cursors.
  void scatterSide(int k);
  // Waits for side k's scatter, all-gathers every rank's fills (one
  // collective), then enqueues the chunks' exchanges back to back.  false:
  // some rank overflowed (nothing of this side was exchanged; every rank
  // returns false at the same point).
  bool exchangeSide(int k);

  data::Window *window(int k) { return sides[k].window.get(); }
  uint32_t sampleStride(int k) const { return sides[k].stride; }
  uint64_t sliceCapacity(int k) const { return sides[k].capTotal; }

 private:
  struct Side {
    data::Relation *relation = nullptr;
    histograms::LocalHistogram *local = nullptr;  // geometry, chunks, blocks per chunk (owned by hc)
    uint32_t chunks = 1, stride = 1;
    uint64_t *sampled = nullptr;         // [C][G][F] sampled counts (pinned staging)
    std::vector<uint64_t> estimate;      // [C][F] scaled estimates (the assignment's input)
    std::vector<uint64_t> start, cap;    // [C][G][F] slice start / capacity (tuples)
    std::vector<uint32_t> cur32, end32;  // asynchronous upload sources (alive until the join ends)
    std::vector<uint64_t> end64;
    void *gcur = nullptr, *gend = nullptr;
    bool narrow = true;
    uint64_t capTotal = 0;               // send buffer slots
    kernels::RoundMap rm;                // round-interleaved send buffer (kernels::RoundMap), else identity
    uint32_t *roundMeta = nullptr;       // device copy of rm for the scatter
    uint64_t *send = nullptr;            // claim slices (8-byte words)
    void *cursorsBack = nullptr;         // [C][G][F] final claim cursors (pinned staging)
    std::vector<hipEvent_t> scattered;   // [C]
    histograms::ExchangePlan xp;         // filled chunk by chunk (the window holds a reference)
    std::unique_ptr<data::Window> window;
    std::vector<uint64_t> windowCap;     // [N] receive capacity of every rank (same on all ranks)
  };
  uint64_t receiveCapacity(int k, uint32_t rank) const;

  uint32_t nodes, me;
  core::ExecContext *ctx;
  const core::JoinPlan &plan;
  uint32_t requestedStride;
  HistogramComputation *hc;
  Side sides[2];
};

}  // namespace tasks
}  // namespace hpcjoin
