// Single-rank network pass without the exact histogram read.
//
// With one rank nothing is exchanged, so the network histogram is only needed
// to size the partition regions -- and reading both relations once just to
// count costs a full pass over the input (16 B per tuple, ~20% of a 1B x 1B
// join).  Here every workgroup histograms 1 tile in `sampleStride` of its own
// range; each (XCD group, digit) claim slice gets the estimate plus a
// statistical margin (6 sigma of the sampling error + 2%), and the bounded
// claim-mode scatter (kernels::netScatter with gend) fills the slices.  The
// final claim cursors give every slice's exact fill; the window's plan lists
// the filled slices as segments, which is all the local pass needs.  If a
// slice overflowed (skew the sample missed), the caller discards this pass and
// runs the exact histogram path (HashJoin keeps using it afterwards).
//
// Replaces, for N == 1, HistogramComputation + NetworkPartitioning
// (reference: histograms/LocalHistogram.cpp:35-53 + tasks/NetworkPartitioning.cpp:74-222).
#pragma once

#include <memory>
#include <vector>

#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../data/Window.h"
#include "../histograms/ExchangePlan.h"
#include "../kernels/kernels.h"

namespace hpcjoin {
namespace tasks {

class SampledNetworkPartitioning {
 public:
  SampledNetworkPartitioning(data::Relation *innerRelation, data::Relation *outerRelation, core::ExecContext *ctx,
                             const core::JoinPlan &plan, uint32_t maxBlocks, uint32_t sampleStride);
  ~SampledNetworkPartitioning();
  SampledNetworkPartitioning(const SampledNetworkPartitioning &) = delete;
  SampledNetworkPartitioning &operator=(const SampledNetworkPartitioning &) = delete;

  // Per side k (0 = inner, 1 = outer), so the host work of one side overlaps
  // the other side's kernels: sample() enqueues both sampled histograms;
  // layoutSide(k) enqueues side k's slice layout (on the device, from the
  // sampled totals: no wait) and sizes its window by the layout's bound;
  // scatterSide(k) enqueues the bounded scatter and the read-back of its
  // slices and final cursors; finishSide(k) waits for those and builds the
  // window plan (false = a slice overflowed).
  void sample();
  void layoutSide(int k);
  void scatterSide(int k);
  bool finishSide(int k);
  // Both sides in order (one wait per side).
  void layout();
  bool scatter();

  data::Window *innerWindow() { return sides[0].window.get(); }
  data::Window *outerWindow() { return sides[1].window.get(); }
  uint64_t capacity(int side) const { return sides[side].capacityTotal; }
  uint32_t roundLp() const;

 private:
  struct SidePlan {
    kernels::PartitionGeometry geom;
    uint32_t stride = 1;
    kernels::SampleScale sc{};
    uint64_t bound = 0;  // sum of the slice capacities can not exceed this
  };
  const SidePlan &sidePlan(uint64_t n) const;
  struct Side {
    data::Relation *relation = nullptr;
    kernels::PartitionGeometry geom;
    uint32_t stride = 1;  // sampled tile stride (kernels::sampleStrideFor)
    kernels::SampleScale sc{};
    histograms::ExchangePlan xp;
    std::unique_ptr<data::Window> window;
    uint64_t *groupTotalsDev = nullptr;  // [groups][F] sampled (or exact) counts
    void *cursorsBack = nullptr;         // [3][groups][F] slice starts, final claim cursors, slice ends (pinned)
    hipEvent_t cursorsReady = nullptr;
    std::vector<uint64_t> start;  // [groups][F] slice start (tuples), read back with the cursors
    std::vector<uint64_t> fill;   // [groups][F] claimed after the scatter
    void *gstart = nullptr, *gcur = nullptr, *gend = nullptr;  // device [groups][F] each, adjacent
    uint32_t *roundMeta = nullptr;                              // device {lp, lv, lns, 0} after gend
    bool narrow = true;
    uint64_t capacityTotal = 0;  // window slots: the layout's capacity bound
  };
  void finishPlan(Side &s);

  core::ExecContext *ctx;
  const core::JoinPlan &plan;
  uint32_t maxBlocks, sampleStride;
  Side sides[2];
};

}  // namespace tasks
}  // namespace hpcjoin
