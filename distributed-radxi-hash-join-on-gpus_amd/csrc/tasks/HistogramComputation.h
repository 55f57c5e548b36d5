// Histogram phase: local histograms (HIP kernels) -> one fused all-gather ->
// assignment -> offsets / exchange plans.  Reference:
// /root/reference/tasks/HistogramComputation.cpp:63-76.
#pragma once

#include <memory>
#include <vector>

#include "../core/ExecContext.h"
#include "../data/Relation.h"
#include "../histograms/AssignmentMap.h"
#include "../histograms/GlobalHistogram.h"
#include "../histograms/LocalHistogram.h"
#include "../histograms/OffsetMap.h"
#include "Task.h"

namespace hpcjoin {
namespace tasks {

class HistogramComputation : public Task {
 public:
  HistogramComputation(uint32_t numberOfNodes, uint32_t nodeId, data::Relation *innerRelation,
                       data::Relation *outerRelation, core::ExecContext *ctx, const core::JoinPlan &plan,
                       uint32_t maxBlocks);
  ~HistogramComputation();

  void execute();
  task_type_t getType() { return TASK_HISTOGRAM; }

  // Split pipeline (JoinPlan::splitHistogram, device, N > 1): the outer
  // relation's exact histogram leaves the head of the join.
  //  executeInner(): inner exact + outer sampled estimate, one all-gather,
  //    assignment (LPT on the estimate), inner offsets.
  //  launchOuter(s): outer exact histogram on the compute stream and its
  //    all-gather enqueued on `s` (the exchange stream, after the inner
  //    chunks already issued there), then a copy to pinned host memory.
  //  finishOuter(): waits for that copy only, then outer offsets.
  void executeInner(uint32_t sampleStride);
  // Sampled N > 1 network pass (tasks/SampledShuffle): per-chunk estimates of
  // both relations ([chunks][F] each) -> one fused all-gather -> assignment.
  // No offsets: the exchange layout is built from the exact slice fills.
  void assignFromEstimates(const uint64_t *innerEstimate, const uint64_t *outerEstimate);
  void launchOuter(hipStream_t exchangeStream);
  void finishOuter();

  uint32_t *getAssignment();
  uint64_t *getInnerRelationLocalHistogram();
  uint64_t *getOuterRelationLocalHistogram();
  uint64_t *getInnerRelationGlobalHistogram();
  uint64_t *getOuterRelationGlobalHistogram();
  uint64_t *getInnerRelationBaseOffsets();
  uint64_t *getOuterRelationBaseOffsets();
  uint64_t *getInnerRelationWriteOffsets();
  uint64_t *getOuterRelationWriteOffsets();

  histograms::LocalHistogram *innerLocal() { return innerRelationLocalHistogram.get(); }
  histograms::LocalHistogram *outerLocal() { return outerRelationLocalHistogram.get(); }
  histograms::GlobalHistogram *innerGlobal() { return innerRelationGlobalHistogram.get(); }
  histograms::GlobalHistogram *outerGlobal() { return outerRelationGlobalHistogram.get(); }
  histograms::AssignmentMap *assignmentMap() { return assignment.get(); }
  histograms::OffsetMap *innerOffsetMap() { return innerOffsets.get(); }
  histograms::OffsetMap *outerOffsetMap() { return outerOffsets.get(); }

  // Sub-phase host times (µs) for Measurements.
  uint64_t localUs = 0, globalUs = 0, assignUs = 0, offsetUs = 0;

 protected:
  void computeLocalHistograms();
  void computeGlobalInformation();

 protected:
  uint32_t nodeId;
  uint32_t numberOfNodes;
  data::Relation *innerRelation;
  data::Relation *outerRelation;
  std::unique_ptr<histograms::LocalHistogram> innerRelationLocalHistogram;
  std::unique_ptr<histograms::LocalHistogram> outerRelationLocalHistogram;
  std::unique_ptr<histograms::GlobalHistogram> innerRelationGlobalHistogram;
  std::unique_ptr<histograms::GlobalHistogram> outerRelationGlobalHistogram;
  std::unique_ptr<histograms::AssignmentMap> assignment;
  std::unique_ptr<histograms::OffsetMap> innerOffsets;
  std::unique_ptr<histograms::OffsetMap> outerOffsets;

 private:
  core::ExecContext *ctx;
  hipEvent_t outerHistDone = nullptr, outerGatherDone = nullptr;
  uint64_t *outerGatherHost = nullptr;  // pinned (staging arena); host path: outerGatherHostVec
  std::vector<uint64_t> outerGatherHostVec;
  bool outerLaunched = false;
};

}  // namespace tasks
}  // namespace hpcjoin
