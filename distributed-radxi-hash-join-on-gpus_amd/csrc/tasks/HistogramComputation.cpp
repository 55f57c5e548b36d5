#include "HistogramComputation.h"

#include "../comm/Communicator.h"
#include "../memory/Arena.h"
#include "../performance/Clock.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../utils/Debug.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

HistogramComputation::HistogramComputation(uint32_t numberOfNodes, uint32_t nodeId, data::Relation *innerRelation,
                                           data::Relation *outerRelation, core::ExecContext *ctx,
                                           const core::JoinPlan &plan, uint32_t maxBlocks)
    : nodeId(nodeId), numberOfNodes(numberOfNodes), innerRelation(innerRelation), outerRelation(outerRelation),
      ctx(ctx) {
  innerRelationLocalHistogram.reset(
      new histograms::LocalHistogram(innerRelation, ctx, plan.networkBits, plan.chunks, maxBlocks,
                                     kernels::KeyMix{plan.keyMix ? 1u : 0u, plan.keyBits}));
  outerRelationLocalHistogram.reset(
      new histograms::LocalHistogram(outerRelation, ctx, plan.networkBits, plan.chunks, maxBlocks,
                                     kernels::KeyMix{plan.keyMix ? 1u : 0u, plan.keyBits}));
  innerRelationGlobalHistogram.reset(new histograms::GlobalHistogram(innerRelationLocalHistogram.get(), ctx->comm()));
  outerRelationGlobalHistogram.reset(new histograms::GlobalHistogram(outerRelationLocalHistogram.get(), ctx->comm()));
  assignment.reset(new histograms::AssignmentMap(numberOfNodes, innerRelationGlobalHistogram.get(),
                                                 outerRelationGlobalHistogram.get(), plan.assignment));
  assignment->setSkewSplit(plan.skewSplit);
  assignment->setPieces(std::max<uint32_t>(1, plan.chunks));
  innerOffsets.reset(new histograms::OffsetMap(numberOfNodes, nodeId, innerRelationLocalHistogram.get(),
                                               innerRelationGlobalHistogram.get(), assignment.get()));
  outerOffsets.reset(new histograms::OffsetMap(numberOfNodes, nodeId, outerRelationLocalHistogram.get(),
                                               outerRelationGlobalHistogram.get(), assignment.get()));
}

HistogramComputation::~HistogramComputation() = default;  // events belong to the context pool

void HistogramComputation::executeInner(uint32_t sampleStride) {
  uint64_t t0 = performance::nowUs();
  performance::Timeline &tl = ctx->timeline();
  tl.begin("HILOCAL", ctx->stream());
  innerRelationLocalHistogram->computeLocalHistogram();
  tl.end("HILOCAL", ctx->stream());
  tl.begin("HOLOCAL", ctx->stream());
  outerRelationLocalHistogram->computeSampledEstimate(sampleStride);
  tl.end("HOLOCAL", ctx->stream());
  ctx->synchronize();
  outerRelationLocalHistogram->scaleEstimate();
  localUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  histograms::GlobalHistogram::computeGlobalHistograms(*innerRelationGlobalHistogram, *outerRelationGlobalHistogram);
  globalUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  assignment->computePartitionAssignment();  // outer side: the estimate
  assignUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  innerOffsets->computeOffsets();
  offsetUs = performance::nowUs() - t0;
}

void HistogramComputation::assignFromEstimates(const uint64_t *innerEstimate, const uint64_t *outerEstimate) {
  innerRelationLocalHistogram->setChunkHistograms(innerEstimate);
  outerRelationLocalHistogram->setChunkHistograms(outerEstimate);
  uint64_t t0 = performance::nowUs();
  histograms::GlobalHistogram::computeGlobalHistograms(*innerRelationGlobalHistogram, *outerRelationGlobalHistogram);
  globalUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  assignment->computePartitionAssignment();
  assignUs = performance::nowUs() - t0;
}

void HistogramComputation::launchOuter(hipStream_t exchangeStream) {
  histograms::LocalHistogram *h = outerRelationLocalHistogram.get();
  const size_t per = (size_t)h->getChunkCount() * h->getPartitionCount();
  if (!ctx->onDevice()) {  // host path: the same sequence, completed in place
    ctx->timeline().begin("HOLOCAL");
    h->computeLocalHistogram();
    ctx->timeline().end("HOLOCAL");
    outerGatherHostVec.resize(per * numberOfNodes);
    ctx->timeline().begin("HOGLOBAL");
    ctx->comm()->allGatherHost(h->getChunkHistograms(), outerGatherHostVec.data(), per);
    ctx->timeline().end("HOGLOBAL");
    outerGatherHost = outerGatherHostVec.data();
    outerLaunched = true;
    return;
  }
  if (!outerHistDone) outerHistDone = ctx->acquireEvent();
  if (!outerGatherDone) outerGatherDone = ctx->acquireEvent();
  ctx->timeline().begin("HOLOCAL", ctx->stream());
  h->computeLocalHistogramDevice();
  ctx->timeline().end("HOLOCAL", ctx->stream());
  HIP_CHECK(hipEventRecord(outerHistDone, ctx->stream()));
  uint64_t *gatherDev = ctx->workspace().getArray<uint64_t>(per * numberOfNodes);
  outerGatherHost = ctx->staging().getArray<uint64_t>(per * numberOfNodes);
  HIP_CHECK(hipStreamWaitEvent(exchangeStream, outerHistDone, 0));
  ctx->timeline().begin("HOGLOBAL", exchangeStream);
  ctx->comm()->allGatherDevice(h->chunkTotalsDevice(), gatherDev, per, exchangeStream);
  ctx->timeline().end("HOGLOBAL", exchangeStream);
  ctx->readBack(outerGatherHost, gatherDev, per * numberOfNodes * 8, exchangeStream);
  HIP_CHECK(hipEventRecord(outerGatherDone, exchangeStream));
  outerLaunched = true;
}

void HistogramComputation::finishOuter() {
  JOIN_ASSERT(outerLaunched, "HistogramComputation", "finishOuter() before launchOuter()");
  if (ctx->onDevice()) utils::waitEvent(outerGatherDone, ctx->comm(), "outer histogram all-gather");
  histograms::LocalHistogram *h = outerRelationLocalHistogram.get();
  const size_t per = (size_t)h->getChunkCount() * h->getPartitionCount();
  h->setChunkHistograms(outerGatherHost + per * nodeId);
  outerRelationGlobalHistogram->setGathered(outerGatherHost);
  outerOffsets->computeOffsets();
  outerLaunched = false;
}

void HistogramComputation::execute() {
  computeLocalHistograms();
  computeGlobalInformation();
}

void HistogramComputation::computeLocalHistograms() {
  const uint64_t t0 = performance::nowUs();
  performance::Timeline &tl = ctx->timeline();
  tl.begin("HILOCAL", ctx->stream());
  innerRelationLocalHistogram->computeLocalHistogram();
  tl.end("HILOCAL", ctx->stream());
  tl.begin("HOLOCAL", ctx->stream());
  outerRelationLocalHistogram->computeLocalHistogram();
  tl.end("HOLOCAL", ctx->stream());
  ctx->synchronize();  // the host needs the totals for the collective
  localUs = performance::nowUs() - t0;
}

void HistogramComputation::computeGlobalInformation() {
  uint64_t t0 = performance::nowUs();
  histograms::GlobalHistogram::computeGlobalHistograms(*innerRelationGlobalHistogram, *outerRelationGlobalHistogram);
  globalUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  assignment->computePartitionAssignment();
  assignUs = performance::nowUs() - t0;
  t0 = performance::nowUs();
  innerOffsets->computeOffsets();
  outerOffsets->computeOffsets();
  offsetUs = performance::nowUs() - t0;
}

uint32_t *HistogramComputation::getAssignment() { return assignment->getPartitionAssignment(); }
uint64_t *HistogramComputation::getInnerRelationLocalHistogram() { return innerRelationLocalHistogram->getLocalHistogram(); }
uint64_t *HistogramComputation::getOuterRelationLocalHistogram() { return outerRelationLocalHistogram->getLocalHistogram(); }
uint64_t *HistogramComputation::getInnerRelationGlobalHistogram() { return innerRelationGlobalHistogram->getGlobalHistogram(); }
uint64_t *HistogramComputation::getOuterRelationGlobalHistogram() { return outerRelationGlobalHistogram->getGlobalHistogram(); }
uint64_t *HistogramComputation::getInnerRelationBaseOffsets() { return innerOffsets->getBaseOffsets(); }
uint64_t *HistogramComputation::getOuterRelationBaseOffsets() { return outerOffsets->getBaseOffsets(); }
uint64_t *HistogramComputation::getInnerRelationWriteOffsets() { return innerOffsets->getAbsoluteWriteOffsets(); }
uint64_t *HistogramComputation::getOuterRelationWriteOffsets() { return outerOffsets->getAbsoluteWriteOffsets(); }

}  // namespace tasks
}  // namespace hpcjoin
