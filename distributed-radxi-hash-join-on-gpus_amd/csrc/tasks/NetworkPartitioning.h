// Network partitioning: per relation, derive every workgroup's scatter
// cursors from the per-workgroup histogram and the exchange plan, run the
// LDS write-combining scatter (CompressedTuple packing fused in), and hand
// each finished chunk to the window's RCCL all-to-allv on the exchange
// stream.  Chunk k's exchange overlaps chunk k+1's scatter, and the inner
// relation's exchange overlaps the outer relation's scatter.
// Reference: /root/reference/tasks/NetworkPartitioning.cpp:64-222 (software
// write-combining + double-buffered MPI_Put).
#pragma once

#include <functional>

#include "../core/ExecContext.h"
#include "../data/Relation.h"
#include "../data/Window.h"
#include "HistogramComputation.h"
#include "Task.h"

namespace hpcjoin {
namespace tasks {

class NetworkPartitioning : public Task {
 public:
  NetworkPartitioning(uint32_t nodeId, data::Relation *innerRelation, data::Relation *outerRelation,
                      data::Window *innerWindow, data::Window *outerWindow, HistogramComputation *histograms,
                      core::ExecContext *ctx, const core::JoinPlan &plan);
  ~NetworkPartitioning();

  void execute();
  task_type_t getType() { return TASK_NET_PARTITION; }

  // Split histogram pipeline (HistogramComputation::launchOuter): the inner
  // relation first, with a hook after each chunk has been handed to the
  // exchange; the outer relation once its window exists.
  void partitionInner(const std::function<void(uint32_t)> &afterChunk);
  void partitionOuter(data::Window *window);

 protected:
  void partition(data::Relation *relation, data::Window *window, histograms::LocalHistogram *local,
                 const histograms::ExchangePlan &xp, const std::function<void(uint32_t)> &afterChunk = {});

 protected:
  uint32_t nodeId;
  data::Relation *innerRelation;
  data::Relation *outerRelation;
  data::Window *innerWindow;
  data::Window *outerWindow;

 private:
  HistogramComputation *histograms;
  core::ExecContext *ctx;
  core::JoinPlan plan;
};

}  // namespace tasks
}  // namespace hpcjoin
