// Local (second) radix pass over the received window so that every final
// partition's inner side fits one LDS hash table.  Reference:
// /root/reference/tasks/LocalPartitioning.cpp:59-250 (per network partition,
// host histogram + padded prefix sum + write-combined scatter, disabled by
// default).  Here all owned partitions of a relation are processed by three
// launches: per-item LDS histograms, per-partition cursor scan, LDS
// write-combining scatter.  Work items never cross a (chunk, source,
// partition) segment of the window, so the source-major RCCL layout needs
// no compaction pass.
//
// Sampled mode (device, JoinPlan::localHistogram): the per-item histograms
// read 1 tile in sampleStride, each final partition gets a slot sized from
// the estimate plus 6 sigma of the sampling error, and the bounded scatter
// fills them (one claim stream per network partition).  Partitions then have
// tail gaps, so the window gets explicit partition ends (the final claim
// cursors) for the build/probe.  An overflowing slot raises a device flag
// that HashJoin reads after the build/probe; it then redoes the local pass
// exactly (forceExact) and the build/probe.
#pragma once

#include <vector>

#include "../core/ExecContext.h"
#include "../data/CompressedTuple.h"
#include "../data/Window.h"
#include "../kernels/kernels.h"
#include "Task.h"

namespace hpcjoin {
namespace tasks {

class LocalPartitioning : public Task {
 public:
  LocalPartitioning(data::Window *innerWindow, data::Window *outerWindow, core::ExecContext *ctx,
                    const core::JoinPlan &plan, bool forceExact = false);
  ~LocalPartitioning();

  void execute();
  task_type_t getType() { return TASK_PARTITION; }

  // One side at a time (pipelined outer relation: one call per chunk view of
  // the outer window, slot >= 1 distinct per call).
  void partitionSide(data::Window *window, int slot) {
    partition(window, slot);
    if (slot == 0) innerDone = true;
  }

  uint64_t partitionedElements() const { return elements; }
  uint64_t workItems() const { return itemTotal; }
  bool sampled() const { return anySampled; }
  // After the stream is synchronised: did a sampled slot overflow?
  bool overflowed() const;

 protected:
  void partition(data::Window *window, int which);
  void partitionImpl(data::Window *window, int which);
  void *alloc(uint64_t bytes);

 private:
  data::Window *windows[2];
  core::ExecContext *ctx;
  core::JoinPlan plan;
  // Per side (slot): host item lists stay alive until the join ends (async H2D sources).
  std::vector<std::vector<kernels::LocalItem>> items;
  std::vector<std::vector<uint32_t>> lpItemBegin;
  uint64_t itemTotal = 0;
  std::vector<uint64_t> zero;
  uint64_t elements = 0;
  bool forceExact;
  bool anySampled = false;
  bool innerDone = false;  // partitionSide(inner, 0) ran already: execute() does the outer side only
  // Per side (`which`): a device flag raised by an overflowing sampled slot
  // and its pinned copy, read back on the stream that ran that side (the
  // inner side may run on a stream of its own, JoinConfig::overlapLocal).
  std::vector<unsigned int *> overflowFlag;  // device
  std::vector<unsigned int *> overflowBack;  // pinned
};

}  // namespace tasks
}  // namespace hpcjoin
