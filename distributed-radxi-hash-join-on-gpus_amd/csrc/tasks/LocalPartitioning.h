// Local (second) radix pass over the received window so that every final
// partition's inner side fits one LDS hash table.  Reference:
// /root/reference/tasks/LocalPartitioning.cpp:59-250 (per network partition,
// host histogram + padded prefix sum + write-combined scatter, disabled by
// default).  Here all owned partitions of a relation are processed by three
// launches: per-item LDS histograms, per-partition cursor scan, LDS
// write-combining scatter.  Work items never cross a (chunk, source,
// partition) segment of the window, so the source-major RCCL layout needs
// no compaction pass.
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
                    const core::JoinPlan &plan);
  ~LocalPartitioning();

  void execute();
  task_type_t getType() { return TASK_PARTITION; }

  uint64_t partitionedElements() const { return elements; }
  uint64_t workItems() const { return items[0].size() + items[1].size(); }

 protected:
  void partition(data::Window *window, int which);

 private:
  data::Window *windows[2];
  core::ExecContext *ctx;
  core::JoinPlan plan;
  std::vector<kernels::LocalItem> items[2];
  std::vector<uint32_t> lpItemBegin[2];
  std::vector<uint64_t> zero;
  uint64_t elements = 0;
};

}  // namespace tasks
}  // namespace hpcjoin
