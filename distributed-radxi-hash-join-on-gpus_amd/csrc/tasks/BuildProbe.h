// Build/probe phase.  Reference: /root/reference/tasks/BuildProbe.cpp:47-121
// (host bucket chaining per partition pair) and the GPU offload of
// tasks/gpu/GPUWrapper.cu + operators/gpu/eth.cu (whose result was never
// read back).  Device flow, all stream-ordered:
//   plan counts -> wave64 scan (item count stays on the device) -> emit items
//   -> persistent LDS build/probe kernel -> one 64-bit atomic per workgroup.
// The host reads the counters once, after the join's single final sync.
#pragma once

#include <vector>

#include "../core/ExecContext.h"
#include "../data/CompressedTuple.h"
#include "../data/Window.h"
#include "../kernels/kernels.h"
#include "Task.h"

namespace hpcjoin {
namespace tasks {

class BuildProbe : public Task {
 public:
  // Reference-compatible: one (inner, outer) partition pair in host memory,
  // reference bit layout (compare value >> 32, hash bits from 37).
  BuildProbe(uint64_t innerPartitionSize, data::CompressedTuple *innerPartition, uint64_t outerPartitionSize,
             data::CompressedTuple *outerPartition);
  BuildProbe(data::Window *innerWindow, data::Window *outerWindow, core::ExecContext *ctx, const core::JoinPlan &plan,
             uint64_t outputCapacity);
  ~BuildProbe();

  void execute();
  task_type_t getType() { return TASK_BUILD_PROBE; }

  // After the caller synchronised the streams: pull the counters; returns
  // true if the work-item list or the output buffer overflowed and
  // execute() must run again (it then sizes both exactly).
  bool collect();

 private:
  void readBackCounters();

 public:
  uint64_t getMatches() const { return matches; }
  uint64_t getOutputCount() const { return outputCount; }
  uint32_t getWorkItems() const { return workItems; }
  const ulonglong2 *getOutput() const { return outPairs; }
  bool outputOverflowed() const { return overflowOut; }
  // Fused row output (device, split layout): the materialize pass writes whole
  // rows to the sink.  A sink overflow is reported, not re-run (the caller
  // owns the buffer).
  void setRowSink(const kernels::RowSink *s) { sink = s; }
  // Pairs go to this pinned host buffer (JoinConfig::outputHost, outputCapacity
  // pairs); an overflow is reported, not re-run.
  void setHostOutput(void *host) { hostOut = static_cast<ulonglong2 *>(host); }
  // The quotient table chained copies of a key (repeated inner keys), or a
  // span filled its overflow table and this task re-ran on counted tables.
  bool sawDuplicateChains() const { return duplicateChains; }
  bool rowsFused() const { return fused; }

 protected:
  uint64_t innerPartitionSize;
  data::CompressedTuple *innerPartition;
  uint64_t outerPartitionSize;
  data::CompressedTuple *outerPartition;

 private:
  void configure();
  core::ExecContext *ctx = nullptr;
  core::JoinPlan plan;
  data::Window *windows[2] = {nullptr, nullptr};
  kernels::BPArgs args;
  uint32_t capacity = 0;
  uint64_t outputCapacity = 0;
  // [0] matches [1] out cursor [2] item count (u32) [3] materialize: count-pass
  // matches / key spans: quotient-table side-list overflow flag
  unsigned long long *counters = nullptr;
  unsigned long long *countersBack = nullptr;  // pinned copy, enqueued at the end of execute()
  ulonglong2 *outPairs = nullptr;
  std::vector<uint64_t> refBounds;  // reference ctor: partition begin arrays
  uint64_t matches = 0, outputCount = 0;
  uint32_t workItems = 0;
  bool reference = false, overflowOut = false, fused = false;
  bool duplicateChains = false;   // copies of a key chained in the quotient table
  bool countedAll = false;        // a quotient span overflowed: this task counts every partition on counted tables
  bool deduped = false;           // heavy inner partitions compacted in place (kernels::bpKeyDedup)
  uint32_t *dedupCounts = nullptr;
  uint64_t *dedupLen = nullptr;
  const kernels::RowSink *sink = nullptr;
  ulonglong2 *hostOut = nullptr;
  uint64_t hostCursor = 0;
};

}  // namespace tasks
}  // namespace hpcjoin
