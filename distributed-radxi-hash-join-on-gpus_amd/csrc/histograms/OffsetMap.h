// Offsets of this rank's tuples inside the owners' windows.  Same three
// arrays as /root/reference/histograms/OffsetMap.cpp:43-93 (base offset of a
// partition in its owner's partition-major layout, this rank's relative
// offset inside the partition = exclusive prefix over ranks, absolute = sum),
// computed from the all-gathered table instead of MPI_Exscan, plus the full
// ExchangePlan for the RCCL all-to-allv and the local pass.
#pragma once

#include <cstdint>
#include <vector>

#include "AssignmentMap.h"
#include "ExchangePlan.h"
#include "GlobalHistogram.h"
#include "LocalHistogram.h"

namespace hpcjoin {
namespace histograms {

class OffsetMap {
 public:
  OffsetMap(uint32_t numberOfProcesses, LocalHistogram *localHistogram, GlobalHistogram *globalHistogram,
            AssignmentMap *assignment);  // nodeId from comm::world()
  OffsetMap(uint32_t numberOfProcesses, uint32_t nodeId, LocalHistogram *localHistogram,
            GlobalHistogram *globalHistogram, AssignmentMap *assignment);
  ~OffsetMap();

  void computeOffsets();
  uint64_t *getBaseOffsets();
  uint64_t *getRelativeWriteOffsets();
  uint64_t *getAbsoluteWriteOffsets();
  const ExchangePlan &getExchangePlan() const { return plan; }

 protected:
  void computeBaseOffsets();
  void computeRelativePrivateOffsets();
  void computeAbsolutePrivateOffsets();
  void computeExchangePlan();

 protected:
  uint32_t numberOfProcesses;
  uint32_t nodeId;
  LocalHistogram *localHistogram;
  GlobalHistogram *globalHistogram;
  AssignmentMap *assignment;
  std::vector<uint64_t> baseOffsets;
  std::vector<uint64_t> relativeWriteOffsets;
  std::vector<uint64_t> absoluteWriteOffsets;
  ExchangePlan plan;
};

}  // namespace histograms
}  // namespace hpcjoin
