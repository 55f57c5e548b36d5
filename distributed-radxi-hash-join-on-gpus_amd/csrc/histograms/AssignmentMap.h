// Partition -> owner node.  The reference assigns round-robin p % N and
// ignores the histograms it is given (/root/reference/histograms/AssignmentMap.cpp:34-49,
// SURVEY §2.9 #13).  Here RoundRobin is kept for parity and LPT (longest
// processing time first on |R_p| + |S_p|, ties by partition id, then by the
// lowest-loaded / lowest node) balances skewed inputs.  Both are pure
// functions of the global histograms, so every rank computes the same map.
#pragma once

#include <cstdint>
#include <vector>

#include "../core/JoinConfig.h"
#include "GlobalHistogram.h"

namespace hpcjoin {
namespace histograms {

class AssignmentMap {
 public:
  AssignmentMap(uint32_t numberOfNodes, GlobalHistogram *innerRelationGlobalHistogram,
                GlobalHistogram *outerRelationGlobalHistogram,
                core::AssignmentPolicy policy = core::AssignmentPolicy::RoundRobin);
  ~AssignmentMap();

  void computePartitionAssignment();
  uint32_t *getPartitionAssignment();
  uint64_t nodeLoad(uint32_t node) const { return loads.at(node); }  // |R| + |S| assigned
  core::AssignmentPolicy policy() const { return pol; }

 protected:
  uint32_t numberOfNodes;
  GlobalHistogram *innerRelationGlobalHistogram;
  GlobalHistogram *outerRelationGlobalHistogram;
  std::vector<uint32_t> assignment;

 private:
  core::AssignmentPolicy pol;
  std::vector<uint64_t> loads;
};

}  // namespace histograms
}  // namespace hpcjoin
