#include "AssignmentMap.h"

#include <algorithm>
#include <numeric>

#include "../utils/Debug.h"

namespace hpcjoin {
namespace histograms {

AssignmentMap::AssignmentMap(uint32_t numberOfNodes, GlobalHistogram *inner, GlobalHistogram *outer,
                             core::AssignmentPolicy policy)
    : numberOfNodes(numberOfNodes), innerRelationGlobalHistogram(inner), outerRelationGlobalHistogram(outer),
      pol(policy) {}

AssignmentMap::~AssignmentMap() {}

void AssignmentMap::computePartitionAssignment() {
  const uint32_t F = innerRelationGlobalHistogram->getPartitionCount();
  JOIN_ASSERT(F == outerRelationGlobalHistogram->getPartitionCount(), "AssignmentMap",
              "inner/outer fan-out mismatch");
  const uint64_t *r = innerRelationGlobalHistogram->getGlobalHistogram();
  const uint64_t *s = outerRelationGlobalHistogram->getGlobalHistogram();
  assignment.assign(F, 0);
  loads.assign(numberOfNodes, 0);
  if (pol == core::AssignmentPolicy::RoundRobin) {
    for (uint32_t p = 0; p < F; ++p) {
      assignment[p] = p % numberOfNodes;
      loads[assignment[p]] += r[p] + s[p];
    }
    return;
  }
  std::vector<uint32_t> order(F);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return r[a] + s[a] > r[b] + s[b]; });
  for (uint32_t p : order) {
    uint32_t best = 0;
    for (uint32_t n = 1; n < numberOfNodes; ++n)
      if (loads[n] < loads[best]) best = n;
    assignment[p] = best;
    loads[best] += r[p] + s[p];
  }
}

uint32_t *AssignmentMap::getPartitionAssignment() { return assignment.data(); }

}  // namespace histograms
}  // namespace hpcjoin
