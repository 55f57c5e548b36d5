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
  helpers.assign(F, {});
  splitSide.assign(F, 0);
  nSplit = 0;
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
  uint64_t total = 0;
  for (uint32_t p = 0; p < F; ++p) total += r[p] + s[p];
  const uint64_t fair = total / numberOfNodes;
  const uint64_t target = fair / 2;  // a helper's share of a divided partition
  const uint64_t pieces = (uint64_t)numberOfNodes * chunks;
  for (uint32_t p : order) {
    const uint64_t load = r[p] + s[p];
    const uint64_t big = std::max(r[p], s[p]), small = std::min(r[p], s[p]);
    // Divided: partitions above a rank's fair share, and those above half of
    // it whose larger side dominates (left whole, such lumps are what the
    // greedy placement cannot even out: Zipf(0.99) over 5 keys on 8 ranks went
    // from 1.41x to ~1.1x the mean load).
    const bool hot = load > fair || (load > target && big > 2 * small);
    if (split && numberOfNodes > 1 && fair > 0 && hot && big > small) {
      // k helpers: the smallest divisor of the piece count (so every helper
      // gets the same number of pieces) that brings a helper's share down to
      // half a fair share, at most every rank; the least loaded ranks (ties:
      // lowest id).
      uint32_t k = 0;
      for (uint32_t c = 2; c <= numberOfNodes; ++c) {
        if (pieces % c) continue;
        k = c;
        if (big / c + small <= target) break;
      }
      if (k == 0) k = (uint32_t)std::min<uint64_t>(numberOfNodes, std::max<uint64_t>(2, (load + fair - 1) / fair));
      std::vector<uint32_t> byLoad(numberOfNodes);
      std::iota(byLoad.begin(), byLoad.end(), 0u);
      std::stable_sort(byLoad.begin(), byLoad.end(), [&](uint32_t a, uint32_t b) { return loads[a] < loads[b]; });
      std::vector<uint32_t> h(byLoad.begin(), byLoad.begin() + k);
      std::sort(h.begin(), h.end());
      for (uint32_t n : h) loads[n] += small + (big + k - 1) / k;
      assignment[p] = h[0];
      splitSide[p] = s[p] >= r[p] ? 1 : 0;
      helpers[p] = std::move(h);
      ++nSplit;
      continue;
    }
    uint32_t best = 0;
    for (uint32_t n = 1; n < numberOfNodes; ++n)
      if (loads[n] < loads[best]) best = n;
    assignment[p] = best;
    loads[best] += r[p] + s[p];
  }
}

uint32_t *AssignmentMap::getPartitionAssignment() { return assignment.data(); }

bool AssignmentMap::receives(int side, uint32_t source, uint32_t chunk, uint32_t chunks, uint32_t p,
                             uint32_t node) const {
  if (!isSplit(p)) return assignment[p] == node;
  const std::vector<uint32_t> &h = helpers[p];
  if (side == splitSide[p]) return h[((uint64_t)source * chunks + chunk) % h.size()] == node;
  return std::binary_search(h.begin(), h.end(), node);
}

bool AssignmentMap::owns(uint32_t p, uint32_t node) const {
  if (!isSplit(p)) return assignment[p] == node;
  return std::binary_search(helpers[p].begin(), helpers[p].end(), node);
}

}  // namespace histograms
}  // namespace hpcjoin
