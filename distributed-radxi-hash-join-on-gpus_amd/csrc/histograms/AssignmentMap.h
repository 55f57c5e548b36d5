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

  // Cross-rank splitting of a hot partition (the
  // skew_detect / probe_skew_pth_large idea of
  // /root/reference/operators/gpu/kernels_optimized.cu:301-457,591-672, moved
  // from workgroups to ranks).  With LPT and splitting on, a partition holding
  // more than one rank's fair share of |R| + |S| gets k helper ranks: its
  // larger side is divided among them by (source rank, chunk), its smaller
  // side is replicated to all of them, so every match is found exactly once
  // (each tuple of the divided side meets the whole other side on exactly one
  // rank).  Every rank derives the same map from the same histograms.
  void setSkewSplit(bool on) { split = on; }
  // Exchange chunks per rank: a divided side travels as numberOfNodes x
  // chunks pieces (source rank, chunk), so helper counts that divide it give
  // every helper the same share.
  void setPieces(uint32_t chunksPerRank) { chunks = chunksPerRank ? chunksPerRank : 1; }
  bool isSplit(uint32_t p) const { return p < helpers.size() && !helpers[p].empty(); }
  const std::vector<uint32_t> &helpersOf(uint32_t p) const { return helpers.at(p); }
  int splitSideOf(uint32_t p) const { return splitSide.at(p); }  // 0 inner, 1 outer: the divided side
  uint32_t splitPartitions() const { return nSplit; }
  // Does `node` receive relation `side`'s (0 inner, 1 outer) tuples of
  // partition p from chunk `chunk` (of `chunks`) of rank `source`?
  bool receives(int side, uint32_t source, uint32_t chunk, uint32_t chunks, uint32_t p, uint32_t node) const;
  // Does `node` join partition p (owner or helper)?
  bool owns(uint32_t p, uint32_t node) const;
  int sideOf(const GlobalHistogram *h) const { return h == outerRelationGlobalHistogram ? 1 : 0; }

 protected:
  uint32_t numberOfNodes;
  GlobalHistogram *innerRelationGlobalHistogram;
  GlobalHistogram *outerRelationGlobalHistogram;
  std::vector<uint32_t> assignment;

 private:
  core::AssignmentPolicy pol;
  std::vector<uint64_t> loads;
  bool split = false;
  uint32_t chunks = 1;
  uint32_t nSplit = 0;
  std::vector<std::vector<uint32_t>> helpers;  // [F]: empty unless split
  std::vector<uint8_t> splitSide;             // [F]
};

}  // namespace histograms
}  // namespace hpcjoin
