// Everything a rank needs to scatter, exchange and locally re-partition one
// relation, derived from the all-gathered histogram table + assignment.
//
// Send buffer (per chunk c): destination-major; inside a destination its
// owned partitions in increasing order.  Receive window: chunk-major, then
// source-major (what one grouped ncclSend/ncclRecv per peer produces), then
// owned partitions in increasing order.  Because every count is known before
// any byte moves, every write offset is exact and disjoint (the property of
// /root/reference/histograms/OffsetMap.cpp:59-93 the RMA design relied on).
#pragma once

#include <cstdint>
#include <vector>

namespace hpcjoin {
namespace histograms {

struct Segment {
  uint64_t begin;  // tuple offset in the window
  uint64_t len;
  uint32_t lp;     // local index of the owned partition
  uint32_t chunk;
  uint32_t source;
};

// A run the scatter writes once but that goes to several destinations (the
// replicated side of a split hot partition, AssignmentMap): copied inside the
// send buffer after the chunk's scatter.
struct Replica {
  uint32_t chunk;
  uint64_t src, dst, len;  // send-buffer tuple offsets
};

struct ExchangePlan {
  uint32_t numberOfNodes = 1, nodeId = 0, partitions = 0, chunks = 1;
  std::vector<uint32_t> owned;        // lp -> partition id (ascending)
  std::vector<int32_t> localIndex;    // partition id -> lp, or -1
  std::vector<uint64_t> digitBase;    // [chunks][F] send-buffer offset of (chunk, partition) run
  std::vector<uint64_t> sendCounts;   // [chunks][N]
  std::vector<uint64_t> sendDispls;   // [chunks][N]
  std::vector<uint64_t> recvCounts;   // [chunks][N]
  std::vector<uint64_t> recvDispls;   // [chunks][N]
  uint64_t sendTotal = 0, recvTotal = 0;
  uint64_t scatterTotal = 0;          // tuples the scatter writes (sendTotal minus replicas)
  std::vector<uint32_t> digitDest;    // [chunks][F] destination of the scattered (chunk, partition) run
  std::vector<Replica> replicas;
  std::vector<uint64_t> partSize;     // [owned]
  std::vector<uint64_t> lpBase;       // [owned + 1]
  std::vector<Segment> segments;      // by lp, then chunk, then source
  // Sampled single-rank pass: partitions are runs of estimated slices with
  // unused tail room between them (segments give the filled parts).
  bool gapped = false;
  // True when the window is already partition-major (N == 1 and one chunk).
  bool windowIsPartitionMajor() const { return numberOfNodes == 1 && chunks == 1 && !gapped; }
};

}  // namespace histograms
}  // namespace hpcjoin
