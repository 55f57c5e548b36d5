// Global histogram = sum of all ranks' local histograms.  The reference runs
// MPI_Allreduce here and a separate MPI_Exscan in OffsetMap
// (/root/reference/histograms/GlobalHistogram.cpp:31-48, OffsetMap.cpp:75-85).
// Here ONE all-gather of every rank's per-chunk histograms (inner and outer
// fused into one message) gives each rank the full [rank][chunk][partition]
// table, from which the global sums, the exclusive prefix over ranks and the
// whole exchange plan are derived locally and identically on every rank.
#pragma once

#include <cstdint>
#include <vector>

#include "LocalHistogram.h"

namespace hpcjoin {
namespace comm {
class Communicator;
}
namespace histograms {

class GlobalHistogram {
 public:
  explicit GlobalHistogram(LocalHistogram *localHistogram);  // uses comm::world()
  GlobalHistogram(LocalHistogram *localHistogram, comm::Communicator *comm);
  ~GlobalHistogram();

  void computeGlobalHistogram();
  // One collective for both relations (what HistogramComputation uses).
  static void computeGlobalHistograms(GlobalHistogram &inner, GlobalHistogram &outer);

  // Take the [rank][chunk][partition] table of this relation alone from an
  // all-gather done elsewhere (e.g. on device, overlapped with an exchange).
  void setGathered(const uint64_t *gathered);

  uint64_t *getGlobalHistogram();  // [F]
  // count of partition p in chunk c on rank r
  uint64_t rankCount(uint32_t r, uint32_t c, uint32_t p) const {
    return table[((size_t)r * chunks + c) * partitions + p];
  }
  uint32_t numberOfNodes() const { return nodes; }
  uint32_t getChunkCount() const { return chunks; }
  uint32_t getPartitionCount() const { return partitions; }
  LocalHistogram *getLocalHistogram() const { return localHistogram; }

 protected:
  LocalHistogram *localHistogram;
  std::vector<uint64_t> values;  // [F]

 private:
  void absorb(const uint64_t *gathered, size_t stride, size_t offset);
  comm::Communicator *comm;
  uint32_t nodes = 1, chunks = 1, partitions = 0;
  std::vector<uint64_t> table;  // [N][chunks][F]
};

}  // namespace histograms
}  // namespace hpcjoin
