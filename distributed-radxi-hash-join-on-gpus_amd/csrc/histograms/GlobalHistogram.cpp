#include "GlobalHistogram.h"

#include <cstring>

#include "../comm/World.h"
#include "../utils/Debug.h"

namespace hpcjoin {
namespace histograms {

GlobalHistogram::GlobalHistogram(LocalHistogram *localHistogram)
    : localHistogram(localHistogram), comm(comm::world()) {}

GlobalHistogram::GlobalHistogram(LocalHistogram *localHistogram, comm::Communicator *comm)
    : localHistogram(localHistogram), comm(comm) {}

GlobalHistogram::~GlobalHistogram() {}

void GlobalHistogram::absorb(const uint64_t *gathered, size_t stride, size_t offset) {
  nodes = comm->size();
  chunks = localHistogram->getChunkCount();
  partitions = localHistogram->getPartitionCount();
  const size_t per = (size_t)chunks * partitions;
  table.resize(nodes * per);
  values.assign(partitions, 0);
  for (uint32_t r = 0; r < nodes; ++r) {
    std::memcpy(&table[r * per], gathered + r * stride + offset, per * 8);
    for (uint32_t c = 0; c < chunks; ++c)
      for (uint32_t p = 0; p < partitions; ++p) values[p] += table[r * per + (size_t)c * partitions + p];
  }
}

void GlobalHistogram::computeGlobalHistogram() {
  const size_t per = (size_t)localHistogram->getChunkCount() * localHistogram->getPartitionCount();
  std::vector<uint64_t> all(per * comm->size());
  comm->allGatherHost(localHistogram->getChunkHistograms(), all.data(), per);
  absorb(all.data(), per, 0);
}

void GlobalHistogram::computeGlobalHistograms(GlobalHistogram &inner, GlobalHistogram &outer) {
  JOIN_ASSERT(inner.comm == outer.comm, "GlobalHistogram", "fused histograms need one communicator");
  const size_t a = (size_t)inner.localHistogram->getChunkCount() * inner.localHistogram->getPartitionCount();
  const size_t b = (size_t)outer.localHistogram->getChunkCount() * outer.localHistogram->getPartitionCount();
  std::vector<uint64_t> send(a + b), all((a + b) * inner.comm->size());
  std::memcpy(send.data(), inner.localHistogram->getChunkHistograms(), a * 8);
  std::memcpy(send.data() + a, outer.localHistogram->getChunkHistograms(), b * 8);
  inner.comm->allGatherHost(send.data(), all.data(), a + b);
  inner.absorb(all.data(), a + b, 0);
  outer.absorb(all.data(), a + b, a);
}

void GlobalHistogram::setGathered(const uint64_t *gathered) {
  const size_t per = (size_t)localHistogram->getChunkCount() * localHistogram->getPartitionCount();
  absorb(gathered, per, 0);
}

uint64_t *GlobalHistogram::getGlobalHistogram() { return values.data(); }

}  // namespace histograms
}  // namespace hpcjoin
