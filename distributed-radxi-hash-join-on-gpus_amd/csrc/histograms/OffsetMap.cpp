#include "OffsetMap.h"

#include "../comm/World.h"
#include "../utils/Debug.h"

namespace hpcjoin {
namespace histograms {

OffsetMap::OffsetMap(uint32_t numberOfProcesses, LocalHistogram *localHistogram, GlobalHistogram *globalHistogram,
                     AssignmentMap *assignment)
    : OffsetMap(numberOfProcesses, comm::world()->rank(), localHistogram, globalHistogram, assignment) {}

OffsetMap::OffsetMap(uint32_t numberOfProcesses, uint32_t nodeId, LocalHistogram *localHistogram,
                     GlobalHistogram *globalHistogram, AssignmentMap *assignment)
    : numberOfProcesses(numberOfProcesses), nodeId(nodeId), localHistogram(localHistogram),
      globalHistogram(globalHistogram), assignment(assignment) {}

OffsetMap::~OffsetMap() {}

void OffsetMap::computeOffsets() {
  JOIN_ASSERT(globalHistogram->numberOfNodes() == numberOfProcesses, "OffsetMap",
              "histogram table has %u ranks, expected %u", globalHistogram->numberOfNodes(), numberOfProcesses);
  computeBaseOffsets();
  computeRelativePrivateOffsets();
  computeAbsolutePrivateOffsets();
  computeExchangePlan();
}

// Base offset of partition p inside its owner's partition-major layout.
void OffsetMap::computeBaseOffsets() {
  const uint32_t F = globalHistogram->getPartitionCount();
  const uint32_t *owner = assignment->getPartitionAssignment();
  const uint64_t *g = globalHistogram->getGlobalHistogram();
  std::vector<uint64_t> run(numberOfProcesses, 0);
  baseOffsets.assign(F, 0);
  for (uint32_t p = 0; p < F; ++p) {
    baseOffsets[p] = run[owner[p]];
    run[owner[p]] += g[p];
  }
}

// Exclusive prefix over ranks (the MPI_Exscan of OffsetMap.cpp:75-85).
void OffsetMap::computeRelativePrivateOffsets() {
  const uint32_t F = globalHistogram->getPartitionCount(), C = globalHistogram->getChunkCount();
  relativeWriteOffsets.assign(F, 0);
  for (uint32_t r = 0; r < nodeId; ++r)
    for (uint32_t c = 0; c < C; ++c)
      for (uint32_t p = 0; p < F; ++p) relativeWriteOffsets[p] += globalHistogram->rankCount(r, c, p);
}

void OffsetMap::computeAbsolutePrivateOffsets() {
  const uint32_t F = globalHistogram->getPartitionCount();
  absoluteWriteOffsets.assign(F, 0);
  for (uint32_t p = 0; p < F; ++p) absoluteWriteOffsets[p] = baseOffsets[p] + relativeWriteOffsets[p];
}

void OffsetMap::computeExchangePlan() {
  const uint32_t N = numberOfProcesses, F = globalHistogram->getPartitionCount(),
                 C = globalHistogram->getChunkCount(), me = nodeId;
  const int side = assignment->sideOf(globalHistogram);
  const AssignmentMap &am = *assignment;
  ExchangePlan &x = plan;
  x = ExchangePlan();
  x.numberOfNodes = N;
  x.nodeId = me;
  x.partitions = F;
  x.chunks = C;
  // Partitions each rank joins: its own, plus the hot ones it helps with.
  std::vector<std::vector<uint32_t>> ownedBy(N);
  for (uint32_t p = 0; p < F; ++p)
    for (uint32_t d = 0; d < N; ++d)
      if (am.owns(p, d)) ownedBy[d].push_back(p);
  x.owned = ownedBy[me];
  x.localIndex.assign(F, -1);
  for (uint32_t lp = 0; lp < x.owned.size(); ++lp) x.localIndex[x.owned[lp]] = (int32_t)lp;

  // send side: the scatter writes each (chunk, partition) run once, into the
  // first destination that receives it; replicated runs are copied after.
  constexpr uint64_t UNSET = ~0ull;
  x.digitBase.assign((size_t)C * F, UNSET);
  x.digitDest.assign((size_t)C * F, 0);
  x.sendCounts.assign((size_t)C * N, 0);
  x.sendDispls.assign((size_t)C * N, 0);
  uint64_t cur = 0;
  for (uint32_t c = 0; c < C; ++c) {
    for (uint32_t d = 0; d < N; ++d) {
      x.sendDispls[(size_t)c * N + d] = cur;
      for (uint32_t p : ownedBy[d]) {
        if (!am.receives(side, me, c, C, p, d)) continue;
        const uint64_t n = globalHistogram->rankCount(me, c, p);
        uint64_t &db = x.digitBase[(size_t)c * F + p];
        if (db == UNSET) {
          db = cur;
          x.digitDest[(size_t)c * F + p] = d;
          x.scatterTotal += n;
        } else if (n) {
          x.replicas.push_back(Replica{c, db, cur, n});
        }
        cur += n;
      }
      x.sendCounts[(size_t)c * N + d] = cur - x.sendDispls[(size_t)c * N + d];
    }
    for (uint32_t p = 0; p < F; ++p) {
      uint64_t &db = x.digitBase[(size_t)c * F + p];
      JOIN_ASSERT(db != UNSET || globalHistogram->rankCount(me, c, p) == 0, "OffsetMap",
                  "partition %u (chunk %u) has no destination", p, c);
      if (db == UNSET) db = cur;  // empty run
    }
  }
  x.sendTotal = cur;

  // receive side
  const uint32_t owned = (uint32_t)x.owned.size();
  x.recvCounts.assign((size_t)C * N, 0);
  x.recvDispls.assign((size_t)C * N, 0);
  std::vector<uint64_t> segStart((size_t)C * N * owned, 0), segLen((size_t)C * N * owned, 0);
  cur = 0;
  for (uint32_t c = 0; c < C; ++c)
    for (uint32_t s = 0; s < N; ++s) {
      x.recvDispls[(size_t)c * N + s] = cur;
      for (uint32_t lp = 0; lp < owned; ++lp) {
        const size_t i = ((size_t)c * N + s) * owned + lp;
        segStart[i] = cur;
        segLen[i] = am.receives(side, s, c, C, x.owned[lp], me) ? globalHistogram->rankCount(s, c, x.owned[lp]) : 0;
        cur += segLen[i];
      }
      x.recvCounts[(size_t)c * N + s] = cur - x.recvDispls[(size_t)c * N + s];
    }
  x.recvTotal = cur;

  x.partSize.assign(owned, 0);
  x.lpBase.assign(owned + 1, 0);
  for (uint32_t lp = 0; lp < owned; ++lp) {
    for (uint32_t c = 0; c < C; ++c)
      for (uint32_t s = 0; s < N; ++s) {
        const size_t i = ((size_t)c * N + s) * owned + lp;
        x.partSize[lp] += segLen[i];
        if (segLen[i]) x.segments.push_back(Segment{segStart[i], segLen[i], lp, c, s});
      }
    x.lpBase[lp + 1] = x.lpBase[lp] + x.partSize[lp];
  }
  JOIN_ASSERT(x.lpBase[owned] == x.recvTotal, "OffsetMap", "window accounting mismatch %lu != %lu",
              (unsigned long)x.lpBase[owned], (unsigned long)x.recvTotal);
}

uint64_t *OffsetMap::getBaseOffsets() { return baseOffsets.data(); }
uint64_t *OffsetMap::getRelativeWriteOffsets() { return relativeWriteOffsets.data(); }
uint64_t *OffsetMap::getAbsoluteWriteOffsets() { return absoluteWriteOffsets.data(); }

}  // namespace histograms
}  // namespace hpcjoin
