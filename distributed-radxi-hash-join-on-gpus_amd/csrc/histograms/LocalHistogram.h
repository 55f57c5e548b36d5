// Per-rank radix histogram of the network partition bits.  Reference:
// /root/reference/histograms/LocalHistogram.cpp:35-53 (a host loop over key & 31).
// On MI355X it is the netHistogram kernel (LDS wave-private histograms,
// digit-major per-workgroup output) followed by a per-digit reduction; the
// per-workgroup histogram stays in HBM and is reused by NetworkPartitioning
// to derive every workgroup's scatter cursors.
#pragma once

#include <cstdint>
#include <vector>

#include "../core/ExecContext.h"
#include "../data/Relation.h"
#include "../kernels/kernels.h"

namespace hpcjoin {
namespace histograms {

class LocalHistogram {
 public:
  explicit LocalHistogram(data::Relation *relation);  // reference: host, Configuration fan-out, 1 chunk
  LocalHistogram(data::Relation *relation, core::ExecContext *ctx, uint32_t bits, uint32_t chunks,
                 uint32_t maxBlocks = 2048, kernels::KeyMix mix = kernels::KeyMix());
  ~LocalHistogram();

  void computeLocalHistogram();  // device: enqueued; host values valid after ctx->synchronize()
  // Device only: per-workgroup histogram and per-chunk totals stay in HBM
  // (chunkTotalsDevice()); no copy to the host.
  void computeLocalHistogramDevice();
  const uint64_t *chunkTotalsDevice() const { return totalsDev; }
  // Estimate from 1 tile in `stride` per workgroup (device: enqueued; call
  // scaleEstimate() after ctx->synchronize()).  Per-chunk counts are scaled to
  // the chunk's tuple count.  Used for the partition assignment only.
  void computeSampledEstimate(uint32_t stride);
  void scaleEstimate();
  void setChunkHistograms(const uint64_t *v);  // [chunks][F] (e.g. this rank's row of a gather)
  uint64_t *getLocalHistogram();  // [F], summed over chunks
  uint64_t *getChunkHistograms();  // [chunks][F]

  // Tuple range [begin, end) of exchange chunk c for a relation of n tuples:
  // the same block split as the constructor's (chunks may shrink for tiny n).
  static void chunkRange(uint64_t n, uint32_t chunks, uint32_t maxBlocks, uint32_t c, uint64_t *begin,
                         uint64_t *end);

  uint32_t getPartitionBits() const { return bits; }
  uint32_t getPartitionCount() const { return 1u << bits; }
  uint32_t getChunkCount() const { return chunks; }
  uint32_t blocksPerChunk() const { return bpc; }
  const kernels::PartitionGeometry &geometry() const { return geom; }
  const uint32_t *blockHistogram() const { return blockHist; }  // [F][blocks] (ctx location)
  data::Relation *getRelation() const { return relation; }

 protected:
  data::Relation *relation;
  std::vector<uint64_t> values;   // [F]
  std::vector<uint64_t> chunkValues;  // [chunks][F]

 private:
  core::ExecContext *ctx;
  std::unique_ptr<core::ExecContext> ownedCtx;
  std::unique_ptr<comm::Communicator> ownedComm;
  uint32_t bits, chunks, bpc;
  kernels::PartitionGeometry geom;
  uint32_t *blockHist = nullptr;
  uint64_t *totalsDev = nullptr;
  kernels::KeyMix mix;
  bool summed = false;
};

}  // namespace histograms
}  // namespace hpcjoin
