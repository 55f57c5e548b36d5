#include "LocalHistogram.h"

#include <algorithm>

#include "../comm/World.h"
#include "../core/Configuration.h"
#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../utils/Debug.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace histograms {

LocalHistogram::LocalHistogram(data::Relation *relation)
    : relation(relation), ctx(nullptr), bits((uint32_t)core::Configuration::NETWORK_PARTITIONING_FANOUT), chunks(1) {
  ownedComm.reset(new comm::LocalCommunicator());
  ownedCtx.reset(new core::ExecContext(relation->location(), relation->device(), ownedComm.get()));
  ctx = ownedCtx.get();
  geom = kernels::partitionGeometry(relation->getLocalSize());
  bpc = geom.blocks;
}

LocalHistogram::LocalHistogram(data::Relation *relation, core::ExecContext *ctx, uint32_t bits, uint32_t chunks,
                               uint32_t maxBlocks, kernels::KeyMix mix)
    : relation(relation), ctx(ctx), bits(bits), chunks(std::max<uint32_t>(1, chunks)), mix(mix) {
  geom = kernels::partitionGeometry(relation->getLocalSize(), std::max<uint32_t>(maxBlocks, this->chunks));
  if (this->chunks > geom.blocks) this->chunks = geom.blocks;
  bpc = (uint32_t)ceilDiv(geom.blocks, this->chunks);
  this->chunks = (uint32_t)ceilDiv(geom.blocks, bpc);
}

LocalHistogram::~LocalHistogram() {}

void LocalHistogram::chunkRange(uint64_t n, uint32_t chunks, uint32_t maxBlocks, uint32_t c, uint64_t *begin,
                                uint64_t *end) {
  chunks = std::max<uint32_t>(1, chunks);
  const kernels::PartitionGeometry g = kernels::partitionGeometry(n, std::max<uint32_t>(maxBlocks, chunks));
  if (chunks > g.blocks) chunks = g.blocks;
  const uint64_t bpc = ceilDiv(g.blocks, chunks);
  const uint64_t per = bpc * g.tuplesPerBlock();
  *begin = std::min<uint64_t>(n, (uint64_t)c * per);
  *end = std::min<uint64_t>(n, *begin + per);
}

void LocalHistogram::computeLocalHistogram() {
  const uint32_t F = 1u << bits;
  values.assign(F, 0);
  chunkValues.assign((size_t)chunks * F, 0);
  summed = false;
  blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * geom.blocks);
  if (ctx->onDevice()) {
    totalsDev = ctx->workspace().getArray<uint64_t>((uint64_t)chunks * F);
    kernels::netHistogram(relation->getData(), relation->getLocalSize(), bits, geom, blockHist, ctx->stream(), mix);
    kernels::digitTotals(blockHist, F, geom.blocks, bpc, chunks, totalsDev, ctx->stream());
    ctx->copy(chunkValues.data(), totalsDev, chunkValues.size() * 8, false, true);
  } else {
    host::netHistogram(relation->getData(), relation->getLocalSize(), bits, geom, blockHist, mix);
    host::digitTotals(blockHist, F, geom.blocks, bpc, chunks, chunkValues.data());
  }
}

void LocalHistogram::computeLocalHistogramDevice() {
  const uint32_t F = 1u << bits;
  JOIN_ASSERT(ctx->onDevice(), "LocalHistogram", "device histogram on a host context");
  summed = false;
  blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * geom.blocks);
  totalsDev = ctx->workspace().getArray<uint64_t>((uint64_t)chunks * F);
  kernels::netHistogram(relation->getData(), relation->getLocalSize(), bits, geom, blockHist, ctx->stream(), mix);
  kernels::digitTotals(blockHist, F, geom.blocks, bpc, chunks, totalsDev, ctx->stream());
}

void LocalHistogram::computeSampledEstimate(uint32_t stride) {
  const uint32_t F = 1u << bits;
  values.assign(F, 0);
  chunkValues.assign((size_t)chunks * F, 0);
  summed = false;
  uint32_t *sampleHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * geom.blocks);
  if (ctx->onDevice()) {
    uint64_t *t = ctx->workspace().getArray<uint64_t>((uint64_t)chunks * F);
    kernels::netHistogram(relation->getData(), relation->getLocalSize(), bits, geom, sampleHist, ctx->stream(), mix,
                          std::max<uint32_t>(1, stride));
    kernels::digitTotals(sampleHist, F, geom.blocks, bpc, chunks, t, ctx->stream());
    ctx->copy(chunkValues.data(), t, chunkValues.size() * 8, false, true);
  } else {
    host::netHistogram(relation->getData(), relation->getLocalSize(), bits, geom, sampleHist, mix);
    host::digitTotals(sampleHist, F, geom.blocks, bpc, chunks, chunkValues.data());
  }
}

void LocalHistogram::scaleEstimate() {
  const uint32_t F = 1u << bits;
  const uint64_t n = relation->getLocalSize(), per = (uint64_t)bpc * geom.tuplesPerBlock();
  for (uint32_t c = 0; c < chunks; ++c) {
    const uint64_t b = std::min<uint64_t>(n, (uint64_t)c * per), e = std::min<uint64_t>(n, b + per);
    uint64_t *v = &chunkValues[(size_t)c * F];
    uint64_t sampledTuples = 0;
    for (uint32_t d = 0; d < F; ++d) sampledTuples += v[d];
    if (!sampledTuples) continue;
    const double scale = (double)(e - b) / (double)sampledTuples;
    for (uint32_t d = 0; d < F; ++d) v[d] = (uint64_t)(v[d] * scale + 0.5);
  }
  summed = false;
}

void LocalHistogram::setChunkHistograms(const uint64_t *v) {
  chunkValues.assign(v, v + (size_t)chunks * (1u << bits));
  summed = false;
}

uint64_t *LocalHistogram::getChunkHistograms() { return chunkValues.data(); }

uint64_t *LocalHistogram::getLocalHistogram() {
  if (!summed) {
    const uint32_t F = 1u << bits;
    values.assign(F, 0);
    for (uint32_t c = 0; c < chunks; ++c)
      for (uint32_t d = 0; d < F && !chunkValues.empty(); ++d) values[d] += chunkValues[(size_t)c * F + d];
    summed = true;
  }
  return values.data();
}

}  // namespace histograms
}  // namespace hpcjoin
