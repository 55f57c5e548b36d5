// Single-thread host implementations of every device kernel, with the SAME
// data layouts (digit-major block histograms, per-block cursors, per-item
// local cursors, partition begin arrays).  They are the reference CPU path
// of BASELINE config 1 (plumbing, no GPU), and the oracle the GPU kernels are
// tested against.  Build/probe uses the reference's bucket-chained table
// (/root/reference/tasks/BuildProbe.cpp:47-121) rather than the GPU's LDS
// open addressing, so the two paths are independent implementations.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "../kernels/kernels.h"

namespace hpcjoin {
namespace host {

kernels::ZipfParams makeZipf(uint64_t n, double theta);

void generate(data::Tuple *out, uint64_t n, const kernels::GenParams &p);

void netHistogram(const data::Tuple *in, uint64_t n, uint32_t bits, const kernels::PartitionGeometry &g,
                  uint32_t *blockHist, kernels::KeyMix mix = kernels::KeyMix());
void digitTotals(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk, uint32_t chunks,
                 uint64_t *totals);
void netCursors(const uint32_t *blockHist, uint32_t F, uint32_t blocks, uint32_t blocksPerChunk,
                const uint64_t *base, uint64_t *cursors);
void netScatter(const data::Tuple *in, uint64_t n, uint32_t bits, uint32_t keyShift,
                const kernels::PartitionGeometry &g, uint32_t blockBegin, uint32_t blockEnd, const uint64_t *cursors,
                void *out, bool wide, kernels::KeyMix mix = kernels::KeyMix(), bool withRids = true);

void localHistogram(const void *in, bool wide, const kernels::LocalItem *items, uint32_t nItems, uint32_t shift,
                    uint32_t bits, uint32_t *itemHist);
void localCursors(const uint32_t *itemHist, const uint32_t *lpItemBegin, uint32_t owned, uint32_t bits,
                  const uint64_t *lpBase, uint64_t *itemCursors, uint64_t *partBegin);
void localScatter(const void *in, bool wide, const kernels::LocalItem *items, uint32_t nItems, uint32_t shift,
                  uint32_t bits, const uint64_t *itemCursors, void *out);

// Bucket-chained build/probe per final partition; returns matches and (when
// a.materialize) writes pairs through a.outPairs / a.outCursor (host memory).
uint64_t buildProbe(const kernels::BPArgs &a);

// Wire codec (kernels.h, WireCodec) over host segment lists.
void wirePack(const uint64_t *raw, uint64_t *wire, const kernels::WireSeg *segs, uint32_t nSegs,
              const kernels::WireCodec &c);
void wireUnpack(const uint64_t *wire, uint64_t *raw, const kernels::WireSeg *segs, uint32_t nSegs,
                const kernels::WireCodec &c);

uint64_t npjJoin(const data::Tuple *R, uint64_t nR, const data::Tuple *S, uint64_t nS);
// (inner rid, outer rid) of every match, outer order, inner copies in input order.
std::vector<std::pair<uint64_t, uint64_t>> npjPairs(const data::Tuple *R, uint64_t nR, const data::Tuple *S,
                                                    uint64_t nS);

}  // namespace host
}  // namespace hpcjoin
