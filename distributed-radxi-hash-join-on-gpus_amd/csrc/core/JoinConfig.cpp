#include "JoinConfig.h"

#include <algorithm>

#include "../utils/Debug.h"

namespace hpcjoin {
namespace core {

std::string JoinConfig::describe() const {
  return utils::format("JoinConfig(networkBits=%u localBits=%u twoLevel=%d keyShift=%u assignment=%s format=%s "
                       "materialize=%d buildTarget=%lu rChunk=%u sChunk=%u chunks=%u)",
                       networkBits, localBits, (int)twoLevel, keyShift,
                       assignment == AssignmentPolicy::LPT ? "lpt" : "round_robin",
                       format == TupleFormat::Wide ? "wide" : "compressed", (int)materialize,
                       (unsigned long)buildTarget, rChunk, sChunk, chunks);
}

std::string JoinPlan::describe() const {
  return utils::format("JoinPlan(nodes=%u networkBits=%u localBits=%u twoLevel=%d keyShift=%u fragShift=%u "
                       "rChunk=%u sChunk=%u chunks=%u wide=%d materialize=%d keyMix=%d sampled=%d assignment=%s wire=%u/%u "
                       "split=%d splitHist=%d pipeOuter=%d bitmap=%d/%u%s%s%s%s%s)",
                       numberOfNodes, networkBits, localBits, (int)twoLevel, keyShift, fragShift, rChunk, sChunk,
                       chunks, (int)wide, (int)materialize, (int)keyMix, (int)sampledNetwork,
                       assignment == AssignmentPolicy::LPT ? "lpt" : "round_robin", wireBits[0], wireBits[1],
                       (int)splitLocal, (int)splitHistogram, (int)pipelineOuter, (int)bitmapJoin, bitmapBits,
                       bitmapReplicated ? " replicated" : "", keyOnly ? " keyOnly" : "",
                       oneSided ? " oneSided" : "", fragments && !bitmapJoin ? " fragments" : "",
                       innerRepeats ? " innerRepeats" : "");
}

JoinPlan makePlan(const JoinConfig &cfg, uint32_t numberOfNodes, uint64_t globalInner, uint64_t globalOuter,
                  uint64_t maxKey, uint64_t maxRid) {
  JoinPlan p;
  p.numberOfNodes = numberOfNodes;
  p.twoLevel = cfg.twoLevel;
  p.wide = cfg.format == TupleFormat::Wide;
  p.materialize = cfg.materialize;
  p.directCount = cfg.directCount;
  p.localItemTiles = std::max<uint32_t>(1, std::min<uint32_t>(cfg.localItemTiles, 1024));
  p.localGeometry = cfg.localGeometry;
  p.variants = cfg.variants;
  p.assignment = cfg.assignment;
  p.skewSplit = cfg.skewSplit && cfg.assignment == AssignmentPolicy::LPT && numberOfNodes > 1;
  p.chunks = std::max<uint32_t>(1, cfg.chunks);
  p.localHistogram = cfg.localHistogram;
  p.sampleStride = std::max<uint32_t>(1, cfg.sampleStride);
  p.localSampleStride = std::max<uint32_t>(1, cfg.localSampleStride);
  p.roundLp = std::min<uint32_t>(cfg.roundLp, 16);
  p.sChunk = std::max<uint32_t>(1024, cfg.sChunk);

  const uint32_t maxBits = Configuration::GPU_MAX_FANOUT_BITS - 1;  // 1024-way per pass
  // Materializing compressed tuples: final partitions of <= 2048 inner tuples
  // fit one 32 KiB (fragment, rid) table of the split materializing kernel.
  // At N = 1 (where rows can be written by the build/probe itself) the target
  // is 1024: with their 32-byte payload rows (32 KiB) they fit the LDS of the
  // fused row-output kernel, 3 workgroups per CU (kernels/build_probe.hip,
  // bpMatRowsKernel).  SF100: 35.6 ms fused vs 42.0 ms join + separate pass.
  const bool matNarrow = p.materialize && !p.wide && !cfg.rChunk;
  const uint32_t matTarget = numberOfNodes == 1 ? 1024 : 2048;
  // >= 8 network partitions per node so LPT has room to balance.
  const uint32_t minNet = std::max<uint32_t>(4, ceilLog2(numberOfNodes) + 3);
  auto splitBits = [&](uint64_t target) {
    const uint32_t totalBits = ceilLog2(ceilDiv(std::max<uint64_t>(globalInner, 1), std::max<uint64_t>(256, target)));
    if (cfg.networkBits) {
      p.networkBits = cfg.networkBits;
    } else if (p.twoLevel) {
      p.networkBits = std::min(maxBits, std::max(minNet, (totalBits + 1) / 2));
    } else {
      p.networkBits = std::min(maxBits, std::max(minNet, totalBits));
    }
    if (!p.twoLevel) {
      p.localBits = 0;
    } else if (cfg.localBits) {
      p.localBits = cfg.localBits;
    } else {
      p.localBits = totalBits > p.networkBits ? std::min(maxBits, totalBits - p.networkBits) : 1;
    }
  };
  splitBits(matNarrow ? std::min<uint64_t>(cfg.buildTarget, matTarget) : cfg.buildTarget);
  JOIN_ASSERT(p.networkBits >= 1 && p.networkBits <= Configuration::GPU_MAX_FANOUT_BITS, "Plan",
              "networkBits=%u out of range", p.networkBits);
  JOIN_ASSERT(p.localBits <= Configuration::GPU_MAX_FANOUT_BITS, "Plan", "localBits=%u out of range", p.localBits);

  const uint32_t ridBits = maxRid == ~0ull ? 64 : ceilLog2(maxRid + 1);
  const uint32_t keyBits = maxKey == ~0ull ? 64 : ceilLog2(maxKey + 1);
  p.keyBits = keyBits;
  // Mixed keys stay below 2^keyBits; a full 64-bit domain could map a key onto
  // the wide format's reserved empty marker, so mixing needs keyBits < 64.
  p.keyMix = cfg.keyHashing == KeyHashing::On && keyBits < 64;
  if (!p.wide) {
    // Keys too wide for a CompressedTuple (sparse 63-bit keys, rids beyond
    // 2^32 next to them): counting joins carry 8-byte key-only words, and
    // materializing ones the 16-byte Tuple format end to end.
    const uint32_t ks = cfg.keyShift ? cfg.keyShift : std::max<uint32_t>(32, ridBits);
    const uint32_t high = keyBits > p.networkBits ? keyBits - p.networkBits : 0;
    const uint32_t local = p.twoLevel ? p.localBits : 0;
    if (ks >= 64 || high > 64 - ks || high > 31 + local) {
      if (p.materialize)
        p.wide = true;
      else
        p.keyOnly = true;
    }
  }
  if (p.keyOnly) {
    // 8-byte table entries: final partitions of <= 2048 inner tuples give 36 KiB
    // LDS tables (4 workgroups per CU).  Measured on 1B x 1B sparse keys:
    // 24.7 ms per join against 28.5 ms with 4096-tuple partitions (2 per CU).
    if (!cfg.rChunk) splitBits(std::min<uint64_t>(cfg.buildTarget, 2048));
    p.keyShift = 0;
    p.fragShift = p.twoLevel ? p.localBits : 0;
  } else if (p.wide) {
    p.keyShift = 64;
    p.fragShift = 64;
    JOIN_ASSERT(maxKey != ~0ull, "Plan", "wide format reserves key 0xFFFFFFFFFFFFFFFF as the empty slot");
  } else {
    p.keyShift = cfg.keyShift ? cfg.keyShift : std::max<uint32_t>(32, ridBits);
    JOIN_ASSERT(ridBits <= p.keyShift, "Plan", "rids need %u bits but keyShift=%u", ridBits, p.keyShift);
    JOIN_ASSERT(p.keyShift >= 32, "Plan", "keyShift=%u: the rid field of a CompressedTuple is at least 32 bits",
                p.keyShift);
    const uint32_t keyHighBits = keyBits > p.networkBits ? keyBits - p.networkBits : 0;
    JOIN_ASSERT(keyHighBits <= 64 - p.keyShift, "Plan",
                "keys need %u bits: %u above the %u network bits do not fit the %u bits of a CompressedTuple above "
                "keyShift=%u; use TupleFormat::Wide",
                keyBits, keyHighBits, p.networkBits, 64 - p.keyShift, p.keyShift);
    p.fragShift = p.keyShift + (p.twoLevel ? p.localBits : 0);
    // The LDS table uses 0xFFFFFFFF as its empty marker: fragments must stay below it.
    JOIN_ASSERT(keyHighBits <= 31 + (p.twoLevel ? p.localBits : 0), "Plan",
                "key fragment (%u bits) would reach the LDS empty marker 0xFFFFFFFF", keyHighBits);
  }

  if (!p.wide && p.twoLevel) {
    const uint32_t passBits = p.networkBits + p.localBits;
    const uint32_t fragBits = p.keyBits > passBits ? p.keyBits - passBits : 0;
    // Compressed: u32 rid + u16 fragment.  Key-only: the fragment above both
    // digits as u32 + u16 (<= 48 bits: 63-bit keys leave 44 after 10 + 9).
    p.splitLocal = cfg.splitLocal && (p.keyOnly ? fragBits <= 48 : ridBits <= 32 && fragBits <= 16);
  }

  // LDS budget: a 32 KiB table (counting, 4-byte fragments) lets 5 workgroups
  // (20 wave64s) share a CU; materializing compressed tuples also uses 32 KiB
  // (4 per CU); wide entries get 64 KiB (2 per CU).
  if (cfg.rChunk) {
    p.rChunk = cfg.rChunk;
  } else {
    const uint32_t entry = p.wide ? (p.materialize ? 16 : 8) : (p.materialize || p.keyOnly ? 8 : 4);
    const uint32_t budget = (entry == 4 || p.keyOnly) ? 32 * 1024 : matNarrow ? 16 * matTarget : 64 * 1024;
    p.rChunk = (budget / entry) / 2;
  }
  return p;
}

}  // namespace core
}  // namespace hpcjoin
