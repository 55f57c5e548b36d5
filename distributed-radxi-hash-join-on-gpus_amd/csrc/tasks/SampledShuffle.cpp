#include "SampledShuffle.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../comm/Communicator.h"
#include "../memory/Arena.h"
#include "../performance/Timeline.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace tasks {

using kernels::CLAIM_GROUPS;
using kernels::PART_TILE;

SampledShuffle::SampledShuffle(uint32_t numberOfNodes, uint32_t nodeId, HistogramComputation *hc,
                               core::ExecContext *ctx, const core::JoinPlan &plan, uint32_t sampleStride)
    : nodes(numberOfNodes), me(nodeId), ctx(ctx), plan(plan), requestedStride(std::max<uint32_t>(1, sampleStride)),
      hc(hc) {
  JOIN_ASSERT(ctx->onDevice() && nodes > 1, "SampledShuffle", "multi-rank device path only");
  JOIN_ASSERT(!plan.wide, "SampledShuffle", "needs 8-byte tuples (packed or raw on the wire)");
  sides[0].local = hc->innerLocal();
  sides[1].local = hc->outerLocal();
  for (Side &s : sides) {
    s.relation = s.local->getRelation();
    s.chunks = s.local->getChunkCount();
  }
}

SampledShuffle::~SampledShuffle() = default;  // events belong to the context pool

namespace {
// Tuples chunk c's claim group g scatters, and how many of them the sampled
// histogram reads (netHistogramKernel: tiles begin, begin + stride, ... of
// every workgroup's range).
void groupScale(const histograms::LocalHistogram &h, uint64_t n, uint32_t stride, std::vector<double> &total,
                std::vector<double> &seen) {
  const kernels::PartitionGeometry &g = h.geometry();
  const uint32_t C = h.getChunkCount(), bpc = h.blocksPerChunk();
  total.assign((size_t)C * CLAIM_GROUPS, 0.0);
  seen.assign((size_t)C * CLAIM_GROUPS, 0.0);
  const uint64_t span = g.tuplesPerBlock();
  for (uint32_t b = 0; b < g.blocks; ++b) {
    const uint32_t c = b / bpc, grp = (b - c * bpc) % CLAIM_GROUPS;
    const uint64_t begin = (uint64_t)b * span, end = std::min(n, begin + span);
    if (begin >= end) continue;
    total[(size_t)c * CLAIM_GROUPS + grp] += (double)(end - begin);
    for (uint64_t base = begin; base < end; base += (uint64_t)PART_TILE * stride)
      seen[(size_t)c * CLAIM_GROUPS + grp] += (double)std::min<uint64_t>(PART_TILE, end - base);
  }
}
}  // namespace

void SampledShuffle::sampleAndAssign() {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  for (int k = 0; k < 2; ++k) {
    Side &s = sides[k];
    const uint64_t n = s.relation->getLocalSize();
    const kernels::PartitionGeometry &g = s.local->geometry();
    // At least ~64 sampled tuples per (chunk, group, digit) cell on average;
    // small inputs end at stride 1 (an exact count, no margins).
    const uint64_t cells = (uint64_t)s.chunks * G * F * 64;
    s.stride = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(requestedStride, n / std::max<uint64_t>(cells, 1)));
    const char *key = k == 0 ? "HILOCAL" : "HOLOCAL";
    ctx->timeline().begin(key, ctx->stream());
    uint32_t *blockHist = ctx->workspace().getArray<uint32_t>((uint64_t)F * std::max<uint32_t>(g.blocks, 1));
    uint64_t *groupDev = ctx->workspace().getArray<uint64_t>((uint64_t)s.chunks * G * F);
    if (n) {
      kernels::netHistogram(s.relation->getData(), n, plan.networkBits, g, blockHist, ctx->stream(), mix, s.stride);
      kernels::netChunkGroupTotals(blockHist, F, g.blocks, s.local->blocksPerChunk(), s.chunks, groupDev,
                                   ctx->stream());
    } else {
      ctx->zero(groupDev, (size_t)s.chunks * G * F * 8);
    }
    ctx->timeline().end(key, ctx->stream());
    s.sampled = ctx->staging().getArray<uint64_t>((uint64_t)s.chunks * G * F);
    ctx->readBack(s.sampled, groupDev, (size_t)s.chunks * G * F * 8);
  }
  utils::waitStream(ctx->stream(), ctx->comm(), "sampled network histograms");
  for (Side &s : sides) {
    const uint64_t n = s.relation->getLocalSize();
    std::vector<double> total, seen;
    groupScale(*s.local, n, s.stride, total, seen);
    const size_t cells = (size_t)s.chunks * G * F;
    s.start.assign(cells, 0);
    s.cap.assign(cells, 0);
    s.estimate.assign((size_t)s.chunks * F, 0);
    // Exact counts (stride 1) need no margin; otherwise 6 sigma of the
    // sampling error + 2% + 256 (the single-rank pass's statistics).
    const bool exact = s.stride == 1;
    const double sigmas = exact ? 0 : 6.0, frac = exact ? 0 : 0.02, floor = exact ? 0 : 256.0;
    uint64_t cur = 0;
    for (uint32_t c = 0; c < s.chunks; ++c)
      for (uint32_t d = 0; d < F; ++d) {
        double sum = 0;
        for (uint32_t g = 0; g < G; ++g) {
          const size_t cg = (size_t)c * G + g, i = cg * F + d;
          double est = 0, c2 = 0;
          if (seen[cg] > 0) {
            const double scale = total[cg] / seen[cg];
            est = (double)s.sampled[i] * scale;
            const double margin = sigmas * std::sqrt(std::max(est, scale) * scale) + frac * est + floor;
            c2 = std::min(std::ceil(est + margin), total[cg]);
          }
          sum += est;
          // whole 128-byte lines per slice: slices never share a line
          s.cap[i] = ((uint64_t)c2 + 15) & ~15ull;
          s.start[i] = cur;
          cur += s.cap[i];
        }
        s.estimate[(size_t)c * F + d] = (uint64_t)std::llround(sum);
      }
    s.capTotal = cur;
    // Round-interleaved send buffer (kernels::RoundMap): slice i = (c G + g) F
    // + d starts at logical i << lv; taken when its slots stay within half
    // again the linear total (uneven slices keep linear ones).
    s.rm = kernels::RoundMap();
    uint64_t logical = cur;
    if (const uint32_t lp = kernels::roundLpFor(plan.roundLp, 8)) {
      uint64_t maxCap = 0;
      for (uint64_t c : s.cap) maxCap = std::max(maxCap, c);
      uint32_t lns = 0, lv = lp;
      while ((1ull << lns) < cells) ++lns;
      while ((1ull << lv) < maxCap) ++lv;
      const uint64_t slots = kernels::roundSlots(maxCap, lp, lns);
      if (maxCap && lns + lv < 48 && slots <= cur + cur / 2 + (1ull << 20)) {
        s.rm.lp = lp;
        s.rm.lv = lv;
        s.rm.lns = lns;
        for (size_t i = 0; i < cells; ++i) s.start[i] = (uint64_t)i << lv;
        s.capTotal = slots;
        logical = (uint64_t)cells << lv;
      }
    }
    // Claims may run past a slice end by up to n before the overflow is seen.
    s.narrow = kernels::cursorsNarrow(logical + n);
  }
  hc->assignFromEstimates(sides[0].estimate.data(), sides[1].estimate.data());
}

uint64_t SampledShuffle::receiveCapacity(int k, uint32_t rank) const {
  // The estimated receive total of `rank` (every rank computes the same value
  // from the gathered estimates) + 1/16 + 64K tuples: the total of many
  // sampled cells is far more accurate than one cell.
  histograms::GlobalHistogram *gh = k == 0 ? hc->innerGlobal() : hc->outerGlobal();
  const histograms::AssignmentMap &am = *hc->assignmentMap();
  const uint32_t F = 1u << plan.networkBits, C = sides[k].chunks;
  uint64_t e = 0;
  for (uint32_t p = 0; p < F; ++p) {
    if (!am.owns(p, rank)) continue;
    for (uint32_t s = 0; s < nodes; ++s)
      for (uint32_t c = 0; c < C; ++c)
        if (am.receives(k, s, c, C, p, rank)) e += gh->rankCount(s, c, p);
  }
  return e + e / 16 + (64ull << 10);
}

void SampledShuffle::layoutSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  Side &s = sides[k];
  const size_t cells = (size_t)s.chunks * G * F;
  const size_t cb = s.narrow ? 4 : 8;
  s.gcur = ctx->workspace().get(cells * cb);
  s.gend = ctx->workspace().get(cells * cb);
  if (s.narrow) {
    s.cur32.resize(cells);
    s.end32.resize(cells);
    for (size_t i = 0; i < cells; ++i) {
      s.cur32[i] = (uint32_t)s.start[i];
      s.end32[i] = (uint32_t)(s.start[i] + s.cap[i]);
    }
    ctx->copy(s.gcur, s.cur32.data(), cells * 4, true, false);
    ctx->copy(s.gend, s.end32.data(), cells * 4, true, false);
  } else {
    s.end64.resize(cells);
    for (size_t i = 0; i < cells; ++i) s.end64[i] = s.start[i] + s.cap[i];
    ctx->copy(s.gcur, s.start.data(), cells * 8, true, false);
    ctx->copy(s.gend, s.end64.data(), cells * 8, true, false);
  }
  // Window plan skeleton: owned partitions now, segments chunk by chunk.
  const histograms::AssignmentMap &am = *hc->assignmentMap();
  histograms::ExchangePlan &x = s.xp;
  x = histograms::ExchangePlan();
  x.numberOfNodes = nodes;
  x.nodeId = me;
  x.partitions = F;
  x.chunks = s.chunks;
  x.localIndex.assign(F, -1);
  for (uint32_t p = 0; p < F; ++p)
    if (am.owns(p, me)) {
      x.localIndex[p] = (int32_t)x.owned.size();
      x.owned.push_back(p);
    }
  x.sendCounts.assign((size_t)s.chunks * nodes, 0);
  x.sendDispls.assign((size_t)s.chunks * nodes, 0);
  x.recvCounts.assign((size_t)s.chunks * nodes, 0);
  x.recvDispls.assign((size_t)s.chunks * nodes, 0);
  x.scatterTotal = x.sendTotal = s.relation->getLocalSize();
  s.windowCap.resize(nodes);
  for (uint32_t r = 0; r < nodes; ++r) s.windowCap[r] = receiveCapacity(k, r);
  s.window.reset(new data::Window(x, s.windowCap[me], ctx, false));
  s.window->setSendRounded(s.rm.on());
  kernels::WireCodec codec;
  codec.w = plan.wireBits[k];
  codec.ridBits = plan.wireRidBits[k];
  codec.keyShift = plan.keyShift;
  s.window->setWireCodec(codec, plan.ridBase[k]);
}

void SampledShuffle::scatterSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS;
  const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
  Side &s = sides[k];
  const uint64_t n = s.relation->getLocalSize();
  kernels::PartitionGeometry g = s.local->geometry();
  g.ipt = plan.variants.netIpt;
  g.nth = plan.variants.netThreads;
  const uint32_t bpc = s.local->blocksPerChunk();
  const size_t perChunk = (size_t)G * F * (s.narrow ? 4 : 8);
  s.send = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(s.capTotal, 1));
  s.cursorsBack = ctx->staging().get(perChunk * s.chunks);
  s.roundMeta = nullptr;
  if (s.rm.on()) {
    uint32_t *m = static_cast<uint32_t *>(ctx->staging().get(16));
    m[0] = s.rm.lp;
    m[1] = s.rm.lv;
    m[2] = s.rm.lns;
    m[3] = 0;
    s.roundMeta = ctx->workspace().getArray<uint32_t>(4);
    ctx->copy(s.roundMeta, m, 16, true, false);
  }
  s.scattered.assign(s.chunks, nullptr);
  s.window->start();
  const char *key = k == 0 ? "MIMAINPART" : "MOMAINPART";
  ctx->timeline().begin(key, ctx->stream());
  for (uint32_t c = 0; c < s.chunks; ++c) {
    const uint32_t b0 = c * bpc, b1 = std::min(g.blocks, b0 + bpc);
    uint8_t *gc = static_cast<uint8_t *>(s.gcur) + c * perChunk;
    const uint8_t *ge = static_cast<const uint8_t *>(s.gend) + c * perChunk;
    if (b1 > b0)
      kernels::netScatter(s.relation->getData(), n, plan.networkBits, plan.keyShift, g, b0, b1, gc, s.send,
                          ctx->stream(), plan.keyBits, mix, ge, s.narrow ? 1 : 0, !plan.keyOnly, s.roundMeta);
    ctx->readBack(static_cast<uint8_t *>(s.cursorsBack) + c * perChunk, gc, perChunk);
    s.scattered[c] = ctx->acquireEvent();
    HIP_CHECK(hipEventRecord(s.scattered[c], ctx->stream()));
  }
  ctx->timeline().end(key, ctx->stream());
}

bool SampledShuffle::exchangeSide(int k) {
  const uint32_t F = 1u << plan.networkBits, G = CLAIM_GROUPS, N = nodes;
  Side &s = sides[k];
  histograms::ExchangePlan &x = s.xp;
  const histograms::AssignmentMap &am = *hc->assignmentMap();
  const uint32_t C = s.chunks;
  const size_t GF = (size_t)G * F;
  const kernels::WireCodec &codec = s.window->wireCodec();
  const size_t ridChunks = plan.ridBase[k].size() / N;
  JOIN_ASSERT(ridChunks >= C, "SampledShuffle", "rid bases for %zu chunks, %u needed", ridChunks, C);
  std::vector<std::vector<uint32_t>> ownedBy(N);
  for (uint32_t p = 0; p < F; ++p)
    for (uint32_t d = 0; d < N; ++d)
      if (am.owns(p, d)) ownedBy[d].push_back(p);
  // One all-gather per relation, after its whole scatter: every rank's exact
  // fills of every chunk (u32 pairs) + its overflow flag.  (Per-chunk gathers
  // would start the first exchange earlier, but each one waits behind the
  // previous chunk's all-to-allv on the communicator and so leaves a host
  // round trip between consecutive chunks on the links.)
  const size_t cells = (size_t)C * GF, W = (cells + 1) / 2 + 1;
  std::vector<uint64_t> mine(W, 0), all(W * N);
  auto fillOf = [&](uint32_t r, uint32_t c, size_t i) -> uint64_t {
    const size_t j = (size_t)c * GF + i;
    const uint64_t w = all[(size_t)r * W + j / 2];
    return (j & 1) ? (w >> 32) : (w & 0xffffffffull);
  };
  const char *kFlush = k == 0 ? "MIFLUSHPART" : "MOFLUSHPART";
  ctx->timeline().begin(kFlush, ctx->stream());
  utils::waitEvent(s.scattered[C - 1], ctx->comm(), "sampled network scatter");  // one stream: all chunks done
  // Checks raise flags that travel in the fill all-gather instead of throwing
  // here: a rank that threw before the collective would leave its peers
  // blocked in it.  A cell past u32 is an overflow (exact re-run);
  // claims that do not add up to the chunk are an engine fault, raised on
  // every rank after the gather.
  bool over = false;
  uint64_t brokenChunk = 0;  // 1 + the first chunk whose claims do not add up
  {
    const uint32_t *c32 = static_cast<const uint32_t *>(s.cursorsBack);
    const uint64_t *c64 = static_cast<const uint64_t *>(s.cursorsBack);
    const uint64_t n = s.relation->getLocalSize(), span = s.local->geometry().tuplesPerBlock();
    const uint32_t bpc = s.local->blocksPerChunk(), blocks = s.local->geometry().blocks;
    for (uint32_t c = 0; c < C; ++c) {
      uint64_t sum = 0;
      for (size_t i = 0; i < GF; ++i) {
        const size_t at = (size_t)c * GF + i;
        const uint64_t fill = (s.narrow ? c32[at] : c64[at]) - s.start[at];
        over = over || fill > s.cap[at] || fill > 0xffffffffull;  // the fill all-gather packs u32
        sum += fill;
        mine[at / 2] |= std::min<uint64_t>(fill, 0xffffffffull) << (32 * (at & 1));
      }
      const uint64_t b = std::min<uint64_t>(n, (uint64_t)c * bpc * span);
      const uint64_t e = std::min<uint64_t>(n, (uint64_t)std::min<uint32_t>(blocks, (c + 1) * bpc) * span);
      if (sum != e - b && !brokenChunk) brokenChunk = 1 + c;
    }
  }
  mine[W - 1] = (over ? 1 : 0) | (brokenChunk << 1);
  ctx->comm()->allGatherHost(mine.data(), all.data(), W);
  bool anyOver = false;
  for (uint32_t r = 0; r < N; ++r) {
    const uint64_t flags = all[(size_t)r * W + W - 1];
    HJ_CHECK((flags >> 1) == 0, "sampled network pass: rank %u's chunk %lu claims do not add up to its tuples", r,
             (unsigned long)((flags >> 1) - 1));
    anyOver = anyOver || (flags & 1) != 0;
  }
  // Receive totals of every rank vs its window capacity (same verdict everywhere).
  for (uint32_t r = 0; r < N && !anyOver; ++r) {
    uint64_t got = 0;
    for (uint32_t c = 0; c < C; ++c)
      for (uint32_t q : ownedBy[r])
        for (uint32_t src = 0; src < N; ++src)
          if (am.receives(k, src, c, C, q, r))
            for (uint32_t g = 0; g < G; ++g) got += fillOf(src, c, (size_t)g * F + q);
    anyOver = got > s.windowCap[r];
  }
  if (anyOver) {
    ctx->timeline().end(kFlush, ctx->stream());
    return false;
  }
  uint64_t cur = 0;  // window tuples laid out so far
  for (uint32_t c = 0; c < C; ++c) {
    data::Window::SegmentedChunk sc;
    sc.sendMap = s.rm;
    sc.sendWords.assign(N, 0);
    sc.sendDispls.assign(N, 0);
    sc.recvWords.assign(N, 0);
    sc.recvDispls.assign(N, 0);
    // Send side: my filled runs per peer, in the peer's owned-partition order.
    const uint64_t myBase = plan.ridBase[k][(size_t)me * ridChunks + c];
    uint64_t off = 0;
    for (uint32_t p = 0; p < N; ++p) {
      sc.sendDispls[p] = off;
      uint64_t tuples = 0;
      for (uint32_t q : ownedBy[p]) {
        if (!am.receives(k, me, c, C, q, p)) continue;
        for (uint32_t g = 0; g < G; ++g) {
          const size_t at = (size_t)c * GF + (size_t)g * F + q;
          const uint64_t n = fillOf(me, c, (size_t)g * F + q);
          tuples += n;
          if (!n || p == me) continue;
          sc.send.push_back(kernels::WireSeg{s.start[at], off, n, myBase, 0});
          off += codec.w ? codec.words(n) : n;  // raw: the exact run
        }
      }
      sc.sendWords[p] = off - sc.sendDispls[p];
      x.sendCounts[(size_t)c * N + p] = tuples;
    }
    // Receive side: exact window layout of chunk c, source-major, then owned
    // partitions, each partition's G runs back to back (the exact exchange's
    // order, histograms/ExchangePlan.h).
    uint64_t roff = 0;
    for (uint32_t src = 0; src < N; ++src) {
      x.recvDispls[(size_t)c * N + src] = cur;
      if (!codec.w) roff = cur;  // raw: received straight into the window (same run order as the sender's)
      sc.recvDispls[src] = roff;
      const uint64_t base = plan.ridBase[k][(size_t)src * ridChunks + c];
      const uint64_t first = cur;
      for (uint32_t lp = 0; lp < x.owned.size(); ++lp) {
        const uint32_t q = x.owned[lp];
        if (!am.receives(k, src, c, C, q, me)) continue;
        const uint64_t segBegin = cur;
        for (uint32_t g = 0; g < G; ++g) {
          const uint64_t n = fillOf(src, c, (size_t)g * F + q);
          if (!n) continue;
          if (src == me) {
            sc.self.push_back(kernels::WireSeg{s.start[(size_t)c * GF + (size_t)g * F + q], cur, n, 0, 0});
          } else {
            sc.recv.push_back(kernels::WireSeg{cur, roff, n, base, 0});
            roff += codec.w ? codec.words(n) : n;
          }
          cur += n;
        }
        if (cur > segBegin) x.segments.push_back(histograms::Segment{segBegin, cur - segBegin, lp, c, src});
      }
      x.recvCounts[(size_t)c * N + src] = cur - first;
      sc.recvWords[src] = roff - sc.recvDispls[src];
    }
    JOIN_ASSERT(cur <= s.windowCap[me], "SampledShuffle", "window overrun %lu > %lu", (unsigned long)cur,
                (unsigned long)s.windowCap[me]);
    s.window->exchangeSegmented(s.send, c, std::move(sc), s.scattered[c]);
  }
  ctx->timeline().end(kFlush, s.window->completionStream());
  // Segments by partition, then chunk, then source (what the local pass and
  // the chunk views expect).
  std::stable_sort(x.segments.begin(), x.segments.end(), [](const histograms::Segment &a, const histograms::Segment &b) {
    return a.lp != b.lp ? a.lp < b.lp : a.chunk != b.chunk ? a.chunk < b.chunk : a.source < b.source;
  });
  const uint32_t owned = (uint32_t)x.owned.size();
  x.partSize.assign(owned, 0);
  x.lpBase.assign(owned + 1, 0);
  for (const histograms::Segment &sg : x.segments) x.partSize[sg.lp] += sg.len;
  for (uint32_t lp = 0; lp < owned; ++lp) x.lpBase[lp + 1] = x.lpBase[lp] + x.partSize[lp];
  x.recvTotal = cur;
  return true;
}

}  // namespace tasks
}  // namespace hpcjoin
