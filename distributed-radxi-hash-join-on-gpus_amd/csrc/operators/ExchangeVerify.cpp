#include "ExchangeVerify.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../comm/Communicator.h"
#include "../memory/Arena.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace operators {

namespace {

// How the window words of relation `side` hold (mixed key, rid).
kernels::ChecksumFormat formatOf(const core::JoinPlan &plan, int side) {
  kernels::ChecksumFormat f;
  f.bits = plan.networkBits;
  if (plan.wide) {
    f.kind = kernels::ChecksumFormat::Wide;
    f.withRid = 1;
  } else if (plan.keyOnly) {
    f.keyShift = 0;  // value = mk >> bits, no rid
    f.withRid = 0;
  } else {
    f.keyShift = plan.keyShift;
    // Count-only wire codecs carry no rid (the receiver decodes the sender's base).
    f.withRid = (plan.wireBits[side] == 0 || plan.wireRidBits[side] > 0) ? 1 : 0;
  }
  return f;
}

// Input range of exchange chunk c (the scatter's block ranges).
void chunkRange(const histograms::LocalHistogram &lh, uint64_t n, uint32_t c, uint64_t *b, uint64_t *e) {
  const kernels::PartitionGeometry &g = lh.geometry();
  const uint64_t bpc = lh.blocksPerChunk(), span = g.tuplesPerBlock();
  *b = std::min<uint64_t>(n, (uint64_t)c * bpc * span);
  *e = std::min<uint64_t>(n, std::min<uint64_t>(g.blocks, (uint64_t)(c + 1) * bpc) * span);
}

uint64_t hostWindowHash(const void *window, const kernels::ChecksumFormat &f, uint64_t i, uint32_t p) {
  if (f.kind == kernels::ChecksumFormat::Wide) {
    const data::Tuple &t = static_cast<const data::Tuple *>(window)[i];
    return kernels::exchangeHash(t.key, f.withRid ? t.rid : 0);
  }
  const uint64_t v = static_cast<const uint64_t *>(window)[i];
  const uint64_t mk = ((v >> f.keyShift) << f.bits) | p;
  return kernels::exchangeHash(mk, f.withRid ? (v & ((1ull << f.keyShift) - 1)) : 0);
}

}  // namespace

ExchangeCheck verifyExchange(JoinEnv &env, JoinRun &run) {
  core::ExecContext *ctx = env.ctx;
  const core::JoinPlan &plan = env.plan;
  JOIN_ASSERT(run.hc, "verifyExchange", "no histogram state (N > 1 exchanges only)");
  const uint32_t N = env.nodes, F = 1u << plan.networkBits;
  const bool dev = ctx->onDevice();
  const hipStream_t st = ctx->stream();
  histograms::AssignmentMap *am = run.hc->assignmentMap();
  data::Window *wins[2] = {run.inner, run.outer};
  data::Relation *rels[2] = {env.inner, env.outer};
  histograms::LocalHistogram *lhs[2] = {run.hc->innerLocal(), run.hc->outerLocal()};
  // Fault injection: one word of this rank's inner window flipped after it
  // arrived -- the check below must fail (tests/test_failure.py).
  if (utils::faultHit("corrupt_window") && run.inner->computeLocalWindowSize() > 0) {
    if (dev)
      kernels::flipWindowWord(run.inner->getData(), 0, st);
    else
      static_cast<uint64_t *>(run.inner->getData())[0] ^= 0x5A5A5A5A5A5A5A5Aull;
  }
  ExchangeCheck out;
  std::string first;
  for (int k = 0; k < 2; ++k) {
    data::Window *w = wins[k];
    const histograms::ExchangePlan &xp = w->getPlan();
    const uint32_t C = std::max<uint32_t>(1, xp.chunks);
    const kernels::ChecksumFormat fmt = formatOf(plan, k);
    const kernels::KeyMix mix{plan.keyMix ? 1u : 0u, plan.keyBits};
    const uint64_t n = rels[k]->getLocalSize();
    const size_t sentCells = (size_t)C * F, recvCells = (size_t)N * C * F;
    std::vector<uint64_t> sent(sentCells, 0), recv(recvCells, 0);
    std::vector<kernels::ChecksumSeg> segs;
    segs.reserve(xp.segments.size());
    for (const histograms::Segment &s : xp.segments)
      if (s.len)
        segs.push_back(kernels::ChecksumSeg{s.begin, s.len, xp.owned[s.lp],
                                            (uint32_t)(((size_t)s.source * C + s.chunk) * F + xp.owned[s.lp])});
    if (dev) {
      memory::Arena &ws = ctx->workspace();
      auto *dSent = ws.getArray<unsigned long long>(sentCells);
      auto *dRecv = ws.getArray<unsigned long long>(recvCells);
      kernels::zeroWords(dSent, sentCells, st);
      kernels::zeroWords(dRecv, recvCells, st);
      for (uint32_t c = 0; c < C; ++c) {
        uint64_t b, e;
        chunkRange(*lhs[k], n, c, &b, &e);
        kernels::exchangeChecksumSend(rels[k]->getData(), b, e, plan.networkBits, mix, fmt.withRid != 0,
                                      dSent + (size_t)c * F, st);
      }
      auto *dSegs = ws.getArray<kernels::ChecksumSeg>(std::max<size_t>(1, segs.size()));
      ctx->copy(dSegs, segs.data(), segs.size() * sizeof(kernels::ChecksumSeg), true, false);
      kernels::exchangeChecksumRecv(w->getData(), fmt, dSegs, (uint32_t)segs.size(), dRecv, st);
      HIP_CHECK(hipMemcpyAsync(sent.data(), dSent, sentCells * 8, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipMemcpyAsync(recv.data(), dRecv, recvCells * 8, hipMemcpyDeviceToHost, st));
      utils::waitStream(st, ctx->comm(), "exchange verification");
    } else {
      const data::Tuple *in = rels[k]->getData();
      for (uint32_t c = 0; c < C; ++c) {
        uint64_t b, e;
        chunkRange(*lhs[k], n, c, &b, &e);
        for (uint64_t i = b; i < e; ++i) {
          const uint64_t mk = mix.apply(in[i].key);
          sent[(size_t)c * F + (mk & (F - 1))] += kernels::exchangeHash(mk, fmt.withRid ? in[i].rid : 0);
        }
      }
      for (const kernels::ChecksumSeg &s : segs)
        for (uint64_t i = 0; i < s.len; ++i) recv[s.slot] += hostWindowHash(w->getData(), fmt, s.begin + i, s.partition);
    }
    std::vector<uint64_t> sentAll(sentCells * N);
    ctx->comm()->allGatherHost(sent.data(), sentAll.data(), sentCells);
    ctx->comm()->allReduceSumHost(recv.data(), recvCells);
    for (uint32_t src = 0; src < N; ++src)
      for (uint32_t c = 0; c < C; ++c)
        for (uint32_t p = 0; p < F; ++p) {
          uint64_t copies = 0;
          for (uint32_t r = 0; r < N; ++r) copies += am->receives(k, src, c, C, p, r) ? 1 : 0;
          const uint64_t want = sentAll[(size_t)src * sentCells + (size_t)c * F + p] * copies;
          const uint64_t got = recv[((size_t)src * C + c) * F + p];
          ++out.cells;
          if (got != want) {
            if (!out.mismatches)
              first = utils::format("%s relation, source rank %u, chunk %u, partition %u: received hash %016llx, "
                                    "expected %016llx (%llu cop%s)",
                                    k ? "outer" : "inner", src, c, p, (unsigned long long)got,
                                    (unsigned long long)want, (unsigned long long)copies, copies == 1 ? "y" : "ies");
            ++out.mismatches;
          }
        }
  }
  HJ_CHECK(out.mismatches == 0,
           "exchange verification: %llu of %llu (source, chunk, partition) runs did not arrive intact%s; first: %s",
           (unsigned long long)out.mismatches, (unsigned long long)out.cells,
           plan.oneSided ? " (one-sided windows)" : "", first.c_str());
  return out;
}

}  // namespace operators
}  // namespace hpcjoin
