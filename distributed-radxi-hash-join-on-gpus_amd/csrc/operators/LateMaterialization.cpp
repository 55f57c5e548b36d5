#include "LateMaterialization.h"

#include "../performance/Clock.h"

#include <algorithm>
#include <cstring>
#include <vector>

#include "../comm/Communicator.h"
#include "../kernels/kernels.h"
#include "../memory/Arena.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace operators {

using kernels::ROW_WORDS;

LateMaterialization::LateMaterialization(core::ExecContext *ctx, const PayloadColumn &inner,
                                         const PayloadColumn &outer, uint32_t matVariant)
    : ctx(ctx), matVariant(matVariant) {
  cols[0] = inner;
  cols[1] = outer;
}

static uint32_t ownerOf(uint64_t rid, uint64_t ridsPerRank, uint32_t nodes) {
  uint64_t o = ridsPerRank ? rid / ridsPerRank : 0;
  return (uint32_t)std::min<uint64_t>(o, nodes - 1);
}

LateMaterialization::~LateMaterialization() {
  for (auto &side : marks)
    for (hipEvent_t &e : side)
      if (e) (void)hipEventDestroy(e);
}

// After the final synchronisation: phase k of a side = mark k -> mark k + 1.
void LateMaterialization::resolveMarks() {
  double *acc[PHASES] = {&st.bucketMs, &st.requestMs, &st.gatherMs, &st.responseMs, &st.placeMs};
  for (int side = 0; side < 2; ++side) {
    if (!marked[side]) continue;
    for (int k = 0; k < PHASES; ++k) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, marks[side][k], marks[side][k + 1]));
      *acc[k] += ms;
    }
    marked[side] = false;
  }
}

void LateMaterialization::materialize(const ulonglong2 *pairs, uint64_t n, uint64_t *out) {
  static_assert(OUT_WORDS == 2 + 2 * ROW_WORDS, "output row layout");
  if (ctx->onDevice() && ctx->comm()->size() == 1) {
    kernels::materializeLocal(pairs, n, cols[0].rows, cols[0].ridOffset, cols[1].rows, cols[1].ridOffset, out,
                              ctx->stream(), matVariant);
    HIP_CHECK(hipStreamSynchronize(ctx->stream()));
    return;
  }
  for (int side = 0; side < 2; ++side) {
    if (ctx->onDevice())
      fetchDevice(pairs, n, side, cols[side], out);
    else
      fetchHost(pairs, n, side, cols[side], out);
  }
  // rid columns
  if (ctx->onDevice()) {
    if (n)
      HIP_CHECK(hipMemcpy2DAsync(out, OUT_WORDS * 8, pairs, 16, 16, n, hipMemcpyDeviceToDevice, ctx->stream()));
    HIP_CHECK(hipStreamSynchronize(ctx->stream()));
    resolveMarks();
  } else {
    for (uint64_t i = 0; i < n; ++i) {
      out[i * OUT_WORDS] = pairs[i].x;
      out[i * OUT_WORDS + 1] = pairs[i].y;
    }
  }
}

void LateMaterialization::fetchDevice(const ulonglong2 *pairs, uint64_t n, int side, const PayloadColumn &col,
                                      uint64_t *out) {
  comm::Communicator *c = ctx->comm();
  const uint32_t N = c->size(), me = c->rank();
  const uint64_t ridsPerRank = col.globalRows / N;
  hipStream_t s = ctx->stream();
  memory::Arena &ws = ctx->workspace();
  const uint32_t col0 = 2 + side * ROW_WORDS;
  ulonglong2 *req = ws.getArray<ulonglong2>(std::max<uint64_t>(n, 1));
  kernels::makeRequests(pairs, n, side, ridsPerRank, N, req, s);
  uint64_t *rids = ws.getArray<uint64_t>(std::max<uint64_t>(n, 1));
  uint64_t *idx = ws.getArray<uint64_t>(std::max<uint64_t>(n, 1));
  std::vector<uint64_t> sendCounts(N, 0);
  if (N == 1) {
    kernels::splitRequests(req, n, rids, idx, s);
    uint64_t *rows = ws.getArray<uint64_t>(std::max<uint64_t>(n, 1) * ROW_WORDS);
    kernels::gatherRows(rids, n, col.ridOffset, col.rows, rows, s);
    kernels::placeRows(rows, idx, n, out, OUT_WORDS, col0, s);
    return;
  }
  // Bucket requests by owner with the LDS radix kernels (digit = owner).
  // Phase boundaries are timing events on the stream (resolveMarks).
  for (hipEvent_t &e : marks[side])
    if (!e) HIP_CHECK(hipEventCreate(&e));
  int mark = 0;
  auto lap = [&]() { HIP_CHECK(hipEventRecord(marks[side][mark++], s)); };
  lap();
  const uint32_t bits = std::max<uint32_t>(1, ceilLog2(N)), F = 1u << bits;
  const kernels::PartitionGeometry g = kernels::partitionGeometry(n);
  uint32_t *blockHist = ws.getArray<uint32_t>((uint64_t)F * g.blocks);
  uint64_t *totals = ws.getArray<uint64_t>(F);
  ulonglong2 *sorted = ws.getArray<ulonglong2>(std::max<uint64_t>(n, 1));
  std::vector<uint64_t> tot(F, 0), base(F, 0);
  if (n) {
    kernels::netHistogram(reinterpret_cast<const data::Tuple *>(req), n, bits, g, blockHist, s);
    kernels::digitTotals(blockHist, F, g.blocks, g.blocks, 1, totals, s);
    HIP_CHECK(hipMemcpyAsync(tot.data(), totals, F * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (uint32_t d = 1; d < F; ++d) base[d] = base[d - 1] + tot[d - 1];
    uint64_t *baseDev = ws.getArray<uint64_t>(F);
    HIP_CHECK(hipMemcpyAsync(baseDev, base.data(), F * 8, hipMemcpyHostToDevice, s));
    const bool narrow = kernels::cursorsNarrow(n);
    void *gcur = ws.get((uint64_t)kernels::CLAIM_GROUPS * F * (narrow ? 4 : 8));
    kernels::netGroupCursors(blockHist, F, g.blocks, g.blocks, baseDev, gcur, narrow, s);
    kernels::netScatterWide(reinterpret_cast<const data::Tuple *>(req), n, bits, g, 0, g.blocks, gcur,
                            reinterpret_cast<data::Tuple *>(sorted), s);
    kernels::splitRequests(sorted, n, rids, idx, s);
  }
  for (uint32_t d = 0; d < N; ++d) sendCounts[d] = tot[d];
  // request counts -> receive counts
  std::vector<uint64_t> all((size_t)N * N);
  c->allGatherHost(sendCounts.data(), all.data(), N);
  std::vector<uint64_t> recvCounts(N), sd(N, 0), rd(N, 0);
  uint64_t m = 0;
  for (uint32_t r = 0; r < N; ++r) {
    recvCounts[r] = all[(size_t)r * N + me];
    rd[r] = m;
    m += recvCounts[r];
    if (r) sd[r] = sd[r - 1] + sendCounts[r - 1];
  }
  uint64_t *recvRids = ws.getArray<uint64_t>(std::max<uint64_t>(m, 1));
  lap();
  c->allToAllV(rids, sendCounts.data(), sd.data(), recvRids, recvCounts.data(), rd.data(), Location::Device, s);
  lap();
  for (uint32_t r = 0; r < N; ++r)
    if (r != me) {
      st.requestBytes += sendCounts[r] * 8;
      st.responseBytes += recvCounts[r] * ROW_WORDS * 8;
    }
  // serve
  uint64_t *resp = ws.getArray<uint64_t>(std::max<uint64_t>(m, 1) * ROW_WORDS);
  kernels::gatherRows(recvRids, m, col.ridOffset, col.rows, resp, s);
  // rows back: counts x ROW_WORDS words
  std::vector<uint64_t> bsc(N), bsd(N), brc(N), brd(N);
  for (uint32_t r = 0; r < N; ++r) {
    bsc[r] = recvCounts[r] * ROW_WORDS;
    bsd[r] = rd[r] * ROW_WORDS;
    brc[r] = sendCounts[r] * ROW_WORDS;
    brd[r] = sd[r] * ROW_WORDS;
  }
  uint64_t *rowsBack = ws.getArray<uint64_t>(std::max<uint64_t>(n, 1) * ROW_WORDS);
  lap();
  c->allToAllV(resp, bsc.data(), bsd.data(), rowsBack, brc.data(), brd.data(), Location::Device, s);
  lap();
  kernels::placeRows(rowsBack, idx, n, out, OUT_WORDS, col0, s);
  lap();
  marked[side] = true;
}

void LateMaterialization::fetchHost(const ulonglong2 *pairs, uint64_t n, int side, const PayloadColumn &col,
                                    uint64_t *out) {
  comm::Communicator *c = ctx->comm();
  const uint32_t N = c->size(), me = c->rank();
  const uint64_t ridsPerRank = col.globalRows / N;
  const uint32_t col0 = 2 + side * ROW_WORDS;
  std::vector<std::vector<uint64_t>> byOwner(N), idxByOwner(N);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t rid = side == 0 ? pairs[i].x : pairs[i].y;
    const uint32_t o = ownerOf(rid, ridsPerRank, N);
    byOwner[o].push_back(rid);
    idxByOwner[o].push_back(i);
  }
  std::vector<uint64_t> sendRids, sendIdx, sc(N), sd(N);
  for (uint32_t r = 0; r < N; ++r) {
    sd[r] = sendRids.size();
    sc[r] = byOwner[r].size();
    sendRids.insert(sendRids.end(), byOwner[r].begin(), byOwner[r].end());
    sendIdx.insert(sendIdx.end(), idxByOwner[r].begin(), idxByOwner[r].end());
  }
  std::vector<uint64_t> all((size_t)N * N);
  c->allGatherHost(sc.data(), all.data(), N);
  std::vector<uint64_t> rc(N), rd(N);
  uint64_t m = 0;
  for (uint32_t r = 0; r < N; ++r) {
    rc[r] = all[(size_t)r * N + me];
    rd[r] = m;
    m += rc[r];
  }
  std::vector<uint64_t> recvRids(std::max<uint64_t>(m, 1));
  sendRids.resize(std::max<size_t>(sendRids.size(), 1));
  c->allToAllV(sendRids.data(), sc.data(), sd.data(), recvRids.data(), rc.data(), rd.data(), Location::Host, nullptr);
  std::vector<uint64_t> resp(std::max<uint64_t>(m, 1) * ROW_WORDS);
  for (uint64_t j = 0; j < m; ++j)
    std::memcpy(&resp[j * ROW_WORDS], col.rows + (recvRids[j] - col.ridOffset) * ROW_WORDS, ROW_WORDS * 8);
  std::vector<uint64_t> bsc(N), bsd(N), brc(N), brd(N);
  for (uint32_t r = 0; r < N; ++r) {
    bsc[r] = rc[r] * ROW_WORDS;
    bsd[r] = rd[r] * ROW_WORDS;
    brc[r] = sc[r] * ROW_WORDS;
    brd[r] = sd[r] * ROW_WORDS;
  }
  std::vector<uint64_t> back(std::max<uint64_t>(n, 1) * ROW_WORDS);
  c->allToAllV(resp.data(), bsc.data(), bsd.data(), back.data(), brc.data(), brd.data(), Location::Host, nullptr);
  for (uint64_t j = 0; j < n; ++j)
    std::memcpy(out + sendIdx[j] * OUT_WORDS + col0, &back[j * ROW_WORDS], ROW_WORDS * 8);
}

}  // namespace operators
}  // namespace hpcjoin
