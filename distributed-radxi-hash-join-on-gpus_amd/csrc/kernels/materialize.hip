// Late materialization kernels (BASELINE config 5: 32-byte payloads).
//
// The join itself moves only 8-byte CompressedTuples (key + rid); payload
// rows stay where they were generated.  After the join, each materialized
// (rid_inner, rid_outer) pair fetches its two rows: requests are bucketed by
// the rank that owns the rid (the same LDS partition kernels, digit = owner),
// exchanged with an RCCL all-to-allv, served by a row gather on the owner,
// exchanged back and placed next to the pair.  Counterpart of the reference's
// dormant result materialization (probe kernels writing (rid, sid) pairs,
// kernels.cu:199-246) extended to distributed payload fetch.
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

constexpr int MT = 256;

static uint32_t gridFor(uint64_t n) {
  const uint64_t b = ceilDiv(n, MT);
  return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);
}

__global__ __launch_bounds__(MT) void generatePayloadKernel(uint64_t *rows, uint64_t n, uint64_t ridOffset,
                                                            uint64_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x; i < n; i += stride) {
    const uint64_t rid = ridOffset + i;
    ulonglong2 a = make_ulonglong2(payloadWord(seed, rid, 0), payloadWord(seed, rid, 1));
    ulonglong2 b = make_ulonglong2(payloadWord(seed, rid, 2), payloadWord(seed, rid, 3));
    reinterpret_cast<ulonglong2 *>(rows)[2 * i] = a;
    reinterpret_cast<ulonglong2 *>(rows)[2 * i + 1] = b;
  }
}

void generatePayload(uint64_t *rows, uint64_t n, uint64_t ridOffset, uint64_t seed, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(generatePayloadKernel, dim3(gridFor(n)), dim3(MT), 0, s, rows, n, ridOffset, seed);
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(MT) void makeRequestsKernel(const ulonglong2 *__restrict__ pairs, uint64_t n, int side,
                                                         uint64_t ridsPerRank, uint32_t nodes,
                                                         ulonglong2 *__restrict__ req) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x; i < n; i += stride) {
    const ulonglong2 p = pairs[i];
    const uint64_t rid = side == 0 ? p.x : p.y;
    uint64_t owner = ridsPerRank ? rid / ridsPerRank : 0;
    if (owner >= nodes) owner = nodes - 1;  // last rank holds the remainder
    req[i] = make_ulonglong2(owner | (i << 8), rid);
  }
}

void makeRequests(const ulonglong2 *pairs, uint64_t n, int side, uint64_t ridsPerRank, uint32_t nodes,
                  ulonglong2 *req, hipStream_t s) {
  if (!n) return;
  HJ_CHECK(nodes <= 256 && n < (1ull << 56), "makeRequests: %u nodes / %lu pairs out of range", nodes,
           (unsigned long)n);
  hipLaunchKernelGGL(makeRequestsKernel, dim3(gridFor(n)), dim3(MT), 0, s, pairs, n, side, ridsPerRank, nodes, req);
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(MT) void splitRequestsKernel(const ulonglong2 *__restrict__ req, uint64_t n,
                                                          uint64_t *__restrict__ rids, uint64_t *__restrict__ idx) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x; i < n; i += stride) {
    const ulonglong2 r = req[i];
    rids[i] = r.y;
    idx[i] = r.x >> 8;
  }
}

void splitRequests(const ulonglong2 *req, uint64_t n, uint64_t *rids, uint64_t *idx, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(splitRequestsKernel, dim3(gridFor(n)), dim3(MT), 0, s, req, n, rids, idx);
  HIP_CHECK_LAUNCH();
}

// One 32-byte row per lane pair: lanes 2j and 2j+1 move the two 16-byte halves
// of row j, so a wave moves 32 rows with 16-byte accesses.
__global__ __launch_bounds__(MT) void gatherRowsKernel(const uint64_t *__restrict__ rids, uint64_t n,
                                                       uint64_t ridOffset, const ulonglong2 *__restrict__ payload,
                                                       ulonglong2 *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t t = (uint64_t)blockIdx.x * MT + threadIdx.x; t < 2 * n; t += stride) {
    const uint64_t j = t >> 1, half = t & 1;
    out[2 * j + half] = payload[2 * (rids[j] - ridOffset) + half];
  }
}

void gatherRows(const uint64_t *rids, uint64_t n, uint64_t ridOffset, const uint64_t *payload, uint64_t *rowsOut,
                hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(gatherRowsKernel, dim3(gridFor(2 * n)), dim3(MT), 0, s, rids, n, ridOffset,
                     reinterpret_cast<const ulonglong2 *>(payload), reinterpret_cast<ulonglong2 *>(rowsOut));
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(MT) void placeRowsKernel(const ulonglong2 *__restrict__ rows,
                                                      const uint64_t *__restrict__ idx, uint64_t n,
                                                      uint64_t *__restrict__ out, uint32_t strideWords,
                                                      uint32_t colWord) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t t = (uint64_t)blockIdx.x * MT + threadIdx.x; t < 2 * n; t += stride) {
    const uint64_t j = t >> 1, half = t & 1;
    const ulonglong2 v = rows[2 * j + half];
    uint64_t *dst = out + idx[j] * strideWords + colWord + 2 * half;
    dst[0] = v.x;
    dst[1] = v.y;
  }
}

void placeRows(const uint64_t *rows, const uint64_t *idx, uint64_t n, uint64_t *out, uint32_t strideWords,
               uint32_t colWord, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(placeRowsKernel, dim3(gridFor(2 * n)), dim3(MT), 0, s, reinterpret_cast<const ulonglong2 *>(rows),
                     idx, n, out, strideWords, colWord);
  HIP_CHECK_LAUNCH();
}

// Single-rank fast path: both payload columns are local, so one pass per pair
// reads the pair, gathers its two 32-byte rows and writes the whole 80-byte
// output row (no request buckets, no intermediate row buffers).
__global__ __launch_bounds__(MT) void materializeLocalKernel(const ulonglong2 *__restrict__ pairs, uint64_t n,
                                                             const ulonglong2 *__restrict__ rowsA, uint64_t offA,
                                                             const ulonglong2 *__restrict__ rowsB, uint64_t offB,
                                                             ulonglong2 *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * MT;
  for (uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x; i < n; i += stride) {
    const ulonglong2 p = pairs[i];
    const uint64_t a = 2 * (p.x - offA), b = 2 * (p.y - offB);
    const ulonglong2 a0 = rowsA[a], a1 = rowsA[a + 1], b0 = rowsB[b], b1 = rowsB[b + 1];
    ulonglong2 *o = out + 5 * i;  // 80-byte row = 5 x 16 bytes
    o[0] = p;
    o[1] = a0;
    o[2] = a1;
    o[3] = b0;
    o[4] = b1;
  }
}

void materializeLocal(const ulonglong2 *pairs, uint64_t n, const uint64_t *rowsA, uint64_t offA,
                      const uint64_t *rowsB, uint64_t offB, uint64_t *out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(materializeLocalKernel, dim3(gridFor(n)), dim3(MT), 0, s, pairs, n,
                     reinterpret_cast<const ulonglong2 *>(rowsA), offA, reinterpret_cast<const ulonglong2 *>(rowsB),
                     offB, reinterpret_cast<ulonglong2 *>(out));
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
