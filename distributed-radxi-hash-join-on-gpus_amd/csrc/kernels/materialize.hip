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

#include <cstdlib>

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
//
// A wave owns 64 consecutive pairs per step.  Gathers go by lane pairs: lanes
// 2j and 2j+1 read the two 16-byte halves of one row, so each load instruction
// touches 32 whole rows instead of 64 half rows.  The 64 output rows (5 KiB,
// contiguous in the output) are assembled in a wave-private LDS buffer and
// written by 5 instructions of 64 consecutive 16-byte pieces.  The direct form
// (5 stores per lane at an 80-byte lane stride) cost 43.9 ms for the SF100
// 600M pairs (profiles/r1_tpch_sf100_kernel_stats.md).
constexpr int MAT_WAVES = MT / 64;
using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));

// NT: non-temporal output stores.  XCD: the grid's 8 XCD groups (blockIdx % 8)
// each walk one contiguous eighth of the pairs, so the ~4 pairs that share an
// inner row (one build/probe item) are served from one XCD's L2.  Measured on
// SF100: direct stores 42.3 ms, LDS-staged 39.3, + XCD walk 38.6 (variants
// without NT within 1%); the rest is the random 32-byte row gathers, fetched
// as 64-byte requests (FETCH_SIZE 89 GB for 600M pairs).
// BNT: the lineitem-side (B) rows, each read once at a random position, are
// loaded non-temporally so their lines do not push the ~4x-reused inner (A)
// rows out of the XCD's L2 (FETCH_SIZE showed 64 B fetched per A access: no
// reuse survived the B stream).  Write-through (`sc1`, `sc1 nt`) output
// stores that leave L2 at once measured no faster (31.5 / 31.0 vs 30.9 ms).
template <bool NT, bool XCD, bool BNT = false>
__global__ __launch_bounds__(MT) void materializeLocalKernel(const ulonglong2 *__restrict__ pairs, uint64_t n,
                                                             const ulonglong2 *__restrict__ rowsA, uint64_t offA,
                                                             const ulonglong2 *__restrict__ rowsB, uint64_t offB,
                                                             ulonglong2 *__restrict__ out) {
  __shared__ ulonglong2 stage[MAT_WAVES][5 * 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  ulonglong2 *w = stage[wave];
  const uint64_t steps = ceilDiv(n, 64);
  uint64_t first = (uint64_t)blockIdx.x * MAT_WAVES + wave, last = steps, waveStride = (uint64_t)gridDim.x * MAT_WAVES;
  if (XCD) {  // gridDim.x % 8 == 0: XCD x = blockIdx % 8 walks the x-th eighth of the steps
    const uint32_t x = blockIdx.x & 7;
    const uint64_t seg0 = steps * x / 8;
    last = steps * (x + 1) / 8;
    first = seg0 + (uint64_t)(blockIdx.x >> 3) * MAT_WAVES + wave;
    waveStride = (uint64_t)(gridDim.x >> 3) * MAT_WAVES;
  }
  for (uint64_t st = first; st < last; st += waveStride) {
    const uint64_t base = st * 64;
    const uint32_t m = (uint32_t)(n - base < 64 ? n - base : 64);
    const ulonglong2 p = lane < m ? pairs[base + lane] : make_ulonglong2(offA, offB);
    const uint32_t half = lane & 1;
    ulonglong2 ra[2], rb[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t j = (lane >> 1) + 32 * k;  // pair whose row half this lane moves
      const uint64_t x = __shfl(p.x, j, 64), y = __shfl(p.y, j, 64);
      if (j < m) {
        ra[k] = rowsA[2 * (x - offA) + half];
        if (BNT) {
          const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(rowsB + 2 * (y - offB) + half));
          rb[k] = make_ulonglong2(v.x, v.y);
        } else {
          rb[k] = rowsB[2 * (y - offB) + half];
        }
      }
    }
    w[5 * lane] = p;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t j = (lane >> 1) + 32 * k;
      w[5 * j + 1 + half] = ra[k];
      w[5 * j + 3 + half] = rb[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ulonglong2 *o = out + 5 * base;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint32_t q = 64 * k + lane;
      if (q < 5 * m) {
        const ulonglong2 v = w[q];
        if (NT) {
          const u64x2 vv = {v.x, v.y};
          __builtin_nontemporal_store(vv, reinterpret_cast<u64x2 *>(o + q));
        } else {
          o[q] = v;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

void materializeLocal(const ulonglong2 *pairs, uint64_t n, const uint64_t *rowsA, uint64_t offA,
                      const uint64_t *rowsB, uint64_t offB, uint64_t *out, hipStream_t s, uint32_t variant) {
  if (!n) return;
  const uint64_t blocks = ceilDiv(ceilDiv(n, 64), MAT_WAVES);
  const uint32_t grid = (uint32_t)(blocks < 8192 ? (blocks + 7) / 8 * 8 : 8192);
  const auto *ra = reinterpret_cast<const ulonglong2 *>(rowsA);
  const auto *rb = reinterpret_cast<const ulonglong2 *>(rowsB);
  auto *o = reinterpret_cast<ulonglong2 *>(out);
  switch (variant) {  // sweep: NT stores / non-temporal B loads
    case 0: hipLaunchKernelGGL((materializeLocalKernel<true, true, false>), dim3(grid), dim3(MT), 0, s, pairs, n, ra, offA, rb, offB, o); break;
    case 2: hipLaunchKernelGGL((materializeLocalKernel<false, true, true>), dim3(grid), dim3(MT), 0, s, pairs, n, ra, offA, rb, offB, o); break;
    case 3: hipLaunchKernelGGL((materializeLocalKernel<false, true, false>), dim3(grid), dim3(MT), 0, s, pairs, n, ra, offA, rb, offB, o); break;
    default: hipLaunchKernelGGL((materializeLocalKernel<true, true, true>), dim3(grid), dim3(MT), 0, s, pairs, n, ra, offA, rb, offB, o); break;
  }
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadMaterialize() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&generatePayloadKernel)));
}

}  // namespace kernels
}  // namespace hpcjoin
