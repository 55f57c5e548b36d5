// Streaming micro-kernels used by the phase micro-benchmarks (the analog of
// the reference's UVA_benchmark / shared_memory_PT drivers,
// /root/reference/operators/gpu/small_data_optimized.cu:254-399,1664-1729):
// 16-byte-per-lane copy and read give the HBM ceiling the partition kernels
// are judged against.
#include "kernels.h"
#include "device_common.h"

namespace hpcjoin {
namespace kernels {

__global__ __launch_bounds__(256) void copyKernelImpl(const ulonglong2 *__restrict__ in, ulonglong2 *__restrict__ out,
                                                      uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

__global__ __launch_bounds__(256) void readKernelImpl(const ulonglong2 *__restrict__ in, uint64_t n,
                                                      unsigned long long *sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const ulonglong2 v = in[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x9E3779B97F4A7C15ull) *sink = acc;  // keeps the loads live
}

// Stream-mix ceiling of a pass's exact byte mix (tools/stream_mix_bench.py):
// up to two read streams of RA / RB bytes per element and two write streams
// of WA / WB bytes per element, all in order, no partitioning.  A lane moves
// 8 elements per step as 16-byte vectors (8 x RA / 16 loads of stream A, ...),
// so every stream is read / written with the widest access whatever its
// element size; written words are XORs of read words (nothing folds away).
using mixv = unsigned int __attribute__((ext_vector_type(4)));
// A wave moves 512 elements per step: stream A's 512 x RA bytes are LA x 64
// 16-byte vectors, vector k * 64 + lane of the wave's block -- every load and
// store instruction is 64 consecutive 16-byte vectors (1 KiB, coalesced).
template <int RA, int RB, int WA, int WB>
__global__ __launch_bounds__(256) void streamMixKernel(const mixv *__restrict__ a, const mixv *__restrict__ b,
                                                       mixv *__restrict__ wa, mixv *__restrict__ wb, uint64_t steps,
                                                       unsigned long long *sink) {
  constexpr int LA = RA / 2, LB = RB / 2, SA = WA / 2, SB = WB / 2;  // 16-byte vectors per lane and step
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (256 / WAVE);
  mixv acc = {0, 0, 0, 0};
  for (uint64_t w = (uint64_t)blockIdx.x * (256 / WAVE) + threadIdx.x / WAVE; w < steps; w += waves) {
    mixv x = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < LA; ++k) x ^= __builtin_nontemporal_load(a + (w * LA + k) * WAVE + lane);
#pragma unroll
    for (int k = 0; k < LB; ++k) x ^= __builtin_nontemporal_load(b + (w * LB + k) * WAVE + lane);
#pragma unroll
    for (int k = 0; k < SA; ++k) wa[(w * SA + k) * WAVE + lane] = x + (unsigned)k;
#pragma unroll
    for (int k = 0; k < SB; ++k) wb[(w * SB + k) * WAVE + lane] = x - (unsigned)k;
    acc ^= x;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) *sink = acc.x;  // keeps read-only mixes live
}

void streamMix(int ra, int rb, int wa, int wb, const void *a, const void *b, void *oa, void *ob, uint64_t n,
               unsigned long long *sink, hipStream_t s) {
  const uint64_t steps = n / 512;  // wave steps of 512 elements
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ceilDiv(steps, 256 / WAVE), 256 * 16);
#define HJ_MIX(RA, RB, WA, WB)                                                                                    \
  if (ra == RA && rb == RB && wa == WA && wb == WB) {                                                             \
    hipLaunchKernelGGL((streamMixKernel<RA, RB, WA, WB>), dim3(grid), dim3(256), 0, s, (const mixv *)a,          \
                       (const mixv *)b, (mixv *)oa, (mixv *)ob, steps, sink);                                  \
    HIP_CHECK_LAUNCH();                                                                                            \
    return;                                                                                                        \
  }
  HJ_MIX(16, 0, 8, 0)  // general-path network pass: tuple in, key-only word out
  HJ_MIX(16, 0, 4, 0)  // count-only network pass: tuple in, u32 fragment out
  HJ_MIX(16, 0, 16, 0) // copy
  HJ_MIX(8, 0, 4, 2)   // split local pass: key-only word in, u32 + u16 columns out
  HJ_MIX(8, 0, 8, 0)   // unsplit local pass
  HJ_MIX(4, 0, 2, 0)   // fragment local pass (two-level fragments)
  HJ_MIX(4, 2, 0, 0)   // key-only build/probe: u32 + u16 columns read
  HJ_MIX(4, 0, 0, 0)   // bitmap join: u32 fragments read
  HJ_MIX(2, 0, 0, 0)   // direct-count build/probe: u16 column read
  HJ_MIX(16, 0, 0, 0)  // read only
#undef HJ_MIX
  HJ_CHECK(false, "streamMix: no instantiation for read %d+%d / write %d+%d bytes", ra, rb, wa, wb);
}

// Random 32-byte row gather shapes (tools/gather_bench.py): MODE 0 a lane
// per 16-byte half row; 1 a lane per whole row (two loads); 2 as 0 with four
// rows per lane pair in flight; 3 as 0 with non-temporal loads.
using gx2 = unsigned long long __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(256) void gatherVariantKernel(const uint64_t *__restrict__ rids, uint64_t n,
                                                           const ulonglong2 *__restrict__ rows,
                                                           ulonglong2 *__restrict__ out) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  if constexpr (MODE == 1) {
    for (uint64_t j = tid; j < n; j += stride) {
      const uint64_t r = rids[j];
      const ulonglong2 a = rows[2 * r], b = rows[2 * r + 1];
      out[2 * j] = a;
      out[2 * j + 1] = b;
    }
  } else if constexpr (MODE == 2) {
    // lane pair p handles rows 4p .. 4p+3 of each 4-row group step
    for (uint64_t t = tid; t < 2 * ((n + 3) / 4); t += stride) {
      const uint64_t g = t >> 1, half = t & 1;
      ulonglong2 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t j = 4 * g + k;
        if (j < n) v[k] = rows[2 * rids[j] + half];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t j = 4 * g + k;
        if (j < n) out[2 * j + half] = v[k];
      }
    }
  } else {
    for (uint64_t t = tid; t < 2 * n; t += stride) {
      const uint64_t j = t >> 1, half = t & 1;
      if constexpr (MODE == 3) {
        const gx2 x = __builtin_nontemporal_load(reinterpret_cast<const gx2 *>(rows + 2 * rids[j] + half));
        out[2 * j + half] = make_ulonglong2(x.x, x.y);
      } else {
        out[2 * j + half] = rows[2 * rids[j] + half];
      }
    }
  }
}

void gatherVariant(int mode, const uint64_t *rids, uint64_t n, const ulonglong2 *rows, ulonglong2 *out,
                   hipStream_t s) {
  const uint32_t grid = 256 * 8;
  switch (mode) {
    case 1: hipLaunchKernelGGL(gatherVariantKernel<1>, dim3(grid), dim3(256), 0, s, rids, n, rows, out); break;
    case 2: hipLaunchKernelGGL(gatherVariantKernel<2>, dim3(grid), dim3(256), 0, s, rids, n, rows, out); break;
    case 3: hipLaunchKernelGGL(gatherVariantKernel<3>, dim3(grid), dim3(256), 0, s, rids, n, rows, out); break;
    default: hipLaunchKernelGGL(gatherVariantKernel<0>, dim3(grid), dim3(256), 0, s, rids, n, rows, out); break;
  }
  HIP_CHECK_LAUNCH();
}

// Streaming ceiling of the count-only network pass's byte mix: read a
// 16-byte tuple, write a 4-byte fragment (no partitioning), IPT tuples per
// thread per step.
template <int IPT>
__global__ __launch_bounds__(256) void projectKeysKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                         uint32_t shift, uint32_t *__restrict__ out) {
  const uint64_t step = (uint64_t)gridDim.x * 256 * IPT;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * IPT + threadIdx.x; b < n; b += step) {
    ulonglong2 v[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (b + (uint64_t)k * 256 < n) v[k] = in[b + (uint64_t)k * 256];
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (b + (uint64_t)k * 256 < n) out[b + (uint64_t)k * 256] = (uint32_t)(v[k].x >> shift);
  }
}

void projectKeys(const ulonglong2 *in, uint64_t n, uint32_t shift, uint32_t *out, int ipt, hipStream_t s) {
  const uint32_t grid = 256 * 8;
  switch (ipt) {
    case 1: hipLaunchKernelGGL(projectKeysKernel<1>, dim3(grid), dim3(256), 0, s, in, n, shift, out); break;
    case 4: hipLaunchKernelGGL(projectKeysKernel<4>, dim3(grid), dim3(256), 0, s, in, n, shift, out); break;
    default: hipLaunchKernelGGL(projectKeysKernel<8>, dim3(grid), dim3(256), 0, s, in, n, shift, out); break;
  }
  HIP_CHECK_LAUNCH();
}

// Probe ceiling of a whole-key-space bitmap kept in the Infinity Cache: every
// tuple's key tests one bit of a 2^bits-bit global bitmap (random 4-byte
// reads), keys streamed from 16-byte tuples, IPT tuples in flight per lane.
template <int IPT>
__global__ __launch_bounds__(256) void probeBitmapGlobalKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                               const uint32_t *__restrict__ bm, uint64_t keyMask,
                                                               unsigned long long *count) {
  const uint64_t step = (uint64_t)gridDim.x * 256 * IPT;
  uint32_t c = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * IPT + threadIdx.x; b < n; b += step) {
    uint64_t k[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) k[j] = b + (uint64_t)j * 256 < n ? (in[b + (uint64_t)j * 256].x & keyMask) : 0;
    uint32_t w[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) w[j] = bm[k[j] >> 5];
#pragma unroll
    for (int j = 0; j < IPT; ++j) c += (b + (uint64_t)j * 256 < n) ? (w[j] >> (k[j] & 31)) & 1u : 0u;
  }
  c = waveReduceSum<uint32_t>(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, (unsigned long long)c);
}

void probeBitmapGlobal(const ulonglong2 *in, uint64_t n, const uint32_t *bm, uint64_t keyMask,
                       unsigned long long *count, int ipt, hipStream_t s) {
  const uint32_t grid = 256 * 16;
  if (ipt == 16)
    hipLaunchKernelGGL(probeBitmapGlobalKernel<16>, dim3(grid), dim3(256), 0, s, in, n, bm, keyMask, count);
  else
    hipLaunchKernelGGL(probeBitmapGlobalKernel<8>, dim3(grid), dim3(256), 0, s, in, n, bm, keyMask, count);
  HIP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void keyRidMaxKernel(const ulonglong2 *__restrict__ in, uint64_t n,
                                                       unsigned long long *out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  unsigned long long k = 0, r = 0, rmin = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const ulonglong2 v = in[i];
    k = v.x > k ? v.x : k;
    r = v.y > r ? v.y : r;
    rmin = v.y < rmin ? v.y : rmin;
  }
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) {
    const unsigned long long k2 = __shfl_xor(k, o, WAVE), r2 = __shfl_xor(r, o, WAVE),
                             m2 = __shfl_xor(rmin, o, WAVE);
    k = k2 > k ? k2 : k;
    r = r2 > r ? r2 : r;
    rmin = m2 < rmin ? m2 : rmin;
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    atomicMax(&out[0], k);
    atomicMax(&out[1], r);
    atomicMin(&out[2], rmin);
  }
}

// Plan-time duplicate probe of the inner keys (HashJoin::makeJoinPlan, for
// relations whose generator did not say): S keys at evenly spaced positions
// go into a global open-addressing set of 2^tbits >= 2S entries (CAS); a key
// that finds itself already there counts one repeat.  ~0 (the empty marker)
// is skipped.  One launch, no sort, ~20 us for 64K samples.
__global__ __launch_bounds__(256) void sampleRepeatsKernel(const ulonglong2 *__restrict__ in, uint64_t n, uint32_t S,
                                                           unsigned long long *__restrict__ set, uint32_t tbits,
                                                           unsigned int *__restrict__ repeats) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= S) return;
  const unsigned long long key = in[(uint64_t)((unsigned __int128)i * n / S)].x;
  if (key == ~0ull) return;
  const uint32_t mask = (1u << tbits) - 1;
  uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tbits));
  for (uint32_t w = 0; w <= mask; ++w) {  // 2^tbits >= 2S: an empty entry is always reached
    const unsigned long long o = atomicCAS(&set[h], ~0ull, key);
    if (o == ~0ull) return;
    if (o == key) {
      atomicAdd(repeats, 1u);
      return;
    }
    h = (h + 1) & mask;
  }
}

size_t sampleRepeatsBytes(uint32_t S) { return ((size_t)8 << ceilLog2(2ull * std::max<uint32_t>(S, 1))) + 16; }

void sampleRepeats(const data::Tuple *in, uint64_t n, uint32_t S, void *ws, unsigned int *repeats, hipStream_t s) {
  if (n == 0 || S == 0) return;
  const uint32_t tbits = ceilLog2(2ull * S);
  auto *set = static_cast<unsigned long long *>(ws);
  HIP_CHECK(hipMemsetAsync(set, 0xFF, (size_t)8 << tbits, s));
  HIP_CHECK(hipMemsetAsync(repeats, 0, sizeof(unsigned int), s));
  hipLaunchKernelGGL(sampleRepeatsKernel, dim3(ceilDiv(S, 256)), dim3(256), 0, s,
                     reinterpret_cast<const ulonglong2 *>(in), n, S, set, tbits, repeats);
  HIP_CHECK_LAUNCH();
}

void keyRidMax(const data::Tuple *in, uint64_t n, unsigned long long *out, hipStream_t s) {
  if (n == 0) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceilDiv(n, 256), 2048);
  hipLaunchKernelGGL(keyRidMaxKernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const ulonglong2 *>(in), n,
                     out);
  HIP_CHECK_LAUNCH();
}

void copyKernel(const ulonglong2 *in, ulonglong2 *out, uint64_t n16, hipStream_t s) {
  hipLaunchKernelGGL(copyKernelImpl, dim3(4096), dim3(256), 0, s, in, out, n16);
  HIP_CHECK_LAUNCH();
}

void readKernel(const ulonglong2 *in, uint64_t n16, unsigned long long *sink, hipStream_t s) {
  hipLaunchKernelGGL(readKernelImpl, dim3(4096), dim3(256), 0, s, in, n16, sink);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
