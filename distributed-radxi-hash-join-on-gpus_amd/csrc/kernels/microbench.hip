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
