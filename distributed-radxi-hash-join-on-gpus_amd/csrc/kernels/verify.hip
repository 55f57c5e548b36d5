// Exchange verification (JoinConfig::verifyExchange): content checksums of
// every (source rank, exchange chunk, partition) run, computed on the sender
// from its input and on every receiver from what landed in its window.
//
// The reference's completion check is a count (Window::assertAllTuplesWritten,
// /root/reference/data/Window.cpp:180-191): it compares plan counts and never
// looks at the data, so a put that lands in the wrong place or not at all is
// silent.  Here each tuple contributes exchangeHash(mixed key, rid) (kernels.h)
// to the sum of its run; operators/ExchangeVerify.cpp compares the sums.
#include "kernels.h"
#include "device_common.h"

#include <algorithm>

namespace hpcjoin {
namespace kernels {

constexpr int VT = 256;

// sums[d] += hash of every tuple of in[begin, end) with digit d (F digits).
__global__ __launch_bounds__(VT) void checksumSendKernel(const ulonglong2 *__restrict__ in, uint64_t begin,
                                                          uint64_t end, uint32_t bits, KeyMix mix, uint32_t withRid,
                                                          unsigned long long *__restrict__ sums) {
  extern __shared__ unsigned long long acc[];
  const uint32_t F = 1u << bits;
  for (uint32_t d = threadIdx.x; d < F; d += VT) acc[d] = 0;
  __syncthreads();
  for (uint64_t i = begin + (uint64_t)blockIdx.x * VT + threadIdx.x; i < end; i += (uint64_t)gridDim.x * VT) {
    const ulonglong2 t = in[i];
    const uint64_t mk = mix.apply(t.x);
    atomicAdd(&acc[mk & (F - 1)], (unsigned long long)exchangeHash(mk, withRid ? t.y : 0));
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < F; d += VT)
    if (acc[d]) atomicAdd(&sums[d], acc[d]);
}

void exchangeChecksumSend(const data::Tuple *in, uint64_t begin, uint64_t end, uint32_t bits, KeyMix mix,
                          bool withRid, unsigned long long *sums, hipStream_t s) {
  HJ_CHECK(bits <= MAX_PART_BITS, "exchangeChecksumSend: bits=%u", bits);
  if (end <= begin) return;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (end - begin + VT - 1) / VT);
  hipLaunchKernelGGL(checksumSendKernel, dim3(grid), dim3(VT), (size_t)8 << bits, s,
                     reinterpret_cast<const ulonglong2 *>(in), begin, end, bits, mix, withRid ? 1u : 0u, sums);
  HIP_CHECK_LAUNCH();
}

// One workgroup per segment: sums[seg.slot] += hash of every tuple of the
// window run [seg.begin, seg.begin + seg.len) of partition seg.partition.
__global__ __launch_bounds__(VT) void checksumRecvKernel(const void *__restrict__ window, ChecksumFormat fmt,
                                                          const ChecksumSeg *__restrict__ segs,
                                                          unsigned long long *__restrict__ sums) {
  __shared__ unsigned long long wt[VT / WAVE];
  const ChecksumSeg sg = segs[blockIdx.x];
  unsigned long long mine = 0;
  for (uint64_t i = threadIdx.x; i < sg.len; i += VT) {
    uint64_t mk, rid;
    if (fmt.kind == ChecksumFormat::Wide) {
      const ulonglong2 t = static_cast<const ulonglong2 *>(window)[sg.begin + i];
      mk = t.x;
      rid = t.y;
    } else {
      const uint64_t v = static_cast<const uint64_t *>(window)[sg.begin + i];
      mk = ((v >> fmt.keyShift) << fmt.bits) | sg.partition;
      rid = v & ((1ull << fmt.keyShift) - 1);
    }
    mine += exchangeHash(mk, fmt.withRid ? rid : 0);
  }
  const unsigned long long total = blockReduceSum<VT, unsigned long long>(mine, wt);
  if (threadIdx.x == 0 && total) atomicAdd(&sums[sg.slot], total);
}

void exchangeChecksumRecv(const void *window, const ChecksumFormat &fmt, const ChecksumSeg *segs, uint32_t nSegs,
                          unsigned long long *sums, hipStream_t s) {
  if (nSegs == 0) return;
  hipLaunchKernelGGL(checksumRecvKernel, dim3(nSegs), dim3(VT), 0, s, window, fmt, segs, sums);
  HIP_CHECK_LAUNCH();
}

// One word of the window flipped (fault injection "corrupt_window": the
// verification must catch it).
__global__ void flipWordKernel(uint64_t *p) { *p ^= 0x5A5A5A5A5A5A5A5Aull; }

void flipWindowWord(void *window, uint64_t word, hipStream_t s) {
  hipLaunchKernelGGL(flipWordKernel, dim3(1), dim3(1), 0, s, static_cast<uint64_t *>(window) + word);
  HIP_CHECK_LAUNCH();
}

}  // namespace kernels
}  // namespace hpcjoin
