// Exchange wire codec (kernels.h, WireCodec): bit-packs 8-byte
// CompressedTuples into w-bit wire values before the RCCL all-to-allv and
// unpacks them into the receive window after it.  The reference sends full
// 8-byte CompressedTuples in 64 KB MPI_Puts
// (/root/reference/tasks/NetworkPartitioning.cpp:146-165); on MI355X the
// xGMI links, not HBM, bound the distributed join, so bytes on the wire are
// what to save.
//
// One wave64 per group of 64 tuples.  Pack: lane i encodes tuple i, then lane
// j < w assembles wire word j (stream bits [64j, 64j + 64)) from the <= 3
// (for w >= 32) values that overlap it, fetched with cross-lane shuffles --
// no LDS, no atomics, one coalesced load and one coalesced store per wave.
// Unpack: lane i reads the one or two words holding stream bits
// [iw, iw + w).  Both kernels are HBM streaming kernels (8 B read + w/8 B
// written, or the reverse) that run on their own streams next to RCCL.
#include "device_common.h"
#include "kernels.h"

namespace hpcjoin {
namespace kernels {

namespace {

constexpr uint32_t WIRE_THREADS = 256;
constexpr uint32_t WIRE_WAVES = WIRE_THREADS / WAVE;
constexpr uint32_t WIRE_MAX_SEGS_LDS = 256;

// Segment of global group gi (last segment with group0 <= gi).
__device__ __forceinline__ uint32_t findSeg(const WireSeg *segs, uint32_t nSegs, uint64_t gi) {
  uint32_t lo = 0, hi = nSegs;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (segs[mid].group0 <= gi)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

template <bool kLds>
__device__ __forceinline__ const WireSeg *stageSegs(const WireSeg *segs, uint32_t nSegs, WireSeg *lds) {
  if (!kLds) return segs;
  for (uint32_t i = threadIdx.x; i < nSegs; i += WIRE_THREADS) lds[i] = segs[i];
  __syncthreads();
  return lds;
}

// Every wave walks a contiguous run of `per` groups: one search for its first
// group's segment, then a forward walk.  Segments may be many (the sampled
// N > 1 exchange lists one per (peer, partition, XCD group) slice), so no
// per-group search; a wave's groups are also contiguous in memory.
struct GroupRun {
  uint64_t gi, ge;
  uint32_t si;
  __device__ __forceinline__ GroupRun(const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups, uint64_t per) {
    const uint64_t wave = (uint64_t)blockIdx.x * WIRE_WAVES + threadIdx.x / WAVE;
    gi = wave * per;
    ge = min(totalGroups, gi + per);
    si = gi < ge ? findSeg(segs, nSegs, gi) : 0;
  }
  // Segment of group gi (advanced monotonically).
  __device__ __forceinline__ const WireSeg &seg(const WireSeg *segs, uint32_t nSegs) {
    while (si + 1 < nSegs && segs[si + 1].group0 <= gi) ++si;
    return segs[si];
  }
};

template <bool kLds>
__global__ __launch_bounds__(WIRE_THREADS) void wirePackKernel(const uint64_t *__restrict__ raw,
                                                               uint64_t *__restrict__ wire,
                                                               const WireSeg *__restrict__ gsegs, uint32_t nSegs,
                                                               uint64_t totalGroups, uint64_t per, WireCodec c,
                                                               RoundMap rm) {
  __shared__ WireSeg lds[kLds ? WIRE_MAX_SEGS_LDS : 1];
  const WireSeg *segs = stageSegs<kLds>(gsegs, nSegs, lds);
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t w = c.w;
  const uint64_t wmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
  // Word `lane` of a group starts at stream bit 64*lane: first overlapping value a, offset o in it.
  const uint32_t a = (64u * lane) / w, o = 64u * lane - a * w;
  const uint32_t K = (64u + w - 1) / w + 1;  // values overlapping one word (uniform)
  GroupRun r(segs, nSegs, totalGroups, per);
  for (; r.gi < r.ge; ++r.gi) {
    const WireSeg &sg = r.seg(segs, nSegs);
    const uint64_t g = r.gi - sg.group0, t = g * 64 + lane;
    const uint64_t e = t < sg.n ? (c.encode(raw[rm(sg.raw + t)], sg.base) & wmask) : 0ull;
    uint64_t word = 0;
    for (uint32_t k = 0; k < K; ++k) {
      const uint32_t idx = a + k;
      const uint64_t x = __shfl(e, (int)(idx & (WAVE - 1)), WAVE);
      const int sh = (int)(k * w) - (int)o;  // value idx's bit 0 relative to the word's bit 0
      if (idx < 64) {
        if (sh < 0)
          word |= x >> (-sh);
        else if (sh < 64)
          word |= x << sh;
      }
    }
    if (lane < w) wire[sg.wire + g * w + lane] = word;
  }
}

template <bool kLds>
__global__ __launch_bounds__(WIRE_THREADS) void wireUnpackKernel(const uint64_t *__restrict__ wire,
                                                                 uint64_t *__restrict__ raw,
                                                                 const WireSeg *__restrict__ gsegs, uint32_t nSegs,
                                                                 uint64_t totalGroups, uint64_t per, WireCodec c) {
  __shared__ WireSeg lds[kLds ? WIRE_MAX_SEGS_LDS : 1];
  const WireSeg *segs = stageSegs<kLds>(gsegs, nSegs, lds);
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint32_t w = c.w;
  const uint64_t wmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
  const uint32_t bit0 = lane * w, j0 = bit0 >> 6, o = bit0 & 63;
  const bool two = o + w > 64;
  GroupRun r(segs, nSegs, totalGroups, per);
  for (; r.gi < r.ge; ++r.gi) {
    const WireSeg &sg = r.seg(segs, nSegs);
    const uint64_t g = r.gi - sg.group0, t = g * 64 + lane;
    if (t >= sg.n) continue;
    const uint64_t *gw = wire + sg.wire + g * w;
    uint64_t e = gw[j0] >> o;
    if (two) e |= gw[j0 + 1] << (64 - o);
    raw[sg.raw + t] = c.decode(e & wmask, sg.base);
  }
}

// Raw gather: dst[seg.wire + t] = src[rm(seg.raw + t)] (a rank's own runs,
// which never touch the wire, into its window; or every run into the raw send
// buffer).
template <bool kLds>
__global__ __launch_bounds__(WIRE_THREADS) void segCopyKernel(const uint64_t *__restrict__ src,
                                                              uint64_t *__restrict__ dst,
                                                              const WireSeg *__restrict__ gsegs, uint32_t nSegs,
                                                              uint64_t totalGroups, uint64_t per, RoundMap rm) {
  __shared__ WireSeg lds[kLds ? WIRE_MAX_SEGS_LDS : 1];
  const WireSeg *segs = stageSegs<kLds>(gsegs, nSegs, lds);
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  GroupRun r(segs, nSegs, totalGroups, per);
  for (; r.gi < r.ge; ++r.gi) {
    const WireSeg &sg = r.seg(segs, nSegs);
    const uint64_t t = (r.gi - sg.group0) * 64 + lane;
    if (t < sg.n) dst[sg.wire + t] = __builtin_nontemporal_load(src + rm(sg.raw + t));
  }
}

// Waves of a launch over totalGroups groups (~8 per SIMD of 256 CUs, or one
// per group for small launches) and the groups each walks.
struct WireLaunch {
  uint32_t blocks;
  uint64_t per;
};
WireLaunch wireLaunch(uint64_t totalGroups) {
  const uint64_t maxWaves = 256ull * 4 * 8;
  const uint64_t waves = std::max<uint64_t>(1, std::min<uint64_t>(totalGroups, maxWaves));
  const uint64_t per = ceilDiv(totalGroups, waves);
  return WireLaunch{(uint32_t)ceilDiv(ceilDiv(totalGroups, per), WIRE_WAVES), per};
}

}  // namespace

void wirePack(const uint64_t *raw, uint64_t *wire, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
              const WireCodec &c, hipStream_t s, RoundMap rm) {
  if (totalGroups == 0) return;
  HJ_CHECK(c.w >= 1 && c.w <= 64 && nSegs >= 1, "wirePack: w=%u nSegs=%u", c.w, nSegs);
  const WireLaunch l = wireLaunch(totalGroups);
  if (nSegs <= WIRE_MAX_SEGS_LDS)
    hipLaunchKernelGGL(wirePackKernel<true>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, raw, wire, segs, nSegs,
                       totalGroups, l.per, c, rm);
  else
    hipLaunchKernelGGL(wirePackKernel<false>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, raw, wire, segs, nSegs,
                       totalGroups, l.per, c, rm);
  HIP_CHECK_LAUNCH();
}

void wireUnpack(const uint64_t *wire, uint64_t *raw, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
                const WireCodec &c, hipStream_t s) {
  if (totalGroups == 0) return;
  HJ_CHECK(c.w >= 1 && c.w <= 64 && nSegs >= 1, "wireUnpack: w=%u nSegs=%u", c.w, nSegs);
  const WireLaunch l = wireLaunch(totalGroups);
  if (nSegs <= WIRE_MAX_SEGS_LDS)
    hipLaunchKernelGGL(wireUnpackKernel<true>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, wire, raw, segs, nSegs,
                       totalGroups, l.per, c);
  else
    hipLaunchKernelGGL(wireUnpackKernel<false>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, wire, raw, segs, nSegs,
                       totalGroups, l.per, c);
  HIP_CHECK_LAUNCH();
}

void segCopy(const uint64_t *src, uint64_t *dst, const WireSeg *segs, uint32_t nSegs, uint64_t totalGroups,
             hipStream_t s, RoundMap rm) {
  if (totalGroups == 0) return;
  HJ_CHECK(nSegs >= 1, "segCopy: no segments for %lu groups", (unsigned long)totalGroups);
  const WireLaunch l = wireLaunch(totalGroups);
  if (nSegs <= WIRE_MAX_SEGS_LDS)
    hipLaunchKernelGGL(segCopyKernel<true>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, src, dst, segs, nSegs,
                       totalGroups, l.per, rm);
  else
    hipLaunchKernelGGL(segCopyKernel<false>, dim3(l.blocks), dim3(WIRE_THREADS), 0, s, src, dst, segs, nSegs,
                       totalGroups, l.per, rm);
  HIP_CHECK_LAUNCH();
}

// Loads this file's code object at engine start (kernels::preloadCodeObjects).
void preloadWire() {
  hipFuncAttributes a;
  HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&wirePackKernel<true>)));
}

}  // namespace kernels
}  // namespace hpcjoin
