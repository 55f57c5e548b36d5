// Counter-based generators shared by the HIP datagen kernels and the host
// reference path (bit-identical on both, so host and device relations match).
//
// The reference builds unique keys with a sequential Sattolo-style shuffle plus
// an MPI pairwise swap (/root/reference/data/Relation.cpp:63-141).  On the GPU
// that is replaced by a keyed Feistel bijection over [0, domain) evaluated per
// element with cycle walking: rank r simply evaluates its slice of ONE global
// permutation, so no shuffle and no distribute() exchange is needed.
#pragma once

#include "../core/Types.h"

namespace hpcjoin {
namespace kernels {

HJ_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

struct FeistelPermutation {
  uint64_t domain;
  uint32_t halfBits;
  uint64_t halfMask;
  uint64_t roundKey[4];

  static FeistelPermutation make(uint64_t domain, uint64_t seed) {
    FeistelPermutation p;
    p.domain = domain < 1 ? 1 : domain;
    uint32_t bits = ceilLog2(p.domain);
    p.halfBits = (bits + 1) / 2;
    if (p.halfBits == 0) p.halfBits = 1;
    p.halfMask = (uint64_t(1) << p.halfBits) - 1;
    uint64_t s = seed * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL;
    for (int r = 0; r < 4; ++r) {
      s = mix64(s + 0x9E3779B97F4A7C15ULL * (r + 1));
      p.roundKey[r] = s;
    }
    return p;
  }

  HJ_HD uint64_t once(uint64_t x) const {
    uint64_t L = x >> halfBits, R = x & halfMask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint64_t f = mix64(R ^ roundKey[r]) & halfMask;
      uint64_t nl = R;
      R = L ^ f;
      L = nl;
    }
    return (L << halfBits) | R;
  }

  // Bijection on [0, domain): cycle-walk until the image falls in range.
  HJ_HD uint64_t operator()(uint64_t i) const {
    uint64_t x = i;
    do {
      x = once(x);
    } while (x >= domain);
    return x;
  }
};

HJ_HD double uniform01(uint64_t seed, uint64_t i) {
  return double(mix64(seed ^ mix64(i + 0x5851F42D4C957F2DULL)) >> 11) * (1.0 / 9007199254740992.0);
}

// Zipf(theta) over ranks [0, n): Gray et al., "Quickly generating billion-record
// synthetic databases" (SIGMOD'94).  zetan is precomputed on the host.
struct ZipfParams {
  uint64_t n;
  double theta, alpha, zetan, eta, half_pow_theta;
};

}  // namespace kernels
}  // namespace hpcjoin
