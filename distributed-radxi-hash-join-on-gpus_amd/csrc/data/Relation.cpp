#include "Relation.h"

#include <algorithm>
#include <cstring>
#include <vector>

#include "../comm/Communicator.h"
#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../memory/Pool.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace data {

using kernels::KeyDistribution;

Relation::Relation(uint64_t localSize, uint64_t globalSize)
    : localSize(localSize), globalSize(globalSize), loc_(Location::Host), device_(0), owns_(true), fromPool_(true) {
  data = static_cast<Tuple *>(memory::Pool::getMemory(localSize * sizeof(Tuple)));
  std::memset(data, 0, localSize * sizeof(Tuple));
}

Relation::Relation(uint64_t localSize, uint64_t globalSize, Location loc, int device)
    : localSize(localSize), globalSize(globalSize), loc_(loc), device_(device), owns_(true), fromPool_(false) {
  data = static_cast<Tuple *>(memory::Arena::rawAlloc(loc, localSize * sizeof(Tuple), device));
}

Relation::Relation(Tuple *external, uint64_t localSize, uint64_t globalSize, Location loc, int device)
    : localSize(localSize), globalSize(globalSize), data(external), loc_(loc), device_(device), owns_(false),
      fromPool_(false) {}

Relation::~Relation() {
  // Pool memory is released by Pool::freeAll (the reference freed it here).
  if (owns_ && !fromPool_) memory::Arena::rawFree(loc_, data);
}

uint64_t Relation::getLocalSize() { return localSize; }
uint64_t Relation::getGlobalSize() { return globalSize; }
Tuple *Relation::getData() { return data; }

uint64_t Relation::localSizeFor(uint64_t globalSize, uint32_t nodeId, uint32_t numberOfNodes) {
  // Same split as /root/reference/main.cpp:73-79: the last rank takes the remainder.
  const uint64_t base = globalSize / numberOfNodes;
  return nodeId < numberOfNodes - 1 ? base : globalSize - (uint64_t)(numberOfNodes - 1) * base;
}

uint64_t Relation::localOffsetFor(uint64_t globalSize, uint32_t nodeId, uint32_t numberOfNodes) {
  return (uint64_t)nodeId * (globalSize / numberOfNodes);
}

static void runGenerate(Tuple *out, uint64_t n, const kernels::GenParams &p, Location loc, int device) {
  if (deviceAccessible(loc)) {  // pinned: the GPU writes host memory over the host link
    HIP_CHECK(hipSetDevice(device));
    kernels::generate(out, n, p, nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::generate(out, n, p);
  }
}

void Relation::fillUniqueValues(uint64_t startKeyValue, uint64_t startRidValue) {
  kernels::GenParams p;
  p.dist = KeyDistribution::Unique;
  p.globalOffset = 0;
  p.ridOffset = startRidValue;
  p.keyOffset = startKeyValue;
  p.domain = localSize;
  p.perm = kernels::FeistelPermutation::make(localSize, 1234 + startKeyValue * 7 + startRidValue);
  runGenerate(data, localSize, p, loc_, device_);
  maxKey_ = startKeyValue + (localSize ? localSize - 1 : 0);
  setGenerated(startRidValue, true);
  keyRepeats_ = 0;  // unique here; other ranks' slices may overlap (the reference fills per rank)
}

void Relation::fillModuloValues(uint64_t startKeyValue, uint64_t startRidValue, uint64_t innerRelationSize) {
  JOIN_ASSERT(innerRelationSize > 0, "Relation", "modulo size must be > 0");
  kernels::GenParams p;
  p.dist = KeyDistribution::Modulo;
  p.ridOffset = startRidValue;
  p.keyOffset = startKeyValue;
  p.modulo = innerRelationSize;
  p.domain = innerRelationSize;
  p.perm = kernels::FeistelPermutation::make(innerRelationSize, 4321 + startKeyValue);
  runGenerate(data, localSize, p, loc_, device_);
  maxKey_ = startKeyValue + innerRelationSize - 1;
  setGenerated(startRidValue, true);
  keyRepeats_ = localSize > innerRelationSize ? 2 : 0;
}

void Relation::generate(const GenSpec &spec, uint64_t globalOffset) {
  kernels::GenParams p;
  p.dist = spec.distribution;
  p.globalOffset = globalOffset;
  p.ridOffset = globalOffset;
  p.keyOffset = spec.keyOffset;
  p.domain = spec.domain ? spec.domain : globalSize;
  p.modulo = p.domain;
  p.seed = spec.seed;
  p.perm = kernels::FeistelPermutation::make(p.domain, spec.seed);
  if (spec.distribution == KeyDistribution::Zipf) p.zipf = host::makeZipf(p.domain, spec.zipfTheta);
  p.tpchSparse = spec.tpchSparse;
  p.sparse64 = spec.sparse64;
  runGenerate(data, localSize, p, loc_, device_);
  maxKey_ = spec.keyOffset + (spec.distribution == KeyDistribution::Dense ? globalSize : p.domain) - 1;
  if (spec.tpchSparse) maxKey_ = kernels::tpchSparseKey(maxKey_);
  if (spec.sparse64) maxKey_ = kernels::SPARSE_KEY_MAX;
  // Keys are permutations / draws over a dense domain (or a bijective mix of
  // one): uniform low bits.  The TPC-H layout leaves digits empty.
  setGenerated(globalOffset, !spec.tpchSparse);
  // Unique / dense draws are a permutation of the domain; uniform and Zipf
  // draws repeat keys once the birthday bound is passed (G^2 > 2 domain);
  // modulo keys once the relation is larger than the domain.
  const double G = (double)globalSize, D = (double)p.domain;
  switch (spec.distribution) {
    case KeyDistribution::Unique:
    case KeyDistribution::Dense: keyRepeats_ = globalSize <= p.domain || spec.distribution == KeyDistribution::Dense ? 1 : 0; break;
    case KeyDistribution::Modulo: keyRepeats_ = globalSize > p.domain ? 2 : 1; break;
    default: keyRepeats_ = G * G > 2.0 * D ? 2 : 0; break;
  }
}

void Relation::inheritBounds(const Relation &parent, uint64_t maxKey, uint64_t ridMax) {
  keyBoundKnown_ = true;
  maxKey_ = maxKey;
  ridsPositional_ = false;
  ridBoundKnown_ = true;
  ridMax_ = ridMax;
  lowBitsUniform_ = parent.lowBitsUniform_;
  keyRepeats_ = parent.keyRepeats_;
}

void Relation::setGenerated(uint64_t ridBase, bool lowBitsUniform) {
  keyBoundKnown_ = true;
  ridsPositional_ = true;
  ridBase_ = ridBase;
  lowBitsUniform_ = lowBitsUniform;
}

uint64_t Relation::expectedMatches(const GenSpec &inner, uint64_t innerGlobal, const GenSpec &outer,
                                   uint64_t outerGlobal) {
  if (inner.tpchSparse != outer.tpchSparse || inner.sparse64 != outer.sparse64)
    return UINT64_MAX;  // the key transforms must match
  const uint64_t innerDomain = inner.domain ? inner.domain : innerGlobal;
  const bool innerIsKeySet = (inner.distribution == KeyDistribution::Unique ||
                              inner.distribution == KeyDistribution::Dense) &&
                             innerDomain == innerGlobal;
  if (!innerIsKeySet) return UINT64_MAX;  // inner = every key of [off, off + G_R) exactly once
  const uint64_t lo = inner.keyOffset, hi = inner.keyOffset + innerGlobal;
  const uint64_t outerDomain = outer.domain ? outer.domain : outerGlobal;
  const uint64_t olo = outer.keyOffset, ohi = outer.keyOffset + outerDomain;
  switch (outer.distribution) {
    case KeyDistribution::Unique:
    case KeyDistribution::Dense:
      // every outer key of [olo, ohi) once
      if (outerDomain != outerGlobal) return UINT64_MAX;
      return std::min(hi, ohi) > std::max(lo, olo) ? std::min(hi, ohi) - std::max(lo, olo) : 0;
    case KeyDistribution::Modulo:
    case KeyDistribution::Uniform:
    case KeyDistribution::Zipf:
      // foreign keys drawn from the outer domain: all match when it lies inside the inner key set
      if (olo >= lo && ohi <= hi) return outerGlobal;
      return UINT64_MAX;
  }
  return UINT64_MAX;
}

void Relation::randomOrder() {
  // Only used by the host reference generators (kept for parity).
  if (loc_ != Location::Host || localSize < 2) return;
  uint64_t s = 0x2545F4914F6CDD1DULL;
  for (uint64_t i = localSize - 1; i > 0; --i) {
    s = kernels::mix64(s + i);
    const uint64_t j = s % i;  // Sattolo-style j < i, as in Relation.cpp:90-96
    std::swap(data[i].key, data[j].key);
  }
}

void Relation::distribute(uint32_t nodeId, uint32_t numberOfNodes, comm::Communicator *comm) {
  // Reference (Relation.cpp:99-141): pairwise swap of sections, then reshuffle.
  // Here: section k of every rank goes to rank k in one all-to-all.
  if (numberOfNodes <= 1) return;
  JOIN_ASSERT(loc_ != Location::Pinned, "Relation", "distribute() of a pinned host relation is not supported");
  JOIN_ASSERT(comm && comm->size() == numberOfNodes && comm->rank() == nodeId, "Relation",
              "distribute needs the job communicator");
  std::vector<uint64_t> sendCounts(numberOfNodes), sendDispls(numberOfNodes), recvCounts(numberOfNodes),
      recvDispls(numberOfNodes);
  const uint64_t section = localSize / numberOfNodes;
  for (uint32_t k = 0; k < numberOfNodes; ++k) {
    sendDispls[k] = k * section * 2;
    sendCounts[k] = (k == numberOfNodes - 1 ? localSize - section * (numberOfNodes - 1) : section) * 2;
  }
  std::vector<uint64_t> all(numberOfNodes * numberOfNodes);
  comm->allGatherHost(sendCounts.data(), all.data(), numberOfNodes);
  uint64_t total = 0;
  for (uint32_t k = 0; k < numberOfNodes; ++k) {
    recvCounts[k] = all[(uint64_t)k * numberOfNodes + nodeId];
    recvDispls[k] = total;
    total += recvCounts[k];
  }
  JOIN_ASSERT(total == localSize * 2, "Relation", "distribute changes local sizes (%lu != %lu)",
              (unsigned long)total / 2, (unsigned long)localSize);
  Tuple *incoming = static_cast<Tuple *>(memory::Arena::rawAlloc(loc_, localSize * sizeof(Tuple), device_));
  comm->allToAllV(reinterpret_cast<uint64_t *>(data), sendCounts.data(), sendDispls.data(),
                  reinterpret_cast<uint64_t *>(incoming), recvCounts.data(), recvDispls.data(), loc_, nullptr);
  if (loc_ == Location::Device) {
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(data, incoming, localSize * sizeof(Tuple), hipMemcpyDeviceToDevice));
  } else {
    std::memcpy(data, incoming, localSize * sizeof(Tuple));
    randomOrder();
  }
  memory::Arena::rawFree(loc_, incoming);
  ridsPositional_ = false;  // rids moved with their tuples; keys keep their bound
}

void Relation::debugKeyPrint(uint64_t limit) {
  const uint64_t n = std::min(limit, localSize);
  std::vector<Tuple> h(n);
  if (deviceAccessible(loc_))
    HIP_CHECK(hipMemcpy(h.data(), data, n * sizeof(Tuple), hipMemcpyDefault));
  else
    std::memcpy(h.data(), data, n * sizeof(Tuple));
  for (uint64_t i = 0; i < n; ++i) std::fprintf(stdout, "%lu, ", (unsigned long)h[i].key);
  std::fprintf(stdout, "\n");
  std::fflush(stdout);
}

}  // namespace data
}  // namespace hpcjoin
