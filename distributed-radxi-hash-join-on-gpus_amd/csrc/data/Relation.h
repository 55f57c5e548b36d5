// Local slice of a relation plus its global size.  Same public API as
// /root/reference/data/Relation.h:17-61 (getLocalSize / getGlobalSize /
// getData / fillUniqueValues / fillModuloValues / distribute / debugKeyPrint),
// but the tuples can live in HBM and every generator runs as a HIP kernel
// (datagen.hip).  The generate() family evaluates each rank's slice of ONE
// global relation (Feistel permutation, Zipf, ...) so distribute() is no
// longer needed to mix keys across ranks; it is kept (RCCL all-to-all) for
// API parity.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../core/Types.h"
#include "../kernels/kernels.h"
#include "Tuple.h"

namespace hpcjoin {
namespace comm {
class Communicator;
}
namespace data {

struct GenSpec {
  kernels::KeyDistribution distribution = kernels::KeyDistribution::Unique;
  uint64_t seed = 1234;
  uint64_t domain = 0;       // key domain (0 = global size); FK relations use the inner size
  uint64_t keyOffset = 0;
  double zipfTheta = 0.75;
  bool tpchSparse = false;   // TPC-H O_ORDERKEY layout applied to the generated key (both sides alike)
  bool sparse64 = false;     // sparse random 63-bit keys (kernels::sparseKey), both sides alike
};

class Relation {
 public:
  // Reference constructor: host memory from memory::Pool.
  Relation(uint64_t localSize, uint64_t globalSize);
  // Owning relation in HBM (Location::Device) or host memory.
  Relation(uint64_t localSize, uint64_t globalSize, Location loc, int device = 0);
  // Non-owning view of caller memory (e.g. a torch tensor).
  Relation(Tuple *external, uint64_t localSize, uint64_t globalSize, Location loc, int device = 0);
  ~Relation();
  Relation(const Relation &) = delete;
  Relation &operator=(const Relation &) = delete;

  uint64_t getLocalSize();
  uint64_t getGlobalSize();
  Tuple *getData();
  Location location() const { return loc_; }
  int device() const { return device_; }

  // Reference generators (Relation.cpp:63-85): keys start..start+n-1 in a
  // random order, rids startRid + i.
  void fillUniqueValues(uint64_t startKeyValue, uint64_t startRidValue);
  void fillModuloValues(uint64_t startKeyValue, uint64_t startRidValue, uint64_t innerRelationSize);
  // MI355X generators: this rank's slice [globalOffset, globalOffset + n) of a
  // global relation.  Returns nothing; see expectedMatches() for the oracle.
  void generate(const GenSpec &spec, uint64_t globalOffset);
  void distribute(uint32_t nodeId, uint32_t numberOfNodes, comm::Communicator *comm = nullptr);
  void debugKeyPrint(uint64_t limit = 64);

  // Helpers for rank slices: [offset, offset + size) of the global relation.
  static uint64_t localSizeFor(uint64_t globalSize, uint32_t nodeId, uint32_t numberOfNodes);
  static uint64_t localOffsetFor(uint64_t globalSize, uint32_t nodeId, uint32_t numberOfNodes);
  // Exact |R join S| for generate()d inner/outer pairs when it is known
  // analytically (unique inner keys over [0, G_R)); UINT64_MAX otherwise.
  static uint64_t expectedMatches(const GenSpec &inner, uint64_t innerGlobal, const GenSpec &outer,
                                  uint64_t outerGlobal);
  uint64_t maxKey() const { return maxKey_; }
  // Bounds the planner can use without reading the tuples (set by the
  // generators, cleared by distribute()/external data): every key <= maxKey(),
  // the rid of local tuple i is ridBase() + i, and the low key bits are
  // uniform (no key mixing needed).
  bool keyBoundKnown() const { return keyBoundKnown_; }
  bool ridsPositional() const { return ridsPositional_; }
  uint64_t ridBase() const { return ridBase_; }
  bool lowBitsUniform() const { return lowBitsUniform_; }
  // What the generator knows about repeated keys in the GLOBAL relation:
  // 0 unknown (external data), 1 every key unique, 2 keys repeat.  The
  // planner decides bitmap vs two-level and the key-only table kind from it
  // before the first join (HashJoin::makeJoinPlan samples when 0).
  int keyRepeats() const { return keyRepeats_; }
  // A pass view of a subset of `parent`'s tuples (capacity spill,
  // operators/HashJoin::runPasses): the parent's key bound (maxKey), its
  // repeated-key knowledge and low-bit uniformity carry over; rids are
  // bounded by ridMax but no longer positional.
  void inheritBounds(const Relation &parent, uint64_t maxKey, uint64_t ridMax);
  bool ridBoundKnown() const { return ridBoundKnown_; }
  uint64_t ridMax() const { return ridMax_; }

 protected:
  void randomOrder();
  void ensureHostMirror();
  void setGenerated(uint64_t ridBase, bool lowBitsUniform);

 protected:
  uint64_t localSize;
  uint64_t globalSize;
  Tuple *data;

 private:
  Location loc_;
  int device_;
  bool owns_;
  bool fromPool_;
  uint64_t maxKey_ = 0;
  bool keyBoundKnown_ = false;
  bool ridsPositional_ = false;
  uint64_t ridBase_ = 0;
  bool lowBitsUniform_ = false;
  int keyRepeats_ = 0;
  bool ridBoundKnown_ = false;
  uint64_t ridMax_ = 0;
};

}  // namespace data
}  // namespace hpcjoin
