// Runtime configuration of one join (the reference is compile-time only:
// core/Configuration.h + CMake -D macros, SURVEY §5 "Config / flag system").
// JoinPlan is what the engine actually runs with once sizes are known.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "Configuration.h"
#include "Types.h"

namespace hpcjoin {
namespace core {

enum class AssignmentPolicy : int {
  RoundRobin = 0,  // partition p -> node p % N (reference AssignmentMap.cpp:41-43)
  LPT = 1,         // longest-processing-time greedy on |R_p| + |S_p| (skew-aware)
};

enum class TupleFormat : int {
  Compressed = 0,  // 8-byte CompressedTuple after the network pass (reference format)
  Wide = 1,        // 16-byte Tuple end to end: full 64-bit keys (the RCD / AoS path)
};

// Radix digits from the raw key (optimal for dense keys) or from a bijective
// mix of it (keys with structured low bits: sparse TPC-H order keys, strides).
enum class KeyHashing : int {
  Auto = 0,  // decided at plan time from a histogram of the inner keys' low bits
  Off = 1,
  On = 2,
};

// How a radix pass sizes its partitions: an exact histogram read of the input,
// or a sampled one with statistical slack and an exact re-run on overflow.
//   network pass: Sampled only for N == 1 on a device with one chunk (the
//                 exchange needs exact counts); Auto = Sampled there when both
//                 relations have >= 16M tuples (tasks/SampledNetworkPartitioning)
//   local pass:   Sampled on a device (any N); Auto = Sampled when the window
//                 holds >= 16M tuples (tasks/LocalPartitioning)
enum class HistogramMode : int {
  Auto = 0,
  Exact = 1,
  Sampled = 2,
};

// Exchange wire format (kernels.h, WireCodec): bit-packed frame-of-reference
// tuples on the xGMI links instead of full 8-byte CompressedTuples.
enum class WireCodecMode : int {
  Auto = 0,  // device engine, N > 1, when the link time it saves exceeds its extra passes (HashJoin::codecPays)
  Off = 1,
  On = 2,    // whenever the tuple fits < 64 bits (also the host path: tests)
};

// Tri-state switch of an optional plan (Auto = the planner's cost model decides).
enum class PlanChoice : int {
  Auto = 0,
  Off = 1,
  On = 2,
};

// How NetworkPartitioning moves tuples to their owners (N > 1).
enum class ExchangeMode : int {
  Rccl = 0,      // two-sided: grouped ncclSend/ncclRecv all-to-allv per chunk (default)
  OneSided = 1,  // the MPI_Put analog: each rank copies its runs straight into the owner's window
                 // (IPC-mapped peer allocations; plain pointers for in-process ranks), then a barrier
};

struct JoinConfig {
  uint32_t networkBits = 0;   // radix bits of the network pass (0 = auto)
  uint32_t localBits = 0;     // radix bits of the local pass (0 = auto; ignored if !twoLevel)
  bool twoLevel = true;       // run the local (second) partitioning pass
  uint32_t keyShift = 0;      // CompressedTuple key position (0 = auto: max(32, rid bits))
  AssignmentPolicy assignment = AssignmentPolicy::LPT;
  TupleFormat format = TupleFormat::Compressed;
  bool materialize = false;   // also write (rid_inner, rid_outer) pairs
  uint64_t outputCapacity = 0;  // materialize: pair capacity (0 = auto from oracle bound)
  // materialize: write the (rid_inner, rid_outer) pairs straight into this
  // caller-owned pinned host buffer of outputCapacity pairs (device-mapped:
  // the place kernel stores over the host link), not into the workspace --
  // the output of a join may then exceed HBM, and a materializing join can
  // spill (capacity passes append to it).  The reference's UVA driver writes
  // its probe output to host memory the same way
  // (operators/gpu/small_data_optimized.cu:1193-1195).
  void *outputHost = nullptr;
  uint64_t buildTarget = 4096;  // target inner tuples per final partition (= one 256 x 16 LDS build batch)
  uint32_t rChunk = 0;          // max inner tuples per LDS table (0 = auto from LDS budget)
  uint32_t sChunk = 65536;      // max outer tuples per build/probe work item
  uint32_t chunks = 1;          // exchange pipeline slices per relation (>1: scatter(k+1) || all-to-all(k))
  bool checks = true;           // cheap always-on invariants (all tuples written, sizes)
  // Network-pass grid cap: 512 = two workgroups per CU, each walking a long
  // contiguous range (1B tuples: 477 tiles per workgroup).  Same-process A/B
  // on MI355X, 1B x 1B: general path 19.23 -> 18.99 ms, headline 9.54 -> 9.47
  // ms against 2048 (fewer workgroup prologues / epilogues per CU;
  // profiles/r6/README.md).
  uint32_t maxPartitionBlocks = 512;
  KeyHashing keyHashing = KeyHashing::Auto;
  HistogramMode networkHistogram = HistogramMode::Auto;
  HistogramMode localHistogram = HistogramMode::Auto;
  uint32_t sampleStride = 64;   // sampled network pass: histogram 1 tile in sampleStride (per-slot counts ~1e5+)
  uint32_t localSampleStride = 16;  // sampled local pass: 1 tile in localSampleStride of every work item
  // Single-rank sampled network windows: claim slices in rounds of
  // 2^roundLp-slot pieces (kernels::RoundMap) when the slices are even enough
  // to fit; 0 = linear slices.
  uint32_t roundLp = 9;
  WireCodecMode wireCodec = WireCodecMode::Auto;
  bool splitLocal = true;       // device: split local pass output (u32 rid + u16 fragment columns) when they fit
  // N > 1, LPT: a network partition above one rank's fair share of |R| + |S|
  // is joined by several ranks (larger side divided, smaller replicated;
  // histograms/AssignmentMap).
  bool skewSplit = true;
  bool directCount = true;      // count-only build/probe: direct-addressed LDS counts when fragments are <= 13 bits
  bool splitHistogram = true;   // N > 1 on device: outer exact histogram overlaps the inner exchange
  bool pipelineOuter = true;    // N > 1 on device, counting: outer local pass + build/probe per received chunk
  bool bitmapJoin = true;       // N == 1 on device, counting, sampled network pass: one LDS bitmap per network
                                // partition instead of the local pass when the fragment range fits (unique inner
                                // keys; a duplicate falls back to the two-level pass)
  // N > 1 counting joins of unique inner keys whose key range fits bitmaps
  // (tasks/BitmapJoin): every rank builds the bitmaps of its own inner keys,
  // one RCCL all-reduce ORs them, and every rank probes its own outer tuples
  // -- no tuple crosses a link.  Auto: on a device engine when its link bytes
  // (2 (N-1)/N * 2^keyBits / 8) undercut the shuffle's; On: whenever the key
  // range fits (host path and N == 1 included); Off: never.
  PlanChoice replicateBitmap = PlanChoice::Auto;
  ExchangeMode exchange = ExchangeMode::Rccl;
  // N > 1: check the exchanged data, not only the counts -- content hashes
  // of every (source, chunk, partition) run on the sender vs what arrived
  // (operators/ExchangeVerify.h).  One extra read of the input and of the
  // windows per join.  Auto: on for one-sided windows (IPC puts, where a lost
  // or misdirected put would otherwise be silent), off for RCCL all-to-allv.
  PlanChoice verifyExchange = PlanChoice::Auto;
  // Capacity spill (kernels/spill.hip): run the join in this many passes,
  // each over the tuples whose key hashes to it (counting joins).  0 = auto:
  // on a device engine, as many as it takes for one pass's buffers and
  // workspace to fit what HBM has free (capped by workspaceBudget).
  uint32_t passes = 0;
  uint32_t localItemTiles = 64; // local pass work item: up to this many 4096-tuple tiles of one segment
  uint32_t localGeometry = 0;   // local scatter workgroup geometry (0 = 1024 x 8; 1-4: sweep alternatives)
  KernelVariants variants;      // kernel-shape variants (sweeps; core/Types.h)
  // Device engines: grow the workspace arena to the plan's size estimate at
  // HashJoin construction (and touch the new pages once), so that the first
  // join allocates nothing (HashJoin::workspaceEstimate).
  bool reserveWorkspace = true;
  // Upper bound in bytes of that reservation (0 = 85 % of the HBM free at
  // construction).  The arena never frees on its own; ExecContext's trim
  // (Python: ExecContext.trim_workspace) gives it back between joins.
  uint64_t workspaceBudget = 0;
  // Link model of the N > 1 plan choice / prediction: one-way GB/s one rank
  // reaches to one peer (0 = kDefaultLinkGBpsPerPeer; bench.py calibrates it
  // with an RCCL all-to-all).
  double linkGBpsPerPeer = 0;
  // Wire codec cost (WireCodecMode::Auto): picoseconds per tuple the pack +
  // unpack passes cost beyond raw words' gather of the filled runs (MI355X:
  // ~7 ps pack + unpack vs ~3.5 ps gather per tuple, bench.py scale_model).
  double codecExtraPsPerTuple = 3.5;

  std::string describe() const;
};

// Fully resolved plan for a given pair of relations.
struct JoinPlan {
  uint32_t numberOfNodes = 1;
  uint32_t networkBits = 5;
  uint32_t localBits = 0;
  uint32_t keyShift = 32;
  uint32_t fragShift = 32;    // compressed: key fragment shift after both passes
  uint32_t keyBits = 64;      // bits of the largest key over both relations
  uint32_t rChunk = 4096;
  uint32_t sChunk = 65536;
  uint32_t chunks = 1;
  bool twoLevel = true;
  bool wide = false;
  bool materialize = false;
  bool keyMix = false;        // radix digits from kernels::KeyMix{keyBits} of the key
  // Counting join whose keys do not fit a CompressedTuple (sparse 63-bit keys):
  // after the network pass a tuple is the 8-byte word key >> networkBits (no
  // rid: a count never reads one), keyShift = 0.  The wide format's 16 bytes
  // are kept only for materializing joins and when TupleFormat::Wide is asked.
  bool keyOnly = false;
  bool innerRepeats = false;    // inner keys repeat (generator metadata or a plan-time sample): no bitmap plan
  bool sampledNetwork = false;  // single-rank network pass sized from a sampled histogram
  bool splitHistogram = false;  // N > 1: assignment from an outer estimate, outer exact histogram off the head
  bool pipelineOuter = false;   // N > 1 counting: outer local pass + build/probe per exchange chunk
  bool bitmapJoin = false;      // single-level bitmap join (kernels::bitmapJoin) after the sampled network pass
  uint32_t bitmapBits = 0;      // fragment bits per network partition (bitmap size 2^bitmapBits)
  bool bitmapReplicated = false;  // bitmaps all-reduced over ranks, outer probed in place (tasks/BitmapJoin)
  bool oneSided = false;          // ExchangeMode::OneSided in effect (data::Window::enableOneSided)
  // Cost model of the N > 1 plan choice: bytes one rank puts on its links per
  // join for the replicated bitmaps and for the tuple shuffle, and the
  // predicted link time of each at linkGBps per rank (7 xGMI peers).
  double replicatedLinkBytes = 0, shuffleLinkBytes = 0;
  double linkGBps = 0;
  HistogramMode localHistogram = HistogramMode::Exact;  // resolved per window size by LocalPartitioning
  uint32_t sampleStride = 64;
  uint32_t localSampleStride = 16;
  uint32_t roundLp = 0;  // round-interleaved sampled network window (JoinConfig::roundLp; 0 = linear)
  AssignmentPolicy assignment = AssignmentPolicy::LPT;
  // Wire codec per relation (0 = inner, 1 = outer): bits per tuple (0 = off),
  // rid bits, and the rid base of every (rank, exchange chunk), rank-major.
  // Set by HashJoin::planWireCodec.
  bool splitLocal = false;    // local pass writes split columns (kernels.h, SplitLayout)
  // Count-only two-level pass (N = 1, sampled network pass): the network pass
  // writes u32 key fragments and the local pass only the u16 fragment column
  // -- no rid is written, since a count never reads one.
  bool fragments = false;
  bool skewSplit = false;     // hot network partitions may be split across ranks
  bool directCount = true;    // build/probe may use direct-addressed count tables
  uint32_t localItemTiles = 64;
  uint32_t localGeometry = 0;
  KernelVariants variants;
  uint32_t wireBits[2] = {0, 0};
  uint32_t wireRidBits[2] = {0, 0};
  // Capacity spill of the N = 1 bitmap plan (tasks/BitmapJoin, partition-group
  // passes): bytes the fragment windows of one pass may take; 0 = one pass.
  uint64_t groupBudget = 0;
  std::vector<uint64_t> ridBase[2];
  uint64_t networkPartitions() const { return uint64_t(1) << networkBits; }
  uint64_t localPartitions() const { return twoLevel ? (uint64_t(1) << localBits) : 1; }
  std::string describe() const;
};

// maxKey / maxRid: upper bounds over both relations (all ranks).
JoinPlan makePlan(const JoinConfig &cfg, uint32_t numberOfNodes, uint64_t globalInner, uint64_t globalOuter,
                  uint64_t maxKey, uint64_t maxRid);

}  // namespace core
}  // namespace hpcjoin
