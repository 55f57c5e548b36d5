// Late materialization of join results with fixed-width payload rows
// (BASELINE config 5: TPC-H-like orders x lineitem, 32-byte payloads).
//
// Payload columns stay on the rank that generated them (rid ranges follow
// Relation::localOffsetFor).  For every materialized (rid_inner, rid_outer)
// pair the operator fetches both rows: requests bucketed by owner rank with
// the LDS partition kernels, RCCL all-to-allv of rids, row gather on the
// owner, all-to-allv of rows back, placement next to the pair.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../core/ExecContext.h"

namespace hpcjoin {
namespace operators {

struct PayloadColumn {
  const uint64_t *rows = nullptr;  // [localRows][ROW_WORDS] in the context's memory
  uint64_t localRows = 0;
  uint64_t ridOffset = 0;          // rid of local row 0
  uint64_t globalRows = 0;         // rows over all ranks (owner of rid = rid / (globalRows / N))
};

class LateMaterialization {
 public:
  static constexpr uint32_t OUT_WORDS = 2 + 2 * 4;  // rid_inner, rid_outer, inner row, outer row
  // Device-timeline phase times (both sides summed; timing events recorded on
  // the engine stream between the phases and resolved after materialize()'s
  // final synchronisation -- no extra host syncs) and the bytes this rank put
  // on its links.
  struct Stats {
    double bucketMs = 0;    // requests bucketed by owner rank (LDS radix kernels)
    double requestMs = 0;   // all-to-allv of the requested rids
    double gatherMs = 0;    // owner-side row gather
    double responseMs = 0;  // all-to-allv of the rows back
    double placeMs = 0;     // rows placed next to their pairs
    uint64_t requestBytes = 0, responseBytes = 0;  // to other ranks
  };
  const Stats &stats() const { return st; }

  // matVariant: KernelVariants::matVariant of the single-rank gather kernel.
  LateMaterialization(core::ExecContext *ctx, const PayloadColumn &inner, const PayloadColumn &outer,
                      uint32_t matVariant = 1);
  ~LateMaterialization();
  LateMaterialization(const LateMaterialization &) = delete;
  LateMaterialization &operator=(const LateMaterialization &) = delete;
  // out: [n][OUT_WORDS] u64 in the context's memory.  Collective: every rank calls it.
  void materialize(const ulonglong2 *pairs, uint64_t n, uint64_t *out);

 private:
  void fetchDevice(const ulonglong2 *pairs, uint64_t n, int side, const PayloadColumn &col, uint64_t *out);
  void fetchHost(const ulonglong2 *pairs, uint64_t n, int side, const PayloadColumn &col, uint64_t *out);
  core::ExecContext *ctx;
  PayloadColumn cols[2];
  uint32_t matVariant = 1;
  Stats st;
  static constexpr int PHASES = 5;             // bucket, request, gather, response, place
  hipEvent_t marks[2][PHASES + 1] = {};        // per side: start + one per phase end (timing events)
  bool marked[2] = {false, false};
  void resolveMarks();
};

}  // namespace operators
}  // namespace hpcjoin
