// 8-byte packed tuple: layout-identical to /root/reference/data/CompressedTuple.h:14-20
// with the packing rule of /root/reference/tasks/NetworkPartitioning.cpp:128-129:
//
//   value = rid | ((key >> networkBits) << keyShift)
//
// The reference fixes networkBits = 5 and keyShift = NPF + PAYLOAD_BITS = 32.
// Here both are runtime parameters (JoinConfig) so that (a) a larger network
// fan-out can be chosen for 8 GPUs and (b) rids wider than 32 bits (the
// 1B x 16B skew config) still fit.  The network partition bits are implicit in
// the partition a tuple lives in, exactly as in the reference.
#pragma once

#include "../core/Types.h"

namespace hpcjoin {
namespace data {

class CompressedTuple {
 public:
  unsigned long long value;

  static HJ_HD unsigned long long pack(uint64_t key, uint64_t rid, uint32_t networkBits, uint32_t keyShift) {
    return (unsigned long long)(rid | ((key >> networkBits) << keyShift));
  }
  // Key bits above the network partition id, i.e. key >> networkBits.
  static HJ_HD uint64_t keyHigh(unsigned long long v, uint32_t keyShift) { return v >> keyShift; }
  static HJ_HD uint64_t rid(unsigned long long v, uint32_t keyShift) {
    return keyShift >= 64 ? v : (v & ((uint64_t(1) << keyShift) - 1));
  }
  // Full key, given the network partition the tuple was routed to.
  static HJ_HD uint64_t key(unsigned long long v, uint32_t networkBits, uint32_t keyShift, uint64_t partition) {
    return ((v >> keyShift) << networkBits) | partition;
  }
};

static_assert(sizeof(CompressedTuple) == 8, "CompressedTuple must stay 8 bytes");

}  // namespace data
}  // namespace hpcjoin
