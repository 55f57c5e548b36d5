// RCCL communicator: one process per MI355X, bootstrapped from a 128-byte
// ncclUniqueId that the launcher distributes (torch.distributed store, a file,
// or MPI).  The shuffle is a grouped ncclSend/ncclRecv per peer: on a fully
// connected 8 x MI355X node every pair has its own xGMI link, so a direct
// all-to-allv is link-parallel (7 x ~153 GB/s egress per GPU) where a ring
// collective would be per-link bound.
#pragma once

#include <string>
#include <vector>

#include "Communicator.h"

namespace hpcjoin {
namespace comm {

class RcclCommunicator : public Communicator {
 public:
  static constexpr size_t UNIQUE_ID_BYTES = 128;
  static std::vector<uint8_t> uniqueId();

  RcclCommunicator(const std::vector<uint8_t> &id, uint32_t rank, uint32_t size, int device);
  ~RcclCommunicator() override;

  uint32_t rank() const override { return rank_; }
  uint32_t size() const override { return size_; }
  bool supports(Location loc) const override { return loc == Location::Device; }
  std::string name() const override { return "rccl"; }
  void allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) override;
  void allGatherDevice(const uint64_t *send, uint64_t *recv, size_t count, hipStream_t stream) override;
  void allReduceSumHost(uint64_t *data, size_t count) override;
  void allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream) override;
  void barrier() override;
  void allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls, uint64_t *recv,
                 const uint64_t *recvCounts, const uint64_t *recvDispls, Location loc, hipStream_t stream) override;
  int device() const { return device_; }
  void checkHealth() override;
  void abort(const std::string &why) override;

 private:
  uint64_t *scratch(size_t words);
  void *comm_ = nullptr;  // ncclComm_t
  uint32_t rank_, size_;
  int device_;
  hipStream_t stream_ = nullptr;  // for the small blocking collectives
  uint64_t *scratch_ = nullptr;
  std::vector<uint64_t *> retired_;  // outgrown scratch buffers (freed with the communicator)
  size_t scratchWords_ = 0;
  std::string abortReason_;
};

}  // namespace comm
}  // namespace hpcjoin
