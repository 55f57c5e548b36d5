// Communicator over a torch.distributed ProcessGroup (c10d).  Used for the
// host reference path across processes (gloo backend on CPU: the
// multi-process tests) and as a fallback on GPUs (nccl backend = RCCL).  The
// MI355X production path is RcclCommunicator (stream-ordered, direct links).
#pragma once

#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include "../comm/Communicator.h"

namespace hpcjoin {
namespace comm {

class ProcessGroupCommunicator : public Communicator {
 public:
  explicit ProcessGroupCommunicator(c10::intrusive_ptr<c10d::ProcessGroup> pg);
  uint32_t rank() const override { return (uint32_t)pg_->getRank(); }
  uint32_t size() const override { return (uint32_t)pg_->getSize(); }
  bool supports(Location loc) const override { return loc == Location::Host; }
  std::string name() const override { return "process_group:" + pg_->getBackendName(); }
  void allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) override;
  void allReduceSumHost(uint64_t *data, size_t count) override;
  void barrier() override;
  void allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls, uint64_t *recv,
                 const uint64_t *recvCounts, const uint64_t *recvDispls, Location loc, hipStream_t stream) override;

 private:
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
};

}  // namespace comm
}  // namespace hpcjoin
