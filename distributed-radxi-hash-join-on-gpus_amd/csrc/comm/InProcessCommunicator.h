// N ranks as threads of one process ("a fake communicator
// (in-process threads exchanging buffers) lets the host-side offset and
// assignment logic be tested without a cluster").  Works for host buffers and
// for device buffers on one GPU (D2D copies), so the complete distributed
// device path -- exchange plans, windows, chunked exchange, segments -- runs
// under test on a single MI355X, where RCCL refuses two ranks per device.
// Collectives are blocking; allToAllV synchronises the caller's stream first
// so a sender's scatter kernel has finished before peers copy from it.
#pragma once

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "Communicator.h"

namespace hpcjoin {
namespace comm {

class InProcessGroup {
 public:
  explicit InProcessGroup(uint32_t size);
  uint32_t size() const { return size_; }
  // Blocks until all ranks arrive.  Throws if the group was aborted (a peer
  // failed) or after utils::commTimeoutMs(), aborting the group itself then.
  void barrier();
  void abort(const std::string &why);
  bool aborted();
  // Shared slots: each rank publishes one pointer-sized value per phase.
  std::vector<const void *> slots;
  std::vector<const uint64_t *> counts, displs;
  std::vector<uint64_t> scratch;  // all-gather staging

 private:
  uint32_t size_;
  std::mutex m_;
  std::condition_variable cv_;
  uint32_t waiting_ = 0;
  uint64_t generation_ = 0;
  bool aborted_ = false;
  std::string reason_;
};

class InProcessCommunicator : public Communicator {
 public:
  InProcessCommunicator(std::shared_ptr<InProcessGroup> group, uint32_t rank) : group_(std::move(group)), rank_(rank) {}
  ~InProcessCommunicator() override;
  uint32_t rank() const override { return rank_; }
  uint32_t size() const override { return group_->size(); }
  bool supports(Location) const override { return true; }
  std::string name() const override { return "in_process"; }
  bool sharesAddressSpace() const override { return true; }
  void allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) override;
  void allReduceSumHost(uint64_t *data, size_t count) override;
  // Device buffers of ranks on one device: each rank sums its slice of all
  // buffers with one kernel (no host staging); completes before returning.
  // Blocking (stream sync + barriers per call): an in-process rehearsal of the
  // replicated bitmap plan therefore runs its all-reduce ranges one after the
  // other -- the overlap of build, reduce and probe ranges is the RCCL path's.
  void allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream) override;
  void barrier() override { group_->barrier(); }
  void checkHealth() override;
  void abort(const std::string &why) override { group_->abort(why); }
  void allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls, uint64_t *recv,
                 const uint64_t *recvCounts, const uint64_t *recvDispls, Location loc, hipStream_t stream) override;

 private:
  std::shared_ptr<InProcessGroup> group_;
  uint32_t rank_;
  uint64_t **ptrTable_ = nullptr;  // device table of the ranks' buffer pointers (allocated once)
  int ptrTableDevice_ = -1;
  uint32_t ptrTableSize_ = 0;
};

}  // namespace comm
}  // namespace hpcjoin
