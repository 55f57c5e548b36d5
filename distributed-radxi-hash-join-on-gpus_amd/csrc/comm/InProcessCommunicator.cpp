#include "InProcessCommunicator.h"

#include "../kernels/kernels.h"

#include <chrono>
#include <cstring>

#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace comm {

InProcessGroup::InProcessGroup(uint32_t size)
    : slots(size, nullptr), counts(size, nullptr), displs(size, nullptr), size_(size) {}

void InProcessGroup::barrier() {
  std::unique_lock<std::mutex> lk(m_);
  JOIN_ASSERT(!aborted_, "InProcess", "group aborted: %s", reason_.c_str());
  const uint64_t gen = generation_;
  if (++waiting_ == size_) {
    waiting_ = 0;
    ++generation_;
    cv_.notify_all();
    return;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(utils::commTimeoutMs());
  if (!cv_.wait_until(lk, deadline, [&] { return generation_ != gen || aborted_; })) {
    aborted_ = true;
    reason_ = utils::format("barrier timed out after %lu ms with %u of %u ranks present (rank %d: %s)",
                            (unsigned long)utils::commTimeoutMs(), waiting_, size_, utils::debugRank(),
                            utils::watchdogContext().c_str());
    cv_.notify_all();
  }
  if (generation_ == gen) {  // woken by an abort, not by the last arrival
    --waiting_;
    JOIN_ASSERT(false, "InProcess", "group aborted: %s", reason_.c_str());
  }
}

void InProcessGroup::abort(const std::string &why) {
  std::lock_guard<std::mutex> lk(m_);
  if (!aborted_) {
    aborted_ = true;
    reason_ = why;
  }
  cv_.notify_all();
}

bool InProcessGroup::aborted() {
  std::lock_guard<std::mutex> lk(m_);
  return aborted_;
}

void InProcessCommunicator::checkHealth() {
  JOIN_ASSERT(!group_->aborted(), "InProcess", "a peer rank aborted the group");
}

void InProcessCommunicator::allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) {
  InProcessGroup &g = *group_;
  g.slots[rank_] = send;
  g.barrier();
  for (uint32_t r = 0; r < g.size(); ++r)
    std::memcpy(recv + r * count, g.slots[r], count * sizeof(uint64_t));
  g.barrier();
}

void InProcessCommunicator::allReduceSumHost(uint64_t *data, size_t count) {
  std::vector<uint64_t> all(count * size());
  allGatherHost(data, all.data(), count);
  for (size_t i = 0; i < count; ++i) {
    uint64_t s = 0;
    for (uint32_t r = 0; r < size(); ++r) s += all[r * count + i];
    data[i] = s;
  }
}

InProcessCommunicator::~InProcessCommunicator() {
  if (ptrTable_) (void)hipFree(ptrTable_);
}

void InProcessCommunicator::allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream) {
  const uint32_t N = size(), me = rank_;
  if (N == 1 || count == 0) return;
  hipPointerAttribute_t attr;
  const bool dev = hipPointerGetAttributes(&attr, data) == hipSuccess && attr.type == hipMemoryTypeDevice;
  (void)hipGetLastError();
  std::vector<uint64_t> ptrs(N);
  const uint64_t mine[2] = {(uint64_t)(uintptr_t)data, dev ? (uint64_t)attr.device : ~0ull};
  std::vector<uint64_t> all(2 * N);
  HIP_CHECK(hipStreamSynchronize(stream));  // my buffer is final
  allGatherHost(mine, all.data(), 2);       // (a barrier: every buffer is final)
  bool sameDevice = dev;
  for (uint32_t r = 0; r < N; ++r) {
    ptrs[r] = all[2 * r];
    sameDevice = sameDevice && all[2 * r + 1] == mine[1];
  }
  if (!sameDevice) {  // ranks on different devices (or host memory): the staged default
    Communicator::allReduceSumDevice(data, count, stream);
    return;
  }
  if (!ptrTable_ || ptrTableDevice_ != (int)attr.device || ptrTableSize_ < N) {
    if (ptrTable_) HIP_CHECK(hipFree(ptrTable_));
    HIP_CHECK(hipMalloc((void **)&ptrTable_, N * sizeof(uint64_t)));
    ptrTableDevice_ = (int)attr.device;
    ptrTableSize_ = N;
  }
  HIP_CHECK(hipMemcpyAsync((void *)ptrTable_, ptrs.data(), N * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  kernels::sumSlices(ptrTable_, N, count * me / N, count * (me + 1) / N, stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  group_->barrier();  // every slice of every buffer written
}

void InProcessCommunicator::allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls,
                                      uint64_t *recv, const uint64_t *recvCounts, const uint64_t *recvDispls,
                                      Location loc, hipStream_t stream) {
  InProcessGroup &g = *group_;
  const bool dev = loc == Location::Device;
  if (dev) HIP_CHECK(hipStreamSynchronize(stream));  // my scatter output is complete
  g.slots[rank_] = send;
  g.counts[rank_] = sendCounts;
  g.displs[rank_] = sendDispls;
  g.barrier();
  for (uint32_t src = 0; src < g.size(); ++src) {
    const uint64_t n = recvCounts[src];
    JOIN_ASSERT(g.counts[src][rank_] == n, "InProcess", "rank %u expects %lu words from %u, which sends %lu", rank_,
                (unsigned long)n, src, (unsigned long)g.counts[src][rank_]);
    if (!n) continue;
    const uint64_t *from = static_cast<const uint64_t *>(g.slots[src]) + g.displs[src][rank_];
    if (dev)
      HIP_CHECK(hipMemcpyAsync(recv + recvDispls[src], from, n * 8, hipMemcpyDeviceToDevice, stream));
    else
      std::memcpy(recv + recvDispls[src], from, n * 8);
  }
  if (dev) HIP_CHECK(hipStreamSynchronize(stream));
  g.barrier();  // nobody reuses a send buffer before every peer copied from it
}

}  // namespace comm
}  // namespace hpcjoin
