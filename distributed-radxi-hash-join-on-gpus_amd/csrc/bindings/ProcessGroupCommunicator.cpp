#include "ProcessGroupCommunicator.h"

#include <cstring>

#include "../utils/Debug.h"
#include "../utils/Fault.h"

namespace hpcjoin {
namespace comm {

ProcessGroupCommunicator::ProcessGroupCommunicator(c10::intrusive_ptr<c10d::ProcessGroup> pg) : pg_(std::move(pg)) {
  utils::setDebugRank(pg_->getRank());
}

// Every collective waits at most the engine's watchdog deadline
// (HPCJOIN_COMM_TIMEOUT_S): a peer that stopped making progress ends this
// rank's wait with a message naming the rank, phase and last collective,
// instead of gloo's 30-minute default.
static void waitBounded(const c10::intrusive_ptr<c10d::Work> &work, const char *what) {
  try {
    work->wait(std::chrono::milliseconds(utils::commTimeoutMs()));
  } catch (const std::exception &e) {
    utils::fail("WATCHDOG", __FILE__, __LINE__,
                utils::format("%s did not complete within %lu ms (%s): %s", what,
                              (unsigned long)utils::commTimeoutMs(), utils::watchdogContext().c_str(), e.what()));
  }
  utils::noteCollective(what, true);
}

static at::Tensor hostWords(const uint64_t *p, size_t n) {
  at::Tensor t = at::empty({(int64_t)n}, at::TensorOptions().dtype(at::kLong));
  if (n) std::memcpy(t.data_ptr(), p, n * 8);
  return t;
}

void ProcessGroupCommunicator::allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) {
  std::vector<at::Tensor> in{hostWords(send, count)};
  std::vector<std::vector<at::Tensor>> out(1);
  for (uint32_t r = 0; r < size(); ++r) out[0].push_back(at::empty({(int64_t)count}, at::kLong));
  waitBounded(pg_->allgather(out, in), "gloo allgather");
  for (uint32_t r = 0; r < size(); ++r) std::memcpy(recv + r * count, out[0][r].data_ptr(), count * 8);
}

void ProcessGroupCommunicator::allReduceSumHost(uint64_t *data, size_t count) {
  std::vector<at::Tensor> t{hostWords(data, count)};
  waitBounded(pg_->allreduce(t), "gloo allreduce");
  std::memcpy(data, t[0].data_ptr(), count * 8);
}

void ProcessGroupCommunicator::barrier() { waitBounded(pg_->barrier(), "gloo barrier"); }

void ProcessGroupCommunicator::allToAllV(const uint64_t *send, const uint64_t *sendCounts,
                                         const uint64_t *sendDispls, uint64_t *recv, const uint64_t *recvCounts,
                                         const uint64_t *recvDispls, Location loc, hipStream_t) {
  JOIN_ASSERT(loc == Location::Host, "PGComm", "ProcessGroupCommunicator moves host buffers only");
  const uint32_t N = size();
  std::vector<int64_t> ss(N), rs(N);
  uint64_t st = 0, rt = 0;
  for (uint32_t p = 0; p < N; ++p) {
    JOIN_ASSERT(sendDispls[p] == sendDispls[0] + st && recvDispls[p] == recvDispls[0] + rt, "PGComm",
                "all-to-allv regions must be contiguous and peer-ordered");
    ss[p] = (int64_t)sendCounts[p];
    rs[p] = (int64_t)recvCounts[p];
    st += sendCounts[p];
    rt += recvCounts[p];
  }
  at::Tensor in = at::from_blob(const_cast<uint64_t *>(send) + sendDispls[0], {(int64_t)st}, at::kLong);
  at::Tensor out = at::from_blob(recv + recvDispls[0], {(int64_t)rt}, at::kLong);
  waitBounded(pg_->alltoall_base(out, in, rs, ss), "gloo all-to-allv");
}

}  // namespace comm
}  // namespace hpcjoin
