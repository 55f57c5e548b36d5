#include "RcclCommunicator.h"

#include <rccl/rccl.h>

#include <cstring>

#include "../utils/Fault.h"
#include "../utils/Hip.h"

#define RCCL_CHECK(expr)                                                                      \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess)                                                                    \
      ::hpcjoin::utils::fail("RCCL", __FILE__, __LINE__,                                      \
                             ::hpcjoin::utils::format("%s -> %s", #expr, ncclGetErrorString(_r))); \
  } while (0)

namespace hpcjoin {
namespace comm {

static_assert(sizeof(ncclUniqueId) == RcclCommunicator::UNIQUE_ID_BYTES, "unexpected ncclUniqueId size");

std::vector<uint8_t> RcclCommunicator::uniqueId() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  std::vector<uint8_t> out(sizeof(id));
  std::memcpy(out.data(), &id, sizeof(id));
  return out;
}

RcclCommunicator::RcclCommunicator(const std::vector<uint8_t> &id, uint32_t rank, uint32_t size, int device)
    : rank_(rank), size_(size), device_(device) {
  JOIN_ASSERT(id.size() == sizeof(ncclUniqueId), "RCCL", "unique id must be %zu bytes", sizeof(ncclUniqueId));
  utils::setDebugRank((int)rank);
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  ncclUniqueId uid;
  std::memcpy(&uid, id.data(), sizeof(uid));
  ncclComm_t c;
  RCCL_CHECK(ncclCommInitRank(&c, (int)size, uid, (int)rank));
  comm_ = c;
}

void RcclCommunicator::checkHealth() {
  JOIN_ASSERT(comm_ != nullptr, "RCCL", "communicator was aborted: %s", abortReason_.c_str());
  ncclResult_t st = ncclSuccess;
  RCCL_CHECK(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &st));
  if (st != ncclSuccess && st != ncclInProgress) {
    std::string why = utils::format("asynchronous RCCL error: %s", ncclGetErrorString(st));
    abort(why);
    utils::fail("RCCL", __FILE__, __LINE__, why);
  }
}

void RcclCommunicator::abort(const std::string &why) {
  if (!comm_) return;
  abortReason_ = why;
  (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
  comm_ = nullptr;
}

RcclCommunicator::~RcclCommunicator() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
  if (scratch_) (void)hipFree(scratch_);
  for (uint64_t *p : retired_) (void)hipFree(p);
  if (stream_) (void)hipStreamDestroy(stream_);
}

uint64_t *RcclCommunicator::scratch(size_t words) {
  if (words > scratchWords_) {
    // The outgrown buffer is kept until the communicator goes: hipFree
    // synchronises the whole device, and between ranks that would wait on
    // this process's in-flight collectives (e.g. an exchange still on the
    // links while a host collective grows the scratch).
    if (scratch_) retired_.push_back(scratch_);
    scratchWords_ = words < 4096 ? 4096 : words;
    HIP_CHECK(hipMalloc(&scratch_, scratchWords_ * 8));
  }
  return scratch_;
}

void RcclCommunicator::allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) {
  uint64_t *buf = scratch(count * size_);
  HIP_CHECK(hipMemcpyAsync(buf + count * rank_, send, count * 8, hipMemcpyHostToDevice, stream_));
  checkHealth();
  RCCL_CHECK(ncclAllGather(buf + count * rank_, buf, count, ncclUint64, static_cast<ncclComm_t>(comm_), stream_));
  HIP_CHECK(hipMemcpyAsync(recv, buf, count * size_ * 8, hipMemcpyDeviceToHost, stream_));
  utils::waitStream(stream_, this, "ncclAllGather");
  utils::noteCollective("ncclAllGather", true);
}

void RcclCommunicator::allGatherDevice(const uint64_t *send, uint64_t *recv, size_t count, hipStream_t stream) {
  checkHealth();
  RCCL_CHECK(ncclAllGather(send, recv, count, ncclUint64, static_cast<ncclComm_t>(comm_), stream));
  utils::noteCollective("ncclAllGather (stream)", false);
}

void RcclCommunicator::allReduceSumHost(uint64_t *data, size_t count) {
  uint64_t *buf = scratch(count);
  HIP_CHECK(hipMemcpyAsync(buf, data, count * 8, hipMemcpyHostToDevice, stream_));
  checkHealth();
  RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, static_cast<ncclComm_t>(comm_), stream_));
  HIP_CHECK(hipMemcpyAsync(data, buf, count * 8, hipMemcpyDeviceToHost, stream_));
  utils::waitStream(stream_, this, "ncclAllReduce");
  utils::noteCollective("ncclAllReduce", true);
}

void RcclCommunicator::allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream) {
  if (count == 0) return;
  checkHealth();
  RCCL_CHECK(ncclAllReduce(data, data, count, ncclUint64, ncclSum, static_cast<ncclComm_t>(comm_), stream));
  utils::noteCollective("ncclAllReduce (stream)", false);
}

void RcclCommunicator::barrier() {
  uint64_t one = 1;
  allReduceSumHost(&one, 1);
}

void RcclCommunicator::allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls,
                                 uint64_t *recv, const uint64_t *recvCounts, const uint64_t *recvDispls,
                                 Location loc, hipStream_t stream) {
  JOIN_ASSERT(loc == Location::Device, "RCCL", "all-to-all buffers must be in HBM");
  checkHealth();
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  // Own slice: plain D2D copy on the same stream (no RCCL channel needed).
  HJ_CHECK(sendCounts[rank_] == recvCounts[rank_], "self slice mismatch %lu != %lu",
           (unsigned long)sendCounts[rank_], (unsigned long)recvCounts[rank_]);
  if (sendCounts[rank_])
    HIP_CHECK(hipMemcpyAsync(recv + recvDispls[rank_], send + sendDispls[rank_], sendCounts[rank_] * 8,
                             hipMemcpyDeviceToDevice, stream));
  RCCL_CHECK(ncclGroupStart());
  // Stagger peers (rank+1, rank+2, ...) so that at every step each GPU talks
  // to a different partner: every xGMI link is busy, none is oversubscribed.
  for (uint32_t k = 1; k < size_; ++k) {
    const uint32_t to = (rank_ + k) % size_;
    const uint32_t from = (rank_ + size_ - k) % size_;
    if (sendCounts[to]) RCCL_CHECK(ncclSend(send + sendDispls[to], sendCounts[to], ncclUint64, (int)to, c, stream));
    if (recvCounts[from])
      RCCL_CHECK(ncclRecv(recv + recvDispls[from], recvCounts[from], ncclUint64, (int)from, c, stream));
  }
  RCCL_CHECK(ncclGroupEnd());
  utils::noteCollective("ncclSend/ncclRecv all-to-allv", false);
}

}  // namespace comm
}  // namespace hpcjoin
