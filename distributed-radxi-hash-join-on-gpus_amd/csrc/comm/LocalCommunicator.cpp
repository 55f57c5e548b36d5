#include <cstring>
#include <vector>

#include "../utils/Hip.h"
#include "Communicator.h"

namespace hpcjoin {
namespace comm {

void Communicator::allGatherDevice(const uint64_t *send, uint64_t *recv, size_t count, hipStream_t stream) {
  std::vector<uint64_t> mine(count), all(count * size());
  HIP_CHECK(hipStreamSynchronize(stream));
  if (count) HIP_CHECK(hipMemcpy(mine.data(), send, count * 8, hipMemcpyDeviceToHost));
  allGatherHost(mine.data(), all.data(), count);
  if (count) HIP_CHECK(hipMemcpy(recv, all.data(), all.size() * 8, hipMemcpyHostToDevice));
}

void Communicator::allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream) {
  if (size() == 1 || count == 0) return;
  std::vector<uint64_t> h(count);
  HIP_CHECK(hipStreamSynchronize(stream));
  HIP_CHECK(hipMemcpy(h.data(), data, count * 8, hipMemcpyDeviceToHost));
  allReduceSumHost(h.data(), count);
  HIP_CHECK(hipMemcpy(data, h.data(), count * 8, hipMemcpyHostToDevice));
}

void LocalCommunicator::allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) {
  if (send != recv) std::memmove(recv, send, count * sizeof(uint64_t));
}

void LocalCommunicator::allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls,
                                  uint64_t *recv, const uint64_t *recvCounts, const uint64_t *recvDispls,
                                  Location loc, hipStream_t stream) {
  HJ_CHECK(sendCounts[0] == recvCounts[0], "local all-to-all: send %lu != recv %lu",
           (unsigned long)sendCounts[0], (unsigned long)recvCounts[0]);
  const uint64_t *src = send + sendDispls[0];
  uint64_t *dst = recv + recvDispls[0];
  if (src == dst || sendCounts[0] == 0) return;
  if (loc == Location::Device)
    HIP_CHECK(hipMemcpyAsync(dst, src, sendCounts[0] * 8, hipMemcpyDeviceToDevice, stream));
  else
    std::memmove(dst, src, sendCounts[0] * 8);
}

}  // namespace comm
}  // namespace hpcjoin
