// Communication layer.  The reference uses MPI-3:
// Allreduce + Exscan for histograms, one-sided RMA (Win_create / Put /
// flush) for the tuple shuffle, Send/Recv for distribute() and results.
// Here every one of those maps onto three primitives:
//   allGatherHost  - histograms of all ranks (replaces Allreduce + Exscan: each
//                    rank derives the global histogram AND its exclusive prefix
//                    over ranks locally from one all-gather)
//   allToAllV      - the tuple shuffle (replaces Win_create/Put/flush): RCCL
//                    grouped ncclSend/ncclRecv over direct xGMI peer links,
//                    stream-ordered so it overlaps the next scatter kernel
//   allReduceSumHost / barrier - result count and phase fences
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../core/Types.h"

namespace hpcjoin {
namespace comm {

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual uint32_t rank() const = 0;
  virtual uint32_t size() const = 0;
  // Where allToAllV buffers must live (Device for RCCL, Host for gloo).
  virtual bool supports(Location loc) const = 0;
  virtual std::string name() const = 0;
  // True when every rank runs in this process (threads): one-sided windows
  // are then plain pointers instead of IPC-mapped allocations.
  virtual bool sharesAddressSpace() const { return size() == 1; }
  // Failure detection: throw if the communicator has seen an asynchronous
  // error (RCCL) or a peer aborted (in-process).  Polled by blocking waits.
  virtual void checkHealth() {}
  // Tear the communicator down so that peers blocked in collectives fail
  // instead of hanging (ncclCommAbort / group abort).  Idempotent.
  virtual void abort(const std::string &why) { (void)why; }

  // recv[r * count + i] = rank r's send[i]   (host buffers, blocking)
  virtual void allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) = 0;
  // Same on device buffers, enqueued on `stream` in issue order with the
  // stream's other collectives (RCCL: no host sync).  The default stages
  // through the host and completes before returning.
  virtual void allGatherDevice(const uint64_t *send, uint64_t *recv, size_t count, hipStream_t stream);
  // data[i] = sum over ranks (host buffer, blocking)
  virtual void allReduceSumHost(uint64_t *data, size_t count) = 0;
  // Same on a device buffer, in place, enqueued on `stream` (RCCL: ncclAllReduce,
  // no host sync).  The default stages through the host and completes before
  // returning.  Used for the replicated bitmaps (disjoint bits: sum == OR).
  virtual void allReduceSumDevice(uint64_t *data, size_t count, hipStream_t stream);
  virtual void barrier() = 0;
  // Variable all-to-all of 8-byte words.  Counts / displacements are per peer
  // and in words.  Device communicators enqueue on `stream` and return;
  // host communicators complete before returning.
  virtual void allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls,
                         uint64_t *recv, const uint64_t *recvCounts, const uint64_t *recvDispls,
                         Location loc, hipStream_t stream) = 0;
};

// World of one: no communication at all (single GPU / single process).
class LocalCommunicator : public Communicator {
 public:
  uint32_t rank() const override { return 0; }
  uint32_t size() const override { return 1; }
  bool supports(Location) const override { return true; }
  std::string name() const override { return "local"; }
  void allGatherHost(const uint64_t *send, uint64_t *recv, size_t count) override;
  void allReduceSumHost(uint64_t *, size_t) override {}
  void barrier() override {}
  void allToAllV(const uint64_t *send, const uint64_t *sendCounts, const uint64_t *sendDispls, uint64_t *recv,
                 const uint64_t *recvCounts, const uint64_t *recvDispls, Location loc, hipStream_t stream) override;
};

}  // namespace comm
}  // namespace hpcjoin
