// Receive window of one relation.  Reference: /root/reference/data/Window.cpp
// (MPI_Win over MPI_Alloc_mem, lock_all / Put / flush_local / unlock_all).
//
// On MI355X the window is an HBM buffer carved from the engine arena, sized
// exactly from the exchange plan, and filled by stream-ordered RCCL
// all-to-allv chunks on the exchange stream.  start()/stop()/flush() keep
// the reference's epoch API: stop() makes the compute stream wait for every
// exchange of this window (the MPI_Win_unlock_all + MPI_Barrier analog),
// without a host round trip.
#pragma once

#include <memory>

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../core/ExecContext.h"
#include "../histograms/AssignmentMap.h"
#include "../histograms/ExchangePlan.h"
#include "../histograms/GlobalHistogram.h"
#include "../kernels/kernels.h"
#include "CompressedTuple.h"
#include "Tuple.h"

namespace hpcjoin {
namespace data {

class Window {
 public:
  // ipcWindow: the receive buffer comes from ExecContext::windows() (a
  // one-sided window that peers IPC-map) instead of the workspace.
  Window(const histograms::ExchangePlan &plan, histograms::GlobalHistogram *globalHistogram,
         histograms::AssignmentMap *assignment, core::ExecContext *ctx, bool wide, bool ipcWindow = false);
  // Window of `capacityTuples` whose plan is filled in after the scatter
  // (sampled network passes: single-rank, no exchange; or N > 1, exchanged
  // with exchangeSegmented as the plan's chunks become known).
  // elemBytes 4: the window holds u32 key fragments (JoinPlan::fragments).
  Window(const histograms::ExchangePlan &plan, uint64_t capacityTuples, core::ExecContext *ctx, bool wide,
         uint32_t elemBytes = 0);
  ~Window();
  // View of exchange chunk c alone (its segments; the data is shared): stop()
  // waits for that chunk only, so the local pass and build/probe can run on a
  // chunk while later chunks are still on the links.
  std::unique_ptr<Window> chunkView(uint32_t chunk) const;
  Window(const Window &) = delete;
  Window &operator=(const Window &) = delete;

  void start();
  void stop();
  void flush();
  // Enqueue the all-to-allv of one chunk once the compute stream reaches this
  // point (the chunk's scatter kernel is already enqueued on it).
  void exchange(const void *sendBuffer, uint32_t chunk);
  // Stream on which this window's last exchange step completes.
  hipStream_t completionStream() const;
  // One-sided exchange (the reference's MPI_Win_create + MPI_Put,
  // data/Window.cpp:35-144): collective.  Every rank publishes where its
  // window lives (an IPC handle of the allocation + offset, or a plain
  // pointer for in-process ranks) and where each source's chunks land in
  // it; exchange() then copies this rank's runs straight into the owners'
  // windows, and stop() is the unlock_all + barrier: this rank's puts are
  // complete, then every rank's (HashJoin.cpp:119-121).  No receive-side
  // RCCL call, no staging through a second buffer on the receiver.
  void enableOneSided();
  bool isOneSided() const { return oneSided; }
  // Device one-sided windows: the network scatter writes every run straight
  // into its owner's window (no local send buffer, no copy afterwards).
  // directDigitBase() gives, per (chunk, partition), the absolute tuple index
  // (address / tuple bytes) of the run's first slot in the owner's window --
  // the scatter's cursors then address peer memory from a null base.
  // (Not with replicated runs of split hot partitions: those need a send buffer.)
  bool directScatter() const { return oneSided && ctx->onDevice() && plan.replicas.empty(); }
  std::vector<uint64_t> directDigitBase() const;
  // Sampled N > 1 exchange of one chunk (tasks/SampledShuffle): the send
  // buffer holds gapped claim slices, so the caller lists the filled runs.
  // send: runs per peer in peer order, `wire` = absolute word offset in the
  // packed send buffer; recv: runs per source, `raw` = window tuple offset,
  // `wire` = absolute word offset in the packed receive buffer; self: own runs,
  // `raw` = send-buffer offset, `wire` = window offset.  Words and word
  // displacements are per peer.  group0 is filled in here.  The pack waits
  // for `scattered` (the chunk's scatter) on the exchange stream.  Needs the
  // wire codec (setWireCodec); the plan's segments describe the result.
  struct SegmentedChunk {
    std::vector<kernels::WireSeg> send, recv, self;
    std::vector<uint64_t> sendWords, sendDispls, recvWords, recvDispls;
    kernels::RoundMap sendMap;  // slot map of the send buffer (send / self `raw` are logical positions)
  };
  void exchangeSegmented(const uint64_t *sendBuffer, uint32_t chunk, SegmentedChunk &&sc, hipEvent_t scattered);
  // Bit-pack tuples on the wire (kernels.h, WireCodec); ridBase[rank * C + c]
  // is the rid base of sender `rank`'s chunk c (C = ridBase.size() / ranks).
  // Call before the first exchange.
  void setWireCodec(const kernels::WireCodec &codec, const std::vector<uint64_t> &ridBase);
  const kernels::WireCodec &wireCodec() const { return codec; }
  uint64_t wireBytesSent() const { return wireSent * 8; }  // bytes this rank put on the links (all chunks)

  CompressedTuple *getPartition(uint32_t partitionId);  // partition-major (after local partitioning)
  Tuple *getWidePartition(uint32_t partitionId);
  uint64_t getPartitionSize(uint32_t partitionId);
  uint64_t computeLocalWindowSize();
  uint64_t computeWindowSize(uint32_t nodeId);
  void assertAllTuplesWritten();

  void *getData() { return data; }
  // Slot map of a sampled single-rank network window (kernels::RoundMap):
  // the plan's segment offsets are logical positions; identity by default.
  void setRoundMap(const kernels::RoundMap &m) { roundMap_ = m; }
  const kernels::RoundMap &roundMap() const { return roundMap_; }
  // N > 1: the send buffer feeding this window had round-interleaved slices
  // (informational: the window itself is linear).
  void setSendRounded(bool on) { sendRounded_ = on; }
  bool sendRounded() const { return sendRounded_; }
  // An event recorded behind every kernel that writes the window's data (the
  // sampled single-rank scatter), or null: the local pass may then start its
  // histogram on another stream as soon as this event has fired.
  void setDataReady(hipEvent_t e) { dataReady_ = e; }
  hipEvent_t dataReady() const { return dataReady_; }
  uint32_t tupleBytes() const { return elemBytes ? elemBytes : (wide ? 16 : 8); }
  bool holdsFragments() const { return elemBytes == 4; }
  bool isWide() const { return wide; }
  const histograms::ExchangePlan &getPlan() const { return plan; }
  // Local partitioning hands back its partition-major output.
  // partEnd: null when partitions are contiguous (end of p = partBegin[p + 1]).
  // hi: the fragment column of the split layout (kernels.h, SplitLayout);
  // partitioned is then the u32 rid column.
  // capacity: elements of the partitioned buffers (0 = the window size).
  void setPartitioned(void *partitioned, const uint64_t *partBegin, uint32_t localBits,
                      const uint64_t *partEnd = nullptr, uint16_t *hi = nullptr, uint64_t capacity = 0);
  uint64_t getPartitionedCapacity() const { return partitionedCapacity; }
  const uint16_t *getPartitionedHi() const { return partitionedHi; }  // null unless split
  void *getPartitionedData() const { return partitioned; }
  const uint64_t *getPartitionBegin() const { return partBegin; }  // [owned * 2^localBits + 1] (ctx location)
  const uint64_t *getPartitionEnd() const { return partEnd; }      // null, or [owned * 2^localBits] (gapped)
  uint32_t getLocalBits() const { return localBits; }

 protected:
  uint64_t localWindowSize;
  void *data;

 private:
  Window(std::unique_ptr<histograms::ExchangePlan> ownPlan, void *data, core::ExecContext *ctx, bool wide,
         hipEvent_t arrived);
  std::unique_ptr<histograms::ExchangePlan> ownedPlan;  // chunk views only
  const histograms::ExchangePlan &plan;
  hipEvent_t viewArrived = nullptr;  // chunk views: the parent's event for that chunk
  histograms::GlobalHistogram *globalHistogram;
  histograms::AssignmentMap *assignment;
  core::ExecContext *ctx;
  bool wide;
  kernels::RoundMap roundMap_;
  bool sendRounded_ = false;
  hipEvent_t dataReady_ = nullptr;
  uint32_t elemBytes = 0;  // 0: the tuple format's size
  bool open = false;
  std::vector<hipEvent_t> ready, done;
  std::vector<bool> exchanged;
  void exchangePacked(const uint64_t *send, uint32_t chunk);
  kernels::WireCodec codec;
  std::vector<uint64_t> ridBase;
  uint32_t ridBaseChunks = 1;
  // Per-chunk segment lists: kept alive until the join ends (async H2D source).
  std::vector<std::vector<kernels::WireSeg>> sendSegs, recvSegs;
  std::vector<SegmentedChunk> segmented;  // exchangeSegmented chunks (host copies, for inspection)
  void createExchangeEvents();
  std::vector<hipEvent_t> wired;  // chunk's all-to-allv done (exchange stream -> decode stream)
  uint64_t wireSent = 0;
  void *partitioned = nullptr;
  const uint64_t *partBegin = nullptr;
  const uint64_t *partEnd = nullptr;
  uint32_t localBits = 0;
  uint16_t *partitionedHi = nullptr;
  uint64_t partitionedCapacity = 0;
  // One-sided state: peer p's window base (mapped), and the tuple offset of
  // this rank's chunk-c run in it: peerOffset[p * chunks + c].
  bool oneSided = false, oneSidedComplete = false;
  std::vector<uint8_t *> peerBase;
  std::vector<uint64_t> peerOffset;
  void putChunk(const void *send, uint32_t chunk);
};

}  // namespace data
}  // namespace hpcjoin
