// Per-engine execution state shared by the tasks of one HashJoin: where the
// data lives, the HIP streams, the communicator and the workspace arenas.
// The reference has none of this (everything is a static or an MPI global).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "JoinConfig.h"
#include "Types.h"

namespace hpcjoin {
namespace comm {
class Communicator;
}
namespace memory {
class Arena;
}
namespace performance {
class Timeline;
}
namespace kernels {
struct DeviceControl;
struct ResultMailbox;
}

namespace core {

class ExecContext {
 public:
  // device < 0 selects the host reference path.
  ExecContext(Location loc, int device, comm::Communicator *comm);
  ~ExecContext();
  ExecContext(const ExecContext &) = delete;
  ExecContext &operator=(const ExecContext &) = delete;

  Location location() const { return loc_; }
  bool onDevice() const { return loc_ == Location::Device; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }          // compute stream
  hipStream_t commStream() const { return commStream_; }  // exchange stream (overlaps compute)
  hipStream_t decodeStream() const { return decodeStream_; }  // wire unpack (overlaps the next exchange)
  comm::Communicator *comm() const { return comm_; }
  uint32_t nodeId() const;
  uint32_t numberOfNodes() const;
  memory::Arena &workspace() { return *workspace_; }  // data-side scratch (HBM or host), reset per join
  memory::Arena &staging() { return *staging_; }      // pinned host scratch for plans/results, reset per join
  // Receive windows of one-sided exchanges (peers IPC-map them): rewound per
  // join like the workspace but never freed before the context is -- a
  // freed allocation's address can come back with the same IPC handle bytes,
  // and the runtime then hands a peer's re-open its still-referenced mapping
  // of the freed memory (see ipcExport).  Growth adds allocations at new
  // addresses, so an exported handle always names live memory.
  memory::Arena &windows() { return *windows_; }
  performance::Timeline &timeline() { return *timeline_; }  // sub-phase spans of the current join (.perf keys)

  void synchronize() const;                 // compute + comm streams
  // Async on s (default: stream()).
  void copy(void *dst, const void *src, uint64_t bytes, bool toDevice, bool fromDevice, hipStream_t s = nullptr) const;
  // Device -> host read-back on stream s (default: stream()).  Into the
  // pinned staging arena it is one of the engine's own kernels writing the
  // mapped host memory (no copy engine, no runtime blit kernel); elsewhere a
  // runtime copy.  The host reads dst after an event recorded behind it.
  void readBack(void *dst, const void *src, uint64_t bytes, hipStream_t s = nullptr) const;
  // Zero device memory on stream s (default: stream()) with the engine's own
  // kernel when 8-byte aligned, else a runtime fill.
  void zero(void *dev, uint64_t bytes, hipStream_t s = nullptr) const;
  void resetScratch();
  // Synchronisation event (timing disabled) from a per-context pool, valid
  // until the next resetScratch(): joins reuse the same events instead of
  // creating and destroying several per join.
  hipEvent_t acquireEvent();
  // One-sided exchange (JoinConfig::exchange = OneSided): the IPC handle of
  // the device allocation holding `p` (8 words), p's offset in it, the
  // workspace generation (memory::Arena::generation), and the allocation's
  // tag (offset of its Arena::TAG_BYTES tail, and the nonce this export
  // wrote there); and the mapping of a peer's exported allocation, cached per
  // (peer, handle) while the peer's generation is unchanged.
  //
  // ROCm's handle is derived from the allocation's address: a new allocation
  // at a freed one's address exports the SAME handle bytes, and while this
  // process still holds any open mapping of the old handle, opening the new
  // one returns that mapping of the FREED memory -- puts through it are lost
  // (tests/ipc_order_worker.py; round 4's inexact one-sided join).  So a
  // peer whose generation moved has its mappings closed before the open, and
  // every fresh open reads the tag back: a nonce other than the one the
  // exporter sent means a stale mapping, and the import throws.
  void ipcExport(const void *p, uint64_t handle[8], uint64_t *offset, uint64_t *generation, uint64_t *tagOffset,
                 uint64_t *nonce);
  void *ipcImport(uint32_t peer, const uint64_t handle[8], uint64_t generation, uint64_t tagOffset, uint64_t nonce);
  size_t ipcMappings() const { return ipcImported_.size(); }
  // Between joins, before any rank frees workspace memory (trim_workspace,
  // a plan that re-lays the workspace out at N > 1): every rank closes its
  // mappings of peers' memory, then a barrier, then the frees -- so no
  // mapping outlives the allocation it names and no handle is opened after
  // its allocation is gone (HashJoin::makeJoinPlan, module.cpp trim_workspace).
  // Imports are re-opened at the next join.
  void releaseImports();
  // Every export / open / close of this context, in order (the last 4096):
  // op 'E' export (cached = true: the allocation's handle of this
  // generation was handed out again), 'O' open, 'C' close of a stale
  // mapping, 'R' releaseImports.  handleHash = FNV-1a of the 64 handle bytes.
  struct IpcEvent {
    char op;
    bool cached;
    uint32_t peer;
    uint64_t generation;
    uint64_t handleHash;
    const void *ptr;
  };
  const std::vector<IpcEvent> &ipcLog() const { return ipcLog_; }

  // Persistent join scratch of a device engine (kernels::DeviceControl):
  // zeroed once here; the kernels that consume it return it to zero, so the
  // bitmap join issues no memset.  A join that ends in an exception may leave
  // it dirty: beginControl() re-zeroes it before the next use then.
  kernels::DeviceControl *control() const { return control_; }
  void beginControl();
  void endControl() { controlDirty_ = false; }
  // Host-mapped result mailbox (kernels::ResultMailbox): the device alias for
  // kernels, the next sequence number, and a spin wait for it (no runtime
  // call, no interrupt wake-up).  waitMailbox returns false when seq did not
  // arrive within the communicator timeout (the caller then synchronises the
  // streams, which reports a device fault).
  kernels::ResultMailbox *mailboxDevice() const { return mailboxDev_; }
  const kernels::ResultMailbox &mailbox() const { return *mailboxHost_; }
  uint64_t nextMailboxSeq() { return ++mailboxSeq_; }
  bool waitMailbox(uint64_t seq) const;

 private:
  kernels::DeviceControl *control_ = nullptr;
  bool controlDirty_ = false;
  kernels::ResultMailbox *mailboxHost_ = nullptr;
  kernels::ResultMailbox *mailboxDev_ = nullptr;
  uint64_t mailboxSeq_ = 0;
  void warmRuntimeCopies();
  static constexpr uint64_t kStagingReserve = 4ull << 20;

  Location loc_;
  std::vector<hipEvent_t> events_;
  size_t eventsUsed_ = 0;
  int device_;
  comm::Communicator *comm_;
  hipStream_t stream_ = nullptr;
  // IPC tag reads / writes: a private non-blocking stream and pinned words,
  // so the checks never wait behind work queued on the engine's streams.
  hipStream_t tagStream_ = nullptr;
  uint64_t *tagHost_ = nullptr;
  void tagRead(const void *devTag, uint64_t out[2]);
  void tagWrite(void *devTag, const uint64_t in[2]);
  hipStream_t commStream_ = nullptr;
  hipStream_t decodeStream_ = nullptr;
  std::unique_ptr<memory::Arena> workspace_;
  std::unique_ptr<memory::Arena> staging_;
  std::unique_ptr<memory::Arena> windows_;
  std::unique_ptr<performance::Timeline> timeline_;
  struct IpcMapping {
    uint32_t peer;
    std::vector<uint64_t> handle;
    uint64_t generation;
    void *base;
    uint64_t nonce;
  };
  std::vector<IpcMapping> ipcImported_;
  // One export per allocation and arena generation: a second
  // hipIpcGetMemHandle of the same allocation (the join's second window in
  // the same chunk) while a peer is still opening the first handle was the
  // suspected cause of intermittent open failures ("invalid device pointer")
  // and one inexact one-sided join at 4 ranks.
  struct IpcExport {
    const memory::Arena *arena;
    void *base;
    uint64_t generation;
    hipIpcMemHandle_t handle;
    uint64_t tagOffset, nonce;
  };
  uint64_t exportSerial_ = 0;
  std::vector<IpcExport> ipcExported_;
  std::vector<IpcEvent> ipcLog_;
  void logIpc(char op, bool cached, uint32_t peer, uint64_t generation, const void *handle, const void *ptr);
};

}  // namespace core
}  // namespace hpcjoin
