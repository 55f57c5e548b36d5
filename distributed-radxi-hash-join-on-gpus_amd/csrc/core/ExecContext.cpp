#include "ExecContext.h"

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <mutex>
#include <set>
#include <immintrin.h>

#include "../comm/Communicator.h"
#include "../kernels/kernels.h"
#include "../memory/Arena.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../performance/Trace.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace core {

ExecContext::ExecContext(Location loc, int device, comm::Communicator *comm)
    : loc_(loc), device_(device < 0 ? 0 : device), comm_(comm) {
  JOIN_ASSERT(comm_ != nullptr, "ExecContext", "a communicator is required");
  JOIN_ASSERT(comm_->size() == 1 || comm_->supports(loc), "ExecContext", "communicator %s cannot move %s buffers",
              comm_->name().c_str(), locationName(loc));
  utils::setDebugRank((int)comm_->rank());
  workspace_.reset(new memory::Arena(loc, device_));
  windows_.reset(new memory::Arena(loc, device_));
  // Pinned on a device engine: host->device uploads and device->host result
  // copies through it are true DMA transfers that never block the host.
  staging_.reset(new memory::Arena(onDevice() ? Location::Pinned : Location::Host, device_));
  timeline_.reset(new performance::Timeline(onDevice()));
  if (onDevice()) {
    HIP_CHECK(hipSetDevice(device_));
    {
      // Code objects of the join kernels, once per process and device.
      static std::mutex m;
      static std::set<int> loaded;
      std::lock_guard<std::mutex> g(m);
      if (loaded.insert(device_).second) kernels::preloadCodeObjects();
    }
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    // The exchange stream (RCCL collectives, window copies) gets the highest
    // priority: its few long-running blocks are dispatched ahead of the
    // remaining blocks of a partitioning kernel it overlaps, instead of
    // waiting for CUs behind them.
    int leastPrio = 0, greatestPrio = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&leastPrio, &greatestPrio));
    HIP_CHECK(hipStreamCreateWithPriority(&commStream_, hipStreamNonBlocking, greatestPrio));
    HIP_CHECK(hipStreamCreateWithFlags(&decodeStream_, hipStreamNonBlocking));
    HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&control_), sizeof(kernels::DeviceControl)));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&mailboxHost_), sizeof(kernels::ResultMailbox),
                            hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(mailboxHost_, 0, sizeof(kernels::ResultMailbox));
    HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&mailboxDev_), mailboxHost_, 0));
    // Event pools filled now (a join uses ~6 timing and a few sync events):
    // creating them lazily put ~0.1 ms of hipEventCreate into the first join.
    timeline_->reserveEvents(32);
    for (int i = 0; i < 32; ++i) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      events_.push_back(e);
    }
    warmRuntimeCopies();
  }
  // First uses that would otherwise land in the first join: the roctx
  // library's lazy start (a join opens its range first thing) and the
  // measurement key table (built on the first startJoin).
  { performance::TraceRange warm("hpcjoin::engine_start"); }
  (void)performance::Measurements::referenceKeys();
}

// The runtime loads its copy / fill kernels on first use: the first join of
// a process paid ~17 ms in its network phase for it (docs/ROUND4.md, 1e8 x
// 4e8 sparse keys; nothing of it under rocprofv3, whose copies are kernels
// it loads itself).  One tiny fill and one copy of each direction on the
// engine's compute stream move that cost here, and the fill zeroes the
// control block.
void ExecContext::warmRuntimeCopies() {
  // Pinned scratch for a join's small read-backs (claim cursors, counters:
  // tens of KiB): reserved now, so a first join does not pay a pinned
  // allocation (~ms) in the middle of its network phase.
  staging_->ensure(kStagingReserve);
  // One timed span, queried and resolved the way a join's timeline is, so the
  // runtime's first-use work for timing events (first record / query /
  // elapsed-time) happens here and not around the first join.
  hipEvent_t t0 = timeline_->mark(stream_), t1 = nullptr;
  kernels::zeroWords(control_, sizeof(kernels::DeviceControl) / 8, stream_);
  t1 = timeline_->mark(stream_);
  if (t1) utils::waitEvent(t1, comm_, "engine start");
  HIP_CHECK(hipStreamSynchronize(stream_));
  {
    float ms = 0;
    if (t0 && t1) HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
  }
  timeline_->reset();
  const char *w = std::getenv("HPCJOIN_WARM_COPIES");
  if (w && w[0] == '0') {
    HIP_CHECK(hipStreamSynchronize(stream_));
    return;
  }
  HIP_CHECK(hipMemsetAsync(reinterpret_cast<uint8_t *>(control_) + offsetof(kernels::DeviceControl, pad), 0, 16,
                           stream_));
  void *pinned = staging_->get(256);
  std::memset(pinned, 0, 256);
  uint8_t *dev = reinterpret_cast<uint8_t *>(control_) + offsetof(kernels::DeviceControl, pad);
  HIP_CHECK(hipMemcpyAsync(dev, pinned, 32, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t *>(pinned) + 64, dev, 32, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(dev + 32, dev, 16, hipMemcpyDeviceToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  staging_->reset();
}

void ExecContext::beginControl() {
  if (controlDirty_) kernels::zeroWords(control_, sizeof(kernels::DeviceControl) / 8, stream_);
  controlDirty_ = true;
}

bool ExecContext::waitMailbox(uint64_t seq) const {
  using clk = std::chrono::steady_clock;
  const auto deadline = clk::now() + std::chrono::milliseconds(utils::commTimeoutMs());
  const volatile unsigned long long *p = &mailboxHost_->seq;
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(p, __ATOMIC_ACQUIRE) >= seq) return true;
    _mm_pause();
    if ((spin & 4095) == 0) {
      // A faulted kernel never publishes: poll the stream for its error.
      const hipError_t e = hipStreamQuery(stream_);
      if (e != hipSuccess && e != hipErrorNotReady) HIP_CHECK(e);
      if (e == hipSuccess && __atomic_load_n(p, __ATOMIC_ACQUIRE) < seq) return false;
      if (clk::now() > deadline) return false;
    }
  }
}

ExecContext::~ExecContext() {
  for (auto &m : ipcImported_) (void)hipIpcCloseMemHandle(m.base);
  if (control_) (void)hipFree(control_);
  if (mailboxHost_) (void)hipHostFree(mailboxHost_);
  for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  timeline_.reset();
  workspace_.reset();
  staging_.reset();
  windows_.reset();
  if (stream_) (void)hipStreamDestroy(stream_);
  if (tagStream_) (void)hipStreamDestroy(tagStream_);
  if (tagHost_) (void)hipHostFree(tagHost_);
  if (commStream_) (void)hipStreamDestroy(commStream_);
  if (decodeStream_) (void)hipStreamDestroy(decodeStream_);
}

uint32_t ExecContext::nodeId() const { return comm_->rank(); }
uint32_t ExecContext::numberOfNodes() const { return comm_->size(); }

// Polled waits (utils::waitStream): a lost peer cannot hang this rank
// forever, and the host sees the end of the join's last kernel within
// microseconds instead of after a runtime sleep on an interrupt.
void ExecContext::synchronize() const {
  if (!onDevice()) return;
  utils::waitStream(commStream_, comm_, "exchange stream");
  utils::waitStream(decodeStream_, comm_, "decode stream");
  utils::waitStream(stream_, comm_, "compute stream");
}

void ExecContext::copy(void *dst, const void *src, uint64_t bytes, bool toDevice, bool fromDevice,
                       hipStream_t s) const {
  if (bytes == 0) return;
  if (!s) s = stream_;
  if (!onDevice()) {
    std::memcpy(dst, src, bytes);
    return;
  }
  hipMemcpyKind k = toDevice ? (fromDevice ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                             : (fromDevice ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
  // Small uploads go through the pinned staging arena (rewound per join,
  // after the previous join's final synchronisation), so they are DMA
  // transfers ordered on the stream rather than runtime-staged pageable
  // copies.  (A/B on the 1B and 128M joins: no measurable change there; it
  // keeps uploads issued mid-exchange from depending on pageable staging.)
  if (toDevice && !fromDevice && bytes <= (64ull << 20) && !staging_->owns(src)) {
    void *p = staging_->get(bytes);
    std::memcpy(p, src, bytes);
    src = p;
  }
  // Uploads out of the staging arena are read by one of the engine's own
  // kernels over the host link (no copy engine: bench_skew's first join paid
  // ~5-10 ms in its local pass for the first SDMA upload of a process).
  if (toDevice && !fromDevice && staging_->owns(src)) {
    kernels::copyFromHost(dst, src, bytes, s);
    return;
  }
  HIP_CHECK(hipMemcpyAsync(dst, src, bytes, k, s));
}

void ExecContext::readBack(void *dst, const void *src, uint64_t bytes, hipStream_t s) const {
  if (bytes == 0) return;
  if (!onDevice()) {
    std::memcpy(dst, src, bytes);
    return;
  }
  if (!s) s = stream_;
  if (staging_->owns(dst))
    kernels::copyToHost(dst, src, bytes, s);
  else
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
}

void ExecContext::zero(void *dev, uint64_t bytes, hipStream_t s) const {
  if (bytes == 0) return;
  if (!onDevice()) {
    std::memset(dev, 0, bytes);
    return;
  }
  if (!s) s = stream_;
  if (((reinterpret_cast<uintptr_t>(dev) | bytes) & 7) == 0)
    kernels::zeroWords(dev, bytes / 8, s);
  else
    HIP_CHECK(hipMemsetAsync(dev, 0, bytes, s));
}

void ExecContext::resetScratch() {
  workspace_->reset();
  staging_->reset();
  windows_->reset();
  eventsUsed_ = 0;
}

void ExecContext::logIpc(char op, bool cached, uint32_t peer, uint64_t generation, const void *handle,
                         const void *ptr) {
  uint64_t h = 1469598103934665603ull;
  if (handle)
    for (size_t i = 0; i < sizeof(hipIpcMemHandle_t); ++i) h = (h ^ static_cast<const uint8_t *>(handle)[i]) * 1099511628211ull;
  if (ipcLog_.size() >= 4096) ipcLog_.erase(ipcLog_.begin(), ipcLog_.begin() + 1024);
  ipcLog_.push_back(IpcEvent{op, cached, peer, generation, handle ? h : 0, ptr});
}

// The 16-byte IPC tag of an allocation, read or written with the engine's own
// copy kernels on a private non-blocking stream (no null-stream copy, nothing
// queued on the join's streams in front of it).
void ExecContext::tagRead(const void *devTag, uint64_t out[2]) {
  HIP_CHECK(hipSetDevice(device_));
  if (!tagStream_) HIP_CHECK(hipStreamCreateWithFlags(&tagStream_, hipStreamNonBlocking));
  if (!tagHost_) HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&tagHost_), 64, hipHostMallocMapped));
  kernels::copyToHost(tagHost_, devTag, 16, tagStream_);
  utils::waitStream(tagStream_, nullptr, "IPC tag read");
  out[0] = tagHost_[0];
  out[1] = tagHost_[1];
}

void ExecContext::tagWrite(void *devTag, const uint64_t in[2]) {
  HIP_CHECK(hipSetDevice(device_));
  if (!tagStream_) HIP_CHECK(hipStreamCreateWithFlags(&tagStream_, hipStreamNonBlocking));
  if (!tagHost_) HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&tagHost_), 64, hipHostMallocMapped));
  tagHost_[2] = in[0];
  tagHost_[3] = in[1];
  kernels::copyFromHost(devTag, tagHost_ + 2, 16, tagStream_);
  // Complete before the handle is published (importers read the tag).
  utils::waitStream(tagStream_, nullptr, "IPC tag write");
}

void ExecContext::ipcExport(const void *p, uint64_t handle[8], uint64_t *offset, uint64_t *generation,
                            uint64_t *tagOffset, uint64_t *nonce) {
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "unexpected hipIpcMemHandle_t size");
  JOIN_ASSERT(onDevice(), "ExecContext", "IPC export of host memory");
  memory::Arena *arena = windows_->allocationOf(p) ? windows_.get() : workspace_.get();
  void *base = arena->allocationOf(p);
  JOIN_ASSERT(base != nullptr, "ExecContext", "IPC export: %p is not in the workspace", p);
  const uint64_t gen = arena->generation();
  // Entries of older generations name freed allocations: drop them.
  ipcExported_.erase(std::remove_if(ipcExported_.begin(), ipcExported_.end(),
                                    [&](const IpcExport &x) { return x.arena == arena && x.generation != gen; }),
                     ipcExported_.end());
  const IpcExport *hit = nullptr;
  for (const auto &x : ipcExported_)
    if (x.base == base) hit = &x;
  const bool cached = hit != nullptr;
  if (hit) {
    // The tag must still be this export's: anything else is a write past
    // the end of a workspace buffer (the tag is the allocation's tail).
    uint64_t stamp[2] = {0, 0};
    tagRead(static_cast<const uint8_t *>(hit->base) + hit->tagOffset, stamp);
    JOIN_ASSERT(stamp[0] == hit->nonce && stamp[1] == gen, "ExecContext",
                "IPC export: the tag of allocation %p (generation %lu) was overwritten: nonce %016lx gen %lu, "
                "expected %016lx gen %lu -- a write past the end of a workspace buffer",
                hit->base, (unsigned long)gen, (unsigned long)stamp[0], (unsigned long)stamp[1],
                (unsigned long)hit->nonce, (unsigned long)gen);
  }
  if (!hit) {
    IpcExport x{arena, base, gen, {}, 0, 0};
    HIP_CHECK(hipIpcGetMemHandle(&x.handle, base));
    uint8_t *tag = static_cast<uint8_t *>(arena->tagOf(base));
    JOIN_ASSERT(tag != nullptr, "ExecContext", "IPC export: allocation %p has no tag", base);
    x.tagOffset = (uint64_t)(tag - static_cast<uint8_t *>(base));
    // Unique per process and export: pid, a serial, and the clock.
    x.nonce = ((uint64_t)getpid() << 40) ^ (++exportSerial_ << 20) ^
              (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    const uint64_t stamp[2] = {x.nonce, gen};
    // Complete before the handle is published (a synchronous hipMemcpy from
    // pageable memory may return once the source is staged, before the DMA
    // lands: importers then read the previous tag, seen at 8 ranks).
    tagWrite(tag, stamp);
    ipcExported_.push_back(x);
    hit = &ipcExported_.back();
  }
  logIpc('E', cached, comm_ ? comm_->rank() : 0, gen, &hit->handle, base);
  std::memcpy(handle, &hit->handle, sizeof(hit->handle));
  *offset = (uint64_t)(static_cast<const uint8_t *>(p) - static_cast<const uint8_t *>(base));
  *generation = gen;
  *tagOffset = hit->tagOffset;
  *nonce = hit->nonce;
}

void *ExecContext::ipcImport(uint32_t peer, const uint64_t handle[8], uint64_t generation, uint64_t tagOffset,
                             uint64_t nonce) {
  std::vector<uint64_t> key(handle, handle + 8);
  for (size_t i = 0; i < ipcImported_.size();) {
    IpcMapping &m = ipcImported_[i];
    // Stale: the peer FREED memory since this mapping was opened (its arena's
    // generation counts frees only, and frees happen between joins), so no
    // window of the current join points into it.  Growth inside a join (a
    // fallback allocation behind the peer's second window) keeps the
    // generation: the first window's mapping stays open.
    if (m.peer == peer && m.generation != generation) {
      logIpc('C', false, peer, m.generation, m.handle.data(), m.base);
      HIP_CHECK(hipIpcCloseMemHandle(m.base));
      ipcImported_.erase(ipcImported_.begin() + i);
      continue;
    }
    if (m.peer == peer && m.handle == key) {
      JOIN_ASSERT(m.nonce == nonce, "ExecContext",
                  "IPC import from rank %u: a cached mapping of generation %lu carries another export's tag", peer,
                  (unsigned long)generation);
      return m.base;
    }
    ++i;
  }
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  void *ptr = nullptr;
  HIP_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
  logIpc('O', false, peer, generation, &h, ptr);
  uint64_t stamp[2] = {0, 0};
  tagRead(static_cast<uint8_t *>(ptr) + tagOffset, stamp);
  if (stamp[0] != nonce || stamp[1] != generation) {
    (void)hipIpcCloseMemHandle(ptr);
    JOIN_ASSERT(false, "ExecContext",
                "stale IPC mapping: rank %u's handle (generation %lu, nonce %016lx) opened memory tagged by "
                "another export (generation %lu, nonce %016lx) -- a mapping of a freed allocation at the same "
                "address is still open in this process, so puts through it would be lost",
                peer, (unsigned long)generation, (unsigned long)nonce, (unsigned long)stamp[1],
                (unsigned long)stamp[0]);
  }
  ipcImported_.push_back(IpcMapping{peer, std::move(key), generation, ptr, nonce});
  return ptr;
}

void ExecContext::releaseImports() {
  if (!ipcImported_.empty()) logIpc('R', false, 0, 0, nullptr, nullptr);
  for (auto &m : ipcImported_) HIP_CHECK(hipIpcCloseMemHandle(m.base));
  ipcImported_.clear();
}

hipEvent_t ExecContext::acquireEvent() {
  if (eventsUsed_ == events_.size()) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events_.push_back(e);
  }
  return events_[eventsUsed_++];
}

}  // namespace core
}  // namespace hpcjoin
