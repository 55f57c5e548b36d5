#include "Window.h"

#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "../comm/Communicator.h"
#include "../host/HostOps.h"
#include "../memory/Arena.h"
#include "../performance/Measurements.h"
#include "../performance/Timeline.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace data {

Window::Window(const histograms::ExchangePlan &plan, histograms::GlobalHistogram *globalHistogram,
               histograms::AssignmentMap *assignment, core::ExecContext *ctx, bool wide, bool ipcWindow)
    : plan(plan), globalHistogram(globalHistogram), assignment(assignment), ctx(ctx), wide(wide) {
  localWindowSize = plan.recvTotal;
  data = (ipcWindow ? ctx->windows() : ctx->workspace()).get(localWindowSize * tupleBytes());
  exchanged.assign(plan.chunks, false);
  createExchangeEvents();
}

void Window::createExchangeEvents() {
  if (!ctx->onDevice() || plan.numberOfNodes == 1) return;
  ready.resize(plan.chunks);
  done.resize(plan.chunks);
  for (uint32_t c = 0; c < plan.chunks; ++c) {
    ready[c] = ctx->acquireEvent();
    done[c] = ctx->acquireEvent();
  }
}

Window::Window(const histograms::ExchangePlan &plan, uint64_t capacityTuples, core::ExecContext *ctx, bool wide,
               uint32_t elemBytes)
    : plan(plan), globalHistogram(nullptr), assignment(nullptr), ctx(ctx), wide(wide), elemBytes(elemBytes) {
  localWindowSize = capacityTuples;
  data = ctx->workspace().get(std::max<uint64_t>(capacityTuples, 1) * tupleBytes());
  exchanged.assign(std::max<uint32_t>(plan.chunks, 1), false);
  createExchangeEvents();
}

Window::Window(std::unique_ptr<histograms::ExchangePlan> ownPlan, void *data, core::ExecContext *ctx, bool wide,
               hipEvent_t arrived)
    : ownedPlan(std::move(ownPlan)), plan(*ownedPlan), globalHistogram(nullptr), assignment(nullptr), ctx(ctx),
      wide(wide), viewArrived(arrived) {
  localWindowSize = plan.recvTotal;
  this->data = data;
  exchanged.assign(std::max<uint32_t>(plan.chunks, 1), true);
}

std::unique_ptr<Window> Window::chunkView(uint32_t chunk) const {
  JOIN_ASSERT(chunk < plan.chunks, "Window", "chunk view %u of %u chunks", chunk, plan.chunks);
  std::unique_ptr<histograms::ExchangePlan> v(new histograms::ExchangePlan(plan));
  const uint32_t owned = (uint32_t)plan.owned.size();
  v->segments.clear();
  v->partSize.assign(owned, 0);
  for (const histograms::Segment &s : plan.segments)
    if (s.chunk == chunk) {
      v->segments.push_back(s);
      v->partSize[s.lp] += s.len;
    }
  v->lpBase.assign(owned + 1, 0);
  for (uint32_t lp = 0; lp < owned; ++lp) v->lpBase[lp + 1] = v->lpBase[lp] + v->partSize[lp];
  v->recvTotal = v->lpBase[owned];
  hipEvent_t arrived = chunk < done.size() ? done[chunk] : nullptr;
  return std::unique_ptr<Window>(new Window(std::move(v), data, ctx, wide, arrived));
}

Window::~Window() = default;  // events belong to the context pool

hipStream_t Window::completionStream() const {
  if (!ctx->onDevice() || plan.numberOfNodes == 1) return ctx->stream();
  return codec.w ? ctx->decodeStream() : ctx->commStream();
}

void Window::setWireCodec(const kernels::WireCodec &c, const std::vector<uint64_t> &bases) {
  JOIN_ASSERT(!wide || c.w == 0, "Window", "the wire codec packs 8-byte CompressedTuples only");
  JOIN_ASSERT(c.w == 0 || (bases.size() >= plan.numberOfNodes && bases.size() % plan.numberOfNodes == 0 &&
                            bases.size() / plan.numberOfNodes >= plan.chunks),
              "Window", "need one rid base per (rank, chunk)");
  codec = c;
  ridBase = bases;
  ridBaseChunks = c.w ? (uint32_t)(bases.size() / plan.numberOfNodes) : 1;
  if (codec.w && ctx->onDevice() && plan.numberOfNodes > 1 && wired.empty()) {
    wired.resize(plan.chunks);
    for (auto &e : wired) e = ctx->acquireEvent();
  }
}

// Packed exchange of one chunk: pack (compute stream) -> own slice copied raw
// + all-to-allv of the wire words (exchange stream) -> unpack into the window
// (decode stream, so the next chunk's all-to-allv starts right away).
void Window::exchangePacked(const uint64_t *send, uint32_t chunk) {
  const uint32_t N = plan.numberOfNodes, me = plan.nodeId;
  if (sendSegs.empty()) {
    sendSegs.resize(plan.chunks);
    recvSegs.resize(plan.chunks);
  }
  std::vector<kernels::WireSeg> &ss = sendSegs[chunk], &rs = recvSegs[chunk];
  ss.clear();
  rs.clear();
  std::vector<uint64_t> sc(N, 0), sd(N, 0), rc(N, 0), rd(N, 0);
  uint64_t sOff = 0, rOff = 0, sGroups = 0, rGroups = 0;
  for (uint32_t p = 0; p < N; ++p) {
    if (p == me) continue;
    const uint64_t n = plan.sendCounts[(size_t)chunk * N + p], m = plan.recvCounts[(size_t)chunk * N + p];
    if (n) ss.push_back({plan.sendDispls[(size_t)chunk * N + p], sOff, n, ridBase[(size_t)me * ridBaseChunks + chunk],
                         sGroups});
    sc[p] = codec.words(n);
    sd[p] = sOff;
    sOff += sc[p];
    sGroups += ceilDiv(n, 64);
    if (m) rs.push_back({plan.recvDispls[(size_t)chunk * N + p], rOff, m, ridBase[(size_t)p * ridBaseChunks + chunk],
                         rGroups});
    rc[p] = codec.words(m);
    rd[p] = rOff;
    rOff += rc[p];
    rGroups += ceilDiv(m, 64);
  }
  wireSent += sOff;
  const uint64_t selfN = plan.sendCounts[(size_t)chunk * N + me];
  const uint64_t selfSrc = plan.sendDispls[(size_t)chunk * N + me], selfDst = plan.recvDispls[(size_t)chunk * N + me];
  JOIN_ASSERT(selfN == plan.recvCounts[(size_t)chunk * N + me], "Window", "own slice mismatch");
  uint64_t *wsend = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(sOff, 1));
  uint64_t *wrecv = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(rOff, 1));
  uint64_t *dst = static_cast<uint64_t *>(data);
  if (ctx->onDevice() && N > 1) {
    kernels::WireSeg *dS = ctx->workspace().getArray<kernels::WireSeg>(std::max<size_t>(ss.size(), 1));
    kernels::WireSeg *dR = ctx->workspace().getArray<kernels::WireSeg>(std::max<size_t>(rs.size(), 1));
    ctx->copy(dS, ss.data(), ss.size() * sizeof(kernels::WireSeg), true, false);
    ctx->copy(dR, rs.data(), rs.size() * sizeof(kernels::WireSeg), true, false);
    kernels::wirePack(send, wsend, dS, (uint32_t)ss.size(), sGroups, codec, ctx->stream());
    HIP_CHECK(hipEventRecord(ready[chunk], ctx->stream()));
    HIP_CHECK(hipStreamWaitEvent(ctx->commStream(), ready[chunk], 0));
    ctx->timeline().begin("MWINPUT", ctx->commStream());
    if (selfN)
      HIP_CHECK(hipMemcpyAsync(dst + selfDst, send + selfSrc, selfN * 8, hipMemcpyDeviceToDevice,
                               ctx->commStream()));
    ctx->comm()->allToAllV(wsend, sc.data(), sd.data(), wrecv, rc.data(), rd.data(), Location::Device,
                           ctx->commStream());
    ctx->timeline().end("MWINPUT", ctx->commStream());
    HIP_CHECK(hipEventRecord(wired[chunk], ctx->commStream()));
    HIP_CHECK(hipStreamWaitEvent(ctx->decodeStream(), wired[chunk], 0));
    kernels::wireUnpack(wrecv, dst, dR, (uint32_t)rs.size(), rGroups, codec, ctx->decodeStream());
    HIP_CHECK(hipEventRecord(done[chunk], ctx->decodeStream()));
  } else {
    host::wirePack(send, wsend, ss.data(), (uint32_t)ss.size(), codec);
    if (selfN) std::memcpy(dst + selfDst, send + selfSrc, selfN * 8);
    ctx->timeline().begin("MWINPUT");
    ctx->comm()->allToAllV(wsend, sc.data(), sd.data(), wrecv, rc.data(), rd.data(), ctx->location(),
                           ctx->stream());
    ctx->timeline().end("MWINPUT");
    host::wireUnpack(wrecv, dst, rs.data(), (uint32_t)rs.size(), codec);
  }
}

void Window::exchangeSegmented(const uint64_t *send, uint32_t chunk, SegmentedChunk &&sc, hipEvent_t scattered) {
  const uint32_t N = plan.numberOfNodes;
  JOIN_ASSERT(ctx->onDevice() && N > 1 && !wide && chunk < plan.chunks, "Window",
              "segmented exchange: device, N > 1, compressed tuples");
  JOIN_ASSERT(sc.sendWords.size() == N && sc.sendDispls.size() == N && sc.recvWords.size() == N &&
                  sc.recvDispls.size() == N,
              "Window", "segmented exchange: per-peer word counts for %u ranks", N);
  auto prefix = [](std::vector<kernels::WireSeg> &v) {
    uint64_t g = 0;
    for (kernels::WireSeg &x : v) {
      x.group0 = g;
      g += ceilDiv(x.n, 64);
    }
    return g;
  };
  const uint64_t sG = prefix(sc.send), rG = prefix(sc.recv), cG = prefix(sc.self);
  uint64_t sTotal = 0, rTotal = 0;
  for (uint32_t p = 0; p < N; ++p) {
    sTotal = std::max(sTotal, sc.sendDispls[p] + sc.sendWords[p]);
    rTotal = std::max(rTotal, sc.recvDispls[p] + sc.recvWords[p]);
    if (p != plan.nodeId) wireSent += sc.sendWords[p];
  }
  uint64_t *wsend = ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(sTotal, 1));
  uint64_t *wrecv = codec.w ? ctx->workspace().getArray<uint64_t>(std::max<uint64_t>(rTotal, 1)) : nullptr;
  uint64_t *dst = static_cast<uint64_t *>(data);
  hipStream_t xs = ctx->commStream();
  HIP_CHECK(hipStreamWaitEvent(xs, scattered, 0));
  // Segment tables: pinned staging -> HBM, ordered on the exchange stream.
  auto upload = [&](const std::vector<kernels::WireSeg> &v) -> kernels::WireSeg * {
    if (v.empty()) return nullptr;
    const size_t bytes = v.size() * sizeof(kernels::WireSeg);
    void *pinned = ctx->staging().get(bytes);
    std::memcpy(pinned, v.data(), bytes);
    kernels::WireSeg *d = ctx->workspace().getArray<kernels::WireSeg>(v.size());
    HIP_CHECK(hipMemcpyAsync(d, pinned, bytes, hipMemcpyHostToDevice, xs));
    return d;
  };
  kernels::WireSeg *dS = upload(sc.send), *dR = upload(sc.recv), *dC = upload(sc.self);
  if (!codec.w) {
    // Raw words (the planner found the codec's extra pass dearer than the link
    // bytes it saves, HashJoin::planWireCodec): the filled runs are gathered
    // out of the claim slices and the all-to-allv lands them straight in the
    // window -- the receive displacements ARE window offsets, no unpack pass.
    kernels::segCopy(send, wsend, dS, (uint32_t)sc.send.size(), sG, xs, sc.sendMap);
    kernels::segCopy(send, dst, dC, (uint32_t)sc.self.size(), cG, xs, sc.sendMap);
    ctx->timeline().begin("MWINPUT", xs);
    ctx->comm()->allToAllV(wsend, sc.sendWords.data(), sc.sendDispls.data(), dst, sc.recvWords.data(),
                           sc.recvDispls.data(), Location::Device, xs);
    ctx->timeline().end("MWINPUT", xs);
    HIP_CHECK(hipEventRecord(done[chunk], xs));
    performance::Measurements::add("MWINPUTCNT", 1, "calls");
    if (segmented.size() < plan.chunks) segmented.resize(plan.chunks);
    segmented[chunk] = std::move(sc);
    exchanged[chunk] = true;
    return;
  }
  kernels::wirePack(send, wsend, dS, (uint32_t)sc.send.size(), sG, codec, xs, sc.sendMap);
  kernels::segCopy(send, dst, dC, (uint32_t)sc.self.size(), cG, xs, sc.sendMap);
  ctx->timeline().begin("MWINPUT", xs);
  ctx->comm()->allToAllV(wsend, sc.sendWords.data(), sc.sendDispls.data(), wrecv, sc.recvWords.data(),
                         sc.recvDispls.data(), Location::Device, xs);
  ctx->timeline().end("MWINPUT", xs);
  if (wired.size() < plan.chunks) {
    wired.resize(plan.chunks, nullptr);
    for (auto &e : wired)
      if (!e) e = ctx->acquireEvent();
  }
  HIP_CHECK(hipEventRecord(wired[chunk], xs));
  HIP_CHECK(hipStreamWaitEvent(ctx->decodeStream(), wired[chunk], 0));
  kernels::wireUnpack(wrecv, dst, dR, (uint32_t)sc.recv.size(), rG, codec, ctx->decodeStream());
  HIP_CHECK(hipEventRecord(done[chunk], ctx->decodeStream()));
  performance::Measurements::add("MWINPUTCNT", 1, "calls");
  if (segmented.size() < plan.chunks) segmented.resize(plan.chunks);
  segmented[chunk] = std::move(sc);
  exchanged[chunk] = true;
}

void Window::start() { open = true; }

void Window::enableOneSided() {
  const uint32_t N = plan.numberOfNodes, me = plan.nodeId, C = plan.chunks;
  JOIN_ASSERT(N > 1 && codec.w == 0, "Window", "one-sided windows: N > 1, raw tuples (no wire codec)");
  const bool shared = ctx->comm()->sharesAddressSpace();
  JOIN_ASSERT(shared || ctx->onDevice(), "Window", "one-sided host windows need in-process ranks");
  // Per rank: {pid, raw pointer, IPC handle (8 words), offset, workspace
  // generation, device, tag offset, tag nonce, recvDispls[C][N]}.
  const size_t H = 15, R = H + (size_t)C * N;
  std::vector<uint64_t> mine(R, 0), all(R * N);
  mine[0] = (uint64_t)getpid();
  mine[1] = (uint64_t)(uintptr_t)data;
  if (!shared) ctx->ipcExport(data, &mine[2], &mine[10], &mine[11], &mine[13], &mine[14]);
  mine[12] = ctx->onDevice() ? (uint64_t)ctx->device() : ~0ull;
  for (size_t i = 0; i < (size_t)C * N; ++i) mine[H + i] = plan.recvDispls[i];
  ctx->comm()->allGatherHost(mine.data(), all.data(), R);
  peerBase.assign(N, nullptr);
  peerOffset.assign((size_t)N * C, 0);
  for (uint32_t p = 0; p < N; ++p) {
    const uint64_t *r = &all[R * p];
    if (p == me) {
      peerBase[p] = static_cast<uint8_t *>(data);
    } else if (shared) {
      // In-process ranks pass raw pointers: the scatter kernel and the peer
      // copies dereference them from this rank's device, which needs peer
      // access when the ranks sit on different GPUs.
      if (ctx->onDevice() && r[12] != mine[12]) {
        int can = 0;
        HIP_CHECK(hipDeviceCanAccessPeer(&can, ctx->device(), (int)r[12]));
        JOIN_ASSERT(can, "Window", "one-sided window: device %d cannot access peer device %d", ctx->device(),
                    (int)r[12]);
        const hipError_t e = hipDeviceEnablePeerAccess((int)r[12], 0);
        if (e == hipErrorPeerAccessAlreadyEnabled)
          (void)hipGetLastError();
        else
          HIP_CHECK(e);
      }
      peerBase[p] = reinterpret_cast<uint8_t *>((uintptr_t)r[1]);
    } else {
      peerBase[p] = static_cast<uint8_t *>(ctx->ipcImport(p, &r[2], r[11], r[13], r[14])) + r[10];
    }
    for (uint32_t c = 0; c < C; ++c) peerOffset[(size_t)p * C + c] = r[H + (size_t)c * N + me];
  }
  // Every rank has opened its peers' handles before any rank goes on to
  // export, free or re-lay out memory (an exporter's later runtime calls must
  // not race a peer's open of the handle it just sent).
  if (!shared) ctx->comm()->barrier();
  oneSided = true;
  oneSidedComplete = false;
}

std::vector<uint64_t> Window::directDigitBase() const {
  JOIN_ASSERT(oneSided && assignment, "Window", "direct scatter needs a one-sided window with an assignment");
  const uint32_t N = plan.numberOfNodes, C = plan.chunks, F = plan.partitions;
  const uint64_t tb = tupleBytes();
  JOIN_ASSERT(plan.replicas.empty(), "Window", "replicated runs need a send buffer");
  std::vector<uint64_t> db((size_t)C * F, 0);
  for (uint32_t c = 0; c < C; ++c)
    for (uint32_t p = 0; p < F; ++p) {
      // The destination lays out source me's chunk-c runs exactly as my send
      // buffer does for it: same partitions, same order, same counts.
      const uint32_t d = plan.digitDest[(size_t)c * F + p];
      const uint64_t within = plan.digitBase[(size_t)c * F + p] - plan.sendDispls[(size_t)c * N + d];
      const uintptr_t addr = (uintptr_t)peerBase[d] + (peerOffset[(size_t)d * C + c] + within) * tb;
      JOIN_ASSERT(addr % tb == 0, "Window", "peer window misaligned for %lu-byte tuples", (unsigned long)tb);
      db[(size_t)c * F + p] = addr / tb;
    }
  return db;
}

// This rank's runs of chunk c, each copied into its owner's window at the
// owner's receive displacement for (c, this rank) -- MPI_Put at an exact,
// disjoint offset.  Device: peer copies on the exchange stream once the
// chunk's scatter is done.
void Window::putChunk(const void *send, uint32_t chunk) {
  const uint32_t N = plan.numberOfNodes, me = plan.nodeId, C = plan.chunks;
  const uint64_t tb = tupleBytes();
  if (directScatter()) {  // the scatter kernel already wrote the runs into the owners' windows
    for (uint32_t p = 0; p < N; ++p)
      if (p != me) wireSent += plan.sendCounts[(size_t)chunk * N + p] * tb / 8;
    HIP_CHECK(hipEventRecord(done[chunk], ctx->stream()));
    performance::Measurements::add("MWINPUTCNT", 1, "calls");
    return;
  }
  const uint8_t *src = static_cast<const uint8_t *>(send);
  const bool dev = ctx->onDevice();
  if (dev) {
    HIP_CHECK(hipEventRecord(ready[chunk], ctx->stream()));
    HIP_CHECK(hipStreamWaitEvent(ctx->commStream(), ready[chunk], 0));
  }
  ctx->timeline().begin("MWINPUT", dev ? ctx->commStream() : nullptr);
  for (uint32_t k = 0; k < N; ++k) {
    const uint32_t p = (me + k) % N;  // staggered: every link busy, none oversubscribed
    const uint64_t n = plan.sendCounts[(size_t)chunk * N + p];
    if (!n) continue;
    uint8_t *dst = peerBase[p] + peerOffset[(size_t)p * C + chunk] * tb;
    const uint8_t *from = src + plan.sendDispls[(size_t)chunk * N + p] * tb;
    if (dev)
      HIP_CHECK(hipMemcpyAsync(dst, from, n * tb, hipMemcpyDeviceToDevice, ctx->commStream()));
    else
      std::memcpy(dst, from, n * tb);
    if (p != me) wireSent += n * tb / 8;
    performance::Measurements::add("MWINPUTCNT", 1, "calls");
  }
  ctx->timeline().end("MWINPUT", dev ? ctx->commStream() : nullptr);
  if (dev) HIP_CHECK(hipEventRecord(done[chunk], ctx->commStream()));
}

void Window::exchange(const void *sendBuffer, uint32_t chunk) {
  JOIN_ASSERT(chunk < plan.chunks, "Window", "chunk %u out of range", chunk);
  if (oneSided) {
    putChunk(sendBuffer, chunk);
    exchanged[chunk] = true;
    return;
  }
  performance::Measurements::add("MWINPUTCNT", 1, "calls");  // one all-to-allv per chunk (the MPI_Put analog)
  if (codec.w && plan.numberOfNodes > 1) {
    exchangePacked(static_cast<const uint64_t *>(sendBuffer), chunk);
    exchanged[chunk] = true;
    return;
  }
  const uint32_t N = plan.numberOfNodes;
  const uint64_t w = tupleBytes() / 8;  // 8-byte words per tuple
  std::vector<uint64_t> sc(N), sd(N), rc(N), rd(N);
  for (uint32_t p = 0; p < N; ++p) {
    sc[p] = plan.sendCounts[(size_t)chunk * N + p] * w;
    sd[p] = plan.sendDispls[(size_t)chunk * N + p] * w;
    rc[p] = plan.recvCounts[(size_t)chunk * N + p] * w;
    rd[p] = plan.recvDispls[(size_t)chunk * N + p] * w;
  }
  for (uint32_t p = 0; p < N; ++p)
    if (p != plan.nodeId) wireSent += sc[p];
  const uint64_t *src = static_cast<const uint64_t *>(sendBuffer);
  uint64_t *dst = static_cast<uint64_t *>(data);
  if (ctx->onDevice() && N > 1) {
    HIP_CHECK(hipEventRecord(ready[chunk], ctx->stream()));
    HIP_CHECK(hipStreamWaitEvent(ctx->commStream(), ready[chunk], 0));
    ctx->timeline().begin("MWINPUT", ctx->commStream());
    ctx->comm()->allToAllV(src, sc.data(), sd.data(), dst, rc.data(), rd.data(), Location::Device,
                           ctx->commStream());
    ctx->timeline().end("MWINPUT", ctx->commStream());
    HIP_CHECK(hipEventRecord(done[chunk], ctx->commStream()));
  } else {
    ctx->timeline().begin("MWINPUT");
    ctx->comm()->allToAllV(src, sc.data(), sd.data(), dst, rc.data(), rd.data(), ctx->location(), ctx->stream());
    ctx->timeline().end("MWINPUT");
  }
  exchanged[chunk] = true;
}

void Window::stop() {
  if (ownedPlan) {  // chunk view
    if (viewArrived) HIP_CHECK(hipStreamWaitEvent(ctx->stream(), viewArrived, 0));
    open = false;
    return;
  }
  if (oneSided) {
    if (!oneSidedComplete) {
      // unlock_all + barrier: my puts have landed, then everyone's have.
      if (ctx->onDevice())
        utils::waitStream(directScatter() ? ctx->stream() : ctx->commStream(), ctx->comm(), "one-sided puts");
      ctx->comm()->barrier();
      oneSidedComplete = true;
      performance::Measurements::add("MWINWAITCNT", 1, "calls");
    }
    open = false;
    return;
  }
  if (ctx->onDevice() && plan.numberOfNodes > 1)
    for (uint32_t c = 0; c < plan.chunks; ++c)
      if (exchanged[c]) HIP_CHECK(hipStreamWaitEvent(ctx->stream(), done[c], 0));
  if (plan.numberOfNodes > 1 && open) performance::Measurements::add("MWINWAITCNT", 1, "calls");
  open = false;
}

void Window::flush() { stop(); }

void Window::setPartitioned(void *p, const uint64_t *pb, uint32_t bits, const uint64_t *pe, uint16_t *hi,
                            uint64_t capacity) {
  partitionedHi = hi;
  partitionedCapacity = capacity ? capacity : localWindowSize;
  partitioned = p;
  partBegin = pb;
  partEnd = pe;
  localBits = bits;
}

uint64_t Window::getPartitionSize(uint32_t partitionId) {
  JOIN_ASSERT(partitionId < plan.partitions, "Window", "partition %u out of range", partitionId);
  const int32_t lp = plan.localIndex[partitionId];
  return lp < 0 ? 0 : plan.partSize[lp];
}

CompressedTuple *Window::getPartition(uint32_t partitionId) {
  JOIN_ASSERT(!wide, "Window", "wide window: use getWidePartition");
  const int32_t lp = plan.localIndex.at(partitionId);
  JOIN_ASSERT(lp >= 0, "Window", "partition %u is not owned by node %u", partitionId, plan.nodeId);
  JOIN_ASSERT(!partEnd, "Window", "gapped local output: use getPartitionBegin/getPartitionEnd");
  JOIN_ASSERT(!partitionedHi, "Window", "split local output: use getPartitionedData / getPartitionedHi");
  void *base = partitioned ? partitioned : (plan.windowIsPartitionMajor() ? data : nullptr);
  JOIN_ASSERT(base, "Window", "partition-major view requires local partitioning first");
  return static_cast<CompressedTuple *>(base) + plan.lpBase[lp];
}

Tuple *Window::getWidePartition(uint32_t partitionId) {
  JOIN_ASSERT(wide, "Window", "compressed window: use getPartition");
  const int32_t lp = plan.localIndex.at(partitionId);
  JOIN_ASSERT(lp >= 0, "Window", "partition %u is not owned by node %u", partitionId, plan.nodeId);
  JOIN_ASSERT(!partEnd, "Window", "gapped local output: use getPartitionBegin/getPartitionEnd");
  void *base = partitioned ? partitioned : (plan.windowIsPartitionMajor() ? data : nullptr);
  JOIN_ASSERT(base, "Window", "partition-major view requires local partitioning first");
  return static_cast<Tuple *>(base) + plan.lpBase[lp];
}

uint64_t Window::computeLocalWindowSize() { return plan.recvTotal; }

uint64_t Window::computeWindowSize(uint32_t nodeId) {
  if (!globalHistogram) return nodeId == plan.nodeId ? plan.recvTotal : 0;
  const int side = assignment->sideOf(globalHistogram);
  const uint32_t C = globalHistogram->getChunkCount();
  uint64_t s = 0;
  for (uint32_t p = 0; p < plan.partitions; ++p) {
    if (!assignment->owns(p, nodeId)) continue;
    for (uint32_t r = 0; r < plan.numberOfNodes; ++r)
      for (uint32_t c = 0; c < C; ++c)
        if (assignment->receives(side, r, c, C, p, nodeId)) s += globalHistogram->rankCount(r, c, p);
  }
  return s;
}

void Window::assertAllTuplesWritten() {
  // Every source's chunk was exchanged and the plan's receive total equals the
  // global histogram mass of the partitions this node owns.
  for (uint32_t c = 0; c < plan.chunks; ++c)
    HJ_CHECK(exchanged[c] || plan.numberOfNodes == 1, "window chunk %u was never exchanged", c);
  HJ_CHECK(computeWindowSize(plan.nodeId) == plan.recvTotal, "window holds %lu tuples, owners expect %lu",
           (unsigned long)plan.recvTotal, (unsigned long)computeWindowSize(plan.nodeId));
}

}  // namespace data
}  // namespace hpcjoin
