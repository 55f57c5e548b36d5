#include "Window.h"

#include <algorithm>

#include "../comm/Communicator.h"
#include "../memory/Arena.h"
#include "../utils/Hip.h"

namespace hpcjoin {
namespace data {

Window::Window(const histograms::ExchangePlan &plan, histograms::GlobalHistogram *globalHistogram,
               histograms::AssignmentMap *assignment, core::ExecContext *ctx, bool wide)
    : plan(plan), globalHistogram(globalHistogram), assignment(assignment), ctx(ctx), wide(wide) {
  localWindowSize = plan.recvTotal;
  data = ctx->workspace().get(localWindowSize * tupleBytes());
  exchanged.assign(plan.chunks, false);
  if (ctx->onDevice() && plan.numberOfNodes > 1) {
    ready.resize(plan.chunks);
    done.resize(plan.chunks);
    for (uint32_t c = 0; c < plan.chunks; ++c) {
      HIP_CHECK(hipEventCreateWithFlags(&ready[c], hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&done[c], hipEventDisableTiming));
    }
  }
}

Window::Window(const histograms::ExchangePlan &plan, uint64_t capacityTuples, core::ExecContext *ctx, bool wide)
    : plan(plan), globalHistogram(nullptr), assignment(nullptr), ctx(ctx), wide(wide) {
  localWindowSize = capacityTuples;
  data = ctx->workspace().get(std::max<uint64_t>(capacityTuples, 1) * tupleBytes());
  exchanged.assign(std::max<uint32_t>(plan.chunks, 1), false);
}

Window::~Window() {
  for (auto e : ready) (void)hipEventDestroy(e);
  for (auto e : done) (void)hipEventDestroy(e);
}

void Window::start() { open = true; }

void Window::exchange(const void *sendBuffer, uint32_t chunk) {
  JOIN_ASSERT(chunk < plan.chunks, "Window", "chunk %u out of range", chunk);
  const uint32_t N = plan.numberOfNodes;
  const uint64_t w = tupleBytes() / 8;  // 8-byte words per tuple
  std::vector<uint64_t> sc(N), sd(N), rc(N), rd(N);
  for (uint32_t p = 0; p < N; ++p) {
    sc[p] = plan.sendCounts[(size_t)chunk * N + p] * w;
    sd[p] = plan.sendDispls[(size_t)chunk * N + p] * w;
    rc[p] = plan.recvCounts[(size_t)chunk * N + p] * w;
    rd[p] = plan.recvDispls[(size_t)chunk * N + p] * w;
  }
  const uint64_t *src = static_cast<const uint64_t *>(sendBuffer);
  uint64_t *dst = static_cast<uint64_t *>(data);
  if (ctx->onDevice() && N > 1) {
    HIP_CHECK(hipEventRecord(ready[chunk], ctx->stream()));
    HIP_CHECK(hipStreamWaitEvent(ctx->commStream(), ready[chunk], 0));
    ctx->comm()->allToAllV(src, sc.data(), sd.data(), dst, rc.data(), rd.data(), Location::Device,
                           ctx->commStream());
    HIP_CHECK(hipEventRecord(done[chunk], ctx->commStream()));
  } else {
    ctx->comm()->allToAllV(src, sc.data(), sd.data(), dst, rc.data(), rd.data(), ctx->location(), ctx->stream());
  }
  exchanged[chunk] = true;
}

void Window::stop() {
  if (ctx->onDevice() && plan.numberOfNodes > 1)
    for (uint32_t c = 0; c < plan.chunks; ++c)
      if (exchanged[c]) HIP_CHECK(hipStreamWaitEvent(ctx->stream(), done[c], 0));
  open = false;
}

void Window::flush() { stop(); }

void Window::setPartitioned(void *p, const uint64_t *pb, uint32_t bits, const uint64_t *pe) {
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
  const uint32_t *owner = assignment->getPartitionAssignment();
  const uint64_t *g = globalHistogram->getGlobalHistogram();
  uint64_t s = 0;
  for (uint32_t p = 0; p < plan.partitions; ++p)
    if (owner[p] == nodeId) s += g[p];
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
