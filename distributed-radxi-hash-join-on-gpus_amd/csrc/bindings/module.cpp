// pybind11 bindings of the native engine (built in-tree as hpcjoin/_C*.so).
// The C++ core is the source of truth; Python adds launch/bootstrap glue,
// the oracle and the benchmark harness.
#include <torch/extension.h>

#include <hip/hip_runtime.h>

#include <memory>
#include <tuple>
#include <vector>

#include "../comm/InProcessCommunicator.h"
#include "../comm/RcclCommunicator.h"
#include "../comm/World.h"
#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../host/HostOps.h"
#include "../kernels/kernels.h"
#include "../memory/Arena.h"
#include "../memory/Pool.h"
#include "../operators/HashJoin.h"
#include "../operators/LateMaterialization.h"
#include "../performance/Measurements.h"
#include "../utils/Fault.h"
#include "../utils/Hip.h"
#include "ProcessGroupCommunicator.h"

namespace py = pybind11;
using namespace hpcjoin;

namespace {

Location locOf(const at::Tensor &t) { return t.is_cuda() ? Location::Device : Location::Host; }

void syncIfDevice(Location l) {
  if (l == Location::Device) HIP_CHECK(hipDeviceSynchronize());
}

void checkTuples(const at::Tensor &t, const char *name) {
  TORCH_CHECK(t.dim() == 2 && t.size(1) == 2 && t.scalar_type() == at::kLong && t.is_contiguous(), name,
              " must be a contiguous int64 tensor of shape [n, 2] (key, rid)");
}

void checkWords(const at::Tensor &t, const char *name) {
  TORCH_CHECK(t.dim() == 1 && t.scalar_type() == at::kLong && t.is_contiguous(), name,
              " must be a contiguous 1-D int64 tensor");
}

template <typename T>
T *ptr(const at::Tensor &t) {
  return reinterpret_cast<T *>(t.data_ptr());
}

at::TensorOptions like(const at::Tensor &t, at::ScalarType st = at::kLong) {
  return at::TensorOptions().dtype(st).device(t.device());
}

void setDevice(const at::Tensor &t) {
  if (t.is_cuda()) HIP_CHECK(hipSetDevice(t.get_device()));
}

// ---- single-relation network pass (one "rank", all partitions local) ------
std::tuple<at::Tensor, at::Tensor> opNetPartition(const at::Tensor &tuples, int64_t bits, int64_t keyShift,
                                                  bool wide, int64_t maxBlocks, int64_t keyBits) {
  checkTuples(tuples, "tuples");
  setDevice(tuples);
  const uint64_t n = tuples.size(0);
  const uint32_t F = 1u << bits;
  const Location l = locOf(tuples);
  const auto g = kernels::partitionGeometry(n, (uint32_t)maxBlocks);
  at::Tensor blockHist = at::empty({(int64_t)F * g.blocks}, like(tuples, at::kInt));
  at::Tensor totals = at::empty({(int64_t)F}, like(tuples));
  at::Tensor cursors = at::empty({(int64_t)F * g.blocks}, like(tuples));
  at::Tensor out = wide ? at::empty({(int64_t)n, 2}, like(tuples)) : at::empty({(int64_t)n}, like(tuples));
  const data::Tuple *in = ptr<const data::Tuple>(tuples);
  if (l == Location::Device) {
    kernels::netHistogram(in, n, bits, g, ptr<uint32_t>(blockHist), nullptr);
    kernels::digitTotals(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, 1, ptr<uint64_t>(totals), nullptr);
  } else {
    host::netHistogram(in, n, bits, g, ptr<uint32_t>(blockHist));
    host::digitTotals(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, 1, ptr<uint64_t>(totals));
  }
  at::Tensor begin = at::zeros({(int64_t)F + 1}, at::kLong);
  begin.slice(0, 1).copy_(at::cumsum(totals.cpu(), 0));
  at::Tensor base = begin.slice(0, 0, F).to(tuples.device()).contiguous();
  if (l == Location::Device) {
    const bool narrow = kernels::cursorsNarrow(n);
    at::Tensor gcur = at::empty({(int64_t)kernels::CLAIM_GROUPS * F}, like(tuples));
    kernels::netGroupCursors(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, ptr<uint64_t>(base), gcur.data_ptr(),
                             narrow, nullptr);
    if (wide)
      kernels::netScatterWide(in, n, bits, g, 0, g.blocks, gcur.data_ptr(), ptr<data::Tuple>(out), nullptr);
    else
      kernels::netScatter(in, n, bits, (uint32_t)keyShift, g, 0, g.blocks, gcur.data_ptr(), ptr<uint64_t>(out),
                          nullptr, (uint32_t)keyBits);
  } else {
    host::netCursors(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, ptr<uint64_t>(base), ptr<uint64_t>(cursors));
    host::netScatter(in, n, bits, (uint32_t)keyShift, g, 0, g.blocks, ptr<uint64_t>(cursors), out.data_ptr(), wide);
  }
  syncIfDevice(l);
  return {out, begin};
}

at::Tensor opNetHistogram(const at::Tensor &tuples, int64_t bits, int64_t maxBlocks) {
  checkTuples(tuples, "tuples");
  setDevice(tuples);
  const uint64_t n = tuples.size(0);
  const uint32_t F = 1u << bits;
  const auto g = kernels::partitionGeometry(n, (uint32_t)maxBlocks);
  at::Tensor blockHist = at::empty({(int64_t)F * g.blocks}, like(tuples, at::kInt));
  at::Tensor totals = at::empty({(int64_t)F}, like(tuples));
  if (tuples.is_cuda()) {
    kernels::netHistogram(ptr<data::Tuple>(tuples), n, bits, g, ptr<uint32_t>(blockHist), nullptr);
    kernels::digitTotals(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, 1, ptr<uint64_t>(totals), nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::netHistogram(ptr<data::Tuple>(tuples), n, bits, g, ptr<uint32_t>(blockHist));
    host::digitTotals(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, 1, ptr<uint64_t>(totals));
  }
  return totals;
}

// ---- local pass over a partition-major buffer (each input partition = one lp)
std::tuple<at::Tensor, at::Tensor> opLocalPartition(const at::Tensor &values, const at::Tensor &partBeginIn,
                                                    int64_t shift, int64_t bits, bool wide) {
  if (wide)
    checkTuples(values, "values");
  else
    checkWords(values, "values");
  setDevice(values);
  at::Tensor pbIn = partBeginIn.cpu().contiguous();
  const uint32_t owned = (uint32_t)pbIn.size(0) - 1;
  const uint32_t F = 1u << bits;
  std::vector<kernels::LocalItem> items;
  std::vector<uint32_t> lb(owned + 1);
  std::vector<uint64_t> base(owned + 1);
  for (uint32_t lp = 0; lp < owned; ++lp) {
    lb[lp] = (uint32_t)items.size();
    const uint64_t b = pbIn[lp].item<int64_t>(), e = pbIn[lp + 1].item<int64_t>();
    base[lp] = b;
    for (uint64_t o = b; o < e; o += kernels::LOCAL_ITEM_MAX)
      items.push_back({o, (uint32_t)std::min<uint64_t>(kernels::LOCAL_ITEM_MAX, e - o), lp, 0, 0});
  }
  lb[owned] = (uint32_t)items.size();
  base[owned] = owned ? (uint64_t)pbIn[owned].item<int64_t>() : 0;
  const uint32_t nItems = (uint32_t)items.size();
  at::Tensor out = at::empty_like(values);
  at::Tensor partBegin = at::empty({(int64_t)owned * F + 1}, like(values));
  at::Tensor itemHist = at::empty({std::max<int64_t>(1, (int64_t)nItems * F)}, like(values, at::kInt));
  at::Tensor itemCursors = at::empty({std::max<int64_t>(1, (int64_t)nItems * F)}, like(values));
  if (values.is_cuda()) {
    const uint32_t streams = kernels::assignLocalStreams(items.data(), nItems);
    const bool narrow = kernels::cursorsNarrow(values.size(0));
    at::Tensor gcur = at::empty({std::max<int64_t>(1, (int64_t)streams * F)}, like(values));
    at::Tensor dItems = at::empty({std::max<int64_t>(1, (int64_t)nItems * 3)}, like(values));
    at::Tensor dLb = at::empty({(int64_t)owned + 1}, like(values, at::kInt));
    at::Tensor dBase = at::empty({(int64_t)owned + 1}, like(values));
    HIP_CHECK(hipMemcpy(dItems.data_ptr(), items.data(), nItems * sizeof(kernels::LocalItem), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dLb.data_ptr(), lb.data(), (owned + 1) * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dBase.data_ptr(), base.data(), (owned + 1) * 8, hipMemcpyHostToDevice));
    const auto *di = ptr<const kernels::LocalItem>(dItems);
    kernels::localHistogram(values.data_ptr(), wide, di, nItems, (uint32_t)shift, (uint32_t)bits, ptr<uint32_t>(itemHist),
                            nullptr);
    kernels::localCursors(ptr<uint32_t>(itemHist), ptr<uint32_t>(dLb), owned, (uint32_t)bits, ptr<uint64_t>(dBase), di,
                          gcur.data_ptr(), narrow, ptr<uint64_t>(partBegin), nullptr);
    kernels::localScatter(values.data_ptr(), wide, di, nItems, (uint32_t)shift, (uint32_t)bits, gcur.data_ptr(), narrow,
                          out.data_ptr(), nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::localHistogram(values.data_ptr(), wide, items.data(), nItems, (uint32_t)shift, (uint32_t)bits,
                         ptr<uint32_t>(itemHist));
    host::localCursors(ptr<uint32_t>(itemHist), lb.data(), owned, (uint32_t)bits, base.data(),
                       ptr<uint64_t>(itemCursors), ptr<uint64_t>(partBegin));
    host::localScatter(values.data_ptr(), wide, items.data(), nItems, (uint32_t)shift, (uint32_t)bits,
                       ptr<uint64_t>(itemCursors), out.data_ptr());
  }
  return {out, partBegin};
}

// ---- build/probe over partition-major inputs -----------------------------
py::dict opBuildProbe(const at::Tensor &R, const at::Tensor &S, const at::Tensor &partR, const at::Tensor &partS,
                      int64_t fragShift, int64_t keyShift, bool wide, bool materialize, int64_t rChunk,
                      int64_t sChunk, int64_t outCapacity) {
  setDevice(R);
  kernels::BPArgs a;
  a.R = R.data_ptr();
  a.S = S.data_ptr();
  at::Tensor pr = partR.to(R.device()).contiguous(), ps = partS.to(R.device()).contiguous();
  a.partR = ptr<uint64_t>(pr);
  a.partS = ptr<uint64_t>(ps);
  a.P = (uint32_t)pr.size(0) - 1;
  a.rChunk = (uint32_t)rChunk;
  a.sChunk = (uint32_t)sChunk;
  a.fragShift = (uint32_t)fragShift;
  a.keyShift = (uint32_t)keyShift;
  a.wide = wide;
  a.materialize = materialize;
  at::Tensor pairs = at::empty({std::max<int64_t>(outCapacity, 1), 2}, like(R));
  a.outPairs = reinterpret_cast<ulonglong2 *>(pairs.data_ptr());
  a.outCapacity = materialize ? (uint64_t)outCapacity : 0;
  py::dict d;
  if (R.is_cuda()) {
    at::Tensor ctr = at::zeros({4}, like(R));
    a.result = reinterpret_cast<unsigned long long *>(ctr.data_ptr());
    a.outCursor = a.result + 1;
    uint32_t *nItems = reinterpret_cast<uint32_t *>(a.result + 2);
    at::Tensor counts = at::empty({std::max<int64_t>(a.P, 1)}, like(R, at::kInt));
    at::Tensor offsets = at::empty({std::max<int64_t>(a.P, 1)}, like(R, at::kInt));
    at::Tensor scanWs = at::empty({(int64_t)kernels::scanWorkspaceBytes(a.P) / 4 + 1}, like(R, at::kInt));
    uint32_t capacity = 2 * a.P + (uint32_t)(S.size(0) / a.sChunk + R.size(0) / a.rChunk) + 1024;
    for (int attempt = 0; attempt < 2; ++attempt) {
      at::Tensor items = at::empty({(int64_t)capacity * 2}, like(R));
      ctr.zero_();
      kernels::bpPlanCounts(a, ptr<uint32_t>(counts), nullptr);
      kernels::scanExclusiveU32(ptr<uint32_t>(counts), ptr<uint32_t>(offsets), a.P, nItems, scanWs.data_ptr(), nullptr);
      kernels::bpEmit(a, ptr<uint32_t>(counts), ptr<uint32_t>(offsets), ptr<kernels::BPItem>(items), capacity, nullptr);
      kernels::buildProbe(a, ptr<kernels::BPItem>(items), nItems, capacity, nullptr);
      HIP_CHECK(hipDeviceSynchronize());
      at::Tensor h = ctr.cpu();
      const uint32_t need = (uint32_t)(h[2].item<int64_t>() & 0xFFFFFFFF);
      d["matches"] = (uint64_t)h[0].item<int64_t>();
      d["output_count"] = (uint64_t)h[1].item<int64_t>();
      d["work_items"] = need;
      if (need <= capacity) break;
      capacity = need;
    }
  } else {
    uint64_t cursor = 0;
    a.outCursor = reinterpret_cast<unsigned long long *>(&cursor);
    d["matches"] = host::buildProbe(a);
    d["output_count"] = cursor;
    d["work_items"] = a.P;
  }
  d["pairs"] = pairs;
  return d;
}

at::Tensor opGenerate(int64_t n, int64_t globalOffset, int64_t globalSize, const data::GenSpec &spec,
                      const std::string &device) {
  at::Tensor out = at::empty({n, 2}, at::TensorOptions().dtype(at::kLong).device(device));
  setDevice(out);
  const uint64_t domain = spec.domain ? spec.domain : (uint64_t)globalSize;
  kernels::GenParams p;
  p.dist = spec.distribution;
  p.globalOffset = globalOffset;
  p.ridOffset = globalOffset;
  p.keyOffset = spec.keyOffset;
  p.domain = domain;
  p.modulo = domain;
  p.seed = spec.seed;
  p.perm = kernels::FeistelPermutation::make(domain, spec.seed);
  if (spec.distribution == kernels::KeyDistribution::Zipf) p.zipf = host::makeZipf(domain, spec.zipfTheta);
  p.tpchSparse = spec.tpchSparse;
  p.sparse64 = spec.sparse64;
  if (out.is_cuda()) {
    kernels::generate(ptr<data::Tuple>(out), n, p, nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::generate(ptr<data::Tuple>(out), n, p);
  }
  return out;
}

at::Tensor opScan(const at::Tensor &in) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kInt && in.dim() == 1, "scan expects a 1-D int32 HIP tensor");
  setDevice(in);
  const uint64_t n = in.size(0);
  at::Tensor out = at::empty({(int64_t)n + 1}, like(in, at::kInt));
  at::Tensor ws = at::empty({(int64_t)kernels::scanWorkspaceBytes(n) / 4 + 1}, like(in, at::kInt));
  kernels::scanExclusiveU32(ptr<uint32_t>(in), ptr<uint32_t>(out), n, ptr<uint32_t>(out) + n, ws.data_ptr(), nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  return out;
}

uint64_t opNpjCount(const at::Tensor &R, const at::Tensor &S) {
  checkTuples(R, "R");
  checkTuples(S, "S");
  setDevice(R);
  if (!R.is_cuda()) return host::npjJoin(ptr<data::Tuple>(R), R.size(0), ptr<data::Tuple>(S), S.size(0));
  const uint64_t slots = kernels::npjTableSlots(R.size(0));
  at::Tensor table = at::empty({(int64_t)slots}, like(R));
  at::Tensor res = at::zeros({1}, like(R));
  kernels::npjBuild(ptr<data::Tuple>(R), R.size(0), ptr<unsigned long long>(table), slots, nullptr);
  kernels::npjProbe(ptr<data::Tuple>(S), S.size(0), ptr<unsigned long long>(table), slots, ptr<unsigned long long>(res),
                    nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  return (uint64_t)res.cpu()[0].item<int64_t>();
}

// (inner rid, outer rid) pairs of the no-partitioning join, [matches, 2] int64
// on the inputs' device: count pass, exact allocation, materializing pass.
at::Tensor opNpjJoin(const at::Tensor &R, const at::Tensor &S) {
  checkTuples(R, "R");
  checkTuples(S, "S");
  setDevice(R);
  if (!R.is_cuda()) {
    const auto v = host::npjPairs(ptr<data::Tuple>(R), R.size(0), ptr<data::Tuple>(S), S.size(0));
    at::Tensor out = at::empty({(int64_t)v.size(), 2}, like(R));
    int64_t *o = out.data_ptr<int64_t>();
    for (size_t i = 0; i < v.size(); ++i) {
      o[2 * i] = (int64_t)v[i].first;
      o[2 * i + 1] = (int64_t)v[i].second;
    }
    return out;
  }
  const uint64_t slots = kernels::npjTableSlots(R.size(0));
  at::Tensor table = at::empty({(int64_t)slots}, like(R));
  at::Tensor rids = at::empty({(int64_t)slots}, like(R));
  at::Tensor res = at::zeros({2}, like(R));
  kernels::npjBuildRids(ptr<data::Tuple>(R), R.size(0), ptr<unsigned long long>(table), ptr<unsigned long long>(rids),
                        slots, nullptr);
  kernels::npjProbe(ptr<data::Tuple>(S), S.size(0), ptr<unsigned long long>(table), slots,
                    ptr<unsigned long long>(res), nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  const int64_t m = res.cpu()[0].item<int64_t>();
  at::Tensor out = at::empty({m, 2}, like(R));
  kernels::npjProbePairs(ptr<data::Tuple>(S), S.size(0), ptr<unsigned long long>(table),
                         ptr<unsigned long long>(rids), slots, reinterpret_cast<ulonglong2 *>(out.data_ptr()),
                         (uint64_t)m, ptr<unsigned long long>(res) + 1, nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  TORCH_CHECK(res.cpu()[1].item<int64_t>() == m, "npj_join: the materializing pass found another match count");
  return out;
}

at::Tensor opNetScatterGlobalAtomic(const at::Tensor &tuples, int64_t bits, int64_t keyShift,
                                    const at::Tensor &partBegin) {
  checkTuples(tuples, "tuples");
  TORCH_CHECK(tuples.is_cuda(), "global-atomic scatter is a device ablation");
  setDevice(tuples);
  at::Tensor cur = partBegin.slice(0, 0, partBegin.size(0) - 1).to(tuples.device()).contiguous().clone();
  at::Tensor out = at::empty({tuples.size(0)}, like(tuples));
  kernels::netScatterGlobalAtomic(ptr<data::Tuple>(tuples), tuples.size(0), bits, keyShift, ptr<uint64_t>(cur),
                                  ptr<uint64_t>(out), nullptr);
  HIP_CHECK(hipDeviceSynchronize());
  return out;
}

// Timed device micro-benchmarks: returns milliseconds per call (median of iters).
double timeDevice(const std::function<void(hipStream_t)> &fn, int iters) {
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  std::vector<float> ms;
  fn(nullptr);  // warm
  for (int i = 0; i < iters; ++i) {
    HIP_CHECK(hipEventRecord(a, nullptr));
    fn(nullptr);
    HIP_CHECK(hipEventRecord(b, nullptr));
    HIP_CHECK(hipEventSynchronize(b));
    float m;
    HIP_CHECK(hipEventElapsedTime(&m, a, b));
    ms.push_back(m);
  }
  HIP_CHECK(hipEventDestroy(a));
  HIP_CHECK(hipEventDestroy(b));
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

// Times the network scatter kernel alone (cursors precomputed) in one of the
// ablation modes; returns ms per call.
double benchScatter(const at::Tensor &tuples, int64_t bits, int64_t mode, int iters, int64_t maxBlocks,
                    int64_t geometry, int64_t roundLp) {
  checkTuples(tuples, "tuples");
  setDevice(tuples);
  const uint64_t n = tuples.size(0);
  const uint32_t F = 1u << bits;
  const auto g = kernels::partitionGeometry(n, (uint32_t)maxBlocks);
  at::Tensor blockHist = at::empty({(int64_t)F * g.blocks}, like(tuples, at::kInt));
  at::Tensor totals = at::empty({(int64_t)F}, like(tuples));
  at::Tensor cursors = at::empty({(int64_t)F * g.blocks}, like(tuples));
  // mode 3 (round-interleaved slices): slice i = g * F + d starts at logical
  // i << lv; the write-out sends logical [i | j | o] to physical [j | i | o].
  uint32_t rs[3] = {(uint32_t)roundLp, 0, 0};
  while ((1u << rs[2]) < 8 * F) ++rs[2];
  while ((double)(1ull << rs[1]) < 1.05 * (double)n / (8.0 * F) + 64) ++rs[1];
  JOIN_ASSERT(mode != 3 || rs[1] + rs[2] <= 32, "benchScatter", "mode 3 logical space past 32 bits");
  at::Tensor out = at::empty({mode == 3 ? (int64_t)1 << (rs[1] + rs[2]) : (int64_t)n}, like(tuples));
  kernels::netHistogram(ptr<data::Tuple>(tuples), n, bits, g, ptr<uint32_t>(blockHist), nullptr);
  kernels::digitTotals(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, 1, ptr<uint64_t>(totals), nullptr);
  at::Tensor base = (at::cumsum(totals, 0) - totals).contiguous();
  kernels::netCursors(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, ptr<uint64_t>(base), ptr<uint64_t>(cursors),
                      nullptr);
  at::Tensor gcur32 = at::empty({8 * (int64_t)F}, like(tuples, at::kInt));
  kernels::netGroupCursors(ptr<uint32_t>(blockHist), F, g.blocks, g.blocks, ptr<uint64_t>(base), gcur32.data_ptr(),
                           true, nullptr);
  if (mode == 3)
    gcur32 = (at::arange(8 * (int64_t)F, like(tuples, at::kLong)) * ((int64_t)1 << rs[1])).to(at::kInt).contiguous();
  at::Tensor work = gcur32.clone();
  at::Tensor meta = at::tensor({(int32_t)rs[0], (int32_t)rs[1], (int32_t)rs[2], 0}, like(tuples, at::kInt));
  HIP_CHECK(hipDeviceSynchronize());
  return timeDevice(
      [&](hipStream_t s) {
        HIP_CHECK(hipMemcpyAsync(work.data_ptr(), gcur32.data_ptr(), 8 * F * 4, hipMemcpyDeviceToDevice, s));
        kernels::scatterAblation(ptr<data::Tuple>(tuples), n, bits, 32, g, ptr<uint64_t>(cursors), ptr<uint64_t>(out),
                                 (int)mode, (int)geometry, s, work.data_ptr(),
                                 mode == 3 ? static_cast<const uint32_t *>(meta.data_ptr()) : nullptr);
      },
      iters);
}

double benchHistogram(const at::Tensor &tuples, int64_t bits, int iters) {
  setDevice(tuples);
  const uint64_t n = tuples.size(0);
  const auto g = kernels::partitionGeometry(n, 2048);
  at::Tensor blockHist = at::empty({(int64_t)(1u << bits) * g.blocks}, like(tuples, at::kInt));
  return timeDevice(
      [&](hipStream_t s) { kernels::netHistogram(ptr<data::Tuple>(tuples), n, bits, g, ptr<uint32_t>(blockHist), s); },
      iters);
}

// Wire codec on explicit segments [(raw offset, n, rid base)] (tests and the
// wire micro-benchmark).  Segments are packed back to back.
std::vector<kernels::WireSeg> wireSegs(const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> &segs,
                                       const kernels::WireCodec &c, uint64_t *words, uint64_t *groups) {
  std::vector<kernels::WireSeg> out;
  uint64_t off = 0, g = 0;
  for (const auto &t : segs) {
    const uint64_t n = std::get<1>(t);
    if (n) out.push_back({std::get<0>(t), off, n, std::get<2>(t), g});
    off += c.words(n);
    g += ceilDiv(n, 64);
  }
  *words = off;
  *groups = g;
  return out;
}

kernels::WireCodec makeCodec(uint32_t w, uint32_t ridBits, uint32_t keyShift) {
  TORCH_CHECK(w >= 1 && w <= 64 && ridBits <= w && keyShift >= ridBits && keyShift < 64, "bad wire codec");
  kernels::WireCodec c;
  c.w = w;
  c.ridBits = ridBits;
  c.keyShift = keyShift;
  return c;
}

at::Tensor opWirePack(const at::Tensor &raw, uint32_t w, uint32_t ridBits, uint32_t keyShift,
                      const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> &segs) {
  checkWords(raw, "raw");
  setDevice(raw);
  const kernels::WireCodec c = makeCodec(w, ridBits, keyShift);
  uint64_t words, groups;
  std::vector<kernels::WireSeg> sg = wireSegs(segs, c, &words, &groups);
  for (const auto &x : sg) TORCH_CHECK(x.raw + x.n <= (uint64_t)raw.numel(), "segment out of range");
  at::Tensor wire = at::zeros({(int64_t)std::max<uint64_t>(words, 1)}, like(raw));
  if (raw.is_cuda()) {
    at::Tensor d = at::empty({(int64_t)(std::max<size_t>(sg.size(), 1) * sizeof(kernels::WireSeg))},
                             like(raw, at::kByte));
    HIP_CHECK(hipMemcpy(d.data_ptr(), sg.data(), sg.size() * sizeof(kernels::WireSeg), hipMemcpyHostToDevice));
    kernels::wirePack(ptr<uint64_t>(raw), ptr<uint64_t>(wire), ptr<kernels::WireSeg>(d), (uint32_t)sg.size(), groups,
                      c, nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::wirePack(ptr<uint64_t>(raw), ptr<uint64_t>(wire), sg.data(), (uint32_t)sg.size(), c);
  }
  return wire;
}

void opWireUnpack(const at::Tensor &wire, const at::Tensor &raw, uint32_t w, uint32_t ridBits, uint32_t keyShift,
                  const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> &segs) {
  checkWords(wire, "wire");
  checkWords(raw, "raw");
  setDevice(raw);
  const kernels::WireCodec c = makeCodec(w, ridBits, keyShift);
  uint64_t words, groups;
  std::vector<kernels::WireSeg> sg = wireSegs(segs, c, &words, &groups);
  TORCH_CHECK(words <= (uint64_t)wire.numel(), "wire buffer too small");
  for (const auto &x : sg) TORCH_CHECK(x.raw + x.n <= (uint64_t)raw.numel(), "segment out of range");
  if (raw.is_cuda()) {
    at::Tensor d = at::empty({(int64_t)(std::max<size_t>(sg.size(), 1) * sizeof(kernels::WireSeg))},
                             like(raw, at::kByte));
    HIP_CHECK(hipMemcpy(d.data_ptr(), sg.data(), sg.size() * sizeof(kernels::WireSeg), hipMemcpyHostToDevice));
    kernels::wireUnpack(ptr<uint64_t>(wire), ptr<uint64_t>(raw), ptr<kernels::WireSeg>(d), (uint32_t)sg.size(),
                        groups, c, nullptr);
    HIP_CHECK(hipDeviceSynchronize());
  } else {
    host::wireUnpack(ptr<uint64_t>(wire), ptr<uint64_t>(raw), sg.data(), (uint32_t)sg.size(), c);
  }
}

// Pack + unpack of one n-tuple segment, device ms each (median).
py::dict benchWire(const at::Tensor &raw, uint32_t w, uint32_t ridBits, uint32_t keyShift, int iters) {
  checkWords(raw, "raw");
  TORCH_CHECK(raw.is_cuda(), "bench_wire needs a HIP tensor");
  setDevice(raw);
  const kernels::WireCodec c = makeCodec(w, ridBits, keyShift);
  uint64_t words, groups;
  std::vector<kernels::WireSeg> sg = wireSegs({{0, (uint64_t)raw.numel(), 0}}, c, &words, &groups);
  at::Tensor wire = at::empty({(int64_t)words}, like(raw));
  at::Tensor back = at::empty_like(raw);
  at::Tensor d = at::empty({(int64_t)sizeof(kernels::WireSeg)}, like(raw, at::kByte));
  HIP_CHECK(hipMemcpy(d.data_ptr(), sg.data(), sizeof(kernels::WireSeg), hipMemcpyHostToDevice));
  const auto *ds = ptr<kernels::WireSeg>(d);
  py::dict out;
  out["pack_ms"] = timeDevice(
      [&](hipStream_t s) { kernels::wirePack(ptr<uint64_t>(raw), ptr<uint64_t>(wire), ds, 1, groups, c, s); }, iters);
  out["unpack_ms"] = timeDevice(
      [&](hipStream_t s) { kernels::wireUnpack(ptr<uint64_t>(wire), ptr<uint64_t>(back), ds, 1, groups, c, s); },
      iters);
  out["wire_bytes"] = words * 8;
  return out;
}

double benchCopy(const at::Tensor &src, const at::Tensor &dst, int iters) {
  setDevice(src);
  const uint64_t n16 = src.numel() * src.element_size() / 16;
  return timeDevice(
      [&](hipStream_t s) {
        kernels::copyKernel(ptr<const ulonglong2>(src), ptr<ulonglong2>(dst), n16, s);
      },
      iters);
}

double benchRead(const at::Tensor &src, int iters) {
  setDevice(src);
  const uint64_t n16 = src.numel() * src.element_size() / 16;
  at::Tensor sink = at::zeros({1}, like(src));
  return timeDevice(
      [&](hipStream_t s) { kernels::readKernel(ptr<const ulonglong2>(src), n16, ptr<unsigned long long>(sink), s); },
      iters);
}

// Host-link ceilings (the reference's dormant UVA_benchmark,
// operators/gpu/small_data_optimized.cu): DMA copies both ways between pinned
// host memory and HBM, and kernels reading pinned memory in place (the path
// the engine uses for relations kept in pinned host memory).
py::dict benchHostLink(uint64_t bytes, int device, int iters) {
  HIP_CHECK(hipSetDevice(device));
  bytes = std::max<uint64_t>(16, bytes / 16 * 16);
  void *h = memory::Arena::rawAlloc(Location::Pinned, bytes, device);
  void *d = memory::Arena::rawAlloc(Location::Device, bytes, device);
  unsigned long long *sink = static_cast<unsigned long long *>(memory::Arena::rawAlloc(Location::Device, 8, device));
  std::memset(h, 1, bytes);
  py::dict out;
  try {
    const double h2d = timeDevice([&](hipStream_t s) { HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s)); }, iters);
    const double d2h = timeDevice([&](hipStream_t s) { HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s)); }, iters);
    const double zc = timeDevice(
        [&](hipStream_t s) { kernels::readKernel(static_cast<const ulonglong2 *>(h), bytes / 16, sink, s); }, iters);
    out["bytes"] = bytes;
    out["h2d_GBps"] = bytes / h2d / 1e6;
    out["d2h_GBps"] = bytes / d2h / 1e6;
    out["zero_copy_read_GBps"] = bytes / zc / 1e6;
  } catch (...) {
    memory::Arena::rawFree(Location::Pinned, h);
    memory::Arena::rawFree(Location::Device, d);
    memory::Arena::rawFree(Location::Device, sink);
    throw;
  }
  memory::Arena::rawFree(Location::Pinned, h);
  memory::Arena::rawFree(Location::Device, d);
  memory::Arena::rawFree(Location::Device, sink);
  return out;
}

py::dict resultToDict(const operators::JoinResult &r) {
  py::dict d;
  d["local_matches"] = r.localMatches;
  d["global_matches"] = r.globalMatches;
  d["output_pairs"] = r.outputPairs;
  d["output_overflow"] = r.outputOverflow;
  d["rows_fused"] = r.rowsFused;
  d["split_partitions"] = r.splitPartitions;
  d["direct_scatter"] = r.directScatter;
  d["reruns"] = r.reruns;
  d["sampled_network"] = r.sampledNetwork;
  d["network_fallbacks"] = r.networkFallbacks;
  d["round_windows"] = r.roundWindows;
  d["sampled_local"] = r.sampledLocal;
  d["bitmap_join"] = r.bitmapJoin;
  d["local_fallbacks"] = r.localFallbacks;
  d["join_ms"] = r.joinMs;
  d["histogram_ms"] = r.histogramMs;
  d["window_ms"] = r.windowMs;
  d["network_ms"] = r.networkMs;
  d["local_ms"] = r.localMs;
  d["dev_histogram_ms"] = r.devHistogramMs;
  d["dev_network_ms"] = r.devNetworkMs;
  d["dev_local_partition_ms"] = r.devLocalPartitionMs;
  d["dev_build_probe_ms"] = r.devBuildProbeMs;
  d["setup_ms"] = r.setupMs;
  d["teardown_ms"] = r.teardownMs;
  d["enqueue_ms"] = r.enqueueMs;
  d["host_wait_ms"] = r.hostWaitMs;
  d["dev_span_ms"] = r.devSpanMs;
  d["exchange_checked"] = r.exchangeChecked;
  d["passes"] = r.passes;
  d["compact_ms"] = r.compactMs;
  d["verify_ms"] = r.verifyMs;
  d["group_passes"] = r.groupPasses;
  d["inner_received"] = r.innerReceived;
  d["wire_bytes"] = r.wireBytes;
  d["outer_received"] = r.outerReceived;
  d["local_items"] = r.localItems;
  d["build_probe_items"] = r.buildProbeItems;
  d["inner_local"] = r.innerLocal;
  d["outer_local"] = r.outerLocal;
  return d;
}

// Relation wrapper that can keep a torch tensor alive for views.
struct PyRelation {
  std::shared_ptr<data::Relation> rel;
  py::object keepAlive;
};

}  // namespace

// Payload columns must hold a row for every rid of this rank's relation
// slices: the gather kernels index rows by rid - offset on the device.
static py::dict statsToDict(const operators::LateMaterialization::Stats &st) {
  py::dict d;
  d["bucket_ms"] = st.bucketMs;
  d["request_ms"] = st.requestMs;
  d["gather_ms"] = st.gatherMs;
  d["response_ms"] = st.responseMs;
  d["place_ms"] = st.placeMs;
  d["request_bytes"] = st.requestBytes;
  d["response_bytes"] = st.responseBytes;
  return d;
}

static void checkPayloadCover(const operators::HashJoin &j, const at::Tensor &a, uint64_t offA, const at::Tensor &b,
                              uint64_t offB) {
  const uint64_t off[2] = {offA, offB}, rows[2] = {(uint64_t)a.size(0), (uint64_t)b.size(0)};
  for (int r = 0; r < 2; ++r) {
    const uint64_t lo = j.ridMin(r), hi = j.ridMax(r);
    TORCH_CHECK(lo > hi || (lo >= off[r] && hi - off[r] < rows[r]), r ? "outer" : "inner", " payload rows [", off[r],
                ", ", off[r] + rows[r], ") do not cover this rank's rids [", lo, ", ", hi, "]");
  }
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native distributed radix hash join engine (native core)";
  m.attr("ARCH") = "gfx950";

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });

  py::enum_<kernels::KeyDistribution>(m, "KeyDistribution")
      .value("UNIQUE", kernels::KeyDistribution::Unique)
      .value("MODULO", kernels::KeyDistribution::Modulo)
      .value("UNIFORM", kernels::KeyDistribution::Uniform)
      .value("ZIPF", kernels::KeyDistribution::Zipf)
      .value("DENSE", kernels::KeyDistribution::Dense);
  py::enum_<core::AssignmentPolicy>(m, "AssignmentPolicy")
      .value("ROUND_ROBIN", core::AssignmentPolicy::RoundRobin)
      .value("LPT", core::AssignmentPolicy::LPT);
  py::enum_<core::TupleFormat>(m, "TupleFormat")
      .value("COMPRESSED", core::TupleFormat::Compressed)
      .value("WIDE", core::TupleFormat::Wide);

  py::enum_<core::KeyHashing>(m, "KeyHashing")
      .value("AUTO", core::KeyHashing::Auto)
      .value("OFF", core::KeyHashing::Off)
      .value("ON", core::KeyHashing::On);
  py::enum_<core::HistogramMode>(m, "HistogramMode")
      .value("AUTO", core::HistogramMode::Auto)
      .value("EXACT", core::HistogramMode::Exact)
      .value("SAMPLED", core::HistogramMode::Sampled);
  m.attr("NetworkHistogram") = m.attr("HistogramMode");
  py::enum_<core::WireCodecMode>(m, "WireCodecMode")
      .value("AUTO", core::WireCodecMode::Auto)
      .value("OFF", core::WireCodecMode::Off)
      .value("ON", core::WireCodecMode::On);
  py::enum_<core::PlanChoice>(m, "PlanChoice")
      .value("AUTO", core::PlanChoice::Auto)
      .value("OFF", core::PlanChoice::Off)
      .value("ON", core::PlanChoice::On);
  py::enum_<core::ExchangeMode>(m, "ExchangeMode")
      .value("RCCL", core::ExchangeMode::Rccl)
      .value("ONE_SIDED", core::ExchangeMode::OneSided);
  py::class_<core::JoinConfig>(m, "JoinConfig")
      .def(py::init<>())
      .def_readwrite("network_bits", &core::JoinConfig::networkBits)
      .def_readwrite("local_bits", &core::JoinConfig::localBits)
      .def_readwrite("two_level", &core::JoinConfig::twoLevel)
      .def_readwrite("key_shift", &core::JoinConfig::keyShift)
      .def_readwrite("assignment", &core::JoinConfig::assignment)
      .def_readwrite("format", &core::JoinConfig::format)
      .def_readwrite("materialize", &core::JoinConfig::materialize)
      .def_readwrite("key_hashing", &core::JoinConfig::keyHashing)
      .def_readwrite("network_histogram", &core::JoinConfig::networkHistogram)
      .def_readwrite("local_histogram", &core::JoinConfig::localHistogram)
      .def_readwrite("sample_stride", &core::JoinConfig::sampleStride)
      .def_readwrite("wire_codec", &core::JoinConfig::wireCodec)
      .def_readwrite("split_local", &core::JoinConfig::splitLocal)
      .def_readwrite("skew_split", &core::JoinConfig::skewSplit)
      .def_readwrite("direct_count", &core::JoinConfig::directCount)
      .def_readwrite("bitmap_join", &core::JoinConfig::bitmapJoin)
      .def_readwrite("replicate_bitmap", &core::JoinConfig::replicateBitmap)
      .def_readwrite("verify_exchange", &core::JoinConfig::verifyExchange)
      .def_readwrite("passes", &core::JoinConfig::passes)
      .def_readwrite("exchange", &core::JoinConfig::exchange)
      .def_readwrite("split_histogram", &core::JoinConfig::splitHistogram)
      .def_readwrite("pipeline_outer", &core::JoinConfig::pipelineOuter)
      .def_readwrite("local_item_tiles", &core::JoinConfig::localItemTiles)
      .def_readwrite("local_geometry", &core::JoinConfig::localGeometry)
      .def_readwrite("local_sample_stride", &core::JoinConfig::localSampleStride)
      .def_readwrite("round_lp", &core::JoinConfig::roundLp)
      .def_readwrite("output_capacity", &core::JoinConfig::outputCapacity)
      .def_readwrite("codec_extra_ps_per_tuple", &core::JoinConfig::codecExtraPsPerTuple)
      .def_property(
          "output_host", [](const core::JoinConfig &c) { return (uint64_t)(uintptr_t)c.outputHost; },
          [](core::JoinConfig &c, uint64_t addr) { c.outputHost = reinterpret_cast<void *>((uintptr_t)addr); },
          "address of a pinned host buffer of output_capacity (rid, rid) pairs (e.g. hpcjoin.pinned_pairs(n)): a "
          "materializing join writes its pairs there instead of the workspace (0 = workspace)")
      .def_readwrite("build_target", &core::JoinConfig::buildTarget)
      .def_readwrite("r_chunk", &core::JoinConfig::rChunk)
      .def_readwrite("s_chunk", &core::JoinConfig::sChunk)
      .def_readwrite("chunks", &core::JoinConfig::chunks)
      .def_readwrite("checks", &core::JoinConfig::checks)
      .def_readwrite("max_partition_blocks", &core::JoinConfig::maxPartitionBlocks)
      .def_readwrite("reserve_workspace", &core::JoinConfig::reserveWorkspace)
      .def_readwrite("workspace_budget", &core::JoinConfig::workspaceBudget)
      .def_readwrite("link_gbps_per_peer", &core::JoinConfig::linkGBpsPerPeer)
      // KernelVariants, flattened (sweeps / A-B tests; core/Types.h)
      .def_property("net_ipt", [](const core::JoinConfig &c) { return c.variants.netIpt; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.netIpt = v; })
      .def_property("net_threads", [](const core::JoinConfig &c) { return c.variants.netThreads; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.netThreads = v; })
      .def_property("bm_threads", [](const core::JoinConfig &c) { return c.variants.bmThreads; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.bmThreads = v; })
      .def_property("bm_flat", [](const core::JoinConfig &c) { return c.variants.bmFlat; },
                    [](core::JoinConfig &c, int32_t v) { c.variants.bmFlat = v; })
      .def_property("reduce_chunks", [](const core::JoinConfig &c) { return c.variants.reduceChunks; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.reduceChunks = v; })
      .def_property("key_count", [](const core::JoinConfig &c) { return c.variants.keyCount; },
                    [](core::JoinConfig &c, uint32_t v) {
                      HJ_CHECK(v >= 7 && v <= 9, "key_count: 7 (v2 buckets), 8 (quotient) or 9 (counted), got %u", v);
                      c.variants.keyCount = v;
                    })
      .def_property("rows_lds", [](const core::JoinConfig &c) { return c.variants.rowsLds; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.rowsLds = v; })
      .def_property("mat_variant", [](const core::JoinConfig &c) { return c.variants.matVariant; },
                    [](core::JoinConfig &c, uint32_t v) { c.variants.matVariant = v; })
      .def("__repr__", &core::JoinConfig::describe);

  py::class_<core::JoinPlan>(m, "JoinPlan")
      .def_readonly("number_of_nodes", &core::JoinPlan::numberOfNodes)
      .def_readonly("network_bits", &core::JoinPlan::networkBits)
      .def_readonly("key_mix", &core::JoinPlan::keyMix)
      .def_readonly("sampled_network", &core::JoinPlan::sampledNetwork)
      .def_readonly("bitmap_join", &core::JoinPlan::bitmapJoin)
      .def_readonly("bitmap_bits", &core::JoinPlan::bitmapBits)
      .def_readonly("bitmap_replicated", &core::JoinPlan::bitmapReplicated)
      .def_readonly("key_only", &core::JoinPlan::keyOnly)
      .def_readonly("inner_repeats", &core::JoinPlan::innerRepeats)
      .def_readonly("one_sided", &core::JoinPlan::oneSided)
      .def_readonly("replicated_link_bytes", &core::JoinPlan::replicatedLinkBytes)
      .def_readonly("shuffle_link_bytes", &core::JoinPlan::shuffleLinkBytes)
      .def_readonly("link_gbps", &core::JoinPlan::linkGBps)
      .def_readonly("split_histogram", &core::JoinPlan::splitHistogram)
      .def_readonly("pipeline_outer", &core::JoinPlan::pipelineOuter)
      .def_readonly("local_bits", &core::JoinPlan::localBits)
      .def_readonly("key_shift", &core::JoinPlan::keyShift)
      .def_readonly("frag_shift", &core::JoinPlan::fragShift)
      .def_readonly("key_bits", &core::JoinPlan::keyBits)
      .def_readonly("split_local", &core::JoinPlan::splitLocal)
      .def_readonly("fragments", &core::JoinPlan::fragments)
      .def_readonly("skew_split", &core::JoinPlan::skewSplit)
      .def_property_readonly("wire_bits", [](const core::JoinPlan &p) {
        return std::vector<uint32_t>{p.wireBits[0], p.wireBits[1]};
      })
      .def_readonly("r_chunk", &core::JoinPlan::rChunk)
      .def_readonly("s_chunk", &core::JoinPlan::sChunk)
      .def_readonly("chunks", &core::JoinPlan::chunks)
      .def_readonly("two_level", &core::JoinPlan::twoLevel)
      .def_readonly("wide", &core::JoinPlan::wide)
      .def_readonly("materialize", &core::JoinPlan::materialize)
      .def("__repr__", &core::JoinPlan::describe);
  m.def("make_plan", &core::makePlan, py::arg("config"), py::arg("number_of_nodes"), py::arg("global_inner"),
        py::arg("global_outer"), py::arg("max_key"), py::arg("max_rid"));

  py::class_<comm::Communicator, std::shared_ptr<comm::Communicator>>(m, "Communicator")
      .def("rank", &comm::Communicator::rank)
      .def("size", &comm::Communicator::size)
      .def("name", &comm::Communicator::name)
      .def("barrier", &comm::Communicator::barrier, py::call_guard<py::gil_scoped_release>())
      .def("check_health", &comm::Communicator::checkHealth)
      .def("abort", &comm::Communicator::abort, py::arg("why"), py::call_guard<py::gil_scoped_release>())
      .def("all_gather", [](comm::Communicator &c, std::vector<uint64_t> v) {
        std::vector<uint64_t> out(v.size() * c.size());
        {
          py::gil_scoped_release nogil;
          c.allGatherHost(v.data(), out.data(), v.size());
        }
        return out;
      })
      .def("all_to_all_v",
           [](comm::Communicator &c, at::Tensor send, std::vector<uint64_t> sendCounts, at::Tensor recv,
              std::vector<uint64_t> recvCounts) {
             // Words (int64 elements); displacements are the running sums.
             TORCH_CHECK(send.scalar_type() == at::kLong && recv.scalar_type() == at::kLong, "int64 tensors");
             const uint32_t n = c.size();
             TORCH_CHECK(sendCounts.size() == n && recvCounts.size() == n, "one count per rank");
             std::vector<uint64_t> sd(n), rd(n);
             for (uint32_t p = 1; p < n; ++p) {
               sd[p] = sd[p - 1] + sendCounts[p - 1];
               rd[p] = rd[p - 1] + recvCounts[p - 1];
             }
             const Location l = locOf(send);
             if (l == Location::Device) HIP_CHECK(hipDeviceSynchronize());
             py::gil_scoped_release nogil;
             c.allToAllV(ptr<uint64_t>(send), sendCounts.data(), sd.data(), ptr<uint64_t>(recv), recvCounts.data(),
                         rd.data(), l, nullptr);
             if (l == Location::Device) HIP_CHECK(hipDeviceSynchronize());
           })
      .def("all_reduce_sum", [](comm::Communicator &c, std::vector<uint64_t> v) {
        {
          py::gil_scoped_release nogil;
          c.allReduceSumHost(v.data(), v.size());
        }
        return v;
      });
  py::class_<comm::LocalCommunicator, comm::Communicator, std::shared_ptr<comm::LocalCommunicator>>(
      m, "LocalCommunicator")
      .def(py::init<>());
  py::class_<comm::RcclCommunicator, comm::Communicator, std::shared_ptr<comm::RcclCommunicator>>(m,
                                                                                                   "RcclCommunicator")
      .def(py::init([](py::bytes id, uint32_t rank, uint32_t size, int device) {
             std::string s = id;
             std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;
             return std::make_shared<comm::RcclCommunicator>(v, rank, size, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("size"), py::arg("device"));
  py::class_<comm::InProcessGroup, std::shared_ptr<comm::InProcessGroup>>(m, "InProcessGroup")
      .def(py::init<uint32_t>(), py::arg("size"))
      .def("size", &comm::InProcessGroup::size)
      .def("abort", &comm::InProcessGroup::abort, py::arg("why"))
      .def("aborted", &comm::InProcessGroup::aborted)
      .def("communicator", [](std::shared_ptr<comm::InProcessGroup> g, uint32_t rank) {
        return std::static_pointer_cast<comm::Communicator>(std::make_shared<comm::InProcessCommunicator>(g, rank));
      });
  m.def("device_info", [](int dev) {
    // Identity of a device as this process sees it (bench.py topology record).
    hipDeviceProp_t pr;
    HIP_CHECK(hipGetDeviceProperties(&pr, dev));
    char bus[64] = {0};
    HIP_CHECK(hipDeviceGetPCIBusId(bus, sizeof(bus), dev));
    int count = 0;
    HIP_CHECK(hipGetDeviceCount(&count));
    py::dict d;
    d["device"] = dev;
    d["pci_bus_id"] = std::string(bus);
    d["name"] = std::string(pr.name);
    d["arch"] = std::string(pr.gcnArchName);
    d["compute_units"] = pr.multiProcessorCount;
    d["hbm_bytes"] = (uint64_t)pr.totalGlobalMem;
    d["visible_devices"] = count;
    return d;
  }, py::arg("device"));
  m.def("rccl_unique_id", []() {
    auto v = comm::RcclCommunicator::uniqueId();
    return py::bytes(reinterpret_cast<const char *>(v.data()), v.size());
  });
  py::class_<comm::ProcessGroupCommunicator, comm::Communicator, std::shared_ptr<comm::ProcessGroupCommunicator>>(
      m, "ProcessGroupCommunicator")
      .def(py::init<c10::intrusive_ptr<c10d::ProcessGroup>>(), py::arg("process_group"));
  m.def("set_world", [](std::shared_ptr<comm::Communicator> c) {
    static std::shared_ptr<comm::Communicator> keep;
    keep = c;
    comm::setWorld(c.get());
  });

  py::class_<core::ExecContext, std::shared_ptr<core::ExecContext>>(m, "ExecContext")
      .def(py::init([](const std::string &loc, int device, std::shared_ptr<comm::Communicator> c) {
             TORCH_CHECK(loc == "device" || loc == "host", "engine location must be device|host");
             auto ctx = std::shared_ptr<core::ExecContext>(
                 new core::ExecContext(loc == "device" ? Location::Device : Location::Host, device, c.get()),
                 [c](core::ExecContext *p) { delete p; });
             return ctx;
           }),
           py::arg("location"), py::arg("device"), py::arg("communicator"))
      .def_property_readonly("on_device", &core::ExecContext::onDevice)
      .def_property_readonly("device", &core::ExecContext::device)
      .def_property_readonly("node_id", &core::ExecContext::nodeId)
      .def_property_readonly("number_of_nodes", &core::ExecContext::numberOfNodes)
      .def("workspace_capacity", [](core::ExecContext &c) { return c.workspace().capacity(); })
      .def("workspace_peak", [](core::ExecContext &c) { return c.workspace().peak(); })
      .def("reset_scratch", &core::ExecContext::resetScratch, py::call_guard<py::gil_scoped_release>(),
           "Rewind the arenas; if the last join spilled into fallback allocations, re-reserve one block of "
           "the observed peak now (so the next join does not pay for it)")
      .def("reserve_workspace", [](core::ExecContext &c, uint64_t b) { c.workspace().reserve(b); })
      .def("trim_workspace", [](core::ExecContext &c, uint64_t keep) {
             // Collective when the communicator has several ranks (every rank
             // calls it together): all ranks close their mappings of peers'
             // memory before any rank frees, and no rank starts a join
             // before every free is done.
             c.synchronize();
             c.releaseImports();
             const bool multi = c.comm()->size() > 1;
             if (multi) c.comm()->barrier();
             const uint64_t freed = c.workspace().trim(keep);
             if (multi) c.comm()->barrier();
             return freed;
           },
           py::arg("keep") = 0,
           "Between joins, on every rank together: shrink the workspace to one chunk of `keep` bytes; returns the "
           "bytes freed")
      .def("workspace_generation", [](core::ExecContext &c) { return c.workspace().generation(); })
      .def("ensure_workspace", [](core::ExecContext &c, uint64_t b) { return c.workspace().ensure(b); })
      .def("workspace_scratch", [](core::ExecContext &c, uint64_t b) {
             return reinterpret_cast<uintptr_t>(c.workspace().get(b));
           }, "Hand out b bytes of the workspace (tests of the arena's growth rules)")
      .def("synchronize", &core::ExecContext::synchronize)
      // One-sided window plumbing, for the IPC ordering tests (tests/ipc_order_worker.py)
      .def("ipc_export", [](core::ExecContext &c, uintptr_t p) {
             uint64_t h[8], off = 0, gen = 0, tagOff = 0, nonce = 0;
             c.ipcExport(reinterpret_cast<const void *>(p), h, &off, &gen, &tagOff, &nonce);
             return py::make_tuple(py::bytes(reinterpret_cast<const char *>(h), sizeof(h)), off, gen, tagOff, nonce);
           }, py::arg("ptr"),
           "(handle bytes, offset in its allocation, workspace generation, tag offset, tag nonce) of a workspace "
           "address")
      .def("ipc_import", [](core::ExecContext &c, uint32_t peer, const py::bytes &handle, uint64_t gen,
                            uint64_t tagOff, uint64_t nonce) {
             const std::string s = handle;
             TORCH_CHECK(s.size() == 64, "an IPC handle is 64 bytes");
             uint64_t h[8];
             std::memcpy(h, s.data(), 64);
             return reinterpret_cast<uintptr_t>(c.ipcImport(peer, h, gen, tagOff, nonce));
           }, py::arg("peer"), py::arg("handle"), py::arg("generation"), py::arg("tag_offset"), py::arg("nonce"),
           "Base address of the mapping of a peer's exported allocation (cached per handle and generation; a "
           "fresh open checks the allocation's tag and throws on a stale mapping)")
      .def("release_imports", &core::ExecContext::releaseImports)
      .def("ipc_mappings", &core::ExecContext::ipcMappings)
      .def("ipc_log", [](const core::ExecContext &c) {
             py::list out;
             for (const auto &e : c.ipcLog())
               out.append(py::make_tuple(std::string(1, e.op), e.cached, e.peer, e.generation, e.handleHash,
                                         reinterpret_cast<uintptr_t>(e.ptr)));
             return out;
           }, "(op, cached, peer, generation, handle hash, address) per export 'E' / open 'O' / stale close 'C' / "
              "releaseImports 'R', in order");

  py::class_<data::GenSpec>(m, "GenSpec")
      .def(py::init<>())
      .def(py::init([](kernels::KeyDistribution d, uint64_t seed, uint64_t domain, uint64_t keyOffset, double theta) {
             data::GenSpec s;
             s.distribution = d;
             s.seed = seed;
             s.domain = domain;
             s.keyOffset = keyOffset;
             s.zipfTheta = theta;
             return s;
           }),
           py::arg("distribution") = kernels::KeyDistribution::Unique, py::arg("seed") = 1234, py::arg("domain") = 0,
           py::arg("key_offset") = 0, py::arg("zipf_theta") = 0.75)
      .def(py::init([](kernels::KeyDistribution d, uint64_t seed, uint64_t domain, uint64_t keyOffset, double theta,
                       bool sparse) {
             data::GenSpec s;
             s.distribution = d;
             s.seed = seed;
             s.domain = domain;
             s.keyOffset = keyOffset;
             s.zipfTheta = theta;
             s.tpchSparse = sparse;
             return s;
           }),
           py::arg("distribution"), py::arg("seed"), py::arg("domain"), py::arg("key_offset"), py::arg("zipf_theta"),
           py::arg("tpch_sparse"))
      .def_readwrite("distribution", &data::GenSpec::distribution)
      .def_readwrite("seed", &data::GenSpec::seed)
      .def_readwrite("domain", &data::GenSpec::domain)
      .def_readwrite("key_offset", &data::GenSpec::keyOffset)
      .def_readwrite("zipf_theta", &data::GenSpec::zipfTheta)
      .def_readwrite("tpch_sparse", &data::GenSpec::tpchSparse)
      .def_readwrite("sparse64", &data::GenSpec::sparse64);

  py::class_<PyRelation>(m, "Relation")
      .def(py::init([](uint64_t localSize, uint64_t globalSize, const std::string &loc, int device) {
             PyRelation r;
             TORCH_CHECK(loc == "device" || loc == "host" || loc == "pinned", "location must be device|host|pinned");
             r.rel = std::make_shared<data::Relation>(
                 localSize, globalSize,
                 loc == "device" ? Location::Device : (loc == "pinned" ? Location::Pinned : Location::Host), device);
             return r;
           }),
           py::arg("local_size"), py::arg("global_size"), py::arg("location") = "device", py::arg("device") = 0)
      .def_static(
          "from_tensor",
          [](at::Tensor t, uint64_t globalSize) {
            checkTuples(t, "tuples");
            if (t.is_cuda()) HIP_CHECK(hipDeviceSynchronize());
            PyRelation r;
            r.rel = std::make_shared<data::Relation>(ptr<data::Tuple>(t), t.size(0), globalSize, locOf(t),
                                                     t.is_cuda() ? t.get_device() : 0);
            r.keepAlive = py::cast(t);
            return r;
          },
          py::arg("tuples"), py::arg("global_size"))
      .def("local_size", [](PyRelation &r) { return r.rel->getLocalSize(); })
      .def("global_size", [](PyRelation &r) { return r.rel->getGlobalSize(); })
      .def("location", [](PyRelation &r) { return std::string(locationName(r.rel->location())); })
      .def("fill_unique_values", [](PyRelation &r, uint64_t k, uint64_t rid) { r.rel->fillUniqueValues(k, rid); })
      .def("fill_modulo_values",
           [](PyRelation &r, uint64_t k, uint64_t rid, uint64_t inner) { r.rel->fillModuloValues(k, rid, inner); })
      .def("generate", [](PyRelation &r, const data::GenSpec &s, uint64_t off) { r.rel->generate(s, off); },
           py::arg("spec"), py::arg("global_offset"))
      .def("distribute",
           [](PyRelation &r, uint32_t node, uint32_t n, std::shared_ptr<comm::Communicator> c) {
             py::gil_scoped_release nogil;
             r.rel->distribute(node, n, c.get());
           })
      .def("to_tensor",
           [](PyRelation &r) {
             const auto &rel = r.rel;
             auto opts = at::TensorOptions().dtype(at::kLong);
             if (rel->location() == Location::Device) opts = opts.device(at::kCUDA, rel->device());
             at::Tensor out = at::empty({(int64_t)rel->getLocalSize(), 2}, opts);
             if (rel->location() == Location::Device)
               HIP_CHECK(hipMemcpy(out.data_ptr(), rel->getData(), rel->getLocalSize() * 16, hipMemcpyDeviceToDevice));
             else
               std::memcpy(out.data_ptr(), rel->getData(), rel->getLocalSize() * 16);
             return out;
           })
      .def("count_keys",
           [](PyRelation &r, at::Tensor counts, uint64_t lo) {
             // Oracle of skewed joins: counts (int32, zeroed, on the relation's
             // device) += one per key in [lo, lo + counts.numel()); returns the
             // number of keys outside that range.
             const auto &rel = r.rel;
             TORCH_CHECK(rel->location() == Location::Device && counts.is_cuda(), "count_keys: device relations");
             TORCH_CHECK(counts.scalar_type() == at::kInt && counts.is_contiguous(), "count_keys: contiguous int32");
             at::Tensor out = at::zeros({1}, at::TensorOptions().dtype(at::kLong).device(counts.device()));
             kernels::countKeys(rel->getData(), rel->getLocalSize(), lo, (uint64_t)counts.numel(),
                                reinterpret_cast<uint32_t *>(counts.data_ptr()),
                                reinterpret_cast<unsigned long long *>(out.data_ptr()), nullptr);
             HIP_CHECK(hipDeviceSynchronize());
             return out.item<int64_t>();
           },
           py::arg("counts"), py::arg("lo") = 0)
      .def_static("local_size_for", &data::Relation::localSizeFor)
      .def_static("local_offset_for", &data::Relation::localOffsetFor)
      .def_static("expected_matches", [](const data::GenSpec &i, uint64_t gi, const data::GenSpec &o, uint64_t go) {
        uint64_t v = data::Relation::expectedMatches(i, gi, o, go);
        return v == UINT64_MAX ? py::object(py::none()) : py::object(py::int_(v));
      });

  py::class_<operators::HashJoin, std::shared_ptr<operators::HashJoin>>(m, "HashJoin")
      .def_static("codec_pays", &operators::HashJoin::codecPays, py::arg("wire_bits"), py::arg("nodes"),
                  py::arg("link_gbps_per_peer"), py::arg("extra_ps_per_tuple") = 3.5,
                  "The wire codec's cost model: packing w-bit tuples pays at this world size and link rate")
      .def(py::init([](PyRelation &inner, PyRelation &outer, std::shared_ptr<core::ExecContext> ctx,
                       const core::JoinConfig &cfg) {
             py::gil_scoped_release nogil;
             return std::make_shared<operators::HashJoin>(inner.rel.get(), outer.rel.get(), ctx.get(), cfg);
           }),
           py::arg("inner"), py::arg("outer"), py::arg("context"), py::arg("config") = core::JoinConfig(),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def("run",
           [](operators::HashJoin &j) {
             operators::JoinResult r;
             {
               py::gil_scoped_release nogil;
               r = j.run();
             }
             return resultToDict(r);
           })
      .def("join", [](operators::HashJoin &j) {
        py::gil_scoped_release nogil;
        j.join();
      })
      .def_property_readonly("plan", &operators::HashJoin::getPlan)
      .def("workspace_estimate", &operators::HashJoin::workspaceEstimate)
      .def_property_readonly("reserved_bytes", &operators::HashJoin::reservedBytes)
      .def_property_readonly("spill_passes", &operators::HashJoin::spillPasses)
      .def_property_readonly("spill_info", [](const operators::HashJoin &j) {
        py::dict d;
        d["passes"] = j.spillPasses();
        d["estimate_bytes"] = j.spill.estimate;
        d["available_bytes"] = j.spill.available;
        d["pass_buffer_bytes"] = j.spill.passBuffers;
        d["pass_estimate_bytes"] = j.spill.passEstimate;
        d["pass_workspace_bytes"] = j.spill.passReserved;
        d["pass_peak_bytes"] = j.spill.passPeak;
        d["group_budget_bytes"] = j.spill.groupBudget;
        return d;
      })
      .def_property_readonly("plan_ms", &operators::HashJoin::planMilliseconds)
      .def_property_readonly("reserve_ms", &operators::HashJoin::reserveMilliseconds)
      .def(
          "materialize_payloads",
          [](operators::HashJoin &j, std::shared_ptr<core::ExecContext> ctx, at::Tensor innerRows, uint64_t innerOffset,
             uint64_t innerGlobal, at::Tensor outerRows, uint64_t outerOffset, uint64_t outerGlobal,
             bool returnStats) -> py::object {
            // Collective.  Returns [pairs, 10] int64: rid_inner, rid_outer, inner row (4), outer row (4)
            // (return_stats: (rows, phase times and link bytes of the request/response exchange)).
            TORCH_CHECK(j.getConfig().materialize, "join was not run with materialize=True");
            TORCH_CHECK(!j.lastResult().rowsFused, "the last run wrote rows directly (join_materialized)");
            TORCH_CHECK(innerRows.dim() == 2 && innerRows.size(1) == (int64_t)kernels::ROW_WORDS &&
                            outerRows.dim() == 2 && outerRows.size(1) == (int64_t)kernels::ROW_WORDS,
                        "payload rows must be [n, 4] int64 (32 bytes)");
            checkPayloadCover(j, innerRows, innerOffset, outerRows, outerOffset);
            operators::PayloadColumn a{ptr<uint64_t>(innerRows), (uint64_t)innerRows.size(0), innerOffset, innerGlobal};
            operators::PayloadColumn b{ptr<uint64_t>(outerRows), (uint64_t)outerRows.size(0), outerOffset, outerGlobal};
            const uint64_t n = j.lastResult().outputPairs;
            at::Tensor out = at::empty({(int64_t)n, (int64_t)operators::LateMaterialization::OUT_WORDS},
                                       at::TensorOptions().dtype(at::kLong).device(innerRows.device()));
            if (innerRows.is_cuda()) HIP_CHECK(hipDeviceSynchronize());
            operators::LateMaterialization::Stats st;
            {
              py::gil_scoped_release nogil;
              operators::LateMaterialization lm(ctx.get(), a, b, j.getConfig().variants.matVariant);
              lm.materialize(j.getOutput(), n, ptr<uint64_t>(out));
              st = lm.stats();
            }
            if (returnStats) return py::make_tuple(out, statsToDict(st));
            return py::cast(out);
          },
          py::arg("context"), py::arg("inner_rows"), py::arg("inner_rid_offset"), py::arg("inner_global_rows"),
          py::arg("outer_rows"), py::arg("outer_rid_offset"), py::arg("outer_global_rows"),
          py::arg("return_stats") = false)
      .def_property_readonly("can_fuse_rows", &operators::HashJoin::canFuseRows)
      .def(
          "join_materialized",
          [](operators::HashJoin &j, std::shared_ptr<core::ExecContext> ctx, at::Tensor innerRows, uint64_t innerOffset,
             uint64_t innerGlobal, at::Tensor outerRows, uint64_t outerOffset, uint64_t outerGlobal) {
            // Collective.  One join + both payload rows of every result pair:
            // returns (result dict, [pairs, 10] int64 rows).  Device joins at
            // N = 1 write the rows from the build/probe's materialize pass
            // (no pair array); otherwise run() + LateMaterialization.
            TORCH_CHECK(j.getConfig().materialize, "join_materialized needs materialize=True");
            TORCH_CHECK(innerRows.dim() == 2 && innerRows.size(1) == (int64_t)kernels::ROW_WORDS &&
                            outerRows.dim() == 2 && outerRows.size(1) == (int64_t)kernels::ROW_WORDS,
                        "payload rows must be [n, 4] int64 (32 bytes)");
            TORCH_CHECK(innerRows.is_contiguous() && outerRows.is_contiguous(), "payload rows must be contiguous");
            checkPayloadCover(j, innerRows, innerOffset, outerRows, outerOffset);
            const auto opts = at::TensorOptions().dtype(at::kLong).device(innerRows.device());
            constexpr int64_t W = operators::LateMaterialization::OUT_WORDS;
            operators::JoinResult r;
            if (innerRows.is_cuda()) HIP_CHECK(hipDeviceSynchronize());  // payloads written on other streams
            if (innerRows.is_cuda() && outerRows.is_cuda() && j.canFuseRows()) {
              struct Clear {
                operators::HashJoin &j;
                ~Clear() { j.clearRowSink(); }
              } clear{j};
              uint64_t cap = j.getConfig().outputCapacity ? j.getConfig().outputCapacity
                                                          : (uint64_t)outerRows.size(0) + 1024;
              for (int attempt = 0; attempt < 2; ++attempt) {
                at::Tensor out = at::empty({(int64_t)cap, W}, opts);
                kernels::RowSink sk;
                sk.rowsA = ptr<uint64_t>(innerRows);
                sk.offA = innerOffset;
                sk.rowsAN = (uint64_t)innerRows.size(0);
                sk.rowsB = ptr<uint64_t>(outerRows);
                sk.offB = outerOffset;
                sk.rowsBN = (uint64_t)outerRows.size(0);
                sk.out = ptr<uint64_t>(out);
                sk.capacity = cap;
                j.setRowSink(sk);
                {
                  py::gil_scoped_release nogil;
                  r = j.run();
                }
                if (!r.rowsFused) break;  // this run took another layout: materialize the pairs below
                if (!r.outputOverflow)
                  return py::make_tuple(resultToDict(r), out.narrow(0, 0, (int64_t)r.outputPairs));
                cap = r.outputPairs;  // more matches than the first guess: once more, exactly sized
              }
              TORCH_CHECK(!r.rowsFused, "join_materialized: row output overflowed twice");
            } else {
              py::gil_scoped_release nogil;
              r = j.run();
            }
            operators::PayloadColumn a{ptr<uint64_t>(innerRows), (uint64_t)innerRows.size(0), innerOffset, innerGlobal};
            operators::PayloadColumn b{ptr<uint64_t>(outerRows), (uint64_t)outerRows.size(0), outerOffset, outerGlobal};
            const uint64_t n = r.outputPairs;
            at::Tensor out = at::empty({(int64_t)n, W}, opts);
            operators::LateMaterialization::Stats st;
            {
              py::gil_scoped_release nogil;
              operators::LateMaterialization lm(ctx.get(), a, b, j.getConfig().variants.matVariant);
              lm.materialize(j.getOutput(), n, ptr<uint64_t>(out));
              st = lm.stats();
            }
            py::dict d = resultToDict(r);
            d["materialize_phases"] = statsToDict(st);
            return py::make_tuple(d, out);
          },
          py::arg("context"), py::arg("inner_rows"), py::arg("inner_rid_offset"), py::arg("inner_global_rows"),
          py::arg("outer_rows"), py::arg("outer_rid_offset"), py::arg("outer_global_rows"))
      .def("output", [](operators::HashJoin &j) {
        const auto &r = j.lastResult();
        const uint64_t n = r.outputPairs;
        at::Tensor out = at::empty({(int64_t)n, 2}, at::kLong);
        if (n && j.getOutput()) {
          HJ_CHECK(j.outputValid(),
                   "HashJoin.output(): the pairs of the last run were in the engine workspace, which a later join, "
                   "plan or trim_workspace on the same context has since reused; read output() right after run()");
          if (j.context()->onDevice())  // workspace pairs, or the pinned host buffer (outputHost)
            HIP_CHECK(hipMemcpy(out.data_ptr(), j.getOutput(), n * 16, hipMemcpyDefault));
          else
            std::memcpy(out.data_ptr(), j.getOutput(), n * 16);
        }
        return out;
      });
  m.def("result_counter", []() { return operators::HashJoin::RESULT_COUNTER; });
  m.def(
      "pinned_pairs",
      [](uint64_t n) {
        // Page-locked, device-mapped host memory for JoinConfig.output_host:
        // the place kernel writes pairs into it over the host link.
        void *p = nullptr;
        HIP_CHECK(hipHostMalloc(&p, std::max<uint64_t>(n, 1) * 16, hipHostMallocMapped | hipHostMallocPortable));
        return at::from_blob(
            p, {(int64_t)n, 2}, [](void *q) { (void)hipHostFree(q); }, at::TensorOptions().dtype(at::kLong));
      },
      py::arg("pairs"), "A pinned, device-mapped host tensor [pairs, 2] (int64) for JoinConfig.output_host");

  auto fault = m.def_submodule("fault", "failure detection and fault injection");
  py::register_exception<utils::InjectedFault>(fault, "InjectedFault", PyExc_RuntimeError);
  fault.def("arm", &utils::armFault, py::arg("phase"), py::arg("rank") = -1,
            "Arm a one-shot fault for the calling thread at phase histogram|network|local|build_probe "
            "(rank -1: any rank).  An empty phase disarms.");
  fault.def("set_comm_timeout_ms", &utils::setCommTimeoutMs, py::arg("ms"));
  fault.def("comm_timeout_ms", &utils::commTimeoutMs);

  auto ipc = m.def_submodule("ipc", "raw HIP IPC calls and host copies, for the IPC ordering tests");
  ipc.def("get_handle", [](uintptr_t p) {
    hipIpcMemHandle_t h;
    HIP_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void *>(p)));
    return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h));
  });
  ipc.def("open", [](const py::bytes &handle) {
    const std::string s = handle;
    TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "an IPC handle is 64 bytes");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void *p = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    return reinterpret_cast<uintptr_t>(p);
  });
  ipc.def("close", [](uintptr_t p) { HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void *>(p))); });
  ipc.def("is_device_pointer", [](uintptr_t p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, reinterpret_cast<void *>(p)) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeDevice;
  });
  ipc.def("write", [](uintptr_t p, const py::bytes &b) {
    const std::string s = b;
    HIP_CHECK(hipMemcpy(reinterpret_cast<void *>(p), s.data(), s.size(), hipMemcpyHostToDevice));
  });
  ipc.def("read", [](uintptr_t p, size_t n) {
    std::string s(n, '\0');
    HIP_CHECK(hipMemcpy(s.data(), reinterpret_cast<const void *>(p), n, hipMemcpyDeviceToHost));
    return py::bytes(s);
  });

  auto meas = m.def_submodule("measurements");
  meas.def("init", &performance::Measurements::init, py::arg("node_id"), py::arg("number_of_nodes"),
           py::arg("tag") = "experiment", py::arg("directory") = "");
  meas.def("write_meta", [](const std::string &k, const std::string &v) {
    performance::Measurements::writeMetaData(k.c_str(), v.c_str());
  });
  meas.def("print_measurements", [](std::shared_ptr<comm::Communicator> c) {
    py::gil_scoped_release nogil;
    performance::Measurements::printMeasurements(c.get());
  });
  meas.def("store_all", &performance::Measurements::storeAllMeasurements);
  meas.def("snapshot", &performance::Measurements::snapshot);
  meas.def("reference_keys", &performance::Measurements::referenceKeys,
           "The reference's .perf keys (performance/Measurements.cpp:136-542), all present after every join");
  meas.def("serialize", &performance::Measurements::serializeResults);

  auto ops = m.def_submodule("ops", "kernel-level entry points on torch tensors (device or host)");
  ops.def("net_histogram", &opNetHistogram, py::arg("tuples"), py::arg("bits"), py::arg("max_blocks") = 2048);
  ops.def("net_partition", &opNetPartition, py::arg("tuples"), py::arg("bits"), py::arg("key_shift") = 32,
          py::arg("wide") = false, py::arg("max_blocks") = 2048, py::arg("key_bits") = 64);
  ops.def("local_partition", &opLocalPartition, py::arg("values"), py::arg("part_begin"), py::arg("shift"),
          py::arg("bits"), py::arg("wide") = false);
  ops.def("build_probe", &opBuildProbe, py::arg("R"), py::arg("S"), py::arg("part_r"), py::arg("part_s"),
          py::arg("frag_shift"), py::arg("key_shift"), py::arg("wide") = false, py::arg("materialize") = false,
          py::arg("r_chunk") = 4096, py::arg("s_chunk") = 65536, py::arg("out_capacity") = 0);
  ops.def("generate", &opGenerate, py::arg("n"), py::arg("global_offset"), py::arg("global_size"), py::arg("spec"),
          py::arg("device") = "cpu");
  ops.def("scan_u32", &opScan);
  ops.def(
      "generate_payload",
      [](int64_t n, uint64_t ridOffset, uint64_t seed, const std::string &device) {
        at::Tensor out = at::empty({n, (int64_t)kernels::ROW_WORDS}, at::TensorOptions().dtype(at::kLong).device(device));
        if (out.is_cuda()) {
          setDevice(out);
          kernels::generatePayload(ptr<uint64_t>(out), n, ridOffset, seed, nullptr);
          HIP_CHECK(hipDeviceSynchronize());
        } else {
          uint64_t *o = ptr<uint64_t>(out);
          for (int64_t i = 0; i < n; ++i)
            for (uint32_t w = 0; w < kernels::ROW_WORDS; ++w)
              o[i * kernels::ROW_WORDS + w] = kernels::payloadWord(seed, ridOffset + i, w);
        }
        return out;
      },
      py::arg("n"), py::arg("rid_offset"), py::arg("seed"), py::arg("device") = "cpu");
  ops.def("npj_count", &opNpjCount);
  ops.def("scatter_profile", [](bool reset) {
    unsigned long long v[10];
    kernels::scatterProfile(v, reset);
    return std::vector<unsigned long long>(v, v + 10);
  }, py::arg("reset") = true,
          "Claim-scatter shader-clock sums per phase (rank, barrier A, claims+prefetch, scan, staging, write bases, "
          "barrier B, write-out), tiles, ranges; zeros unless built with -DHPCJOIN_SCATTER_PROF");
  ops.def("scatter_profile_built", &kernels::scatterProfileBuilt);
  ops.def("npj_join", &opNpjJoin, py::arg("R"), py::arg("S"),
          "(inner rid, outer rid) pairs of the no-partitioning hash join, [matches, 2] int64");
  ops.def("wire_pack", &opWirePack, py::arg("raw"), py::arg("w"), py::arg("rid_bits"), py::arg("key_shift"),
          py::arg("segments"));
  ops.def("wire_unpack", &opWireUnpack, py::arg("wire"), py::arg("raw"), py::arg("w"), py::arg("rid_bits"),
          py::arg("key_shift"), py::arg("segments"));
  ops.def("bench_wire", &benchWire, py::arg("raw"), py::arg("w"), py::arg("rid_bits"), py::arg("key_shift"),
          py::arg("iters") = 10);
  ops.def("net_scatter_global_atomic", &opNetScatterGlobalAtomic);
  ops.def("bench_copy_ms", &benchCopy, py::arg("src"), py::arg("dst"), py::arg("iters") = 10);
  ops.def("bench_read_ms", &benchRead, py::arg("src"), py::arg("iters") = 10);
  // Single un-timed launches on the null stream (MALL probe, tools/mall_probe.py).
  ops.def(
      "gather_rows",
      [](const at::Tensor &rids, uint64_t ridOffset, const at::Tensor &payload, int mode) {
        // out[i] = payload[rids[i] - ridOffset] for 32-byte rows (device; microbenchmark of the random row
        // gather).  mode -1: the operator's gatherRows; 0..3: kernels::gatherVariant shapes (rid_offset 0).
        TORCH_CHECK(rids.is_cuda() && payload.is_cuda() && rids.scalar_type() == at::kLong &&
                        payload.dim() == 2 && payload.size(1) == 4 && payload.is_contiguous() && rids.is_contiguous(),
                    "gather_rows: device int64 rids and [n, 4] int64 payload");
        at::Tensor out = at::empty({rids.size(0), 4}, payload.options());
        if (mode < 0)
          kernels::gatherRows(ptr<uint64_t>(rids), (uint64_t)rids.size(0), ridOffset, ptr<uint64_t>(payload),
                              ptr<uint64_t>(out), nullptr);
        else
          kernels::gatherVariant(mode, ptr<uint64_t>(rids), (uint64_t)rids.size(0), ptr<const ulonglong2>(payload),
                                 ptr<ulonglong2>(out), nullptr);
        return out;
      },
      py::arg("rids"), py::arg("rid_offset"), py::arg("payload"), py::arg("mode") = -1);
  ops.def(
      "project_keys",
      [](const at::Tensor &tuples, uint32_t shift, int ipt) {
        // [n, 2] int64 tuples -> [n] int32 (key >> shift): the count-only network pass's byte mix, no partitioning
        TORCH_CHECK(tuples.is_cuda() && tuples.dim() == 2 && tuples.size(1) == 2 && tuples.is_contiguous(),
                    "project_keys: device [n, 2] int64 tuples");
        at::Tensor out = at::empty({tuples.size(0)}, tuples.options().dtype(at::kInt));
        kernels::projectKeys(ptr<const ulonglong2>(tuples), (uint64_t)tuples.size(0), shift, ptr<uint32_t>(out), ipt,
                             nullptr);
        return out;
      },
      py::arg("tuples"), py::arg("shift") = 10, py::arg("ipt") = 8);
  ops.def(
      "probe_bitmap_global",
      [](const at::Tensor &tuples, const at::Tensor &bitmap, uint64_t keyMask, int ipt) {
        // Count tuples whose key bit is set in a global bitmap (microbenchmark of a whole-key-space probe)
        TORCH_CHECK(tuples.is_cuda() && bitmap.is_cuda() && tuples.dim() == 2 && tuples.size(1) == 2 &&
                        bitmap.scalar_type() == at::kInt && bitmap.is_contiguous(),
                    "probe_bitmap_global: device [n, 2] int64 tuples and an int32 bitmap");
        TORCH_CHECK((uint64_t)bitmap.numel() * 32 > keyMask, "probe_bitmap_global: bitmap smaller than the key mask");
        at::Tensor cnt = at::zeros({1}, tuples.options());
        kernels::probeBitmapGlobal(ptr<const ulonglong2>(tuples), (uint64_t)tuples.size(0), ptr<uint32_t>(bitmap),
                                   keyMask, reinterpret_cast<unsigned long long *>(cnt.data_ptr()), ipt, nullptr);
        return cnt;
      },
      py::arg("tuples"), py::arg("bitmap"), py::arg("key_mask"), py::arg("ipt") = 8);
  ops.def("copy_into", [](const at::Tensor &src, const at::Tensor &dst) {
    setDevice(src);
    HJ_CHECK(dst.numel() * dst.element_size() >= src.numel() * src.element_size(), "copy_into: dst too small");
    kernels::copyKernel(ptr<const ulonglong2>(src), ptr<ulonglong2>(dst), src.numel() * src.element_size() / 16, nullptr);
  });
  ops.def(
      "stream_mix",
      [](uint64_t n, int ra, int rb, int wa, int wb, const at::Tensor &a, const at::Tensor &b, const at::Tensor &oa,
         const at::Tensor &ob, const at::Tensor &sink) {
        // One in-order pass over n elements with the given byte mix (stream-mix ceiling of a pass)
        setDevice(a);
        auto need = [&](const at::Tensor &t, int bytes, const char *what) {
          if (bytes) HJ_CHECK(t.is_cuda() && (uint64_t)(t.numel() * t.element_size()) >= n * bytes,
                              "stream_mix: %s holds fewer than n x %d bytes", what, bytes);
        };
        need(a, ra, "a");
        need(b, rb, "b");
        need(oa, wa, "oa");
        need(ob, wb, "ob");
        HJ_CHECK(n % 512 == 0, "stream_mix: n must be a multiple of 512");
        kernels::streamMix(ra, rb, wa, wb, a.data_ptr(), b.data_ptr(), oa.data_ptr(), ob.data_ptr(), n,
                           reinterpret_cast<unsigned long long *>(sink.data_ptr()), nullptr);
      },
      py::arg("n"), py::arg("ra"), py::arg("rb"), py::arg("wa"), py::arg("wb"), py::arg("a"), py::arg("b"),
      py::arg("oa"), py::arg("ob"), py::arg("sink"));
  ops.def("read_sink", [](const at::Tensor &src, const at::Tensor &sink) {
    setDevice(src);
    kernels::readKernel(ptr<const ulonglong2>(src), src.numel() * src.element_size() / 16,
                        ptr<unsigned long long>(sink), nullptr);
  });
  ops.def("bench_host_link", &benchHostLink, py::arg("bytes") = (uint64_t)1 << 30, py::arg("device") = 0,
          py::arg("iters") = 5);
  ops.def("bench_scatter_ms", &benchScatter, py::arg("tuples"), py::arg("bits"), py::arg("mode") = 0,
          py::arg("iters") = 10, py::arg("max_blocks") = 2048, py::arg("geometry") = 0, py::arg("round_lp") = 6);
  ops.def("bench_histogram_ms", &benchHistogram, py::arg("tuples"), py::arg("bits"), py::arg("iters") = 10);
  ops.def("partition_tile", []() { return kernels::PART_TILE; });
  // Round-interleaved window slots (kernels::RoundMap), for the layout tests.
  ops.def(
      "round_slot",
      [](uint64_t logical, uint32_t lp, uint32_t lv, uint32_t lns) {
        kernels::RoundMap m;
        m.lp = lp;
        m.lv = lv;
        m.lns = lns;
        return m(logical);
      },
      py::arg("logical"), py::arg("lp"), py::arg("lv"), py::arg("lns"));
  ops.def("round_slots", &kernels::roundSlots, py::arg("max_cap"), py::arg("lp"), py::arg("lns"));
}
