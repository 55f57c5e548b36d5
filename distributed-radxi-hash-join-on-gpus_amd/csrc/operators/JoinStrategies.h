// The per-plan pieces of HashJoin::run() (reference: the phase sequence of
// operators/HashJoin.cpp:45-220).  A join is
//   exchange   histogram -> windows -> network partitioning, one strategy per plan:
//                SampledSingleRankExchange  N == 1, sampled histogram, bounded claim scatter
//                SampledShuffleExchange     N > 1, sampled histogram, exact fills gathered per relation
//                SplitHistogramExchange     N > 1, outer histogram behind the inner exchange
//                ExactExchange              exact histograms, then windows and the chunked exchange
//   local      second radix pass + build/probe (LocalPhase; pipelined per outer chunk at N > 1)
// and, for count-only joins of unique dense keys, BitmapPlan replaces both.
// Every strategy shares the JoinRun state, the timeline events and the
// Measurements hooks of the join (JoinEnv).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "../core/ExecContext.h"
#include "../core/JoinConfig.h"
#include "../data/Relation.h"
#include "../data/Window.h"
#include "../kernels/kernels.h"
#include "../performance/Trace.h"
#include "../tasks/BuildProbe.h"
#include "../tasks/HistogramComputation.h"
#include "../tasks/LocalPartitioning.h"
#include "../tasks/SampledNetworkPartitioning.h"
#include "../tasks/SampledShuffle.h"

namespace hpcjoin {
namespace operators {

struct JoinResult;

// What every strategy of one HashJoin reads: the engine, the plan, both
// relations and the join's five timing events (ev[0] = join start).
struct JoinEnv {
  core::ExecContext *ctx;
  const core::JoinConfig &config;
  core::JoinPlan &plan;
  data::Relation *inner;
  data::Relation *outer;
  hipEvent_t *ev;
  uint32_t nodes, nodeId;
};

// State of one run() shared by the exchange strategy and the local phase.
struct JoinRun {
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;  // host clock: start, histogram done, windows done, network done
  std::unique_ptr<performance::TraceRange> trace;
  std::unique_ptr<tasks::HistogramComputation> hc;
  std::unique_ptr<tasks::SampledNetworkPartitioning> sp;
  std::unique_ptr<tasks::SampledShuffle> ss;  // N > 1 sampled pass (owns its windows' plans)
  std::unique_ptr<data::Window> innerOwned, outerOwned;
  data::Window *inner = nullptr, *outer = nullptr;
  // Local pass: created by the exchange when it starts the inner side early.
  std::unique_ptr<tasks::LocalPartitioning> lp;
  bool networkEventRecorded = false;  // ev[2] already recorded by the exchange
  bool sampled = false;               // the single-rank sampled pass produced the windows
  // Pops the current roctx range (ranges nest) and opens `name`.
  void phase(const char *name);
};

class ExchangeStrategy {
 public:
  explicit ExchangeStrategy(JoinEnv &env) : env(env) {}
  virtual ~ExchangeStrategy() = default;
  virtual const char *name() const = 0;
  // Leaves run.inner / run.outer set; false = a sampled slice overflowed (the
  // caller re-runs the join with ExactExchange and keeps using it).
  virtual bool exchange(JoinRun &run) = 0;

 protected:
  JoinEnv &env;
  std::unique_ptr<data::Window> makeWindow(tasks::HistogramComputation &hc, int side) const;
};

// N == 1: sampled histogram, bounded claim scatter, the inner local pass
// started while the outer scatter still runs (tasks/SampledNetworkPartitioning).
class SampledSingleRankExchange : public ExchangeStrategy {
 public:
  SampledSingleRankExchange(JoinEnv &env, bool localExact) : ExchangeStrategy(env), localExact(localExact) {}
  const char *name() const override { return "sampled_single_rank"; }
  bool exchange(JoinRun &run) override;

 private:
  bool localExact;
};

// N > 1, sampled: estimates instead of the exact pre-read, bounded claim
// slices, exact fills all-gathered per relation and packed runs on the wire
// (tasks/SampledShuffle).  false = a slice or window would overflow on some
// rank (every rank agrees; the caller re-runs with ExactExchange).
class SampledShuffleExchange : public ExchangeStrategy {
 public:
  using ExchangeStrategy::ExchangeStrategy;
  const char *name() const override { return "sampled_shuffle"; }
  bool exchange(JoinRun &run) override;
};

// N > 1: the inner relation's exact histogram heads the join; the outer
// histogram's all-gather runs on the exchange stream behind the inner exchange.
class SplitHistogramExchange : public ExchangeStrategy {
 public:
  using ExchangeStrategy::ExchangeStrategy;
  const char *name() const override { return "split_histogram"; }
  bool exchange(JoinRun &run) override;
};

// Exact histograms of both relations, then windows and the chunked exchange
// (the reference's sequence; also the fallback of the sampled pass).
class ExactExchange : public ExchangeStrategy {
 public:
  // afterSampledOverflow: the measurement spans were opened by the failed
  // sampled pass (they are not restarted).
  ExactExchange(JoinEnv &env, bool afterSampledOverflow) : ExchangeStrategy(env), retry(afterSampledOverflow) {}
  const char *name() const override { return "exact"; }
  bool exchange(JoinRun &run) override;

 private:
  bool retry;
};

// Local phase: second radix pass and build/probe over the windows, with the
// sampled pass's exact re-run and the build/probe overflow re-runs.
class LocalPhase {
 public:
  LocalPhase(JoinEnv &env, bool &localOverflowed, const kernels::RowSink *sink)
      : env(env), localOverflowed(localOverflowed), sink(sink) {}
  // Runs to completion (all streams synchronised); fills the counts of `r`.
  void run(JoinRun &run, JoinResult &r);
  std::vector<std::unique_ptr<tasks::BuildProbe>> &buildProbes() { return bps; }
  void release() {
    bps.clear();
    outerViews.clear();
  }

 private:
  tasks::BuildProbe *addBuildProbe(data::Window *inner, data::Window *outer);
  JoinEnv &env;
  bool &localOverflowed;
  const kernels::RowSink *sink;  // fused row output (N = 1 materializing joins), or null
  std::vector<std::unique_ptr<tasks::BuildProbe>> bps;
  std::vector<std::unique_ptr<data::Window>> outerViews;
};

// Count-only single-level bitmap join (tasks/BitmapJoin): N == 1 LDS bitmaps,
// N > 1 replicated bitmaps combined by one RCCL all-reduce.
class BitmapPlan {
 public:
  BitmapPlan(JoinEnv &env, bool &exact) : env(env), exact(exact) {}
  // false: a repeated inner key (the caller continues on the two-level plan).
  bool run(uint64_t t0, JoinResult &r);

 private:
  JoinEnv &env;
  bool &exact;  // sticky: exact histograms (small inputs, or after an overflow)
};

}  // namespace operators
}  // namespace hpcjoin
