#include "Fault.h"

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../comm/Communicator.h"
#include "Hip.h"

namespace hpcjoin {
namespace utils {

namespace {
thread_local std::string t_phase;
thread_local int t_rank = -1;
thread_local bool t_armed = false;
std::atomic<uint64_t> g_timeoutMs{0};
// Watchdog context of this rank.
thread_local const char *t_current = "setup";
thread_local const char *t_lastDone = nullptr;
thread_local const char *t_lastQueued = nullptr;
thread_local uint64_t t_doneCount = 0, t_queuedCount = 0;
thread_local comm::Communicator *t_watchComm = nullptr;
thread_local bool t_stalled = false;

bool envMatch(const char *var, const char *phase) {
  const char *e = std::getenv(var);
  if (!e || !e[0]) return false;
  const char *colon = std::strchr(e, ':');
  const size_t n = colon ? (size_t)(colon - e) : std::strlen(e);
  if (std::strlen(phase) != n || std::strncmp(e, phase, n) != 0) return false;
  return !colon || std::atoi(colon + 1) == debugRank();
}
}  // namespace

void armFault(const std::string &phase, int rank) {
  t_phase = phase;
  t_rank = rank;
  t_armed = !phase.empty();
}

bool faultHit(const char *phase) {
  const bool hit =
      (t_armed && t_phase == phase && (t_rank < 0 || t_rank == debugRank())) || envMatch("HPCJOIN_FAULT", phase);
  if (hit) t_armed = false;  // one shot
  return hit;
}

template <typename Query>
static void waitUntil(Query query, comm::Communicator *comm, const char *what);

void faultPoint(const char *phase) {
  setPhase(phase);
  if (faultHit(phase))
    throw InjectedFault(format("[FAULT][rank %d] injected fault at phase '%s'", debugRank(), phase));
  if (!t_stalled && envMatch("HPCJOIN_STALL", phase)) {
    t_stalled = true;  // one shot per rank
    const std::string what = format("injected stall at phase '%s'", phase);
    waitUntil([] { return hipErrorNotReady; }, t_watchComm, what.c_str());
  }
}

void setPhase(const char *phase) { t_current = phase; }

void noteCollective(const char *name, bool completed) {
  if (completed) {
    t_lastDone = name;
    ++t_doneCount;
  } else {
    t_lastQueued = name;
    ++t_queuedCount;
  }
}

std::string watchdogContext() {
  std::string s = format("phase '%s', last completed collective ", t_current);
  s += t_lastDone ? format("%s #%lu", t_lastDone, (unsigned long)t_doneCount) : std::string("none");
  if (t_lastQueued) s += format(", last enqueued %s #%lu", t_lastQueued, (unsigned long)t_queuedCount);
  return s;
}

void setWatchComm(comm::Communicator *comm) { t_watchComm = comm; }

uint64_t commTimeoutMs() {
  uint64_t v = g_timeoutMs.load(std::memory_order_relaxed);
  if (v) return v;
  const char *e = std::getenv("HPCJOIN_COMM_TIMEOUT_S");
  v = (e && e[0]) ? (uint64_t)(std::atof(e) * 1000.0) : 600000;
  return v ? v : 1;
}

void setCommTimeoutMs(uint64_t ms) { g_timeoutMs.store(ms, std::memory_order_relaxed); }

template <typename Query>
static void waitUntil(Query query, comm::Communicator *comm, const char *what) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const auto deadline = t0 + std::chrono::milliseconds(commTimeoutMs());
  for (uint64_t spin = 0;; ++spin) {
    hipError_t e = query();
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    if (comm) comm->checkHealth();
    const auto now = clk::now();
    if (now > deadline) {
      std::string why = format("%s did not complete within %lu ms (%s)", what, (unsigned long)commTimeoutMs(),
                               watchdogContext().c_str());
      if (comm) comm->abort(why);
      fail("WATCHDOG", __FILE__, __LINE__, why);
    }
    // Yield-spin for the first 100 ms (a join's waits end within
    // microseconds of its last kernel; a sleep would add its granularity to
    // every join), then back off so a stuck collective does not burn a core.
    (void)spin;
    if (now - t0 < std::chrono::milliseconds(100)) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void waitStream(hipStream_t stream, comm::Communicator *comm, const char *what) {
  waitUntil([stream] { return hipStreamQuery(stream); }, comm, what);
}

void waitEvent(hipEvent_t event, comm::Communicator *comm, const char *what) {
  waitUntil([event] { return hipEventQuery(event); }, comm, what);
}

}  // namespace utils
}  // namespace hpcjoin
