// Failure detection and fault injection (the reference has none --
// MPI errors are fatal and most CUDA errors unchecked).
//
// * faultPoint(phase): deterministic fault injection.  A fault is armed either
//   programmatically per thread (in-process ranks are threads) or through
//   HPCJOIN_FAULT="<phase>[:<rank>]" in the environment; the armed rank throws
//   InjectedFault when it reaches that phase.  Tests use it to prove that a
//   failing rank does not hang its peers.
// * HPCJOIN_STALL="<phase>[:<rank>]": the armed rank stops making progress at
//   that phase (a wait that never completes, as a hung kernel or a lost peer
//   would leave it).  Its own watchdog and every peer's must then end the run.
// * commTimeoutMs(): deadline for every blocking wait on communication
//   (HPCJOIN_COMM_TIMEOUT_S, default 600 s).  Waits poll the communicator's
//   health (RCCL async errors, aborted in-process groups) and give up with an
//   exception instead of hanging forever.  The exception names the rank, the
//   join phase it was in, the wait site and the last collective the rank
//   completed (watchdogContext): on a real multi-GPU run every rank's message
//   says where it stopped.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace hpcjoin {
namespace comm {
class Communicator;
}
namespace utils {

struct InjectedFault : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Arm a fault for the calling thread (rank < 0: any rank). Empty phase disarms.
void armFault(const std::string &phase, int rank = -1);
void faultPoint(const char *phase);
// Non-throwing variant: true (once) when a fault is armed for this phase --
// the caller injects it (e.g. "corrupt_window": flip a word of a window).
bool faultHit(const char *phase);

uint64_t commTimeoutMs();
void setCommTimeoutMs(uint64_t ms);  // process-wide override (tests)

// Per rank (thread: in-process ranks are threads) diagnostic state for the
// watchdog.  faultPoint() records the phase; communicators record every
// collective they complete on the host (and the last one they enqueue on a
// stream).  watchdogContext() formats it: "phase 'network', last completed
// collective ncclAllGather #7, last enqueued ncclSend/Recv (all-to-allv) #3".
void setPhase(const char *phase);
void noteCollective(const char *name, bool completed);
std::string watchdogContext();
// Communicator a stall injected by HPCJOIN_STALL waits on (HashJoin::run sets
// it for its duration; null: the stall waits without health polling).
void setWatchComm(comm::Communicator *comm);

// Wait until `stream` is idle.  Polls comm->checkHealth() and throws after
// commTimeoutMs() (after aborting the communicator so peers fail fast, too).
void waitStream(hipStream_t stream, comm::Communicator *comm, const char *what);
// Same for one event (work queued behind it on its stream is not waited for).
void waitEvent(hipEvent_t event, comm::Communicator *comm, const char *what);

}  // namespace utils
}  // namespace hpcjoin
