// Content verification of a join's exchange (JoinConfig::verifyExchange).
//
// The reference checks an exchange by counts only (Window::
// assertAllTuplesWritten, /root/reference/data/Window.cpp:180-191, and the
// per-partition write counters of Window::write, :121-124): a put that lands
// at a wrong offset, in a freed or unmapped window, or never, is silent.  Here
// every sender hashes its input per (exchange chunk, partition) and every
// receiver hashes what arrived in its window per (source, chunk, partition)
// segment (kernels::exchangeHash of the mixed key and, where it travels, the
// rid).  After one all-gather and one all-reduce every rank holds both tables
// and checks received == sent x copies for every (source, chunk, partition),
// copies = the ranks the assignment sends that run to (1, or the helpers of a
// split partition's replicated side) -- so all ranks reach the same verdict
// and either all continue or all throw.
#pragma once

#include "JoinStrategies.h"

namespace hpcjoin {
namespace operators {

struct ExchangeCheck {
  uint64_t cells = 0;       // (source, chunk, partition, side) entries compared
  uint64_t mismatches = 0;
};

// Collective.  Both windows must be complete on this rank (stop()); throws
// (every rank) on a mismatch.
ExchangeCheck verifyExchange(JoinEnv &env, JoinRun &run);

}  // namespace operators
}  // namespace hpcjoin
