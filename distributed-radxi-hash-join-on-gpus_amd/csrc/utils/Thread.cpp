#include "Thread.h"

#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <pthread.h>
#include <sched.h>

namespace hpcjoin {
namespace utils {

bool Thread::pin(uint32_t coreId) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(coreId, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

int Thread::currentCore() { return sched_getcpu(); }

}  // namespace utils
}  // namespace hpcjoin
