// Logging / assertion macros with the reference names (/root/reference/utils/Debug.h:16-60).
// Differences: JOIN_ASSERT throws (so Python callers and tests see the failure
// with rank + site) instead of exit(-1), and HJ_CHECK is an always-on cheap
// invariant check used for the "all tuples written" style checks of SURVEY §4.5.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace hpcjoin {
namespace utils {

int debugRank();            // rank used in messages (set by the communicator)
void setDebugRank(int r);
bool debugEnabled();        // HPCJOIN_DEBUG=1 in the environment or JOIN_DEBUG_PRINT at build time

[[noreturn]] void fail(const char *tag, const char *file, int line, const std::string &msg);
std::string format(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
unsigned long vmSizeBytes();  // /proc/self/statm (JOIN_MEM_DEBUG analog)

}  // namespace utils
}  // namespace hpcjoin

#define JOIN_DEBUG(tag, ...)                                                                 \
  do {                                                                                       \
    if (::hpcjoin::utils::debugEnabled()) {                                                  \
      std::fprintf(stdout, "[%s][%d] %s\n", tag, ::hpcjoin::utils::debugRank(),              \
                   ::hpcjoin::utils::format(__VA_ARGS__).c_str());                           \
      std::fflush(stdout);                                                                   \
    }                                                                                        \
  } while (0)

#define JOIN_ASSERT(cond, tag, ...)                                                          \
  do {                                                                                       \
    if (!(cond)) ::hpcjoin::utils::fail(tag, __FILE__, __LINE__, ::hpcjoin::utils::format(__VA_ARGS__)); \
  } while (0)

#define JOIN_MEM_DEBUG(msg)                                                                  \
  do {                                                                                       \
    if (::hpcjoin::utils::debugEnabled())                                                    \
      std::fprintf(stdout, "[MEMORY][%s] %lu bytes\n", msg, ::hpcjoin::utils::vmSizeBytes()); \
  } while (0)

#define HJ_CHECK(cond, ...) JOIN_ASSERT(cond, "CHECK", __VA_ARGS__)
