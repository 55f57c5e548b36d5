#include "Debug.h"

#include <cstdarg>
#include <cstring>
#include <unistd.h>

namespace hpcjoin {
namespace utils {

static thread_local int g_rank = 0;
int debugRank() { return g_rank; }
void setDebugRank(int r) { g_rank = r; }

bool debugEnabled() {
#ifdef JOIN_DEBUG_PRINT
  return true;
#else
  // Magic static: initialised once, thread-safe (in-process ranks are threads;
  // the earlier lazily written int was a data race found by the TSan build).
  static const bool enabled = [] {
    const char *e = std::getenv("HPCJOIN_DEBUG");
    return e && e[0] && std::strcmp(e, "0") != 0;
  }();
  return enabled;
#endif
}

std::string format(const char *fmt, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return std::string(buf);
}

void fail(const char *tag, const char *file, int line, const std::string &msg) {
  std::string m = format("[%s][rank %d] %s (%s:%d)", tag, g_rank, msg.c_str(), file, line);
  throw std::runtime_error(m);
}

unsigned long vmSizeBytes() {
  unsigned long pages = 0;
  FILE *f = std::fopen("/proc/self/statm", "r");
  if (f) {
    if (std::fscanf(f, "%lu", &pages) != 1) pages = 0;
    std::fclose(f);
  }
  return pages * (unsigned long)sysconf(_SC_PAGESIZE);
}

}  // namespace utils
}  // namespace hpcjoin
