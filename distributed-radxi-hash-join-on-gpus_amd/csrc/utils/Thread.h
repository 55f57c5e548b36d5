// Thread pinning helper (reference: /root/reference/utils/Thread.h:15-20, never
// called there).  Here it is used by the host reference path and by the
// standalone CLI to pin the rank's host thread next to its GPU.
#pragma once

#include <cstdint>

namespace hpcjoin {
namespace utils {

class Thread {
 public:
  static bool pin(uint32_t coreId);
  static int currentCore();
};

}  // namespace utils
}  // namespace hpcjoin
