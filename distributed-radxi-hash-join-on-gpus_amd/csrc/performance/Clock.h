#pragma once

#include <chrono>
#include <cstdint>

namespace hpcjoin {
namespace performance {

inline uint64_t nowUs() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace performance
}  // namespace hpcjoin
