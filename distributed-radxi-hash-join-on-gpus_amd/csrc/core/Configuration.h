// Compile-time defaults.  Same class name, member names and values as the
// reference (/root/reference/core/Configuration.h:15-40) so code written
// against hpcjoin::core::Configuration keeps compiling.  On MI355X these are
// only *defaults*: the runtime JoinConfig (core/JoinConfig.h) derives the real
// fan-outs from the relation sizes and the 160 KiB LDS / 288 GB HBM budget.
#pragma once

#include <cstdint>

namespace hpcjoin {
namespace core {

class Configuration {
 public:
  static const uint32_t RESULT_AGGREGATION_NODE = 0;

  // Host (reference) write-combining geometry (NetworkPartitioning.cpp:82-110).
  static const uint32_t CACHELINE_SIZE_BYTES = 64;
  static const uint32_t CACHELINES_PER_MEMORY_BUFFER = 1024;
  static const uint32_t MEMORY_BUFFERS_PER_PARTITION = 2;
  static const uint64_t MEMORY_BUFFER_SIZE_BYTES = CACHELINES_PER_MEMORY_BUFFER * CACHELINE_SIZE_BYTES;
  static const uint64_t MEMORY_PARTITION_SIZE_BYTES = MEMORY_BUFFERS_PER_PARTITION * MEMORY_BUFFER_SIZE_BYTES;

  // The reference ships with the second pass disabled (Configuration.h:28);
  // on the GPU the second (LDS-sized) pass is what makes build/probe fit LDS,
  // so JoinConfig enables it by default and this constant only seeds the
  // host reference path.
  static const bool ENABLE_TWO_LEVEL_PARTITIONING = false;

  static const uint64_t NETWORK_PARTITIONING_FANOUT = 5;
  static const uint64_t LOCAL_PARTITIONING_FANOUT = 5;
  static const uint64_t NETWORK_PARTITIONING_COUNT = (1 << NETWORK_PARTITIONING_FANOUT);
  static const uint64_t LOCAL_PARTITIONING_COUNT = (1 << LOCAL_PARTITIONING_FANOUT);

  static constexpr double ALLOCATION_FACTOR = 1.1;

  static const uint32_t PAYLOAD_BITS = 27;

  // --- MI355X (gfx950) device geometry used by the kernels -----------------
  static const uint32_t GPU_WAVE_SIZE = 64;
  static const uint32_t GPU_CU_COUNT = 256;
  static const uint32_t GPU_XCD_COUNT = 8;
  static const uint32_t GPU_LDS_BYTES = 160 * 1024;
  static const uint32_t GPU_L2_LINE_BYTES = 128;
  static const uint32_t GPU_MAX_FANOUT_BITS = 11;  // per radix pass (LDS histogram / cursors)
};

}  // namespace core
}  // namespace hpcjoin
