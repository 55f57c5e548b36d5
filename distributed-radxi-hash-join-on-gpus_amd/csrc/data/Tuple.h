// 16-byte row {key, rid}: layout-identical to /root/reference/data/Tuple.h:15-22.
#pragma once

#include <cstdint>

namespace hpcjoin {
namespace data {

class Tuple {
 public:
  uint64_t key;
  uint64_t rid;
};

static_assert(sizeof(Tuple) == 16, "Tuple must stay 16 bytes (source compatibility)");

}  // namespace data
}  // namespace hpcjoin
