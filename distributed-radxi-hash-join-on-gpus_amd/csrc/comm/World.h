// Process-wide default communicator used by the reference-compatible
// constructors that take no communicator (e.g. GlobalHistogram(LocalHistogram*)).
#pragma once

#include "Communicator.h"

namespace hpcjoin {
namespace comm {

Communicator *world();             // LocalCommunicator unless set
void setWorld(Communicator *comm);  // not owned

}  // namespace comm
}  // namespace hpcjoin
