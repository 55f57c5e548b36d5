#include "World.h"

namespace hpcjoin {
namespace comm {

static LocalCommunicator g_local;
static Communicator *g_world = nullptr;

Communicator *world() { return g_world ? g_world : &g_local; }
void setWorld(Communicator *comm) { g_world = comm; }

}  // namespace comm
}  // namespace hpcjoin
