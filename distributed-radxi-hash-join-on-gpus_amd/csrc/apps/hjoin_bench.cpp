// Standalone driver: the analog of the reference's `program`
// (/root/reference/main.cpp:28-149) without MPI or Python.
//
//   hjoin_bench [--inner N] [--outer N] [--dist unique|modulo|uniform|zipf]
//               [--theta T] [--device D] [--host] [--iters K] [--warmup W]
//               [--rank R --world W --id-file PATH]   (one process per GPU; rank 0
//                                                      writes the ncclUniqueId to PATH)
//               [--chunks C] [--net-bits B] [--local-bits B] [--materialize] [--wide]
//               [--round-robin] [--perf-dir DIR]
// Default workload per rank: 20M x 20M unique keys, as in main.cpp:70-71.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../comm/RcclCommunicator.h"
#include "../comm/World.h"
#include "../core/ExecContext.h"
#include "../data/Relation.h"
#include "../operators/HashJoin.h"
#include "../performance/Measurements.h"
#include "../utils/Hip.h"

using namespace hpcjoin;

int main(int argc, char **argv) {
  uint32_t rank = 0, world = 1;
  int device = -1;
  std::string idFile = "/tmp/hjoin_bench.id", dist = "unique", perfDir;
  uint64_t inner = 0, outer = 0;
  double theta = 0.75;
  int iters = 5, warmup = 1;
  bool host = false;
  core::JoinConfig cfg;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--inner") inner = std::stoull(next());
    else if (a == "--outer") outer = std::stoull(next());
    else if (a == "--dist") dist = next();
    else if (a == "--theta") theta = std::stod(next());
    else if (a == "--device") device = std::stoi(next());
    else if (a == "--host") host = true;
    else if (a == "--iters") iters = std::stoi(next());
    else if (a == "--warmup") warmup = std::stoi(next());
    else if (a == "--rank") rank = std::stoul(next());
    else if (a == "--world") world = std::stoul(next());
    else if (a == "--id-file") idFile = next();
    else if (a == "--chunks") cfg.chunks = std::stoul(next());
    else if (a == "--net-bits") cfg.networkBits = std::stoul(next());
    else if (a == "--local-bits") cfg.localBits = std::stoul(next());
    else if (a == "--materialize") cfg.materialize = true;
    else if (a == "--wide") cfg.format = core::TupleFormat::Wide;
    else if (a == "--round-robin") cfg.assignment = core::AssignmentPolicy::RoundRobin;
    else if (a == "--two-level-only") cfg.bitmapJoin = false;  // no single-level bitmap join (N == 1)
    else if (a == "--perf-dir") perfDir = next();
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (!inner) inner = (uint64_t)world * 20000000ull;
  if (!outer) outer = inner;
  if (device < 0) device = (int)rank;

  std::unique_ptr<comm::Communicator> comm;
  if (world == 1 || host) {
    comm.reset(new comm::LocalCommunicator());
    world = 1;
    rank = 0;
  } else {
    std::vector<uint8_t> id;
    if (rank == 0) {
      id = comm::RcclCommunicator::uniqueId();
      std::string tmp = idFile + ".tmp";
      std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char *>(id.data()), id.size());
      std::rename(tmp.c_str(), idFile.c_str());
    } else {
      for (int t = 0; t < 600; ++t) {
        std::ifstream f(idFile, std::ios::binary);
        id.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
        if (id.size() == comm::RcclCommunicator::UNIQUE_ID_BYTES) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
      }
    }
    comm.reset(new comm::RcclCommunicator(id, rank, world, device));
  }
  comm::setWorld(comm.get());
  const Location loc = host ? Location::Host : Location::Device;

  performance::Measurements::init(rank, world, "experiment", perfDir);
  performance::Measurements::writeMetaData("GISZ", inner);
  performance::Measurements::writeMetaData("GOSZ", outer);

  data::GenSpec is, os;
  is.seed = 1234;
  os.seed = 4321;
  if (dist == "unique") {
  } else if (dist == "modulo") {
    os.distribution = kernels::KeyDistribution::Modulo;
    os.domain = inner;
  } else if (dist == "uniform") {
    os.distribution = kernels::KeyDistribution::Uniform;
    os.domain = inner;
  } else if (dist == "zipf") {
    os.distribution = kernels::KeyDistribution::Zipf;
    os.domain = inner;
    os.zipfTheta = theta;
  } else {
    std::fprintf(stderr, "unknown --dist %s\n", dist.c_str());
    return 2;
  }
  const uint64_t li = data::Relation::localSizeFor(inner, rank, world);
  const uint64_t lo = data::Relation::localSizeFor(outer, rank, world);
  performance::Measurements::writeMetaData("LISZ", li);
  performance::Measurements::writeMetaData("LOSZ", lo);
  data::Relation R(li, inner, loc, device), S(lo, outer, loc, device);
  R.generate(is, data::Relation::localOffsetFor(inner, rank, world));
  S.generate(os, data::Relation::localOffsetFor(outer, rank, world));
  const uint64_t expected = data::Relation::expectedMatches(is, inner, os, outer);

  core::ExecContext ctx(loc, device, comm.get());
  operators::HashJoin join(&R, &S, &ctx, cfg);
  if (rank == 0) std::printf("[INFO] %s\n", join.getPlan().describe().c_str());
  for (int w = 0; w < warmup; ++w) join.run();
  ctx.resetScratch();  // grow the arena to the warmup peak before timing
  std::vector<double> times;
  uint64_t matches = 0;
  for (int it = 0; it < iters; ++it) {
    comm->barrier();
    operators::JoinResult r = join.run();
    std::vector<uint64_t> mine{(uint64_t)(r.joinMs * 1000.0)}, all(world);
    comm->allGatherHost(mine.data(), all.data(), 1);
    times.push_back(*std::max_element(all.begin(), all.end()) / 1000.0);
    matches = r.globalMatches;
  }
  performance::Measurements::printMeasurements(comm.get());
  performance::Measurements::storeAllMeasurements();
  std::sort(times.begin(), times.end());
  const double med = times.empty() ? 0 : times[times.size() / 2];
  if (rank == 0) {
    std::printf("{\"metric\": \"join_throughput\", \"value\": %.4f, \"unit\": \"billion tuples/s\", \"n_gpus\": %u, "
                "\"ms_per_join\": %.3f, \"matches\": %lu, \"expected\": %s%lu, \"correct\": %s}\n",
                med > 0 ? (inner + outer) / (med * 1e6) : 0.0, world, med, (unsigned long)matches,
                expected == UINT64_MAX ? "-" : "", (unsigned long)(expected == UINT64_MAX ? 0 : expected),
                (expected == UINT64_MAX || expected == matches) ? "true" : "false");
  }
  return (expected == UINT64_MAX || expected == matches) ? 0 : 1;
}
