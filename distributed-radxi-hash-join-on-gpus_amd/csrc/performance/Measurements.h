// Timers, counters and reporting.  Keeps the reference's phase structure and
// output keys (/root/reference/performance/Measurements.cpp: JTOTAL, JHIST,
// JMPI, JPROC, SWINALLOC, SNETCOMPL, SLOCPREP, HILOCAL, ..., BPPROBEELEM in
// <rank>.perf; NUMNODES, NODEID, HOST, GISZ, ... in <rank>.info; the rank-0
// "[RESULTS]" table) so runs stay comparable, and adds device-side phase
// times from hipEvents (D* keys) and a JSON-friendly key/value dump.
// Differences: std::chrono instead of gettimeofday, no PAPI (not in this
// image), aggregation through the engine communicator instead of MPI_Send.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace hpcjoin {
namespace comm {
class Communicator;
}
namespace performance {

class Measurements {
 public:
  static void init(uint32_t nodeId, uint32_t numberOfNodes, const std::string &tag, const std::string &directory = "");
  static void writeMetaData(const char *key, const char *value);
  static void writeMetaData(const char *key, uint64_t value);

  static void startJoin();
  static void stopJoin();
  static void startHistogramComputation();
  static void stopHistogramComputation();
  static void startWindowAllocation();
  static void stopWindowAllocation();
  static void startNetworkPartitioning();
  static void stopNetworkPartitioning();
  static void startWaitingForNetworkCompletion();
  static void stopWaitingForNetworkCompletion();
  static void startLocalProcessingPreparations();
  static void stopLocalProcessingPreparations();
  static void startLocalProcessing();
  static void stopLocalProcessing();

  static void storeHistogramDetails(uint64_t localUs, uint64_t innerElements, uint64_t outerElements,
                                    uint64_t globalUs, uint64_t assignUs, uint64_t offsetUs);
  static void storeNetworkDetails(uint64_t innerElements, uint64_t outerElements, uint64_t chunks);
  static void storeLocalPartitioningDetails(uint64_t elements, uint64_t items);
  static void storeBuildProbeDetails(uint64_t buildElements, uint64_t probeElements, uint64_t items);
  static void storeDevicePhase(const std::string &key, double ms);  // DHIST, DNET, DLOCPART, DBP
  static void storeResultTuples(uint64_t tuples);

  // 10 values per rank, reference order: tuples, join, histogram, network,
  // local, winalloc, partwait, localprep, localpart, localbp (µs).
  static std::vector<uint64_t> serializeResults();
  static void printMeasurements(comm::Communicator *comm);  // gathers to everyone, rank 0 prints
  static void storeAllMeasurements();                     // <dir>/<rank>.perf when a directory was given
  static std::map<std::string, double> snapshot();        // everything, for Python / JSON

  static uint64_t joinUs();

  // Detailed keys (sub-phases, counts, bytes): set / accumulate into this
  // join's table.  Every reference key exists from startJoin() on (0 when a
  // plan has no such step), so reports always carry the full key set.
  static void put(const std::string &key, double v, const char *unit);
  static void add(const std::string &key, double v, const char *unit);
  static const std::vector<std::string> &referenceKeys();
};

}  // namespace performance
}  // namespace hpcjoin
