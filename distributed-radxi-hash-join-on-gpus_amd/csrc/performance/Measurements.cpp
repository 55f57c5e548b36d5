#include "Measurements.h"

#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <mutex>

#include "../comm/Communicator.h"
#include "Clock.h"

namespace hpcjoin {
namespace performance {

namespace {
struct State {
  uint32_t nodeId = 0, numberOfNodes = 1;
  std::string tag = "experiment", dir;
  std::map<std::string, std::string> meta;
  std::map<std::string, std::pair<double, std::string>> values;
  uint64_t joinStart = 0, joinStop = 0, cycleStart = 0;
  uint64_t phaseStart[8] = {0};
  uint64_t phaseTime[8] = {0};
  uint64_t tuples = 0;
};
State &st() {
  static thread_local State s;  // one per rank thread (in-process ranks)
  return s;
}
enum Phase { HIST = 0, WINALLOC, NET, NETWAIT, LOCPREP, LOCAL, NPHASE };
void begin(int p) { st().phaseStart[p] = nowUs(); }
void end(int p) { st().phaseTime[p] = nowUs() - st().phaseStart[p]; }
}  // namespace

void Measurements::put(const std::string &key, double v, const char *unit) { st().values[key] = {v, unit}; }
void Measurements::add(const std::string &key, double v, const char *unit) {
  auto &e = st().values[key];
  e.first += v;
  e.second = unit;
}

// The reference's .perf keys (performance/Measurements.cpp:136-542) and units.
static const std::vector<std::pair<std::string, const char *>> &refKeyUnits() {
  static const std::vector<std::pair<std::string, const char *>> k = {
      {"CTOTAL", "cycles"},     {"JTOTAL", "us"},         {"JHIST", "us"},          {"JMPI", "us"},
      {"JPROC", "us"},          {"SWINALLOC", "us"},      {"SNETCOMPL", "us"},      {"SLOCPREP", "us"},
      {"HILOCAL", "us"},        {"HILOCELEM", "tuples"},  {"HILOCRATE", "Mbytes/sec"}, {"HOLOCAL", "us"},
      {"HOLOCELEM", "tuples"},  {"HOLOCRATE", "Mbytes/sec"}, {"HIGLOBAL", "us"},    {"HOGLOBAL", "us"},
      {"HASSIGN", "us"},        {"HIOFFCOMP", "us"},      {"HOOFFCOMP", "us"},      {"MIMEMALLOC", "us"},
      {"MIMAINPART", "us"},     {"MIFLUSHPART", "us"},    {"MOMEMALLOC", "us"},     {"MOMAINPART", "us"},
      {"MOFLUSHPART", "us"},    {"MWINPUT", "us"},        {"MWINPUTCNT", "calls"},  {"MWINWAIT", "us"},
      {"MWINWAITCNT", "calls"}, {"LPTASKTIME", "us"},     {"LPTASKCOUNT", "tasks"}, {"LPHISTCOMP", "us"},
      {"LPHISTELEM", "tuples"}, {"LPOFFSET", "us"},       {"LPMEMALLOC", "us"},     {"LPMEMSIZE", "bytes"},
      {"LPPART", "us"},         {"LPELEMENTS", "tuples"}, {"BPTASKTIME", "us"},     {"BPTASKCOUNT", "tasks"},
      {"BPMEMALLOC", "us"},     {"BPMEMSIZE", "bytes"},   {"BPBUILD", "us"},        {"BPBUILDELEM", "tuples"},
      {"BPPROBE", "us"},        {"BPPROBEELEM", "tuples"}};
  return k;
}

const std::vector<std::string> &Measurements::referenceKeys() {
  static const std::vector<std::string> keys = [] {
    std::vector<std::string> v;
    for (auto &ku : refKeyUnits()) v.push_back(ku.first);
    return v;
  }();
  return keys;
}

// Host CPU cycles (the reference reads PAPI_TOT_CYC, Measurements.cpp:90-107;
// PAPI is not in this image, the TSC is the same clock on x86).
static uint64_t cycles() {
#if defined(__x86_64__)
  return __builtin_ia32_rdtsc();
#else
  return 0;
#endif
}

void Measurements::init(uint32_t nodeId, uint32_t numberOfNodes, const std::string &tag, const std::string &dir) {
  State &s = st();
  s = State();
  s.nodeId = nodeId;
  s.numberOfNodes = numberOfNodes;
  s.tag = tag;
  s.dir = dir;
  if (!dir.empty()) mkdir(dir.c_str(), 0755);
  writeMetaData("NUMNODES", numberOfNodes);
  writeMetaData("NODEID", nodeId);
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  writeMetaData("HOST", host);
}

void Measurements::writeMetaData(const char *key, const char *value) { st().meta[key] = value; }
void Measurements::writeMetaData(const char *key, uint64_t value) { st().meta[key] = std::to_string(value); }

void Measurements::startJoin() {
  State &s = st();
  s.values.clear();
  for (auto &ku : refKeyUnits()) s.values[ku.first] = {0.0, ku.second};
  for (uint64_t &t : s.phaseTime) t = 0;
  s.joinStart = nowUs();
  s.cycleStart = cycles();
}
void Measurements::stopJoin() {
  State &s = st();
  s.joinStop = nowUs();
  put("CTOTAL", (double)(cycles() - s.cycleStart), "cycles");
  put("JTOTAL", (double)(s.joinStop - s.joinStart), "us");
  put("MWINWAIT", (double)s.phaseTime[NETWAIT], "us");
  for (const char *side : {"I", "O"}) {  // histogram read rate: 16-byte tuples per µs = MB/s
    const double us = s.values[std::string("H") + side + "LOCAL"].first;
    const double el = s.values[std::string("H") + side + "LOCELEM"].first;
    put(std::string("H") + side + "LOCRATE", us > 0 ? el * 16.0 / us : 0.0, "Mbytes/sec");
  }
  put("JHIST", (double)s.phaseTime[HIST], "us");
  put("JMPI", (double)(s.phaseTime[WINALLOC] + s.phaseTime[NET] + s.phaseTime[NETWAIT]), "us");
  put("JPROC", (double)(s.phaseTime[LOCPREP] + s.phaseTime[LOCAL]), "us");
  put("SWINALLOC", (double)s.phaseTime[WINALLOC], "us");
  put("SNETCOMPL", (double)s.phaseTime[NETWAIT], "us");
  put("SLOCPREP", (double)s.phaseTime[LOCPREP], "us");
}
uint64_t Measurements::joinUs() { return st().joinStop - st().joinStart; }

void Measurements::startHistogramComputation() { begin(HIST); }
void Measurements::stopHistogramComputation() { end(HIST); }
void Measurements::startWindowAllocation() { begin(WINALLOC); }
void Measurements::stopWindowAllocation() { end(WINALLOC); }
void Measurements::startNetworkPartitioning() { begin(NET); }
void Measurements::stopNetworkPartitioning() { end(NET); }
void Measurements::startWaitingForNetworkCompletion() { begin(NETWAIT); }
void Measurements::stopWaitingForNetworkCompletion() { end(NETWAIT); }
void Measurements::startLocalProcessingPreparations() { begin(LOCPREP); }
void Measurements::stopLocalProcessingPreparations() { end(LOCPREP); }
void Measurements::startLocalProcessing() { begin(LOCAL); }
void Measurements::stopLocalProcessing() { end(LOCAL); }

void Measurements::storeHistogramDetails(uint64_t localUs, uint64_t innerElements, uint64_t outerElements,
                                         uint64_t globalUs, uint64_t assignUs, uint64_t offsetUs) {
  // The device computes both relations' histograms in one enqueue + sync; the
  // time is split by element count for the per-relation keys.
  // HILOCAL / HOLOCAL: each relation's histogram kernels (Timeline spans);
  // the rates follow at stopJoin().
  (void)localUs;
  put("HILOCELEM", (double)innerElements, "tuples");
  put("HOLOCELEM", (double)outerElements, "tuples");
  // One fused all-gather carries both relations' histograms (unless the
  // outer one runs behind the inner exchange: HOGLOBAL is then timed on its
  // own stream by the Timeline): each relation is charged half of it.
  put("HIGLOBAL", globalUs / 2.0, "us");
  put("HOGLOBAL", globalUs / 2.0, "us");
  put("HASSIGN", (double)assignUs, "us");
  put("HIOFFCOMP", offsetUs / 2.0, "us");
  put("HOOFFCOMP", offsetUs / 2.0, "us");
}

void Measurements::storeNetworkDetails(uint64_t innerElements, uint64_t outerElements, uint64_t chunks) {
  (void)chunks;  // MWINPUTCNT counts the exchanges themselves (Window::exchange)
  put("MIELEM", (double)innerElements, "tuples");
  put("MOELEM", (double)outerElements, "tuples");
}

void Measurements::storeLocalPartitioningDetails(uint64_t elements, uint64_t items) {
  put("LPELEMENTS", (double)elements, "tuples");
  put("LPTASKCOUNT", (double)items, "tasks");
}

void Measurements::storeBuildProbeDetails(uint64_t buildElements, uint64_t probeElements, uint64_t items) {
  put("BPBUILDELEM", (double)buildElements, "tuples");
  put("BPPROBEELEM", (double)probeElements, "tuples");
  put("BPTASKCOUNT", (double)items, "tasks");
}

void Measurements::storeDevicePhase(const std::string &key, double ms) { put(key, ms * 1000.0, "us"); }

void Measurements::storeResultTuples(uint64_t tuples) {
  st().tuples = tuples;
  put("RTUPLES", (double)tuples, "tuples");
}

std::vector<uint64_t> Measurements::serializeResults() {
  State &s = st();
  auto dev = [&](const char *k) -> uint64_t {
    auto it = s.values.find(k);
    return it == s.values.end() ? 0 : (uint64_t)it->second.first;
  };
  return {s.tuples,
          s.joinStop - s.joinStart,
          s.phaseTime[HIST],
          s.phaseTime[WINALLOC] + s.phaseTime[NET] + s.phaseTime[NETWAIT],
          s.phaseTime[LOCPREP] + s.phaseTime[LOCAL],
          s.phaseTime[WINALLOC],
          s.phaseTime[NETWAIT],
          s.phaseTime[LOCPREP],
          dev("DLOCPART"),
          dev("DBP")};
}

void Measurements::printMeasurements(comm::Communicator *comm) {
  std::vector<uint64_t> mine = serializeResults();
  const uint32_t N = comm->size();
  std::vector<uint64_t> all(mine.size() * N);
  comm->allGatherHost(mine.data(), all.data(), mine.size());
  if (comm->rank() != 0) return;
  const char *names[] = {"Tuples", "Join", "Histogram", "Network", "Local",
                         "WinAlloc", "PartWait", "LocalPrep", "LocalPart", "LocalBP"};
  uint64_t totalTuples = 0;
  for (size_t k = 0; k < mine.size(); ++k) {
    std::printf("[RESULTS] %s:\t", names[k]);
    for (uint32_t r = 0; r < N; ++r) {
      const uint64_t v = all[r * mine.size() + k];
      if (k == 0) {
        std::printf("%lu\t", (unsigned long)v);
        totalTuples += v;
      } else {
        std::printf("%.3f\t", v / 1000.0);
      }
    }
    std::printf("\n");
  }
  uint64_t maxJoin = 0;
  for (uint32_t r = 0; r < N; ++r) maxJoin = std::max(maxJoin, all[r * mine.size() + 1]);
  std::printf("[RESULTS] Summary:\t%lu\t%.3f\n", (unsigned long)totalTuples, maxJoin / 1000.0);
  std::fflush(stdout);
}

void Measurements::storeAllMeasurements() {
  State &s = st();
  if (s.dir.empty()) return;
  const std::string base = s.dir + "/" + std::to_string(s.nodeId);
  if (FILE *f = std::fopen((base + ".perf").c_str(), "w")) {
    for (auto &kv : s.values) std::fprintf(f, "%s\t%.3f\t%s\n", kv.first.c_str(), kv.second.first, kv.second.second.c_str());
    std::fclose(f);
  }
  if (FILE *f = std::fopen((base + ".info").c_str(), "w")) {
    for (auto &kv : s.meta) std::fprintf(f, "%s\t%s\n", kv.first.c_str(), kv.second.c_str());
    std::fclose(f);
  }
}

std::map<std::string, double> Measurements::snapshot() {
  std::map<std::string, double> m;
  for (auto &kv : st().values) m[kv.first] = kv.second.first;
  return m;
}

}  // namespace performance
}  // namespace hpcjoin
