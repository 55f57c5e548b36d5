// Host-path self test for sanitizer builds (SURVEY §5 "race detection /
// sanitizers": the reference has none and its kernels race).  GPU sanitizers
// are not available on the MI355X pool, so the host runtime -- tasks,
// histograms, offsets, windows, the in-process communicator's threads, late
// materialization and failure propagation -- is exercised here under
// AddressSanitizer + UBSan and, in a second build, ThreadSanitizer
// (tools/sanitize_host.sh, tests/test_sanitizers.py).
//
//   host_selftest [--ranks N] [--size G]
// Exit code 0 iff every join matches its oracle.
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../comm/InProcessCommunicator.h"
#include "../core/ExecContext.h"
#include "../data/Relation.h"
#include "../kernels/kernels.h"
#include "../operators/HashJoin.h"
#include "../operators/LateMaterialization.h"
#include "../utils/Fault.h"

using namespace hpcjoin;

namespace {

struct Case {
  const char *name;
  kernels::KeyDistribution outer;
  bool wide, materialize, tpch;
  core::KeyHashing hashing;
  bool wire = false;  // bit-packed exchange (host twin of kernels/wire.hip)
};

bool runCase(const Case &c, uint32_t ranks, uint64_t G) {
  auto group = std::make_shared<comm::InProcessGroup>(ranks);
  std::vector<std::string> errors(ranks);
  std::vector<uint64_t> matches(ranks, 0), pairs(ranks, 0);
  data::GenSpec is, os;
  is.seed = 11;
  is.tpchSparse = c.tpch;
  os.seed = 12;
  os.distribution = c.outer;
  os.domain = c.outer == kernels::KeyDistribution::Unique ? 0 : G;
  os.tpchSparse = c.tpch;
  const uint64_t GS = c.outer == kernels::KeyDistribution::Unique ? G : 3 * G;
  auto rankMain = [&](uint32_t r) {
    try {
      comm::InProcessCommunicator comm(group, r);
      core::ExecContext ctx(Location::Host, -1, &comm);
      data::Relation R(data::Relation::localSizeFor(G, r, ranks), G, Location::Host, 0);
      data::Relation S(data::Relation::localSizeFor(GS, r, ranks), GS, Location::Host, 0);
      R.generate(is, data::Relation::localOffsetFor(G, r, ranks));
      S.generate(os, data::Relation::localOffsetFor(GS, r, ranks));
      core::JoinConfig cfg;
      cfg.format = c.wide ? core::TupleFormat::Wide : core::TupleFormat::Compressed;
      cfg.materialize = c.materialize;
      cfg.keyHashing = c.hashing;
      cfg.chunks = 2;
      cfg.wireCodec = c.wire ? core::WireCodecMode::On : core::WireCodecMode::Off;
      operators::HashJoin j(&R, &S, &ctx, cfg);
      operators::JoinResult res = j.run();
      matches[r] = res.globalMatches;
      pairs[r] = res.outputPairs;
      if (c.materialize) {  // fetch 32-byte payload rows of both sides from their owners
        const uint64_t oR = data::Relation::localOffsetFor(G, r, ranks), oS = data::Relation::localOffsetFor(GS, r, ranks);
        std::vector<uint64_t> rowsR(R.getLocalSize() * kernels::ROW_WORDS), rowsS(S.getLocalSize() * kernels::ROW_WORDS);
        for (uint64_t i = 0; i < R.getLocalSize(); ++i)
          for (uint32_t w = 0; w < kernels::ROW_WORDS; ++w) rowsR[i * kernels::ROW_WORDS + w] = kernels::payloadWord(1, oR + i, w);
        for (uint64_t i = 0; i < S.getLocalSize(); ++i)
          for (uint32_t w = 0; w < kernels::ROW_WORDS; ++w) rowsS[i * kernels::ROW_WORDS + w] = kernels::payloadWord(2, oS + i, w);
        operators::PayloadColumn a{rowsR.data(), R.getLocalSize(), oR, G}, b{rowsS.data(), S.getLocalSize(), oS, GS};
        operators::LateMaterialization lm(&ctx, a, b);
        std::vector<uint64_t> out(res.outputPairs * operators::LateMaterialization::OUT_WORDS + 1);
        lm.materialize(j.getOutput(), res.outputPairs, out.data());
        for (uint64_t i = 0; i < res.outputPairs; ++i) {
          const uint64_t *row = &out[i * operators::LateMaterialization::OUT_WORDS];
          for (uint32_t w = 0; w < kernels::ROW_WORDS; ++w)
            if (row[2 + w] != kernels::payloadWord(1, row[0], w) || row[6 + w] != kernels::payloadWord(2, row[1], w))
              throw std::runtime_error("payload row does not belong to its rid");
        }
      }
    } catch (const std::exception &e) {
      errors[r] = e.what();
    }
  };
  std::vector<std::thread> ts;
  for (uint32_t r = 0; r < ranks; ++r) ts.emplace_back(rankMain, r);
  for (auto &t : ts) t.join();
  const uint64_t expected = data::Relation::expectedMatches(is, G, os, GS);
  bool ok = true;
  for (uint32_t r = 0; r < ranks; ++r) {
    if (!errors[r].empty()) {
      std::printf("[%s] rank %u failed: %s\n", c.name, r, errors[r].c_str());
      ok = false;
    } else if (matches[r] != expected) {
      std::printf("[%s] rank %u: %lu matches, expected %lu\n", c.name, r, (unsigned long)matches[r],
                  (unsigned long)expected);
      ok = false;
    }
  }
  if (ok && c.materialize) {
    uint64_t total = 0;
    for (uint64_t p : pairs) total += p;
    if (total != expected) {
      std::printf("[%s] %lu pairs, expected %lu\n", c.name, (unsigned long)total, (unsigned long)expected);
      ok = false;
    }
  }
  std::printf("[%s] ranks=%u %s\n", c.name, ranks, ok ? "OK" : "FAIL");
  return ok;
}

// A rank failing mid-join must make every peer fail (not hang), under the sanitizers too.
bool runFaultCase(uint32_t ranks, uint64_t G) {
  auto group = std::make_shared<comm::InProcessGroup>(ranks);
  std::vector<int> failed(ranks, 0);
  auto rankMain = [&](uint32_t r) {
    try {
      utils::armFault("network", 1);
      comm::InProcessCommunicator comm(group, r);
      core::ExecContext ctx(Location::Host, -1, &comm);
      data::Relation R(data::Relation::localSizeFor(G, r, ranks), G, Location::Host, 0);
      data::Relation S(data::Relation::localSizeFor(G, r, ranks), G, Location::Host, 0);
      R.generate(data::GenSpec(), data::Relation::localOffsetFor(G, r, ranks));
      S.generate(data::GenSpec(), data::Relation::localOffsetFor(G, r, ranks));
      operators::HashJoin j(&R, &S, &ctx, core::JoinConfig());
      j.run();
    } catch (const std::exception &) {
      failed[r] = 1;
    }
    utils::armFault("", -1);
  };
  std::vector<std::thread> ts;
  for (uint32_t r = 0; r < ranks; ++r) ts.emplace_back(rankMain, r);
  for (auto &t : ts) t.join();
  bool ok = true;
  for (int f : failed) ok = ok && f;
  std::printf("[fault] ranks=%u %s\n", ranks, ok ? "OK" : "FAIL");
  return ok;
}

}  // namespace

int main(int argc, char **argv) {
  uint32_t ranks = 3;
  uint64_t G = 50000;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--ranks") && i + 1 < argc) ranks = (uint32_t)std::stoul(argv[++i]);
    else if (!std::strcmp(argv[i], "--size") && i + 1 < argc) G = std::stoull(argv[++i]);
  }
  utils::setCommTimeoutMs(60000);
  const Case cases[] = {
      {"unique", kernels::KeyDistribution::Unique, false, false, false, core::KeyHashing::Auto},
      {"zipf", kernels::KeyDistribution::Zipf, false, false, false, core::KeyHashing::Auto},
      {"wide_materialize", kernels::KeyDistribution::Uniform, true, true, false, core::KeyHashing::Auto},
      {"tpch_materialize", kernels::KeyDistribution::Modulo, false, true, true, core::KeyHashing::Auto},
      {"mix_on_wide", kernels::KeyDistribution::Modulo, true, false, false, core::KeyHashing::On},
      {"wire_zipf", kernels::KeyDistribution::Zipf, false, false, false, core::KeyHashing::Auto, true},
      {"wire_tpch_materialize", kernels::KeyDistribution::Modulo, false, true, true, core::KeyHashing::Auto, true},
  };
  bool ok = true;
  for (const Case &c : cases) ok = runCase(c, ranks, G) && ok;
  ok = runFaultCase(ranks, G) && ok;
  std::printf("%s\n", ok ? "ALL OK" : "FAILED");
  return ok ? 0 : 1;
}
