#!/usr/bin/env python3
"""Where the claim scatter's time goes, phase by phase (shader clock).

Needs a build with the phase stamps compiled in:

    HPCJOIN_EXTRA_HIPFLAGS=-DHPCJOIN_SCATTER_PROF python -c "import __graft_entry__ as g; g.build()"

(tools/gpu.sh `phases` does that in a copy of the tree under ab/prof).  Runs
the headline join (1B x 1B dense unique keys: the fragment scatter only)
and the general path (random 63-bit keys: key-only network scatter + local
split scatter, summed) and prints one JSON line per workload: each phase's
share of wave 0's tile-loop cycles and its cycles per tile.

Phases (partition.hip, ScatterProf): rank (includes waiting for the tile's
loads), barrier A, claims + next-tile prefetch issue, scan, staging, write
bases (the claim atomics land), barrier B, write-out issue.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hpcjoin  # noqa: E402

PHASES = ["rank", "barrier_A", "claims_prefetch", "scan", "staging", "write_bases", "barrier_B", "write_out"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    C = hpcjoin.require_native()
    if not C.ops.scatter_profile_built():
        sys.exit("scatter_phases.py: this build has no phase stamps (HPCJOIN_EXTRA_HIPFLAGS=-DHPCJOIN_SCATTER_PROF)")
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G = int(args.size)
    for name, sparse in (("headline", False), ("general", True)):
        inner, outer = C.GenSpec(seed=1234), C.GenSpec(seed=4321)
        inner.sparse64 = outer.sparse64 = sparse
        R = C.Relation(G, G, "device", 0)
        S = C.Relation(G, G, "device", 0)
        R.generate(inner, 0)
        S.generate(outer, 0)
        j = C.HashJoin(R, S, ctx, C.JoinConfig())
        for _ in range(2):
            j.run()
        C.ops.scatter_profile(True)
        ms = []
        for _ in range(args.steps):
            res = j.run()
            assert res["global_matches"] == G, (name, res["global_matches"])
            ms.append(res["join_ms"])
        v = C.ops.scatter_profile(True)
        total = sum(v[:8]) or 1
        tiles = max(v[8], 1)
        print(json.dumps({
            "workload": name, "join_ms": round(sum(ms) / len(ms), 3), "ranges": v[9], "tiles": v[8],
            "share": {p: round(v[i] / total, 4) for i, p in enumerate(PHASES)},
            "cycles_per_tile": {p: round(v[i] / tiles, 1) for i, p in enumerate(PHASES)},
        }), flush=True)
        del j, R, S
        ctx.reset_scratch()


if __name__ == "__main__":
    main()
