#!/usr/bin/env python3
"""Within one process: the general-path join's local pass after the engine's
workspace is trimmed and re-reserved behind a dummy allocation of a given
size (does the 5.97 / 6.45 ms local-pass spread follow the allocations?).

    python tools/placement_probe.py [dummy MiB sizes ...]
    PROBE_SKEWS=lo:hi+lo:hi+...  HPCJOIN_LP_SKEW values to cycle per placement
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402

C = hpcjoin.require_native()


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [0, 2, 64, 1024, 2, 0, 4096, 0]
    G = 10**9
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    R, S = C.Relation(G, G, "device", 0), C.Relation(G, G, "device", 0)
    a, b = C.GenSpec(seed=1234), C.GenSpec(seed=4321)
    a.sparse64 = b.sparse64 = True
    R.generate(a, 0)
    S.generate(b, 0)
    keep = []
    for mib in sizes:
        ctx.trim_workspace(0)
        if mib:
            keep.append(torch.empty(mib << 20, dtype=torch.uint8, device="cuda"))
        j = C.HashJoin(R, S, ctx, C.JoinConfig())
        # HPCJOIN_LP_SKEW (read per join): start offsets of the local output
        # columns inside their allocations, same placement otherwise.
        for skew in os.environ.get("PROBE_SKEWS", "0:0").split("+"):
            os.environ["HPCJOIN_LP_SKEW"] = skew
            res = [j.run() for _ in range(2)]
            row = {"dummy_MiB": mib, "skew": skew, "join_ms": [round(r["join_ms"], 3) for r in res],
                   "local_ms": [round(r["dev_local_partition_ms"], 3) for r in res],
                   "network_ms": [round(r["dev_network_ms"], 3) for r in res],
                   "correct": all(r["global_matches"] == G for r in res)}
            print(json.dumps(row), flush=True)
        del j


if __name__ == "__main__":
    main()
