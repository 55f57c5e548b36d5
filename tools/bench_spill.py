#!/usr/bin/env python3
"""Capacity spill benchmark: a join whose relations plus workspace exceed
what HBM holds (or a forced workspace budget) runs in K key-hash passes
(JoinConfig.passes, kernels/spill.hip) or, for the bitmap plan, in partition-
group passes (tasks/BitmapJoin: `group_passes`).  One JSON line per configuration.

    python tools/bench_spill.py --size 1e9 --budget-frac 0.25      # 1B x 1B, workspace budget = estimate / 4
    python tools/bench_spill.py --size 6e9                          # 6B x 6B in HBM: 192 GB of relations
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_SDMA", "0")

import torch  # noqa: E402

import hpcjoin  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=1e9, help="tuples per relation (inner; outer too unless --outer-size)")
    ap.add_argument("--outer-size", type=float, default=0, help="outer tuples (0: --size)")
    ap.add_argument("--outer-dist", default="unique", choices=["unique", "zipf", "uniform"],
                    help="outer keys: unique, or Zipf / uniform over the inner key domain (BASELINE config 4: "
                         "--size 1e9 --outer-size 16e9 --outer-dist zipf, 272 GB of relations on one GPU)")
    ap.add_argument("--theta", type=float, default=0.75)
    ap.add_argument("--budget-frac", type=float, default=0.0,
                    help="memory budget of one pass (its pass buffers + its workspace) as a fraction of the "
                         "single-pass workspace estimate; 0: what HBM has free")
    ap.add_argument("--passes", type=int, default=0, help="force the pass count (0: planner)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--input", default="device", choices=["device", "pinned"])
    ap.add_argument("--reference", default="auto", choices=["auto", "on", "off"],
                    help="also time the single-pass join when it fits (auto: when no budget is forced)")
    args = ap.parse_args()
    C = hpcjoin.require_native()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G = int(args.size)
    GS = int(args.outer_size) or G
    R = C.Relation(G, G, args.input, 0)
    S = C.Relation(GS, GS, args.input, 0)
    inner = C.GenSpec(seed=1234)
    outer = (C.GenSpec(seed=4321) if args.outer_dist == "unique" else
             C.GenSpec(distribution=getattr(C.KeyDistribution, args.outer_dist.upper()), seed=4321, domain=G,
                       zipf_theta=args.theta))
    R.generate(inner, 0)
    S.generate(outer, 0)
    expected = C.Relation.expected_matches(inner, G, outer, GS)
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()
    probe = C.JoinConfig()
    probe.reserve_workspace = False
    probe.passes = 1
    est = C.HashJoin(R, S, ctx, probe).workspace_estimate()
    cfg = C.JoinConfig()
    cfg.passes = args.passes
    if args.budget_frac > 0:
        cfg.workspace_budget = int(est * args.budget_frac)
    t0 = time.perf_counter()
    j = C.HashJoin(R, S, ctx, cfg)
    setup_ms = (time.perf_counter() - t0) * 1e3
    try:
        first = j.run()
    except Exception as e:  # noqa: BLE001 -- report what the planner decided
        print(json.dumps({"bench": "capacity_spill", "size": G, "error": str(e)[:300],
                          "spill": {k: (round(v / 1e9, 2) if k.endswith("bytes") else v)
                                    for k, v in j.spill_info.items()},
                          "single_pass_workspace_estimate_GB": round(est / 1e9, 1),
                          "hbm_free_after_relations_GB": round(free0 / 1e9, 1)}), flush=True)
        raise
    times, res, results = [], first, []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = j.run()
        times.append((time.perf_counter() - t0) * 1e3)
        results.append(res)
    out = {"bench": "capacity_spill", "size": G, "outer_size": GS, "outer_dist": args.outer_dist,
           "input": args.input, "relations_GB": round((G + GS) * 16 / 1e9, 1),
           "hbm_total_GB": round(total / 1e9, 1), "hbm_free_after_relations_GB": round(free0 / 1e9, 1),
           "single_pass_workspace_estimate_GB": round(est / 1e9, 1),
           "workspace_budget_GB": round(cfg.workspace_budget / 1e9, 1) if cfg.workspace_budget else None,
           "passes": j.spill_passes, "group_passes": res["group_passes"] if res else None, "setup_ms": round(setup_ms, 1), "first_join_ms": round(first["join_ms"], 2),
           "ms_per_join": round(sum(times) / len(times), 2), "join_ms": [round(t, 2) for t in times],
           "compact_ms": round(res["compact_ms"], 2),
           "value_Gtuples_per_s": round((G + GS) / (sum(times) / len(times)) / 1e6, 2),
           "matches": res["global_matches"], "expected_matches": expected,
           "correct": all(r["global_matches"] == expected for r in [first] + results),
           "spill": {k: (round(v / 1e9, 2) if k.endswith("bytes") else v) for k, v in j.spill_info.items()},
           "plan": repr(j.plan)}
    del j
    if args.reference == "on" or (args.reference == "auto" and args.budget_frac > 0):
        one = C.JoinConfig()
        one.passes = 1
        jr = C.HashJoin(R, S, ctx, one)
        jr.run()
        t = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            r1 = jr.run()
            t.append((time.perf_counter() - t0) * 1e3)
        out["single_pass_ms"] = round(sum(t) / len(t), 2)
        out["single_pass_correct"] = r1["global_matches"] == expected
        del jr
    print(json.dumps(out), flush=True)
    del ctx


if __name__ == "__main__":
    main()
