#!/usr/bin/env python3
"""Per-join device sub-phase spans (the engine's Timeline events: network
scatters, local histogram / layout / scatter, build/probe) of one workload,
without a profiler attached.  Use it when a phase's time differs between a
profiled and a plain run (a profiler serialises dispatches).

    python tools/phase_spans.py --sparse --steps 6            # general path, 1B x 1B
    python tools/phase_spans.py --size 1e9 --keys MIMAINPART,LPPART
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_SDMA", "0")

import torch  # noqa: E402

import hpcjoin  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=1e9)
    ap.add_argument("--sparse", action="store_true", help="random 63-bit keys (the general path)")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--env-cycle", default="",
                    help="NAME=v1|v2|...: set the environment variable to each value in turn, one join each, "
                         "cycling (same-process A/B of an environment knob read per join)")
    ap.add_argument("--ab", default="",
                    help="FIELD=v1|v2|...: one join per JoinConfig value, built on the same relations and run in "
                         "turn (same-process A/B of a config field)")
    ap.add_argument("--after-headline", action="store_true",
                    help="first run the dense-key headline join on the same context (as bench.py does before "
                         "its general path), then free its relations")
    ap.add_argument("--trim", action="store_true", help="with --after-headline: trim the workspace in between")
    ap.add_argument("--keys", default="", help="comma- or colon-separated measurement keys (default: every device span)")
    args = ap.parse_args()
    C = hpcjoin.require_native()
    ctx = C.ExecContext("device", 0, C.LocalCommunicator())
    G = int(args.size)
    if args.after_headline:
        Rh, Sh = C.Relation(G, G, "device", 0), C.Relation(G, G, "device", 0)
        Rh.generate(C.GenSpec(seed=1234), 0)
        Sh.generate(C.GenSpec(seed=4321), 0)
        jh = C.HashJoin(Rh, Sh, ctx, C.JoinConfig())
        for _ in range(3):
            jh.run()
        del jh, Rh, Sh
        ctx.reset_scratch()
        if args.trim:
            ctx.trim_workspace(0)
        torch.cuda.synchronize()
    R = C.Relation(G, G, "device", 0)
    S = C.Relation(G, G, "device", 0)
    a, b = C.GenSpec(seed=1234), C.GenSpec(seed=4321)
    a.sparse64 = b.sparse64 = args.sparse
    R.generate(a, 0)
    S.generate(b, 0)
    torch.cuda.synchronize()
    joins = []
    if args.ab:
        field, vals = args.ab.split("=", 1)
        for v in vals.split("|"):
            cfg = C.JoinConfig()
            setattr(cfg, field, type(getattr(cfg, field))(int(v) if v.lstrip("-").isdigit() else v))
            joins.append((f"{field}={v}", C.HashJoin(R, S, ctx, cfg)))
    else:
        joins.append((None, C.HashJoin(R, S, ctx, C.JoinConfig())))
    for _, j in joins:
        j.run()
    want = [k for k in args.keys.replace(":", ",").split(",") if k]
    cyc = None
    if args.env_cycle:
        name, vals = args.env_cycle.split("=", 1)
        cyc = (name, vals.split("|"))
    for step in range(args.steps):
        tag, j = joins[step % len(joins)]
        if cyc:
            tag = cyc[1][step % len(cyc[1])]
            os.environ[cyc[0]] = tag
        r = j.run()
        snap = C.measurements.snapshot()
        keys = want or sorted(k for k in snap if k.isupper())
        print(json.dumps({"step": step, "env": tag, "join_ms": round(r["join_ms"], 3), "dev_span_ms": round(r["dev_span_ms"], 3),
                          "correct": r["global_matches"] == G,
                          "spans": {k: round(snap[k], 1) for k in keys if k in snap}}), flush=True)


if __name__ == "__main__":
    main()
