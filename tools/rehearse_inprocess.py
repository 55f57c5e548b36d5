#!/usr/bin/env python3
"""N ranks as threads of one process on one GPU (InProcessCommunicator, device
buffers): the full N-rank join logic at full size -- split histogram, wire
codec, chunked exchange, per-chunk outer pass -- with device copies standing
in for RCCL.  Times are not multi-GPU times; this checks correctness at scale.

    python tools/rehearse_inprocess.py --ranks 4 --size 1e9
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import hpcjoin  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--size", type=float, default=1e9)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--sparse", action="store_true", help="unique random 63-bit keys (the general path)")
    ap.add_argument("--shuffle", action="store_true", help="hash-partition shuffle instead of replicated bitmaps")
    ap.add_argument("--one-sided", action="store_true")
    args = ap.parse_args()
    C = hpcjoin.require_native()
    n, G = args.ranks, int(args.size)
    group = C.InProcessGroup(n)
    inner = C.GenSpec(seed=1234)
    outer = C.GenSpec(seed=4321)
    inner.sparse64 = outer.sparse64 = args.sparse
    out, errors = [None] * n, []

    def rank_main(r):
        try:
            ctx = C.ExecContext("device", 0, group.communicator(r))
            lo = C.Relation.local_offset_for(G, r, n)
            R = C.Relation(C.Relation.local_size_for(G, r, n), G, "device", 0)
            S = C.Relation(C.Relation.local_size_for(G, r, n), G, "device", 0)
            R.generate(inner, lo)
            S.generate(outer, lo)
            cfg = C.JoinConfig()
            cfg.chunks = args.chunks
            if args.shuffle:
                cfg.bitmap_join = False
            if args.one_sided:
                cfg.exchange = C.ExchangeMode.ONE_SIDED
            j = C.HashJoin(R, S, ctx, cfg)
            res = [j.run() for _ in range(2)]
            out[r] = {"plan": repr(j.plan), "global_matches": [x["global_matches"] for x in res],
                      "local_matches": res[-1]["local_matches"], "wire_bytes": res[-1]["wire_bytes"],
                      "local_fallbacks": sum(x["local_fallbacks"] for x in res), "join_ms": res[-1]["join_ms"]}
            del j, R, S, ctx
        except Exception as e:  # surface in the main thread
            errors.append((r, repr(e)))

    t0 = time.time()
    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    ok = not errors and all(o["global_matches"] == [G, G] for o in out)
    print(json.dumps({"ranks": n, "size": G, "ok": ok, "errors": errors, "wall_s": round(time.time() - t0, 1),
                      "rank0": out[0] if out[0] else None,
                      "local_matches": [o["local_matches"] for o in out] if not errors else None}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
