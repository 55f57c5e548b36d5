#!/usr/bin/env python3
"""Random 32-byte row gather ceiling on one MI355X (the outer-row gather of the
TPC-H-like late materialization): out[i] = payload[rids[i]] for n rows of a
table of n rows, rids random / sorted.  Prints GB/s of HBM traffic assuming a
64-byte fetch per random row."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402


def main():
    C = hpcjoin.require_native()
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 600_000_000
    payload = C.ops.generate_payload(n, 0, 7, "cuda:0")
    modes = [int(m) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1]
    for order in ("random", "sorted"):
        rids = torch.randperm(n, device="cuda", dtype=torch.int64) if order == "random" else \
            torch.arange(n, device="cuda", dtype=torch.int64)
        for mode in modes:
            out = C.ops.gather_rows(rids, 0, payload, mode)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = C.ops.gather_rows(rids, 0, payload, mode)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = min(ts)
            fetch = n * 8 + n * (64 if order == "random" else 32)
            write = n * 32
            print(json.dumps({"bench": "gather_rows", "order": order, "mode": mode, "rows": n, "ms": round(ms, 3),
                              "Grows_per_s": round(n / ms / 1e6, 2),
                              "TBps_64B_lines": round((fetch + write) / ms / 1e9, 3)}), flush=True)
            del out
        del rids
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
