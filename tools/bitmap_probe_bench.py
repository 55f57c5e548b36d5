#!/usr/bin/env python3
"""Whole-key-space bitmap probe ceiling: 1B tuples with keys 0..2^30-1 each
test one bit of a 128 MiB bitmap (fits the 256 MiB Infinity Cache), keys read
from the 16-byte tuples in input order.  Compare with the partitioned outer
path (scatter ~4.4 ms + probe share of the bitmap join)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402


def main():
    C = hpcjoin.require_native()
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    R = C.Relation(n, n, "device", 0)
    R.generate(C.GenSpec(seed=3), 0)
    t = R.to_tensor()
    bits = max(5, (n - 1).bit_length())
    bm = torch.full(((1 << bits) // 32,), -1, dtype=torch.int32, device="cuda")
    for ipt in (8, 16):
        C.ops.probe_bitmap_global(t, bm, (1 << bits) - 1, ipt)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c = C.ops.probe_bitmap_global(t, bm, (1 << bits) - 1, ipt)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"bench": "probe_bitmap_global", "ipt": ipt, "tuples": n, "bitmap_MiB": (1 << bits) // 8 >> 20,
                          "ms": round(min(ts), 3), "count_ok": int(c.item()) == n}), flush=True)


if __name__ == "__main__":
    main()
