#!/usr/bin/env python3
"""Infinity Cache (MALL) probe: does a buffer written by one kernel and read
by the next stay on-chip when it is small enough?

Pattern A (all HBM):   for each slice i of a big input: copy in[i] -> out[i] (big), read out[i]
Pattern B (reuse):     for each slice i of a big input: copy in[i] -> buf (reused), read buf

Prints one JSON line per slice size.  If B is much faster than A, a pipeline
that consumes a pass's output while it is still in MALL saves HBM traffic.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402


def main():
    C = hpcjoin.require_native()
    total = 4 << 30
    src = torch.ones(total // 8, dtype=torch.int64, device="cuda")
    big = torch.empty_like(src)
    sink = torch.zeros(1, dtype=torch.int64, device="cuda")
    for mb in (16, 32, 64, 96, 128, 192, 256, 512):
        sl = (mb << 20) // 8
        nsl = src.numel() // sl
        buf = torch.empty(sl, dtype=torch.int64, device="cuda")
        res = {"slice_MB": mb}
        for name, reuse in (("hbm", False), ("reuse", True)):
            def run():
                for i in range(nsl):
                    a = src[i * sl:(i + 1) * sl]
                    b = buf if reuse else big[i * sl:(i + 1) * sl]
                    C.ops.copy_into(a, b)
                    C.ops.read_sink(b, sink)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 3
            # bytes moved if everything went to HBM: read src + write + read back
            res[name + "_ms"] = round(ms, 3)
            res[name + "_TBps_equiv"] = round(3 * total / ms / 1e9, 2)
        # copy-only and read-only of a reused slice
        res["launches"] = 2 * nsl
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
