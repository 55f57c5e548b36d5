#!/usr/bin/env python3
"""Stream-mix ceilings: for every pass of the joins, the time of ONE in-order
pass over the same element count with the pass's exact byte mix (read streams
and write streams, each moved with 16-byte vectors, no partitioning, no LDS)
-- `ops.stream_mix`, microbench.hip streamMixKernel.  A partitioning kernel's
efficiency is ceiling_ms / kernel_ms.

    python tools/stream_mix_bench.py [elements=1e9]

One JSON line per mix: {"mix", "pass", "read_B", "write_B", "ms", "TBps"}.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402

# (pass, read A, read B, write A, write B) in bytes per element
MIXES = [
    ("general network pass (tuple -> key-only word)", 16, 0, 8, 0),
    ("count-only network pass (tuple -> u32 fragment)", 16, 0, 4, 0),
    ("split local pass (word -> u32 + u16 columns)", 8, 0, 4, 2),
    ("key-only build/probe (u32 + u16 columns)", 4, 2, 0, 0),
    ("fragment local pass (u32 -> u16)", 4, 0, 2, 0),
    ("bitmap join (u32 fragments)", 4, 0, 0, 0),
    ("copy 16 B", 16, 0, 16, 0),
    ("read 16 B", 16, 0, 0, 0),
]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


def main():
    C = hpcjoin.require_native()
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    n -= n % 512
    dev = torch.device("cuda", 0)
    buf = lambda b: torch.empty(max(n * b, 16), dtype=torch.uint8, device=dev) if b else torch.empty(16, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    for name, ra, rb, wa, wb in MIXES:
        a, b, oa, ob = buf(ra), buf(rb), buf(wa), buf(wb)
        a.random_(0, 255)
        if rb:
            b.random_(0, 255)
        ms = timed(lambda: C.ops.stream_mix(n, ra, rb, wa, wb, a, b, oa, ob, sink))
        rd, wr = ra + rb, wa + wb
        print(json.dumps({"mix": f"r{ra}+{rb}/w{wa}+{wb}", "pass": name, "elements": n, "read_B": rd, "write_B": wr,
                          "ms": round(ms, 3), "TBps": round(n * (rd + wr) / ms / 1e9, 3)}), flush=True)
        del a, b, oa, ob
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
