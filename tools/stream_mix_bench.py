#!/usr/bin/env python3
"""Streaming ceiling for the count-only network pass's byte mix (read 16 B,
write 4 B per tuple, no partitioning) next to the plain copy, on cuda:0."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hpcjoin  # noqa: E402


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
    R = C.Relation(n, n, "device", 0)
    R.generate(C.GenSpec(seed=1), 0)
    t = R.to_tensor()
    for ipt in (1, 4, 8):
        ms = timed(lambda: C.ops.project_keys(t, 10, ipt))
        print(json.dumps({"bench": "project_keys", "ipt": ipt, "tuples": n, "ms": round(ms, 3),
                          "TBps": round(n * 20 / ms / 1e9, 3)}), flush=True)
    dst = torch.empty_like(t)
    ms = timed(lambda: C.ops.copy_into(t, dst))
    print(json.dumps({"bench": "copy", "bytes": n * 16, "ms": round(ms, 3), "TBps": round(n * 32 / ms / 1e9, 3)}))


if __name__ == "__main__":
    main()
