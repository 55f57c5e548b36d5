"""Network scatter with round-interleaved slices vs the linear slice layout
(scatterAblation mode 3 vs 0, 1 = coalesced write-out ceiling): is the
1024-way scatter bound by how many pages its concurrent write streams touch?

    python tools/round_probe.py [n=1e9] [bits=10]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hpcjoin  # noqa: E402,F401
from hpcjoin.utils import microbench as mb  # noqa: E402

C = hpcjoin.require_native()


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
    bits = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    t = mb.gen(n)
    for geo in (9,):
        row = {"n": n, "bits": bits, "geometry": geo}
        row["linear"] = round(C.ops.bench_scatter_ms(t, bits, 0, 5, 512, geo), 4)
        row["coalesced"] = round(C.ops.bench_scatter_ms(t, bits, 1, 5, 512, geo), 4)
        for lp in (3, 4, 5, 6, 7, 8, 9):
            row[f"rounds_lp{lp}"] = round(C.ops.bench_scatter_ms(t, bits, 3, 5, 512, geo, lp), 4)
        row["linear_again"] = round(C.ops.bench_scatter_ms(t, bits, 0, 5, 512, geo), 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
