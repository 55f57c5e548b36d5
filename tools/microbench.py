#!/usr/bin/env python3
"""Run the per-phase micro-benchmarks on cuda:0 and print one JSON line each.

    python tools/microbench.py [copy|host_link|partition|local|bp|npj|wire|ablation|all] [--n N] [--bits B]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hpcjoin  # noqa: E402
from hpcjoin.utils import microbench as mb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all")
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--bits", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    todo = ["copy", "host_link", "partition", "local", "bp", "npj", "wire"] if a.what == "all" else [a.what]
    for w in todo:
        if w == "copy":
            r = mb.copy_ceiling()
        elif w == "host_link":
            r = mb.host_link()
        elif w == "partition":
            r = mb.partition_phase(a.n, a.bits, iters=a.iters)
        elif w == "local":
            r = mb.local_phase(a.n, iters=a.iters)
        elif w == "bp":
            r = mb.build_probe_phase(a.n, iters=a.iters)
        elif w == "ablation":
            for r in mb.scatter_ablation(a.n, (8, 9, 10, 11), a.iters, geometries=(0, 3, 6, 7, 8, 9)):
                print(json.dumps({"bench": "scatter_ablation", **r}), flush=True)
            continue
        elif w == "wire":
            r = mb.wire_phase(a.n, iters=a.iters)
        elif w == "npj":
            r = mb.npj_phase(min(a.n, 1 << 26), iters=a.iters)
        else:
            raise SystemExit(f"unknown {w}")
        print(json.dumps({"bench": w, **r}), flush=True)


if __name__ == "__main__":
    main()
