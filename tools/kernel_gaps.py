#!/usr/bin/env python3
"""Kernel timeline from a rocprofv3 kernel_trace.csv: duration of every
dispatch and the idle gap before it (host enqueue stalls show up as gaps).

    python tools/kernel_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--last N]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    prev, out = None, []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        out.append((r["Kernel_Name"].replace("hpcjoin::kernels::", "")[:64], (e - s) / 1e3,
                    (s - prev) / 1e3 if prev else 0.0))
        prev = e
    for name, dur, gap in out[-a.last:]:
        print(f"{name:<64} {dur:10.1f} us   gap {gap:8.1f} us")


if __name__ == "__main__":
    main()
