#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into markdown.

    python tools/rocprof_summary.py gpurun_out/prof_1b/run_kernel_stats.csv [--bytes KERNEL=GB ...]

Optional --bytes annotates kernels with the algorithmic bytes they move per
call so the table shows effective HBM bandwidth (GB/s) next to time.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--bytes", nargs="*", default=[], help="substring=GB_per_call")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    bmap = {}
    for kv in a.bytes:
        k, v = kv.split("=")
        bmap[k] = float(v)
    rows = list(csv.DictReader(open(a.stats)))
    if a.title:
        print(f"### {a.title}\n")
    print("| kernel | calls | avg ms | total % | algorithmic GB/call | eff. TB/s |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        name = r["Name"].split("(")[0].replace("void ", "").replace("hpcjoin::kernels::", "")
        avg_ms = float(r["AverageNs"]) / 1e6
        gb = next((v for k, v in bmap.items() if k in name), None)
        bw = f"{gb / avg_ms:.2f}" if gb and avg_ms > 0 else ""
        print(f"| {name} | {r['Calls']} | {avg_ms:.3f} | {float(r['Percentage']):.1f} | {gb or ''} | {bw} |")


if __name__ == "__main__":
    main()
