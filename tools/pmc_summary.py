#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel.

    python tools/pmc_summary.py gpurun_out/p12_sq gpurun_out/p12_fetch gpurun_out/p12_write
Prints one markdown row per kernel with counters averaged per dispatch and
derived quantities (wait fraction, LDS conflict ratio, HBM GB moved).
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hpcjoin::kernels::", "")
            k = k.split("<")[0] if "Scatter" not in k else k[:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return agg, calls


def main():
    merged = collections.defaultdict(dict)
    ncalls = {}
    for d in sys.argv[1:]:
        agg, calls = load(d)
        for k, v in agg.items():
            n = max(1, len(calls[k]))
            ncalls[k] = n
            for c, x in v.items():
                merged[k][c] = x / n
    print("| kernel | calls | wait% (SQ_WAIT_ANY/WAVE_CYCLES) | LDS conflict cycles / LDS insts | FETCH GB* | WRITE GB | L2 hit % |")
    print("|---|---|---|---|---|---|---|")
    for k, v in sorted(merged.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wait = 100 * v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"] if v.get("SQ_WAVE_CYCLES") else float("nan")
        lds = v["SQ_LDS_BANK_CONFLICT"] / v["SQ_INSTS_LDS"] if v.get("SQ_INSTS_LDS") else float("nan")
        fetch = v.get("FETCH_SIZE", float("nan")) / 1e6
        write = v.get("WRITE_SIZE", float("nan")) / 1e6
        hit = v.get("TCC_HIT_sum", 0)
        miss = v.get("TCC_MISS_sum", 0)
        hr = 100 * hit / (hit + miss) if hit + miss else float("nan")
        print(f"| {k} | {ncalls[k]} | {wait:.0f} | {lds:.2f} | {fetch:.2f} | {write:.2f} | {hr:.0f} |")
    print("\n*FETCH_SIZE/WRITE_SIZE are in KB per dispatch in rocprofv3; shown as GB. On gfx950 FETCH_SIZE reports "
          "~1/2 of the bytes of wide streaming reads (MI355X_MICROARCH.md §HBM); L2 hit % mixes the fetch/write passes.")


if __name__ == "__main__":
    main()
