"""Per-call durations of the general path's big kernels from a rocprofv3
kernel trace (run_kernel_trace.csv): one line per kernel name, calls in
launch order (inner side first within a join unless the run reorders them)."""
import csv
import sys

KEYS = ("netScatterClaim", "localScatterPersist", "localHistogramKernel", "bpKeyQuotient")


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    for k in KEYS:
        v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if k in r["Kernel_Name"]]
        if v:
            print(f"{k:22s} " + " ".join(f"{x:.0f}" for x in v))


if __name__ == "__main__":
    main(sys.argv[1])
