"""Per-dispatch PMC values of the big kernels of a rocprofv3 --pmc run
(run_counter_collection.csv + run_kernel_trace.csv in one directory)."""
import collections
import csv
import os
import sys

KEYS = ("netScatter", "localScatter", "bpKey", "bitmapJoin", "bpMat")


def main(d):
    trace = {r["Dispatch_Id"]: r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))}
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        agg[r["Dispatch_Id"]][r["Counter_Name"]] = agg[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        agg[r["Dispatch_Id"]]["name"] = r["Kernel_Name"]
    for did, v in sorted(agg.items(), key=lambda x: int(x[0])):
        name = v.pop("name")
        if not any(k in name for k in KEYS):
            continue
        t = trace.get(did)
        dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3 if t else float("nan")
        vals = " ".join(f"{k.replace('TCP_UTCL1_', 'U1_')}={x:.3g}" for k, x in sorted(v.items()))
        print(f"{did:>5} {name.split('<')[0].split('::')[-1][:24]:24s} {dur:8.0f}us {vals}")


if __name__ == "__main__":
    main(sys.argv[1])
