#!/usr/bin/env python3
"""Mean of every PMC counter per kernel (and grid size) from a rocprofv3
`run_counter_collection.csv`, with the mean dispatch duration.  Used for the
round-5 translation / IO passes (r05o, r05p):

    python3 profiles/r05/scripts/pmc_by_kernel.py profiles/r05/r05o/tcp/run_counter_collection.csv
"""
import collections
import csv
import sys


def main(paths, only="uinet"):
    for p in paths:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(p)):
            if only and only not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = name.split("(")[0].split("::")[-1]
            k = f"{name} grid={r['Grid_Size']}"
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[k]["_dur_us"].append(d)
        print(p)
        for k, v in sorted(agg.items()):
            n = len(v["_dur_us"]) // max(1, len(v) - 1)
            print(f"  {k}  dispatches={n}")
            for c, xs in sorted(v.items()):
                print(f"    {c:40s} {sum(xs) / len(xs):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
