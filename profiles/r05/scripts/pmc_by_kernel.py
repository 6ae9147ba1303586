#!/usr/bin/env python3
"""PMC counters per kernel (and grid size) from a rocprofv3
`run_counter_collection.csv`, with the dispatch duration: the mean over
dispatches, or every dispatch with --per-dispatch.  Used for the round-5
translation / IO passes (r05o-r05r).  Read per dispatch where one kernel runs
in different roles: in r05o / r05p the zero-copy path's hook calls launch the
parse and walk kernels, which find the mbufs unregistered and exit in ~20 µs,
and those dispatches pull the means down.

    python3 profiles/r05/scripts/pmc_by_kernel.py [--per-dispatch] <csv> ...
"""
import collections
import csv
import sys


def kernel_key(r):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    return f"{name.split('(')[0].split('::')[-1]} grid={r['Grid_Size']}"


def main(argv, only="uinet"):
    per = "--per-dispatch" in argv
    for p in [a for a in argv if not a.startswith("--")]:
        disp = collections.defaultdict(dict)  # (kernel, dispatch id) -> counters
        for r in csv.DictReader(open(p)):
            if only and only not in r["Kernel_Name"]:
                continue
            d = disp[(kernel_key(r), int(r["Dispatch_Id"]))]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["_dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        by = collections.defaultdict(list)
        for (k, i), d in sorted(disp.items(), key=lambda kv: kv[0][1]):
            by[k].append((i, d))
        print(p)
        for k, ds in sorted(by.items()):
            print(f"  {k}  dispatches={len(ds)}")
            names = sorted({c for _, d in ds for c in d})
            if per:
                for i, d in ds:
                    print(f"    #{i}: " + ", ".join(f"{c}={d.get(c, 0):.0f}" for c in names))
            else:
                for c in names:
                    print(f"    {c:40s} {sum(d.get(c, 0) for _, d in ds) / len(ds):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
