#!/usr/bin/env python3
"""Mean per-dispatch PMC values of the engine's kernels from pmc_sets.sh output."""
import csv, glob, statistics, sys, collections, re
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+<[^>]*>)", r["Kernel_Name"])
        if m:
            d[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in d.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {statistics.mean(v):16.1f}")
