#!/usr/bin/env python3
"""Instruction counters per KiB of algorithmic bytes for one kernel family,
from a rocprofv3 --pmc directory (SQ_INSTS_* are per-wave instruction counts
summed over the dispatch).

Usage: insts_summary.py <pmc_dir> --kernel k_chains_pipe --bytes ALGO_BYTES
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--bytes", type=float, required=True, help="algorithmic bytes per dispatch")
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    names = set()
    for f in glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                names.add(r["Kernel_Name"].split("(")[0])
    kib = a.bytes / 1024
    out = {"kernel": sorted(names), "algorithmic_kib": kib}
    for k, v in sorted(vals.items()):
        m = sum(v) / len(v)
        out[k] = {"per_dispatch": m, "dispatches": len(v), "per_kib": round(m / kib, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
