#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the checksum kernels.

  kernel-trace stats -> mean/min duration per kernel (ns)
  --pmc FETCH_SIZE   -> HBM read bytes per dispatch = FETCH_SIZE * 1024 * 2
                        (gfx950: FETCH_SIZE counts half the bytes of a wide
                        16-B/lane streaming read -- MI355X_MICROARCH.md "HBM";
                        calibrated here on tools/hbm_read's known byte count)

Usage: pmc_summary.py <prof_dir> [--key KEY --bytes ALGO_BYTES] [--out json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics


def short(name: str) -> str:
    m = re.search(r"(k_\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2).replace(' ', '')}>"
    return name.split("(")[0][-60:]


def load_csv(d: str, suffix: str):
    files = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--kernel", default="k_")
    ap.add_argument("--key")
    ap.add_argument("--bytes", type=float, help="algorithmic bytes per dispatch")
    ap.add_argument("--out")
    ap.add_argument("--last", type=int, default=100,
                    help="also average the last N dispatches of each kernel (the bench's "
                         "timed launches; the first ones are its untimed warmup)")
    a = ap.parse_args()

    res = {}
    stats = load_csv(a.prof_dir, "kernel_stats.csv")
    for r in stats:
        if a.kernel in r["Name"]:
            res.setdefault(short(r["Name"]), {}).update(
                calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]),
                max_ns=float(r["MaxNs"]))
    trace = load_csv(a.prof_dir, "kernel_trace.csv")
    durs = {}
    for r in sorted(trace, key=lambda r: int(r["Start_Timestamp"])):
        if a.kernel in r["Kernel_Name"]:
            durs.setdefault(short(r["Kernel_Name"]), []).append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, d in durs.items():
        if k in res and a.last and len(d) > a.last:
            res[k][f"avg_ns_last{a.last}"] = statistics.mean(d[-a.last:])
    pmc = load_csv(a.prof_dir, "counter_collection.csv")
    per = {}
    for r in pmc:
        if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            per.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    for k, v in per.items():
        fs = statistics.mean(v)
        e = res.setdefault(k, {})
        e.update(fetch_size_kb_mean=fs, dispatches=len(v),
                 hbm_read_bytes_per_launch=fs * 1024 * 2)
        if a.bytes:
            e["traffic_over_algorithmic"] = fs * 1024 * 2 / a.bytes
    print(json.dumps(res, indent=1))
    if a.out and a.key:
        cur = {}
        if os.path.exists(a.out):
            with open(a.out) as fh:
                cur = json.load(fh)
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import kernel_src_sha

        for k, e in res.items():
            if "hbm_read_bytes_per_launch" in e:
                # src_sha: the kernel's sources at measurement time (bench.py
                # reports the traffic only while they are unchanged)
                cur[a.key] = dict(e, kernel=k, source=os.path.relpath(a.prof_dir),
                                  src_sha=kernel_src_sha(k))
        with open(a.out, "w") as fh:
            json.dump(cur, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
