#!/usr/bin/env python3
"""Markdown table of a measurement set (profiles/r04/scripts/r04_set.sh / prof_all.sh):
one row per bench_<tag>.log, with its trace and FETCH_SIZE summaries.

Usage: set_table.py profiles/r04/r04s1 [profiles/r04/r04s2 ...]"""
from __future__ import annotations

import glob
import json
import os
import sys


def line(path):
    with open(path) as f:
        ls = [x for x in f if x.startswith("{")]
    return json.loads(ls[-1]) if ls else None


def main():
    print("| config | kernel | ms / launch | achieved | frac | trace avg (µs) | traffic ÷ algorithmic "
          "| reference 1 thread / 16 floating / 16 pinned (GiB/s) | bit-identical |")
    print("|---|---|---|---|---|---|---|---|---|")
    for d in sys.argv[1:]:
        for b in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
            tag = os.path.basename(b)[len("bench_"):-len(".log")]
            j = line(b)
            if j is None:
                continue
            r = j["roofline"]
            tr = os.path.join(d, f"trace_{tag}.summary.json")
            pm = os.path.join(d, f"pmc_{tag}.summary.json")
            tavg = ""
            if os.path.exists(tr):
                t = json.load(open(tr))
                k = r.get("instance")
                if k in t:
                    tavg = f"{t[k].get('avg_ns', 0) / 1e3:.1f}"
            traf = ""
            if os.path.exists(pm):
                p = json.load(open(pm))
                k = r.get("instance")
                if k in p and "traffic_over_algorithmic" in p[k]:
                    traf = f"{p[k]['traffic_over_algorithmic']:.3f}"
            cb = j.get("cpu_baseline", {}).get("runs_gibs", {})
            ref = " / ".join(str(cb.get(k, "")) for k in ("1_floating", "16_floating", "16_pinned"))
            lf = r.get("layout_floor")
            frac = f"{r['frac']:.3f}" + (f" ({lf['frac']:.3f} floor)" if lf else "")
            print(f"| {tag} | `{r.get('instance', r['kernel'])}` | {r['kernel_ms_mean']:.4f} | "
                  f"{r['achieved'] / 1000:.2f} TB/s | {frac} | {tavg} | {traf} | {ref} | "
                  f"{j.get('bit_identical')} |")


if __name__ == "__main__":
    main()
