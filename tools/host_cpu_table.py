#!/usr/bin/env python3
"""Markdown table of tests/perf/host_cpu.py runs: for each workload, the
median over the given runs (processes) of wall ms, host CPU ms and host CPU
µs per 1,000 packets, per engine path and host_threads, beside the
reference's one-thread figures.

Usage: host_cpu_table.py run1.log [run2.log ...]"""
from __future__ import annotations

import json
import statistics
import sys

WORK = (("c2", "host-mbuf batch, config 2 (1,048,576 x 1500 B, one mbuf each)"),
        ("c3", "host-mbuf batch, config 3 (262,144 chains of 1..256-B mbufs, skip 20)"),
        ("tx_hook", "TX offload hook, 65,536 mixed frames"),
        ("rx_hook", "RX offload hook, 65,536 mixed frames"),
        ("echo", "config 1, echo TX + RX call sequence, 65,536 segments"))
PATHS = ("staged", "zero_copy", "span", "span_gpu", "dev_walk", "dev_walk2")


def load(path):
    lines = [ln for ln in open(path) if ln.startswith('{"threads"')]
    return json.loads(lines[-1])


def med(runs, key, field):
    vals = [r[key][field] for r in runs if key in r]
    return statistics.median(vals) if vals else None


def main():
    runs = [load(p) for p in sys.argv[1:]]
    threads = runs[0]["threads"]
    print("| workload | path | " + " | ".join(f"{t} thread{'s' if t > 1 else ''}: wall ms / CPU ms (CPU µs per 1k pkts)" for t in threads) + " |")
    print("|---|---|" + "---|" * len(threads))
    for w, title in WORK:
        ref = f"{w}/reference/1t"
        if not any(ref in r for r in runs) and not any(f"{w}/staged/{threads[0]}t" in r for r in runs):
            continue
        for p in PATHS:
            cells = []
            for t in threads:
                k = f"{w}/{p}/{t}t"
                if med(runs, k, "wall_ms") is None:
                    cells.append("—")
                    continue
                ok = all(r[k].get("bit_identical", True) for r in runs if k in r)
                cells.append(f"{med(runs, k, 'wall_ms'):.2f} / {med(runs, k, 'cpu_ms'):.2f} "
                             f"({med(runs, k, 'cpu_us_per_1k_pkts'):.1f}){'' if ok else ' MISMATCH'}")
            print(f"| {title} | engine, {p.replace('_', '-')} | " + " | ".join(cells) + " |")
        if med(runs, ref, "wall_ms") is not None:
            print(f"| {title} | reference, 1 thread | {med(runs, ref, 'wall_ms'):.2f} / "
                  f"{med(runs, ref, 'cpu_ms'):.2f} ({med(runs, ref, 'cpu_us_per_1k_pkts'):.1f})"
                  + " | —" * (len(threads) - 1) + " |")


if __name__ == "__main__":
    main()
