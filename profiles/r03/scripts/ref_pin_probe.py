#!/usr/bin/env python3
"""The reference's 16-thread in_cksum_skip on host mbufs with its threads
pinned to the first 16 CPUs of the process mask (what bench.py's
cpu_baseline does) and left to the scheduler, alternating; median of 5 each.
Config 2 (1 M x 1500 B, one mbuf each) and config 3 (262 K chained)."""
from __future__ import annotations

import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes  # noqa: E402
from libuinet_amd.workloads import build_config3  # noqa: E402


def main():
    R = oracle.Reference()
    allowed = sorted(os.sched_getaffinity(0))
    res = {"cpus_in_mask": len(allowed), "os_cpu_count": os.cpu_count()}
    n = 1 << 20
    arena = aligned_empty(1500 * n + 64)
    splitmix64_bytes(arena.size, 2, out=arena)
    c2 = MbufChains.contiguous(arena, 1500 * np.arange(n), 1500)
    c3 = build_config3(1 << 18, seed=3)
    ch3 = MbufChains(c3["arena"], c3["seg_off"], c3["seg_len"], c3["pkt_seg"])
    shapes = [("c2", c2.heads, np.full(n, 1500), np.zeros(n), n * 1500),
              ("c3", ch3.heads, c3["lens"], np.full(c3["lens"].size, 20), int((c3["lens"] - 20).sum()))]
    for name, heads, ln, sk, nbytes in shapes:
        t = {"pinned": [], "floating": []}
        for _ in range(5):
            t["pinned"].append(R.time_skip(heads, ln, sk, nthreads=16, cpus=allowed[:16], reps=1)[0])
            t["floating"].append(R.time_skip(heads, ln, sk, nthreads=16, cpus=None, reps=1)[0])
        res[name] = {k: round(nbytes / statistics.median(v) / 2**30, 2) for k, v in t.items()}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
