#!/usr/bin/env python3
"""Host-resident rates: the host-mbuf batch API (staging vs zero-copy over a
registered region) against the reference's scalar in_cksum_skip on the same
host mbufs.  Config-2 shape (1500-B packets, one mbuf each) and config-3
shape (mixed lengths chained into 1..256-B mbufs, skip 20)."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: F401,E402  (one HIP runtime)

import libuinet_amd as u  # noqa: E402
import oracle  # noqa: E402
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes  # noqa: E402
from libuinet_amd.workloads import build_config3  # noqa: E402


def best(fn, reps=5):
    t = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        t = min(t, time.perf_counter() - t0)
    return t, r


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c2,c3", help="c2 (65,536 and 1 M x 1500 B), c3")
    ap.add_argument("--no-reference", action="store_true", help="engine only (A/B runs)")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    R = oracle.Reference() if oracle.have_reference() and not a.no_reference else None
    res = {}
    shapes = []
    for n in ((65536, 1 << 20) if "c2" in a.shapes else ()):
        arena = aligned_empty(1500 * n + 64)
        splitmix64_bytes(arena.size, 2, out=arena)
        ch = MbufChains.contiguous(arena, 1500 * np.arange(n), 1500)
        shapes.append((f"c2_{n}", arena, ch, 1500, 0, n * 1500))
    if "c3" in a.shapes:
        c3 = build_config3(1 << 18, seed=3)
        ch3 = MbufChains(c3["arena"], c3["seg_off"], c3["seg_len"], c3["pkt_seg"])
        shapes.append(("c3_262144", c3["arena"], ch3, c3["lens"], 20,
                       int((c3["lens"] - 20).sum())))
    for name, arena, ch, ln, sk, nbytes in shapes:
        gib = nbytes / 2**30
        u.in_cksum_skip_batch(ch.heads, ln, sk)
        t_stage, r_stage = best(lambda: u.in_cksum_skip_batch(ch.heads, ln, sk), a.reps)
        u.register_host(arena)
        try:
            u.in_cksum_skip_batch(ch.heads, ln, sk)
            t_zc, r_zc = best(lambda: u.in_cksum_skip_batch(ch.heads, ln, sk), a.reps)
        finally:
            u.unregister_host(arena)
        e = {"staging_gibs": round(gib / t_stage, 2), "zero_copy_gibs": round(gib / t_zc, 2),
             "equal": bool(np.array_equal(r_stage, r_zc))}
        if R is not None:
            t1, r1 = R.time_skip(ch.heads, ln, sk, nthreads=1, reps=3)
            e["reference_1thread_gibs"] = round(gib / t1, 2)
            cpus = sorted(os.sched_getaffinity(0))[:16]
            # 16 threads pinned to the first CPUs of the mask, and floating:
            # the faster is the baseline (profiles/r02/host_pin/)
            t16p, r16 = R.time_skip(ch.heads, ln, sk, nthreads=len(cpus), cpus=cpus, reps=5)
            t16f, r16f = R.time_skip(ch.heads, ln, sk, nthreads=len(cpus), cpus=None, reps=5)
            t16 = min(t16p, t16f)
            e[f"reference_{len(cpus)}thread_gibs"] = round(gib / t16, 2)
            e[f"reference_{len(cpus)}thread_pinned_gibs"] = round(gib / t16p, 2)
            e[f"reference_{len(cpus)}thread_floating_gibs"] = round(gib / t16f, 2)
            e["equal_reference"] = bool(np.array_equal(r1, r_zc) and np.array_equal(r16, r_zc)
                                        and np.array_equal(r16f, r_zc))
        res[name] = e
        print(name, e, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
