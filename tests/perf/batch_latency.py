#!/usr/bin/env python3
"""Latency and host CPU of SMALL host-mbuf batches and hook batches, per path:
staged (nothing registered), zero-copy (bytes registered, the host walks) and
device (bytes and mbufs registered: the GPU walks; for the hooks it also parses
and writes the verdicts).  Median of many calls per size.  Decides where the
device path starts to pay in latency (round 5; DESIGN.md "Host CPU time")."""
from __future__ import annotations

import argparse
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


def med(fn, reps):
    ws, cs = [], []
    for _ in range(reps):
        u.host_cpu(reset=True)
        t0 = time.perf_counter()
        out = fn()
        ws.append(time.perf_counter() - t0)
        cs.append(u.host_cpu(reset=True)["cpu_ns"] / 1e3)
    return round(float(np.median(ws)) * 1e6, 1), round(float(np.median(cs)), 1), out


class Regs:
    def __init__(self, bufs):
        self.bufs = bufs

    def __enter__(self):
        for b in self.bufs:
            u.register_host(b)

    def __exit__(self, *a):
        for b in self.bufs:
            u.unregister_host(b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=60)
    a = ap.parse_args()
    O = oracle.Oracle()
    res = {"reps": a.reps}
    n_max = 16384
    arena = aligned_empty(1500 * n_max + 64)
    splitmix64_bytes(arena.size, 1, out=arena)
    ch = MbufChains.contiguous(arena, 1500 * np.arange(n_max), 1500)
    u.set_tuning("host_threads", 1)
    for nb in (1, 8, 64, 256, 1024, 4096, 16384):
        heads = ch.heads[:nb]
        want = O.skip_batch(heads, 1500, 0)
        row = {}
        for path, bufs in (("staged", []), ("zero_copy", [arena]), ("device", [arena, ch.mbufs])):
            with Regs(bufs):
                u.in_cksum_skip_batch(heads, 1500, 0)
                w, c, out = med(lambda: u.in_cksum_skip_batch(heads, 1500, 0), a.reps)
            row[path] = {"us": w, "cpu_us": c, "ok": bool(np.array_equal(out, want))}
        res[f"skip_batch_{nb}"] = row
        print(json.dumps({f"skip_batch_{nb}": row}), flush=True)
    from libuinet_amd.frames import FrameBatch

    for nf in (16, 64, 256, 1024, 4096):
        fb = FrameBatch(nf, seed=3)
        rx, arena_rx, _ = fb.rx(seed=4, corrupt=0.0)
        want = None
        row = {}
        for path, bufs in (("staged", []), ("zero_copy", [arena_rx]),
                           ("device", [arena_rx, rx.mbufs])):
            def f():
                rx.mbufs["csum_flags"][:] = 0
                rx.mbufs["csum_data"][:] = 0
                return u.rx_offload(rx.heads)
            with Regs(bufs):
                f()
                w, c, out = med(f, a.reps)
            want = out if want is None else want
            row[path] = {"us": w, "cpu_us": c, "ok": bool(np.array_equal(out, want))}
        res[f"rx_hook_{nf}"] = row
        print(json.dumps({f"rx_hook_{nf}": row}), flush=True)
    u.set_tuning("host_threads", min(16, os.cpu_count() or 1))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
