#!/usr/bin/env python3
"""Config 1 (TCP echo call sequence, libuinet_amd/echo.py) timed end to end:
the reference's scalar calls (one thread, the stack's own per-packet loop)
against the engine's host-mbuf batch API, staged and zero-copy.  Each phase
is one batch call over all segments; the TX sums and RX verifications are
checked to be identical / zero for every engine."""
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
from libuinet_amd.echo import SEG, EchoBatch, GpuEngine  # noqa: E402


def run(echo, eng, rx):
    """One full sequence; returns per-phase seconds and the results."""
    t = {}
    echo.reset_tx()
    t0 = time.perf_counter()
    th = eng.skip_batch(echo.tx.heads, SEG, 20)
    t["tx_tcp"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    ip = eng.skip_batch(echo.tx.heads, 20, 0)
    t["tx_ip"] = time.perf_counter() - t0
    echo.arena[echo.hdr_off[:, None] + np.array([36, 37])] = th.view(np.uint8).reshape(-1, 2)
    echo.arena[echo.hdr_off[:, None] + np.array([10, 11])] = ip.view(np.uint8).reshape(-1, 2)
    ips = echo.rx_arena.ctypes.data + echo.rx_off.astype(np.uint64)
    t0 = time.perf_counter()
    hs = eng.hdr_batch(ips)
    t["rx_ip"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    ps = eng.pseudo_header_batch(rx.heads, SEG - 20, 20, echo.src, echo.dst, 6)
    t["rx_tcp"] = time.perf_counter() - t0
    return t, (th, ip, hs, ps)


def best(echo, eng, rx, reps):
    out = None
    bt = None
    for _ in range(reps):
        t, r = run(echo, eng, rx)
        if bt is None or sum(t.values()) < sum(bt.values()):
            bt, out = t, r
    return bt, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    echo = EchoBatch(args.packets)
    O = oracle.Oracle()
    echo.reset_tx()
    want = echo.transmit(O)
    rx = echo.deliver_fast()
    engines = {"gpu_staged": GpuEngine()}
    if oracle.have_reference():
        engines = {"reference_1thread": oracle.Reference(), **engines}
    res = {"packets": args.packets, "segment_bytes": SEG,
           "bytes_per_sequence": args.packets * (2 * (SEG - 20) + 2 * 20)}
    for name, eng in list(engines.items()) + [("gpu_zero_copy", engines["gpu_staged"])]:
        if name == "gpu_zero_copy":
            u.register_host(echo.arena)
            u.register_host(echo.rx_arena)
        try:
            run(echo, eng, rx)
            t, (th, ip, hs, ps) = best(echo, eng, rx, args.reps)
        finally:
            if name == "gpu_zero_copy":
                u.unregister_host(echo.arena)
                u.unregister_host(echo.rx_arena)
        tot = sum(t.values())
        e = {k: round(v * 1e3, 3) for k, v in t.items()}
        e.update(total_ms=round(tot * 1e3, 3),
                 segments_per_s=round(args.packets / tot),
                 gibs=round(res["bytes_per_sequence"] / tot / 2**30, 2),
                 tx_equal=bool(np.array_equal(th, want[0]) and np.array_equal(ip, want[1])),
                 rx_all_zero=bool(not hs.any() and not ps.any()))
        res[name] = e
        print(name, e, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
