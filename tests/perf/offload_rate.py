#!/usr/bin/env python3
"""Driver offload hooks timed on a 64 K-frame batch (libuinet_amd/frames.py):
uinet_cksum_tx_offload / uinet_cksum_rx_offload, staged and zero-copy,
against the reference object's own per-packet calls doing the same sums on
one thread (what the software stack runs for these packets).  Checks the
hooks' results against the oracle restatement."""
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
from libuinet_amd.frames import FrameBatch, pkthdr_fields  # noqa: E402


def best(fn, reps):
    t = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t = min(t, time.perf_counter() - t0)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    t0 = time.perf_counter()
    fb = FrameBatch(a.frames, seed=31)
    ref_fb = FrameBatch(a.frames, seed=31)
    print(f"built {a.frames} frames in {time.perf_counter() - t0:.1f}s", flush=True)
    O = oracle.Oracle()
    st_o = O.tx_offload(ref_fb.tx.heads)
    nbytes = int(sum(fb.tx.seg_len))
    res = {"frames": a.frames, "frame_bytes": nbytes}

    # TX: the hook rewrites sums in place; re-arm flags between repetitions
    def tx():
        fb.set_tx_flags()
        return u.tx_offload(fb.tx.heads)

    st = tx()
    res["tx_equal_oracle"] = bool(np.array_equal(st, st_o) and np.array_equal(fb.arena, ref_fb.arena))
    done = fb.arena.copy()
    # (repeats re-sum packets whose fields now hold final sums: same work)
    res["tx_staged_ms"] = round(best(tx, a.reps) * 1e3, 3)
    u.register_host(fb.arena)
    try:
        tx()
        res["tx_zero_copy_ms"] = round(best(tx, a.reps) * 1e3, 3)
    finally:
        u.unregister_host(fb.arena)
    fb.arena[:] = done

    rx, arena, _ = fb.rx(seed=7, corrupt=0.05)
    rx_o, _, _ = ref_fb.rx(seed=7, corrupt=0.05)
    want = O.rx_offload(rx_o.heads)

    def rxf():
        rx.mbufs["csum_flags"][:] = 0
        rx.mbufs["csum_data"][:] = 0
        return u.rx_offload(rx.heads)

    st = rxf()
    res["rx_equal_oracle"] = bool(np.array_equal(st, want) and all(
        np.array_equal(x, y) for x, y in zip(pkthdr_fields(rx), pkthdr_fields(rx_o))))
    res["rx_staged_ms"] = round(best(rxf, a.reps) * 1e3, 3)
    u.register_host(arena)
    try:
        rxf()
        res["rx_zero_copy_ms"] = round(best(rxf, a.reps) * 1e3, 3)
    finally:
        u.unregister_host(arena)

    if oracle.have_reference():
        R = oracle.Reference()
        # the same sums through the reference's per-packet functions, 1 thread
        l4 = np.flatnonzero((st_o & 1) != 0)
        ipd = np.flatnonzero((st_o & 2) != 0)
        first = rx_o.pkt_seg[:-1]
        ip_len = np.array([int.from_bytes(rx_o.arena[rx_o.seg_off[first[i]] + fb.l3[i] + 2:
                                                     rx_o.seg_off[first[i]] + fb.l3[i] + 4].tobytes(),
                                          "big") for i in range(fb.n)])
        txl = (fb.l3 + ip_len)[l4]
        txs = (fb.l3 + fb.hlen)[l4]
        t_tx = best(lambda: (R.skip_batch(ref_fb.tx.heads[l4], txl, txs),
                             R.skip_batch(ref_fb.tx.heads[ipd], (fb.l3 + fb.hlen)[ipd],
                                          fb.l3[ipd])), a.reps)
        ips = np.array([rx_o.arena.ctypes.data + rx_o.seg_off[first[i]] + fb.l3[i]
                        for i in ipd], np.uint64)
        proto = np.where(np.isin(fb.kinds[l4], ["udp"]), 17, 6)
        t_rx = best(lambda: (R.hdr_batch(ips),
                             R.pseudo_header_batch(rx_o.heads[l4], (ip_len - fb.hlen)[l4],
                                                   (fb.l3 + fb.hlen)[l4], fb.src[l4], fb.dst[l4],
                                                   proto)), a.reps)
        res["reference_1thread_tx_ms"] = round(t_tx * 1e3, 3)
        res["reference_1thread_rx_ms"] = round(t_rx * 1e3, 3)
        # the same calls split over the box's host threads (ctypes releases the
        # GIL, so the slices run in parallel on up to 16 cores)
        from concurrent.futures import ThreadPoolExecutor
        nt = min(16, len(os.sched_getaffinity(0)))
        pool = ThreadPoolExecutor(nt)

        def par(fn, idx):
            return list(pool.map(fn, np.array_split(idx, nt)))

        t_tx16 = best(lambda: (par(lambda k: R.skip_batch(ref_fb.tx.heads[l4][k], txl[k], txs[k]),
                                   np.arange(l4.size)),
                               par(lambda k: R.skip_batch(ref_fb.tx.heads[ipd][k],
                                                          (fb.l3 + fb.hlen)[ipd][k], fb.l3[ipd][k]),
                                   np.arange(ipd.size))), a.reps)
        plen4 = (ip_len - fb.hlen)[l4]
        off4 = (fb.l3 + fb.hlen)[l4]
        t_rx16 = best(lambda: (par(lambda k: R.hdr_batch(ips[k]), np.arange(ips.size)),
                               par(lambda k: R.pseudo_header_batch(rx_o.heads[l4][k], plen4[k], off4[k],
                                                                   fb.src[l4][k], fb.dst[l4][k],
                                                                   proto[k]), np.arange(l4.size))),
                      a.reps)
        pool.shutdown()
        res[f"reference_{nt}thread_tx_ms"] = round(t_tx16 * 1e3, 3)
        res[f"reference_{nt}thread_rx_ms"] = round(t_rx16 * 1e3, 3)
    for k in ("tx_staged", "tx_zero_copy", "rx_staged", "rx_zero_copy", "reference_1thread_tx",
              "reference_1thread_rx", "reference_16thread_tx", "reference_16thread_rx"):
        if f"{k}_ms" in res:
            res[f"{k}_gibs"] = round(nbytes / (res[f"{k}_ms"] * 1e-3) / 2**30, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
