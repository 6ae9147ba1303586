#!/usr/bin/env python3
"""Host-resident long packets through the host-mbuf batch API: 131,072 x
9000-B frames in registered host memory (zero-copy, folded over PCIe), with
the chain kernel forced to the 32-packet tile kernel (knob chains_wide 1) or
one wave per packet (2), alternating; the host walk (bytes registered) and
the device walk (mbufs registered too).  Prints one JSON line per mode."""
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


def main():
    n, ln = 131072, 9000
    arena = aligned_empty(n * ln + 64)
    splitmix64_bytes(arena.size, 77, out=arena)
    ch = MbufChains.contiguous(arena, ln * np.arange(n, dtype=np.int64), ln)
    length = np.full(n, ln, np.int64)
    want = oracle.Oracle().skip_batch(ch.heads[:4096], length[:4096], 20)
    res = {}
    for mode, regs in (("host_walk", (arena,)), ("device_walk", (arena, ch.mbufs))):
        for b in regs:
            u.register_host(b)
        try:
            for r in range(3):
                for wide in (1, 2):
                    u.set_tuning("chains_wide", wide)
                    t0 = time.perf_counter()
                    got = u.in_cksum_skip_batch(ch.heads, length, 20)
                    dt = time.perf_counter() - t0
                    assert np.array_equal(got[:4096], want), (mode, wide)
                    res.setdefault((mode, wide), []).append(dt)
        finally:
            u.set_tuning("chains_wide", 0)
            for b in regs:
                u.unregister_host(b)
    for (mode, wide), ts in sorted(res.items()):
        print(json.dumps({"mode": mode, "chains_wide": wide, "ms": [round(1e3 * t, 2) for t in ts],
                          "best_GBps": round(n * (ln - 20) / min(ts) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
