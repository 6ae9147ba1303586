#!/usr/bin/env python3
"""Latency of the per-call drop-in ABI (a GPU batch of one) and of host
batches of various sizes, vs the reference object on the same host mbufs."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: F401  (one HIP runtime)
import libuinet_amd as u
import oracle
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes

arena = aligned_empty(1500 * 65536 + 64)
splitmix64_bytes(arena.size, 1, out=arena)
ch = MbufChains.contiguous(arena, 1500 * np.arange(65536), 1500)
res = {}
h = ch.head(0)
for _ in range(100):
    u.in_cksum_skip(h, 1500, 0)
t0 = time.perf_counter(); N = 2000
for i in range(N):
    u.in_cksum_skip(ch.head(i), 1500, 0)
res["per_call_in_cksum_skip_us"] = (time.perf_counter() - t0) / N * 1e6
R = oracle.Reference() if oracle.have_reference() else None
if R:
    t0 = time.perf_counter()
    for i in range(N):
        R.cksum_skip(ch.head(i), 1500, 0)
    res["per_call_reference_us_incl_ctypes"] = (time.perf_counter() - t0) / N * 1e6
for nb in (64, 1024, 16384, 65536):
    heads = ch.heads[:nb]
    u.in_cksum_skip_batch(heads, 1500, 0)
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter(); u.in_cksum_skip_batch(heads, 1500, 0); best = min(best, time.perf_counter() - t0)
    res[f"host_batch_{nb}_us"] = best * 1e6
    res[f"host_batch_{nb}_gibs"] = nb * 1500 / best / 2**30
print(json.dumps(res, indent=1))
