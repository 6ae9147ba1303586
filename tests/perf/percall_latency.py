#!/usr/bin/env python3
"""Latency of the per-call drop-in ABI (a host fold on the calling thread)
and of host batches of various sizes (GPU), vs the reference object on the
same host mbufs.  The per-call numbers come twice: through ctypes, and from
tests/perf/percall_bench.c (plain C, no interpreter in the loop)."""
import json, os, subprocess, sys, tempfile, time
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
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if R:
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "percall_bench")
        lib, ref = os.path.join(REPO, "libuinet_amd"), os.path.join(REPO, "oracle", "_ref")
        subprocess.run(["gcc", "-O2", "-std=c11", "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "perf", "percall_bench.c"), "-L", lib,
                        "-luinet_cksum", f"-Wl,-rpath,{lib}", os.path.join(ref, "libref_cksum.so"),
                        f"-Wl,-rpath,{ref}", "-o", exe], check=True)
        res["c_percall"] = [json.loads(subprocess.run([exe, str(n)], capture_output=True, text=True,
                                                      check=True).stdout) for n in (64, 1500, 9000)]
print(json.dumps(res, indent=1))
