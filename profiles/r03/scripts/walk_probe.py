#!/usr/bin/env python3
"""Why does the zero-copy batch walk config 3 slower than the staged batch?
Times the staged host batch (per-phase trace on stderr) with the arena
unregistered, then with an unrelated buffer registered (so batches still take
the staged path after one group's walk), then the zero-copy batch with the
arena registered, then the staged batch again after unregistering it."""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("UINET_CKSUM_TRACE_HOST", "1")
import torch  # noqa: F401,E402

import libuinet_amd as u  # noqa: E402
from libuinet_amd.mbuf import MbufChains, aligned_empty  # noqa: E402
from libuinet_amd.workloads import build_config3  # noqa: E402


def run(tag, ch, ln, reps=4):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        u.in_cksum_skip_batch(ch.heads, ln, 20)
        ts.append(time.perf_counter() - t0)
    print(f"{tag}: best {min(ts) * 1e3:.3f} ms", flush=True)
    sys.stderr.write(f"== {tag}\n")


def main():
    c3 = build_config3(1 << 18, seed=3)
    ch = MbufChains(c3["arena"], c3["seg_off"], c3["seg_len"], c3["pkt_seg"])
    ln = c3["lens"]
    run("staged, nothing registered", ch, ln)
    other = aligned_empty(1 << 20)
    u.register_host(other)
    run("staged after a zero-copy attempt (an unrelated buffer registered)", ch, ln)
    u.unregister_host(other)
    u.register_host(c3["arena"])
    run("zero-copy, arena registered", ch, ln)
    u.unregister_host(c3["arena"])
    run("staged, arena unregistered again", ch, ln)


if __name__ == "__main__":
    main()
