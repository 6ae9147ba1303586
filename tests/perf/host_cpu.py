#!/usr/bin/env python3
"""What the GPU path costs the host CPU (SURVEY.md section 7
step 7): every host-resident path timed for wall time AND host CPU time, per
1,000 packets, at host_threads 1 and 16, beside the reference object's own
scalar functions on one thread over the same mbufs.

Engine CPU time comes from uinet_cksum_host_cpu (include/uinet_cksum.h 2f):
CLOCK_THREAD_CPUTIME_ID of the calling thread inside the call, plus the CPU
time of the engine's host-pool helpers spent on it.  The reference's CPU time
is time.thread_time() around its single-threaded call (a scalar loop: CPU time
= wall time).

Engine paths per workload:
  staged      the host walks the chains and packs the bytes into pinned staging
              (nothing registered)
  zero_copy   the packet bytes are registered; the host walks the chains and
              writes descriptors, the GPU reads the bytes in place over PCIe
  span_gpu    bytes AND mbufs registered, one mbuf per packet: the span path
              with the head mbufs read by the GPU (k_span_walk)
  dev_walk    bytes AND mbufs registered; the GPU walks the chains and folds
              their bytes in one launch (csrc/cksum_mbufs.hip, knob walk_device
              3) -- the host only writes the jobs
  dev_walk2   the same, walked into a segment list (csrc/cksum_walk.hip) and
              folded by the chain kernel (knob walk_device 2)

Workloads: c2 (1,048,576 x 1500-B packets, one mbuf each), c3 (262,144
config-3 chains of 1..256-B mbufs, skip 20), the RX and TX offload hooks on
65,536 mixed frames, and config 1's echo call sequence on 65,536 segments.
Prints one JSON object per row and a final JSON summary."""
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
from libuinet_amd.workloads import build_config3  # noqa: E402


def meter(fn, reps):
    """Median-wall rep of fn(): wall ms and the engine's host CPU counters."""
    rows = []
    out = None
    for _ in range(reps):
        u.host_cpu(reset=True)
        t0 = time.perf_counter()
        out = fn()
        wall = time.perf_counter() - t0
        rows.append((wall, u.host_cpu(reset=True)))
    rows.sort(key=lambda r: r[0])
    wall, st = rows[len(rows) // 2]
    return {"wall_ms": round(wall * 1e3, 3), "cpu_ms": round(st["cpu_ns"] / 1e6, 3),
            "_st": st,
            "caller_cpu_ms": round(st["caller_cpu_ns"] / 1e6, 3),
            "helper_cpu_ms": round(st["helper_cpu_ns"] / 1e6, 3),
            "calls": st["calls"], "device_walks": st["device_walks"],
            "cpu_ms_all_reps": [round(r[1]["cpu_ns"] / 1e6, 3) for r in rows]}, out


def ref_meter(fn, reps):
    best = None
    out = None
    for _ in range(reps):
        c0, t0 = time.thread_time(), time.perf_counter()
        out = fn()
        w, c = time.perf_counter() - t0, time.thread_time() - c0
        if best is None or w < best[0]:
            best = (w, c)
    return {"wall_ms": round(best[0] * 1e3, 3), "cpu_ms": round(best[1] * 1e3, 3)}, out


def per_k(e, n, nbytes):
    e["cpu_us_per_1k_pkts"] = round(e["cpu_ms"] * 1e3 / (n / 1000), 3)
    e["wall_us_per_1k_pkts"] = round(e["wall_ms"] * 1e3 / (n / 1000), 3)
    e["gibs"] = round(nbytes / (e["wall_ms"] * 1e-3) / 2**30, 2)
    return e


class Regs:
    """Registers the given buffers for one path (and unregisters them)."""

    def __init__(self, bufs):
        self.bufs = bufs

    def __enter__(self):
        for b in self.bufs:
            u.register_host(b)

    def __exit__(self, *a):
        for b in self.bufs:
            u.unregister_host(b)


PATHS = ("staged", "zero_copy", "dev_walk")


def run_paths(name, n, nbytes, fn, bytes_bufs, mbuf_bufs, threads, reps, check, res):
    """Every engine path x host_threads for one workload; check(out) -> bool."""
    paths = (("staged", []), ("zero_copy", bytes_bufs), ("span", bytes_bufs),
             ("span_gpu", bytes_bufs + mbuf_bufs),
             ("dev_walk", bytes_bufs + mbuf_bufs), ("dev_walk2", bytes_bufs + mbuf_bufs))
    for path, bufs in paths:
        if path not in PATHS:
            continue
        for t in threads:
            u.set_tuning("host_threads", t)
            # dev_walk: the fused walk + fold (walk_device 3); dev_walk2: the
            # walk into a segment list, then the chain kernel (walk_device 2)
            u.set_tuning("walk_device", 2 if path == "dev_walk2" else 3)
            # span: the single-mbuf span path (only one-mbuf sums take it);
            # the other paths with it off
            u.set_tuning("span_fast", 1 if path in ("span", "span_gpu") else 0)
            with Regs(bufs):
                fn()  # warm: staging buffers, pool threads, walk row size
                e, out = meter(fn, reps)
            u.set_tuning("walk_device", 1)
            u.set_tuning("span_fast", 1)
            e["span_batches"] = e.pop("_st")["span_batches"]
            e = per_k(e, n, nbytes)
            e["bit_identical"] = bool(check(out))
            key = f"{name}/{path}/{t}t"
            res[key] = e
            print(json.dumps({key: e}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default="c2,c3,hooks,echo")
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--c2-packets", type=int, default=1 << 20)
    ap.add_argument("--c3-packets", type=int, default=1 << 18)
    ap.add_argument("--paths", default="staged,zero_copy,dev_walk")
    a = ap.parse_args()
    global PATHS
    PATHS = tuple(a.paths.split(","))
    threads = [int(x) for x in a.threads.split(",")]
    work = a.work.split(",")
    R = oracle.Reference() if oracle.have_reference() else None
    O = oracle.Oracle()
    res = {"threads": threads, "reps": a.reps,
           "reference": "oracle/_ref (the reference's in_cksum.c)" if R else "oracle port"}
    ref = R if R is not None else O

    if "c2" in work:
        n = a.c2_packets
        arena = aligned_empty(1500 * n + 64)
        splitmix64_bytes(arena.size, 2, out=arena)
        ch = MbufChains.contiguous(arena, 1500 * np.arange(n), 1500)
        want = O.skip_batch(ch.heads, 1500, 0)
        e, _ = ref_meter(lambda: ref.skip_batch(ch.heads, 1500, 0), 3)
        res["c2/reference/1t"] = per_k(e, n, 1500 * n)
        print(json.dumps({"c2/reference/1t": e}), flush=True)
        run_paths("c2", n, 1500 * n, lambda: u.in_cksum_skip_batch(ch.heads, 1500, 0),
                  [arena], [ch.mbufs], threads, a.reps, lambda o: np.array_equal(o, want), res)
        del arena, ch
    if "c3" in work:
        c3 = build_config3(a.c3_packets, seed=3)
        ch3 = MbufChains(c3["arena"], c3["seg_off"], c3["seg_len"], c3["pkt_seg"])
        n = ch3.n
        nb = int((c3["lens"] - 20).sum())
        want = O.skip_batch(ch3.heads, c3["lens"], 20)
        e, _ = ref_meter(lambda: ref.skip_batch(ch3.heads, c3["lens"], 20), 3)
        res["c3/reference/1t"] = per_k(e, n, nb)
        print(json.dumps({"c3/reference/1t": e}), flush=True)
        run_paths("c3", n, nb, lambda: u.in_cksum_skip_batch(ch3.heads, c3["lens"], 20),
                  [c3["arena"]], [ch3.mbufs], threads, a.reps, lambda o: np.array_equal(o, want),
                  res)
        del c3, ch3
    if "hooks" in work:
        from libuinet_amd.frames import FrameBatch

        nf = 65536
        fb = FrameBatch(nf, seed=31)
        ref_fb = FrameBatch(nf, seed=31)
        nbytes = int(sum(fb.tx.seg_len))
        st_o = O.tx_offload(ref_fb.tx.heads)

        def tx():
            fb.set_tx_flags()
            return u.tx_offload(fb.tx.heads)

        run_paths("tx_hook", nf, nbytes, tx, [fb.arena], [fb.tx.mbufs], threads, a.reps,
                  lambda o: np.array_equal(o, st_o), res)
        # the repeated TX runs re-summed fields that already held final sums:
        # back to the state after one TX pass (the oracle's) before RX
        fb.arena[:] = ref_fb.arena
        rx, arena_rx, _ = fb.rx(seed=7, corrupt=0.05)
        rx_o, _, _ = ref_fb.rx(seed=7, corrupt=0.05)
        want_rx = O.rx_offload(rx_o.heads)

        def rxf():
            rx.mbufs["csum_flags"][:] = 0
            rx.mbufs["csum_data"][:] = 0
            return u.rx_offload(rx.heads)

        run_paths("rx_hook", nf, nbytes, rxf, [arena_rx], [rx.mbufs], threads, a.reps,
                  lambda o: np.array_equal(o, want_rx), res)
        # the reference's per-packet calls doing the same sums, one thread
        # (tests/perf/offload_rate.py restates which calls)
        l4 = np.flatnonzero((st_o & 1) != 0)
        ipd = np.flatnonzero((st_o & 2) != 0)
        first = rx_o.pkt_seg[:-1]
        ip_len = np.array([int.from_bytes(rx_o.arena[rx_o.seg_off[first[i]] + fb.l3[i] + 2:
                                                     rx_o.seg_off[first[i]] + fb.l3[i] + 4].tobytes(),
                                          "big") for i in range(nf)])
        txl, txs = (fb.l3 + ip_len)[l4], (fb.l3 + fb.hlen)[l4]
        e, _ = ref_meter(lambda: (ref.skip_batch(ref_fb.tx.heads[l4], txl, txs),
                                  ref.skip_batch(ref_fb.tx.heads[ipd], (fb.l3 + fb.hlen)[ipd],
                                                 fb.l3[ipd])), a.reps)
        res["tx_hook/reference/1t"] = per_k(e, nf, nbytes)
        ips = np.array([rx_o.arena.ctypes.data + rx_o.seg_off[first[i]] + fb.l3[i] for i in ipd],
                       np.uint64)
        proto = np.where(np.isin(fb.kinds[l4], ["udp"]), 17, 6)
        e, _ = ref_meter(lambda: (ref.hdr_batch(ips),
                                  ref.pseudo_header_batch(rx_o.heads[l4], (ip_len - fb.hlen)[l4],
                                                          (fb.l3 + fb.hlen)[l4], fb.src[l4],
                                                          fb.dst[l4], proto)), a.reps)
        res["rx_hook/reference/1t"] = per_k(e, nf, nbytes)
        print(json.dumps({k: res[k] for k in ("tx_hook/reference/1t", "rx_hook/reference/1t")}),
              flush=True)
    if "echo" in work:
        from libuinet_amd.echo import SEG, EchoBatch, GpuEngine

        ne = 65536
        echo = EchoBatch(ne)
        echo.reset_tx()
        want = echo.transmit(O)
        rxc = echo.deliver_fast()
        nbytes = ne * (2 * (SEG - 20) + 2 * 20)

        def seq(eng):
            echo.reset_tx()
            th = eng.skip_batch(echo.tx.heads, SEG, 20)
            ip = eng.skip_batch(echo.tx.heads, 20, 0)
            echo.arena[echo.hdr_off[:, None] + np.array([36, 37])] = th.view(np.uint8).reshape(-1, 2)
            echo.arena[echo.hdr_off[:, None] + np.array([10, 11])] = ip.view(np.uint8).reshape(-1, 2)
            ips = echo.rx_arena.ctypes.data + echo.rx_off.astype(np.uint64)
            hs = eng.hdr_batch(ips)
            ps = eng.pseudo_header_batch(rxc.heads, SEG - 20, 20, echo.src, echo.dst, 6)
            return th, ip, hs, ps

        def ok(r):
            th, ip, hs, ps = r
            return (np.array_equal(th, want[0]) and np.array_equal(ip, want[1])
                    and not hs.any() and not ps.any())

        eng = GpuEngine()
        run_paths("echo", ne, nbytes, lambda: seq(eng), [echo.arena, echo.rx_arena],
                  [echo.tx.mbufs, rxc.mbufs], threads, a.reps, ok, res)
        e, r = ref_meter(lambda: seq(ref), a.reps)
        e["bit_identical"] = bool(ok(r))
        res["echo/reference/1t"] = per_k(e, ne, nbytes)
        print(json.dumps({"echo/reference/1t": e}), flush=True)
    u.set_tuning("host_threads", min(16, os.cpu_count() or 1))
    try:  # how much of the process is on transparent huge pages (UINET_MBUF_HUGEPAGES)
        with open("/proc/self/smaps_rollup") as f:
            res["anon_huge_kb"] = int(next(ln for ln in f if ln.startswith("AnonHugePages")).split()[1])
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as f:
            res["thp_mode"] = f.read().strip()
    except (OSError, StopIteration, ValueError):
        pass
    res["hugepages_env"] = os.environ.get("UINET_MBUF_HUGEPAGES", "")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
