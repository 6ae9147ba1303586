#!/usr/bin/env python3
"""Interleaved A/B of engine tuning variants in ONE process (so DVFS and
device-to-device spread hit every variant alike).

  python tools/ab.py --config 3 --variants 'chains_long=128' 'chains_long=0'

Each variant is a comma list of key=value pairs for uinet_cksum_set_tuning;
the pseudo-key desc=1 launches with packed descriptors (uinet_cksum_spans32 /
uinet_cksum_chains32) instead of wide ones (desc=0, the default).
Prints one JSON object: per variant the median / min kernel ms and GB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# the engine's knob defaults (include/uinet_cksum.h); host_threads defaults to
# min(16, hardware threads)
DEFAULTS = {"blocks_per_cu": 0, "chains_long": 128, "xcd_remap": 1, "multi_gather": 0,
            "chains_wide": 0, "walk_device": 1,
            "host_threads": min(16, os.cpu_count() or 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="2")
    ap.add_argument("--api", default="spans")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--packets", type=int, default=None, help="batch size (default: the config's)")
    a = ap.parse_args()
    import torch

    import bench
    import libuinet_amd as u

    w = bench.build_workload(a.config, a.packets, 0)
    out = torch.empty(w["n"], dtype=torch.uint16, device="cuda")
    s = torch.cuda.current_stream()
    if a.config in bench.CHAIN_CONFIGS:
        w["packed"] = u.pack_segments(w["seg_off"], w["seg_len"])
    elif a.api == "spans":
        w["packed"] = u.pack_segments(w["off"], w["len"])
    launches = {0: bench.make_launch(a.config, w, a.api, out),
                1: bench.make_launch(a.config, w, a.api, out, "packed") if "packed" in w else None}
    variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv)
                for v in a.variants]
    # Every key any variant names goes back to its default before each variant
    # is applied.  (Until round 3 a variant inherited the keys the previous one
    # had set, so e.g. "xcd_remap=1" after "blocks_per_cu=4096" ran at 4096.)
    for v in variants:
        for k in v:
            if k == "desc":
                if launches.get(v[k]) is None:
                    raise SystemExit(f"tools/ab.py: desc={v[k]} does not apply here")
                continue
            if k not in DEFAULTS:
                raise SystemExit(f"tools/ab.py: no default recorded for knob {k!r}")
    times = {i: [] for i in range(len(variants))}
    ref = None
    for r in range(a.rounds):
        for i, v in enumerate(variants):
            for k in {k for vv in variants for k in vv} - {"desc"}:
                u.set_tuning(k, DEFAULTS[k])
            for k, val in v.items():
                if k != "desc":
                    u.set_tuning(k, val)
            launch = launches[v.get("desc", 0)]
            launch(s)  # warm
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif not torch.equal(out, ref):
                raise SystemExit(f"variant {a.variants[i]} changed results")
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.launches):
                launch(s)
            e1.record(s)
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.launches)
    res = {}
    for i, v in enumerate(a.variants):
        t = times[i]
        res[v] = {"median_ms": round(statistics.median(t), 5), "min_ms": round(min(t), 5),
                  "GBps_median": round(w["bytes"] / (statistics.median(t) * 1e-3) / 1e9, 1)}
    print(json.dumps({"config": a.config, "api": a.api, "results": res}, indent=1))


if __name__ == "__main__":
    main()
