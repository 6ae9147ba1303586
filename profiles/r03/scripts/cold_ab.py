#!/usr/bin/env python3
"""Interleaved cold-start A/B: which kernel variants slow down in the first
launches after an idle gap (the driver's 5-warmup / 20-step window)?

One process builds config 2 once; then, for each repetition and each
variant in turn: sleep --idle-s, run --launches back-to-back launches with a
HIP event pair around each, and record the rate over launches
[warmup, warmup + steps) and over the last 10.  Variants are engine tuning
settings (uinet_cksum_set_tuning, "key=value,..."), plus "pure-read": a
torch sum over the same arena viewed as int64 (a streaming read with next to
no arithmetic), for the platform's own behaviour in the same process.

Prints one JSON object: per variant the per-repetition window and tail
rates (TB/s) and the per-launch ms of every repetition.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--idle-s", type=float, default=1.5)
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tail", type=int, default=10, help="launches in the tail rate")
    ap.add_argument("--api", default="spans", choices=["spans", "strided"])
    ap.add_argument("--variants", nargs="+",
                    default=["", "blocks_per_cu=256", "blocks_per_cu=32", "pure-read"])
    a = ap.parse_args()
    import torch

    import bench
    import libuinet_amd as u

    torch.cuda.set_device(0)
    assert u.device_ok()
    w = bench.build_workload("2", None, 0)
    out = torch.empty(w["n"], dtype=torch.uint16, device="cuda")
    s = torch.cuda.current_stream()
    spans = bench.make_launch("2", w, a.api, out)
    arena64 = w["arena"][: (w["arena"].numel() // 8) * 8].view(torch.int64)
    sink = torch.empty((), dtype=torch.int64, device="cuda")
    # the engine's defaults (cksum_api.hip TuningLive), restored before each variant
    defaults = {"blocks_per_cu": 0, "spans_sdesc": 1, "spans_lut": 1, "xcd_remap": 1,
                "spans_geo": 0}
    ref = None
    res = {v or "default": {"window_tbs": [], "tail_tbs": [], "ms": []} for v in a.variants}
    for _ in range(a.reps):
        for v in a.variants:
            for k, val in defaults.items():
                u.set_tuning(k, val)
            if v == "pure-read":
                launch = lambda st: torch.sum(arena64, dim=(0,), out=sink)  # noqa: E731
                nbytes = arena64.numel() * 8
            else:
                for kv in filter(None, v.split(",")):
                    k, val = kv.split("=")
                    u.set_tuning(k, int(val))
                launch, nbytes = spans, w["bytes"]
            torch.cuda.synchronize()
            time.sleep(a.idle_s)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.launches)]
            for e0, e1 in ev:
                e0.record(s)
                launch(s)
                e1.record(s)
            torch.cuda.synchronize()
            ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
            if v != "pure-read":
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    raise SystemExit(f"variant {v!r} changed results")
            win = ms[a.warmup:a.warmup + a.steps]
            r = res[v or "default"]
            r["window_tbs"].append(round(nbytes * len(win) / (win.sum() * 1e-3) / 1e12, 3))
            r["tail_tbs"].append(round(nbytes * a.tail / (ms[-a.tail:].sum() * 1e-3) / 1e12, 3))
            r["ms"].append([round(float(x), 4) for x in ms])
        print({k: (r["window_tbs"][-1], r["tail_tbs"][-1]) for k, r in res.items()}, flush=True)
    for r in res.values():
        r["window_median"] = float(np.median(r["window_tbs"]))
        r["tail_median"] = float(np.median(r["tail_tbs"]))
    print(json.dumps({"workload": w["desc"], "api": a.api, "idle_s": a.idle_s, "results": res}))


if __name__ == "__main__":
    main()
