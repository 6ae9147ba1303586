#!/usr/bin/env python3
"""Per-launch kernel time over a long back-to-back run (HIP events around
each launch), per tuning variant: shows clock/power drift under sustained
HBM streaming.  python tools/drift.py --config 2 --launches 300 --variants spans_lut=0 spans_lut=1"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="2")
    ap.add_argument("--api", default="spans")
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--variants", nargs="+", default=[""])
    a = ap.parse_args()
    import torch

    import bench
    import libuinet_amd as u

    w = bench.build_workload(a.config, None, 0)
    out = torch.empty(w["n"], dtype=torch.uint16, device="cuda")
    s = torch.cuda.current_stream()
    launch = bench.make_launch(a.config, w, a.api, out)
    res = {}
    for v in a.variants:
        for kv in filter(None, v.split(",")):
            k, x = kv.split("=")
            u.set_tuning(k, int(x))
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        torch.cuda.synchronize()
        for e0, e1 in ev:
            e0.record(s)
            launch(s)
            e1.record(s)
        torch.cuda.synchronize()
        ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
        k = max(1, a.launches // 10)
        res[v or "default"] = {
            "first10pct_ms": round(float(ms[:k].mean()), 5),
            "last10pct_ms": round(float(ms[-k:].mean()), 5),
            "mean_ms": round(float(ms.mean()), 5),
            "GBps_mean": round(w["bytes"] / (ms.mean() * 1e-3) / 1e9, 1),
            "deciles_ms": [round(float(x), 4) for x in ms.reshape(10, -1).mean(1)]
            if a.launches % 10 == 0 else None,
        }
        print(v, res[v or "default"], flush=True)
        torch.cuda.synchronize()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
