#!/usr/bin/env python3
"""Where do the slow first launches of a fresh bench process come from?

Runs the bench's own config-2 workload and launch, exactly as bench.py builds
them, with a HIP event pair around EVERY launch, while a thread samples the
GPU's clocks and power through amdsmi (gpu_metrics) about every millisecond:

  phase "driver":  W untimed + K timed launches, back to back (the driver's
                   --warmup 5 --steps 20 shape), then more launches up to
                   --launches so the settled state is visible;
  phase "idle":    sleep --idle-s seconds, then --launches again (does the
                   ramp recur after idle?).

Prints one JSON object: per-launch ms, clock samples (t, gfxclk, uclk,
fclk, socket power, activity), and per-phase deciles.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class ClockSampler(threading.Thread):
    KEYS = ("current_gfxclk", "current_uclk", "current_fclk", "current_socclk",
            "current_socket_power", "average_gfx_activity", "average_umc_activity",
            "temperature_hotspot", "temperature_mem", "throttle_status")

    def __init__(self, period_s=0.001):
        super().__init__(daemon=True)
        self.period = period_s
        self.samples = []
        self.err = None
        self.stop_ev = threading.Event()
        self.t0 = time.perf_counter()

    def run(self):
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            h = amdsmi.amdsmi_get_processor_handles()[0]
        except Exception as e:  # pragma: no cover - box dependent
            self.err = f"amdsmi init: {e!r}"
            return
        while not self.stop_ev.is_set():
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            except Exception as e:  # pragma: no cover
                self.err = f"metrics: {e!r}"
                return
            row = {"t": round(time.perf_counter() - self.t0, 5)}
            for k in self.KEYS:
                v = m.get(k)
                if isinstance(v, list):
                    v = v[0] if v else None
                row[k] = v if isinstance(v, (int, float)) else None
            self.samples.append(row)
            time.sleep(self.period)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--idle-s", type=float, default=1.0)
    ap.add_argument("--config", default="2")
    ap.add_argument("--api", default="spans", help="spans | strided")
    a = ap.parse_args()

    sampler = ClockSampler()
    sampler.start()
    import torch

    import bench
    import libuinet_amd as u

    torch.cuda.set_device(0)
    assert u.device_ok()
    t_build0 = time.perf_counter() - sampler.t0
    w = bench.build_workload(a.config, None, 0)
    outs = [torch.empty(w["n"], dtype=torch.uint16, device="cuda") for _ in range(2)]
    launches = [bench.make_launch(a.config, w, a.api, o) for o in outs]
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t_build1 = time.perf_counter() - sampler.t0

    def run(nl):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(nl)]
        torch.cuda.synchronize()
        t_start = time.perf_counter() - sampler.t0
        for i, (e0, e1) in enumerate(ev):
            e0.record(s)
            launches[i & 1](s)
            e1.record(s)
        torch.cuda.synchronize()
        t_end = time.perf_counter() - sampler.t0
        ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
        return ms, t_start, t_end

    res = {"workload": w["desc"], "api": a.api, "bytes": w["bytes"],
           "build_s": [t_build0, t_build1]}
    for phase in ("driver", "idle"):
        if phase == "idle":
            time.sleep(a.idle_s)
        n = max(a.launches, a.warmup + a.steps)
        ms, t0, t1 = run(n)
        gbs = w["bytes"] / (ms * 1e-3) / 1e9
        d = {"t_start": round(t0, 4), "t_end": round(t1, 4),
             "ms": [round(float(x), 5) for x in ms],
             "first_gbs": round(float(gbs[0]), 1),
             "driver_window_gbs": round(w["bytes"] * a.steps /
                                        (ms[a.warmup:a.warmup + a.steps].sum() * 1e-3) / 1e9, 1),
             "last100_gbs": round(w["bytes"] * 100 / (ms[-100:].sum() * 1e-3) / 1e9, 1),
             "deciles_gbs": [round(float(x), 1) for x in
                             (w["bytes"] / (np.array_split(ms, 10)[i].mean() * 1e-3) / 1e9
                              for i in range(10))]}
        res[phase] = d
        print(phase, {k: v for k, v in d.items() if k != "ms"}, flush=True)
    sampler.stop_ev.set()
    sampler.join(2)
    res["clock_err"] = sampler.err
    res["clock_samples"] = sampler.samples
    print(json.dumps(res))


if __name__ == "__main__":
    main()
