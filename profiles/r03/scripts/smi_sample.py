#!/usr/bin/env python3
"""Sample the GPU's clocks, power, activity and throttle status through amdsmi
(gpu_metrics) every --period-s until SIGTERM / SIGINT, then write the samples
as JSON: run it in the background beside a bench (it never touches the GPU's
compute queues).  python tools/smi_sample.py OUT.json [--period-s 0.005]"""
from __future__ import annotations

import argparse
import json
import signal
import time

KEYS = ("current_gfxclk", "current_uclk", "current_fclk", "current_socket_power",
        "average_gfx_activity", "average_umc_activity", "temperature_hotspot",
        "temperature_mem", "throttle_status")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--period-s", type=float, default=0.005)
    ap.add_argument("--max-s", type=float, default=300.0)
    a = ap.parse_args()
    stop = []
    signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
    signal.signal(signal.SIGINT, lambda *_: stop.append(1))
    rows, err = [], None
    t0 = time.time()
    try:
        import amdsmi

        amdsmi.amdsmi_init()
        h = amdsmi.amdsmi_get_processor_handles()[0]
        while not stop and time.time() - t0 < a.max_s:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            row = {"t": round(time.time(), 4)}
            for k in KEYS:
                v = m.get(k)
                if isinstance(v, list):
                    v = v[0] if v else None
                row[k] = v if isinstance(v, (int, float)) else None
            rows.append(row)
            time.sleep(a.period_s)
    except Exception as e:  # pragma: no cover - box dependent
        err = repr(e)
    with open(a.out, "w") as f:
        json.dump({"error": err, "t0": t0, "samples": rows}, f)


if __name__ == "__main__":
    main()
