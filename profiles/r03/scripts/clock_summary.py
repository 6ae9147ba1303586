#!/usr/bin/env python3
"""Steady-state clocks and power per config from tools/cold_start.py outputs.

  python tools/clock_summary.py profiles/r02/clocks/c*.json

For each file: the kernel's rate over the last 100 launches of the first
phase, and the median gfxclk / uclk / socket power / activity / throttle
status over the samples in the last 40 % of that phase (the settled state)."""
from __future__ import annotations

import json
import statistics
import sys


def main():
    for path in sys.argv[1:]:
        text = open(path).read()
        res = json.loads(text[text.index('{"workload"'):])
        ph = res["driver"]
        t0, t1 = ph["t_start"], ph["t_end"]
        lo = t0 + 0.6 * (t1 - t0)
        win = [s for s in res["clock_samples"] if lo <= s["t"] <= t1]

        def med(k):
            v = [s[k] for s in win if s.get(k) is not None]
            return statistics.median(v) if v else None

        thr = sorted({s.get("throttle_status") for s in win})
        print(json.dumps({
            "file": path, "workload": res["workload"][:60],
            "last100_GBps": ph["last100_gbs"], "samples": len(win),
            "gfxclk_MHz": med("current_gfxclk"), "uclk_MHz": med("current_uclk"),
            "socket_W": med("current_socket_power"), "gfx_activity": med("average_gfx_activity"),
            "umc_activity": med("average_umc_activity"), "throttle_status": thr}))


if __name__ == "__main__":
    main()
