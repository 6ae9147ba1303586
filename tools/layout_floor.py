#!/usr/bin/env python3
"""HBM-traffic floor of a chained batch's layout: the bytes of the distinct
64-B and 128-B lines that hold at least one summed byte, plus the segment
and packet descriptors the chain kernel reads (12 B per segment for the wide
form, 6 B packed; pkt_seg + len + skip + seed per packet).  What no kernel
reading these packets from this layout can avoid fetching -- the denominator
for "fraction of the layout floor" beside the algorithmic fraction.

  python tools/layout_floor.py --config 3tx      (3, 3tx, 5tso; CPU only)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="3", choices=["3", "3tx", "5tso"])
    ap.add_argument("--packets", type=int, default=1 << 20)
    a = ap.parse_args()
    import libuinet_amd.workloads as W

    if a.config == "3":
        lay = W.config3_layout(a.packets)
        lens, skip, seed = lay["lens"], np.full(a.packets, 20), False
    else:
        lay = W.chain_layout(a.config, a.packets if a.config == "3tx" else None)
        lens, skip, seed = lay["lens"], lay["skip"], lay["seed"] is not None
    nseg, npkt = lay["seg_len"].size, lay["pkt_seg"].size - 1
    res = {"config": a.config, "packets": npkt, "segments": nseg}
    for line in (64, 128):
        wide = W.layout_floor(lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lens, skip, seed, line)
        packed = W.layout_floor(lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lens, skip, seed,
                                line, seg_desc_bytes=6)
        algo = wide["algorithmic_bytes"]
        res["algorithmic_bytes"] = algo
        res[f"arena_lines_{line}B"] = wide["arena_bytes"]
        res[f"floor_wide_{line}B"] = wide["floor_bytes"]
        res[f"floor_packed_{line}B"] = packed["floor_bytes"]
        res[f"floor_wide_{line}B_over_algorithmic"] = round(wide["floor_bytes"] / algo, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
