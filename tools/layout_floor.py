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


def clipped_segments(seg_off, seg_len, pkt_seg, lens, skip):
    """Per segment, the [start, end) arena bytes in_cksum_skip sums."""
    n = pkt_seg.size - 1
    seg_pkt = np.repeat(np.arange(n), np.diff(pkt_seg))
    pos = np.cumsum(seg_len) - seg_len                      # global running position
    pos = pos - (np.cumsum(seg_len) - seg_len)[pkt_seg[:-1]][seg_pkt]  # position in its chain
    lo = np.clip(skip[seg_pkt] - pos, 0, seg_len)
    hi = np.clip(lens[seg_pkt] - pos, 0, seg_len)
    keep = hi > lo
    return seg_off[keep] + lo[keep], seg_off[keep] + hi[keep], int((hi - lo)[keep].sum())


def lines_touched(a, b, line):
    first, last = a // line, (b - 1) // line
    # union of [first, last] ranges over all segments
    order = np.argsort(first, kind="stable")
    f, l = first[order], last[order]
    runmax = np.maximum.accumulate(l)
    new = np.concatenate([[True], f[1:] > runmax[:-1]])
    starts = f[new]
    ends = np.maximum.reduceat(l, np.flatnonzero(new))
    return int((ends - starts + 1).sum())


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
    s, e, algo = clipped_segments(lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lens, skip)
    nseg, npkt = lay["seg_len"].size, lay["pkt_seg"].size - 1
    desc_pkt = npkt * (4 + 4 + 4 + (4 if seed else 0)) + 4
    res = {"config": a.config, "packets": npkt, "segments": nseg, "algorithmic_bytes": algo}
    for line in (64, 128):
        arena = lines_touched(s, e, line) * line
        res[f"arena_lines_{line}B"] = arena
        res[f"floor_wide_{line}B"] = arena + 12 * nseg + desc_pkt
        res[f"floor_packed_{line}B"] = arena + 6 * nseg + desc_pkt
        res[f"floor_wide_{line}B_over_algorithmic"] = round(res[f"floor_wide_{line}B"] / algo, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
