#!/usr/bin/env python3
"""Where the wave-per-packet chain kernel (k_chains_wide) overtakes the
32-packet tile kernel (k_chains_pipe): device-resident chains of 1, 2 or 4
segments of one length each (--long: jumbo / TSO shapes, some with a 40-B
header mbuf first), ~1.2 GB summed per launch, segments laid back to back,
skip 0; both kernels forced by the chains_wide knob, alternating, in one
process.  Prints one JSON line per shape (median kernel ms of each)."""
from __future__ import annotations

import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import libuinet_amd as u

    total = 1_200_000_000
    arena = torch.randint(0, 256, (total + 4096,), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    shapes = [(nseg, seg, 0) for nseg in (1, 2, 4)
              for seg in (256, 512, 768, 1024, 1500, 2048, 3000, 4096)]
    if len(sys.argv) > 1 and sys.argv[1] == "--long":
        # jumbo frames, TSO payloads, and a 40-B header mbuf before 1-16 page slices
        shapes = [(1, 9000, 0), (1, 16384, 0), (2, 8192, 0), (1, 8960, 40), (2, 4096, 40),
                  (4, 4096, 40), (16, 4096, 40), (8, 2048, 40)]
    for nseg, seg, hdr in shapes:
        if True:
            per = nseg + (1 if hdr else 0)
            n = total // (seg * nseg + hdr)
            seg_len = np.tile(np.array(([hdr] if hdr else []) + [seg] * nseg, np.int64), n)
            seg_off = np.concatenate([[0], np.cumsum(seg_len)[:-1]]).astype(np.int64)
            pkt_seg = np.arange(n + 1, dtype=np.int64) * per
            d_so = torch.from_numpy(seg_off).cuda()
            d_sl = torch.from_numpy(seg_len.astype(np.int32)).cuda()
            d_ps = torch.from_numpy(pkt_seg.astype(np.int32)).cuda()
            out = torch.empty(n, dtype=torch.uint16, device="cuda")
            t = {1: [], 2: []}
            ref = None
            for r in range(4):
                for wide in (1, 2):
                    u.set_tuning("chains_wide", wide)
                    u.cksum_chains(arena, d_so, d_sl, d_ps, out=out, stream=s)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out.clone()
                    assert torch.equal(out, ref), (nseg, seg, wide)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(10):
                        u.cksum_chains(arena, d_so, d_sl, d_ps, out=out, stream=s)
                    e1.record(s)
                    e1.synchronize()
                    t[wide].append(e0.elapsed_time(e1) / 10)
            u.set_tuning("chains_wide", 0)
            a, b = statistics.median(t[1]), statistics.median(t[2])
            print(json.dumps({"segs_per_packet": nseg, "seg_bytes": seg, "header_mbuf": hdr, "packets": n,
                              "tile_ms": round(a, 4), "wide_ms": round(b, 4),
                              "wide_vs_tile": round(b / a, 3)}), flush=True)
            del d_so, d_sl, d_ps, out


if __name__ == "__main__":
    main()
