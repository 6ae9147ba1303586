#!/usr/bin/env python3
"""ADVICE r04 (cksum_kernels.hip pick_geometry): span batches with a mean
length above 6144 B take 64 lanes x 9 loads; only 9000-B frames were measured.
This times large spans (16, 32, 64 KiB; ~1.5 GB per launch, device-resident)
on the picked geometry against 64 x 3 forced with the spans_geo knob,
alternating, HIP events around 20 back-to-back launches, bit-exact against
each other."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import numpy as np
import torch

import libuinet_amd as u


def timed(fn, k=20):
    s = torch.cuda.current_stream()
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(k):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k


res = {}
arena = torch.randint(0, 256, (3 << 29,), dtype=torch.uint8, device="cuda")  # 1.5 GiB
for span in (9000, 16384, 32768, 65000):
    n = (1536 << 20) // span
    off = torch.arange(n, dtype=torch.int64, device="cuda") * span
    ln = torch.full((n,), span, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    nbytes = n * span
    row = {}
    ref = None
    for r in range(3):
        for name, geo in (("picked", 0), ("64x3", 64 * 16 + 3)):
            u.set_tuning("spans_geo", geo)
            ms = timed(lambda: u.cksum_spans(arena, off, ln, out=out, len_hint=span))
            kern = u.last_kernel()
            got = out.cpu().numpy().copy()
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), (span, name)
            row.setdefault(name, []).append(round(ms, 4))
            row[name + "_kernel"] = kern.split("(")[0][-70:]
    u.set_tuning("spans_geo", 0)
    for name in ("picked", "64x3"):
        row[name + "_frac"] = round(nbytes / (np.median(row[name]) * 1e-3) / 8e12, 4)
    res[span] = row
    print(json.dumps({span: row}), flush=True)
print(json.dumps(res))
