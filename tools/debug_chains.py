import sys, os, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import libuinet_amd as u, oracle
from test_gpu_parity import rand_arena, random_chain_layout, dev, host16
ora = oracle.Oracle()
for case in range(4):
    rng = np.random.default_rng(1000 + case)
    arena = rand_arena(1 << 20, 31)
    zero_frac = [0.08, 0.0, 0.08, 0.0][case]
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 5000, arena.size, max_seg=256)
    if zero_frac == 0: seg_len[seg_len == 0] = 5
    if case >= 2: seg_off = seg_off & ~15  # aligned segments
    want = ora.chains(arena, seg_off, seg_len, pkt_seg)
    got = host16(u.cksum_chains(dev(torch, arena), dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)), dev(torch, pkt_seg.astype(np.int32))))
    bad = np.nonzero(got != want)[0]
    nseg = np.diff(pkt_seg)
    print(f"case {case} zero={zero_frac} aligned={case>=2}: bad {bad.size}/{want.size}")
    if bad.size:
        t = bad // 32; first_seg_in_tile = pkt_seg[t*32]
        rel0 = pkt_seg[bad] - first_seg_in_tile; rel1 = pkt_seg[bad+1] - first_seg_in_tile
        cross = (rel0 // 64) != ((rel1 - 1) // 64)
        print("  pkt in tile:", np.bincount(bad % 32, minlength=32))
        print("  crosses round:", cross.mean(), " nseg mean bad/all:", nseg[bad].mean(), nseg.mean())
        # is it a rotation (byte swap) error?
        sw = ((want[bad] >> 8) | (want[bad] << 8)) & 0xffff
        print("  got==bswap(want):", (got[bad] == sw).mean())
        print("  first bad:", bad[:10], got[bad[:5]], want[bad[:5]])
