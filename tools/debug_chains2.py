import sys, os, numpy as np, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import libuinet_amd as u, oracle
from test_gpu_parity import rand_arena, random_chain_layout, dev, host16
ora = oracle.Oracle()
rng = np.random.default_rng(1001)
arena = rand_arena(1 << 20, 31)
seg_off, seg_len, pkt_seg = random_chain_layout(rng, 5000, arena.size, max_seg=256)
seg_len[seg_len == 0] = 5
d = dev(torch, arena)
assert d.data_ptr() % 16 == 0
want = ora.chains(arena, seg_off, seg_len, pkt_seg)
got = host16(u.cksum_chains(d, dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)), dev(torch, pkt_seg.astype(np.int32))))
bad = set(np.nonzero(got != want)[0].tolist())
stats = collections.Counter(); tot = collections.Counter()
for t in range(0, 5000 // 32 + 1):
    P0 = t * 32; P1 = min(5000, P0 + 32)
    if P0 >= 5000: break
    S0, S1 = pkt_seg[P0], pkt_seg[P1]
    for r0 in range(S0, S1, 64):
        segs = np.arange(r0, min(S1, r0 + 64))
        head = seg_off[segs] & 15
        nch = (head + seg_len[segs] + 15) >> 4
        cst = np.concatenate([[0], np.cumsum(nch)[:-1]])
        C = nch.sum()
        for p in range(P0, P1):
            a, b = pkt_seg[p], pkt_seg[p + 1]
            m = (segs >= a) & (segs < b)
            if not m.any(): continue
            if a < r0 or b > r0 + 64: key = "crossround"
            else:
                c_first = cst[m][0]; c_last = cst[m][-1] + nch[m][-1] - 1
                key = f"round{(r0-S0)//64} batch{c_first//256}-{c_last//256} C>256:{C>256}"
            tot[key] += 1
            stats[key] += p in bad
for k in sorted(tot): print(f"{k:45s} bad {stats[k]:5d} / {tot[k]:5d}")
