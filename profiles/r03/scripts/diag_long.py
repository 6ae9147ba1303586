"""Lab diagnostic (not a test): single-segment chains of 9000 B, all zero but
one 16-bit word of 1 at byte p; prints which p give a wrong sum."""
import numpy as np
import torch
import libuinet_amd as u

L = 9000
n = L // 2
arena = np.zeros(n * L + 64, np.uint8)
for i in range(n):
    arena[i * L + 2 * i] = 1  # packet i: word at byte 2*i
seg_off = (np.arange(n, dtype=np.int64) * L)
seg_len = np.full(n, L, np.int64)
pkt_seg = np.arange(n + 1, dtype=np.int64)
d = lambda a: torch.from_numpy(a).cuda()
got = u.cksum_chains(d(arena), d(seg_off), d(seg_len.astype(np.int32)), d(pkt_seg.astype(np.int32)))
g = got.cpu().numpy().view(np.uint16)
want = np.full(n, 0xFFFF ^ 1, np.uint16)
bad = np.nonzero(g != want)[0]
print("bad", bad.size, "of", n)
if bad.size:
    chunks = (2 * bad) // 16
    print("bad chunks:", np.unique(chunks)[:80], "...", np.unique(chunks)[-20:])
    print("sample got", [hex(x) for x in g[bad[:8]]])
