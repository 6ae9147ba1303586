#!/usr/bin/env python3
"""Generate tests/golden/golden_in6.npz from the REFERENCE's own IPv6 code.

Run in the build container after ``make -C oracle``: the expected values are
what /root/reference/sys/netinet6/in6_cksum.c (with in6_getscope from
scope6.c; oracle/Makefile) returns for the stored inputs.

  arena, seg_off, seg_len, pkt_seg   IPv6 TCP/UDP/ICMPv6 packets as mbuf chains
                                     (tests/test_in6.py::build_ipv6: link-local,
                                     multicast and global addresses, extension
                                     headers, 0-300-B mbufs at 0-7-B offsets;
                                     len >= 1: the reference dereferences NULL
                                     for len 0 at the very end of a chain)
  nxt, off, len, expected            in6_cksum(m, nxt, off, len)
  p_hdr, p_len, p_nxt, p_csum, p_expected
                                     in6_cksum_pseudo(ip6, len, nxt, csum) on the
                                     same packets' headers
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from test_in6 import build_ipv6  # noqa: E402


def main() -> None:
    R = oracle.Reference()
    ch, nxt, off, ln, pkts = build_ipv6(300, seed=61, min_len=1)
    expected = R.in6_cksum_batch(ch.heads, nxt, off, ln)
    rng = np.random.default_rng(62)
    hdr = np.stack([np.frombuffer(p[:40], np.uint8) for p in pkts])
    p_len = rng.integers(0, 1 << 32, len(pkts), dtype=np.uint64).astype(np.uint32)
    p_len[::3] = ln[::3]
    p_nxt = nxt.astype(np.uint8)
    p_csum = rng.integers(0, 1 << 16, len(pkts)).astype(np.uint16)
    p_exp = np.array([R.in6_cksum_pseudo(hdr[i].ctypes.data, int(p_len[i]), int(p_nxt[i]),
                                         int(p_csum[i])) for i in range(len(pkts))], np.int32)
    np.savez_compressed(os.path.join(HERE, "golden_in6.npz"), arena=np.asarray(ch.arena),
                        seg_off=ch.seg_off, seg_len=ch.seg_len, pkt_seg=ch.pkt_seg,
                        nxt=nxt.astype(np.uint8), off=off.astype(np.uint32),
                        len=ln.astype(np.uint32), expected=expected, p_hdr=hdr, p_len=p_len,
                        p_nxt=p_nxt, p_csum=p_csum, p_expected=p_exp)
    print(f"golden_in6.npz: {len(pkts)} packets")


if __name__ == "__main__":
    main()
