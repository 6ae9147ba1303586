"""The oracle (CPU restatement) pinned against the reference's golden vectors,
the reference object itself, and the reference's pcap fixture."""
from __future__ import annotations

import numpy as np
import pytest

from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes


def test_golden_skip(ora, arena, golden):
    g = golden("skip")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    got = ora.skip_batch(ch.heads, g["len"], g["skip"])
    np.testing.assert_array_equal(got, g["expected"])


def test_golden_skip_per_call(ora, arena, golden):
    g = golden("skip")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    for i in range(0, ch.n, 7):
        assert ora.cksum_skip(ch.head(i), int(g["len"][i]), int(g["skip"][i])) == g["expected"][i]


def test_golden_pseudo(ora, arena, golden):
    g = golden("pseudo")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    got = ora.pseudo_header_batch(ch.heads, g["plen"], g["off0"], g["src"], g["dst"], g["proto"])
    np.testing.assert_array_equal(got, g["expected"])


def test_golden_hdr(ora, arena, golden):
    g = golden("hdr")
    got = ora.hdr_batch(arena.ctypes.data + g["off"].astype(np.uint64))
    np.testing.assert_array_equal(got, g["expected"])


def test_golden_fold(ora, golden):
    g = golden("fold")
    for a, b, c, e in zip(g["pa"], g["pb"], g["pc"], g["pseudo"]):
        assert ora.in_pseudo(int(a), int(b), int(c)) == e
    for a, b, e in zip(g["wa"], g["wb"], g["addword"]):
        assert ora.in_addword(int(a), int(b)) == e


def test_golden_config_shapes(ora, arena, golden):
    g = golden("configs")
    for tag in ("c2", "c2rx"):
        ch = MbufChains.contiguous(arena, g[f"{tag}_off"], 1500)
        np.testing.assert_array_equal(ora.skip_batch(ch.heads, 1500, 0), g[f"{tag}_expected"])
        # the flat span form computes the same thing
        np.testing.assert_array_equal(ora.spans(arena, g[f"{tag}_off"], 1500), g[f"{tag}_expected"])
    ch = MbufChains(arena, g["c3_seg_off"], g["c3_seg_len"], g["c3_pkt_seg"])
    np.testing.assert_array_equal(ora.skip_batch(ch.heads, g["c3_len"], 20), g["c3_expected"])
    ch = MbufChains.contiguous(arena, g["c5_off"], 9000)
    got = ora.pseudo_header_batch(ch.heads, 8980, 20, g["c5_src"], g["c5_dst"], g["c5_proto"])
    np.testing.assert_array_equal(got, g["c5_expected"])


def test_edge_values(ora):
    a = aligned_empty(8192)
    ch = MbufChains.contiguous(a, [0, 1, 2, 3, 4097], [1500, 7, 0, 33, 1])
    # all-zero data -> 0xffff (never 0: end-around carry, in_cksum.c:65-71)
    assert list(ora.skip_batch(ch.heads, [1500, 7, 0, 33, 1], 0)) == [0xFFFF] * 5
    a[:] = 0xFF
    # even-length all-0xff -> folded 0xffff -> 0; the empty range stays 0xffff
    got = ora.skip_batch(ch.heads, [1500, 7, 0, 33, 1], 0)
    assert got[0] == 0 and got[2] == 0xFFFF


def test_empty_and_null_chains(ora):
    a = aligned_empty(64)
    ch = MbufChains(a, [], [], [0, 0, 0])
    assert list(ora.skip_batch(ch.heads, [10, 0], [0, 0])) == [0xFFFF, 0xFFFF]


def test_oracle_vs_reference_fuzz(ora, ref):
    """200k-style fuzz (scaled to 20k here) of random chains, the survey's
    verification, against the reference object itself."""
    rng = np.random.default_rng(11)
    arena = aligned_empty(1 << 20)
    splitmix64_bytes(arena.size, 3, out=arena)
    n = 20000
    nseg = rng.integers(1, 6, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)])
    s = int(pkt_seg[-1])
    seg_len = rng.integers(0, 1600, s)
    seg_off = rng.integers(0, arena.size - 1700, s)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = (rng.random(n) * tot * 0.5).astype(np.int64)
    ln = (skip + rng.random(n) * (tot - skip + 3)).astype(np.int64)
    np.testing.assert_array_equal(ora.skip_batch(ch.heads, ln, skip), ref.skip_batch(ch.heads, ln, skip))
    first = seg_len[pkt_seg[:-1]]
    off0 = (rng.random(n) * (first + 1)).astype(np.int64)
    plen = (rng.random(n) * (tot - off0 + 1)).astype(np.int64)
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    pr = rng.integers(0, 256, n)
    np.testing.assert_array_equal(ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, pr),
                                  ref.pseudo_header_batch(ch.heads, plen, off0, src, dst, pr))


def _pcap_packets(frames):
    """(ip-offset, frame) pairs of the IPv4/TCP frames of the fixture."""
    out = []
    for f in frames:
        if len(f) >= 34 and f[12:14] == b"\x08\x00" and f[23] == 6:
            out.append(f)
    return out


def pcap_cases(frames):
    """Lay the fixture's frames out RX-style (IP header at cluster + 14,
    uinet_if_pcap.c:690-715) and return chains + in_cksum_pseudo_header args."""
    pk = _pcap_packets(frames)
    arena = aligned_empty(2048 * len(pk))
    off, ln, hl, plen, src, dst = [], [], [], [], [], []
    for i, f in enumerate(pk):
        arena[2048 * i : 2048 * i + len(f)] = np.frombuffer(f, np.uint8)
        ip = f[14:]
        ihl = (ip[0] & 0xF) * 4
        tot = int.from_bytes(ip[2:4], "big")
        off.append(2048 * i + 14)
        ln.append(len(f) - 14)
        hl.append(ihl)
        plen.append(tot - ihl)
        src.append(int.from_bytes(ip[12:16], "little"))
        dst.append(int.from_bytes(ip[16:20], "little"))
    return arena, np.array(off), np.array(ln), np.array(hl), np.array(plen), np.array(src, np.uint64), np.array(dst, np.uint64)


def test_pcap_kat(ora, pcap_frames):
    """The reference's own fixture lib/libuinet_demo/passive_extract_test.pcap:
    all 113 captured IPv4/TCP packets carry valid IP and TCP checksums, so
    in_cksum_hdr and in_cksum_pseudo_header must both return 0
    (ip_input.c:460-471, tcp_input.c:711-717)."""
    arena, off, ln, hl, plen, src, dst = pcap_cases(pcap_frames)
    assert off.size == 113
    ips = arena.ctypes.data + off.astype(np.uint64)
    assert not ora.hdr_batch(ips).any()
    ch = MbufChains.contiguous(arena, off, ln)
    assert not ora.pseudo_header_batch(ch.heads, plen, hl, src, dst, 6).any()


def test_pcap_kat_refragmented(ora, pcap_frames):
    """Same KAT after re-chaining every packet into random 1..256-B fragments at
    random 0-7-B offsets (m_fragment, sys/kern/uipc_mbuf.c:1693-1761)."""
    arena, off, ln, hl, plen, src, dst = pcap_cases(pcap_frames)
    rng = np.random.default_rng(5)
    frag = aligned_empty(8 * arena.size)
    seg_off, seg_len, pkt_seg, cur = [], [], [0], 0
    for o, L, h in zip(off, ln, hl):
        pos = 0
        first = True
        while pos < L:
            piece = int(min(L - pos, max(h, rng.integers(1, 257)) if first else rng.integers(1, 257)))
            cur += int(rng.integers(0, 8))
            frag[cur : cur + piece] = arena[o + pos : o + pos + piece]
            seg_off.append(cur)
            seg_len.append(piece)
            cur += piece
            pos += piece
            first = False
        pkt_seg.append(len(seg_off))
    ch = MbufChains(frag, seg_off, seg_len, pkt_seg)
    assert not ora.pseudo_header_batch(ch.heads, plen, hl, src, dst, 6).any()
