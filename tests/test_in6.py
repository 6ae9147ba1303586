"""IPv6: in6_cksum / in6_cksum_pseudo / in6_cksum_batch.

The reference's sys/netinet6/in6_cksum.c is not compiled by its own build
(INET6 off); oracle/Makefile compiles it with libuinet's kernel flags, plus
the one function it calls from scope6.c (in6_getscope), into the reference
object.  Parity is pinned to that object directly (in6_cksum and
in6_cksum_pseudo on the same chains and headers, and the committed
golden_in6.npz it generated, which the GPU box checks without the
reference tree), and in two halves as before: the data walk against the
reference's in_cksum_skip, the pseudo header against an independent Python
restatement; plus the self-verification property every receiver relies on:
a segment whose checksum field holds in6_cksum's result sums to 0."""
from __future__ import annotations

import numpy as np
import pytest

from libuinet_amd.mbuf import MbufChains, aligned_empty


def _pseudo_py(h: bytes, length: int, nxt: int) -> int:
    def words(b):
        return [b[i] | b[i + 1] << 8 for i in range(0, len(b), 2)]

    def scope(a):
        ll = a[0] == 0xFE and (a[1] & 0xC0) == 0x80
        mc = a[0] == 0xFF and (a[1] & 0x0F) in (1, 2)
        return (a[2] | a[3] << 8) if (ll or mc) else 0

    ph = length.to_bytes(4, "big") + b"\0\0\0" + bytes([nxt])
    s = sum(words(ph)) + sum(words(h[8:40])) - scope(h[8:24]) - scope(h[24:40])
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _addr(rng):
    k = rng.integers(0, 5)
    a = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
    if k == 0:
        a[0], a[1] = 0xFE, 0x80 | (a[1] & 0x3F)          # link-local, zone in word 1
    elif k == 1:
        a[0], a[1] = 0xFF, (a[1] & 0xF0) | 0x02          # link-local multicast
    elif k == 2:
        a[0], a[1] = 0xFF, (a[1] & 0xF0) | 0x01          # interface-local multicast
    elif k == 3:
        a[0], a[1] = 0xFF, (a[1] & 0xF0) | 0x05          # site-local multicast: no zone
    return bytes(a)


def build_ipv6(n: int, seed: int = 6, min_len: int = 0):
    """n IPv6 TCP/UDP/ICMPv6 packets; the first mbuf holds the whole IPv6
    header (in6_cksum's contract), the rest is cut into 0-300-B mbufs."""
    rng = np.random.default_rng(seed)
    pkts, nxts, offs, lens = [], [], [], []
    for _ in range(n):
        nxt = int(rng.choice([6, 17, 58]))
        ext = int(rng.choice([0, 0, 0, 8, 16]))   # extension headers before L4
        plen = int(rng.integers(min_len, 1500))
        hdr = bytearray(40)
        hdr[0] = 0x60
        hdr[4:6] = (ext + plen).to_bytes(2, "big")
        hdr[6] = 0 if ext else nxt
        hdr[7] = 64
        hdr[8:24] = _addr(rng)
        hdr[24:40] = _addr(rng)
        body = rng.integers(0, 256, ext + plen, dtype=np.uint8).tobytes()
        pkts.append(bytes(hdr) + body)
        nxts.append(nxt)
        offs.append(40 + ext)
        lens.append(plen)
    sizes = np.array([len(p) for p in pkts])
    arena = aligned_empty(int(sizes.sum()) + 8 * n + 64)
    seg_off, seg_len, pkt_seg, cur = [], [], [0], 0
    for p in pkts:
        cur += int(rng.integers(0, 8))
        arena[cur:cur + len(p)] = np.frombuffer(p, np.uint8)
        first = min(len(p), 40 + int(rng.integers(0, 200)))
        cuts = [0, first]
        while cuts[-1] < len(p):
            cuts.append(min(len(p), cuts[-1] + int(rng.integers(0, 300))))
        for a, b in zip(cuts[:-1], cuts[1:]):
            seg_off.append(cur + a)
            seg_len.append(b - a)
        pkt_seg.append(len(seg_off))
        cur += len(p)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    return ch, np.array(nxts), np.array(offs), np.array(lens), pkts


@pytest.fixture(scope="module")
def v6():
    return build_ipv6(3000)


def test_in6_oracle_pinned(v6, ora, ref):
    ch, nxt, off, ln, pkts = v6
    got = ora.in6_cksum_batch(ch.heads, nxt, off, ln)
    data = ref.skip_batch(ch.heads, off + ln, off).astype(np.int64)   # reference object
    dfold = (~data) & 0xFFFF
    want = []
    for i in range(ch.n):
        s = _pseudo_py(pkts[i], int(ln[i]), int(nxt[i])) + int(dfold[i])
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        want.append(~s & 0xFFFF)
    np.testing.assert_array_equal(got, np.array(want, np.uint16))


def test_in6_reference_pinned(ora, ref):
    """The reference's own in6_cksum / in6_cksum_pseudo (in6_cksum.c:86-357)
    against the oracle and the engine's per-call host fold.  Segments of at
    least one byte: with len 0 and off at the very end of the chain the
    reference dereferences the NULL m_next (in6_cksum.c:208-217), outside its
    contract (a transport header is never empty)."""
    import libuinet_amd as u

    ch, nxt, off, ln, pkts = build_ipv6(1500, seed=9, min_len=1)
    want = ref.in6_cksum_batch(ch.heads, nxt, off, ln)
    np.testing.assert_array_equal(ora.in6_cksum_batch(ch.heads, nxt, off, ln), want)
    got = [u.in6_cksum(int(ch.heads[i]), int(nxt[i]), int(off[i]), int(ln[i]))
           for i in range(ch.n)]
    np.testing.assert_array_equal(np.array(got, np.uint16), want)
    rng = np.random.default_rng(3)
    for i in range(0, ch.n, 5):
        h = np.frombuffer(pkts[i][:40], np.uint8).copy()
        length = int(rng.integers(0, 1 << 32))
        csum = int(rng.integers(0, 1 << 16))
        w = ref.in6_cksum_pseudo(h.ctypes.data, length, int(nxt[i]), csum)
        assert ora.in6_cksum_pseudo(h.ctypes.data, length, int(nxt[i]), csum) == w
        assert u.in6_cksum_pseudo(h.ctypes.data, length, int(nxt[i]), csum) == w


def _golden_in6(golden):
    g = golden("in6")
    arena = aligned_empty(g["arena"].size)
    arena[:] = g["arena"]
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    return g, ch


def test_in6_golden_per_call_and_oracle(golden, ora):
    import libuinet_amd as u

    g, ch = _golden_in6(golden)
    np.testing.assert_array_equal(ora.in6_cksum_batch(ch.heads, g["nxt"], g["off"], g["len"]),
                                  g["expected"])
    for i in range(ch.n):
        assert u.in6_cksum(int(ch.heads[i]), int(g["nxt"][i]), int(g["off"][i]),
                           int(g["len"][i])) == g["expected"][i]
    for i in range(g["p_hdr"].shape[0]):
        h = np.ascontiguousarray(g["p_hdr"][i])
        args = (h.ctypes.data, int(g["p_len"][i]), int(g["p_nxt"][i]), int(g["p_csum"][i]))
        assert u.in6_cksum_pseudo(*args) == g["p_expected"][i]
        assert ora.in6_cksum_pseudo(*args) == g["p_expected"][i]


@pytest.mark.gpu
def test_in6_golden_gpu(torch_dev, golden):
    import libuinet_amd as u

    g, ch = _golden_in6(golden)
    np.testing.assert_array_equal(u.in6_cksum_batch(ch.heads, g["nxt"], g["off"], g["len"]),
                                  g["expected"])


def test_in6_pseudo_oracle_and_engine(v6, ora):
    import libuinet_amd as u

    ch, nxt, off, ln, pkts = v6
    for i in range(0, ch.n, 7):
        h = np.frombuffer(pkts[i][:40], np.uint8).copy()
        csum = (i * 7919) & 0xFFFF
        want = _pseudo_py(pkts[i], int(ln[i]), int(nxt[i])) + csum
        while want >> 16:
            want = (want & 0xFFFF) + (want >> 16)
        assert ora.in6_cksum_pseudo(h.ctypes.data, int(ln[i]), int(nxt[i]), csum) == want
        assert u.in6_cksum_pseudo(h.ctypes.data, int(ln[i]), int(nxt[i]), csum) == want


def test_in6_self_verification(ora):
    """Store in6_cksum's result in the TCP/UDP checksum field: the segment
    then sums to 0 (what tcp6_input / udp6_input check)."""
    ch, nxt, off, ln, pkts = build_ipv6(400, seed=8)
    keep = [i for i in range(ch.n) if nxt[i] in (6, 17) and ln[i] >= (20 if nxt[i] == 6 else 8)]
    for i in keep:
        fld = int(off[i]) + (16 if nxt[i] == 6 else 6)
        b = bytearray(pkts[i])
        b[fld:fld + 2] = b"\0\0"
        arena = aligned_empty(len(b) + 64)
        arena[:len(b)] = np.frombuffer(bytes(b), np.uint8)
        one = MbufChains.contiguous(arena, [0], len(b))
        c = int(ora.in6_cksum_batch(one.heads, nxt[i], off[i], ln[i])[0])
        arena[fld:fld + 2] = np.frombuffer(np.uint16(c).tobytes(), np.uint8)
        assert int(ora.in6_cksum_batch(one.heads, nxt[i], off[i], ln[i])[0]) == 0


@pytest.mark.gpu
def test_in6_gpu(torch_dev, v6, ora):
    import libuinet_amd as u

    ch, nxt, off, ln, _ = v6
    want = ora.in6_cksum_batch(ch.heads, nxt, off, ln)
    np.testing.assert_array_equal(u.in6_cksum_batch(ch.heads, nxt, off, ln), want)
    for i in range(0, 40):
        assert u.in6_cksum(int(ch.heads[i]), int(nxt[i]), int(off[i]), int(ln[i])) == want[i]
    u.register_host(ch.arena)
    try:
        np.testing.assert_array_equal(u.in6_cksum_batch(ch.heads, nxt, off, ln), want)
        # the mbufs registered too: the GPU walks the chains (csrc/cksum_walk.hip)
        u.register_host(ch.mbufs)
        u.set_tuning("span_fast", 0)  # the device walk even where a chain's sum is in one mbuf
        try:
            w0 = u.host_cpu()["device_walks"]
            np.testing.assert_array_equal(u.in6_cksum_batch(ch.heads, nxt, off, ln), want)
            assert u.host_cpu()["device_walks"] == w0 + 1
        finally:
            u.set_tuning("span_fast", 1)
            u.unregister_host(ch.mbufs)
    finally:
        u.unregister_host(ch.arena)


@pytest.mark.gpu
def test_in6_gpu_single_mbuf_spans(torch_dev, v6, ora):
    """The same IPv6 packets laid out one mbuf each (the RX shape) in one
    registered arena: in6_cksum_batch takes the single-mbuf span path, each
    packet's pseudo-header fold riding as its seed, packet after packet in
    the common-packet run (span_run) -- bit-exact against the oracle."""
    import libuinet_amd as u

    _, nxt, off, ln, pkts = v6
    sizes = np.array([len(p) for p in pkts], np.int64)
    starts = 1 + np.concatenate([[0], np.cumsum(sizes)[:-1]])  # odd and even starts
    arena = aligned_empty(int(starts[-1] + sizes[-1] + 64))
    for s, p in zip(starts, pkts):
        arena[s:s + len(p)] = np.frombuffer(p, np.uint8)
    ch = MbufChains.contiguous(arena, starts, sizes)
    want = ora.in6_cksum_batch(ch.heads, nxt, off, ln)
    u.register_host(arena)
    try:
        s0 = u.host_cpu()["span_batches"]
        np.testing.assert_array_equal(u.in6_cksum_batch(ch.heads, nxt, off, ln), want)
        assert u.host_cpu()["span_batches"] == s0 + 1
    finally:
        u.unregister_host(arena)
