"""Driver batch offload hooks (include/uinet_cksum.h section 2d, SURVEY.md
8f items 1-2): uinet_cksum_tx_offload fills deferred ip_sum / th_sum / uh_sum
like in_delayed_cksum; uinet_cksum_rx_offload verifies a received batch and
marks m_pkthdr the way ip_input / tcp_input / udp_input read an offloading
NIC's verdict.

CPU: the oracle's restatement (oracle/offload_oracle.c) is pinned against the
reference object's own in_cksum_hdr / in_cksum_skip / in_cksum_pseudo_header
on the same frames.  GPU: the engine's hooks equal the oracle's byte for byte
(packet bytes, csum_flags, csum_data, status), staged and zero-copy."""
from __future__ import annotations

import numpy as np
import pytest

from libuinet_amd.frames import FrameBatch, pkthdr_fields

RX_IPV4, RX_IP_OK, RX_L4, RX_L4_OK, RX_NOSUM, RX_FRAG = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
RX_IPV6 = 0x40
TX_L4, TX_IP, TX_L4_LOST, TX_SKIP, TX_IPV6 = 0x01, 0x02, 0x04, 0x08, 0x10
CSUM_IP_CHECKED, CSUM_IP_VALID, CSUM_DATA_VALID, CSUM_PSEUDO_HDR = 0x100, 0x200, 0x400, 0x800


def _ref_rx_verdicts(ref, fb, rx):
    """What the software stack computes for each received frame, with the
    reference object's own functions (m_data at the frame start, so offsets
    count the link header)."""
    n = fb.n
    l3, hl = fb.l3, fb.hlen
    ip_ptr = np.array([rx.arena.ctypes.data + rx.seg_off[rx.pkt_seg[i]] + l3[i] for i in range(n)],
                      np.uint64)
    hdr = ref.hdr_batch(ip_ptr[hl == 20]).astype(np.int64)
    ip_sum = np.zeros(n, np.int64)
    ip_sum[hl == 20] = hdr
    opt = np.flatnonzero(hl != 20)
    if opt.size:
        ip_sum[opt] = ref.skip_batch(rx.heads[opt], (l3 + hl)[opt], l3[opt])
    return ip_sum


def _ip_len(b, l3):
    return int(b[l3 + 2]) << 8 | int(b[l3 + 3])


@pytest.fixture(scope="module")
def frames():
    return lambda seed=11, n=2500, l2=True, ipv6=0.0: FrameBatch(n, seed=seed, l2=l2, ipv6=ipv6)


def test_tx_oracle_against_reference(frames, ora, ref):
    """After the oracle TX hook, every packet it handled verifies with the
    reference's own functions, and the stored sums are what in_cksum_skip of
    the reference returns."""
    fb = frames()
    st = ora.tx_offload(fb.tx.heads)
    assert set(np.unique(st)) <= {TX_IP, TX_L4 | TX_IP, TX_SKIP}
    fl, _ = pkthdr_fields(fb.tx)
    done = (st & TX_IP) != 0
    assert not (fl[done] & 0x7).any()  # handled flags cleared
    # ip_sum: re-zero it in a copy and recompute with the reference object
    for i in np.flatnonzero(done)[:400]:
        b = bytearray(fb.frame_bytes(i))
        l3, hl = int(fb.l3[i]), int(fb.hlen[i])
        stored = b[l3 + 10] | b[l3 + 11] << 8
        b[l3 + 10:l3 + 12] = b"\0\0"
        buf = np.frombuffer(bytes(b), np.uint8).copy()
        from libuinet_amd.mbuf import MbufChains
        ch = MbufChains.contiguous(buf, [l3], hl)
        assert int(ref.skip_batch(ch.heads, hl, 0)[0]) == stored
    # and the receiver's view: everything handled verifies to 0
    rx, arena, _ = fb.rx(seed=4, corrupt=0.0)
    ip_sum = _ref_rx_verdicts(ref, fb, rx)
    assert not ip_sum[done].any()
    l4 = np.flatnonzero((st & TX_L4) != 0)
    plen = np.array([_ip_len(np.frombuffer(fb.frame_bytes(i)[:120], np.uint8), int(fb.l3[i]))
                     for i in l4]) - fb.hlen[l4]
    proto = np.where(np.isin(fb.kinds[l4], ["udp", "udp0"]), 17, 6)
    got = ref.pseudo_header_batch(rx.heads[l4], plen, (fb.l3 + fb.hlen)[l4], fb.src[l4],
                                  fb.dst[l4], proto)
    assert not got.any()


def test_rx_oracle_against_reference(frames, ora, ref):
    """The oracle RX hook's marks encode exactly the software stack's
    verdicts, computed here with the reference object, corrupted frames
    included."""
    fb = frames(seed=12)
    ora.tx_offload(fb.tx.heads)
    rx, arena, bad = fb.rx(seed=5, corrupt=0.2)
    st = ora.rx_offload(rx.heads)
    fl, cd = pkthdr_fields(rx)
    ipv4 = (st & RX_IPV4) != 0
    assert (ipv4 == (fb.kinds != "arp")).all()
    ip_sum = _ref_rx_verdicts(ref, fb, rx)
    assert ((fl & CSUM_IP_CHECKED) != 0).tolist() == ipv4.tolist()
    assert (((fl & CSUM_IP_VALID) != 0) == (ipv4 & (ip_sum == 0))).all()
    assert (((st & RX_IP_OK) != 0) == (ipv4 & (ip_sum == 0))).all()
    l4 = np.flatnonzero((st & RX_L4) != 0)
    assert ((fl[l4] & (CSUM_DATA_VALID | CSUM_PSEUDO_HDR)) == (CSUM_DATA_VALID | CSUM_PSEUDO_HDR)).all()
    # recompute each L4 verdict with the reference from the received bytes
    for i in l4:
        b = np.frombuffer(rx.packet_bytes(i), np.uint8)
        l3, hl = int(fb.l3[i]), int(fb.hlen[i])
        proto = int(b[l3 + 9])
        plen = _ip_len(b, l3) - hl
        if proto == 17:
            plen = int(b[l3 + hl + 4]) << 8 | int(b[l3 + hl + 5])
        src = b[l3 + 12:l3 + 16].view(np.uint32)  # as received (may be corrupted)
        dst = b[l3 + 16:l3 + 20].view(np.uint32)
        want = int(ref.pseudo_header_batch(rx.heads[i:i + 1], plen, l3 + hl, src, dst, proto)[0])
        assert (int(cd[i]) ^ 0xFFFF) == want
        assert bool(st[i] & RX_L4_OK) == (want == 0)
    # uncorrupted TCP/UDP frames all verify; a corrupted one never both verifies
    good = ~bad & np.isin(fb.kinds, ["tcp", "udp"]) & ((fb.flags & 0x20) == 0)
    assert ((st[good] & (RX_IP_OK | RX_L4_OK)) == (RX_IP_OK | RX_L4_OK)).all()
    assert ((st[np.isin(fb.kinds, ["udp0"])] & RX_NOSUM) != 0).all()
    assert ((st[fb.kinds == "frag"] & RX_FRAG) != 0).all()


def test_rx_oracle_header_splits_invariant(frames, ora):
    """RX verdicts do not depend on where the first mbuf ends: the stack pulls
    the headers up (ip_input.c:426,443 m_pullup, tcp_input.c:686) and the
    sums run over the chain.  The oracle marks the same frames identically
    with their headers cut across mbufs (and zero-length mbufs), IPv4 and IPv6
    with extension headers -- the inputs tests/test_device_walk.py
    ::test_hooks_headers_split_across_mbufs gives the engine."""
    from libuinet_amd.frames import split_headers

    fb = frames(seed=14, ipv6=0.3)
    ora.tx_offload(fb.tx.heads)
    rx, _, _ = fb.rx(seed=8, corrupt=0.1)
    whole = ora.rx_offload(rx.heads)
    f_whole = pkthdr_fields(rx)
    split = split_headers(rx, 9)
    assert split.n == rx.n and int(split.pkt_seg[-1]) > int(rx.pkt_seg[-1])
    for x in pkthdr_fields(split):  # fresh marks
        x[:] = 0
    split.mbufs["csum_flags"][split.pkt_seg[:-1]] = 0
    split.mbufs["csum_data"][split.pkt_seg[:-1]] = 0
    rx.mbufs["csum_flags"][rx.pkt_seg[:-1]] = 0
    rx.mbufs["csum_data"][rx.pkt_seg[:-1]] = 0
    assert np.array_equal(ora.rx_offload(split.heads), whole)
    for x, y in zip(pkthdr_fields(split), f_whole):
        assert np.array_equal(x, y)


# ---- IPv6 (ip6_output.c:188-209,966-981; tcp_input.c:627-639; udp6_usrreq.c:216-246)

def _zoned(a: np.ndarray) -> bool:
    """A link-local / link- or interface-local multicast address with a zone
    word (ip6_input.c:658-661 drops the packet)."""
    ll = a[0] == 0xFE and (a[1] & 0xC0) == 0x80
    mc = a[0] == 0xFF and (a[1] & 0x0F) in (1, 2)
    return bool((ll or mc) and (a[2] or a[3]))


def _from_l3(ch, fb, idx):
    """Packets ``idx`` of chains ``ch`` copied from their network header on,
    one mbuf each (the view in6_cksum reads: m_data at the IPv6 header)."""
    from libuinet_amd.mbuf import MbufChains, aligned_empty

    bufs = [ch.packet_bytes(int(i))[int(fb.l3[i]):] for i in idx]
    arena = aligned_empty(2048 * max(1, len(bufs)) + 64)
    for j, b in enumerate(bufs):
        arena[2048 * j:2048 * j + len(b)] = np.frombuffer(b, np.uint8)
    return MbufChains.contiguous(arena, 2048 * np.arange(len(bufs)), [len(b) for b in bufs]), bufs


def _walk6(b: bytes, rx: bool):
    """The IPv6 header chain of ``b`` (bytes from the IPv6 header on) as the
    reference's stack walks it (ip6_input.c:906-913,986-1019, dest6.c:62-123,
    route6.c:59-108, frag6.c:165): (transport offset, next header), ("frag",
    offset) at a fragment header, or None for a packet the stack drops."""
    plen = b[4] << 8 | b[5]
    o, x = 40, b[6]
    for k in range(16 if x == 0 else 15):  # hop-by-hop is outside the nest count
        if x == 0 and k > 0:
            return None
        if x not in (0, 43, 60):
            if o > 40 + plen:
                return None
            return ("frag", o) if x == 44 else (o, x)
        if o + 8 > 40 + plen or len(b) < o + 4:
            return None
        if rx and x == 43 and b[o + 3] != 0:
            return None
        x, o = b[o], o + 8 * (b[o + 1] + 1)
    return None


def test_tx6_oracle_against_reference(frames, ora, ref):
    """IPv6 TX, extension headers included: the frames' checksum-field seeds
    are the reference's own in6_cksum_pseudo; after the oracle TX hook every
    handled IPv6 packet verifies to 0 with the reference's in6_cksum over
    its transport (past the extension headers), and the handled CSUM_*_IPV6
    bits are cleared."""
    fb = frames(seed=13, ipv6=0.5)
    v6 = np.flatnonzero(fb.v6 & ((fb.flags & 0x6000) != 0))
    assert v6.size > 500 and fb.ext6[v6].sum() > 40
    for i in v6:  # the builder's seed == the reference's in6_cksum_pseudo(ip6, len, nxt, 0)
        if fb.rt_left[i] or _zoned(fb.addr6[i][:16]) or _zoned(fb.addr6[i][16:]):
            continue  # routing header with segments left: the seed holds its final address
        b = np.frombuffer(fb.frame_bytes(i), np.uint8)
        l3, off = int(fb.l3[i]), int(fb.hlen[i])
        ip6 = b[l3:l3 + 40].copy()
        nxt, plen = int(fb.nxt6[i]), int(ip6[4]) << 8 | int(ip6[5])
        at = l3 + off + (16 if nxt == 6 else 6)
        stored = int(b[at]) | int(b[at + 1]) << 8
        assert _walk6(bytes(b[l3:]), False) == (off, nxt)
        assert ref.in6_cksum_pseudo(ip6.ctypes.data, plen + 40 - off, nxt, 0) == stored
    st = ora.tx_offload(fb.tx.heads)
    tso = (fb.flags & 0x20) != 0
    want = fb.v6 & ((fb.flags & 0x6000) != 0) & ~tso
    assert (((st & TX_IPV6) != 0) == want).all()
    assert ((st[want] & (TX_L4 | TX_L4_LOST)) == TX_L4).all()
    fl, _ = pkthdr_fields(fb.tx)
    assert not (fl[want] & 0x6000).any()
    assert ((st[fb.v6 & ~want] & TX_SKIP) != 0).all()
    ok = np.array([i for i in np.flatnonzero(want & ~fb.rt_left)
                   if not (_zoned(fb.addr6[i][:16]) or _zoned(fb.addr6[i][16:]))])
    ch, bufs = _from_l3(fb.tx, fb, ok)
    off = fb.hlen[ok]
    plen = np.array([b[4] << 8 | b[5] for b in bufs])
    assert not ref.in6_cksum_batch(ch.heads, fb.nxt6[ok], off, plen + 40 - off).any()


def test_rx6_oracle_against_reference(frames, ora, ref):
    """IPv6 RX: every L4 mark the oracle hook writes encodes the reference's
    own in6_cksum over the received bytes, corrupted frames included; the
    frames the stack would not checksum through tcp6/udp6 get none."""
    fb = frames(seed=14, ipv6=0.5)
    ora.tx_offload(fb.tx.heads)
    rx, arena, bad = fb.rx(seed=7, corrupt=0.2)
    st = ora.rx_offload(rx.heads)
    fl, cd = pkthdr_fields(rx)
    assert (((st & RX_IPV6) != 0) == fb.v6).all()
    assert not (st[fb.v6] & (RX_IPV4 | RX_IP_OK)).any()
    l4 = np.flatnonzero(fb.v6 & ((st & RX_L4) != 0))
    assert l4.size > 500
    ch, bufs = _from_l3(rx, fb, l4)
    walks = [_walk6(b, True) for b in bufs]
    off = np.array([w[0] for w in walks])
    nxt = np.array([w[1] for w in walks])
    plen = np.array([b[4] << 8 | b[5] for b in bufs])
    assert set(np.unique(nxt)) <= {6, 17}
    want = ref.in6_cksum_batch(ch.heads, nxt, off, plen + 40 - off)
    np.testing.assert_array_equal(cd[l4] ^ 0xFFFF, want)
    np.testing.assert_array_equal((st[l4] & RX_L4_OK) != 0, want == 0)
    assert ((fl[l4] & 0xC00) == 0xC00).all()
    zoned = np.array([_zoned(a[:16]) or _zoned(a[16:]) for a in fb.addr6])
    clean = fb.v6 & ~bad & ~zoned
    dropped = fb.rt_left | fb.frag_ext  # route6 drops; frag6 reassembles first
    good = clean & ~dropped & np.isin(fb.kinds, ["tcp", "udp"]) & ((fb.flags & 0x20) == 0)
    assert ((st[good] & (RX_L4 | RX_L4_OK)) == (RX_L4 | RX_L4_OK)).all()
    assert (good & fb.ext6).sum() > 40  # extension headers walked to the transport
    assert not (st[fb.v6 & zoned] & RX_L4).any()
    assert not (st[fb.v6 & dropped] & RX_L4).any()
    assert ((st[clean & (fb.kinds == "udp0")] & RX_NOSUM) != 0).all()
    assert ((st[clean & ((fb.kinds == "frag") | fb.frag_ext)] & RX_FRAG) != 0).all()


# ---- GPU: engine == oracle ------------------------------------------------------

def _twin(frames, seed, l2):
    return frames(seed=seed, l2=l2), frames(seed=seed, l2=l2)


@pytest.mark.gpu
@pytest.mark.parametrize("l2,zero_copy", [(True, False), (True, True), (False, False)])
def test_offload_gpu_matches_oracle(torch_dev, frames, ora, l2, zero_copy):
    import libuinet_amd as u

    l2len = -1 if l2 else 0
    a, b = _twin(frames, 21, l2)
    if zero_copy:
        u.register_host(a.arena)
    try:
        st_g = u.tx_offload(a.tx.heads, l2len)
    finally:
        if zero_copy:
            u.unregister_host(a.arena)
    st_o = ora.tx_offload(b.tx.heads, l2len)
    np.testing.assert_array_equal(st_g, st_o)
    np.testing.assert_array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        np.testing.assert_array_equal(x, y)
    rx_a, arena_a, _ = a.rx(seed=6, corrupt=0.15)
    rx_b, arena_b, _ = b.rx(seed=6, corrupt=0.15)
    if zero_copy:
        u.register_host(arena_a)
    try:
        st_g = u.rx_offload(rx_a.heads, l2len)
    finally:
        if zero_copy:
            u.unregister_host(arena_a)
    st_o = ora.rx_offload(rx_b.heads, l2len)
    np.testing.assert_array_equal(st_g, st_o)
    for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
        np.testing.assert_array_equal(x, y)
    assert ((st_g & RX_L4_OK) != 0).any() and (((st_g & RX_L4) != 0) & ((st_g & RX_L4_OK) == 0)).any()


@pytest.mark.gpu
@pytest.mark.parametrize("l2,zero_copy", [(True, False), (True, True), (False, False)])
def test_offload6_gpu_matches_oracle(torch_dev, frames, ora, l2, zero_copy):
    """A mixed IPv4 / IPv6 batch through both hooks: the engine's bytes,
    marks and status equal the oracle's."""
    import libuinet_amd as u

    l2len = -1 if l2 else 0
    a, b = frames(seed=23, l2=l2, ipv6=0.4), frames(seed=23, l2=l2, ipv6=0.4)
    if zero_copy:
        u.register_host(a.arena)
    try:
        st_g = u.tx_offload(a.tx.heads, l2len)
    finally:
        if zero_copy:
            u.unregister_host(a.arena)
    st_o = ora.tx_offload(b.tx.heads, l2len)
    np.testing.assert_array_equal(st_g, st_o)
    np.testing.assert_array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        np.testing.assert_array_equal(x, y)
    assert ((st_g & (TX_IPV6 | TX_L4)) == (TX_IPV6 | TX_L4)).sum() > 300
    rx_a, arena_a, _ = a.rx(seed=8, corrupt=0.15)
    rx_b, arena_b, _ = b.rx(seed=8, corrupt=0.15)
    if zero_copy:
        u.register_host(arena_a)
    try:
        st_g = u.rx_offload(rx_a.heads, l2len)
    finally:
        if zero_copy:
            u.unregister_host(arena_a)
    st_o = ora.rx_offload(rx_b.heads, l2len)
    np.testing.assert_array_equal(st_g, st_o)
    for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
        np.testing.assert_array_equal(x, y)
    v6 = (st_g & RX_IPV6) != 0
    assert (v6 & ((st_g & RX_L4_OK) != 0)).sum() > 300
    assert (v6 & ((st_g & RX_L4) != 0) & ((st_g & RX_L4_OK) == 0)).any()


@pytest.mark.gpu
def test_offload_gpu_empty_and_bad_args(torch_dev):
    import libuinet_amd as u

    assert u.rx_offload(np.zeros(0, np.uint64)).size == 0
    assert u.tx_offload(np.zeros(0, np.uint64)).size == 0
    with pytest.raises(u.CksumError):
        u.rx_offload(np.zeros(1, np.uint64), l2len=-2)
    # NULL packets are skipped, not dereferenced
    assert u.tx_offload(np.zeros(3, np.uint64)).tolist() == [TX_SKIP] * 3
    assert u.rx_offload(np.zeros(3, np.uint64)).tolist() == [0] * 3


def _pcap_rx(frames):
    """Every frame of the reference's passive_extract_test.pcap as received:
    one cluster each, m_data at the Ethernet header."""
    from libuinet_amd.mbuf import MbufChains, aligned_empty

    arena = aligned_empty(2048 * len(frames) + 64)
    for i, f in enumerate(frames):
        arena[2048 * i:2048 * i + len(f)] = np.frombuffer(f, np.uint8)
    return MbufChains.contiguous(arena, 2048 * np.arange(len(frames)),
                                 [len(f) for f in frames]), arena


def test_pcap_rx_offload_oracle(ora, pcap_frames):
    """The reference's own capture through the RX hook (SURVEY.md 8f item 3,
    without libpcap): every IPv4/TCP frame is marked IP-valid and
    data-valid with csum_data 0xffff, exactly what if_loop.c:96-101 sets."""
    rx, _ = _pcap_rx(pcap_frames)
    st = ora.rx_offload(rx.heads)
    fl, cd = pkthdr_fields(rx)
    tcp = (st & RX_L4) != 0
    assert tcp.sum() >= 113
    assert ((st[tcp] & (RX_IPV4 | RX_IP_OK | RX_L4 | RX_L4_OK)) == 0x0F).all()
    assert (cd[tcp] == 0xFFFF).all()
    assert ((fl[tcp] & 0xF00) == 0xF00).all()


@pytest.mark.gpu
def test_pcap_rx_offload_gpu(torch_dev, ora, pcap_frames):
    import libuinet_amd as u

    rx_g, _ = _pcap_rx(pcap_frames)
    rx_o, _ = _pcap_rx(pcap_frames)
    np.testing.assert_array_equal(u.rx_offload(rx_g.heads), ora.rx_offload(rx_o.heads))
    for x, y in zip(pkthdr_fields(rx_g), pkthdr_fields(rx_o)):
        np.testing.assert_array_equal(x, y)


def _pcap_fragmented(frames, seed):
    """The capture's frames re-chained as m_fragment() does under
    MBUF_STRESS_TEST (uipc_mbuf.c:1693-1761): random 1-256-B mbufs, each at a
    random 0-7-B offset (SURVEY.md section 4's KAT)."""
    from libuinet_amd.mbuf import MbufChains, aligned_empty

    rng = np.random.default_rng(seed)
    arena = aligned_empty(sum(len(f) for f in frames) * 2 + 8 * 4096)
    seg_off, seg_len, pkt_seg, cur = [], [], [0], 0
    for f in frames:
        b = np.frombuffer(f, np.uint8)
        i = 0
        while i < b.size:
            k = min(int(rng.integers(1, 257)), b.size - i)
            cur += int(rng.integers(0, 8))
            arena[cur:cur + k] = b[i:i + k]
            seg_off.append(cur)
            seg_len.append(k)
            cur += k
            i += k
        pkt_seg.append(len(seg_off))
    return MbufChains(arena, seg_off, seg_len, pkt_seg), arena


def test_pcap_rx_offload_fragmented_oracle(ora, pcap_frames):
    """the capture verifies to 0 also when every frame
    is re-chained into random 1-256-B fragments -- through the RX hook's
    restatement (the stack's pull-ups modelled) every TCP frame is still
    marked IP-valid and data-valid, exactly as unfragmented."""
    for seed in (1, 2, 3):
        rx, _ = _pcap_fragmented(pcap_frames, seed)
        st = ora.rx_offload(rx.heads)
        tcp = (st & RX_L4) != 0
        assert tcp.sum() >= 113
        assert ((st[tcp] & (RX_IPV4 | RX_IP_OK | RX_L4 | RX_L4_OK)) == 0x0F).all()
        _, cd = pkthdr_fields(rx)
        assert (cd[tcp] == 0xFFFF).all()


@pytest.mark.gpu
@pytest.mark.parametrize("registered", [False, True])
def test_pcap_rx_offload_fragmented_gpu(torch_dev, ora, pcap_frames, registered):
    """The same fragmented capture through the engine's RX hook: the host hook
    (staged), and with mbufs and bytes registered the device hook (the capture
    repeated 20 times, 2,260 frames: a device-sized batch), against the oracle."""
    import libuinet_amd as u

    frames = list(pcap_frames) * (20 if registered else 1)
    rx_g, arena_g = _pcap_fragmented(frames, 4)
    rx_o, _ = _pcap_fragmented(frames, 4)
    regs = (arena_g, rx_g.mbufs) if registered else ()
    for b in regs:
        u.register_host(b)
    try:
        before = u.host_cpu()["device_walks"]
        st = u.rx_offload(rx_g.heads)
        walked = u.host_cpu()["device_walks"] - before
    finally:
        for b in regs:
            u.unregister_host(b)
    assert walked == (1 if registered else 0)
    np.testing.assert_array_equal(st, ora.rx_offload(rx_o.heads))
    for x, y in zip(pkthdr_fields(rx_g), pkthdr_fields(rx_o)):
        np.testing.assert_array_equal(x, y)


# ---- IPv6 header-nest limit (ip6_input.c:906-913,986-990; in6_proto.c:406) -------

def _nest_frames(cases):
    """Ethernet + IPv6 + the given extension headers (hop-by-hop first when
    `hbh`, then `ndst` destination-options headers of 8 bytes) + a TCP header
    with a correct th_sum + 32 payload bytes, one cluster per frame."""
    from libuinet_amd.frames import pseudo6
    from libuinet_amd.mbuf import MbufChains, aligned_empty

    rng = np.random.default_rng(77)
    frames = []
    for hbh, ndst in cases:
        types = ([0] if hbh else []) + [60] * ndst
        ext = bytearray()
        for j, _t in enumerate(types):
            nxt = types[j + 1] if j + 1 < len(types) else 6
            ext += bytes([nxt, 0, 1, 4, 0, 0, 0, 0])  # PadN over the option space
        tcp = bytearray(rng.integers(0, 256, 20 + 32, dtype=np.uint8).tobytes())
        tcp[12] = 5 << 4  # data offset 5
        tcp[16:18] = b"\0\0"
        src = bytes([0x20, 0x01]) + rng.integers(0, 256, 14, dtype=np.uint8).tobytes()
        dst = bytes([0x20, 0x01]) + rng.integers(0, 256, 14, dtype=np.uint8).tobytes()
        s = pseudo6(src, dst, len(tcp), 6) + int(np.frombuffer(bytes(tcp), "<u2").sum())
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        tcp[16:18] = (~s & 0xFFFF).to_bytes(2, "little")
        plen = len(ext) + len(tcp)
        ip6 = bytes([0x60, 0, 0, 0]) + plen.to_bytes(2, "big") + bytes(
            [types[0] if types else 6, 64]) + src + dst
        eth = rng.integers(0, 256, 12, dtype=np.uint8).tobytes() + b"\x86\xdd"
        frames.append(eth + ip6 + bytes(ext) + bytes(tcp))
    arena = aligned_empty(2048 * len(frames) + 64)
    for i, f in enumerate(frames):
        arena[2048 * i:2048 * i + len(f)] = np.frombuffer(f, np.uint8)
    ch = MbufChains.contiguous(arena, 2048 * np.arange(len(frames)), [len(f) for f in frames])
    return ch, frames


NEST_CASES = [(True, 13), (True, 14), (True, 15), (False, 13), (False, 14), (False, 15),
              (True, 0), (False, 0)]
# the stack reaches tcp6_input (and so reads an offload mark) when the loop's
# headers, transport included, are at most 15: hop-by-hop + 14, or 14 alone
NEST_OK = [True, True, False, True, True, False, True, True]


def test_ipv6_nest_limit_oracle(ora):
    ch, frames = _nest_frames(NEST_CASES)
    for f, ok in zip(frames, NEST_OK):
        w = _walk6(f[14:], True)
        assert (w is not None) == ok and (not ok or w[1] == 6)
    st = ora.rx_offload(ch.heads)
    assert ((st & RX_IPV6) != 0).all()
    for s, ok in zip(st, NEST_OK):
        assert ((s & (RX_L4 | RX_L4_OK)) == (RX_L4 | RX_L4_OK)) == ok, (hex(s), ok)


@pytest.mark.gpu
def test_ipv6_nest_limit_gpu(torch_dev, ora):
    import libuinet_amd as u

    ch_g, _ = _nest_frames(NEST_CASES)
    ch_o, _ = _nest_frames(NEST_CASES)
    np.testing.assert_array_equal(u.rx_offload(ch_g.heads), ora.rx_offload(ch_o.heads))
    for x, y in zip(pkthdr_fields(ch_g), pkthdr_fields(ch_o)):
        np.testing.assert_array_equal(x, y)
