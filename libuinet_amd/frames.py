"""Synthetic Ethernet/IPv4 frame batches for the driver offload hooks
(``uinet_cksum_rx_offload`` / ``uinet_cksum_tx_offload``): tests and
tests/perf/offload_rate.py.

A TX batch is laid out the way tcp_output / udp_output hand packets to the
driver when the interface advertises checksum offload: a header mbuf holding
the link + IP + L4 headers (M_PKTHDR, csum_flags CSUM_IP | CSUM_TCP or
CSUM_UDP, csum_data = offsetof(th_sum) 16 or offsetof(uh_sum) 6, the
in_pseudo seed already in the L4 checksum field, tcp_output.c:1062,1080-1081
and udp_usrreq.c:1184-1197) chained to payload slices of 4-KiB page clusters.
An RX batch is the same frames as a driver receives them: one 2-KiB cluster
each, or split into 2-3 mbufs after the headers.

The mix covers what the hooks must tell apart: TCP, UDP, UDP without a
checksum, IP options, 802.1Q tags, fragments, other protocols, non-IP
frames, and (RX) corrupted headers / payloads / checksum fields.

With ``ipv6 > 0`` that share of the IP frames is IPv6 instead (Ethernet type
0x86dd): TCP / UDP after the fixed header with the in6_cksum_pseudo seed in
the checksum field and CSUM_TCP_IPV6 / CSUM_UDP_IPV6 (tcp_output.c:
1069-1071, udp6_usrreq.c:786), UDP with a zero checksum, fragments (next
header 44), ICMPv6, and global, link-local and (rarely) zone-carrying
link-local addresses.  12 % of the IPv6 TCP / UDP frames carry extension
headers (``ext6``): hop-by-hop and destination options (PadN), routing
headers with no segments left, a routing header with one segment left
(``rt_left``: the receiver drops it, route6.c:99-105; the seed holds the
final destination, the address in the routing header) or a fragment header
after hop-by-hop options (``frag_ext``, no offload flags).  ``nxt6`` is the
transport protocol.  The IPv4 frames' random stream does not depend on
``ipv6``.
"""
from __future__ import annotations

import numpy as np

from .mbuf import MbufChains, aligned_empty

CSUM_IP, CSUM_TCP, CSUM_UDP, CSUM_TSO = 0x1, 0x2, 0x4, 0x20
CSUM_UDP_IPV6, CSUM_TCP_IPV6 = 0x2000, 0x4000


def _in_pseudo(a: int, b: int, c: int) -> int:
    s = a + b + c
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _bs16(x: int) -> int:
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


def pseudo6(src: bytes, dst: bytes, length: int, nxt: int) -> int:
    """in6_cksum_pseudo(ip6, len, nxt, 0) for wire addresses (in6_cksum.c:
    86-140): both addresses, htonl(len) and nxt as little-endian 16-bit
    words, folded with end-around carry, not complemented."""
    a = np.frombuffer(bytes(src) + bytes(dst), "<u2")
    s = int(a.sum()) + _bs16(length >> 16) + _bs16(length & 0xFFFF) + _bs16(nxt)
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _addr6(rng) -> np.ndarray:
    """Mostly global unicast; 15 % link-local (zone word 0 as on the wire);
    3 % link-local with a nonzero zone word (ip6_input drops those)."""
    a = rng.integers(0, 256, 16, dtype=np.uint8)
    r = rng.random()
    if r < 0.82:
        a[0] = 0x20 | (a[0] & 0x0F)
    else:
        a[0:8] = (0xFE, 0x80, 0, 0, 0, 0, 0, 0)
        if r > 0.97:
            a[2:4] = (0, 1 + int(rng.integers(0, 255)))
    return a


class FrameBatch:
    """n frames (TX shape): ``tx`` chains + per-packet metadata."""

    def __init__(self, n: int, seed: int = 1, vlan: float = 0.1, l2: bool = True,
                 ipv6: float = 0.0):
        rng = np.random.default_rng(seed)
        rng6 = np.random.default_rng(seed + 0x6600)
        self.n = n
        self.l2 = l2
        kinds = rng.choice(["tcp", "udp", "udp0", "frag", "icmp", "arp"], n,
                           p=[0.6, 0.22, 0.04, 0.05, 0.05, 0.04] if l2 else
                           [0.62, 0.24, 0.04, 0.05, 0.05, 0.0])
        self.kinds = kinds
        self.v6 = (rng6.random(n) < ipv6) & (kinds != "arp")
        self.ext6 = self.v6 & np.isin(kinds, ["tcp", "udp"]) & (rng6.random(n) < 0.12)
        self.rt_left = np.zeros(n, bool)
        self.frag_ext = np.zeros(n, bool)
        self.nxt6 = np.zeros(n, np.int64)
        self.addr6 = np.zeros((n, 32), np.uint8)
        hdr_slot = 256
        pay = np.where(rng.random(n) < 0.15, rng.integers(0, 64, n), rng.integers(64, 1461, n))
        total_pay = int(pay.sum())
        nclus = total_pay // 4096 + 2
        self.clus0 = hdr_slot * n
        self.arena = aligned_empty(self.clus0 + nclus * 4096 + 64)
        self.arena[self.clus0:] = rng.integers(0, 256, self.arena.size - self.clus0, dtype=np.uint8)
        perm = rng.permutation(nclus)
        seg_off, seg_len, pkt_seg = [], [], [0]
        self.flags = np.zeros(n, np.int32)
        self.cdata = np.zeros(n, np.int32)
        self.hlen = np.zeros(n, np.int64)
        self.l3 = np.zeros(n, np.int64)
        self.hdr_off = np.zeros(n, np.int64)
        self.hdr_len = np.zeros(n, np.int64)
        self.src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        self.dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        cursor = 0
        for i in range(n):
            k = kinds[i]
            p = int(pay[i])
            if self.v6[i]:
                h = self._header6(i, k, p, l2, vlan, rng6)
            else:
                h = self._header4(i, k, p, l2, vlan, rng)
            if self.v6[i] and rng6.random() < 0.02:
                self.flags[i] |= CSUM_TSO  # the hooks leave TSO packets to the driver
            ho = hdr_slot * i + 104  # m_pktdat (88) + max_linkhdr (16); <= 98 header bytes
            self.arena[ho:ho + h.size] = h
            self.hdr_off[i], self.hdr_len[i] = ho, h.size
            seg_off.append(ho)
            seg_len.append(h.size)
            # payload: the socket buffer's next p bytes, 1-2 page-cluster slices
            s0 = cursor
            cursor += p
            c, o = divmod(s0, 4096)
            first = min(p, 4096 - o)
            if p:
                seg_off.append(self.clus0 + int(perm[c]) * 4096 + o)
                seg_len.append(first)
                if first < p:
                    seg_off.append(self.clus0 + int(perm[c + 1]) * 4096)
                    seg_len.append(p - first)
            pkt_seg.append(len(seg_off))
        self.tx = MbufChains(self.arena, seg_off, seg_len, pkt_seg)
        self.set_tx_flags()

    def _ext_chain(self, i, k, rng):
        """The extension headers of frame i as (next-header type, bytes) in
        wire order (each header's first byte is filled in by the caller), and
        the final destination a routing header with segments left carries."""
        if k == "frag":
            return [(44, rng.integers(0, 256, 8, dtype=np.uint8))], None
        if not self.ext6[i]:
            return [], None

        def opts(n8):  # n8 x 8 bytes of options: one PadN
            h = np.zeros(8 * n8, np.uint8)
            h[1], h[2], h[3] = n8 - 1, 1, 8 * n8 - 4
            return h

        def rt(left, final):
            h = np.zeros(24, np.uint8)
            h[1], h[2], h[3] = 2, 2, left  # type 2 (one address), segments left
            h[8:24] = final
            return h

        final = None
        r = rng.random()
        if r < 0.30:
            chain = [(0, opts(1))]
        elif r < 0.50:
            chain = [(60, opts(2))]
        elif r < 0.65:
            chain = [(0, opts(1)), (43, rt(0, _addr6(rng)))]
        elif r < 0.80:
            chain = [(0, opts(1)), (60, opts(1)), (43, rt(0, _addr6(rng)))]
        elif r < 0.88:
            chain = [(60, opts(1)), (43, rt(0, _addr6(rng))), (60, opts(1))]
        elif r < 0.94:
            final = _addr6(rng)
            chain = [(43, rt(1, final))]
            self.rt_left[i] = True
        else:
            chain = [(0, opts(1)), (44, rng.integers(0, 256, 8, dtype=np.uint8))]
            self.frag_ext[i] = True
        return chain, final

    def _header6(self, i, k, p, l2, vlan, rng):
        """Link + IPv6 (+ extension headers) + L4 header of frame i."""
        tag = l2 and rng.random() < vlan
        l3 = (18 if tag else 14) if l2 else 0
        nxt = {"tcp": 6, "frag": 6, "udp": 17, "udp0": 17, "icmp": 58}[k]
        chain, final = self._ext_chain(i, k, rng)
        ext = sum(int(b.size) for _, b in chain)
        l4h = 20 if nxt == 6 else 8
        plen = ext + l4h + p
        h = np.zeros(l3 + 40 + ext + l4h, np.uint8)
        if l2:
            h[0:12] = rng.integers(0, 256, 12, dtype=np.uint8)
            if tag:
                h[12:14] = (0x81, 0x00)
                h[14:16] = rng.integers(0, 256, 2, dtype=np.uint8)
            h[l3 - 2:l3] = (0x86, 0xDD)
        ip6 = h[l3:l3 + 40]
        ip6[0] = 0x60
        ip6[1:4] = rng.integers(0, 256, 3, dtype=np.uint8)
        ip6[1] &= 0x0F
        ip6[4:6] = (plen >> 8, plen & 0xFF)
        ip6[6] = chain[0][0] if chain else nxt
        ip6[7] = 64
        src, dst = _addr6(rng), _addr6(rng)
        ip6[8:24], ip6[24:40] = src, dst
        self.addr6[i] = np.concatenate([src, dst])
        o = l3 + 40
        for j, (_, b) in enumerate(chain):
            h[o:o + b.size] = b
            h[o] = chain[j + 1][0] if j + 1 < len(chain) else nxt
            o += b.size
        l4 = h[l3 + 40 + ext:]
        l4[:] = rng.integers(0, 256, l4h, dtype=np.uint8)
        fdst = dst if final is None else final  # the pseudo header's destination
        offload = k != "frag" and not self.frag_ext[i]
        fl, cd = 0, 0
        if nxt == 6:
            l4[12] = 0x50
            seed16 = pseudo6(src, fdst, l4h + p, 6)
            l4[16:18] = (seed16 & 0xFF, seed16 >> 8)
            if offload:
                fl, cd = CSUM_TCP_IPV6, 16
        elif nxt == 17:
            ulen = 8 + p
            l4[4:6] = (ulen >> 8, ulen & 0xFF)
            if k == "udp0":
                l4[6:8] = 0
            else:
                seed16 = pseudo6(src, fdst, ulen, 17)
                l4[6:8] = (seed16 & 0xFF, seed16 >> 8)
                if offload:
                    fl, cd = CSUM_UDP_IPV6, 6
        self.flags[i], self.cdata[i] = fl, cd
        self.l3[i], self.hlen[i], self.nxt6[i] = l3, 40 + ext, nxt
        return h

    def _header4(self, i, k, p, l2, vlan, rng):
        """Link + IPv4 + L4 header of frame i (the original stream)."""
        tag = l2 and rng.random() < vlan
        l3 = (18 if tag else 14) if l2 else 0
        hl = 20 if rng.random() < 0.85 else int(rng.integers(6, 16)) * 4
        proto = {"tcp": 6, "udp": 17, "udp0": 17, "frag": 6, "icmp": 1, "arp": 0}[k]
        l4h = 20 if proto == 6 else 8 if proto == 17 else 0
        ip_len = hl + l4h + p
        h = np.zeros(l3 + hl + l4h, np.uint8)
        if l2:
            h[0:12] = rng.integers(0, 256, 12, dtype=np.uint8)
            if tag:
                h[12:14] = (0x81, 0x00)
                h[14:16] = rng.integers(0, 256, 2, dtype=np.uint8)
            h[l3 - 2:l3] = (0x08, 0x06) if k == "arp" else (0x08, 0x00)
        ip = h[l3:l3 + hl]
        ip[0] = 0x40 | (hl // 4)
        ip[2:4] = (ip_len >> 8, ip_len & 0xFF)
        ip[4:6] = rng.integers(0, 256, 2, dtype=np.uint8)
        ip[6] = 0x20 if k == "frag" else 0x40
        ip[8] = 64
        ip[9] = proto
        ip[12:16] = np.frombuffer(self.src[i].tobytes(), np.uint8)
        ip[16:20] = np.frombuffer(self.dst[i].tobytes(), np.uint8)
        if hl > 20:
            ip[20:hl] = rng.integers(0, 256, hl - 20, dtype=np.uint8)
        l4 = h[l3 + hl:]
        l4[:] = rng.integers(0, 256, l4h, dtype=np.uint8)
        fl = 0 if k == "arp" else CSUM_IP
        if proto == 6:
            l4[12] = 0x50
            seed16 = _in_pseudo(int(self.src[i]), int(self.dst[i]), _bs16(l4h + 6 + p))
            l4[16:18] = (seed16 & 0xFF, seed16 >> 8)  # native-order u16 store
            if k != "frag":
                fl |= CSUM_TCP
                self.cdata[i] = 16
        elif proto == 17:
            ulen = 8 + p
            l4[4:6] = (ulen >> 8, ulen & 0xFF)
            if k == "udp0":
                l4[6:8] = 0
            else:
                seed16 = _in_pseudo(int(self.src[i]), int(self.dst[i]), _bs16(ulen + 17))
                l4[6:8] = (seed16 & 0xFF, seed16 >> 8)
                fl |= CSUM_UDP
                self.cdata[i] = 6
        if rng.random() < 0.02:
            fl |= CSUM_TSO  # the hooks leave TSO packets to the driver
        self.flags[i] = fl
        self.l3[i], self.hlen[i] = l3, hl
        return h

    def set_tx_flags(self) -> None:
        first = self.tx.pkt_seg[:-1]
        self.tx.mbufs["csum_flags"][first] = self.flags
        self.tx.mbufs["csum_data"][first] = self.cdata

    def frame_bytes(self, i: int) -> bytes:
        return self.tx.packet_bytes(i)

    def rx(self, seed: int = 2, split: float = 0.3, corrupt: float = 0.1):
        """The frames as received: (MbufChains, arena, corrupted mask).  Each
        frame sits in its own 2-KiB cluster at a 0-3-B offset; ``split`` of
        them are cut into 2-3 mbufs after the L4 header; ``corrupt`` of them
        get one byte flipped (header, checksum field or payload)."""
        rng = np.random.default_rng(seed)
        n = self.n
        arena = aligned_empty(n * 2048 + 64)
        seg_off, seg_len, pkt_seg = [], [], [0]
        bad = np.zeros(n, bool)
        for i in range(n):
            b = np.frombuffer(self.frame_bytes(i), np.uint8).copy()
            l3 = int(self.l3[i])
            if rng.random() < corrupt and b.size > l3 + 1:
                # any byte after the link header and the version/IHL byte
                j = int(rng.integers(l3 + 1, b.size))
                b[j] ^= np.uint8(1 << int(rng.integers(0, 8)))
                bad[i] = True
            o = 2048 * i + int(rng.integers(0, 4))
            arena[o:o + b.size] = b
            hdr_end = int(self.l3[i] + self.hlen[i] + 20)
            if rng.random() < split and b.size > hdr_end + 2:
                cut1 = int(rng.integers(hdr_end, b.size))
                cuts = [0, cut1]
                if rng.random() < 0.5 and b.size > cut1 + 1:
                    cuts.append(int(rng.integers(cut1 + 1, b.size)))
                cuts.append(b.size)
                for a, e in zip(cuts[:-1], cuts[1:]):
                    seg_off.append(o + a)
                    seg_len.append(e - a)
            else:
                seg_off.append(o)
                seg_len.append(b.size)
            pkt_seg.append(len(seg_off))
        return MbufChains(arena, seg_off, seg_len, pkt_seg), arena, bad


def pkthdr_fields(ch: MbufChains):
    """(csum_flags, csum_data) of every packet's first mbuf."""
    first = ch.pkt_seg[:-1]
    return ch.mbufs["csum_flags"][first].copy(), ch.mbufs["csum_data"][first].copy()


def split_headers(ch: MbufChains, seed: int, frac: float = 0.7, upto: int = 80) -> MbufChains:
    """The same frames with the first mbuf of `frac` of them cut inside the
    headers (at 1 .. `upto` bytes), sometimes with a zero-length mbuf after the
    cut: the parse's reads that leave the first mbuf (offload_parse.h,
    View::bytes / read) -- no generated batch splits a header otherwise."""
    rng = np.random.default_rng(seed)
    so, sl, ps = [], [], [0]
    for i in range(ch.n):
        a, e = int(ch.pkt_seg[i]), int(ch.pkt_seg[i + 1])
        offs = [int(x) for x in ch.seg_off[a:e]]
        lens = [int(x) for x in ch.seg_len[a:e]]
        if lens and lens[0] > 1 and rng.random() < frac:
            c = int(rng.integers(1, min(lens[0], upto)))
            head = [(offs[0], c)] + ([(offs[0] + c, 0)] if rng.random() < 0.2 else [])
            segs = head + [(offs[0] + c, lens[0] - c)] + list(zip(offs[1:], lens[1:]))
        else:
            segs = list(zip(offs, lens))
        for o, ln in segs:
            so.append(o)
            sl.append(ln)
        ps.append(len(so))
    out = MbufChains(ch.arena, np.array(so, np.int64), np.array(sl, np.int64),
                     np.array(ps, np.int64))
    f_old, f_new = ch.pkt_seg[:-1], out.pkt_seg[:-1]
    out.mbufs["csum_flags"][f_new] = ch.mbufs["csum_flags"][f_old]
    out.mbufs["csum_data"][f_new] = ch.mbufs["csum_data"][f_old]
    return out


def mangle_headers(ch: MbufChains, fb: FrameBatch, seed: int, frac: float = 0.5) -> MbufChains:
    """The same frames with `frac` of them made malformed the ways the stack's
    input checks name (ip_input.c:416-500, ip6_input.c:519-700, udp_usrreq.c:
    404-420, udp6_usrreq.c:216-230): a wrong version or header length nibble,
    a wrong ethertype, IP / IPv6 / UDP length fields too short or too long, a
    transport or extension-header type or length changed, the chain cut
    inside its headers, or nothing but empty mbufs.  Header bytes are changed
    in `ch`'s arena in place (apply the same seed to a twin batch for the
    oracle); the returned chains carry the cuts.  `fb` is the batch the frames
    came from (its l3 / header offsets)."""
    rng = np.random.default_rng(seed)
    so, sl, ps = [], [], [0]
    for i in range(ch.n):
        a, e = int(ch.pkt_seg[i]), int(ch.pkt_seg[i + 1])
        offs = [int(x) for x in ch.seg_off[a:e]]
        lens = [int(x) for x in ch.seg_len[a:e]]
        size = sum(lens)

        def poke(j, v):
            for o, ln in zip(offs, lens):
                if j < ln:
                    ch.arena[o + j] = v & 0xFF
                    return
                j -= ln

        def peek(j):
            for o, ln in zip(offs, lens):
                if j < ln:
                    return int(ch.arena[o + j])
                j -= ln
            return 0

        l3, hl, v6 = int(fb.l3[i]), int(fb.hlen[i]), bool(fb.v6[i])
        kind = int(rng.integers(0, 9)) if size > l3 and rng.random() < frac else -1
        if kind == 0:  # header length nibble
            poke(l3, (peek(l3) & 0xF0) | int(rng.integers(0, 16)))
        elif kind == 1:  # version nibble
            poke(l3, int(rng.integers(0, 16)) << 4 | (peek(l3) & 0x0F))
        elif kind == 2 and l3 >= 14:  # ethertype
            t = [(0x08, 0x00), (0x86, 0xDD), (0x81, 0x00), (0x08, 0x06),
                 tuple(int(x) for x in rng.integers(0, 256, 2))][int(rng.integers(0, 5))]
            poke(l3 - 2, t[0])
            poke(l3 - 1, t[1])
        elif kind == 3:  # IP total / IPv6 payload length
            act = size - l3 - (40 if v6 else 0)
            v = int(rng.choice([0, 1, 7, max(hl - 1, 0), hl, act - 1, act + 1, 65535,
                                int(rng.integers(0, 65536))])) & 0xFFFF
            poke(l3 + (4 if v6 else 2), v >> 8)
            poke(l3 + (5 if v6 else 3), v)
        elif kind == 4 and fb.kinds[i] in ("udp", "udp0"):  # UDP length
            act = size - l3 - hl
            v = int(rng.choice([0, 7, 8, act - 1, act + 1, 65535])) & 0xFFFF
            poke(l3 + hl + 4, v >> 8)
            poke(l3 + hl + 5, v)
        elif kind == 5:  # the chain cut inside or just past its headers
            keep = int(rng.integers(0, min(size, l3 + hl + 28) + 1))
            nl = []
            for ln in lens:
                nl.append(min(ln, keep))
                keep -= nl[-1]
            lens = nl
        elif kind == 6 and v6:  # the first extension header's length
            poke(l3 + 41, int(rng.integers(0, 256)))
        elif kind == 7:  # only empty mbufs
            lens = [0] * len(lens)
        elif kind == 8:  # transport / next-header type
            pool = [0, 6, 17, 43, 44, 58, 59, 60] if v6 else [0, 1, 6, 17, 44, 58]
            poke(l3 + (6 if v6 else 9), int(rng.choice(pool + [int(rng.integers(0, 256))])))
        so.extend(offs)
        sl.extend(lens)
        ps.append(len(so))
    out = MbufChains(ch.arena, np.array(so, np.int64), np.array(sl, np.int64),
                     np.array(ps, np.int64))
    f_old, f_new = ch.pkt_seg[:-1], out.pkt_seg[:-1]
    out.mbufs["csum_flags"][f_new] = ch.mbufs["csum_flags"][f_old]
    out.mbufs["csum_data"][f_new] = ch.mbufs["csum_data"][f_old]
    return out
