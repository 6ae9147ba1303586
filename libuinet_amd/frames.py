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
"""
from __future__ import annotations

import numpy as np

from .mbuf import MbufChains, aligned_empty

CSUM_IP, CSUM_TCP, CSUM_UDP, CSUM_TSO = 0x1, 0x2, 0x4, 0x20


def _in_pseudo(a: int, b: int, c: int) -> int:
    s = a + b + c
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _bs16(x: int) -> int:
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


class FrameBatch:
    """n frames (TX shape): ``tx`` chains + per-packet metadata."""

    def __init__(self, n: int, seed: int = 1, vlan: float = 0.1, l2: bool = True):
        rng = np.random.default_rng(seed)
        self.n = n
        self.l2 = l2
        kinds = rng.choice(["tcp", "udp", "udp0", "frag", "icmp", "arp"], n,
                           p=[0.6, 0.22, 0.04, 0.05, 0.05, 0.04] if l2 else
                           [0.62, 0.24, 0.04, 0.05, 0.05, 0.0])
        self.kinds = kinds
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
            tag = l2 and rng.random() < vlan
            l3 = (18 if tag else 14) if l2 else 0
            hl = 20 if rng.random() < 0.85 else int(rng.integers(6, 16)) * 4
            proto = {"tcp": 6, "udp": 17, "udp0": 17, "frag": 6, "icmp": 1, "arp": 0}[k]
            l4h = 20 if proto == 6 else 8 if proto == 17 else 0
            p = int(pay[i])
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
            ho = hdr_slot * i + 104  # m_pktdat (88) + max_linkhdr (16); <= 98 header bytes
            self.arena[ho:ho + h.size] = h
            self.hdr_off[i], self.hdr_len[i] = ho, h.size
            self.l3[i], self.hlen[i] = l3, hl
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
