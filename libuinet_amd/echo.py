"""BASELINE config 1: the checksum calls of a `multitool --echo` TCP flow,
replayed on synthetic segments in the reference's own mbuf shapes.

libuinet's loopback interface claims hardware checksums (sys/net/if_loop.c
:255-258), so a real echo over lo0 never calls in_cksum*; over netmap/pcap
every segment goes through these calls, which is what is replayed here:

TX (tcp_output -> ip_output -> in_delayed_cksum), per segment:
  * a header mbuf with the 40-B IP+TCP header at m_data + max_linkhdr
    (tcp_output.c:844-846) chained to m_copy slices of the 4-KiB page
    clusters of the socket buffer (tcp_output.c:858; about a third of the
    1460-B payloads span two clusters);
  * th_sum = in_pseudo(src, dst, htons(sizeof(tcphdr) + IPPROTO_TCP + len))
    (tcp_output.c:1080-1081), stored uncomplemented;
  * th_sum = in_cksum_skip(m, ip_len, ip_hl << 2) (ip_output.c:961,
    in_delayed_cksum; csum_data = offsetof(tcphdr, th_sum), tcp_output.c:1062);
  * ip_sum = in_cksum(m, hlen) (ip_output.c:665-667).
RX (ether_input -> ip_input -> tcp_input), per segment copied to a 2-KiB
cluster at +14 (uinet_if_netmap.c:1504-1523):
  * in_cksum_hdr(ip) == 0 (ip_input.c:464);
  * in_cksum_pseudo_header(m, ip_len - hlen, hlen, src, dst, IPPROTO_TCP) == 0
    (tcp_input.c:711-713).

`engine` is anything with skip_batch / hdr_batch / pseudo_header_batch over
mbuf heads (the GPU engine adapter below, or the oracle / reference objects
used by the tests and tests/perf/echo_replay.py).
"""
from __future__ import annotations

import numpy as np

from .mbuf import SEED_BASE, MbufChains, aligned_empty, splitmix64_bytes

MSS = 1460
HDR = 40
SEG = HDR + MSS
CLUSTER = 4096          # MJUMPAGESIZE socket-buffer clusters
RX_CLUSTER = 2048       # MCLBYTES receive buffers
MAX_LINKHDR = 16        # tcp_output.c:844, uipc_domain.c:275


def _bswap16(x):
    x = np.asarray(x, np.uint32)
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


def in_pseudo_np(a, b, c) -> np.ndarray:
    """Vectorised in_pseudo (in_cksum.c:181-191): folded, not complemented."""
    s = np.asarray(a, np.uint64) + np.asarray(b, np.uint64) + np.asarray(c, np.uint64)
    for _ in range(4):
        s = (s & np.uint64(0xFFFF)) + (s >> np.uint64(16))
    return s.astype(np.uint16)


class EchoBatch:
    """n TCP segments of SEG bytes in the reference TX and RX shapes."""

    def __init__(self, n: int = 65536, seed: int = 1):
        rng = np.random.default_rng(seed)
        self.n = n
        nclus = (n * MSS + CLUSTER - 1) // CLUSTER + 1
        hdr_bytes = n * 256                      # one 256-B mbuf per header
        self.clus0 = hdr_bytes
        self.arena = aligned_empty(hdr_bytes + nclus * CLUSTER + 64)
        self.arena[:] = 0
        # socket-buffer payload stream in shuffled page clusters
        stream = splitmix64_bytes(nclus * CLUSTER, SEED_BASE + 1)
        perm = rng.permutation(nclus)
        clus = self.arena[self.clus0 : self.clus0 + nclus * CLUSTER].reshape(nclus, CLUSTER)
        clus[perm] = stream.reshape(nclus, CLUSTER)
        self.perm = perm
        # headers
        self.hdr_off = 256 * np.arange(n, dtype=np.int64) + MAX_LINKHDR + 32
        self.src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        self.dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        h = self.arena[self.hdr_off[:, None] + np.arange(HDR)]
        h[:, 0] = 0x45
        h[:, 2:4] = np.frombuffer(np.uint16(SEG).byteswap().tobytes(), np.uint8)
        ipid = (np.arange(n) & 0xFFFF).astype(">u2").view(np.uint8).reshape(n, 2)
        h[:, 4:6] = ipid
        h[:, 6] = 0x40                            # DF
        h[:, 8] = 64                              # ttl
        h[:, 9] = 6                               # IPPROTO_TCP
        h[:, 12:16] = self.src.view(np.uint8).reshape(n, 4)
        h[:, 16:20] = self.dst.view(np.uint8).reshape(n, 4)
        h[:, 20:22] = np.frombuffer(np.uint16(5001).byteswap().tobytes(), np.uint8)
        h[:, 22:24] = np.frombuffer(np.uint16(2222).byteswap().tobytes(), np.uint8)
        seq = (np.uint32(1000) + np.arange(n, dtype=np.uint32) * np.uint32(MSS)).astype(">u4")
        h[:, 24:28] = seq.view(np.uint8).reshape(n, 4)
        h[:, 32] = 0x50                           # th_off 5
        h[:, 33] = 0x18                           # PSH|ACK
        h[:, 34:36] = np.frombuffer(np.uint16(65535).byteswap().tobytes(), np.uint8)
        # tcp_output.c:1080-1081: uncomplemented pseudo seed in th_sum (native order)
        seed = in_pseudo_np(self.src, self.dst, _bswap16(20 + 6 + MSS))
        h[:, 36:38] = seed.view(np.uint8).reshape(n, 2)
        self.arena[self.hdr_off[:, None] + np.arange(HDR)] = h
        # TX chains: header mbuf -> 1 or 2 cluster slices
        s0 = np.arange(n, dtype=np.int64) * MSS
        c0, o0 = s0 // CLUSTER, s0 % CLUSTER
        first = np.minimum(MSS, CLUSTER - o0)
        two = first < MSS
        nseg = 2 + two.astype(np.int64)
        pkt_seg = np.concatenate([[0], np.cumsum(nseg)])
        seg_off = np.zeros(int(pkt_seg[-1]), np.int64)
        seg_len = np.zeros_like(seg_off)
        seg_off[pkt_seg[:-1]] = self.hdr_off
        seg_len[pkt_seg[:-1]] = HDR
        seg_off[pkt_seg[:-1] + 1] = self.clus0 + perm[c0] * CLUSTER + o0
        seg_len[pkt_seg[:-1] + 1] = first
        k = pkt_seg[:-1][two] + 2
        seg_off[k] = self.clus0 + perm[c0[two] + 1] * CLUSTER
        seg_len[k] = MSS - first[two]
        self.tx = MbufChains(self.arena, seg_off, seg_len, pkt_seg)
        self.rx_arena = aligned_empty(n * RX_CLUSTER + 64)
        self.rx_off = RX_CLUSTER * np.arange(n, dtype=np.int64) + 14

    # ---- TX -------------------------------------------------------------------
    def transmit(self, engine) -> tuple[np.ndarray, np.ndarray]:
        """in_delayed_cksum then ip_sum for every segment; the sums are stored
        into the headers like the stack does.  Returns (th_sum, ip_sum)."""
        th = engine.skip_batch(self.tx.heads, SEG, 20)              # ip_output.c:961
        self.arena[self.hdr_off[:, None] + np.array([36, 37])] = th.view(np.uint8).reshape(-1, 2)
        ips = engine.skip_batch(self.tx.heads, 20, 0)               # ip_output.c:667
        self.arena[self.hdr_off[:, None] + np.array([10, 11])] = ips.view(np.uint8).reshape(-1, 2)
        return th, ips

    def reset_tx(self) -> None:
        """Restore the pre-TX header state (seed in th_sum, ip_sum 0)."""
        seed = in_pseudo_np(self.src, self.dst, _bswap16(20 + 6 + MSS))
        self.arena[self.hdr_off[:, None] + np.array([36, 37])] = seed.view(np.uint8).reshape(-1, 2)
        self.arena[self.hdr_off[:, None] + np.array([10, 11])] = 0

    # ---- RX -------------------------------------------------------------------
    def deliver(self) -> MbufChains:
        """Copy every transmitted segment into its RX cluster at +14."""
        for i in range(self.n):
            b = self.tx.packet_bytes(i)
            self.rx_arena[self.rx_off[i] : self.rx_off[i] + SEG] = np.frombuffer(b, np.uint8)
        return MbufChains.contiguous(self.rx_arena, self.rx_off, SEG)

    def deliver_fast(self) -> MbufChains:
        """Vectorised deliver(): gather the TX pieces with numpy."""
        rx = self.rx_arena
        pk = self.tx.pkt_seg
        dst0 = self.rx_off.copy()
        for j in range(3):
            k = pk[:-1] + j
            ok = k < pk[1:]
            kk = k[ok]
            ln = self.tx.seg_len[kk]
            so = self.tx.seg_off[kk]
            d = dst0[ok]
            maxl = int(ln.max()) if ln.size else 0
            idx = np.arange(maxl)
            m = idx[None, :] < ln[:, None]
            rows = np.broadcast_to(np.arange(kk.size)[:, None], m.shape)[m]
            cols = np.broadcast_to(idx[None, :], m.shape)[m]
            rx[d[rows] + cols] = self.arena[so[rows] + cols]
            dst0[ok] += ln
        return MbufChains.contiguous(rx, self.rx_off, SEG)

    def receive(self, engine, rx: MbufChains) -> tuple[np.ndarray, np.ndarray]:
        """in_cksum_hdr and in_cksum_pseudo_header for every received segment
        (both 0 when the transmitted sums are right)."""
        ips = self.rx_arena.ctypes.data + self.rx_off.astype(np.uint64)
        hs = engine.hdr_batch(ips)
        ps = engine.pseudo_header_batch(rx.heads, SEG - 20, 20, self.src, self.dst, 6)
        return hs, ps


class GpuEngine:
    """The engine's host-mbuf batch API in the shape EchoBatch expects."""

    def __init__(self):
        from . import in_cksum_hdr_batch, in_cksum_pseudo_header_batch, in_cksum_skip_batch

        self.skip_batch = in_cksum_skip_batch
        self.hdr_batch = in_cksum_hdr_batch
        self.pseudo_header_batch = in_cksum_pseudo_header_batch
