"""Host-memory mbuf chains in libuinet's ``struct mbuf`` layout.

The checksum reads three fields of ``struct m_hdr``
(/root/reference/sys/sys/mbuf.h:90-98): ``m_next`` at offset 0, ``m_data`` at
16 and ``m_len`` (int) at 24; an mbuf is MSIZE = 256 bytes
(sys/sys/param.h:159).  :class:`MbufChains` lays real records out with that
ABI so the very same chains can be handed to the engine's C ABI, to the
oracle and to the reference object.

A chain set is described the way ``m_fragment`` (sys/kern/uipc_mbuf.c:1693-1761)
leaves a packet: packet ``i`` is the in-order list of mbufs
``[pkt_seg[i], pkt_seg[i+1])``, mbuf ``k`` holding ``seg_len[k]`` bytes at
``arena[seg_off[k]:]``.
"""
from __future__ import annotations

import os

import numpy as np

MSIZE = 256
M_PKTHDR = 0x2  # sys/sys/mbuf.h:182
# struct m_hdr (mbuf.h:90-98, M_HDR_PAD 6 on amd64) then struct pkthdr
# (:116-133), valid in the first mbuf of a packet (M_PKTHDR); the driver
# offload hooks read/write csum_flags and csum_data.
MBUF_DTYPE = np.dtype(
    [
        ("m_next", "<u8"),
        ("m_nextpkt", "<u8"),
        ("m_data", "<u8"),
        ("m_len", "<i4"),
        ("m_flags", "<i4"),
        ("m_type", "<i2"),
        ("m_pad", "V6"),
        ("rcvif", "<u8"),
        ("header", "<u8"),
        ("pkt_len", "<i4"),
        ("flowid", "<u4"),
        ("csum_flags", "<i4"),
        ("csum_data", "<i4"),
        ("tso_segsz", "<u2"),
        ("vtag", "<u2"),
        ("ph_pad", "V4"),
        ("tags", "<u8"),
        ("m_pktdat", "V168"),
    ]
)
assert MBUF_DTYPE.itemsize == MSIZE
assert MBUF_DTYPE.fields["m_data"][1] == 16 and MBUF_DTYPE.fields["m_len"][1] == 24
assert MBUF_DTYPE.fields["csum_flags"][1] == 64 and MBUF_DTYPE.fields["csum_data"][1] == 68
assert MBUF_DTYPE.fields["m_pktdat"][1] == 88


HUGE = 2 << 20


def aligned_empty(nbytes: int, align: int = 4096, pad: int = 64) -> np.ndarray:
    """A zeroed uint8 buffer whose element 0 is ``align``-aligned, with ``pad``
    bytes of readable slack before and after it (the reference reads whole
    aligned words around a span, in_cksum.c:106-115,165-167).

    With UINET_MBUF_HUGEPAGES=1 in the environment, buffers of 2 MiB and more
    come from an anonymous mapping advised MADV_HUGEPAGE (transparent huge
    pages, as a UMA arena mapped with huge pages would be: uinet_vm_kern.c
    maps one region for every zone) -- the device walk's A/B of page size."""
    if os.environ.get("UINET_MBUF_HUGEPAGES") == "1" and nbytes >= HUGE:
        import mmap

        size = (nbytes + 2 * pad + 2 * HUGE + HUGE - 1) // HUGE * HUGE
        m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        m.madvise(mmap.MADV_HUGEPAGE)
        raw = np.frombuffer(m, dtype=np.uint8)
        start = (-(raw.ctypes.data + pad)) % HUGE + pad  # 2 MiB aligned
        return raw[start : start + nbytes]
    raw = np.zeros(nbytes + align + 2 * pad, dtype=np.uint8)
    start = (-(raw.ctypes.data + pad)) % align + pad
    return raw[start : start + nbytes]  # the view keeps `raw` alive


class MbufChains:
    """A set of mbuf chains over a byte arena (see module docstring)."""

    def __init__(self, arena: np.ndarray, seg_off, seg_len, pkt_seg):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        seg_off = np.asarray(seg_off, dtype=np.int64)
        seg_len = np.asarray(seg_len, dtype=np.int64)
        pkt_seg = np.asarray(pkt_seg, dtype=np.int64)
        if seg_off.shape != seg_len.shape or pkt_seg.ndim != 1 or pkt_seg[0] != 0:
            raise ValueError("bad chain description")
        if pkt_seg[-1] != seg_off.size or np.any(np.diff(pkt_seg) < 0):
            raise ValueError("pkt_seg must be a non-decreasing prefix array ending at nseg")
        self.arena = arena
        self.seg_off = seg_off
        self.seg_len = seg_len
        self.pkt_seg = pkt_seg
        nseg = seg_off.size
        # page-aligned records (zeroed), so the mbufs can be registered with
        # the engine (uinet_cksum_register_host) as a region of their own, as
        # libuinet's UMA slabs are (the device walk reads them in place)
        self.mbufs = aligned_empty(max(nseg, 1) * MSIZE).view(MBUF_DTYPE)
        base = self.mbufs.ctypes.data
        addr = base + MSIZE * np.arange(nseg, dtype=np.uint64)
        nxt = addr + np.uint64(MSIZE)
        npk = pkt_seg.size - 1
        nonempty = pkt_seg[1:] > pkt_seg[:-1]
        last = pkt_seg[1:][nonempty] - 1
        if nseg:
            nxt[last] = 0
            self.mbufs["m_next"][:nseg] = nxt
            self.mbufs["m_data"][:nseg] = np.uint64(arena.ctypes.data) + seg_off.astype(np.uint64)
            self.mbufs["m_len"][:nseg] = seg_len.astype(np.int32)
        heads = np.zeros(npk, dtype=np.uint64)
        if nseg:
            heads[nonempty] = addr[pkt_seg[:-1][nonempty]]
            first = pkt_seg[:-1][nonempty]
            self.mbufs["m_flags"][first] = M_PKTHDR
            self.mbufs["pkt_len"][first] = np.add.reduceat(seg_len, first) if first.size else 0
        self.heads = heads

    @property
    def n(self) -> int:
        return self.heads.size

    def head(self, i: int) -> int:
        return int(self.heads[i])

    def first_mbuf(self, i: int) -> int:
        """Index into ``mbufs`` of packet ``i``'s head (its pkthdr)."""
        return int(self.pkt_seg[i])

    def packet_bytes(self, i: int) -> bytes:
        """The concatenated bytes of packet ``i``'s chain (test helper)."""
        parts = [
            self.arena[o : o + l].tobytes()
            for o, l in zip(self.seg_off[self.pkt_seg[i] : self.pkt_seg[i + 1]],
                            self.seg_len[self.pkt_seg[i] : self.pkt_seg[i + 1]])
        ]
        return b"".join(parts)

    @classmethod
    def contiguous(cls, arena: np.ndarray, off, length) -> "MbufChains":
        """One mbuf per packet (the RX shape: data in a single cluster)."""
        off = np.asarray(off, dtype=np.int64)
        length = np.broadcast_to(np.asarray(length, dtype=np.int64), off.shape)
        return cls(arena, off, length, np.arange(off.size + 1, dtype=np.int64))


def splitmix64_bytes(nbytes: int, seed: int, out: np.ndarray | None = None) -> np.ndarray:
    """Deterministic payload bytes: the splitmix64 stream of BASELINE.md
    (seed 0x6C69627569657401 + config index), little-endian, vectorised in
    blocks so multi-GB arenas stay within a few hundred MB of temporaries."""
    if out is None:
        out = np.empty(nbytes, dtype=np.uint8)
    nwords = (nbytes + 7) // 8
    block = 1 << 22
    with np.errstate(over="ignore"):
        for w0 in range(0, nwords, block):
            w1 = min(nwords, w0 + block)
            i = np.arange(w0 + 1, w1 + 1, dtype=np.uint64)
            z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            b = z.view(np.uint8)
            lo, hi = 8 * w0, min(nbytes, 8 * w1)
            out[lo:hi] = b[: hi - lo]
    return out


SEED_BASE = 0x6C69627569657401
