"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes loaders for
  * ``liboracle_cksum.so`` -- the CPU restatement in cksum_oracle.c (always
    built by ``make -C oracle``), and
  * ``_ref/libref_cksum.so`` -- the reference's own
    sys/amd64/amd64/in_cksum.c compiled from /root/reference (built here when
    the reference tree is present; the built .so travels to the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (libuinet_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle_cksum.so")
REF_SO = os.path.join(HERE, "_ref", "libref_cksum.so")

F_UDP = 0x1
F_NO_COMPLEMENT = 0x2

_vp, _i32, _u32, _u64, _u16, _u8 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32,
                                    ctypes.c_uint64, ctypes.c_uint16, ctypes.c_uint8)


def _p(a: Optional[np.ndarray]) -> int:
    return 0 if a is None else a.ctypes.data


def _c(a, dtype, n=None):
    if a is None:
        return None
    a = np.asarray(a)
    if n is not None:
        a = np.broadcast_to(a, (n,))
    return np.ascontiguousarray(a, dtype=dtype)


class Oracle:
    """The CPU restatement (cksum_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        sig = {
            "oracle_cksum_skip": (_u16, [_vp, _i32, _i32]),
            "oracle_cksum_pseudo_header": (_u16, [_vp, _i32, _i32, _u32, _u32, _u8]),
            "oracle_cksum_hdr": (ctypes.c_uint, [_vp]),
            "oracle_in_pseudo": (_u16, [_u32, _u32, _u32]),
            "oracle_in_addword": (_u16, [_u16, _u16]),
            "oracle_spans": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32]),
            "oracle_chains": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32]),
            "oracle_cksum_skip_batch": (None, [_vp, _vp, _vp, _vp, _i32, _i32]),
            "oracle_cksum_pseudo_header_batch": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32]),
            "oracle_cksum_hdr_batch": (None, [_vp, _vp, _i32]),
            "oracle_rx_offload": (None, [_vp, _i32, _i32, _vp]),
            "oracle_in6_cksum_pseudo": (_i32, [_vp, _u32, _u8, _u16]),
            "oracle_in6_cksum_batch": (None, [_vp, _vp, _vp, _vp, _vp, _i32]),
            "oracle_tx_offload": (None, [_vp, _i32, _i32, _vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.L = L

    # per-call
    def cksum_skip(self, m: int, length: int, skip: int) -> int:
        return self.L.oracle_cksum_skip(m, length, skip)

    def cksum_pseudo_header(self, m, plen, off0, src, dst, proto) -> int:
        return self.L.oracle_cksum_pseudo_header(m, plen, off0, src, dst, proto)

    def cksum_hdr(self, ip: int) -> int:
        return self.L.oracle_cksum_hdr(ip)

    def in_pseudo(self, a, b, c) -> int:
        return self.L.oracle_in_pseudo(a, b, c)

    def in_addword(self, a, b) -> int:
        return self.L.oracle_in_addword(a, b)

    # batches
    def skip_batch(self, heads, length, skip, nthreads: int = 8) -> np.ndarray:
        heads = _c(heads, np.uint64)
        n = heads.size
        length, skip = _c(length, np.int32, n), _c(skip, np.int32, n)
        out = np.zeros(n, np.uint16)
        self.L.oracle_cksum_skip_batch(_p(heads), _p(length), _p(skip), _p(out), n, nthreads)
        return out

    def pseudo_header_batch(self, heads, plen, off0, src, dst, proto) -> np.ndarray:
        heads = _c(heads, np.uint64)
        n = heads.size
        arrs = [_c(plen, np.int32, n), _c(off0, np.int32, n), _c(src, np.uint32, n),
                _c(dst, np.uint32, n), _c(proto, np.uint8, n)]
        out = np.zeros(n, np.uint16)
        self.L.oracle_cksum_pseudo_header_batch(_p(heads), *[_p(a) for a in arrs], _p(out), n)
        return out

    def hdr_batch(self, ips) -> np.ndarray:
        ips = _c(ips, np.uint64)
        out = np.zeros(ips.size, np.uint32)
        self.L.oracle_cksum_hdr_batch(_p(ips), _p(out), ips.size)
        return out

    def in6_cksum_batch(self, heads, nxt, off, length) -> np.ndarray:
        """in6_cksum(m, nxt, off, len) per packet (sys/netinet6/in6_cksum.c)."""
        heads = _c(heads, np.uint64)
        n = heads.size
        arrs = [_c(nxt, np.uint8, n), _c(off, np.uint32, n), _c(length, np.uint32, n)]
        out = np.zeros(n, np.uint16)
        self.L.oracle_in6_cksum_batch(_p(heads), *[_p(a) for a in arrs], _p(out), n)
        return out

    def in6_cksum_pseudo(self, ip6: int, length: int, nxt: int, csum: int) -> int:
        return self.L.oracle_in6_cksum_pseudo(ip6, length, nxt, csum)

    def rx_offload(self, heads, l2len: int = -1) -> np.ndarray:
        """offload_oracle.c: the RX hook restated packet by packet (marks pkthdrs)."""
        heads = _c(heads, np.uint64)
        st = np.zeros(heads.size, np.uint8)
        self.L.oracle_rx_offload(_p(heads), heads.size, l2len, _p(st))
        return st

    def tx_offload(self, heads, l2len: int = -1) -> np.ndarray:
        """offload_oracle.c: the TX hook restated (writes sums into the packets)."""
        heads = _c(heads, np.uint64)
        st = np.zeros(heads.size, np.uint8)
        self.L.oracle_tx_offload(_p(heads), heads.size, l2len, _p(st))
        return st

    def spans(self, base: np.ndarray, off, length, seed=None, parity=None, flags=0) -> np.ndarray:
        off = _c(off, np.uint64)
        n = off.size
        length = _c(length, np.uint32, n)
        seed = _c(seed, np.uint32, n)
        parity = _c(parity, np.uint8, n)
        out = np.zeros(n, np.uint16)
        self.L.oracle_spans(_p(base), _p(off), _p(length), _p(seed), _p(parity), _p(out), n, flags)
        return out

    def chains(self, base: np.ndarray, seg_off, seg_len, pkt_seg, length=None, skip=None,
               seed=None, flags=0) -> np.ndarray:
        """in_cksum_skip(chain_i, length[i], skip[i]) over segment-list chains."""
        seg_off = _c(seg_off, np.uint64)
        seg_len = _c(seg_len, np.uint32)
        pkt_seg = _c(pkt_seg, np.uint64)
        n = pkt_seg.size - 1
        length = _c(length, np.int64, n)
        skip = _c(skip, np.int64, n)
        seed = _c(seed, np.uint32, n)
        out = np.zeros(n, np.uint16)
        self.L.oracle_chains(_p(base), _p(seg_off), _p(seg_len), _p(pkt_seg), _p(length),
                             _p(skip), _p(seed), _p(out), n, flags)
        return out


class Reference:
    """The reference object itself (oracle/_ref/libref_cksum.so)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        L = ctypes.CDLL(path)
        sig = {
            "refh_in_cksum_skip": (ctypes.c_ushort, [_vp, _i32, _i32]),
            "refh_in_cksum_pseudo_header": (_u16, [_vp, _i32, _i32, _u32, _u32, _u8]),
            "refh_in_cksum_hdr": (ctypes.c_uint, [_vp]),
            "refh_in_pseudo": (ctypes.c_ushort, [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]),
            "refh_in_addword": (ctypes.c_ushort, [ctypes.c_ushort, ctypes.c_ushort]),
            "refh_skip_batch": (None, [_vp, _vp, _vp, _vp, _i32]),
            "refh_pseudo_batch": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32]),
            "refh_hdr_batch": (None, [_vp, _vp, _i32]),
            "refh_time_batch": (ctypes.c_double, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32,
                                                  _i32, _vp, _i32, _vp]),
            "refh_time_read": (ctypes.c_double, [_vp, ctypes.c_long, _i32, _vp, _i32, _vp, _vp]),
            "refh_in6_cksum": (_i32, [_vp, _u8, _u32, _u32]),
            "refh_in6_cksum_pseudo": (_i32, [_vp, _u32, _u8, _u16]),
            "refh_in6_batch": (None, [_vp, _vp, _vp, _vp, _vp, _i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.L = L

    def cksum_skip(self, m, length, skip) -> int:
        return self.L.refh_in_cksum_skip(m, length, skip)

    def cksum_pseudo_header(self, m, plen, off0, src, dst, proto) -> int:
        return self.L.refh_in_cksum_pseudo_header(m, plen, off0, src, dst, proto)

    def cksum_hdr(self, ip) -> int:
        return self.L.refh_in_cksum_hdr(ip)

    def in_pseudo(self, a, b, c) -> int:
        return self.L.refh_in_pseudo(a, b, c)

    def in_addword(self, a, b) -> int:
        return self.L.refh_in_addword(a, b)

    def skip_batch(self, heads, length, skip) -> np.ndarray:
        heads = _c(heads, np.uint64)
        n = heads.size
        length, skip = _c(length, np.int32, n), _c(skip, np.int32, n)
        out = np.zeros(n, np.uint16)
        self.L.refh_skip_batch(_p(heads), _p(length), _p(skip), _p(out), n)
        return out

    def pseudo_header_batch(self, heads, plen, off0, src, dst, proto) -> np.ndarray:
        heads = _c(heads, np.uint64)
        n = heads.size
        arrs = [_c(plen, np.int32, n), _c(off0, np.int32, n), _c(src, np.uint32, n),
                _c(dst, np.uint32, n), _c(proto, np.uint8, n)]
        out = np.zeros(n, np.uint16)
        self.L.refh_pseudo_batch(_p(heads), *[_p(a) for a in arrs], _p(out), n)
        return out

    def hdr_batch(self, ips) -> np.ndarray:
        ips = _c(ips, np.uint64)
        out = np.zeros(ips.size, np.uint32)
        self.L.refh_hdr_batch(_p(ips), _p(out), ips.size)
        return out

    def in6_cksum_pseudo(self, ip6: int, length: int, nxt: int, csum: int) -> int:
        """sys/netinet6/in6_cksum.c:129-140, the reference's own."""
        return self.L.refh_in6_cksum_pseudo(ip6, length, nxt, csum)

    def in6_cksum_batch(self, heads, nxt, off, length) -> np.ndarray:
        """in6_cksum(m, nxt, off, len) per packet, the reference's own
        (in6_cksum.c:150-357; the chain must hold off + len bytes)."""
        heads = _c(heads, np.uint64)
        n = heads.size
        arrs = [_c(nxt, np.uint8, n), _c(off, np.uint32, n), _c(length, np.uint32, n)]
        out = np.zeros(n, np.uint16)
        self.L.refh_in6_batch(_p(heads), *[_p(a) for a in arrs], _p(out), n)
        return out

    @staticmethod
    def _stamps(nthreads, with_stamps):
        return np.zeros(2 * max(1, nthreads), np.float64) if with_stamps else None

    def time_skip(self, heads, length, skip, nthreads=1, cpus=None, reps=5, stamps=False):
        """Best-of-``reps`` pass, seconds, of in_cksum_skip over the batch:
        every worker stamps its own start and end, a pass is max(end) -
        min(start).  Returns (t, out) or, with ``stamps``, (t, out, the last
        pass's per-worker [start, end] pairs)."""
        heads = _c(heads, np.uint64)
        n = heads.size
        length, skip = _c(length, np.int32, n), _c(skip, np.int32, n)
        out = np.zeros(n, np.uint16)
        cpus_a = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.int32)
        st = self._stamps(nthreads, stamps)
        t = self.L.refh_time_batch(0, _p(heads), _p(length), _p(skip), 0, 0, 0, _p(out), n,
                                   nthreads, _p(cpus_a), reps, _p(st))
        return (t, out, st.reshape(-1, 2)[:nthreads]) if stamps else (t, out)

    def time_pseudo(self, heads, plen, off0, src, dst, proto, nthreads=1, cpus=None, reps=5,
                    stamps=False):
        heads = _c(heads, np.uint64)
        n = heads.size
        arrs = [_c(plen, np.int32, n), _c(off0, np.int32, n), _c(src, np.uint32, n),
                _c(dst, np.uint32, n), _c(proto, np.uint8, n)]
        out = np.zeros(n, np.uint16)
        cpus_a = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.int32)
        st = self._stamps(nthreads, stamps)
        t = self.L.refh_time_batch(1, _p(heads), *[_p(a) for a in arrs], _p(out), n, nthreads,
                                   _p(cpus_a), reps, _p(st))
        return (t, out, st.reshape(-1, 2)[:nthreads]) if stamps else (t, out)

    def time_read(self, buf: np.ndarray, nthreads=1, cpus=None, reps=1, stamps=False):
        """The host's read bandwidth over ``buf``: best-of-``reps`` pass,
        seconds, of a plain streaming 64-bit sum on ``nthreads`` threads,
        timed like time_skip (ref_harness.c refh_time_read)."""
        buf = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
        cpus_a = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.int32)
        st = self._stamps(nthreads, stamps)
        sink = np.zeros(1, np.uint64)
        t = self.L.refh_time_read(_p(buf), buf.size, nthreads, _p(cpus_a), reps, _p(st), _p(sink))
        return (t, st.reshape(-1, 2)[:nthreads]) if stamps else t


def have_reference() -> bool:
    return os.path.exists(REF_SO)
