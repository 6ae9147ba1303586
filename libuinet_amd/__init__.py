"""libuinet_amd -- MI355X-native engine for libuinet's Internet checksum.

Python mirror of the engine's C ABI (``include/uinet_cksum.h``), which keeps
the reference KPI of /root/reference/sys/amd64/include/in_cksum.h:44,76-83:

* per-call, same names and argument meaning as the reference:
  :func:`in_cksum_skip`, :func:`in_cksum` (macro), :func:`in_cksum_pseudo_header`,
  :func:`in_cksum_hdr`, :func:`in_pseudo`, :func:`in_addword`;
* host-mbuf batches: :func:`in_cksum_skip_batch`, :func:`in_cksum_pseudo_header_batch`,
  :func:`in_cksum_hdr_batch`;
* the device-resident hot path over HBM buffers held in torch tensors:
  :func:`cksum_spans`, :func:`cksum_strided`, :func:`cksum_chains`, and
  :func:`cksum_mbufs` over struct mbuf chains that live in HBM.

Everything that touches packet bytes runs in the HIP library
``libuinet_amd/libuinet_cksum.so``; if it is missing or no gfx950 device is
usable the calls raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from .mbuf import MBUF_DTYPE, MSIZE, MbufChains, SEED_BASE, aligned_empty, splitmix64_bytes

__all__ = [
    "LIB_PATH", "CksumError", "lib", "in_cksum", "in_cksum_skip", "in_cksum_pseudo_header",
    "in_cksum_hdr", "in_pseudo", "in_addword", "in_cksum_skip_batch",
    "in_cksum_pseudo_header_batch", "in_cksum_hdr_batch", "cksum_spans", "cksum_strided",
    "cksum_chains", "pack_segments", "F_UDP", "F_NO_COMPLEMENT", "MbufChains", "MBUF_DTYPE", "MSIZE",
    "SEED_BASE", "aligned_empty", "splitmix64_bytes", "EXPORTED_SYMBOLS", "cksum_spans_multi",
    "in_cksum_skip_batch_multi", "host_cpu", "cksum_mbufs", "MBUF_TRUNC", "MBUF_BADLEN",
    "MBUF_BADARG", "MBUF_HOPS_MAX",
]

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libuinet_cksum.so")

F_UDP = 0x1
F_NO_COMPLEMENT = 0x2

OK, EINVAL, ENODEV, ENOMEM, EHIP = 0, -22, -19, -12, -5

# Every function include/uinet_cksum.h declares (tests check the .so exports
# exactly these).
EXPORTED_SYMBOLS = (
    "in_cksum_skip", "in_cksum_pseudo_header", "in_cksum_hdr", "in_pseudo", "in_addword",
    "uinet_cksum_version", "uinet_cksum_strerror", "uinet_cksum_last_hip_error",
    "uinet_cksum_last_kernel", "uinet_cksum_device_ok", "uinet_cksum_set_tuning", "uinet_cksum_spans", "uinet_cksum_spans32",
    "uinet_cksum_strided", "uinet_cksum_chains", "uinet_cksum_chains32",
    "in_cksum_skip_batch", "in_cksum_pseudo_header_batch", "in_cksum_hdr_batch",
    "uinet_cksum_register_host", "uinet_cksum_unregister_host",
    "uinet_cksum_rx_offload", "uinet_cksum_tx_offload",
    "in6_cksum", "in6_cksum_pseudo", "in6_cksum_batch",
    "uinet_cksum_spans_multi", "uinet_cksum_multi_last_gather", "in_cksum_skip_batch_multi",
    "uinet_cksum_host_cpu", "uinet_cksum_mbufs",
)

# uinet_cksum_mbufs status bits and hop bound (include/uinet_cksum.h section 2b).
MBUF_TRUNC, MBUF_BADLEN, MBUF_BADARG = 0x1, 0x2, 0x4
MBUF_HOPS_MAX = 0x20000

# Driver offload status bits (include/uinet_cksum.h section 2d).
RX_IPV4, RX_IP_OK, RX_L4, RX_L4_OK, RX_NOSUM, RX_FRAG = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
TX_L4, TX_IP, TX_L4_LOST, TX_SKIP = 0x01, 0x02, 0x04, 0x08


class CksumError(RuntimeError):
    """A negative UINET_CKSUM_E* status from the engine."""

    def __init__(self, fn: str, code: int):
        self.code = code
        msg = lib().uinet_cksum_strerror(code).decode()
        hip = lib().uinet_cksum_last_hip_error()
        super().__init__(f"{fn}: {msg} (code {code}, hip error {hip})")


_LIB: Optional[ctypes.CDLL] = None

_vp, _u64, _u32, _i32, _u16, _u8 = (ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_int, ctypes.c_uint16, ctypes.c_uint8)


def lib() -> ctypes.CDLL:
    """Load the engine library (torch first, so both share one HIP runtime:
    torch's bundled libamdhip64 and ROCm's carry the same SONAME)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is part of the image
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is not built; run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "in_cksum_skip": (ctypes.c_ushort, [_vp, _i32, _i32]),
        "in_cksum_pseudo_header": (_u16, [_vp, _i32, _i32, _u32, _u32, _u8]),
        "in_cksum_hdr": (ctypes.c_uint, [_vp]),
        "in_pseudo": (ctypes.c_ushort, [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]),
        "in_addword": (ctypes.c_ushort, [ctypes.c_ushort, ctypes.c_ushort]),
        "uinet_cksum_version": (ctypes.c_char_p, []),
        "uinet_cksum_last_kernel": (ctypes.c_char_p, []),
        "uinet_cksum_strerror": (ctypes.c_char_p, [_i32]),
        "uinet_cksum_last_hip_error": (_i32, []),
        "uinet_cksum_device_ok": (_i32, []),
        "uinet_cksum_set_tuning": (_i32, [ctypes.c_char_p, _i32]),
        "uinet_cksum_spans": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]),
        "uinet_cksum_spans32": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]),
        "uinet_cksum_strided": (_i32, [_vp, _u64, _u32, _vp, _vp, _u32, _u32, _vp]),
        "uinet_cksum_chains": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32,
                                       _vp]),
        "uinet_cksum_chains32": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32,
                                         _u32, _vp]),
        "in_cksum_skip_batch": (_i32, [_vp, _vp, _vp, _vp, _i32]),
        "in_cksum_pseudo_header_batch": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32]),
        "in_cksum_hdr_batch": (_i32, [_vp, _vp, _i32]),
        "uinet_cksum_register_host": (_i32, [_vp, ctypes.c_size_t]),
        "uinet_cksum_unregister_host": (_i32, [_vp]),
        "uinet_cksum_rx_offload": (_i32, [_vp, _i32, _i32, _vp]),
        "uinet_cksum_tx_offload": (_i32, [_vp, _i32, _i32, _vp]),
        "in6_cksum": (_i32, [_vp, _u8, _u32, _u32]),
        "in6_cksum_pseudo": (_i32, [_vp, _u32, _u8, _u16]),
        "in6_cksum_batch": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32]),
        "uinet_cksum_spans_multi": (_i32, [_vp, _i32, _u32, _u32, _i32, _vp]),
        "uinet_cksum_multi_last_gather": (_i32, []),
        "in_cksum_skip_batch_multi": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _i32]),
        "uinet_cksum_host_cpu": (_i32, [_vp, _i32]),
        "uinet_cksum_mbufs": (_i32, [_vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def _check(fn: str, rc: int) -> None:
    if rc != OK:
        raise CksumError(fn, rc)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---- per-call ABI (sys/amd64/include/in_cksum.h) ----------------------------

def in_cksum_skip(m: int, len: int, skip: int) -> int:  # noqa: A002 - reference name
    """in_cksum.c:193-232.  ``m`` is the address of a ``struct mbuf``."""
    return lib().in_cksum_skip(m, len, skip)


def in_cksum(m: int, len: int) -> int:  # noqa: A002
    """in_cksum.h:44 -- ``in_cksum_skip(m, len, 0)``."""
    return lib().in_cksum_skip(m, len, 0)


def in_cksum_pseudo_header(m: int, plen: int, off0: int, src: int, dst: int, protonum: int) -> int:
    """in_cksum.c:241-276; ``src``/``dst`` as stored in the header (network
    order read as a native u32)."""
    return lib().in_cksum_pseudo_header(m, plen, off0, src, dst, protonum)


def in_cksum_hdr(ip: int) -> int:
    """in_cksum.c:278-285.  ``ip`` is the address of the 20-byte header."""
    return lib().in_cksum_hdr(ip)


def in_pseudo(a: int, b: int, c: int) -> int:
    """in_cksum.c:181-191 (folded, not complemented)."""
    return lib().in_pseudo(a, b, c)


def in_addword(a: int, b: int) -> int:
    """in_cksum.c:172-179."""
    return lib().in_addword(a, b)


# ---- host-mbuf batches --------------------------------------------------------

def in_cksum_skip_batch(heads, length, skip) -> np.ndarray:
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    n = heads.size
    length = np.ascontiguousarray(np.broadcast_to(length, (n,)), dtype=np.int32)
    skip = np.ascontiguousarray(np.broadcast_to(skip, (n,)), dtype=np.int32)
    out = np.zeros(n, dtype=np.uint16)
    _check("in_cksum_skip_batch",
           lib().in_cksum_skip_batch(_ptr(heads), _ptr(length), _ptr(skip), _ptr(out), n))
    return out


def in_cksum_pseudo_header_batch(heads, plen, off0, src, dst, proto) -> np.ndarray:
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    n = heads.size
    arrs = [np.ascontiguousarray(np.broadcast_to(a, (n,)), dtype=t)
            for a, t in ((plen, np.int32), (off0, np.int32), (src, np.uint32),
                         (dst, np.uint32), (proto, np.uint8))]
    out = np.zeros(n, dtype=np.uint16)
    _check("in_cksum_pseudo_header_batch",
           lib().in_cksum_pseudo_header_batch(_ptr(heads), *[_ptr(a) for a in arrs], _ptr(out), n))
    return out


def register_host(buf: np.ndarray) -> None:
    """uinet_cksum_register_host over a host buffer: batches whose bytes lie in
    it are folded in place over PCIe (zero-copy)."""
    _check("uinet_cksum_register_host",
           lib().uinet_cksum_register_host(buf.ctypes.data, buf.nbytes))


def unregister_host(buf: np.ndarray) -> None:
    _check("uinet_cksum_unregister_host", lib().uinet_cksum_unregister_host(buf.ctypes.data))


def in6_cksum(m: int, nxt: int, off: int, length: int) -> int:
    """sys/netinet6/in6_cksum.c:150-357 (per call, a GPU batch of one)."""
    return lib().in6_cksum(m, nxt, off, length)


def in6_cksum_pseudo(ip6: int, length: int, nxt: int, csum: int) -> int:
    """in6_cksum.c:129-140: folded pseudo-header sum + csum (host fold)."""
    return lib().in6_cksum_pseudo(ip6, length, nxt, csum)


def in6_cksum_batch(heads, nxt, off, length) -> np.ndarray:
    """in6_cksum(m[i], nxt[i], off[i], len[i]) for a batch, one GPU launch."""
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    n = heads.size
    nxt = np.ascontiguousarray(np.broadcast_to(nxt, (n,)), dtype=np.uint8)
    off = np.ascontiguousarray(np.broadcast_to(off, (n,)), dtype=np.uint32)
    length = np.ascontiguousarray(np.broadcast_to(length, (n,)), dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint16)
    _check("in6_cksum_batch", lib().in6_cksum_batch(_ptr(heads), _ptr(nxt), _ptr(off),
                                                   _ptr(length), _ptr(out), n))
    return out


def rx_offload(heads, l2len: int = -1) -> np.ndarray:
    """uinet_cksum_rx_offload: verify a received batch and mark m_pkthdr
    (csum_flags / csum_data) like a checksum-offloading NIC; RX_* bits."""
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    st = np.zeros(heads.size, dtype=np.uint8)
    _check("uinet_cksum_rx_offload",
           lib().uinet_cksum_rx_offload(_ptr(heads), heads.size, l2len, _ptr(st)))
    return st


def tx_offload(heads, l2len: int = -1) -> np.ndarray:
    """uinet_cksum_tx_offload: fill the deferred ip_sum / th_sum / uh_sum of a
    transmit batch in place (in_delayed_cksum semantics); TX_* bits."""
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    st = np.zeros(heads.size, dtype=np.uint8)
    _check("uinet_cksum_tx_offload",
           lib().uinet_cksum_tx_offload(_ptr(heads), heads.size, l2len, _ptr(st)))
    return st


def in_cksum_hdr_batch(ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint64)
    out = np.zeros(ips.size, dtype=np.uint32)
    _check("in_cksum_hdr_batch", lib().in_cksum_hdr_batch(_ptr(ips), _ptr(out), ips.size))
    return out


# ---- device-resident hot path (torch tensors in HBM) -------------------------

def _dev(t, dtype, name):
    import torch

    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a device tensor")
    if t.dtype != dtype or not t.is_contiguous():
        raise TypeError(f"{name} must be a contiguous {dtype} tensor")
    return t


def _dp(t) -> int:
    return 0 if t is None else t.data_ptr()


def _stream(stream) -> int:
    import torch

    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def _out(n, out, like):
    import torch

    if out is None:
        return torch.empty(n, dtype=torch.uint16, device=like.device)
    return _dev(out, torch.uint16, "out")


def cksum_spans(base, off, length, seed=None, parity=None, out=None, flags: int = 0,
                len_hint: int = 0, stream=None):
    """out[i] = checksum of ``base[off[i] : off[i] + length[i]]`` (device u8 tensor
    ``base``; optional uint32-valued int32 ``seed``; optional uint8 ``parity``).
    Wide descriptors (int64 ``off``, int32 ``length``) call uinet_cksum_spans;
    packed ones (uint32-valued int32 ``off``, uint16 or uint16-valued int16
    ``length``: arenas < 4 GiB, spans <= 65535 B; see :func:`pack_segments`)
    call uinet_cksum_spans32."""
    import torch

    _dev(base, torch.uint8, "base")
    packed = off is not None and off.dtype == torch.int32
    if packed:
        _dev(off, torch.int32, "off")
        if length is not None and length.dtype == torch.uint16:
            length = length.view(torch.int16)
        _dev(length, torch.int16, "length")
    else:
        _dev(off, torch.int64, "off")
        _dev(length, torch.int32, "length")
    _dev(seed, torch.int32, "seed")
    _dev(parity, torch.uint8, "parity")
    n = off.numel()
    if length.numel() != n:
        raise ValueError("off/length size mismatch")
    out = _out(n, out, base)
    fn = "uinet_cksum_spans32" if packed else "uinet_cksum_spans"
    _check(fn, getattr(lib(), fn)(
        _dp(base), _dp(off), _dp(length), _dp(seed), _dp(parity), _dp(out), n, flags,
        len_hint, _stream(stream)))
    return out


def cksum_strided(base, stride: int, length: int, n: int, seed=None, out=None,
                  flags: int = 0, stream=None):
    """out[i] = checksum of ``base[i*stride : i*stride + length]``."""
    import torch

    _dev(base, torch.uint8, "base")
    _dev(seed, torch.int32, "seed")
    if n and (n - 1) * stride + length > base.numel():
        raise ValueError("strided batch exceeds base")
    out = _out(n, out, base)
    _check("uinet_cksum_strided", lib().uinet_cksum_strided(
        _dp(base), stride, length, _dp(seed), _dp(out), n, flags, _stream(stream)))
    return out


def cksum_chains(base, seg_off, seg_len, pkt_seg, length=None, skip=None, seed=None, out=None,
                 flags: int = 0, len_hint: int = 0, stream=None):
    """``in_cksum_skip(chain_i, length[i], skip[i])`` for device-resident chains:
    packet i = segments [pkt_seg[i], pkt_seg[i+1]) of ``base`` (int32 pkt_seg of
    n+1 entries; optional int32 length/skip/seed).  Wide descriptors (int64
    seg_off, int32 seg_len) call uinet_cksum_chains; packed ones (uint32-valued
    int32 seg_off, uint16 or uint16-valued int16 seg_len: arenas < 4 GiB,
    mbufs <= 65535 B; see :func:`pack_segments`) call uinet_cksum_chains32."""
    import torch

    _dev(base, torch.uint8, "base")
    packed = seg_off is not None and seg_off.dtype == torch.int32
    if packed:
        _dev(seg_off, torch.int32, "seg_off")
        if seg_len is not None and seg_len.dtype == torch.uint16:
            seg_len = seg_len.view(torch.int16)
        _dev(seg_len, torch.int16, "seg_len")
    else:
        _dev(seg_off, torch.int64, "seg_off")
        _dev(seg_len, torch.int32, "seg_len")
    if seg_off.numel() != seg_len.numel():
        raise ValueError("seg_off/seg_len size mismatch")
    _dev(pkt_seg, torch.int32, "pkt_seg")
    for t, nm in ((length, "length"), (skip, "skip"), (seed, "seed")):
        _dev(t, torch.int32, nm)
    n = pkt_seg.numel() - 1
    out = _out(n, out, base)
    fn = "uinet_cksum_chains32" if packed else "uinet_cksum_chains"
    _check(fn, getattr(lib(), fn)(
        _dp(base), _dp(seg_off), _dp(seg_len), _dp(pkt_seg), _dp(length), _dp(skip), _dp(seed),
        _dp(out), n, flags, len_hint, _stream(stream)))
    return out


def cksum_mbufs(heads, length=None, skip=None, seed=None, out=None, flags: int = 0,
                seg_hint: int = 0, status=None, stream=None):
    """``in_cksum_skip(heads[i], length[i], skip[i])`` (+ ``seed[i]``) over
    struct mbuf chains that live in HBM: ``heads`` is an int64 device tensor
    of first-mbuf device addresses whose m_next / m_data are device addresses
    too (see :func:`libuinet_amd.workloads.device_mbufs`); optional int32
    ``length`` / ``skip`` / ``seed`` (None: whole chain / 0 / 0).  ``status``
    (an int32 device tensor of one element, optional) receives the OR of
    MBUF_* bits.  One launch of uinet_cksum_mbufs walks and folds."""
    import torch

    _dev(heads, torch.int64, "heads")
    for t, nm in ((length, "length"), (skip, "skip"), (seed, "seed"), (status, "status")):
        _dev(t, torch.int32, nm)
    n = heads.numel()
    for t, nm in ((length, "length"), (skip, "skip"), (seed, "seed")):
        if t is not None and t.numel() != n:
            raise ValueError(f"{nm} must hold one entry per packet")
    if status is not None and status.numel() < 1:
        raise ValueError("status needs one element")
    out = _out(n, out, heads)
    _check("uinet_cksum_mbufs", lib().uinet_cksum_mbufs(
        _dp(heads), _dp(length), _dp(skip), _dp(seed), _dp(out), n, flags, seg_hint,
        _dp(status), _stream(stream)))
    return out


def pack_segments(seg_off, seg_len):
    """Wide chain or span descriptors (int64 offsets, int32 lengths; numpy or
    torch) to the packed form of uinet_cksum_chains32 / uinet_cksum_spans32:
    int32 holding the uint32 offset,
    int16 holding the uint16 length.  Raises ValueError when an offset is not
    below 4 GiB or a length exceeds 65535, instead of truncating."""
    if hasattr(seg_off, "cpu"):
        import torch

        if seg_off.numel() and (int(seg_off.min()) < 0 or int(seg_off.max()) >= 1 << 32
                                or int(seg_len.min()) < 0 or int(seg_len.max()) > 0xffff):
            raise ValueError("segments do not fit the packed descriptor form")
        off32 = (seg_off - ((seg_off >> 31) << 32)).to(torch.int32)
        len16 = (seg_len - ((seg_len >> 15) << 16)).to(torch.int16)
        return off32, len16
    seg_off = np.asarray(seg_off, dtype=np.int64)
    seg_len = np.asarray(seg_len, dtype=np.int64)
    if seg_off.size and (seg_off.min() < 0 or seg_off.max() >= 1 << 32
                         or seg_len.min() < 0 or seg_len.max() > 0xffff):
        raise ValueError("segments do not fit the packed descriptor form")
    return seg_off.astype(np.uint32).view(np.int32), seg_len.astype(np.uint16).view(np.int16)


class Shard(ctypes.Structure):
    """struct uinet_cksum_shard (include/uinet_cksum.h section 2e)."""

    _fields_ = [("device", ctypes.c_int), ("n", ctypes.c_uint32), ("base", _vp), ("off", _vp),
                ("len", _vp), ("seed", _vp), ("parity", _vp)]


def cksum_spans_multi(shards, root_device: int = 0, out=None, flags: int = 0,
                      len_hint: int = 0):
    """uinet_cksum_spans_multi: ``shards`` is a list of dicts with device tensors
    ``base`` (uint8), ``off`` (int64), ``length`` (int32) and optional ``seed``
    (int32) / ``parity`` (uint8), each on its own device; returns the gathered
    uint16 results on ``root_device`` (shard order)."""
    import torch

    arr = (Shard * len(shards))()
    total = 0
    for k, sh in enumerate(shards):
        base, off, ln = sh["base"], sh["off"], sh["length"]
        _dev(base, torch.uint8, "base")
        _dev(off, torch.int64, "off")
        _dev(ln, torch.int32, "length")
        _dev(sh.get("seed"), torch.int32, "seed")
        _dev(sh.get("parity"), torch.uint8, "parity")
        if off.numel() != ln.numel():
            raise ValueError("off/length size mismatch")
        arr[k] = Shard(base.device.index, off.numel(), _dp(base), _dp(off), _dp(ln),
                       _dp(sh.get("seed")), _dp(sh.get("parity")))
        total += off.numel()
    if out is None:
        out = torch.empty(total, dtype=torch.uint16, device=f"cuda:{root_device}")
    _dev(out, torch.uint16, "out")
    if out.numel() < total or out.device.index != root_device:
        raise ValueError("out must hold every result on root_device")
    for sh in shards:  # the shards' inputs were written on the callers' streams
        torch.cuda.synchronize(sh["base"].device)
    _check("uinet_cksum_spans_multi", lib().uinet_cksum_spans_multi(
        ctypes.addressof(arr), len(shards), flags, len_hint, root_device, _dp(out)))
    return out


def multi_last_gather() -> int:
    """How this thread's last cksum_spans_multi gathered: 1 one RCCL gather,
    0 peer copies, -1 no call yet."""
    return lib().uinet_cksum_multi_last_gather()


def in_cksum_skip_batch_multi(devices, heads, length, skip) -> np.ndarray:
    """in_cksum_skip_batch spread over ``devices`` (byte-balanced contiguous ranges)."""
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    heads = np.ascontiguousarray(heads, dtype=np.uint64)
    n = heads.size
    length = np.ascontiguousarray(np.broadcast_to(length, (n,)), dtype=np.int32)
    skip = np.ascontiguousarray(np.broadcast_to(skip, (n,)), dtype=np.int32)
    out = np.zeros(n, dtype=np.uint16)
    _check("in_cksum_skip_batch_multi", lib().in_cksum_skip_batch_multi(
        _ptr(devs), devs.size, _ptr(heads), _ptr(length), _ptr(skip), _ptr(out), n))
    return out


class HostCpu(ctypes.Structure):
    """struct uinet_cksum_host_cpu (include/uinet_cksum.h section 2f)."""

    _fields_ = [("calls", _u64), ("packets", _u64), ("wall_ns", _u64), ("caller_cpu_ns", _u64),
                ("helper_cpu_ns", _u64), ("device_walks", _u64), ("span_batches", _u64),
                ("span_dma_bytes", _u64)]


def host_cpu(reset: bool = False) -> dict:
    """uinet_cksum_host_cpu: this thread's host-batch counters (wall time,
    calling-thread CPU time and host-pool helper CPU time, in ns)."""
    st = HostCpu()
    _check("uinet_cksum_host_cpu", lib().uinet_cksum_host_cpu(ctypes.byref(st), int(reset)))
    d = {k: int(getattr(st, k)) for k, _ in HostCpu._fields_}
    d["cpu_ns"] = d["caller_cpu_ns"] + d["helper_cpu_ns"]
    return d


def set_tuning(key: str, value: int) -> None:
    """uinet_cksum_set_tuning: performance knobs that never change results."""
    _check("uinet_cksum_set_tuning", lib().uinet_cksum_set_tuning(key.encode(), value))


def last_kernel() -> str:
    """The kernel instantiation this thread's last launch started (demangled;
    "" before any launch): uinet_cksum_last_kernel."""
    return lib().uinet_cksum_last_kernel().decode()


def device_ok() -> bool:
    return bool(lib().uinet_cksum_device_ok())
