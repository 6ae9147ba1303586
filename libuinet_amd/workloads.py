"""Synthetic packet batches in the shapes of BASELINE.json's configs.

Payload bytes are the splitmix64 stream of BASELINE.md (seed
0x6C69627569657401 + config index [+ rank]) so host- and device-built batches
are byte-identical.  Device batches are generated with torch integer ops
straight into HBM (no multi-GB host round trip).

config 2  1,048,576 x 1500 B contiguous packets at stride 1500 (4-B aligned
          starts), in_cksum_skip(m, 1500, 0); RX variant stride 1514, +14.
config 3  1,048,576 packets of 64/576/1500 B (uniform), each chained into
          m_fragment(-2)-style random 1..256-B segments
          (sys/kern/uipc_mbuf.c:1724-1735) laid out in order with random
          0-7-B gaps; in_cksum_skip(m, len, 20).
config 4  config 2's kernel per GPU, 2,097,152 packets per GPU (bench --packets).
config 5  131,072 x 9000 B jumbo frames, in_cksum_pseudo_header(m, 8980, 20,
          src, dst, TCP/UDP): the pseudo-header seed per packet + 8980 bytes.
"""
from __future__ import annotations

import numpy as np

from .mbuf import SEED_BASE, aligned_empty, splitmix64_bytes

_M64 = (1 << 64) - 1


def _signed(x: int) -> int:
    x &= _M64
    return x - (1 << 64) if x >> 63 else x


def splitmix64_fill_device(out, seed: int, block_words: int = 1 << 24):
    """Fill the uint8 device tensor ``out`` with the splitmix64 stream of
    :func:`libuinet_amd.mbuf.splitmix64_bytes` (same bytes), using wrapping
    int64 torch ops on the GPU."""
    import torch

    nbytes = out.numel()
    nwords = (nbytes + 7) // 8
    g = _signed(0x9E3779B97F4A7C15)
    m1 = _signed(0xBF58476D1CE4E5B9)
    m2 = _signed(0x94D049BB133111EB)

    def lsr(z, k):  # logical shift right on int64
        return (z >> k) & ((1 << (64 - k)) - 1)

    for w0 in range(0, nwords, block_words):
        w1 = min(nwords, w0 + block_words)
        i = torch.arange(w0 + 1, w1 + 1, dtype=torch.int64, device=out.device)
        z = i * g + _signed(seed)
        z = (z ^ lsr(z, 30)) * m1
        z = (z ^ lsr(z, 27)) * m2
        z = z ^ lsr(z, 31)
        b = z.view(torch.uint8)
        lo, hi = 8 * w0, min(nbytes, 8 * w1)
        out[lo:hi].copy_(b[: hi - lo])
    return out


def config2_device(n: int = 1 << 20, stride: int = 1500, length: int = 1500, base: int = 0,
                   rank: int = 0, device="cuda"):
    """Device-resident config-2 batch: dict(arena, off, len, n, bytes)."""
    import torch

    arena = torch.empty(base + stride * n + 64, dtype=torch.uint8, device=device)
    splitmix64_fill_device(arena, SEED_BASE + 2 + 1000 * rank)
    off = base + stride * torch.arange(n, dtype=torch.int64, device=device)
    ln = torch.full((n,), length, dtype=torch.int32, device=device)
    return dict(arena=arena, off=off, len=ln, n=n, stride=stride, length=length, base=base,
                bytes=n * length)


def config3_layout(n: int, seed: int = 3):
    """Host-side layout of config 3 (no payload): lengths, segments, arena size."""
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array([64, 576, 1500], np.int64), n)
    bounds = np.concatenate([[0], np.cumsum(lens)])
    total = int(bounds[-1])
    steps = rng.integers(1, 257, int(total / 128.5 * 1.05) + 1024)
    cuts = np.cumsum(steps)
    while cuts[-1] < total:  # pragma: no cover - the 5 % margin covers it
        cuts = np.concatenate([cuts, cuts[-1] + np.cumsum(rng.integers(1, 257, 1024))])
    cuts = np.union1d(cuts[cuts < total], bounds)  # sorted, unique, includes 0 and total
    seg_start = cuts[:-1]
    seg_len = np.diff(cuts)
    pkt_seg = np.searchsorted(cuts, bounds)
    gaps = rng.integers(0, 8, seg_len.size)
    seg_off = np.cumsum(seg_len + gaps) - seg_len  # each segment at cursor + its gap
    arena_bytes = int(seg_off[-1] + seg_len[-1] + 64)
    return dict(lens=lens, seg_start=seg_start, seg_off=seg_off.astype(np.int64),
                seg_len=seg_len.astype(np.int64), pkt_seg=pkt_seg.astype(np.int64),
                arena_bytes=arena_bytes, total=total, n=n)


def build_config3(n: int = 1 << 20, seed: int = 3, rank: int = 0):
    """Host config-3 batch (payload included) for tests: each segment k holds
    the logical packet bytes [seg_start[k], + seg_len[k]) of a splitmix64
    stream, placed at arena offset seg_off[k]."""
    lay = config3_layout(n, seed)
    stream = splitmix64_bytes(lay["total"], SEED_BASE + 3 + 1000 * rank)
    arena = aligned_empty(lay["arena_bytes"])
    arena[:] = 0
    # scatter the stream into the gapped layout, segment by segment (vectorised
    # by per-byte index arithmetic in blocks)
    seg_of_byte_start = lay["seg_off"] - lay["seg_start"]  # arena = stream + shift[k]
    k = np.searchsorted(lay["seg_start"], np.arange(lay["total"]), side="right") - 1
    arena[np.arange(lay["total"]) + seg_of_byte_start[k]] = stream
    lay.update(arena=arena, mean_seg=int(lay["total"] / max(1, lay["seg_len"].size)),
               skip=np.full(n, 20, np.int64), bytes=int((lay["lens"] - 20).sum()))
    return lay


def config3_device(n: int = 1 << 20, seed: int = 3, rank: int = 0, device="cuda"):
    """Device-resident config-3 batch.  The payload is generated in HBM and
    the segment placement (stream byte -> gapped arena) is applied there."""
    import torch

    lay = config3_layout(n, seed)
    stream = torch.empty(lay["total"], dtype=torch.uint8, device=device)
    splitmix64_fill_device(stream, SEED_BASE + 3 + 1000 * rank)
    arena = torch.zeros(lay["arena_bytes"], dtype=torch.uint8, device=device)
    shift = torch.from_numpy(lay["seg_off"] - lay["seg_start"]).to(device)
    starts = torch.from_numpy(lay["seg_start"]).to(device)
    block = 1 << 26
    for b0 in range(0, lay["total"], block):
        idx = torch.arange(b0, min(lay["total"], b0 + block), dtype=torch.int64, device=device)
        k = torch.searchsorted(starts, idx, right=True) - 1
        arena[idx + shift[k]] = stream[idx]
    del stream
    return dict(arena=arena,
                seg_off=torch.from_numpy(lay["seg_off"]).to(device),
                seg_len=torch.from_numpy(lay["seg_len"].astype(np.int32)).to(device),
                pkt_seg=torch.from_numpy(lay["pkt_seg"].astype(np.int32)).to(device),
                len=torch.from_numpy(lay["lens"].astype(np.int32)).to(device),
                skip=torch.full((n,), 20, dtype=torch.int32, device=device),
                n=n, mean_seg=int(lay["total"] / lay["seg_len"].size),
                nseg=int(lay["seg_len"].size), bytes=int((lay["lens"] - 20).sum()), layout=lay)


def pseudo_seed(src, dst, proto, plen) -> np.ndarray:
    """in_cksum.c:252-253 seed (src + dst + htons(proto) + htons(plen)),
    end-around folded to 16 bits so it fits the engine's u32 seed slot."""
    src = np.asarray(src, np.uint64)
    dst = np.asarray(dst, np.uint64)
    proto = np.asarray(proto, np.uint64)
    plen = np.asarray(plen, np.uint64) & np.uint64(0xFFFF)

    def bs(x):
        return ((x & np.uint64(0xFF)) << np.uint64(8)) | (x >> np.uint64(8))

    s = src + dst + bs(proto) + bs(plen)
    for _ in range(4):
        s = (s & np.uint64(0xFFFF)) + (s >> np.uint64(16))
    return s.astype(np.uint32)


def config5_device(n: int = 131072, frame: int = 9000, off0: int = 20, rank: int = 0,
                   device="cuda"):
    """Device-resident config-5 batch: jumbo frames + per-packet pseudo seeds."""
    import torch

    rng = np.random.default_rng(5 + 1000 * rank)
    arena = torch.empty(frame * n + 64, dtype=torch.uint8, device=device)
    splitmix64_fill_device(arena, SEED_BASE + 5 + 1000 * rank)
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    proto = rng.choice(np.array([6, 17], np.uint64), n)
    plen = frame - off0
    seed = pseudo_seed(src, dst, proto, plen)
    off = off0 + frame * torch.arange(n, dtype=torch.int64, device=device)
    return dict(arena=arena, off=off, len=torch.full((n,), plen, dtype=torch.int32, device=device),
                seed=torch.from_numpy(seed.view(np.int32)).to(device), n=n, bytes=n * plen,
                src=src, dst=dst, proto=proto, plen=plen, off0=off0, frame=frame)
