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

Chain-shaped variants (uinet_cksum_chains), built by one layout function and
materialised identically on the host (tests, oracle) or in HBM (bench):
config 3tx  config 3's lengths in the reference TX shape: a header mbuf with
          the 40-B IP+TCP header (tcp_output.c:844-846) chained to m_copy
          slices of shuffled 4-KiB socket-buffer page clusters (:858); the
          in_pseudo seed sits in th_sum (:1080-1081); in_cksum_skip(m, len, 20).
config 5tso  TSO-style: 1-MiB sends cut at MSS 8960 (117 full segments + one
          of 256 B); per segment a 40-B header chained to its payload slice of
          the send buffer, in_cksum_pseudo_header(m, 20 + seglen, 20, src,
          dst, TCP) -- the per-segment sums a TSO engine fills in.
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


# ---- chain-shaped variants ------------------------------------------------------

def _bswap16(x):
    x = np.asarray(x, np.uint64)
    return ((x & np.uint64(0xFF)) << np.uint64(8)) | ((x >> np.uint64(8)) & np.uint64(0xFF))


def _in_pseudo(a, b, c) -> np.ndarray:
    s = np.asarray(a, np.uint64) + np.asarray(b, np.uint64) + np.asarray(c, np.uint64)
    for _ in range(4):
        s = (s & np.uint64(0xFFFF)) + (s >> np.uint64(16))
    return s.astype(np.uint16)


def _u16_patch(pos0, vals) -> tuple[np.ndarray, np.ndarray]:
    """Byte positions/values that store the u16s `vals` (native LE) at pos0."""
    v = np.asarray(vals, np.uint16)
    pos = np.stack([pos0, pos0 + 1], 1).reshape(-1)
    return pos.astype(np.int64), v.view(np.uint8).reshape(-1).copy()


def config3tx_layout(n: int, seed: int = 33):
    """Config 3's lengths in the reference TX chain shape (see module doc)."""
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array([64, 576, 1500], np.int64), n)
    pay = lens - 40
    clus0 = 256 * n                      # header mbufs first, then page clusters
    hdr_off = 256 * np.arange(n, dtype=np.int64) + 88 + 16   # pktdat + max_linkhdr
    s0 = np.concatenate([[0], np.cumsum(pay)])[:-1]
    total = int(pay.sum())
    nclus = total // 4096 + 2
    perm = rng.permutation(nclus).astype(np.int64)
    c0, o0 = s0 // 4096, s0 % 4096
    first = np.minimum(pay, 4096 - o0)
    two = first < pay
    nseg = 2 + two.astype(np.int64)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)])
    seg_off = np.zeros(int(pkt_seg[-1]), np.int64)
    seg_len = np.zeros_like(seg_off)
    h = pkt_seg[:-1]
    seg_off[h], seg_len[h] = hdr_off, 40
    seg_off[h + 1], seg_len[h + 1] = clus0 + perm[c0] * 4096 + o0, first
    seg_off[h[two] + 2] = clus0 + perm[c0[two] + 1] * 4096
    seg_len[h[two] + 2] = pay[two] - first[two]
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    th = _in_pseudo(src, dst, _bswap16(6 + lens - 20))       # tcp_output.c:1080-1081
    p1, v1 = _u16_patch(hdr_off + 36, th)
    p2, v2 = _u16_patch(hdr_off + 10, np.zeros(n, np.uint16))  # ip_sum not yet set
    return dict(n=n, lens=lens, skip=np.full(n, 20, np.int64), seed=None,
                seg_off=seg_off, seg_len=seg_len, pkt_seg=pkt_seg,
                patch_pos=np.concatenate([p1, p2]), patch_val=np.concatenate([v1, v2]),
                arena_bytes=int(clus0 + nclus * 4096 + 64), stream_seed=SEED_BASE + 3 + 100,
                bytes=int((lens - 20).sum()), hdr_off=hdr_off)


def config5tso_layout(sends: int = 1111, mss: int = 8960, send_bytes: int = 1 << 20,
                      seed: int = 55):
    """TSO-style per-segment sums of 1-MiB sends (see module doc)."""
    rng = np.random.default_rng(seed)
    per = -(-send_bytes // mss)
    seglen1 = np.full(per, mss, np.int64)
    seglen1[-1] = send_bytes - mss * (per - 1)
    n = sends * per
    seglen = np.tile(seglen1, sends)
    hdr_bytes = 64 * n
    hdr_off = 64 * np.arange(n, dtype=np.int64)
    pay_off = (hdr_bytes + send_bytes * np.repeat(np.arange(sends, dtype=np.int64), per)
               + np.tile(mss * np.arange(per, dtype=np.int64), sends))
    pkt_seg = 2 * np.arange(n + 1, dtype=np.int64)
    seg_off = np.stack([hdr_off, pay_off], 1).reshape(-1)
    seg_len = np.stack([np.full(n, 40, np.int64), seglen], 1).reshape(-1)
    src = np.repeat(rng.integers(0, 2**32, sends, dtype=np.uint64), per)   # one flow per send
    dst = np.repeat(rng.integers(0, 2**32, sends, dtype=np.uint64), per)
    plen = 20 + seglen
    p1, v1 = _u16_patch(hdr_off + 36, np.zeros(n, np.uint16))   # th_sum left to the engine
    p2, v2 = _u16_patch(hdr_off + 10, np.zeros(n, np.uint16))
    return dict(n=n, lens=40 + seglen, skip=np.full(n, 20, np.int64),
                seed=pseudo_seed(src, dst, 6, plen), src=src, dst=dst, plen=plen, off0=20,
                seg_off=seg_off, seg_len=seg_len, pkt_seg=pkt_seg,
                patch_pos=np.concatenate([p1, p2]), patch_val=np.concatenate([v1, v2]),
                arena_bytes=int(hdr_bytes + sends * send_bytes + 64),
                stream_seed=SEED_BASE + 5 + 100, bytes=int(plen.sum()), sends=sends,
                per_send=per, mss=mss)


def chain_layout(cfg: str, n=None):
    if cfg == "3tx":
        return config3tx_layout(n or (1 << 20))
    if cfg == "5tso":
        return config5tso_layout(n or 1111)
    raise ValueError(cfg)


def materialize_host(lay) -> np.ndarray:
    """The layout's arena in host memory (4-KiB aligned)."""
    arena = aligned_empty(lay["arena_bytes"])
    splitmix64_bytes(lay["arena_bytes"], lay["stream_seed"], out=arena)
    arena[lay["patch_pos"]] = lay["patch_val"]
    return arena


def materialize_device(lay, device="cuda"):
    """The same arena generated in HBM, plus the chain descriptors there."""
    import torch

    arena = torch.empty(lay["arena_bytes"], dtype=torch.uint8, device=device)
    splitmix64_fill_device(arena, lay["stream_seed"])
    arena[torch.from_numpy(lay["patch_pos"]).to(device)] = torch.from_numpy(lay["patch_val"]).to(device)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(device)  # noqa: E731
    nseg = int(lay["seg_len"].size)
    return dict(arena=arena, seg_off=t(lay["seg_off"], np.int64),
                seg_len=t(lay["seg_len"], np.int32), pkt_seg=t(lay["pkt_seg"], np.int32),
                len=t(lay["lens"], np.int32), skip=t(lay["skip"], np.int32),
                seed=None if lay["seed"] is None else t(lay["seed"].view(np.int32), np.int32),
                n=lay["n"], nseg=nseg, mean_seg=int(lay["seg_len"].sum() // max(1, nseg)),
                bytes=lay["bytes"], layout=lay)


# ---- the same chains as struct mbufs in HBM (uinet_cksum_mbufs) ----------------

def device_mbufs(arena, seg_off, seg_len, pkt_seg, shuffle: int | None = None,
                 inline_first: int | None = None):
    """struct mbuf chains in HBM over a device arena, one 256-B record
    (MSIZE, sys/sys/param.h:159) per segment, the way MbufChains lays them out
    on the host: m_next (offset 0) and m_data (16) are DEVICE addresses, m_len
    (24) the segment length, M_PKTHDR in the first mbuf's m_flags (28).
    Records sit in chain order, or -- with ``shuffle`` a seed -- at a random
    permutation of the slots (a UMA zone's free list hands mbufs out in no
    particular order).  ``inline_first`` = k: every packet's first segment
    lies INSIDE its own mbuf, k bytes into the record (m_pktdat + max_linkhdr:
    a header mbuf as tcp_output.c:844-846 builds it, config 3tx's layout puts
    those records in the arena), so that record is written into the arena at
    seg_off - k instead of the record array.  Returns dict(mbufs=int64 tensor
    (nseg, 32), heads=int64 tensor of the first mbufs' addresses, 0 for an
    empty chain)."""
    import torch

    dev = arena.device
    seg_off = torch.as_tensor(seg_off).to(dev, torch.int64)
    seg_len = torch.as_tensor(seg_len).to(dev, torch.int64)
    pkt_seg = torch.as_tensor(pkt_seg).to(dev, torch.int64)
    nseg, n = seg_off.numel(), pkt_seg.numel() - 1
    mb = torch.zeros((max(nseg, 1), 32), dtype=torch.int64, device=dev)
    if shuffle is None:
        slot = torch.arange(nseg, dtype=torch.int64, device=dev)
    else:
        g = torch.Generator(device="cpu").manual_seed(int(shuffle))
        slot = torch.randperm(nseg, generator=g).to(dev)
    addr = mb.data_ptr() + 256 * slot
    nonempty = pkt_seg[1:] > pkt_seg[:-1]
    first = pkt_seg[:-1][nonempty]
    last = pkt_seg[1:][nonempty] - 1
    if inline_first is not None:
        rec = seg_off[first] - int(inline_first)
        if bool((rec < 0).any()) or bool((rec % 8 != 0).any()):
            raise ValueError("inline_first: records must lie 8-B aligned inside the arena")
        addr[first] = arena.data_ptr() + rec
    nxt = torch.zeros(nseg, dtype=torch.int64, device=dev)
    if nseg > 1:
        nxt[:-1] = addr[1:]
    nxt[last] = 0
    flags = torch.zeros(nseg, dtype=torch.int64, device=dev)
    flags[first] = 0x2  # M_PKTHDR
    fields = torch.stack([nxt, torch.zeros_like(nxt), arena.data_ptr() + seg_off,
                          (seg_len & 0xFFFFFFFF) | (flags << 32)], 1)
    if nseg:
        mb[slot, :4] = fields
    if inline_first is not None and first.numel():
        # the header mbufs' m_hdr words, written into their records in the arena
        words = arena.view(-1)[: arena.numel() // 8 * 8].view(torch.int64)
        w0 = (seg_off[first] - int(inline_first)) // 8
        for j in range(4):
            words[w0 + j] = fields[first, j]
    heads = torch.zeros(n, dtype=torch.int64, device=dev)
    heads[nonempty] = addr[first]
    return dict(mbufs=mb, heads=heads)


def tx_inline_offset(lay) -> int:
    """Where config 3tx's header bytes sit in their 256-B header mbuf record
    (m_pktdat 88 + max_linkhdr 16): device_mbufs(inline_first=...)."""
    return int(lay["hdr_off"][0] % 256)


def mbufs_walked(seg_len, pkt_seg, lens, skip) -> int:
    """How many mbufs in_cksum_skip(m, len, skip) reads (in_cksum.c:203-229):
    every mbuf that starts before byte len of its chain (the skip walk reads
    the ones before `skip` too), when len > skip; none otherwise."""
    seg_len = np.asarray(seg_len, np.int64)
    pkt_seg = np.asarray(pkt_seg, np.int64)
    n = pkt_seg.size - 1
    seg_pkt = np.repeat(np.arange(n), np.diff(pkt_seg))
    run = np.cumsum(seg_len) - seg_len
    pos = run - run[np.minimum(pkt_seg[:-1], max(run.size - 1, 0))][seg_pkt]
    lens = np.asarray(lens, np.int64) if lens is not None else np.full(n, np.iinfo(np.int64).max)
    skip = np.zeros(n, np.int64) if skip is None else np.broadcast_to(np.asarray(skip, np.int64), (n,))
    lens = np.broadcast_to(lens, (n,))
    want = (lens > skip)[seg_pkt]
    return int(np.count_nonzero(want & (pos < lens[seg_pkt])))


def clipped_segments(seg_off, seg_len, pkt_seg, lens, skip):
    """Per segment, the arena bytes [start, end) that in_cksum_skip(m, len,
    skip) sums (in_cksum.c:203-229: len counts from the chain start), for the
    segments that contribute; and the algorithmic byte count."""
    seg_off, seg_len = np.asarray(seg_off, np.int64), np.asarray(seg_len, np.int64)
    pkt_seg = np.asarray(pkt_seg, np.int64)
    n = pkt_seg.size - 1
    seg_pkt = np.repeat(np.arange(n), np.diff(pkt_seg))
    run = np.cumsum(seg_len) - seg_len                      # running position over all chains
    pos = run - run[np.minimum(pkt_seg[:-1], max(run.size - 1, 0))][seg_pkt]  # within its chain
    lens = np.full(n, np.iinfo(np.int64).max) if lens is None else np.asarray(lens, np.int64)
    skip = np.zeros(n, np.int64) if skip is None else np.asarray(skip, np.int64)
    lo = np.clip(skip[seg_pkt] - pos, 0, seg_len)
    hi = np.clip(lens[seg_pkt] - pos, 0, seg_len)
    keep = hi > lo
    return seg_off[keep] + lo[keep], seg_off[keep] + hi[keep], int((hi - lo)[keep].sum())


def lines_touched(a, b, line: int) -> int:
    """Distinct `line`-byte lines holding at least one byte of the [a, b) ranges."""
    if a.size == 0:
        return 0
    first, last = a // line, (b - 1) // line
    order = np.argsort(first, kind="stable")
    f, l = first[order], last[order]
    runmax = np.maximum.accumulate(l)
    new = np.concatenate([[True], f[1:] > runmax[:-1]])
    starts = f[new]
    ends = np.maximum.reduceat(l, np.flatnonzero(new))
    return int((ends - starts + 1).sum())


def layout_floor(seg_off, seg_len, pkt_seg, lens, skip, seed: bool, line: int = 128,
                 seg_desc_bytes: int = 12) -> dict:
    """HBM-traffic floor of a chained batch: the distinct lines holding a
    summed byte plus the descriptors the chain kernel reads (seg_desc_bytes
    per segment: 12 wide, 6 packed; pkt_seg + len + skip [+ seed] per
    packet).  What no kernel reading these packets from this layout can
    avoid fetching."""
    s, e, algo = clipped_segments(seg_off, seg_len, pkt_seg, lens, skip)
    nseg, npkt = int(np.asarray(seg_len).size), int(np.asarray(pkt_seg).size) - 1
    arena = lines_touched(s, e, line) * line
    desc = seg_desc_bytes * nseg + npkt * (4 + 4 + 4 + (4 if seed else 0)) + 4
    return dict(line=line, arena_bytes=arena, descriptor_bytes=desc, floor_bytes=arena + desc,
                algorithmic_bytes=algo)
