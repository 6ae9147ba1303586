"""GPU parity: every entry point of the HIP engine, bit-exact against the
oracle (itself pinned to the reference's golden vectors) and against the
golden vectors directly.  Runs on an MI355X (`pytest -m gpu`)."""
from __future__ import annotations

import threading

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes

from test_oracle import pcap_cases

pytestmark = pytest.mark.gpu

HINTS = (0, 64, 80, 200, 500, 1500, 4000, 9000)  # every kernel geometry (4000: 64 x 3, 9000: 64 x 9)


@pytest.fixture(scope="module")
def torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert u.device_ok(), "device is not gfx950"
    return torch


def dev(torch, a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host16(t) -> np.ndarray:
    return t.cpu().view(__import__("torch").int16).numpy().view(np.uint16)


def rand_arena(nbytes: int, seed: int) -> np.ndarray:
    a = aligned_empty(nbytes)
    splitmix64_bytes(nbytes, seed, out=a)
    return a


def rand_spans(rng, n, arena_size, max_len):
    ln = rng.integers(0, max_len + 1, n)
    edge = rng.random(n)
    ln = np.where(edge < 0.05, rng.choice([0, 1, 2, 3, 4, 15, 16, 17, 31, 32, 33], n), ln)
    off = rng.integers(0, arena_size - max_len - 1, n)
    return off.astype(np.int64), ln.astype(np.int64)


# ---- device-resident API ------------------------------------------------------

@pytest.mark.parametrize("hint", HINTS)
@pytest.mark.parametrize("flags", [0, u.F_UDP, u.F_NO_COMPLEMENT])
def test_spans_random(torch_dev, ora, hint, flags):
    torch = torch_dev
    rng = np.random.default_rng(hint * 7 + flags)
    arena = rand_arena(1 << 21, 17 + hint)
    n = 6000
    off, ln = rand_spans(rng, n, arena.size, 3000)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    seed[rng.random(n) < 0.3] = 0
    par = rng.integers(0, 2, n).astype(np.uint8)
    want = ora.spans(arena, off, ln, seed, par, flags)
    got = u.cksum_spans(dev(torch, arena), dev(torch, off), dev(torch, ln.astype(np.int32)),
                        seed=dev(torch, seed.view(np.int32)), parity=dev(torch, par),
                        flags=flags, len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)


@pytest.mark.parametrize("hint", HINTS)
def test_spans_no_seed_no_parity(torch_dev, ora, hint):
    torch = torch_dev
    rng = np.random.default_rng(99 + hint)
    arena = rand_arena(1 << 20, 5)
    off, ln = rand_spans(rng, 4000, arena.size, 1600)
    want = ora.spans(arena, off, ln)
    got = u.cksum_spans(dev(torch, arena), dev(torch, off), dev(torch, ln.astype(np.int32)),
                        len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)


@pytest.mark.parametrize("pipe", [1])
@pytest.mark.parametrize("n", [1, 7, 6000, 70001])
def test_spans_every_kernel(torch_dev, ora, n, pipe):
    """Every span kernel family (k_spans_lean, k_spans_quad, k_spans) at
    every geometry, and the strided kernel at 64 and 60 B: each
    packet folded exactly once, ragged tails."""
    torch = torch_dev
    rng = np.random.default_rng(500 + n + 7 * pipe)
    arena = rand_arena(1 << 21, 31)
    off, ln = rand_spans(rng, n, arena.size, 1600)
    want = ora.spans(arena, off, ln)
    d_arena = dev(torch, arena)
    for hint in HINTS:
        got = u.cksum_spans(d_arena, dev(torch, off), dev(torch, ln.astype(np.int32)),
                            len_hint=hint)
        np.testing.assert_array_equal(host16(got), want)
    m = min(n, (arena.size - 64) // 64)
    for length in (64, 60):
        got = u.cksum_strided(d_arena, 64, length, m)
        want_s = ora.spans(arena, 64 * np.arange(m, dtype=np.int64),
                           np.full(m, length, np.int64))
        np.testing.assert_array_equal(host16(got), want_s)


@pytest.mark.parametrize("pipe,bpc", [(1, 1), (1, 3), (1, 0)])
def test_spans_pipe_grids(torch_dev, ora, pipe, bpc):
    """The persistent span kernel at 32 and 64 lanes per packet
    (k_spans_lean), on grids small enough that every wave walks many steps:
    ragged batches, seeds, parity, UDP, spans longer than one round, empty
    spans."""
    torch = torch_dev
    rng = np.random.default_rng(700 + 10 * pipe + bpc)
    arena = rand_arena(1 << 22, 41)
    u.set_tuning("blocks_per_cu", bpc)
    try:
        for n in (1, 7, 6000, 70001):
            off, ln = rand_spans(rng, n, arena.size, 12000)
            seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            par = rng.integers(0, 2, n).astype(np.uint8)
            d = dict(arena=dev(torch, arena), off=dev(torch, off), ln=dev(torch, ln.astype(np.int32)))
            for hint in (1500, 9000):
                want = ora.spans(arena, off, ln, seed, par, u.F_UDP)
                got = u.cksum_spans(d["arena"], d["off"], d["ln"], seed=dev(torch, seed.view(np.int32)),
                                    parity=dev(torch, par), flags=u.F_UDP, len_hint=hint)
                np.testing.assert_array_equal(host16(got), want)
                got = u.cksum_spans(d["arena"], d["off"], d["ln"], len_hint=hint)
                np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln))
    finally:
        u.set_tuning("blocks_per_cu", 0)


@pytest.mark.parametrize("pipe,bpc", [(1, 1), (1, 3), (1, 0)])
def test_strided_pipe_grids(torch_dev, ora, pipe, bpc):
    """The strided API on the persistent kernel (k_spans_lean; 32 / 64 lanes
    per packet), with grids small
    enough that every lane group walks many packets: packet lengths of one
    round and of several, aligned and unaligned strides and bases, seeds and
    UDP, ragged counts."""
    torch = torch_dev
    rng = np.random.default_rng(900 + 10 * pipe + bpc)
    arena = rand_arena(24 << 20, 43)
    d_arena = dev(torch, arena)
    u.set_tuning("blocks_per_cu", bpc)
    try:
        for length, stride, base in ((1500, 1500, 0), (1500, 1514, 14), (1480, 1501, 3),
                                     (9000, 9000, 0), (8980, 9017, 5), (2000, 2048, 1)):
            for n in (1, 5, 2049):
                n = min(n, (arena.size - base - length) // stride)
                seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                off = base + stride * np.arange(n, dtype=np.int64)
                got = u.cksum_strided(d_arena[base:], stride, length, n,
                                      seed=dev(torch, seed.view(np.int32)), flags=u.F_UDP)
                want = ora.spans(arena, off, np.full(n, length, np.int64), seed, None, u.F_UDP)
                np.testing.assert_array_equal(host16(got), want)
    finally:
        u.set_tuning("blocks_per_cu", 0)


@pytest.mark.parametrize("pipe", [1])
def test_spans_far_apart(torch_dev, ora, pipe):
    """Neighbouring packets (one wave's pair at 32 lanes per packet, one
    wave's 16 at 4) that lie 4 GiB and more apart in one arena: the lean
    kernel's loads are relative to one scalar base, and such a pair takes its
    64-bit fallback."""
    torch = torch_dev
    rng = np.random.default_rng(4242)
    win = 1 << 16
    far = (1 << 32) + 4096 + 7  # > 4 GiB between the two windows
    d = torch.empty(far + win, dtype=torch.uint8, device="cuda")
    lo, hi = rand_arena(win, 51), rand_arena(win, 52)
    d[:win].copy_(torch.from_numpy(lo))
    d[far:far + win].copy_(torch.from_numpy(hi))
    host = np.concatenate([lo, hi])  # the two windows back to back, for the oracle
    n = 2000
    ln = rng.integers(0, 3000, n)
    ln[::97] = 0
    o = rng.integers(0, win - 3000, n)
    side = (np.arange(n) // rng.integers(1, 3)) % 2  # alternate windows, pairs and singles
    off_dev = np.where(side == 1, far + o, o).astype(np.int64)
    off_host = np.where(side == 1, win + o, o).astype(np.int64)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    par = rng.integers(0, 2, n).astype(np.uint8)
    try:
        for hint in (64, 1500, 9000):
            got = u.cksum_spans(d, dev(torch, off_dev), dev(torch, ln.astype(np.int32)),
                                seed=dev(torch, seed.view(np.int32)), parity=dev(torch, par),
                                flags=u.F_UDP, len_hint=hint)
            want = ora.spans(host, off_host, ln.astype(np.int64), seed, par, u.F_UDP)
            np.testing.assert_array_equal(host16(got), want)
    finally:
        del d
        torch.cuda.empty_cache()


@pytest.mark.parametrize("pipe,bpc", [(1, 0), (1, 1), (1, 3)])
def test_spans_small_packets(torch_dev, ora, pipe, bpc):
    """The small-packet geometries (4, 8 and 16 lanes per packet; the 4-lane
    shapes run k_spans_quad, the 8 and 16 k_spans), also on
    grids small enough that every wave walks many steps: ragged counts, spans
    longer than the geometry's round, empty spans, seeds, parity, UDP; the
    strided API at 64-B packets, 16-B aligned and not."""
    torch = torch_dev
    u.set_tuning("blocks_per_cu", bpc)
    try:
        _small_packets(torch, ora)
    finally:
        u.set_tuning("blocks_per_cu", 0)


def _small_packets(torch, ora):
    rng = np.random.default_rng(1300)
    arena = rand_arena(24 << 20, 45)
    d_arena = dev(torch, arena)
    for hint, max_len in ((64, 80), (90, 120), (200, 300), (600, 900)):
        for n in (1, 63, 64, 65, 1000, 70001):
            # offsets leave room for the 5000-B spans (longer than the
            # geometry's round) that 1 % of the packets get
            off, ln = rand_spans(rng, n, arena.size - 5000, max_len)
            ln[rng.random(n) < 0.01] = 5000
            seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            par = rng.integers(0, 2, n).astype(np.uint8)
            d_off, d_ln = dev(torch, off), dev(torch, ln.astype(np.int32))
            got = u.cksum_spans(d_arena, d_off, d_ln, seed=dev(torch, seed.view(np.int32)),
                                parity=dev(torch, par), flags=u.F_UDP, len_hint=hint)
            np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln, seed, par, u.F_UDP))
            got = u.cksum_spans(d_arena, d_off, d_ln, len_hint=hint)
            np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln))
    for length, stride, base in ((64, 64, 0), (64, 80, 16), (60, 67, 3), (40, 64, 2)):
        for n in (1, 65, 100003):
            seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            off = base + stride * np.arange(n, dtype=np.int64)
            got = u.cksum_strided(d_arena[base:], stride, length, n,
                                  seed=dev(torch, seed.view(np.int32)), flags=u.F_UDP)
            want = ora.spans(arena, off, np.full(n, length, np.int64), seed, None, u.F_UDP)
            np.testing.assert_array_equal(host16(got), want)


def test_spans_long(torch_dev, ora):
    """Spans far longer than one unrolled round of any geometry."""
    torch = torch_dev
    arena = rand_arena(40 << 20, 23)
    off = np.array([0, 1, 3, 4097, 5 << 20, 7], np.int64)
    ln = np.array([1 << 16, (1 << 20) + 3, 9000, 65535, 32 << 20, 0], np.int64)
    want = ora.spans(arena, off, ln)
    for hint in HINTS:
        got = u.cksum_spans(dev(torch, arena), dev(torch, off), dev(torch, ln.astype(np.int32)),
                            len_hint=hint)
        np.testing.assert_array_equal(host16(got), want)


@pytest.mark.parametrize("hint", [1500, 4000, 9000])
def test_spans_round_edges(torch_dev, ora, hint):
    """Span lengths at and around the 64-lane geometries' round sizes (3 KB
    for 64 x 3, 9 KB for 64 x 9: one, two and three rounds and a byte either
    side) at every head offset 0-15, with seeds, parity and UDP, in batches
    where the wave's two packets differ (32 lanes) or a wave holds one packet
    of each length in turn (64 lanes)."""
    torch = torch_dev
    rng = np.random.default_rng(4242)
    edges = [1, 15, 16, 17, 1535, 1536, 1537, 3071, 3072, 3073, 6143, 6144, 6145,
             9199, 9200, 9201, 9215, 9216, 9217, 18431, 18432, 18433, 27648, 27649]
    ln = np.array([e for e in edges for _ in range(16)], np.int64)
    n = ln.size
    ln = np.concatenate([ln, ln[rng.permutation(n)]])
    head = np.tile(np.arange(16, dtype=np.int64), 2 * len(edges))
    arena = rand_arena(4 << 20, 77)
    off = (rng.integers(0, (arena.size - 28000) // 16, ln.size) * 16 + head).astype(np.int64)
    seed = rng.integers(0, 2**32, ln.size, dtype=np.uint64).astype(np.uint32)
    par = rng.integers(0, 2, ln.size).astype(np.uint8)
    d_arena, d_off, d_ln = dev(torch, arena), dev(torch, off), dev(torch, ln.astype(np.int32))
    got = u.cksum_spans(d_arena, d_off, d_ln, seed=dev(torch, seed.view(np.int32)),
                        parity=dev(torch, par), flags=u.F_UDP, len_hint=hint)
    np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln, seed, par, u.F_UDP))
    got = u.cksum_spans(d_arena, d_off, d_ln, len_hint=hint)
    np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln))
    # strided: every packet the same length, at each edge
    for e in (3072, 3073, 9216, 9217):
        m = 257
        got = u.cksum_strided(d_arena[3:], e + 5, e, m)
        want = ora.spans(arena, 3 + (e + 5) * np.arange(m, dtype=np.int64), np.full(m, e, np.int64))
        np.testing.assert_array_equal(host16(got), want)


def test_spans_zero_and_ff(torch_dev, ora):
    torch = torch_dev
    for fill in (0x00, 0xFF):
        arena = aligned_empty(1 << 16)
        arena[:] = fill
        off = np.arange(0, 64 * 17, 17, dtype=np.int64)
        ln = np.arange(64, dtype=np.int64) * 13
        want = ora.spans(arena, off, ln)
        got = u.cksum_spans(dev(torch, arena), dev(torch, off), dev(torch, ln.astype(np.int32)))
        np.testing.assert_array_equal(host16(got), want)
        if fill == 0:
            assert (want == 0xFFFF).all()


def test_empty_batch(torch_dev):
    torch = torch_dev
    arena = torch.zeros(16, dtype=torch.uint8, device="cuda")
    e64 = torch.zeros(0, dtype=torch.int64, device="cuda")
    e32 = torch.zeros(0, dtype=torch.int32, device="cuda")
    assert u.cksum_spans(arena, e64, e32).numel() == 0
    assert u.cksum_strided(arena, 16, 16, 0).numel() == 0


@pytest.mark.parametrize("stride,length,base", [(1500, 1500, 0), (1514, 1500, 14), (9000, 9000, 0),
                                                (1501, 1500, 1), (64, 64, 0), (600, 576, 3),
                                                # 16-B aligned packets of <= 64 B (one chunk
                                                # per lane) and their unaligned neighbours
                                                (16, 16, 0), (48, 33, 0), (64, 1, 0), (80, 64, 16),
                                                (64, 64, 8), (96, 63, 2)])
def test_strided(torch_dev, ora, stride, length, base):
    torch = torch_dev
    n = 3000
    arena = rand_arena(base + stride * n + 64, stride)
    off = base + stride * np.arange(n, dtype=np.int64)
    want = ora.spans(arena, off, length)
    d = dev(torch, arena)
    got = u.cksum_strided(d[base:], stride, length, n)
    np.testing.assert_array_equal(host16(got), want)


TILE32_MIN = 32 * 4096  # launch_chains_t: 32-packet tiles from this many packets, 8 below


def pad_for_tile(tile, pkt_seg, *arrs):
    """Append empty chains (no segments, zeros in `arrs`) so the chain kernel
    runs `tile`-packet tiles (the tile follows the batch size, 8 below
    TILE32_MIN packets); tile 8 / 0 returns the inputs unchanged."""
    n = pkt_seg.size - 1
    if tile != 32 or n >= TILE32_MIN:
        return (pkt_seg, *arrs)
    pad = TILE32_MIN - n
    out = [np.concatenate([pkt_seg, np.full(pad, pkt_seg[-1], pkt_seg.dtype)])]
    for a in arrs:
        out.append(None if a is None else np.concatenate([a, np.zeros(pad, a.dtype)]))
    return tuple(out)


def random_chain_layout(rng, n, arena_size, max_seg=256, max_segs=8):
    nseg = rng.integers(1, max_segs + 1, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(1, max_seg + 1, s)
    seg_len[rng.random(s) < 0.08] = 0
    seg_off = rng.integers(0, arena_size - max_seg - 1, s)
    return seg_off.astype(np.int64), seg_len.astype(np.int64), pkt_seg


@pytest.mark.parametrize("hint", HINTS)
def test_chains_random(torch_dev, ora, hint):
    torch = torch_dev
    rng = np.random.default_rng(1000 + hint)
    arena = rand_arena(1 << 20, 31)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 5000, arena.size,
                                                   max_seg=max(hint, 64) if hint else 256)
    seed = rng.integers(0, 2**32, pkt_seg.size - 1, dtype=np.uint64).astype(np.uint32)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, seed=seed)
    got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)),
                         dev(torch, pkt_seg.astype(np.int32)), seed=dev(torch, seed.view(np.int32)),
                         len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)
    # and the same chains as host mbufs through the reference-shaped walk
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    np.testing.assert_array_equal(ora.chains(arena, seg_off, seg_len, pkt_seg),
                                  ora.skip_batch(ch.heads, tot, 0))


# ---- host-mbuf batch API (the per-call ABI is a host fold: test_percall_host.py) --

def test_golden_skip_batch(torch_dev, arena, golden):
    g = golden("skip")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, g["len"], g["skip"]), g["expected"])


def test_golden_pseudo_batch(torch_dev, arena, golden):
    g = golden("pseudo")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    got = u.in_cksum_pseudo_header_batch(ch.heads, g["plen"], g["off0"], g["src"], g["dst"], g["proto"])
    np.testing.assert_array_equal(got, g["expected"])


def test_golden_hdr_batch(torch_dev, arena, golden):
    g = golden("hdr")
    ips = arena.ctypes.data + g["off"].astype(np.uint64)
    np.testing.assert_array_equal(u.in_cksum_hdr_batch(ips), g["expected"])


def test_golden_configs(torch_dev, arena, golden):
    torch = torch_dev
    g = golden("configs")
    d = dev(torch, arena)
    for tag in ("c2", "c2rx"):
        ch = MbufChains.contiguous(arena, g[f"{tag}_off"], 1500)
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, 1500, 0), g[f"{tag}_expected"])
        got = u.cksum_spans(d, dev(torch, g[f"{tag}_off"]),
                            dev(torch, np.full(64, 1500, np.int32)), len_hint=1500)
        np.testing.assert_array_equal(host16(got), g[f"{tag}_expected"])
    ch = MbufChains(arena, g["c3_seg_off"], g["c3_seg_len"], g["c3_pkt_seg"])
    np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, g["c3_len"], 20), g["c3_expected"])
    ch = MbufChains.contiguous(arena, g["c5_off"], 9000)
    got = u.in_cksum_pseudo_header_batch(ch.heads, 8980, 20, g["c5_src"], g["c5_dst"], g["c5_proto"])
    np.testing.assert_array_equal(got, g["c5_expected"])


def test_pcap_kat_gpu(torch_dev, pcap_frames):
    arena, off, ln, hl, plen, src, dst = pcap_cases(pcap_frames)
    assert not u.in_cksum_hdr_batch(arena.ctypes.data + off.astype(np.uint64)).any()
    ch = MbufChains.contiguous(arena, off, ln)
    assert not u.in_cksum_pseudo_header_batch(ch.heads, plen, hl, src, dst, 6).any()


def test_zero_copy_registered_arena(torch_dev, arena, golden):
    """Registered host memory: the batches are folded in place over PCIe by
    the chain kernel (no staging copy) -- same golden results."""
    u.register_host(arena)
    try:
        g = golden("skip")
        ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, g["len"], g["skip"]),
                                      g["expected"])
        g = golden("pseudo")
        ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
        got = u.in_cksum_pseudo_header_batch(ch.heads, g["plen"], g["off0"], g["src"], g["dst"],
                                             g["proto"])
        np.testing.assert_array_equal(got, g["expected"])
        g = golden("hdr")
        even = (g["off"] % 2) == 0  # odd header addresses take the staging path
        ips = arena.ctypes.data + g["off"].astype(np.uint64)
        np.testing.assert_array_equal(u.in_cksum_hdr_batch(ips[even]), g["expected"][even])
        np.testing.assert_array_equal(u.in_cksum_hdr_batch(ips), g["expected"])
        g = golden("configs")
        ch = MbufChains(arena, g["c3_seg_off"], g["c3_seg_len"], g["c3_pkt_seg"])
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, g["c3_len"], 20),
                                      g["c3_expected"])
        with pytest.raises(u.CksumError):
            u.register_host(arena)  # overlapping registration is refused
    finally:
        u.unregister_host(arena)


def test_zero_copy_partial_registration(torch_dev, ora):
    """Pieces outside registered memory send the batch through staging."""
    rng = np.random.default_rng(81)
    arena = rand_arena(1 << 20, 81)
    half = arena[: 1 << 19]
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 3000, arena.size)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    want = ora.skip_batch(ch.heads, tot, 0)
    u.register_host(half)
    try:
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, tot, 0), want)
        inside = np.array([seg_off[pkt_seg[i]:pkt_seg[i + 1]].max(initial=0) < (1 << 19) - 300
                           for i in range(ch.n)])
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads[inside], tot[inside], 0),
                                      want[inside])
    finally:
        u.unregister_host(half)


def test_host_batch_threads(torch_dev, ora):
    """Concurrent callers (RX threads + TX app threads)."""
    rng = np.random.default_rng(77)
    arena = rand_arena(1 << 20, 77)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 4000, arena.size)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    want = ora.skip_batch(ch.heads, tot, 0)
    results, errors = {}, []

    def worker(k):
        try:
            sl = slice(k * 1000, (k + 1) * 1000)
            for _ in range(5):
                results[k] = u.in_cksum_skip_batch(ch.heads[sl], tot[sl], 0)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    np.testing.assert_array_equal(np.concatenate([results[k] for k in range(4)]), want)


# ---- BASELINE.json sizes --------------------------------------------------------

def test_full_config2(torch_dev, ora):
    """1 M x 1500 B contiguous packets (config 2), stride 1500 and the RX
    stride-1514/+14 variant, whole batch vs the oracle."""
    torch = torch_dev
    n = 1 << 20
    for stride, base in ((1500, 0), (1514, 14)):
        d = torch.randint(0, 256, (base + stride * n + 64,), dtype=torch.uint8, device="cuda")
        off = base + stride * torch.arange(n, dtype=torch.int64, device="cuda")
        ln = torch.full((n,), 1500, dtype=torch.int32, device="cuda")
        got = u.cksum_spans(d, off, ln, len_hint=1500)
        got_s = u.cksum_strided(d[base:], stride, 1500, n)
        want = ora.spans(d.cpu().numpy(), off.cpu().numpy(), 1500)
        np.testing.assert_array_equal(host16(got), want)
        np.testing.assert_array_equal(host16(got_s), want)
        del d


def test_full_config3_chains(torch_dev, ora):
    """1 M mixed 64/576/1500-B packets as m_fragment-style chains of 1..256-B
    segments at random 0-7-B offsets, skip 20 (config 3)."""
    from libuinet_amd.workloads import config3_device

    c = config3_device(1 << 20, seed=3)
    got = u.cksum_chains(c["arena"], c["seg_off"], c["seg_len"], c["pkt_seg"], length=c["len"],
                         skip=c["skip"], len_hint=c["mean_seg"])
    lay = c["layout"]
    want = ora.chains(c["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=20)
    np.testing.assert_array_equal(host16(got), want)


def test_config3_host_layout_matches_device(torch_dev):
    """The host and device config-3 builders place identical bytes."""
    from libuinet_amd.workloads import build_config3, config3_device

    h = build_config3(4096, seed=9)
    d = config3_device(4096, seed=9)
    np.testing.assert_array_equal(d["arena"].cpu().numpy(), h["arena"])


@pytest.mark.parametrize("hint", [0, 40, 200, 500])
def test_chains_many_segments(torch_dev, ora, hint):
    """Chains of 0..300 segments (the tiled kernel carries chain positions
    across 64-segment descriptor rounds), empty chains, 1-byte segments."""
    torch = torch_dev
    rng = np.random.default_rng(7000 + hint)
    arena = rand_arena(1 << 21, 43)
    n = 700
    nseg = rng.integers(0, 301, n)
    nseg[rng.random(n) < 0.1] = 0
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = np.where(rng.random(s) < 0.3, rng.integers(0, 3, s), rng.integers(1, 80, s))
    seg_off = rng.integers(0, arena.size - 100, s).astype(np.int64)
    tot = np.zeros(n, np.int64)
    nz = nseg > 0
    tot[nz] = np.add.reduceat(seg_len, pkt_seg[:-1][nz])
    skip = (rng.random(n) * (tot + 1) * 0.3).astype(np.int64)
    length = skip + (rng.random(n) * (tot - skip + 10)).astype(np.int64)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed)
    got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)),
                         dev(torch, pkt_seg.astype(np.int32)),
                         length=dev(torch, length.astype(np.int32)),
                         skip=dev(torch, skip.astype(np.int32)),
                         seed=dev(torch, seed.view(np.int32)), len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)


@pytest.mark.parametrize("hint", HINTS)
def test_chains_len_skip(torch_dev, ora, hint):
    """in_cksum_skip(chain, len, skip) semantics on device chains: skip
    landing inside / exactly on segment boundaries, len short of, equal to
    and beyond the chain, len <= skip."""
    torch = torch_dev
    rng = np.random.default_rng(4000 + hint)
    arena = rand_arena(1 << 20, 41)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 4000, arena.size)
    n = pkt_seg.size - 1
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    cum = np.concatenate([[0], np.cumsum(seg_len)])
    skip = (rng.random(n) * (tot + 1)).astype(np.int64)
    k = pkt_seg[:-1] + (rng.random(n) * np.diff(pkt_seg)).astype(np.int64)
    skip = np.where(rng.random(n) < 0.25, cum[k] - cum[pkt_seg[:-1]], skip)
    length = skip + (rng.random(n) * (tot - skip + 40)).astype(np.int64)
    length = np.where(rng.random(n) < 0.1, skip - rng.integers(0, 3, n), length)
    length = np.maximum(length, 0)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    np.testing.assert_array_equal(want, ora.skip_batch(ch.heads, length, skip))
    got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)),
                         dev(torch, pkt_seg.astype(np.int32)),
                         length=dev(torch, length.astype(np.int32)),
                         skip=dev(torch, skip.astype(np.int32)), len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)


def test_full_config5_jumbo(torch_dev, ora):
    """131072 x 9000-B jumbo frames, in_cksum_pseudo_header(m, 8980, 20, ...)
    semantics via seeds (config 5); the host batch API on a slice."""
    torch = torch_dev
    n = 131072
    rng = np.random.default_rng(55)
    d = torch.randint(0, 256, (9000 * n,), dtype=torch.uint8, device="cuda")
    host = d.cpu().numpy()
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    proto = rng.choice([6, 17], n).astype(np.uint64)
    bs = lambda x: ((x & 0xFF) << 8) | (x >> 8)  # noqa: E731
    seed64 = src + dst + bs(proto) + bs(np.uint64(8980))
    seed = ((seed64 & 0xFFFFFFFF) + (seed64 >> 32)).astype(np.uint64)
    seed = ((seed & 0xFFFF) + (seed >> 16)).astype(np.uint32)
    off = 9000 * np.arange(n, dtype=np.int64) + 20
    got = u.cksum_spans(d, dev(torch, off), dev(torch, np.full(n, 8980, np.int32)),
                        seed=dev(torch, seed.view(np.int32)), len_hint=8980)
    want = ora.spans(host, off, 8980, seed)
    np.testing.assert_array_equal(host16(got), want)
    # cross-check the seed convention against the per-packet pseudo-header walk
    ch = MbufChains.contiguous(host, 9000 * np.arange(256, dtype=np.int64), 9000)
    np.testing.assert_array_equal(
        ora.pseudo_header_batch(ch.heads, 8980, 20, src[:256], dst[:256], proto[:256]), want[:256])
    np.testing.assert_array_equal(
        u.in_cksum_pseudo_header_batch(ch.heads, 8980, 20, src[:256], dst[:256], proto[:256]),
        want[:256])


@pytest.mark.parametrize("host_threads", [1, 3, 8])
def test_host_batch_chunked(torch_dev, ora, host_threads):
    """Batches large enough to be walked/packed in chunks by the host pool
    (staging and zero-copy), with concurrent callers contending for it."""
    rng = np.random.default_rng(90 + host_threads)
    arena = rand_arena(1 << 22, 90)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 24000, arena.size)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = rng.integers(0, 40, ch.n).astype(np.int32)
    want = ora.skip_batch(ch.heads, tot, skip)
    u.set_tuning("host_threads", host_threads)
    try:
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, tot, skip), want)
        u.register_host(arena)
        try:
            np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, tot, skip), want)
            results, errors = {}, []

            def worker(k):
                try:
                    sl = slice(k * 6000, (k + 1) * 6000)
                    for _ in range(3):
                        results[k] = u.in_cksum_skip_batch(ch.heads[sl], tot[sl], skip[sl])
                except Exception as e:  # pragma: no cover
                    errors.append(e)

            th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            assert not errors
            np.testing.assert_array_equal(np.concatenate([results[k] for k in range(4)]), want)
        finally:
            u.unregister_host(arena)
    finally:
        u.set_tuning("host_threads", 16)


def test_host_walk_prefetch(torch_dev, ora):
    """The host walk with its header prefetch gives the oracle's sums: chains longer
    than the bytes wanted (the prefetch must stop where the walk stops), short
    chains, len <= skip, and pseudo-header batches, staged and zero-copy."""
    rng = np.random.default_rng(301)
    arena = rand_arena(1 << 22, 300)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 20000, arena.size, max_segs=12)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1]).astype(np.int64)
    length = (tot * rng.uniform(0.2, 1.2, ch.n)).astype(np.int32)  # some past the chain end
    skip = rng.integers(0, 60, ch.n).astype(np.int32)
    want = ora.skip_batch(ch.heads, length, skip)
    first = seg_len[pkt_seg[:-1]].astype(np.int32)
    off0 = np.minimum(first, 20).astype(np.int32)
    plen = np.maximum(length - off0, 0).astype(np.int32)
    src = rng.integers(0, 2**32, ch.n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, ch.n, dtype=np.uint64).astype(np.uint32)
    proto = np.where(rng.random(ch.n) < 0.5, 6, 17).astype(np.uint8)
    want_ph = ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
    for registered in (False, True):
        if registered:
            u.register_host(arena)
        try:
            np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, length, skip), want)
            np.testing.assert_array_equal(
                u.in_cksum_pseudo_header_batch(ch.heads, plen, off0, src, dst, proto), want_ph)
        finally:
            if registered:
                u.unregister_host(arena)


@pytest.mark.parametrize("host_threads", [2, 16])
def test_zero_copy_pipeline_ring(torch_dev, ora, host_threads):
    """Zero-copy batches are walked and launched group by group through a
    descriptor ring in pinned memory: on a fresh thread (1 MiB ring) 40 K
    chains of ~8 pieces wrap the ring (2 threads: 300-KB groups) or grow it
    (16 threads: 2-MB groups).  An odd-address header in the LAST group sends
    a batch whose earlier groups are already launched down the staging path."""
    rng = np.random.default_rng(300 + host_threads)
    arena = rand_arena(1 << 22, 301)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 40000, arena.size, max_segs=16)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    want = ora.skip_batch(ch.heads, tot, 0)
    hoff = rng.integers(0, arena.size - 64, 40000) & ~1
    hoff[-1] |= 1
    ips = arena.ctypes.data + hoff.astype(np.uint64)
    want_hdr = ora.hdr_batch(ips)
    got, errors = {}, []

    def fresh_thread():
        try:
            for k in range(2):
                got[("skip", k)] = u.in_cksum_skip_batch(ch.heads, tot, 0)
                got[("hdr", k)] = u.in_cksum_hdr_batch(ips)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    u.set_tuning("host_threads", host_threads)
    u.register_host(arena)
    try:
        t = threading.Thread(target=fresh_thread)
        t.start()
        t.join()
    finally:
        u.unregister_host(arena)
        u.set_tuning("host_threads", 16)
    assert not errors
    for k in range(2):
        np.testing.assert_array_equal(got[("skip", k)], want)
        np.testing.assert_array_equal(got[("hdr", k)], want_hdr)


@pytest.mark.parametrize("long_ch,n", [(0, 1 << 17), (16, 3000), (16, 1 << 17), (64, 3000),
                                       (200, 3000)])
def test_chains_long_segments(torch_dev, ora, long_ch, n):
    """Chains mixing short and long (wave-streamed) segments, with len/skip
    clipping that cuts into long segments, over both tile sizes of the
    chunk-stream kernel (8 packets below 128 K packets, 32 from there)."""
    torch = torch_dev
    rng = np.random.default_rng(5100 + long_ch + n % 97)
    arena = rand_arena(1 << 23, 51)
    nseg = rng.integers(1, 7, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = np.where(rng.random(s) < 0.5, rng.integers(0, 200, s), rng.integers(200, 9000, s))
    seg_off = rng.integers(0, arena.size - 9100, s).astype(np.int64)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = np.where(rng.random(n) < 0.5, 20, (rng.random(n) * tot * 0.6).astype(np.int64))
    length = np.where(rng.random(n) < 0.7, tot, skip + (rng.random(n) * (tot - skip + 1)).astype(np.int64))
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed)
    u.set_tuning("chains_long", long_ch)
    try:
        for flags in (0, u.F_UDP):
            w = want if flags == 0 else ora.chains(arena, seg_off, seg_len, pkt_seg, length=length,
                                                   skip=skip, seed=seed, flags=flags)
            got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off),
                                 dev(torch, seg_len.astype(np.int32)),
                                 dev(torch, pkt_seg.astype(np.int32)),
                                 length=dev(torch, length.astype(np.int32)),
                                 skip=dev(torch, skip.astype(np.int32)),
                                 seed=dev(torch, seed.view(np.int32)), flags=flags)
            np.testing.assert_array_equal(host16(got), w)
    finally:
        u.set_tuning("chains_long", 128)


@pytest.mark.parametrize("long_ch", [0, 200])
def test_chains_full_rounds(torch_dev, ora, long_ch):
    """Descriptor rounds whose chunk list is longer than 4096 chunks: 64
    segments of 1900-2031 B each (up to 127 chunks), mixed with rounds of tiny
    and empty segments; 128 K packets, so the 32-packet tile (full 64-segment
    rounds) runs."""
    torch = torch_dev
    rng = np.random.default_rng(6100 + long_ch)
    arena = rand_arena(1 << 24, 61)
    n = 1 << 17
    nseg = rng.integers(1, 9, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    big = (np.arange(s) // 256) % 2 == 0
    seg_len = np.where(big, rng.integers(1900, 2032, s), rng.integers(0, 40, s))
    seg_off = rng.integers(0, arena.size - 2100, s).astype(np.int64)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = np.where(rng.random(n) < 0.5, 20, (rng.random(n) * tot * 0.5).astype(np.int64))
    length = np.where(rng.random(n) < 0.7, tot, skip + (rng.random(n) * (tot - skip + 1)).astype(np.int64))
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip)
    u.set_tuning("chains_long", long_ch)
    try:
        got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off),
                             dev(torch, seg_len.astype(np.int32)),
                             dev(torch, pkt_seg.astype(np.int32)),
                             length=dev(torch, length.astype(np.int32)),
                             skip=dev(torch, skip.astype(np.int32)), len_hint=1000)
        np.testing.assert_array_equal(host16(got), want)
    finally:
        u.set_tuning("chains_long", 128)


def test_chains_kernel_variants(torch_dev, ora):
    """The chain kernel on chains of 0..150 segments with len/skip/seed and
    the UDP flag."""
    torch = torch_dev
    rng = np.random.default_rng(8802)
    arena = rand_arena(1 << 21, 47)
    n = 1500
    nseg = rng.integers(0, 151, n)
    nseg[rng.random(n) < 0.1] = 0
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = np.where(rng.random(s) < 0.2, rng.integers(0, 4, s), rng.integers(1, 300, s))
    seg_off = rng.integers(0, arena.size - 400, s).astype(np.int64)
    tot = np.zeros(n, np.int64)
    nz = nseg > 0
    tot[nz] = np.add.reduceat(seg_len, pkt_seg[:-1][nz])
    skip = (rng.random(n) * (tot + 1) * 0.3).astype(np.int64)
    length = skip + (rng.random(n) * (tot - skip + 10)).astype(np.int64)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for flags in (0, u.F_UDP):
        want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip,
                          seed=seed, flags=flags)
        got = u.cksum_chains(dev(torch, arena), dev(torch, seg_off),
                             dev(torch, seg_len.astype(np.int32)),
                             dev(torch, pkt_seg.astype(np.int32)),
                             length=dev(torch, length.astype(np.int32)),
                             skip=dev(torch, skip.astype(np.int32)),
                             seed=dev(torch, seed.view(np.int32)), flags=flags, len_hint=120)
        np.testing.assert_array_equal(host16(got), want)


def test_chains_beyond_4gib_window(torch_dev, ora):
    """A 4.5 GiB arena: even tiles keep their segments within 1 MiB of a tile
    base anywhere in the arena (one 4 GiB window: 32-bit buffer offsets),
    odd tiles scatter them over the whole arena (descriptor rounds that take
    the 64-bit address path)."""
    torch = torch_dev
    size = (9 << 29) + 4096
    d = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda")
    host = d.cpu().numpy()
    rng = np.random.default_rng(4242)
    n = 4096
    nseg = rng.integers(1, 20, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(0, 300, s)
    # every 40th segment is long (2-9 KB: the wave-streamed path), at offsets
    # on both sides of 2 GiB and 4 GiB (64-bit bases whose low word has bit 31)
    seg_len[::40] = rng.integers(2048, 9000, seg_len[::40].size)
    pkt = np.repeat(np.arange(n), nseg)
    tile_base = rng.integers(0, size - (2 << 20) - 9100, n // 32 + 1)
    local = tile_base[pkt // 32] + rng.integers(0, 1 << 20, s)
    scattered = rng.integers(0, size - 9100, s)
    seg_off = np.where((pkt // 32) % 2 == 0, local, scattered).astype(np.int64)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    skip = np.full(n, 3, np.int64)
    want = ora.chains(host, seg_off, seg_len, pkt_seg, skip=skip, seed=seed)
    got = u.cksum_chains(d, dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)),
                         dev(torch, pkt_seg.astype(np.int32)),
                         skip=dev(torch, skip.astype(np.int32)),
                         seed=dev(torch, seed.view(np.int32)), len_hint=150)
    np.testing.assert_array_equal(host16(got), want)
    # the wave-per-packet kernel over the same chains (mean segment >= 2 KiB picks it)
    got = u.cksum_chains(d, dev(torch, seg_off), dev(torch, seg_len.astype(np.int32)),
                         dev(torch, pkt_seg.astype(np.int32)), skip=dev(torch, skip.astype(np.int32)),
                         seed=dev(torch, seed.view(np.int32)), len_hint=4096)
    assert "k_chains_wide" in u.last_kernel()
    np.testing.assert_array_equal(host16(got), want)
    # spans and strided packets past the 4 GiB mark (64-bit offsets)
    off = rng.integers((1 << 32) - 4096, size - 10000, 3000).astype(np.int64)
    ln = rng.integers(0, 9000, 3000)
    for hint in (64, 4000):
        got = u.cksum_spans(d, dev(torch, off), dev(torch, ln.astype(np.int32)), len_hint=hint)
        np.testing.assert_array_equal(host16(got), ora.spans(host, off, ln))
    got = u.cksum_strided(d[(1 << 32) - 7:], 1514, 1500, 2000)
    np.testing.assert_array_equal(
        host16(got), ora.spans(host, (1 << 32) - 7 + 1514 * np.arange(2000), 1500))
    del d
    torch.cuda.empty_cache()


def test_host_batch_stream_copy(torch_dev, ora):
    """A staged host batch large enough (>= 32 MiB of packet bytes) to be
    packed and shipped to HBM in overlapped groups; chained and odd-offset
    packets included, so every group boundary lands mid-layout."""
    rng = np.random.default_rng(77)
    n = 64000  # ~45 MB of summed bytes
    arena = rand_arena(1500 * n + 8192, 77)
    lens = rng.choice([64, 576, 1500], n)
    off = (np.arange(n) * 1500 + rng.integers(0, 7, n)).astype(np.int64)
    ch = MbufChains.contiguous(arena, off, lens)
    skip = rng.integers(0, 30, n).astype(np.int32)
    want = ora.skip_batch(ch.heads, lens, skip)
    np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, lens, skip), want)
    # chained: every packet re-cut into 1..256-B segments
    seg_off, seg_len, pkt_seg = [], [], [0]
    for i in range(n):
        cuts = np.cumsum(rng.integers(1, 257, 12))
        cuts = np.concatenate([[0], cuts[cuts < lens[i]], [lens[i]]])
        seg_off.extend(off[i] + cuts[:-1])
        seg_len.extend(np.diff(cuts))
        pkt_seg.append(len(seg_off))
    cc = MbufChains(arena, np.array(seg_off), np.array(seg_len), np.array(pkt_seg))
    np.testing.assert_array_equal(u.in_cksum_skip_batch(cc.heads, lens, skip), want)


def test_device_api_on_side_streams(torch_dev, ora):
    """The device-resident entry points enqueue on the caller's stream: four
    side streams with a span, a strided, a chain and a seeded span batch in
    flight together, then four host threads each looping on its own stream."""
    torch = torch_dev
    rng = np.random.default_rng(606)
    arena = rand_arena(1 << 22, 66)
    d = dev(torch, arena)
    n = 20000
    off = rng.integers(0, arena.size - 3000, n)
    ln = rng.integers(0, 2000, n)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 3000, arena.size)
    want = [ora.spans(arena, off, ln), ora.spans(arena, 1514 * np.arange(2000) + 14, 1500),
            ora.chains(arena, seg_off, seg_len, pkt_seg), ora.spans(arena, off, ln, seed)]
    t_off, t_ln, t_seed = dev(torch, off), dev(torch, ln.astype(np.int32)), dev(torch, seed.view(np.int32))
    t_so, t_sl = dev(torch, seg_off), dev(torch, seg_len.astype(np.int32))
    t_ps = dev(torch, pkt_seg.astype(np.int32))
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = [torch.empty(w.size, dtype=torch.uint16, device="cuda") for w in want]
    torch.cuda.synchronize()
    for _ in range(3):
        u.cksum_spans(d, t_off, t_ln, out=outs[0], stream=streams[0])
        u.cksum_strided(d[14:], 1514, 1500, 2000, out=outs[1], stream=streams[1])
        u.cksum_chains(d, t_so, t_sl, t_ps, out=outs[2], stream=streams[2])
        u.cksum_spans(d, t_off, t_ln, seed=t_seed, out=outs[3], stream=streams[3])
    torch.cuda.synchronize()
    for o, w in zip(outs, want):
        np.testing.assert_array_equal(host16(o), w)

    errors, got = [], {}

    def worker(k):
        try:
            s = torch.cuda.Stream()
            o = torch.empty(n, dtype=torch.uint16, device="cuda")
            for _ in range(5):
                u.cksum_spans(d, t_off, t_ln, seed=t_seed if k % 2 else None, out=o, stream=s)
            s.synchronize()
            got[k] = host16(o)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    for k in range(4):
        np.testing.assert_array_equal(got[k], want[3] if k % 2 else want[0])
