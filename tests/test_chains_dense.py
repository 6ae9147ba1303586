"""Chain batches whose segments are carved densely out of the arena -- in
order, shuffled inside a round, overlapping, scattered blocks between them,
1-byte and empty segments, len/skip clipping, long segments inside a dense
run, rounds whose chunk list runs 1,023 chunks, segments ending on the
arena's last byte, all-0x00 / all-0xff bytes -- through the chain kernel at
both tile sizes, both batch widths and both descriptor widths, against the
oracle's in_cksum_skip walk (/root/reference/sys/amd64/amd64/in_cksum.c
:203-229).  (Round 4 measured an address-sweep formulation on these layouts
and removed it, profiles/r04/pruned/; the layouts stay as parity cases.)"""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import aligned_empty

from test_gpu_parity import dev, host16, pad_for_tile, rand_arena, torch_dev  # noqa: F401

pytestmark = pytest.mark.gpu


def dense_layout(rng, n, arena_size, shape, max_seg=256, max_segs=12):
    """Chains whose segments are carved one after another out of the arena
    (gaps of 0-7 B).  shape: "in" (placement = chain order), "shuffled"
    (placement permuted inside blocks of 48 segments), "overlap" (each
    segment starts up to 40 B before the previous one ends), "mixed" (every
    third block of chains scattered over the whole arena)."""
    nseg = rng.integers(0, max_segs + 1, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    r = rng.random(s)
    seg_len = rng.integers(1, max_seg + 1, s)
    seg_len = np.where(r < 0.06, 0, seg_len)
    seg_len = np.where((r >= 0.06) & (r < 0.12), rng.integers(1, 4, s), seg_len)
    gaps = rng.integers(0, 8, s)
    order = np.arange(s)
    if shape == "shuffled":
        for b in range(0, s, 48):
            order[b:b + 48] = b + rng.permutation(min(48, s - b))
    step = seg_len[order] + gaps
    if shape == "overlap":
        step = np.maximum(seg_len[order] - rng.integers(0, 41, s), 0)
    start = 64 + np.cumsum(step) - step  # placement k at start[k]
    seg_off = np.empty(s, np.int64)
    seg_off[order] = start
    if shape == "mixed":
        blk = (np.arange(s) // 150) % 3 == 2
        seg_off[blk] = rng.integers(0, arena_size - max_seg - 1, int(blk.sum()))
    assert seg_off.max(initial=0) + max_seg < arena_size
    return seg_off, seg_len.astype(np.int64), pkt_seg


def clip_args(rng, seg_len, pkt_seg):
    n = pkt_seg.size - 1
    tot = np.zeros(n, np.int64)
    nz = np.diff(pkt_seg) > 0
    tot[nz] = np.add.reduceat(seg_len, pkt_seg[:-1][nz])
    skip = np.where(rng.random(n) < 0.5, np.minimum(20, tot),
                    (rng.random(n) * (tot + 1) * 0.5).astype(np.int64))
    length = np.where(rng.random(n) < 0.6, tot,
                      skip + (rng.random(n) * (tot - skip + 30)).astype(np.int64))
    length = np.where(rng.random(n) < 0.05, np.maximum(skip - 1, 0), length)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    return length, skip, seed


def run_chains(torch, arena, seg_off, seg_len, pkt_seg, length, skip, seed, packed, flags=0):
    if packed:
        so, sl = u.pack_segments(seg_off, seg_len)
        so, sl = dev(torch, so), dev(torch, sl)
    else:
        so, sl = dev(torch, seg_off), dev(torch, seg_len.astype(np.int32))
    return host16(u.cksum_chains(dev(torch, arena), so, sl, dev(torch, pkt_seg.astype(np.int32)),
                                 length=dev(torch, length.astype(np.int32)),
                                 skip=dev(torch, skip.astype(np.int32)),
                                 seed=dev(torch, seed.view(np.int32)), flags=flags, len_hint=110))


def with_knobs(knobs, fn):
    dflt = {"chains_long": 128}
    for k, v in knobs.items():
        u.set_tuning(k, v)
    try:
        return fn()
    finally:
        for k in knobs:
            u.set_tuning(k, dflt[k])


@pytest.mark.parametrize("shape", ["in", "shuffled", "overlap", "mixed"])
def test_dense_layouts(torch_dev, ora, shape):
    torch = torch_dev
    rng = np.random.default_rng(12000 + len(shape))
    arena = rand_arena(1 << 23, 120)
    seg_off, seg_len, pkt_seg = dense_layout(rng, 6000, arena.size, shape)
    length, skip, seed = clip_args(rng, seg_len, pkt_seg)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed)
    for packed in (False, True):
        got = run_chains(torch, arena, seg_off, seg_len, pkt_seg, length, skip, seed, packed)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("tile,long_ch", [(8, 128), (32, 128), (32, 16), (8, 0)])
def test_dense_geometries(torch_dev, ora, tile, long_ch):
    """Dense rounds at both tile sizes (tile 32: padded with empty chains to
    128 K packets), with long segments (streamed wave-wide) inside the dense
    run."""
    torch = torch_dev
    rng = np.random.default_rng(13000 + tile + 2 + long_ch)
    arena = rand_arena(1 << 23, 130)
    seg_off, seg_len, pkt_seg = dense_layout(rng, 3000, arena.size, "in", max_seg=600)
    length, skip, seed = clip_args(rng, seg_len, pkt_seg)
    pkt_seg, length, skip, seed = pad_for_tile(tile, pkt_seg, length, skip, seed)
    for flags in (0, u.F_UDP):
        want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed,
                          flags=flags)
        got = with_knobs({"chains_long": long_ch},
                         lambda: run_chains(torch, arena, seg_off, seg_len, pkt_seg, length, skip,
                                            seed, False, flags))
        np.testing.assert_array_equal(got, want)


def test_dense_extremes(torch_dev, ora):
    """All-0x00 and all-0xff bytes (0 vs 0xffff after the fold), rounds of 64
    one-byte segments, segments ending on the arena's last byte, and rounds
    whose list runs 1023 chunks (the longest the chunk list takes)."""
    torch = torch_dev
    rng = np.random.default_rng(14000)
    for fill in (0x00, 0xFF):
        arena = aligned_empty(1 << 22)
        arena[:] = fill
        seg_off, seg_len, pkt_seg = dense_layout(rng, 2000, arena.size, "in")
        length, skip, seed = clip_args(rng, seg_len, pkt_seg)
        seed[:] = 0
        want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed)
        got = run_chains(torch, arena, seg_off, seg_len, pkt_seg, length, skip, seed, False)
        np.testing.assert_array_equal(got, want)
    arena = rand_arena(1 << 24, 140)
    n = 400
    nseg = np.full(n, 64)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = np.ones(s, np.int64)
    seg_len[s // 2:] = rng.integers(16300, 16368, s - s // 2) // 64  # ~255-B pieces
    seg_len[-128:] = 16360  # ~1023 chunks each: the list's limit; one dense 1-MB round
    seg_off = np.cumsum(seg_len) - seg_len + rng.integers(0, 16)
    seg_off[-1] = arena.size - seg_len[-1]  # the last segment ends on the last byte
    seg_off[-2] = seg_off[-1] - seg_len[-2]  # (the last round: scattered, the chunk list)
    length, skip, seed = clip_args(rng, seg_len, pkt_seg)
    for tile in (8, 32):
        ps, ln, sk, sd = pad_for_tile(tile, pkt_seg, length, skip, seed)
        want = ora.chains(arena, seg_off, seg_len, ps, length=ln, skip=sk, seed=sd)
        got = with_knobs({"chains_long": 0},
                         lambda: run_chains(torch, arena, seg_off, seg_len, ps, ln, sk, sd, False))
        np.testing.assert_array_equal(got, want)


def test_config3_slice(torch_dev, ora):
    """Config 3's own layout (m_fragment chains, in order, 0-7-B gaps) at
    65,536 packets, wide and packed descriptors."""
    torch = torch_dev
    from libuinet_amd.workloads import config3_device

    c = config3_device(1 << 16, seed=21)
    lay = c["layout"]
    want = ora.chains(c["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=np.full(c["n"], 20, np.int64))
    packed = u.pack_segments(c["seg_off"], c["seg_len"])

    fl = 0
    a = host16(u.cksum_chains(c["arena"], c["seg_off"], c["seg_len"], c["pkt_seg"],
                              length=c["len"], skip=c["skip"], flags=fl, len_hint=c["mean_seg"]))
    b = host16(u.cksum_chains(c["arena"], packed[0], packed[1], c["pkt_seg"],
                              length=c["len"], skip=c["skip"], flags=fl, len_hint=c["mean_seg"]))
    np.testing.assert_array_equal(a, want)
    np.testing.assert_array_equal(b, want)
