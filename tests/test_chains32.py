"""Packed chain descriptors (uinet_cksum_chains32: u32 segment offset, u16
segment length) against the oracle's in_cksum_skip chain walk
(oracle/cksum_oracle.c, after /root/reference/sys/amd64/amd64/in_cksum.c
:193-232), and against the wide-descriptor path on the same chains.

The packing helper's range checks run on CPU; everything else is `-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import HINTS, dev, host16, pad_for_tile, rand_arena, random_chain_layout


def packed_dev(torch, seg_off, seg_len):
    o32, l16 = u.pack_segments(seg_off, seg_len)
    return dev(torch, o32), dev(torch, l16)


# ---- CPU: the packing helper -------------------------------------------------

def test_pack_segments_round_trip():
    off = np.array([0, 1, (1 << 31) - 1, 1 << 31, (1 << 32) - 1], np.int64)
    ln = np.array([0, 1, 0x7fff, 0x8000, 0xffff], np.int64)
    o32, l16 = u.pack_segments(off, ln)
    assert o32.dtype == np.int32 and l16.dtype == np.int16
    np.testing.assert_array_equal(o32.view(np.uint32).astype(np.int64), off)
    np.testing.assert_array_equal(l16.view(np.uint16).astype(np.int64), ln)


@pytest.mark.parametrize("off,ln", [(1 << 32, 1), (-1, 1), (0, 0x10000), (0, -1)])
def test_pack_segments_rejects_out_of_range(off, ln):
    with pytest.raises(ValueError):
        u.pack_segments(np.array([off], np.int64), np.array([ln], np.int64))


def test_pack_segments_torch_matches_numpy():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    off = rng.integers(0, 1 << 32, 1000)
    ln = rng.integers(0, 1 << 16, 1000)
    a32, a16 = u.pack_segments(off, ln)
    t32, t16 = u.pack_segments(torch.from_numpy(off), torch.from_numpy(ln.astype(np.int32)))
    np.testing.assert_array_equal(t32.numpy(), a32)
    np.testing.assert_array_equal(t16.numpy(), a16)
    with pytest.raises(ValueError):
        u.pack_segments(torch.tensor([1 << 32]), torch.tensor([1], dtype=torch.int32))


# ---- GPU parity ----------------------------------------------------------------

@pytest.fixture(scope="module")
def torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert u.device_ok(), "device is not gfx950"
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("hint", HINTS)
def test_chains32_len_skip_seed(torch_dev, ora, hint):
    torch = torch_dev
    rng = np.random.default_rng(9100 + hint)
    arena = rand_arena(1 << 20, 61)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 4000, arena.size)
    n = pkt_seg.size - 1
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = (rng.random(n) * (tot + 1) * 0.5).astype(np.int64)
    length = skip + (rng.random(n) * (tot - skip + 40)).astype(np.int64)
    length = np.where(rng.random(n) < 0.1, np.maximum(skip - 1, 0), length)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed)
    so, sl = packed_dev(torch, seg_off, seg_len)
    got = u.cksum_chains(dev(torch, arena), so, sl, dev(torch, pkt_seg.astype(np.int32)),
                         length=dev(torch, length.astype(np.int32)),
                         skip=dev(torch, skip.astype(np.int32)),
                         seed=dev(torch, seed.view(np.int32)), len_hint=hint)
    np.testing.assert_array_equal(host16(got), want)


@pytest.mark.gpu
@pytest.mark.parametrize("long_ch,tile", [(128, 0), (16, 8), (0, 32), (128, 32)])
def test_chains32_long_and_many_segments(torch_dev, ora, long_ch, tile):
    """Segments up to 65535 B (the u16 limit) mixed with 0..3-B ones, chains of
    up to 200 segments across descriptor rounds, both tile sizes (tile 32: the
    batch padded with empty chains to 128 K packets)."""
    torch = torch_dev
    rng = np.random.default_rng(9200 + 14 + long_ch + tile)
    arena = rand_arena(1 << 23, 62)
    n = 900
    nseg = rng.integers(0, 200, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    r = rng.random(s)
    seg_len = np.where(r < 0.3, rng.integers(0, 4, s), rng.integers(4, 300, s))
    seg_len = np.where(r > 0.995, rng.integers(9000, 0x10000, s), seg_len)
    seg_len[: 2] = 0xffff
    seg_off = rng.integers(0, arena.size - 0x10000, s).astype(np.int64)
    tot = np.zeros(n, np.int64)
    nz = nseg > 0
    tot[nz] = np.add.reduceat(seg_len, pkt_seg[:-1][nz])
    skip = np.where(rng.random(n) < 0.5, 20, (rng.random(n) * tot * 0.4).astype(np.int64))
    length = np.where(rng.random(n) < 0.7, tot, skip + (rng.random(n) * (tot - skip + 1)).astype(np.int64))
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    pkt_seg, length, skip, seed = pad_for_tile(tile, pkt_seg, length, skip, seed)
    d_arena, d_ps = dev(torch, arena), dev(torch, pkt_seg.astype(np.int32))
    d_len, d_skip = dev(torch, length.astype(np.int32)), dev(torch, skip.astype(np.int32))
    d_seed = dev(torch, seed.view(np.int32))
    so, sl = packed_dev(torch, seg_off, seg_len)
    u.set_tuning("chains_long", long_ch)
    try:
        for flags in (0, u.F_UDP):
            want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip,
                              seed=seed, flags=flags)
            got = u.cksum_chains(d_arena, so, sl, d_ps, length=d_len, skip=d_skip, seed=d_seed,
                                 flags=flags, len_hint=200)
            np.testing.assert_array_equal(host16(got), want)
    finally:
        u.set_tuning("chains_long", 128)


@pytest.mark.gpu
def test_chains32_offsets_above_2gib(torch_dev, ora):
    """Offsets in [2^31, 2^32): the packed offset is unsigned.  The chains'
    bytes are a 1-MiB window placed 3 GiB + 16 into a 3.25-GiB device arena
    (16-B aligned, so every address parity and alignment matches the compact
    host copy the oracle sums)."""
    torch = torch_dev
    rng = np.random.default_rng(9300)
    win = rand_arena(1 << 20, 63)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 3000, win.size)
    W = (3 << 30) + 16
    big = torch.zeros(W + win.size + 4096, dtype=torch.uint8, device="cuda")
    big[W:W + win.size] = dev(torch, win)
    want = ora.chains(win, seg_off, seg_len, pkt_seg, skip=np.full(pkt_seg.size - 1, 3))
    so, sl = packed_dev(torch, seg_off + W, seg_len)
    assert int(so.min()) < 0  # really above 2^31 when read as signed
    d_ps = dev(torch, pkt_seg.astype(np.int32))
    d_skip = dev(torch, np.full(pkt_seg.size - 1, 3, np.int32))
    got = u.cksum_chains(big, so, sl, d_ps, skip=d_skip)
    np.testing.assert_array_equal(host16(got), want)
    wide = u.cksum_chains(big, dev(torch, seg_off + W), dev(torch, seg_len.astype(np.int32)), d_ps,
                          skip=d_skip)
    np.testing.assert_array_equal(host16(wide), want)
    del big


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["3", "3tx", "5tso"])
def test_chains32_full_configs(torch_dev, ora, shape):
    """The benchmarked chain batches (configs 3, 3tx, 5tso at full size) with
    packed descriptors give the oracle's sums and the wide path's."""
    from libuinet_amd import workloads as W

    if shape == "3":
        c = W.config3_device(1 << 20, seed=3)
        lay = c["layout"]
        skip, seed = np.full(c["n"], 20, np.int64), None
    else:
        lay = W.chain_layout(shape)
        c = W.materialize_device(lay)
        skip, seed = lay["skip"], lay["seed"]
    so, sl = u.pack_segments(c["seg_off"], c["seg_len"])
    got = u.cksum_chains(c["arena"], so, sl, c["pkt_seg"], length=c["len"], skip=c["skip"],
                         seed=c.get("seed"), len_hint=c["mean_seg"])
    wide = u.cksum_chains(c["arena"], c["seg_off"], c["seg_len"], c["pkt_seg"], length=c["len"],
                          skip=c["skip"], seed=c.get("seed"), len_hint=c["mean_seg"])
    want = ora.chains(c["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=skip, seed=seed)
    np.testing.assert_array_equal(host16(got), want)
    np.testing.assert_array_equal(host16(wide), want)
