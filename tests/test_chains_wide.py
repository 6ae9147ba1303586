"""k_chains_wide (cksum_chains.hip): one wave per packet, for chains of few
long segments (config 5tso's 40-B header mbuf + 9 KB payload slice).  Every
shape the tile kernel's tests use -- empty chains, zero-length and 1-byte
segments, hundreds of segments per chain, len / skip cutting inside and on
segment boundaries, len <= skip, segments longer than one 9 KiB load round,
seeds, UDP and no-complement flags, wide and packed descriptors -- bit-exact
against the oracle with the kernel forced (knob chains_wide = 2) and picked by
the mean segment length (len_hint 4096-9216)."""
from __future__ import annotations

import zlib

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import dev, host16, rand_arena

pytestmark = pytest.mark.gpu


@pytest.fixture
def wide(torch_dev):
    u.set_tuning("chains_wide", 2)
    try:
        yield torch_dev
    finally:
        u.set_tuning("chains_wide", 0)


def _layout(rng, n, arena_size, max_segs, lens):
    nseg = rng.integers(0, max_segs + 1, n)
    nseg[rng.random(n) < 0.05] = 0
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = lens(s)
    seg_off = rng.integers(0, arena_size - int(seg_len.max(initial=0)) - 32, s).astype(np.int64)
    return seg_off, seg_len.astype(np.int64), pkt_seg


SHAPES = {
    "short": lambda rng, s: np.where(rng.random(s) < 0.2, rng.integers(0, 3, s), rng.integers(1, 300, s)),
    "long": lambda rng, s: np.where(rng.random(s) < 0.4, rng.integers(0, 200, s), rng.integers(200, 30000, s)),
    "tso": lambda rng, s: np.where(np.arange(s) % 2 == 0, 40, rng.integers(8000, 9300, s)),
}


@pytest.mark.parametrize("shape,max_segs", [("short", 40), ("short", 300), ("long", 6), ("tso", 2)])
@pytest.mark.parametrize("desc", ["wide", "packed"])
def test_chains_wide_matches_oracle(wide, ora, shape, max_segs, desc):
    torch = wide
    rng = np.random.default_rng(zlib.crc32(f"{shape}{max_segs}{desc}".encode()))
    arena = rand_arena(1 << 23, 61)
    n = 2000
    seg_off, seg_len, pkt_seg = _layout(rng, n, arena.size, max_segs,
                                        lambda s: SHAPES[shape](rng, s))
    if desc == "packed":
        seg_len = np.minimum(seg_len, 65535)
    tot = np.zeros(n, np.int64)
    nz = np.diff(pkt_seg) > 0
    tot[nz] = np.add.reduceat(seg_len, pkt_seg[:-1][nz])
    cum = np.concatenate([[0], np.cumsum(seg_len)])
    skip = np.where(rng.random(n) < 0.5, np.minimum(20, tot), (rng.random(n) * (tot + 1) * 0.5).astype(np.int64))
    first_end = np.where(nz, cum[np.minimum(pkt_seg[:-1] + 1, cum.size - 1)] - cum[pkt_seg[:-1]], 0)
    skip = np.where(rng.random(n) < 0.2, first_end, skip)  # skip on the first boundary
    length = np.where(rng.random(n) < 0.6, tot, skip + (rng.random(n) * (tot - skip + 50)).astype(np.int64))
    length = np.where(rng.random(n) < 0.05, np.maximum(skip - rng.integers(0, 3, n), 0), length)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d_arena = dev(torch, arena)
    if desc == "packed":
        so, sl = u.pack_segments(seg_off, seg_len.astype(np.int32))
        d_so, d_sl = dev(torch, so), dev(torch, sl)
    else:
        d_so, d_sl = dev(torch, seg_off), dev(torch, seg_len.astype(np.int32))
    for flags in (0, u.F_UDP, u.F_NO_COMPLEMENT):
        for use_len, use_skip, use_seed in ((True, True, True), (False, False, False)):
            want = ora.chains(arena, seg_off, seg_len, pkt_seg,
                              length=length if use_len else None, skip=skip if use_skip else None,
                              seed=seed if use_seed else None, flags=flags)
            got = u.cksum_chains(d_arena, d_so, d_sl, dev(torch, pkt_seg.astype(np.int32)),
                                 length=dev(torch, length.astype(np.int32)) if use_len else None,
                                 skip=dev(torch, skip.astype(np.int32)) if use_skip else None,
                                 seed=dev(torch, seed.view(np.int32)) if use_seed else None,
                                 flags=flags)
            assert "k_chains_wide" in u.last_kernel()
            np.testing.assert_array_equal(host16(got), want)


def test_chains_wide_picked_by_hint(torch_dev, ora):
    """Auto (chains_wide 0): a mean segment of 4-9 KiB takes the
    wave-per-packet kernel, shorter and longer ones the tile kernel; both
    equal the oracle on the same TSO-shaped batch."""
    torch = torch_dev
    from libuinet_amd.workloads import chain_layout, materialize_device

    w = materialize_device(chain_layout("5tso", 40))
    lay = w["layout"]
    want = ora.chains(w["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=lay["skip"], seed=lay["seed"])
    for hint, kern in ((w["mean_seg"], "k_chains_wide"), (300, "k_chains_pipe"),
                       (16384, "k_chains_pipe")):
        got = u.cksum_chains(w["arena"], w["seg_off"], w["seg_len"], w["pkt_seg"], length=w["len"],
                             skip=w["skip"], seed=w["seed"], len_hint=int(hint))
        assert kern in u.last_kernel(), (hint, u.last_kernel())
        np.testing.assert_array_equal(host16(got), want)


def test_chains_wide_packed_lengths_off_word(wide, ora):
    """Packed u16 lengths whose array starts 2 B past a 4-B boundary: the
    kernel reads each length out of its aligned 32-bit word (seg_len_at), so
    both halves of a word and the array's first and last entries are checked
    against the oracle."""
    torch = wide
    rng = np.random.default_rng(77)
    arena = rand_arena(1 << 22, 62)
    n = 1500
    seg_off, seg_len, pkt_seg = _layout(rng, n, arena.size, 3,
                                        lambda s: rng.integers(0, 9300, s))
    so, sl = u.pack_segments(seg_off, seg_len.astype(np.int32))
    big = torch.zeros(sl.size + 1, dtype=torch.int16, device="cuda")
    big[1:] = dev(torch, sl).to(torch.int16)
    d_sl = big[1:]  # storage offset 1: the array starts 2 B into a word
    assert d_sl.data_ptr() % 4 == 2
    want = ora.chains(arena, seg_off, seg_len, pkt_seg)
    got = u.cksum_chains(dev(torch, arena), dev(torch, so), d_sl, dev(torch, pkt_seg.astype(np.int32)))
    assert "k_chains_wide" in u.last_kernel()
    np.testing.assert_array_equal(host16(got), want)
