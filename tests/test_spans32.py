"""Packed span descriptors (uinet_cksum_spans32: u32 offset, u16 length per
packet) against the oracle's span fold (oracle/cksum_oracle.c, after
/root/reference/sys/amd64/amd64/in_cksum.c:91-170,193-232 and the
in_cksum_pseudo_header seed of :241-276), and against the wide-descriptor
path (uinet_cksum_spans) on the same spans.  Every span kernel family and
geometry the wide API dispatches to runs here with packed descriptors.

The ABI export is checked on CPU by tests/test_abi.py; everything here is
`-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import HINTS, dev, host16, rand_arena, rand_spans

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert u.device_ok(), "device is not gfx950"
    return torch


def packed(torch, off, ln):
    o32, l16 = u.pack_segments(off, ln)
    return dev(torch, o32), dev(torch, l16)


@pytest.mark.parametrize("pipe", [1])
@pytest.mark.parametrize("n", [1, 2, 7, 6000, 70001])
def test_spans32_every_kernel(torch_dev, ora, pipe, n):
    """Every geometry (len_hint) under both kernel families, seeds, parity,
    UDP; odd and even packet counts (a u16 length is read from the dword that
    holds it)."""
    torch = torch_dev
    rng = np.random.default_rng(8100 + 3 * n + pipe)
    arena = rand_arena(1 << 21, 81)
    off, ln = rand_spans(rng, n, arena.size, 3000)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    par = rng.integers(0, 2, n).astype(np.uint8)
    d_arena = dev(torch, arena)
    d_off, d_ln = packed(torch, off, ln)
    d_seed, d_par = dev(torch, seed.view(np.int32)), dev(torch, par)
    for hint in HINTS:
        want = ora.spans(arena, off, ln, seed, par, u.F_UDP)
        got = u.cksum_spans(d_arena, d_off, d_ln, seed=d_seed, parity=d_par, flags=u.F_UDP,
                            len_hint=hint)
        np.testing.assert_array_equal(host16(got), want)
        got = u.cksum_spans(d_arena, d_off, d_ln, len_hint=hint)
        np.testing.assert_array_equal(host16(got), ora.spans(arena, off, ln))


@pytest.mark.parametrize("bpc", [0, 1, 3])
def test_spans32_small_packets_and_grids(torch_dev, ora, bpc):
    """k_spans_quad (4 lanes per packet) and k_spans_lean on grids small
    enough that every wave walks many steps: ragged counts, empty spans,
    spans longer than the geometry's round, the u16 maximum of 65535 B."""
    torch = torch_dev
    rng = np.random.default_rng(8200 + bpc)
    arena = rand_arena(24 << 20, 82)
    d_arena = dev(torch, arena)
    u.set_tuning("blocks_per_cu", bpc)
    try:
        for hint, max_len in ((64, 80), (64, 64), (1500, 1600), (9000, 9100)):
            for n in (1, 63, 64, 65, 1000, 70001):
                off, ln = rand_spans(rng, n, arena.size - 70000, max_len)
                ln[rng.random(n) < 0.01] = 0xffff
                ln[rng.random(n) < 0.01] = 5000
                seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                par = rng.integers(0, 2, n).astype(np.uint8)
                d_off, d_ln = packed(torch, off, ln)
                got = u.cksum_spans(d_arena, d_off, d_ln, seed=dev(torch, seed.view(np.int32)),
                                    parity=dev(torch, par), flags=u.F_UDP, len_hint=hint)
                want = ora.spans(arena, off, ln, seed, par, u.F_UDP)
                np.testing.assert_array_equal(host16(got), want)
    finally:
        u.set_tuning("blocks_per_cu", 0)


def test_spans32_offsets_above_2gib(torch_dev, ora):
    """Offsets in [2^31, 2^32): the packed offset is unsigned.  The spans lie
    in a 1-MiB window placed 3 GiB + 16 into a device arena (16-B aligned, so
    address parity and alignment match the host copy the oracle sums)."""
    torch = torch_dev
    rng = np.random.default_rng(8300)
    win = rand_arena(1 << 20, 83)
    W = (3 << 30) + 16
    big = torch.zeros(W + win.size + 4096, dtype=torch.uint8, device="cuda")
    big[W:W + win.size] = dev(torch, win)
    try:
        n = 5000
        off, ln = rand_spans(rng, n, win.size, 3000)
        d_off, d_ln = packed(torch, off + W, ln)
        assert int(d_off.min()) < 0  # really above 2^31 when read as signed
        for hint in (64, 500, 1500, 9000):
            got = u.cksum_spans(big, d_off, d_ln, len_hint=hint)
            np.testing.assert_array_equal(host16(got), ora.spans(win, off, ln))
    finally:
        del big
        torch.cuda.empty_cache()


@pytest.mark.parametrize("base", [0, 2])
def test_spans32_full_2s(torch_dev, ora, base):
    """The benchmarked small-packet batch at full size (config 2s / 2su:
    16,777,216 x 64 B at stride 64, +0 / +2) with packed descriptors equals
    the oracle and the wide path."""
    import libuinet_amd.workloads as Wl

    n = 1 << 24
    w = Wl.config2_device(n, stride=64, length=64, base=base)
    o32, l16 = u.pack_segments(w["off"], w["len"])
    got = u.cksum_spans(w["arena"], o32, l16, len_hint=64)
    wide = u.cksum_spans(w["arena"], w["off"], w["len"], len_hint=64)
    host = w["arena"].cpu().numpy()
    want = ora.spans(host, base + 64 * np.arange(n, dtype=np.int64), np.full(n, 64, np.int64))
    np.testing.assert_array_equal(host16(got), want)
    np.testing.assert_array_equal(host16(wide), want)


def test_spans32_rejects_bad_args(torch_dev):
    torch = torch_dev
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    o, l16 = packed(torch, np.array([0, 16]), np.array([8, 8]))
    with pytest.raises(ValueError):
        u.cksum_spans(arena, o, l16[:1])
    rc = u.lib().uinet_cksum_spans32(arena.data_ptr(), 0, l16.data_ptr(), None, None,
                                     arena.data_ptr(), 2, 0, 0, None)
    assert rc == -22
    assert u.lib().uinet_cksum_spans32(0, 0, 0, None, None, 0, 0, 0, 0, None) == 0
