"""Config 1: the TX/RX checksum call sequence of a TCP echo flow
(libuinet_amd/echo.py).  CPU: oracle and reference agree on every TX sum and
the receiver verifies to zero.  GPU: the engine's host-mbuf batch API produces
the same TX sums and zero RX verifications, staged and zero-copy."""
from __future__ import annotations

import numpy as np
import pytest

from libuinet_amd.echo import SEG, EchoBatch, in_pseudo_np


@pytest.fixture(scope="module")
def echo():
    return EchoBatch(4096, seed=7)


def test_in_pseudo_np_matches_oracle(ora):
    rng = np.random.default_rng(3)
    a, b, c = (rng.integers(0, 2**32, 1000, dtype=np.uint64).astype(np.uint32) for _ in range(3))
    want = np.array([ora.in_pseudo(int(x), int(y), int(z)) for x, y, z in zip(a, b, c)], np.uint16)
    assert np.array_equal(in_pseudo_np(a, b, c), want)


def test_echo_shape(echo):
    nseg = np.diff(echo.tx.pkt_seg)
    assert set(np.unique(nseg)) == {2, 3}                       # header + 1..2 cluster slices
    assert 0.2 < (nseg == 3).mean() < 0.5
    assert all(len(echo.tx.packet_bytes(i)) == SEG for i in (0, 1, echo.n - 1))


def test_echo_oracle_roundtrip(echo, ora):
    echo.reset_tx()
    th, ip = echo.transmit(ora)
    rx = echo.deliver_fast()
    for i in (0, 17, echo.n - 1):
        assert echo.tx.packet_bytes(i) == bytes(echo.rx_arena[echo.rx_off[i] : echo.rx_off[i] + SEG])
    hs, ps = echo.receive(ora, rx)
    assert not hs.any() and not ps.any()
    assert th.dtype == np.uint16 and ip.dtype == np.uint16
    # corrupt one payload byte: that packet, and only it, fails RX verification
    rx.arena[echo.rx_off[5] + 100] ^= 0x40
    hs2, ps2 = echo.receive(ora, rx)
    assert np.flatnonzero(ps2).tolist() == [5] and not hs2.any()
    rx.arena[echo.rx_off[5] + 100] ^= 0x40


def test_echo_oracle_vs_reference(echo, ora, ref):
    echo.reset_tx()
    th_r, ip_r = echo.transmit(ref)
    rx = echo.deliver_fast()
    hs, ps = echo.receive(ref, rx)
    assert not hs.any() and not ps.any()
    echo.reset_tx()
    th_o, ip_o = echo.transmit(ora)
    assert np.array_equal(th_r, th_o) and np.array_equal(ip_r, ip_o)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [False, True])
def test_echo_gpu(echo, ora, zero_copy):
    _echo_gpu(echo, ora, zero_copy)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [False, True])
def test_echo_gpu_config1_full(ora, zero_copy):
    """Config 1 at its BASELINE size: 65,536 segments (the flow
    tests/perf/echo_replay.py times), every TX sum equal to the oracle's and
    every RX verification zero."""
    _echo_gpu(EchoBatch(65536, seed=11), ora, zero_copy)


def _echo_gpu(echo, ora, zero_copy):
    import torch  # noqa: F401  (one HIP runtime)

    import libuinet_amd as u
    from libuinet_amd.echo import GpuEngine

    g = GpuEngine()
    echo.reset_tx()
    th_o, ip_o = echo.transmit(ora)
    echo.reset_tx()
    if zero_copy:
        u.register_host(echo.arena)
        u.register_host(echo.rx_arena)
    try:
        th, ip = echo.transmit(g)
        assert np.array_equal(th, th_o) and np.array_equal(ip, ip_o)
        rx = echo.deliver_fast()
        hs, ps = echo.receive(g, rx)
        assert not hs.any() and not ps.any()
    finally:
        if zero_copy:
            u.unregister_host(echo.arena)
            u.unregister_host(echo.rx_arena)
