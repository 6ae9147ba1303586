"""Config 3tx (config 3's lengths in the reference TX chain shape) and config
5tso (TSO-style per-segment pseudo-header sums of 1-MiB sends), see
libuinet_amd/workloads.py.  CPU: the layout's chain-descriptor semantics
(oracle_chains with len/skip/seed) equal the reference's own in_cksum_skip /
in_cksum_pseudo_header over the same bytes as host mbufs.  GPU: the chain
kernel equals the oracle, at test size and at the bench size."""
from __future__ import annotations

import numpy as np
import pytest

from libuinet_amd.mbuf import MbufChains
from libuinet_amd.workloads import (config3tx_layout, config5tso_layout, materialize_device,
                                    materialize_host)


@pytest.fixture(scope="module")
def tx3():
    lay = config3tx_layout(6000, seed=9)
    return lay, materialize_host(lay)


@pytest.fixture(scope="module")
def tso5():
    lay = config5tso_layout(sends=6, seed=10)
    return lay, materialize_host(lay)


def test_config3tx_shape(tx3):
    lay, arena = tx3
    nseg = np.diff(lay["pkt_seg"])
    assert set(np.unique(nseg)) <= {2, 3} and (nseg == 3).any()
    assert (lay["seg_len"][lay["pkt_seg"][:-1]] == 40).all()
    tot = np.add.reduceat(lay["seg_len"], lay["pkt_seg"][:-1])
    assert np.array_equal(tot, lay["lens"])
    assert (lay["seg_off"] + lay["seg_len"]).max() <= arena.size - 64


def test_config3tx_oracle_vs_reference(tx3, ora, ref):
    lay, arena = tx3
    got = ora.chains(arena, lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lay["lens"],
                     lay["skip"])
    ch = MbufChains(arena, lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
    assert np.array_equal(got, ref.skip_batch(ch.heads, lay["lens"], 20))
    assert np.array_equal(got, ora.skip_batch(ch.heads, lay["lens"], 20))


def test_config5tso_shape(tso5):
    lay, _ = tso5
    assert lay["per_send"] == 118
    sl = lay["seg_len"][1::2].reshape(lay["sends"], -1)
    assert (sl.sum(1) == 1 << 20).all() and sl[0, -1] == 256


def test_config5tso_oracle_vs_reference(tso5, ora, ref):
    lay, arena = tso5
    got = ora.chains(arena, lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lay["lens"],
                     lay["skip"], lay["seed"])
    ch = MbufChains(arena, lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
    want = ref.pseudo_header_batch(ch.heads, lay["plen"], 20, lay["src"], lay["dst"], 6)
    assert np.array_equal(got, want)


def _gpu_vs_oracle(lay, ora, host=None):
    import libuinet_amd as u

    w = materialize_device(lay)
    out = u.cksum_chains(w["arena"], w["seg_off"], w["seg_len"], w["pkt_seg"], length=w["len"],
                         skip=w["skip"], seed=w["seed"], len_hint=w["mean_seg"])
    got = out.cpu().view(__import__("torch").int16).numpy().view(np.uint16)
    if host is None:
        host = w["arena"].cpu().numpy()
    want = ora.chains(host, lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lay["lens"],
                      lay["skip"], lay["seed"])
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_config3tx_gpu(torch_dev, tx3, ora):
    lay, arena = tx3
    _gpu_vs_oracle(lay, ora, arena)


@pytest.mark.gpu
def test_config5tso_gpu(torch_dev, tso5, ora):
    lay, arena = tso5
    _gpu_vs_oracle(lay, ora, arena)


@pytest.mark.gpu
def test_full_config3tx(torch_dev, ora):
    _gpu_vs_oracle(config3tx_layout(1 << 20), ora)


@pytest.mark.gpu
def test_full_config5tso(torch_dev, ora):
    _gpu_vs_oracle(config5tso_layout(1111), ora)


def test_layout_floor_small_cases():
    """workloads.layout_floor on hand-checked chains: clipping to [skip, len)
    counted from the chain start, shared and straddled lines, empty
    contributions, descriptor bytes."""
    import libuinet_amd.workloads as W

    # packet 0: segments [0, 100) + [130, 330), len 300, skip 20 -> bytes
    # [20, 100) and [130, 330); packet 1: segment [1000, 1040), whole chain
    seg_off = np.array([0, 130, 1000], np.int64)
    seg_len = np.array([100, 200, 40], np.int64)
    pkt_seg = np.array([0, 2, 3], np.int64)
    lens = np.array([300, 40], np.int64)
    skip = np.array([20, 0], np.int64)
    s, e, algo = W.clipped_segments(seg_off, seg_len, pkt_seg, lens, skip)
    assert s.tolist() == [20, 130, 1000] and e.tolist() == [100, 330, 1040]
    assert algo == 80 + 200 + 40
    # 128-B lines: [20, 100) -> 0; [130, 330) -> 1, 2; [1000, 1040) -> 7, 8
    f = W.layout_floor(seg_off, seg_len, pkt_seg, lens, skip, False, 128)
    assert f["arena_bytes"] == 5 * 128
    assert f["descriptor_bytes"] == 12 * 3 + 2 * 12 + 4
    assert f["floor_bytes"] == f["arena_bytes"] + f["descriptor_bytes"]
    # len cutting a chain short: packet 0 stops inside its first segment
    s, e, algo = W.clipped_segments(seg_off, seg_len, pkt_seg, np.array([60, 40]), skip)
    assert s.tolist() == [20, 1000] and e.tolist() == [60, 1040] and algo == 80
    assert W.lines_touched(np.array([0, 64]), np.array([64, 65]), 64) == 2
