"""The single-mbuf span path of the host-mbuf batch API (cksum_api.hip,
span_fast_batch): over registered packet bytes, a batch whose every sum lies
in its packet's first mbuf is folded as spans -- the host reads each head
mbuf, the GPU only the bytes.  Bit-exact against the oracle on the edges of
"lies in the first mbuf" (in_cksum.c:203-229, :254-272), and every batch that
needs a second mbuf, an unregistered byte or a piece over 65,535 B goes to
the general paths with the same results."""
from __future__ import annotations

import contextlib

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains

from test_gpu_parity import rand_arena

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def registered(*bufs):
    for b in bufs:
        u.register_host(b)
    try:
        yield
    finally:
        for b in bufs:
            u.unregister_host(b)


@pytest.fixture(autouse=True, params=[1, 2], ids=["host-heads", "gpu-heads"])
def span_mode(request):
    """Every test under both span forms: the calling thread reads the head
    mbufs (span_fast 1), or -- where the mbufs are registered -- the GPU does
    (span_fast 2, k_span_walk; with only the bytes registered it is form 1)."""
    u.set_tuning("span_fast", request.param)
    yield request.param
    u.set_tuning("span_fast", 1)


def spans(fn):
    """(result, span batches during fn())."""
    before = u.host_cpu()["span_batches"]
    r = fn()
    return r, u.host_cpu()["span_batches"] - before


@pytest.fixture(scope="module")
def arena(torch_dev):
    return rand_arena(8 << 20, 991)


def _one_mbuf(rng, arena, n, max_len=3000):
    off = rng.integers(0, arena.size - max_len - 1, n)
    ln = rng.integers(0, max_len + 1, n)
    return MbufChains.contiguous(arena, off, ln), ln


@pytest.mark.parametrize("mbufs_registered", [False, True])
def test_span_path_skip_batch(ora, arena, mbufs_registered, span_mode):
    """One mbuf per packet at random offsets (odd addresses included), len
    short of / equal to / beyond the mbuf, skip inside / at / past its end,
    len <= skip, empty mbufs; with only the bytes or also the mbufs
    registered (the span path needs only the bytes and runs before the device
    walk; with the mbufs registered far from the bytes its descriptors are
    packed relative to the largest region)."""
    rng = np.random.default_rng(11)
    n = 20000
    ch, ln = _one_mbuf(rng, arena, n)
    length = np.where(rng.random(n) < 0.2, ln + rng.integers(0, 100, n), ln)
    length = np.where(rng.random(n) < 0.2, rng.integers(0, ln + 1), length)
    skip = np.where(rng.random(n) < 0.5, rng.integers(0, 60, n), 0)
    skip = np.where(rng.random(n) < 0.05, ln, skip)           # skip == m_len
    skip = np.where(rng.random(n) < 0.05, ln + 7, skip)       # skip past the only mbuf
    want = ora.skip_batch(ch.heads, length, skip)
    bufs = (arena, ch.mbufs) if mbufs_registered else (arena,)
    w0 = u.host_cpu()["device_walks"]
    with registered(*bufs):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, length, skip))
    assert ns == 1
    # the GPU read the heads exactly when asked to and able to
    gpu_read = u.host_cpu()["device_walks"] - w0
    assert gpu_read == (1 if (span_mode == 2 and mbufs_registered) else 0)
    np.testing.assert_array_equal(got, want)


def test_span_path_chained_packets_whose_sum_fits_the_first_mbuf(ora, arena):
    """Chains of several mbufs whose [skip, len) ends inside the first one
    (a header-only sum over a TX chain) take the span path; one chain whose
    sum reaches its second mbuf sends the whole batch to the general path."""
    rng = np.random.default_rng(12)
    n = 5000
    nseg = rng.integers(1, 5, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(40, 400, s)
    seg_off = rng.integers(0, arena.size - 401, s).astype(np.int64)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    first = seg_len[pkt_seg[:-1]]
    length = rng.integers(20, first + 1)
    skip = np.minimum(rng.integers(0, 20, n), length)
    want = ora.skip_batch(ch.heads, length, skip)
    with registered(arena):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, length, skip))
        assert ns == 1
        np.testing.assert_array_equal(got, want)
        length2 = length.copy()
        length2[n - 3] = first[n - 3] + 5 if nseg[n - 3] > 1 else length2[n - 3]
        k = int(np.flatnonzero(nseg > 1)[-1])
        length2[k] = first[k] + 5
        want2 = ora.skip_batch(ch.heads, length2, skip)
        got2, ns2 = spans(lambda: u.in_cksum_skip_batch(ch.heads, length2, skip))
    assert ns2 == 0
    np.testing.assert_array_equal(got2, want2)


def test_span_path_pseudo_header(ora, arena):
    """in_cksum_pseudo_header_batch over one-mbuf packets (config 5's
    shape): off0 inside the mbuf and at its end; off0 past it (outside the
    reference's contract) sends the batch to the general path."""
    rng = np.random.default_rng(13)
    n = 6000
    ch, ln = _one_mbuf(rng, arena, n, max_len=9000)
    off0 = np.minimum(ln, rng.integers(0, 41, n))
    plen = np.maximum(0, ln - off0 - rng.integers(0, 30, n))
    src, dst = (rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(2))
    proto = rng.choice(np.array([6, 17], np.uint8), n)
    want = ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
    with registered(arena):
        got, ns = spans(lambda: u.in_cksum_pseudo_header_batch(ch.heads, plen, off0, src, dst,
                                                                proto))
        assert ns == 1
        np.testing.assert_array_equal(got, want)


def test_span_path_long_pieces_and_unregistered(ora, arena):
    """A piece over 65,535 B (the packed descriptor's limit) sends the batch
    round again with wide descriptors, still as spans; a byte outside the
    registered regions sends it to the general path.  Same results."""
    rng = np.random.default_rng(14)
    n = 600
    big = rand_arena(1 << 20, 15)
    off = rng.integers(0, arena.size - 70001, n)
    ln = rng.integers(0, 1500, n)
    ln[300] = 70000
    ch = MbufChains.contiguous(arena, off, ln)
    want = ora.skip_batch(ch.heads, ln, 0)
    with registered(arena):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, ln, 0))
    assert ns == 1
    np.testing.assert_array_equal(got, want)
    ch2 = MbufChains.contiguous(big, rng.integers(0, big.size - 1501, n), ln.clip(0, 1500))
    want2 = ora.skip_batch(ch2.heads, 1500, 0)
    with registered(arena):  # `big` not registered
        got2, ns2 = spans(lambda: u.in_cksum_skip_batch(ch2.heads, 1500, 0))
    assert ns2 == 0
    np.testing.assert_array_equal(got2, want2)


def test_span_path_many_groups(ora, arena):
    """A batch of several pipeline groups (64 K packets each), ragged tail,
    the mbufs registered too (the span path still comes first)."""
    rng = np.random.default_rng(16)
    n = 3 * 65536 + 777
    ch, ln = _one_mbuf(rng, arena, n, max_len=1600)
    want = ora.skip_batch(ch.heads, ln, 0)
    with registered(arena, ch.mbufs):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, ln, 0))
    assert ns == 1
    np.testing.assert_array_equal(got, want)


def test_span_path_retries_wide_after_launched_groups(ora, arena):
    """A piece over 65,535 B in the third pipeline group: the first two groups
    were already folded with packed descriptors when the batch goes round
    again with wide ones; every result is the wide round's."""
    rng = np.random.default_rng(17)
    n = 2 * 65536 + 1000
    off = rng.integers(0, arena.size - 70001, n)
    ln = rng.integers(0, 1501, n)
    ln[2 * 65536 + 500] = 70000
    ch = MbufChains.contiguous(arena, off, ln)
    want = ora.skip_batch(ch.heads, ln, 3)
    with registered(arena, ch.mbufs):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, ln, 3))
    assert ns == 1
    np.testing.assert_array_equal(got, want)


def test_span_path_dense_groups_copy_to_hbm(ora):
    """Packets back to back in one registered region (config 2's layout, at
    odd and even starts, empty and short packets among them): each pipeline
    group's byte range goes to HBM by one DMA copy and is folded there
    (host_cpu()["span_dma_bytes"]; groups under 1 MiB are read in place);
    results equal the oracle.  The same
    packets spread out (gaps over 1/16 of the bytes) are read in place."""
    rng = np.random.default_rng(18)
    n = 2 * 65536 + 333
    ln = rng.integers(600, 1501, n)
    ln[rng.random(n) < 0.01] = 0
    ln[rng.random(n) < 0.01] = 1
    off = 3 + np.concatenate([[0], np.cumsum(ln)[:-1]])
    arena = rand_arena(int(off[-1] + ln[-1] + 64), 19)
    ch = MbufChains.contiguous(arena, off, ln)
    skip = rng.integers(0, 3, n)
    want = ora.skip_batch(ch.heads, ln, skip)
    before = u.host_cpu()["span_dma_bytes"]
    with registered(arena, ch.mbufs):
        got, ns = spans(lambda: u.in_cksum_skip_batch(ch.heads, ln, skip))
    moved = u.host_cpu()["span_dma_bytes"] - before
    assert ns == 1
    np.testing.assert_array_equal(got, want)
    # the two full groups (64 K packets each) by DMA; the 333-packet tail
    # (under 1 MiB) in place
    summed = ln - np.minimum(skip, ln)
    assert int(summed[:2 * 65536].sum()) <= moved <= int(summed.sum()) + 3 * 4096
    # spread: every packet followed by a gap of its own length
    off2 = 5 + np.concatenate([[0], np.cumsum(2 * ln)[:-1]])
    arena2 = rand_arena(int(off2[-1] + ln[-1] + 64), 20)
    ch2 = MbufChains.contiguous(arena2, off2, ln)
    want2 = ora.skip_batch(ch2.heads, ln, skip)
    before = u.host_cpu()["span_dma_bytes"]
    with registered(arena2):
        got2, ns2 = spans(lambda: u.in_cksum_skip_batch(ch2.heads, ln, skip))
    assert ns2 == 1 and u.host_cpu()["span_dma_bytes"] == before
    np.testing.assert_array_equal(got2, want2)


def test_span_path_dense_pseudo_header(ora):
    """The pseudo-header form over a dense layout (config 5's jumbo frames
    back to back): DMA copies, seeds, results equal the oracle."""
    rng = np.random.default_rng(21)
    n = 40000
    ln = np.full(n, 9000)
    off = np.arange(n, dtype=np.int64) * 9000
    arena = rand_arena(int(off[-1] + 9000 + 64), 22)
    ch = MbufChains.contiguous(arena, off, ln)
    off0 = np.full(n, 20)
    plen = ln - 20
    src, dst = (rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(2))
    proto = rng.choice(np.array([6, 17], np.uint8), n)
    want = ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
    before = u.host_cpu()["span_dma_bytes"]
    with registered(arena):
        got, ns = spans(lambda: u.in_cksum_pseudo_header_batch(ch.heads, plen, off0, src, dst,
                                                                proto))
    assert ns == 1 and u.host_cpu()["span_dma_bytes"] > before
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("first", ["a", "b"])
def test_span_path_two_regions_interleaved(ora, arena, first):
    """Packets from two registered regions, in runs and then alternating at
    random: the common-packet run (span_run) holds one region's bounds, so a
    packet from the other leaves it for the general code (above the group's
    origin: offsets from it across regions; below: the group's offsets move
    to the batch's base) and the next one re-enters it.  Either region first.
    Edge packets (empty sums, skip at and past the mbuf's end) among them."""
    rng = np.random.default_rng(23 if first == "a" else 24)
    other = rand_arena(4 << 20, 25)
    n = 30000
    src = np.zeros(n, bool)
    src[1000:2000] = True
    src[2000:] = rng.random(n - 2000) < 0.3
    if first == "b":
        src = ~src
    ln = rng.integers(0, 1501, n)
    offs = np.where(src, rng.integers(0, other.size - 1502, n), rng.integers(0, arena.size - 1502, n))
    ch_a = MbufChains.contiguous(arena, offs, ln)
    ch_b = MbufChains.contiguous(other, offs, ln)
    heads = np.where(src, ch_b.heads, ch_a.heads)
    skip = np.where(rng.random(n) < 0.5, rng.integers(0, 60, n), 0)
    skip = np.where(rng.random(n) < 0.02, ln, skip)
    skip = np.where(rng.random(n) < 0.02, ln + 3, skip)
    length = np.where(rng.random(n) < 0.1, rng.integers(0, ln + 1), ln)
    want = ora.skip_batch(heads, length, skip)
    with registered(arena, other):
        got, ns = spans(lambda: u.in_cksum_skip_batch(heads, length, skip))
    assert ns == 1
    np.testing.assert_array_equal(got, want)


def test_span_path_two_regions_pseudo_header(ora, arena):
    """The pseudo-header form (seeds in the common-packet run) over packets
    from two registered regions, alternating in runs of random length."""
    rng = np.random.default_rng(26)
    other = rand_arena(4 << 20, 27)
    n = 20000
    src = np.repeat(rng.random(200) < 0.5, 100)
    ln = rng.integers(0, 1501, n)
    offs = np.where(src, rng.integers(0, other.size - 1502, n), rng.integers(0, arena.size - 1502, n))
    ch_a = MbufChains.contiguous(arena, offs, ln)
    ch_b = MbufChains.contiguous(other, offs, ln)
    heads = np.where(src, ch_b.heads, ch_a.heads)
    off0 = np.minimum(ln, rng.integers(0, 41, n))
    plen = np.maximum(0, ln - off0 - rng.integers(0, 30, n))
    s_ip, d_ip = (rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(2))
    proto = rng.choice(np.array([6, 17], np.uint8), n)
    want = ora.pseudo_header_batch(heads, plen, off0, s_ip, d_ip, proto)
    with registered(arena, other):
        got, ns = spans(lambda: u.in_cksum_pseudo_header_batch(heads, plen, off0, s_ip, d_ip,
                                                                proto))
    assert ns == 1
    np.testing.assert_array_equal(got, want)
