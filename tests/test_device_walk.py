"""The device-side chain walk: host-mbuf batches whose mbufs and packet bytes
all lie in registered host memory are walked by the GPU (m_next / m_data /
m_len read over PCIe) -- in one launch that also folds the bytes
(csrc/cksum_mbufs.hip, knob walk_device 3; the hooks' default) or into a
segment list that the chain kernel folds (csrc/cksum_walk.hip, walk_device 2;
the chain batches' default); every test runs under both.
Every case is checked bit-exact against the oracle, and
uinet_cksum_host_cpu().device_walks says whether the GPU walked the batch or
the host walk took it (a pointer outside the regions, a pseudo-header off0
past the first mbuf, a chain longer than the walk takes)."""
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


def walks(fn):
    """(result, device walks during fn())."""
    before = u.host_cpu()["device_walks"]
    r = fn()
    return r, u.host_cpu()["device_walks"] - before


def chains(rng, arena, n, max_seg=12, max_len=300, zero_frac=0.1):
    nseg = rng.integers(1, max_seg + 1, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(0, max_len + 1, s)
    seg_len[rng.random(s) < zero_frac] = 0
    seg_off = rng.integers(0, arena.size - max_len - 1, s).astype(np.int64)
    return MbufChains(arena, seg_off, seg_len, pkt_seg), seg_len, pkt_seg


@pytest.fixture(scope="module")
def arena(torch_dev):
    return rand_arena(4 << 20, 777)


@pytest.fixture(autouse=True, params=[3, 2], ids=["fused", "seglist"])
def walk_form(request):
    # the single-mbuf span path (test_span_fast.py) off: every batch here
    # exercises the device walk, one-mbuf chains included
    u.set_tuning("span_fast", 0)
    u.set_tuning("walk_device", request.param)
    yield request.param
    u.set_tuning("walk_device", 1)
    u.set_tuning("span_fast", 1)


def test_device_walk_skip_batch_edges(ora, arena):
    """Zero-length mbufs, skip exactly on an mbuf boundary, len beyond the
    chain, len < skip, len 0, single-mbuf and long chains."""
    rng = np.random.default_rng(1)
    n = 4096
    ch, seg_len, pkt_seg = chains(rng, arena, n)
    cs = np.concatenate([[0], np.cumsum(seg_len)])
    tot = cs[pkt_seg[1:]] - cs[pkt_seg[:-1]]
    length = tot.copy()
    skip = np.zeros(n, np.int64)
    k = np.arange(n) % 8
    # skip on the first mbuf boundary
    first_end = seg_len[pkt_seg[:-1]]
    skip[k == 1] = first_end[k == 1]
    length[k == 2] = tot[k == 2] + 100       # len beyond the chain
    length[k == 3] = 0
    skip[k == 4] = 20
    length[k == 4] = 10                      # len < skip
    skip[k == 5] = np.minimum(tot[k == 5], 41)
    length[k == 6] = np.maximum(0, tot[k == 6] - 7)
    skip[k == 7] = tot[k == 7]               # skip == whole chain
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, length, skip))
    assert nw == 1, "the GPU did not walk this batch"
    want = ora.skip_batch(ch.heads, length, skip)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]


def test_device_walk_long_chains_grow_rows(ora, arena):
    """Chains longer than the walk's first row size: walked again with room."""
    rng = np.random.default_rng(2)
    n = 700
    ch, seg_len, pkt_seg = chains(rng, arena, n, max_seg=300, max_len=40)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 30, 3))
    assert nw == 1
    assert np.array_equal(got, ora.skip_batch(ch.heads, 1 << 30, 3))


def test_device_walk_chain_past_row_limit(ora, arena, walk_form):
    """A chain of 5,000 one-byte mbufs among short ones: longer than any
    segment-list row (4,096), so that walk stops at the limit and hands the
    batch to the host walk (it never follows a chain without bound); the
    fused walk takes it on the device.  Same results either way."""
    rng = np.random.default_rng(12)
    n = 300
    nseg = rng.integers(1, 5, n)
    nseg[137] = 5000
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(1, 100, s)
    seg_len[pkt_seg[137]:pkt_seg[138]] = 1
    seg_off = rng.integers(0, arena.size - 101, s).astype(np.int64)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    want = ora.skip_batch(ch.heads, 1 << 30, 2)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 30, 2))
    assert nw == (1 if walk_form == 3 else 0)
    assert np.array_equal(got, want)


def test_device_walk_pipelined_groups(ora, arena):
    """A batch large enough for the walk/fold pipeline (groups of consecutive
    packets alternating between two streams), with a row size that has to
    grow on the way (a few long chains), and skip / len cutting the chains."""
    rng = np.random.default_rng(7)
    n = 100_003
    ch, seg_len, pkt_seg = chains(rng, arena, n, max_seg=5, max_len=200)
    cs = np.concatenate([[0], np.cumsum(seg_len)])
    tot = cs[pkt_seg[1:]] - cs[pkt_seg[:-1]]
    length = np.maximum(0, tot - rng.integers(0, 30, n))
    skip = np.minimum(rng.integers(0, 41, n), length)
    want = ora.skip_batch(ch.heads, length, skip)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, length, skip))
        assert nw == 1 and np.array_equal(got, want), np.flatnonzero(got != want)[:8]
        # chains of up to 60 mbufs near the end of the batch: the walk grows its rows
        long = MbufChains(arena, *_long_tail(rng, arena, n))
        with registered(long.mbufs):
            want2 = ora.skip_batch(long.heads, 1 << 30, 0)
            got2, nw2 = walks(lambda: u.in_cksum_skip_batch(long.heads, 1 << 30, 0))
    assert nw2 == 1 and np.array_equal(got2, want2), np.flatnonzero(got2 != want2)[:8]


def _long_tail(rng, arena, n):
    nseg = rng.integers(1, 4, n)
    nseg[-50:] = rng.integers(30, 61, 50)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(0, 100, s)
    seg_off = rng.integers(0, arena.size - 101, s).astype(np.int64)
    return seg_off, seg_len, pkt_seg


def test_device_walk_falls_back_outside_regions(ora, arena):
    """A chain whose mbufs, or one of whose data pointers, lie outside the
    registered regions goes to the host walk, with the same results."""
    rng = np.random.default_rng(3)
    n = 2000
    ch, _, _ = chains(rng, arena, n)
    want = ora.skip_batch(ch.heads, 1 << 20, 0)
    with registered(arena):  # mbufs not registered
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 20, 0))
    assert nw == 0 and np.array_equal(got, want)
    # one mbuf mid-chain points into an unregistered buffer
    other = rand_arena(1 << 16, 9)
    long_pk = int(np.flatnonzero(np.diff(ch.pkt_seg) >= 3)[0])
    mid = int(ch.pkt_seg[long_pk]) + 1
    ch.mbufs["m_data"][mid] = other.ctypes.data
    ch.mbufs["m_len"][mid] = 64
    want = ora.skip_batch(ch.heads, 1 << 20, 0)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 20, 0))
    assert nw == 0 and np.array_equal(got, want)
    with registered(arena, ch.mbufs, other):  # now it is registered too
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 20, 0))
    assert nw == 1 and np.array_equal(got, want)


def test_device_walk_pseudo_header(ora, arena):
    """in_cksum_pseudo_header_batch: off0 inside the first mbuf walks on the
    GPU; an off0 past the first mbuf (where the reference's sum differs from
    the skip form) takes the host walk."""
    rng = np.random.default_rng(4)
    n = 3000
    ch, seg_len, pkt_seg = chains(rng, arena, n, zero_frac=0.0)
    first = seg_len[pkt_seg[:-1]]
    cs = np.concatenate([[0], np.cumsum(seg_len)])
    tot = cs[pkt_seg[1:]] - cs[pkt_seg[:-1]]
    off0 = np.minimum(first, rng.integers(0, 41, n))
    plen = np.maximum(0, tot - off0 - rng.integers(0, 20, n))
    src, dst = (rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(2))
    proto = rng.choice(np.array([6, 17], np.uint8), n)
    want = ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_pseudo_header_batch(ch.heads, plen, off0, src, dst, proto))
        assert nw == 1 and np.array_equal(got, want)
        off0b = off0.copy()
        off0b[5] = first[5] + 3  # outside the reference's contract: host walk
        plenb = np.maximum(0, plen - 3)
        wantb = ora.pseudo_header_batch(ch.heads, plenb, off0b, src, dst, proto)
        got, nw = walks(lambda: u.in_cksum_pseudo_header_batch(ch.heads, plenb, off0b, src, dst,
                                                                proto))
    assert nw == 0 and np.array_equal(got, wantb)


def test_device_walk_knob_off(ora, arena):
    rng = np.random.default_rng(5)
    ch, _, _ = chains(rng, arena, 500)
    u.set_tuning("walk_device", 0)  # the fixture restores the default
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 20, 0))
    assert nw == 0 and np.array_equal(got, ora.skip_batch(ch.heads, 1 << 20, 0))


def test_device_walk_hooks(ora, torch_dev):
    """The RX / TX hooks (headers parsed on the host, payload chains walked on
    the GPU), mbufs and frames registered (in6_cksum_batch: tests/test_in6.py)."""
    from libuinet_amd.frames import FrameBatch, pkthdr_fields

    a = FrameBatch(3000, seed=11, ipv6=0.3)
    b = FrameBatch(3000, seed=11, ipv6=0.3)
    with registered(a.arena, a.tx.mbufs):
        st, nw = walks(lambda: u.tx_offload(a.tx.heads))
    assert nw == 1
    assert np.array_equal(st, ora.tx_offload(b.tx.heads))
    assert np.array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        assert np.array_equal(x, y)
    rx_a, arena_a, _ = a.rx(seed=3, corrupt=0.05)
    rx_b, _, _ = b.rx(seed=3, corrupt=0.05)
    with registered(arena_a, rx_a.mbufs):
        st, nw = walks(lambda: u.rx_offload(rx_a.heads))
    assert nw == 1
    assert np.array_equal(st, ora.rx_offload(rx_b.heads))
    for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("on_device", [True, False])
def test_hooks_headers_split_across_mbufs(ora, torch_dev, on_device):
    """RX and TX hooks on frames whose link / IP / L4 headers straddle the
    first mbuf boundary (and zero-length mbufs), IPv4 with options and IPv6
    with extension headers among them: on the device (mbufs registered, a
    device-sized batch) and on the host hook, bit-exact against the oracle --
    statuses, the sums written into the frames and the pkthdr marks."""
    from libuinet_amd.frames import FrameBatch, pkthdr_fields, split_headers as resplit

    n = 2600 if on_device else 1500
    a = FrameBatch(n, seed=21, ipv6=0.3)
    b = FrameBatch(n, seed=21, ipv6=0.3)
    ta, tb = resplit(a.tx, 5), resplit(b.tx, 5)
    regs = (a.arena, ta.mbufs) if on_device else ()
    with registered(*regs):
        st, nw = walks(lambda: u.tx_offload(ta.heads))
    assert nw == (1 if on_device else 0)
    assert np.array_equal(st, ora.tx_offload(tb.heads))
    assert np.array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(ta), pkthdr_fields(tb)):
        assert np.array_equal(x, y)
    rx_a, arena_a, _ = a.rx(seed=6, corrupt=0.05)
    rx_b, _, _ = b.rx(seed=6, corrupt=0.05)
    ra, rb = resplit(rx_a, 7), resplit(rx_b, 7)
    regs = (arena_a, ra.mbufs) if on_device else ()
    with registered(*regs):
        st, nw = walks(lambda: u.rx_offload(ra.heads))
    assert nw == (1 if on_device else 0)
    assert np.array_equal(st, ora.rx_offload(rb.heads))
    for x, y in zip(pkthdr_fields(ra), pkthdr_fields(rb)):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("mode", ["device", "bytes", "host"])
def test_hooks_malformed_frames(ora, torch_dev, mode):
    """RX and TX hooks on batches where most frames are malformed the ways the
    stack's input checks name (frames.mangle_headers: version / header-length
    nibbles, ethertype, IP / IPv6 / UDP lengths, next-header types, extension
    lengths, chains cut inside their headers, only empty mbufs), headers also
    cut across mbufs: on the device hook (mbufs and frames registered), the
    host hook over registered frames, and the staged host hook -- statuses,
    stored sums and marks bit-exact against the oracle."""
    from libuinet_amd.frames import FrameBatch, mangle_headers, pkthdr_fields, split_headers

    n = 2600 if mode == "device" else 1500
    for l2, seed in ((True, 41), (False, 42)):
        l2len = -1 if l2 else 0
        a = FrameBatch(n, seed=seed, l2=l2, ipv6=0.4)
        b = FrameBatch(n, seed=seed, l2=l2, ipv6=0.4)
        ta, tb = mangle_headers(a.tx, a, seed, 0.7), mangle_headers(b.tx, b, seed, 0.7)
        ta, tb = split_headers(ta, seed + 1, 0.3), split_headers(tb, seed + 1, 0.3)
        regs = {"device": (a.arena, ta.mbufs), "bytes": (a.arena,), "host": ()}[mode]
        with registered(*regs):
            st, nw = walks(lambda: u.tx_offload(ta.heads, l2len))
        assert nw == (1 if mode == "device" else 0)
        assert np.array_equal(st, ora.tx_offload(tb.heads, l2len)), (l2, "TX")
        assert np.array_equal(a.arena, b.arena)
        for x, y in zip(pkthdr_fields(ta), pkthdr_fields(tb)):
            assert np.array_equal(x, y)
        rx_a, arena_a, _ = a.rx(seed=seed + 2, corrupt=0.05)
        rx_b, _, _ = b.rx(seed=seed + 2, corrupt=0.05)
        ra, rb = mangle_headers(rx_a, a, seed + 3, 0.7), mangle_headers(rx_b, b, seed + 3, 0.7)
        ra, rb = split_headers(ra, seed + 4, 0.3), split_headers(rb, seed + 4, 0.3)
        regs = {"device": (arena_a, ra.mbufs), "bytes": (arena_a,), "host": ()}[mode]
        with registered(*regs):
            st, nw = walks(lambda: u.rx_offload(ra.heads, l2len))
        assert nw == (1 if mode == "device" else 0)
        want = ora.rx_offload(rb.heads, l2len)
        assert np.array_equal(st, want), (l2, "RX", np.flatnonzero(st != want)[:8])
        for x, y in zip(pkthdr_fields(ra), pkthdr_fields(rb)):
            assert np.array_equal(x, y)
        assert (want & 0x08).any() and (want == 0).any()  # verified frames and unmarked ones


def _payload_outside(ch, arena, k, other):
    """Point frame k's second mbuf at a copy of its bytes in `other` (outside
    the registered regions); returns the copy's offset in `other`."""
    seg = int(ch.pkt_seg[k]) + 1
    ln = int(ch.mbufs["m_len"][seg])
    src = int(ch.mbufs["m_data"][seg]) - arena.ctypes.data
    other[:ln] = arena[src:src + ln]
    ch.mbufs["m_data"][seg] = other.ctypes.data


def test_device_hooks_walk_flag_in_last_group(ora, torch_dev):
    """Batches of 20,000 frames (the device hook walks them in several groups
    on two streams): one frame in the last group has a payload mbuf outside the
    registered regions.  The parse, which reads only the first mbuf, takes it;
    the walk flags it, so the apply writes nothing in any group and the host
    hook takes the whole batch -- equal to the oracle, TX and RX.  (Writing
    the other groups on the device and redoing only the flagged one measured
    no faster: profiles/r05/pruned/hook_apply_per_group.diff.)"""
    from libuinet_amd.frames import FrameBatch, pkthdr_fields

    n = 20000
    a = FrameBatch(n, seed=41)
    b = FrameBatch(n, seed=41)
    k = int(np.flatnonzero(np.diff(a.tx.pkt_seg) >= 2)[-1])  # a chained frame near the end
    oa, ob = rand_arena(1 << 16, 3), rand_arena(1 << 16, 3)
    _payload_outside(a.tx, a.arena, k, oa)
    _payload_outside(b.tx, b.arena, k, ob)
    with registered(a.arena, a.tx.mbufs):
        st, nw = walks(lambda: u.tx_offload(a.tx.heads))
    assert nw == 0  # the host hook took the batch
    assert np.array_equal(st, ora.tx_offload(b.tx.heads))
    assert np.array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        assert np.array_equal(x, y)
    rx_a, arena_a, _ = a.rx(seed=42, corrupt=0.05)
    rx_b, arena_b, _ = b.rx(seed=42, corrupt=0.05)
    k = int(np.flatnonzero(np.diff(rx_a.pkt_seg) >= 2)[-1])
    _payload_outside(rx_a, arena_a, k, oa)
    _payload_outside(rx_b, arena_b, k, ob)
    with registered(arena_a, rx_a.mbufs):
        st, nw = walks(lambda: u.rx_offload(rx_a.heads))
    assert nw == 0
    assert np.array_equal(st, ora.rx_offload(rx_b.heads))
    for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
        assert np.array_equal(x, y)


def test_device_hooks_fall_back_outside_regions(ora, torch_dev):
    """A TX batch one of whose frames has its first mbuf's data outside the
    registered regions: the device hook writes nothing and the host hook takes
    the batch, with the oracle's results."""
    from libuinet_amd.frames import FrameBatch, pkthdr_fields

    a = FrameBatch(2500, seed=12, ipv6=0.3)  # >= 2,048 frames: the device hook's size
    b = FrameBatch(2500, seed=12, ipv6=0.3)
    other = rand_arena(1 << 16, 5)
    first = int(a.tx.pkt_seg[3])
    ln = int(a.tx.mbufs["m_len"][first])
    src = int(a.tx.mbufs["m_data"][first]) - a.arena.ctypes.data
    if 0 <= src <= a.arena.size - ln:  # move frame 3's first mbuf data out of the regions
        other[:ln] = a.arena[src:src + ln]
        a.tx.mbufs["m_data"][first] = other.ctypes.data
        bf = int(b.tx.pkt_seg[3])
        b.tx.mbufs["m_data"][bf] = other.ctypes.data + (1 << 15)
        other[1 << 15:(1 << 15) + ln] = b.arena[src:src + ln]
    else:  # headers in the mbuf itself: point at a copy outside
        mb = a.tx.mbufs.view(np.uint8).reshape(-1, 256)
        off = int(a.tx.mbufs["m_data"][first]) - a.tx.mbufs.ctypes.data - 256 * first
        other[:ln] = mb[first, off:off + ln]
        a.tx.mbufs["m_data"][first] = other.ctypes.data
        other[1 << 15:(1 << 15) + ln] = mb[first, off:off + ln]
        b.tx.mbufs["m_data"][int(b.tx.pkt_seg[3])] = other.ctypes.data + (1 << 15)
    with registered(a.arena, a.tx.mbufs):
        st, nw = walks(lambda: u.tx_offload(a.tx.heads))
    assert nw == 0
    assert np.array_equal(st, ora.tx_offload(b.tx.heads))
    assert np.array_equal(a.arena, b.arena)
    assert np.array_equal(other[:ln], other[1 << 15:(1 << 15) + ln])
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        assert np.array_equal(x, y)


def test_small_batches_are_staged(ora, arena, torch_dev):
    """Over registered memory, batches of at most 128 packets and hook batches
    below 2,048 frames are staged (one launch out of mapped memory answers
    sooner, profiles/r05/r05k/); results equal the oracle's either way."""
    from libuinet_amd.frames import FrameBatch, pkthdr_fields

    rng = np.random.default_rng(8)
    ch, _, _ = chains(rng, arena, 129)
    with registered(arena, ch.mbufs):
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads[:128], 1 << 20, 0))
        assert nw == 0 and np.array_equal(got, ora.skip_batch(ch.heads[:128], 1 << 20, 0))
        got, nw = walks(lambda: u.in_cksum_skip_batch(ch.heads, 1 << 20, 0))
        assert nw == 1 and np.array_equal(got, ora.skip_batch(ch.heads, 1 << 20, 0))
    a = FrameBatch(2047, seed=13)
    b = FrameBatch(2047, seed=13)
    with registered(a.arena, a.tx.mbufs):
        st, nw = walks(lambda: u.tx_offload(a.tx.heads))
    assert nw == 0 and np.array_equal(st, ora.tx_offload(b.tx.heads))
    assert np.array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(a.tx), pkthdr_fields(b.tx)):
        assert np.array_equal(x, y)


def test_host_cpu_counters(arena):
    """uinet_cksum_host_cpu counts calls, packets, wall and CPU time on the
    calling thread, and resets."""
    rng = np.random.default_rng(6)
    ch, _, _ = chains(rng, arena, 5000)
    u.host_cpu(reset=True)
    u.in_cksum_skip_batch(ch.heads, 1 << 20, 0)
    u.in_cksum_skip_batch(ch.heads, 1 << 20, 0)
    st = u.host_cpu(reset=True)
    assert st["calls"] == 2 and st["packets"] == 10000
    assert st["wall_ns"] > 0 and st["caller_cpu_ns"] > 0
    assert st["cpu_ns"] == st["caller_cpu_ns"] + st["helper_cpu_ns"]
    assert u.host_cpu()["calls"] == 0


def test_device_paths_concurrent_threads(ora, arena, torch_dev):
    """An RX thread and a TX thread (libuinet's per-interface kthreads,
    uinet_if_netmap.c:1648-1665) and a host-batch thread calling the device
    paths at once, each on its own registered batch: every call equals the
    oracle (each thread has its own stream and staging; regions are shared)."""
    import threading

    from libuinet_amd.frames import FrameBatch

    rng = np.random.default_rng(9)
    ch, _, _ = chains(rng, arena, 3000)
    want_skip = ora.skip_batch(ch.heads, 1 << 20, 0)
    tx_a, tx_b = FrameBatch(2500, seed=21, ipv6=0.3), FrameBatch(2500, seed=21, ipv6=0.3)
    want_tx = ora.tx_offload(tx_b.tx.heads)
    rx_src = FrameBatch(2500, seed=22, ipv6=0.3)
    rx, rx_arena, _ = rx_src.rx(seed=2, corrupt=0.05)
    rx_ref, _, _ = FrameBatch(2500, seed=22, ipv6=0.3).rx(seed=2, corrupt=0.05)
    want_rx = ora.rx_offload(rx_ref.heads)
    errors = []

    def tx_loop():
        try:
            for _ in range(10):
                # re-armed flags; the sums of a repeat differ (their fields now
                # hold final sums), the per-frame status does not
                tx_a.set_tx_flags()
                st = u.tx_offload(tx_a.tx.heads)
                assert np.array_equal(st, want_tx)
        except Exception as e:  # reported below
            errors.append(("tx", e))

    def rx_loop():
        try:
            for _ in range(10):
                rx.mbufs["csum_flags"][:] = 0
                rx.mbufs["csum_data"][:] = 0
                assert np.array_equal(u.rx_offload(rx.heads), want_rx)
        except Exception as e:
            errors.append(("rx", e))

    def skip_loop():
        try:
            for _ in range(10):
                assert np.array_equal(u.in_cksum_skip_batch(ch.heads, 1 << 20, 0), want_skip)
        except Exception as e:
            errors.append(("skip", e))

    with registered(arena, ch.mbufs, tx_a.arena, tx_a.tx.mbufs, rx_arena, rx.mbufs):
        ts = [threading.Thread(target=f) for f in (tx_loop, rx_loop, skip_loop)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
    assert not errors, errors
