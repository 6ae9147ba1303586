"""uinet_cksum_mbufs: in_cksum_skip over struct mbuf chains that live in HBM
(the fused walk + fold of csrc/cksum_mbufs.hip), bit-exact against the
reference's golden vectors, the oracle and -- through the same records built
on the host -- the reference's own chain walk (in_cksum.c:193-232).

The CPU tests check the record builder (workloads.device_mbufs) itself: built
over a CPU tensor its records are real host mbufs, which the oracle walks."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u
import libuinet_amd.workloads as W
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes

torch = pytest.importorskip("torch")


def rand_arena(nbytes: int, seed: int) -> np.ndarray:
    a = aligned_empty(nbytes)
    splitmix64_bytes(nbytes, seed, out=a)
    return a


def chain_layout(rng, n, arena_size, max_seg=256, max_segs=8, zero_frac=0.08):
    nseg = rng.integers(1, max_segs + 1, n)
    nseg[rng.random(n) < 0.03] = 0  # empty chains (head NULL)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = rng.integers(1, max_seg + 1, s)
    seg_len[rng.random(s) < zero_frac] = 0
    seg_off = rng.integers(0, arena_size - max_seg - 1, s)
    return seg_off.astype(np.int64), seg_len.astype(np.int64), pkt_seg


def len_skip(rng, seg_len, pkt_seg, extra=40):
    """len / skip covering the edges: skip inside and exactly on mbuf
    boundaries, len short of / equal to / beyond the chain, len <= skip."""
    n = pkt_seg.size - 1
    cum = np.concatenate([[0], np.cumsum(seg_len)])
    tot = cum[pkt_seg[1:]] - cum[pkt_seg[:-1]]
    skip = (rng.random(n) * (tot + 1)).astype(np.int64)
    k = pkt_seg[:-1] + (rng.random(n) * np.diff(pkt_seg)).astype(np.int64)
    k = np.minimum(k, max(cum.size - 2, 0))
    skip = np.where((rng.random(n) < 0.25) & (np.diff(pkt_seg) > 0),
                    cum[k] - cum[pkt_seg[:-1]], skip)
    length = skip + (rng.random(n) * (tot - skip + extra)).astype(np.int64)
    length = np.where(rng.random(n) < 0.1, skip - rng.integers(0, 3, n), length)
    length = np.where(rng.random(n) < 0.05, tot, length)
    return np.maximum(length, 0), skip


# ---- the record builder (CPU) -----------------------------------------------------

@pytest.mark.parametrize("shuffle", [None, 5])
def test_device_mbufs_records_walk_like_host_chains(ora, shuffle):
    rng = np.random.default_rng(3 + (shuffle or 0))
    arena = rand_arena(1 << 18, 8)
    seg_off, seg_len, pkt_seg = chain_layout(rng, 500, arena.size)
    t = torch.from_numpy(arena)
    d = W.device_mbufs(t, seg_off, seg_len, pkt_seg, shuffle=shuffle)
    length, skip = len_skip(rng, seg_len, pkt_seg)
    heads = d["heads"].numpy().view(np.uint64)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip)
    np.testing.assert_array_equal(ora.skip_batch(heads, length, skip), want)
    rec = d["mbufs"].numpy()
    assert rec.shape[1] * 8 == u.MSIZE
    firsts = pkt_seg[:-1][np.diff(pkt_seg) > 0]
    slots = ((heads[heads != 0] - np.uint64(d["mbufs"].data_ptr())) // np.uint64(256)).astype(np.int64)
    assert np.all((rec[slots, 3] >> 32) & 0x2)  # M_PKTHDR on the first mbuf of each chain
    assert slots.size == firsts.size


def test_device_mbufs_inline_first_records(ora):
    """inline_first: each packet's first segment inside its own record (the
    config-3tx header mbuf); the records written into the arena walk like
    host chains and leave the summed bytes alone."""
    lay = W.config3tx_layout(512)
    arena = W.materialize_host(lay)
    before = arena.copy()
    t = torch.from_numpy(arena)
    d = W.device_mbufs(t, lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                       inline_first=W.tx_inline_offset(lay))
    heads = d["heads"].numpy().view(np.uint64)
    assert np.array_equal(heads - np.uint64(arena.ctypes.data),
                          (lay["hdr_off"] - W.tx_inline_offset(lay)).astype(np.uint64))
    want = ora.chains(before, lay["seg_off"], lay["seg_len"], lay["pkt_seg"], length=lay["lens"],
                      skip=20)
    np.testing.assert_array_equal(ora.skip_batch(heads, lay["lens"], 20), want)
    s, e, _ = W.clipped_segments(lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lay["lens"],
                                 np.full(512, 20))
    for a, b in zip(s[:200], e[:200]):
        assert np.array_equal(arena[a:b], before[a:b])


def test_mbufs_walked_counts():
    seg_len = np.array([5, 0, 7, 3, 4, 4], np.int64)
    pkt_seg = np.array([0, 4, 6], np.int64)
    # packet 0: offsets 0, 5, 5, 12 -- len 5 reads the first mbuf only; len 6
    # reads through the 7-B one (the zero-length one at 5 too)
    assert W.mbufs_walked(seg_len, pkt_seg, [5, 8], [0, 0]) == 1 + 2
    assert W.mbufs_walked(seg_len, pkt_seg, [6, 8], [0, 0]) == 3 + 2
    assert W.mbufs_walked(seg_len, pkt_seg, [6, 2], [0, 2]) == 3 + 0  # len <= skip: none
    assert W.mbufs_walked(seg_len, pkt_seg, None, None) == 6


def test_cksum_mbufs_rejects_host_tensors():
    with pytest.raises(TypeError):
        u.cksum_mbufs(torch.zeros(4, dtype=torch.int64))


# ---- the kernel (GPU) ----------------------------------------------------------------

@pytest.fixture(scope="module")
def torch_dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert u.device_ok(), "device is not gfx950"
    return torch


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host16(t) -> np.ndarray:
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def run(arena_d, seg_off, seg_len, pkt_seg, length=None, skip=None, seed=None, flags=0,
        shuffle=None, seg_hint=0):
    d = W.device_mbufs(arena_d, seg_off, seg_len, pkt_seg, shuffle=shuffle)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    got = u.cksum_mbufs(d["heads"],
                        length=None if length is None else dev(np.asarray(length, np.int32)),
                        skip=None if skip is None else dev(np.asarray(skip, np.int32)),
                        seed=None if seed is None else dev(np.asarray(seed, np.uint32).view(np.int32)),
                        flags=flags, seg_hint=seg_hint, status=st)
    torch.cuda.synchronize()
    return host16(got), int(st.item()), d




@pytest.mark.gpu
def test_golden_skip_vectors(torch_dev, arena, golden):
    """The reference's own outputs (tests/golden, from oracle/_ref)."""
    g = golden("skip")
    got, st, _ = run(dev(arena), g["seg_off"], g["seg_len"], g["pkt_seg"], g["len"], g["skip"])
    np.testing.assert_array_equal(got, g["expected"])
    assert st == 0


@pytest.mark.gpu
def test_golden_config3_vectors(torch_dev, arena, golden):
    g = golden("configs")
    n = g["c3_pkt_seg"].size - 1
    got, _, _ = run(dev(arena), g["c3_seg_off"], g["c3_seg_len"], g["c3_pkt_seg"], g["c3_len"],
                    np.full(n, 20))
    np.testing.assert_array_equal(got, g["c3_expected"])


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [None, 11])
@pytest.mark.parametrize("flags", [0, u.F_UDP, u.F_NO_COMPLEMENT])
@pytest.mark.parametrize("seg_hint", [0, 128])  # non-temporal / temporal byte loads
def test_random_chains(torch_dev, ora, shuffle, flags, seg_hint):
    rng = np.random.default_rng(70 + flags + (shuffle or 0) + seg_hint)
    arena = rand_arena(1 << 21, 71)
    seg_off, seg_len, pkt_seg = chain_layout(rng, 20000, arena.size)
    length, skip = len_skip(rng, seg_len, pkt_seg)
    n = pkt_seg.size - 1
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    seed[rng.random(n) < 0.3] = 0
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed,
                      flags=flags)
    got, st, _ = run(dev(arena), seg_off, seg_len, pkt_seg, length, skip, seed, flags, shuffle,
                     seg_hint)
    np.testing.assert_array_equal(got, want)
    assert st == 0


@pytest.mark.gpu
def test_null_len_skip_whole_chain(torch_dev, ora):
    rng = np.random.default_rng(5)
    arena = rand_arena(1 << 20, 6)
    seg_off, seg_len, pkt_seg = chain_layout(rng, 3000, arena.size)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg)
    got, _, _ = run(dev(arena), seg_off, seg_len, pkt_seg)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_long_chains_and_long_segments(torch_dev, ora):
    """Chains of 0..3000 one-byte mbufs (thousands of rounds per lane), and
    segments of 2 KiB .. 64 KiB (the wave-wide stream), mixed in one batch."""
    rng = np.random.default_rng(9)
    arena = rand_arena(1 << 23, 10)
    n = 400
    kind = rng.integers(0, 3, n)
    nseg = np.where(kind == 0, rng.integers(0, 3001, n), rng.integers(1, 5, n))
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_pkt = np.repeat(np.arange(n), nseg)
    seg_len = np.where(kind[seg_pkt] == 0, rng.integers(0, 2, s),
                       np.where(kind[seg_pkt] == 1, rng.integers(2048, 9001, s),
                                rng.integers(1, 65536, s)))
    seg_off = rng.integers(0, arena.size - 65536 - 1, s).astype(np.int64)
    length, skip = len_skip(rng, seg_len, pkt_seg, extra=100)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip)
    got, st, _ = run(dev(arena), seg_off, seg_len, pkt_seg, length, skip)
    np.testing.assert_array_equal(got, want)
    assert st == 0


@pytest.mark.gpu
def test_edge_chains(torch_dev, ora):
    """Hand-made edges: empty chain, all-zero-length chain, skip exactly on a
    boundary, skip past the chain, len == skip, len < skip, len beyond the
    chain, a zero-length mbuf at the skip point, odd addresses."""
    arena = rand_arena(1 << 16, 12)
    segs = [
        [],                                   # NULL head
        [(100, 0), (200, 0)],                 # only empty mbufs
        [(101, 20), (301, 33)],               # skip 20: exactly on the boundary
        [(1, 7), (513, 0), (777, 9)],         # zero-length mbuf where skip lands
        [(3, 5)],                             # skip past the chain
        [(10, 50), (90, 50)],                 # len == skip
        [(10, 50), (90, 50)],                 # len < skip
        [(11, 50), (93, 51)],                 # len beyond the chain
        [(5, 1)] * 40,                        # 40 one-byte mbufs
        [(4097, 4096), (1, 1)],               # a long one, then a byte
    ]
    lens = [10, 10, 53, 16, 10, 30, 30, 10_000, 37, 5000]
    skips = [0, 0, 20, 7, 9, 30, 31, 20, 3, 1]
    seg_off = np.array([o for c in segs for o, _ in c], np.int64)
    seg_len = np.array([ln for c in segs for _, ln in c], np.int64)
    pkt_seg = np.concatenate([[0], np.cumsum([len(c) for c in segs])]).astype(np.int64)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=lens, skip=skips)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    np.testing.assert_array_equal(ora.skip_batch(ch.heads, lens, skips), want)
    for shuffle, hint in ((None, 0), (3, 100)):
        got, st, _ = run(dev(arena), seg_off, seg_len, pkt_seg, lens, skips, shuffle=shuffle,
                         seg_hint=hint)
        np.testing.assert_array_equal(got, want)
        assert st == 0


@pytest.mark.gpu
def test_bad_inputs_are_flagged_and_bounded(torch_dev, ora):
    """Outside the contract: a negative m_len ends its chain (BADLEN), a
    negative skip sums nothing (BADARG), and a cyclic chain of zero-length
    mbufs stops after MBUF_HOPS_MAX hops (TRUNC) -- every wave finishes."""
    arena_h = rand_arena(1 << 16, 13)
    a = dev(arena_h)
    seg_off = np.array([0, 64, 128, 300], np.int64)
    seg_len = np.array([30, 40, 50, 20], np.int64)
    pkt_seg = np.array([0, 3, 4], np.int64)
    d = W.device_mbufs(a, seg_off, seg_len, pkt_seg)
    mb = d["mbufs"]
    # mbuf 1 (second of packet 0): m_len = -1
    mb[1, 3] = (mb[1, 3] & ~0xFFFFFFFF) | 0xFFFFFFFF
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    got = host16(u.cksum_mbufs(d["heads"], length=dev(np.array([120, 20], np.int32)),
                               skip=dev(np.array([0, -1], np.int32)), status=st))
    want0 = ora.chains(arena_h, seg_off[:1], seg_len[:1], np.array([0, 1]), length=[120])
    assert got[0] == want0[0]             # summed up to the bad mbuf
    assert got[1] == 0xFFFF               # nothing summed
    assert int(st.item()) == u.MBUF_BADLEN | u.MBUF_BADARG
    # a 2-mbuf cycle of empty mbufs
    mb2 = W.device_mbufs(a, np.array([0, 0], np.int64), np.array([0, 0], np.int64),
                         np.array([0, 2], np.int64))
    mb2["mbufs"][1, 0] = mb2["heads"][0]  # m_next of the last -> the first
    st.zero_()
    got = host16(u.cksum_mbufs(mb2["heads"], length=dev(np.array([100], np.int32)), status=st))
    torch.cuda.synchronize()
    assert got[0] == 0xFFFF and int(st.item()) == u.MBUF_TRUNC


@pytest.mark.gpu
def test_full_config3_mbufs(torch_dev, ora):
    """BASELINE config 3 in its own form: 1 M mixed 64/576/1500-B packets as
    m_fragment-style chains of 1..256-B mbufs in HBM, in_cksum_skip(m, len,
    20), against the oracle; the same bytes as the segment-list form."""
    c = W.config3_device(1 << 20, seed=3)
    lay = c["layout"]
    d = W.device_mbufs(c["arena"], c["seg_off"], c["seg_len"], c["pkt_seg"])
    want = ora.chains(c["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=20)
    for hint in (0, c["mean_seg"]):
        got = host16(u.cksum_mbufs(d["heads"], length=c["len"], skip=c["skip"], seg_hint=hint))
        np.testing.assert_array_equal(got, want)
    seglist = host16(u.cksum_chains(c["arena"], c["seg_off"], c["seg_len"], c["pkt_seg"],
                                    length=c["len"], skip=c["skip"], len_hint=c["mean_seg"]))
    np.testing.assert_array_equal(seglist, want)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["3tx", "5tso"])
def test_full_chain_variants_mbufs(torch_dev, ora, cfg):
    """Config 3tx (40-B header mbuf -> 4-KiB page-cluster slices) and 5tso
    (TSO segments, pseudo-header seeds) as HBM mbuf chains, full size."""
    w = W.materialize_device(W.chain_layout(cfg))
    lay = w["layout"]
    d = W.device_mbufs(w["arena"], w["seg_off"], w["seg_len"], w["pkt_seg"], shuffle=1,
                       inline_first=W.tx_inline_offset(lay) if cfg == "3tx" else None)
    got = host16(u.cksum_mbufs(d["heads"], length=w["len"], skip=w["skip"], seed=w.get("seed")))
    want = ora.chains(w["arena"].cpu().numpy(), lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                      length=lay["lens"], skip=lay["skip"], seed=lay["seed"])
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_streams_and_empty_batch(torch_dev, ora):
    """n = 0 is a no-op; a launch on a side stream orders like any other."""
    out = torch.empty(0, dtype=torch.uint16, device="cuda")
    u.cksum_mbufs(torch.empty(0, dtype=torch.int64, device="cuda"), out=out)
    rng = np.random.default_rng(21)
    arena = rand_arena(1 << 20, 22)
    seg_off, seg_len, pkt_seg = chain_layout(rng, 5000, arena.size)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg)
    a = dev(arena)
    d = W.device_mbufs(a, seg_off, seg_len, pkt_seg)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        got = u.cksum_mbufs(d["heads"], stream=s)
    s.synchronize()
    np.testing.assert_array_equal(host16(got), want)
