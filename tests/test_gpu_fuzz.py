"""Randomised differential test of the device-resident entry points against the
oracle: every trial draws an API (spans wide / packed, strided, chains wide /
packed, HBM mbuf chains), a batch shape (counts, length families from empty to 20 KB, head
offsets, lengths and skips that cut chains short), a length hint that may not
match the batch, flags, seeds and parity, and a setting of every performance
knob (which must never change a result: include/uinet_cksum.h).  Seeded, so a
failure names its trial and replays."""
from __future__ import annotations

import os

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import dev, host16, rand_arena

pytestmark = pytest.mark.gpu

DEFAULTS = {"blocks_per_cu": 0, "chains_long": 128, "xcd_remap": 1, "chains_wide": 0}
KNOBS = {"blocks_per_cu": [0, 0, 1, 3, 64], "chains_long": [128, 0, 16], "xcd_remap": [1, 0],
         "chains_wide": [0, 0, 1, 2]}
HINTS = (0, 64, 80, 200, 500, 1500, 4000, 9000)
ARENA = 8 << 20
TRIALS = int(os.environ.get("UINET_FUZZ_TRIALS", "300"))  # longer hunts: set it
BASE = int(os.environ.get("UINET_FUZZ_BASE", "0"))  # and this, for seeds not yet run


def _lengths(rng, n):
    fam = rng.integers(0, 5)
    hi = (64, 300, 2000, 9300, 20000)[fam]
    ln = rng.integers(0, hi + 1, n)
    edge = rng.random(n) < 0.05
    ln[edge] = rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 1500, 3072, 9216, 9217], int(edge.sum()))
    return ln.astype(np.int64)


def _trial(torch, ora, arena, d_arena, t):
    rng = np.random.default_rng(90000 + BASE + t)
    knobs = {k: int(rng.choice(vals)) for k, vals in KNOBS.items()}
    for k, v in knobs.items():
        u.set_tuning(k, v)
    api = ("spans", "spans32", "strided", "chains", "chains32", "mbufs")[rng.integers(0, 6)]
    n = int(rng.choice([1, 2, 3, 63, 64, 65, int(rng.integers(1, 3000))]))
    hint = int(rng.choice(HINTS)) if rng.random() < 0.8 else int(rng.integers(0, 12000))
    flags = int(rng.choice([0, u.F_UDP, u.F_NO_COMPLEMENT]))
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.5 else None
    d_seed = dev(torch, seed.view(np.int32)) if seed is not None else None
    if api in ("spans", "spans32", "strided"):
        if api == "strided":
            length = int(_lengths(rng, 1)[0])
            stride = length + int(rng.integers(0, 40))
            n = max(1, min(n, (ARENA - 64) // max(stride, 1)))
            seed = seed[:n] if seed is not None else None
            d_seed = dev(torch, seed.view(np.int32)) if seed is not None else None
            base = int(rng.integers(0, 64))
            got = u.cksum_strided(d_arena[base:], stride, length, n, seed=d_seed, flags=flags)
            off = base + stride * np.arange(n, dtype=np.int64)
            want = ora.spans(arena, off, np.full(n, length, np.int64), seed, None, flags)
        else:
            ln = _lengths(rng, n)
            off = rng.integers(0, ARENA - 20001, n).astype(np.int64)
            par = rng.integers(0, 2, n).astype(np.uint8) if rng.random() < 0.5 else None
            d_par = dev(torch, par) if par is not None else None
            if api == "spans32":
                po, pl = u.pack_segments(off, ln.astype(np.int32))
                d_off, d_ln = dev(torch, po), dev(torch, pl)
            else:
                d_off, d_ln = dev(torch, off), dev(torch, ln.astype(np.int32))
            got = u.cksum_spans(d_arena, d_off, d_ln, seed=d_seed, parity=d_par, flags=flags,
                                len_hint=hint)
            want = ora.spans(arena, off, ln, seed, par, flags)
    else:
        nseg = rng.integers(0 if rng.random() < 0.1 else 1, int(rng.choice([2, 8, 40])) + 1, n)
        nseg[0] = max(nseg[0], 1)  # at least one segment in the batch
        pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
        s = int(pkt_seg[-1])
        seg_len = _lengths(rng, s)
        if rng.random() < 0.5:  # segments laid out in order, 0-7 B apart (config-3 shape)
            gaps = rng.integers(0, 8, s)
            seg_off = np.cumsum(np.concatenate([[int(rng.integers(0, 16))], (seg_len + gaps)[:-1]]))
            seg_off = (seg_off % (ARENA - 20001)).astype(np.int64)
        else:
            seg_off = rng.integers(0, ARENA - 20001, s).astype(np.int64)
        cs = np.concatenate([[0], np.cumsum(seg_len)])
        tot = cs[pkt_seg[1:]] - cs[pkt_seg[:-1]]
        length = skip = None
        if rng.random() < 0.5:
            length = np.maximum(0, tot + rng.integers(-40, 41, n)).astype(np.int64)
        if rng.random() < 0.5:
            skip = np.minimum(rng.integers(0, 61, n), tot if length is None else length)
            skip = skip.astype(np.int64)
        d_len = dev(torch, length.astype(np.int32)) if length is not None else None
        d_skip = dev(torch, skip.astype(np.int32)) if skip is not None else None
        if api == "mbufs":  # the same chains as struct mbufs in HBM
            from libuinet_amd.workloads import device_mbufs

            mb = device_mbufs(d_arena, seg_off, seg_len, pkt_seg,
                              shuffle=int(rng.integers(0, 99)) if rng.random() < 0.5 else None)
            got = u.cksum_mbufs(mb["heads"], length=d_len, skip=d_skip, seed=d_seed, flags=flags,
                                seg_hint=hint)
        else:
            if api == "chains32":
                so, sl = u.pack_segments(seg_off, seg_len.astype(np.int32))
                d_so, d_sl = dev(torch, so), dev(torch, sl)
            else:
                d_so, d_sl = dev(torch, seg_off), dev(torch, seg_len.astype(np.int32))
            got = u.cksum_chains(d_arena, d_so, d_sl, dev(torch, pkt_seg.astype(np.int32)),
                                 length=d_len, skip=d_skip, seed=d_seed, flags=flags,
                                 len_hint=hint)
        want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip, seed=seed,
                          flags=flags)
    bad = np.flatnonzero(host16(got) != want)
    _trial.packets = getattr(_trial, "packets", 0) + n
    assert bad.size == 0, (f"trial {t}: api={api} n={n} hint={hint} flags={flags} "
                           f"knobs={knobs} first mismatches {bad[:5].tolist()}")


def test_fuzz_device_entry_points(ora):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    arena = rand_arena(ARENA, 2024)
    d_arena = dev(torch, arena)
    try:
        for t in range(TRIALS):
            _trial(torch, ora, arena, d_arena, t)
            if t % 1000 == 999:
                print(f"fuzz: {t + 1} trials", flush=True)
        print(f"fuzz: {TRIALS} trials, {_trial.packets} packets")
    finally:
        for k, v in DEFAULTS.items():
            u.set_tuning(k, v)


HOST_DEFAULTS = {"host_threads": min(16, os.cpu_count() or 1), "walk_device": 1, "span_fast": 1}


def _host_trial(ora, arena, t):
    from libuinet_amd.mbuf import MbufChains

    rng = np.random.default_rng(70000 + BASE + t)
    u.set_tuning("host_threads", int(rng.choice([1, 2, 5, 16])))
    u.set_tuning("walk_device", int(rng.integers(0, 4)))
    u.set_tuning("span_fast", int(rng.choice([0, 1, 1, 2, 2])))
    n = int(rng.choice([1, 7, 64, 200, int(rng.integers(1, 2500))]))
    nseg = rng.integers(1, int(rng.choice([2, 6, 30])) + 1, n)  # a chain is >= 1 mbuf
    if rng.random() < 0.3:  # one mbuf per packet: the single-mbuf span path's shape
        nseg[:] = 1
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    seg_len = _lengths(rng, s)
    if rng.random() < 0.15:  # pieces past 65535 B: the zero-copy path's wide descriptors
        seg_len[rng.integers(0, s)] = int(rng.integers(65536, 90000))
    seg_off = rng.integers(0, ARENA - 90001, s).astype(np.int64)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    cs = np.concatenate([[0], np.cumsum(seg_len)])
    tot = cs[pkt_seg[1:]] - cs[pkt_seg[:-1]]
    zero_copy = rng.random() < 0.5
    # with the mbufs registered too, the GPU walks the chains (cksum_walk.hip)
    walk_mbufs = zero_copy and rng.random() < 0.5
    if zero_copy:
        u.register_host(arena)
    if walk_mbufs:
        u.register_host(ch.mbufs)
    try:
        if rng.random() < 0.7:
            length = np.maximum(0, tot + rng.integers(-30, 31, n)).astype(np.int64)
            skip = np.minimum(rng.integers(0, 41, n), length).astype(np.int64)
            got = u.in_cksum_skip_batch(ch.heads, length, skip)
            want = ora.skip_batch(ch.heads, length, skip)
            what = "skip"
        else:
            off0 = np.minimum(rng.integers(0, 41, n), tot)
            plen = np.maximum(0, tot - off0 - rng.integers(0, 20, n))
            src, dst = (rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(2))
            proto = rng.choice(np.array([6, 17], np.uint8), n)
            got = u.in_cksum_pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
            want = ora.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
            what = "pseudo"
    finally:
        if zero_copy:
            u.unregister_host(arena)
        if walk_mbufs:
            u.unregister_host(ch.mbufs)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (f"host trial {t}: {what} n={n} zero_copy={zero_copy} "
                           f"mbufs registered={walk_mbufs} "
                           f"first mismatches {bad[:5].tolist()}")
    return n


def test_fuzz_host_batches(ora):
    """The host-mbuf batch API (in_cksum_skip_batch, in_cksum_pseudo_header_batch)
    over random chains, staged and zero-copy, under random host-pool knobs."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    arena = rand_arena(ARENA, 2025)
    packets = 0
    try:
        for t in range(max(1, TRIALS // 3)):
            packets += _host_trial(ora, arena, t)
            if t % 200 == 199:  # long hunts: a sign of life every few seconds
                print(f"host fuzz: {t + 1} trials", flush=True)
        print(f"host fuzz: {max(1, TRIALS // 3)} trials, {packets} packets")
    finally:
        for k, v in HOST_DEFAULTS.items():
            u.set_tuning(k, v)


def test_fuzz_offload_hooks(ora):
    """The RX / TX driver hooks over random frame batches (IPv4 and IPv6 in random
    proportions, with and without the link header, random corruption), staged and
    zero-copy, under random host-pool knobs: status, packet bytes and m_pkthdr
    marks equal the oracle's."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from libuinet_amd.frames import FrameBatch, mangle_headers, pkthdr_fields, split_headers

    frames = 0
    try:
        for t in range(max(1, TRIALS // 10)):
            rng = np.random.default_rng(50000 + BASE + t)
            u.set_tuning("host_threads", int(rng.choice([1, 3, 16])))
            u.set_tuning("walk_device", int(rng.integers(0, 4)))
            # batches of 2,048 frames and more take the device hook when their
            # mbufs are registered (cksum_hookdev.hip); smaller ones the host hook
            n = int(rng.choice([1, 2, int(rng.integers(1, 1500)), int(rng.integers(2048, 3000))]))
            l2 = bool(rng.integers(0, 2))
            l2len = -1 if l2 else 0
            ipv6 = float(rng.choice([0.0, 0.3, 1.0]))
            seed = int(rng.integers(0, 2**31))
            a = FrameBatch(n, seed=seed, l2=l2, ipv6=ipv6)
            b = FrameBatch(n, seed=seed, l2=l2, ipv6=ipv6)
            zc = bool(rng.integers(0, 2))
            mb = zc and bool(rng.integers(0, 2))  # mbufs registered: the GPU walks
            # a third of the trials cut headers across the first mbuf boundary
            sp = bool(rng.integers(0, 3) == 0)
            ss = int(rng.integers(0, 2**31))
            # a quarter make half their frames malformed (frames.mangle_headers)
            mg = float(rng.choice([0.0, 0.0, 0.0, 0.5]))
            ta, tb = (mangle_headers(a.tx, a, ss, mg), mangle_headers(b.tx, b, ss, mg)) if mg else (a.tx, b.tx)
            ta, tb = (split_headers(ta, ss), split_headers(tb, ss)) if sp else (ta, tb)
            if zc:
                u.register_host(a.arena)
            if mb:
                u.register_host(ta.mbufs)
            try:
                st_g = u.tx_offload(ta.heads, l2len)
            finally:
                if zc:
                    u.unregister_host(a.arena)
                if mb:
                    u.unregister_host(ta.mbufs)
            st_o = ora.tx_offload(tb.heads, l2len)
            ctx = (f"offload trial {t}: n={n} l2={l2} ipv6={ipv6} zero_copy={zc} mbufs={mb} "
                   f"split={sp} malformed={mg}")
            assert np.array_equal(st_g, st_o), ctx + " (TX status)"
            assert np.array_equal(a.arena, b.arena), ctx + " (TX bytes)"
            for x, y in zip(pkthdr_fields(ta), pkthdr_fields(tb)):
                assert np.array_equal(x, y), ctx + " (TX marks)"
            corrupt = float(rng.choice([0.0, 0.05, 0.5]))
            rs = int(rng.integers(0, 2**31))
            rx_a, arena_a, _ = a.rx(seed=rs, corrupt=corrupt)
            rx_b, _, _ = b.rx(seed=rs, corrupt=corrupt)
            if mg:
                rx_a, rx_b = mangle_headers(rx_a, a, ss + 2, mg), mangle_headers(rx_b, b, ss + 2, mg)
            if sp:
                rx_a, rx_b = split_headers(rx_a, ss + 1), split_headers(rx_b, ss + 1)
            if zc:
                u.register_host(arena_a)
            if mb:
                u.register_host(rx_a.mbufs)
            try:
                st_g = u.rx_offload(rx_a.heads, l2len)
            finally:
                if zc:
                    u.unregister_host(arena_a)
                if mb:
                    u.unregister_host(rx_a.mbufs)
            st_o = ora.rx_offload(rx_b.heads, l2len)
            assert np.array_equal(st_g, st_o), ctx + f" corrupt={corrupt} (RX status)"
            for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
                assert np.array_equal(x, y), ctx + f" corrupt={corrupt} (RX marks)"
            frames += n
            if t % 50 == 49:
                print(f"offload fuzz: {t + 1} trials", flush=True)
        print(f"offload fuzz: {max(1, TRIALS // 10)} trials, {frames} frames each way")
    finally:
        for k, v in HOST_DEFAULTS.items():
            u.set_tuning(k, v)
