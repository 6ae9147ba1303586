"""The driver hooks' header parse on the CPU (no GPU): offload_parse.h through
the host hook's own view (offload_hostview.h), built with g++ from
tests/native/parse_host.cpp, makes each frame's two checksum jobs and its plan;
the oracle folds the jobs and the verdicts are written the way the hooks write
them (cksum_offload.hip's apply steps, restated below).  Statuses, stored sums
and m_pkthdr marks must equal the oracle's own hooks (oracle/offload_oracle.c)
on the same frames -- IPv4 with options, IPv6 with extension headers, with and
without the link header, corrupted frames, and headers cut across the first
mbuf boundary.  The GPU tests cover the same parse on the device view."""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from libuinet_amd.frames import FrameBatch, mangle_headers, pkthdr_fields, split_headers

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "libuinet_amd", "csrc")

RX_IP_OK, RX_L4, RX_L4_OK = 0x02, 0x04, 0x08
TX_L4, TX_IP, TX_L4_LOST = 0x01, 0x02, 0x04
CSUM_IP = 0x1
CSUM_IP_CHECKED, CSUM_IP_VALID, CSUM_DATA_VALID, CSUM_PSEUDO_HDR = 0x100, 0x200, 0x400, 0x800
M_PKTHDR = 0x2


@pytest.fixture(scope="module")
def parse_lib(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    so = tmp_path_factory.mktemp("parse") / "libparse_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-shared", "-fPIC",
                    f"-I{CSRC}", f"-I{os.path.join(REPO, 'include')}",
                    os.path.join(HERE, "native", "parse_host.cpp"), "-o", str(so)], check=True)
    return ctypes.CDLL(str(so))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _jobs(n):
    return (np.zeros(2 * n, np.uint64), np.zeros(2 * n, np.int32), np.zeros(2 * n, np.int32),
            np.zeros(2 * n, np.uint32))


def _fold(x):
    while x >> 16:
        x = (x & 0xFFFF) + (x >> 16)
    return x


def _results(ora, jm, jl, js, jd):
    """Each job's u16 as the engine computes it: ~fold(sum + seed), by the oracle's
    in_cksum_skip (which returns ~fold(sum))."""
    res = np.zeros(jm.size, np.int64)
    live = np.flatnonzero(jm != 0)
    if live.size:
        r = ora.skip_batch(jm[live], jl[live], js[live]).astype(np.int64)
        res[live] = [~_fold((~int(a) & 0xFFFF) + int(s)) & 0xFFFF for a, s in zip(r, jd[live])]
    return res


def _rx_apply(ch, st, ip_job, l4_job, res):
    """cksum_offload.hip's RX apply (ip_input.c:460-471, tcp_input.c:697-718)."""
    first = ch.pkt_seg[:-1]
    for k in range(ch.n):
        if ch.heads[k] == 0:
            continue
        f = int(first[k])
        hdr = (int(ch.mbufs["m_flags"][f]) & M_PKTHDR) != 0
        fl = int(ch.mbufs["csum_flags"][f])
        if ip_job[k]:
            ok = res[2 * k] == 0
            st[k] |= RX_IP_OK if ok else 0
            fl |= CSUM_IP_CHECKED | (CSUM_IP_VALID if ok else 0)
        if l4_job[k]:
            r = int(res[2 * k + 1])
            st[k] |= RX_L4 | (RX_L4_OK if r == 0 else 0)
            fl |= CSUM_DATA_VALID | CSUM_PSEUDO_HDR
            if hdr:
                ch.mbufs["csum_data"][f] = r ^ 0xFFFF
        if hdr and (ip_job[k] or l4_job[k]):
            ch.mbufs["csum_flags"][f] = fl
    return st


def _put16(arena, addr, c):
    o = int(addr) - arena.ctypes.data
    arena[o] = c & 0xFF
    arena[o + 1] = c >> 8


def _tx_apply(ch, arena, st, ip_job, l4_job, udp, l4_store, ip_l3, clear, res):
    """cksum_offload.hip's TX apply (ip_output.c:665-667,953-976)."""
    first = ch.pkt_seg[:-1]
    for k in range(ch.n):
        f = int(first[k])
        if not (ip_job[k] or l4_job[k]):
            continue
        fl = int(ch.mbufs["csum_flags"][f])
        data = int(ch.mbufs["m_data"][f])
        if l4_job[k]:
            c = int(res[2 * k + 1])
            if udp[k] and c == 0:
                c = 0xFFFF
            if l4_store[k] + 2 > int(ch.mbufs["m_len"][f]):
                st[k] |= TX_L4_LOST
            else:
                _put16(arena, data + int(l4_store[k]), c)
                st[k] |= TX_L4
            fl &= ~int(clear[k])
        if ip_job[k]:
            _put16(arena, data + int(ip_l3[k]) + 10, int(res[2 * k]))
            st[k] |= TX_IP
            fl &= ~CSUM_IP
        ch.mbufs["csum_flags"][f] = fl
    return st


CASES = [  # (seed, ipv6 share, link header, cut headers across mbufs, malformed share)
    (31, 0.0, True, False, 0.0), (32, 0.3, True, False, 0.0), (33, 1.0, False, False, 0.0),
    (34, 0.3, True, True, 0.0), (35, 0.5, False, True, 0.0),
    (36, 0.0, True, False, 0.6), (37, 0.5, True, True, 0.6), (38, 1.0, False, True, 0.6)]


@pytest.mark.parametrize("seed,ipv6,l2,cut,bad", CASES)
def test_host_parse_matches_oracle_hooks(parse_lib, ora, seed, ipv6, l2, cut, bad):
    n = 1200
    l2len = -1 if l2 else 0
    a = FrameBatch(n, seed=seed, l2=l2, ipv6=ipv6)
    b = FrameBatch(n, seed=seed, l2=l2, ipv6=ipv6)
    ta, tb = (split_headers(a.tx, seed), split_headers(b.tx, seed)) if cut else (a.tx, b.tx)
    if bad:  # malformed headers, cut chains, empty mbufs (frames.mangle_headers)
        ta, tb = mangle_headers(ta, a, seed + 3, bad), mangle_headers(tb, b, seed + 3, bad)

    # TX
    jm, jl, js, jd = _jobs(n)
    ip_job, l4_job, udp, st = (np.zeros(n, np.uint8) for _ in range(4))
    l4_store, ip_l3, clear = (np.zeros(n, np.int32) for _ in range(3))
    heads = np.ascontiguousarray(ta.heads, np.uint64)
    parse_lib.parse_tx(_ptr(heads), n, l2len, _ptr(jm), _ptr(jl), _ptr(js), _ptr(jd), _ptr(ip_job),
                       _ptr(l4_job), _ptr(udp), _ptr(l4_store), _ptr(ip_l3), _ptr(clear), _ptr(st))
    res = _results(ora, jm, jl, js, jd)
    st = _tx_apply(ta, a.arena, st, ip_job, l4_job, udp, l4_store, ip_l3, clear, res)
    want = ora.tx_offload(tb.heads, l2len)
    assert np.array_equal(st, want), np.flatnonzero(st != want)[:8]
    assert np.array_equal(a.arena, b.arena)
    for x, y in zip(pkthdr_fields(ta), pkthdr_fields(tb)):
        assert np.array_equal(x, y)

    # RX over the transmitted frames, some corrupted
    rx_a, _, _ = a.rx(seed=seed + 1, corrupt=0.1)
    rx_b, _, _ = b.rx(seed=seed + 1, corrupt=0.1)
    if bad:
        rx_a, rx_b = mangle_headers(rx_a, a, seed + 4, bad), mangle_headers(rx_b, b, seed + 4, bad)
    if cut:
        rx_a, rx_b = split_headers(rx_a, seed + 2), split_headers(rx_b, seed + 2)
    jm, jl, js, jd = _jobs(n)
    ip_job, l4_job, st = (np.zeros(n, np.uint8) for _ in range(3))
    heads = np.ascontiguousarray(rx_a.heads, np.uint64)
    parse_lib.parse_rx(_ptr(heads), n, l2len, _ptr(jm), _ptr(jl), _ptr(js), _ptr(jd), _ptr(ip_job),
                       _ptr(l4_job), _ptr(st))
    res = _results(ora, jm, jl, js, jd)
    st = _rx_apply(rx_a, st, ip_job, l4_job, res)
    want = ora.rx_offload(rx_b.heads, l2len)
    assert np.array_equal(st, want), np.flatnonzero(st != want)[:8]
    for x, y in zip(pkthdr_fields(rx_a), pkthdr_fields(rx_b)):
        assert np.array_equal(x, y)
    assert (want & RX_L4).any() and (want & RX_L4_OK).any()  # the sums did run


def test_host_parse_fragmented_capture(parse_lib, ora, pcap_frames):
    """The reference's capture re-chained into random 1-256-B fragments
    (SURVEY.md section 4's KAT): the shared parse's jobs, folded by the oracle,
    verify every TCP frame to 0 -- the same marks as the oracle's RX hook."""
    from test_offload import _pcap_fragmented

    for seed in (5, 6):
        rx, _ = _pcap_fragmented(pcap_frames, seed)
        rx_b, _ = _pcap_fragmented(pcap_frames, seed)
        n = rx.n
        jm, jl, js, jd = _jobs(n)
        ip_job, l4_job, st = (np.zeros(n, np.uint8) for _ in range(3))
        heads = np.ascontiguousarray(rx.heads, np.uint64)
        parse_lib.parse_rx(_ptr(heads), n, -1, _ptr(jm), _ptr(jl), _ptr(js), _ptr(jd),
                           _ptr(ip_job), _ptr(l4_job), _ptr(st))
        st = _rx_apply(rx, st, ip_job, l4_job, _results(ora, jm, jl, js, jd))
        want = ora.rx_offload(rx_b.heads)
        assert np.array_equal(st, want)
        assert ((want & 0x0F) == 0x0F).sum() >= 113
