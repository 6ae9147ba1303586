"""Multi-device entry points of the C ABI (include/uinet_cksum.h section 2e;
SURVEY.md 8e).  On a one-GPU box the device lists repeat
device 0 -- every shard still runs on its own host thread and stream, and the
gather goes through the same copy path -- and the gathered results must equal
the oracle over the whole batch."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes

from conftest import gpu_available


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_multi_no_device_and_bad_args():
    L = u.lib()
    a = aligned_empty(4096)
    ch = MbufChains.contiguous(a, [0], [100])
    devs = np.zeros(2, np.int32)
    ln = np.array([100], np.int32)
    sk = np.zeros(1, np.int32)
    out = np.zeros(1, np.uint16)
    p = lambda x: x.ctypes.data  # noqa: E731
    assert L.in_cksum_skip_batch_multi(p(devs), 0, p(ch.heads), p(ln), p(sk), p(out), 1) == u.EINVAL
    assert L.in_cksum_skip_batch_multi(p(devs), 2, None, p(ln), p(sk), p(out), 1) == u.EINVAL
    assert L.in_cksum_skip_batch_multi(p(devs), 2, p(ch.heads), p(ln), p(sk), p(out), 1) == u.ENODEV
    sh = (u.Shard * 1)(u.Shard(0, 1, 16, 16, 16, None, None))
    assert L.uinet_cksum_spans_multi(ctypes.addressof(sh), 1, 0, 0, 0, 16) == u.ENODEV
    assert L.uinet_cksum_spans_multi(None, 1, 0, 0, 0, 16) == u.EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("nshards", [1, 3, 8])
def test_spans_multi_gather(torch_dev, ora, nshards):
    torch = torch_dev
    rng = np.random.default_rng(nshards)
    arena = aligned_empty(4 << 20)
    splitmix64_bytes(arena.size, 99 + nshards, out=arena)
    n = 20000
    off = rng.integers(0, arena.size - 3000, n).astype(np.int64)
    ln = rng.integers(0, 3000, n).astype(np.int32)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    par = rng.integers(0, 2, n).astype(np.uint8)
    want = ora.spans(arena, off, ln, seed=seed, parity=par)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    base = d(arena)
    cuts = np.sort(rng.integers(0, n, nshards - 1))
    cuts = np.concatenate([[0], cuts, [n]])
    cuts[1] = cuts[0] if nshards > 2 else cuts[1]  # one empty shard when there are several
    shards = [dict(base=base, off=d(off[a:b]), length=d(ln[a:b]), seed=d(seed[a:b].view(np.int32)),
                   parity=d(par[a:b])) for a, b in zip(cuts[:-1], cuts[1:])]
    got = u.cksum_spans_multi(shards, root_device=0, len_hint=1500)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().view(torch.int16).numpy().view(np.uint16), want)
    # one shard per device (here: the one device) takes the in-process RCCL
    # gather; a device that appears twice takes the peer copies
    assert u.multi_last_gather() == (1 if nshards == 1 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [0, 1])
def test_spans_multi_rccl_single_device(torch_dev, ora, gather):
    """The RCCL branch of uinet_cksum_spans_multi on a one-device list (a
    communicator of one rank, the gather in place on the root) against the
    peer-copy branch (knob multi_gather=1), config-2 shaped, twice in a row
    (the second call reuses the cached communicator)."""
    torch = torch_dev
    arena = aligned_empty(1500 * 40000 + 64)
    splitmix64_bytes(arena.size, 7, out=arena)
    off = 1500 * np.arange(40000, dtype=np.int64)
    ln = np.full(40000, 1500, np.int32)
    want = ora.spans(arena, off, ln)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    sh = [dict(base=d(arena), off=d(off), length=d(ln))]
    u.set_tuning("multi_gather", gather)
    try:
        for _ in range(2):
            got = u.cksum_spans_multi(sh, root_device=0, len_hint=1500)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(got.cpu().view(torch.int16).numpy().view(np.uint16), want)
            assert u.multi_last_gather() == (1 if gather == 0 else 0)
    finally:
        u.set_tuning("multi_gather", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0]])
def test_host_batch_multi(torch_dev, ora, devices):
    from libuinet_amd.workloads import build_config3

    lay = build_config3(30000, seed=5)
    ch = MbufChains(lay["arena"], lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
    want = ora.skip_batch(ch.heads, lay["lens"], 20)
    np.testing.assert_array_equal(u.in_cksum_skip_batch_multi(devices, ch.heads, lay["lens"], 20),
                                  want)
    u.register_host(lay["arena"])  # zero-copy shards: every byte in registered memory
    try:
        got = u.in_cksum_skip_batch_multi(devices, ch.heads, lay["lens"], 20)
        np.testing.assert_array_equal(got, want)
        # the mbufs registered too: every shard's chains walked by its device
        u.register_host(ch.mbufs)
        u.set_tuning("span_fast", 0)
        try:
            w0 = u.host_cpu()["device_walks"]
            got = u.in_cksum_skip_batch_multi(devices, ch.heads, lay["lens"], 20)
            if len(devices) == 1:  # one shard: it runs on the calling thread
                assert u.host_cpu()["device_walks"] == w0 + 1
        finally:
            u.set_tuning("span_fast", 1)
            u.unregister_host(ch.mbufs)
    finally:
        u.unregister_host(lay["arena"])
    np.testing.assert_array_equal(got, want)
