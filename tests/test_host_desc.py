"""Zero-copy host-mbuf batches write packed 6-B chain descriptors (u32
offset, u16 length: the uinet_cksum_chains32 kernels) when every registered
byte lies within 4 GiB and no piece exceeds 65535 B, and 12-B wide ones for
a pipeline group holding a longer piece.  Both against the oracle's
reference-shaped walk (in_cksum.c:193-232)."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains

from test_gpu_parity import rand_arena, random_chain_layout

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("host_threads", [1, 4])
@pytest.mark.parametrize("long_every", [0, 7000, 400])
def test_zero_copy_packed_and_wide_groups(torch_dev, ora, host_threads, long_every):
    rng = np.random.default_rng(500 + host_threads + long_every)
    arena = rand_arena(1 << 23, 500)
    seg_off, seg_len, pkt_seg = random_chain_layout(rng, 30000, arena.size - 100000, max_segs=10)
    if long_every:  # pieces past the u16 limit in some groups
        k = np.arange(0, seg_len.size, long_every)
        seg_len[k] = rng.integers(65536, 90000, k.size)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    skip = rng.integers(0, 30, ch.n).astype(np.int32)
    want = ora.skip_batch(ch.heads, tot, skip)
    u.set_tuning("host_threads", host_threads)
    u.register_host(arena)
    try:
        np.testing.assert_array_equal(u.in_cksum_skip_batch(ch.heads, tot, skip), want)
    finally:
        u.unregister_host(arena)
        u.set_tuning("host_threads", 16)
