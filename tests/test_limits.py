"""Size limits of the device API: chain segments may hold up to
2^32 - 1 bytes; spans are limited to UINET_CKSUM_MAX_SPAN bytes, which the
strided entry point enforces."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import aligned_empty, splitmix64_bytes

MAX_SPAN = 0x7FFFF000


def test_max_span_declared_and_enforced():
    from conftest import REPO
    import os

    text = open(os.path.join(REPO, "include", "uinet_cksum.h")).read()
    assert "#define UINET_CKSUM_MAX_SPAN 0x7ffff000u" in text
    p = 16  # never dereferenced: the check comes first
    assert u.lib().uinet_cksum_strided(p, MAX_SPAN, MAX_SPAN, None, p, 1, 0, None) == u.EINVAL
    assert u.lib().uinet_cksum_strided(p, 1 << 32, 0xFFFFFFFF, None, p, 1, 0, None) == u.EINVAL


@pytest.mark.gpu
def test_chain_segment_over_256_mib(torch_dev, ora):
    """One mbuf of 2^28 + 4099 bytes at an odd address, between short ones:
    its length no longer fits the 28 bits a packed (length << 4 | head) word
    kept, which summed only the first len mod 2^28 bytes."""
    torch = torch_dev
    big = (1 << 28) + 4099
    arena = aligned_empty(big + (1 << 16))
    splitmix64_bytes(arena.size, 4242, out=arena)
    # packet 0: 37 B -> the big mbuf -> 30 B -> 999 B, skip 7; packet 1: the big
    # mbuf alone, len and skip inside it
    seg_off = np.array([5, 101, 101 + big + 3, 101 + big + 40, 101], np.int64)
    seg_len = np.array([37, big, 30, 999, big], np.int64)
    pkt_seg = np.array([0, 4, 5], np.int64)
    length = np.array([int(seg_len[:4].sum()), big - 5], np.int64)
    skip = np.array([7, 3], np.int64)
    want = ora.chains(arena, seg_off, seg_len, pkt_seg, length=length, skip=skip)
    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).cuda()  # noqa: E731
    got = u.cksum_chains(d(arena, np.uint8), d(seg_off, np.int64), d(seg_len, np.int32),
                         d(pkt_seg, np.int32), length=d(length, np.int32),
                         skip=d(skip, np.int32), len_hint=int(seg_len.mean()))
    got = got.cpu().view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(got, want)
