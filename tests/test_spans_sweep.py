"""Small packets through the span API whose 64-packet super-steps lie in one
dense address range (k_spans_quad's address sweep, cksum_device.h): packets
back to back at every alignment, 0-7-B gaps, empty and 1-byte packets,
lengths up to the sweep's 16-KiB limit, seeds, parity bytes, UDP and
no-complement flags, wide and packed descriptors, batches whose dense and
scattered super-steps alternate, and ragged batch ends.  Every result against
the oracle's span fold (oracle/cksum_oracle.c after
/root/reference/sys/amd64/amd64/in_cksum.c:91-170,193-276)."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import dev, host16, rand_arena

pytestmark = pytest.mark.gpu


def dense_spans(rng, n, arena_size, max_len=100, base=0, scatter_every=0):
    ln = rng.integers(0, max_len + 1, n)
    ln = np.where(rng.random(n) < 0.05, rng.choice([0, 1, 2, 15, 16, 17], n), ln)
    gaps = rng.integers(0, 8, n)
    off = base + np.cumsum(ln + gaps) - ln - gaps
    if scatter_every:  # every k-th block of 64 packets scattered over the arena
        blk = (np.arange(n) // 64) % scatter_every == scatter_every - 1
        off[blk] = rng.integers(0, arena_size - max_len - 1, int(blk.sum()))
    assert off.max() + max_len < arena_size
    return off.astype(np.int64), ln.astype(np.int64)


def run(torch, arena, off, ln, packed, seed=None, par=None, flags=0, hint=64):
    if packed:
        o, l_ = u.pack_segments(off, ln)
        o, l_ = dev(torch, o), dev(torch, l_)
    else:
        o, l_ = dev(torch, off), dev(torch, ln.astype(np.int32))
    return host16(u.cksum_spans(dev(torch, arena), o, l_,
                                seed=None if seed is None else dev(torch, seed.view(np.int32)),
                                parity=None if par is None else dev(torch, par),
                                flags=flags, len_hint=hint))


@pytest.mark.parametrize("base", [0, 1, 2, 14])
@pytest.mark.parametrize("scatter", [0, 3])
def test_dense_small_spans(torch_dev, ora, base, scatter):
    torch = torch_dev
    rng = np.random.default_rng(15000 + 10 * base + scatter)
    arena = rand_arena(1 << 22, 150)
    n = 30000 + base  # ragged: the last super-step is partial
    off, ln = dense_spans(rng, n, arena.size, base=base, scatter_every=scatter)
    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    par = rng.integers(0, 2, n).astype(np.uint8)
    for packed in (False, True):
        np.testing.assert_array_equal(run(torch, arena, off, ln, packed), ora.spans(arena, off, ln))
        for flags in (0, u.F_UDP, u.F_NO_COMPLEMENT):
            np.testing.assert_array_equal(
                run(torch, arena, off, ln, packed, seed, par, flags),
                ora.spans(arena, off, ln, seed, par, flags))


def test_dense_spans_extremes(torch_dev, ora):
    """All-0x00 / all-0xff bytes, every span empty, 1-B spans, spans of up to
    16,368 B (the sweep's limit is 1,024 chunks: longer ones take the quads),
    and a super-step whose spans run backwards (the quads)."""
    torch = torch_dev
    rng = np.random.default_rng(15100)
    from libuinet_amd.mbuf import aligned_empty

    for fill in (0x00, 0xFF):
        arena = aligned_empty(1 << 21)
        arena[:] = fill
        off, ln = dense_spans(rng, 8000, arena.size, base=3)
        np.testing.assert_array_equal(run(torch, arena, off, ln, False), ora.spans(arena, off, ln))
    arena = rand_arena(1 << 24, 151)
    n = 640
    ln = np.zeros(n, np.int64)
    ln[64:128] = 1
    ln[128:192] = rng.integers(16300, 16369, 64)
    ln[192:256] = rng.integers(16369, 17000, 64)  # over the limit: quads
    ln[256:] = rng.integers(0, 80, n - 256)
    off = np.cumsum(ln) - ln + 5
    off[320:384] = off[320:384][::-1].copy()  # backwards: quads
    np.testing.assert_array_equal(run(torch, arena, off, ln, False), ora.spans(arena, off, ln))
    np.testing.assert_array_equal(run(torch, arena, off, ln, False, hint=1500),
                                  ora.spans(arena, off, ln))
