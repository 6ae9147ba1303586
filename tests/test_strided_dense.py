"""The dense strided kernel (k_strided_dense, cksum_spans.hip): small strided
packets laid (nearly) back to back, read as one run of aligned chunks per
wave and split at the packet boundaries.  Against the oracle's span fold
(oracle/cksum_oracle.c, after /root/reference/sys/amd64/amd64/in_cksum.c
:91-170,193-232) on every shape the dispatcher sends it: strides 32-256,
lengths down to 3/4 of the stride, every start alignment, odd strides
(packets alternating between even and odd start addresses), ragged counts,
seeds, UDP / no-complement flags, grids small enough for many steps per wave.

CPU: the kernel's slot arithmetic (a multiply by ceil(2^20 / stride) for
floor(r / stride), r < 1024) is exact on its whole domain."""
from __future__ import annotations

import numpy as np
import pytest

import libuinet_amd as u

from test_gpu_parity import dev, host16, rand_arena


def test_slot_division_exact():
    r = np.arange(1024, dtype=np.int64)
    for s in range(32, 257):
        recip = ((1 << 20) + s - 1) // s
        np.testing.assert_array_equal((r * recip) >> 20, r // s)


@pytest.fixture(scope="module")
def torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert u.device_ok(), "device is not gfx950"
    return torch


# (stride, len); the dispatcher sends these to the dense kernel when base or
# stride is off 16-B alignment (bases 1, 2, 3, 7, 14, 15; odd strides), to
# k_spans_quad / k_spans otherwise (base 0 with a multiple-of-16 stride)
SHAPES = [(64, 64), (64, 60), (64, 48), (32, 32), (32, 24), (33, 33), (65, 64), (80, 64),
          (96, 90), (127, 100), (128, 128), (200, 150), (256, 256), (256, 192), (255, 254)]


@pytest.mark.gpu
@pytest.mark.parametrize("bpc", [0, 1])
def test_strided_dense_shapes(torch_dev, ora, bpc):
    torch = torch_dev
    rng = np.random.default_rng(7700 + bpc)
    arena = rand_arena(8 << 20, 77)
    d_arena = dev(torch, arena)
    u.set_tuning("blocks_per_cu", bpc)
    try:
        for stride, length in SHAPES:
            for base in (0, 1, 2, 3, 7, 14, 15):
                for n in (1, 2, 14, 15, 16, 31, 1000, 20011):
                    n = min(n, (arena.size - base - length) // stride)
                    seed = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                    flags = int(rng.choice([0, u.F_UDP, u.F_NO_COMPLEMENT]))
                    use_seed = rng.random() < 0.5
                    got = u.cksum_strided(d_arena[base:], stride, length, n,
                                          seed=dev(torch, seed.view(np.int32)) if use_seed else None,
                                          flags=flags)
                    off = base + stride * np.arange(n, dtype=np.int64)
                    want = ora.spans(arena, off, np.full(n, length, np.int64),
                                     seed if use_seed else None, None, flags)
                    np.testing.assert_array_equal(host16(got), want,
                                                  err_msg=f"{stride=} {length=} {base=} {n=}")
    finally:
        u.set_tuning("blocks_per_cu", 0)


@pytest.mark.gpu
def test_strided_dense_full_2s(torch_dev, ora):
    """The benchmarked strided small-packet batches (2s / 2su: 16,777,216 x
    64 B at stride 64, +0 / +2) and all-0x00 / all-0xff packets."""
    import libuinet_amd.workloads as Wl

    torch = torch_dev
    n = 1 << 24
    for base in (0, 2):
        w = Wl.config2_device(n, stride=64, length=64, base=base)
        got = u.cksum_strided(w["arena"][base:], 64, 64, n)
        host = w["arena"].cpu().numpy()
        want = ora.spans(host, base + 64 * np.arange(n, dtype=np.int64), np.full(n, 64, np.int64))
        np.testing.assert_array_equal(host16(got), want)
        del w
    for fill in (0x00, 0xFF):
        a = torch.full((64 * 5000 + 64,), fill, dtype=torch.uint8, device="cuda")
        got = host16(u.cksum_strided(a[3:], 64, 64, 5000))
        assert (got == (0xFFFF if fill == 0 else 0)).all()
