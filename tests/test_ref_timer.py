"""The reference timer behind bench.py's cpu_baseline (oracle/ref_harness.c).

A pass is max(worker end) - min(worker start), stamped by the workers
themselves, so the measuring thread's own scheduling never shortens it
(main-thread stamps read 1.3-2.3 TB/s passes on a
~1.2 TB/s host).  Checked with more workers than this process may run at
once, where a late-scheduled stamping thread used to matter most."""
from __future__ import annotations

import os

import numpy as np

from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes


def _batch(n=4096, length=1500):
    a = aligned_empty(n * length)
    splitmix64_bytes(a.size, 77, out=a)
    return a, MbufChains.contiguous(a, length * np.arange(n), length)


def _oversubscribed() -> int:
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        ncpu = os.cpu_count() or 1
    return min(4 * ncpu, 256)


def test_pass_covers_every_worker(ref):
    a, ch = _batch()
    nt = _oversubscribed()
    t, out, st = ref.time_skip(ch.heads, 1500, 0, nthreads=nt, reps=1, stamps=True)
    assert st.shape == (nt, 2)
    assert np.all(st[:, 1] >= st[:, 0])
    # the pass is the union of the workers' spans, never shorter than any one
    assert t >= float(np.max(st[:, 1] - st[:, 0]))
    assert abs(t - (st[:, 1].max() - st[:, 0].min())) < 1e-9
    # and the results are the reference's, whatever the split
    np.testing.assert_array_equal(out, ref.skip_batch(ch.heads, 1500, 0))


def test_pseudo_pass_covers_every_worker(ref):
    a, ch = _batch(n=1024, length=9000)
    nt = _oversubscribed()
    t, out, st = ref.time_pseudo(ch.heads, 8980, 20, 0x0a000001, 0x0a000002, 6, nthreads=nt,
                                 reps=1, stamps=True)
    assert t >= float(np.max(st[:, 1] - st[:, 0]))
    np.testing.assert_array_equal(
        out, ref.pseudo_header_batch(ch.heads, 8980, 20, 0x0a000001, 0x0a000002, 6))


def test_read_pass_covers_every_worker(ref):
    a, _ = _batch()
    nt = _oversubscribed()
    t, st = ref.time_read(a, nthreads=nt, reps=1, stamps=True)
    assert t > 0 and t >= float(np.max(st[:, 1] - st[:, 0]))
    assert abs(t - (st[:, 1].max() - st[:, 0].min())) < 1e-9


def test_best_of_reps_is_a_pass(ref):
    """reps > 1 returns the best pass; it can only be faster than one pass
    measured the same way, never faster than the read of the same bytes
    would allow by more than noise."""
    a, ch = _batch(n=2048)
    t1 = ref.time_skip(ch.heads, 1500, 0, nthreads=2, reps=1)[0]
    t3 = ref.time_skip(ch.heads, 1500, 0, nthreads=2, reps=3)[0]
    assert 0 < t3 <= t1 * 1.5
