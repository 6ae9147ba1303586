"""N>1 path on CPU: byte-balanced sharding + the single gather of 16-bit
results, world_size 2 over gloo (the GPU runs use the same code over RCCL)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from libuinet_amd.dist import shard_bounds, shard_range


def test_shard_bounds_equal_counts():
    for n, w in ((10, 3), (1 << 20, 8), (7, 8), (0, 2)):
        b = shard_bounds(n, w)
        assert b[0] == 0 and b[-1] == n and (np.diff(b) >= 0).all()
        assert np.diff(b).max() - np.diff(b).min() <= 1


def test_shard_bounds_by_bytes():
    rng = np.random.default_rng(0)
    lens = rng.choice([64, 576, 1500], 100000)
    b = shard_bounds(lens.size, 8, lens)
    per = np.add.reduceat(lens, b[:-1])
    assert b[-1] == lens.size and (np.diff(b) > 0).all()
    assert per.max() / per.min() < 1.01


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_path):
    import torch
    import torch.distributed as dist

    import oracle
    from libuinet_amd.dist import gather_results
    from libuinet_amd.mbuf import aligned_empty, splitmix64_bytes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        n = 5000
        lens = rng.choice([64, 576, 1500], n)
        off = np.concatenate([[0], np.cumsum(lens)[:-1]])
        arena = aligned_empty(int(lens.sum()) + 64)
        splitmix64_bytes(arena.size, 9, out=arena)
        b = shard_bounds(n, world, lens)
        lo, hi = int(b[rank]), int(b[rank + 1])
        # per-rank fold (the oracle stands in for the GPU on this CPU test)
        local = oracle.Oracle().spans(arena, off[lo:hi], lens[lo:hi])
        got = gather_results(torch.from_numpy(local.view(np.int16)), np.diff(b))
        if rank == 0:
            want = oracle.Oracle().spans(arena, off, lens)
            np.save(result_path, np.stack([got.view(torch.int16).numpy().view(np.uint16), want]))
    finally:
        dist.destroy_process_group()


def test_gather_world2_gloo(tmp_path):
    import torch.multiprocessing as mp

    path = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    got, want = np.load(path)
    np.testing.assert_array_equal(got, want)


def test_shard_range_matches_bounds():
    b = shard_bounds(1001, 4)
    assert [shard_range(1001, r, 4) for r in range(4)] == [(int(b[r]), int(b[r + 1])) for r in range(4)]


def _worker_async(rank, world, port, result_path):
    import torch
    import torch.distributed as dist

    from libuinet_amd.dist import ResultGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts = [3, 5, 4][:world]
        rg = ResultGather(counts, "cpu")
        got = []
        for step in range(5):  # the bench's double-buffered pattern
            slot = step & 1
            rg.wait(slot)
            local = torch.arange(counts[rank], dtype=torch.int16) + 100 * rank + 1000 * step
            rg.start(local, slot)
            if step >= 1:
                prev = (step - 1) & 1
                rg.wait(prev)
                if rank == 0:
                    got.append(rg.result(prev).numpy().copy())
        rg.wait_all()
        if rank == 0:
            got.append(rg.result(4 & 1).numpy().copy())
            np.save(result_path, np.stack(got))
    finally:
        dist.destroy_process_group()


def test_async_result_gather_world3_gloo(tmp_path):
    import torch.multiprocessing as mp

    path = str(tmp_path / "res.npy")
    mp.spawn(_worker_async, args=(3, _free_port(), path), nprocs=3, join=True)
    got = np.load(path)
    for step in range(5):
        want = np.concatenate([np.arange(c) + 100 * r + 1000 * step
                               for r, c in enumerate([3, 5, 4])])
        np.testing.assert_array_equal(got[step], want)
