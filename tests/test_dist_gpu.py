"""N>1 on the GPU: the same chained batch sharded over
1, 2 and 4 ranks -- byte-balanced packet ranges, each rank folding its range
with the engine's chain kernel on the GPU, one gather of the u16 results to
rank 0 -- must give byte-identical results, equal to the oracle.  On a
one-GPU box every rank shares cuda:0 and the gather runs over gloo; the
8-GPU runs use the same code over RCCL (bench.py, dist.py)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_PKT = 20000


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _layout():
    from libuinet_amd.workloads import build_config3

    return build_config3(N_PKT, seed=21)


def _worker(rank, world, port, result_path):
    import torch
    import torch.distributed as dist

    import libuinet_amd as u
    from libuinet_amd.dist import gather_results, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        lay = _layout()
        b = shard_bounds(N_PKT, world, lay["lens"])
        lo, hi = int(b[rank]), int(b[rank + 1])
        s0, s1 = int(lay["pkt_seg"][lo]), int(lay["pkt_seg"][hi])
        # the rank's shard: its packets' segment descriptors, rebased
        dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).cuda()  # noqa: E731
        out = u.cksum_chains(dev(lay["arena"], np.uint8), dev(lay["seg_off"][s0:s1], np.int64),
                             dev(lay["seg_len"][s0:s1], np.int32),
                             dev(lay["pkt_seg"][lo:hi + 1] - s0, np.int32),
                             length=dev(lay["lens"][lo:hi], np.int32),
                             skip=dev(lay["skip"][lo:hi], np.int32), len_hint=lay["mean_seg"])
        torch.cuda.synchronize()
        got = gather_results(out.view(torch.int16), np.diff(b))
        if rank == 0:
            np.save(result_path, got.cpu().numpy().view(np.uint16))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def want():
    import oracle

    lay = _layout()
    return oracle.Oracle().chains(lay["arena"], lay["seg_off"], lay["seg_len"], lay["pkt_seg"],
                                  length=lay["lens"], skip=lay["skip"])


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_chains_gather_gpu(tmp_path, want, world):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp

    path = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), path), nprocs=world, join=True)
    np.testing.assert_array_equal(np.load(path), want)
