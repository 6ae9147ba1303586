"""bench.py's own multi-rank path on the GPU.

* ``bench.py --gpus 2`` with no launcher and UINET_BENCH_BACKEND=gloo: the
  script spawns two ranks (both on cuda:0 of a one-GPU box), each folds its
  full config-4 shard of 2,097,152 x 1500-B packets with the span kernel, and
  the per-step gather brings every rank's u16 results to rank 0.  The saved
  array must equal the oracle over each rank's bytes, byte for byte.
* ``torch.distributed.run --nproc-per-node 1 bench.py --gpus 1`` on the
  default ``nccl`` backend: init_process_group("nccl") and the RCCL gather
  (ResultGather with device buffers) run, and the gathered array is checked
  the same way.

Both runs keep the bench's own reference check on (its cpu_baseline leg): the
JSON line must carry ``bit_identical: true`` over every rank's packets.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(cmd, env_extra, timeout):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _want_config2(n: int, world: int) -> np.ndarray:
    """Oracle over every rank's config-2 arena (the same device generator the
    bench uses, copied to the host), concatenated in rank order."""
    import torch

    import oracle
    import libuinet_amd.workloads as W

    ora = oracle.Oracle()
    parts = []
    for r in range(world):
        w = W.config2_device(n, rank=r)
        host = w["arena"].cpu().numpy()
        del w
        torch.cuda.empty_cache()
        parts.append(ora.spans(host, 1500 * np.arange(n, dtype=np.int64), 1500))
    return np.concatenate(parts)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_gpus2_config4_full_shard_gloo(tmp_path, torch_dev):
    path = str(tmp_path / "res.npy")
    d = _bench([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
                "--save-results", path],
               {"UINET_BENCH_BACKEND": "gloo"}, timeout=400)
    assert d["n_gpus"] == 2
    assert d["bit_identical"] is True and d["parity"]["packets"] == 2 * 2097152
    assert d["config"]["workload"].startswith("config4: 4,194,304 x 1500 B")
    assert d["config"]["packets_per_gpu"] == 2097152
    # every rank's kernel, not only rank 0's
    rk = d["ranks"]
    assert len(rk["ranks_kernel_ms"]) == 2 and all(x > 0 for x in rk["ranks_kernel_ms"])
    assert rk["kernel_ms_max_rank"] == max(rk["ranks_kernel_ms"])
    assert rk["slowest_rank"] in (0, 1)
    assert rk["step_ms"] == round(d["ms_per_step"], 4)
    assert abs(rk["gather_exposed_ms"] - (rk["step_ms"] - rk["kernel_ms_max_rank"])) < 1e-3
    assert rk["per_gpu_gbs_min"] > 0
    got = np.load(path)
    assert got.dtype == np.uint16 and got.size == 2 * 2097152
    np.testing.assert_array_equal(got, _want_config2(2097152, 2))


def test_bench_nccl_world1_rccl_gather(tmp_path, torch_dev):
    path = str(tmp_path / "res.npy")
    n = 65536
    d = _bench([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node=1", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
                "bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1", "--packets", str(n),
                "--save-results", path],
               {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}, timeout=300)
    assert d["n_gpus"] == 1
    assert d["bit_identical"] is True
    assert "RCCL gather" in d["config"]["parallelism"]
    assert d["config"]["launcher"] == "torch.distributed.run"
    got = np.load(path)
    np.testing.assert_array_equal(got, _want_config2(n, 1))


def test_bench_n1_host_resident_cpu_line(torch_dev):
    """The N = 1 line folds its batch once more as host mbufs in registered
    memory and reports the host CPU that cost, beside the reference's
    one-thread pass; bit-identical to the timed step.  One mbuf per packet
    takes the single-mbuf span path, with the mbufs registered or not."""
    d = _bench([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--packets", "65536"],
               {}, timeout=300)
    h = d["host_resident_cpu"]
    assert "error" not in h, h
    assert h["bit_identical"] is True and h["path"] == "single-mbuf spans"
    b = h["bytes_only"]
    assert b["bit_identical"] is True and b["path"] == "single-mbuf spans"
    assert b["wall_ms"] > 0 and b["host_cpu_us_per_1k_pkts"] > 0
    assert h["wall_ms"] > 0 and h["host_cpu_us_per_1k_pkts"] > 0
    assert h["reference_1thread_cpu_us_per_1k_pkts"] > 0
    # the link's own DMA rate, measured in the same run, and the batch against it
    assert h["link_h2d_gbs"] and h["link_h2d_gbs"] > 1.0
    assert 0 < h["frac_of_link"] < 1.5
