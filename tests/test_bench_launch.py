"""bench.py's launch contract on CPU: ``--gpus N`` yields N ranks (spawned
through torch.distributed.run when no launcher set WORLD_SIZE), a WORLD_SIZE
that disagrees with --gpus is an error, and the distributed default workload
is config 4 (2,097,152 packets per GPU).  ``--dry-run`` stops every rank after
the gloo rendezvous, before anything touches a GPU."""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout, cwd="/tmp")


def _plans(stdout):
    return [json.loads(m) for m in re.findall(r"\{[^{}]*\"rank\"[^{}]*\}", stdout)]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_gpus_n_spawns_n_ranks_with_config4_default():
    r = _run(["--gpus", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    plans = _plans(r.stdout)
    assert sorted(p["rank"] for p in plans) == [0, 1, 2]
    assert {p["world"] for p in plans} == {3}
    assert {p["config"] for p in plans} == {"4"}
    assert {p["packets_per_gpu"] for p in plans} == {2097152}


def test_single_gpu_default_is_config2_without_launcher():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    (p,) = _plans(r.stdout)
    assert p == {"rank": 0, "local_rank": 0, "world": 1, "config": "2",
                 "packets_per_gpu": 1048576, "backend": None}
