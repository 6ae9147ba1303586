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
    """Every rank's plan object (ranks share the launcher's stdout, so two
    lines may run together)."""
    dec = json.JSONDecoder()
    out, i = [], stdout.find('{"rank"')
    while i >= 0:
        obj, end = dec.raw_decode(stdout, i)
        out.append(obj)
        i = stdout.find('{"rank"', end)
    return out


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_strided_api_only_for_strided_configs():
    """--api strided measures packets at a fixed stride (configs 2, 2rx, 2s,
    2su); asked of another config the bench stops instead of timing the span
    API under a strided label."""
    for cfg in ("3", "4", "5", "5tso"):
        r = _run(["--config", cfg, "--api", "strided", "--dry-run"])
        assert r.returncode != 0 and "--api strided" in r.stderr, (cfg, r.stderr[-500:])
    r = _run(["--config", "2su", "--api", "strided", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]


def test_gpus_n_spawns_n_ranks_with_config4_default():
    r = _run(["--gpus", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    plans = _plans(r.stdout)
    assert sorted(p["rank"] for p in plans) == [0, 1, 2]
    assert {p["world"] for p in plans} == {3}
    assert {p["config"] for p in plans} == {"4"}
    assert {p["packets_per_gpu"] for p in plans} == {2097152}


def test_rank_fields_gathered_over_gloo():
    """The N > 1 line's per-rank fields (ranks_kernel_ms, kernel_ms_max_rank,
    slowest_rank, step_ms, gather_exposed_ms, per_gpu_gbs_min) come from one
    all_gather of every rank's kernel times: rehearsed at world 2 over gloo
    with stand-in times (rank r: 0.4 + 0.01 r ms)."""
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    plans = _plans(r.stdout)
    assert len(plans) == 2
    for p in plans:
        f = p["rank_fields_rehearsal"]
        assert f["ranks_kernel_ms"] == [0.4, 0.41]
        assert f["kernel_ms_max_rank"] == 0.41 and f["slowest_rank"] == 1
        assert f["step_ms"] == 0.45 and f["gather_exposed_ms"] == 0.04
        assert f["per_gpu_gbs_min"] == round(3145728000 / 0.41e-3 / 1e9, 1)



def test_single_gpu_default_is_config2_without_launcher():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    (p,) = _plans(r.stdout)
    assert p == {"rank": 0, "local_rank": 0, "world": 1, "config": "2",
                 "packets_per_gpu": 1048576, "backend": None}


def _rank_procs(n, env_extra, args=("--dry-run",)):
    """n ranks of bench.py started directly (the launcher's env contract:
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), so each rank's own exit status
    and output are seen, not a launcher's."""
    port = str(__import__("bench").free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port}, **env_extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"),
                                       "--gpus", str(n), *args], env=env, cwd="/tmp",
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    return procs


def _watchdog_lines(stdout):
    return [json.loads(m) for m in re.findall(r"\{[^{}]*\"watchdog\"[^{}]*\}", stdout)]


def test_watchdog_ends_every_rank_of_a_stalled_run():
    """Rank 1 hangs on entering the plan phase (injected); rank 0 waits for it
    in the plan barrier.  Both must end non-zero within the deadline, each
    with one JSON line naming its phase and rank."""
    import time

    deadline = 6.0
    t0 = time.monotonic()
    procs = _rank_procs(2, {"UINET_BENCH_WATCHDOG_S": str(deadline), "UINET_BENCH_STALL": "1:plan"})
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:  # pragma: no cover - the failure under test
            for q in procs:
                q.kill()
            raise AssertionError("a rank outlived its watchdog")
        outs.append((p.returncode, o, e))
    took = time.monotonic() - t0
    for r, (rc, o, e) in enumerate(outs):
        assert rc != 0, (r, o, e[-2000:])
        lines = _watchdog_lines(o)
        assert len(lines) == 1, (r, o, e[-2000:])
        assert lines[0]["rank"] == r and lines[0]["phase"] == "plan", lines
        assert lines[0]["watchdog"] in ("deadline", "error"), lines
    stalled = _watchdog_lines(outs[1][1])[0]
    assert stalled["watchdog"] == "deadline" and outs[1][0] == 124
    assert stalled["phase_s"] >= deadline
    # the deadline bounds the run (plus interpreter and torch start-up)
    assert took < 90, took


def test_watchdog_quiet_on_a_healthy_run():
    procs = _rank_procs(2, {"UINET_BENCH_WATCHDOG_S": "60"})
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-2000:]
        assert not _watchdog_lines(o)
        assert len(_plans(o)) == 1
