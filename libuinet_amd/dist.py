"""Multi-GPU sharding of packet batches (one process per GPU).

The checksum has no cross-packet term, so a batch is cut into
contiguous packet ranges -- balanced by bytes when lengths vary -- every rank
folds its range on its own GPU with no data-path collective, and the one
exchange step is a single gather of the 16-bit results to the root over RCCL
(torch.distributed "nccl" is RCCL on ROCm; gloo on CPU in the tests).
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n: int, world: int, weights=None) -> np.ndarray:
    """Packet-index bounds ``b`` (world + 1 entries) so rank r owns
    ``[b[r], b[r+1])``: equal counts, or equal ``weights`` (bytes) sums."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if weights is None:
        return (np.arange(world + 1, dtype=np.int64) * n) // world
    w = np.asarray(weights, dtype=np.float64)
    if w.size != n:
        raise ValueError("weights must have one entry per packet")
    cum = np.concatenate([[0.0], np.cumsum(w)])
    targets = cum[-1] * np.arange(world + 1) / world
    b = np.searchsorted(cum, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, n
    return np.maximum.accumulate(b)


def shard_range(n: int, rank: int, world: int, weights=None) -> tuple[int, int]:
    b = shard_bounds(n, world, weights)
    return int(b[rank]), int(b[rank + 1])


def gather_results(local, counts, group=None, dst: int = 0):
    """Gather every rank's 16-bit results (``local``: 1-D uint16/int16 tensor,
    ``counts[r]`` entries on rank r) into one tensor on ``dst`` with one
    collective; other ranks get None.  Ranks with fewer packets are padded
    to the largest shard so the collective moves equal-sized buffers."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cmax = 2 * int(max(counts))
    # Moved as bytes: every backend (gloo, RCCL) carries uint8.  gloo's
    # gather takes host tensors only.
    home = local.device
    if dist.get_backend(group) == "gloo" and local.is_cuda:
        local = local.cpu()
    send = local.contiguous().view(torch.uint8)
    if send.numel() < cmax:
        pad = torch.zeros(cmax, dtype=torch.uint8, device=send.device)
        pad[: send.numel()] = send
        send = pad
    gl = [torch.empty(cmax, dtype=torch.uint8, device=send.device) for _ in range(world)] \
        if rank == dst else None
    dist.gather(send, gather_list=gl, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([g[: 2 * int(c)] for g, c in zip(gl, counts)]).view(local.dtype).to(home)


class ResultGather:
    """The per-step gather of u16 results, asynchronous and double-buffered:
    step k's gather runs on the collective stream while step k+1's kernel
    runs on the compute stream (xGMI traffic and an HBM-bound fold overlap);
    a slot is only rewritten after its previous gather completed.

    ``start(local, slot)`` enqueues the gather of ``local`` (the rank's
    results, written on the current stream); ``wait(slot)`` orders the
    current stream after it; ``result(slot)`` is the concatenated array on
    ``dst`` (None elsewhere) once waited."""

    def __init__(self, counts, device, group=None, dst: int = 0, depth: int = 2):
        import torch
        import torch.distributed as dist

        self.group, self.dst = group, dst
        self.counts = [int(c) for c in counts]
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.host = dist.get_backend(group) == "gloo"
        dev = torch.device("cpu") if self.host else torch.device(device)
        self.cmax = 2 * max(self.counts)
        self.pad = [torch.zeros(self.cmax, dtype=torch.uint8, device=dev) for _ in range(depth)]
        self.recv = [[torch.empty(self.cmax, dtype=torch.uint8, device=dev)
                      for _ in range(self.world)] if self.rank == dst else None
                     for _ in range(depth)]
        self.work = [None] * depth

    def start(self, local, slot: int):
        import torch.distributed as dist

        self.wait(slot)
        send = local.contiguous().view(__import__("torch").uint8)
        if self.host and send.is_cuda:
            send = send.cpu()
        if send.numel() < self.cmax or send.device != self.pad[slot].device:
            self.pad[slot][: send.numel()].copy_(send)
            send = self.pad[slot]
        self.work[slot] = dist.gather(send, gather_list=self.recv[slot], dst=self.dst,
                                      group=self.group, async_op=True)

    def wait(self, slot: int) -> None:
        if self.work[slot] is not None:
            self.work[slot].wait()
            self.work[slot] = None

    def wait_all(self) -> None:
        for s in range(len(self.work)):
            self.wait(s)

    def result(self, slot: int, dtype=None):
        import torch

        if self.rank != self.dst:
            return None
        out = torch.cat([g[: 2 * c] for g, c in zip(self.recv[slot], self.counts)])
        return out.view(dtype or torch.int16)


class Watchdog:
    """Bounded time for every phase of a multi-process run.

    A daemon thread watches the phase this rank is in.  When a phase outlives
    its deadline (a rendezvous that never completes, an RCCL init or a gather
    stuck on a peer), the rank prints ONE JSON diagnostic line -- phase, rank,
    seconds in the phase and since start -- and leaves with ``os._exit`` (no
    cleanup that could block on the stuck collective, no re-exec, no retry).
    ``fail(exc)`` does the same for an exception raised inside a phase, so every
    rank of a broken run ends non-zero with a line that says where.

    Deadlines (seconds) default to :data:`DEFAULTS`; the environment variable
    ``UINET_BENCH_WATCHDOG_S`` sets one value for every phase.  For tests,
    ``UINET_BENCH_STALL="<rank>:<phase>"`` makes that rank hang on entering
    that phase (the watchdog must end it).  The reference's concurrency this
    guards is one RX/TX kthread per interface
    (/root/reference/lib/libuinet/uinet_if_netmap.c:1648-1665): one stuck
    worker must not hang the others silently."""

    DEFAULTS = {"rendezvous": 300.0, "workload": 600.0, "warmup": 300.0, "timed": 300.0,
                "parity": 900.0, "plan": 120.0, "teardown": 120.0}
    EXIT_DEADLINE = 124  # timeout(1)'s status
    EXIT_ERROR = 125

    def __init__(self, rank: int, deadlines=None, stream=None):
        import os
        import sys
        import threading
        import time

        self._os, self._time = os, time
        self.rank = int(rank)
        self.stream = stream or sys.stdout
        self.deadlines = dict(self.DEFAULTS, **(deadlines or {}))
        flat = os.environ.get("UINET_BENCH_WATCHDOG_S")
        if flat:
            self.deadlines = {k: float(flat) for k in self.deadlines}
        self.t0 = time.monotonic()
        self.phase, self.t_phase, self.deadline = None, self.t0, None
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._watch, name="uinet-watchdog", daemon=True)
        self._thread.start()

    def enter(self, phase: str) -> None:
        now = self._time.monotonic()
        with self._lock:
            self.phase, self.t_phase = phase, now
            self.deadline = now + self.deadlines.get(phase, max(self.deadlines.values()))
        if self._os.environ.get("UINET_BENCH_STALL") == f"{self.rank}:{phase}":
            while True:  # injected hang (tests): only the watchdog ends it
                self._time.sleep(3600)

    def done(self) -> None:
        with self._lock:
            self.phase, self.deadline = None, None

    def _line(self, what: str, **extra) -> None:
        import json

        now = self._time.monotonic()
        rec = {"watchdog": what, "phase": self.phase, "rank": self.rank,
               "phase_s": round(now - self.t_phase, 3), "elapsed_s": round(now - self.t0, 3),
               "deadline_s": self.deadlines.get(self.phase) if self.phase else None}
        rec.update(extra)
        try:
            self.stream.write(json.dumps(rec) + "\n")
            self.stream.flush()
        except Exception:  # pragma: no cover - nothing left to report with
            pass

    def fail(self, exc: BaseException) -> None:
        """Report an exception raised inside the current phase and exit."""
        self._line("error", error=f"{type(exc).__name__}: {exc}"[:500])
        self._os._exit(self.EXIT_ERROR)

    def _watch(self) -> None:
        while True:
            with self._lock:
                dl = self.deadline
            now = self._time.monotonic()
            if dl is not None and now >= dl:
                with self._lock:
                    if self.deadline is None or self._time.monotonic() < self.deadline:
                        continue
                    self._line("deadline")
                self._os._exit(self.EXIT_DEADLINE)
            self._time.sleep(0.2 if dl is None else min(0.2, max(0.01, dl - now)))
