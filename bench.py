#!/usr/bin/env python3
"""Device-resident Internet-checksum throughput on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch that already sits in
HBM: a single launch of the engine's span kernel (``uinet_cksum_spans``, the
C ABI the libuinet shim calls) over the rank's packets, plus -- for N > 1 --
the one RCCL gather of the 16-bit results to rank 0.  Workload at N = 1 is
BASELINE.json configs[1] (config 2): 1,048,576 x 1500-B contiguous packets,
in_cksum_skip(m, 1500, 0).  For N > 1 the default is config 4 (configs[3]):
every rank folds its own 2,097,152 x 1500-B packets (16 M over 8 GPUs, weak
scaling) and the u16 results meet on rank 0 in one gather per step.

Launch: ``python bench.py --gpus N``.  Without a launcher (no WORLD_SIZE in
the environment) and N > 1, this process starts N ranks itself with
``torch.distributed.run`` as a child process -- before anything touches the
GPU -- and exits with its status; under torchrun WORLD_SIZE must equal N.

Rank 0 prints ONE JSON line.  ``roofline`` prices the span kernel: algorithmic
bytes per launch (sum of packet lengths) / its mean HIP-event duration on the
launch stream, against the 8 TB/s HBM3E peak; ``traffic`` is the PMC-measured
HBM read bytes per launch from profiles/ (FETCH_SIZE x 1024 x 2, the gfx950
correction of MI355X_MICROARCH.md section HBM) when present for this workload.
``cpu_baseline`` is the reference's own scalar in_cksum_skip
(oracle/_ref/libref_cksum.so, compiled from /root/reference) on the same
bytes laid out as host mbufs, timed on this box's host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
CHAIN_CONFIGS = ("3", "3tx", "5tso")


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=200,
                    help="untimed steps first: the first ~30-100 back-to-back launches run "
                    "up to 25 %% slower while clocks settle (profiles/r01/)")
    ap.add_argument("--config", choices=["2", "2rx", "2s", "2su", "3", "3tx", "4", "5", "5tso"],
                    default=None,
                    help="BASELINE.json config shape (default: 2 = the headline at N = 1, 4 = "
                    "2,097,152 packets per GPU when distributed; 2s = 16 M x 64 B packets, a "
                    "small-packet shape outside BASELINE.json)")
    ap.add_argument("--packets", type=int, default=None, help="packets per GPU")
    ap.add_argument("--api", choices=["spans", "strided"], default="spans")
    ap.add_argument("--desc", choices=["wide", "packed"], default="wide",
                    help="12-B wide (uinet_cksum_chains / uinet_cksum_spans) or packed "
                    "6-B (uinet_cksum_chains32 / uinet_cksum_spans32) descriptors")
    ap.add_argument("--form", choices=["seglist", "mbufs"], default="seglist",
                    help="chain configs (3, 3tx, 5tso): a segment list resolved from the chains "
                    "(uinet_cksum_chains) or the struct mbuf chains themselves in HBM, walked "
                    "on the GPU (uinet_cksum_mbufs)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--host-offload", choices=["auto", "off"], default="auto",
                    help="N = 1: also fold the batch as host-resident registered mbufs "
                    "(device walk) and report its host CPU per 1,000 packets")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM traffic measured by rocprofv3 --pmc")
    ap.add_argument("--scaling-ref", default=os.path.join(REPO, "profiles", "scaling_ref.json"),
                    help="single-GPU config-4 shard rate (committed) carried in the line")
    ap.add_argument("--host-path", action="store_true",
                    help="also time H2D + kernel + D2H (host-resident rate)")
    ap.add_argument("--save-results", default=None, metavar="NPY",
                    help="rank 0 saves the last timed step's u16 results (every rank's, "
                    "gathered, in rank order) to this .npy file")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch (and rendezvous, over gloo) as usual, print each rank's plan "
                    "as JSON and exit before touching the GPU")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start ``n`` ranks of this script under torch.distributed.run as a
    child process (never an exec: nothing here has touched the GPU, and the
    box forbids replacing a process) and return its exit status."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    return subprocess.run(cmd, env=env).returncode


def metric_name() -> str:
    try:
        with open(os.path.join(REPO, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except Exception:  # pragma: no cover
        return "device-resident checksum GiB/s"


def build_workload(cfg: str, n, rank: int, world: int = 1):
    import libuinet_amd.workloads as W

    if cfg == "4":
        n = n or (1 << 21)
        w = W.config2_device(n, rank=rank)
        w["desc"] = (f"config4: {n * world:,} x 1500 B packets sharded {n:,} per GPU over "
                     f"{world} GPU{'s' if world > 1 else ''} (stride 1500, device-resident), "
                     f"in_cksum_skip(m,1500,0); u16 results gathered to rank 0")
        w["hint"] = 1500
    elif cfg in ("2", "2rx"):
        n = n or (1 << 20)
        w = W.config2_device(n, stride=1514 if cfg == "2rx" else 1500,
                             base=14 if cfg == "2rx" else 0, rank=rank)
        w["desc"] = (f"config{cfg}: {n:,} x 1500 B contiguous packets (stride {w['stride']}"
                     f"{', +14' if cfg == '2rx' else ''}), device-resident, in_cksum_skip(m,1500,0)")
        w["hint"] = 1500
    elif cfg in ("2s", "2su"):
        n = n or (1 << 24)
        # 2su: the same packets 2 B off 16-B alignment (an IP packet behind a
        # 14-B Ethernet header at a 16-B aligned frame): every span touches 5 chunks
        base = 2 if cfg == "2su" else 0
        w = W.config2_device(n, stride=64, length=64, base=base, rank=rank)
        w["desc"] = (f"config{cfg}: {n:,} x 64 B contiguous packets (stride 64"
                     f"{', +2' if base else ''}), device-resident, in_cksum_skip(m,64,0) -- "
                     f"small-packet shape, not a BASELINE.json config")
        w["hint"] = 64
    elif cfg == "3":
        n = n or (1 << 20)
        w = W.config3_device(n, rank=rank)
        w["desc"] = (f"config3: {n:,} mixed 64/576/1500 B packets as {w['nseg']:,} chained "
                     f"1..256 B mbuf segments, in_cksum_skip(m,len,20)")
        w["hint"] = w["mean_seg"]
    elif cfg in ("3tx", "5tso"):
        w = W.materialize_device(W.chain_layout(cfg, n))
        w["hint"] = w["mean_seg"]
        n = w["n"]
        if cfg == "3tx":
            w["desc"] = (f"config3tx: {n:,} mixed 64/576/1500 B packets in the reference TX "
                         f"shape (40-B header mbuf -> 4-KiB page-cluster slices, {w['nseg']:,} "
                         f"segments), in_cksum_skip(m,len,20)")
        else:
            w["desc"] = (f"config5tso: {w['layout']['sends']:,} 1-MiB sends cut at MSS 8960 into "
                         f"{n:,} segments (40-B header -> payload slice), "
                         f"in_cksum_pseudo_header(m,20+seglen,20,src,dst,TCP)")
    else:
        n = n or 131072
        w = W.config5_device(n, rank=rank)
        w["desc"] = (f"config5: {n:,} x 9000 B jumbo frames, in_cksum_pseudo_header(m,8980,20,"
                     f"src,dst,TCP/UDP)")
        w["hint"] = 8980
    return w


def make_launch(cfg: str, w, api: str, out, desc: str = "wide", flags: int = 0,
                form: str = "seglist"):
    import libuinet_amd as u

    if cfg in CHAIN_CONFIGS and form == "mbufs":
        return lambda s: u.cksum_mbufs(w["heads"], length=w["len"], skip=w["skip"],
                                       seed=w.get("seed"), out=out, flags=flags,
                                       seg_hint=w["hint"], stream=s)
    if cfg in CHAIN_CONFIGS:
        so, sl = (w["seg_off"], w["seg_len"]) if desc == "wide" else w["packed"]
        return lambda s: u.cksum_chains(w["arena"], so, sl, w["pkt_seg"],
                                        length=w["len"], skip=w["skip"], seed=w.get("seed"),
                                        out=out, flags=flags, len_hint=w["hint"], stream=s)
    if api == "strided" and cfg in ("2", "2rx", "2s", "2su"):
        base = w["arena"][w["base"]:]
        return lambda s: u.cksum_strided(base, w["stride"], w["length"], w["n"], out=out, stream=s)
    seed = w.get("seed")
    off, ln = (w["off"], w["len"]) if desc == "wide" else w["packed"]
    return lambda s: u.cksum_spans(w["arena"], off, ln, seed=seed, out=out,
                                   len_hint=w["hint"], stream=s)


def kernel_name(cfg: str, api: str, desc: str = "wide", form: str = "seglist") -> str:
    if cfg in CHAIN_CONFIGS and form == "mbufs":
        return "k_mbufs"
    if cfg in CHAIN_CONFIGS:
        return "k_chains32" if desc == "packed" else "k_chains"
    if api == "strided":
        return "k_strided"
    return "k_spans32" if desc == "packed" else "k_spans"


# The sources each kernel family is compiled from: a FETCH_SIZE entry counts
# only while they are byte-identical to the ones it was measured on.
KERNEL_SOURCES = {
    "k_chains_pipe": ("cksum_chains.hip", "cksum_device.h"),
    "k_chains_wide": ("cksum_chains.hip", "cksum_device.h"),
    "k_spans_lean": ("cksum_spans.hip", "cksum_device.h"),
    "k_spans_quad": ("cksum_spans.hip", "cksum_device.h"),
    "k_strided_dense": ("cksum_spans.hip", "cksum_device.h"),
    "k_spans": ("cksum_kernels.hip", "cksum_device.h"),
    "k_mbufs": ("cksum_mbufs.hip", "cksum_device.h", "walk_xlate.h"),
}


def short_kernel(name: str) -> str:
    """A demangled kernel name as tools/pmc_summary.py keys it:
    'k_chains_pipe<2,32,2,unsignedlong,unsignedint>'."""
    import re

    m = re.search(r"(k_\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2).replace(' ', '')}>"
    return name.split("(")[0][-60:]


def kernel_src_sha(kernel: str):
    """sha256 (16 hex digits) of the sources the kernel (short or family
    name) is built from; None for an unknown family."""
    import hashlib

    fam = kernel.split("<")[0]
    files = KERNEL_SOURCES.get(fam)
    if files is None:
        return None
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(REPO, "libuinet_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_traffic(path: str, key: str, kernel: str):
    """HBM bytes per launch from the FETCH_SIZE passes folded into `path`
    (tools/prof_all.sh), with where they were measured.  None unless the
    entry was measured on exactly this instantiation (`kernel`, the short name
    of what the engine launched) built from today's sources."""
    try:
        with open(path) as f:
            e = json.load(f).get(key)
    except Exception:
        e = None
    if e is None:
        return None, {"key": key, "note": "no FETCH_SIZE entry"}
    src = {"key": key, "source": e.get("source"), "measured_kernel": e.get("kernel"),
           "launched_kernel": kernel}
    if e.get("kernel") != kernel:
        src["note"] = "measured on another kernel: not reported"
        return None, src
    if e.get("src_sha") is None or e.get("src_sha") != kernel_src_sha(kernel):
        src["note"] = "measured on an older build of this kernel: not reported"
        return None, src
    return float(e["hbm_read_bytes_per_launch"]), src


def layout_floor_line(cfg: str, w, desc: str, kms, form: str = "seglist") -> dict:
    """Chain configs: the layout's HBM-traffic floor (distinct 128-B lines
    holding a summed byte + the descriptors the kernel reads) and the kernel's
    rate measured against it, beside the algorithmic roofline."""
    import libuinet_amd.workloads as W

    lay = w["layout"]
    skip = lay.get("skip")
    if skip is None:  # config 3: in_cksum_skip(m, len, 20)
        skip = np.full(w["n"], 20, np.int64)
    seeded = w.get("seed") is not None
    fl = W.layout_floor(lay["seg_off"], lay["seg_len"], lay["pkt_seg"], lay["lens"], skip,
                        seeded, 128, 6 if desc == "packed" else 12)
    floor = fl["floor_bytes"]
    extra = {}
    if form == "mbufs":
        # no descriptors: the packet bytes' lines, one 128-B line per mbuf
        # header the walk reads (records 256 B apart: a line each), and the
        # jobs (head u64, len, skip [, seed] per packet)
        # (a header mbuf that holds its packet's first bytes shares its first
        # line with them: counted once, with the bytes)
        walked = W.mbufs_walked(lay["seg_len"], lay["pkt_seg"], lay["lens"], skip)
        own = walked - (w["n"] if w.get("inline_first") is not None else 0)
        floor = fl["arena_bytes"] + 128 * own + w["n"] * (16 + (4 if seeded else 0))
        extra = {"mbufs_walked": walked, "header_line_bytes": 128 * own}
    achieved = floor / (float(kms.mean()) * 1e-3) / 1e9
    return {"bytes": floor, "line": 128, **extra,
            "over_algorithmic": round(floor / w["bytes"], 4),
            "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4)}


def gather_rank_kernels(kms, world: int, backend: str):
    """Every rank's kernel times (mean, min, max ms per launch), gathered to
    every rank in rank order: a (world, 3) array.  One tiny all_gather after
    the timed region (RCCL on the GPU box, gloo in the CPU rehearsal)."""
    import torch
    import torch.distributed as dist

    dev = "cuda" if backend == "nccl" else "cpu"
    kms = np.asarray(kms, dtype=np.float64)
    t = torch.tensor([kms.mean(), kms.min(), kms.max()], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.stack([p.cpu().numpy() for p in parts])


def rank_fields(stats, bytes_per_gpu: int, step_ms: float) -> dict:
    """The N > 1 line's per-rank view: which GPU is the
    slowest, and how much of a step the result gather leaves exposed."""
    means = np.asarray(stats, dtype=np.float64)[:, 0]
    slow = int(np.argmax(means))
    kmax = float(means[slow])
    return {
        "ranks_kernel_ms": [round(float(x), 5) for x in means],
        "kernel_ms_max_rank": round(kmax, 5),
        "slowest_rank": slow,
        "step_ms": round(step_ms, 4),
        "gather_exposed_ms": round(step_ms - kmax, 4),
        "per_gpu_gbs_min": round(bytes_per_gpu / (kmax * 1e-3) / 1e9, 1),
    }


def scaling_ref(path: str):
    """The single-GPU config-4 shard rate (``bench.py --gpus 1 --config 4``)
    from a committed profiles/ entry, so a 1 -> N efficiency can be computed
    from like workloads (every N > 1 point is config 4; the N = 1 headline is
    config 2).  None when the file is absent."""
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    import platform

    return platform.processor() or "unknown"


def reference_results(cfg: str, w, threads: int):
    """The reference's (or, without oracle/_ref, the oracle restatement's)
    results over this rank's bytes, computed on the host after the timed
    region: the distributed line's parity check (cpu_baseline leg)."""
    import oracle
    from libuinet_amd.mbuf import MbufChains

    host = w["arena"].cpu().numpy()
    R = oracle.Reference() if oracle.have_reference() else None
    kind = "reference" if R is not None else "port"
    threads = max(1, threads)
    if cfg in CHAIN_CONFIGS:
        lay = w["layout"]
        ch = MbufChains(host, lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
        if cfg == "5tso":
            args = (ch.heads, lay["plen"], 20, lay["src"], lay["dst"], 6)
            out = R.time_pseudo(*args, nthreads=threads, reps=1)[1] if R else \
                oracle.Oracle().pseudo_header_batch(*args)
        else:
            args = (ch.heads, lay["lens"], 20)
            out = R.time_skip(*args, nthreads=threads, reps=1)[1] if R else \
                oracle.Oracle().skip_batch(*args, nthreads=threads)
    elif cfg == "5":
        ch = MbufChains.contiguous(host, w["frame"] * np.arange(w["n"], dtype=np.int64), w["frame"])
        args = (ch.heads, w["plen"], w["off0"], w["src"], w["dst"], w["proto"])
        out = R.time_pseudo(*args, nthreads=threads, reps=1)[1] if R else \
            oracle.Oracle().pseudo_header_batch(*args)
    else:
        ch = MbufChains.contiguous(host, w["off"].cpu().numpy(), w["length"])
        out = R.time_skip(ch.heads, w["length"], 0, nthreads=threads, reps=1)[1] if R else \
            oracle.Oracle().skip_batch(ch.heads, w["length"], 0, nthreads=threads)
    return kind, np.ascontiguousarray(out, dtype=np.uint16)


def cpu_baseline(cfg: str, w, gpu_out, threads: int, keep=None):
    """The reference's scalar in_cksum_skip / in_cksum_pseudo_header over the same
    bytes as host mbufs; returns the cpu_baseline object (and checks parity).
    ``keep`` (a dict) receives the host mbufs and call arguments for
    host_offload_line."""
    import oracle
    from libuinet_amd.mbuf import MbufChains

    from libuinet_amd.mbuf import aligned_empty

    kind = "reference" if oracle.have_reference() else "port"
    R = oracle.Reference() if kind == "reference" else None
    # page-aligned, so host_offload_line can register it with the engine
    src = w["arena"].cpu().numpy()
    host = aligned_empty(src.size)
    host[:] = src
    del src
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        allowed = list(range(os.cpu_count() or 1))
    threads = max(1, min(threads, len(allowed)))
    cpus = allowed[:threads]
    if cfg == "5tso":
        lay = w["layout"]
        ch = MbufChains(host, lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
        args = (ch.heads, lay["plen"], 20, lay["src"], lay["dst"], 6)
        timer = (lambda nt, cp, r: R.time_pseudo(*args, nthreads=nt, cpus=cp, reps=r)) if R else None
        port = lambda: oracle.Oracle().pseudo_header_batch(*args)  # noqa: E731
    elif cfg in ("3", "3tx"):
        lay = w["layout"]
        ch = MbufChains(host, lay["seg_off"], lay["seg_len"], lay["pkt_seg"])
        args = (ch.heads, lay["lens"], 20)
        timer = (lambda nt, cp, r: R.time_skip(*args, nthreads=nt, cpus=cp, reps=r)) if R else None
        port = lambda: oracle.Oracle().skip_batch(*args, nthreads=threads)  # noqa: E731
    elif cfg == "5":
        ch = MbufChains.contiguous(host, w["frame"] * np.arange(w["n"], dtype=np.int64), w["frame"])
        args = (ch.heads, w["plen"], w["off0"], w["src"], w["dst"], w["proto"])
        timer = (lambda nt, cp, r: R.time_pseudo(*args, nthreads=nt, cpus=cp, reps=r)) if R else None
        port = lambda: oracle.Oracle().pseudo_header_batch(*args)  # noqa: E731
    else:
        off = w["off"].cpu().numpy()
        ch = MbufChains.contiguous(host, off, w["length"])
        args = (ch.heads, w["length"], 0)
        timer = (lambda nt, cp, r: R.time_skip(*args, nthreads=nt, cpus=cp, reps=r)) if R else None
        port = lambda: oracle.Oracle().skip_batch(*args, nthreads=threads)  # noqa: E731
    if keep is not None:
        keep.update(host=host, ch=ch, args=args,
                    pseudo=cfg in ("5", "5tso"))
        if keep.get("before_passes"):
            keep["before_passes"]()
    gib = w["bytes"] / 2**30
    runs, spread, read = {}, {}, {}
    if timer is not None:
        # median of 5 single passes per (threads, placement): the threads pinned
        # to the first CPUs of the process mask, and left to the scheduler.
        # `threads` is the box's CPU share (16 per GPU): the rest of the mask
        # belongs to the other GPUs' jobs on the machine; plus every CPU of the
        # process mask (SURVEY.md 8d "1 thread, then all host cores"; one
        # thread per CPU, at most 256).  Every pass is max(worker end) -
        # min(worker start), stamped by the workers themselves
        # (ref_harness.c): round 5 stamped on the main thread, which a busy
        # mask scheduled late, and read passes of 1.3-2.3 TB/s, above the
        # host's memory bandwidth.  Beside each checksum setting, passes of a
        # plain streaming read of the same host bytes with the same threads
        # and placement: the host's read bandwidth, which no checksum pass can
        # beat (`within_read_ceiling`).
        outs = []
        n_all = min(len(allowed), 256)
        spread_cpus = l3_spread(allowed, threads)
        for nt in sorted({1, threads, n_all}):
            # "spread": one thread per L3 domain (CCD) of the mask, where the
            # host has more domains than threads: what `threads` cores pull at
            # best (first CPUs of the mask share a few CCDs' links; floating
            # threads land anywhere)
            places = ("pinned", "floating") + (("spread",) if nt == threads and spread_cpus else ())
            for placement in places:
                if placement == "spread":
                    pin = spread_cpus
                else:
                    pin = ((allowed[:nt] if nt > threads else cpus[:nt]) if placement == "pinned"
                           else None)
                # checksum and read passes alternate (same box conditions for
                # both).  From 16 threads up both are bound by the host's
                # memory system and spread by 2-10x from pass to pass on the
                # shared host, so the ceiling takes the fastest of 40 read
                # passes per setting (with 10, a checksum pass now and then
                # beat every read pass by 3-25 %: profiles/r06/NOTES.md); one
                # thread reads 15-20 % faster than it sums, 10 suffice there
                rr, rd = [], []
                for _ in range(5):
                    rr.append(timer(nt, pin, 1))
                    rd += [R.time_read(host, nthreads=nt, cpus=pin, reps=1)
                           for _ in range(2 if nt == 1 else 8)]
                runs[f"{nt}_{placement}"] = float(np.median([r[0] for r in rr]))
                spread[f"{nt}_{placement}"] = (min(r[0] for r in rr), max(r[0] for r in rr))
                outs.append(rr[-1][1])
                read[f"{nt}_{placement}"] = (float(np.median(rd)), min(rd))
        best = min((k for k in runs if k.startswith(f"{threads}_")), key=runs.get)
        tn = runs[best]
        t1 = min(runs["1_pinned"], runs["1_floating"])
        best_all = min((k for k in runs if k.startswith(f"{n_all}_")), key=runs.get)
    else:  # oracle restatement, timed the same way
        t0 = time.perf_counter(); o = port(); t1 = time.perf_counter() - t0  # noqa: E702
        outs, tn, best = [o], t1, f"{threads}_port"
        runs[best] = t1
        spread[best] = (t1, t1)
        best_all, n_all = best, threads
    parity = bool(all(np.array_equal(o, gpu_out) for o in outs))
    rates = {k: round(gib / t, 3) for k, t in runs.items()}
    # min / max GiB/s of the 5 passes: the many-thread figure swings by 4x
    # from box to box (64.8 .. 271.2 GiB/s for one command on one CPU model,
    # VERDICT r03); the 1-thread figure is the stable comparison
    minmax = {k: [round(gib / hi, 3), round(gib / lo, 3)] for k, (lo, hi) in spread.items()}
    host_gib = host.nbytes / 2**30
    read_gibs = {k: round(host_gib / med, 3) for k, (med, _) in read.items()}
    ceiling = round(max((host_gib / best_t for _, best_t in read.values()), default=0.0), 3)
    fastest = max((v[1] for v in minmax.values()), default=0.0)
    return {
        "value": round(gib / tn, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
        "cpu_model": cpu_model(),
        "sample": (f"{w['n']:,} packets ({gib:.3f} GiB algorithmic) of the benchmarked batch, "
                   f"host copy as {'chained ' if cfg in CHAIN_CONFIGS else ''}struct mbuf; median "
                   f"of 5 passes per thread count and placement (GiB/s: "
                   + ", ".join(f"{k.replace('_', ' threads ')} {v}" for k, v in rates.items())
                   + f"); value = {best.replace('_', ' threads ')} (its 5 passes: "
                   + "{}-{} GiB/s".format(*minmax[best])
                   + f"); every pass max(worker end) - min(worker start); host streaming-read "
                   f"ceiling {ceiling} GiB/s; results bit-identical to the GPU in every run: "
                   f"{parity}"),
        "runs_gibs": rates,
        "runs_minmax_gibs": minmax,
        "value_from": best,
        "placement": best.split("_")[1],
        "one_thread_gibs": round(gib / t1, 3),
        # the reference on every CPU of the mask (median of 5, the faster
        # placement); `value` stays the `cores`-thread figure (the GPU box's
        # CPU share per GPU)
        "all_cores_gibs": round(gib / runs[best_all], 3),
        "all_cores_threads": n_all,
        "all_cores_from": best_all,
        "mask_cpus": len(allowed),
        # the host's streaming-read rate over the same host bytes (the arena)
        # per thread count and placement (median of 10 or 40), and its fastest pass:
        # the ceiling every checksum pass above must stay under
        "host_read_gibs": read_gibs or None,
        "host_read_max_gibs": {k: round(host_gib / b, 3) for k, (_, b) in read.items()} or None,
        "host_read_ceiling_gibs": ceiling or None,
        "fastest_pass_gibs": fastest,
        "within_read_ceiling": (fastest <= ceiling) if ceiling else None,
        "bit_identical_to_gpu": parity,
    }


def l3_spread(allowed, nt):
    """`nt` CPUs of `allowed`, one per L3 cache domain (sysfs
    cache/index3/shared_cpu_list), or None when the mask has fewer domains
    than `nt` or the topology is not readable."""
    seen, picks = set(), []
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                dom = f.read().strip()
        except OSError:
            return None
        if dom not in seen:
            seen.add(dom)
            picks.append(c)
    return picks[:nt] if len(picks) >= nt else None


def host_offload_line(keep, n: int, nbytes: int, gpu_out, reps: int = 7):
    """The benchmarked batch once more as HOST-resident mbufs, the way libuinet
    holds them: packet bytes and mbufs registered with the engine
    (uinet_cksum_register_host), folded through the host-mbuf batch API --
    the GPU walks the chains and reads the bytes over PCIe.  Reports wall time
    and the host CPU the call cost (uinet_cksum_host_cpu: calling thread +
    engine pool helpers) per 1,000 packets, beside the reference's 1-thread
    pass over the same mbufs (a scalar loop: its CPU time is its wall time;
    the caller adds those fields from cpu_baseline's one-thread figure).
    One mbuf per packet (configs 2, 5) takes the single-mbuf span path: the
    host reads each head mbuf and hands the GPU spans; chains take the device
    walk.  `bytes_only` repeats it with only the packet bytes registered (the
    zero-copy netmap setup: spans, or the host walk for chains).
    Never `value`; SURVEY.md section 7 step 7 / VERDICT r04 item 1."""
    ch, args = keep["ch"], keep["args"]
    link = link_h2d_gbs(keep["host"], [keep["host"], ch.mbufs])
    row = host_offload_row(keep, [keep["host"], ch.mbufs], n, nbytes, gpu_out, link, reps)
    row["bytes_only"] = host_offload_row(keep, [keep["host"]], n, nbytes, gpu_out, link, reps)
    return row


def host_offload_row(keep, bufs, n, nbytes, gpu_out, link, reps):
    """One host_offload_line measurement with `bufs` registered."""
    import libuinet_amd as u

    fn = u.in_cksum_pseudo_header_batch if keep["pseudo"] else u.in_cksum_skip_batch
    args = keep["args"]
    for b in bufs:
        u.register_host(b)
    try:
        fn(*args)  # warm: staging, walk row size
        rows = []
        for _ in range(reps):
            u.host_cpu(reset=True)
            t0 = time.perf_counter()
            out = fn(*args)
            rows.append((time.perf_counter() - t0, u.host_cpu(reset=True), out))
    finally:
        for b in bufs:
            u.unregister_host(b)
    k = n / 1000
    cpu_us = [r[1]["cpu_ns"] / 1e3 / k for r in rows]  # per call, in call order
    rows.sort(key=lambda r: r[0])
    wall, st, out = rows[len(rows) // 2]
    return {
        "what": "the benchmarked batch as host mbufs (%s registered), through the host-mbuf "
                "batch API (the GPU reads the bytes in place over PCIe); medians of %d calls"
                % ("packet bytes and mbufs" if len(bufs) > 1 else "packet bytes only", reps),
        "wall_ms": round(wall * 1e3, 3),
        "gibs": round(nbytes / wall / 2**30, 2),
        # the median over the calls (each call's own CPU time: a busy host now
        # and then doubles one call's, independent of its wall time)
        "host_cpu_us_per_1k_pkts": round(float(np.median(cpu_us)), 3),
        "host_cpu_us_per_1k_pkts_calls": [round(x, 3) for x in cpu_us],
        # which host-resident path the engine took: one mbuf per packet goes
        # as spans (the host reads each head mbuf, the link carries the packet
        # bytes and 6 B per packet); chains to the device walk when the mbufs
        # are registered, else to the host walk
        "path": ("single-mbuf spans" if st["span_batches"] == st["calls"] else
                 "device walk" if st["device_walks"] == st["calls"] else "host walk"),
        "device_walked": bool(st["device_walks"] == st["calls"]),
        # on the span path: whether the GPU read the head mbufs (mbufs
        # registered) or the calling thread did
        "heads_read_by": ("gpu" if st["device_walks"] == st["calls"] else "host")
                         if st["span_batches"] == st["calls"] else None,
        "dma_bytes": int(st.get("span_dma_bytes", 0)),
        "bit_identical": bool(all(np.array_equal(r[2], gpu_out) for r in rows)),
        # the link's own rate, measured here: one DMA copy of the same registered
        # bytes to HBM; the batch's summed bytes over its wall time against it
        # (mbuf lines the walk reads also cross the link and are not counted)
        "link_h2d_gbs": link,
        "frac_of_link": round(nbytes / wall / 1e9 / link, 4) if link else None,
    }


def link_h2d_gbs(host, bufs):
    """GB/s of a DMA copy of `host` (registered again for the copy) into HBM,
    best of 3; None if it cannot be measured."""
    import torch

    import libuinet_amd as u

    try:
        for b in bufs:
            u.register_host(b)
        try:
            h = torch.from_numpy(host)
            d = torch.empty(h.shape, dtype=h.dtype, device="cuda")
            d.copy_(h)
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                d.copy_(h)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            del d
            return round(host.nbytes / best / 1e9, 2)
        finally:
            for b in bufs:
                u.unregister_host(b)
    except Exception:  # a report, never the measurement
        return None


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # the ranks print the JSON line
    distributed = env_world is not None
    if distributed and int(env_world) != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}; launch with "
                 f"torchrun --nproc-per-node {args.gpus} (or drop the launcher)")
    if args.config is None:
        args.config = "4" if distributed else "2"
    if args.api == "strided" and args.config not in ("2", "2rx", "2s", "2su"):
        sys.exit(f"bench: --api strided runs configs 2, 2rx, 2s and 2su, not {args.config}")
    # N > 1: every phase has a deadline (libuinet_amd.dist.Watchdog).  A rank
    # stuck in the rendezvous, RCCL init, a step or the parity gather -- or
    # failing in one -- prints one JSON line naming the phase and exits
    # non-zero, instead of leaving the launcher to kill a silent run.
    wd = None
    if distributed:
        from libuinet_amd.dist import Watchdog

        wd = Watchdog(int(os.environ.get("RANK", "0")))
    try:
        run(args, distributed, wd)
    except Exception as e:
        if wd is None:
            raise
        import traceback

        traceback.print_exc()
        wd.fail(e)


def run(args, distributed: bool, wd):
    def phase(name):
        if wd is not None:
            wd.enter(name)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if distributed:
            phase("rendezvous")
            dist.init_process_group("gloo")
            phase("plan")
        plan = {"rank": rank, "local_rank": local,
                "world": dist.get_world_size() if distributed else 1, "config": args.config,
                "packets_per_gpu": args.packets or {"4": 1 << 21, "2s": 1 << 24, "2su": 1 << 24,
                                                    "5": 131072}.get(args.config, 1 << 20),
                "backend": os.environ.get("UINET_BENCH_BACKEND", "nccl") if distributed else None}
        if distributed:
            # the N > 1 line's per-rank fields, rehearsed over gloo with stand-in
            # kernel times (rank r: 0.4 + 0.01 r ms per launch) through the same
            # gather and arithmetic the timed run uses
            fake = 0.4 + 0.01 * rank + np.array([0.0, -0.001, 0.001])
            st = gather_rank_kernels(fake, plan["world"], "gloo")
            plan["rank_fields_rehearsal"] = rank_fields(st, 3145728000, 0.45)
        print(json.dumps(plan), flush=True)
        if distributed:
            dist.barrier()
            phase("teardown")
            dist.destroy_process_group()
            wd.done()
        return
    # UINET_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # one GPU (CI / 1-GPU boxes); the real runs use RCCL, one rank per GPU.
    backend = os.environ.get("UINET_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and local >= ndev:
        sys.exit(f"bench: rank {rank} has LOCAL_RANK {local} but {ndev} GPU(s) are visible "
                 "(RCCL needs one GPU per rank; UINET_BENCH_BACKEND=gloo shares one)")
    dev = local % max(1, ndev)
    phase("rendezvous")
    torch.cuda.set_device(dev)
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    world = dist.get_world_size() if distributed else 1

    import libuinet_amd as u
    from libuinet_amd.dist import ResultGather

    if not u.device_ok():
        raise SystemExit("bench: no gfx950 device visible")
    phase("workload")
    w = build_workload(args.config, args.packets, rank, world)
    n = w["n"]
    # three result buffers (N > 1): step k's gather is enqueued after step
    # k+1's kernel and overlaps it; a buffer is rewritten only after the
    # gather that read it has completed
    NBUF = 3
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(NBUF)]
    out = outs[0]
    stream = torch.cuda.current_stream()
    if distributed:
        # a non-blocking stream of its own for the kernels (made current, so
        # the collectives and gloo's host copies order themselves after it)
        # instead of the null stream: 0.481 vs 0.489 ms per step at world 1
        # (profiles/r02/gather/).  High priority: a hardware queue apart from
        # RCCL's normal-priority stream, so that step k's gather kernel does
        # not sit between the kernels of steps k + 1 and k + 2.  Both backends
        # run this same layout (round 2's gloo rehearsal kept the null stream
        # after a side-stream run exited non-zero before the ordering below
        # existed; profiles/r03/gather/)
        stream = torch.cuda.Stream(priority=-1)
        # it does not synchronise with the null stream: the workload's
        # generation and descriptor uploads (null stream) must be complete
        # before its first kernel reads them
        stream.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        torch.cuda.set_stream(stream)
    if args.desc == "packed" and args.config in CHAIN_CONFIGS:
        w["packed"] = u.pack_segments(w["seg_off"], w["seg_len"])
    elif args.desc == "packed" and args.api == "spans":
        w["packed"] = u.pack_segments(w["off"], w["len"])
    if args.form == "mbufs" and args.config in CHAIN_CONFIGS:
        import libuinet_amd.workloads as W

        # the same chains as struct mbufs in HBM (records in chain order); 3tx's
        # 40-B IP + TCP header lives inside its header mbuf (m_pktdat +
        # max_linkhdr, 104 B into the record, tcp_output.c:844-846), the
        # payload slices in page clusters
        inline = W.tx_inline_offset(w["layout"]) if args.config == "3tx" else None
        w.update(W.device_mbufs(w["arena"], w["seg_off"], w["seg_len"], w["pkt_seg"],
                                inline_first=inline))
        w["inline_first"] = inline
        w["desc"] += "; as struct mbuf chains in HBM, walked on the GPU (m_next / m_data / m_len)"
    launches = [make_launch(args.config, w, args.api, o, args.desc, form=args.form) for o in outs]
    counts = [n] * world
    rg = ResultGather(counts, "cuda", depth=NBUF) if distributed else None
    K, Wm = args.steps, args.warmup
    # Kernel time from HIP events on the launch stream.  At N = 1 a step IS
    # one launch, so one event pair brackets the K back-to-back launches (no
    # per-launch event overhead; inter-launch gaps count against us).  At
    # N > 1 each launch is bracketed so the gather stays out of it.
    per_launch = distributed
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K if per_launch else 1)]

    def step(k=None, i=0):
        slot = i % NBUF
        if rg is not None:
            rg.wait(slot)  # the gather that last read this buffer is done
        if per_launch and k is not None:
            ev[k][0].record(stream)
        launches[slot](stream)
        if per_launch and k is not None:
            ev[k][1].record(stream)
        if rg is not None and i > 0:
            # the one exchange, u16 results -> rank 0, for the PREVIOUS step:
            # enqueued behind this step's kernel, so the kernels run back to
            # back and each gather overlaps the next kernel
            prev = (i - 1) % NBUF
            rg.start(outs[prev], prev)

    def drain(i_last):
        if rg is not None:
            rg.start(outs[i_last % NBUF], i_last % NBUF)
            rg.wait_all()

    phase("warmup")
    for i in range(Wm):
        step(None, i)
    if Wm:
        drain(Wm - 1)
    torch.cuda.synchronize()
    phase("timed")
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if not per_launch:
        ev[0][0].record(stream)
    for k in range(K):
        step(k, k)
    if not per_launch:
        ev[0][1].record(stream)
    drain(K - 1)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if per_launch:
        kms = np.array([a.elapsed_time(b) for a, b in ev])  # ms, kernel only
    else:
        kms = np.array([ev[0][0].elapsed_time(ev[0][1]) / K])  # mean ms per launch
    rank_stats = gather_rank_kernels(kms, world, backend) if distributed else None

    phase("parity")
    result = None
    if rank == 0:
        total_bytes = w["bytes"] * world * K
        value = total_bytes / elapsed / 2**30
        achieved = w["bytes"] / (kms.mean() * 1e-3) / 1e9
        key = f"{kernel_name(args.config, args.api, args.desc, args.form)}:config{args.config}:{n}"
        # the instantiation that really ran (never a re-derivation of the C
        # dispatch rule: a knob set at run time would fool that)
        launched = short_kernel(u.last_kernel())
        kern = launched.split("<")[0]
        traffic, traffic_src = load_traffic(args.pmc, key, launched)
        result = {
            "metric": metric_name(),
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "packets_per_s": round(n * world * K / elapsed, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16 one's-complement (u32 loads, u64 accumulate)",
            "data": "synthetic (splitmix64 payload, BASELINE.md seeds)",
            "config": {
                "workload": w["desc"],
                "packets_per_gpu": n,
                "algorithmic_bytes_per_gpu": w["bytes"],
                "api": {"spans": "uinet_cksum_spans" + ("32" if args.desc == "packed" else ""),
                        "strided": "uinet_cksum_strided"}[args.api]
                if args.config not in CHAIN_CONFIGS else "uinet_cksum_mbufs" if args.form == "mbufs"
                else {"wide": "uinet_cksum_chains", "packed": "uinet_cksum_chains32"}[args.desc],
                "parallelism": f"dp{world} packet shards" + (
                    f" + {'RCCL' if backend == 'nccl' else backend} gather of u16 results, "
                    "overlapped with the next step's kernel" if distributed else ""),
                "launcher": "torch.distributed.run" if distributed else "none",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kern,
                "instance": launched,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": w["bytes"],
                "kernel_ms_mean": round(float(kms.mean()), 5),
                "kernel_ms_min": round(float(kms.min()), 5),
            },
        }
        if args.config in CHAIN_CONFIGS:
            result["roofline"]["layout_floor"] = layout_floor_line(args.config, w, args.desc, kms,
                                                                   args.form)
        if distributed:
            # rank 0's kernel is the roofline above; these are every rank's
            result["ranks"] = rank_fields(rank_stats, w["bytes"], elapsed / K * 1e3)
        ref = scaling_ref(args.scaling_ref)
        if ref is not None:
            result["scaling_ref"] = ref
        if args.host_path:
            result["host_resident"] = host_path_rate(args, w)
    if world == 1 and rank == 0 and args.cpu_baseline == "auto":
        torch.cuda.synchronize()
        gpu_out = outs[(K - 1) % NBUF].cpu().view(torch.int16).numpy().view(np.uint16)
        keep = {}
        if args.host_offload == "auto":
            # the host-resident line runs once the host mbufs exist and before
            # the reference's passes, whose all-core runs leave the host's
            # cores clocked down for a while after
            def before_passes():
                try:
                    result["host_resident_cpu"] = host_offload_line(keep, n, w["bytes"], gpu_out)
                except Exception as e:  # a report, never the measurement: say what failed
                    result["host_resident_cpu"] = {"error": f"{type(e).__name__}: {e}"}
            keep["before_passes"] = before_passes
        result["cpu_baseline"] = cpu_baseline(args.config, w, gpu_out, args.cpu_threads, keep)
        result["bit_identical"] = result["cpu_baseline"]["bit_identical_to_gpu"]
        h = result.get("host_resident_cpu")
        if h is not None and "error" not in h:
            t1 = result["cpu_baseline"].get("one_thread_gibs")
            ref_1t = w["bytes"] / 2**30 / t1 if t1 else None
            h["reference_1thread_ms"] = round(ref_1t * 1e3, 3) if ref_1t else None
            h["reference_1thread_cpu_us_per_1k_pkts"] = (round(ref_1t * 1e6 / (n / 1000), 3)
                                                         if ref_1t else None)
        result["parity"] = {"packets": n, "against": result["cpu_baseline"]["kind"],
                            "how": "the last timed step's results vs the reference's "
                                   "in_cksum_* over the same bytes as host mbufs"}
    elif distributed and args.cpu_baseline == "auto":
        # every rank folds its own bytes with the reference on its host cores
        # (after the timed region), the expected results meet on rank 0 in
        # one more gather, and rank 0 compares them with the gathered GPU
        # results of the last timed step: the N > 1 line proves its own parity
        torch.cuda.synchronize()
        kind, want = reference_results(args.config, w, args.cpu_threads)
        from libuinet_amd.dist import gather_results

        allwant = gather_results(torch.from_numpy(want.view(np.int16)).to(
            "cuda" if backend == "nccl" else "cpu"), counts)
        if rank == 0:
            got = rg.result((K - 1) % NBUF).cpu().numpy().view(np.uint16)
            exp = allwant.cpu().numpy().view(np.uint16)
            result["bit_identical"] = bool(got.shape == exp.shape and np.array_equal(got, exp))
            result["parity"] = {"packets": int(exp.size), "against": kind,
                                "how": "the last timed step's gathered results vs the "
                                       "reference's in_cksum_* over every rank's bytes as host "
                                       "mbufs, computed on each rank's host cores and gathered"}
    if args.save_results and rank == 0:
        last = (K - 1) % NBUF
        res = rg.result(last) if rg is not None else outs[last].view(torch.int16)
        np.save(args.save_results, res.cpu().numpy().view(np.uint16))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        phase("teardown")
        dist.barrier()
        dist.destroy_process_group()
        wd.done()


def host_path_rate(args, w):
    """H2D of the whole batch from pinned host memory + kernel + D2H of the
    results (the rate when packets start and end in host memory)."""
    import torch
    import libuinet_amd as u

    if args.config not in ("2", "2rx", "5"):
        return None
    host = w["arena"].cpu().pin_memory()
    dev = torch.empty_like(w["arena"])
    res = torch.empty(w["n"], dtype=torch.uint16).pin_memory()
    out = torch.empty(w["n"], dtype=torch.uint16, device="cuda")
    s = torch.cuda.current_stream()
    best = 1e30
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.copy_(host, non_blocking=True)
        u.cksum_spans(dev, w["off"], w["len"], seed=w.get("seed"), out=out, len_hint=w["hint"],
                      stream=s)
        res.copy_(out, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return {"gibs": round(w["bytes"] / best / 2**30, 3), "ms": round(best * 1e3, 3),
            "what": "pinned host arena -> HBM copy + span kernel + u16 results -> pinned host"}


if __name__ == "__main__":
    main()
