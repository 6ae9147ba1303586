"""The per-call drop-in ABI (in_cksum_skip / in_cksum / in_cksum_pseudo_header /
in_cksum_hdr / in6_cksum) is a host fold that never touches a device and
never fails, like the reference (/root/reference/sys/amd64/amd64/in_cksum.c
:193-285 has no error path).  Checked here on CPU:

* through ctypes against every golden vector of the reference object;
* from a plain C consumer compiled against include/uinet_cksum.h and linked
  with -luinet_cksum, run with no visible GPU (HIP_VISIBLE_DEVICES empty);
* against the oracle on random chains with 0-7-B start offsets, empty mbufs
  and skip/len edges;
* the batch entry points keep refusing to run without a device
  (test_abi.py::test_no_silent_cpu_fallback)."""
from __future__ import annotations

import os
import struct
import subprocess

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes

from conftest import REPO


def test_golden_skip_per_call(arena, golden):
    g = golden("skip")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    for i in range(ch.n):
        assert u.in_cksum_skip(ch.head(i), int(g["len"][i]), int(g["skip"][i])) == g["expected"][i], i
        if g["skip"][i] == 0:
            assert u.in_cksum(ch.head(i), int(g["len"][i])) == g["expected"][i]


def test_golden_pseudo_per_call(arena, golden):
    g = golden("pseudo")
    ch = MbufChains(arena, g["seg_off"], g["seg_len"], g["pkt_seg"])
    for i in range(ch.n):
        assert u.in_cksum_pseudo_header(ch.head(i), int(g["plen"][i]), int(g["off0"][i]),
                                        int(g["src"][i]), int(g["dst"][i]),
                                        int(g["proto"][i])) == g["expected"][i], i


def test_golden_hdr_per_call(arena, golden):
    g = golden("hdr")
    for off, want in zip(g["off"], g["expected"]):
        assert u.in_cksum_hdr(arena.ctypes.data + int(off)) == want, off


def test_golden_configs_per_call(arena, golden):
    g = golden("configs")
    for tag in ("c2", "c2rx"):
        ch = MbufChains.contiguous(arena, g[f"{tag}_off"], 1500)
        assert [u.in_cksum(ch.head(i), 1500) for i in range(ch.n)] == list(g[f"{tag}_expected"])
    ch = MbufChains(arena, g["c3_seg_off"], g["c3_seg_len"], g["c3_pkt_seg"])
    assert [u.in_cksum_skip(ch.head(i), int(g["c3_len"][i]), 20)
            for i in range(ch.n)] == list(g["c3_expected"])
    ch = MbufChains.contiguous(arena, g["c5_off"], 9000)
    assert [u.in_cksum_pseudo_header(ch.head(i), 8980, 20, int(g["c5_src"][i]),
                                     int(g["c5_dst"][i]), int(g["c5_proto"][i]))
            for i in range(ch.n)] == list(g["c5_expected"])


def test_random_chains_vs_oracle(ora):
    rng = np.random.default_rng(77)
    arena = aligned_empty(1 << 20)
    splitmix64_bytes(arena.size, 77, out=arena)
    arena[:4096] = 0        # all-zero and all-0xff regions: the 0xffff / 0 edge
    arena[4096:8192] = 0xFF
    seg_off, seg_len, pkt_seg = [], [], [0]
    for _ in range(3000):
        k = int(rng.integers(1, 6))
        base = int(rng.choice([0, 4096, int(rng.integers(8192, arena.size - 9000))]))
        for _ in range(k):
            ln = int(rng.choice([0, 1, 2, 3, int(rng.integers(0, 1600))]))
            seg_off.append(base + int(rng.integers(0, 8)))
            seg_len.append(ln)
            base += ln + 8
        pkt_seg.append(len(seg_off))
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    tot = np.add.reduceat(np.array(seg_len), np.array(pkt_seg[:-1]))
    length = np.minimum(tot, rng.integers(0, 2 * tot + 2))
    skip = np.minimum(length, rng.integers(0, 64, ch.n))
    want = ora.skip_batch(ch.heads, length, skip)
    got = [u.in_cksum_skip(ch.head(i), int(length[i]), int(skip[i])) for i in range(ch.n)]
    np.testing.assert_array_equal(np.array(got, np.uint16), want)


def _write_input(path, arena, golden):
    gs, gp, gh = golden("skip"), golden("pseudo"), golden("hdr")
    seg_off = np.concatenate([gs["seg_off"], gp["seg_off"]]).astype(np.uint64)
    seg_len = np.concatenate([gs["seg_len"], gp["seg_len"]]).astype(np.int32)
    pkt_seg = np.concatenate([gs["pkt_seg"], gp["pkt_seg"][1:] + gs["pkt_seg"][-1]]).astype(np.uint32)
    recs = []
    for i in range(gs["len"].size):
        recs.append(struct.pack("<BiiIIB", 0, int(gs["len"][i]), int(gs["skip"][i]), 0, 0, 0))
    for i in range(gp["plen"].size):
        recs.append(struct.pack("<BiiIIB", 1, int(gp["plen"][i]), int(gp["off0"][i]),
                                int(gp["src"][i]), int(gp["dst"][i]), int(gp["proto"][i])))
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", arena.size))
        f.write(arena.tobytes())
        f.write(struct.pack("<II", seg_off.size, pkt_seg.size - 1))
        f.write(seg_off.tobytes() + seg_len.tobytes() + pkt_seg.tobytes())
        f.write(b"".join(recs))
        f.write(struct.pack("<I", gh["off"].size))
        f.write(gh["off"].astype(np.uint64).tobytes())
    return np.concatenate([gs["expected"], gp["expected"]]), gh["expected"]


def test_c_consumer_without_gpu(tmp_path, arena, golden):
    exe = tmp_path / "percall_golden"
    libdir = os.path.dirname(u.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Werror",
                    "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "native", "percall_golden.c"),
                    "-L", libdir, "-luinet_cksum", f"-Wl,-rpath,{libdir}", "-o", str(exe)],
                   check=True)
    inp = tmp_path / "in.bin"
    want16, want32 = _write_input(str(inp), arena, golden)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([str(exe), str(inp)], capture_output=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    n16 = want16.size
    got16 = np.frombuffer(r.stdout[: 2 * n16], np.uint16)
    got32 = np.frombuffer(r.stdout[2 * n16:], np.uint32)
    np.testing.assert_array_equal(got16, want16)
    np.testing.assert_array_equal(got32, want32)


def test_percall_fold_sanitized(tmp_path, arena, golden):
    """The per-call fold (csrc/cksum_percall.cpp) built with AddressSanitizer
    and UndefinedBehaviorSanitizer into the same C consumer, linked through
    a test-only shim instead of the HIP library: every golden chain, pseudo
    header and IP header, with no out-of-piece read, unaligned-access UB or
    overflow reported, and the golden results."""
    flags = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
             "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"),
             "-I", os.path.join(REPO, "libuinet_amd", "csrc")]
    objs = []
    for cc, std, src in (("gcc", "-std=c11", "tests/native/percall_golden.c"),
                         ("g++", "-std=c++17", "libuinet_amd/csrc/cksum_percall.cpp"),
                         ("g++", "-std=c++17", "tests/native/percall_shim.cpp")):
        o = tmp_path / (os.path.basename(src) + ".o")
        subprocess.run([cc, std, *flags, "-c", os.path.join(REPO, src), "-o", str(o)], check=True)
        objs.append(str(o))
    exe = tmp_path / "percall_san"
    subprocess.run(["g++", "-fsanitize=address,undefined", *objs, "-o", str(exe)], check=True)
    inp = tmp_path / "in.bin"
    want16, want32 = _write_input(str(inp), arena, golden)
    # verify_asan_link_order=0: the environment may preload a library of its own
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(inp)], capture_output=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"runtime error" not in r.stderr, r.stderr.decode()[-3000:]
    n16 = want16.size
    np.testing.assert_array_equal(np.frombuffer(r.stdout[: 2 * n16], np.uint16), want16)
    np.testing.assert_array_equal(np.frombuffer(r.stdout[2 * n16:], np.uint32), want32)


@pytest.mark.parametrize("length", [0, 1, 19, 20, 21, 1500, 65535])
def test_per_call_edge_lengths(ora, length):
    arena = aligned_empty(70000)
    splitmix64_bytes(arena.size, length, out=arena)
    for off in range(8):
        ch = MbufChains.contiguous(arena, [off], [length])
        for skip in (0, 1, min(length, 20)):
            want = ora.skip_batch(ch.heads, length, skip)[0]
            assert u.in_cksum_skip(ch.head(0), length, skip) == want, (off, skip)


def test_per_call_simd_edges(ora):
    """Piece lengths around the vector folds' thresholds and steps (AVX2 from
    128 B in 64-B steps, AVX-512 from 256 B in 128-B steps, cksum_percall.cpp)
    at every start offset within a 64-B line, whole and cut by skip, against
    the oracle: the scalar tail after a vector run keeps each byte's weight."""
    arena = aligned_empty(1 << 16)
    splitmix64_bytes(arena.size, 99, out=arena)
    lengths = [127, 128, 129, 191, 192, 255, 256, 257, 383, 384, 385, 511, 512, 513, 1023, 4097]
    offs, lens = [], []
    for ln in lengths:
        for off in range(64):
            offs.append(64 * len(offs) % 40000 + off)
            lens.append(ln)
    ch = MbufChains(arena, offs, lens, np.arange(len(offs) + 1))
    for skip in (0, 1, 3):
        want = ora.skip_batch(ch.heads, np.array(lens), skip)
        got = np.array([u.in_cksum_skip(ch.head(i), lens[i], skip) for i in range(ch.n)])
        np.testing.assert_array_equal(got, want)
