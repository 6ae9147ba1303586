#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE OBJECT.

Run in the build container (where /root/reference exists) after
``make -C oracle``: every expected value below is what
/root/reference/sys/amd64/amd64/in_cksum.c -- compiled unmodified with
libuinet's kernel flags into oracle/_ref/libref_cksum.so -- returns for the
stored inputs.  Inputs are plain data: one shared byte arena plus mbuf-chain
descriptions (offsets/lengths into the arena), so the fixtures stay small.

Files written:
  golden_arena.npz    arena bytes (splitmix64 payload, an all-0x00 and an
                      all-0xff region)
  golden_skip.npz     in_cksum_skip over random chains + edge cases
  golden_pseudo.npz   in_cksum_pseudo_header over random chains
  golden_hdr.npz      in_cksum_hdr at every address alignment
  golden_fold.npz     in_pseudo / in_addword
  golden_configs.npz  small samples in the shapes of BASELINE.json configs 1-3, 5
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from libuinet_amd.mbuf import MbufChains, aligned_empty, splitmix64_bytes, SEED_BASE  # noqa: E402
import oracle  # noqa: E402

ARENA = 256 * 1024
ZERO_AT = ARENA            # 4 KiB of 0x00
FF_AT = ARENA + 4096       # 4 KiB of 0xff
ARENA_TOTAL = ARENA + 8192


def make_arena() -> np.ndarray:
    a = aligned_empty(ARENA_TOTAL)
    splitmix64_bytes(ARENA, SEED_BASE + 100, out=a[:ARENA])
    a[ZERO_AT:ZERO_AT + 4096] = 0
    a[FF_AT:FF_AT + 4096] = 0xFF
    return a


def random_chains(rng, n, max_segs=5, region=(0, ARENA)):
    nseg = rng.integers(1, max_segs + 1, n)
    pkt_seg = np.concatenate([[0], np.cumsum(nseg)]).astype(np.int64)
    s = int(pkt_seg[-1])
    kind = rng.random(s)
    seg_len = np.where(kind < 0.10, 0,
               np.where(kind < 0.30, rng.integers(1, 9, s),
               np.where(kind < 0.75, rng.integers(1, 257, s), rng.integers(1, 1601, s))))
    lo, hi = region
    seg_off = rng.integers(lo, hi - 1601, s)
    return seg_off.astype(np.int64), seg_len.astype(np.int64), pkt_seg


def skip_cases(rng, arena, R):
    seg_off, seg_len, pkt_seg = random_chains(rng, 2500)
    # Edge chains over the all-zero and all-0xff regions.
    e_off, e_len, e_ps = random_chains(rng, 250, region=(ZERO_AT, ZERO_AT + 4096 + 1601))
    e_off = np.clip(e_off, ZERO_AT, ZERO_AT + 4096 - 1600)
    f_off, f_len, f_ps = random_chains(rng, 250, region=(FF_AT, FF_AT + 4096 + 1601))
    f_off = np.clip(f_off, FF_AT, FF_AT + 4096 - 1600)
    seg_off = np.concatenate([seg_off, e_off, f_off])
    seg_len = np.concatenate([seg_len, e_len, f_len])
    pkt_seg = np.concatenate([pkt_seg, e_ps[1:] + pkt_seg[-1], f_ps[1:] + pkt_seg[-1] + e_ps[-1]])
    n = pkt_seg.size - 1
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    tot[np.diff(pkt_seg) == 0] = 0
    mode = rng.random(n)
    skip = np.where(mode < 0.3, 0, (rng.random(n) * (tot + 1)).astype(np.int64))
    # skip exactly on an mbuf boundary for a fifth of the cases
    bnd = mode > 0.8
    cum = np.concatenate([[0], np.cumsum(seg_len)])
    k = (pkt_seg[:-1] + (rng.random(n) * np.diff(pkt_seg)).astype(np.int64))
    skip = np.where(bnd, cum[k] - cum[pkt_seg[:-1]], skip)
    length = skip + (rng.random(n) * (tot - skip + 40)).astype(np.int64)  # may exceed chain
    length = np.where(rng.random(n) < 0.05, skip, length)               # empty range
    length = np.where(rng.random(n) < 0.05, tot, length)                # whole chain
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    exp = R.skip_batch(ch.heads, length, skip)
    return dict(seg_off=seg_off, seg_len=seg_len, pkt_seg=pkt_seg, len=length.astype(np.int32),
                skip=skip.astype(np.int32), expected=exp)


def pseudo_cases(rng, arena, R):
    seg_off, seg_len, pkt_seg = random_chains(rng, 1500)
    n = pkt_seg.size - 1
    # in_cksum_pseudo_header reads the first mbuf: give every chain one with
    # room for the IP header (its callers m_pullup first, tcp_input.c:684-690).
    first = pkt_seg[:-1]
    seg_len[first] = np.maximum(seg_len[first], rng.integers(20, 200, n))
    tot = np.add.reduceat(seg_len, pkt_seg[:-1])
    off0 = np.minimum(rng.choice([0, 20, 24, 40, 60], n), seg_len[first])
    plen = (rng.random(n) * (tot - off0 + 30)).astype(np.int64)
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    proto = rng.choice([6, 17, 1, 0, 255], n)
    src[:8] = 0
    dst[:8] = 0
    proto[:8] = 0
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    exp = R.pseudo_header_batch(ch.heads, plen, off0, src, dst, proto)
    return dict(seg_off=seg_off, seg_len=seg_len, pkt_seg=pkt_seg, plen=plen.astype(np.int32),
                off0=off0.astype(np.int32), src=src.astype(np.uint32), dst=dst.astype(np.uint32),
                proto=proto.astype(np.uint8), expected=exp)


def hdr_cases(rng, arena, R):
    off = np.concatenate([rng.integers(0, ARENA - 64, 512), ZERO_AT + np.arange(16),
                          FF_AT + np.arange(16)]).astype(np.int64)
    exp = R.hdr_batch(arena.ctypes.data + off.astype(np.uint64))
    return dict(off=off, expected=exp)


def fold_cases(rng, R):
    a = rng.integers(0, 2**32, 2000, dtype=np.uint64)
    b = rng.integers(0, 2**32, 2000, dtype=np.uint64)
    c = rng.integers(0, 2**32, 2000, dtype=np.uint64)
    edge = np.array([0, 1, 0xffff, 0x10000, 0xfffe, 0xffffffff, 0x7fffffff, 0x80000000], np.uint64)
    g = np.array(np.meshgrid(edge, edge, edge)).reshape(3, -1)
    a, b, c = (np.concatenate([a, g[0]]), np.concatenate([b, g[1]]), np.concatenate([c, g[2]]))
    ps = np.array([R.in_pseudo(int(x), int(y), int(z)) for x, y, z in zip(a, b, c)], np.uint16)
    wa = np.concatenate([rng.integers(0, 2**16, 2000), [0, 0, 0xffff, 0xffff, 1, 0x8000]])
    wb = np.concatenate([rng.integers(0, 2**16, 2000), [0, 0xffff, 0xffff, 1, 0xffff, 0x8000]])
    aw = np.array([R.in_addword(int(x), int(y)) for x, y in zip(wa, wb)], np.uint16)
    return dict(pa=a.astype(np.uint32), pb=b.astype(np.uint32), pc=c.astype(np.uint32),
                pseudo=ps, wa=wa.astype(np.uint16), wb=wb.astype(np.uint16), addword=aw)


def config_cases(rng, arena, R):
    out = {}
    # config 2: 1500-B packets at stride 1500 (4-B aligned) and the RX variant
    # at stride 1514 with +14 (IP header at 2 mod 4), in_cksum_skip(m,1500,0).
    for tag, stride, base in (("c2", 1500, 0), ("c2rx", 1514, 14)):
        off = base + stride * np.arange(64, dtype=np.int64)
        ch = MbufChains.contiguous(arena, off, 1500)
        out[f"{tag}_off"] = off
        out[f"{tag}_expected"] = R.skip_batch(ch.heads, 1500, 0)
    # config 3: mixed 64/576/1500-B packets chained into random fragments at
    # random 0-7-B start offsets, in_cksum_skip(m, len, 20).
    lens = rng.choice([64, 576, 1500], 96)
    seg_off, seg_len, pkt_seg, cur = [], [], [0], 0
    for L in lens:
        start = int(rng.integers(0, ARENA - 2000)) & ~7
        pos = 0
        while pos < L:
            piece = int(min(L - pos, rng.integers(1, 257)))
            seg_off.append(start + pos + int(rng.integers(0, 8)))
            seg_len.append(piece)
            pos += piece
        pkt_seg.append(len(seg_off))
    seg_off = np.array(seg_off, np.int64)
    seg_len = np.array(seg_len, np.int64)
    pkt_seg = np.array(pkt_seg, np.int64)
    ch = MbufChains(arena, seg_off, seg_len, pkt_seg)
    out.update(c3_seg_off=seg_off, c3_seg_len=seg_len, c3_pkt_seg=pkt_seg,
               c3_len=lens.astype(np.int32),
               c3_expected=R.skip_batch(ch.heads, lens, 20))
    # config 5: 9000-B jumbo frames, in_cksum_pseudo_header(m, 8980, 20, src, dst, TCP/UDP).
    off = rng.integers(0, ARENA - 9100, 16).astype(np.int64)
    src = rng.integers(0, 2**32, 16, dtype=np.uint64)
    dst = rng.integers(0, 2**32, 16, dtype=np.uint64)
    proto = rng.choice([6, 17], 16)
    ch = MbufChains.contiguous(arena, off, 9000)
    out.update(c5_off=off, c5_src=src.astype(np.uint32), c5_dst=dst.astype(np.uint32),
               c5_proto=proto.astype(np.uint8),
               c5_expected=R.pseudo_header_batch(ch.heads, 8980, 20, src, dst, proto))
    return out


def main() -> None:
    R = oracle.Reference()
    rng = np.random.default_rng(0x75696E6574)
    arena = make_arena()
    np.savez_compressed(os.path.join(HERE, "golden_arena.npz"), arena=arena)
    np.savez_compressed(os.path.join(HERE, "golden_skip.npz"), **skip_cases(rng, arena, R))
    np.savez_compressed(os.path.join(HERE, "golden_pseudo.npz"), **pseudo_cases(rng, arena, R))
    np.savez_compressed(os.path.join(HERE, "golden_hdr.npz"), **hdr_cases(rng, arena, R))
    np.savez_compressed(os.path.join(HERE, "golden_fold.npz"), **fold_cases(rng, R))
    np.savez_compressed(os.path.join(HERE, "golden_configs.npz"), **config_cases(rng, arena, R))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
