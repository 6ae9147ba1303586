"""The chunk-sum helper's machine code (CPU suite: hipcc cross-compiles for
gfx950, nothing runs).  hipcc has compiled ``__builtin_bit_cast(us2, v.y)``
taken straight off an ext-vector element as ``v.x``: the four
``v_dot2_u32_u16`` of a 16-byte chunk then read one register four times and
the checksum silently covers 4 of its 16 bytes.  tests/native/dot2_repro.hip
holds that pattern (k_elem) beside the engine's helper chunk_halves()
(libuinet_amd/csrc/cksum_device.h, k_helper) in the loop where it struck.
Every chunk's four dot2 in k_helper must read four distinct VGPRs."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

DOT2 = re.compile(r"^\s*v_dot2_u32_u16\s+(v\d+),\s*(v\d+),\s*([sv]\d+|\d+),\s*(\S+)")


def compile_isa(tmp_path) -> str:
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path / "dot2.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-I" + os.path.join(REPO, "include"),
                    "-I" + os.path.join(REPO, "libuinet_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "dot2_repro.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


def dot2_chains(isa: str, fn: str):
    """The kernel's v_dot2_u32_u16 source registers, grouped into chains of
    four that feed one another's accumulator (a chunk's four words)."""
    body = isa[isa.index(f"{fn}:"):]
    body = body[:body.index("s_endpgm")]
    ops = [DOT2.match(line).groups() for line in body.splitlines() if DOT2.match(line)]
    chains, cur = [], []
    for dst, src, _one, acc in ops:
        if cur and acc != cur[-1][0]:
            chains.append(cur)
            cur = []
        cur.append((dst, src))
    if cur:
        chains.append(cur)
    return ops, chains


def distinct_words(chain) -> bool:
    # a chain of 8 is two chunks back to back: check each chunk's four
    return all(len({s for _, s in chain[i:i + 4]}) == len(chain[i:i + 4])
               for i in range(0, len(chain), 4))


def test_helper_reads_four_words(tmp_path):
    isa = compile_isa(tmp_path)
    ops, chains = dot2_chains(isa, "k_helper")
    assert len(ops) == 8, ops  # two chunks of four words
    assert all(distinct_words(c) for c in chains), chains


def test_checker_sees_the_miscompile(tmp_path):
    """The checker is sensitive: on the element pattern it reports the
    collapse when this hipcc still produces it."""
    isa = compile_isa(tmp_path)
    _ops, chains = dot2_chains(isa, "k_elem")
    if all(distinct_words(c) for c in chains):
        pytest.skip("this hipcc compiles the element pattern correctly")
    assert not all(distinct_words(c) for c in chains)
