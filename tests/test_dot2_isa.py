"""The chunk-sum helper's machine code (CPU suite: hipcc cross-compiles for
gfx950, nothing runs).  hipcc has compiled ``__builtin_bit_cast(us2, v.y)``
taken straight off an ext-vector element as ``v.x``: the four
``v_dot2_u32_u16`` of a 16-byte chunk then read one register four times and
the checksum silently covers 4 of its 16 bytes.  tests/native/dot2_repro.hip
holds that pattern (k_elem) beside the engine's helper chunk_halves()
(libuinet_amd/csrc/cksum_device.h, k_helper) in the loop where it struck.
Every chunk's four dot2 in k_helper must read four distinct VGPRs -- and so
must every chunk's four dot2 in the kernels the library ships, disassembled
from the built objects (libuinet_amd/build/*.o), where the helper is inlined
into other contexts."""
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
    # the dependency-chain reading used on the shipped kernels sees it too
    body = isa[isa.index("k_elem:"):]
    body = body[:body.index("s_endpgm")]
    deps = [c for c in dependency_chains(body) if len(c) % 4 == 0]
    assert deps and not all(len(set(c[i:i + 4])) == 4 for c in deps for i in range(0, len(c), 4))


# ---- the shipped kernels ------------------------------------------------------

LLVM = "/opt/rocm/lib/llvm/bin"
SHIPPED = ("cksum_spans", "cksum_chains", "cksum_kernels")
KERNEL = re.compile(r"^[0-9a-f]+ <(_Z\S+)>:", re.M)


def shipped_disasm(name: str, tmp_path) -> str:
    """The gfx950 code object of libuinet_amd/build/<name>.o, disassembled."""
    obj = os.path.join(REPO, "libuinet_amd", "build", f"{name}.o")
    if not os.path.exists(obj):
        pytest.skip(f"{obj} not built")
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("ROCm llvm tools not available")
    fat, co = tmp_path / f"{name}.fatbin", tmp_path / f"{name}.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, str(fat)],
                   check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                          check=True, capture_output=True, text=True).stdout


FIRST_OPERAND = re.compile(r"^\s*[a-z_0-9]+\s+(v\d+|v\[\d+:\d+\])")


def vregs(op: str):
    """'v7' -> ['v7'], 'v[4:7]' -> ['v4', ..., 'v7']."""
    if op.startswith("v["):
        a, b = (int(x) for x in op[2:-1].split(":"))
        return [f"v{i}" for i in range(a, b + 1)]
    return [op]


def dependency_chains(body: str):
    """v_dot2_u32_u16 source registers grouped by accumulator dependency (the
    next dot2 of a chain takes the previous one's result as its accumulator);
    chains may interleave."""
    open_, chains = {}, []
    for line in body.splitlines():
        m = DOT2.match(line)
        if not m:
            # any other write to a chain's result register ends that chain
            w = FIRST_OPERAND.match(line)
            if w:
                for reg in vregs(w.group(1)):
                    open_.pop(reg, None)
            continue
        dst, src, _one, acc = m.groups()
        ch = open_.pop(acc, None) if acc.startswith("v") else None
        if ch is None:
            ch = []
            chains.append(ch)
        ch.append(src)
        open_[dst] = ch
    return chains


@pytest.mark.parametrize("name", SHIPPED)
def test_shipped_kernels_read_four_words(name, tmp_path):
    dis = shipped_disasm(name, tmp_path)
    heads = list(KERNEL.finditer(dis))
    assert heads, "no kernels in the code object"
    chunks = 0
    for k, h in enumerate(heads):
        body = dis[h.end():heads[k + 1].start() if k + 1 < len(heads) else len(dis)]
        for ch in dependency_chains(body):
            if len(ch) % 4:
                # a lone dot2 is k_chains_pipe's mask-index / bin key, not a chunk sum
                assert len(ch) == 1, (h.group(1), ch)
                continue
            for i in range(0, len(ch), 4):
                assert len(set(ch[i:i + 4])) == 4, (h.group(1), ch)
                chunks += 1
    assert chunks >= 8, chunks  # the chunk sums are there and were checked
