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
    if not gpu_available():
        assert u.last_kernel() == ""  # nothing launched on this thread


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


def _ip_fold(h: bytes) -> int:
    s = sum(int.from_bytes(h[k:k + 2], "big") for k in range(0, len(h), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def test_in_cksum_update_inline(tmp_path):
    """The header's static inline uinet_in_cksum_update, compiled by gcc from
    include/uinet_cksum.h, against in_cksum.h:55-61 (ntohs(ip_sum) + 256,
    end-around carry, htons) on every ip_sum value, and as the forwarding
    path uses it: after ip_ttl -= 1 the header still verifies."""
    import ctypes

    src = tmp_path / "upd.c"
    src.write_text('#include "uinet_cksum.h"\nvoid upd(void *h) { uinet_in_cksum_update(h); }\n')
    so = tmp_path / "upd.so"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-shared", "-fPIC",
                    "-I", os.path.join(REPO, "include"), "-o", str(so), str(src)], check=True)
    upd = ctypes.CDLL(str(so)).upd
    upd.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_uint8 * 20)()
    for s in range(0x10000):  # every ip_sum
        buf[10], buf[11] = s >> 8, s & 0xFF
        upd(buf)
        t = s + 256
        assert (buf[10] << 8 | buf[11]) == (t + (t >> 16)) & 0xFFFF, s
    rng = np.random.default_rng(11)
    for _ in range(2000):
        h = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
        h[8] = int(rng.integers(1, 256))  # ttl >= 1
        h[10:12] = b"\0\0"
        h[10:12] = (~_ip_fold(h) & 0xFFFF).to_bytes(2, "big")
        assert _ip_fold(h) == 0xFFFF
        h[8] -= 1  # ip_fastfwd.c: ip->ip_ttl -= IPTTLDEC, then in_cksum_update(ip)
        ctypes.memmove(buf, bytes(h), 20)
        upd(buf)
        assert _ip_fold(bytes(buf)) == 0xFFFF


def test_in_cksum_update_matches_reference(tmp_path):
    """include/uinet_cksum.h's in_cksum_update against the reference's own
    (machine/in_cksum.h:46-72, compiled into oracle/_ref by oracle/Makefile as
    ref_in_cksum_update): every ip_sum value and 2000 random headers give the
    same 20 bytes."""
    import ctypes

    import oracle

    if not oracle.have_reference():
        pytest.skip("oracle/_ref/libref_cksum.so not built (needs /root/reference)")
    ref = ctypes.CDLL(oracle.REF_SO)
    if not hasattr(ref, "ref_in_cksum_update"):
        pytest.skip("oracle/_ref predates ref_in_cksum_update: run `make -C oracle ref`")
    ref.ref_in_cksum_update.argtypes = [ctypes.c_void_p]
    src = tmp_path / "upd.c"
    src.write_text('#include "uinet_cksum.h"\nvoid upd(void *h) { uinet_in_cksum_update(h); }\n')
    so = tmp_path / "upd.so"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-shared", "-fPIC",
                    "-I", os.path.join(REPO, "include"), "-o", str(so), str(src)], check=True)
    upd = ctypes.CDLL(str(so)).upd
    upd.argtypes = [ctypes.c_void_p]
    ours, theirs = (ctypes.c_uint8 * 20)(), (ctypes.c_uint8 * 20)()
    rng = np.random.default_rng(12)
    hdrs = [bytes([0x45, 0] + [0] * 8 + [s >> 8, s & 0xFF] + [0] * 8) for s in range(0x10000)]
    hdrs += [rng.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(2000)]
    for h in hdrs:
        ctypes.memmove(ours, h, 20)
        ctypes.memmove(theirs, h, 20)
        upd(ours)
        ref.ref_in_cksum_update(theirs)
        assert bytes(ours) == bytes(theirs), h.hex()


@pytest.mark.parametrize("order", ["reference_first", "opt_out_macro", "ours_only"])
def test_in_cksum_update_include_order(tmp_path, order):
    """The reference-named in_cksum_update shim next to a reference-style
    definition (in_cksum.h:46-61 under its _MACHINE_IN_CKSUM_H_ guard): with
    the reference header first, or with UINET_CKSUM_NO_IN_CKSUM_UPDATE, the
    unit compiles with one definition; alone, the shim provides it."""
    ref_like = ("#ifndef _MACHINE_IN_CKSUM_H_\n#define _MACHINE_IN_CKSUM_H_\n"
                "static inline void in_cksum_update(struct ip *ip) { (void)ip; }\n#endif\n")
    head = "#define IPVERSION 4\nstruct ip;\n"
    if order == "reference_first":
        body = head + ref_like + '#include "uinet_cksum.h"\n'
    elif order == "opt_out_macro":
        body = head + '#define UINET_CKSUM_NO_IN_CKSUM_UPDATE\n#include "uinet_cksum.h"\n' + \
            ref_like.replace("#ifndef _MACHINE_IN_CKSUM_H_\n#define _MACHINE_IN_CKSUM_H_\n", "") \
            .replace("#endif\n", "")
    else:
        body = head + '#include "uinet_cksum.h"\n'
    src = tmp_path / "order.c"
    src.write_text(body + "void use(struct ip *ip) { in_cksum_update(ip); }\n")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", "-I", os.path.join(REPO, "include"),
                    "-o", str(tmp_path / "order.o"), str(src)], check=True)


def test_set_tuning_validation():
    """uinet_cksum_set_tuning accepts each documented knob's range and rejects
    unknown keys and out-of-range values (no device needed)."""
    L = u.lib()
    ok = [("blocks_per_cu", 0), ("blocks_per_cu", 4096), ("chains_long", 0),
          ("chains_long", 16), ("xcd_remap", 0), ("host_threads", 64), ("multi_gather", 1),
          ("walk_device", 0), ("walk_device", 1), ("walk_device", 2), ("walk_device", 3),
          ("chains_wide", 2),
          ("span_fast", 0), ("span_fast", 1), ("span_fast", 2)]
    # chains_variant, spans_lut, spans_contig and spans_pipe 2 (k_spans_pp)
    # were removed in round 3; spans_sdesc, host_group and walk_prefetch 2 in
    # round 4; spans_pipe, spans_geo, chains_pass, chains_tile, host_pin and
    # walk_prefetch in round 6 (profiles/r06/pruned/)
    bad = [("blocks_per_cu", -1), ("chains_long", 15), ("xcd_remap", 2), ("host_threads", 0),
           ("spans_sdesc", 0), ("host_group", 1), ("chains_sweep", 2), ("multi_gather", 2),
           ("chains_variant", 0), ("spans_lut", 1), ("spans_contig", 0), ("walk_device", 4),
           ("walk_device", -1), ("chains_wide", 3), ("spans_pipe", 1), ("spans_geo", 0),
           ("chains_pass", 2), ("chains_tile", 0), ("host_pin", 0), ("walk_prefetch", 1),
           ("span_fast", 3), ("no_such_knob", 1)]
    try:
        for k, v in ok:
            assert L.uinet_cksum_set_tuning(k.encode(), v) == 0, (k, v)
        for k, v in bad:
            assert L.uinet_cksum_set_tuning(k.encode(), v) == u.EINVAL, (k, v)
        assert L.uinet_cksum_set_tuning(None, 1) == u.EINVAL
    finally:  # back to the defaults
        for k, v in [("blocks_per_cu", 0), ("chains_long", 128), ("xcd_remap", 1),
                     ("host_threads", min(16, os.cpu_count() or 1)), ("multi_gather", 0),
                     ("walk_device", 1), ("chains_wide", 0), ("span_fast", 1)]:
            L.uinet_cksum_set_tuning(k.encode(), v)


def test_header_lists_at_most_eight_knobs():
    """The knob list in include/uinet_cksum.h is the set the engine accepts,
    and it stays short."""
    import re

    with open(os.path.join(REPO, "include", "uinet_cksum.h")) as f:
        h = f.read()
    block = h[h.index("Performance knobs"):h.index("int uinet_cksum_set_tuning")]
    keys = re.findall(r'^ \*   "(\w+)"', block, re.M)
    assert 1 <= len(keys) <= 8, keys
    for k in keys:
        assert u.lib().uinet_cksum_set_tuning(k.encode(), -12345) == u.EINVAL
    assert set(keys) == {"blocks_per_cu", "chains_long", "xcd_remap", "host_threads",
                         "multi_gather", "walk_device", "chains_wide", "span_fast"}


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


def test_device_api_rejects_oversized_launch():
    """More than UINET_CKSUM_MAX_PACKETS packets in one launch is EINVAL,
    decided before anything touches a device; n == 0 is a no-op."""
    L = u.lib()
    p = 16  # never dereferenced: both checks come first
    big = 0x80000001
    assert L.uinet_cksum_spans(p, p, p, None, None, p, big, 0, 0, None) == u.EINVAL
    assert L.uinet_cksum_strided(p, 1500, 1500, None, p, big, 0, None) == u.EINVAL
    assert L.uinet_cksum_chains(p, p, p, p, None, None, None, p, big, 0, 0, None) == u.EINVAL
    assert L.uinet_cksum_spans(p, p, p, None, None, p, 0, 0, 0, None) == 0
    text = open(HEADER).read()
    assert "#define UINET_CKSUM_MAX_PACKETS 0x80000000u" in text
