"""The register-only fold helpers on the GPU box, so the round's GPU record
covers every §8(a) function: in_pseudo / in_addword against the reference
object's golden grid (in_cksum.c:172-191), and in_cksum_update
(in_cksum.h:55-61) through the header inline, next to a device batch of the
same headers.  These functions fold two or three register words on the
calling thread by design (DESIGN.md boundary item 1); the device path below
is the batch API's in_cksum_hdr_batch."""
import os
import subprocess

import numpy as np
import pytest

import libuinet_amd as u

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_in_pseudo_in_addword_golden(torch_dev, golden):
    g = golden("fold")
    got = [u.in_pseudo(int(a), int(b), int(c)) for a, b, c in zip(g["pa"], g["pb"], g["pc"])]
    np.testing.assert_array_equal(got, g["pseudo"])
    got = [u.in_addword(int(a), int(b)) for a, b in zip(g["wa"], g["wb"])]
    np.testing.assert_array_equal(got, g["addword"])


def test_in_cksum_update_then_device_verify(torch_dev, ora, tmp_path):
    """Forwarding: ip_ttl -= 1 then in_cksum_update (ip_fastfwd.c), then the
    updated headers verify to 0 through the GPU batch in_cksum_hdr_batch and
    the oracle alike."""
    import ctypes

    src = tmp_path / "upd.c"
    # the reference's name and type: struct ip * with IPVERSION 4 (in_cksum.h:46-61)
    src.write_text('#define IPVERSION 4\nstruct ip;\n#include "uinet_cksum.h"\n'
                   'void upd(void *h) { in_cksum_update((struct ip *)h); }\n')
    so = tmp_path / "upd.so"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-shared", "-fPIC",
                    "-I", os.path.join(REPO, "include"), "-o", str(so), str(src)], check=True)
    upd = ctypes.CDLL(str(so)).upd
    upd.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(355)
    n = 4096
    hdrs = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    hdrs[:, 0] = 0x45
    hdrs[:, 8] = rng.integers(1, 256, n)  # ttl >= 1
    hdrs[:, 10:12] = 0
    words = hdrs.reshape(n, 10, 2).astype(np.uint32)
    s = (words[:, :, 0] << 8 | words[:, :, 1]).sum(axis=1)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    ck = ~s & 0xFFFF
    hdrs[:, 10], hdrs[:, 11] = ck >> 8, ck & 0xFF
    hdrs[:, 8] -= 1
    for i in range(n):
        row = np.ascontiguousarray(hdrs[i])
        upd(row.ctypes.data)
        hdrs[i] = row
    # in_cksum_hdr over each updated header: 0 when it verifies
    buf = np.ascontiguousarray(hdrs).reshape(-1)
    ips = [buf.ctypes.data + 20 * i for i in range(n)]
    got = u.in_cksum_hdr_batch(ips)
    np.testing.assert_array_equal(got, np.zeros(n, np.uint32))
    np.testing.assert_array_equal(ora.hdr_batch(np.array(ips, np.uint64)), np.zeros(n))
