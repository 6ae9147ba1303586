"""libuinet links unchanged against the engine.

integration/Makefile compiles the reference's netinet callers of the
checksum KPI (ip_input, ip_output, ip_icmp, ip_fastfwd, igmp, tcp_input,
tcp_output, tcp_lro, udp_usrreq) with libuinet's kernel flags and runs
libuinet's library step on them (lib/libuinet/Makefile:420-424): ld -r,
localize every defined symbol, globalize the API symlist.

* stock (in_cksum.c in MACHINE_SRCS, Makefile:274-275): the five checksum
  symbols are defined and localized inside the library object;
* patched (in_cksum.c removed): all five stay undefined, and the consumer's
  final link binds every one of them to libuinet_cksum.so.

Needs /root/reference (the build container); skipped elsewhere."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

from conftest import REPO

REF = "/root/reference"
SYMS = ("in_cksum_skip", "in_cksum_pseudo_header", "in_cksum_hdr", "in_pseudo", "in_addword")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "sys/netinet/ip_input.c")),
                                reason="reference tree absent")


@pytest.fixture(scope="module")
def out(tmp_path_factory):
    d = tmp_path_factory.mktemp("link")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "integration"), f"OUT={d}"],
                   check=True, capture_output=True, timeout=600)
    return d


def _nm(path):
    syms = {}
    for line in open(path):
        parts = line.split()
        if len(parts) >= 2:
            syms[parts[-1]] = parts[-2]
    return syms


def test_stock_library_defines_and_localizes(out):
    nm = _nm(out / "stock.nm")
    for s in SYMS:
        assert nm.get(s) == "t", (s, nm.get(s))  # defined, local: nothing outside binds it


def test_patched_library_leaves_them_undefined(out):
    nm = _nm(out / "patched.nm")
    for s in SYMS:
        assert nm.get(s) == "U", (s, nm.get(s))
    assert "in_cksumdata" not in nm


def test_final_link_binds_them_to_the_engine(out):
    trace = (out / "final_link.trace").read_text()
    lib = os.path.join(REPO, "libuinet_amd", "libuinet_cksum.so")
    for s in SYMS:
        assert f"patched.ro: reference to {s}" in trace
        assert f"{lib}: definition of {s}" in trace
    assert re.search(r"\(NEEDED\)\s+Shared library: \[libuinet_cksum\.so\]", trace)
