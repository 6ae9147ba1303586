"""Offline replay of the reference's own capture through the receive path's
checksum stages (SURVEY.md 8f item 3 without libpcap or the stack itself):
tests/native/pcap_replay.c reads lib/libuinet_demo/passive_extract_test.pcap
(copied to tests/golden/), restates the verdict steps of ip_input /
tcp_input / udp_input in the stack's order and prints the bad-sum counters
(uinet_api.c:170 exports them as tcps_rcvbadsum / ips_badsum).

CPU: with the engine's per-call functions every counter is 0 on the clean
capture, and on a copy with 30 flipped bits the counters equal those the
reference's own functions (oracle/_ref) give.  GPU: the same with every
frame first marked by uinet_cksum_rx_offload, the stack reading the marks."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PCAP = os.path.join(REPO, "tests", "golden", "passive_extract_test.pcap")
LIBDIR = os.path.join(REPO, "libuinet_amd")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_cksum.so")


@pytest.fixture(scope="module")
def replay(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    if not os.path.exists(os.path.join(LIBDIR, "libuinet_cksum.so")):
        pytest.skip("engine library not built")
    exe = str(tmp_path_factory.mktemp("replay") / "pcap_replay")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-std=c11", "-D_GNU_SOURCE",
                    "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "native", "pcap_replay.c"), "-o", exe,
                    "-L", LIBDIR, "-luinet_cksum", f"-Wl,-rpath,{LIBDIR}", "-ldl"], check=True)

    def run(mode: str, corrupt: int = 0) -> dict:
        r = subprocess.run([exe, PCAP, mode, str(corrupt), REF_SO], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, (mode, r.returncode, r.stderr)
        return {k: int(v) for k, v in (t.split("=") for t in r.stdout.split())}

    return run


def _verdicts(c: dict) -> dict:
    return {k: v for k, v in c.items() if k != "marked"}


def test_replay_capture_software_path(replay):
    """The engine's per-call functions: zero bad sums on the reference's
    capture, the reference's own counters on a corrupted copy."""
    if not os.path.exists(REF_SO):
        pytest.skip("reference object not built")
    clean = replay("software")
    assert clean["frames"] == clean["ipv4"] == clean["tcp"] == 113
    assert clean["ips_badsum"] == clean["tcps_rcvbadsum"] == clean["udps_badsum"] == 0
    assert _verdicts(clean) == _verdicts(replay("reference"))
    bad = replay("software", 30)
    assert bad["ips_badsum"] + bad["tcps_rcvbadsum"] == 30
    assert _verdicts(bad) == _verdicts(replay("reference", 30))


@pytest.mark.gpu
def test_replay_capture_rx_offload(replay):
    """Every frame marked by the GPU RX hook first: the stack reads the marks
    and reaches the reference's verdicts, zero bad sums on the capture."""
    import libuinet_amd as u

    if not u.device_ok():
        pytest.skip("no gfx950 device")
    clean = replay("offload")
    assert clean["marked"] == 113
    assert clean["ips_badsum"] == clean["tcps_rcvbadsum"] == clean["udps_badsum"] == 0
    assert _verdicts(clean) == _verdicts(replay("reference"))
    bad = replay("offload", 30)
    assert bad["ips_badsum"] + bad["tcps_rcvbadsum"] == 30
    assert _verdicts(bad) == _verdicts(replay("reference", 30))
