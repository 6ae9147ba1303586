"""The device chain walk's pointer translation (libuinet_amd/csrc/walk_xlate.h)
run on the host: an address it accepts is read by the GPU, so it must accept
exactly the byte ranges that lie inside one registered region."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "libuinet_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_walk_xlate_matches_linear_scan(tmp_path):
    exe = tmp_path / "walk_xlate_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", f"-I{CSRC}",
                    os.path.join(HERE, "native", "walk_xlate_test.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout
    hits = int(r.stdout.split("hits=")[1].split()[0])
    assert hits > 1000  # the probes do land inside regions
