"""The host pool (libuinet_amd/csrc/host_pool.h) that walks and packs large
host-mbuf batches: built host-only with g++ under ThreadSanitizer and
stress-tested with concurrent callers -- every job runs exactly once."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_pool_stress(tmp_path):
    exe = tmp_path / "host_pool_test"
    src = os.path.join(HERE, "native", "host_pool_test.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-fsanitize=thread", src, "-o",
                    str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout and "ThreadSanitizer" not in r.stderr
