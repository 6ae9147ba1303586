"""Shared fixtures.  `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


def _ensure_built() -> None:
    """Build the oracle and the engine in-tree if a fresh checkout lacks them
    (the same recipes __graft_entry__.build() runs)."""
    if not os.path.exists(os.path.join(REPO, "oracle", "liboracle_cksum.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all"], check=True)
    if not os.path.exists(os.path.join(REPO, "libuinet_amd", "libuinet_cksum.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "libuinet_amd")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def ora():
    import oracle

    return oracle.Oracle()


@pytest.fixture(scope="session")
def ref():
    import oracle

    if not oracle.have_reference():
        pytest.skip("oracle/_ref (reference object) not built here")
    return oracle.Reference()


def load_golden(name: str):
    return np.load(os.path.join(GOLDEN, f"golden_{name}.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def arena():
    """The golden arena, re-materialised at a 4 KiB-aligned address so every
    stored offset has the alignment the reference saw."""
    from libuinet_amd.mbuf import aligned_empty

    src = load_golden("arena")["arena"]
    a = aligned_empty(src.size)
    a[:] = src
    return a


@pytest.fixture(scope="session")
def golden():
    return load_golden


def read_pcap(path: str):
    """Minimal libpcap reader (linktype 1): returns a list of frame byte strings."""
    with open(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[:4], "little")
    order = "little" if magic in (0xA1B2C3D4, 0xA1B23C4D) else "big"
    linktype = int.from_bytes(data[20:24], order)
    assert linktype == 1, "Ethernet captures only"
    frames, pos = [], 24
    while pos + 16 <= len(data):
        incl = int.from_bytes(data[pos + 8 : pos + 12], order)
        frames.append(data[pos + 16 : pos + 16 + incl])
        pos += 16 + incl
    return frames


@pytest.fixture(scope="session")
def pcap_frames():
    return read_pcap(os.path.join(GOLDEN, "passive_extract_test.pcap"))


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="session")
def torch_dev():
    """torch on a visible gfx950 device (GPU tests only)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import libuinet_amd as u

    assert u.device_ok(), "device is not gfx950"
    return torch
