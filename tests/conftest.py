"""Shared test setup.

Markers: `gpu` tests need an MI355X (run on the GPU box with `-m gpu`); everything else runs on
the CPU.  The CPU restatement (oracle/) is the checker for every parity test.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "path-tracer-cuda-opengl_amd")
for p in (os.path.join(PKG, "python"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a GPU (MI355X); run with -m gpu on the GPU box")


def _ensure_built():
    lib = os.path.join(PKG, "libpt.so")
    if not os.path.exists(lib):
        import subprocess
        subprocess.run(["make", "-s", "-C", PKG], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def pt():
    import ptamd
    return ptamd


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def gpu(pt):
    """The GPU tests fail (not skip) when no device is visible: there is no CPU fallback."""
    n = pt.device_count()
    assert n > 0, "no GPU visible to libpt.so"
    return 0
