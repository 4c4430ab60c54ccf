"""Test configuration: marker registration, import paths, in-tree builds.

`-m "not gpu"` runs the oracle against the reference's golden vectors, the host logic and the
C-ABI library's exports (no GPU compute).  `-m gpu` runs the parity tests through the C ABI on
an MI355X.  The oracle (oracle/) is the checker only.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "qt-raytracer_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhippt.so on the device)")


def _ensure_built():
    lib = os.path.join(REPO, "qt-raytracer_amd", "libhippt.so")
    olib = os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all"], check=True)
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "qt-raytracer_amd")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
