# SPDX-License-Identifier: BSD-3-Clause
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# a failing HIP call inside libgrout_hip.so names itself on stderr (captured
# with the failing test's output)
os.environ.setdefault("GR_HIP_TRACE_ERRORS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgrout_hip.so)")


def _built():
    return all(os.path.exists(os.path.join(ROOT, p)) for p in
               ("grout_amd/libgrout_hip.so", "grout_amd/libgrout_host.so", "oracle/liboracle.so"))


@pytest.fixture(scope="session", autouse=True)
def built_libs():
    if not _built():
        subprocess.run(["make", "-C", ROOT, "-j8"], check=True, stdout=subprocess.DEVNULL)
    yield


@pytest.fixture(scope="session")
def fastpath():
    """One HIP context for the whole GPU session (one process, one device)."""
    from grout_amd.fwd import FastPath
    fp = FastPath(0)
    yield fp
    fp.close()
