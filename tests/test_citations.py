# SPDX-License-Identifier: BSD-3-Clause
"""Every `file.c:N-M` citation in the repo's sources, tests and docs names
lines that exist in the mounted reference (or in the repo file it names),
and those lines hold what the citation talks about (an identifier from its
clause, or for a smoke script's line the address it configures):
tools/check_citations.py. Runs where /root/reference is mounted (this
container), skipped elsewhere; reads the reference as text only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/modules"), reason="reference not mounted")
def test_citations_resolve():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_citations.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-500:]
