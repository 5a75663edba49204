# SPDX-License-Identifier: BSD-3-Clause
"""bench.py's host helpers (CPU only): the CPU baseline's view of the box and
the worker placements tools/node_workers.py and tools/cpu_baseline.py use."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _pkg(c):
    return bench._cpu_sysfs(c, "topology/physical_package_id")


def test_host_cpus():
    h = bench.host_cpus()
    assert h["allowed"] >= 1
    assert h["quota_cpus"] is None or h["quota_cpus"] > 0


def test_cpu_placement_spread():
    allowed = sorted(os.sched_getaffinity(0))
    assert bench.cpu_placement(1, "none") is None
    for n in (1, 2, len(allowed)):
        p = bench.cpu_placement(n)
        if p is None:  # fewer physical cores than n (SMT siblings are skipped), or no sysfs
            continue
        assert len(p) == n and len(set(p)) == n and set(p) <= set(allowed)
        # one hardware thread per core: no two of them SMT siblings
        cores = {bench._cpu_sysfs(c, "topology/thread_siblings_list") for c in p}
        assert len(cores) == n
    assert bench.cpu_placement(len(allowed) * 2 + 1) is None


def test_cpu_placement_one_socket():
    p = bench.cpu_placement(1, "socket")
    if p is None:
        return
    pkg = _pkg(p[0])
    q = bench.cpu_placement(2, "socket")
    if q is not None:
        assert {_pkg(c) for c in q} == {pkg}
