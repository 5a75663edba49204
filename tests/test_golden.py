# SPDX-License-Identifier: BSD-3-Clause
"""The committed golden fixtures (tests/golden/*.npz) are reproduced by the
oracle (CPU) and by the HIP fast path (GPU) bit for bit."""
import os

import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import topology as T
from golden_util import GOLDEN, topo_for, load, run_gpu

from golden.make_golden import digest


@pytest.mark.parametrize("name", ["corpus", "single", "fullview", "imix", "fullview6", "eth_cache"])
def test_topology_unchanged(name):
    g = load(name)
    assert digest(topo_for(name)) == str(g["topo_sha256"])


@pytest.mark.parametrize("name", ["corpus", "single", "fullview", "imix", "fullview6", "eth_cache"])
def test_oracle_reproduces_golden(name):
    g = load(name)
    out, v, st = oracle.Oracle(topo_for(name)).process(g["frames"], g["meta"], lines_only=bool(g["lines_only"]))
    assert np.array_equal(v, g["verdicts"])
    assert np.array_equal(out, g["out"])
    assert np.array_equal(st[g["stats_ifaces"]], g["stats"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["corpus", "single", "fullview", "imix", "fullview6", "eth_cache"])
def test_gpu_matches_golden(fastpath, name):
    g = load(name)
    out, v, st = run_gpu(fastpath, topo_for(name), g["frames"], g["meta"], lines_only=bool(g["lines_only"]))
    bad = np.nonzero(v != g["verdicts"])[0]
    labels = g["labels"]
    assert len(bad) == 0, [(labels[i] if len(labels) else i, v[i], g["verdicts"][i]) for i in bad[:10]]
    assert np.array_equal(out, g["out"])
    assert np.array_equal(st[g["stats_ifaces"]], g["stats"])
