# SPDX-License-Identifier: BSD-3-Clause
"""Step-by-step run of tests/test_graph_walk.py's corpus walk with a line
printed before each native call (finds a host-side crash without a debugger)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import scenarios as SC  # noqa: E402
import test_graph_walk as G  # noqa: E402
from grout_amd import abi  # noqa: E402


def step(msg):
    print(msg, flush=True)


step("lib")
L = G.lib()
step("gh_init")
print(L.gh_init(0, 1024, 1 << 17, G.BATCH, G.BURST, G.DELAY_NS), flush=True)
step("graph_create")
print(L.gh_graph_create(b"gh"), flush=True)
from grout_amd.fwd import FastPath  # noqa: E402
fp = FastPath.borrow(L.gh_hip_ctx())
t, _ = SC.corpus_topology()
fr, me, lab = SC.corpus_arrays()
step("load")
G.load(fp, t)
step("queue_stats reset")
print(L.gh_queue_stats(None, 0, 1), flush=True)
ns0 = np.zeros(1, dtype=abi.NODE_STATS_DT)
step("node_stats")
print(L.gh_node_stats(ns0.ctypes.data, None), flush=True)
step("oracle")
o = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True)
step("walk")
got, lines, ns, walks = G.walk(fr, me)
step(f"walked {walks}")
