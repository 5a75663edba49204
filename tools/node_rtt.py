#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""One node batch's round trip on an idle GPU: gr_hip_node_start (stage,
send) to gr_hip_node_finish (waited for, handed back onto the views), per
batch size, with the resident kernel (knob "resident") and with a launch per
batch, alternating. Medians over --iters batches after --warm. The batch's
RX accumulation is not in it (tests/perf_node_chain.py measures latency
from port_rx with it).

    python3 tools/node_rtt.py --sizes 64,1024,4096,15360
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,1024,4096,15360")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--warm", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--tiles", default="8", help="resident_tiles settings to compare, e.g. 8,32")
    ap.add_argument("--wgs", default="4", help="resident_wgs (rings per queue) settings to compare, e.g. 4,8")
    a = ap.parse_args()
    from golden_util import fresh_fastpath_state
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath
    from test_node_shim import mbufs_for

    fp = FastPath(0)
    topo = T.config_fullview(count=100_000)
    fresh_fastpath_state(fp, topo, {})
    sizes = [int(x) for x in a.sizes.split(",")]
    fr, me = S.stream(max(sizes), 0x277, routes=topo.route_array())
    res = {}
    for _ in range(a.rounds):
        for resident, wgs in [(0, 0)] + [(int(t), int(w)) for t in a.tiles.split(",") for w in a.wgs.split(",")]:
            fp.tune("resident", 1 if resident else 0)  # 0: a launch per batch
            if resident:
                fp.tune("resident_tiles", resident)
                fp.tune("resident_wgs", wgs)
            q = fp.queue()
            for n in sizes:
                times = []
                for i in range(a.warm + a.iters):
                    bufs, m = mbufs_for(fr[:n], me[:n])  # fresh views: the hand-back rewrites them
                    t = time.perf_counter()
                    q.node_start(m)
                    q.node_finish()
                    if i >= a.warm:
                        times.append(time.perf_counter() - t)
                res.setdefault((resident, wgs, n), []).append(float(np.median(times)) * 1e6)
            q.close()
    for (resident, wgs, n), v in sorted(res.items()):
        print(json.dumps({"resident_tiles": resident, "resident_wgs": wgs, "packets": n,
                          "rtt_us_median": round(float(np.median(v)), 1),
                          "rounds": [round(x, 1) for x in v]}), flush=True)
    fp.tune("resident", 0)
    fp.close()


if __name__ == "__main__":
    main()
