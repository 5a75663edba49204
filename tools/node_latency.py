# SPDX-License-Identifier: BSD-3-Clause
"""Latency of the rte_graph node's walk (gr_hip_node_process: stage, forward
on the GPU, hand back) against the flush size, from one worker thread: the
node flushes when the RX queue drains, so small flushes are what a lightly
loaded grout worker sees. Median of --reps calls per size,
on warm mbufs (the same ones each call; reset in between, outside the timing).

    python tools/node_latency.py > out.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,256,1024,4096,16384,65536,262144")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    sizes = [int(x) for x in args.sizes.split(",")]
    nmax = max(sizes)
    fr, me = S.stream(nmax, S.SEED_GPU_BASE, routes=topo.route_array())
    bufs = np.zeros((nmax, 256), dtype=np.uint8)
    mb = np.zeros(nmax, dtype=abi.MBUF_DT)
    mb["frame"] = bufs.ctypes.data + np.arange(nmax, dtype=np.uint64) * 256
    mb["pkt_len"] = me["pkt_len"]
    mb["data_len"] = me["pkt_len"]
    mb["data_off"] = 128
    mb["rss"] = me["rss"]
    mb["iface"] = me["iface"]
    q = fp.queue()
    for n in sizes:
        m = mb[:n].copy()
        t = []
        for r in range(args.reps + 3):
            m[:] = mb[:n]
            bufs[:n, :64] = fr[:n]
            t0 = time.perf_counter()
            q.node_process(m)
            if r >= 3:
                t.append(time.perf_counter() - t0)
        d = float(np.median(t))
        print(json.dumps({"flush_pkts": n, "us_median": round(d * 1e6, 1), "us_p90": round(float(np.percentile(t, 90)) * 1e6, 1),
                          "mpps": round(n / d / 1e6, 2), "mode": "staged lines (default)"}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
