#!/usr/bin/env python3
"""What the resident kernel's idle polls cost the PCIe link:
the PCIe-inclusive host path (gr_hip_fwd4_host_ex on pinned header lines,
the kernel's own PCIe loads and stores) timed with no resident kernel, then
with Q queues' rings idle on a live resident kernel (each queue's first ring
polls its descriptor in pinned host memory; one ring per queue, so the
probe sees the polls and not the CUs the rings hold), Q = 0, 8, 16, 32, in
turn and twice over. One JSON line per measurement.

    python tools/poll_cost_probe.py [--pkts 4194304] [--reps 5]
"""
import argparse
import json
import sys
import time

import numpy as np

sys.path[:0] = [".", "tests"]
from grout_amd import abi  # noqa: E402
from grout_amd import synth as S  # noqa: E402
from grout_amd import topology as T  # noqa: E402
from grout_amd.fwd import FastPath  # noqa: E402
from test_node_shim import mbufs_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pkts", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    fp = FastPath(0)
    topo = T.config_fullview(count=50_000)
    fp.load(topo)
    fp.tune("resident", 1)
    fp.tune("resident_ms", 10000)  # the kernel stays live (polling) through each measurement
    n = a.pkts
    fr, me = S.stream(n, 0x9011, routes=topo.route_array())
    lines = torch.from_numpy(np.ascontiguousarray(fr[:, :abi.LINE]).reshape(-1)).pin_memory()
    meta = torch.from_numpy(me.view(np.uint8)).pin_memory()
    out = torch.empty(n * abi.LINE, dtype=torch.uint8).pin_memory()
    v = torch.empty(n * 8, dtype=torch.uint8).pin_memory()
    hq = fp.queue()
    fx = fp.lib.gr_hip_fwd4_host_ex
    sfr, sme = S.stream(1024, 0x9012, routes=topo.route_array())

    def host_rate():
        abi.check("host", fx(hq._h, lines.data_ptr(), meta.data_ptr(), n, out.data_ptr(), abi.LINE, v.data_ptr()))
        t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            abi.check("host", fx(hq._h, lines.data_ptr(), meta.data_ptr(), n, out.data_ptr(), abi.LINE,
                                 v.data_ptr()))
            t.append(time.perf_counter() - t0)
        return n / float(np.median(t)) / 1e6

    fp.tune("resident_wgs", 1)  # one ring (its first) per idle queue: the polls, not the CUs they hold
    for rnd in range(2):
        for q_idle in (0, 8, 16, 32):
            fp.tune("resident_hold", 1)  # the live kernel leaves ...
            time.sleep(0.02)
            fp.tune("resident_hold", 0)  # ... and the idle queues' first batches launch it again
            qs = []
            for _ in range(q_idle):  # each takes its rings with one batch, then idles
                q = fp.queue()
                bufs, m = mbufs_for(sfr, sme)
                q.node_start(m)
                q.node_finish()
                qs.append(q)
            rate = host_rate()
            print(json.dumps(dict(round=rnd, idle_queues=q_idle, idle_first_rings=q_idle,
                                  live=fp.tune("resident_launches"), host_path_mpps=round(rate, 1))), flush=True)
            for q in qs:
                q.close()
            time.sleep(0.05)
    hq.close()
    fp.close()


if __name__ == "__main__":
    main()
