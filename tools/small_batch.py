#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Small launches, one process, settings interleaved: the kernel time of a
--n-packet batch (HIP events, device-resident lines) and the host's
submit-to-done time of the same batch on pinned host memory (the node's
host-direct path: the kernel reads and writes the lines over PCIe), for each
gr_hip_tune setting given (e.g. stage_min_tiles=0 vs 4). Medians over --iters
launches after --warm, --rounds passes over the settings.

    python3 tools/small_batch.py --n 1024 --set stage_min_tiles=4 --set stage_min_tiles=0
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
    ap.add_argument("--n", default="1024", help="packets per launch, comma-separated sizes")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE[,KEY=VALUE]")
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    fp.tune("time_every", 1)
    sizes = [int(x) for x in a.n.split(",")]
    nmax = max(sizes)
    fr, me = S.stream(nmax, 0x5A11, routes=topo.route_array())
    d_in = torch.from_numpy(fr.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(me.view(np.uint8)).to(dev)
    d_out = torch.empty(nmax * abi.LINE, dtype=torch.uint8, device=dev)
    d_v = torch.empty(nmax * 8, dtype=torch.uint8, device=dev)
    h_in = torch.from_numpy(np.ascontiguousarray(fr)).pin_memory()
    h_me = torch.from_numpy(me.view(np.uint8).copy()).pin_memory()
    h_out = torch.zeros(nmax * abi.LINE, dtype=torch.uint8).pin_memory()
    h_v = torch.zeros(nmax * 8, dtype=torch.uint8).pin_memory()
    q = fp.queue(shared_stream(dev))
    settings = a.set or ["stage_min_tiles=4"]

    def apply(st):
        for kv in st.split(","):
            k, v = kv.split("=")
            fp.tune(k, int(v))

    res = {}
    for _ in range(a.rounds):
        for n in sizes:
            for st in settings:
                apply(st)
                for _ in range(a.warm):
                    q.submit(d_in, d_out, d_meta, d_v, n)
                q.sync()
                ks = []
                for _ in range(a.iters // 50):
                    for _ in range(50):
                        q.submit(d_in, d_out, d_meta, d_v, n)
                    q.sync()
                    ms, cnt = q.kernel_ms(50)
                    ks.append(ms / max(cnt, 1))
                lat = []
                for i in range(a.warm + a.iters):
                    t = time.perf_counter()
                    abi.check("gr_hip_fwd4_host", fp.lib.gr_hip_fwd4_host(
                        q._h, h_in.data_ptr(), h_me.data_ptr(), n, h_out.data_ptr(), h_v.data_ptr()))
                    if i >= a.warm:
                        lat.append(time.perf_counter() - t)
                r = res.setdefault((n, st), {"kernel_us": [], "host_us": []})
                r["kernel_us"].append(float(np.median(ks)) * 1e3)
                r["host_us"].append(float(np.median(lat)) * 1e6)
    for (n, st), r in res.items():
        print(json.dumps({"n": n, "set": st, "kernel_us": round(float(np.median(r["kernel_us"])), 2),
                          "host_submit_to_done_us": round(float(np.median(r["host_us"])), 2),
                          "rounds": {k: [round(x, 2) for x in v] for k, v in r.items()}}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
