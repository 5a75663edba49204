# SPDX-License-Identifier: BSD-3-Clause
"""Kernel time against batch size (full view, 64 B) for ring geometries,
interleaved in one process. One JSON line per (batch, geometry): median
kernel µs (HIP events) and the median wall µs of submit + sync (what one
burst waits for)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rings", default="2")
    ap.add_argument("--log2", default="10,12,14,16,18,20,22,24")
    args = ap.parse_args()
    import torch

    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    sizes = [1 << int(x) for x in args.log2.split(",")]
    kernels = [int(x) for x in args.rings.split(",")]
    nmax = max(sizes)
    frames, meta = S.stream(nmax, S.SEED_GPU_BASE, routes=topo.route_array())
    d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_out = torch.empty_like(d_in)
    d_v = torch.empty(nmax * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    kt = {(n, k): [] for n in sizes for k in kernels}
    wt = {(n, k): [] for n in sizes for k in kernels}
    for _ in range(args.rounds):
        for n in sizes:
            for k in kernels:
                fp.tune("ring", k)
                q.submit(d_in, d_out, d_meta, d_v, n)
                q.sync()
                walls = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    q.submit(d_in, d_out, d_meta, d_v, n)
                    q.sync()
                    walls.append(time.perf_counter() - t0)
                ms, cnt = q.kernel_ms(args.reps)
                kt[(n, k)].append(ms / cnt)
                wt[(n, k)].append(float(np.median(walls)))
    for n in sizes:
        for k in kernels:
            kus = float(np.median(kt[(n, k)])) * 1e3
            print(json.dumps({"batch": n, "ring": k, "kernel_us": round(kus, 2),
                              "wall_us": round(float(np.median(wt[(n, k)])) * 1e6, 2),
                              "mpps": round(n / kus, 1)}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
