# SPDX-License-Identifier: BSD-3-Clause
"""A/B the kernel variants in ONE process, interleaved rounds (methodology
rule 24 of cdna_hip_programming.md): staging x stats x workgroups per CU on
the headline workload. Prints one JSON line per variant (median / min ms)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--wg", default="0,2,4")
    args = ap.parse_args()
    import torch

    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = args.batch
    frames, meta = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array())
    d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_out = torch.empty_like(d_in)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(torch.cuda.current_stream(dev).cuda_stream)
    variants = []
    for st in (0, 1):
        for stats in (1, 0):
            for wg in [int(x) for x in args.wg.split(",")]:
                variants.append((st, stats, wg))
    times = {v: [] for v in variants}
    occ = {}
    for r in range(args.rounds):
        for v in variants:
            fp.tune("staging", v[0])
            fp.tune("stats", v[1])
            fp.tune("wg_per_cu", v[2])
            occ[v] = fp.tune("occupancy")
            q.submit(d_in, d_out, d_meta, d_v, n)  # warm
            for _ in range(args.reps):
                q.submit(d_in, d_out, d_meta, d_v, n)
            q.sync()
            ms, cnt = q.kernel_ms(args.reps)
            times[v].append(ms / cnt)
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"staging": ["lds", "direct"][v[0]], "stats": v[1], "wg_per_cu": v[2] or occ[v],
                          "median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                          "mpps": round(n / float(np.median(t)) / 1e3, 1)}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
