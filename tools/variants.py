# SPDX-License-Identifier: BSD-3-Clause
"""A/B the kernel variants in ONE process, interleaved rounds (methodology
rule 24 of cdna_hip_programming.md) on a bench workload: counters on/off,
nontemporal loads/stores, grid shape, FIB entry size. One JSON line per
variant (median / min kernel ms from the library's HIP events)."""
import argparse
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ints(s):
    return [int(x) for x in s.split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--workload", default="fullview64", choices=["fullview64", "single64", "fullview6"])
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--wg", default="0,6")
    ap.add_argument("--fib16", default="2,1,0", help="gr_hip_tune fib_format values")
    ap.add_argument("--stats", default="1")
    ap.add_argument("--ring", default="1", help="ring geometries (fwd4_ring.hip ring_cfgN)")
    ap.add_argument("--place", default="out", help="out = separate lines; in = in place")
    args = ap.parse_args()
    import torch

    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    if args.workload == "single64":
        topo = T.config_single_route()
        kw = dict(dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    elif args.workload == "fullview6":
        topo = T.config_fullview6()
    else:
        topo = T.config_fullview()
        kw = dict(routes=topo.route_array())
    fp = FastPath(0)
    fp.load(topo)
    n = args.batch
    if args.workload == "fullview6":
        r6 = topo.route6_array()
        frames, meta = S.stream6(n, S.SEED_GPU_BASE, r6[r6["prefixlen"] < 128])
    else:
        frames, meta = S.stream(n, S.SEED_GPU_BASE, **kw)
    d_src = torch.from_numpy(frames.reshape(-1)).to(dev)
    bufs = [torch.empty_like(d_src) for _ in range(args.reps + 1)]
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_out = torch.empty_like(d_src)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    variants = list(itertools.product(ints(args.fib16), ints(args.stats), ints(args.nt), ints(args.wg),
                                      ints(args.ring), args.place.split(",")))
    times = {v: [] for v in variants}
    refv = refo = None
    for r in range(args.rounds):
        for v in variants:
            f16, st, nt, wg, ring, place = v
            fp.tune("ring", ring)
            if args.workload != "fullview6":
                fp.tune("fib_format", f16)
                fp.fib_commit(T.VRF_MAIN)  # re-uploads when the format changes
            fp.tune("stats", st)
            fp.tune("nt", nt)
            fp.tune("wg_per_cu", wg)
            # every launch gets a fresh batch (in place rewrites it), all
            # copied before the launches, for every variant alike; the warm
            # launch absorbs the write-back of the last copy
            for b in bufs:
                b.copy_(d_src)
            for b in bufs:
                q.submit(b, b if place != "out" else d_out, d_meta, d_v, n)
            q.sync()
            ms, cnt = q.kernel_ms(args.reps)
            times[v].append(ms / cnt)
            if r == 0:  # every variant must produce the same verdicts and lines
                hv = int(torch.sum(d_v.view(torch.int32).to(torch.int64)).item())
                refv = hv if refv is None else refv
                assert hv == refv, ("verdicts differ", v, hv, refv)
                if place == "out":
                    ho = int(torch.sum(d_out.view(torch.int32).to(torch.int64)).item())
                    refo = ho if refo is None else refo
                    assert ho == refo, ("lines differ", v, ho, refo)
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"workload": args.workload, "fib16": v[0], "stats": v[1], "nt": v[2],
                          "wg_per_cu": v[3], "ring": v[4], "place": v[5], "median_ms": round(float(np.median(t)), 4),
                          "min_ms": round(float(t.min()), 4), "mpps": round(n / float(np.median(t)) / 1e3, 1)}),
              flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
