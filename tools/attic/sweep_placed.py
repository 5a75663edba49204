"""Kernel variants in one process on ONE placed batch (gr_hip_batch_alloc +
gr_hip_batch_place, so the in/out placement is the same for every variant),
interleaved rounds: ring geometry x tile order (x nt). One JSON line per
variant (median / min kernel ms, HIP events).

    python tools/sweep_placed.py [--rings 0,1,...] [--orders 0,1,2] [--rounds 3]
"""
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
    ap.add_argument("--rings", default="0,1,2,3,4,5,6,7,8")
    ap.add_argument("--orders", default="0,1,2")
    ap.add_argument("--nt", default="1")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--workload", default="fullview64", choices=["fullview64", "single64"])
    a = ap.parse_args()
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    if a.workload == "single64":
        topo = T.config_single_route()
        kw = dict(dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    else:
        topo = T.config_fullview()
        kw = dict(routes=topo.route_array())
    fp = FastPath(0)
    fp.load(topo)
    n = 1 << 24
    frames, meta = S.stream(n, S.SEED_GPU_BASE, **kw)
    L = fp.lib
    b = fp.batch_alloc(n)
    for dst, src in ((b.in_frames, frames), (b.meta, meta)):
        abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
    fp.batch_place(b, 6)
    q = fp.queue()
    variants = list(itertools.product(ints(a.rings), ints(a.orders), ints(a.nt)))
    times = {v: [] for v in variants}
    ref = None
    vh = np.empty(n, dtype=abi.VERDICT_DT)
    for r in range(a.rounds):
        for v in variants:
            ring, order, nt = v
            fp.tune("ring", ring)
            fp.tune("tile_order", order)
            fp.tune("nt", nt)
            for _ in range(2 + a.reps):
                q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
            q.sync()
            ms, cnt = q.kernel_ms(a.reps)
            times[v].append(ms / cnt)
            if r == 0:
                abi.check("d2h", L.gr_hip_memcpy_d2h(fp.h, vh.ctypes.data, b.verdicts, vh.nbytes))
                h = int(vh.view(np.uint32).astype(np.uint64).sum())
                ref = h if ref is None else ref
                assert h == ref, ("verdicts differ", v)
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"workload": a.workload, "ring": v[0], "tile_order": v[1], "nt": v[2],
                          "median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                          "mpps": round(n / float(np.median(t)) / 1e3, 1)}), flush=True)
    fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
