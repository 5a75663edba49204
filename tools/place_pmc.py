#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Which counter separates slow buffer pairings from fast ones (VERDICT r04,
next #5)? The headline kernel over one input batch (config 3, 2^24 x 64 B)
and each of --cands separately allocated output-line buffers in turn
(plain torch allocations, as the bench's plain leg), --steps launches each
after --warm untimed ones. Run it under rocprofv3 --pmc, one pass per counter
group (each pass a new process: new pages, its own fast and slow pairings):
within a pass every candidate has its dispatches' mean duration and counters,
and `--analyze` correlates each counter per launch with the duration over
the candidates of each pass.

    rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum ... -d OUT/p0 -o run -- python3 tools/place_pmc.py
    python3 tools/place_pmc.py --analyze OUT
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    fp = FastPath(0)
    topo = T.config_fullview()
    fp.load(topo)
    n = a.batch
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    outs = [torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev) for _ in range(a.cands)]
    torch.cuda.synchronize()
    q = fp.queue(shared_stream(dev))
    fp.tune("time_every", 1)
    res = []
    for c, d_out in enumerate(outs):
        for _ in range(a.warm):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        q.kernel_ms(10 ** 6)  # drop the warm-up's events
        for _ in range(a.steps):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        ms, cnt = q.kernel_ms(a.steps)
        res.append(round(ms / max(cnt, 1), 4))
    print(json.dumps({"cands": a.cands, "warm": a.warm, "steps": a.steps, "kernel_ms": res}), flush=True)
    q.close()
    fp.close()


def analyze(a):
    out = {}
    for f in sorted(glob.glob(os.path.join(a.analyze, "**", "*counter_collection.csv"), recursive=True)):
        d = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            if "ring" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            e = d.setdefault(k, {"dur_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ks = list(d)
        per = a.warm + a.steps
        if len(ks) < a.cands * per:
            continue
        rows = []
        for c in range(a.cands):
            sel = [d[k] for k in ks[c * per + a.warm:(c + 1) * per]]
            rows.append({x: float(np.mean([s[x] for s in sel])) for x in sel[0]})
        dur = np.array([r["dur_ms"] for r in rows])
        corr = {}
        for x in rows[0]:
            if x == "dur_ms":
                continue
            v = np.array([r[x] for r in rows])
            corr[x] = {"r": round(float(np.corrcoef(v, dur)[0, 1]), 3) if v.std() > 0 else None,
                       "fast": round(float(v[dur.argmin()]), 0), "slow": round(float(v[dur.argmax()]), 0),
                       "slow_over_fast": round(float(v[dur.argmax()] / v[dur.argmin()]), 3) if v[dur.argmin()] else None}
        out[os.path.relpath(f, a.analyze)] = {"dur_ms": [round(x, 4) for x in dur],
                                              "spread": round(float(dur.max() / dur.min()), 3), "counters": corr}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", type=int, default=10)
    ap.add_argument("--warm", type=int, default=6)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--analyze", default=None, help="a directory of rocprofv3 --pmc passes")
    a = ap.parse_args()
    if a.analyze:
        analyze(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
