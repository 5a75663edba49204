#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""The headline kernel out of place (frames in, lines out) against in place
(the lines rewritten over the frames, as grout rewrites its mbufs), on the
same buffers, alternating, kernel time by HIP events only.

A frame forwarded in place is no longer the frame that arrived (its L2
header names the next hop), so before every launch of either mode the
pristine stream is copied into the work buffer on the queue's stream
(outside the events): both modes run on identical input. Several allocation
sets, since the pages a buffer gets move a launch by up to 15 % (DESIGN.md
§6.2): each set is timed in both modes.

    python3 tools/inplace_probe.py --sets 4 --launches 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 24)
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--launches", type=int, default=20, help="timed launches per mode and set")
    ap.add_argument("--rounds", type=int, default=2, help="A/B alternations per set")
    a = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    fp = FastPath(0)
    topo = T.config_fullview()
    fp.load(topo)
    n = a.n
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    q = fp.queue(shared_stream(dev))
    pristine = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    ref_v = None
    out = []
    for s in range(a.sets):
        work = torch.empty_like(pristine)
        lines = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
        d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)

        def launch(inplace):
            work.copy_(pristine)
            q.submit(work, work if inplace else lines, d_meta, d_v, n)

        fp.tune("untimed", 1)  # settle: the GPU's steady clock
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            launch(False)
            torch.cuda.synchronize()
        fp.tune("untimed", 0)
        res = {"set": s, "out_of_place": [], "in_place": []}
        for _ in range(a.rounds):
            for inplace in (False, True):
                fp.tune("time_every", 1)
                for _ in range(a.launches):
                    launch(inplace)
                torch.cuda.synchronize()
                q.sync()
                ms, cnt = q.kernel_ms(a.launches)
                res["in_place" if inplace else "out_of_place"].append(round(ms / max(cnt, 1), 4))
                v = d_v.cpu().numpy()
                if ref_v is None:
                    ref_v = v.copy()
                assert np.array_equal(v, ref_v), "verdicts differ between modes"
        for k in ("out_of_place", "in_place"):
            res[k + "_ms"] = float(np.median(res[k]))
        res["in_over_out"] = round(res["in_place_ms"] / res["out_of_place_ms"], 4)
        print(json.dumps(res), flush=True)
        out.append(res)
        del work, lines, d_v
        torch.cuda.empty_cache()
    r = [x["in_over_out"] for x in out]
    print(json.dumps({"summary": {"in_over_out_median": float(np.median(r)), "sets": len(r),
                                  "out_ms_median": float(np.median([x["out_of_place_ms"] for x in out])),
                                  "in_ms_median": float(np.median([x["in_place_ms"] for x in out])),
                                  "n": n}}), flush=True)


if __name__ == "__main__":
    main()
