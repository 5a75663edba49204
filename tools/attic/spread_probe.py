"""Output-line candidates for one input buffer, allocated back to back or
with a spacer allocation between them: how far apart must candidates be
for some of them to avoid the in/out placement conflict?

    python tools/spread_probe.py [--cands 12] [--spacer-mb 0,1024]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", type=int, default=12)
    ap.add_argument("--spacer-mb", default="0,1024")
    ap.add_argument("--steps", type=int, default=10)
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
    n = 1 << 24
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    for sp in [int(x) for x in a.spacer_mb.split(",")]:
        keep, ts = [], []
        for k in range(a.cands):
            o = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
            keep.append(o)
            if sp:
                keep.append(torch.empty(sp << 20, dtype=torch.uint8, device=dev))
            for _ in range(3 + a.steps):
                q.submit(d_in, o, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
            torch.cuda.synchronize()
            ms, cnt = q.kernel_ms(a.steps)
            ts.append(round(ms / cnt, 4))
        print(json.dumps({"spacer_mb": sp, "ms": ts, "min": min(ts), "max": max(ts)}), flush=True)
        del keep
        torch.cuda.empty_cache()
    fp.close()


if __name__ == "__main__":
    main()
