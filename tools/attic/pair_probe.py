"""Kernel time for every pairing of SETS input-line buffers with SETS
output-line buffers (separate allocations; metadata and verdicts fixed):
is the placement effect a property of one buffer or of the pair?

    python tools/pair_probe.py [--sets 8] [--steps 20]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--orders", default="0", help="tile_order values, one matrix each")
    ap.add_argument("--proxy", type=int, default=0, help="also time each pair on an empty context")
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
    n = a.batch
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    ins, outs = [], []
    for _ in range(a.sets):
        ins.append(torch.from_numpy(frames.reshape(-1)).to(dev))
        outs.append(torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev))
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    if a.proxy:
        fpe = FastPath(0)  # nothing loaded: every packet ends at iface_input
        qe = fpe.queue(shared_stream(dev))
    for order in [int(x) for x in a.orders.split(",")]:
        assert fp.tune("tile_order", order) == 0
        m = np.zeros((a.sets, a.sets))
        pm = np.zeros((a.sets, a.sets))
        for i in range(a.sets):
            for o in range(a.sets):
                if a.proxy:
                    for _ in range(8):
                        qe.submit(ins[i], outs[o], d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
                    torch.cuda.synchronize()
                    ms, cnt = qe.kernel_ms(5)
                    pm[i, o] = ms / cnt
                for _ in range(3 + a.steps):
                    q.submit(ins[i], outs[o], d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
                torch.cuda.synchronize()
                ms, cnt = q.kernel_ms(a.steps)
                m[i, o] = ms / cnt
            print(json.dumps({"order": order, "in": i, "ms_by_out": [round(x, 4) for x in m[i]],
                              **({"proxy_ms_by_out": [round(x, 4) for x in pm[i]]} if a.proxy else {})}), flush=True)
        if a.proxy:
            pick = pm.argmin(axis=1)
            print(json.dumps({"proxy_corr": round(float(np.corrcoef(m.ravel(), pm.ravel())[0, 1]), 3),
                              "picked_ms": [round(m[i, pick[i]], 4) for i in range(a.sets)],
                              "best_ms": [round(x, 4) for x in m.min(axis=1)],
                              "row_mean_ms": [round(x, 4) for x in m.mean(axis=1)]}), flush=True)
        # additive model: m[i,o] ~ mu + r_i + c_o; the residual is the pair interaction
        mu = m.mean()
        r = m.mean(axis=1) - mu
        c = m.mean(axis=0) - mu
        resid = m - (mu + r[:, None] + c[None, :])
        print(json.dumps({"summary": True, "order": order, "mean": round(mu, 4), "in_effect": [round(x, 4) for x in r],
                          "out_effect": [round(x, 4) for x in c],
                          "resid_rms": round(float(np.sqrt((resid ** 2).mean())), 4),
                          "min": round(m.min(), 4), "max": round(m.max(), 4)}), flush=True)
    fp.close()


if __name__ == "__main__":
    main()
