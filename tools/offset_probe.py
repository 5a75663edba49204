#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Is the slow buffer-pairing class a property of the pages
or of where the two streams sit relative to each other? The headline kernel
(config 3, 2^24 x 64 B) over the input lines and an output pointer shifted by
k x --step inside ONE over-sized allocation: the shifted buffers use almost
the same physical pages, at other offsets from the input stream. If the time
follows k, the effect is relative placement (TLB sets, channel phase) and a
chosen offset makes placement deterministic; if it stays with the allocation,
it is the pages'. Then the same with the input shifted against a fixed output.
Several allocations (--allocs) so that fast and slow ones are both seen.

    python3 tools/offset_probe.py [--allocs 4] [--shifts 0,1,2,3,...] [--step 2097152]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--shifts", default="0,1,2,3,4,5,6,7,8,12,16,24,31")
    ap.add_argument("--step", type=int, default=2 << 20, help="bytes per shift unit")
    ap.add_argument("--warm", type=int, default=10)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1 << 24)
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
    n = a.batch
    shifts = [int(x) for x in a.shifts.split(",")]
    span = n * abi.LINE + max(shifts) * a.step
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    t_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    q = fp.queue(shared_stream(dev))

    def timed(d_in, d_out):
        for _ in range(a.warm):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        q.kernel_ms(10 ** 6)
        for _ in range(a.steps):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        ms, cnt = q.kernel_ms(a.steps)
        return round(ms / max(cnt, 1), 4)

    bigs = [torch.empty(span, dtype=torch.uint8, device=dev) for _ in range(a.allocs)]
    ins = [torch.empty(span, dtype=torch.uint8, device=dev) for _ in range(a.allocs)]
    for i, big in enumerate(bigs):  # the output shifted against the input
        res = [timed(t_in.data_ptr(), big.data_ptr() + s * a.step) for s in shifts]
        print(json.dumps({"shifted": "out", "alloc": i, "base": hex(big.data_ptr()), "in": hex(t_in.data_ptr()),
                          "step": a.step, "shifts": shifts, "kernel_ms": res,
                          "spread": round(max(res) / min(res), 3)}), flush=True)
    out = bigs[0].data_ptr()
    for i, bi in enumerate(ins):  # the input shifted against the first output allocation
        res = []
        for s in shifts:
            p = bi.data_ptr() + s * a.step
            bi[s * a.step: s * a.step + n * abi.LINE].copy_(t_in)
            res.append(timed(p, out))
        print(json.dumps({"shifted": "in", "alloc": i, "base": hex(bi.data_ptr()), "out": hex(out),
                          "step": a.step, "shifts": shifts, "kernel_ms": res,
                          "spread": round(max(res) / min(res), 3)}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
