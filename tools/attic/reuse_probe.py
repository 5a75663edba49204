# SPDX-License-Identifier: BSD-3-Clause
"""Why do tools/variants.py and bench.py time the same kernel differently on
one box (0.447 against 0.468 ms per 2^24 packets)? The two differ in what
happens around the launches. This probe times the headline kernel on plain
torch allocations, in one process, under each launch pattern, interleaved
over --rounds:

  same        one input and one output buffer, launches back to back (bench.py)
  same_sync   the same with a host sync between launches
  copy_first  the input rewritten by a device copy before every launch
  rotate      --inputs input buffers filled once, used in turn, no copies
  variants    tools/variants.py's pattern: copy every input, then one launch
              on each (the first untimed)

Kernel ms per launch from the library's HIP events (median over the timed
launches of a round).

    python tools/reuse_probe.py [--rounds 3] > out.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--inputs", type=int, default=6)
    ap.add_argument("--modes", default="same,same_sync,copy_first,rotate,variants")
    args = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = 1 << 24
    fr, me = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array())
    src = torch.from_numpy(fr.reshape(-1)).to(dev)
    ins = [torch.empty_like(src) for _ in range(args.inputs)]
    for b in ins:
        b.copy_(src)
    out = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
    meta = torch.from_numpy(me.view(np.uint8)).to(dev)
    v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))

    def timed(k):  # the last k launches, per launch
        ms, cnt = q.kernel_ms(k)
        return ms / cnt

    def run(mode):
        if mode == "same":
            for _ in range(2 + args.reps):
                q.submit(ins[0], out, meta, v, n)
            q.sync()
            return timed(args.reps)
        if mode == "same_sync":
            t = []
            for r in range(2 + args.reps):
                q.submit(ins[0], out, meta, v, n)
                q.sync()
                if r >= 2:
                    t.append(timed(1))
            return float(np.median(t))
        if mode == "copy_first":
            t = []
            for r in range(2 + args.reps):
                ins[0].copy_(src)
                q.submit(ins[0], out, meta, v, n)
                q.sync()
                if r >= 2:
                    t.append(timed(1))
            return float(np.median(t))
        if mode == "rotate":
            for r in range(2 + args.reps):
                q.submit(ins[r % len(ins)], out, meta, v, n)
            q.sync()
            return timed(args.reps)
        if mode == "variants":
            for b in ins:
                b.copy_(src)
            for b in ins:
                q.submit(b, out, meta, v, n)
            q.sync()
            return timed(len(ins) - 1)
        raise ValueError(mode)

    modes = args.modes.split(",")
    res = {m: [] for m in modes}
    for rnd in range(args.rounds):
        for m in modes:
            ms = run(m)
            res[m].append(ms)
            print(json.dumps({"round": rnd, "mode": m, "kernel_ms": round(ms, 4)}), flush=True)
    for m in modes:
        print(json.dumps({"mode": m, "median_ms": round(float(np.median(res[m])), 4)}), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
