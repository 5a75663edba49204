"""Kernel time against the relative placement of the batch's buffers.

One device pool; the input lines at offset 0, the output lines at
n*64 + DELTA, then metadata and verdicts. Each DELTA is timed in PASSES
round-robin passes (STEPS launches each, HIP events), so a placement
effect shows as a per-DELTA pattern that repeats across passes.

    python tools/offset_probe.py [--passes 2] [--steps 30] [--what out|meta|v]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

DELTAS_KB = [0, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--what", default="out", choices=["out", "meta", "v"])
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
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    L, M, V = n * 64, n * 8, n * 8
    slack = max(DELTAS_KB) * 1024 + (1 << 21)
    pool = torch.empty(L * 2 + M + V + slack * 3, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    base = pool.data_ptr()
    print(json.dumps({"pool_addr": hex(base), "pool_mod_2m": base % (1 << 21)}), flush=True)

    def views(d):
        off_out = L + (d if a.what == "out" else 0)
        off_meta = off_out + L + (d if a.what == "meta" else 0)
        off_v = off_meta + M + (d if a.what == "v" else 0)
        return (pool[0:L], pool[off_out:off_out + L], pool[off_meta:off_meta + M], pool[off_v:off_v + V])

    host_in = torch.from_numpy(frames.reshape(-1))
    host_meta = torch.from_numpy(meta.view(np.uint8))
    res = np.zeros((a.passes, len(DELTAS_KB)))
    for p in range(a.passes):
        for k, dkb in enumerate(DELTAS_KB):
            d_in, d_out, d_meta, d_v = views(dkb * 1024)
            d_in.copy_(host_in)
            d_meta.copy_(host_meta)
            for _ in range(3):
                q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
            for _ in range(a.steps):
                q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
            torch.cuda.synchronize()
            ms, cnt = q.kernel_ms(a.steps)
            res[p, k] = ms / max(cnt, 1)
            print(json.dumps({"pass": p, "what": a.what, "delta_kb": dkb, "kernel_ms": round(res[p, k], 4)}),
                  flush=True)
    print(json.dumps({"summary": True, "what": a.what, "deltas_kb": DELTAS_KB,
                      "mean_ms": [round(x, 4) for x in res.mean(axis=0)],
                      "pass_spread": round(float(np.abs(res[0] - res[-1]).max()), 4)}))
    fp.close()


if __name__ == "__main__":
    main()
