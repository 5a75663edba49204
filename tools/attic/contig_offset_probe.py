"""Input and output lines inside one physically contiguous allocation
(hipDeviceMallocContiguous), the output at byte distance DELTA from the
input: which distances avoid the in/out placement conflict
(tools/pair_probe.py)? Metadata and verdicts: fixed torch buffers.

    python tools/contig_offset_probe.py [--steps 20] [--passes 2]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

GIB = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--contiguous", type=int, default=1)
    ap.add_argument("--orders", default="0")
    ap.add_argument("--far", type=int, default=0, help="deltas from 1 to 7.5 GiB in 512 MiB steps")
    a = ap.parse_args()
    import torch
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    fp = FastPath(0)
    topo = T.config_fullview()
    fp.load(topo)
    n = 1 << 24
    L = n * 64
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    src = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    pool_bytes = (9 if a.far else 4) * GIB + (64 << 20)
    p = ctypes.c_void_p()
    flags = 0x4 if a.contiguous else 0
    r = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(pool_bytes), ctypes.c_uint(flags))
    assert r == 0, r
    base = p.value
    assert hip.hipMemcpy(ctypes.c_void_p(base), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(L), 3) == 0
    q = fp.queue(shared_stream(dev))
    if a.far:
        deltas = [GIB + k * (GIB // 2) for k in range(14)]
    else:
        deltas = [GIB] + [GIB + (1 << k) for k in range(12, 31)] + [2 * GIB + (1 << 29), 3 * GIB]
    orders = [int(x) for x in a.orders.split(",")]
    res = np.zeros((a.passes * len(orders), len(deltas)))
    for ps in range(a.passes * len(orders)):
        order = orders[ps % len(orders)]
        assert fp.tune("tile_order", order) == 0
        for j, d in enumerate(deltas):
            for _ in range(3 + a.steps):
                q.submit(base, base + d, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
            torch.cuda.synchronize()
            ms, cnt = q.kernel_ms(a.steps)
            res[ps, j] = ms / cnt
            print(json.dumps({"pass": ps, "order": order, "delta": hex(d), "kernel_ms": round(res[ps, j], 4)}),
                  flush=True)
    for oi, order in enumerate(orders):
        rr = res[oi::len(orders)]
        print(json.dumps({"summary": True, "order": order, "contiguous": a.contiguous, "pool": hex(base),
                          "by_delta": {hex(d): round(float(rr[:, j].mean()), 4) for j, d in enumerate(deltas)}}))
    fp.close()


if __name__ == "__main__":
    main()
