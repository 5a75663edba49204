"""Does physically contiguous device memory remove the placement spread?

SETS (input lines, output lines) pairs per allocation kind, each timed with
STEPS launches (HIP events); metadata and verdicts fixed. Kinds: hipMalloc,
hipExtMallocWithFlags(hipDeviceMallocContiguous), and torch's allocator.

    python tools/contig_probe.py [--sets 6] [--steps 40]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

HIP_D2D = 3
CONTIGUOUS = 0x4  # hipDeviceMallocContiguous


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=1 << 24)
    a = ap.parse_args()
    import torch
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = a.batch
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    src = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    L = n * 64
    keep = []

    def alloc(kind):
        if kind == "torch":
            t = torch.empty(L, dtype=torch.uint8, device=dev)
            keep.append(t)
            return t.data_ptr()
        p = ctypes.c_void_p()
        if kind == "hipMalloc":
            r = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(L))
        else:
            r = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(L), ctypes.c_uint(CONTIGUOUS))
        assert r == 0, (kind, r)
        return p.value

    def time_pair(d_in, d_out):
        for _ in range(3):
            q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
        for _ in range(a.steps):
            q.submit(d_in, d_out, d_meta, d_v, n, in_stride=abi.LINE, out_stride=abi.LINE)
        torch.cuda.synchronize()
        ms, cnt = q.kernel_ms(a.steps)
        return ms / cnt

    out = {}
    for kind in ["hipMalloc", "contiguous", "torch", "hipMalloc", "contiguous"]:
        ts = []
        for s in range(a.sets):
            d_in, d_out = alloc(kind), alloc(kind)
            assert hip.hipMemcpy(ctypes.c_void_p(d_in), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(L), HIP_D2D) == 0
            ts.append(round(time_pair(d_in, d_out), 4))
            print(json.dumps({"kind": kind, "set": s, "kernel_ms": ts[-1], "in": hex(d_in), "out": hex(d_out)}),
                  flush=True)
        out.setdefault(kind, []).extend(ts)
    print(json.dumps({"summary": True, **{k: {"min": min(v), "max": max(v), "mean": round(sum(v) / len(v), 4)}
                                          for k, v in out.items()}}))


if __name__ == "__main__":
    main()
