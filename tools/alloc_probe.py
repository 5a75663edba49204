#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Does the allocation kind remove the buffer-pairing spread (DESIGN.md §6,
"placement")? Slow pairings stall on address translation (tools/place_pmc.py:
TCP_UTCL1_STALL_INFLIGHT_MAX and TA_ADDR_STALLED_BY_TC grow with the kernel
time, DRAM requests and credit stalls do not), so an allocation the driver
maps with large fragments should translate fast whatever its pages.

The headline kernel (config 3, 2^24 x 64 B) over the input lines and each of
--cands output buffers of one kind, --steps timed launches each after --warm:
kinds torch (the bench's plain leg), hipMalloc, hipExtMallocWithFlags
(hipDeviceMallocContiguous); and the input itself of that kind too ("+in").
One JSON line per kind: every candidate's kernel ms, min / median / max.

    python3 tools/alloc_probe.py [--cands 8] [--kinds torch,malloc,contig,contig+in] [--orders 0,1,2]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4  # hip_runtime_api.h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", type=int, default=8)
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--kinds", default="torch,malloc,contig,contig+in")
    ap.add_argument("--fib-contig", default="1", help="FIB tables contiguous (the \"alloc_contig\" knob at load), "
                    "e.g. 0,1: one context each, interleaved")
    ap.add_argument("--rounds", type=int, default=1, help="passes over every (fib, kind)")
    ap.add_argument("--orders", default="0", help="tile orders (the \"tile_order\" knob), e.g. 0,1,2,3:16 (order 3 with "
                    "runs of 16 tiles): every candidate "
                    "timed under each")
    a = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    dev = torch.device("cuda", 0)
    topo = T.config_fullview()
    fps = {}
    for fc in [int(x) for x in a.fib_contig.split(",")]:
        fps[fc] = FastPath(0)
        fps[fc].tune("alloc_contig", fc)
        fps[fc].load(topo)
    n = a.batch
    frames, meta = S.stream(n, 0x67721000, routes=topo.route_array())
    t_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    stream = shared_stream(dev)
    qs = {fc: f.queue(stream) for fc, f in fps.items()}

    def alloc(kind, size):
        if kind == "torch":
            t = torch.empty(size, dtype=torch.uint8, device=dev)
            return t.data_ptr(), t
        p = ctypes.c_void_p()
        r = hip.hipMalloc(ctypes.byref(p), size) if kind == "malloc" else \
            hip.hipExtMallocWithFlags(ctypes.byref(p), size, HIP_DEVICE_MALLOC_CONTIGUOUS)
        if r != 0:
            raise MemoryError(f"{kind}: hip error {r}")
        return p.value, p

    orders = a.orders.split(",")  # "3:16" = tile order 3, runs of 16 tiles

    def timed(q, fp, d_in, d_out):
        res = []
        for o in orders:
            order, _, run = o.partition(":")
            fp.tune("tile_order", int(order))
            fp.tune("tile_run", int(run or 16))
            res.append(timed1(q, d_in, d_out))
        return res

    def timed1(q, d_in, d_out):
        for _ in range(a.warm):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        for _ in range(a.steps):
            q.submit(d_in, d_out, d_meta, d_v, n)
        q.sync()
        ms, cnt = q.kernel_ms(a.steps)
        return ms / max(cnt, 1)

    for _, fc, kind in [(r, fc, k) for r in range(a.rounds) for fc in fps for k in a.kinds.split(",")]:
        q = qs[fc]
        base, _, in_too = kind.partition("+")
        keep = []
        d_in = t_in.data_ptr()
        if in_too:
            d_in, h = alloc(base, n * abi.LINE)
            keep.append(h)
            assert hip.hipMemcpy(d_in, t_in.data_ptr(), n * abi.LINE, 3) == 0  # device to device
        res = []
        for _ in range(a.cands):
            d_out, h = alloc(base, n * abi.LINE)
            keep.append(h)
            res.append(timed(q, fps[fc], d_in, d_out))
        for i, o in enumerate(orders):
            r = [round(x[i], 4) for x in res]
            print(json.dumps({"fib_contig": fc, "kind": kind, "tile_order": o, "kernel_ms": r, "min": min(r),
                              "median": float(np.median(r)), "max": max(r), "spread": round(max(r) / min(r), 3)}), flush=True)
        for h in keep:
            if isinstance(h, ctypes.c_void_p):
                hip.hipFree(h)
        del keep
        torch.cuda.synchronize()
    for fc in fps:
        qs[fc].close()
        fps[fc].close()


if __name__ == "__main__":
    main()
