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
VMM (hipMemCreate handles of the whole size or of chunks, mapped into a
reservation aligned to 1 GiB: "vmm", "vmm:<chunk MiB>[:<align MiB>]"; --keep).
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
    ap.add_argument("--keep", action="store_true", help="free nothing until the end (no VA reuse between kinds)")
    ap.add_argument("--check", action="store_true", help="every candidate's output lines and verdicts equal those of "
                    "the torch buffers (themselves parity-tested against the oracle)")
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

    P, Z, U = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_ulonglong
    hip.hipMemAddressReserve.argtypes = [ctypes.POINTER(P), Z, Z, P, U]
    hip.hipMemCreate.argtypes = [ctypes.POINTER(P), Z, P, U]
    hip.hipMemMap.argtypes = [P, Z, Z, P, U]
    hip.hipMemSetAccess.argtypes = [P, Z, P, Z]
    hip.hipMemGetAllocationGranularity.argtypes = [ctypes.POINTER(Z), P, ctypes.c_int]

    class Loc(ctypes.Structure):  # hipMemLocation
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Prop(ctypes.Structure):  # hipMemAllocationProp
        _fields_ = [("type", ctypes.c_int), ("handle_type", ctypes.c_int), ("location", Loc),
                    ("win32", ctypes.c_void_p), ("compression", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte),
                    ("usage", ctypes.c_ushort)]

    class Access(ctypes.Structure):  # hipMemAccessDesc
        _fields_ = [("location", Loc), ("flags", ctypes.c_int)]

    prop = Prop(type=1, handle_type=0, location=Loc(type=1, id=0))  # pinned, no export, device 0
    gran = {}
    for k, f in (("min", 0), ("recommended", 1)):
        g = ctypes.c_size_t()
        gran[k] = g.value if hip.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), f) == 0 else None
    print(json.dumps({"vmm_granularity": gran}), flush=True)

    def vmm(size, chunk, align):
        """VA reserved at `align`, backed by physical handles of `chunk` bytes
        (the whole size when chunk is 0), mapped in order. Never freed here
        (run with --keep)."""
        g = gran["recommended"] or gran["min"] or (2 << 20)
        size = -(-size // g) * g
        chunk = size if chunk == 0 else -(-chunk // g) * g
        va = ctypes.c_void_p()
        if hip.hipMemAddressReserve(ctypes.byref(va), size, align, None, 0) != 0:
            raise MemoryError("hipMemAddressReserve")
        for off in range(0, size, chunk):
            h = ctypes.c_void_p()
            if hip.hipMemCreate(ctypes.byref(h), min(chunk, size - off), ctypes.byref(prop), 0) != 0:
                raise MemoryError("hipMemCreate")
            if hip.hipMemMap(va.value + off, min(chunk, size - off), 0, h, 0) != 0:
                raise MemoryError("hipMemMap")
        acc = Access(location=Loc(type=1, id=0), flags=3)
        if hip.hipMemSetAccess(va, size, ctypes.byref(acc), 1) != 0:
            raise MemoryError("hipMemSetAccess")
        assert hip.hipDeviceSynchronize() == 0
        return va.value, None

    def d2d(dst, src, size):  # hipMemcpy device to device does not block the host
        assert hip.hipMemcpy(dst, src, size, 3) == 0 and hip.hipDeviceSynchronize() == 0

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
        if kind.startswith("vmm"):  # vmm[:chunk MiB[:align MiB]]
            assert a.keep, "vmm kinds need --keep"
            f = kind.split(":")
            return vmm(size, int(f[1]) << 20 if len(f) > 1 else 0, (int(f[2]) if len(f) > 2 else 1024) << 20)
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

    ref = None
    if a.check:  # reference output of plain torch buffers
        q0 = next(iter(qs.values()))
        t_out = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
        q0.submit(t_in.data_ptr(), t_out.data_ptr(), d_meta, d_v, n)
        q0.sync()
        ref = (t_out, d_v.clone())
        scratch = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)

    def same(d_out):
        if ref is None:
            return None
        torch.cuda.synchronize()
        d2d(scratch.data_ptr(), d_out, n * abi.LINE)
        return bool(torch.equal(scratch, ref[0]) and torch.equal(d_v, ref[1]))

    kept = []
    for _, fc, kind in [(r, fc, k) for r in range(a.rounds) for fc in fps for k in a.kinds.split(",")]:
        q = qs[fc]
        base, _, in_too = kind.partition("+")  # "+in": the input of that kind too
        keep = []
        d_in = t_in.data_ptr()
        if in_too:
            d_in, h = alloc(base, n * abi.LINE)
            keep.append(h)
            d2d(d_in, t_in.data_ptr(), n * abi.LINE)
            if ref is not None:  # the copy itself
                d2d(scratch.data_ptr(), d_in, n * abi.LINE)
                assert torch.equal(scratch, t_in), f"{kind}: input copy differs"
        res, ok, addrs = [], [], []
        for _ in range(a.cands):
            d_out, h = alloc(base, n * abi.LINE)
            keep.append(h)
            res.append(timed(q, fps[fc], d_in, d_out))
            ok.append(same(d_out))
            addrs.append(hex(d_out))
        for i, o in enumerate(orders):
            r = [round(x[i], 4) for x in res]
            print(json.dumps({"fib_contig": fc, "kind": kind, "tile_order": o, "kernel_ms": r, "min": min(r),
                              "median": float(np.median(r)), "max": max(r), "spread": round(max(r) / min(r), 3),
                              "in": hex(d_in), "out": addrs, "equal": ok}), flush=True)
        torch.cuda.synchronize()
        if a.keep:
            kept.append(keep)
            continue
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
