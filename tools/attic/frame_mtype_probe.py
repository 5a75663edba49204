# SPDX-License-Identifier: BSD-3-Clause
"""Config 4's whole frames (one 64-byte head per 2240-byte mbuf-like slot):
does the memory type of the frame buffer change what a head read costs?
On the default (coarse-grained, cached) allocation the L2 fetches a whole
128-byte line per head (profiles/r02_pmc_imix_frames.json). The same batch
with its frames in hipExtMallocWithFlags(flag) memory -- 0 default,
1 fine-grained, 3 uncached -- timed in alternation in one process (HIP
events around each launch on the queue's stream).

    python tools/frame_mtype_probe.py [--flags 0,1,3] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hip_lib():
    for line in open("/proc/self/maps"):
        p = line.split()[-1]
        if "libamdhip64.so" in p:
            return ctypes.CDLL(p)
    raise RuntimeError("no HIP runtime loaded")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0,1,3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--slot", type=int, default=2240)
    a = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda")
    topo = T.config_fullview()
    fp = FastPath()
    fp.load(topo)
    H = hip_lib()
    H.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    H.hipFree.argtypes = [ctypes.c_void_p]
    n = a.batch
    frames, meta = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array(), imix=True, stride=a.slot)
    frames = np.ascontiguousarray(frames)
    bufs = {}
    for fl in [int(x) for x in a.flags.split(",")]:
        p = ctypes.c_void_p()
        assert H.hipExtMallocWithFlags(ctypes.byref(p), frames.nbytes, fl) == 0, fl
        abi.check("gr_hip_memcpy_h2d", fp.lib.gr_hip_memcpy_h2d(fp.h, p.value, frames.ctypes.data, frames.nbytes))
        bufs[fl] = p.value
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_out = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    res = {fl: [] for fl in bufs}
    for fl in bufs:  # warm-up and a bit-exact check between memory types
        for _ in range(20):
            q.submit(bufs[fl], d_out, d_meta, d_v, n, in_stride=a.slot)
        q.sync()
    ref = None
    for r in range(a.rounds):
        for fl, p in bufs.items():
            for _ in range(a.reps):
                q.submit(p, d_out, d_meta, d_v, n, in_stride=a.slot)
            q.sync()
            tot, cnt = q.kernel_ms(a.reps)
            assert cnt == a.reps, cnt
            ms = tot / cnt
            v = d_v.cpu().numpy()
            if ref is None:
                ref = v.copy()
            assert np.array_equal(v, ref), fl
            res[fl].append(ms)
            print(json.dumps({"round": r, "flag": fl, "kernel_ms": round(ms, 4),
                              "mpps": round(n / ms / 1e3, 1)}), flush=True)
    print(json.dumps({"summary": {str(fl): round(float(np.median(v)), 4) for fl, v in res.items()},
                      "batch": n, "slot": a.slot,
                      "flags": "0 = hipDeviceMallocDefault, 1 = Finegrained, 3 = Uncached"}), flush=True)
    q.close()
    for p in bufs.values():
        H.hipFree(p)


if __name__ == "__main__":
    main()
