# SPDX-License-Identifier: BSD-3-Clause
"""Does the headline kernel's time depend on how long the GPU has been busy?
The headline workload (config 3, 2^24 packets) on two buffer sets, the
calibrated one (gr_hip_batch_place, as bench.py) and plain torch allocations,
in alternating blocks of --block launches for --seconds after an idle pause;
per block: time since the first launch, mean kernel ms (HIP events on the
queue's stream). A time trend common to both sets is the clock / power
state; a constant gap between them is placement.

    python tools/clock_probe.py > out.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--block", type=int, default=20)
    ap.add_argument("--idle", type=float, default=2.0)
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
    b = fp.batch_alloc(n, abi.LINE)
    cf, cm = S.stream(n, S.SEED_GPU_BASE ^ 0xCA11B, routes=topo.route_array())
    for dst, src in ((b.in_frames, cf), (b.meta, cm)):
        src = np.ascontiguousarray(src)
        abi.check("h2d", fp.lib.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
    fp.batch_place(b, 6)
    for dst, src in ((b.in_frames, fr), (b.meta, me)):
        src = np.ascontiguousarray(src)
        abi.check("h2d", fp.lib.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
    sets = {
        "calibrated": (b.in_frames, b.out_lines, b.meta, b.verdicts),
        "plain": (torch.from_numpy(fr.reshape(-1)).to(dev), torch.empty(n * 64, dtype=torch.uint8, device=dev),
                  torch.from_numpy(me.view(np.uint8)).to(dev), torch.empty(n * 8, dtype=torch.uint8, device=dev)),
    }
    q = fp.queue(shared_stream(dev))
    fp.tune("untimed", 1)
    torch.cuda.synchronize()
    time.sleep(args.idle)
    t_start = time.perf_counter()
    k = 0
    while time.perf_counter() - t_start < args.seconds:
        name = ("calibrated", "plain")[k % 2]
        d_in, d_out, d_meta, d_v = sets[name]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter() - t_start
        e0.record()
        for _ in range(args.block):
            q.submit(d_in, d_out, d_meta, d_v, n)
        e1.record()
        e1.synchronize()
        print(json.dumps({"block": k, "set": name, "t_s": round(t0, 3),
                          "ms_per_launch": round(e0.elapsed_time(e1) / args.block, 4)}), flush=True)
        k += 1
    q.sync()
    fp.tune("untimed", 0)
    fp.batch_free(b)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
