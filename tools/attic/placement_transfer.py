# SPDX-License-Identifier: BSD-3-Clause
"""Does a placement found on one batch hold for another batch of the same
workload? gr_hip_batch_place times candidate output-line allocations over
the batch in place; bench.py calibrates on a stream drawn with
another seed than the one it measures. This probe, in one process:

  for each calibration stream X in (A, B): place on X, then time the placed
  buffers on A and on B (the input loaded into the same frames buffer);
  and plain torch allocations on A and B.

Kernel ms per 2^24-packet launch, median of --reps timed launches.

    python tools/placement_transfer.py [--workload fullview64] [--reps 8] > out.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--candidates", type=int, default=6)
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
    streams = {k: S.stream(n, s, routes=topo.route_array()) for k, s in (("A", S.SEED_GPU_BASE),
                                                                           ("B", S.SEED_GPU_BASE ^ 0xCA11B))}
    q = fp.queue(shared_stream(dev))
    L = fp.lib

    def h2d(dst, src):
        src = np.ascontiguousarray(src)
        abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))

    def time_on(bufs):
        d_in, d_out, d_meta, d_v = bufs
        for _ in range(2):
            q.submit(d_in, d_out, d_meta, d_v, n)
        ms = []
        for _ in range(args.reps):
            q.submit(d_in, d_out, d_meta, d_v, n)
            q.sync()
            ms.append(q.kernel_ms(1)[0])
        return float(np.median(ms))

    for rnd in range(args.rounds):
        for cal in ("A", "B"):
            b = fp.batch_alloc(n)
            h2d(b.in_frames, streams[cal][0])
            h2d(b.meta, streams[cal][1])
            fp.batch_place(b, args.candidates)
            for meas in ("A", "B"):
                h2d(b.in_frames, streams[meas][0])
                h2d(b.meta, streams[meas][1])
                ms = time_on((b.in_frames, b.out_lines, b.meta, b.verdicts))
                print(json.dumps({"round": rnd, "placed_on": cal, "measured_on": meas, "kernel_ms": round(ms, 4)}),
                      flush=True)
            fp.batch_free(b)
        for meas in ("A", "B"):
            fr, me = streams[meas]
            bufs = (torch.from_numpy(fr.reshape(-1)).to(dev), torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev),
                    torch.from_numpy(me.view(np.uint8)).to(dev), torch.empty(n * 8, dtype=torch.uint8, device=dev))
            ms = time_on(bufs)
            print(json.dumps({"round": rnd, "placed_on": "plain", "measured_on": meas, "kernel_ms": round(ms, 4)}),
                  flush=True)
            del bufs
            torch.cuda.synchronize()
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
