"""Do consecutive launches overlap usefully when alternate batches go to two
queues (two streams)? Wall ms per step over STEPS steps, one queue + one
batch against two queues + two batches, events off, interleaved rounds.

    python tools/overlap_probe.py [--steps 200] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = 1 << 24
    frames, meta = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array())
    L = fp.lib
    bs = []
    for _ in range(2):
        b = fp.batch_alloc(n)
        for dst, src in ((b.in_frames, frames), (b.meta, meta)):
            abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
        fp.batch_place(b, 6)
        bs.append(b)
    qs = [fp.queue(), fp.queue()]
    fp.tune("untimed", 1)
    res = {1: [], 2: []}
    for r in range(a.rounds):
        for nq in (1, 2):
            for k in range(10):
                qs[k % nq].submit(bs[k % nq].in_frames, bs[k % nq].out_lines, bs[k % nq].meta, bs[k % nq].verdicts, n)
            for q in qs:
                q.sync()
            t0 = time.perf_counter()
            for k in range(a.steps):
                b = bs[k % nq]
                qs[k % nq].submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
            for q in qs:
                q.sync()
            res[nq].append((time.perf_counter() - t0) / a.steps * 1e3)
    fp.tune("untimed", 0)
    print(json.dumps({"steps": a.steps, "ms_per_step_1q": [round(x, 4) for x in res[1]],
                      "ms_per_step_2q": [round(x, 4) for x in res[2]]}))
    for b in bs:
        fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
