"""Wall time per step of back-to-back launches on one placed headline batch,
with and without the library's HIP events around each launch ("untimed"),
interleaved rounds: what the per-launch events cost the bench's clock.

    python tools/event_cost.py [--steps 200] [--rounds 4]
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
    ap.add_argument("--rounds", type=int, default=4)
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
    b = fp.batch_alloc(n)
    for dst, src in ((b.in_frames, frames), (b.meta, meta)):
        abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
    fp.batch_place(b, 6)
    q = fp.queue()
    res = {0: [], 1: []}
    for r in range(a.rounds):
        for untimed in (0, 1):
            fp.tune("untimed", untimed)
            for _ in range(10):
                q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
            q.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
            q.sync()
            res[untimed].append((time.perf_counter() - t0) / a.steps * 1e3)
    fp.tune("untimed", 0)
    print(json.dumps({"steps": a.steps, "ms_per_step_timed": [round(x, 4) for x in res[0]],
                      "ms_per_step_untimed": [round(x, 4) for x in res[1]]}))
    fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
