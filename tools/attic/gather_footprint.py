"""FIB gather cost against the tbl24 footprint, on one placed batch: the
full-view FIB, destinations drawn uniformly from a window of W tbl24
entries (W x 2 bytes of table), re-filled into the same buffers per W so the
in/out placement is constant. Interleaved rounds; kernel ms by HIP events.

    python tools/gather_footprint.py [--rounds 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = 1 << 24
    L = fp.lib
    base = 1 << 16  # tbl24 index of 1.0.0.0
    windows = [1, 64, 4096, 1 << 16, 1 << 18, 1 << 20, 1 << 21, 3 << 20]
    streams = {}
    for w in windows:
        lo = base << 8
        streams[w] = S.stream(n, S.SEED_GPU_BASE, dst_range=(lo, lo + (w << 8) - 1))
    streams["fullview"] = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array())
    b = fp.batch_alloc(n)

    def fill(k):
        fr, me = streams[k]
        for dst, src in ((b.in_frames, fr), (b.meta, me)):
            abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))

    fill("fullview")
    fp.batch_place(b, 6)
    q = fp.queue()
    vh = np.empty(n, dtype=abi.VERDICT_DT)
    res = {k: [] for k in streams}
    fwd = {}
    for r in range(a.rounds):
        for k in streams:
            fill(k)
            for _ in range(2 + a.reps):
                q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
            q.sync()
            ms, cnt = q.kernel_ms(a.reps)
            res[k].append(ms / cnt)
            if r == 0:
                abi.check("d2h", L.gr_hip_memcpy_d2h(fp.h, vh.ctypes.data, b.verdicts, vh.nbytes))
                fwd[k] = float((vh["edge"] == abi.EDGE["port_output"]).mean())
    for k in streams:
        t = np.array(res[k])
        print(json.dumps({"window_tbl24": k, "table_bytes": (k * 2 if k != "fullview" else 7 << 20),
                          "median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                          "forwarded": round(fwd[k], 4)}), flush=True)
    fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
