"""Per-workgroup start / end times of one ring launch (measurement build
with -DRING_TRACE: copy it over grout_amd/libgrout_hip.so first), on a
placed headline batch: how long the grid's tail is, and per XCD.

    python tools/ring_trace.py
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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
    fn = L.gr_fwd4_ring_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:  # settle: the GPU's steady state
        for _ in range(8):
            q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
        q.sync()
    out = []
    for rep in range(5):
        q.submit(b.in_frames, b.out_lines, b.meta, b.verdicts, n)
        q.sync()
        ms, _ = q.kernel_ms(1)
        tr = np.zeros(2 * 4096, dtype=np.uint64)
        assert fn(tr.ctypes.data, len(tr)) == 0
        g = 256
        st, en = tr[0:2 * g:2].astype(np.int64), tr[1:2 * g:2].astype(np.int64)
        t0 = st.min()
        st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0  # s_memrealtime: 100 MHz
        xcd = np.arange(g) % 8
        out.append({"rep": rep, "kernel_ms": round(ms, 4), "start_spread_us": round(float(st_us.max()), 2),
                    "end_min_us": round(float(en_us.min()), 2), "end_median_us": round(float(np.median(en_us)), 2),
                    "end_max_us": round(float(en_us.max()), 2),
                    "tail_us": round(float(en_us.max() - np.median(en_us)), 2),
                    "end_mean_by_xcd_us": [round(float(en_us[xcd == x].mean()), 1) for x in range(8)]})
        print(json.dumps(out[-1]), flush=True)
    fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
