# SPDX-License-Identifier: BSD-3-Clause
"""Cost of the node's staging copy (gr_hip_node_stage: 64-byte header line +
8-byte metadata per mbuf) by destination: pageable host memory against the
pinned, device-mapped memory the node stages into (gr_hip_host_alloc, the
queue's walk slots), on warm frames (a pass before each timing) and on frames
spread over a large region (cold). Median ns per packet.

    python tools/stage_probe.py > out.jsonl
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=21)
    args = ap.parse_args()

    from grout_amd import abi
    from grout_amd.fwd import FastPath

    fp = FastPath(0)
    L = fp.lib
    n = args.n
    room = 2304
    frames = np.zeros(n * room, dtype=np.uint8)
    frames.reshape(n, room)[:, :64] = 0x45
    m = np.zeros(n, dtype=abi.MBUF_DT)
    m["frame"] = frames.ctypes.data + np.arange(n, dtype=np.uint64) * room
    m["pkt_len"] = 60
    m["data_len"] = 60
    m["iface"] = 2
    meta_pg = np.zeros(n, dtype=abi.META_DT)
    lines_pg = np.zeros((n, 64), dtype=np.uint8)
    p_lines, p_meta = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check("gr_hip_host_alloc", L.gr_hip_host_alloc(fp.h, n * 64, ctypes.byref(p_lines)))
    abi.check("gr_hip_host_alloc", L.gr_hip_host_alloc(fp.h, n * 8, ctypes.byref(p_meta)))
    dests = {"pageable": (lines_pg.ctypes.data, meta_pg.ctypes.data), "pinned": (p_lines.value, p_meta.value)}
    for warm in (True, False):
        for name, (dl, dm) in dests.items():
            t = []
            for _ in range(args.reps):
                if warm:
                    L.gr_hip_node_stage(m.ctypes.data, n, 64, None, dl, dm)
                else:
                    junk = np.ones(1 << 25, dtype=np.uint64)  # 256 MB: evict the frames
                    junk.sum()
                    del junk
                t0 = time.perf_counter()
                abi.check("gr_hip_node_stage", L.gr_hip_node_stage(m.ctypes.data, n, 64, None, dl, dm))
                t.append(time.perf_counter() - t0)
            print(json.dumps({"dest": name, "frames": "warm" if warm else "cold", "pkts": n,
                              "ns_per_pkt": round(float(np.median(t)) / n * 1e9, 2)}), flush=True)
    L.gr_hip_host_free(fp.h, p_lines)
    L.gr_hip_host_free(fp.h, p_meta)
    fp.close()


if __name__ == "__main__":
    main()
