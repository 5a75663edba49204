# SPDX-License-Identifier: BSD-3-Clause
"""Forwarding rate of the grout node itself (gpu_fwd4_node.c) inside a whole
rte_graph walk, driven from C: the walk harness's port_rx stand-in feeds
full 64-packet bursts of the full-view stream, the node accumulates them into
batches of --batch packets, the GPU forwards them and the node hands every
mbuf to the recorder node of its edge (walk_harness.c). One worker thread,
one graph; depth 1 (each batch waited for) against depth 2 (pipelined,
the default), alternating, --reps times each. Mpps = mbufs / wall time of
gh_run (one C call: no Python in the loop). The hold time (--max-delay-us)
is long enough that --batch sets the flush (full RX bursts never flush
early): each line reports the batches the node started and the largest.
Compare with bench.py's cpu_baseline.single_core_mpps run on the same box
(the oracle is test infrastructure: only bench.py's baseline leg runs it).

    python tools/node_graph_rate.py --batch 16384 > out.jsonl
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--mbufs", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--pin", type=int, default=0, help="1: frames by address (node_ptrs)")
    ap.add_argument("--depths", default="1,2")
    ap.add_argument("--rx-touch", default="0", help="harness port_rx leaves mbuf and frame cached (PMD + DDIO): 0,1")
    ap.add_argument("--max-delay-us", type=float, default=20_000.0, help="the node's hold time")
    args = ap.parse_args()

    import test_graph_walk as G  # the harness bindings and the fan-out control plane
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T

    L = G.lib()
    L.gpu_fwd4_prof.argtypes = [ctypes.c_int, ctypes.c_void_p]
    L.gpu_fwd4_prof.restype = None
    devs = (ctypes.c_int * 1)(0)
    r = L.gh_init(ctypes.cast(devs, ctypes.c_void_p), 1, 1024, 1 << 17, args.batch, 64, int(args.max_delay_us * 1e3))
    assert r == 0, r
    assert L.gh_graph_create(0, 0) == 0
    G._gh["fp"] = fp = G.FanOutPath(L)
    topo = T.config_fullview()
    G.load(fp, topo)
    fp.tune("node_ptrs", args.pin)
    L.gh_set_pin(args.pin)
    fr, me = S.stream(args.mbufs, S.SEED_GPU_BASE, routes=topo.route_array())
    fr = np.ascontiguousarray(fr)
    me = np.ascontiguousarray(me)
    L.gh_set_rx_touch.argtypes = [ctypes.c_int]
    variants = [(int(d), int(t)) for d in args.depths.split(",") for t in args.rx_touch.split(",")]
    for rep in range(args.reps + 1):
        for depth, touch in variants:
            assert L.gpu_fwd4_set_depth(depth) == 0
            L.gh_set_rx_touch(touch)
            # the walk as it runs in production: no phase clocks
            assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, len(me)) == 0
            t0 = time.perf_counter()
            assert L.gh_run(1 << 24) > 0
            dt_plain = time.perf_counter() - t0
            # the same with the node's and the library's phase clocks
            fp.tune("node_prof", 1)
            assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, len(me)) == 0
            L.gpu_fwd4_prof(1, None)
            H = abi.hip()
            H.gr_hip_node_prof(None, 0, 1)
            wi0 = G.walk_info()
            t0 = time.perf_counter()
            walks = L.gh_run(1 << 24)
            dt = time.perf_counter() - t0
            wi = G.walk_info()
            ph = np.zeros(6, dtype=np.uint64)  # GPU_FWD4_PROF_COUNT
            L.gpu_fwd4_prof(0, ph.ctypes.data)
            lp = np.zeros(9, dtype=np.uint64)
            H.gr_hip_node_prof(lp.ctypes.data, 9, 1)
            fp.tune("node_prof", 0)
            assert walks > 0, walks
            if rep == 0:
                continue  # warm-up: staging buffers grown, pages touched
            # ns per packet in each phase of the node, clocks on (depth 2: start and finish
            # are the library's halves; depth 1 runs gr_hip_node_process, not split)
            names = ["accumulate", "start", "finish", "deliver", "poll", "flush_node"]
            per = {k: round(float(v) / len(me), 2) for k, v in zip(names, ph)}
            # poll and flush_node overlap the four phases (the flush node's hand-backs and flushes)
            per["rest_of_walk"] = round(dt * 1e9 / len(me) - sum(per[k] for k in names[:4]), 2)
            print(json.dumps({"batch": args.batch, "max_delay_us": args.max_delay_us, "depth": depth, "rx_touch": touch,
                              "mbufs": len(me), "graph_walks": walks,
                              "node_batches": int(wi["batches"] - wi0["batches"]), "max_batch": int(wi["max_batch"]),
                              "ms": round(dt * 1e3, 2), "mpps": round(len(me) / dt / 1e6, 1),
                              "mpps_unprofiled": round(len(me) / dt_plain / 1e6, 1),
                              "ns_per_pkt_unprofiled": round(dt_plain * 1e9 / len(me), 2),
                              "ns_per_pkt": per,
                              "start_ns_per_pkt": {k: round(float(v) / len(me), 2) for k, v in zip(
                                  ["layout", "prep", "lock", "stage", "launch", "record", "fin_wait", "fin_scan",
                                   "fin_apply"], lp)},
                              "mode": "frames by address" if args.pin else "staged lines"}), flush=True)



if __name__ == "__main__":
    main()
