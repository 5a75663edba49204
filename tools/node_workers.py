#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Several grout workers on one GPU: the fast path's node (gpu_fwd4_node.c)
in K worker graphs at once, each walked from its own pthread (the walk
harness's gh_workers_run: one graph per worker as grout's worker.c, each
polling its own share of the full-view stream like an RX queue, the
recorders behind the edges only counting). One GPU context, one queue per
graph. Aggregate Mpps = all packets / the wall time of the slowest worker;
compare with bench.py's cpu_baseline on the same box (16 cores).

--recycle P: each worker's packets go through a pool of P mbufs of its own
(a mempool: port_rx refills an mbuf from the stream when the recorder gives
it back), --passes times over its share, instead of one mbuf per packet.
--lcores spread: worker k pinned to bench.cpu_placement's k-th core (one
core per L3 domain in turn), as a deployment places its lcores. The node's
cost is the median over --reps back-to-back pairs of (node run - harness-
alone run): the host's other tenants move both alike.

    python tools/node_workers.py --threads 1,4,8,16 --recycle 65536 --passes 8 --lcores spread
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--per-thread", type=int, default=1 << 18, help="mbufs per worker")
    ap.add_argument("--batch", type=int, default=15360)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rx-touch", type=int, default=1, help="port_rx writes the mbuf and touches the frame (PMD + DDIO)")
    ap.add_argument("--pin", type=int, default=0, help="1: frames by address (node_ptrs, mbuf memory registered)")
    ap.add_argument("--recycle", type=int, default=0,
                    help="mbufs per worker's pool (a mempool: port_rx refills them from the stream); 0: one per packet")
    ap.add_argument("--passes", type=int, default=1, help="with --recycle: times each worker goes over its share")
    ap.add_argument("--ring-cfg", type=int, default=-1, help="the \"ring\" knob (kernel geometry, fwd4_ring.hip ring_cfgN); -1: the default")
    ap.add_argument("--wg-per-cu", type=int, default=-1, help="the \"wg_per_cu\" knob; -1: the default")
    ap.add_argument("--prof", type=int, default=0,
                    help="1: one more node run per line with the node's and the library's phase clocks")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE", help="gr_hip_tune knobs (repeatable)")
    ap.add_argument("--lcores", default="none", choices=["none", "allowed", "spread", "socket"],
                    help="worker placement: the scheduler's, the k-th allowed CPU, or bench.cpu_placement's spread")
    args = ap.parse_args()
    threads = [int(x) for x in args.threads.split(",")]

    import test_graph_walk as G  # the harness bindings and the fan-out control plane
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T

    L = G.lib()
    L.gh_workers_run.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.gh_set_rx_touch.argtypes = [ctypes.c_int]
    L.gpu_fwd4_prof.argtypes = [ctypes.c_int, ctypes.c_void_p]
    L.gpu_fwd4_prof.restype = None
    devs = (ctypes.c_int * 1)(0)
    kmax = max(threads)
    r = L.gh_init(ctypes.cast(devs, ctypes.c_void_p), 1, 1024, 1 << 17, args.batch, 64, 20_000_000)
    assert r == 0, r
    for k in range(kmax):
        assert L.gh_graph_create(k, 0) == k
    fp = G.FanOutPath(L)
    topo = T.config_fullview()
    fp.load(topo)
    n = kmax * args.per_thread
    fr, me = S.stream(n, 0x67720002, routes=topo.route_array())
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    fp.tune("node_ptrs", args.pin)
    if args.ring_cfg >= 0:
        fp.tune("ring", args.ring_cfg)
    if args.wg_per_cu >= 0:
        fp.tune("wg_per_cu", args.wg_per_cu)
    for kv in args.tune:
        k, v = kv.split("=")
        fp.tune(k, int(v))
    L.gh_set_pin(args.pin)  # 0: staged header lines, the node's default
    L.gh_set_rx_touch(args.rx_touch)
    L.gh_set_null_node.argtypes = [ctypes.c_int]
    L.gh_set_recycle.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.gh_set_recycle.restype = None
    L.gh_set_recycle(args.recycle, args.passes)
    from bench import cpu_placement

    def place(k):
        cpus = []
        if args.lcores == "allowed":
            cpus = sorted(os.sched_getaffinity(0))[:k]
        elif args.lcores in ("spread", "socket"):
            cpus = cpu_placement(k, args.lcores) or []
        arr = (ctypes.c_int * max(1, len(cpus)))(*cpus)
        assert L.gh_set_lcores(arr, len(cpus)) == 0
        return cpus
    per = args.passes if args.recycle else 1  # packets through each worker: its share, `passes` times

    def once(k, m, null):
        L.gh_set_null_node(null)
        try:
            assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, m) == 0  # the frames as they came
            s, w = ctypes.c_double(), ctypes.c_uint64()
            rr = L.gh_workers_run(k, ctypes.byref(s), ctypes.byref(w))
            assert rr == 0, rr
            return s.value
        finally:
            L.gh_set_null_node(0)

    def run(k, m):
        """(node, harness alone) wall times, medians over --reps pairs run
        back to back: the host's other tenants move both alike."""
        once(k, m, 0)  # warm-up: pages, queues, pinned slots
        once(k, m, 1)
        pairs = [(once(k, m, 0), once(k, m, 1)) for _ in range(args.reps)]
        return float(np.median([p[0] for p in pairs])), float(np.median([p[1] for p in pairs])), \
            float(np.median([p[0] - p[1] for p in pairs]))

    for k in threads:
        cpus = place(k)
        m = k * args.per_thread
        # t0: the same walks with port_rx handing its bursts straight to
        # port_output: the harness's own cost, which the node's walk pays too
        t, t0, dt = run(k, m)
        prof = None
        if args.prof:  # every worker's clocks add into the same counters
            fp.tune("node_prof", 1)
            L.gpu_fwd4_prof(1, None)
            H = abi.hip()
            H.gr_hip_node_prof(None, 0, 1)
            once(k, m, 0)
            ph = np.zeros(6, dtype=np.uint64)  # GPU_FWD4_PROF_COUNT
            L.gpu_fwd4_prof(0, ph.ctypes.data)
            lp = np.zeros(9, dtype=np.uint64)
            H.gr_hip_node_prof(lp.ctypes.data, 9, 1)
            fp.tune("node_prof", 0)
            pk = m * per  # the clocks add up every worker's time: ns of a worker per packet it takes
            prof = {"node": {a: round(float(v) / pk, 2) for a, v in zip(["accumulate", "start", "finish", "deliver", "poll", "flush_node"], ph)},
                    "library": {a: round(float(v) / pk, 2) for a, v in zip(
                        ["layout", "prep", "lock", "stage", "launch", "record", "fin_wait", "fin_scan", "fin_apply"], lp)}}
        m_loaded, m = m, m * per
        print(json.dumps({"threads": k, "gpus": 1, "packets": m, "batch": args.batch, "rx_touch": args.rx_touch,
                          "harness_alone_mpps": round(m / t0 / 1e6, 1),
                          "node_ns_per_pkt_per_worker": round(dt * 1e9 * k / m, 1), "mode": "frames by address" if args.pin else "staged lines",
                          "recycle": args.recycle, "passes": per, "lcores": args.lcores, "cpus": cpus, "ring_cfg": args.ring_cfg, "wg_per_cu": args.wg_per_cu, "tune": args.tune, "mbufs_loaded": m_loaded,
                          "ms": round(t * 1e3, 2), "mpps_aggregate": round(m / t / 1e6, 1),
                          "mpps_per_worker": round(m / t / 1e6 / k, 1),
                          "cpu_ns_per_pkt_per_worker": round(t * 1e9 * k / m, 1),
                          "prof_ns_per_pkt": prof}), flush=True)
    L.gh_fini()


if __name__ == "__main__":
    main()
