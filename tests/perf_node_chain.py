#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Host-memory deployment, like for like: grout's CPU chain and the GPU node
in the same walk harness. TEST INFRASTRUCTURE: it runs
the oracle's restatement of grout's nodes as the CPU chain, so it lives under
tests/ (not collected: no test_ prefix; tests/test_graph_walk.py runs --check).

Both modes are K worker graphs walked from K pinned pthreads (the harness's
gh_workers_run: one graph per worker as grout's worker.c, each polling its own
share of the full-view stream like an RX queue, through the same port_rx
stand-in, per-worker mempools of --recycle mbufs and the same recorders behind
the edges):

  gpu    port_rx -> iface_input = the fast path's node (gpu_fwd4_node.c):
         stage, GPU, hand back onto the mbufs (one GPU, one queue per worker)
  chain  port_rx_chain -> cpu_chain = grout's node chain iface_input ..
         iface_output run on the CPU over the mbufs in place (the oracle's
         restatement, or_walk_frames: DIR24_8 with 8-byte entries, one FIB
         shared by every worker as grout's rte_fib), then grout's mbuf fields
         and private data, enqueued on the same edges

For each K: Mpps (all packets / the slowest worker's wall time) and CPU ns
per packet per worker (= wall x K / packets) of each mode, medians over
--reps back-to-back rounds (gpu, chain, harness alone), and in a separate
run per mode with latency on, the p50 / p99 of each packet's time from
port_rx to the recorder behind its edge (TSC, one read per burst at RX and
per recorder call). One JSON line per K.

    python tests/perf_node_chain.py --threads 1,8,16 --recycle 65536 --passes 8 --lcores spread
    python tests/perf_node_chain.py --check      # CPU: the chain graph against the oracle's mbufs
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

GH_LAT_BUCKETS = 64 * 16


def chain_bind(L, o):
    """Point the harness's cpu_chain node at the oracle's or_walk_frames on o."""
    import oracle
    fn = oracle.lib().or_walk_frames
    L.gh_set_chain.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.gh_set_chain.restype = None
    L.gh_set_chain(ctypes.cast(fn, ctypes.c_void_p), o.h)


def check(L, G):
    """The chain graph's walk (single-threaded, recording) ends every mbuf of
    the exception corpus and of a full-view stream as the oracle's mbuf-level
    chain does (edge, lengths, data_off, packet_type, frame bytes): the
    comparison measures the same work in both modes."""
    import oracle
    import scenarios as SC
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    k = L.gh_graph_create_chain(0, 0)
    assert k >= 0, k
    assert L.gh_graph_use(k) == 0
    cases = [(SC.corpus_topology()[0],) + tuple(SC.corpus_arrays()[:2])]
    tf = T.config_fullview(count=100_000)
    cases.append((tf,) + S.stream(20_000, 0xC4A1, routes=tf.route_array()))
    for topo, fr, me in cases:
        fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
        ifs = np.ascontiguousarray(topo.ifaces[topo.ifaces["id"] != 0])
        nh = np.ascontiguousarray(topo.nh[1:topo.n_nh + 1])
        assert L.gh_set_objects(ifs.ctypes.data, len(ifs), nh.ctypes.data, 1, len(nh)) == 0
        o = oracle.Oracle(topo)
        chain_bind(L, o)
        lines_w, v, _, want, _ = o.process_mbufs(fr, me, burst=64)
        n = len(me)
        assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, n) == 0
        assert L.gh_run(1 << 22) > 0
        out = np.zeros(n, dtype=G.OUT_DT)
        lines = np.zeros((n, abi.LINE), dtype=np.uint8)
        assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
        # packets the continuation nodes take further (ip_output_snat,
        # ip_input_local_ct: the module's CPU nodes, behind either node) and
        # the checksum status no ol_flags value expresses (the corpus's 3)
        # are not compared
        cont = np.isin(want["edge"], [abi.EDGE["ip_output_snat"], abi.EDGE["ip_input_local_ct"]])
        keep = ~cont & (((me["vlan_ck"] >> 12) & 3) != 3)
        out, want, lines, lines_w = out[keep], want[keep], lines[keep], lines_w[keep]
        for f in ("edge", "pkt_len", "data_len", "data_off", "packet_type"):
            bad = np.nonzero(out[f] != want[f])[0]
            assert len(bad) == 0, (f, bad[:5], out[f][bad[:5]], want[f][bad[:5]])
        fwd = out["edge"] == abi.EDGE["port_output"]
        assert fwd.sum() > 40, fwd.sum()
        assert (out["iface"][fwd] == want["iface"][fwd]).all(), (out["iface"][fwd][:8], want["iface"][fwd][:8])
        assert np.array_equal(lines, lines_w)  # the frames rewritten in place as grout's nodes do
        L.gh_set_chain(None, None)
        o.close()
    print(json.dumps({"check": "ok", "cases": [len(c[2]) for c in cases]}), flush=True)


def percentiles(hist, cycles_per_ns, floor, qs=(0.5, 0.99)):
    tot = hist.sum()
    cum = np.cumsum(hist)
    out = {}
    for q in qs:
        b = int(np.searchsorted(cum, q * tot))
        out[f"p{int(q * 100)}_us"] = round(floor[b] / cycles_per_ns / 1e3, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="only the chain graph against the oracle (no GPU)")
    ap.add_argument("--threads", default="1,8,16")
    ap.add_argument("--per-thread", type=int, default=1 << 18, help="mbufs loaded per worker")
    ap.add_argument("--batch", type=int, default=15360)
    ap.add_argument("--batches", default=None,
                    help="GPU node batch sizes to sweep at each K (gpu_fwd4_set_batch), e.g. 1024,4096,15360; "
                         "the chain and the harness alone are measured once per K")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--budget-us", type=float, default=0,
                    help="the GPU node's latency budget (gpu_fwd4_set_latency_budget): batches sized so that their "
                         "oldest packet comes back within it; --batch is then the largest batch")
    ap.add_argument("--recycle", type=int, default=65536, help="mbufs per worker's pool (0: one per packet)")
    ap.add_argument("--passes", type=int, default=8, help="with --recycle: passes over each worker's share")
    ap.add_argument("--lcores", default="spread", choices=["none", "allowed", "spread", "socket"])
    ap.add_argument("--out", default=None, help="also append the lines to this JSONL file")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="gr_hip_tune knobs of the GPU node's contexts, e.g. resident=1, or launch_per_batch (the module's) (repeatable)")
    ap.add_argument("--alt", action="append", default=[], metavar="KEY=VALUE/BACK",
                    help="also run the GPU node with knob KEY at VALUE (gpu_alt), interleaved with the other "
                         "modes in every rep, KEY set back to BACK after each run, e.g. resident=0/1 (repeatable)")
    args = ap.parse_args()

    import test_graph_walk as G
    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T

    L = G.lib()
    for name, res, argt in [("gh_graph_create_chain", ctypes.c_int, [ctypes.c_uint, ctypes.c_int]),
                            ("gh_workers_first", ctypes.c_int, [ctypes.c_uint32]),
                            ("gh_set_latency", None, [ctypes.c_int]),
                            ("gh_latency", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32,
                                                          ctypes.POINTER(ctypes.c_double)]),
                            ("gh_lat_bucket_floor", ctypes.c_uint64, [ctypes.c_uint32]),
                            ("gh_workers_run", ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                                              ctypes.POINTER(ctypes.c_uint64)]),
                            ("gh_set_rx_touch", None, [ctypes.c_int]), ("gh_set_null_node", None, [ctypes.c_int]),
                            ("gh_set_recycle", None, [ctypes.c_uint32, ctypes.c_uint32]),
                            ("gh_walk_info_at", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
                            ("gh_node_stats_at", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
                            ("gpu_fwd4_set_latency_budget", ctypes.c_int, [ctypes.c_uint64])]:
        f = getattr(L, name)
        f.restype, f.argtypes = res, argt

    threads = [int(x) for x in args.threads.split(",")]
    kmax = 1 if args.check else max(threads)
    devs = (ctypes.c_int * 1)(0)
    r = L.gh_init(ctypes.cast(devs, ctypes.c_void_p), 1, 1024, 1 << 17, args.batch, 64, 20_000_000)
    if args.check:
        assert r in (0, -19), r  # -ENODEV without a GPU: the chain needs none
        check(L, G)
        L.gh_fini()
        return
    assert r == 0, r
    import oracle
    for k in range(kmax):  # slots 0 .. kmax-1: the GPU node's graphs
        assert L.gh_graph_create(k, 0) == k
    for k in range(kmax):  # slots kmax .. 2 kmax-1: the chain's
        assert L.gh_graph_create_chain(k, 0) == kmax + k
    fp = G.FanOutPath(L)
    topo = T.config_fullview()
    fp.load(topo)
    L.gpu_fwd4_set_launch_per_batch.argtypes = [ctypes.c_int]
    L.gpu_fwd4_set_depth.argtypes = [ctypes.c_uint32]

    def set_knob(key, v):
        """launch_per_batch, depth: the module's own (gpu_fwd4_set_launch_per_batch,
        gpu_fwd4_set_depth); else a gr_hip_tune knob of every context."""
        if key == "launch_per_batch":
            assert L.gpu_fwd4_set_launch_per_batch(v) == 0
        elif key == "depth":
            assert L.gpu_fwd4_set_depth(v) == 0
        else:
            fp.tune(key, v)

    for kv in args.tune:
        k, v = kv.split("=")
        set_knob(k, int(v))
    alt = [(kv.split("=")[0], int(kv.split("=")[1].split("/")[0])) for kv in args.alt]
    alt_back = [(kv.split("=")[0], int(kv.split("/")[1])) for kv in args.alt]
    ifs = np.ascontiguousarray(topo.ifaces[topo.ifaces["id"] != 0])
    nh = np.ascontiguousarray(topo.nh[1:topo.n_nh + 1])
    assert L.gh_set_objects(ifs.ctypes.data, len(ifs), nh.ctypes.data, 1, len(nh)) == 0
    o = oracle.Oracle(topo)
    chain_bind(L, o)
    n = kmax * args.per_thread
    fr, me = S.stream(n, 0x67720002, routes=topo.route_array())
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    L.gh_set_pin(0)  # staged header lines, the node's default
    L.gh_set_rx_touch(1)
    L.gh_set_recycle(args.recycle, args.passes)
    per = args.passes if args.recycle else 1
    floor = np.array([L.gh_lat_bucket_floor(b) for b in range(GH_LAT_BUCKETS)], dtype=np.float64)
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

    def once(k, m, mode, lat=False):
        """One workers run of mode gpu / chain / alone (port_rx straight to
        port_output): wall seconds (and the latency histogram)."""
        assert L.gh_workers_first(kmax if mode == "chain" else 0) == 0
        L.gh_set_null_node(1 if mode == "alone" else 0)
        L.gh_set_latency(1 if lat else 0)
        for key, v in (alt if mode == "gpu_alt" else []):
            set_knob(key, v)
        try:
            assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, m) == 0
            s, w = ctypes.c_double(), ctypes.c_uint64()
            rr = L.gh_workers_run(k, ctypes.byref(s), ctypes.byref(w))
            assert rr == 0, (mode, rr)
            hist = None
            if lat:
                hist = np.zeros(GH_LAT_BUCKETS, dtype=np.uint64)
                cpn = ctypes.c_double()
                assert L.gh_latency(hist.ctypes.data, GH_LAT_BUCKETS, ctypes.byref(cpn)) == GH_LAT_BUCKETS
                hist = (hist, cpn.value)
            return s.value, hist
        finally:
            for key, v in (alt_back if mode == "gpu_alt" else []):
                set_knob(key, v)
            L.gh_set_null_node(0)
            L.gh_set_latency(0)
            L.gh_workers_first(0)

    out = open(args.out, "a") if args.out else None
    L.gpu_fwd4_set_batch.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    batches = [int(x) for x in args.batches.split(",")] if args.batches else [args.batch]
    assert L.gpu_fwd4_set_latency_budget(int(args.budget_us * 1e3)) == 0
    for k, batch in [(k, b) for k in threads for b in batches]:
        assert L.gpu_fwd4_set_batch(batch, 20_000_000) == 0
        cpus = place(k)
        m = k * args.per_thread
        pk = m * per
        gmodes = ("gpu", "gpu_alt") if alt else ("gpu",)
        for mode in gmodes + ("chain", "alone"):  # warm-up: pages, queues, pinned slots, FIB in cache
            once(k, m, mode)
        t = {mode: [] for mode in gmodes + ("chain", "alone")}
        for _ in range(args.reps):
            for mode in t:
                t[mode].append(once(k, m, mode)[0])
        med = {mode: float(np.median(v)) for mode, v in t.items()}
        lat = {}
        caps, health = {}, {}
        for mode in gmodes + ("chain",):
            _, (hist, cpn) = once(k, m, mode, lat=True)
            assert int(hist.sum()) == pk, (mode, int(hist.sum()), pk)
            lat[mode] = percentiles(hist.astype(np.float64), cpn, floor)
            if mode != "chain":  # each worker graph's batch cap where the run left it, and what went wrong
                wi = np.zeros(1, dtype=G.WALK_INFO_DT)
                cs, over, errs = [], 0, 0
                for g in range(k):
                    assert L.gh_walk_info_at(g, wi.ctypes.data) == 0
                    cs.append(int(wi[0]["batch_cap"]))
                    over += int(wi[0]["over_budget"])
                    e = ctypes.c_uint64()
                    assert L.gh_node_stats_at(g, None, ctypes.byref(e)) == 0
                    errs += e.value
                caps[mode] = cs
                health[mode] = {"over_budget_batches": over, "gpu_errors": errs,
                                "resident_cancels": abi.hip().gr_hip_tune(L.gh_hip_ctx(), b"resident_cancels", 0)}
        line = {"threads": k, "packets": pk, "lcores": args.lcores, "cpus": cpus, "recycle": args.recycle,
                "passes": per, "batch": batch, "reps": args.reps, "tune": args.tune, "alt": args.alt,
                **({"budget_us": args.budget_us, "batch_caps": caps} if args.budget_us else {}),
                "gpu_health": health,
                "workload": "config3 full view (fib_inject 1M routes), 64 B, seeded stream 0x67720002"}
        for mode in gmodes + ("chain",):
            line[mode] = {"mpps": round(pk / med[mode] / 1e6, 1),
                          "cpu_ns_per_pkt_per_worker": round(med[mode] * 1e9 * k / pk, 1),
                          "walk_ns_per_pkt_per_worker": round((med[mode] - med["alone"]) * 1e9 * k / pk, 1),
                          **lat[mode]}
        line["harness_alone"] = {"mpps": round(pk / med["alone"] / 1e6, 1),
                                 "cpu_ns_per_pkt_per_worker": round(med["alone"] * 1e9 * k / pk, 1)}
        line["gpu_over_chain"] = round(med["chain"] / med["gpu"], 3)
        if alt:
            line["gpu_over_gpu_alt"] = round(med["gpu_alt"] / med["gpu"], 3)
        s = json.dumps(line)
        print(s, flush=True)
        if out:
            out.write(s + "\n")
            out.flush()
    o.close()
    L.gh_fini()


if __name__ == "__main__":
    main()
