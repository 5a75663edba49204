# SPDX-License-Identifier: BSD-3-Clause
"""FIB load rate and forwarding under route churn.

1. Load: the 1M-route fib_inject -4 view (--ipv6: fib_inject -6's 200k-route
   view; smoke/fib_inject.c:245-254 times the injection and prints
   routes/s) into an empty VRF, one route per gr_hip_route4_add /
   gr_hip_route6_add call like fib_inject's one request per route, then one
   commit; and again in one batched call. routes/s = routes / (adds + commit).
2. Churn: the headline batch (2^24 packets over that view) submitted back to
   back for --seconds, without and then with a control thread applying
   --rate route changes per second (nexthop replacements, deletes and
   re-adds of random full-view routes, in --period-ms batches, one commit
   per batch). Mpps by wall clock over each window, and the commit latency.

    python tools/fib_churn.py [--ipv6] [--seconds 3] [--rate 10000] [--period-ms 10] > out.json
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--rate", type=int, default=10_000, help="route changes per second")
    ap.add_argument("--period-ms", type=float, default=10.0, help="one commit per period")
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--no-per-route", action="store_true")
    ap.add_argument("--ipv6", action="store_true", help="fib_inject -6's view and an IPv6 stream")
    args = ap.parse_args()
    v6 = args.ipv6
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    out = {"tool": "fib_churn", "family": "ipv6" if v6 else "ipv4"}
    if v6:
        topo = T.config_fullview6()
        routes = topo.route6_array()
        count = T.FULLVIEW6_ROUTES
    else:
        topo = T.config_fullview()
        routes = topo.route_array()
        count = 1_000_000
    view = routes[:count]
    vrf = int(view["vrf_id"][0])
    add_fn = "gr_hip_route6_add" if v6 else "gr_hip_route4_add"
    rsize = view.dtype.itemsize

    def fresh():
        fp = FastPath(0)
        fp.set_ifaces(topo.ifaces)
        fp.set_nexthops(topo.nh[1:topo.n_nh + 1], first=1)
        fp.set_reta(topo.reta)
        for v, (mr, nt) in topo.fibs.items():
            fp.fib_create(v, mr, nt)
        for v, (mr, ng) in topo.fibs6.items():
            fp.fib6_create(v, mr, ng)
        return fp

    def add(fp, r, replace=False):
        (fp.route6_add if v6 else fp.route_add)(r, replace=replace)

    def delete(fp, x):
        if v6:
            fp.route6_del(vrf, bytes(x["ip"]), int(x["prefixlen"]), int(x["iface_id"]))
        else:
            fp.route_del(vrf, int(x["ip"]), int(x["prefixlen"]))

    def commit(fp):
        (fp.fib6_commit if v6 else fp.fib_commit)(vrf)

    # 1. load rates
    if not args.no_per_route:
        fp = fresh()
        L, h = fp.lib, fp.h
        base = view.ctypes.data
        fn = getattr(L, add_fn)
        t0 = time.perf_counter()
        for i in range(count):
            r = fn(h, ctypes.c_void_p(base + rsize * i), 1, 0)
            if r:
                abi.check(add_fn, r)
        t1 = time.perf_counter()
        commit(fp)
        t2 = time.perf_counter()
        out["load_per_route"] = {"routes": count, "add_s": round(t1 - t0, 3), "commit_s": round(t2 - t1, 4),
                                 "routes_per_s": round(count / (t2 - t0)),
                                 "note": "one %s per route from Python ctypes, then one commit" % add_fn}
        print(json.dumps(out["load_per_route"]), file=sys.stderr, flush=True)
        fp.close()
    fp = fresh()
    t0 = time.perf_counter()
    add(fp, view)
    t1 = time.perf_counter()
    commit(fp)
    t2 = time.perf_counter()
    if len(routes) > count:
        add(fp, routes[count:])  # the address route: the bench topology exactly
    if v6:
        fp.route_add(topo.route_array())  # the IPv4 routes of the topology
        fp.fib_commit(vrf)
    commit(fp)
    t3 = time.perf_counter()
    out["load_batched"] = {"routes": count, "add_s": round(t1 - t0, 3), "commit_s": round(t2 - t1, 4),
                           "routes_per_s": round(count / (t2 - t0)),
                           "second_commit_s": round(t3 - t2, 4),
                           "note": "one route add call of all routes (gr_hip_route4_add / gr_hip_route6_add), then one commit (the first writes one "
                                   "copy whole; the second commit writes the other copy whole)"}
    print(json.dumps(out["load_batched"]), file=sys.stderr, flush=True)

    # 2. churn
    dev = torch.device("cuda", 0)
    n = args.batch
    if v6:
        frames, meta = S.stream6(n, S.SEED_FULLVIEW6, routes[routes["prefixlen"] < 128])
    else:
        frames, meta = S.stream(n, S.SEED_GPU_BASE, routes=routes)
    fin = torch.from_numpy(frames.reshape(-1)).to(dev)
    me = torch.from_numpy(meta.view(np.uint8)).to(dev)
    fo = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
    vo = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    del frames
    q = fp.queue(shared_stream(dev))
    fp.tune("untimed", 1)

    def forward(seconds):
        launches = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(4):
                q.submit(fin, fo, me, vo, n)
            q.sync()
            launches += 4
        dt = time.perf_counter() - t0
        return {"launches": launches, "s": round(dt, 3), "mpps": round(launches * n / dt / 1e6, 1)}

    forward(0.5)  # warm-up
    base = forward(args.seconds)
    print(json.dumps({"base": base}), file=sys.stderr, flush=True)

    nh_slots = np.unique(view["nh"])
    rng = np.random.default_rng(0xC4A9)
    per_commit = max(1, int(round(args.rate * args.period_ms / 1000)))
    stop = threading.Event()
    lat, clat, phases, applied = [], [], [], [0]
    deleted = []
    live = np.ones(count, dtype=bool)

    def control():
        period = args.period_ms / 1000
        nxt = time.perf_counter()
        while not stop.is_set():
            k_rep = per_commit // 2
            k_del = (per_commit - k_rep) // 2
            k_add = per_commit - k_rep - k_del
            idx = rng.choice(np.nonzero(live)[0], size=k_rep + k_del, replace=False)
            rep = view[idx[:k_rep]].copy()
            rep["nh"] = rng.choice(nh_slots, size=k_rep)
            t0 = time.perf_counter()
            add(fp, rep, replace=True)
            for i in idx[k_rep:]:
                delete(fp, view[i])
                live[i] = False
                deleted.append(i)
            back = [deleted.pop(0) for _ in range(min(k_add, len(deleted) - k_del))] if len(deleted) > k_del else []
            if back:
                add(fp, view[np.array(back)])
                live[np.array(back)] = True
            tc = time.perf_counter()
            commit(fp)
            t1 = time.perf_counter()
            lat.append(t1 - t0)
            clat.append(t1 - tc)
            phases.append([fp.tune(k) for k in ("commit_us_stage", "commit_us_enqueue", "commit_us_publish")])
            applied[0] += k_rep + k_del + len(back)
            nxt += period
            d = nxt - time.perf_counter()
            if d > 0:
                time.sleep(d)

    th = threading.Thread(target=control)
    t0 = time.perf_counter()
    th.start()
    churn = forward(args.seconds)
    stop.set()
    th.join()
    dt = time.perf_counter() - t0
    la = np.array(lat) * 1e3
    churn.update({"route_changes": applied[0], "changes_per_s": round(applied[0] / dt),
                  "commits": len(lat), "commit_ms_p50": round(float(np.percentile(la, 50)), 3),
                  "commit_ms_p99": round(float(np.percentile(la, 99)), 3), "commit_ms_max": round(float(la.max()), 3),
                  "changes_per_commit": per_commit,
                  "commit_call_ms_p50": round(float(np.percentile(np.array(clat) * 1e3, 50)), 3),
                  "commit_phase_us_p50": dict(zip(("stage", "enqueue", "publish"),
                                                  np.percentile(np.array(phases), 50, axis=0).round(1).tolist()))})
    out.update({"batch": n, "base": base, "churn": churn, "mpps_ratio": round(churn["mpps"] / base["mpps"], 4),
                "note": "wall-clock Mpps, submits of 4 launches then a sync, untimed launches; commit latency = "
                        "route adds/deletes + gr_hip_fib%s_commit" % ("6" if v6 else "4")})
    print(json.dumps(out), flush=True)
    q.close()
    fp.close()


if __name__ == "__main__":
    main()
