# SPDX-License-Identifier: BSD-3-Clause
"""The rte_graph node's whole walk (gr_hip_node_process: stage from the
mbufs, forward on the GPU, hand back onto the mbufs) from K worker threads at
once, each with its own queue and its own mbufs, like K grout workers sharing
one GPU. Per round: every thread resets its mbufs, a barrier,
every thread walks its batch, a barrier; the round's time is the wall clock
between the barriers. Aggregate Mpps = K x batch / that time (median round).

    python tools/node_scale.py [--threads 1,2,4,8] [--batch 1048576] > out.jsonl
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mode", default="frame_ptrs", choices=["frame_ptrs", "staged"])
    args = ap.parse_args()

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    fp.tune("host_direct", 1)
    fp.tune("node_ptrs", 1 if args.mode == "frame_ptrs" else 0)
    n = args.batch
    kmax = max(int(k) for k in args.threads.split(","))
    workers = []
    for w in range(kmax):
        fr, me = S.stream(n, S.SEED_GPU_BASE + w, routes=topo.route_array())
        bufs = np.zeros((n, 256), dtype=np.uint8)  # mbuf data rooms (frame at offset 0)
        bufs[:, :64] = fr
        mb = np.zeros(n, dtype=abi.MBUF_DT)
        mb["frame"] = bufs.ctypes.data + np.arange(n, dtype=np.uint64) * 256
        mb["pkt_len"] = me["pkt_len"]
        mb["data_len"] = me["pkt_len"]
        mb["data_off"] = 128
        mb["rss"] = me["rss"]
        mb["iface"] = me["iface"]
        abi.check("gr_hip_host_register", fp.lib.gr_hip_host_register(fp.h, bufs.ctypes.data, bufs.nbytes))
        workers.append({"fr": fr, "bufs": bufs, "mb": mb, "m": mb.copy(), "q": fp.queue()})
        workers[-1]["q"].node_process(workers[-1]["m"])  # warm-up: staging buffers grown
    for k in (int(x) for x in args.threads.split(",")):
        bar = threading.Barrier(k + 1)
        err = []

        def run(wk):
            try:
                for _ in range(args.rounds):
                    wk["m"][:] = wk["mb"]
                    wk["bufs"][:, :64] = wk["fr"]
                    bar.wait()
                    wk["q"].node_process(wk["m"])
                    bar.wait()
            except Exception as e:  # reported below
                err.append(e)
                bar.abort()

        ths = [threading.Thread(target=run, args=(workers[i],)) for i in range(k)]
        for t in ths:
            t.start()
        times = []
        try:
            for _ in range(args.rounds):
                bar.wait()
                t0 = time.perf_counter()
                bar.wait()
                times.append(time.perf_counter() - t0)
        except threading.BrokenBarrierError:
            pass
        for t in ths:
            t.join()
        if err:
            raise err[0]
        d = float(np.median(times))
        print(json.dumps({"mode": args.mode, "threads": k, "batch_per_thread": n, "ms_per_round": round(d * 1e3, 2),
                          "mpps_aggregate": round(k * n / d / 1e6, 1), "mpps_per_thread": round(n / d / 1e6, 1),
                          "pcie_bytes_per_pkt": 16 + 64 + 64 + 8 if args.mode == "frame_ptrs" else 72 + 72}),
              flush=True)
    for wk in workers:
        abi.check("gr_hip_host_unregister", fp.lib.gr_hip_host_unregister(fp.h, wk["bufs"].ctypes.data))
        wk["q"].close()
    fp.close()


if __name__ == "__main__":
    main()
