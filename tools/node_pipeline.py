# SPDX-License-Identifier: BSD-3-Clause
"""The rte_graph node's walk done in flushes of F packets, one flush waited
for at a time (depth 1: gr_hip_node_process) or pipelined two deep (depth 2:
gr_hip_node_start of flush i, then gr_hip_node_finish of flush i-1, as the
grout node does, gpu_fwd4_node.c). K worker threads at once, each with its
own queue and 2^20 mbufs of the full-view stream (staged header lines, the
node's default). Per round every thread resets its mbufs, a barrier, walks
them all, a barrier; aggregate Mpps = K x mbufs / the median round.

    python tools/node_pipeline.py [--threads 1,4,8] [--flush 4096,16384,65536] [--thp] > out.jsonl

--thp puts the data rooms and the gr_hip_mbuf views on transparent huge
pages, as DPDK's mempools are on hugepages (4 KiB pages cost a TLB miss per
mbuf).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def walk(q, m, flush, depth):
    n = len(m)
    if depth == 1:
        for o in range(0, n, flush):
            q.node_process(m[o:o + flush])
        return
    for o in range(0, n, flush):
        q.node_start(m[o:o + flush])
        if o:
            q.node_finish()
    q.node_finish()


def zeros(shape, dtype, thp):
    if not thp:
        return np.zeros(shape, dtype=dtype)
    import mmap
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    mm = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    mm.madvise(mmap.MADV_HUGEPAGE)
    return np.frombuffer(mm, dtype=dtype).reshape(shape)  # zero-filled; the array keeps the map


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4,8")
    ap.add_argument("--flush", default="4096,16384,65536")
    ap.add_argument("--mbufs", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--driver", default="python", choices=["python", "c"],
                    help="c: the threads are C pthreads in tools/libnode_mt.so (no Python between the calls)")
    ap.add_argument("--thp", action="store_true", help="mbufs and data rooms on transparent huge pages")
    args = ap.parse_args()

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    fp = FastPath(0)
    fp.load(topo)
    n = args.mbufs
    threads = [int(x) for x in args.threads.split(",")]
    workers = []
    for w in range(max(threads)):
        fr, me = S.stream(n, S.SEED_GPU_BASE + w, routes=topo.route_array())
        bufs = zeros((n, 256), np.uint8, args.thp)  # mbuf data rooms (frame at offset 0)
        bufs[:, :64] = fr
        mb = zeros(n, abi.MBUF_DT, False)
        mb["frame"] = bufs.ctypes.data + np.arange(n, dtype=np.uint64) * 256
        mb["pkt_len"] = me["pkt_len"]
        mb["data_len"] = me["pkt_len"]
        mb["data_off"] = 128
        mb["rss"] = me["rss"]
        mb["iface"] = me["iface"]
        m = zeros(n, abi.MBUF_DT, args.thp)
        m[:] = mb
        wk = {"fr": fr, "bufs": bufs, "mb": mb, "m": m, "q": fp.queue()}
        walk(wk["q"], wk["m"], 1 << 16, 2)  # warm-up: both staging slots grown
        workers.append(wk)
    check = None
    if args.driver == "c":
        import ctypes
        C = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnode_mt.so"))
        C.node_mt_round.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    for flush in (int(x) for x in args.flush.split(",")):
        for k in threads:
            for depth in (1, 2):
                if args.driver == "c":
                    qs = (ctypes.c_void_p * k)(*[workers[i]["q"]._h.value for i in range(k)])
                    ms = (ctypes.c_void_p * k)(*[workers[i]["m"].ctypes.data for i in range(k)])
                    times = []
                    for _ in range(args.rounds):
                        for i in range(k):
                            workers[i]["m"][:] = workers[i]["mb"]
                            workers[i]["bufs"][:, :64] = workers[i]["fr"]
                        sec = ctypes.c_double()
                        abi.check("node_mt_round", C.node_mt_round(qs, ms, k, n, flush, depth, ctypes.byref(sec)))
                        times.append(sec.value)
                    d = float(np.median(times))
                    print(json.dumps({"driver": "c", "thp": args.thp, "flush_pkts": flush, "threads": k, "depth": depth,
                                      "mbufs_per_thread": n, "ms_per_round": round(d * 1e3, 2),
                                      "mpps_aggregate": round(k * n / d / 1e6, 1),
                                      "mpps_per_thread": round(n / d / 1e6, 1)}), flush=True)
                    continue
                bar = threading.Barrier(k + 1)
                err = []

                def run(wk):
                    try:
                        for _ in range(args.rounds):
                            wk["m"][:] = wk["mb"]
                            wk["bufs"][:, :64] = wk["fr"]
                            bar.wait()
                            walk(wk["q"], wk["m"], flush, depth)
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
                # both depths leave the same mbufs: edges and rewritten frames
                got = (workers[0]["m"]["edge"].copy(), workers[0]["bufs"][:, :32].copy())
                if check is None:
                    check = got
                same = bool(np.array_equal(got[0], check[0]) and np.array_equal(got[1], check[1]))
                d = float(np.median(times))
                print(json.dumps({"thp": args.thp, "flush_pkts": flush, "threads": k, "depth": depth, "mbufs_per_thread": n,
                                  "ms_per_round": round(d * 1e3, 2), "mpps_aggregate": round(k * n / d / 1e6, 1),
                                  "mpps_per_thread": round(n / d / 1e6, 1), "same_results": same}), flush=True)
    for wk in workers:
        wk["q"].close()
    fp.close()


if __name__ == "__main__":
    main()
