#!/usr/bin/env python3
"""Round 5's lost counter flushes (test_ring_give_up_is_reported):
the per-iface counters read and reset two ways, interleaved, many times.

Each iteration is the test's sequence: a launch forced to give up
(spin_max 1), the reset read, a full launch of 2^20 single-route packets, and
the read of every shard (gr_hip_queue_stats_shards), in one of two modes:

  copy    round 5's path ("stats_copy" 1): a hipMemcpy of the shards, and a
          hipMemsetAsync on the queue's stream to reset
  atomic  the library's path: gr_stats_collect, one agent-scope atomic per
          counter (fetch-add 0 to read, exchange with 0 to reset)

A read whose rx total differs from the packets sent names the shards that are
off. One JSON line per mode at the end (and one per miss as it happens).

  python tools/stats_read_probe.py --iters 200
"""
import argparse
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from grout_amd import abi  # noqa: E402
from grout_amd import synth as S  # noqa: E402
from grout_amd import topology as T  # noqa: E402
from grout_amd.fwd import FastPath  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--no-give-up", action="store_true", help="leave out the forced give-up launch")
    a = ap.parse_args()
    fp = FastPath()
    t = T.config_single_route()
    fp.load(t)
    n = 1 << 20
    fr, me = S.stream(n, 0x5A1, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    L = fp.lib
    b = fp.batch_alloc(n)
    for dst, src in ((b.in_frames, fr), (b.meta, me)):
        abi.check("h2d", L.gr_hip_memcpy_h2d(fp.h, dst, src.ctypes.data, src.nbytes))
    q = fp.queue()
    rx_if = int(me["iface"][0])
    res = {m: dict(mode=m, iters=0, misses=0, lost_packets=0, shard_hist={}) for m in ("copy", "atomic")}
    for it in range(a.iters):
        for mode in (("copy", "atomic") if it % 2 == 0 else ("atomic", "copy")):
            fp.tune("stats_copy", 1 if mode == "copy" else 0)
            if not a.no_give_up:
                fp.tune("spin_max", 1)
                abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
                L.gr_hip_queue_sync(q._h)
                L.gr_hip_queue_sync(q._h)
                fp.tune("spin_max", 0)
            q.stats(reset=True)
            abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
            r = L.gr_hip_queue_sync(q._h)
            sh = q.stats_shards(16)
            per = sh["rx_packets"][:, rx_if].astype(np.int64)
            R = res[mode]
            R["iters"] += 1
            if r != 0 or per.sum() != n:
                med = int(np.median(per))
                off = {int(s): int(per[s]) for s in np.nonzero(per != med)[0]}
                R["misses"] += 1
                R["lost_packets"] += int(n - per.sum())
                for s in off:
                    R["shard_hist"][str(s)] = R["shard_hist"].get(str(s), 0) + 1
                print(json.dumps(dict(miss=mode, iter=it, sync=r, got=int(per.sum()), median=med, off=off)),
                      flush=True)
        if it % 50 == 49:
            print(json.dumps(dict(progress=it + 1, **{m: res[m]["misses"] for m in res})), flush=True)
    fp.tune("stats_copy", 0)
    for m in res:
        print(json.dumps(res[m]), flush=True)
    q.close()
    fp.batch_free(b)
    fp.close()


if __name__ == "__main__":
    main()
