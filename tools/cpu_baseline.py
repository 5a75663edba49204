#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""The CPU baseline leg of bench.py alone, repeated: is it a steady state?

Each repetition times the oracle's restatement of grout's node chain
(oracle.c or_bench) on the full-view stream's 1M-packet
sample: one core, then `--threads` pinned cores each with its own IPv4 FIB
copy on THP, then the same with one shared FIB (grout's layout). Every
worker warms up with one untimed pass over the sample first. One JSON line
per repetition; VERDICT r03 asks single-core figures within 10 % of each
other and of the multi-core figure / cores."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import oracle  # noqa: E402  (test infrastructure: the CPU baseline only)
from bench import cpu_placement, host_cpus  # noqa: E402
from grout_amd import synth as S  # noqa: E402
from grout_amd import topology as T  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--seconds", type=float, default=4.0, help="timed part of each multi-core run")
    p.add_argument("--placement", default="allowed", choices=["allowed", "spread"],
                   help="worker i on the i-th allowed CPU, or bench.cpu_placement's spread")
    a = p.parse_args()
    t = T.config_fullview()
    fr, me = S.stream(1 << 20, 0x67720002, routes=t.route_array())
    o = oracle.Oracle(t)
    threads = max(1, min(a.threads, os.cpu_count() or 1))
    cpus = cpu_placement(threads, a.placement)
    for rep in range(a.reps):
        t0 = time.time()
        m1, _ = o.bench(fr, me, 1, 10_000_000)
        mN, _ = o.bench(fr, me, threads, int(m1 * 1e6 * a.seconds), cpus=cpus)
        mS, _ = o.bench(fr, me, threads, int(m1 * 1e6 * a.seconds), fib_copy=False, cpus=cpus)
        print(json.dumps({"rep": rep, "single_core_mpps": round(m1, 2), "cores": threads,
                          "fib_copy_mpps": round(mN, 2), "fib_copy_per_core": round(mN / threads, 2),
                          "shared_fib_mpps": round(mS, 2), "shared_fib_per_core": round(mS / threads, 2),
                          "host_cpus": host_cpus(), "placement": a.placement, "cpus": cpus, "wall_s": round(time.time() - t0, 1)}), flush=True)
    o.close()


if __name__ == "__main__":
    main()
