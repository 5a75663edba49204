#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""How busy the GPU was during each burst of kernels in a rocprofv3 kernel
trace (`--kernel-trace`: the *_kernel_trace.csv, or the *_results.db that
ROCm 7's rocprofv3 writes by default): kernels are grouped into
runs separated by more than --gap-ms of idle GPU, and each run reports its
span, the time at least one kernel was running (the union of the kernels'
intervals), that as a fraction of the span, the summed kernel time (above
the union when kernels of several queues overlap) and the mean kernel.

    python tools/kernel_busy.py gpurun_out/prof_w16/w16_results.db --kernel gr_fwd4_ring
"""
import argparse
import csv
import json
import sqlite3


def runs(intervals, gap_ns):
    out, cur = [], []
    for s, e in sorted(intervals):
        if cur and s - max(x[1] for x in cur) > gap_ns:
            out.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        out.append(cur)
    return out


def union(iv):
    busy, end = 0, None
    for s, e in sorted(iv):
        if end is None or s > end:
            busy += e - s
            end = e
        elif e > end:
            busy += e - end
            end = e
    return busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=5.0)
    ap.add_argument("--kernel", default="", help="only kernels whose name contains this")
    a = ap.parse_args()
    iv = []
    if a.trace.endswith(".db"):
        db = sqlite3.connect(a.trace)
        for name, s, e in db.execute("select name, start, end from kernels"):
            if a.kernel in name:
                iv.append((int(s), int(e)))
    else:
        with open(a.trace, newline="") as f:
            for row in csv.DictReader(f):
                if a.kernel in row["Kernel_Name"]:
                    iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    for k, r in enumerate(runs(iv, a.gap_ms * 1e6)):
        span = max(e for _, e in r) - min(s for s, _ in r)
        busy = union(r)
        total = sum(e - s for s, e in r)
        print(json.dumps({"run": k, "kernels": len(r), "span_ms": round(span / 1e6, 3),
                          "busy_ms": round(busy / 1e6, 3), "busy_frac": round(busy / span, 3) if span else None,
                          "kernel_ms_sum": round(total / 1e6, 3), "kernel_us_mean": round(total / len(r) / 1e3, 1)}))


if __name__ == "__main__":
    main()
