#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""Per-launch counters of the ring kernel by workload, from
tools/pmc_compare.sh's passes: mean over the dispatches of each pass (the
first one dropped), one JSON object per workload, and the ratio of each
counter to the first workload's."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    out = collections.OrderedDict()
    def order(x):  # single64 first, spans by size, then the rest
        return (x != "single64", not x.startswith("span"), int(x[4:]) if x[4:].isdigit() else 0, x)
    for wl in sorted(os.listdir(root), key=order):
        if not os.path.isdir(os.path.join(root, wl)):
            continue
        c, durs = {}, []
        for f in sorted(glob.glob(os.path.join(root, wl, "**", "*counter_collection.csv"), recursive=True)):
            d = collections.OrderedDict()
            for r in csv.DictReader(open(f)):
                if "ring" not in r["Kernel_Name"]:
                    continue
                e = d.setdefault(int(r["Dispatch_Id"]), {"_dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            rows = list(d.values())[1:]
            if not rows:
                continue
            durs += [x["_dur"] for x in rows]
            for k in rows[0]:
                if k != "_dur":
                    c[k] = sum(x[k] for x in rows) / len(rows)
        out[wl] = {"kernel_ms_mean": round(sum(durs) / len(durs), 4) if durs else None,
                   "counters": {k: round(v) for k, v in sorted(c.items())}}
    names = list(out)
    if len(names) > 1:
        base = out[names[0]]["counters"]
        for wl in names[1:]:
            out[wl]["over_" + names[0]] = {k: round(v / base[k], 3) for k, v in out[wl]["counters"].items()
                                           if base.get(k)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
