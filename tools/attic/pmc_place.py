"""Per-set counters from a rocprofv3 --pmc run of placement_probe.py
(--sets S --passes 1 --steps K): ring dispatches in schedule order are
S*5 warm-up, then S*K timed, then the 16 buffer mixes. Prints, per set,
the timed dispatches' mean duration and counters (per launch).

    python tools/pmc_place.py DIR [--sets 8] [--steps 5]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)[0]
    d = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "ring" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = d.setdefault(k, {"dur_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    ks = list(d)
    w = a.sets * 5
    for s in range(a.sets):
        sel = [d[k] for k in ks[w + s * a.steps: w + (s + 1) * a.steps]]
        avg = {c: sum(x[c] for x in sel) / len(sel) for c in sel[0]}
        print(json.dumps({"set": s, **{c: round(v, 4 if c == "dur_ms" else 0) for c, v in avg.items()}}))


if __name__ == "__main__":
    main()
