# SPDX-License-Identifier: BSD-3-Clause
"""Summarise rocprofv3 --pmc counter CSVs per kernel (average per dispatch).

    python tools/pmc_summary.py OUTDIR [OUTDIR ...] > summary.json

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide streaming read, so
the corrected read bytes are 2 x FETCH_SIZE x 1024 -- checked here against the
1 GiB calibration copy the runner performs (tools/pmc_run.py).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "?")
                fw = [x for x in ("gr_fwd4_ring", "gr_fwd4_pipe", "gr_fwd4_kernel") if x in k]
                k = fw[0] if fw else ("copy" if "copy" in k.lower() or "elementwise" in k else k[:60])
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, ctrs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        out[k]["_dispatch_samples"] = max(len(v) for v in ctrs.values())
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
