"""Longer differential fuzz run than tests/test_fuzz.py: many seeds, HIP
path against the oracle (whole frames, header lines, in place), one line
per mismatching seed and a JSON summary at the end.

    python tests/fuzz_sweep.py --seeds 300 [--first 0x10000]

Test infrastructure (it runs the oracle as the checker), so it lives under tests/.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]

import oracle  # noqa: E402
import test_fuzz as F  # noqa: E402
from golden_util import run_gpu  # noqa: E402
from grout_amd.fwd import FastPath  # noqa: E402


def diff(o, g):
    bad_v = np.nonzero(o[1] != g[1])[0]
    bad_l = np.nonzero((o[0] != g[0]).any(axis=1))[0]
    return len(bad_v), len(bad_l), bool(np.array_equal(o[2], g[2])), [int(i) for i in bad_v[:4]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=300)
    ap.add_argument("--first", type=lambda s: int(s, 0), default=0x10000)
    a = ap.parse_args()
    fp = FastPath(0)
    fails, t0 = [], time.time()
    for k in range(a.seeds):
        seed = a.first + k
        t, fr, me = F.fuzz_case(seed)
        o = oracle.Oracle(t)
        fr64 = np.ascontiguousarray(fr[:, :64])
        o_full = o.process(fr, me)
        for mode, want, got in [
                ("frames", o_full, lambda: run_gpu(fp, t, fr, me)),
                ("lines", o.process(fr64, me, lines_only=True), lambda: run_gpu(fp, t, fr64, me, lines_only=True)),
                ("inplace", o_full, lambda: run_gpu(fp, t, fr, me, inplace=True))]:
            r = diff(want, got())
            if r[0] or r[1] or not r[2]:
                fails.append({"seed": seed, "mode": mode, "bad_verdicts": r[0], "bad_lines": r[1],
                              "stats_equal": r[2], "first": r[3]})
                print(json.dumps(fails[-1]), flush=True)
        if k % 50 == 49:
            print(f"# {k + 1} seeds, {len(fails)} mismatches, {time.time() - t0:.0f}s", flush=True)
    print(json.dumps({"seeds": a.seeds, "first": a.first, "pkts_per_seed": F.N_PKTS, "modes": 3,
                      "mismatches": len(fails), "seconds": round(time.time() - t0, 1)}))
    fp.close()
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
