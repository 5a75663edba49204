# SPDX-License-Identifier: BSD-3-Clause
"""PCIe ceilings of the box: pinned host <-> device copy rates, one direction
at a time and both at once (two streams), at the host path's chunk sizes."""
import json
import time

import torch


def rate(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    dev = torch.device("cuda", 0)
    for mb in (4, 18, 64, 256):
        n = mb << 20
        h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
        h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
        d_a = torch.empty(n, dtype=torch.uint8, device=dev)
        d_b = torch.empty(n, dtype=torch.uint8, device=dev)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

        def h2d():
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)

        def d2h():
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)

        def both():
            h2d()
            d2h()
        r = {"mib": mb, "h2d_GBps": round(rate(h2d, n), 1), "d2h_GBps": round(rate(d2h, n), 1),
             "both_GBps_per_dir": round(rate(both, n), 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
