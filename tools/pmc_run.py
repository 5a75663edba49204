# SPDX-License-Identifier: BSD-3-Clause
"""Minimal runner for rocprofv3 --pmc passes: the headline workload
(1M-route view, 2^24 x 64 B) launched `--reps` times, plus one 1 GiB
device-to-device copy as the byte-count calibration for FETCH/WRITE_SIZE.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- \
        python3 tools/pmc_run.py
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--workload", default="fullview64",
                    choices=["fullview64", "single64", "fullview6", "imix", "imix_frames"])
    ap.add_argument("--slot", type=int, default=2240, help="imix_frames: bytes per frame slot (bench.py)")
    ap.add_argument("--ring", type=int, default=None, help="gr_hip_tune ring geometry")
    ap.add_argument("--wg", type=int, default=None, help="gr_hip_tune wg_per_cu")
    ap.add_argument("--stats", type=int, default=None)
    ap.add_argument("--nt", type=int, default=None)
    ap.add_argument("--fib-format", type=int, default=None, help="gr_hip_tune fib_format (0: 4-byte DIR24_8)")
    ap.add_argument("--no-calib", action="store_true")
    ap.add_argument("--span-bits", type=int, default=None,
                    help="fullview64 with destinations uniform in an aligned 2^N-address range (from 16.0.0.0 when "
                         "N <= 28, else from 0.0.0.0): the FIB lookups touch 2^(N-8) x 2 bytes of tbl24")
    args = ap.parse_args()
    import torch

    from grout_amd import abi
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath, shared_stream

    dev = torch.device("cuda", 0)
    if args.workload == "single64":
        topo = T.config_single_route()
        kw = dict(dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    elif args.workload == "fullview6":
        topo = T.config_fullview6()
        kw = None
    else:
        topo = T.config_fullview()
        kw = dict(routes=topo.route_array())
        if args.span_bits is not None:
            lo = 0x10000000 if args.span_bits <= 28 else 0
            kw = dict(dst_range=(lo, lo + (1 << args.span_bits) - 1))
        if args.workload == "imix_frames":  # whole IMIX frames in mbuf-like slots, as bench.py
            kw.update(imix=True, stride=args.slot)
        elif args.workload == "imix":  # IMIX header lines staged, as bench.py
            kw.update(imix=True, lines_only=True)
    fp = FastPath(0)
    if args.fib_format is not None:
        fp.tune("fib_format", args.fib_format)
    fp.load(topo)
    for k in ("ring", "wg", "stats", "nt"):
        v = getattr(args, k)
        if v is not None:
            fp.tune("wg_per_cu" if k == "wg" else k, v)
    n = args.batch
    if kw is None:
        r6 = topo.route6_array()
        frames, meta = S.stream6(n, S.SEED_GPU_BASE, r6[r6["prefixlen"] < 128])
    else:
        frames, meta = S.stream(n, S.SEED_GPU_BASE, **kw)
    stride = frames.shape[1]
    d_in = torch.from_numpy(frames.reshape(-1)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.uint8)).to(dev)
    d_out = torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev)
    d_v = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    q = fp.queue(shared_stream(dev))
    for _ in range(args.reps):
        q.submit(d_in, d_out, d_meta, d_v, n, in_stride=stride, out_stride=abi.LINE,
                 lines_only=args.workload == "imix")
    torch.cuda.synchronize()
    if args.no_calib:
        return
    # calibration: 1 GiB read + 1 GiB written by a streaming copy kernel
    a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    print("pmc_run done", n, args.reps)
    q.close()
    fp.close()
    del abi


if __name__ == "__main__":
    main()
