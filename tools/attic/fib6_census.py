# SPDX-License-Identifier: BSD-3-Clause
"""Where the IPv6 trie's lookups go (host only, no GPU): fib_inject -6's view
built with the product's FIB6 builder (fib6.c), a sample of the bench's
IPv6 stream walked through the painted image as the kernel walks it
(chain_fib6), and per dependent gather: the kind of table read (first
level, group, wide group, skip node), the distinct 128-byte lines the sample
touches there, and those lines by the matching route's prefix length.

    python tools/fib6_census.py [--packets 65536] > census.json
"""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from grout_amd import abi  # noqa: E402
from grout_amd import synth as S  # noqa: E402
from grout_amd import topology as T  # noqa: E402

EXT, SKIP, WIDE, IDX = 0x80000000, 0x40000000, 0x20000000, 0x1FFFFFFF
LINE = 128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 16)
    ap.add_argument("--routes", type=int, default=T.FULLVIEW6_ROUTES)
    a = ap.parse_args()
    t = T.config_fullview6(count=a.routes)
    r = t.route6_array()
    H = abi.host()
    for name, res, args in (("gr_fib6_new", ctypes.c_void_p, [ctypes.c_uint32, ctypes.c_uint32]),
                            ("gr_fib6_add", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8,
                                                           ctypes.c_uint32, ctypes.c_int]),
                            ("gr_fib6_build", ctypes.c_int, [ctypes.c_void_p]),
                            ("gr_fib6_top", ctypes.c_void_p, [ctypes.c_void_p]),
                            ("gr_fib6_groups", ctypes.c_void_p, [ctypes.c_void_p]),
                            ("gr_fib6_skips", ctypes.c_void_p, [ctypes.c_void_p]),
                            ("gr_fib6_groups_used", ctypes.c_uint32, [ctypes.c_void_p]),
                            ("gr_fib6_skips_used", ctypes.c_uint32, [ctypes.c_void_p]),
                            ("gr_fib6_free", None, [ctypes.c_void_p])):
        fn = getattr(H, name)
        fn.restype, fn.argtypes = res, args
    fmax = t.fibs6[T.VRF_MAIN]
    f = H.gr_fib6_new(fmax[0], fmax[1])
    for x in r:
        ip = np.ascontiguousarray(x["ip"])
        assert H.gr_fib6_add(f, ip.ctypes.data, int(x["prefixlen"]), int(x["nh"]), 0) == 0
    assert H.gr_fib6_build(f) == 0
    ng, nk = H.gr_fib6_groups_used(f), H.gr_fib6_skips_used(f)
    top = np.ctypeslib.as_array((ctypes.c_uint32 * 65536).from_address(H.gr_fib6_top(f)))
    groups = np.ctypeslib.as_array((ctypes.c_uint32 * (ng * 256)).from_address(H.gr_fib6_groups(f))) if ng else []
    skips = np.ctypeslib.as_array((ctypes.c_uint32 * (4 * nk)).from_address(H.gr_fib6_skips(f))).reshape(-1, 4) \
        if nk else np.zeros((0, 4), np.uint32)
    frames, _ = S.stream6(a.packets, S.SEED_GPU_BASE, r)
    dst = np.asarray(frames)[:, 38:54]
    # the matching route's length per packet (longest match in the RIB sample)
    lines = collections.defaultdict(set)  # (depth, kind) -> lines
    by_len = collections.defaultdict(set)  # (depth, kind, plen) -> lines
    pkts = collections.Counter()
    depth_hist = collections.Counter()
    plen_of = {}
    for x in r:
        plen_of[(bytes(x["ip"]), int(x["prefixlen"]))] = int(x["prefixlen"])
    # route per packet: stream6 picks a route and keeps its prefix, so match by mask
    for i in range(len(dst)):
        ip = bytes(dst[i])
        ent = int(top[(ip[0] << 8) | ip[1]])
        path = [(0, "top", ((ip[0] << 8) | ip[1]) * 4 // LINE)]
        b = 2
        while b < 16 and ent & EXT:
            if ent & SKIP and ent & WIDE:  # range group: 8-byte entries by byte b
                o = (ent & IDX) * 256 + 2 * ip[b]
                path.append((len(path), "range", ("g", o * 4 // LINE)))
                q0, q1 = int(groups[o]), int(groups[o + 1])
                ent = (q0 if (q0 >> 24) <= ip[b + 1] <= (q1 >> 24) else q1) & 0xFFFFFF
                b += 2
            elif ent & SKIP:
                k = ent & IDX
                path.append((len(path), "skip", ("s", k * 16 // LINE)))
                sk = skips[k]
                key = bytes(int(sk[0] >> (8 * j)) & 0xFF for j in range(4)) + bytes(int(sk[1] >> (8 * j)) & 0xFF
                                                                                   for j in range(3))
                n = int(sk[1] >> 24)
                match = b + n <= 16 and ip[b:b + n] == key[:n]
                ent = int(sk[2] if match else sk[3])
                b += n
            elif ent & WIDE:
                sh = (ent >> 26) & 7  # fib6.h: a narrow wide group keeps 2^(8-sh) entries per row
                o = (ent & 0x03FFFFFF) * 256 + (ip[b] << (8 - sh)) + (ip[b + 1] >> sh)
                path.append((len(path), "wide", ("g", o * 4 // LINE)))
                ent = int(groups[o])
                b += 2
            else:
                o = (ent & IDX) * 256 + ip[b]
                path.append((len(path), "group", ("g", o * 4 // LINE)))
                ent = int(groups[o])
                b += 1
        depth_hist[len(path)] += 1
        # the route this packet was drawn under: longest RIB prefix among the view's lengths
        plen = next((L for L in (128, 48, 46, 44, 42, 40, 38, 36, 32)
                     if (bytes(np.bitwise_and(np.frombuffer(ip, np.uint8),
                                              np.frombuffer(_mask(L), np.uint8))), L) in plen_of), -1)
        for d, kind, ln in path:
            lines[(d, kind)].add(ln)
            by_len[(d, kind, plen)].add(ln)
            pkts[(d, kind)] += 1
    out = {"routes": len(r), "groups_used": int(ng), "skips_used": int(nk), "packets": len(dst),
           "gathers_per_packet": {str(k): v / len(dst) for k, v in sorted(depth_hist.items())},
           "levels": [{"depth": d, "kind": kind, "packets": pkts[(d, kind)], "lines": len(v),
                       "bytes": len(v) * LINE,
                       "by_prefixlen": {str(L): len(by_len[(d, kind, L)]) for (dd, kk, L) in sorted(by_len)
                                        if dd == d and kk == kind}}
                      for (d, kind), v in sorted(lines.items())]}
    print(json.dumps(out))
    H.gr_fib6_free(f)


def _mask(L):
    m = bytearray(16)
    for i in range(16):
        k = min(8, max(0, L - 8 * i))
        m[i] = (0xFF << (8 - k)) & 0xFF
    return bytes(m)


if __name__ == "__main__":
    main()
