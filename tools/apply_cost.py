#!/usr/bin/env python3
# SPDX-License-Identifier: BSD-3-Clause
"""CPU cost of the node's hand-back on this box's CPU, in ns per packet: the
apply of gr_hip_node_finish_mbufs (gr_node_apply_ex straight onto the mbufs,
grout_amd/csrc/gr_node.cpp) over batches of the full-view stream, and the
staging of the same batches (gr_hip_node_stage). No rte_graph around it and
no GPU wait: the verdicts and header lines come from one GPU pass over the
stream (gr_hip_fwd4_host) before the clocks start. The mbufs (rte_mbuf,
private area, frame: 2304-byte objects) sit on transparent huge pages, as
DPDK's mempools sit on hugepages. Variants on one library: with and without
the per-iface and per-node counters, so that each part's share shows, and
with the frames taken as already rewritten (lines NULL: what the hand-back
would cost if the GPU wrote its prefixes into the frames itself).
Compare library builds by running this once per build, alternating
(--lib build/ab/<name>.so; tools/ab_libs.sh's pattern).

    python tools/apply_cost.py [--lib PATH] [--batch 15360] > out.jsonl
"""
import argparse
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# grout's rte_mbuf and private-data offsets (DPDK rte_mbuf_core.h; grout
# mbuf.h:29-41, rxtx.h:45-48, eth.h:23-36, l3.h:9), as tests/test_node_shim.py
LAYOUT = dict(data_off=16, data_len=40, pkt_len=36, packet_type=32, priv=128, priv_iface=16, priv_vlan_id=24,
              priv_domain=24, priv_eth_nh=32, priv_l3_nh=24)
OBJ, FRAME = 2304, 320  # object size (rte_mbuf 128 + priv 64 + headroom 128 + data), frame offset


class Layout(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint16) for k in LAYOUT] + [
        ("n_ifaces", ctypes.c_uint32), ("n_nh", ctypes.c_uint32), ("ifaces", ctypes.c_void_p), ("nh", ctypes.c_void_p),
        ("buf_addr", ctypes.c_uint16), ("ol_flags", ctypes.c_uint16), ("rss", ctypes.c_uint16),
        ("iface_id", ctypes.c_uint16), ("ck_mask", ctypes.c_uint64), ("ck_good", ctypes.c_uint64),
        ("ck_bad", ctypes.c_uint64)]


class Direct(ctypes.Structure):
    _fields_ = [("mbufs", ctypes.c_void_p), ("lay", ctypes.c_void_p), ("edges", ctypes.c_void_p),
                ("stale", ctypes.c_uint32), ("meta", ctypes.c_void_p)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None, help="library build to time (default: the in-tree one)")
    ap.add_argument("--pkts", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=15360)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from grout_amd import abi
    if args.lib:
        abi.LIB_HIP = os.path.abspath(args.lib)
    from grout_amd import synth as S
    from grout_amd import topology as T
    from grout_amd.fwd import FastPath

    topo = T.config_fullview()
    n = args.pkts
    fr, me = S.stream(n, S.SEED_GPU_BASE, routes=topo.route_array())
    fp = FastPath(0)
    fp.load(topo)
    q = fp.queue()
    lines, v = q.forward_host(np.ascontiguousarray(fr[:, :abi.LINE]), me)
    q.close()
    fp.close()
    out32 = np.ascontiguousarray(lines[:, :abi.PREFIX])  # what the node's walk gets back

    mm = mmap.mmap(-1, n * OBJ + (2 << 20))
    mm.madvise(mmap.MADV_HUGEPAGE)
    mem = np.frombuffer(mm, dtype=np.uint8)
    base = (mem.ctypes.data + (2 << 20) - 1) & ~((2 << 20) - 1)
    off = base - mem.ctypes.data
    objs = mem[off:off + n * OBJ].reshape(n, OBJ)
    objs[:, FRAME:FRAME + abi.LINE] = fr[:, :abi.LINE]
    ptrs = (base + np.arange(n, dtype=np.uint64) * OBJ).astype(np.uint64)
    m = np.zeros(n, dtype=abi.MBUF_DT)
    m["frame"] = ptrs + FRAME
    m["pkt_len"] = me["pkt_len"]
    m["data_len"] = me["pkt_len"]
    m["data_off"] = 128
    m["rss"] = me["rss"]
    m["iface"] = me["iface"]
    m["vlan_id"] = me["vlan_ck"] & 0xFFF
    m["ck"] = (me["vlan_ck"] >> 12) & 3
    m["flags"][::64] = abi.MBUF_F_WALK

    reg_if = np.zeros(topo.max_ifaces, dtype=np.uint64)
    live = topo.ifaces["id"] != 0
    reg_if[live] = 0x7F0000001000 + np.nonzero(live)[0]  # registry "pointers": never dereferenced
    reg_nh = (0x7F0000100000 + np.arange(len(topo.nh), dtype=np.uint64)).astype(np.uint64)
    reg_nh[0] = 0
    lay = Layout(**LAYOUT, n_ifaces=len(reg_if), n_nh=len(reg_nh), ifaces=reg_if.ctypes.data, nh=reg_nh.ctypes.data)
    ifaces = np.ascontiguousarray(topo.ifaces)
    nh = np.ascontiguousarray(topo.nh)
    st = np.zeros(topo.max_ifaces, dtype=abi.STATS_DT)
    ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
    vl = np.zeros(3, dtype=np.uint64)  # struct gr_node_vlans: no VLAN sub-interfaces in this view
    edges = np.zeros(args.batch, dtype=np.uint8)
    stage_lines = np.zeros((args.batch, abi.LINE), dtype=np.uint8)
    stage_meta = np.zeros(args.batch, dtype=abi.META_DT)

    L = ctypes.CDLL(abi.LIB_HIP)
    P, U32 = ctypes.c_void_p, ctypes.c_uint32
    L.gr_node_apply_ex.argtypes = [P, U32, U32, P, P, U32, P, P, U32, P, U32, P, P, P, U32, P]
    L.gr_hip_node_stage.argtypes = [P, U32, U32, P, P, P]
    B = args.batch
    starts = list(range(0, n - B + 1, B))

    m0 = m.copy()

    def apply_pass(ifst, stats, direct=True, in_place=False):
        t = 0.0
        for s in starts:
            if not direct:  # the views are written: each pass starts from the RX state
                m[s:s + B] = m0[s:s + B]
            d = Direct(mbufs=int(ptrs.ctypes.data) + 8 * s, lay=ctypes.addressof(lay), edges=edges.ctypes.data)
            t0 = time.perf_counter()
            r = L.gr_node_apply_ex(int(m.ctypes.data) + m.itemsize * s, B, 64, None,
                                   None if in_place else int(out32.ctypes.data) + abi.PREFIX * s, abi.PREFIX,
                                   int(v.ctypes.data) + v.itemsize * s, ifaces.ctypes.data, len(ifaces),
                                   nh.ctypes.data, len(nh), ns.ctypes.data if stats else None, vl.ctypes.data,
                                   st.ctypes.data if ifst else None, len(st),
                                   ctypes.addressof(d) if direct else None)
            t += time.perf_counter() - t0
            assert r == 0, r
        return t * 1e9 / (len(starts) * B)

    def stage_pass():
        t = 0.0
        for s in starts:
            t0 = time.perf_counter()
            r = L.gr_hip_node_stage(int(m.ctypes.data) + m.itemsize * s, B, 64, None, stage_lines.ctypes.data,
                                    stage_meta.ctypes.data)
            t += time.perf_counter() - t0
            assert r == 0, r
        return t * 1e9 / (len(starts) * B)

    variants = {"apply": (1, 1, True), "apply_no_iface_counters": (0, 1, True), "apply_no_counters": (0, 0, True),
                "apply_onto_views": (1, 1, False), "apply_frames_rewritten_by_gpu": (0, 1, True, True)}
    apply_pass(1, 1)  # warm-up: pages, code
    res = {k: [] for k in variants}
    res["stage"] = []
    for _ in range(args.reps):
        for k, a in variants.items():
            res[k].append(apply_pass(*a))
        res["stage"].append(stage_pass())
    fwd = float((v["edge"] == abi.EDGE["port_output"]).mean())
    print(json.dumps({"lib": os.path.relpath(abi.LIB_HIP, ROOT), "pkts": len(starts) * B, "batch": B,
                      "forwarded_frac": round(fwd, 4), "mbufs": f"{OBJ}-byte objects on THP",
                      "ns_per_pkt_median": {k: round(float(np.median(x)), 2) for k, x in res.items()},
                      "ns_per_pkt_all": {k: [round(y, 2) for y in x] for k, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
