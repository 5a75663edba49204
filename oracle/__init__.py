# SPDX-License-Identifier: BSD-3-Clause
"""TEST INFRASTRUCTURE ONLY: ctypes binding of the oracle (see oracle.h).

A CPU restatement of grout's IPv4 forwarding node chain, used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker and the
CPU baseline. The product (grout_amd/) never imports this package.
"""
import ctypes
import os

import numpy as np

from grout_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.environ.get("GR_LIBDIR") or HERE, "liboracle.so")  # GR_LIBDIR: `make asan-test`

_P, _U8, _U16, _U32, _U64, _I = (ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32,
                                 ctypes.c_uint64, ctypes.c_int)
API = {
    "or_topo_new": (_P, [_U32, _U32]),
    "or_topo_free": (None, [_P]),
    "or_edge_eth_type": (_I, [_P, _U16, _U8]),
    "or_edge_iface_mode": (_I, [_P, _U8, _U8]),
    "or_edge_ip_input_nh_type": (_I, [_P, _U8, _U8]),
    "or_edge_ip_output_nh_type": (_I, [_P, _U8, _U8]),
    "or_edge_ip_output_iface_type": (_I, [_P, _U8, _U8]),
    "or_edge_iface_output_type": (_I, [_P, _U8, _U8]),
    "or_iface_set": (_I, [_P, _P, _U32]),
    "or_nh_set": (_I, [_P, _U32, _P, _U32]),
    "or_reta_set": (_I, [_P, _U32, _P, _U32]),
    "or_fib_create": (_I, [_P, _U16, _U32]),
    "or_route_add": (_I, [_P, _P, _U32, _I]),
    "or_route_del": (_I, [_P, _U16, _U32, _U8]),
    "or_fib_build": (_I, [_P, _U16]),
    "or_lpm_hash": (_U32, [_P, _U16, _U32]),
    "or_lpm_dir24": (_U32, [_P, _U16, _U32]),
    "or_lpm_brute": (_U32, [_P, _U16, _U32]),
    "or_edge_ip6_input_nh_type": (_I, [_P, _U8, _U8]),
    "or_edge_ip6_output_nh_type": (_I, [_P, _U8, _U8]),
    "or_edge_ip6_output_iface_type": (_I, [_P, _U8, _U8]),
    "or_fib6_create": (_I, [_P, _U16]),
    "or_route6_add": (_I, [_P, _P, _U32, _I]),
    "or_route6_del": (_I, [_P, _U16, _U16, _P, _U8]),
    "or_lpm6": (_U32, [_P, _U16, _U16, _P]),
    "or_lpm6_brute": (_U32, [_P, _U16, _U16, _P]),
    "or_process": (_I, [_P, _P, _U32, _P, _U32, _P, _U32, _P, _P, _U32]),
    "or_process_ex": (_I, [_P, _P, _U32, _P, _U32, _P, _U32, _P, _P, _U32, _P, _P]),
    "or_bench": (ctypes.c_double, [_P, _P, _U32, _P, _U32, _I, _U64, _U32, ctypes.POINTER(_U64)]),
}

OR_F_MBUF_WALKS = 0x80000000  # oracle.h

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"oracle not built: {LIB} (run make)")
        _lib = ctypes.CDLL(LIB)
        for k, (r, a) in API.items():
            f = getattr(_lib, k)
            f.restype = r
            f.argtypes = a
    return _lib


def _ck(fn, r):
    if r < 0:
        raise RuntimeError(f"{fn}: {r} ({os.strerror(-r)})")
    return r


class Oracle:
    """The restated grout node chain over a Topology."""

    def __init__(self, topo, build_dir24=True):
        L = lib()
        self.L = L
        self.max_ifaces = topo.max_ifaces
        self.h = L.or_topo_new(topo.max_ifaces, topo.max_nexthops)
        if not self.h:
            raise MemoryError("or_topo_new")
        live = np.ascontiguousarray(topo.ifaces[topo.ifaces["id"] != 0])
        _ck("or_iface_set", L.or_iface_set(self.h, live.ctypes.data, len(live)))
        if topo.n_nh:
            nh = np.ascontiguousarray(topo.nh[1:topo.n_nh + 1])
            _ck("or_nh_set", L.or_nh_set(self.h, 1, nh.ctypes.data, len(nh)))
        if len(topo.reta):
            r = np.ascontiguousarray(topo.reta, dtype=np.uint32)
            _ck("or_reta_set", L.or_reta_set(self.h, 0, r.ctypes.data, len(r)))
        for vrf_id, (_mr, num_tbl8) in topo.fibs.items():
            ntbl8 = num_tbl8 or max(256, _mr // 500)
            _ck("or_fib_create", L.or_fib_create(self.h, vrf_id, ntbl8))
        routes = topo.route_array()
        if len(routes):
            _ck("or_route_add", L.or_route_add(self.h, routes.ctypes.data, len(routes), 0))
        for vrf_id in getattr(topo, "fibs6", {}):
            _ck("or_fib6_create", L.or_fib6_create(self.h, vrf_id))
        routes6 = topo.route6_array() if hasattr(topo, "route6_array") else []
        if len(routes6):
            _ck("or_route6_add", L.or_route6_add(self.h, routes6.ctypes.data, len(routes6), 0))
        if build_dir24:
            for vrf_id in topo.fibs:
                _ck("or_fib_build", L.or_fib_build(self.h, vrf_id))

    def close(self):
        if self.h:
            self.L.or_topo_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def edge(self, kind, key, edge):
        fn = {"eth_type": "or_edge_eth_type", "iface_mode": "or_edge_iface_mode",
              "ip_input_nh_type": "or_edge_ip_input_nh_type",
              "ip_output_nh_type": "or_edge_ip_output_nh_type",
              "ip_output_iface_type": "or_edge_ip_output_iface_type",
              "iface_output_type": "or_edge_iface_output_type",
              "ip6_input_nh_type": "or_edge_ip6_input_nh_type",
              "ip6_output_nh_type": "or_edge_ip6_output_nh_type",
              "ip6_output_iface_type": "or_edge_ip6_output_iface_type"}[kind]
        _ck(fn, getattr(self.L, fn)(self.h, key, edge))

    def lpm(self, vrf_id, ip_host, how="hash"):
        return getattr(self.L, "or_lpm_" + how)(self.h, vrf_id, ip_host)

    def lpm6(self, vrf_id, ip16, iface_id=0, brute=False):
        a = np.frombuffer(bytes(ip16), np.uint8).copy()
        fn = self.L.or_lpm6_brute if brute else self.L.or_lpm6
        return fn(self.h, vrf_id, iface_id, a.ctypes.data)

    def process(self, frames, meta, lines_only=False, stats=None):
        """-> (out_lines n x 64, verdicts)."""
        frames = np.ascontiguousarray(frames)
        meta = np.ascontiguousarray(meta, dtype=abi.META_DT)
        n = len(meta)
        stride = frames.shape[1] if frames.ndim == 2 else frames.itemsize
        out = np.zeros((n, abi.LINE), dtype=np.uint8)
        v = np.zeros(n, dtype=abi.VERDICT_DT)
        st = stats if stats is not None else np.zeros(self.max_ifaces, dtype=abi.STATS_DT)
        _ck("or_process", self.L.or_process(self.h, frames.ctypes.data, stride, meta.ctypes.data, n,
                                            out.ctypes.data, abi.LINE, v.ctypes.data, st.ctypes.data,
                                            abi.BATCH_F_LINES_ONLY if lines_only else 0))
        return out, v, st

    def process_mbufs(self, frames, meta, lines_only=False, burst=64):
        """-> (out_lines, verdicts, stats, mbufs, node_stats): process() plus
        the mbuf state at each edge (abi.MBUF_DT, RX data_off 128) and the
        per-node counters. Graph walks as the rte_graph node cuts mbufs
        (OR_F_MBUF_WALKS): at each abi.META_WALK mark and `burst` (1..256)
        packets after the previous start."""
        if not 1 <= burst <= 256:
            raise ValueError("burst")
        frames = np.ascontiguousarray(frames)
        meta = np.ascontiguousarray(meta, dtype=abi.META_DT)
        n = len(meta)
        stride = frames.shape[1] if frames.ndim == 2 else frames.itemsize
        out = np.zeros((n, abi.LINE), dtype=np.uint8)
        v = np.zeros(n, dtype=abi.VERDICT_DT)
        st = np.zeros(self.max_ifaces, dtype=abi.STATS_DT)
        mb = np.zeros(n, dtype=abi.MBUF_DT)
        ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
        _ck("or_process_ex", self.L.or_process_ex(self.h, frames.ctypes.data, stride, meta.ctypes.data, n,
                                                  out.ctypes.data, abi.LINE, v.ctypes.data, st.ctypes.data,
                                                  (abi.BATCH_F_LINES_ONLY if lines_only else 0) | OR_F_MBUF_WALKS
                                                  | ((burst & 0x1FF) << 16),
                                                  mb.ctypes.data,
                                                  ns.ctypes.data))
        return out, v, st, mb, ns[0]

    def bench(self, frames, meta, threads, pkts_per_thread, fib_copy=True, cpus=None):
        """or_bench (oracle.h): aggregate Mpps of `threads` pinned workers after
        a warm-up pass each; fib_copy: each its own IPv4 FIB copy on THP;
        cpus: worker i on cpus[i] (default: the i-th CPU the process may use)."""
        fwd = ctypes.c_uint64()
        stride = frames.shape[1]
        c = list(cpus or [])
        arr = (ctypes.c_int * max(1, len(c)))(*c)
        if self.L.or_bench_set_cpus(arr, len(c)) != 0:
            raise ValueError(f"or_bench_set_cpus {c}")
        mpps = self.L.or_bench(self.h, frames.ctypes.data, stride, meta.ctypes.data, len(meta), threads,
                               pkts_per_thread, 1 if fib_copy else 0, ctypes.byref(fwd))
        if mpps < 0:
            raise MemoryError("or_bench")
        return mpps, fwd.value
