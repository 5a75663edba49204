# SPDX-License-Identifier: BSD-3-Clause
"""ctypes view of the C ABI in include/grout_hip.h.

numpy dtypes mirror the C structs byte for byte (sizes are asserted against
the header's layout), so topology and packet arrays can be handed to the
library as plain pointers.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GR_LIBDIR: load the libraries from another build (`make asan-test`)
LIBDIR = os.environ.get("GR_LIBDIR") or HERE
LIB_HIP = os.path.join(LIBDIR, "libgrout_hip.so")
LIB_HOST = os.path.join(LIBDIR, "libgrout_host.so")

# ---------------------------------------------------------------------------
# constants (grout_hip.h)
# ---------------------------------------------------------------------------
IFACE_TYPE = dict(UNDEF=0, VRF=1, PORT=2, VLAN=3, IPIP=4, BOND=5, BRIDGE=6, VXLAN=7)
IFACE_MODE = dict(VRF=0, XC=1, BOND=2, BRIDGE=3)
IFACE_F_UP, IFACE_F_PROMISC, IFACE_F_PACKET_TRACE = 0x1, 0x2, 0x4
IFACE_F_SNAT_STATIC, IFACE_F_SNAT_DYNAMIC = 0x8, 0x10
NH_S = dict(NEW=0, PENDING=1, REACHABLE=2, STALE=3, FAILED=4)
NH_F_LOCAL, NH_F_GATEWAY, NH_F_LINK, NH_F_MCAST = 0x1, 0x2, 0x4, 0x8
NH_T = dict(L3=1, SR6_OUTPUT=2, SR6_LOCAL=3, DNAT=4, BLACKHOLE=5, REJECT=6, GROUP=7)
AF_UNSPEC, AF_IP4, AF_IP6 = 0, 1, 2
DOMAIN = dict(UNKNOWN=0, LOOPBACK=1, LOCAL=2, BROADCAST=3, MULTICAST=4, OTHER=5)
CKSUM_UNKNOWN, CKSUM_BAD, CKSUM_GOOD = 0, 1, 2
ABI_VERSION = 3  # GR_HIP_ABI_VERSION
EDGE_CHAIN = 0xFF
EDGE_CHAIN6 = 0xFE  # eth_input type edge: continue into ip6_input on the GPU
LINE = 64
BATCH_F_LINES_ONLY = 0x1
META_WALK = 0x4000  # gr_hip_pkt_meta.vlan_ck: this packet starts a graph walk
MBUF_F_WALK = 0x01  # gr_hip_mbuf.flags: this mbuf starts a graph walk

# enum gr_hip_edge, in order; names are the grout node each value stands for
EDGE_NAMES = [
    "punt",
    "iface_mode_unknown", "iface_input_admin_down", "iface_input_unknown_vlan",
    "xconnect", "bridge_input",
    "eth_input_unknown_type", "eth_input_invalid_iface", "snap_input",
    "arp_input", "ip6_input", "lacp_input",
    "ip_input_local", "ip_input_local_ct", "ip_error_dest_unreach",
    "ip_input_bad_checksum", "ip_input_bad_address", "ip_input_bad_length",
    "ip_input_bad_version", "ip_input_other_host", "ip_blackhole", "dnat44_static",
    "ip_error_ttl_exceeded",
    "ip_hold", "ip_output_error", "ip_fragment", "ip_error_frag_needed",
    "sr6_output", "xvrf", "ipip_output", "ip_output_snat",
    "eth_output_no_mac",
    "iface_output_inval_type", "iface_output_admin_down", "iface_output_vlan_no_parent",
    "bond_output", "vxlan_output", "port_output",
    "ip6_input_local", "ip6_error_dest_unreach", "ip6_input_not_member", "ip6_input_other_host",
    "ip6_input_bad_version", "ip6_input_bad_addr", "ip6_input_bad_length", "ip6_blackhole", "sr6_local",
    "ip6_error_ttl_exceeded",
    "ip6_hold", "ip6_output_error", "ip6_output_too_big",
]
EDGE = {n: i for i, n in enumerate(EDGE_NAMES)}
E_COUNT = len(EDGE_NAMES)

# ---------------------------------------------------------------------------
# struct layouts
# ---------------------------------------------------------------------------
IFACE_DT = np.dtype([
    ("id", "<u2"), ("type", "u1"), ("mode", "u1"), ("flags", "<u2"), ("mtu", "<u2"),
    ("vrf_id", "<u2"), ("port_id", "<u2"), ("vlan_id", "<u2"), ("parent_id", "<u2"),
    ("mac", "u1", (6,)), ("mac_ok", "u1"), ("_pad0", "u1"), ("_pad1", "<u4", (2,)),
])
NH_DT = np.dtype([
    ("type", "u1"), ("state", "u1"), ("flags", "u1"), ("af", "u1"),
    ("iface_id", "<u2"), ("vrf_id", "<u2"),
    ("ipv4", ">u4"),  # network byte order in memory
    ("mac", "u1", (6,)), ("reta_size", "<u2"), ("reta_off", "<u4"), ("single", "<u4"),
    ("n_members", "<u2"), ("_pad0", "<u2"), ("ipv6", "u1", (16,)),
])
ROUTE_DT = np.dtype([
    ("ip", ">u4"), ("prefixlen", "u1"), ("_pad0", "u1"), ("vrf_id", "<u2"), ("nh", "<u4"),
])
ROUTE6_DT = np.dtype([
    ("ip", "u1", (16,)), ("prefixlen", "u1"), ("_pad0", "u1"), ("vrf_id", "<u2"), ("iface_id", "<u2"),
    ("_pad1", "<u2"), ("nh", "<u4"),
])
META_DT = np.dtype([("iface", "<u2"), ("vlan_ck", "<u2"), ("pkt_len", "<u2"), ("rss", "<u2")])
VERDICT_DT = np.dtype([("edge", "u1"), ("domain", "u1"), ("iface", "<u2"), ("nh", "<u4")])
STATS_DT = np.dtype([
    ("rx_packets", "<u8"), ("rx_bytes", "<u8"), ("tx_packets", "<u8"), ("tx_bytes", "<u8"),
])
assert IFACE_DT.itemsize == 32 and NH_DT.itemsize == 48 and ROUTE_DT.itemsize == 12 and ROUTE6_DT.itemsize == 28
assert META_DT.itemsize == 8 and VERDICT_DT.itemsize == 8 and STATS_DT.itemsize == 32
# struct gr_hip_mbuf: the node shim's view of an rte_mbuf + priv (grout_hip.h)
MBUF_DT = np.dtype([("frame", "<u8"), ("pkt_len", "<u4"), ("data_len", "<u2"), ("data_off", "<u2"),
                    ("packet_type", "<u4"), ("rss", "<u4"), ("iface", "<u2"), ("vlan_id", "<u2"),
                    ("ck", "u1"), ("edge", "u1"), ("domain", "u1"), ("flags", "u1"), ("nh", "<u4"),
                    ("_pad1", "<u4")])
assert MBUF_DT.itemsize == 40
NODE_NAMES = ["iface_input", "eth_input", "ip_input", "ip_forward", "ip_output", "eth_output", "iface_output",
              "ip6_input", "ip6_forward", "ip6_output"]
NODE_COUNT = len(NODE_NAMES)
NODE_STATS_DT = np.dtype([("packets", "<u8", NODE_COUNT), ("calls", "<u8", NODE_COUNT)])
PTYPE_L3_IPV4, PTYPE_L3_IPV6 = 0x10, 0x40  # DPDK rte_mbuf_ptype.h
BATCH_F_FRAME_PTRS = 0x2
BATCH_F_PREFIX32 = 0x4  # out_lines: packed 32-byte prefixes (every byte the path changes)
PREFIX = 32
NODE_DEPTH = 4  # GR_HIP_NODE_DEPTH: node walks in flight per queue


class Batch(ctypes.Structure):
    _fields_ = [
        ("in_frames", ctypes.c_void_p), ("out_lines", ctypes.c_void_p),
        ("meta", ctypes.c_void_p), ("verdicts", ctypes.c_void_p),
        ("n", ctypes.c_uint32), ("in_stride", ctypes.c_uint32),
        ("out_stride", ctypes.c_uint32), ("flags", ctypes.c_uint32),
    ]


class SynthStream(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64), ("dst_mode", ctypes.c_uint32), ("size_mode", ctypes.c_uint32),
        ("dst_lo", ctypes.c_uint32), ("dst_hi", ctypes.c_uint32),
        ("routes", ctypes.c_void_p), ("n_routes", ctypes.c_uint32),
        ("in_iface", ctypes.c_uint16), ("dst_mac", ctypes.c_uint8 * 6),
        ("src_mac", ctypes.c_uint8 * 6), ("ttl", ctypes.c_uint8), ("_pad", ctypes.c_uint8),
    ]


# every entry point of include/grout_hip.h: name -> (restype, argtypes)
_P, _U8, _U16, _U32, _U64 = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64
_I = ctypes.c_int
PP = ctypes.POINTER(ctypes.c_void_p)
HIP_API = {
    "gr_hip_abi_version": (_I, []),
    "gr_hip_init": (_I, [_I, _U32, _U32, PP]),
    "gr_hip_fini": (_I, [_P]),
    "gr_hip_strerror": (ctypes.c_char_p, [_I]),
    "gr_hip_edges_eth_type": (_I, [_P, _U16, _U8]),
    "gr_hip_edges_iface_mode": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip_input_nh_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip_output_nh_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip_output_iface_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_iface_output_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip6_input_nh_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip6_output_nh_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_ip6_output_iface_type": (_I, [_P, _U8, _U8]),
    "gr_hip_edges_get": (_I, [_P, _I, _U16]),
    "gr_hip_device_count": (_I, []),
    "gr_hip_device_numa_node": (_I, [_I]),
    "gr_hip_iface_set": (_I, [_P, _P, _U32]),
    "gr_hip_iface_del": (_I, [_P, _U16]),
    "gr_hip_nh_set": (_I, [_P, _U32, _P, _U32]),
    "gr_hip_reta_set": (_I, [_P, _U32, _P, _U32]),
    "gr_hip_fib4_create": (_I, [_P, _U16, _U32, _U32]),
    "gr_hip_fib4_destroy": (_I, [_P, _U16]),
    "gr_hip_route4_add": (_I, [_P, _P, _U32, _I]),
    "gr_hip_route4_del": (_I, [_P, _U16, _U32, _U8]),
    "gr_hip_fib4_commit": (_I, [_P, _U16]),
    "gr_hip_fib4_lookup_host": (_I, [_P, _U16, _U32, ctypes.POINTER(_U32)]),
    "gr_hip_fib4_info": (_I, [_P, _U16, ctypes.POINTER(_U32), ctypes.POINTER(_U32), ctypes.POINTER(_U64)]),
    "gr_hip_fib6_create": (_I, [_P, _U16, _U32, _U32]),
    "gr_hip_fib6_destroy": (_I, [_P, _U16]),
    "gr_hip_route6_add": (_I, [_P, _P, _U32, _I]),
    "gr_hip_route6_del": (_I, [_P, _U16, _U16, _P, _U8]),
    "gr_hip_fib6_commit": (_I, [_P, _U16]),
    "gr_hip_fib6_lookup_host": (_I, [_P, _U16, _U16, _P, ctypes.POINTER(_U32)]),
    "gr_hip_fib6_info": (_I, [_P, _U16, ctypes.POINTER(_U32), ctypes.POINTER(_U32), ctypes.POINTER(_U64)]),
    "gr_hip_queue_create": (_I, [_P, _P, PP]),
    "gr_hip_queue_destroy": (_I, [_P]),
    "gr_hip_queue_stream": (_P, [_P]),
    "gr_hip_fwd4_submit": (_I, [_P, ctypes.POINTER(Batch)]),
    "gr_hip_queue_sync": (_I, [_P]),
    "gr_hip_queue_kernel_ms": (_I, [_P, _U32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_U32)]),
    "gr_hip_tune": (_I, [_P, ctypes.c_char_p, _I]),
    "gr_hip_fwd4_host": (_I, [_P, _P, _P, _U32, _P, _P]),
    "gr_hip_fwd4_host_ex": (_I, [_P, _P, _P, _U32, _P, _U32, _P]),
    "gr_hip_queue_stats": (_I, [_P, _P, _U32, _I]),
    "gr_hip_queue_stats_shards": (_I, [_P, _P, _U32, _I]),
    "gr_hip_host_alloc": (_I, [_P, ctypes.c_size_t, PP]),
    "gr_hip_host_free": (_I, [_P, _P]),
    "gr_hip_dev_alloc": (_I, [_P, ctypes.c_size_t, PP]),
    "gr_hip_dev_free": (_I, [_P, _P]),
    "gr_hip_batch_alloc": (_I, [_P, _U32, _U32, ctypes.POINTER(Batch)]),
    "gr_hip_batch_place": (_I, [_P, ctypes.POINTER(Batch), _U32]),
    "gr_hip_batch_free": (_I, [_P, ctypes.POINTER(Batch)]),
    "gr_hip_memcpy_h2d": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "gr_hip_memcpy_d2h": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "gr_hip_host_register": (_I, [_P, _P, ctypes.c_size_t]),
    "gr_hip_host_unregister": (_I, [_P, _P]),
    "gr_hip_host_dev_addr": (_I, [_P, _P, _P]),
    "gr_hip_edge_node": (_I, [_U8, _U32, _I]),
    "gr_hip_node_layout": (_I, [_P, _U32, _U32, _P]),
    "gr_hip_node_stage": (_I, [_P, _U32, _U32, _P, _P, _P]),
    "gr_hip_node_append": (_I, [_P, _P, _U32, _U32]),
    "gr_hip_node_append_mbufs": (_I, [_P, _P, _U32, _P, _U32]),
    "gr_hip_node_send": (_I, [_P, _P, _U32, _U32]),
    "gr_hip_node_discard": (_I, [_P]),
    "gr_hip_node_apply": (_I, [_P, _U32, _U32, _P, _P, _U32, _P, _P, _U32, _P, _U32, _P]),
    "gr_hip_node_process": (_I, [_P, _P, _U32, _U32, _P]),
    "gr_hip_node_start": (_I, [_P, _P, _U32, _U32]),
    "gr_hip_node_finish": (_I, [_P, _P, _P, _P]),
    "gr_hip_node_finish_mbufs": (_I, [_P, _P, _P, _P, _P, _P]),
    "gr_hip_node_pending": (_I, [_P, _P]),
    "gr_hip_node_iface_stats": (_I, [_P, _P, _U32, _I]),
    "gr_hip_node_prof": (_I, [_P, _U32, _I]),
}

HOST_API = {
    "gr_synth_splitmix64": (_U64, [ctypes.POINTER(_U64)]),
    "gr_synth_fullview_routes": (_I, [_U32, _U16, _U32, _U32, _P]),
    "gr_synth_fullview6_routes": (_I, [_U32, _U16, _U32, _U32, _P]),
    "gr_synth_packets": (_I, [ctypes.POINTER(SynthStream), _U32, _U32, _I, _P, _P]),
    "gr_synth_ip4_cksum": (_U16, [_P, _U32]),
    "gr_fib4_new": (_P, [_U32, _U32]),
    "gr_fib4_free": (None, [_P]),
    "gr_fib4_add": (_I, [_P, _U32, _U8, _U32, _I]),
    "gr_fib4_del": (_I, [_P, _U32, _U8]),
    "gr_fib4_lookup": (_U32, [_P, _U32]),
    "gr_fib4_get": (_U32, [_P, _U32, _U8]),
    "gr_fib4_tbl24": (_P, [_P]),
    "gr_fib4_tbl8": (_P, [_P]),
    "gr_fib4_num_tbl8": (_U32, [_P]),
    "gr_fib4_tbl8_used": (_U32, [_P]),
    "gr_fib4_n_routes": (_U32, [_P]),
    "gr_fib6_new": (_P, [_U32, _U32]),
    "gr_fib6_free": (None, [_P]),
    "gr_fib6_add": (_I, [_P, _P, _U8, _U32, _I]),
    "gr_fib6_del": (_I, [_P, _P, _U8]),
    "gr_fib6_build": (_I, [_P]),
    "gr_fib6_lookup": (_U32, [_P, _P]),
    "gr_fib6_lookup_rib": (_U32, [_P, _P]),
    "gr_fib6_groups_used": (_U32, [_P]),
    "gr_fib6_skips_used": (_U32, [_P]),
    "gr_fib6_groups_painted": (_U32, [_P]),
    "gr_fib6_n_routes": (_U32, [_P]),
    "gr_fib6_groups_live": (_U32, [_P]),
    "gr_fib6_dirty": (_I, [_P, _I, ctypes.POINTER(_P), ctypes.POINTER(_U32)]),
    "gr_fib6_dirty_clear": (None, [_P]),
    "gr_fib6_top": (_P, [_P]),
    "gr_fib6_groups": (_P, [_P]),
    "gr_fib6_skips": (_P, [_P]),
}


def _bind(path, api, what):
    if not os.path.exists(path):
        raise ImportError(f"{what} not built: {path} missing (run `make` or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    # GR_HIP_AB_OLD=1: an older build under A/B (tools/ab_libs.sh) may lack
    # the newest entry points; everything else binds every symbol or fails
    lenient = os.environ.get("GR_HIP_AB_OLD") == "1"
    for name, (res, args) in api.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_hip = None
_host = None


def hip():
    """The HIP fast-path library. Raises if it is not built: no fallback.

    When PyTorch is importable it is imported first: its bundled HIP runtime
    carries the same SONAME (libamdhip64.so.7) as /opt/rocm's, so the library
    then binds to it and the process runs ONE HIP runtime, whose device
    pointers and streams torch tensors also use. Without torch the library
    uses /opt/rocm/lib/libamdhip64.so.7 directly.
    """
    global _hip
    if _hip is None:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _hip = _bind(LIB_HIP, HIP_API, "HIP extension libgrout_hip.so")
    return _hip


def host():
    """Host-only helpers (RIB/FIB builder, synthetic generators)."""
    global _host
    if _host is None:
        _host = _bind(LIB_HOST, HOST_API, "host library libgrout_host.so")
    return _host


def ptr(a):
    """Raw address of a numpy array, a torch tensor or an int."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch.Tensor


class GrHipError(RuntimeError):
    def __init__(self, fn, ret):
        msg = os.strerror(-ret) if ret < 0 else str(ret)
        super().__init__(f"{fn} failed: {ret} ({msg})")
        self.ret = ret


def check(fn, ret):
    if ret < 0:
        raise GrHipError(fn, ret)
    return ret
