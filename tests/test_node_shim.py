# SPDX-License-Identifier: BSD-3-Clause
"""The rte_graph node shim (include/grout_hip.h):
staging mbufs into header lines and handing verdicts back onto mbufs, and
the per-node counters, against the oracle's mbuf-level restatement of the
chain (oracle.c: data_off / data_len / pkt_len through eth_input's adj and
eth_output's prepend, packet_type, vlan_id, priv iface / domain / nexthop).

CPU tests feed the oracle's own lines and verdicts to gr_hip_node_apply (a
pure host function of libgrout_hip.so); the GPU test runs the whole node
walk (gr_hip_node_process: stage, forward on the GPU, apply)."""
import ctypes

import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

RX_DATA_OFF = 128  # RTE_PKTMBUF_HEADROOM


def mbufs_for(frames, meta, data_room=2048):
    """Host 'mbufs': each frame copied into its own buffer, views at RX."""
    n = len(meta)
    stride = frames.shape[1]
    bufs = np.zeros((n, max(stride, abi.LINE)), dtype=np.uint8)
    bufs[:, :stride] = frames
    m = np.zeros(n, dtype=abi.MBUF_DT)
    m["frame"] = bufs.ctypes.data + np.arange(n, dtype=np.uint64) * bufs.shape[1]
    m["pkt_len"] = meta["pkt_len"]
    m["data_len"] = meta["pkt_len"]
    m["data_off"] = RX_DATA_OFF
    m["rss"] = meta["rss"]
    m["iface"] = meta["iface"]
    m["vlan_id"] = meta["vlan_ck"] & 0xfff
    m["ck"] = (meta["vlan_ck"] >> 12) & 3
    return bufs, m


def apply(m, lines, v, topo, burst=64):
    ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
    L = abi.hip()
    ifaces = np.ascontiguousarray(topo.ifaces)
    nh = np.ascontiguousarray(topo.nh)
    abi.check("gr_hip_node_apply", L.gr_hip_node_apply(
        m.ctypes.data, len(m), burst, None, np.ascontiguousarray(lines).ctypes.data, abi.LINE, v.ctypes.data,
        ifaces.ctypes.data, len(ifaces), nh.ctypes.data, len(nh), ns.ctypes.data))
    return ns[0]


FIELDS = ["pkt_len", "data_len", "data_off", "packet_type", "iface", "vlan_id", "edge", "domain", "nh"]


def compare_mbufs(got, want, frames_after, lines_want, labels=None):
    for f in FIELDS:
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, (f, [((labels[i] if labels else i), int(got[f][i]), int(want[f][i]),
                                    abi.EDGE_NAMES[want["edge"][i]]) for i in bad[:6]])
    # the frame ends as the oracle's line: grout's rewrite at that edge
    n = len(got)
    bad = np.nonzero((frames_after[:, :abi.LINE] != lines_want).any(axis=1))[0]
    assert len(bad) == 0, [(labels[i] if labels else i) for i in bad[:6]]
    assert n == len(want)


def test_edge_node_table():
    """Every verdict edge maps to the node that chose it."""
    L = abi.hip()
    N = {n: i for i, n in enumerate(abi.NODE_NAMES)}
    node_of = {e: L.gr_hip_edge_node(i, 0, 0) for i, e in enumerate(abi.EDGE_NAMES)}
    assert node_of["punt"] == -1
    assert node_of["port_output"] == node_of["iface_output_admin_down"] == N["iface_output"]
    assert node_of["ip_hold"] == node_of["ip_output_snat"] == N["ip_output"]
    assert node_of["ip_error_ttl_exceeded"] == N["ip_forward"]
    assert node_of["ip_error_dest_unreach"] == node_of["ip_input_local"] == N["ip_input"]
    assert node_of["snap_input"] == node_of["arp_input"] == node_of["ip6_input"] == N["eth_input"]
    assert node_of["iface_input_admin_down"] == node_of["bridge_input"] == N["iface_input"]
    assert node_of["ip6_input_bad_addr"] == node_of["ip6_error_dest_unreach"] == node_of["sr6_local"] == N["ip6_input"]
    assert node_of["ip6_error_ttl_exceeded"] == N["ip6_forward"]
    assert node_of["ip6_hold"] == node_of["ip6_output_too_big"] == N["ip6_output"]
    # edges two nodes share: the nexthop / the address family tell them apart
    assert L.gr_hip_edge_node(abi.EDGE["bridge_input"], 7, 0) == N["iface_output"]
    assert L.gr_hip_edge_node(abi.EDGE["xvrf"], 7, 0) == N["ip_output"]
    assert L.gr_hip_edge_node(abi.EDGE["xvrf"], 7, 1) == N["ip6_output"]
    assert L.gr_hip_edge_node(abi.EDGE["sr6_output"], 7, 1) == N["ip6_output"]
    assert all(v >= -1 for v in node_of.values())
    assert L.gr_hip_edge_node(abi.E_COUNT, 0, 0) < -1


def test_stage_roundtrip():
    fr, me, _ = SC.corpus_arrays()
    bufs, m = mbufs_for(fr, me)
    lines = np.zeros((len(me), abi.LINE), dtype=np.uint8)
    meta = np.zeros(len(me), dtype=abi.META_DT)
    abi.check("gr_hip_node_stage", abi.hip().gr_hip_node_stage(m.ctypes.data, len(m), 64, None, lines.ctypes.data,
                                                               meta.ctypes.data))
    walk = (meta["vlan_ck"] & abi.META_WALK) != 0
    assert np.array_equal(np.nonzero(walk)[0], np.arange(0, len(me), 64))  # graph walks of 64
    meta["vlan_ck"] &= 0xFFFF ^ abi.META_WALK
    assert np.array_equal(meta, me)
    assert np.array_equal(lines, fr[:, :abi.LINE])  # 64 bytes whatever data_len says


def test_apply_corpus_matches_oracle_mbufs():
    """Every edge of the exception corpus: the hand-back leaves each mbuf as
    grout's chain does at that edge, and the node counters match."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    lines, v, _, want, ns_want = oracle.Oracle(t).process_mbufs(fr, me)
    bufs, m = mbufs_for(fr, me)
    ns = apply(m, lines, v, t)
    compare_mbufs(m, want, bufs, lines, lab)
    assert np.array_equal(ns["packets"], ns_want["packets"]), (ns, ns_want)
    assert np.array_equal(ns["calls"], ns_want["calls"]), (ns, ns_want)
    edges = set(abi.EDGE_NAMES[e] for e in v["edge"])
    assert {"port_output", "ip_hold", "ip_error_ttl_exceeded", "eth_output_no_mac", "snap_input",
            "iface_input_unknown_vlan", "ip_input_bad_checksum", "ip6_hold", "ip6_output_too_big",
            "ip6_error_ttl_exceeded", "ip6_input_bad_addr", "xvrf"} <= edges
    six = (m["packet_type"] == abi.PTYPE_L3_IPV6)
    assert six.sum() > 10 and (m["packet_type"][six] == want["packet_type"][six]).all()


@pytest.mark.parametrize("burst", [1, 7, 64, 128, 256])
def test_node_stats_bursts(burst):
    """Per-node packets / calls follow grout's rule for any walk size up to
    grout's maximum (rx_burst_max / vector_max <= 256, graph.c:612-650): the
    oracle walks the same bursts."""
    t, _ = SC.corpus_topology()
    fr, me, _ = SC.corpus_arrays()
    lines, v, _, want, ns_b = oracle.Oracle(t).process_mbufs(fr, me, burst=burst)
    lines64, _, _, _, ns64 = oracle.Oracle(t).process_mbufs(fr, me)
    bufs, m = mbufs_for(fr, me)
    ns = apply(m, lines, v, t, burst=burst)
    compare_mbufs(m, want, bufs, lines)
    assert np.array_equal(ns["packets"], ns_b["packets"]) and np.array_equal(ns["calls"], ns_b["calls"])
    # packets do not depend on the walk size, calls do
    assert np.array_equal(ns["packets"], ns64["packets"])
    n_walks = -(-len(me) // burst)
    assert (ns["calls"] <= n_walks).all()
    # ip_output / ip6_output return what they sent to eth_output
    N = {n: i for i, n in enumerate(abi.NODE_NAMES)}
    assert ns["packets"][N["ip_output"]] + ns["packets"][N["ip6_output"]] == ns["packets"][N["eth_output"]]


def _vlan_table(topo):
    """The host image of the context's VLAN table (gr_hip.cpp upload_vlans)."""
    ifs = topo.ifaces[(topo.ifaces["id"] != 0) & (topo.ifaces["type"] == abi.IFACE_TYPE["VLAN"])]
    cap = 16
    while cap < 2 * len(ifs):
        cap *= 2
    keys = np.zeros(cap, dtype=np.uint32)
    vals = np.zeros(cap, dtype=np.uint16)
    for i in ifs:
        key = ((int(i["parent_id"]) << 16) | int(i["vlan_id"])) + 1
        h = (key * 0x9E3779B1) & 0xFFFFFFFF & (cap - 1)
        while keys[h] not in (0, key):
            h = (h + 1) & (cap - 1)
        keys[h], vals[h] = key, i["id"]
    return keys, vals


def apply_counting(m, lines, v, topo, burst=64, direct=None, pos=None):
    """gr_node_apply_ex: the hand-back plus the per-iface counters grout's
    iface_input / iface_output would have added (what the node folds into
    grout's iface_stats)."""
    import ctypes
    L = ctypes.CDLL(abi.LIB_HIP)
    keys, vals = _vlan_table(topo)
    vl = (ctypes.c_void_p * 2)(keys.ctypes.data, vals.ctypes.data)
    vl_buf = np.zeros(3, dtype=np.uint64)  # struct gr_node_vlans {keys, vals, cap}
    vl_buf[0], vl_buf[1], vl_buf[2] = vl[0], vl[1], len(keys)
    st = np.zeros(topo.max_ifaces, dtype=abi.STATS_DT)
    ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
    ifaces = np.ascontiguousarray(topo.ifaces)
    nh = np.ascontiguousarray(topo.nh)
    lines = np.ascontiguousarray(lines)
    P, U32 = ctypes.c_void_p, ctypes.c_uint32
    L.gr_node_apply_ex.argtypes = [P, U32, U32, P, P, U32, P, P, U32, P, U32, P, P, P, U32, P]
    n = len(v)
    abi.check("gr_node_apply_ex", L.gr_node_apply_ex(
        None if m is None else m.ctypes.data, n, burst, None if pos is None else pos.ctypes.data,
        lines.ctypes.data, abi.LINE, v.ctypes.data, ifaces.ctypes.data,
        len(ifaces), nh.ctypes.data, len(nh), ns.ctypes.data, vl_buf.ctypes.data, st.ctypes.data, len(st), direct))
    return ns[0], st


_LAYOUT_U16 = ("data_off", "data_len", "pkt_len", "packet_type", "priv", "priv_iface", "priv_vlan_id", "priv_domain",
               "priv_eth_nh", "priv_l3_nh")


class Layout(ctypes.Structure):
    """struct gr_hip_mbuf_layout (include/grout_hip.h)"""
    _fields_ = [(k, ctypes.c_uint16) for k in _LAYOUT_U16] + [
        ("n_ifaces", ctypes.c_uint32), ("n_nh", ctypes.c_uint32), ("ifaces", ctypes.c_void_p), ("nh", ctypes.c_void_p),
        ("buf_addr", ctypes.c_uint16), ("ol_flags", ctypes.c_uint16), ("rss", ctypes.c_uint16),
        ("iface_id", ctypes.c_uint16), ("ck_mask", ctypes.c_uint64), ("ck_good", ctypes.c_uint64),
        ("ck_bad", ctypes.c_uint64)]


class Direct(ctypes.Structure):
    """struct gr_node_direct (grout_amd/csrc/gr_node_priv.h)"""
    _fields_ = [("mbufs", ctypes.c_void_p), ("lay", ctypes.c_void_p), ("edges", ctypes.c_void_p),
                ("stale", ctypes.c_uint32), ("meta", ctypes.c_void_p)]


# grout's rte_mbuf and private-data offsets (DPDK rte_mbuf_core.h; mbuf.h:29-41,
# rxtx.h:45-48, eth.h:23-36, l3.h:9)
GROUT_LAYOUT = dict(data_off=16, data_len=40, pkt_len=36, packet_type=32, priv=128, priv_iface=16, priv_vlan_id=24,
                    priv_domain=24, priv_eth_nh=32, priv_l3_nh=24)
IF_OBJ, NH_OBJ = 0x7F0000001000, 0x7F0000100000  # registry "pointers": base + id
# what the staging reads: rte_mbuf buf_addr, ol_flags, hash.rss (rte_mbuf_core.h)
# and RTE_MBUF_F_RX_IP_CKSUM_MASK / _GOOD / _BAD; iface_id: where the fake iface
# objects below keep their id
GROUT_STAGE = dict(buf_addr=0, ol_flags=24, rss=44, iface_id=8, ck_mask=(1 << 4) | (1 << 7), ck_good=1 << 7,
                   ck_bad=1 << 4)


def test_apply_onto_mbufs_equals_views():
    """The one-pass hand-back (gr_hip_node_finish_mbufs' apply): each mbuf's
    own fields and private data, written through a layout descriptor and the
    caller's registries, are what the view-based hand-back gives its view,
    with grout's private data for the node behind each edge; the views are
    only read; a packet whose nexthop left the registry keeps its mbuf and
    goes to ip_output_error, counted."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    lines, v, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me)
    bufs, m_view = mbufs_for(fr, me)
    ns_view, st_view = apply_counting(m_view, lines, v, t)  # the reference: onto the views
    bufs2, m = mbufs_for(fr, me)
    m0 = m.copy()
    n = len(m)
    mem = np.zeros((n, 256), dtype=np.uint8)  # rte_mbuf (128) + private area (64) + spare
    mem[:, 254:256] = 0xA5  # untouched guard
    L = GROUT_LAYOUT
    mem.view(np.uint16)[:, L["data_off"] // 2] = m0["data_off"]
    mem.view(np.uint16)[:, L["data_len"] // 2] = m0["data_len"]
    mem.view(np.uint32)[:, L["pkt_len"] // 4] = m0["pkt_len"]
    ptrs = (mem.ctypes.data + np.arange(n, dtype=np.uint64) * 256).astype(np.uint64)
    reg_if = np.zeros(t.max_ifaces, dtype=np.uint64)
    live = t.ifaces["id"] != 0
    reg_if[live] = IF_OBJ + np.nonzero(live)[0]
    reg_nh = (NH_OBJ + np.arange(len(t.nh), dtype=np.uint64)).astype(np.uint64)
    gone = int(np.bincount(v["nh"][v["edge"] == abi.EDGE["ip_hold"]]).argmax())  # a nexthop ip_hold names
    reg_nh[gone] = 0
    reg_nh[0] = 0
    lay = Layout(**L, n_ifaces=len(reg_if), n_nh=len(reg_nh), ifaces=reg_if.ctypes.data, nh=reg_nh.ctypes.data)
    edges = np.full(n, 0xEE, dtype=np.uint8)
    d = Direct(mbufs=ptrs.ctypes.data, lay=ctypes.addressof(lay), edges=edges.ctypes.data)
    ns_d, st_d = apply_counting(m, lines, v, t, direct=ctypes.addressof(d))
    assert np.array_equal(m, m0)  # the views: read only
    # the same per-node and per-iface counters (port_output_fast counts as the general loop)
    assert np.array_equal(ns_d, ns_view) and np.array_equal(st_d, st_view)
    assert (v["edge"] == abi.EDGE["port_output"]).sum() > 20
    U16, U32, U64 = mem.view(np.uint16), mem.view(np.uint32), mem.view(np.uint64)
    N = {k: i for i, k in enumerate(abi.NODE_NAMES)}
    six = (lines[:, 12] == 0x86) & (lines[:, 13] == 0xDD)
    node = np.array([abi.hip().gr_hip_edge_node(int(e), int(h), int(x)) for e, h, x in zip(v["edge"], v["nh"], six)])
    punt = v["edge"] == abi.EDGE["punt"]
    stale = ~punt & (v["nh"] == gone) & ~np.isin(node, [N["iface_input"], N["iface_output"]])
    assert stale.sum() > 0 and d.stale == stale.sum()
    assert (edges[stale] == abi.EDGE["ip_output_error"]).all()
    assert np.array_equal(edges[~stale], v["edge"][~stale])
    keep = punt | stale  # mbufs as port_rx left them
    assert (U16[keep, L["data_off"] // 2] == RX_DATA_OFF).all() and (mem[keep, 128:192] == 0).all()
    ok = ~keep
    assert np.array_equal(U16[ok, L["data_off"] // 2], m_view["data_off"][ok])
    assert np.array_equal(U16[ok, L["data_len"] // 2], m_view["data_len"][ok])
    assert np.array_equal(U32[ok, L["pkt_len"] // 4], m_view["pkt_len"][ok])
    assert np.array_equal(U32[ok, L["packet_type"] // 4], m_view["packet_type"][ok])
    priv = mem[:, 128:192]
    pv16, pv32, pv64 = priv.copy().view(np.uint16), priv.copy().view(np.uint32), priv.copy().view(np.uint64)
    want_if = np.where(m_view["iface"] != 0, IF_OBJ + m_view["iface"].astype(np.uint64), 0)
    assert np.array_equal(pv64[ok, 2], want_if[ok])  # mbuf_data.iface
    vl = ok & np.isin(node, [N["iface_input"], N["iface_output"]])
    assert np.array_equal(pv16[vl, 12], m_view["vlan_id"][vl])
    l3 = ok & ~vl & (m_view["nh"] != 0)
    assert np.array_equal(pv64[l3, 3], NH_OBJ + m_view["nh"][l3].astype(np.uint64))
    eo = node == N["eth_output"]
    dom = ok & ~vl & ~eo & (m_view["nh"] == 0)
    assert np.array_equal(pv32[dom, 6], m_view["domain"][dom].astype(np.uint32))
    assert (pv64[ok & ~vl & ~eo, 4] == 0).all()  # eth_input_mbuf_data.nh: NULL
    assert (mem[:, 254:256] == 0xA5).all()
    # frames: rewritten as the view-based hand-back rewrote them
    assert np.array_equal(bufs2[ok][:, :abi.LINE], bufs[ok][:, :abi.LINE])


def test_stage_from_mbufs_equals_views():
    """gr_hip_node_append_mbufs' one pass (gr_node_stage_mbufs): reading
    grout's rte_mbufs through the layout (frame at buf_addr + data_off,
    pkt_len, rss, the iface id through mbuf_data.iface, vlan_id, the checksum
    status from ol_flags) gives the same placement (walks cut at the burst,
    pads before a walk that would straddle a tile) and the same staged lines
    and metadata as gr_hip_node_layout + gr_hip_node_stage on the views the
    grout node used to build, over appends of 1 to 300 mbufs."""
    t, _ = SC.corpus_topology()
    fr, me, _ = SC.corpus_arrays()
    keep = ((me["vlan_ck"] >> 12) & 3) != 3  # no ol_flags value gives the corpus's status 3
    fr, me = np.concatenate([fr[keep]] * 8), np.concatenate([me[keep]] * 8)
    n = len(me)
    rng = np.random.default_rng(7)
    bufs, ref = mbufs_for(fr, me)
    ref["packet_type"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ref["rss"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    L, G = GROUT_LAYOUT, GROUT_STAGE
    mem = np.zeros((n, 256), dtype=np.uint8)
    U16, U32, U64 = mem.view(np.uint16), mem.view(np.uint32), mem.view(np.uint64)
    U64[:, G["buf_addr"] // 8] = ref["frame"] - RX_DATA_OFF
    U16[:, L["data_off"] // 2] = RX_DATA_OFF
    U16[:, L["data_len"] // 2] = ref["data_len"]
    U32[:, L["pkt_len"] // 4] = ref["pkt_len"]
    U32[:, L["packet_type"] // 4] = ref["packet_type"]
    U32[:, G["rss"] // 4] = ref["rss"]
    ck_bits = np.array([0, G["ck_bad"], G["ck_good"]], dtype=np.uint64)
    U64[:, G["ol_flags"] // 8] = ck_bits[ref["ck"]] | np.uint64(1 << 40)  # other flags set too
    ifobj = np.zeros((t.max_ifaces, 64), dtype=np.uint8)
    ifobj.view(np.uint16)[:, G["iface_id"] // 2] = np.arange(t.max_ifaces)
    ifp = np.where(ref["iface"] != 0, ifobj.ctypes.data + 64 * ref["iface"].astype(np.uint64), 0).astype(np.uint64)
    U64[:, (L["priv"] + L["priv_iface"]) // 8] = ifp
    U16[:, (L["priv"] + L["priv_vlan_id"]) // 2] = ref["vlan_id"]
    ptrs = (mem.ctypes.data + np.arange(n, dtype=np.uint64) * 256).astype(np.uint64)
    lay = Layout(**L, **G, n_ifaces=0, n_nh=0, ifaces=None, nh=None)
    # appends of 1 .. 300 mbufs; burst 256 cuts the longer ones
    sizes, i = [], 0
    while i < n:
        k = int(min(n - i, rng.choice([1, 3, 7, 40, 64, 65, 100, 256, 300])))
        sizes.append((i, k))
        i += k
    ref["flags"] = 0
    for i, k in sizes:
        ref["flags"][i] = abi.MBUF_F_WALK
    H = abi.hip()
    pos_ref = np.zeros(n, dtype=np.uint32)
    end = H.gr_hip_node_layout(ref.ctypes.data, n, 256, pos_ref.ctypes.data)
    assert end > n  # pads were needed
    lines_ref = np.full((end, abi.LINE), 0xEE, dtype=np.uint8)
    meta_ref = np.full(end * abi.META_DT.itemsize, 0xEE, dtype=np.uint8).view(abi.META_DT)
    abi.check("gr_hip_node_stage", H.gr_hip_node_stage(ref.ctypes.data, n, 256, pos_ref.ctypes.data,
                                                         lines_ref.ctypes.data, meta_ref.ctypes.data))
    fn = ctypes.CDLL(abi.LIB_HIP).gr_node_stage_mbufs
    P = ctypes.c_void_p
    fn.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32, ctypes.c_uint64, P, P, P]
    fn.restype = ctypes.c_uint64
    pos = np.zeros(n, dtype=np.uint32)
    lines = np.full((end, abi.LINE), 0xEE, dtype=np.uint8)
    meta = np.full(end * abi.META_DT.itemsize, 0xEE, dtype=np.uint8).view(abi.META_DT)
    p = 0
    for i, k in sizes:
        p = fn(ptrs.ctypes.data + 8 * i, k, ctypes.addressof(lay), 256, p, pos.ctypes.data + 4 * i,
               lines.ctypes.data, meta.ctypes.data)
    assert p == end
    assert np.array_equal(pos, pos_ref)
    assert np.array_equal(lines, lines_ref) and np.array_equal(meta, meta_ref)
    assert ((meta["vlan_ck"] & 0x4000) != 0).sum() == sum(1 + (k - 1) // 256 for _, k in sizes)  # one walk flag per cut


def test_apply_onto_mbufs_without_views():
    """The hand-back of a batch appended from the mbufs (no views: each
    packet's fields read from its rte_mbuf through the layout, its iface id
    and walk starts from the staged metadata) leaves every mbuf, private
    area, frame, edge and counter exactly as the hand-back driven by the
    views does, over every edge of the corpus in walks of 64."""
    t, _ = SC.corpus_topology()
    fr, me, _ = SC.corpus_arrays()
    keep = ((me["vlan_ck"] >> 12) & 3) != 3
    fr, me = np.concatenate([fr[keep]] * 4), np.concatenate([me[keep]] * 4)
    n = len(me)
    lines, v, _, _, _ = oracle.Oracle(t).process_mbufs(fr, me)
    L, G = GROUT_LAYOUT, GROUT_STAGE
    ifobj = np.zeros((t.max_ifaces, 64), dtype=np.uint8)
    ifobj.view(np.uint16)[:, G["iface_id"] // 2] = np.arange(t.max_ifaces)
    reg_if = np.zeros(t.max_ifaces, dtype=np.uint64)
    live = t.ifaces["id"] != 0
    reg_if[live] = IF_OBJ + np.nonzero(live)[0]
    reg_nh = (NH_OBJ + np.arange(len(t.nh), dtype=np.uint64)).astype(np.uint64)
    reg_nh[0] = 0
    lay = Layout(**L, **G, n_ifaces=len(reg_if), n_nh=len(reg_nh), ifaces=reg_if.ctypes.data, nh=reg_nh.ctypes.data)
    H = abi.hip()
    res = []
    for own in (False, True):
        bufs, m = mbufs_for(fr, me)  # the frames at RX, each run its own copy
        m["flags"][::64] = abi.MBUF_F_WALK
        mem = np.zeros((n, 256), dtype=np.uint8)
        U16, U32, U64 = mem.view(np.uint16), mem.view(np.uint32), mem.view(np.uint64)
        U64[:, G["buf_addr"] // 8] = m["frame"] - RX_DATA_OFF
        U16[:, L["data_off"] // 2] = RX_DATA_OFF
        U16[:, L["data_len"] // 2] = m["data_len"]
        U32[:, L["pkt_len"] // 4] = m["pkt_len"]
        U16[:, (L["priv"] + L["priv_vlan_id"]) // 2] = m["vlan_id"]
        ptrs = (mem.ctypes.data + np.arange(n, dtype=np.uint64) * 256).astype(np.uint64)
        pos = np.arange(n, dtype=np.uint32)  # walks of 64 on tiles: no pads
        meta = np.zeros(n, dtype=abi.META_DT)
        abi.check("gr_hip_node_stage", H.gr_hip_node_stage(m.ctypes.data, n, 64, pos.ctypes.data, None,
                                                             meta.ctypes.data))
        edges = np.full(n, 0xEE, dtype=np.uint8)
        d = Direct(mbufs=ptrs.ctypes.data, lay=ctypes.addressof(lay), edges=edges.ctypes.data,
                   meta=meta.ctypes.data if own else None)
        ns, st = apply_counting(None if own else m, lines, v, t, direct=ctypes.addressof(d), pos=pos)
        res.append((mem.copy(), bufs.copy(), edges.copy(), ns, st, d.stale))
    (mem0, b0, e0, ns0, st0, s0), (mem1, b1, e1, ns1, st1, s1) = res
    assert np.array_equal(e0, e1) and (e0 != 0xEE).all()
    assert np.array_equal(mem0[:, 16:48], mem1[:, 16:48])  # data_off .. data_len, packet_type
    assert np.array_equal(mem0[:, 128:192], mem1[:, 128:192])  # the private area
    assert np.array_equal(b0[:, :abi.LINE], b1[:, :abi.LINE])  # the frames
    assert np.array_equal(ns0, ns1) and np.array_equal(st0, st1) and s0 == s1
    assert len(set(e0.tolist())) > 20


def test_apply_counts_ifaces_where_grout_does():
    """The hand-back's host-side per-iface counters (rx in iface_input past
    its admin-down and unknown-VLAN drops, VLAN sub-interface and parent; tx
    in iface_output past its no-parent and admin-down drops, VLAN and parent)
    equal the oracle's, over every edge of the corpus and a full-view stream."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    lines, v, st_want, want, _ = oracle.Oracle(t).process_mbufs(fr, me)
    bufs, m = mbufs_for(fr, me)
    _, st = apply_counting(m, lines, v, t)
    compare_mbufs(m, want, bufs, lines, lab)
    bad = np.nonzero(st != st_want)[0]
    assert len(bad) == 0, [(int(i), st[i], st_want[i]) for i in bad[:4]]
    assert st["rx_packets"].sum() > 100 and st["tx_packets"].sum() > 10
    assert (t.ifaces["type"][np.nonzero(st["tx_packets"])[0]] == abi.IFACE_TYPE["VLAN"]).any()  # VLAN + parent
    tf = T.config_fullview(count=50_000)
    fr, me = S.stream(1 << 14, 0xA12, routes=tf.route_array())
    lines, v, st_want, _, _ = oracle.Oracle(tf).process_mbufs(fr, me)
    _, m = mbufs_for(fr, me)
    _, st = apply_counting(m, lines, v, tf)
    assert np.array_equal(st, st_want)


def test_apply_fullview_stream():
    tf = T.config_fullview(count=100_000)
    fr, me = S.stream(1 << 16, 0xA11, routes=tf.route_array())
    lines, v, _, want, ns_want = oracle.Oracle(tf).process_mbufs(fr, me)
    bufs, m = mbufs_for(fr, me)
    ns = apply(m, lines, v, tf)
    compare_mbufs(m, want, bufs, lines)
    assert np.array_equal(ns["packets"], ns_want["packets"]) and np.array_equal(ns["calls"], ns_want["calls"])
    fwd = m["edge"] == abi.EDGE["port_output"]
    assert fwd.mean() > 0.99
    assert (m["data_off"][fwd] == RX_DATA_OFF).all() and (m["packet_type"][fwd] == abi.PTYPE_L3_IPV4).all()
    assert (m["data_off"][~fwd] == RX_DATA_OFF + 14).all()  # no route: left after eth_input's adj


@pytest.mark.gpu
@pytest.mark.parametrize("kernel_counters", [1, 0])
def test_node_process_gpu(fastpath, kernel_counters):
    """The whole node walk on the GPU (stage, fwd4_host, apply) against the
    oracle's mbufs, corpus and a one-route stream. The node stages 64-byte
    header lines, so the oracle runs lines-only: an IPv4 header that does not
    fit is punted to grout's CPU nodes, mbuf untouched. The node's per-iface
    counters are the kernel's (folded in from the queue's device counters),
    or, with the kernel's counters off ("stats" 0), the hand-back's."""
    from golden_util import fresh_fastpath_state
    fastpath.tune("stats", kernel_counters)
    try:
        for topo, fr, me, lab in [(SC.corpus_topology()[0],) + tuple(SC.corpus_arrays()),
                                  (T.config_single_route(),) + S.stream(100_003, 0xB0B, dst_range=(
                                      T.ip4("16.1.0.0"), T.ip4("16.1.255.255"))) + (None,)]:
            fresh_fastpath_state(fastpath, topo)
            lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
            bufs, m = mbufs_for(fr, me)
            q = fastpath.queue()
            ns = q.node_process(m, burst=64)
            compare_mbufs(m, want, bufs, lines, lab)
            assert np.array_equal(ns["packets"], ns_want["packets"])
            assert np.array_equal(ns["calls"], ns_want["calls"])
            if kernel_counters:
                assert np.array_equal(q.stats(), st)  # the iface counters of the same packets
            else:
                assert not q.stats()["rx_packets"].any()
            assert np.array_equal(q.node_iface_stats(), st)  # what the node reports, either way
            q.close()
    finally:
        fastpath.tune("stats", 1)


@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [1, 0])
def test_node_process_registered_frames(fastpath, ptrs):
    """Frames in memory registered with gr_hip_host_register: the node hands
    them to the GPU by address and the kernel rewrites them in place over
    PCIe (node_ptrs 1); the same mbufs staged as lines (node_ptrs 0) must end
    identical."""
    import ctypes
    from golden_util import fresh_fastpath_state
    topo = T.config_fullview(count=100_000)
    fr, me = S.stream(70_001, 0xB0E, routes=topo.route_array())
    fresh_fastpath_state(fastpath, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    L = fastpath.lib
    abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    try:
        dev = ctypes.c_uint64()
        assert L.gr_hip_host_dev_addr(fastpath.h, bufs.ctypes.data + 64, ctypes.byref(dev)) == 0
        assert L.gr_hip_host_register(fastpath.h, bufs.ctypes.data + 64, 64) == -17  # -EEXIST: overlaps
        fastpath.tune("node_ptrs", ptrs)
        q = fastpath.queue()
        ns = q.node_process(m, burst=64)
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(ns["packets"], ns_want["packets"]) and np.array_equal(ns["calls"], ns_want["calls"])
        assert np.array_equal(q.stats(), st)
        q.close()
    finally:
        fastpath.tune("node_ptrs", 0)  # the default
        abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
    assert L.gr_hip_host_dev_addr(fastpath.h, bufs.ctypes.data, ctypes.byref(dev)) == -2  # -ENOENT



@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [1, 0])
def test_node_give_up_hands_back(fastpath, ptrs):
    """A kernel that gives up (spin_max 1) processed each 64-packet tile whole
    or not at all: the node hands back the finished packets as usual and the
    rest as PUNT with frames and mbufs untouched (grout's CPU nodes take
    them), instead of punting frames it already rewrote."""
    from golden_util import fresh_fastpath_state
    topo = T.config_single_route()
    n = 1 << 18
    fr, me = S.stream(n, 0x61FE, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fresh_fastpath_state(fastpath, topo)
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    orig_bufs, orig_m = bufs.copy(), m.copy()
    L = fastpath.lib
    if ptrs:
        abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    q = fastpath.queue()
    try:
        fastpath.tune("node_ptrs", ptrs)
        assert fastpath.tune("spin_max", 1) == 0
        q.node_process(m, burst=64)
    finally:
        fastpath.tune("spin_max", 0)
        fastpath.tune("node_ptrs", 0)  # the default
        if ptrs:
            abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
    punt = m["edge"] == abi.EDGE["punt"]
    assert q.unfinished == punt.sum() > 0  # (frames over PCIe: often every tile gives up)
    assert np.array_equal(bufs[punt], orig_bufs[punt])
    orig_m["edge"] = abi.EDGE["punt"]
    assert np.array_equal(m[punt], orig_m[punt])
    done = ~punt
    compare_mbufs(m[done], want[done], bufs[done], lines[done])
    q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [0, 1])
def test_node_pipelined_walks(fastpath, ptrs):
    """gr_hip_node_start / _finish: walk i+1 is staged and sent while walk i
    is on the GPU, and walks finish in start order; every walk ends exactly
    as gr_hip_node_process leaves it (the oracle's mbufs), counters included.
    Past GR_HIP_NODE_DEPTH walks in flight a start is refused (-EBUSY), and
    so is node_process while walks are in flight; finishing with none in
    flight is -ENOENT."""
    from golden_util import fresh_fastpath_state
    topo = T.config_fullview(count=100_000)
    fr, me = S.stream(50_000, 0xB1F, routes=topo.route_array())
    fresh_fastpath_state(fastpath, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    L = fastpath.lib
    if ptrs:
        abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    q = fastpath.queue()
    try:
        fastpath.tune("node_ptrs", ptrs)
        # walk boundaries on multiples of 64: the oracle's graph walks of 64 stay whole
        cuts = [0, 64 * 100, 64 * 101, 64 * 400, 64 * 401 + 64, len(m)]
        parts = [m[a:b] for a, b in zip(cuts, cuts[1:])]
        total = np.zeros(1, dtype=abi.NODE_STATS_DT)[0]
        D = abi.NODE_DEPTH
        assert len(parts) > D
        for k in range(D):  # the queue full: D walks in flight
            q.node_start(parts[k])
            assert q.node_pending()[0] == k + 1
        assert L.gr_hip_node_start(q._h, parts[D].ctypes.data, len(parts[D]), 64) == -16  # -EBUSY
        assert L.gr_hip_node_process(q._h, parts[D].ctypes.data, len(parts[D]), 64, None) == -16
        done = 0
        for k in range(D, len(parts)):  # one out, one in: still D in flight
            got, ns = q.node_finish()
            assert got is parts[done] and q.unfinished == 0
            done += 1
            total["packets"] += ns["packets"]
            total["calls"] += ns["calls"]
            q.node_start(parts[k])
            assert q.node_pending()[0] == D
        while done < len(parts):
            got, ns = q.node_finish()
            assert got is parts[done]
            done += 1
            total["packets"] += ns["packets"]
            total["calls"] += ns["calls"]
        assert q.node_pending() == (0, False)
        assert L.gr_hip_node_finish(q._h, None, None, None) == -2  # -ENOENT
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(total["packets"], ns_want["packets"])
        assert np.array_equal(total["calls"], ns_want["calls"])
        assert np.array_equal(q.stats(), st)
        # an empty walk passes through the pipeline too
        q.node_start(m[:0])
        got, ns = q.node_finish()
        assert len(got) == 0 and ns["packets"].sum() == 0
    finally:
        fastpath.tune("node_ptrs", 0)
        if ptrs:
            abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
        q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [0, 1])
def test_node_append_send(fastpath, ptrs):
    """gr_hip_node_append / _send: the walks of a batch staged one call at a
    time as they arrive (the grout node's path) end exactly as one
    gr_hip_node_start of the same views (the oracle's mbufs), walks of every
    length up to 256 included. A later append whose first view does not
    start a walk, and a send of other views than were appended, are
    refused (-EINVAL) and leave the queue usable; discard drops an append."""
    from golden_util import fresh_fastpath_state
    topo = T.config_fullview(count=100_000)
    fr, me = S.stream(30_000, 0xA99E, routes=topo.route_array())
    fresh_fastpath_state(fastpath, topo)
    rng = np.random.default_rng(7)
    cuts = [0]
    while cuts[-1] < len(fr):
        cuts.append(min(len(fr), cuts[-1] + int(rng.choice([1, 3, 17, 63, 64, 65, 128, 200, 256]))))
    walks = list(zip(cuts, cuts[1:]))
    meta_walk = me.copy()
    meta_walk["vlan_ck"][[a for a, _ in walks]] |= abi.META_WALK
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, meta_walk, lines_only=True, burst=256)
    bufs, m = mbufs_for(fr, me)
    m["flags"][[a for a, _ in walks]] |= abi.MBUF_F_WALK
    L = fastpath.lib
    if ptrs:
        abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    q = fastpath.queue()
    try:
        fastpath.tune("node_ptrs", ptrs)
        # refused appends and sends, then a discarded one
        assert L.gr_hip_node_append(q._h, m.ctypes.data, 10, 256) > 0
        assert L.gr_hip_node_append(q._h, m[5:].ctypes.data, 3, 256) == -22  # m[5] starts no walk
        assert L.gr_hip_node_send(q._h, m.ctypes.data, 11, 256) == -22  # 10 were appended
        assert q.node_pending()[0] == 0
        assert L.gr_hip_node_append(q._h, m.ctypes.data, 10, 256) > 0
        assert L.gr_hip_node_discard(q._h) == 0
        # the batch, one walk per append, in two halves pipelined
        half = walks[len(walks) // 2][0]
        ns_tot = np.zeros(1, dtype=abi.NODE_STATS_DT)[0]
        for lo, hi in ((0, half), (half, len(m))):
            part = m[lo:hi]
            for a, b in walks:
                if lo <= a < hi:
                    staged = L.gr_hip_node_append(q._h, part[a - lo:].ctypes.data, b - a, 256)
                    assert staged >= b - lo, (a, b, staged)
            abi.check("gr_hip_node_send", L.gr_hip_node_send(q._h, part.ctypes.data, len(part), 256))
            q._walks.append(part)
        for _ in range(2):
            got, ns = q.node_finish()
            assert q.unfinished == 0
            ns_tot["packets"] += ns["packets"]
            ns_tot["calls"] += ns["calls"]
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(ns_tot["packets"], ns_want["packets"])
        assert np.array_equal(ns_tot["calls"], ns_want["calls"])
        assert np.array_equal(q.stats(), st)
    finally:
        fastpath.tune("node_ptrs", 0)
        if ptrs:
            abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
        q.close()


@pytest.mark.gpu
def test_finish_drop_waits_for_the_gpu(fastpath):
    """gr_hip_node_finish on a batch appended from the mbufs drops it with
    -EINVAL (gr_hip_node_finish_mbufs hands such a batch back), but only once
    the GPU is done with it: gpu_fwd4_fini calls it on a graph destroyed with
    a batch in flight and frees the mbufs next, while the kernel rewrites
    registered frames in place. Every forwarded frame is therefore already
    rewritten when the call returns."""
    from golden_util import fresh_fastpath_state
    topo = T.config_single_route()
    n = 1 << 18
    fr, me = S.stream(n, 0xF1A1, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fresh_fastpath_state(fastpath, topo)
    lines, v, _, _, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    orig = bufs[:, :abi.LINE].copy()
    L_, G = GROUT_LAYOUT, GROUT_STAGE
    mem = np.zeros((n, 256), dtype=np.uint8)
    U16, U32, U64 = mem.view(np.uint16), mem.view(np.uint32), mem.view(np.uint64)
    U64[:, G["buf_addr"] // 8] = m["frame"] - RX_DATA_OFF
    U16[:, L_["data_off"] // 2] = RX_DATA_OFF
    U16[:, L_["data_len"] // 2] = m["data_len"]
    U32[:, L_["pkt_len"] // 4] = m["pkt_len"]
    U32[:, G["rss"] // 4] = m["rss"]
    ifobj = np.zeros((topo.max_ifaces, 64), dtype=np.uint8)
    ifobj.view(np.uint16)[:, G["iface_id"] // 2] = np.arange(topo.max_ifaces)
    U64[:, (L_["priv"] + L_["priv_iface"]) // 8] = ifobj.ctypes.data + 64 * m["iface"].astype(np.uint64)
    ptrs = (mem.ctypes.data + np.arange(n, dtype=np.uint64) * 256).astype(np.uint64)
    lay = Layout(**L_, **G, n_ifaces=0, n_nh=0, ifaces=None, nh=None)
    L = fastpath.lib
    abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    q = fastpath.queue()
    try:
        fastpath.tune("node_ptrs", 1)  # frames by address: the kernel rewrites them over PCIe
        assert L.gr_hip_node_append_mbufs(q._h, ptrs.ctypes.data, n, ctypes.addressof(lay), 256) >= n
        abi.check("gr_hip_node_send", L.gr_hip_node_send(q._h, None, n, 256))
        assert L.gr_hip_node_finish(q._h, None, None, None) == -22  # -EINVAL: not handed back ...
        after = bufs[:, :abi.LINE].copy()  # ... but the GPU is done with the frames
        assert q.node_pending()[0] == 0
    finally:
        fastpath.tune("node_ptrs", 0)
        q.close()
        abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
    fwd = v["edge"] == abi.EDGE["port_output"]
    assert fwd.all()
    assert not np.array_equal(after, orig)
    assert np.array_equal(after, lines)
