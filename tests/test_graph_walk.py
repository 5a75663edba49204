# SPDX-License-Identifier: BSD-3-Clause
"""The fast path as a grout node in an rte_graph walk (grout_amd/graph/).

gpu_fwd4_node.c is the node a grout maintainer compiles into grout: it is
registered as "iface_input" through grout's node-info surface, its next
nodes are the verdict edges, and it hands each mbuf to its edge with the
private data grout's chain leaves there. Here it is compiled against the
rte_graph / grout stand-ins (rte_graph_min.h, gr_datapath_min.h) and walked in
a worker-shaped graph: port_rx (bursts of 64) -> iface_input -> recorder
nodes named after every edge (walk_harness.c).

CPU: the stand-in runtime's semantics (graph_selftest.c), the node's
registration (edge names in enum order) and its refusal to join a graph
without the GPU module. GPU: whole walks against the oracle's mbuf-level
chain (oracle.c process_mbufs, lines-only: the node stages 64-byte lines)."""
import ctypes
import os

import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

LIB = os.path.join(os.path.dirname(abi.LIB_HIP), "libgrout_graph.so")

OUT_DT = np.dtype([("pkt_len", "<u4"), ("data_len", "<u2"), ("data_off", "<u2"), ("packet_type", "<u4"),
                   ("iface", "<u2"), ("vlan_id", "<u2"), ("edge", "u1"), ("domain", "u1"), ("_pad", "<u2"),
                   ("nh", "<u4"), ("seq", "<u4"), ("eth_nh", "<u4")])
assert OUT_DT.itemsize == 32

_lib = None


def lib():
    global _lib
    if _lib is None:
        abi.hip()  # libgrout_hip.so first (torch's HIP runtime, abi.py)
        _lib = ctypes.CDLL(LIB)
        _lib.gh_hip_ctx.restype = ctypes.c_void_p
        _lib.gh_init.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_uint64]
        _lib.gh_graph_create.argtypes = [ctypes.c_char_p]
        _lib.rte_node_from_name.argtypes = [ctypes.c_char_p]
        _lib.rte_node_from_name.restype = ctypes.c_uint32
        _lib.rte_node_edge_count.restype = ctypes.c_uint16
        _lib.rte_node_edge_get.restype = ctypes.c_uint16
        _lib.gh_rte_node_counters.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        # pointers as c_void_p (a bare Python int would be passed as a C int)
        _lib.gh_load.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        _lib.gh_run.argtypes = [ctypes.c_uint32]
        _lib.gh_results.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _lib.gh_node_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _lib.gh_queue_stats.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    return _lib


def edges_of(name):
    L = lib()
    nid = L.rte_node_from_name(name.encode())
    assert nid != 0xFFFFFFFF, name
    n = L.rte_node_edge_count(nid)
    names = (ctypes.c_char_p * n)()
    assert L.rte_node_edge_get(nid, names) == n
    return [x.decode() for x in names]


def test_runtime_semantics():
    """Registration, dynamic edges, graph creation from patterns (reachable
    nodes join, dangling edges refused), walk order, stream move, counters."""
    assert lib().gh_graph_selftest() == 0


def test_node_registration():
    L = lib()
    assert L.gh_register() == 0
    want = ["iface_input_cpu"] + abi.EDGE_NAMES[1:]  # PUNT: grout's stock iface_input
    assert edges_of("iface_input") == want
    assert edges_of("gpu_fwd4_flush") == want
    assert edges_of("port_rx") == ["iface_input"]


def test_graph_refused_without_gpu_module():
    """The node's init fails without the fast-path context: no graph, no
    silent CPU path."""
    L = lib()
    assert L.gh_register() == 0
    if L.gh_hip_ctx():
        pytest.skip("module already initialised in this process")
    assert L.gh_graph_create(b"no_gpu") < 0


# ---------------------------------------------------------------------------
# GPU: whole walks
# ---------------------------------------------------------------------------
BATCH, BURST, DELAY_NS = 4096, 64, 2_000_000
_gh = {}


def graph_ctx():
    """One node module (fast-path context) and one worker graph per process."""
    from grout_amd.fwd import FastPath
    L = lib()
    if "fp" not in _gh:
        r = L.gh_init(0, 1024, 1 << 17, BATCH, BURST, DELAY_NS)
        assert r == 0, r
        assert L.gh_graph_create(b"gh") == 0
        _gh["fp"] = FastPath.borrow(L.gh_hip_ctx())
    return _gh["fp"]


def load(fp, topo):
    from golden_util import fresh_fastpath_state
    fresh_fastpath_state(fp, topo, _gh.setdefault("state", {}))


def walk(frames, meta):
    L = lib()
    frames = np.ascontiguousarray(frames)
    meta = np.ascontiguousarray(meta, dtype=abi.META_DT)
    n = len(meta)
    assert L.gh_load(frames.ctypes.data, frames.shape[1], meta.ctypes.data, n) == 0
    walks = L.gh_run(1 << 22)
    assert walks > 0, walks
    out = np.zeros(n, dtype=OUT_DT)
    lines = np.zeros((n, abi.LINE), dtype=np.uint8)
    assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
    ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
    err = ctypes.c_uint64()
    assert L.gh_node_stats(ns.ctypes.data, ctypes.byref(err)) == 0
    assert err.value == 0
    return out, lines, ns[0], walks


def stage_of(edges, nh, ip6):
    L = abi.hip()
    return np.array([L.gr_hip_edge_node(int(e), int(h), int(s)) for e, h, s in zip(edges, nh, ip6)])


def check_walk(topo, fr, me, labels=None):
    fp = graph_ctx()
    load(fp, topo)
    L = lib()
    L.gh_queue_stats(None, 0, 1)  # reset the queue's iface counters
    ns0 = np.zeros(1, dtype=abi.NODE_STATS_DT)
    assert L.gh_node_stats(ns0.ctypes.data, None) == 0
    o_lines, o_v, o_st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    got, lines, ns, _ = walk(fr, me)
    lab = (lambda i: labels[i]) if labels else (lambda i: i)
    for f in ["edge", "pkt_len", "data_len", "data_off", "packet_type", "iface"]:
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, (f, [(lab(i), int(got[f][i]), int(want[f][i])) for i in bad[:6]])
    bad = np.nonzero((lines != o_lines).any(axis=1))[0]
    assert len(bad) == 0, [lab(i) for i in bad[:6]]
    # private data, as the node behind each edge reads it
    ip6 = (fr[:, 12] == 0x86) & (fr[:, 13] == 0xDD)
    st = stage_of(want["edge"], want["nh"], ip6)
    N = {n: i for i, n in enumerate(abi.NODE_NAMES)}
    vl = np.isin(st, [N["iface_input"], N["iface_output"]])
    assert np.array_equal(got["vlan_id"][vl], want["vlan_id"][vl])
    # l3 nexthop: read by ip_output / ip_hold / ip_error ... (l3.h:9); past
    # iface_output the same bytes hold iface_mbuf_data's vlan_id instead
    l3 = (want["nh"] != 0) & ~vl
    bad = np.nonzero(got["nh"][l3] != want["nh"][l3])[0]
    assert len(bad) == 0, [(lab(i), abi.EDGE_NAMES[want["edge"][i]], int(got["nh"][i]), int(want["nh"][i]))
                           for i in np.nonzero(l3)[0][bad[:6]]]
    dom = (st >= 0) & ~vl & (st != N["eth_output"]) & ~l3
    assert np.array_equal(got["domain"][dom], want["domain"][dom])
    assert (got["eth_nh"][dom] == 0).all()
    # each edge receives its packets in RX order
    for e in np.unique(got["edge"]):
        s = got["seq"][got["edge"] == e]
        assert (np.diff(s.astype(np.int64)) > 0).all(), abi.EDGE_NAMES[e]
    # rte_graph counters of the replaced nodes, grout's rule (ip_output returns
    # what it sent to eth_output)
    dn = {k: ns[k] - ns0[0][k] for k in ("packets", "calls")}
    assert np.array_equal(dn["packets"], ns_want["packets"]), (dn, ns_want)
    assert np.array_equal(dn["calls"], ns_want["calls"]), (dn, ns_want)
    qs = np.zeros(fp.max_ifaces, dtype=abi.STATS_DT)
    assert L.gh_queue_stats(qs.ctypes.data, fp.max_ifaces, 1) == 0
    assert np.array_equal(qs, o_st)
    # every packet reached the recorder of its edge, counted by rte_graph
    for e in np.unique(got["edge"]):
        c = np.zeros(3, dtype=np.uint64)
        name = "iface_input_cpu" if e == 0 else abi.EDGE_NAMES[e]
        assert L.gh_rte_node_counters(name.encode(), c.ctypes.data) == 0
        assert c[0] >= (got["edge"] == e).sum()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("pin", [1, 0])
def test_graph_walk_corpus(pin):
    """Every edge. pin 1: the mbuf memory is registered, frames go to the GPU
    by address and come back rewritten in place; pin 0: header lines staged."""
    lib().gh_set_pin(pin)
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    # ol_flags has no value for the corpus's out-of-range status 3 ("ol 3")
    keep = ((me["vlan_ck"] >> 12) & 3) != 3
    fr, me, lab = fr[keep], me[keep], [x for x, k in zip(lab, keep) if k]
    try:
        got = check_walk(t, fr, me, lab)
    finally:
        lib().gh_set_pin(1)
    assert len(set(got["edge"])) > 20


@pytest.mark.gpu
def test_graph_walk_stream_batches():
    """A one-route stream over many batches: 4096-packet batches fill, the
    last RX burst is short and flushes the rest."""
    t = T.config_single_route()
    fr, me = S.stream(100_003, 0xB0C, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    got = check_walk(t, fr, me)
    assert (got["edge"] == abi.EDGE["port_output"]).all()


@pytest.mark.gpu
def test_graph_walk_flush_node():
    """Full bursts only: the packets behind the last full batch wait for the
    flush source node (max_delay), then leave in order."""
    t = T.config_single_route()
    n = BATCH + 2 * BURST
    fr, me = S.stream(n, 0xB0D, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    check_walk(t, fr, me)
    c = np.zeros(3, dtype=np.uint64)
    assert lib().gh_rte_node_counters(b"gpu_fwd4_flush", c.ctypes.data) == 0
    assert c[2] >= 2 * BURST  # the flush node handed those packets on
