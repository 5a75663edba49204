# SPDX-License-Identifier: BSD-3-Clause
"""The fast path as a grout node in an rte_graph walk (grout_amd/module/).

gpu_fwd4_node.c is the node a grout maintainer compiles into grout: it is
registered as "iface_input" through grout's node-info surface, its next
nodes are the verdict edges, and it hands each mbuf to its edge with the
private data grout's chain leaves there. Here the module library
(libgrout_gpu_fwd4.so) is compiled against the rte_graph / grout stand-ins
under grout's header names (tests/standin/include) and loaded by the
stand-in library (tests/standin/libgrout_standin.so), which walks it in a
worker-shaped graph: port_rx (bursts of 64) -> iface_input -> recorder
nodes named after every edge (walk_harness.c).

CPU: the stand-in runtime's semantics (graph_selftest.c), the node's
registration (edge names in enum order) and its refusal to join a graph
without the GPU module. GPU: whole walks against the oracle's mbuf-level
chain (oracle.c process_mbufs, lines-only: the node stages 64-byte lines)."""
import ctypes
import errno
import os

import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "standin", "libgrout_standin.so")  # test infrastructure: the stand-ins + harness
LIB_MODULE = os.path.join(os.path.dirname(abi.LIB_HIP), "libgrout_gpu_fwd4.so")  # the module (product)

OUT_DT = np.dtype([("pkt_len", "<u4"), ("data_len", "<u2"), ("data_off", "<u2"), ("packet_type", "<u4"),
                   ("iface", "<u2"), ("vlan_id", "<u2"), ("edge", "u1"), ("domain", "u1"), ("conn", "<u2"),
                   ("nh", "<u4"), ("seq", "<u4"), ("eth_nh", "<u4"), ("eth_dst", "u1", (6,)), ("eth_type", "<u2"),
                   ("vtep_af", "u1"), ("flow", "u1"), ("_pad", "<u2")])
assert OUT_DT.itemsize == 44
CONN_KEY_DT = np.dtype([("iface_id", "<u2"), ("af", "u1"), ("proto", "u1"), ("src", ">u4"), ("dst", ">u4"),
                        ("src_id", ">u2"), ("dst_id", ">u2")])
assert CONN_KEY_DT.itemsize == 16

_lib = None


def lib():
    global _lib
    if _lib is None:
        abi.hip()  # libgrout_hip.so first (torch's HIP runtime, abi.py)
        _lib = ctypes.CDLL(LIB)
        P, U32, U16 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16
        _lib.gh_hip_ctx.restype = P
        _lib.gh_ctx_at.restype = P
        _lib.gh_ctx_at.argtypes = [U32]
        _lib.gh_n_ctx.restype = U32
        _lib.gh_init.argtypes = [P, U32, U32, U32, U32, U32, ctypes.c_uint64]
        _lib.gh_graph_create.argtypes = [ctypes.c_uint, ctypes.c_int]
        _lib.gh_graph_use.argtypes = [ctypes.c_int]
        _lib.gh_recorder_name.restype = ctypes.c_char_p
        _lib.gh_recorder_name.argtypes = [U32]
        _lib.rte_node_from_name.argtypes = [ctypes.c_char_p]
        _lib.rte_node_from_name.restype = U32
        _lib.rte_node_id_to_name.restype = ctypes.c_char_p
        _lib.rte_node_id_to_name.argtypes = [U32]
        _lib.rte_node_max_count.restype = U32
        _lib.rte_node_edge_count.restype = ctypes.c_uint16
        _lib.rte_node_edge_get.restype = ctypes.c_uint16
        _lib.gh_rte_node_counters.argtypes = [ctypes.c_char_p, P]
        # pointers as c_void_p (a bare Python int would be passed as a C int)
        _lib.gh_load.argtypes = [P, U32, P, U32]
        _lib.gh_run.argtypes = [U32]
        _lib.gh_results.argtypes = [P, P]
        _lib.gh_node_stats.argtypes = [P, P]
        _lib.gh_queue_stats.argtypes = [P, U32, ctypes.c_int]
        _lib.gh_set_objects.argtypes = [P, U32, P, U32, U32]
        _lib.gpu_fwd4_set_depth.argtypes = [U32]
        _lib.gh_conn_add.argtypes = [P, P]
        _lib.gh_snat44_static_add.argtypes = [U16, U32, U32]
        _lib.gh_worker_stats.argtypes = [ctypes.c_char_p, P]
        _lib.gh_iface_stats.argtypes = [U16, P]
        _lib.gh_walk_info.argtypes = [P]
        _lib.gh_rcu_delete_test.argtypes = [U32, U16, U32, P]
        _lib.gh_churn_test.argtypes = [U32, ctypes.c_uint8, U16, U32, U32, U32, U32, P]
        _lib.gh_set_rx_burst.argtypes = [U32]
        _lib.gh_loop_test.argtypes = [U32, ctypes.c_int, ctypes.c_int, U32, U32, U32, P]
        _lib.gpu_fwd4_holding.restype = ctypes.c_uint64
        _lib.gpu_fwd4_set_batch.argtypes = [U32, ctypes.c_uint64]
        _lib.gh_set_gpu_load.argtypes = [U32]
        _lib.gh_set_gpu_load.restype = None
        _lib.gpu_fwd4_diverged.argtypes = [U32]
        _lib.gpu_fwd4_resync.argtypes = [U32]
        _lib.gpu_fwd4_rcu_readers.argtypes = [ctypes.c_int]
        _lib.gpu_fwd4_configure.argtypes = [P]
        _lib.gpu_fwd4_conf_get.argtypes = [P]
        _lib.gh_graph_selftest.restype = ctypes.c_int
        _lib.gh_rcu_selftest.restype = ctypes.c_int
    return _lib


WALK_INFO_DT = np.dtype([("held", "<u4"), ("in_flight", "<u4"), ("batches", "<u8"), ("max_batch", "<u8"),
                         ("stale", "<u8"), ("readers_online", "<u4"), ("diverged", "<i4"), ("append_errors", "<u8"),
                         ("handed", "<u8"), ("drain_punted", "<u8"), ("stranded", "<u8"), ("batch_cap", "<u4"),
                         ("lat_ns", "<u8"), ("over_budget", "<u8"), ("depth", "<u4")], align=True)
assert WALK_INFO_DT.itemsize == 104
LOOP_RES_DT = np.dtype([("walks", "<u4"), ("windows", "<u4"), ("sleeps", "<u4"), ("sleeps_held", "<u4"),
                        ("busy_held", "<u4"), ("blocked", "<u4"), ("recorded_at_block", "<u4"),
                        ("held_at_block", "<u8"), ("readers_online_at_block", "<u4"), ("sync_returned", "<u4"),
                        ("sync_us", "<u8"), ("elapsed_us", "<u8"), ("recorded", "<u4")], align=True)
RCU_RES_DT = np.dtype([("sync_before_handback", "<u4"), ("recorded_at_sync", "<u4"), ("freed_reads", "<u4"),
                       ("recorded", "<u4"), ("stale", "<u8"), ("sync_us", "<u8"), ("walks", "<u4"),
                       ("sync_done", "<u4")])
assert RCU_RES_DT.itemsize == 40
CONF_DT = np.dtype([("n_devs", "<u4"), ("devs", "<i4", (16,)), ("max_ifaces", "<u4"), ("max_nexthops", "<u4"),
                    ("batch", "<u4"), ("rx_burst", "<u4"), ("max_delay_ns", "<u8"), ("depth", "<u4"),
                    ("launch_per_batch", "<u4"), ("latency_budget_ns", "<u8")], align=True)
assert CONF_DT.itemsize == 112
BATCH_MAX = 15360  # GPU_FWD4_BATCH_MAX (gpu_fwd4_node.h)


def walk_info():
    w = np.zeros(1, dtype=WALK_INFO_DT)
    assert lib().gh_walk_info(w.ctypes.data) == 0
    return w[0]


def node_counters(name):
    """rte_graph's counters of a node of the current graph: objects in,
    calls, process() returns, the stream's high-water mark."""
    c = np.zeros(4, dtype=np.uint64)
    assert lib().gh_rte_node_counters(name.encode(), c.ctypes.data) == 0
    return c


def grout_iface_stats(max_ifaces):
    """`grcli interface stats` as grout computes it: every lcore's iface_stats
    summed per iface (stats.c:197-222)."""
    out = np.zeros(max_ifaces, dtype=abi.STATS_DT)
    for i in range(max_ifaces):
        assert lib().gh_iface_stats(i, out[i:i + 1].ctypes.data) == 0
    return out


def grout_node_stats(name):
    """The worker's node statistics for `name` (packets, batches), as
    worker_dump_stats reports them."""
    c = np.zeros(2, dtype=np.uint64)
    assert lib().gh_worker_stats(name.encode(), c.ctypes.data) == 0
    return c


def rec_name(i):
    n = lib().gh_recorder_name(int(i))
    return n.decode() if n else None


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
    nodes join, dangling edges refused), walk order, stream move, counters,
    the stream limit."""
    assert lib().gh_graph_selftest() == 0


def test_rcu_qsbr_semantics():
    """The QSBR stand-in (rte_rcu_min.c) as grout's control plane relies on it:
    synchronize waits for every online registered reader to report quiescent
    (or go offline) after it started, and not for offline or unregistered
    ones; a reader that goes online after the token is not waited for."""
    assert lib().gh_rcu_selftest() == 0


def test_batch_clamped_to_stream_limit():
    """A batch above GPU_FWD4_BATCH_MAX is clamped, so that the node never
    hands rte_graph more than its uint16 streams hold (two batches per walk at
    most, plus bursts of punts)."""
    L = lib()
    if L.gh_hip_ctx():
        pytest.skip("module already initialised in this process")
    c = np.zeros(1, dtype=CONF_DT)
    c["max_ifaces"], c["max_nexthops"], c["batch"], c["rx_burst"] = 1024, 1 << 17, 1 << 16, 64
    c["max_delay_ns"], c["depth"] = 50_000, 2
    assert L.gpu_fwd4_configure(c.ctypes.data) == 0
    got = np.zeros(1, dtype=CONF_DT)
    L.gpu_fwd4_conf_get(got.ctypes.data)
    assert got["batch"][0] == BATCH_MAX and 2 * BATCH_MAX + 4 * 256 < 0xFFFF
    assert L.gpu_fwd4_set_batch(1 << 20, 1000) == 0
    L.gpu_fwd4_conf_get(got.ctypes.data)
    assert got["batch"][0] == BATCH_MAX and got["max_delay_ns"][0] == 1000
    assert L.gpu_fwd4_set_batch(0, 1000) < 0


def test_node_registration():
    L = lib()
    assert L.gh_register() == 0
    want = ["iface_input_cpu"] + abi.EDGE_NAMES[1:]  # PUNT: grout's stock iface_input, renamed
    assert edges_of("iface_input") == want
    assert edges_of("gpu_fwd4_flush") == want
    # port_rx (the harness's stand-in) feeds iface_input; port_output only in the
    # harness-alone measurement (gh_set_null_node)
    assert edges_of("port_rx") == ["iface_input", "port_output"]
    # the CPU continuation nodes and where they go (ip_input.c:20-32, ip_output.c:21-30)
    assert edges_of("ip_input_local_ct") == ["ip_input_local", "dnat44_dynamic"]
    snat = edges_of("ip_output_snat")
    assert snat[:abi.E_COUNT] == want and snat[abi.E_COUNT:] == ["eth_output", "ip_output_drop"]
    # recorder ids of the fast path's edges are the edge values
    assert [rec_name(e) for e in range(abi.E_COUNT)] == want


def _reference_node_names():
    import re
    names = set()
    for root, _, files in os.walk("/root/reference/modules"):
        for f in files:
            if f.endswith(".c"):
                t = open(os.path.join(root, f), encoding="utf-8", errors="replace").read()
                names |= set(re.findall(r'\.name = "([a-z0-9_]+)"', t))
                names |= set(re.findall(r"GR_DROP_REGISTER\((\w+)\)", t))
    names |= {"port_rx", "port_tx"}  # .name = RX_NODE_BASE / TX_NODE_BASE (rxtx.h:20-23)
    return names


@pytest.mark.skipif(not os.path.isdir("/root/reference/modules"), reason="reference not mounted")
def test_graph_nodes_are_grouts():
    """Every node the worker graph can hold is one of grout's, by name, or one
    of the four this integration adds: the fast path's node (taking grout's
    own "iface_input" name), its flush source, the two CPU continuation nodes
    -- and "iface_input_cpu", grout's iface_input under the name
    integration/grout-iface_input_cpu.patch gives it."""
    L = lib()
    assert L.gh_register() == 0
    ours = {"gpu_fwd4_flush", "ip_input_local_ct", "ip_output_snat", "iface_input_cpu"}
    ref = _reference_node_names()
    names, todo = set(), ["port_rx", "gpu_fwd4_flush"]  # what a worker graph holds: reachable nodes
    while todo:
        n = todo.pop()
        if n not in names:
            names.add(n)
            todo += edges_of(n)
    assert "iface_input" in ref and "iface_input" in names
    assert names - ref <= ours, sorted(names - ref - ours)
    assert ours <= names


def test_graph_refused_without_gpu_module():
    """The node's init fails without the fast-path context: no graph, no
    silent CPU path."""
    L = lib()
    assert L.gh_register() == 0
    if L.gh_hip_ctx():
        pytest.skip("module already initialised in this process")
    assert L.gh_graph_create(0, 0) < 0


# ---------------------------------------------------------------------------
# GPU: whole walks
# ---------------------------------------------------------------------------
BATCH, BURST, DELAY_NS = 4096, 64, 2_000_000
_gh = {}


class _FanOut:
    """libgrout_hip's gr_hip_* control calls, routed to the node module's
    gpu_fwd4_* fan-out (every context), so FastPath.load drives them."""

    def __init__(self, L):
        self._L = L

    def __getattr__(self, name):
        fn = getattr(self._L, name.replace("gr_hip_", "gpu_fwd4_", 1))
        res, args = abi.HIP_API[name]
        fn.restype, fn.argtypes = res, args[1:]  # the same call without the context
        return lambda _h, *a: fn(*a)


class FanOutPath:
    """A FastPath-shaped handle on all of the node module's contexts."""

    def __init__(self, L, max_ifaces=1024, max_nexthops=1 << 17):
        from grout_amd.fwd import FastPath
        self.lib = _FanOut(L)
        self.h = None
        self.max_ifaces = max_ifaces
        self.max_nexthops = max_nexthops
        for k in ("set_ifaces", "del_iface", "set_nexthops", "set_reta", "fib_create", "fib_destroy", "route_add",
                  "route_del", "fib_commit", "fib6_create", "fib6_destroy", "route6_add", "route6_del",
                  "fib6_commit", "load", "tune"):
            setattr(self, k, getattr(FastPath, k).__get__(self))


DEVS = (0, 0)  # two fast-path contexts on the one GPU of the box: two "GPUs"


def graph_ctx(devs=DEVS, keep=False):
    """One node module (one fast-path context per entry of devs) and one
    worker graph (cpu 0, socket 0) per process; graph 0 is the current one
    (keep: the current graph stays current)."""
    L = lib()
    if "fp" in _gh:
        if not keep:
            assert L.gh_graph_use(0) == 0
    else:
        d = (ctypes.c_int * len(devs))(*devs)
        r = L.gh_init(ctypes.cast(d, ctypes.c_void_p), len(devs), 1024, 1 << 17, BATCH, BURST, DELAY_NS)
        assert r == 0, r
        assert L.gh_graph_create(0, 0) == 0
        _gh["fp"] = FanOutPath(L)
    return _gh["fp"]


def load(fp, topo):
    from golden_util import fresh_fastpath_state
    fresh_fastpath_state(fp, topo, _gh.setdefault("state", {}))
    L = lib()
    ifs = np.ascontiguousarray(topo.ifaces[topo.ifaces["id"] != 0])
    nh = np.ascontiguousarray(topo.nh[1:topo.n_nh + 1])
    assert L.gh_set_objects(ifs.ctypes.data, len(ifs), nh.ctypes.data, 1, len(nh)) == 0


def walk(frames, meta):
    L = lib()
    frames = np.ascontiguousarray(frames)
    meta = np.ascontiguousarray(meta, dtype=abi.META_DT)
    n = len(meta)
    err0 = ctypes.c_uint64()
    assert L.gh_node_stats(None, ctypes.byref(err0)) == 0
    assert L.gh_load(frames.ctypes.data, frames.shape[1], meta.ctypes.data, n) == 0
    walks = L.gh_run(1 << 22)
    assert walks > 0, walks
    out = np.zeros(n, dtype=OUT_DT)
    lines = np.zeros((n, abi.LINE), dtype=np.uint8)
    assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
    ns = np.zeros(1, dtype=abi.NODE_STATS_DT)
    err = ctypes.c_uint64()
    assert L.gh_node_stats(ns.ctypes.data, ctypes.byref(err)) == 0
    assert err.value == err0.value  # no batch of this walk refused or cut short by the GPU
    return out, lines, ns[0], walks


def stage_of(edges, nh, ip6):
    L = abi.hip()
    return np.array([L.gr_hip_edge_node(int(e), int(h), int(s)) for e, h, s in zip(edges, nh, ip6)])


def check_walk(topo, fr, me, labels=None, burst=BURST, loaded=False):
    """One walk of (fr, me) through the current graph against the oracle on
    `topo`. loaded: the contexts already hold topo (a test that built it
    through grout's control plane and the mirror, test_control_mirror.py)."""
    fp = graph_ctx(keep=True)  # on the current graph
    if not loaded:
        load(fp, topo)
    L = lib()
    L.gh_queue_stats(None, 0, 1)  # reset the queue's iface counters
    L.gh_stats_reset()  # and grout's: iface_stats, the worker's node stats
    ns0 = np.zeros(1, dtype=abi.NODE_STATS_DT)
    assert L.gh_node_stats(ns0.ctypes.data, None) == 0
    o_lines, o_v, o_st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True, burst=burst)
    got, lines, ns, _ = walk(fr, me)
    lab = (lambda i: labels[i]) if labels else (lambda i: i)
    # packets handed to a CPU continuation node (conntrack, SNAT) end further
    # on: checked by test_graph_walk_cpu_continuations
    cont = np.isin(want["edge"], [abi.EDGE["ip_input_local_ct"], abi.EDGE["ip_output_snat"]])
    direct = ~cont
    for f in ["edge", "pkt_len", "data_len", "data_off", "packet_type", "iface"]:
        bad = np.nonzero((got[f] != want[f]) & direct)[0]
        assert len(bad) == 0, (f, [(lab(i), int(got[f][i]), int(want[f][i])) for i in bad[:6]])
    bad = np.nonzero((lines != o_lines).any(axis=1) & direct)[0]
    assert len(bad) == 0, [lab(i) for i in bad[:6]]
    got, want, lines, o_lines, fr = got[direct], want[direct], lines[direct], o_lines[direct], fr[direct]
    if labels:
        labels = [x for x, d in zip(labels, direct) if d]
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
    # what grout reports (row f2): the per-iface counters the node folded
    # into grout's per-lcore iface_stats at the housekeeping ticks, summed the
    # way `grcli interface stats` sums them ...
    qs = np.zeros(fp.max_ifaces, dtype=abi.STATS_DT)
    assert L.gh_queue_stats(qs.ctypes.data, fp.max_ifaces, 0) == 0
    assert not qs["rx_packets"].any() and not qs["tx_packets"].any()  # all folded in
    gs = grout_iface_stats(fp.max_ifaces)
    bad = np.nonzero(gs != o_st)[0]
    assert len(bad) == 0, [(int(i), gs[i], o_st[i]) for i in bad[:4]]
    # ... and the worker's node statistics (`grcli stats`): the replaced nodes
    # read as grout's own would, iface_input is the node itself
    fed = {"eth_output"} if cont.any() else set()  # ip_output_snat feeds grout's eth_output too
    for k, name in enumerate(abi.NODE_NAMES):
        if name == "iface_input" or name in fed:
            continue
        w = grout_node_stats(name)
        assert w[0] == ns_want["packets"][k] and w[1] == ns_want["calls"][k], (name, w, ns_want)
    assert grout_node_stats("iface_input")[0] == len(me)
    # every packet reached the recorder of its edge, counted by rte_graph
    for e in np.unique(got["edge"]):
        c = node_counters(rec_name(e))
        assert c[0] >= (got["edge"] == e).sum()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("pin,ptrs", [(1, 0), (0, 0), (1, 1), (0, 1)],
                         ids=["registered_staged", "staged", "by_address", "by_address_unregistered"])
def test_graph_walk_corpus(pin, ptrs):
    """Every edge. pin 1: the mbuf memory is registered with the contexts;
    ptrs ("node_ptrs") 1: registered frames go to the GPU by address and come
    back rewritten in place (the node appends the mbufs themselves: their
    device addresses are taken through the layout at send), and with the
    memory not registered the lines are staged at send instead, from the
    mbufs; ptrs 0: header lines staged as the walks arrive (the default)."""
    lib().gh_set_pin(pin)
    fp = graph_ctx()
    fp.tune("node_ptrs", ptrs)
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    # ol_flags has no value for the corpus's out-of-range status 3 ("ol 3")
    keep = ((me["vlan_ck"] >> 12) & 3) != 3
    fr, me, lab = fr[keep], me[keep], [x for x, k in zip(lab, keep) if k]
    try:
        got = check_walk(t, fr, me, lab)
    finally:
        lib().gh_set_pin(1)
        fp.tune("node_ptrs", 0)
    assert len(set(got["edge"])) > 20


@pytest.fixture(params=[2, 1, 3, 4], ids=["pipelined", "depth1", "depth3", "depth4"])
def depth(request):
    """Batches in flight per graph: 2 (the default), 1 (each waited for), or
    3 and 4 (two and three on the GPU while the next accumulates)."""
    graph_ctx()
    assert lib().gpu_fwd4_set_depth(request.param) == 0
    yield request.param
    lib().gpu_fwd4_set_depth(0)  # the default: from the budget


@pytest.mark.gpu
def test_graph_walk_stream_batches(depth):
    """A one-route stream over many batches: 4096-packet batches fill, the
    last RX burst is short and flushes the rest. Pipelined, batch i+1 is
    staged while batch i is on the GPU; they still leave in RX order."""
    t = T.config_single_route()
    fr, me = S.stream(100_003, 0xB0C, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    got = check_walk(t, fr, me)
    assert (got["edge"] == abi.EDGE["port_output"]).all()


@pytest.mark.gpu
def test_graph_walk_flush_node(depth):
    """Full bursts only: the packets behind the last full batch wait for the
    flush source node (max_delay), then leave in order. Pipelined, the source
    node also hands back the last batch the GPU finished."""
    t = T.config_single_route()
    n = BATCH + 2 * BURST
    fr, me = S.stream(n, 0xB0D, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    c0 = node_counters("gpu_fwd4_flush")
    check_walk(t, fr, me)
    c = node_counters("gpu_fwd4_flush")
    assert c[2] - c0[2] >= 2 * BURST  # the flush node handed those packets on


@pytest.mark.gpu
def test_graph_walk_two_gpus():
    """grout's multi-worker, multi-GPU shape: the module opens one context
    per configured GPU (here two on the box's one device), worker graphs bind
    to them least-loaded on their NUMA socket, every control-plane change is
    applied to all of them (gpu_fwd4_* fan-out), and each worker graph
    forwards bit-exact on its own GPU."""
    L = lib()
    fp = graph_ctx()
    assert L.gh_n_ctx() == len(DEVS)
    assert L.gh_graph_use(0) == 0 and L.gh_graph_gpu() == 0
    k = L.gh_graph_create(1, 0)  # a second worker, cpu 1
    assert k == 1 and L.gh_graph_gpu() == 1
    try:
        t = T.config_fullview(count=50_000)
        fr, me = S.stream(20_000, 0xB1E, routes=t.route_array())
        for g in (0, 1):
            assert L.gh_graph_use(g) == 0
            got = check_walk(t, fr, me)
            assert (got["edge"] == abi.EDGE["port_output"]).mean() > 0.99
        # a route change reaches both contexts: a /32 of the stream moves
        # to another nexthop, both workers forward it there
        from grout_amd.fwd import FastPath
        dst = int.from_bytes(bytes(fr[0, 30:34]), "big")
        nh_new = int(t.route_array()["nh"][1])
        r = np.zeros(1, dtype=abi.ROUTE_DT)
        r[0] = (dst, 32, 0, 1, nh_new)
        fp.route_add(r, replace=True)
        fp.fib_commit(1)
        for i in range(L.gh_n_ctx()):
            h = FastPath.borrow(L.gh_ctx_at(i))
            assert h.fib_lookup(1, dst) == nh_new
        _gh["state"]["key"] = None  # the topology changed under fresh_fastpath_state: reload
    finally:
        assert L.gh_graph_use(1) == 0
        assert L.gh_graph_destroy() == 0
        L.gh_graph_use(0)


@pytest.mark.gpu
def test_graph_workers_recycled_mbufs():
    """The workers mode tools/node_workers.py measures: two worker graphs
    walked from their own threads at once, each over its share of the
    stream. With gh_set_recycle every worker's packets go through a small
    mempool of its own (port_rx refills an mbuf from the stream when the
    recorder behind the edge gives it back, as port_tx frees them), a pool
    smaller than a batch included (the flush node sends partial batches):
    every edge takes the same number of packets as with one mbuf per packet,
    and `passes` times as many when each worker goes over its share again."""
    L = lib()
    L.gh_workers_run.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.gh_set_recycle.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.gh_set_recycle.restype = None
    fp = graph_ctx()
    t = T.config_fullview(count=20_000)
    load(fp, t)
    assert L.gh_graph_create(1, 0) == 1
    fr, me = S.stream(3 * BATCH + 777, 0xB1F, routes=t.route_array())
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    names = [rec_name(e) for e in range(abi.E_COUNT)]

    def edge_counts():
        c = np.zeros(abi.E_COUNT, dtype=np.int64)
        for g in (0, 1):
            assert L.gh_graph_use(g) == 0
            c += [int(node_counters(x)[0]) for x in names]
        return c

    def run(pool, passes=1):
        L.gh_set_recycle(pool, passes)
        try:
            assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, len(me)) == 0
            c0 = edge_counts()
            s, w = ctypes.c_double(), ctypes.c_uint64()
            assert L.gh_workers_run(2, ctypes.byref(s), ctypes.byref(w)) == 0
            assert s.value > 0 and w.value > 0
            return edge_counts() - c0
        finally:
            L.gh_set_recycle(0, 1)

    try:
        want = run(0)
        assert want.sum() == len(me) and want[abi.EDGE["port_output"]] > 0.9 * len(me)
        for pool in (len(me) // 2, 1000):  # a batch and a half, a quarter batch
            got = run(pool)
            assert (got == want).all(), (pool, got, want)
        assert (run(1000, passes=3) == 3 * want).all()  # each share three times over
        L.gh_set_recycle(len(me), 1)  # two pools of the whole stream: more mbufs than loaded
        try:
            assert L.gh_workers_run(2, None, None) == -errno.EINVAL
        finally:
            L.gh_set_recycle(0, 1)
    finally:
        assert L.gh_graph_use(1) == 0
        assert L.gh_graph_destroy() == 0
        L.gh_graph_use(0)


@pytest.mark.gpu
def test_graph_walk_cpu_continuations():
    """The verdicts that stop at grout's conntrack / NAT hooks continue in
    the CPU nodes ip_input_local_ct (ip_input.c:166-187) and ip_output_snat
    (ip_output.c:108-153), in the graph, with grout's private data:
    a conntrack hit reaches dnat44_dynamic with its connection, a miss
    ip_input_local; a static SNAT rule rewrites the source (RFC 1624 checksum
    update) and the packet reaches eth_output with eth_output_mbuf_data set."""
    L = lib()
    fp = graph_ctx()
    t, nh = SC.corpus_topology()
    load(fp, t)
    fr, me, lab = SC.corpus_arrays()
    pick = [lab.index(x) for x in ("snat dyn local", "snat egress", "fwd 16.1.0.1")]
    fr, me = np.ascontiguousarray(fr[pick * 3]), np.ascontiguousarray(me[pick * 3])
    L.gh_policy_clear()
    # the local packet's flow, seen from the NATed side: a conntrack REV hit
    f = fr[0]
    ihl = (f[14] & 0xF) * 4
    key = np.zeros(2, dtype=CONN_KEY_DT)
    key[1] = (SC.SNATDYN, abi.AF_IP4, f[23], int.from_bytes(bytes(f[26:30]), "big"),
              int.from_bytes(bytes(f[30:34]), "big"), int.from_bytes(bytes(f[14 + ihl:16 + ihl]), "big"),
              int.from_bytes(bytes(f[16 + ihl:18 + ihl]), "big"))
    key[0] = key[1]
    key[0]["src"], key[0]["dst"] = key[1]["dst"], key[1]["src"]
    assert L.gh_conn_add(key[0:1].ctypes.data, key[1:2].ctypes.data) == 0
    src_be = bytes(fr[1, 26:30])
    to = bytes([100, 64, 99, 1])
    assert L.gh_snat44_static_add(SC.P3, int.from_bytes(src_be, "little"), int.from_bytes(to, "little")) == 0
    o_lines, o_v, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True)
    got, lines, _, _ = walk(fr, me)
    names = [rec_name(e) for e in got["edge"]]
    assert names == ["dnat44_dynamic", "eth_output", "port_output"] * 3
    # conntrack hit: the connection and its direction in conn_mbuf_data
    assert (got["conn"][0::3] == 1).all() and (got["flow"][0::3] == 1).all()  # CONN_FLOW_REV
    assert (got["data_off"][0::3] == want["data_off"][0::3]).all()  # after eth_input's adj
    # SNAT: the source rewritten, the header checksum still verifies, the rest
    # of the header as the GPU left it (TTL, the fast path's checksum update)
    s = lines[1::3]
    o = o_lines[1::3]
    assert (s[:, 26:30] == np.frombuffer(to, np.uint8)).all()
    for row in s:
        hdr = bytes(row[14:34])
        tot = sum(int.from_bytes(hdr[i:i + 2], "big") for i in range(0, 20, 2))
        while tot >> 16:
            tot = (tot & 0xFFFF) + (tot >> 16)
        assert tot == 0xFFFF
    assert (s[:, :24] == o[:, :24]).all() and (s[:, 30:] == o[:, 30:]).all()
    # eth_output_mbuf_data: the nexthop's MAC, IPv4, no vtep
    assert (got["eth_dst"][1::3] == np.frombuffer(T.mac_bytes("02:00:00:01:00:15"), np.uint8)).all()
    assert (got["eth_type"][1::3] == 0x0008).all() and (got["vtep_af"][1::3] == 0).all()
    assert (got["iface"][1::3] == SC.P3).all() and (got["packet_type"][1::3] == abi.PTYPE_L3_IPV4).all()
    # ip_output's return rule: the SNAT node counted what it sent to eth_output
    c = node_counters("ip_output_snat")
    assert c[2] >= 3
    # no conntrack entry, no rule: ip_input_local, eth_output with the source kept
    L.gh_policy_clear()
    got, lines, _, _ = walk(fr, me)
    assert [rec_name(e) for e in got["edge"]] == ["ip_input_local", "eth_output", "port_output"] * 3
    assert (lines[1::3] == o_lines[1::3]).all()


# ---------------------------------------------------------------------------
# GPU: the node against grout's RCU and rte_graph's stream limits
# ---------------------------------------------------------------------------
def _slot_of(topo, ipv4):
    nh = topo.nh[1:topo.n_nh + 1]
    return int(np.nonzero((nh["ipv4"] == T.ip4(ipv4)) & (nh["type"] == abi.NH_T["L3"]))[0][0]) + 1


@pytest.mark.gpu
@pytest.mark.parametrize("readers", [1, 0], ids=["qsbr_readers", "no_readers"])
def test_graph_walk_rcu_delete_in_flight(readers):
    """grout deletes a nexthop and its egress iface while a batch that names
    both is on the GPU (iface_destroy / nexthop_destroy, iface.c:702-725,
    nexthop.c:493-518: out of grout's tables, rte_rcu_qsbr_synchronize, then
    the REMOVE / DELETE events and the free). The worker keeps reporting
    quiescent (rte_rcu_qsbr_quiescent, main_loop.c:464). With the node's QSBR readers the
    synchronisation returns only once the batch has been handed back and
    through grout's nodes behind the edges, every packet reaches ip_hold with
    the live nexthop, and nothing freed is read. Without them (round 2's
    node, the negative control) the synchronisation returns while the batch
    is still on the GPU, and the hand-back finds the objects gone."""
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    gw = _slot_of(t, "172.16.0.2")  # 16.0.0.0/16 via 172.16.0.2, unresolved: ip_hold
    oif = int(t.nh[gw]["iface_id"])
    fr, me = S.stream(BATCH, 0xC0C, dst_range=(T.ip4("16.0.0.0"), T.ip4("16.0.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    res = np.zeros(1, dtype=RCU_RES_DT)
    L.gpu_fwd4_rcu_readers(readers)
    # the whole stream is one batch: only a full batch is sent (with DELAY_NS
    # a slow first walk on a fresh process could flush part of it, 2112 of
    # the 4096 packets, and the rest would start after the synchronize)
    assert L.gpu_fwd4_set_batch(BATCH, 10_000_000_000) == 0
    try:
        assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, len(me)) == 0
        assert L.gh_rcu_delete_test(gw, oif, 30, res.ctypes.data) == 0
    finally:
        L.gpu_fwd4_rcu_readers(1)
        assert L.gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0
    r = res[0]
    assert r["sync_done"] == 1 and r["recorded"] == BATCH, r
    if readers:
        assert r["sync_before_handback"] == 0, r
        assert r["recorded_at_sync"] == BATCH, r  # every packet through grout's nodes first
        assert r["freed_reads"] == 0 and r["stale"] == 0, r
        out = np.zeros(BATCH, dtype=OUT_DT)
        lines = np.zeros((BATCH, abi.LINE), dtype=np.uint8)
        assert L.gh_results(out.ctypes.data, lines.ctypes.data) == BATCH
        assert (out["edge"] == abi.EDGE["ip_hold"]).all()
        assert (out["nh"] == gw).all() and (out["iface"] == oif).all()
        assert walk_info()["readers_online"] <= 2  # released one walk after their hand-back
    else:
        assert r["sync_before_handback"] == 1, r
        assert r["stale"] == BATCH, r  # dropped at hand-back: the objects were gone


CHURN_BATCH = 256
CHURN_GPU_LOAD = 1 << 21
CHURN_DT = np.dtype([("cycles", "<u4"), ("commits", "<u4"), ("freed_reads", "<u4"), ("recorded", "<u4"),
                     ("stale", "<u8"), ("walks", "<u4"), ("err", "<u4"), ("inflight_moved", "<u4"),
                     ("inflight_cleared", "<u4")])
assert CHURN_DT.itemsize == 40


@pytest.mark.gpu
@pytest.mark.parametrize("readers,quiesce_each", [(1, 0), (1, 1), (0, 1)],
                         ids=["qsbr_readers", "qsbr_readers_quiesce_each_walk", "no_readers_quiesce_each_walk"])
def test_graph_walk_control_plane_churn(readers, quiesce_each):
    """A control thread cycles a nexthop out and back while the worker
    forwards 2^21 packets through it, over and over, as grout's
    nexthop_destroy orders it: its route moves to another nexthop and is
    published, rte_rcu_qsbr_synchronize, NEXTHOP_DELETE (the registry entry
    cleared), the object freed; then it is created again and the route comes
    back. The worker reports quiescent every 256 walks (and, the worst case
    for a reader held across walks, after every walk). With the node's QSBR
    readers every packet reaches ip_hold with one of the two live nexthops,
    none is dropped stale and nothing freed is read, across tens of
    cycles and their commits. Without them (the negative control) synchronize
    returns while batches naming the nexthop are still on the GPU, and the
    node drops those packets at hand-back instead (stale > 0); the registry
    check at hand-back cannot close the window in which the nexthop is freed
    right after it, so a few freed reads may happen too (round 5: 8 in one run,
    0 in the others) -- what the readers are for."""
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    a = t.add_nexthop(T.PORT_IFACE[1], "172.16.1.50")  # unresolved: ip_hold, the nexthop in l3_mbuf_data
    b = t.add_nexthop(T.PORT_IFACE[1], "172.16.1.51")
    r = t.route_array()
    k = int(np.nonzero((r["prefixlen"] == 16) & (r["ip"] == T.ip4("16.1.0.0")))[0][0])
    t.routes = [r[[i for i in range(len(r)) if i != k]]]
    t.add_route(T.VRF_MAIN, "16.1.0.0/16", a)
    load(fp, t)
    n = 1 << 21
    fr, me = S.stream(n, 0xC4C, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    res = np.zeros(1, dtype=CHURN_DT)
    L.gpu_fwd4_rcu_readers(readers)
    # batches of 4 RX bursts, sent every few walks, and another queue's
    # whole-GPU kernels back to back (another worker's load): the node's
    # batches wait behind them, so one sent before a publication is still on
    # the GPU when the synchronize after it starts. (With BATCH alone, one
    # batch every 64 walks on an idle GPU, that window was hit a few times per
    # run, in some runs never.)
    assert L.gpu_fwd4_set_batch(CHURN_BATCH, DELAY_NS) == 0
    L.gh_set_gpu_load(CHURN_GPU_LOAD)
    if not readers:
        # the negative control needs batches that wait behind the other
        # queue's kernels: one launch per batch (the resident kernel's batches
        # do not queue behind launches, so its window is rarely hit)
        fp.tune("resident", 0)
    try:
        assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, n) == 0
        ip_be = int.from_bytes(T.ip4("16.1.0.0").to_bytes(4, "big"), "little")
        assert L.gh_churn_test(ip_be, 16, T.VRF_MAIN, a, b, 50, quiesce_each, res.ctypes.data) == 0
    finally:
        L.gpu_fwd4_rcu_readers(1)
        fp.tune("resident", 1)  # the module's default
        L.gh_set_gpu_load(0)
        assert L.gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0
    c = res[0]
    print("churn", readers, quiesce_each, c)
    assert c["err"] == 0 and c["recorded"] == n and c["cycles"] >= 10, c
    if readers:  # nothing freed is ever handed to grout's nodes
        assert c["freed_reads"] == 0, c
    out = np.zeros(n, dtype=OUT_DT)
    lines = np.zeros((n, abi.LINE), dtype=np.uint8)
    assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
    dropped = out["edge"] == abi.EDGE["ip_output_error"]
    assert dropped.sum() == c["stale"], c
    held = out["edge"] == abi.EDGE["ip_hold"]
    assert (held | dropped).all()
    assert np.isin(out["nh"][held], [a, b]).all()
    if readers:
        assert c["stale"] == 0, c
        assert (out["nh"] == a).any() and (out["nh"] == b).any()
    else:
        assert c["stale"] > 0, c


@pytest.mark.gpu
def test_graph_walk_full_batches_under_stream_limit():
    """batch = 65536 with a 10 s hold: the node clamps it to
    GPU_FWD4_BATCH_MAX, fills whole batches, hands one back per process()
    call, and no node of the graph ever holds more than two batches plus a
    burst (rte_graph streams are uint16: the stand-in aborts past 65535, as
    DPDK's RTE_VERIFY does)."""
    L = lib()
    graph_ctx()
    assert L.gpu_fwd4_set_batch(1 << 16, 10_000_000_000) == 0
    try:
        t = T.config_single_route()
        n = 3 * BATCH_MAX + 1000  # three full batches, then a short RX burst flushes the rest
        fr, me = S.stream(n, 0xB2A, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
        i0 = walk_info()
        got = check_walk(t, fr, me)
        i1 = walk_info()
    finally:
        assert L.gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0
    assert (got["edge"] == abi.EDGE["port_output"]).all()
    assert i1["max_batch"] == BATCH_MAX
    assert i1["batches"] - i0["batches"] == 4
    hw = node_counters("port_output")[3]
    assert BATCH_MAX <= hw <= 2 * BATCH_MAX + 256, hw


@pytest.mark.gpu
def test_fanout_marks_diverged_context():
    """A control-plane call that fails on one GPU's context only (here a
    route into a VRF that context lacks) leaves that context's mirrors out of
    step: it is marked diverged and the graphs bound to it hand every packet
    to grout's CPU nodes, until the control plane has replayed the change
    into it and calls gpu_fwd4_resync(). The other context keeps forwarding."""
    from grout_amd.fwd import FastPath
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    assert L.gh_n_ctx() == 2
    vrf = 7
    h0, h1 = FastPath.borrow(L.gh_ctx_at(0)), FastPath.borrow(L.gh_ctx_at(1))
    h0.fib_create(vrf, 1024)
    k = L.gh_graph_create(2, 0)  # a worker graph on the least loaded context
    assert k > 0 and L.gh_graph_gpu() == 1
    try:
        r = np.zeros(1, dtype=abi.ROUTE_DT)
        r[0] = (T.ip4("10.9.0.0"), 16, 0, vrf, _slot_of(t, "172.16.1.2"))
        L.gpu_fwd4_route4_add.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        assert L.gpu_fwd4_route4_add(r.ctypes.data, 1, 1) < 0  # -ENONET on context 1 only
        assert L.gpu_fwd4_diverged(0) == 0 and L.gpu_fwd4_diverged(1) == 1
        assert walk_info()["diverged"] == 1
        fr, me = S.stream(3000, 0xD1F, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
        got, _, _, _ = walk(fr, me)
        assert (got["edge"] == abi.EDGE["punt"]).all()  # iface_input_cpu: grout's CPU nodes
        # the control plane replays the change into context 1, then resyncs it
        h1.fib_create(vrf, 1024)
        h1.route_add(r, replace=True)
        assert L.gpu_fwd4_resync(1) == 0 and L.gpu_fwd4_diverged(1) == 0
        got = check_walk(t, fr, me)
        assert (got["edge"] == abi.EDGE["port_output"]).all()
    finally:
        L.gpu_fwd4_resync(1)
        assert L.gh_graph_destroy() == 0
        L.gh_graph_use(0)
        for h in (h0, h1):
            try:
                h.fib_destroy(vrf)
            except Exception:
                pass


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [128, 256])
def test_graph_walk_long_bursts(burst):
    """port_rx bursts of 128 and 256 packets (grout's rx_burst_max /
    vector_max go up to 256, graph.c:612-650): one graph walk per burst, so
    the node's walks span several 64-packet tiles. eth_output's per-walk
    source-MAC cache (eth_output.c:37-59), the per-node calls and the iface
    counters follow grout over whole walks, against the oracle walking the
    same bursts: the cache walks (long ones included), and a stream."""
    L = lib()
    graph_ctx()
    assert L.gh_set_rx_burst(burst) == 0
    try:
        t, _ = SC.corpus_topology()
        fr, me, lab, _ = SC.eth_output_cache_arrays(walks=SC.ETH_OUTPUT_CACHE_WALKS + SC.ETH_OUTPUT_CACHE_LONG_WALKS)
        me = me.copy()
        me["vlan_ck"] &= 0xFFFF ^ abi.META_WALK  # the harness's walks are port_rx's bursts
        got = check_walk(t, fr, me, lab, burst=burst)
        assert (got["edge"] == abi.EDGE["eth_output_no_mac"]).sum() >= 10
        ts = T.config_single_route()
        fr, me = S.stream(20_011, 0xB0E, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
        got = check_walk(ts, fr, me, burst=burst)
        assert (got["edge"] == abi.EDGE["port_output"]).all()
    finally:
        assert L.gh_set_rx_burst(BURST) == 0


RELOAD_DT = np.dtype([("held", "<u4"), ("in_flight", "<u4"), ("left", "<i4"), ("recorded", "<u4"),
                      ("fini_freed", "<u8"), ("graph", "<i4"), ("rx", "<u4"), ("readers_online", "<u4"),
                      ("held_after", "<u4"), ("in_flight_after", "<u4"), ("_pad", "<u4")])
assert RELOAD_DT.itemsize == 48


def _reload(walks, drain):
    res = np.zeros(1, dtype=RELOAD_DT)
    L = lib()
    L.gh_reload_test.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    assert L.gh_reload_test(walks, drain, res.ctypes.data) == 0
    return res[0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["drained", "drained_leave", "not_drained"])
def test_graph_reload_mid_stream(mode):
    """grout reconfigures a worker mid-stream (worker_graph_reload,
    graph.c:263-290): the worker leaves its graph at a housekeeping tick
    (main_loop.c:466-470), the control plane gives it a new graph and
    destroys the old one. grout's nodes hold nothing across walks; the fast
    path's node holds the batch it accumulates (and one on the GPU). With
    the datapath patch the worker runs the datapath hooks' graph_leave first
    (the module's gpu_fwd4_drain), while port_rx keeps delivering the stream:
    every injected mbuf reaches grout's node behind its edge, bit-exact with
    the oracle, nothing is held or freed at the old graph's fini, and the
    node's QSBR readers are all offline. drained_leave: the drain's bound on
    batches handed back set to 0, so that it leaves the GPU at once: the
    batch on the GPU is handed back, the held batch and what RX brings in
    that walk go to grout's CPU nodes (iface_input_cpu) untouched, counted in
    the drain's return. Without the drain (the negative control) the held
    mbufs are freed at fini -- counted (gpu_fwd4_fini_freed), never handed on."""
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    n = 20_000
    fr, me = S.stream(n, 0xD7A, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    _, _, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True, burst=BURST)
    walks = 100  # 64 full bursts fill a batch (sent), 36 more are held
    drain = mode != "not_drained"
    L.gpu_fwd4_set_drain_bound.argtypes = [ctypes.c_int32]
    assert L.gpu_fwd4_set_batch(BATCH, 10_000_000_000) == 0  # no age flush: they stay held
    try:
        assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, n) == 0
        if mode == "drained_leave":
            assert L.gpu_fwd4_set_drain_bound(0) == 0
        r = _reload(walks, drain)
        assert L.gpu_fwd4_set_drain_bound(-1) == 0
        assert r["held"] == walks * BURST - BATCH and r["in_flight"] <= 1, r  # the sent batch may be back already
        if drain:
            assert r["fini_freed"] == 0 and r["held_after"] == 0 and r["in_flight_after"] == 0, r
            assert r["readers_online"] == 0, r  # the drain released the batches' QSBR readers
            # RX kept delivering through the drain, and everything it delivered
            # is through grout's nodes before the switch
            assert r["recorded"] == r["rx"] > walks * BURST, r
            if mode == "drained":
                assert r["left"] == 0, r
            else:  # the held batch + the drain walk's burst, to iface_input_cpu
                assert r["left"] == r["held"] + (r["rx"] - walks * BURST), r
        else:
            assert r["fini_freed"] >= r["held"], r
        w = L.gh_run(1 << 15)  # the new graph goes on with the stream
        assert (w > 0) if drain else (w < 0), w
        out = np.zeros(n, dtype=OUT_DT)
        lines = np.zeros((n, abi.LINE), dtype=np.uint8)
        assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
    finally:
        L.gpu_fwd4_set_drain_bound(-1)
        assert L.gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0
        _reload(0, 1)  # back to a graph in slot 0 for the other tests
        assert L.gh_graph_use(0) == 0
        _gh["state"]["key"] = None
    reached = out["edge"] != 0xFF
    if drain:
        assert reached.all()
    else:
        assert (~reached).sum() == r["fini_freed"], (int((~reached).sum()), r)
    punt = out["edge"] == abi.EDGE["punt"]
    if mode == "drained_leave":
        # the held mbufs and the drain walk's burst: right after the batch on the GPU
        lo = BATCH
        assert np.array_equal(np.nonzero(punt)[0], np.arange(lo, lo + r["left"]))
        assert (out["data_off"][punt] == 128).all()  # as port_rx left them
        assert np.array_equal(lines[punt], fr[punt][:, :abi.LINE])  # frames untouched
    else:
        assert not punt.any()
    fwd = reached & ~punt
    # every other packet leaves on port_output, whose private data is
    # iface_output's vlan_id (over the l3 nexthop's bytes, check_walk)
    assert (out["edge"][fwd] == abi.EDGE["port_output"]).all()
    for f in ("edge", "pkt_len", "data_len", "data_off", "iface", "vlan_id"):
        assert np.array_equal(out[f][fwd], want[f][fwd]), f


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["drained", "drained_leave", "not_drained"])
def test_graph_reload_deep_pipeline(mode):
    """The reload above with depth 4 and 512-packet batches: up to three
    batches on the GPU and one accumulating when the worker leaves its graph.
    Drained, every mbuf reaches grout's node behind its edge in RX order,
    bit-exact, nothing held or freed, no QSBR reader online; drained_leave,
    every batch on the GPU is handed back first (oldest first), then the held
    one and the drain walk's burst go to grout's CPU nodes untouched, right
    after them; not drained, fini frees (and counts) the held and the
    in-flight mbufs, after the GPU is done with them."""
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    n, batch, walks = 20_000, 512, 100
    fr, me = S.stream(n, 0xD7B, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    _, _, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True, burst=BURST)
    sent = walks * BURST // batch * batch  # 12 full batches sent, 256 packets held
    drain = mode != "not_drained"
    L.gpu_fwd4_set_drain_bound.argtypes = [ctypes.c_int32]
    assert L.gpu_fwd4_set_depth(4) == 0
    assert L.gpu_fwd4_set_batch(batch, 10_000_000_000) == 0  # no age flush: the rest stays held
    try:
        assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, n) == 0
        if mode == "drained_leave":
            assert L.gpu_fwd4_set_drain_bound(0) == 0
        r = _reload(walks, drain)
        assert L.gpu_fwd4_set_drain_bound(-1) == 0
        assert r["held"] == walks * BURST - sent and r["in_flight"] <= 3, r
        if drain:
            assert r["fini_freed"] == 0 and r["held_after"] == 0 and r["in_flight_after"] == 0, r
            assert r["readers_online"] == 0, r
            assert r["recorded"] == r["rx"] > walks * BURST, r
            if mode == "drained":
                assert r["left"] == 0, r
            else:
                assert r["left"] == r["held"] + (r["rx"] - walks * BURST), r
        else:
            assert r["fini_freed"] == r["held"] + r["in_flight"] * batch, r  # held + every batch on the GPU
        w = L.gh_run(1 << 15)
        assert (w > 0) if drain else (w < 0), w
        out = np.zeros(n, dtype=OUT_DT)
        lines = np.zeros((n, abi.LINE), dtype=np.uint8)
        assert L.gh_results(out.ctypes.data, lines.ctypes.data) == n
    finally:
        L.gpu_fwd4_set_drain_bound(-1)
        assert L.gpu_fwd4_set_depth(0) == 0
        assert L.gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0
        _reload(0, 1)
        assert L.gh_graph_use(0) == 0
        _gh["state"]["key"] = None
    reached = out["edge"] != 0xFF
    if drain:
        assert reached.all()
    else:
        assert (~reached).sum() == r["fini_freed"], (int((~reached).sum()), r)
    punt = out["edge"] == abi.EDGE["punt"]
    if mode == "drained_leave":
        assert np.array_equal(np.nonzero(punt)[0], np.arange(sent, sent + r["left"]))
        assert (out["data_off"][punt] == 128).all()
        assert np.array_equal(lines[punt], fr[punt][:, :abi.LINE])
    else:
        assert not punt.any()
    fwd = reached & ~punt
    assert (out["edge"][fwd] == abi.EDGE["port_output"]).all()
    for f in ("edge", "pkt_len", "data_len", "data_off", "iface", "vlan_id"):
        assert np.array_equal(out[f][fwd], want[f][fwd]), f


@pytest.mark.gpu
def test_graph_walk_append_failure_punts_one_walk():
    """A graph walk the node cannot stage (gr_hip_node_append fails, e.g. no
    pinned memory to grow the walk slot; the slot is left as it was) goes to
    grout's CPU nodes at once (iface_input_cpu), untouched, and is counted
    (walk_info append_errors). The batch keeps the walks before and after
    it, which forward bit-exact with the oracle (the whole batch
    used to be refused at send)."""
    L = lib()
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    fr, me = S.stream(3000, 0xA9F, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    _, _, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True, burst=BURST)
    i0 = walk_info()
    L.gpu_fwd4_tune.argtypes = [ctypes.c_char_p, ctypes.c_int]
    assert L.gpu_fwd4_tune(b"fail_appends", 1) == 0  # the next append of each context fails
    try:
        got, lines, _, _ = walk(fr, me)
    finally:
        assert L.gpu_fwd4_tune(b"fail_appends", 0) == 0
    assert walk_info()["append_errors"] - i0["append_errors"] == 1
    punt = got["edge"] == abi.EDGE["punt"]
    assert punt[:BURST].all() and punt.sum() == BURST  # the first walk, whole
    assert (got["data_off"][punt] == 128).all() and (got["pkt_len"][punt] == me["pkt_len"][punt]).all()
    assert (lines[punt] == fr[punt, :abi.LINE]).all()  # frames untouched
    assert (got["edge"][~punt] == abi.EDGE["port_output"]).all()  # vlan_id: what port_output reads
    for f in ("edge", "pkt_len", "data_len", "data_off", "iface", "vlan_id"):
        assert np.array_equal(got[f][~punt], want[f][~punt]), f


def test_chain_graph_matches_oracle():
    """The like-for-like measurement's CPU side (tests/perf_node_chain.py):
    a worker graph with grout's CPU chain in the GPU node's place (the
    harness's cpu_chain node over the oracle's or_walk_frames) leaves every
    mbuf of the exception corpus and of a full-view stream -- edge, lengths,
    data_off, packet_type, egress iface, frame bytes -- as the oracle's
    mbuf-level chain does. Run in a process of its own: it initialises the
    harness without a GPU."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "perf_node_chain.py"), "--check"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"check": "ok"' in r.stdout


# ---------------------------------------------------------------------------
# grout's idle logic: the worker sleeps or blocks only when the node holds
# nothing (the holding hook, integration/grout-gpu_fwd4-datapath.patch)
# ---------------------------------------------------------------------------
def _loop(max_sleep_us=0, adaptive=0, ignore_holding=0, block_ms=1000, idle_windows=4, max_walks=50_000_000):
    r = np.zeros(1, dtype=LOOP_RES_DT)
    assert lib().gh_loop_test(max_sleep_us, adaptive, ignore_holding, block_ms, idle_windows, max_walks,
                              r.ctypes.data) == 0
    return r[0]


def _burst_then_silence(n=BATCH_MAX, seed=0x1D1E):
    """One burst of n packets (one full batch: sent when full, then on the GPU
    while RX is quiet), then silence; the oracle's edges for them."""
    fp = graph_ctx()
    t = T.config_single_route()
    load(fp, t)
    fr, me = S.stream(n, seed, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    want = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True, burst=BURST)[3]
    L = lib()
    # no age flush that waits for the GPU inside a walk: the batch is in
    # flight across housekeeping windows, as with a long max_delay_ns
    assert L.gpu_fwd4_set_batch(BATCH_MAX, 20_000_000) == 0
    assert L.gh_load(fr.ctypes.data, fr.shape[1], me.ctypes.data, n) == 0
    _burst_then_silence.keep = (fr, me)  # port_rx reads them while the test walks (gh_load keeps pointers)
    return fp, n, want


def _results(n):
    out = np.zeros(n, dtype=OUT_DT)
    lines = np.zeros((n, abi.LINE), dtype=np.uint8)
    assert lib().gh_results(out.ctypes.data, lines.ctypes.data) == n
    return out


def _restore_batch():
    assert lib().gpu_fwd4_set_batch(BATCH, DELAY_NS) == 0


@pytest.mark.gpu
def test_idle_loop_adaptive_irq_blocks_only_when_nothing_held():
    """Adaptive-IRQ mode (main_loop.c:478-497): one burst, then silence. By
    the time the worker blocks every mbuf is through grout's nodes
    (bit-exact with the oracle), the node's QSBR readers are offline, and a
    control thread's rte_rcu_qsbr_synchronize returns while the worker is
    blocked (the windows the holding hook keeps busy: the deadline test
    below, where the batch is kept on the GPU)."""
    fp, n, want = _burst_then_silence()
    try:
        r = _loop(adaptive=1, block_ms=2000)
    finally:
        _restore_batch()
    assert r["blocked"] == 1, r
    assert r["recorded_at_block"] == n and r["held_at_block"] == 0, r
    assert r["readers_online_at_block"] == 0, r
    assert r["sync_returned"] == 1, r
    got = _results(n)
    bad = np.nonzero(got["edge"] != want["edge"])[0]
    err = ctypes.c_uint64()
    assert lib().gh_node_stats(None, ctypes.byref(err)) == 0
    assert len(bad) == 0, dict(bad=len(bad), first=bad[:4].tolist(), last=bad[-4:].tolist(),
                               got=np.bincount(got["edge"][bad]).nonzero()[0].tolist(), info=walk_info(),
                               gpu_errors=err.value,
                               cancels=abi.hip().gr_hip_tune(lib().gh_hip_ctx(), b"resident_cancels", 0), r=r)
    assert np.array_equal(got["iface"], want["iface"])


@pytest.mark.gpu
def test_idle_loop_deep_pipeline():
    """The adaptive-IRQ loop with depth 4 and 2048-packet batches: when RX
    goes quiet up to three batches are on the GPU and one accumulating; the
    holding hook counts them all, so the worker blocks only once every mbuf
    is through grout's nodes, bit-exact and in order, and every QSBR reader
    is offline."""
    L = lib()
    fp, n, want = _burst_then_silence(n=8 * 2048 + 100, seed=0x1D23)
    assert L.gpu_fwd4_set_depth(4) == 0
    assert L.gpu_fwd4_set_batch(2048, 20_000_000) == 0
    try:
        r = _loop(adaptive=1, block_ms=2000)
    finally:
        assert L.gpu_fwd4_set_depth(0) == 0
        _restore_batch()
    assert r["blocked"] == 1, r
    assert r["recorded_at_block"] == n and r["held_at_block"] == 0, r
    assert r["readers_online_at_block"] == 0 and r["sync_returned"] == 1, r
    got = _results(n)
    assert np.array_equal(got["edge"], want["edge"])
    assert np.array_equal(got["iface"], want["iface"])


@pytest.mark.gpu
def test_idle_loop_without_holding_blocks_with_a_batch_on_the_gpu():
    """The same loop as grout runs it without the hook (the negative
    control): the resident kernel held back (knob "resident_hold") keeps the
    batch on the GPU, the worker blocks after two idle windows with the batch
    and its QSBR reader online, and the synchronize does not return while it
    is blocked. After the wakeup the batch's deadline ("resident_wait_ms")
    retires it: its packets go to grout's CPU nodes and the synchronize
    returns."""
    fp, n, _ = _burst_then_silence(seed=0x1D1F)
    fp.tune("resident_wait_ms", 400)
    fp.tune("resident_hold", 1)
    try:
        r = _loop(adaptive=1, ignore_holding=1, block_ms=100)
    finally:
        fp.tune("resident_hold", 0)
        fp.tune("resident_wait_ms", 500)
        _restore_batch()
    assert r["blocked"] == 1, r
    assert r["recorded_at_block"] < n and r["held_at_block"] > 0, r
    assert r["readers_online_at_block"] > 0, r
    assert r["sync_returned"] == 0, r
    assert lib().gh_run(1 << 20) > 0  # everything through after the wakeup
    assert walk_info()["readers_online"] == 0


@pytest.mark.gpu
def test_idle_loop_resident_deadline_punts_and_counts():
    """A resident kernel that stops serving its rings (knob "resident_hold":
    it leaves and is not relaunched): the node's walks return, the batch is
    retired at its deadline ("resident_wait_ms", measured from the post) and
    every one of its mbufs goes to grout's CPU nodes (iface_input_cpu)
    untouched, counted in the node's gpu_errors and the library's
    "resident_cancels"; then the worker idles and blocks with nothing held.
    Afterwards the kernel is launched again and the GPU forwards as before."""
    fp, n, want = _burst_then_silence(seed=0x1D20)
    L = lib()
    hip = abi.hip()
    ctx = L.gh_hip_ctx()
    c0 = hip.gr_hip_tune(ctx, b"resident_cancels", 0)
    err0 = ctypes.c_uint64()
    assert L.gh_node_stats(None, ctypes.byref(err0)) == 0
    fp.tune("resident_wait_ms", 200)
    fp.tune("resident_hold", 1)
    try:
        r = _loop(adaptive=1, block_ms=2000)
    finally:
        fp.tune("resident_hold", 0)
        fp.tune("resident_wait_ms", 500)
        _restore_batch()
    assert r["blocked"] == 1 and r["recorded_at_block"] == n, r
    assert r["readers_online_at_block"] == 0 and r["sync_returned"] == 1, r
    assert r["busy_held"] > 0, r  # windows with nothing counted, the batch on the GPU: not idle
    assert 200_000 <= r["elapsed_us"] < 3_000_000, r  # past the deadline, well within grout's 5 s
    got = _results(n)
    punt = got["edge"] == abi.EDGE["punt"]
    assert punt.sum() >= BATCH_MAX, int(punt.sum())  # the retired batch, untouched
    ok = ~punt
    assert np.array_equal(got["edge"][ok], want["edge"][ok])
    assert (got["data_off"][punt] == 128).all()  # as port_rx left them (RTE_PKTMBUF_HEADROOM)
    err = ctypes.c_uint64()
    assert L.gh_node_stats(None, ctypes.byref(err)) == 0
    assert err.value > err0.value
    assert hip.gr_hip_tune(ctx, b"resident_cancels", 0) > c0
    assert walk_info()["stranded"] == 0
    # the kernel serves batches again
    check_walk(T.config_single_route(), *S.stream(5000, 0x1D21, dst_range=(T.ip4("16.1.0.0"),
                                                                          T.ip4("16.1.255.255"))))


@pytest.mark.gpu
@pytest.mark.parametrize("ignore_holding", [0, 1], ids=["holding", "no_holding"])
def test_idle_loop_micro_sleep(ignore_holding):
    """Micro-sleep mode (main_loop.c:499-509, max_sleep_us from port.c:833-878):
    with the hook no window sleeps while the node holds packets; without it
    (the batch kept on the GPU by "resident_hold" until its deadline) the
    worker sleeps with the batch held."""
    fp, n, want = _burst_then_silence(seed=0x1D22 + ignore_holding)
    if ignore_holding:
        fp.tune("resident_wait_ms", 200)
        fp.tune("resident_hold", 1)
    try:
        r = _loop(max_sleep_us=20, ignore_holding=ignore_holding, idle_windows=8)
    finally:
        fp.tune("resident_hold", 0)
        fp.tune("resident_wait_ms", 500)
        _restore_batch()
    assert r["recorded"] == n, r
    if ignore_holding:
        assert r["sleeps_held"] > 0, r
    else:
        assert r["sleeps_held"] == 0 and r["busy_held"] > 0, r
        assert r["readers_online_at_block"] == 0, r
        got = _results(n)
        assert np.array_equal(got["edge"], want["edge"])


@pytest.mark.gpu
def test_latency_budget_picks_the_depth():
    """gpu_fwd4_conf.depth 0 (the default): two batches per graph in flight,
    and GR_HIP_NODE_DEPTH under a latency budget of 75 us or less, with the
    resident kernel's ring rotation on; a depth set by hand
    wins. Bit-exact walks either way."""
    L = lib()
    L.gpu_fwd4_set_latency_budget.argtypes = [ctypes.c_uint64]
    fp = graph_ctx()
    t = T.config_single_route()
    fr, me = S.stream(3 * BATCH_MAX, 0x1A7C, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    hip, ctx = abi.hip(), L.gh_hip_ctx()
    assert L.gpu_fwd4_set_depth(0) == 0
    try:
        assert walk_info()["depth"] == 2 and hip.gr_hip_tune(ctx, b"resident_rotating", 0) == 0
        assert L.gpu_fwd4_set_batch(BATCH_MAX, 20_000_000) == 0
        assert L.gpu_fwd4_set_latency_budget(50_000) == 0
        assert walk_info()["depth"] == abi.NODE_DEPTH and hip.gr_hip_tune(ctx, b"resident_rotating", 0) == 1
        check_walk(t, fr, me)
        assert walk_info()["batch_cap"] < BATCH_MAX
        assert L.gpu_fwd4_set_depth(2) == 0  # by hand: no longer the budget's
        assert walk_info()["depth"] == 2 and hip.gr_hip_tune(ctx, b"resident_rotating", 0) == 0
        assert L.gpu_fwd4_set_depth(0) == 0
        assert L.gpu_fwd4_set_latency_budget(100_000) == 0
        assert walk_info()["depth"] == 2 and hip.gr_hip_tune(ctx, b"resident_rotating", 0) == 0
    finally:
        assert L.gpu_fwd4_set_latency_budget(0) == 0
        assert L.gpu_fwd4_set_depth(0) == 0
        _restore_batch()


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [2, 3], ids=["depth2", "depth3"])
def test_latency_budget_sizes_batches(depth):
    """gpu_fwd4_set_latency_budget: under a 100 us budget the graph's batches
    are sized by what their oldest packets took (arrival to hand-back), not by
    the 15360 of gpu_fwd4_set_batch: the cap stays within a few thousand
    packets, and the walk is bit-exact with the oracle as ever (also with two
    batches on the GPU while the next accumulates)."""
    L = lib()
    graph_ctx()
    assert L.gpu_fwd4_set_depth(depth) == 0
    L.gpu_fwd4_set_latency_budget.argtypes = [ctypes.c_uint64]
    fp = graph_ctx()
    t = T.config_single_route()
    fr, me = S.stream(8 * BATCH_MAX, 0x1A7B, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    assert L.gpu_fwd4_set_batch(BATCH_MAX, 20_000_000) == 0
    assert L.gpu_fwd4_set_latency_budget(100_000) == 0
    try:
        i0 = walk_info()
        check_walk(t, fr, me)
        i1 = walk_info()
    finally:
        assert L.gpu_fwd4_set_latency_budget(0) == 0
        assert L.gpu_fwd4_set_depth(0) == 0
        _restore_batch()
    assert 64 <= i1["batch_cap"] <= 4096, i1
    assert i1["max_batch"] <= 4096 + BURST or i1["batches"] - i0["batches"] >= len(me) // 4096, i1
    assert 0 < i1["lat_ns"], i1
