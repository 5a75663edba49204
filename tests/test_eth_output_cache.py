# SPDX-License-Identifier: BSD-3-Clause
"""eth_output's per-walk source-MAC cache (eth_output.c:37-59).

grout looks the source MAC up only when a packet's iface differs from the
last one looked up in the graph walk; a failed lookup (eth_output_no_mac)
zeroes the cached MAC but keeps last_iface_id. So in a walk [X ok, Y no MAC,
X], the third packet is forwarded with source MAC 00:00:00:00:00:00.

The expectations in scenarios.ETH_OUTPUT_CACHE_WALKS are derived by hand from
eth_output.c and rte_graph's pending-queue order; the CPU test pins the
oracle to them, the GPU tests hold the kernel (device batch, walk marks inside
tiles) and the rte_graph node (walks laid out on tiles, padded) to the
oracle bit for bit."""
import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import abi

IFACE_OUT = {abi.EDGE[e] for e in ("port_output", "iface_output_admin_down", "iface_output_vlan_no_parent",
                                   "iface_output_inval_type", "bond_output", "vxlan_output")}


def _src_mac(lines):
    return lines[:, 6:12]


def test_oracle_follows_eth_output_cache():
    t, _ = SC.corpus_topology()
    fr, me, lab, zero = SC.eth_output_cache_arrays()
    lines, v, _ = oracle.Oracle(t).process(fr, me)
    passed = np.isin(v["edge"], list(IFACE_OUT))
    assert passed[zero].all(), "a zero-MAC packet must still go out"
    src = _src_mac(lines)
    assert (src[zero] == 0).all(), [lab[i] for i in np.nonzero(zero & (src != 0).any(axis=1))[0]]
    ok = passed & ~zero
    # everyone else that passed eth_output carries its iface's MAC
    assert (src[ok] != 0).any(axis=1).all(), [lab[i] for i in np.nonzero(ok & (src == 0).all(axis=1))[0]]
    nomac = v["edge"] == abi.EDGE["eth_output_no_mac"]
    assert nomac.sum() >= 10
    # walk marks matter: the same packets as one long walk per 64 differ
    me2 = me.copy()
    me2["vlan_ck"] &= 0xFFFF ^ abi.META_WALK
    lines2, _, _ = oracle.Oracle(t).process(fr, me2)
    assert not np.array_equal(lines2, lines)


def test_oracle_mbuf_walks_match_batch_walks():
    """The same walks given as node mbuf walks (OR_F_MBUF_WALKS, where a walk
    may straddle a multiple of 64) give the same packets out as the batch
    (every walk here is laid out inside a tile by padding)."""
    t, _ = SC.corpus_topology()
    fr, me, lab, zero = SC.eth_output_cache_arrays()
    o = oracle.Oracle(t)
    _, v_b, _ = o.process(fr, me)
    lines_m, v_m, _, mb, _ = o.process_mbufs(fr, me)
    assert np.array_equal(v_b, v_m)
    assert (_src_mac(lines_m)[zero] == 0).all()


def test_oracle_long_walks():
    """Walks of up to 256 packets (grout's maximum burst, graph.c:612-650): the
    oracle's node mbuf walks follow the hand-derived expectations across
    tiles, and the same packets cut into 64-packet walks differ."""
    t, _ = SC.corpus_topology()
    fr, me, lab, zero = SC.eth_output_cache_arrays(walks=SC.ETH_OUTPUT_CACHE_LONG_WALKS)
    o = oracle.Oracle(t)
    lines, v, _, _, _ = o.process_mbufs(fr, me, burst=256)
    passed = np.isin(v["edge"], list(IFACE_OUT))
    assert passed[zero].all()
    src = _src_mac(lines)
    assert (src[zero] == 0).all(), [lab[i] for i in np.nonzero(zero & (src != 0).any(axis=1))[0]]
    ok = passed & ~zero
    assert (src[ok] != 0).any(axis=1).all(), [lab[i] for i in np.nonzero(ok & (src == 0).all(axis=1))[0]]
    lines64, _, _, _, _ = o.process_mbufs(fr, me, burst=64)
    assert not np.array_equal(lines64, lines)


def test_layout_long_walks_start_on_tiles():
    """gr_hip_node_layout with walks up to 256: a walk longer than a tile
    starts on one, shorter ones never straddle one, order kept."""
    L = abi.hip()
    rng = np.random.default_rng(9)
    for burst in (256, 128, 100):
        n = 3000
        m = np.zeros(n, dtype=abi.MBUF_DT)
        m["flags"][rng.random(n) < 0.01] = abi.MBUF_F_WALK
        pos = np.zeros(n, dtype=np.uint32)
        staged = abi.check("gr_hip_node_layout", L.gr_hip_node_layout(m.ctypes.data, n, burst, pos.ctypes.data))
        assert staged == pos[-1] + 1 and (np.diff(pos.astype(np.int64)) >= 1).all()
        start, starts = 0, []
        for i in range(n):
            if i == 0 or m["flags"][i] or i - start == burst:
                start = i
                starts.append(i)
        bounds = starts + [n]
        assert max(b - a for a, b in zip(bounds[:-1], bounds[1:])) > 64
        for a, b in zip(bounds[:-1], bounds[1:]):
            assert np.array_equal(pos[a:b], np.arange(pos[a], pos[a] + b - a))
            if b - a > 64:
                assert pos[a] % 64 == 0, (burst, a, b)
            else:
                assert pos[a] // 64 == pos[b - 1] // 64, (burst, a, b)


def test_layout_pads_walks_onto_tiles():
    """gr_hip_node_layout: no walk straddles a multiple of 64, order kept."""
    L = abi.hip()
    rng = np.random.default_rng(7)
    for burst in (64, 20, 1):
        n = 1000
        m = np.zeros(n, dtype=abi.MBUF_DT)
        m["flags"][rng.random(n) < 0.05] = abi.MBUF_F_WALK
        pos = np.zeros(n, dtype=np.uint32)
        staged = abi.check("gr_hip_node_layout", L.gr_hip_node_layout(m.ctypes.data, n, burst, pos.ctypes.data))
        assert staged >= n and staged == pos[-1] + 1
        assert (np.diff(pos.astype(np.int64)) >= 1).all()
        # walk starts as gr_hip_node_layout defines them
        start, starts = 0, []
        for i in range(n):
            if i == 0 or m["flags"][i] or i - start == burst:
                start = i
                starts.append(i)
        bounds = starts + [n]
        for a, b in zip(bounds[:-1], bounds[1:]):
            assert pos[a] // 64 == pos[b - 1] // 64, (burst, a, b)
            assert np.array_equal(pos[a:b], np.arange(pos[a], pos[a] + b - a))


@pytest.mark.gpu
def test_gpu_device_batch_eth_output_cache(fastpath):
    from golden_util import run_gpu
    from test_gpu_parity import compare
    t, _ = SC.corpus_topology()
    fr, me, lab, zero = SC.eth_output_cache_arrays()
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g, lab)
    assert (_src_mac(g[0])[zero] == 0).all()
    # and shifted by 1..63 packets: walks cut by tile boundaries as well
    for shift in (1, 17, 63):
        fr2 = np.concatenate([np.repeat(fr[:1], shift, axis=0), fr])
        me2 = np.concatenate([np.repeat(me[:1], shift, axis=0), me])
        compare(oracle.Oracle(t).process(fr2, me2), run_gpu(fastpath, t, fr2, me2))


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 128, 256])
@pytest.mark.parametrize("ptrs", [1, 0])
def test_gpu_node_walks_eth_output_cache(fastpath, ptrs, burst):
    """The rte_graph node: mbufs flagged per walk (walks straddle multiples
    of 64 in mbuf order), padded onto tiles by the node, against the oracle's
    mbuf walks; with bursts of 128 and 256 also walks longer than a tile,
    whose eth_output cache the hand-back resolves."""
    from golden_util import fresh_fastpath_state
    from test_node_shim import compare_mbufs, mbufs_for
    t, _ = SC.corpus_topology()
    walks = SC.ETH_OUTPUT_CACHE_WALKS + ([] if burst == 64 else SC.ETH_OUTPUT_CACHE_LONG_WALKS)
    fr, me, lab, zero = SC.eth_output_cache_arrays(walks=walks)
    if burst < 256:  # walks cut at the burst: the hand-derived zeros of longer ones no longer hold
        longw = np.zeros(len(me), bool)
        i = 0
        for spec, _z in walks:
            while lab[i] == "pad":
                i += 1
            k = len(spec.split())
            longw[i:i + k] = k > burst
            i += k
        zero &= ~longw
    fr, me = np.concatenate([fr[:5], fr]), np.concatenate([me[:5], me])  # shift the walks off tile bounds
    zero = np.concatenate([np.zeros(5, bool), zero])
    lab = ["lead %d" % i for i in range(5)] + lab
    fresh_fastpath_state(fastpath, t)
    lines, v, st, want, ns_want = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True, burst=burst)
    bufs, m = mbufs_for(fr, me)
    m["flags"] = np.where(me["vlan_ck"] & abi.META_WALK, abi.MBUF_F_WALK, 0)
    L = fastpath.lib
    if ptrs:
        abi.check("gr_hip_host_register", L.gr_hip_host_register(fastpath.h, bufs.ctypes.data, bufs.nbytes))
    try:
        fastpath.tune("node_ptrs", ptrs)
        q = fastpath.queue()
        ns = q.node_process(m, burst=burst)
        assert q.unfinished == 0
        compare_mbufs(m, want, bufs, lines, lab)
        assert np.array_equal(ns["packets"], ns_want["packets"]) and np.array_equal(ns["calls"], ns_want["calls"])
        assert np.array_equal(q.stats(), st)
        assert (bufs[zero, 6:12] == 0).all()
        q.close()
    finally:
        fastpath.tune("node_ptrs", 0)  # the default
        if ptrs:
            abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fastpath.h, bufs.ctypes.data))
