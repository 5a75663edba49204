# SPDX-License-Identifier: BSD-3-Clause
"""The resident kernel (knob "resident", fwd4_ring.hip gr_fwd4_resident):
node batches posted to descriptor rings in pinned host memory and taken by a
long-lived kernel instead of a launch each (gr_hip.cpp res_post). Every test
here is a node test of test_node_shim.py / test_graph_walk.py run through it:
the same mbufs, lines, verdicts and counters as the oracle (the counters are
the hand-back's: the resident kernel counts none), plus what is its own: a
kernel that left (lifetime over) is relaunched and resumes the ring, a kernel
that gives up hands back what it did not reach, FIB publications and quiesce
wait for the batches posted before them."""
import time

import numpy as np
import pytest

import oracle
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T
from test_node_shim import compare_mbufs, mbufs_for


@pytest.fixture
def resident(fastpath):
    assert fastpath.tune("resident", 1) == 0
    yield fastpath
    fastpath.tune("resident", 0)
    fastpath.tune("resident_ms", 50)


def _pipelined(fp, q, m, cuts):
    """Walks [cuts[i], cuts[i+1]) started two at a time, finished in order."""
    parts = [m[a:b] for a, b in zip(cuts, cuts[1:])]
    tot = np.zeros(1, dtype=abi.NODE_STATS_DT)[0]
    q.node_start(parts[0])
    for k in range(1, len(parts) + 1):
        if k < len(parts):
            q.node_start(parts[k])
        got, ns = q.node_finish()
        assert got is parts[k - 1] and q.unfinished == 0
        tot["packets"] += ns["packets"]
        tot["calls"] += ns["calls"]
    return tot


@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [0, 1], ids=["staged", "by_address"])
def test_resident_pipelined_walks(resident, ptrs):
    """Walks pipelined two deep through the resident kernel end as the oracle
    leaves them: mbufs, frames, node and per-iface counters."""
    from golden_util import fresh_fastpath_state
    fp = resident
    topo = T.config_fullview(count=100_000)
    fr, me = S.stream(50_000, 0xD1F, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    L = fp.lib
    if ptrs:
        abi.check("gr_hip_host_register", L.gr_hip_host_register(fp.h, bufs.ctypes.data, bufs.nbytes))
    q = fp.queue()
    try:
        fp.tune("node_ptrs", ptrs)
        launches0 = fp.tune("resident_launches")
        tot = _pipelined(fp, q, m, [0, 64, 64 * 100, 64 * 101, 64 * 400, 64 * 401 + 64, len(m)])
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(tot["packets"], ns_want["packets"])
        assert np.array_equal(tot["calls"], ns_want["calls"])
        assert np.array_equal(q.node_iface_stats(), st)
        assert not q.stats()["rx_packets"].any()  # nothing counted by a kernel
        assert fp.tune("resident_launches") >= max(launches0, 1)
    finally:
        fp.tune("node_ptrs", 0)
        if ptrs:
            abi.check("gr_hip_host_unregister", L.gr_hip_host_unregister(fp.h, bufs.ctypes.data))
        q.close()


@pytest.mark.gpu
def test_resident_relaunch(resident):
    """A 2 ms lifetime: between walks the idle kernel leaves; the next batch
    launches it again and its workgroup resumes the ring after the last seq
    done. Every walk is still the oracle's."""
    from golden_util import fresh_fastpath_state
    fp = resident
    assert fp.tune("resident_ms", 2) == 0
    topo = T.config_fullview(count=50_000)
    fr, me = S.stream(8 * 3000, 0xD20, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    q = fp.queue()
    try:
        l0 = fp.tune("resident_launches")
        for k in range(8):
            part = m[k * 3000:(k + 1) * 3000]
            q.node_start(part)
            got, _ = q.node_finish()
            assert got is part and q.unfinished == 0
            time.sleep(0.02)  # idle past the lifetime: the kernel leaves
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(q.node_iface_stats(), st)
        assert fp.tune("resident_launches") - l0 >= 4  # relaunched (at most once per walk)
    finally:
        q.close()


@pytest.mark.gpu
def test_resident_queue_joins_a_live_kernel(resident):
    """A queue that takes its rings while the kernel runs (the workgroups of
    rings nobody held left at once) makes it leave; its first batch launches
    one that serves it, and the first queue's batches go on through it."""
    from golden_util import fresh_fastpath_state
    fp = resident
    topo = T.config_fullview(count=50_000)
    fr, me = S.stream(4 * 5000, 0xD23, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    q1 = fp.queue()
    q2 = None
    try:
        q1.node_start(m[:5000])
        q1.node_finish()
        l0 = fp.tune("resident_launches")
        q2 = fp.queue()
        for q, part in ((q2, m[5000:10000]), (q1, m[10000:15000]), (q2, m[15000:])):
            q.node_start(part)
            got, _ = q.node_finish()
            assert got is part and q.unfinished == 0
        assert fp.tune("resident_launches") > l0  # relaunched for q2's rings
        compare_mbufs(m, want, bufs, lines)
    finally:
        q1.close()
        if q2 is not None:
            q2.close()


@pytest.mark.gpu
def test_resident_give_up_hands_back(resident):
    """A resident kernel that gives up (spin_max 1) reports it once (the
    queue's error word), and the node hands back what it finished and punts
    the rest untouched, as after a launch."""
    from golden_util import fresh_fastpath_state
    fp = resident
    topo = T.config_single_route()
    n = 1 << 16
    fr, me = S.stream(n, 0xD21, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    orig_bufs, orig_m = bufs.copy(), m.copy()
    q = fp.queue()
    try:
        assert fp.tune("spin_max", 1) == 0
        q.node_start(m)
        q.node_finish()
    finally:
        fp.tune("spin_max", 0)
    punt = m["edge"] == abi.EDGE["punt"]
    assert q.unfinished == punt.sum()
    assert np.array_equal(bufs[punt], orig_bufs[punt])
    orig_m["edge"] = abi.EDGE["punt"]
    assert np.array_equal(m[punt], orig_m[punt])
    done = ~punt
    compare_mbufs(m[done], want[done], bufs[done], lines[done])
    # the queue goes on: a normal walk after it
    q.node_start(m[:0])
    q.node_finish()
    q.close()


@pytest.mark.gpu
def test_resident_route_change_between_walks(resident):
    """A route committed while the queue's ring holds a batch: the batch
    posted before the commit reads the old FIB whole (the commit waits, on
    the host, for batches posted before the previous publication before it
    rewrites that copy), the walk after it the new one."""
    import copy
    from golden_util import fresh_fastpath_state
    fp = resident
    topo = T.config_fullview(count=20_000)
    fr, me = S.stream(20_000, 0xD22, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    dst = int.from_bytes(bytes(fr[0, 30:34]), "big")
    nh_new = int(topo.route_array()["nh"][1])
    r = np.zeros(1, dtype=abi.ROUTE_DT)
    r[0] = (dst, 32, 0, 1, nh_new)
    topo2 = copy.deepcopy(topo)
    topo2.routes.append(r)
    lines_a, _, _, want_a, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    lines_b, _, _, want_b, _ = oracle.Oracle(topo2).process_mbufs(fr, me, lines_only=True)
    assert not np.array_equal(lines_a, lines_b)  # the new route changes some packets
    bufs_a, m_a = mbufs_for(fr, me)
    bufs_b, m_b = mbufs_for(fr, me)
    q = fp.queue()
    try:
        q.node_start(m_a)  # on the GPU across the commit below
        fp.route_add(r, replace=True)
        fp.fib_commit(1)
        got, _ = q.node_finish()
        assert got is m_a and q.unfinished == 0
        compare_mbufs(m_a, want_a, bufs_a, lines_a)
        q.node_start(m_b)
        got, _ = q.node_finish()
        assert got is m_b and q.unfinished == 0
        compare_mbufs(m_b, want_b, bufs_b, lines_b)
    finally:
        q.close()
        import golden_util
        golden_util._loaded["key"] = None  # the FIB changed under fresh_fastpath_state: reload next time


@pytest.mark.gpu
@pytest.mark.parametrize("ptrs", [0, 1], ids=["staged", "by_address"])
def test_resident_graph_walk_corpus(ptrs):
    """Every edge, in whole rte_graph walks of the grout module's node, its
    batches through the resident kernel: grout's mbufs, node statistics and
    folded per-iface counters as the oracle's."""
    import test_graph_walk as G
    import scenarios as SC
    G.lib().gh_set_pin(1)
    fp = G.graph_ctx()
    fp.tune("resident", 1)  # the module's default
    fp.tune("node_ptrs", ptrs)
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    keep = ((me["vlan_ck"] >> 12) & 3) != 3
    fr, me, lab = fr[keep], me[keep], [x for x, k in zip(lab, keep) if k]
    try:
        got = G.check_walk(t, fr, me, lab)
    finally:
        fp.tune("node_ptrs", 0)
    assert len(set(got["edge"])) > 20


@pytest.mark.gpu
def test_resident_graph_control_plane_churn():
    """test_graph_walk's control-plane churn (nexthops and routes changed
    between and during walks, quiesce on every change) with the batches on the
    resident kernel: quiesce and the FIB publications wait for them."""
    import test_graph_walk as G
    fp = G.graph_ctx()
    fp.tune("resident", 1)  # the module's default
    G.test_graph_walk_control_plane_churn(1, 1)
    G.test_graph_walk_stream_batches(2)


@pytest.fixture
def knobs(resident):
    """The split knobs back at their defaults after the test."""
    yield resident
    resident.tune("resident_wgs", 8)
    resident.tune("resident_tiles", 8)
    resident.tune("resident_split", 0)
    resident.tune("resident_budget", 32)


@pytest.mark.gpu
@pytest.mark.parametrize("wgs,tiles,split,budget", [(1, 8, 0, 32), (2, 1, 0, 32), (3, 2, 0, 32), (8, 1, 0, 0),
                                                   (8, 1000, 0, 32), (8, 1, 5, 0), (8, 1, 0, 3), (4, 8, 0, 1)])
def test_resident_split_knobs(knobs, wgs, tiles, split, budget):
    """Ragged batches (1 to 15360 packets) split over every number of rings
    the knobs allow, one workgroup per `tiles` tiles up to the queue's `wgs`
    rings, at most `split`, at most `budget` over the busy queues (here one,
    two batches in flight): each walk as the oracle's, and the queue no longer
    busy after its last."""
    from golden_util import fresh_fastpath_state
    fp = knobs
    assert fp.tune("resident_wgs", wgs) == 0 and fp.tune("resident_tiles", tiles) == 0
    assert fp.tune("resident_split", split) == 0 and fp.tune("resident_budget", budget) == 0
    topo = T.config_fullview(count=50_000)
    sizes = [1, 63, 64, 65, 129, 640, 1000, 4097, 15360]
    fr, me = S.stream(sum(sizes), 0xD30 + wgs, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    q = fp.queue()
    try:
        tot = _pipelined(fp, q, m, list(np.cumsum([0] + sizes)))
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(tot["packets"], ns_want["packets"])
        assert np.array_equal(q.node_iface_stats(), st)
        assert not q.stats()["rx_packets"].any()  # every batch went to the resident kernel
        assert fp.tune("resident_busy") == 0
    finally:
        q.close()


def _deep(q, m, cuts, depth):
    """Walks [cuts[i], cuts[i+1]) with `depth` of them in flight, finished in order."""
    parts = [m[a:b] for a, b in zip(cuts, cuts[1:])]
    tot = np.zeros(1, dtype=abi.NODE_STATS_DT)[0]
    done = 0
    for k in range(len(parts) + depth):
        if k >= depth or k >= len(parts):
            if done < len(parts):
                got, ns = q.node_finish()
                assert got is parts[done] and q.unfinished == 0
                tot["packets"] += ns["packets"]
                tot["calls"] += ns["calls"]
                done += 1
        if k < len(parts):
            q.node_start(parts[k])
    assert done == len(parts)
    return tot


@pytest.mark.gpu
@pytest.mark.parametrize("wgs,budget", [(8, 32), (3, 32), (8, 2)])
def test_resident_rotate(knobs, wgs, budget):
    """Knob "resident_rotate" (the grout node's depth > 2): a batch of k
    rings posted while others of its queue are in flight runs on a group of
    k helper rings in turn, the first ring only waking them. Ragged batches,
    up to GR_HIP_NODE_DEPTH in flight, rotated over the helpers (those using
    every ring as usual): every walk as the oracle's, in start order, and
    the queue idle after its last."""
    from golden_util import fresh_fastpath_state
    fp = knobs
    assert fp.tune("resident_wgs", wgs) == 0 and fp.tune("resident_budget", budget) == 0
    assert fp.tune("resident_rotate", 1) == 0
    topo = T.config_fullview(count=50_000)
    sizes = [1, 63, 64, 65, 129, 512, 300, 64, 2000, 511, 7, 4097, 128, 256, 15360, 64, 64, 64, 1000, 33]
    fr, me = S.stream(sum(sizes), 0xD40 + wgs, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, ns_want = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    q = fp.queue()
    try:
        tot = _deep(q, m, list(np.cumsum([0] + sizes)), abi.NODE_DEPTH)
        compare_mbufs(m, want, bufs, lines)
        # (calls: ragged batches cut the oracle's 64-packet walks, as in test_resident_split_knobs)
        assert np.array_equal(tot["packets"], ns_want["packets"])
        assert np.array_equal(q.node_iface_stats(), st)
        assert not q.stats()["rx_packets"].any()  # every batch went to the resident kernel
        assert fp.tune("resident_busy") == 0
    finally:
        fp.tune("resident_rotate", 0)
        q.close()


@pytest.mark.gpu
def test_resident_rings_run_out(knobs):
    """A queue takes its rings on its first batch, as many as "resident_wgs"
    says then: groups of different sizes side by side (a group is taken only
    whole and free), and only while the device's CUs can hold every ring that
    queues of any context hold at once ("resident_cap", "resident_held": the
    graph-walk tests' module contexts on the same GPU hold some). Once no
    group of the current size is free, or the device is full, a queue's
    batches get a launch each (its kernel counters show it), and a queue
    closed hands its rings back. Every walk, on every queue, sequential or all
    queues in flight at once, is the oracle's."""
    from golden_util import fresh_fastpath_state
    fp = knobs
    topo = T.config_fullview(count=50_000)
    per = 1000
    fr, me = S.stream(per * 80, 0xD31, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    parts = [m[i * per:(i + 1) * per] for i in range(80)]

    def walk(q, part):
        q.node_start(part)
        got, _ = q.node_finish()
        assert got is part and q.unfinished == 0

    qs = []
    rings = fp.tune("resident_ring_count")
    assert rings >= 32 and rings % 8 == 0
    g8 = (rings - 24) // 8
    # the library's rule, simulated: first free aligned group of w in this
    # context, and the device's held rings + w within its cap
    taken = [False] * rings
    sim = {"held": None, "cap": None}

    def take(w):
        if sim["held"] + w > sim["cap"]:
            return -1
        for r in range(0, rings - w + 1, w):
            if not any(taken[r:r + w]):
                taken[r:r + w] = [True] * w
                sim["held"] += w
                return r
        return -1

    try:
        # of R rings: 0-3 (groups of 4), 8-15 (of 8: 0-7 is not free), 18-20
        # (of 3: 3-5, 6-8, 9-11, 12-14 and 15-17 are not), then 24-31, 32-39,
        # ..., R-8 - R-1 ((R - 24) / 8 groups of 8); 3 more queues find none
        # (fewer get rings when the device holds others' already)
        got_ring = []
        for i, w in enumerate([4, 8, 3] + [8] * (g8 + 3)):
            assert fp.tune("resident_wgs", w) == 0
            if i == 0:
                held0 = fp.tune("resident_held")
            qs.append(fp.queue())
            walk(qs[i], parts[i])
            if i == 0:  # the rings are set up by now
                sim["cap"] = fp.tune("resident_cap")
                sim["held"] = held0
                assert sim["cap"] > 0 and held0 + 4 <= sim["cap"], (held0, sim)
            got_ring.append(take(w))
        assert fp.tune("resident_held") == sim["held"], sim
        launched = [i for i, q in enumerate(qs) if q.stats()["rx_packets"].any()]
        assert launched == [i for i, r in enumerate(got_ring) if r < 0], (launched, got_ring, sim)
        if held0 == 0:  # the device to itself: the layout of the comment above
            assert launched == [3 + g8, 4 + g8, 5 + g8]
        nq = len(qs)
        for i, q in enumerate(qs):  # every queue in flight at once
            q.node_start(parts[nq + i])
        for i, q in enumerate(qs):
            got, _ = q.node_finish()
            assert got is parts[nq + i] and q.unfinished == 0
        compare_mbufs(m[:per * 2 * nq], want[:per * 2 * nq], bufs[:per * 2 * nq], lines[:per * 2 * nq])
        assert fp.tune("resident_busy") == 0
        assert all(qs[i].stats()["rx_packets"].sum() == 2 * per for i in launched)
        # rings 0-3 handed back: with 4-7, never taken, a group of 8 again
        # (if the device has room for 8 more)
        qs[0].close()
        taken[0:4] = [False] * 4
        sim["held"] -= 4
        qs[0] = fp.queue()
        x = 2 * nq
        walk(qs[0], parts[x])
        r0 = take(8)
        assert bool(qs[0].stats()["rx_packets"].any()) == (r0 < 0), (r0, sim)
        if sim["held"] - 8 + 8 <= sim["cap"] and r0 >= 0:
            assert r0 == 0
        compare_mbufs(parts[x], want[per * x:per * (x + 1)], bufs[per * x:per * (x + 1)], lines[per * x:per * (x + 1)])
    finally:
        for q in qs:
            q.close()


@pytest.mark.gpu
def test_resident_lifetime_is_idleness(resident):
    """The kernel leaves when no ring has finished a batch for the lifetime,
    not when one ring has been idle that long: a queue that holds its rings
    and posts nothing does not make the kernel leave under another queue's
    steady walks (no relaunch over ten lifetimes of them); once all are
    idle, it leaves and the next batch launches it again."""
    from golden_util import fresh_fastpath_state
    fp = resident
    assert fp.tune("resident_ms", 50) == 0
    topo = T.config_fullview(count=50_000)
    per = 4096
    fr, me = S.stream(per * 8, 0xD32, routes=topo.route_array())
    fresh_fastpath_state(fp, topo)
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    q1, q2 = fp.queue(), fp.queue()
    try:
        bufs, m = mbufs_for(fr[:per], me[:per])
        q2.node_start(m)  # q2 takes its rings, then stays idle
        q2.node_finish()
        q1.node_start(m)
        q1.node_finish()
        l0 = fp.tune("resident_launches")
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 0.5:  # ten lifetimes of steady walks on q1
            i = k % 8
            bufs, m = mbufs_for(fr[i * per:(i + 1) * per], me[i * per:(i + 1) * per])
            q1.node_start(m)
            got, _ = q1.node_finish()
            assert got is m and q1.unfinished == 0
            compare_mbufs(m, want[i * per:(i + 1) * per], bufs, lines[i * per:(i + 1) * per])
            k += 1
        assert k > 20
        # q2's idle first ring did not stop it (a kernel stopped by one idle ring
        # would relaunch about ten times here; up to two allows for host stalls
        # of a lifetime between walks on a busy box)
        l1 = fp.tune("resident_launches")
        assert l1 - l0 <= 2
        time.sleep(0.25)  # all idle: it leaves
        bufs, m = mbufs_for(fr[:per], me[:per])
        q2.node_start(m)
        q2.node_finish()
        compare_mbufs(m, want[:per], bufs, lines[:per])
        assert fp.tune("resident_launches") == l1 + 1
    finally:
        q1.close()
        q2.close()


@pytest.mark.gpu
def test_resident_deadline_and_dead_context():
    """The library's side of a resident batch past its deadline, on a context
    of its own. With the kernel stopped ("resident_hold") the walk's finish
    returns after "resident_wait_ms" with every packet not reached handed back
    as PUNT, its frame untouched (the batch's descriptors retired: nothing
    runs it later), counted in "resident_cancels"; released, the same queue
    forwards as the oracle's again. When the kernel would not even leave
    ("resident_leave_fail" stands for a workgroup no CU runs), the finish
    returns -EDEADLK without handing the walk back, the queue refuses every
    later walk (-EIO) and the context reports its resident path dead."""
    import errno
    from golden_util import fresh_fastpath_state
    from grout_amd.fwd import FastPath
    topo = T.config_fullview(count=50_000)
    fr, me = S.stream(4096, 0xDEAD, routes=topo.route_array())
    lines, v, st, want, _ = oracle.Oracle(topo).process_mbufs(fr, me, lines_only=True)
    fp = FastPath(0)
    try:
        fresh_fastpath_state(fp, topo, {})
        assert fp.tune("resident", 1) == 0 and fp.tune("resident_wait_ms", 100) == 0
        q = fp.queue()
        bufs, m = mbufs_for(fr, me)
        q.node_start(m)
        q.node_finish()  # the queue takes its rings, the kernel runs
        compare_mbufs(m, want, bufs, lines)
        fp.tune("resident_hold", 1)
        bufs, m = mbufs_for(fr, me)
        t0 = time.perf_counter()
        q.node_start(m)
        got, _ = q.node_finish()
        dt = time.perf_counter() - t0
        assert 0.09 <= dt < 2.0, dt
        assert q.unfinished == len(m)  # every packet: the kernel never started the batch
        assert (m["edge"] == abi.EDGE["punt"]).all() and (m["data_off"] == 128).all()
        assert np.array_equal(bufs[:, :abi.LINE], fr[:, :abi.LINE])  # frames untouched
        assert fp.tune("resident_cancels") == 1 and fp.tune("resident_dead") == 0
        fp.tune("resident_hold", 0)
        bufs, m = mbufs_for(fr, me)
        q.node_start(m)
        q.node_finish()
        compare_mbufs(m, want, bufs, lines)
        # the kernel would not leave
        fp.tune("resident_hold", 1)
        fp.tune("resident_leave_fail", 1)
        bufs, m = mbufs_for(fr, me)
        q.node_start(m)
        r = fp.lib.gr_hip_node_finish(q._h, None, None, None)
        assert r == -errno.EDEADLK, r
        assert fp.tune("resident_dead") == 1
        assert fp.lib.gr_hip_node_start(q._h, m.ctypes.data, len(m), 64) == -errno.EIO
    finally:
        fp.close()  # (the kernel has left: "resident_hold"; its rings are leaked, as for a real one)
