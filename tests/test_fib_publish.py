# SPDX-License-Identifier: BSD-3-Clause
"""Double-buffered FIB publication (gr_hip_fib4_commit).

Each VRF has two device copies of its tables; a commit writes the
unpublished one (its pending list of what it missed, plus the new dirty
ranges) and flips the view generation new launches take. grout's datapath
never waits for a route change either (rte_fib under RCU,
modules/ip/control/route.c:87-95); here a launch sees one table from its
first packet to its last.

  * a run of commits, each checked against the oracle, so the copies
    alternate and the pending lists are exercised, in every device format;
  * launches submitted from another thread while the FIB toggles between
    two states: every launch's verdicts equal the oracle's for one state or
    the other, whole (no launch reads a half-written copy)."""
import threading
import time

import numpy as np
import pytest

import oracle
import scenarios as SC
from golden_util import fresh_fastpath_state, run_gpu
from grout_amd import abi
from grout_amd import topology as T

pytestmark = pytest.mark.gpu


def _route(cidr, slot):
    net = T.ipaddress.IPv4Network(cidr)
    r = np.zeros(1, dtype=abi.ROUTE_DT)
    r["ip"], r["prefixlen"], r["vrf_id"], r["nh"] = int(net.network_address), net.prefixlen, 1, slot
    return r


def _apply(fp, o, ops, nh):
    for op in ops:
        net = T.ipaddress.IPv4Network(op[1])
        if op[0] in ("add", "rep"):
            r = _route(op[1], nh[op[2]])
            fp.route_add(r, replace=op[0] == "rep")
            assert o.L.or_route_add(o.h, r.ctypes.data, 1, 1 if op[0] == "rep" else 0) == 0
        else:
            fp.route_del(1, int(net.network_address), net.prefixlen)
            be = int.from_bytes(int(net.network_address).to_bytes(4, "big"), "little")
            assert o.L.or_route_del(o.h, 1, be, net.prefixlen) == 0


# each step is committed and checked; together they make /16s go from
# uniform to chunked and back (DIR-16-8-8), tbl8 groups get freed and
# reused, and one commit has nothing to publish
STEPS = [
    [("add", "200.1.0.0/16", "fwd")],
    [("add", "16.1.0.0/17", "fwd2"), ("del", "10.90.1.7/32")],
    [("add", "10.66.1.0/24", "fwd"), ("rep", "16.1.0.0/17", "fwd3")],
    [("add", "16.1.5.5/32", "fwd2")],
    [("del", "16.1.5.5/32"), ("add", "16.1.9.9/32", "fwd3")],
    [("add", "0.0.0.0/0", "fwd3"), ("del", "10.66.1.0/24")],
    [],
    [("del", "10.70.0.0/16"), ("del", "200.1.0.0/16"), ("del", "16.1.9.9/32")],
    [("del", "0.0.0.0/0"), ("del", "16.1.0.0/17")],
]


@pytest.mark.parametrize("fmt", [2, 1, 0])
def test_commit_sequence(fastpath, fmt):
    t, nh = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    fastpath.tune("fib_format", fmt)
    fresh_fastpath_state(fastpath, T.config_single_route())  # force a reload in this format
    try:
        run_gpu(fastpath, t, fr, me)  # loads t: first commit
        o = oracle.Oracle(t, build_dir24=False)
        for i, ops in enumerate(STEPS):
            _apply(fastpath, o, ops, nh)
            fastpath.fib_commit(1)
            o.L.or_fib_build(o.h, 1)
            g = run_gpu(fastpath, t, fr, me)
            ref = o.process(fr, me)
            bad = np.nonzero(ref[1] != g[1])[0]
            assert len(bad) == 0, (i, [(lab[k], ref[1][k], g[1][k]) for k in bad[:6]])
            assert np.array_equal(ref[0], g[0]), i
        assert fastpath.tune("fib_format_of", 1) == fmt
    finally:
        fastpath.tune("fib_format", 2)
        fresh_fastpath_state(fastpath, T.config_single_route())  # drop the modified state


TOGGLE_B = [("rep", "16.1.0.0/16", "fwd2"), ("rep", "10.70.0.0/16", "fwd"), ("add", "16.1.7.0/25", "fwd3")]
TOGGLE_A = [("rep", "16.1.0.0/16", "fwd"), ("rep", "10.70.0.0/16", "grp"), ("del", "16.1.7.0/25")]


@pytest.mark.parametrize("fmt", [2, 1])
def test_snapshot_under_churn(fastpath, fmt):
    import torch

    from grout_amd.fwd import shared_stream

    t, nh = SC.corpus_topology()
    fr, me, _ = SC.corpus_arrays()
    fastpath.tune("fib_format", fmt)
    fresh_fastpath_state(fastpath, T.config_single_route())
    try:
        run_gpu(fastpath, t, fr, me)
        # the expected verdicts of each state, on the corpus
        oa = oracle.Oracle(t, build_dir24=False)
        va = oa.process(fr, me)[1].view("<u8")
        ob = oracle.Oracle(t, build_dir24=False)
        for op in TOGGLE_B:  # oracle only
            r = _route(op[1], nh[op[2]])
            assert ob.L.or_route_add(ob.h, r.ctypes.data, 1, 1 if op[0] == "rep" else 0) == 0
        ob.L.or_fib_build(ob.h, 1)
        vb = ob.process(fr, me)[1].view("<u8")
        assert (va != vb).sum() > 4  # the two states tell apart
        # a batch of the corpus tiled, launched K times into K verdict buffers
        reps, K = 2048, 40
        n = len(me) * reps
        dev = torch.device("cuda")
        fin = torch.from_numpy(np.ascontiguousarray(np.tile(fr, (reps, 1))).reshape(-1)).to(dev)
        mt = torch.from_numpy(np.tile(me, reps).view(np.uint8)).to(dev)
        outs = [torch.empty(n * abi.LINE, dtype=torch.uint8, device=dev) for _ in range(2)]
        vs = [torch.zeros(n * 8, dtype=torch.uint8, device=dev) for _ in range(K)]
        q = fastpath.queue(shared_stream(dev))
        stop = threading.Event()
        err = []

        def submitter():
            try:
                for k in range(K):
                    q.submit(fin, outs[k & 1], mt, vs[k], n, in_stride=fr.shape[1])
                    time.sleep(0.002)
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)
            finally:
                stop.set()

        th = threading.Thread(target=submitter)
        dummy = oracle.Oracle(t, build_dir24=False)  # absorbs _apply's oracle half
        commits, state = 0, "A"
        th.start()
        while not stop.is_set():
            _apply(fastpath, dummy, TOGGLE_B if state == "A" else TOGGLE_A, nh)
            fastpath.fib_commit(1)
            state = "B" if state == "A" else "A"
            commits += 1
        th.join()
        q.sync()
        assert not err, err
        seen = []
        for k in range(K):
            got = vs[k].cpu().numpy().view("<u8").reshape(reps, len(me))
            if (got == va).all():
                seen.append("A")
            elif (got == vb).all():
                seen.append("B")
            else:
                rows = np.nonzero((got != va).any(axis=1) & (got != vb).any(axis=1))[0]
                pytest.fail(f"launch {k}: {len(rows)} tiles match neither state (commits {commits})")
        assert commits >= 4 and {"A", "B"} <= set(seen), (commits, seen)
        q.close()
        if state == "B":  # leave state A
            _apply(fastpath, dummy, TOGGLE_A, nh)
            fastpath.fib_commit(1)
    finally:
        fastpath.tune("fib_format", 2)
        fresh_fastpath_state(fastpath, T.config_single_route())


def _two_vrf_topology():
    t = T.Topology(max_ifaces=64, max_nexthops=64)
    t.add_vrf(1)
    t.add_vrf(20)
    t.add_port(2, 0, "02:00:00:00:00:02", vrf_id=1)
    t.add_port(3, 1, "02:00:00:00:00:03", vrf_id=1)
    t.add_port(4, 2, "02:00:00:00:00:04", vrf_id=20)
    t.add_port(5, 3, "02:00:00:00:00:05", vrf_id=20)
    nh = {"a": t.add_nexthop(3, "172.16.3.2", "02:00:00:01:00:0a"),
          "b": t.add_nexthop(3, "172.16.3.3", "02:00:00:01:00:0b"),
          "c": t.add_nexthop(5, "172.16.5.2", "02:00:00:01:00:0c"),
          "d": t.add_nexthop(5, "172.16.5.3", "02:00:00:01:00:0d")}
    t.add_route(1, "10.0.0.0/8", nh["a"])
    t.add_route(20, "10.0.0.0/8", nh["c"])
    t.add_route(20, "10.1.0.0/16", nh["d"])
    return t, nh


@pytest.mark.parametrize("fmt", [2, 1])
def test_commits_interleaved_across_vrfs(fastpath, fmt):
    """Commits of two VRFs interleaved: each publication flips the context's
    view generation, and the other VRF must keep its published copy (not
    the copy it last wrote). Streams enter both VRFs at once."""
    from grout_amd import synth as S
    t, nh = _two_vrf_topology()
    n = 1 << 14
    streams = [S.stream(n, 0x2F0 + k, dst_range=(T.ip4("10.0.0.0"), T.ip4("10.3.255.255")),
                        in_iface=port, dst_mac=mac)
               for k, (port, mac) in enumerate([(2, "02:00:00:00:00:02"), (4, "02:00:00:00:00:04")])]
    fr = np.concatenate([streams[0][0], streams[1][0]])
    me = np.concatenate([streams[0][1], streams[1][1]])
    fastpath.tune("fib_format", fmt)
    try:
        run_gpu(fastpath, t, fr, me)  # loads t: both VRFs committed
        o = oracle.Oracle(t, build_dir24=False)
        steps = [(1, [("add", "10.2.0.0/16", "b")]), (20, [("rep", "10.1.0.0/16", "c")]),
                 (20, [("add", "10.2.3.0/24", "d")]), (1, [("rep", "10.0.0.0/8", "b"), ("del", "10.2.0.0/16")]),
                 (1, []), (20, [("del", "10.1.0.0/16")]), (1, [("add", "10.3.0.0/17", "a")])]
        for vrf, ops in steps:
            for op in ops:
                r = _route(op[1], nh[op[2]]) if op[0] != "del" else None
                if r is not None:
                    r["vrf_id"] = vrf
                    fastpath.route_add(r, replace=op[0] == "rep")
                    assert o.L.or_route_add(o.h, r.ctypes.data, 1, 1 if op[0] == "rep" else 0) == 0
                else:
                    net = T.ipaddress.IPv4Network(op[1])
                    fastpath.route_del(vrf, int(net.network_address), net.prefixlen)
                    be = int.from_bytes(int(net.network_address).to_bytes(4, "big"), "little")
                    assert o.L.or_route_del(o.h, vrf, be, net.prefixlen) == 0
            fastpath.fib_commit(vrf)
            o.L.or_fib_build(o.h, vrf)
            ref, g = o.process(fr, me), run_gpu(fastpath, t, fr, me)
            assert np.array_equal(ref[1], g[1]), (vrf, ops)
            assert np.array_equal(ref[0], g[0]), (vrf, ops)
    finally:
        fastpath.tune("fib_format", 2)
        fresh_fastpath_state(fastpath, T.config_single_route())


def test_queue_destroy_during_commits(fastpath):
    """Queues created, used and destroyed on one thread while another commits
    in a loop: each publication records every queue's retire event and makes
    the control stream wait on it, so a queue must leave the context's list
    (under the exclusive lock, its streams drained) before its events and
    stream are destroyed (gr_hip_queue_destroy). Every forward stays whole on
    one FIB state or the other, and nothing errors."""
    t, nh = SC.corpus_topology()
    fr, me, _ = SC.corpus_arrays()
    fresh_fastpath_state(fastpath, T.config_single_route())
    run_gpu(fastpath, t, fr, me)
    oa = oracle.Oracle(t, build_dir24=False)
    lines = np.ascontiguousarray(fr[:, :abi.LINE])  # the host path takes header lines
    va = oa.process(lines, me, lines_only=True)[1].view("<u8")
    ob = oracle.Oracle(t, build_dir24=False)
    for op in TOGGLE_B:
        r = _route(op[1], nh[op[2]])
        assert ob.L.or_route_add(ob.h, r.ctypes.data, 1, 1 if op[0] == "rep" else 0) == 0
    ob.L.or_fib_build(ob.h, 1)
    vb = ob.process(lines, me, lines_only=True)[1].view("<u8")
    stop = threading.Event()
    err, seen = [], []

    def churn():
        dummy = oracle.Oracle(t, build_dir24=False)
        state = "A"
        try:
            while not stop.is_set():
                _apply(fastpath, dummy, TOGGLE_B if state == "A" else TOGGLE_A, nh)
                fastpath.fib_commit(1)
                state = "B" if state == "A" else "A"
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    th = threading.Thread(target=churn)
    th.start()
    try:
        for _ in range(60):
            q = fastpath.queue()  # created, used once, destroyed, while commits run
            out, v = q.forward_host(lines, np.ascontiguousarray(me))
            q.close()
            got = v.view("<u8")
            seen.append("A" if (got == va).all() else "B" if (got == vb).all() else "mixed")
    finally:
        stop.set()
        th.join()
    assert not err, err
    assert "mixed" not in seen, seen
