# SPDX-License-Identifier: BSD-3-Clause
"""Parity of the HIP fast path (through the C ABI) with the oracle.

Bit-exact on integer/byte work: verdict (edge, domain, iface, nexthop),
the 64-byte header line each packet leaves with, and the per-iface rx/tx
counters, on the same seeded inputs -- from the exception corpus up to the
BASELINE full size (16M packets over the 1M-route view)."""
import ctypes
import functools

import numpy as np
import pytest

import oracle
import scenarios as SC
from golden_util import _fullview, fresh_fastpath_state, run_gpu
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

pytestmark = pytest.mark.gpu


def compare(o_res, g_res, labels=None):
    out_o, v_o, st_o = o_res
    out_g, v_g, st_g = g_res
    bad = np.nonzero(v_o != v_g)[0]
    assert len(bad) == 0, [((labels[i] if labels else i), v_o[i], v_g[i]) for i in bad[:8]]
    badl = np.nonzero((out_o != out_g).any(axis=1))[0]
    assert len(badl) == 0, [(labels[i] if labels else i) for i in badl[:8]]
    assert np.array_equal(st_o, st_g)


def test_corpus_full_frames(fastpath):
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me), lab)


def test_corpus_lines_only(fastpath):
    """Header-only staging: IHL > 12 packets must be punted, others equal."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    fr64 = np.ascontiguousarray(fr[:, :64])
    o = oracle.Oracle(t).process(fr64, me, lines_only=True)
    g = run_gpu(fastpath, t, fr64, me, lines_only=True)
    compare(o, g, lab)
    punted = {lab[i] for i in np.nonzero(g[1]["edge"] == abi.EDGE["punt"])[0]}
    assert {"ihl 13 opts", "ihl 15 opts", "ihl 15 bad"} <= punted


def test_corpus_stride64_full_mode(fastpath):
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    fr64 = np.ascontiguousarray(fr[:, :64])
    compare(oracle.Oracle(t).process(fr64, me), run_gpu(fastpath, t, fr64, me), lab)


def test_corpus_in_place(fastpath):
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me, inplace=True), lab)


def test_in_place_full_frames(fastpath):
    """In place on full frames (grout rewrites mbufs in place): the first 64
    bytes match the oracle, bytes 32 and up are untouched (nothing past the
    IPv4 checksum / IPv6 hop limit is rewritten) and so is everything past
    the 64-byte line. IPv4 and IPv6 corpus frames plus a stream, 128-byte stride."""
    import torch
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    f2, m2 = S.stream(1 << 14, 0x3232, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")), stride=128)
    fr = np.concatenate([np.pad(fr, ((0, 0), (0, 128 - fr.shape[1]))) if fr.shape[1] < 128 else fr[:, :128], f2])
    me = np.concatenate([me, m2])
    rng = np.random.default_rng(32)
    fr[:, 64:] = rng.integers(0, 256, size=(len(fr), 64), dtype=np.uint8)  # sentinels past the line
    fresh_fastpath_state(fastpath, t)
    dev = torch.device("cuda")
    buf = torch.from_numpy(fr.reshape(-1).copy()).to(dev)
    dme = torch.from_numpy(me.view(np.uint8)).to(dev)
    v = torch.zeros(len(me) * 8, dtype=torch.uint8, device=dev)
    q = fastpath.queue()  # private stream: order the uploads first
    torch.cuda.synchronize()
    q.submit(buf, buf, dme, v, len(me), in_stride=128, out_stride=128)
    q.sync()
    q.close()
    out = buf.cpu().numpy().reshape(len(me), 128)
    o_lines, o_v, _ = oracle.Oracle(t).process(fr, me)
    np.testing.assert_array_equal(out[:, :64], o_lines)
    np.testing.assert_array_equal(out[:, 32:], fr[:, 32:])
    np.testing.assert_array_equal(v.cpu().numpy().view(abi.VERDICT_DT), o_v)


def test_single_route_stream(fastpath):
    t = T.config_single_route()
    fr, me = S.stream(1 << 20, S.SEED_SINGLE, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    o = oracle.Oracle(t).process(fr, me)
    assert (o[1]["edge"] == abi.EDGE["port_output"]).all()
    compare(o, run_gpu(fastpath, t, fr, me))


@pytest.mark.parametrize("inplace", [False, True])
def test_fullview_full_size(fastpath, inplace):
    """BASELINE config 3 at full size: 16M x 64 B over the 1M-route FIB,
    into separate lines and in place (the bench's two placements)."""
    t = _fullview()
    fr, me = S.stream(1 << 24, S.SEED_FULLVIEW, routes=t.route_array())
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me, inplace=inplace)
    compare(o, g)
    assert (g[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.99


@pytest.mark.parametrize("g", range(8))
def test_config5_per_gpu_streams(fastpath, g):
    """BASELINE config 5's inputs: the RX stream of GPU g of the 8-GPU node
    (seed 0x67721000 + g; what bench.py --gpus 8's rank g
    forwards), 2^22 packets over the 1M-route view, forwarded on this GPU:
    bit-exact with the oracle, counters included."""
    t = _fullview()
    fr, me = S.stream(1 << 22, S.SEED_GPU_BASE + g, routes=t.route_array())
    o = oracle.Oracle(t).process(fr, me)
    got = run_gpu(fastpath, t, fr, me)
    compare(o, got)
    assert (got[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.99


def test_fullview_random_dst(fastpath):
    """Uniformly random destinations: misses, tbl8 hits, /32s."""
    t = _fullview()
    fr, me = S.stream(1 << 20, 0xD57, dst_range=(0, (1 << 32) - 1))
    compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me))


def test_imix_full_frames(fastpath):
    """BASELINE config 4: IMIX frames in 2048-byte mbuf-like slots."""
    t = _fullview()
    fr, me = S.stream(1 << 17, S.SEED_IMIX, routes=t.route_array(), imix=True, stride=2048)
    compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me))


def test_host_memory_path(fastpath):
    """gr_hip_fwd4_host: header lines in host memory, chunked H2D/D2H."""
    t = _fullview()
    fresh_fastpath_state(fastpath, t)
    fr, me = S.stream(600_000, S.SEED_IMIX, routes=t.route_array(), imix=True, lines_only=True)
    o = oracle.Oracle(t).process(fr, me, lines_only=True)
    q = fastpath.queue()
    q.stats(reset=True)
    lines, v = q.forward_host(fr, me)
    st = q.stats(reset=True)
    q.close()
    compare(o, (lines, v, st))


@pytest.mark.parametrize("inplace", [False, True])
def test_frame_pointer_batch(fastpath, inplace):
    """GR_HIP_BATCH_F_FRAME_PTRS: frames scattered in device memory, handed
    over by address (corpus + a full-view stream, ragged count), lines out of
    place or each frame rewritten in place."""
    import torch
    t = _fullview()
    fr2, me2 = S.stream(50_001, 0xF9, routes=t.route_array(), stride=128)
    tc, _ = SC.corpus_topology()
    frc, mec, lab = SC.corpus_arrays()
    for topo, fr, me in [(tc, frc, mec), (t, fr2, me2)]:
        fresh_fastpath_state(fastpath, topo)
        n, stride = fr.shape
        perm = np.random.default_rng(n).permutation(n)  # frame i lives in slot perm[i]
        slots = np.zeros((n, stride), dtype=np.uint8)
        slots[perm] = fr
        dev = torch.device("cuda")
        d_slots = torch.from_numpy(slots.reshape(-1)).to(dev)
        ptrs = torch.from_numpy((d_slots.data_ptr() + perm.astype(np.uint64) * stride).view(np.int64)).to(dev)
        d_me = torch.from_numpy(me.view(np.uint8)).to(dev)
        d_out = torch.zeros(n * abi.LINE, dtype=torch.uint8, device=dev)
        d_v = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
        q = fastpath.queue()
        torch.cuda.synchronize()
        q.stats(reset=True)
        b = abi.Batch(ptrs.data_ptr(), None if inplace else d_out.data_ptr(), d_me.data_ptr(), d_v.data_ptr(), n, 0,
                      abi.LINE, abi.BATCH_F_FRAME_PTRS)
        abi.check("gr_hip_fwd4_submit", fastpath.lib.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
        q.sync()
        st = q.stats(reset=True)
        q.close()
        lines = (d_slots.cpu().numpy().reshape(n, stride)[perm, :abi.LINE] if inplace
                 else d_out.cpu().numpy().reshape(n, abi.LINE))
        compare(oracle.Oracle(topo).process(fr, me), (lines, d_v.cpu().numpy().view(abi.VERDICT_DT), st))
        if inplace:  # nothing past the line moved
            assert np.array_equal(d_slots.cpu().numpy().reshape(n, stride)[perm, abi.LINE:], fr[:, abi.LINE:])


@pytest.mark.parametrize("direct", [0, 1])
def test_host_memory_path_pinned(fastpath, direct):
    """gr_hip_fwd4_host on pinned buffers: staged copies (direct 0) or the
    kernel reading and writing host memory over PCIe itself (direct 1)."""
    import torch
    t = _fullview()
    fresh_fastpath_state(fastpath, t)
    fr, me = S.stream(300_017, S.SEED_IMIX + 1, routes=t.route_array(), imix=True, lines_only=True)
    o = oracle.Oracle(t).process(fr, me, lines_only=True)
    n = len(me)
    h_in = torch.from_numpy(np.ascontiguousarray(fr).reshape(-1)).pin_memory()
    h_me = torch.from_numpy(me.view(np.uint8)).pin_memory()
    h_out = torch.zeros(n * abi.LINE, dtype=torch.uint8).pin_memory()
    h_v = torch.zeros(n * 8, dtype=torch.uint8).pin_memory()
    fastpath.tune("host_direct", direct)
    try:
        q = fastpath.queue()
        q.stats(reset=True)
        abi.check("gr_hip_fwd4_host", fastpath.lib.gr_hip_fwd4_host(q._h, h_in.data_ptr(), h_me.data_ptr(), n,
                                                                    h_out.data_ptr(), h_v.data_ptr()))
        st = q.stats(reset=True)
        q.close()
    finally:
        fastpath.tune("host_direct", 1)
    compare(o, (h_out.numpy().reshape(n, abi.LINE), h_v.numpy().view(abi.VERDICT_DT), st))


@pytest.mark.parametrize("fmt", [2, 1, 0])
def test_live_fib_updates(fastpath, fmt):
    """Routes added / replaced / deleted after the first commit, in every
    device FIB format (incremental uploads of the dirty ranges)."""
    t, nh = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    fastpath.tune("fib_format", fmt)
    fresh_fastpath_state(fastpath, T.config_single_route())  # force a reload in this format
    run_gpu(fastpath, t, fr, me)  # loads t
    changes = [("add", "200.1.0.0/16", nh["fwd"]), ("add", "16.1.0.0/17", nh["fwd2"]),
               ("del", "10.90.1.7/32", None), ("add", "10.66.1.0/24", nh["fwd"]),
               ("add", "0.0.0.0/0", nh["fwd3"]), ("del", "10.70.0.0/16", None)]
    o = oracle.Oracle(t, build_dir24=False)
    for op, cidr, slot in changes:
        net = T.ipaddress.IPv4Network(cidr)
        if op == "add":
            r = np.zeros(1, dtype=abi.ROUTE_DT)
            r["ip"], r["prefixlen"], r["vrf_id"], r["nh"] = int(net.network_address), net.prefixlen, 1, slot
            fastpath.route_add(r)
            assert o.L.or_route_add(o.h, r.ctypes.data, 1, 0) == 0
        else:
            fastpath.route_del(1, int(net.network_address), net.prefixlen)
            be = int.from_bytes(int(net.network_address).to_bytes(4, "big"), "little")
            assert o.L.or_route_del(o.h, 1, be, net.prefixlen) == 0
    fastpath.fib_commit(1)
    o.L.or_fib_build(o.h, 1)
    compare(o.process(fr, me), run_gpu(fastpath, t, fr, me), lab)
    # control-plane lookup agrees too
    for d in ["200.1.2.3", "16.1.0.1", "16.1.200.1", "10.90.1.7", "10.66.1.9", "1.2.3.4"]:
        assert fastpath.fib_lookup(1, T.ip4(d)) == o.lpm(1, T.ip4(d), "dir24")
    fastpath.tune("fib_format", 2)
    fresh_fastpath_state(fastpath, T.config_single_route())  # drop the modified state


def test_edge_registration(fastpath):
    """gr_hip_edges_* re-route like grout's *_register hooks."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    run_gpu(fastpath, t, fr, me)
    L, h = fastpath.lib, fastpath.h
    o = oracle.Oracle(t)
    # an extra ether type, blackhole treated as forward, XC mode into eth_input
    for fn, ofn, key, e in [("gr_hip_edges_eth_type", "eth_type", 0x3412, abi.EDGE["ip6_input"]),
                            ("gr_hip_edges_ip_input_nh_type", "ip_input_nh_type", abi.NH_T["BLACKHOLE"], abi.EDGE_CHAIN),
                            ("gr_hip_edges_iface_mode", "iface_mode", abi.IFACE_MODE["XC"], abi.EDGE_CHAIN),
                            ("gr_hip_edges_iface_output_type", "iface_output_type", abi.IFACE_TYPE["BOND"], abi.EDGE["port_output"])]:
        assert getattr(L, fn)(h, key, e) == 0
        o.edge(ofn, key, e)
    try:
        compare(o.process(fr, me), run_gpu(fastpath, t, fr, me), lab)
    finally:
        assert L.gr_hip_edges_eth_type(h, 0x3412, abi.EDGE["eth_input_unknown_type"]) == 0
        assert L.gr_hip_edges_ip_input_nh_type(h, abi.NH_T["BLACKHOLE"], abi.EDGE["ip_blackhole"]) == 0
        assert L.gr_hip_edges_iface_mode(h, abi.IFACE_MODE["XC"], abi.EDGE["xconnect"]) == 0
        assert L.gr_hip_edges_iface_output_type(h, abi.IFACE_TYPE["BOND"], abi.EDGE["bond_output"]) == 0


def test_edge_registration_ip6(fastpath):
    """The IPv6 registration tables: ip6_input nh types (ip6_input.c:32),
    ip6_output nh/iface types (ip6_output.c:28,40), and eth_input handing
    0x86DD to the CPU instead of the device chain."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    run_gpu(fastpath, t, fr, me)
    L, h = fastpath.lib, fastpath.h
    o = oracle.Oracle(t)
    sets = [("gr_hip_edges_ip6_input_nh_type", "ip6_input_nh_type", abi.NH_T["BLACKHOLE"], abi.EDGE_CHAIN),
            ("gr_hip_edges_ip6_input_nh_type", "ip6_input_nh_type", abi.NH_T["REJECT"], abi.EDGE["ip6_blackhole"]),
            ("gr_hip_edges_ip6_output_nh_type", "ip6_output_nh_type", abi.NH_T["SR6_OUTPUT"], abi.EDGE_CHAIN),
            ("gr_hip_edges_ip6_output_iface_type", "ip6_output_iface_type", abi.IFACE_TYPE["VRF"],
             abi.EDGE["port_output"])]
    restore = [(fn, ofn, k, e) for (fn, ofn, k, _), e in zip(sets, [
        abi.EDGE["ip6_blackhole"], abi.EDGE["ip6_error_dest_unreach"], abi.EDGE["sr6_output"], abi.EDGE["xvrf"]])]
    try:
        for fn, ofn, key, e in sets:
            assert getattr(L, fn)(h, key, e) == 0
            o.edge(ofn, key, e)
        compare(o.process(fr, me), run_gpu(fastpath, t, fr, me), lab)
        # IPv6 to the CPU from eth_input
        assert L.gr_hip_edges_eth_type(h, 0xDD86, abi.EDGE["ip6_input"]) == 0
        o.edge("eth_type", 0xDD86, abi.EDGE["ip6_input"])
        g = run_gpu(fastpath, t, fr, me)
        compare(o.process(fr, me), g, lab)
        assert (g[1]["edge"] == abi.EDGE["ip6_input"]).sum() > 50
    finally:
        assert L.gr_hip_edges_eth_type(h, 0xDD86, abi.EDGE_CHAIN6) == 0
        for fn, ofn, key, e in restore:
            assert getattr(L, fn)(h, key, e) == 0


def test_batch_alloc_and_place(fastpath):
    """gr_hip_batch_alloc: zeroed buffers of the right sizes that a submit
    can use; gr_hip_batch_place: the re-placed batch still forwards
    bit-exact, the candidates it did not keep are freed, bad arguments are
    refused and leave the batch as it was."""
    t = T.config_single_route()
    fresh_fastpath_state(fastpath, t)
    n, stride = 100_003, 128
    fr, me = S.stream(n, 0xBA7C, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")), stride=stride)
    L = fastpath.lib
    want = oracle.Oracle(t).process(fr, me)
    free0 = torch_free_bytes()
    b = fastpath.batch_alloc(n, stride)
    assert b.n == n and b.in_stride == stride and b.out_stride == abi.LINE and b.flags == 0
    z = np.ones(n, dtype=abi.VERDICT_DT)
    abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, z.ctypes.data, b.verdicts, z.nbytes))
    assert not z.view(np.uint8).any()
    for dst, src in ((b.in_frames, fr), (b.meta, me)):
        abi.check("h2d", L.gr_hip_memcpy_h2d(fastpath.h, dst, src.ctypes.data, src.nbytes))
    q = fastpath.queue()
    for cand in (0, 4):
        if cand:
            fastpath.batch_place(b, cand)
        q.stats(reset=True)
        abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
        q.sync()
        lines = np.empty((n, abi.LINE), dtype=np.uint8)
        v = np.empty(n, dtype=abi.VERDICT_DT)
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, lines.ctypes.data, b.out_lines, lines.nbytes))
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, v.ctypes.data, b.verdicts, v.nbytes))
        compare(want, (lines, v, q.stats()))
    q.close()
    keep = b.out_lines
    b.out_stride = 128
    assert L.gr_hip_batch_place(fastpath.h, ctypes.byref(b), 2) == -22
    b.out_stride = abi.LINE
    assert L.gr_hip_batch_place(fastpath.h, ctypes.byref(b), 17) == -22 and b.out_lines == keep
    fastpath.batch_free(b)
    assert b.in_frames is None and b.n == 0
    assert torch_free_bytes() >= free0 - (64 << 20)  # the candidates did not leak
    bad = abi.Batch()
    assert L.gr_hip_batch_alloc(fastpath.h, 0, 64, ctypes.byref(bad)) == -22
    assert L.gr_hip_batch_alloc(fastpath.h, 64, 72, ctypes.byref(bad)) == -22


def test_ring_give_up_is_reported(fastpath):
    """A ring wait that gives up (forced with spin_max 1) ends the grid and
    the next sync reports it (-ETIMEDOUT) once; the queue then works as before."""
    t = T.config_single_route()
    fresh_fastpath_state(fastpath, t)
    n = 1 << 20
    fr, me = S.stream(n, 0x5A1, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    L = fastpath.lib
    b = fastpath.batch_alloc(n)
    for dst, src in ((b.in_frames, fr), (b.meta, me)):
        abi.check("h2d", L.gr_hip_memcpy_h2d(fastpath.h, dst, src.ctypes.data, src.nbytes))
    q = fastpath.queue()
    try:
        assert fastpath.tune("spin_max", 1) == 0
        abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
        assert L.gr_hip_queue_sync(q._h) == -110
        assert L.gr_hip_queue_sync(q._h) == 0  # reported once
    finally:
        fastpath.tune("spin_max", 0)
    q.stats(reset=True)
    abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
    assert L.gr_hip_queue_sync(q._h) == 0
    lines = np.empty((n, abi.LINE), dtype=np.uint8)
    v = np.empty(n, dtype=abi.VERDICT_DT)
    abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, lines.ctypes.data, b.out_lines, lines.nbytes))
    abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, v.ctypes.data, b.verdicts, v.nbytes))
    o = oracle.Oracle(t).process(fr, me)
    # the counters shard by shard first (workgroup b counts into shard b % 64):
    # a shortfall names the shards, and so the workgroups, that lost counts
    sh = q.stats_shards(16)
    rx_if = int(np.argmax(o[2]["rx_packets"]))
    per = sh["rx_packets"][:, rx_if].astype(np.int64)
    med = int(np.median(per))
    assert per.sum() == o[2]["rx_packets"][rx_if], dict(
        expected=int(o[2]["rx_packets"][rx_if]), got=int(per.sum()), median_per_shard=med,
        off_median={int(s): int(per[s]) for s in np.nonzero(per != med)[0]})
    compare(o, (lines, v, q.stats()))
    q.close()
    fastpath.batch_free(b)


def torch_free_bytes():
    import torch
    return torch.cuda.mem_get_info()[0]


def test_empty_and_ragged_batches(fastpath):
    t = T.config_single_route()
    fresh_fastpath_state(fastpath, t)
    for n in [1, 63, 255, 257, 1000]:
        fr, me = S.stream(n, S.SEED_SINGLE + n, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
        compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me))
    q = fastpath.queue()
    q.submit(0, 0, 0, 0, 0)  # n == 0 is a no-op
    q.sync()
    with pytest.raises(abi.GrHipError):
        q.submit(16, 32, 8, 8, 10, in_stride=40)  # stride not a multiple of 16
    q.close()


def test_kernel_timing_api(fastpath):
    import torch
    t = T.config_single_route()
    fresh_fastpath_state(fastpath, t)
    fr, me = S.stream(1 << 16, 1, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    q = fastpath.queue()
    dev = torch.device("cuda")
    fin = torch.from_numpy(fr.reshape(-1)).to(dev)
    mt = torch.from_numpy(me.view(np.uint8)).to(dev)
    out = torch.empty_like(fin)
    v = torch.empty(len(me) * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for _ in range(3):
        q.submit(fin, out, mt, v, len(me))
    q.sync()
    ms, cnt = q.kernel_ms(3)
    assert cnt == 3 and ms > 0
    q.close()
    # sampled: only submits 0, 3, 6 of a fresh queue carry events
    q = fastpath.queue()
    fastpath.tune("time_every", 3)
    try:
        for _ in range(7):
            q.submit(fin, out, mt, v, len(me))
        q.sync()
        ms, cnt = q.kernel_ms(10)
        assert cnt == 3 and ms > 0
    finally:
        fastpath.tune("time_every", 1)
    q.close()


@pytest.mark.parametrize("nt,stats,wg,fmt", [(1, 1, 0, 1), (0, 0, 1, 1), (1, 0, 2, 0), (0, 1, 0, 0), (1, 1, 3, 0),
                                            (0, 1, 1, 2), (1, 0, 0, 2)])
def test_kernel_variants(fastpath, nt, stats, wg, fmt):
    """Every tuning variant (gr_hip_tune) forwards bit-exact: nontemporal
    streams, counters, grid (wg_per_cu 1-3: every workgroup walks its ring
    many times round), FIB format (0 DIR24_8 4-byte, 1 DIR-16-8-8 2-byte,
    2 DIR24_8 2-byte)."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    tf = _fullview()
    fr2, me2 = S.stream(1 << 20, 0xAB + nt, routes=tf.route_array())
    o1 = oracle.Oracle(t).process(fr, me)
    o2 = oracle.Oracle(tf).process(fr2, me2)
    fastpath.tune("nt", nt)
    fastpath.tune("stats", stats)
    fastpath.tune("wg_per_cu", wg)
    fastpath.tune("fib_format", fmt)
    try:
        fresh_fastpath_state(fastpath, T.config_single_route())  # force a reload (commit)
        g = run_gpu(fastpath, t, fr, me)
        if stats:
            compare(o1, g, lab)
        else:
            compare((o1[0], o1[1], g[2]), g, lab)
            assert not g[2]["rx_packets"].any()
        g2 = run_gpu(fastpath, tf, fr2, me2)
        compare(o2 if stats else (o2[0], o2[1], g2[2]), g2)
        info = fastpath.fib_info(1)
        n8 = max(256, 1_000_010 // 500)
        if fmt == 1:  # DIR-16-8-8: only the non-uniform /16s get a chunk
            assert info["dev_bytes"] < 4 * (1 << 20)
        elif fmt == 2:
            assert info["dev_bytes"] == 2 * (1 << 24) + 512 * n8
        else:
            assert info["dev_bytes"] == 4 * (1 << 24) + 1024 * n8
    finally:
        for k, v in [("nt", 1), ("stats", 1), ("wg_per_cu", 0), ("fib_format", 2)]:
            fastpath.tune(k, v)
        fresh_fastpath_state(fastpath, T.config_single_route())


def test_mirror_updates_propagate(fastpath):
    """Iface / nexthop changes after load reach the precomputed adjacencies."""
    t, nh = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    run_gpu(fastpath, t, fr, me)  # loads t
    # p1 admin down (egress for most forwards), p2 MTU 1500, p0 loses its MAC,
    # one nexthop becomes unresolved, another changes MAC
    t.ifaces[SC.P1]["flags"] = int(t.ifaces[SC.P1]["flags"]) & ~abi.IFACE_F_UP & 0xFFFF
    t.ifaces[SC.P2]["mtu"] = 1500
    t.ifaces[SC.BOND]["mac_ok"] = 0
    t.nh[nh["fwd2"]]["state"] = abi.NH_S["STALE"]
    t.nh[nh["fwd3"]]["mac"] = [2, 0, 0, 1, 0x33, 0x33]
    fastpath.set_ifaces(t.ifaces)
    fastpath.set_nexthops(t.nh[1:t.n_nh + 1], first=1)
    try:
        compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me), lab)
    finally:
        fresh_fastpath_state(fastpath, T.config_single_route())


def _many_nh_topology(n_nh=6000, n_routes=50_000):
    """More nexthops than the ring kernel stages in LDS (2304), a mix of
    plain forwards and nexthops that leave the fast adjacency: unresolved
    (HOLD), on a VLAN, flagged LINK, and on an admin-down port."""
    t = T.base_ports(max_routes=n_routes + 10)
    t.add_vlan(40, T.PORT_IFACE[2], 77)
    t.add_port(41, 3, "02:00:00:00:00:29", up=False)
    first = t.n_nh + 1
    for j in range(1, n_nh + 1):
        slot = first + j - 1
        kind = j % 11
        ip = f"100.{64 + (j >> 16)}.{(j >> 8) & 255}.{j & 255}"
        mac = "02:00:00:02:%02x:%02x" % ((j >> 8) & 255, j & 255)
        if kind == 3:
            t.add_nexthop(T.PORT_IFACE[1], ip, None, slot=slot)  # no MAC: HOLD
        elif kind == 5:
            t.add_nexthop(40, ip, mac, slot=slot)  # VLAN oif
        elif kind == 7:
            t.add_nexthop(T.PORT_IFACE[3], ip, mac, flags=abi.NH_F_LINK, slot=slot)
        elif kind == 9:
            t.add_nexthop(41, ip, mac, slot=slot)  # admin-down port
        else:
            t.add_nexthop(T.PORT_IFACE[1 + j % 3], ip, mac, slot=slot)
    routes = np.zeros(n_routes, dtype=abi.ROUTE_DT)
    abi.check("gr_synth_fullview_routes",
              abi.host().gr_synth_fullview_routes(n_routes, T.VRF_MAIN, first, n_nh, routes.ctypes.data))
    t.add_routes(routes)
    t.add_address(T.PORT_IFACE[0], "172.16.0.1/24")
    return t


def test_many_nexthops_fast_adjacency(fastpath):
    """Nexthop slots past the LDS-staged range read the fast adjacency with a
    gather; non-plain nexthops fall back to the full adjacency."""
    t = _many_nh_topology()
    fr, me = S.stream(1 << 18, 0x5EED, routes=t.route_array())
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g)
    edges = np.bincount(g[1]["edge"], minlength=abi.E_COUNT)
    assert edges[abi.EDGE["port_output"]] > len(me) // 2
    assert edges[abi.EDGE["ip_hold"]] > 0
    assert (g[1]["nh"] > 2304).sum() > len(me) // 4


def test_high_slots_fall_back_to_4byte_fib(fastpath):
    """Nexthop slots past 15 bits (up to the last of 2^17) cannot live in the
    2-byte FIB formats: the commit falls back to 4-byte DIR24_8 entries by
    itself, and forwarding stays bit-exact."""
    t = T.base_ports(max_routes=20_010)
    first = (1 << 17) - 400
    for j in range(400):
        t.add_nexthop(T.PORT_IFACE[1 + j % 3], f"100.66.{j >> 8}.{j & 255}", "02:00:00:03:%02x:%02x" % (j >> 8, j & 255),
                      slot=first + j)
    routes = np.zeros(20_000, dtype=abi.ROUTE_DT)
    abi.check("gr_synth_fullview_routes",
              abi.host().gr_synth_fullview_routes(20_000, T.VRF_MAIN, first, 400, routes.ctypes.data))
    t.add_routes(routes)
    t.add_address(T.PORT_IFACE[0], "172.16.0.1/24")
    fr, me = S.stream(1 << 18, 0x7FFF, routes=t.route_array())
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g)
    assert fastpath.tune("fib_format_of", 1) == 0  # 4-byte entries
    assert (g[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.99
    assert g[1]["nh"].min() >= first and g[1]["nh"].max() > (1 << 15)


@pytest.mark.parametrize("cfg,fmt", [(c, 2) for c in range(12)] + [(c, f) for c in (12, 13, 14) for f in (0, 2, 1)])
def test_ring_geometries(fastpath, cfg, fmt):
    """Every ring geometry (loaders / storers / slots / tiles in flight) of
    fwd4_ring.hip forwards bit-exact; wg_per_cu 1 makes each workgroup walk
    its ring many times round. Geometries 12-14 gather the 4-byte DIR24_8
    entries of some lanes through the scalar cache (fib_tbl24_split): they
    run in every FIB format, 4-byte first (the only one they split)."""
    t, _ = SC.corpus_topology()
    fr, me, lab = SC.corpus_arrays()
    tf = _fullview()
    fr2, me2 = S.stream(1 << 20, 0xC0F + cfg, routes=tf.route_array())
    o1 = oracle.Oracle(t).process(fr, me)
    o2 = oracle.Oracle(tf).process(fr2, me2)
    fastpath.tune("ring", cfg)
    fastpath.tune("wg_per_cu", 1)
    fastpath.tune("fib_format", fmt)
    try:
        compare(o1, run_gpu(fastpath, t, fr, me), lab)
        compare(o2, run_gpu(fastpath, tf, fr2, me2))
        assert fastpath.tune("fib_format_of", 1) == fmt
        n = 64 * 1000 + 17  # ragged last tile; some workgroups get one tile more than others
        compare(oracle.Oracle(tf).process(fr2[:n], me2[:n]), run_gpu(fastpath, tf, fr2[:n], me2[:n]))
    finally:
        fastpath.tune("ring", 2)  # the default geometry
        fastpath.tune("wg_per_cu", 0)
        fastpath.tune("fib_format", 2)
        fresh_fastpath_state(fastpath, T.config_single_route())


@pytest.mark.parametrize("order,run", [(1, 16), (2, 16), (3, 16), (3, 5)])
def test_tile_orders(fastpath, order, run):
    """The other tile orders (one contiguous run per workgroup; one region per
    XCD; interleaved runs of `run` tiles) cover every tile exactly once, ragged
    sizes included, bit-exact."""
    tf = _fullview()
    fr, me = S.stream(1 << 20, 0x7110 + order, routes=tf.route_array())
    fastpath.tune("tile_order", order)
    fastpath.tune("tile_run", run)
    try:
        for n in (1 << 20, 64 * 1000 + 17, 64 * 257 + 1, 63, 1):
            compare(oracle.Oracle(tf).process(fr[:n], me[:n]), run_gpu(fastpath, tf, fr[:n], me[:n]))
    finally:
        fastpath.tune("tile_order", 0)
        fastpath.tune("tile_run", 16)


@pytest.mark.parametrize("stage_min", [0, 1 << 20])
def test_adjacency_staging_threshold(fastpath, stage_min):
    """Fast adjacencies staged in LDS (stage_min_tiles 0: always) or read
    from the global tables (a threshold no launch reaches): the same
    results, bit-exact, large and ragged batches."""
    tf = _fullview()
    fr, me = S.stream(1 << 18, 0x57A6, routes=tf.route_array())
    fastpath.tune("stage_min_tiles", stage_min)
    try:
        for n in (1 << 18, 64 * 300 + 9, 1024, 1):
            compare(oracle.Oracle(tf).process(fr[:n], me[:n]), run_gpu(fastpath, tf, fr[:n], me[:n]))
    finally:
        fastpath.tune("stage_min_tiles", 4)


# ---- IPv6

@functools.lru_cache(maxsize=None)
def _fullview6_big():
    return T.config_fullview6(count=100_000)


def test_fullview6_stream(fastpath):
    """IPv6 forwarding over a 100k-route IPv6 view, 2^20 packets."""
    t = _fullview6_big()
    fr, me = S.stream6(1 << 20, S.SEED_FULLVIEW6 + 1, t.route6_array())
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g)
    assert (g[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.99
    info = fastpath.fib6_info(1)
    # a deep trie, compacted: range groups and narrow wide groups (fib6.h) keep
    # it under 10k group slots (before round 3: over 20k)
    assert info["routes"] == len(t.route6_array()) and 0 < info["groups_used"] < 10_000, info


@pytest.mark.parametrize("seed", [1, 2])
def test_clustered_routes6_stream(fastpath, seed):
    """IPv6 forwarding over clustered tables whose tries widen at bytes 2-5
    (scenarios.clustered_routes6: wide groups and widened one-byte skips
    below the first level, the kernel's WIDE branch at several depths)."""
    t = T.base_ports(max_routes=1 << 10)
    r = SC.clustered_routes6(seed)
    t.fibs6[T.VRF_MAIN] = (len(r) + 10, 1 << 16)
    first = T.fullview6_nexthops(t)
    r["vrf_id"] = T.VRF_MAIN
    r["nh"] = first + np.arange(len(r)) % T.N_FULLVIEW6_NH
    t.add_routes6(r)
    fr, me = S.stream6(1 << 18, 0x6C10 + seed, r)
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g)
    assert (g[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.9


@pytest.mark.parametrize("second_vrf", [False, True], ids=["one_vrf", "two_vrfs"])
def test_routes6_per_vrf(fastpath, second_vrf):
    """The first level's 2000::/4 slice is staged in LDS only when one VRF
    holds IPv6 routes (fwd4_params.top6): packets of a second VRF, whose trie
    holds the same prefixes on other nexthops, must walk their own VRF's trie
    (no slice staged), and lookups outside the slice (3000::/4) gather the
    first level as before. Ingress on p0 (VRF 1) and p3 (VRF 6, or VRF 1;
    VRFs are ifaces: ids 2-5 are the ports)."""
    t = T.Topology()
    t.add_vrf(1, max_routes=1 << 10)
    for p in range(3):
        t.add_port(T.PORT_IFACE[p], p, T.PORT_MAC[p])
    vrf_b = 6 if second_vrf else 1
    if second_vrf:
        t.add_vrf(vrf_b, max_routes=1 << 10)
    t.add_port(T.PORT_IFACE[3], 3, T.PORT_MAC[3], vrf_id=vrf_b)
    first = T.fullview6_nexthops(t, 64)
    r = T.fullview6_routes(20_000, 1, first, 32)
    extra = r.copy()  # the same prefixes under 3000::/4
    extra["ip"][:, 0] += 0x10
    both = np.concatenate([r, extra])
    t.fibs6[1] = (len(both) + 10, 1 << 16)
    t.add_routes6(both)
    if second_vrf:
        rb = both.copy()
        rb["vrf_id"] = vrf_b
        rb["nh"] = first + 32 + (np.arange(len(rb)) % 32)
        t.fibs6[vrf_b] = (len(rb) + 10, 1 << 16)
        t.add_routes6(rb)
    n = 1 << 17
    sel = both[both["prefixlen"] < 128]
    fa, ma = S.stream6(n, 0x6A01, sel)
    fb, mb = S.stream6(n, 0x6A02, sel, in_iface=T.PORT_IFACE[3], dst_mac=T.PORT_MAC[3])
    pick = np.random.default_rng(0x6A03).integers(0, 2, size=n).astype(bool)
    fr = np.where(pick[:, None], fa, fb)
    me = np.where(pick, ma, mb)
    o = oracle.Oracle(t).process(fr, me)
    g = run_gpu(fastpath, t, fr, me)
    compare(o, g)
    assert (g[1]["edge"] == abi.EDGE["port_output"]).mean() > 0.99
    if second_vrf:  # the two VRFs' nexthops differ: each packet took its own VRF's
        nh = g[1]["nh"]
        assert (nh[pick] < first + 32).all() and (nh[~pick] >= first + 32).all()


def test_mixed_v4_v6_stream(fastpath):
    """IPv4 and IPv6 packets interleaved in every wave (divergent chains)."""
    t, _ = SC.corpus_topology()
    rng = np.random.default_rng(46)
    f4, m4 = S.stream(1 << 16, 0x4646, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    r6 = t.route6_array()
    f6, m6 = S.stream6(1 << 16, 0x6464, r6[r6["prefixlen"] < 128])
    pick = rng.integers(0, 2, size=1 << 16).astype(bool)
    fr = np.where(pick[:, None], f4, f6)
    me = np.where(pick, m4, m6)
    compare(oracle.Oracle(t).process(fr, me), run_gpu(fastpath, t, fr, me))


def test_live_route6_updates(fastpath):
    """route6 add / replace / delete after the first commit, then parity
    (rib6_insert_or_replace / rib6_delete, modules/ip6/control/route.c), one
    commit per kind of change so that the trie's two device copies alternate;
    40k routes, so that the /48 bucket gets wide groups (fib6.h)."""
    t = T.config_fullview6(count=40_000)
    r = t.route6_array()
    fr, me = S.stream6(1 << 16, 0x1606, r[r["prefixlen"] < 128])
    run_gpu(fastpath, t, fr, me)  # loads t
    o = oracle.Oracle(t)
    rng = np.random.default_rng(16)
    idx = rng.permutation(len(r) - 1)  # leave the address route alone

    def commit_and_compare():
        fastpath.fib6_commit(1)
        compare(o.process(fr, me), run_gpu(fastpath, t, fr, me))

    for i in idx[:500]:
        fastpath.route6_del(1, bytes(r["ip"][i]), int(r["prefixlen"][i]))
        ip = np.ascontiguousarray(r["ip"][i])
        assert o.L.or_route6_del(o.h, 1, 0, ip.ctypes.data, int(r["prefixlen"][i])) == 0
    commit_and_compare()
    rep = r[idx[500:800]].copy()
    rep["nh"] = np.roll(rep["nh"], 1)
    fastpath.route6_add(rep, replace=True)
    assert o.L.or_route6_add(o.h, rep.ctypes.data, len(rep), 1) == 0
    commit_and_compare()
    new = r[idx[800:900]].copy()
    new["prefixlen"] = np.minimum(new["prefixlen"].astype(np.int32) + 8, 128).astype(np.uint8)
    new["ip"][:, 15] ^= 0x5A  # more-specifics under existing routes
    uniq = {(bytes(x["ip"]), int(x["prefixlen"])) for x in r}
    new = new[[(bytes(x["ip"]), int(x["prefixlen"])) not in uniq for x in new]]
    fastpath.route6_add(new, replace=True)
    assert o.L.or_route6_add(o.h, new.ctypes.data, len(new), 1) == 0
    commit_and_compare()
    g = run_gpu(fastpath, t, fr, me)
    assert (g[1]["edge"] == abi.EDGE["ip6_error_dest_unreach"]).sum() > 0
    for x in list(r[idx[:20]]) + list(rep[:20]) + list(new[:20]):
        assert fastpath.fib6_lookup(1, bytes(x["ip"])) == o.lpm6(1, bytes(x["ip"]))
    # then many small commits through both copies (the incremental uploads:
    # each copy gets the changes it missed, the previous commit's and its own)
    live = np.ones(len(r), dtype=bool)
    live[idx[:500]] = False
    for rnd in range(16):
        for i in rng.choice(len(r) - 1, 60, replace=False):
            ip = np.ascontiguousarray(r["ip"][i])
            pl = int(r["prefixlen"][i])
            if live[i] and rnd % 3 != 2:
                fastpath.route6_del(1, bytes(r["ip"][i]), pl)
                assert o.L.or_route6_del(o.h, 1, 0, ip.ctypes.data, pl) == 0
                live[i] = False
            else:
                x = r[i:i + 1].copy()
                x["nh"] = T.N_FULLVIEW6_NH // 2 + rng.integers(1, T.N_FULLVIEW6_NH // 2)
                x["nh"] += int(r["nh"].min()) - 1
                fastpath.route6_add(x, replace=True)
                assert o.L.or_route6_add(o.h, x.ctypes.data, 1, 1) == 0
                live[i] = True
        commit_and_compare()
    fresh_fastpath_state(fastpath, T.config_single_route())  # drop the modified state


def test_fib6_lookup_host_scoping(fastpath):
    """The context's host lookup scopes link-local destinations like
    fib6_lookup (addr6_linklocal_scope)."""
    t, _ = SC.corpus_topology()
    from golden_util import fresh_fastpath_state
    fresh_fastpath_state(fastpath, t)
    o = oracle.Oracle(t)
    for dst in ["fe80::2", "fe80::1", "2001:db8:100:1::7", "3000:8000::1", "4000::1"]:
        for iface in [T.PORT_IFACE[0], T.PORT_IFACE[1]]:
            ip = T.ip6(dst)
            assert fastpath.fib6_lookup(1, ip, iface) == o.lpm6(1, ip, iface), (dst, iface)


def test_concurrent_queues_and_fib_updates(fastpath):
    """Two worker queues forward full-view streams in their own threads
    while the control thread adds and deletes routes (disjoint from the
    streams' destinations) and switches the device FIB format back and forth
    (full re-uploads, RX views re-pointed). Every batch must equal the
    oracle: a kernel runs entirely before an update or entirely after it
    (grout's RCU around FIB changes, modules/ip/control/route.c:740-771); the routes added last
    take effect."""
    import threading

    import torch
    t = T.config_fullview(count=100_000)
    t.fibs[T.VRF_MAIN] = (100_200, 0)  # room for the routes added below
    fresh_fastpath_state(fastpath, t)
    dev = torch.device("cuda")
    work = []
    for w in range(2):
        fr, me = S.stream(1 << 18, 0xC0C0 + w, routes=t.route_array())
        lines, v, _ = oracle.Oracle(t).process(fr, me)
        work.append(dict(
            d_in=torch.from_numpy(fr.reshape(-1)).to(dev), d_me=torch.from_numpy(me.view(np.uint8)).to(dev),
            want_l=torch.from_numpy(lines.reshape(-1)).to(dev), want_v=torch.from_numpy(v.view(np.uint8)).to(dev),
            n=len(me), bad=0, iters=0))
    torch.cuda.synchronize()
    stop = threading.Event()
    errors = []

    def worker(wk):
        try:
            q = fastpath.queue()  # its own stream
            d_out = torch.empty(wk["n"] * abi.LINE, dtype=torch.uint8, device=dev)
            d_v = torch.empty(wk["n"] * 8, dtype=torch.uint8, device=dev)
            while not stop.is_set() or wk["iters"] < 5:
                d_out.zero_()
                d_v.zero_()
                torch.cuda.synchronize()
                q.submit(wk["d_in"], d_out, wk["d_me"], d_v, wk["n"])
                q.sync()
                if not (torch.equal(d_out, wk["want_l"]) and torch.equal(d_v, wk["want_v"])):
                    wk["bad"] += 1
                wk["iters"] += 1
            q.close()
        except Exception as e:  # reported by the main thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(wk,)) for wk in work]
    for th in threads:
        th.start()
    nh = int(t.route_array()["nh"][0])
    try:
        for i in range(24):
            r = np.zeros(4, dtype=abi.ROUTE_DT)
            for j, (ip, plen) in enumerate([("200.1.%d.0" % i, 24), ("201.%d.0.0" % i, 16),
                                            ("202.0.%d.7" % i, 32), ("203.%d.0.0" % (i % 8), 13)]):
                r[j]["ip"], r[j]["prefixlen"], r[j]["vrf_id"], r[j]["nh"] = T.ip4(ip), plen, 1, nh
            fastpath.route_add(r, replace=True)
            if i % 3 == 2:
                fastpath.route_del(1, T.ip4("200.1.%d.0" % (i - 1)), 24)
            if i % 6 == 5:
                fastpath.tune("fib_format", 1 if (i // 6) % 2 == 0 else 2)
            fastpath.fib_commit(1)
    finally:
        stop.set()
        for th in threads:
            th.join(timeout=120)
        fastpath.tune("fib_format", 2)
    assert not errors, errors
    assert all(not th.is_alive() for th in threads)
    assert all(wk["iters"] >= 5 for wk in work), [wk["iters"] for wk in work]
    assert [wk["bad"] for wk in work] == [0, 0]
    assert fastpath.fib_lookup(1, T.ip4("200.1.23.9")) == nh
    assert fastpath.fib_lookup(1, T.ip4("200.1.22.9")) == 0  # deleted at i = 23
    fastpath.fib_commit(1)
    fresh_fastpath_state(fastpath, T.config_single_route())  # drop the modified state


def test_batch_place_under_timing_knobs(fastpath):
    """gr_hip_batch_place times its probe launches whatever "time_every" /
    "untimed" say (a private always-timed queue), and the placed batch
    forwards bit-exact."""
    t = T.config_single_route()
    fresh_fastpath_state(fastpath, t)
    n = 1 << 18
    fr, me = S.stream(n, 0x91AC, dst_range=(T.ip4("16.1.0.0"), T.ip4("16.1.255.255")))
    L = fastpath.lib
    b = fastpath.batch_alloc(n)
    try:
        for dst, src in ((b.in_frames, fr), (b.meta, me)):
            abi.check("h2d", L.gr_hip_memcpy_h2d(fastpath.h, dst, src.ctypes.data, src.nbytes))
        for key, val in (("time_every", 4), ("untimed", 1)):
            fastpath.tune(key, val)
            try:
                fastpath.batch_place(b, 3)
            finally:
                fastpath.tune(key, 1 if key == "time_every" else 0)
        q = fastpath.queue()
        q.stats(reset=True)
        abi.check("submit", L.gr_hip_fwd4_submit(q._h, ctypes.byref(b)))
        q.sync()
        lines = np.empty((n, abi.LINE), dtype=np.uint8)
        v = np.empty(n, dtype=abi.VERDICT_DT)
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, lines.ctypes.data, b.out_lines, lines.nbytes))
        abi.check("d2h", L.gr_hip_memcpy_d2h(fastpath.h, v.ctypes.data, b.verdicts, v.nbytes))
        compare(oracle.Oracle(t).process(fr, me), (lines, v, q.stats()))
        q.close()
    finally:
        fastpath.batch_free(b)
