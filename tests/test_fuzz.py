# SPDX-License-Identifier: BSD-3-Clause
"""Differential fuzzing: random perturbations of the exception corpus and
its topology, HIP path against the oracle, bit-exact.

The corpus (scenarios.py) places one packet on every edge. Each seed here
perturbs it further. Frames get bit flips in the first 64 bytes, random
destinations under random IPv4 and IPv6 routes, random TTL / hop limits, ingress ifaces,
VLAN ids, checksum offload status, lengths and RSS hashes, and a recomputed
header checksum for most of them, so that packets reach the deep nodes.
The topology gets ifaces brought down, MTUs changed, and nexthop states,
flags and MACs changed. Mixing these reaches combinations no single corpus
case names, such as a VLAN sub-interface on a down parent or a group member
losing its MAC.

The CPU tests feed the oracle's mbuf-level chain through the node
hand-back (gr_hip_node_apply). The GPU tests run the device batch (whole
frames and header lines) and the node walk on the same cases."""
import functools

import numpy as np
import pytest

import oracle
import scenarios as SC
from grout_amd import abi

N_PKTS = 8192
SEEDS = [0xF0221, 0xF0222, 0xF0223, 0xF0224, 0xF0225, 0xF0226]


def mutate_topology(t, rng):
    ids = np.nonzero(t.ifaces["id"])[0]
    for i in rng.choice(ids, size=len(ids) // 3, replace=False):
        r = t.ifaces[i]
        k = rng.integers(3)
        if k == 0:
            r["flags"] ^= abi.IFACE_F_UP
        elif k == 1:
            r["mtu"] = rng.choice([576, 1280, 1400, 1500, 9000])
        else:
            r["flags"] ^= rng.choice([abi.IFACE_F_SNAT_STATIC, abi.IFACE_F_SNAT_DYNAMIC])
    l3 = np.nonzero(t.nh["type"] == abi.NH_T["L3"])[0]
    for s in rng.choice(l3, size=len(l3) // 4, replace=False):
        r = t.nh[s]
        k = rng.integers(3)
        if k == 0:
            r["state"] = rng.choice(list(abi.NH_S.values()))
        elif k == 1:
            r["flags"] ^= rng.choice([abi.NH_F_LINK, abi.NH_F_GATEWAY, abi.NH_F_LOCAL])
        else:
            r["mac"] = rng.integers(0, 256, 6, dtype=np.uint8)
    return t


def ip4_cksum(hdr):
    s = int(np.frombuffer(hdr.tobytes(), ">u2").sum(dtype=np.uint64))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def mutate_frames(fr, me, t, rng, n=N_PKTS):
    idx = rng.integers(len(me), size=n)
    fr = fr[idx].copy()
    me = me[idx].copy()
    stride = fr.shape[1]
    # bit flips, mostly in the Ethernet and IP headers
    for _ in range(3):
        rows = np.nonzero(rng.random(n) < 0.25)[0]
        pos = np.where(rng.random(len(rows)) < 0.8, rng.integers(12, 54, len(rows)), rng.integers(0, 64, len(rows)))
        fr[rows, pos] ^= (1 << rng.integers(0, 8, len(rows))).astype(np.uint8)
    v4 = (fr[:, 12] == 0x08) & (fr[:, 13] == 0x00)
    v6 = (fr[:, 12] == 0x86) & (fr[:, 13] == 0xDD)
    # destinations under random routes (IPv4), hop counts
    routes = t.route_array()
    rows = np.nonzero(v4 & (rng.random(n) < 0.4))[0]
    rt = routes[rng.integers(len(routes), size=len(rows))]
    host = rng.integers(0, 1 << 32, len(rows), dtype=np.uint64).astype(np.uint32)
    plen = rt["prefixlen"].astype(np.uint64)
    mask = ((np.uint64(0xFFFFFFFF) << (np.uint64(32) - plen)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    dst = (rt["ip"].astype(np.uint32) & mask) | (host & ~mask)
    fr[rows, 30:34] = dst.astype(">u4").view(np.uint8).reshape(-1, 4)
    # IPv6 destinations under random routes: prefix bits kept, the rest random
    routes6 = t.route6_array()
    rows = np.nonzero(v6 & (rng.random(n) < 0.4))[0]
    rt6 = routes6[rng.integers(len(routes6), size=len(rows))]
    bits = np.arange(128)
    keep = bits[None, :] < rt6["prefixlen"][:, None].astype(np.int64)  # per bit, MSB first
    pfx = np.unpackbits(rt6["ip"], axis=1).astype(bool)
    rnd = rng.random((len(rows), 128)) < 0.5
    fr[rows, 38:54] = np.packbits(np.where(keep, pfx, rnd), axis=1)
    rows = np.nonzero(v4 & (rng.random(n) < 0.2))[0]
    fr[rows, 22] = rng.choice([0, 1, 2, 255], len(rows))
    rows = np.nonzero(v6 & (rng.random(n) < 0.2))[0]
    fr[rows, 21] = rng.choice([0, 1, 2, 255], len(rows))
    # metadata
    ids = np.concatenate([np.nonzero(t.ifaces["id"])[0], [0, 1, 999, 1023, 4000, 65535]])
    rows = rng.random(n) < 0.1
    me["iface"][rows] = rng.choice(ids, rows.sum())
    rows = rng.random(n) < 0.1
    vlan = rng.choice([0, 100, 200, 13, 4095, int(rng.integers(4096))], rows.sum())
    me["vlan_ck"][rows] = (me["vlan_ck"][rows] & 0xF000) | vlan
    rows = rng.random(n) < 0.2
    me["vlan_ck"][rows] = (me["vlan_ck"][rows] & 0x0FFF) | (rng.integers(0, 4, rows.sum()) << 12).astype(np.uint16)
    rows = rng.random(n) < 0.1
    me["pkt_len"][rows] = rng.integers(0, 2048, rows.sum())
    me["rss"] = rng.integers(0, 1 << 16, n)
    # valid IPv4 header checksums for most, so packets get past ip_input
    for i in np.nonzero(v4 & (rng.random(n) < 0.7))[0]:
        ihl = (fr[i, 14] & 0xF) * 4
        if ihl < 20 or 14 + ihl > stride:
            continue
        fr[i, 24:26] = 0
        fr[i, 24:26] = np.frombuffer(ip4_cksum(fr[i, 14:14 + ihl]).to_bytes(2, "big"), np.uint8)
    return fr, me


@functools.lru_cache(maxsize=1)
def _corpus():
    fr, me, _ = SC.corpus_arrays()
    return fr, me


def fuzz_case(seed):
    rng = np.random.default_rng(seed)
    t, _ = SC.corpus_topology()
    mutate_topology(t, rng)
    fr, me = mutate_frames(*_corpus(), t, rng)
    return t, fr, me


def test_fuzz_reaches_the_edges():
    """The perturbed cases keep covering the graph (not all dropped early)."""
    edges = set()
    for seed in SEEDS[:2]:
        t, fr, me = fuzz_case(seed)
        _, v, _ = oracle.Oracle(t).process(fr, me)
        edges |= {abi.EDGE_NAMES[e] for e in v["edge"]}
        assert (v["edge"] == abi.EDGE["port_output"]).mean() > 0.05
    assert len(edges) >= 35, sorted(edges)


@pytest.mark.parametrize("seed", SEEDS[:3])
def test_fuzz_apply_matches_oracle_mbufs(seed):
    from test_node_shim import apply, compare_mbufs, mbufs_for
    t, fr, me = fuzz_case(seed)
    lines, v, _, want, ns_want = oracle.Oracle(t).process_mbufs(fr, me)
    bufs, m = mbufs_for(fr, me)
    ns = apply(m, lines, v, t)
    compare_mbufs(m, want, bufs, lines)
    assert np.array_equal(ns["packets"], ns_want["packets"]) and np.array_equal(ns["calls"], ns_want["calls"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_gpu(fastpath, seed):
    from golden_util import run_gpu
    from test_gpu_parity import compare
    t, fr, me = fuzz_case(seed)
    o = oracle.Oracle(t)
    compare(o.process(fr, me), run_gpu(fastpath, t, fr, me))
    fr64 = np.ascontiguousarray(fr[:, :64])
    compare(o.process(fr64, me, lines_only=True), run_gpu(fastpath, t, fr64, me, lines_only=True))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:2])
def test_fuzz_node_process_gpu(fastpath, seed):
    from golden_util import fresh_fastpath_state
    from test_node_shim import compare_mbufs, mbufs_for
    t, fr, me = fuzz_case(seed)
    fresh_fastpath_state(fastpath, t)
    lines, v, st, want, ns_want = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True)
    bufs, m = mbufs_for(fr, me)
    q = fastpath.queue()
    try:
        ns = q.node_process(m, burst=64)
        compare_mbufs(m, want, bufs, lines)
        assert np.array_equal(ns["packets"], ns_want["packets"]) and np.array_equal(ns["calls"], ns_want["calls"])
        assert np.array_equal(q.stats(), st)
    finally:
        q.close()
