# SPDX-License-Identifier: BSD-3-Clause
"""Known-answer tests pinning the oracle.

1. The six cases of grout's only hot-path unit test,
   modules/ip/datapath/ip_input.c:302-383, restated on full frames: the
   fake mbuf there holds a bare IPv4 header (data_len = 20, domain LOCAL);
   here the same header follows an Ethernet header addressed to the RX port.
2. ip_forward's incremental checksum (ip_forward.c:29-32), hand-derived.
3. The longest-prefix match of both oracle LPMs against brute force.
4. The five cases of ip6_input's unit test (ip6_input.c:249-316), the hop
   limit of ip6_forward, and the IPv6 LPM (oracle hash, brute force and the
   product's trie) against each other.
"""
import ctypes
import ipaddress

import numpy as np
import pytest

import oracle
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

P0 = T.PORT_IFACE[0]


def kat_topo(snat_dynamic=False, local_nh=False):
    t = T.base_ports()
    if snat_dynamic:
        t.ifaces[P0]["flags"] |= abi.IFACE_F_SNAT_DYNAMIC
    if local_nh:  # nexthop_info_l3 {LOCAL, ipv4 = dst}, ip_input.c:370-374
        nh = t.add_nexthop(P0, None, flags=abi.NH_F_LOCAL)
        t.nh[nh]["af"] = abi.AF_IP4
        t.nh[nh]["ipv4"] = T.ip4("1.9.8.6")
        t.add_route(1, "1.9.8.6/32", nh)
    return t


def kat_header(**kw):
    # ipv4_init_default_mbuf, ip_input.c:275-300 (IPPROTO_RAW = 255)
    d = dict(ihl=5, version=4, total_len=20, tos=0, ident=1, flags_frag=0, ttl=64, proto=255,
             src="0.3.0.1", dst="1.9.8.6", length=34)
    d.update(kw)
    return S.frame(**d)


def run(t, frames, pkt_lens=None):
    arr, meta = S.pack(frames, pkt_lens=pkt_lens)
    _, v, _ = oracle.Oracle(t).process(arr, meta)
    return [abi.EDGE_NAMES[e] for e in v["edge"]]


def test_kat_invalid_mbuf_len():  # ip_input.c:302-312
    assert run(kat_topo(), [kat_header()], pkt_lens=[14 + 10]) == ["ip_input_bad_length"]


def test_kat_invalid_cksum():  # ip_input.c:314-323
    assert run(kat_topo(), [kat_header(cksum=0x666)]) == ["ip_input_bad_checksum"]


def test_kat_invalid_version():  # ip_input.c:325-335
    assert run(kat_topo(), [kat_header(version=5)]) == ["ip_input_bad_version"]


def test_kat_invalid_ihl_raw_cksum():  # ip_input.c:337-349
    f = bytearray(kat_header(version=3, cksum=0))
    s = sum(int.from_bytes(f[14 + i:16 + i], "little") for i in range(0, 20, 2))
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    f[24:26] = s.to_bytes(2, "little")  # rte_raw_cksum, not complemented
    assert run(kat_topo(), [bytes(f)]) == ["ip_input_bad_checksum"]


def test_kat_invalid_total_length():  # ip_input.c:351-361
    assert run(kat_topo(), [kat_header(total_len=10)]) == ["ip_input_bad_length"]


def test_kat_conntrack_dnat():  # ip_input.c:363-383
    # grout's conntrack lookup (mocked to hit in the test) runs on the CPU:
    # the fast path hands such packets to the "local_ct" edge, and to
    # ip_input_local when the iface has no SNAT_DYNAMIC flag.
    assert run(kat_topo(snat_dynamic=True, local_nh=True), [kat_header()]) == ["ip_input_local_ct"]
    assert run(kat_topo(snat_dynamic=False, local_nh=True), [kat_header()]) == ["ip_input_local"]


@pytest.mark.parametrize("field,expect", [
    # checksum field bytes 24-25 as stored, expected after forward
    (b"\x39\x52", b"\x3a\x52"),  # plain: +0x0100 in network order
    (b"\xfe\xff", b"\x00\x00"),  # LE 0xfffe -> 0xffff -> +1 -> 0x0000
    (b"\xff\xff", b"\x01\x00"),  # LE 0xffff -> 0x10000 -> +1 -> 0x0001
    (b"\x00\x00", b"\x01\x00"),
    (b"\xff\x00", b"\x00\x01"),  # LE 0x00ff + 1 = 0x0100
])
def test_ip_forward_cksum_arithmetic(field, expect):
    """ip_forward.c:29-32 applied by the oracle to a GOOD-flagged packet."""
    t = T.config_single_route()
    f = bytearray(S.frame(dst="16.1.0.1"))
    f[24:26] = field
    arr, meta = S.pack([bytes(f)], ck=abi.CKSUM_GOOD)
    out, v, _ = oracle.Oracle(t).process(arr, meta)
    assert abi.EDGE_NAMES[v[0]["edge"]] == "port_output"
    assert bytes(out[0, 24:26]) == expect
    assert out[0, 22] == 63


def test_lpm_vs_brute_force():
    rng = np.random.default_rng(7)
    t = T.base_ports()
    nh = t.add_nexthop(T.PORT_IFACE[1], "172.16.1.2", "02:00:00:01:00:2d")
    seen = set()
    for _ in range(600):
        ln = int(rng.choice([0, 1, 7, 8, 12, 16, 20, 23, 24, 25, 26, 28, 30, 31, 32]))
        ip = int(rng.integers(0, 2**32)) & (((1 << 32) - 1) ^ ((1 << (32 - ln)) - 1))
        if (ip, ln) in seen:
            continue
        seen.add((ip, ln))
        t.add_route(1, f"{T.ipaddress.IPv4Address(ip)}/{ln}", nh + len(seen) % 5)
    for k in range(5):
        t.add_nexthop(T.PORT_IFACE[1], f"172.16.1.{10 + k}", "02:00:00:01:00:2d")
    o = oracle.Oracle(t)
    probes = [int(x) for x in rng.integers(0, 2**32, 3000)]
    for ip, ln in list(seen)[:300]:
        probes += [ip, ip + (1 << (32 - ln)) - 1 if ln else 2**32 - 1]
    for ip in probes:
        b = o.lpm(1, ip, "brute")
        assert o.lpm(1, ip, "hash") == b
        assert o.lpm(1, ip, "dir24") == b


# ---- IPv6: the five cases of modules/ip6/datapath/ip6_input.c:249-316
# (ipv6_init_default_mbuf :217-243: version 6, payload 0, next header NONE,
# hop limit 64, src 0:3:0:3:1:9:8:8, dst 0:3:0:5:2:0:2:4, data_len 40,
# domain OTHER), restated on frames to a MAC that is not the port's.
OTHER_MAC = "02:00:00:aa:bb:cc"


def kat6(**kw):
    d = dict(dst_mac=OTHER_MAC, next_header=59, hop=64, src="0:3:0:3:1:9:8:8", dst="0:3:0:5:2:0:2:4",
             payload_len=0, length=54)
    d.update(kw)
    return S.frame6(**d)


def test_kat6_invalid_version():  # ip6_input.c:249-258
    assert run(kat_topo(), [kat6(version=5)]) == ["ip6_input_bad_version"]


def test_kat6_invalid_src_mcast_addr():  # ip6_input.c:260-271
    assert run(kat_topo(), [kat6(src="ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff")]) == ["ip6_input_bad_addr"]


def test_kat6_invalid_dst_unspec_addr():  # ip6_input.c:273-284
    assert run(kat_topo(), [kat6(dst="::")]) == ["ip6_input_bad_addr"]


def test_kat6_invalid_dst_mcast_addr():  # ip6_input.c:286-305: scope none, iface-local
    assert run(kat_topo(), [kat6(dst="ff00::1"), kat6(dst="ff01::1")]) == ["ip6_input_bad_addr"] * 2


def test_kat6_invalid_mbuf_len():  # ip6_input.c:307-316: data_len = 40 / 2
    assert run(kat_topo(), [kat6()], pkt_lens=[14 + 20]) == ["ip6_input_bad_length"]


def test_kat6_default_is_other_host():
    # the default fake mbuf passes every check above and stops at the
    # domain (ETH_DOMAIN_OTHER, ip6_input.c:115-119)
    assert run(kat_topo(), [kat6()]) == ["ip6_input_other_host"]


def test_kat6_hop_limit():  # ip6_forward.c:25-30: 1 -> error, 2 -> forwarded with 1
    t = T.base_ports()
    nh = t.add_nexthop(T.PORT_IFACE[1], "2001:db8:1::2", "02:00:00:06:00:02")
    t.add_route6(1, "2001:db8:100::/48", nh)
    f = [S.frame6(dst="2001:db8:100::1", hop=h) for h in (0, 1, 2)]
    arr, meta = S.pack(f)
    out, v, _ = oracle.Oracle(t).process(arr, meta)
    assert [abi.EDGE_NAMES[e] for e in v["edge"]] == ["ip6_error_ttl_exceeded"] * 2 + ["port_output"]
    assert out[2][21] == 1 and out[2][12] == 0x86 and out[2][13] == 0xdd
    assert bytes(out[2][:6]) == T.mac_bytes("02:00:00:06:00:02")


def test_lpm6_hash_matches_brute_force():
    rng = np.random.default_rng(6)
    t = T.base_ports()
    nhs = [t.add_nexthop(T.PORT_IFACE[1], "2001:db8:1::%x" % (i + 2), "02:00:00:06:00:%02x" % i) for i in range(8)]
    for i in range(300):
        plen = int(rng.choice([0, 3, 8, 16, 17, 24, 31, 32, 40, 47, 48, 56, 64, 65, 96, 127, 128]))
        a = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        a[0] = 0x20 | (a[0] & 0x0F)
        net = ipaddress.IPv6Network((bytes(a), plen), strict=False)
        t.add_route6(1, str(net), nhs[i % 8])
    # de-duplicate (later identical prefixes would be EEXIST)
    r = t.route6_array()
    _, keep = np.unique(np.concatenate([r["ip"], r["prefixlen"][:, None]], axis=1), axis=0, return_index=True)
    t.routes6 = [r[np.sort(keep)]]
    o = oracle.Oracle(t)
    host = abi.host()
    f = host.gr_fib6_new(1024, 4096)
    for x in t.route6_array():
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_add(f, ip.ctypes.data, int(x["prefixlen"]), int(x["nh"]), 0) == 0
    assert host.gr_fib6_build(f) == 0
    for i in range(2000):
        d = rng.integers(0, 256, 16, dtype=np.uint8)
        if i % 2:  # under a route
            x = t.route6_array()[i % len(t.route6_array())]
            d[:x["prefixlen"] // 8] = x["ip"][:x["prefixlen"] // 8]
        want = o.lpm6(1, bytes(d), brute=True)
        assert o.lpm6(1, bytes(d)) == want
        assert host.gr_fib6_lookup(f, d.ctypes.data) == want  # the product's trie
        assert host.gr_fib6_lookup_rib(f, d.ctypes.data) == want
    host.gr_fib6_free(f)


def _fib6_check(host, f, routes, rng, n):
    """Lookups under random routes (random host bits) and at random
    addresses equal the RIB's longest match."""
    for i in range(n):
        d = rng.integers(0, 256, 16, dtype=np.uint8)
        if i % 4:  # under a route, random host bits
            x = routes[rng.integers(len(routes))]
            nb = int(x["prefixlen"])
            full = nb // 8
            d[:full] = x["ip"][:full]
            if nb % 8:
                m = (0xFF00 >> (nb % 8)) & 0xFF
                d[full] = (int(x["ip"][full]) & m) | (int(d[full]) & (~m & 0xFF))
        assert host.gr_fib6_lookup(f, d.ctypes.data) == host.gr_fib6_lookup_rib(f, d.ctypes.data)


def _fib6_of(host, r):
    f = host.gr_fib6_new(len(r) + 16, max(1 << 16, 4 * len(r)))
    for x in r:
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_add(f, ip.ctypes.data, int(x["prefixlen"]), int(x["nh"]), 0) == 0
    assert host.gr_fib6_build(f) == 0
    return f


def test_fib6_fullview6_trie():
    """The product's IPv6 trie (fib6.c) on fib_inject -6's full view: lookups
    under every route, next to random ones, equal the RIB's longest match,
    also after deletes and a rebuild."""
    host = abi.host()
    r = T.config_fullview6().route6_array()
    assert len(r) == 200_001  # + the address route of p0
    f = _fib6_of(host, r)
    rng = np.random.default_rng(66)
    _fib6_check(host, f, r, rng, 20_000)
    for x in r[::3]:  # delete a third, repaint, compare again
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_del(f, ip.ctypes.data, int(x["prefixlen"])) == 0
    assert host.gr_fib6_build(f) == 0
    _fib6_check(host, f, r, rng, 20_000)
    host.gr_fib6_free(f)


def test_fib6_path_compression():
    """Sparse deep prefixes (random /56 .. /128 under 2000::/3): most of the
    painted groups hold one exception and become skip nodes."""
    host = abi.host()
    rng = np.random.default_rng(67)
    n = 5000
    r = np.zeros(n, dtype=abi.ROUTE6_DT)
    r["ip"] = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    r["ip"][:, 0] = 0x20 | (r["ip"][:, 0] & 0x1F)
    r["prefixlen"] = rng.choice([56, 64, 96, 128], size=n)
    for i in range(n):  # host bits clear
        nb = int(r["prefixlen"][i])
        for b in range(16):
            keep = min(8, max(0, nb - 8 * b))
            r["ip"][i, b] &= (0xFF00 >> keep) & 0xFF
    r["vrf_id"] = 1
    r["nh"] = 1 + np.arange(n) % 64
    f = _fib6_of(host, r)
    painted, kept, skips = host.gr_fib6_groups_painted(f), host.gr_fib6_groups_used(f), host.gr_fib6_skips_used(f)
    assert kept < painted // 4 and skips > 0, (painted, kept, skips)
    _fib6_check(host, f, r, rng, 20_000)
    host.gr_fib6_free(f)


# ---- the same known answers through the GPU (the reference's expectations,
# not the oracle's output, are the check)
def _raw3():
    f = bytearray(kat_header(version=3, cksum=0))
    s = sum(int.from_bytes(f[14 + i:16 + i], "little") for i in range(0, 20, 2))
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    f[24:26] = s.to_bytes(2, "little")
    return bytes(f)


GPU_KATS = [  # (reference test, topology kwargs, frame, pkt_len or None, expected edge)
    ("ip_input.c:302-312", {}, lambda: kat_header(), 14 + 10, "ip_input_bad_length"),
    ("ip_input.c:314-323", {}, lambda: kat_header(cksum=0x666), None, "ip_input_bad_checksum"),
    ("ip_input.c:325-335", {}, lambda: kat_header(version=5), None, "ip_input_bad_version"),
    ("ip_input.c:337-349", {}, _raw3, None, "ip_input_bad_checksum"),
    ("ip_input.c:351-361", {}, lambda: kat_header(total_len=10), None, "ip_input_bad_length"),
    ("ip_input.c:363-383", dict(snat_dynamic=True, local_nh=True), lambda: kat_header(), None, "ip_input_local_ct"),
    ("ip6_input.c:249-258", {}, lambda: kat6(version=5), None, "ip6_input_bad_version"),
    ("ip6_input.c:260-271", {}, lambda: kat6(src="ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff"), None,
     "ip6_input_bad_addr"),
    ("ip6_input.c:273-284", {}, lambda: kat6(dst="::"), None, "ip6_input_bad_addr"),
    ("ip6_input.c:286-305 scope none", {}, lambda: kat6(dst="ff00::1"), None, "ip6_input_bad_addr"),
    ("ip6_input.c:286-305 iface-local", {}, lambda: kat6(dst="ff01::1"), None, "ip6_input_bad_addr"),
    ("ip6_input.c:307-316", {}, lambda: kat6(), 14 + 20, "ip6_input_bad_length"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("ref,topo_kw,frame,pkt_len,expect", GPU_KATS, ids=[k[0] for k in GPU_KATS])
def test_kat_gpu(fastpath, ref, topo_kw, frame, pkt_len, expect):
    """grout's own unit-test cases (ip_input.c, ip6_input.c) on the GPU path."""
    from golden_util import run_gpu
    t = kat_topo(**topo_kw)
    arr, meta = S.pack([frame()], pkt_lens=None if pkt_len is None else [pkt_len])
    _, v, _ = run_gpu(fastpath, t, arr, meta)
    assert abi.EDGE_NAMES[v["edge"][0]] == expect, ref


def _wide_entries(host, f):
    """Wide-group references (GR_FIB6_WIDE) in the painted trie: first
    level, groups and skip-node children."""
    import ctypes
    for fn in ("gr_fib6_top", "gr_fib6_groups", "gr_fib6_skips"):
        getattr(host, fn).restype = ctypes.c_void_p
        getattr(host, fn).argtypes = [ctypes.c_void_p]
    ng, ns = host.gr_fib6_groups_used(f), host.gr_fib6_skips_used(f)
    top = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_top(f), ctypes.POINTER(ctypes.c_uint32)), shape=(65536,))
    grp = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_groups(f), ctypes.POINTER(ctypes.c_uint32)),
                                shape=(max(ng, 1) * 256,))
    sk = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_skips(f), ctypes.POINTER(ctypes.c_uint32)),
                               shape=(max(ns, 1) * 4,)).reshape(-1, 4)
    allv = np.concatenate([top, grp[:ng * 256], sk[:ns, 2]])  # struct gr_fib6_skip: child at byte 8
    return int(((allv & 0xE0000000) == 0xA0000000).sum())


@pytest.mark.parametrize("max_groups", [1 << 16, 200])
def test_fib6_level_compression(max_groups):
    """Dense /48s (fib_inject -6's largest bucket shape: 2400:0:vvvv:vvvv::/48)
    make wide groups (two bytes per gather) when the group capacity allows,
    and the trie stays exact either way (200 group slots: no room for the 256
    slots of a wide group)."""
    host = abi.host()
    n = 40_000
    r = np.zeros(n, dtype=abi.ROUTE6_DT)
    v = np.arange(1, n + 1, dtype=np.uint32)
    r["ip"][:, 0] = 0x24
    for k in range(4):
        r["ip"][:, 2 + k] = (v >> (24 - 8 * k)) & 0xFF
    r["prefixlen"] = 48
    r["vrf_id"] = 1
    r["nh"] = 1 + v % 2048
    f = host.gr_fib6_new(n + 16, max_groups)
    for x in r:
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_add(f, ip.ctypes.data, 48, int(x["nh"]), 0) == 0
    assert host.gr_fib6_build(f) == 0
    wide = _wide_entries(host, f)
    assert (wide > 0) == (max_groups == 1 << 16), wide
    _fib6_check(host, f, r, np.random.default_rng(68), 20_000)
    host.gr_fib6_free(f)


@pytest.mark.parametrize("fanout,wide", [(32, True), (4, False)])
def test_fib6_skip_widening(fanout, wide):
    """A one-byte skip (2400:05xx::/24 is the only branch under 2400::/16)
    over a heavy subtree (byte 3 fans out to `fanout` groups, below
    GR_FIB6_WIDE_MIN) becomes a wide group with its child: 32 groups under it
    qualify, 4 do not (GR_FIB6_SKIP_WIDE_MIN = 16); lookups exact either way."""
    host = abi.host()
    rows = []
    for b3 in range(fanout):
        for b4 in range(0, 256, 3):
            rows.append((b3, b4))
    r = np.zeros(len(rows), dtype=abi.ROUTE6_DT)
    r["ip"][:, 0] = 0x24
    r["ip"][:, 2] = 0x05
    r["ip"][:, 3] = [a for a, _ in rows]
    r["ip"][:, 4] = [b for _, b in rows]
    r["prefixlen"] = 40
    r["vrf_id"] = 1
    r["nh"] = 1 + np.arange(len(rows)) % 1000
    f = _fib6_of(host, r)
    _wide_entries(host, f)  # sets the accessor signatures
    import ctypes
    top = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_top(f), ctypes.POINTER(ctypes.c_uint32)), shape=(65536,))
    ent = int(top[0x2400])
    assert ((ent & 0xE0000000) == 0xA0000000) == wide, hex(ent)
    if not wide:
        assert ent & 0x40000000, hex(ent)  # still the skip node
    _fib6_check(host, f, r, np.random.default_rng(69 + fanout), 10_000)
    host.gr_fib6_free(f)


def _kinds(host, f):
    """Entries of the image by kind (fib6.h): range groups, wide groups by
    shift, skips and plain groups referenced from the first level and groups."""
    import collections
    top, grp, sk = _image(host, f)
    slots, _ = _referenced(top, grp, sk)
    # range groups' own slots hold packed leaves, not entries
    rg = set()
    for v in np.concatenate([top, sk[:, 2]] + ([grp[slots].ravel()] if len(slots) else [])):
        if (int(v) & 0xE0000000) == 0xE0000000:
            rg.update((int(v) & 0x1FFFFFFF) + k for k in (0, 1))
    plain_slots = [x for x in slots.tolist() if x not in rg]
    e = np.concatenate([top, sk[:, 2]] + ([grp[plain_slots].ravel()] if plain_slots else []))
    e = e[(e & 0x80000000) != 0]
    c = collections.Counter()
    for v in e.tolist():
        k = v & 0x60000000
        c["range" if k == 0x60000000 else "skip" if k == 0x40000000 else
          ("wide%d" % ((v >> 26) & 7)) if k == 0x20000000 else "group"] += 1
    return c


def _routes6(rows, plen):
    r = np.zeros(len(rows), dtype=abi.ROUTE6_DT)
    for i, b in enumerate(rows):
        r["ip"][i, :len(b)] = b
    r["prefixlen"] = plen
    r["vrf_id"] = 1
    r["nh"] = 1 + np.arange(len(rows)) % 2000
    return r


def test_fib6_range_groups():
    """fib_inject's /44 shape (2300:0:vvvv:vv00::/44 under nothing shorter):
    each byte-4 node's children hold one run of 16 entries in byte 5, so the
    byte-4 nodes become range groups (8-byte entries, one gather for bytes 4
    and 5). A /48 added under one /44 breaks its run: that byte-4 node falls
    back to a plain or wide group, the others stay range groups; deleting it
    brings the range group back. Lookups equal the RIB's throughout."""
    host = abi.host()
    rows = [(0x23, 0, 0, v >> 8, v & 0xFF) for v in range(1, 3000)]
    r = _routes6(rows, 44)
    f = _fib6_of(host, r)
    k0 = _kinds(host, f)
    assert k0["range"] >= 10, k0
    rng = np.random.default_rng(70)
    _fib6_check(host, f, r, rng, 8000)
    extra = _routes6([(0x23, 0, 0, 5, 7, 0x08)], 48)  # inside 2300:0:5:700::/44's miss range: a new run
    x = np.ascontiguousarray(extra[0]["ip"])
    assert host.gr_fib6_add(f, x.ctypes.data, 48, 77, 0) == 0
    assert host.gr_fib6_build(f) == 0
    k1 = _kinds(host, f)
    assert k1["range"] == k0["range"] - 1, (k0, k1)
    allr = np.concatenate([r, extra])
    _fib6_check(host, f, allr, rng, 8000)
    assert host.gr_fib6_del(f, x.ctypes.data, 48) == 0
    assert host.gr_fib6_build(f) == 0
    assert _kinds(host, f)["range"] == k0["range"]
    _fib6_check(host, f, r, rng, 8000)
    host.gr_fib6_free(f)


def test_fib6_narrow_wide_groups():
    """fib_inject's /36 shape (2100:vvvv:v000::/36: 16 routes per byte-4 node,
    16 entries each): every child of a byte-3 node changes only at multiples
    of 16 in byte 4, so the byte-3 wide groups keep one entry per 16 (shift
    4: 16 slots instead of 256). A /40 under one of them refines that child:
    its wide group goes back to shift 0; deleting it restores shift 4.
    Lookups equal the RIB's throughout."""
    host = abi.host()
    rows = [(0x21, 0, (v << 4) >> 16 & 0xFF, (v << 4) >> 8 & 0xFF, (v << 4) & 0xFF) for v in range(1, 20000)]
    r = _routes6(rows, 36)
    f = _fib6_of(host, r)
    k0 = _kinds(host, f)
    assert k0["wide4"] >= 1 and k0["wide0"] == 0, k0
    rng = np.random.default_rng(71)
    _fib6_check(host, f, r, rng, 8000)
    extra = _routes6([(0x21, 0, 0, 0x12, 0x35)], 40)  # a /40 inside 2100:0:123x::/36
    x = np.ascontiguousarray(extra[0]["ip"])
    assert host.gr_fib6_add(f, x.ctypes.data, 40, 55, 0) == 0
    assert host.gr_fib6_build(f) == 0
    k1 = _kinds(host, f)
    assert k1["wide0"] >= 1, k1
    _fib6_check(host, f, np.concatenate([r, extra]), rng, 8000)
    assert host.gr_fib6_del(f, x.ctypes.data, 40) == 0
    assert host.gr_fib6_build(f) == 0
    assert _kinds(host, f) == k0
    _fib6_check(host, f, r, rng, 8000)
    host.gr_fib6_free(f)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fib6_clustered_rebuilds(seed):
    """Random clusters shaped to trigger both level compressions
    (scenarios.clustered_routes6), rebuilt after random deletes and re-adds:
    every build equals the RIB's longest match."""
    import scenarios as SC
    host = abi.host()
    rng = np.random.default_rng(0x6C0 + seed)
    r = SC.clustered_routes6(seed)
    r["vrf_id"] = 1
    r["nh"] = 1 + rng.integers(0, 4000, len(r))
    f = host.gr_fib6_new(len(r) + 16, 1 << 15)
    for x in r:
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_add(f, ip.ctypes.data, int(x["prefixlen"]), int(x["nh"]), 0) == 0
    live = np.ones(len(r), dtype=bool)
    for step in range(3):
        assert host.gr_fib6_build(f) == 0
        _fib6_check(host, f, r[live], rng, 6000)
        flip = rng.random(len(r)) < 0.3
        for i in np.nonzero(flip)[0]:
            ip = np.ascontiguousarray(r[i]["ip"])
            if live[i]:
                assert host.gr_fib6_del(f, ip.ctypes.data, int(r[i]["prefixlen"])) == 0
            else:
                assert host.gr_fib6_add(f, ip.ctypes.data, int(r[i]["prefixlen"]), int(r[i]["nh"]), 0) == 0
            live[i] = ~live[i]
    if seed != 3:  # seed 3's clusters are too light to widen
        assert _wide_entries(host, f) > 0
    host.gr_fib6_free(f)


def _walk_from(host, f, ip, ent, b):
    """The rest of the fib6.h walk from (ent, b), as chain_fib6 resumes it."""
    G = ctypes.cast(host.gr_fib6_groups(f), ctypes.POINTER(ctypes.c_uint32))
    S = ctypes.cast(host.gr_fib6_skips(f), ctypes.POINTER(ctypes.c_uint8))
    EXT, SKIP, WIDE, IDX = 0x80000000, 0x40000000, 0x20000000, 0x1FFFFFFF
    while b < 16 and ent & EXT:
        if ent & SKIP and ent & WIDE:  # range group (fib6.h)
            q0, q1 = G[(ent & IDX) * 256 + 2 * int(ip[b])], G[(ent & IDX) * 256 + 2 * int(ip[b]) + 1]
            y = int(ip[b + 1])
            ent = (q0 if (q0 >> 24) <= y <= (q1 >> 24) else q1) & 0xFFFFFF
            b += 2
        elif ent & SKIP:
            k = bytes(S[(ent & IDX) * 16 + i] for i in range(16))
            n = k[7]
            match = b + n <= 16 and bytes(ip[b:b + n]) == k[:n]
            ent = int.from_bytes(k[8:12] if match else k[12:16], "little")
            b += n
        elif ent & WIDE:
            sh = (ent >> 26) & 7
            ent = G[(ent & 0x03FFFFFF) * 256 + (int(ip[b]) << (8 - sh)) + (int(ip[b + 1]) >> sh)]
            b += 2
        else:
            ent = G[(ent & IDX) * 256 + int(ip[b])]
            b += 1
    return 0 if ent & EXT else ent


def _image(host, f):
    """The device image of a trie (fib6.h): first level, group slots up to the
    high-water mark, skip nodes (as u32 quadruples)."""
    import ctypes
    _wide_entries(host, f)  # accessor signatures
    host.gr_fib6_dirty.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_uint32)]
    host.gr_fib6_dirty.restype = ctypes.c_int
    ng, ns = host.gr_fib6_groups_used(f), host.gr_fib6_skips_used(f)
    top = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_top(f), ctypes.POINTER(ctypes.c_uint32)), shape=(65536,))
    grp = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_groups(f), ctypes.POINTER(ctypes.c_uint32)),
                                shape=(max(ng, 1) * 256,))[:ng * 256].reshape(-1, 256)
    sk = np.ctypeslib.as_array(ctypes.cast(host.gr_fib6_skips(f), ctypes.POINTER(ctypes.c_uint32)),
                               shape=(max(ns, 1) * 4,))[:ns * 4].reshape(-1, 4)
    return top.copy(), grp.copy(), sk.copy()


def _dirty(host, f, kind):
    import ctypes
    host.gr_fib6_dirty.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_uint32)]
    host.gr_fib6_dirty.restype = ctypes.c_int
    host.gr_fib6_dirty_clear.argtypes = [ctypes.c_void_p]
    p, n = ctypes.c_void_p(), ctypes.c_uint32()
    all_ = host.gr_fib6_dirty(f, kind, ctypes.byref(p), ctypes.byref(n))
    assert all_ >= 0
    v = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(n.value,)).copy() \
        if n.value else np.zeros(0, np.uint32)
    return bool(all_), v


def _referenced(top, grp, sk):
    """Group slots and skip nodes the image reaches from its first level."""
    slots, skips = set(), set()
    todo = [top]
    while todo:
        e = np.concatenate([np.asarray(x, dtype=np.uint32).ravel() for x in todo])
        todo = []
        e = e[(e & 0x80000000) != 0]
        kind = e & 0x60000000
        # range groups: two slots of packed leaves, nothing below them
        slots.update(w + k for w in (e[kind == 0x60000000] & 0x1FFFFFFF).tolist() for k in (0, 1))
        sk_i = (e[kind == 0x40000000] & 0x1FFFFFFF).tolist()
        we = e[kind == 0x20000000]
        wide = list(zip((we & 0x03FFFFFF).tolist(), ((we >> 26) & 7).tolist()))  # first slot, shift: 2^(8-s) slots
        plain = (e[(e & 0x60000000) == 0] & 0x1FFFFFFF).tolist()
        new = [s for s in plain if s not in slots] + [w + k for w, sh in wide for k in range(256 >> sh)
                                                      if w + k not in slots]
        slots.update(new)
        if new:
            todo.append(grp[np.array(new, dtype=np.int64)])
        nk = [k for k in sk_i if k not in skips]
        skips.update(nk)
        if nk:
            todo.append(sk[np.array(nk, dtype=np.int64), 2])  # struct gr_fib6_skip: child at byte 8
    return np.array(sorted(slots), dtype=np.int64), np.array(sorted(skips), dtype=np.int64)


@pytest.mark.parametrize("view", ["fullview6", "clustered"])
def test_fib6_incremental_publication(view):
    """Route churn, committed in rounds, as gr_hip_fib6_commit publishes it:
    two device copies written in turn, each with the changes it missed (the
    previous commit's dirty lists) and this commit's, never the whole trie.
    After every commit the copy just written equals the host image on every
    slot and skip node the image reaches, lookups through the trie equal the
    RIB's longest match, and a commit of 100 changes touches a small share of
    the image (the trie is repainted along the changed paths only)."""
    import scenarios as SC
    host = abi.host()
    rng = np.random.default_rng(0x1C6)
    if view == "fullview6":
        r = T.config_fullview6(count=60_000).route6_array()
    else:
        r = np.ascontiguousarray(SC.clustered_routes6(2), dtype=abi.ROUTE6_DT)
        r["nh"] = 1 + np.arange(len(r)) % 97
    f = host.gr_fib6_new(len(r) + 16, max(1 << 16, 4 * len(r)))
    live = rng.random(len(r)) < 0.9
    for x in r[live]:
        ip = np.ascontiguousarray(x["ip"])
        assert host.gr_fib6_add(f, ip.ctypes.data, int(x["prefixlen"]), int(x["nh"]), 0) == 0
    assert host.gr_fib6_build(f) == 0
    all0, _ = _dirty(host, f, 1)  # (sets the accessors' signatures)
    assert all0  # the first upload is whole
    copies = [_image(host, f), _image(host, f)]  # both written whole
    pend = (np.zeros(0, np.uint32),) * 3
    host.gr_fib6_dirty_clear(f)
    w = 0
    for rnd in range(12):
        for i in rng.choice(len(r), 100, replace=False):  # adds, deletes, nexthop changes
            ip = np.ascontiguousarray(r[i]["ip"])
            pl = int(r[i]["prefixlen"])
            if live[i] and rng.random() < 0.5:
                assert host.gr_fib6_del(f, ip.ctypes.data, pl) == 0
                live[i] = False
            else:
                assert host.gr_fib6_add(f, ip.ctypes.data, pl, int(1 + rng.integers(2000)), 1) == 0
                live[i] = True
        assert host.gr_fib6_build(f) == 0
        top, grp, sk = _image(host, f)
        d = tuple(_dirty(host, f, k)[1] for k in range(3))  # top, slots, skips
        assert not _dirty(host, f, 0)[0]
        w ^= 1
        ct, cg, cs = copies[w]
        if len(cg) < len(grp):  # the device copy is sized for the capacity
            cg = np.concatenate([cg, np.zeros((len(grp) - len(cg), 256), np.uint32)])
        if len(cs) < len(sk):
            cs = np.concatenate([cs, np.zeros((len(sk) - len(cs), 4), np.uint32)])
        ut, us, uk = (np.union1d(a, b).astype(np.int64) for a, b in zip(pend, d))
        ct[ut], cg[us], cs[uk] = top[ut], grp[us], sk[uk]
        copies[w] = (ct, cg, cs)
        pend = d
        host.gr_fib6_dirty_clear(f)
        slots, skips = _referenced(top, grp, sk)
        assert np.array_equal(ct, top)
        assert np.array_equal(cg[slots], grp[slots]) and np.array_equal(cs[skips], sk[skips])
        if view == "fullview6":
            assert len(d[1]) < 0.05 * len(slots), (len(d[1]), len(slots))
        _fib6_check(host, f, r[live], rng, 3000)
    host.gr_fib6_free(f)


def test_fib6_build_recovers_from_enospc():
    """A build that runs out of group slots part way (fib6.c)
    publishes nothing and leaves the trie to be built again whole: once
    routes are deleted, the next build succeeds and every lookup equals the
    RIB's longest match again."""
    host = abi.host()
    rng = np.random.default_rng(0xF6E)
    max_groups = 48
    f = host.gr_fib6_new(4096, max_groups)
    routes = []
    failed = False
    for i in range(400):  # /40s under distinct first-level entries: each needs groups
        a = np.zeros(16, dtype=np.uint8)
        a[0], a[1] = 0x20, 0x01
        a[2:5] = rng.integers(0, 256, 3, dtype=np.uint8)
        a[2] = i % 256
        plen = int(rng.choice([40, 48, 56, 64]))
        ip = np.ascontiguousarray(a)
        if host.gr_fib6_add(f, ip.ctypes.data, plen, 1 + i % 7, 0) != 0:
            continue
        routes.append((ip, plen))
        if i % 8 == 7:
            r = host.gr_fib6_build(f)
            if r < 0:
                assert r == -28, r  # -ENOSPC
                failed = True
                break
    assert failed, "the trie never ran out of groups"
    assert host.gr_fib6_build(f) == -28  # still no room: every path is redone, and fails again
    # delete routes until it fits
    while True:
        ip, plen = routes.pop()
        assert host.gr_fib6_del(f, ip.ctypes.data, plen) == 0
        if len(routes) % 4 == 0 and host.gr_fib6_build(f) == 0:
            break
    r = np.zeros(len(routes), dtype=abi.ROUTE6_DT)
    for k, (ip, plen) in enumerate(routes):
        r[k]["ip"] = ip
        r[k]["prefixlen"] = plen
    _fib6_check(host, f, r, rng, 20_000)
    host.gr_fib6_free(f)
