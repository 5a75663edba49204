# SPDX-License-Identifier: BSD-3-Clause
"""Test scenarios: the exception-corpus topology and crafted frames.

Covers every terminal edge of the replaced sub-graph
and the edge cases SURVEY.md §8d lists: bad checksum, TTL 0/1, dst 0,
version 6, IHL 4, total_len 10, bcast/mcast dst MAC, other-host MAC, no
route, 255.255.255.255, 224.0.0.5, local address, ARP/SNAP/unknown
ethertype, > MTU with/without DF, VLAN, unresolved nexthop, admin-down
ifaces, plus ECMP groups, tbl8 prefixes and the ip_forward checksum quirk;
and the same for IPv6 (ip6_input.c / ip6_forward.c / ip6_output.c): bad
version / length / addresses, multicast scopes, hop limit 0/1/2, local
addresses, link-local scoping, prefixes of every trie level, > MTU, hold,
groups, VLAN / no-MAC / admin-down / xvrf egress.
"""
import numpy as np

from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T
from grout_amd.topology import PORT_MAC, SRC_MAC

P0, P1, P2, P3 = T.PORT_IFACE
DOWN, VLAN100, VLAN200, XC, BR_PORT, IPIP, NOMAC, VLAN_ORPHAN = 6, 7, 8, 9, 10, 11, 12, 13
SNATDYN, BOND, VXLAN, VRF2, VRF3_PORT, BRIDGE = 14, 15, 16, 17, 18, 19
STRIDE = 128  # frames up to 128 bytes: IHL 15 options fit


def corpus_topology():
    t = T.Topology(max_nexthops=4096)
    t.add_vrf(1, max_routes=1 << 16)
    t.add_port(P0, 0, PORT_MAC[0])
    t.add_port(P1, 1, PORT_MAC[1])
    t.add_port(P2, 2, PORT_MAC[2], mtu=1280)
    t.add_port(P3, 3, PORT_MAC[3], flags=abi.IFACE_F_SNAT_STATIC)
    t.add_port(DOWN, 4, "02:00:00:00:00:04", up=False)
    t.add_vlan(VLAN100, P0, 100)
    t.add_vlan(VLAN200, P1, 200, mac="02:00:00:00:c8:01")
    t.add_port(XC, 5, "02:00:00:00:00:05", mode="XC")
    t.add_port(BR_PORT, 6, "02:00:00:00:00:06", mode="BRIDGE")
    t.add_iface(IPIP, "IPIP")
    t.add_port(NOMAC, 7, None)
    t.add_vlan(VLAN_ORPHAN, 40, 13, mac="02:00:00:00:0d:01")
    t.add_port(SNATDYN, 8, "02:00:00:00:00:08", flags=abi.IFACE_F_SNAT_DYNAMIC)
    t.add_iface(BOND, "BOND", mac="02:00:00:00:00:0f")
    t.add_iface(VXLAN, "VXLAN", mac="02:00:00:00:00:10")
    t.add_iface(VRF2, "VRF", vrf_id=VRF2)
    t.add_port(VRF3_PORT, 9, "02:00:00:00:00:12", vrf_id=3)
    t.add_iface(BRIDGE, "BRIDGE", mac="02:00:00:00:00:13")

    t.add_address(P0, "172.16.0.1/24")
    t.add_address(P1, "172.16.1.1/24")
    t.add_address(VLAN100, "10.100.0.1/24")
    t.add_address(SNATDYN, "172.16.14.1/24")
    nh = {}
    nh["fwd"] = t.add_nexthop(P1, "172.16.1.2", "02:00:00:01:00:2d")
    nh["fwd2"] = t.add_nexthop(P2, "100.64.0.2", "02:00:00:01:00:02")
    nh["fwd3"] = t.add_nexthop(P1, "172.16.1.3", "02:00:00:01:00:03")
    nh["unres"] = t.add_nexthop(P0, "172.16.0.2")
    nh["bh"] = t.add_nexthop(0, nh_type="BLACKHOLE", vrf_id=1)
    nh["rej"] = t.add_nexthop(0, nh_type="REJECT", vrf_id=1)
    nh["dnat"] = t.add_nexthop(P0, nh_type="DNAT")
    nh["sr6"] = t.add_nexthop(P1, nh_type="SR6_OUTPUT")
    ga = t.add_nexthop(P1, "172.16.1.10", "02:00:00:01:01:0a")
    gb = t.add_nexthop(P2, "100.64.1.11", "02:00:00:01:01:0b")
    gc = t.add_nexthop(P1, "172.16.1.12", "02:00:00:01:01:0c")
    nh["grp"] = t.add_group([ga, gb, gc], reta_size=16)
    nh["grp1"] = t.add_group([gb])
    nh["grp0"] = t.add_group([], reta_size=4)
    nh["mtu"] = t.add_nexthop(P2, "100.64.0.20", "02:00:00:01:00:14")
    nh["snat"] = t.add_nexthop(P3, "100.64.0.21", "02:00:00:01:00:15")
    nh["down"] = t.add_nexthop(DOWN, "100.64.0.22", "02:00:00:01:00:16")
    nh["vlan"] = t.add_nexthop(VLAN200, "10.200.0.2", "02:00:00:01:00:17")
    nh["ipip"] = t.add_nexthop(IPIP, "100.64.0.24", "02:00:00:01:00:18")
    nh["nomac"] = t.add_nexthop(NOMAC, "100.64.0.25", "02:00:00:01:00:19")
    nh["orphan"] = t.add_nexthop(VLAN_ORPHAN, "100.64.0.26", "02:00:00:01:00:1a")
    nh["bond"] = t.add_nexthop(BOND, "100.64.0.27", "02:00:00:01:00:1b")
    nh["vxlan"] = t.add_nexthop(VXLAN, "100.64.0.28", "02:00:00:01:00:1c")
    nh["xvrf"] = t.add_nexthop(VRF2, "100.64.0.29", "02:00:00:01:00:1d")
    nh["bridge"] = t.add_nexthop(BRIDGE, "100.64.0.30", "02:00:00:01:00:1e")
    nh["noif"] = t.add_nexthop(999, "100.64.0.31", "02:00:00:01:00:1f", vrf_id=1)
    nh["link"] = t.add_nexthop(P1)  # no address: LINK flag, unresolved
    nh["stale"] = t.add_nexthop(P1, "172.16.1.33", "02:00:00:01:00:21", state=abi.NH_S["STALE"])
    routes = [
        ("16.1.0.0/16", "fwd"), ("16.0.0.0/16", "unres"), ("10.66.0.0/16", "bh"),
        ("10.67.0.0/16", "rej"), ("10.68.0.0/16", "dnat"), ("10.69.0.0/16", "sr6"),
        ("10.70.0.0/16", "grp"), ("10.70.1.0/24", "grp1"), ("10.70.2.0/24", "grp0"),
        ("10.71.0.0/16", "mtu"), ("10.72.0.0/16", "snat"), ("10.73.0.0/16", "down"),
        ("10.74.0.0/16", "vlan"), ("10.75.0.0/16", "ipip"), ("10.76.0.0/16", "nomac"),
        ("10.77.0.0/16", "orphan"), ("10.78.0.0/16", "bond"), ("10.79.0.0/16", "vxlan"),
        ("10.80.0.0/16", "xvrf"), ("10.81.0.0/16", "bridge"), ("10.82.0.0/16", "noif"),
        ("10.83.0.0/16", "link"), ("10.84.0.0/16", "stale"),
        ("10.90.0.0/16", "fwd"), ("10.90.1.128/25", "fwd2"), ("10.90.1.7/32", "fwd3"),
        ("10.90.2.0/23", "fwd3"), ("10.90.3.64/26", "fwd2"), ("10.0.0.0/8", "fwd2"),
        ("11.0.0.0/7", "fwd3"),
    ]
    for cidr, k in routes:
        t.add_route(1, cidr, nh[k])

    # IPv6
    t.add_address6(P0, "2001:db8::1/64")
    t.add_address6(P1, "2001:db8:1::1/64")
    t.add_address6(P1, "fe80::1/64")  # link-local, scoped to p1
    nh["fwd6"] = t.add_nexthop(P1, "2001:db8:1::2", "02:00:00:06:00:02")
    nh["fwd6b"] = t.add_nexthop(P2, "2001:db8:2::3", "02:00:00:06:00:03")
    nh["fwd6c"] = t.add_nexthop(P1, "2001:db8:1::4", "02:00:00:06:00:04")
    nh["unres6"] = t.add_nexthop(P0, "2001:db8::2")
    nh["ll6"] = t.add_nexthop(P1, "fe80::2", "02:00:00:06:00:05")
    nh["mtu6"] = t.add_nexthop(P2, "2001:db8:2::6", "02:00:00:06:00:06")  # p2 MTU 1280
    nh["vlan6"] = t.add_nexthop(VLAN200, "2001:db8:c8::2", "02:00:00:06:00:07")
    nh["nomac6"] = t.add_nexthop(NOMAC, "2001:db8:7::2", "02:00:00:06:00:08")
    nh["down6"] = t.add_nexthop(DOWN, "2001:db8:4::2", "02:00:00:06:00:09")
    nh["xvrf6"] = t.add_nexthop(VRF2, "2001:db8:11::2", "02:00:00:06:00:0a")
    nh["stale6"] = t.add_nexthop(P1, "2001:db8:1::33", "02:00:00:06:00:0b", state=abi.NH_S["STALE"])
    nh["noif6"] = t.add_nexthop(999, "2001:db8:99::2", "02:00:00:06:00:0c", vrf_id=1)
    g6a = t.add_nexthop(P1, "2001:db8:1::10", "02:00:00:06:01:0a")
    g6b = t.add_nexthop(P2, "2001:db8:2::11", "02:00:00:06:01:0b")
    nh["grp6"] = t.add_group([g6a, g6b], reta_size=8)
    routes6 = [
        ("2001:db8:100::/48", "fwd6"), ("2001:db8:100:1::/64", "fwd6b"), ("2001:db8:100:1::7/128", "fwd6c"),
        ("2001:db8:100:2::/63", "fwd6c"), ("2001:db8:100:4:8000::/65", "fwd6b"),
        ("2001:db8:101::/48", "unres6"), ("2001:db8:102::/48", "bh"), ("2001:db8:103::/48", "rej"),
        ("2001:db8:104::/48", "grp6"), ("2001:db8:105::/48", "mtu6"), ("2001:db8:106::/48", "vlan6"),
        ("2001:db8:107::/48", "nomac6"), ("2001:db8:108::/48", "down6"), ("2001:db8:109::/48", "xvrf6"),
        ("2001:db8:10a::/48", "stale6"), ("2001:db8:10b::/48", "noif6"), ("2001:db8:10c::/48", "sr6"),
        ("2001:db8::/32", "fwd6b"), ("2000::/3", "fwd6c"), ("3000::/12", "fwd6"), ("3000:8000::/17", "fwd6b"),
        ("2001:db8:200::/40", "fwd6"), ("2001:db8:200:ff00::/56", "fwd6c"),
    ]
    for cidr, k in routes6:
        t.add_route6(1, cidr, nh[k])
    t.add_route6(1, "fe80::2/128", nh["ll6"], iface_id=P1)  # link-local host route on p1 only
    return t, nh


def _cksum_target_id(target_be, **kw):
    """Find an IP id giving header checksum `target_be` (network order)."""
    for ident in range(65536):
        f = S.frame(ident=ident, **kw)
        if int.from_bytes(f[24:26], "big") == target_be:
            return f
    raise AssertionError("no id found")


def _with_cksum_field(f, value_be):
    b = bytearray(f)
    b[24:26] = value_be.to_bytes(2, "big")
    return bytes(b)


def corpus_frames(seed=0x5eed):
    """[(frame bytes, meta dict, label)]."""
    rng = np.random.default_rng(seed)
    F = []

    def add(label, f, iface=P0, vlan=0, ck=abi.CKSUM_UNKNOWN, rss=0, pkt_len=None):
        F.append((f, dict(iface=iface, vlan=vlan, ck=ck, rss=rss,
                          pkt_len=len(f) if pkt_len is None else pkt_len), label))

    fr = S.frame
    for d in ["16.1.0.1", "16.1.255.254", "10.90.0.5", "10.90.1.7", "10.90.1.6", "10.90.1.200",
              "10.90.2.9", "10.90.3.100", "10.90.3.64", "10.1.2.3", "11.200.0.1", "12.0.0.1"]:
        add("fwd " + d, fr(dst=d))
    add("fwd ttl 2", fr(dst="16.1.0.2", ttl=2))
    add("ttl 1", fr(dst="16.1.0.2", ttl=1))
    add("ttl 0", fr(dst="16.1.0.2", ttl=0))
    add("bad cksum", fr(dst="16.1.0.3", cksum=0x666))
    add("ol BAD", fr(dst="16.1.0.3"), ck=abi.CKSUM_BAD)
    add("ol GOOD bad cksum", fr(dst="16.1.0.3", cksum=0x1234), ck=abi.CKSUM_GOOD)
    add("ol 3", fr(dst="16.1.0.3", cksum=0x1234), ck=3)
    add("dst 0", fr(dst="0.0.0.0"))
    add("version 6", fr(dst="16.1.0.4", version=6))
    add("version 5", fr(dst="16.1.0.4", version=5))
    # ip_input.c:337-349: version 3 with an uncomplemented raw checksum
    raw3 = bytearray(fr(dst="1.9.8.6", version=3, cksum=0))
    s = sum(int.from_bytes(raw3[14 + i:16 + i], "little") for i in range(0, 20, 2))
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    raw3[24:26] = s.to_bytes(2, "little")
    add("version 3 raw cksum", bytes(raw3))
    # IHL 4: checksum verified over 16 bytes only
    ihl4 = bytearray(fr(dst="16.1.0.5", cksum=0))
    ihl4[14] = 0x44
    c = S.ip4_cksum(bytes(ihl4[14:30]))
    ihl4[24:26] = c.to_bytes(2, "big")
    add("ihl 4", bytes(ihl4))
    add("ihl 0", bytes(bytearray(fr(dst="16.1.0.5"))[:14]) + bytes([0x40]) + fr(dst="16.1.0.5")[15:])
    add("ihl 6 opts", fr(dst="16.1.0.6", ihl=6, options=b"\x01\x01\x01\x00", length=64))
    add("ihl 12 opts", fr(dst="16.1.0.7", ihl=12, options=b"\x01" * 28, length=80))
    add("ihl 13 opts", fr(dst="16.1.0.7", ihl=13, options=b"\x01" * 32, length=90))
    add("ihl 15 opts", fr(dst="16.1.0.8", ihl=15, options=b"\x01" * 40, length=100))
    add("ihl 15 bad", _with_cksum_field(fr(dst="16.1.0.8", ihl=15, options=b"\x07" * 40, length=100), 0x1111))
    add("total_len 10", fr(dst="16.1.0.9", total_len=10))
    add("total_len 19", fr(dst="16.1.0.9", total_len=19))
    add("data_len 16", fr(dst="16.1.0.10"), pkt_len=30)
    add("pkt_len 10", fr(dst="16.1.0.10"), pkt_len=10)
    add("pkt_len 14", fr(dst="16.1.0.10"), pkt_len=14)
    add("bcast mac", fr(dst_mac="ff:ff:ff:ff:ff:ff", dst="16.1.0.11"))
    add("mcast mac", fr(dst_mac="01:00:5e:00:00:05", dst="224.0.0.5"))
    add("other host mac", fr(dst_mac="02:00:00:aa:bb:cc", dst="16.1.0.12"))
    add("p1 mac on p0", fr(dst_mac=PORT_MAC[1], dst="16.1.0.12"))
    add("dst bcast", fr(dst="255.255.255.255"))
    add("dst 224.0.0.5", fr(dst="224.0.0.5"))
    add("dst 239.1.1.1", fr(dst="239.1.1.1"))
    add("dst 240.0.0.1", fr(dst="240.0.0.1"))
    add("no route", fr(dst="200.1.2.3"))
    add("local addr", fr(dst="172.16.0.1"))
    add("local addr other port", fr(dst="172.16.1.1"))
    add("connected hold", fr(dst="172.16.1.5"))
    add("unresolved gw hold", fr(dst="16.0.3.4"))
    add("link nh hold", fr(dst="10.83.0.1"))
    add("stale nh hold", fr(dst="10.84.0.1"))
    add("blackhole", fr(dst="10.66.1.1"))
    add("reject", fr(dst="10.67.1.1"))
    add("dnat", fr(dst="10.68.1.1"))
    add("sr6 output", fr(dst="10.69.1.1"))
    for r in range(20):
        add("group rss %d" % r, fr(dst="10.70.9.%d" % r), rss=int(rng.integers(0, 65536)))
    add("group single", fr(dst="10.70.1.9"), rss=77)
    add("group empty", fr(dst="10.70.2.9"), rss=78)
    add("mtu ok 1294", fr(dst="10.71.0.1", length=100, total_len=1280), pkt_len=1294)
    add("mtu frag 1295", fr(dst="10.71.0.1", length=100, total_len=1281), pkt_len=1295)
    add("mtu frag needed DF", fr(dst="10.71.0.1", length=100, total_len=1400, flags_frag=0x4000), pkt_len=1414)
    add("mtu frag needed DF+", fr(dst="10.71.0.1", length=100, total_len=1400, flags_frag=0x6000), pkt_len=1414)
    add("snat egress", fr(dst="10.72.0.1"))
    add("egress down", fr(dst="10.73.0.1"))
    add("egress vlan", fr(dst="10.74.0.1"))
    add("ipip", fr(dst="10.75.0.1"))
    add("egress no mac", fr(dst="10.76.0.1"))
    add("vlan no parent", fr(dst="10.77.0.1"))
    add("bond", fr(dst="10.78.0.1"))
    add("vxlan", fr(dst="10.79.0.1"))
    add("xvrf", fr(dst="10.80.0.1"))
    add("bridge egress", fr(dst="10.81.0.1"))
    add("nh iface missing", fr(dst="10.82.0.1"))
    add("arp", fr(ethertype=0x0806, dst="16.1.0.1"))
    add("arp bcast", fr(dst_mac="ff:ff:ff:ff:ff:ff", ethertype=0x0806))
    add("ipv6", fr(ethertype=0x86DD))
    add("lacp", fr(ethertype=0x8809))
    add("snap len", fr(ethertype=0x0100))
    add("snap 1535", fr(ethertype=1535))
    add("jumbo llc", fr(ethertype=0x8870))
    add("type 1536", fr(ethertype=1536))
    add("unknown type", fr(ethertype=0x1234))
    add("vlan tag not stripped", fr(ethertype=0x8100))
    add("vlan 100 local", fr(dst="10.100.0.1"), vlan=100)
    add("vlan 100 fwd", fr(dst="16.1.0.13"), vlan=100)
    add("vlan 100 other mac", fr(dst_mac="02:00:00:aa:bb:cc", dst="16.1.0.13"), vlan=100)
    add("vlan 300 unknown", fr(dst="16.1.0.13"), vlan=300)
    add("vlan on xc port", fr(dst="16.1.0.13", dst_mac="02:00:00:00:00:05"), iface=XC, vlan=100)
    add("ingress down", fr(dst="16.1.0.14", dst_mac="02:00:00:00:00:04"), iface=DOWN)
    add("ingress xc", fr(dst="16.1.0.14"), iface=XC)
    add("ingress bridge", fr(dst="16.1.0.14"), iface=BR_PORT)
    add("ingress no mac", fr(dst="16.1.0.14"), iface=NOMAC)
    add("ingress no mac snap", fr(ethertype=0x0100), iface=NOMAC)
    add("snat dyn local", fr(dst="172.16.14.1", dst_mac="02:00:00:00:00:08"), iface=SNATDYN)
    add("snat dyn fwd", fr(dst="16.1.0.15", dst_mac="02:00:00:00:00:08"), iface=SNATDYN)
    add("vrf missing", fr(dst="16.1.0.16", dst_mac="02:00:00:00:00:12"), iface=VRF3_PORT)
    add("ingress missing", fr(dst="16.1.0.16"), iface=50)
    add("ingress vlan iface id direct", fr(dst="16.1.0.17"), iface=VLAN100)
    # ip_forward.c:29-32 checksum quirk: field (LE u16) 0xfffe -> 0x0000, 0xffff -> 0x0001
    f = _cksum_target_id(0xFEFF, dst="16.1.0.18")
    add("cksum field fffe", f)
    base = S.frame(dst="16.1.0.19", ident=0)
    # find an id whose other words sum to 0xffff: then both 0x0000 and 0xffff verify
    for ident in range(65536):
        g = S.frame(dst="16.1.0.19", ident=ident)
        if int.from_bytes(g[24:26], "big") == 0x0000:
            add("cksum field 0000", g)
            add("cksum field ffff", _with_cksum_field(g, 0xFFFF))
            break
    del base
    for d in ["16.1.0.20", "16.1.0.21"]:
        add("ttl 255 " + d, fr(dst=d, ttl=255))
    # ---- IPv6
    f6 = S.frame6
    for d in ["2001:db8:100::1", "2001:db8:100:1::1", "2001:db8:100:1::7", "2001:db8:100:1::8",
              "2001:db8:100:3::1", "2001:db8:100:4:8000::9", "2001:db8:100:4:7fff::9", "2001:db8:5::1",
              "2fff::1", "3000:1::1", "3000:8000::1", "3000:7fff::1", "2001:db8:200:ff00::1",
              "2001:db8:200:fe00::1"]:
        add("fwd6 " + d, f6(dst=d))
    add("fwd6 hop 2", f6(dst="2001:db8:100::2", hop=2))
    add("hop 1", f6(dst="2001:db8:100::2", hop=1))
    add("hop 0", f6(dst="2001:db8:100::2", hop=0))
    add("ip6 version 4", f6(dst="2001:db8:100::3", version=4))
    add("ip6 version 7", f6(dst="2001:db8:100::3", version=7))
    add("ip6 data_len 39", f6(dst="2001:db8:100::3"), pkt_len=53)
    add("ip6 data_len 40", f6(dst="2001:db8:100::3"), pkt_len=54)
    add("ip6 src mcast", f6(src="ff02::1", dst="2001:db8:100::3"))
    add("ip6 dst unspec", f6(dst="::"))
    add("ip6 mcast scope 0", f6(dst="ff00::1"))
    add("ip6 mcast scope 1", f6(dst="ff01::1"))
    add("ip6 mcast scope 2", f6(dst_mac="33:33:00:00:00:01", dst="ff02::1"))
    add("ip6 mcast scope 5", f6(dst="ff05::1:3"))
    add("ip6 bcast mac", f6(dst_mac="ff:ff:ff:ff:ff:ff", dst="2001:db8:100::4"))
    add("ip6 mcast mac", f6(dst_mac="33:33:00:00:00:09", dst="2001:db8:100::4"))
    add("ip6 other host mac", f6(dst_mac="02:00:00:aa:bb:cc", dst="2001:db8:100::4"))
    add("ip6 no route", f6(dst="4000::1"))
    add("ip6 local addr", f6(dst="2001:db8::1"))
    add("ip6 local addr p1", f6(dst="2001:db8:1::1"))
    add("ip6 connected hold", f6(dst="2001:db8:1::5"))
    add("ip6 unresolved gw hold", f6(dst="2001:db8:101::1"))
    add("ip6 stale hold", f6(dst="2001:db8:10a::1"))
    add("ip6 blackhole", f6(dst="2001:db8:102::1"))
    add("ip6 reject", f6(dst="2001:db8:103::1"))
    add("ip6 sr6 output", f6(dst="2001:db8:10c::1"))
    for r in range(6):
        add("ip6 group rss %d" % r, f6(dst="2001:db8:104::%x" % (r + 1)), rss=int(rng.integers(0, 65536)))
    add("ip6 mtu ok", f6(dst="2001:db8:105::1", payload_len=1240, length=100), pkt_len=1294)
    add("ip6 too big", f6(dst="2001:db8:105::1", payload_len=1241, length=100), pkt_len=1295)
    add("ip6 egress vlan", f6(dst="2001:db8:106::1"))
    add("ip6 egress no mac", f6(dst="2001:db8:107::1"))
    add("ip6 egress down", f6(dst="2001:db8:108::1"))
    add("ip6 xvrf", f6(dst="2001:db8:109::1"))
    add("ip6 nh iface missing", f6(dst="2001:db8:10b::1"))
    add("ip6 link-local on p1", f6(dst_mac=PORT_MAC[1], dst="fe80::2"), iface=P1)
    add("ip6 link-local on p0", f6(dst="fe80::2"))
    add("ip6 link-local local p1", f6(dst_mac=PORT_MAC[1], dst="fe80::1"), iface=P1)
    add("ip6 vlan 100 fwd", f6(dst="2001:db8:100::5"), vlan=100)
    add("ip6 vlan 300 unknown", f6(dst="2001:db8:100::5"), vlan=300)
    add("ip6 ingress down", f6(dst="2001:db8:100::6", dst_mac="02:00:00:00:00:04"), iface=DOWN)
    add("ip6 vrf missing", f6(dst="2001:db8:100::6", dst_mac="02:00:00:00:00:12"), iface=VRF3_PORT)
    for k in range(8):
        b = bytearray(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
        b[12:14] = b"\x86\xdd"
        if k % 2:
            b[0:6] = T.mac_bytes(PORT_MAC[0])
        if k % 4 == 1:
            b[14] = 0x60 | (b[14] & 0x0F)
        add("random6 %d" % k, bytes(b))
    # random bytes frames
    for k in range(32):
        b = bytearray(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
        b[12:14] = b"\x08\x00"
        if k % 2:
            b[0:6] = T.mac_bytes(PORT_MAC[0])
        if k % 4 == 1:
            b[14] = 0x45
            c = S.ip4_cksum(bytes(b[14:34]))
            b[24:26] = c.to_bytes(2, "big")
        add("random %d" % k, bytes(b))
    return F


def corpus_arrays(stride=STRIDE):
    F = corpus_frames()
    n = len(F)
    frames = np.zeros((n, stride), dtype=np.uint8)
    meta = np.zeros(n, dtype=abi.META_DT)
    labels = []
    for i, (f, m, lab) in enumerate(F):
        b = np.frombuffer(f[:stride], np.uint8)
        frames[i, :len(b)] = b
        meta[i]["iface"] = m["iface"]
        meta[i]["vlan_ck"] = (m["vlan"] & 0xFFF) | (m["ck"] << 12)
        meta[i]["pkt_len"] = m["pkt_len"]
        meta[i]["rss"] = m["rss"]
        labels.append(lab)
    return frames, meta, labels


# ---- eth_output's per-walk source-MAC cache (eth_output.c:37-59) ----------
# Graph walks of packets from p0 in the corpus topology, each with the
# positions (in the walk) that grout sends out with source MAC
# 00:00:00:00:00:00, derived by hand from eth_output.c:37-59 and rte_graph's
# pending-queue order (ip6_input before ip_input when it got a packet first).
#   X  forward via p1 (nh "fwd")         Z  forward via p2 (nh "fwd2")
#   Y  egress iface without a MAC        X6 IPv6 forward via p1 (nh "fwd6")
#   Y6 IPv6 egress without a MAC         V  egress VLAN 200 (parent p1)
#   D  egress iface admin down (eth_output runs, iface_output drops)
#   T  ttl 1 (never reaches eth_output)
ETH_OUTPUT_CACHE_WALKS = [
    ("X Y X", {2}),
    ("Y X", set()),
    ("X Y Z X", set()),
    ("X Y X X Z X", {2, 3}),
    ("X6 X Y X X6", {3}),          # ip6_input first: [X6 X6 | X Y X]
    ("X X6 Y X X6", {1, 3, 4}),    # ip_input first: [X Y X | X6 X6]
    ("X Y6 X", set()),             # [X X | Y6]
    ("X Y6 X6", {2}),              # [X | Y6 X6]
    ("V Y V", {2}),
    ("X Y T X", {3}),
    ("D Y D", {2}),
    ("X D Y X", set()),
    ("X Y", set()),
    ("X", set()),                  # a new walk: the cache starts empty
    ("X Y " + "X " * 62, set(range(2, 64))),
    ("Z Y Z Y Z X Y X", {2, 4, 7}),
]


# Walks longer than a 64-packet tile (grout's rx_burst_max / vector_max go up
# to 256, graph.c:612-650): the same rule over the whole walk, derived by hand.
ETH_OUTPUT_CACHE_LONG_WALKS = [
    ("Z " * 63 + "X Y X", {65}),                      # the failed lookup and its victim in the second tile
    ("X " + "Z " * 62 + "Y Z X X X", {64}),           # the lookup fails at the tile's end, Z after it is zeroed
    ("X Y " + "X " * 130, set(range(2, 132))),        # three tiles of zeroed X
    ("X6 " + "X " * 64 + "Y X X6", {66}),             # ip6_input first: [X6 X6 | X*64 Y X], one zero past a tile
    ("X Y " + "X " * 254, set(range(2, 256))),        # a whole 256-packet walk
]


def eth_output_cache_arrays(stride=STRIDE, walks=None):
    """frames, meta (abi.META_WALK at each walk start), labels, zero (bool:
    grout sends the packet with a zero source MAC). walks: (spec, zero set)
    pairs, ETH_OUTPUT_CACHE_WALKS by default; walks longer than 64 are for
    node mbuf walks (oracle burst >= their length), not device batches."""
    walks = ETH_OUTPUT_CACHE_WALKS if walks is None else walks
    fr, f6 = S.frame, S.frame6
    make = {
        "X": lambda k: fr(dst="16.1.7.%d" % (k % 250 + 1)),
        "Z": lambda k: fr(dst="10.90.1.%d" % (200 + k % 50)),
        "Y": lambda k: fr(dst="10.76.0.%d" % (k % 250 + 1)),
        "V": lambda k: fr(dst="10.74.0.%d" % (k % 250 + 1)),
        "D": lambda k: fr(dst="10.73.0.%d" % (k % 250 + 1)),
        "T": lambda k: fr(dst="16.1.7.%d" % (k % 250 + 1), ttl=1),
        "X6": lambda k: f6(dst="2001:db8:100::%x" % (k + 1)),
        "Y6": lambda k: f6(dst="2001:db8:107::%x" % (k + 1)),
    }
    rows, walk, zero, labels = [], [], [], []
    k = 0
    for w, (spec, z) in enumerate(walks):
        syms = spec.split()
        while len(syms) <= 64 and len(rows) % 64 + len(syms) > 64:  # a batch walk never straddles a tile: pad
            rows.append(None)
            walk.append(True)
            zero.append(False)
            labels.append("pad")
        for j, sym in enumerate(syms):
            rows.append(make[sym](k))
            walk.append(j == 0)
            zero.append(j in z)
            labels.append("walk %d %s[%d]" % (w, sym, j))
            k += 1
    n = len(rows)
    frames = np.zeros((n, stride), dtype=np.uint8)
    meta = np.zeros(n, dtype=abi.META_DT)
    for i, f in enumerate(rows):
        if f is None:  # iface 0: punted, counted nowhere, its own walk
            meta[i]["vlan_ck"] = abi.META_WALK
            continue
        frames[i, :len(f)] = np.frombuffer(f[:stride], np.uint8)
        meta[i]["iface"] = P0
        meta[i]["vlan_ck"] = (abi.CKSUM_UNKNOWN << 12) | (abi.META_WALK if walk[i] else 0)
        meta[i]["pkt_len"] = len(f)
    return frames, meta, labels, np.array(zero)


def clustered_routes6(seed):
    """IPv6 prefixes in six clusters shaped to trigger the trie's level
    compressions (fib6.c widen: dense fan-outs of /40-/64 under one-byte
    skips, at bytes 2-5), each with a covering prefix, plus 200 sparse deep
    routes; unique, masked, nh and vrf left to the caller."""
    rng = np.random.default_rng(0x6C0 + seed)
    rows = []
    for c in range(6):
        base = rng.integers(0, 256, 16, dtype=np.uint8)
        base[0] = 0x20 + c
        depth = int(rng.integers(2, 6))  # the byte the cluster fans out at
        fan = int(rng.choice([4, 24, 96]))
        for a in rng.choice(256, size=fan, replace=False):
            for b in rng.choice(256, size=int(rng.integers(2, 40)), replace=False):
                ip = base.copy()
                ip[depth], ip[depth + 1] = a, b
                rows.append((ip, 8 * (depth + 2)))
        rows.append((base, 8 * depth - int(rng.integers(0, 5))))  # a covering prefix
    for _ in range(200):  # sparse deep routes
        ip = rng.integers(0, 256, 16, dtype=np.uint8)
        ip[0] = 0x20 + int(rng.integers(0, 16))
        rows.append((ip, int(rng.integers(17, 129))))
    r = np.zeros(len(rows), dtype=abi.ROUTE6_DT)
    for i, (ip, ln) in enumerate(rows):
        m = np.zeros(16, dtype=np.uint8)
        full = ln // 8
        m[:full] = ip[:full]
        if ln % 8:
            m[full] = ip[full] & ((0xFF00 >> (ln % 8)) & 0xFF)
        r[i]["ip"], r[i]["prefixlen"] = m, ln
    _, keep = np.unique(np.concatenate([r["ip"], r["prefixlen"][:, None]], axis=1), axis=0, return_index=True)
    return r[np.sort(keep)]
