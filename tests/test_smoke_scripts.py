# SPDX-License-Identifier: BSD-3-Clause
"""grout's forwarding smoke scripts restated as packets, on the CPU oracle and
through the rte_graph node walk on the GPU.

Each script builds a topology with grcli, puts Linux namespaces behind the
ports and checks reachability with ping / ping6 / traceroute. DPDK and
network namespaces are not available here, so every probe becomes the frame
it would put on the wire, entering the port it would enter, and the check
is what grout's chain does with it: the next node (edge), the egress port and
VLAN tag, the rewritten Ethernet header, TTL / hop limit and checksum. Each
script runs twice: before the namespaces' neighbours are resolved (ARP / NDP
on the CPU: ip_hold / ip6_hold) and after (the host routes grout installs for
the neighbours it learned, modules/ip/control/nexthop.c:62-90 and
modules/ip6/control/nexthop.c:65-90: packets are forwarded).

The expectations below are written from the scripts and grout's node code,
not taken from the oracle. The CPU test checks the oracle against them; the
GPU test checks the HIP node walk against them and against the oracle, mbuf
for mbuf.

Scripts (under smoke/ in the reference):
  ip6_forward_test.sh       IPv6 gateway and link nexthops, link-local, NDP
  vlan_forward_test.sh      VLAN sub-interfaces on both sides
  vrf_forward_test.sh       two VRFs holding the same addresses and routes
  cross_vrf_forward_test.sh a route whose nexthop is another VRF (xvrf)
  ip_forward_ip6nh_test.sh  IPv4 routes via IPv6 link-local nexthops
  ip_loadbalance_test.sh    an ECMP group of two nexthops
  ip_fragment_test.sh       a 1280-byte MTU: DF (frag needed) and not (fragment)
  ipip_encap_test.sh        an IPIP tunnel interface (ipip_output)
  snat44_test.sh            dynamic SNAT (the CPU's conntrack continuations)
  dnat44_test.sh            a static DNAT nexthop (dnat44_static)
  bridge_test.sh            ports in a bridge domain (bridge_input)
  ip6_same_peer_test.sh     a link-local address only on its own link
  srv6_test.sh              SRv6 encap and local nexthops (sr6_output, sr6_local)
  ip_builtin_icmp_test.sh   grout's own pings: the replies, unroutable and unanswered hosts
  ip6_builtin_icmp_test.sh  the same for IPv6
  iface_mac_test.sh         secondary MACs: frames for them are another host's
  nexthop_ageing_test.sh    neighbours REACHABLE, STALE / FAILED, aged out
  vxlan_test.sh             a VXLAN VTEP, the decapsulated frames back through iface_input
  bond_active_backup_test.sh frames from the active member with the bond as iface, LACP, bond_output
  ip_add_del_test.sh        an IPv4 address deleted and added again
  ip6_add_del_test.sh       an IPv6 address deleted and added again; the port moved to a
                            VRF, then cross-connected
  srv6_end_x_test.sh        an SRv6 End.X SID (sr6_local) beside plain IPv6 forwarding

For the address and ageing scripts, "resolved" names the script's later
state (the address added again, the neighbours answering again), as each
function's docstring says.
"""
import ipaddress
import os

import numpy as np
import pytest

import oracle
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T
from test_node_shim import RX_DATA_OFF, compare_mbufs, mbufs_for

GR_MAC = ["02:00:00:00:00:%02x" % p for p in range(4)]  # grout's ports p0..p3
NS_MAC = ["02:00:00:0a:00:%02x" % n for n in range(4)]  # the namespaces' ends x-p0..x-p3
PORT = [10, 11, 12, 13]  # iface ids of p0..p3 (1 and 2 are left to the VRF ifaces)
REF_SMOKE = "/root/reference/smoke"  # read as text by test_probe_lines_are_the_scripts only


def eui64_ll(mac):
    """fe80::/64 + modified EUI-64 of a MAC (rte_ipv6_llocal_from_ethernet),
    the link-local address grout and Linux give a port."""
    b = bytearray(T.mac_bytes(mac))
    iid = bytes([b[0] ^ 0x02, b[1], b[2], 0xFF, 0xFE, b[3], b[4], b[5]])
    return str(ipaddress.IPv6Address(b"\xfe\x80" + bytes(6) + iid))


def ports(t, n, vrf=None):
    for p in range(n):
        v = vrf[p] if vrf else T.VRF_MAIN
        t.add_port(PORT[p], p, GR_MAC[p], vrf_id=v)
        t.add_address6(PORT[p], eui64_ll(GR_MAC[p]) + "/64")  # the link-local address every port gets


def neighbour(t, vrf, iface, addr, mac):
    """A neighbour grout learned: nexthop + host route (nexthop.c: rib4_insert /32, rib6 /128)."""
    nh = t.add_nexthop(iface, addr, mac)
    if ":" in addr:
        t.add_route6(vrf, addr + "/128", nh, iface_id=iface if addr.startswith("fe80") else 0)
    else:
        t.add_route(vrf, addr + "/32", nh)
    return nh


class Probe:
    """One frame on the wire and what grout does with it.

    before / after: the edge before and after neighbour resolution; `out`:
    (egress port index, VLAN tag, destination MAC) when it is port_output."""

    def __init__(self, script, line, port, frame, before, after=None, out=None, vlan=0, out_any=None, rss=0,
                 iface=None):
        self.script, self.line, self.port, self.frame = script, line, port, frame
        self.before, self.after = before, after if after is not None else before
        self.out, self.out_any, self.vlan, self.rss = out, out_any, vlan, rss
        # the iface port_rx (or a CPU node going back to iface_input) hands the
        # frame over with, when it is not the port itself
        self.iface = iface

    @property
    def label(self):
        return f"{self.script}:{self.line}"


def v4(port, src, dst, ttl=64, proto=1, vlan=0, dst_mac=None, size=56, df=False):
    # ping -s size: ICMP echo, 8-byte header + size bytes (default 56: a 98-byte IP
    # packet); traceroute: UDP probe; df: ping -M do (IP_PMTUDISC_DO)
    length = 14 + 20 + 8 + size if proto == 1 else 14 + 60
    return S.frame(dst_mac=dst_mac or GR_MAC[port], src_mac=NS_MAC[port], src=src, dst=dst, ttl=ttl,
                   proto=proto, length=length, flags_frag=0x4000 if df else 0)


def arp(port, dst_mac="ff:ff:ff:ff:ff:ff", src_mac=None):
    """An ARP frame (a request, broadcast; a reply, to grout's MAC)."""
    return S.frame(dst_mac=dst_mac, src_mac=src_mac or NS_MAC[port], ethertype=0x0806)


def v6(port, src, dst, hop=64, nh=58, dst_mac=None):
    length = 14 + 40 + 64 if nh == 58 else 14 + 40 + 32
    return S.frame6(dst_mac=dst_mac or GR_MAC[port], src_mac=NS_MAC[port], src=src, dst=dst, hop=hop,
                    next_header=nh, length=length)


# ---------------------------------------------------------------------------
# the scripts
# ---------------------------------------------------------------------------
def ip6_forward(resolved):
    """smoke/ip6_forward_test.sh: ports p1, p2 (here p0, p1 of this file's
    numbering: n1 behind p0, n2 behind p1)."""
    s = "ip6_forward_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    P1, P2 = PORT[0], PORT[1]
    t.add_address6(P1, "fd00:ba4:1::1/64")  # :9
    t.add_address6(P2, "fd00:ba4:2::1/64")  # :10
    gw = t.add_nexthop(P1, "fd00:ba4:1::2", NS_MAC[0] if resolved else None)  # :11 (via fd00:ba4:1::2)
    t.add_route6(T.VRF_MAIN, "fd00:f00:1::/64", gw)
    nh45 = t.add_nexthop(P2, None, slot=45)  # :12 no address: GR_AF_UNSPEC + GR_NH_F_LINK (l3_nexthop.c:233-239)
    t.add_route6(T.VRF_MAIN, "fd00:f00:2::/64", nh45)  # :13
    if resolved:
        neighbour(t, T.VRF_MAIN, P1, "fd00:ba4:1::2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, P2, "fd00:ba4:2::2", NS_MAC[1])
        neighbour(t, T.VRF_MAIN, P2, "fd00:f00:2::2", NS_MAC[1])  # on n2's x-p2 (:24): learned through nh45
        neighbour(t, T.VRF_MAIN, P1, eui64_ll(NS_MAC[0]), NS_MAC[0])
        neighbour(t, T.VRF_MAIN, P2, eui64_ll(NS_MAC[1]), NS_MAC[1])
    n1_ll, n2_ll = eui64_ll(NS_MAC[0]), eui64_ll(NS_MAC[1])
    pr = [
        # ping6 to grout's link-local addresses (:29-30)
        Probe(s, 29, 0, v6(0, n1_ll, eui64_ll(GR_MAC[0])), "ip6_input_local"),
        Probe(s, 30, 1, v6(1, n2_ll, eui64_ll(GR_MAC[1])), "ip6_input_local"),
        # n1 -> fd00:f00:2::2 via id 45 (a link nexthop: the neighbour is learned, :31)
        Probe(s, 31, 0, v6(0, "fd00:ba4:1::2", "fd00:f00:2::2"), "ip6_hold", "port_output", (1, 0, NS_MAC[1])),
        # n2 -> fd00:f00:1::2 via the gateway fd00:ba4:1::2 (:32)
        Probe(s, 32, 1, v6(1, "fd00:f00:2::2", "fd00:f00:1::2"), "ip6_hold", "port_output", (0, 0, NS_MAC[0])),
        # the connected /64s (:33-34)
        Probe(s, 33, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:2::2"), "ip6_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 34, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:1::2"), "ip6_hold", "port_output", (0, 0, NS_MAC[0])),
        # the neighbour solicitation for grout's address after the flush (:39-40): to the
        # solicited-node group, whose membership lives on the CPU (mcast6_get_member)
        Probe(s, 40, 0, v6(0, n1_ll, "ff02::1:ff00:1", hop=255, dst_mac="33:33:ff:00:00:01"), "punt"),
        Probe(s, 40, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:1::1"), "ip6_input_local"),
        Probe(s, 40, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:2::1"), "ip6_input_local"),
        # traceroute -N1: the first probe carries hop limit 1 (:46-49)
        Probe(s, 46, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:2::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        Probe(s, 47, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:1::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        Probe(s, 48, 0, v6(0, "fd00:ba4:1::2", "fd00:f00:2::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        Probe(s, 49, 1, v6(1, "fd00:f00:2::2", "fd00:f00:1::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        # a second hop: the probe with hop limit 2 leaves with 1
        Probe(s, 48, 0, v6(0, "fd00:ba4:1::2", "fd00:f00:2::2", hop=2, nh=17), "ip6_hold", "port_output",
              (1, 0, NS_MAC[1])),
    ]
    return t, pr


def vlan_forward(resolved):
    """smoke/vlan_forward_test.sh: p0.42 and p1.43 over ports p0, p1; the
    namespaces tag their frames (port_rx strips the tag into vlan_id,
    port_rx.c:227-232, iface_input demuxes it, iface_input.c:74-86)."""
    s = "vlan_forward_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    V0, V1 = 20, 21
    t.add_vlan(V0, PORT[0], 42)  # :9
    t.add_vlan(V1, PORT[1], 43)  # :10
    t.add_address(V0, "172.16.0.1/24")  # :11
    t.add_address(V1, "172.16.1.1/24")  # :12
    if resolved:
        neighbour(t, T.VRF_MAIN, V0, "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, V1, "172.16.1.2", NS_MAC[1])
    pr = [
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 43, NS_MAC[1]), vlan=42),
        Probe(s, 28, 1, v4(1, "172.16.1.2", "172.16.0.2"), "ip_hold", "port_output", (0, 42, NS_MAC[0]), vlan=43),
        # the namespaces' ARP requests for their gateway, tagged
        Probe(s, 27, 0, S.frame(dst_mac="ff:ff:ff:ff:ff:ff", src_mac=NS_MAC[0], ethertype=0x0806), "arp_input",
              vlan=42),
        # ping the gateway itself
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local", vlan=42),
        # an untagged frame stays on p0 itself, in the same VRF: routed all the same
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 43, NS_MAC[1])),
        # a tag with no VLAN interface (iface_input.c:80-83)
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.1.2"), "iface_input_unknown_vlan", vlan=44),
    ]
    return t, pr


def vrf_forward(resolved):
    """smoke/vrf_forward_test.sh: p0, p1 in gr-vrf1 and p2, p3 in gr-vrf2 with
    the same addresses and routes; n0..n3 behind them, n1 and n3 holding the
    same addresses (only their MACs tell them apart)."""
    s = "vrf_forward_test.sh"
    t = T.Topology()
    t.add_vrf(1)  # gr-vrf1 (:7)
    t.add_vrf(2)  # gr-vrf2 (:8)
    ports(t, 4, vrf=[1, 1, 2, 2])  # :9-12
    for vrf, a, b in ((1, PORT[0], PORT[1]), (2, PORT[2], PORT[3])):
        t.add_address(a, "172.16.0.1/24")  # :13, :17
        t.add_address(b, "172.16.1.1/24")  # :14, :18
        k = 0 if vrf == 1 else 2
        g0 = t.add_nexthop(a, "172.16.0.2", NS_MAC[k] if resolved else None)
        g1 = t.add_nexthop(b, "172.16.1.2", NS_MAC[k + 1] if resolved else None)
        t.add_route(vrf, "16.0.0.0/16", g0)  # :15, :19
        t.add_route(vrf, "16.1.0.0/16", g1)  # :16, :20
        if resolved:
            neighbour(t, vrf, a, "172.16.0.2", NS_MAC[k])
            neighbour(t, vrf, b, "172.16.1.2", NS_MAC[k + 1])
    pr = [
        Probe(s, 31, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 32, 0, v4(0, "172.16.0.2", "16.1.0.1"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 32, 1, v4(1, "16.1.0.1", "172.16.0.2"), "ip_hold", "port_output", (0, 0, NS_MAC[0])),
        Probe(s, 43, 2, v4(2, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (3, 0, NS_MAC[3])),
        Probe(s, 44, 2, v4(2, "172.16.0.2", "16.1.0.1"), "ip_hold", "port_output", (3, 0, NS_MAC[3])),
        Probe(s, 44, 3, v4(3, "16.1.0.1", "172.16.0.2"), "ip_hold", "port_output", (2, 0, NS_MAC[2])),
        # each VRF's own gateway address
        Probe(s, 31, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local"),
        Probe(s, 43, 2, v4(2, "172.16.0.2", "172.16.0.1"), "ip_input_local"),
        # 16.0.0.0/16 has no route in either VRF's view from the far side except via the gateway
        Probe(s, 44, 3, v4(3, "16.1.0.1", "10.9.9.9"), "ip_error_dest_unreach"),
    ]
    return t, pr


def cross_vrf_forward(resolved):
    """smoke/cross_vrf_forward_test.sh: p0 in gr-vrf1, p1 in gr-vrf2. From
    16.0.0.1 to 16.1.0.1 one lookup in gr-vrf1 leaves by p1 (nexthop id 2
    lives in gr-vrf2); the way back looks up gr-vrf2 first, whose nexthop is
    the gr-vrf1 interface: ip_output hands it to xvrf (xvrf.c:61-64), which
    re-enters ip_input in gr-vrf1 on the CPU."""
    s = "cross_vrf_forward_test.sh"
    t = T.Topology()
    t.add_vrf(1)  # :7
    t.add_vrf(2)  # :8
    ports(t, 2, vrf=[1, 2])  # :9-10
    t.add_address(PORT[0], "172.16.0.1/24")  # :11
    t.add_address(PORT[1], "172.16.1.1/24")  # :12
    nh2 = t.add_nexthop(PORT[1], "172.16.1.2", NS_MAC[1] if resolved else None, slot=2)  # :15
    t.add_route(1, "16.1.0.0/16", nh2)  # :16
    t.add_route(2, "16.1.0.0/16", nh2)  # :17
    nh1 = t.add_nexthop(1, None, slot=1)  # :20 l3 iface gr-vrf1 (no address: LINK)
    t.add_route(2, "16.0.0.0/16", nh1)  # :21
    gw = t.add_nexthop(PORT[0], "172.16.0.2", NS_MAC[0] if resolved else None)
    t.add_route(1, "16.0.0.0/16", gw)  # :22
    pr = [
        Probe(s, 34, 0, v4(0, "16.0.0.1", "16.1.0.1"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 35, 1, v4(1, "16.1.0.1", "16.0.0.1"), "xvrf"),
        Probe(s, 35, 1, v4(1, "16.1.0.1", "16.0.0.1", ttl=1), "ip_error_ttl_exceeded"),
        # gr-vrf2 holds no route to 172.16.0.0/24
        Probe(s, 35, 1, v4(1, "16.1.0.1", "172.16.0.2"), "ip_error_dest_unreach"),
    ]
    return t, pr


def ip_forward_ip6nh(resolved):
    """smoke/ip_forward_ip6nh_test.sh: 16.n.0.0/16 via nexthop 42+n, an L3
    nexthop on p_n whose address is n's IPv6 link-local address (:18-20). The
    nexthop is IPv6, the packets IPv4: ip_output only needs it reachable
    (ip_output.c:126-138), and eth_output writes the IPv4 ether type."""
    s = "ip_forward_ip6nh_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    for n in (0, 1):
        nh = t.add_nexthop(PORT[n], eui64_ll(NS_MAC[n]), NS_MAC[n] if resolved else None, slot=42 + n)  # :19
        t.add_route(T.VRF_MAIN, f"16.{n}.0.0/16", nh)  # :20
    pr = [
        # n routes 16.(n^1).0.0/16 via grout's link-local: frames to p_n's MAC (:16, :25)
        Probe(s, 25, 0, v4(0, "16.0.0.1", "16.1.0.1"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 25, 1, v4(1, "16.1.0.1", "16.0.0.1"), "ip_hold", "port_output", (0, 0, NS_MAC[0])),
        Probe(s, 25, 0, v4(0, "16.0.0.1", "16.1.0.1", ttl=1, proto=17), "ip_error_ttl_exceeded"),
    ]
    return t, pr


def ip_loadbalance(resolved):
    """smoke/ip_loadbalance_test.sh: 192.200.0.0/24 via group 10 = {100 on p0,
    101 on p1} (:37-40). The script's own probes are grout-originated pings
    (:43-44, they enter at ip_output, off this path) whose replies come back
    to grout's addresses; transit frames from n1 behind p2 take the group,
    one member per RSS hash (nexthop.h:89-96)."""
    s = "ip_loadbalance_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 3)
    for p in range(3):
        t.add_address(PORT[p], f"172.16.{p}.1/24")  # :32-34
    m100 = t.add_nexthop(PORT[0], "172.16.0.2", NS_MAC[0] if resolved else None, slot=100)  # :37
    m101 = t.add_nexthop(PORT[1], "172.16.1.2", NS_MAC[1] if resolved else None, slot=101)  # :38
    g = t.add_group([m100, m101], slot=10)  # :39
    t.add_route(T.VRF_MAIN, "192.200.0.0/24", g)  # :40
    pr = [
        # the echo replies to grout's pings, one through each member
        Probe(s, 43, 0, v4(0, "192.200.0.2", "172.16.0.1"), "ip_input_local"),
        Probe(s, 44, 1, v4(1, "192.200.0.2", "172.16.1.1"), "ip_input_local"),
    ]
    for rss in range(8):  # n1 -> 192.200.0.2, every reta slot of the group
        pr.append(Probe(s, 40, 2, v4(2, "172.16.2.2", "192.200.0.2"), "ip_hold", "port_output",
                        out_any=[(0, 0, NS_MAC[0]), (1, 0, NS_MAC[1])], rss=rss))
    return t, pr


def ip_fragment(resolved):
    """smoke/ip_fragment_test.sh: p1's MTU is 1280 (:10). A 1260-byte ping is a
    1288-byte IP packet: with DF it must fail (ip_error_frag_needed, :34),
    without DF grout fragments it (ip_fragment, :42); ip_output.c:99-106."""
    s = "ip_fragment_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.ifaces[PORT[1]]["mtu"] = 1280  # port_add p1 mtu 1280 (:10)
    t.add_address(PORT[0], "172.16.0.1/24")  # :11
    t.add_address(PORT[1], "172.16.1.1/24")  # :12
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "172.16.1.2", NS_MAC[1])
    pr = [
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 34, 0, v4(0, "172.16.0.2", "172.16.1.2", size=1260, df=True), "ip_error_frag_needed"),
        Probe(s, 42, 0, v4(0, "172.16.0.2", "172.16.1.2", size=1260), "ip_fragment"),
        # exactly the MTU passes, one byte more does not
        Probe(s, 42, 0, v4(0, "172.16.0.2", "172.16.1.2", size=1252, df=True), "ip_hold", "port_output",
              (1, 0, NS_MAC[1])),
        Probe(s, 42, 0, v4(0, "172.16.0.2", "172.16.1.2", size=1253, df=True), "ip_error_frag_needed"),
        # the replies come back the other way, on the 1500-byte port
        Probe(s, 42, 1, v4(1, "172.16.1.2", "172.16.0.2", size=1260), "ip_hold", "port_output", (0, 0, NS_MAC[0])),
    ]
    return t, pr


def ipip_encap(resolved):
    """smoke/ipip_encap_test.sh: tun1 is an IPIP interface (local 172.16.1.1,
    remote 172.16.1.2) holding 10.98.0.1/24 (:11-12). n0's ping to 10.98.0.2
    leaves ip_output through tun1's type edge, ipip_output (ipip/datapath_out.c:91),
    whether or not a neighbour is resolved (ip_output.c:110-122); the tunnelled
    packets n1 sends back are for grout's own 172.16.1.1 (ipip_input on the CPU)."""
    s = "ipip_encap_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    TUN = 30
    t.add_address(PORT[0], "10.99.0.1/24")  # :9
    t.add_address(PORT[1], "172.16.1.1/24")  # :10
    t.add_iface(TUN, "IPIP")  # :11
    t.add_address(TUN, "10.98.0.1/24")  # :12
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "10.99.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "172.16.1.2", NS_MAC[1])
    pr = [
        Probe(s, 27, 0, v4(0, "10.99.0.2", "10.98.0.2"), "ipip_output"),
        Probe(s, 28, 1, v4(1, "172.16.1.2", "172.16.1.1", proto=4), "ip_input_local"),  # IPIP to grout
        Probe(s, 27, 0, v4(0, "10.99.0.2", "10.98.0.2", ttl=1), "ip_error_ttl_exceeded"),
    ]
    return t, pr


def snat44(resolved):
    """smoke/snat44_test.sh: dynamic SNAT on p0 (:11; GR_IFACE_F_SNAT_DYNAMIC,
    modules/policy/control/snat44_dynamic.c:39). n1's ping to 172.16.0.2 leaves
    through p0: the fast path stops where ip_output calls snat44_process
    (ip_output_snat, run on the CPU); the replies to the SNAT address arrive on
    p0 and stop where ip_input calls into conntrack (ip_input_local_ct)."""
    s = "snat44_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.ifaces[PORT[0]]["flags"] |= abi.IFACE_F_SNAT_DYNAMIC  # :11
    t.add_address(PORT[0], "172.16.0.1/24")  # :9
    t.add_address(PORT[1], "10.99.0.1/24")  # :10
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "10.99.0.99", NS_MAC[1])
    pr = [
        Probe(s, 27, 1, v4(1, "10.99.0.99", "172.16.0.2"), "ip_output_snat"),
        Probe(s, 27, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local_ct"),
        Probe(s, 31, 1, v4(1, "10.99.0.99", "172.16.0.2", proto=6), "ip_output_snat"),  # socat TCP
        Probe(s, 36, 1, v4(1, "10.99.0.99", "172.16.0.2", proto=17), "ip_output_snat"),  # socat UDP
        # p1 has no SNAT policy: n1's ping to grout's own p1 address stays plain local
        Probe(s, 27, 1, v4(1, "10.99.0.99", "10.99.0.1"), "ip_input_local"),
    ]
    return t, pr


def dnat44(resolved):
    """smoke/dnat44_test.sh: a static DNAT of 172.16.0.99 on p0 (:11): a
    GR_NH_T_DNAT nexthop and its /32 route in p0's VRF
    (modules/policy/api/dnat44.c:148-166). n0's ping to 172.16.0.99 leaves
    ip_input by that nexthop type's edge, dnat44_static."""
    s = "dnat44_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address(PORT[0], "172.16.0.1/24")  # :9
    t.add_address(PORT[1], "10.99.0.1/24")  # :10
    t.add_route(T.VRF_MAIN, "172.16.0.99/32", t.add_nexthop(PORT[0], nh_type="DNAT"))  # :11
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "10.99.0.99", NS_MAC[1])
    pr = [
        Probe(s, 26, 0, v4(0, "172.16.0.2", "172.16.0.99"), "dnat44_static"),
        # the address next to it is plain connected
        Probe(s, 26, 0, v4(0, "172.16.0.2", "172.16.0.98"), "ip_hold"),
    ]
    return t, pr


def bridge(resolved):
    """smoke/bridge_test.sh: p0..p2 in bridge br0's domain (:9-11): iface_input's
    mode edge for GR_IFACE_MODE_BRIDGE is bridge_input (bridge_input.c:124),
    which switches on the CPU."""
    s = "bridge_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    BR = 40
    t.add_iface(BR, "BRIDGE", mac=GR_MAC[3])  # :7
    for p in range(3):
        t.add_port(PORT[p], p, GR_MAC[p], mode="BRIDGE")  # :9-11 (the domain itself lives on the CPU)
    t.add_address(BR, "172.16.0.1/24")  # :15
    pr = [
        Probe(s, 26, 0, v4(0, "172.16.0.10", "172.16.0.11", dst_mac=NS_MAC[1]), "bridge_input"),
        Probe(s, 27, 1, v4(1, "172.16.0.11", "172.16.0.12", dst_mac=NS_MAC[2]), "bridge_input"),
        Probe(s, 42, 0, v4(0, "172.16.0.10", "172.16.0.1", dst_mac=GR_MAC[3]), "bridge_input"),
        Probe(s, 26, 0, S.frame(dst_mac="ff:ff:ff:ff:ff:ff", src_mac=NS_MAC[0], ethertype=0x0806), "bridge_input"),
    ]
    return t, pr


def ip6_same_peer(resolved):
    """smoke/ip6_same_peer_test.sh: a link-local address is only reachable on
    its own link (:24: n1's ping to p2's link-local must go unanswered).
    Link-local routes are scoped to their iface (modules/ip6/control/route.c:150-173):
    on p1, fe80::/64 is p1's connected prefix, so the packet is held for a
    neighbour solicitation on p1's link, which nobody answers (ip6_hold in both
    states)."""
    s = "ip6_same_peer_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address6(PORT[0], "fd00:ba4:1::1/64")  # :10
    t.add_address6(PORT[1], "fd00:ba4:2::1/64")  # :11
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "fd00:ba4:1::2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "fd00:ba4:2::2", NS_MAC[1])
        neighbour(t, T.VRF_MAIN, PORT[0], eui64_ll(NS_MAC[0]), NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], eui64_ll(NS_MAC[1]), NS_MAC[1])
    n1_ll, n2_ll = eui64_ll(NS_MAC[0]), eui64_ll(NS_MAC[1])
    pr = [
        Probe(s, 22, 0, v6(0, n1_ll, eui64_ll(GR_MAC[0])), "ip6_input_local"),
        Probe(s, 23, 1, v6(1, n2_ll, eui64_ll(GR_MAC[1])), "ip6_input_local"),
        Probe(s, 24, 0, v6(0, n1_ll, eui64_ll(GR_MAC[1])), "ip6_hold"),  # p2's link-local, asked on p1
        Probe(s, 25, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:2::2"), "ip6_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 26, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:1::2"), "ip6_hold", "port_output", (0, 0, NS_MAC[0])),
        Probe(s, 27, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:1::1"), "ip6_input_local"),
        Probe(s, 28, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:2::1"), "ip6_input_local"),
        Probe(s, 29, 0, v6(0, "fd00:ba4:1::2", "fd00:ba4:2::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        Probe(s, 30, 1, v6(1, "fd00:ba4:2::2", "fd00:ba4:1::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
    ]
    return t, pr


def srv6(resolved):
    """smoke/srv6_test.sh: 192.168.0.0/16 via an SRv6 encap nexthop (id 42,
    :43-44) leaves ip_output by the nexthop type's edge, sr6_output
    (srv6_output.c:152), after ip_forward; fd00:202:100::/48 via an SRv6 local
    End.DT4 nexthop (id 666, :58-59) leaves ip6_input by sr6_local; the
    encapsulated return traffic n1 sends to fd00:202:100:: takes it."""
    s = "srv6_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address6(PORT[1], "fd00:102::1/32")  # :9
    t.add_address(PORT[0], "192.168.61.1/24")  # :10
    sr = t.add_nexthop(0, nh_type="SR6_OUTPUT", slot=42)  # :43
    t.add_route(T.VRF_MAIN, "192.168.0.0/16", sr)  # :44
    gw = t.add_nexthop(PORT[1], "fd00:102::2", NS_MAC[1] if resolved else None)
    t.add_route6(T.VRF_MAIN, "fd00:202::/32", gw)  # :45
    loc = t.add_nexthop(0, nh_type="SR6_LOCAL", slot=666)  # :58
    t.add_route6(T.VRF_MAIN, "fd00:202:100::/48", loc)  # :59
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "192.168.61.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "fd00:102::2", NS_MAC[1])
    pr = [
        Probe(s, 62, 0, v4(0, "192.168.61.2", "192.168.60.1"), "sr6_output"),
        Probe(s, 62, 0, v4(0, "192.168.61.2", "192.168.60.1", ttl=1), "ip_error_ttl_exceeded"),
        Probe(s, 64, 1, v6(1, "fd00:102::2", "fd00:202:100::", nh=43), "sr6_local"),  # IPv6 + routing header
        Probe(s, 64, 1, v6(1, "fd00:102::2", "fd00:202:100::1"), "sr6_local"),
        # the rest of fd00:202::/32 goes back to n1 by the gateway
        Probe(s, 64, 1, v6(1, "fd00:102::2", "fd00:202:200::"), "ip6_hold", "port_output", (1, 0, NS_MAC[1])),
    ]
    return t, pr


def ip_builtin_icmp(resolved):
    """smoke/ip_builtin_icmp_test.sh: p0 holds 172.16.2.1/24 and 172.16.0.1/24,
    p1 172.16.1.1/24 (:9-11). The script's pings and traceroute are grout's
    own (grcli ping, ip_output on the CPU): what comes back on the wire are
    the echo replies, ARP replies and ICMP errors for grout's addresses. The
    two pings that must fail (:30-31) are restated as transit packets from
    n0: no route to 1.1.1.1 (ip_error_dest_unreach, ip_input.c:147-150) and a
    host on p1's link nobody answers ARP for (ip_hold in both states)."""
    s = "ip_builtin_icmp_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address(PORT[0], "172.16.2.1/24")  # :9
    t.add_address(PORT[0], "172.16.0.1/24")  # :10
    t.add_address(PORT[1], "172.16.1.1/24")  # :11
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "172.16.1.2", NS_MAC[1])
    pr = [
        # the echo replies to grcli ping (:24-25), to either of p0's addresses
        Probe(s, 24, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local"),
        Probe(s, 24, 0, v4(0, "172.16.0.2", "172.16.2.1"), "ip_input_local"),
        Probe(s, 25, 1, v4(1, "172.16.1.2", "172.16.1.1"), "ip_input_local"),
        # the ARP replies that resolve the pinged hosts
        Probe(s, 24, 0, arp(0, dst_mac=GR_MAC[0]), "arp_input"),
        Probe(s, 25, 1, arp(1, dst_mac=GR_MAC[1]), "arp_input"),
        # :30 no route, :31 nobody answers
        Probe(s, 30, 0, v4(0, "172.16.0.2", "1.1.1.1"), "ip_error_dest_unreach"),
        Probe(s, 31, 0, v4(0, "172.16.0.2", "172.16.1.3"), "ip_hold"),
        # traceroute's answers (:33): ICMP errors from n0, UDP-probe TTL expiry on the way
        Probe(s, 33, 0, v4(0, "172.16.0.2", "172.16.0.1", proto=1), "ip_input_local"),
        Probe(s, 33, 0, v4(0, "172.16.0.2", "172.16.1.2", ttl=1, proto=17), "ip_error_ttl_exceeded"),
        # and n0 reaching n1 through grout once both are resolved
        Probe(s, 25, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
    ]
    return t, pr


def ip6_builtin_icmp(resolved):
    """smoke/ip6_builtin_icmp_test.sh: fd00:ba4::1/64 on p0, fd00:ba4:1::1/64
    on p1 (:9-10), grcli ping / traceroute of the namespaces (:21-28). The
    replies come back to grout's addresses; the pings that must fail (:25-26)
    are restated as transit: fd00:baa::1 has no route
    (ip6_error_dest_unreach), fd00:ba4:1::3 is never answered (ip6_hold)."""
    s = "ip6_builtin_icmp_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address6(PORT[0], "fd00:ba4:0::1/64")  # :9
    t.add_address6(PORT[1], "fd00:ba4:1::1/64")  # :10
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "fd00:ba4::2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "fd00:ba4:1::2", NS_MAC[1])
    pr = [
        Probe(s, 21, 0, v6(0, "fd00:ba4::2", "fd00:ba4::1"), "ip6_input_local"),
        Probe(s, 22, 1, v6(1, "fd00:ba4:1::2", "fd00:ba4:1::1"), "ip6_input_local"),
        # the neighbour advertisements, unicast to grout's address
        Probe(s, 21, 0, v6(0, "fd00:ba4::2", "fd00:ba4::1", hop=255), "ip6_input_local"),
        Probe(s, 25, 0, v6(0, "fd00:ba4::2", "fd00:baa::1"), "ip6_error_dest_unreach"),
        Probe(s, 26, 0, v6(0, "fd00:ba4::2", "fd00:ba4:1::3"), "ip6_hold"),
        Probe(s, 28, 1, v6(1, "fd00:ba4:1::2", "fd00:ba4:1::1", nh=58), "ip6_input_local"),
        Probe(s, 28, 0, v6(0, "fd00:ba4::2", "fd00:ba4:1::2", hop=1, nh=17), "ip6_error_ttl_exceeded"),
        # the namespaces reach each other over fd00:ba4::/62 (:18)
        Probe(s, 22, 0, v6(0, "fd00:ba4::2", "fd00:ba4:1::2"), "ip6_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 21, 1, v6(1, "fd00:ba4:1::2", "fd00:ba4::2"), "ip6_hold", "port_output", (0, 0, NS_MAC[0])),
    ]
    return t, pr


MAC_SECONDARY = ["02:00:00:00:00:01", "02:00:00:00:00:02", "02:00:00:00:00:03"]  # iface_mac_test.sh:11-13


def iface_mac(resolved):
    """smoke/iface_mac_test.sh: secondary MAC addresses on p0 (:16-18, deleted
    again at :38, :69, :83; resolved = after the deletions). They are the
    port's receive filter (rte_eth_dev_mac_addr_add, modules/infra/control/port.c);
    eth_input compares the destination with the iface's one address,
    iface_get_eth_addr (eth_input.c:62-77): a frame for a secondary MAC is
    ETH_DOMAIN_OTHER and ip_input / ip6_input drop it as for another host,
    in both states. The primary MAC is p0's own (:8: no address, so no route)."""
    s = "iface_mac_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 1)
    pr = [
        Probe(s, 16, 0, v4(0, "10.0.0.2", "10.0.0.1", dst_mac=MAC_SECONDARY[0]), "ip_input_other_host"),
        Probe(s, 17, 0, v4(0, "10.0.0.2", "10.0.0.1", dst_mac=MAC_SECONDARY[1]), "ip_input_other_host"),
        Probe(s, 18, 0, v6(0, eui64_ll(NS_MAC[0]), eui64_ll(GR_MAC[0]), dst_mac=MAC_SECONDARY[2]),
              "ip6_input_other_host"),
        # the primary MAC: no IPv4 address or route on p0, but the link-local address every port gets
        Probe(s, 8, 0, v4(0, "10.0.0.2", "10.0.0.1"), "ip_error_dest_unreach"),
        Probe(s, 8, 0, v6(0, eui64_ll(NS_MAC[0]), eui64_ll(GR_MAC[0])), "ip6_input_local"),
        # ARP to a secondary MAC: eth_input's ether type edge does not look at the domain
        Probe(s, 16, 0, arp(0, dst_mac=MAC_SECONDARY[0]), "arp_input"),
    ]
    return t, pr


def nexthop_ageing(resolved):
    """smoke/nexthop_ageing_test.sh: p0 172.16.0.1/24, p1 172.16.1.1/24
    (:32-33); the namespaces' pings (:44-45) make grout learn both neighbours
    (resolved: REACHABLE, and still so after the lifetime expired and the
    probes were answered, :54-55). With the namespaces' links down the
    nexthops age out and are destroyed (:69-70; l3_age, l3_nexthop.c:313-360):
    not resolved, the /32 routes are gone and the connected prefixes' LINK
    nexthops hold the packets for ARP again (ip_output.c:126-137)."""
    s = "nexthop_ageing_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address(PORT[0], "172.16.0.1/24")  # :32
    t.add_address(PORT[1], "172.16.1.1/24")  # :33
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "172.16.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[1], "172.16.1.2", NS_MAC[1])
    pr = [
        Probe(s, 44, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 45, 1, v4(1, "172.16.1.2", "172.16.0.2"), "ip_hold", "port_output", (0, 0, NS_MAC[0])),
        Probe(s, 44, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local"),
        # the addresses outlive the neighbours (:58-59, :73-74)
        Probe(s, 58, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_input_local"),
        Probe(s, 59, 1, v4(1, "172.16.1.2", "172.16.1.1"), "ip_input_local"),
    ]
    return t, pr


def nexthop_ageing_stale(resolved):
    """smoke/nexthop_ageing_test.sh between :49 and :54: the neighbours'
    lifetime has expired (REACHABLE -> STALE, l3_nexthop.c:351-354) and the
    probes are out; a probe left unanswered makes one FAILED
    (l3_nexthop.c:329-340). Not resolved: 172.16.1.2 STALE and 172.16.0.2
    FAILED, their /32 routes still in place; ip_output holds packets for
    any nexthop that is not REACHABLE (ip_output.c:126-137). Resolved: the
    probes were answered, both REACHABLE again (:54-55)."""
    s = "nexthop_ageing_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 2)
    t.add_address(PORT[0], "172.16.0.1/24")  # :32
    t.add_address(PORT[1], "172.16.1.1/24")  # :33
    st0 = None if resolved else abi.NH_S["FAILED"]
    st1 = None if resolved else abi.NH_S["STALE"]
    n0 = t.add_nexthop(PORT[0], "172.16.0.2", NS_MAC[0], state=st0)
    t.add_route(T.VRF_MAIN, "172.16.0.2/32", n0)
    n1 = t.add_nexthop(PORT[1], "172.16.1.2", NS_MAC[1], state=st1)
    t.add_route(T.VRF_MAIN, "172.16.1.2/32", n1)
    pr = [
        Probe(s, 54, 0, v4(0, "172.16.0.2", "172.16.1.2"), "ip_hold", "port_output", (1, 0, NS_MAC[1])),
        Probe(s, 55, 1, v4(1, "172.16.1.2", "172.16.0.2"), "ip_hold", "port_output", (0, 0, NS_MAC[0])),
        Probe(s, 54, 1, v4(1, "172.16.1.2", "172.16.0.2", ttl=1), "ip_error_ttl_exceeded"),
    ]
    return t, pr


def vxlan(resolved):
    """smoke/vxlan_test.sh: p0 10.0.0.1/24 (:9), bridge br100 (:10) holding
    192.168.100.1/24 (:14), VXLAN vxlan100 (VNI 100, local 10.0.0.1) in
    br100's domain (:11). n1's VXLAN packets are UDP 4789 to grout's
    10.0.0.1: ip_input_local (then l4 and vxlan_input on the CPU). vxlan_input
    hands the inner frame back to iface_input on vxlan100
    (vxlan_input.c:96-101, edge "iface_input"), whose mode edge is
    bridge_input (bridge_input.c:124); bridge_input hands a frame for the
    bridge's own MAC back to iface_input on br100 (bridge_input.c:85-99),
    which eth_input and ip_input take as local. A routed packet for a
    neighbour on br100 leaves by iface_output's type edge for a bridge,
    bridge_input again (bridge_input.c:125)."""
    s = "vxlan_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 1)
    BR, VX = 40, 41
    BR_MAC = "02:00:00:00:01:00"
    t.add_address(PORT[0], "10.0.0.1/24")  # :9
    t.add_iface(BR, "BRIDGE", mac=BR_MAC)  # :10
    t.add_iface(VX, "VXLAN", mode="BRIDGE")  # :11 (the domain itself lives on the CPU)
    t.add_address(BR, "192.168.100.1/24")  # :14
    N1_BR = "02:00:00:0b:00:64"  # n1's br100 (:19, :24)
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "10.0.0.2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, BR, "192.168.100.2", N1_BR)
    inner = v4(0, "192.168.100.2", "192.168.100.1", dst_mac=BR_MAC)
    inner = inner[:6] + T.mac_bytes(N1_BR) + inner[12:]
    pr = [
        # the encapsulated ping (:29): UDP to the VTEP address
        Probe(s, 29, 0, v4(0, "10.0.0.2", "10.0.0.1", proto=17, size=100), "ip_input_local"),
        # the inner frames after vxlan_input: n1's ARP request, the ping itself
        Probe(s, 29, 0, S.frame(dst_mac="ff:ff:ff:ff:ff:ff", src_mac=N1_BR, ethertype=0x0806), "bridge_input",
              iface=VX),
        Probe(s, 29, 0, inner, "bridge_input", iface=VX),
        # ... and bridge_input's hand-back on br100
        Probe(s, 29, 0, inner, "ip_input_local", iface=BR),
        # p0's side reaching n1's bridge address through grout
        Probe(s, 29, 0, v4(0, "10.0.0.2", "192.168.100.2"), "ip_hold", "bridge_input"),
    ]
    return t, pr


def bond_active_backup(resolved):
    """smoke/bond_active_backup_test.sh: bond0 (active-backup, :24) over
    p0..p2 (:26-28) holding 172.16.0.1/24 (:55); its MAC (:35-37) is
    02:f0:00:b4:44:44. port_rx on the active member hands frames over with the bond
    as their iface (rx_bond_process, port_rx.c:414-456; get_bond :123-139),
    LACP frames (ether type 0x8809) with the member itself, whose
    mode BOND edge is eth_input (lacp_input.c:68) and eth_input's ether type
    edge lacp_input (:67). Routed packets leaving by bond0 take iface_output's
    type edge for a bond, bond_output (bond_output.c:250)."""
    s = "bond_active_backup_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    BOND, BMAC = 50, "02:f0:00:b4:44:44"
    t.add_iface(BOND, "BOND", mac=BMAC)  # :24, :37
    for p in range(3):
        t.add_port(PORT[p], p, GR_MAC[p], mode="BOND")  # :26-28 (the domain lives on the CPU)
    t.add_address(BOND, "172.16.0.1/24")  # :55
    if resolved:
        neighbour(t, T.VRF_MAIN, BOND, "172.16.0.2", NS_MAC[0])
    lacp = S.frame(dst_mac="01:80:c2:00:00:02", src_mac=NS_MAC[1], ethertype=0x8809)
    pr = [
        Probe(s, 59, 1, v4(1, "172.16.0.2", "172.16.0.1", dst_mac=BMAC), "ip_input_local", iface=BOND),
        Probe(s, 64, 0, v4(0, "172.16.0.2", "172.16.0.1", dst_mac=BMAC), "ip_input_local", iface=BOND),
        Probe(s, 12, 1, arp(1), "arp_input", iface=BOND),
        Probe(s, 59, 1, lacp, "lacp_input"),
        # a frame for a member's own MAC is not the bond's
        Probe(s, 59, 1, v4(1, "172.16.0.2", "172.16.0.1", dst_mac=GR_MAC[1]), "ip_input_other_host", iface=BOND),
        # transit back out of bond0 to a neighbour on its link
        Probe(s, 59, 1, v4(1, "172.16.0.9", "172.16.0.2", dst_mac=BMAC), "ip_hold", "bond_output", iface=BOND),
    ]
    return t, pr


def ip_add_del(resolved):
    """smoke/ip_add_del_test.sh: 172.16.0.1/24 on p0 added (:9), deleted
    (:11) and added again (:13). Not resolved: after the delete, no route is
    left (ip_error_dest_unreach); resolved: after the second add, the
    address is local again and its prefix connected (ip_hold)."""
    s = "ip_add_del_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 1)
    if resolved:
        t.add_address(PORT[0], "172.16.0.1/24")  # :13
    pr = [
        Probe(s, 11, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_error_dest_unreach", "ip_input_local"),
        Probe(s, 13, 0, v4(0, "172.16.0.2", "172.16.0.3"), "ip_error_dest_unreach", "ip_hold"),
    ]
    return t, pr


def ip6_add_del(resolved):
    """smoke/ip6_add_del_test.sh: 2001::1/64 on p0 added (:11), deleted (:13),
    added again (:15). Not resolved: after the delete; resolved: after the
    second add. p0's link-local address stays through both."""
    s = "ip6_add_del_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 1)
    if resolved:
        t.add_address6(PORT[0], "2001::1/64")  # :15
    pr = [
        Probe(s, 13, 0, v6(0, "2001::2", "2001::1"), "ip6_error_dest_unreach", "ip6_input_local"),
        Probe(s, 15, 0, v6(0, "2001::2", "2001::3"), "ip6_error_dest_unreach", "ip6_hold"),
        Probe(s, 14, 0, v6(0, eui64_ll(NS_MAC[0]), eui64_ll(GR_MAC[0])), "ip6_input_local"),
    ]
    return t, pr


def ip6_add_del_moves(resolved):
    """smoke/ip6_add_del_test.sh, the moves after :15. Not resolved: p0 set
    to VRF foo (:18-19): its addresses are flushed and its link-local
    re-created in foo (GR_EVENT_IFACE_POST_RECONFIG,
    modules/ip6/control/address.c:469-481), so 2001::1 is gone from both
    VRFs. Resolved: p0 cross-connected to p1 (:23-25, mode XC): iface_input's
    mode edge is xconnect (xconnect.c) and p0's addresses are flushed."""
    s = "ip6_add_del_test.sh"
    FOO = 2
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    t.add_vrf(FOO)
    if resolved:
        t.add_port(PORT[0], 0, GR_MAC[0], mode="XC")  # :24
        t.add_port(PORT[1], 1, GR_MAC[1], mode="XC")  # :25
    else:
        t.add_port(PORT[0], 0, GR_MAC[0], vrf_id=FOO)  # :19
        t.add_address6(PORT[0], eui64_ll(GR_MAC[0]) + "/64")
    pr = [
        Probe(s, 19, 0, v6(0, "2001::2", "2001::1"), "ip6_error_dest_unreach", "xconnect"),
        Probe(s, 19, 0, v6(0, eui64_ll(NS_MAC[0]), eui64_ll(GR_MAC[0])), "ip6_input_local", "xconnect"),
        Probe(s, 24, 0, v4(0, "172.16.0.2", "172.16.0.1"), "ip_error_dest_unreach", "xconnect"),
    ]
    return t, pr


def srv6_end_x(resolved):
    """smoke/srv6_end_x_test.sh: p0, p0-bis, p1 (:40-42) on 2001:db8:61::/64,
    :62::/64 and :101::/64 (:44-46); an SRv6 local End.X nexthop (id 200,
    :82) and 5f00:102::100/128 via it (:84). n1 reaches n0 by SRv6-encapsulated
    packets to that SID (:90-91): ip6_input leaves them by the nexthop type's
    edge, sr6_local (whose End.X then sends the inner packet on p0-bis, on
    the CPU), whatever their hop limit (ip6_forward does not run). n0's pings
    to n1 (:123) are plain IPv6 forwarding from p0 to p1."""
    s = "srv6_end_x_test.sh"
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 3)
    t.add_address6(PORT[0], "2001:db8:61::1/64")  # :44
    t.add_address6(PORT[1], "2001:db8:62::1/64")  # :45
    t.add_address6(PORT[2], "2001:db8:101::1/64")  # :46
    endx = t.add_nexthop(PORT[1], nh_type="SR6_LOCAL", slot=200)  # :82
    t.add_route6(T.VRF_MAIN, "5f00:102::100/128", endx)  # :84
    if resolved:
        neighbour(t, T.VRF_MAIN, PORT[0], "2001:db8:61::2", NS_MAC[0])
        neighbour(t, T.VRF_MAIN, PORT[2], "2001:db8:101::2", NS_MAC[2])
    pr = [
        Probe(s, 123, 0, v6(0, "2001:db8:61::2", "2001:db8:101::2"), "ip6_hold", "port_output", (2, 0, NS_MAC[2])),
        Probe(s, 90, 2, v6(2, "2001:db8:101::2", "5f00:102::100", nh=43), "sr6_local"),
        Probe(s, 90, 2, v6(2, "2001:db8:101::2", "5f00:102::100", nh=43, hop=1), "sr6_local"),
        # another SID of 5f00:102::/32, which grout has no route for
        Probe(s, 92, 2, v6(2, "2001:db8:101::2", "5f00:102::101", nh=43), "ip6_error_dest_unreach"),
        # n1's replies on the way back, plain IPv6 before its encap route exists
        Probe(s, 123, 2, v6(2, "2001:db8:101::2", "2001:db8:61::2"), "ip6_hold", "port_output", (0, 0, NS_MAC[0])),
    ]
    return t, pr


SCRIPTS = {f.__name__: f for f in (ip6_forward, vlan_forward, vrf_forward, cross_vrf_forward, ip_forward_ip6nh,
                                   ip_loadbalance, ip_fragment, ipip_encap, snat44, dnat44, bridge, ip6_same_peer,
                                   srv6, ip_builtin_icmp, ip6_builtin_icmp, iface_mac, nexthop_ageing,
                                   nexthop_ageing_stale, vxlan, bond_active_backup, ip_add_del, ip6_add_del,
                                   ip6_add_del_moves, srv6_end_x)}


# ---------------------------------------------------------------------------
# checks
# ---------------------------------------------------------------------------
def _pack(probes):
    fr = [p.frame for p in probes]
    stride = max(128, -(-max(len(f) for f in fr) // 64) * 64)  # whole frames: pkt_len bytes readable
    arr, meta = S.pack(fr, stride=stride, iface=[p.iface or PORT[p.port] for p in probes],
                       vlan=[p.vlan for p in probes])
    meta["rss"] = [p.rss for p in probes]
    return arr, meta


def check(probes, frames_in, lines, m, resolved):
    """lines: the first 64 bytes of each frame after the walk; m: the mbufs."""
    used = set()
    for i, p in enumerate(probes):
        want = p.after if resolved else p.before
        got = abi.EDGE_NAMES[m["edge"][i]]
        assert got == want, (p.label, i, got, want)
        if want != "port_output":
            continue
        outs = [p.out] if p.out else p.out_any
        eg = [o for o in outs if PORT[o[0]] == m["iface"][i]]
        assert len(eg) == 1, (p.label, i, int(m["iface"][i]))
        port, tag, dmac = eg[0]
        used.add((p.label, port))
        assert m["vlan_id"][i] == tag, (p.label, i, int(m["vlan_id"][i]), tag)
        assert m["data_off"][i] == RX_DATA_OFF  # eth_output prepended the header again
        ln, fi = lines[i], frames_in[i]
        assert bytes(ln[0:6]) == T.mac_bytes(dmac), p.label
        assert bytes(ln[6:12]) == T.mac_bytes(GR_MAC[port]), p.label  # a VLAN iface takes its parent's MAC
        six = fi[12] == 0x86
        assert bytes(ln[12:14]) == (b"\x86\xdd" if six else b"\x08\x00")
        if six:
            assert ln[21] == fi[21] - 1  # ip6_forward.c:25-30
            assert m["packet_type"][i] == abi.PTYPE_L3_IPV6
        else:
            assert ln[22] == fi[22] - 1  # ip_forward.c:25-32
            hdr = bytes(ln[14:34])
            s = sum(int.from_bytes(hdr[k:k + 2], "big") for k in range(0, 20, 2))
            s = (s & 0xFFFF) + (s >> 16)
            assert (s + (s >> 16)) & 0xFFFF == 0xFFFF, p.label
            assert m["packet_type"][i] == abi.PTYPE_L3_IPV4
        # the rest of the line is untouched
        assert bytes(ln[14:21]) == bytes(fi[14:21]) and bytes(ln[26:64]) == bytes(fi[26:64]), p.label
    return used


def expect_both_members(used, resolved):
    if resolved:
        lb = {port for label, port in used if label.startswith("ip_loadbalance")}
        assert lb == {0, 1}, lb  # the group spreads over both members


PARAMS = [(name, r) for name in SCRIPTS for r in (False, True)]


@pytest.mark.parametrize("script,resolved", PARAMS)
def test_smoke_script_oracle(script, resolved):
    t, probes = SCRIPTS[script](resolved)
    fr, me = _pack(probes)
    lines, v, _, m, _ = oracle.Oracle(t).process_mbufs(fr, me)
    used = check(probes, fr, lines, m, resolved)
    if script == "ip_loadbalance":
        expect_both_members(used, resolved)


@pytest.mark.gpu
@pytest.mark.parametrize("script,resolved", PARAMS)
def test_smoke_script_gpu(fastpath, script, resolved):
    """The rte_graph node walk (stage, GPU, hand back onto the mbufs)."""
    from golden_util import fresh_fastpath_state
    t, probes = SCRIPTS[script](resolved)
    fr, me = _pack(probes)
    fresh_fastpath_state(fastpath, t)
    bufs, m = mbufs_for(fr, me)
    q = fastpath.queue()
    try:
        q.node_process(m, burst=64)
    finally:
        q.close()
    used = check(probes, fr, bufs[:, :abi.LINE], m, resolved)
    if script == "ip_loadbalance":
        expect_both_members(used, resolved)
    lines_o, _, _, want, _ = oracle.Oracle(t).process_mbufs(fr, me, lines_only=True)
    compare_mbufs(m, want, bufs, lines_o, [p.label for p in probes])


TRAFFIC = ("ping", "traceroute", "socat", "tracepath", "route add", "encap seg6", "mac add", "address add", "address del", "interface add",
           "interface set", "check_nexthop", "address show")


@pytest.mark.skipif(not os.path.isdir(REF_SMOKE), reason="reference not mounted")
@pytest.mark.parametrize("script", list(SCRIPTS))
def test_probe_lines_are_the_scripts(script):
    """Every probe names the script line whose traffic (or configuration
    step) it restates: that line exists and sends or configures something."""
    for resolved in (False, True):
        _, probes = SCRIPTS[script](resolved)
        for p in probes:
            with open(os.path.join(REF_SMOKE, p.script)) as f:
                lines = f.read().split("\n")
            assert 1 <= p.line <= len(lines), p.label
            text = lines[p.line - 1]
            assert any(w in text for w in TRAFFIC), (p.label, text)


def test_group_reta_is_grouts():
    """The test topologies' group reta follows group_import_info /
    group_reta_distribute (group_nexthop.c:27-56,137-154), written out by hand."""
    t = T.Topology()
    t.add_vrf(T.VRF_MAIN)
    ports(t, 3)
    a, b, c = (t.add_nexthop(PORT[p], f"172.16.{p}.2", NS_MAC[p]) for p in range(3))
    cases = [
        (dict(members=[a, b]), [a, b]),  # 2 x 1 -> 2 entries
        (dict(members=[a, b, c]), [a, b, c, a]),  # 3 -> 4, one entry each, then the first member
        (dict(members=[a, b], weights=[1, 3]), [b] * 6 + [a] * 2),  # ordered by weight: 3/1 x 2 = 6 -> 8
        (dict(members=[a, b, c], reta_size=16), [a] * 5 + [b] * 5 + [c] * 5 + [a]),
        (dict(members=[a, b], weights=[0, 0]), [a, b]),  # weight 0 counts as 1
    ]
    for kw, want in cases:
        g = t.add_group(**kw)
        r = t.nh[g]
        got = t.reta[r["reta_off"]:r["reta_off"] + r["reta_size"]]
        assert list(got) == want, (kw, list(got), want)
