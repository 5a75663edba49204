# SPDX-License-Identifier: BSD-3-Clause
"""grout's smoke/ip_forward_test.sh (BASELINE config 1) restated as packets.

The script builds two ports with connected /24s, `16.0.0.0/16 via
172.16.0.2`, nexthop 45 on p1 and `16.1.0.0/16 via id 45` (:7-13), puts a
Linux namespace behind each port (:15-27) and checks reachability with ping
and TTL expiry with traceroute (:29-38). DPDK and network namespaces are not
available here, so each ping / traceroute becomes the frame it would put on
the wire, and the check is the edge and rewrite grout's chain gives it:
before the namespaces' addresses are resolved (ARP on the CPU: ip_hold) and
after (the host routes grout installs for resolved neighbours, forwarded).
The expectations are written out from the script, not taken from the
oracle; the CPU test runs the oracle, the GPU test the HIP path."""
import numpy as np
import pytest

import oracle
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

P0, P1 = T.PORT_IFACE[0], T.PORT_IFACE[1]
N0_MAC, N1_MAC = "02:00:00:0a:00:00", "02:00:00:0a:00:01"  # the namespaces' ends of x-p0, x-p1


def smoke_topology(resolved):
    t = T.base_ports()
    t.add_address(P0, "172.16.0.1/24")  # ip_forward_test.sh:9
    t.add_address(P1, "172.16.1.1/24")  # :10
    gw = t.add_nexthop(P0, "172.16.0.2", N0_MAC if resolved else None)
    t.add_route(T.VRF_MAIN, "16.0.0.0/16", gw)  # :11
    # :12 "nexthop add l3 iface p1 id 45": no address, so GR_AF_UNSPEC + GR_NH_F_LINK
    # (l3_nexthop.c:233-239), like a connected route: every destination is held and learned
    nh45 = t.add_nexthop(P1, None, slot=45)
    t.add_route(T.VRF_MAIN, "16.1.0.0/16", nh45)  # :13
    if resolved:  # the /32 routes grout adds for neighbours it resolved (ARP, nexthop.c:62-90)
        t.add_route(T.VRF_MAIN, "16.1.0.1/32", t.add_nexthop(P1, "16.1.0.1", N1_MAC))  # n1's x-p1 (:24)
        t.add_route(T.VRF_MAIN, "172.16.0.2/32", t.add_nexthop(P0, "172.16.0.2", N0_MAC))
        t.add_route(T.VRF_MAIN, "172.16.1.2/32", t.add_nexthop(P1, "172.16.1.2", N1_MAC))
    return t


# (script line, ingress iface, src MAC, src, dst, ttl, edge before / after resolution, egress iface)
PINGS = [
    (29, P0, N0_MAC, "172.16.0.2", "16.1.0.1", 64, "ip_hold", "port_output", P1),
    (30, P1, N1_MAC, "16.1.0.1", "16.0.0.1", 64, "ip_hold", "port_output", P0),
    (31, P0, N0_MAC, "172.16.0.2", "172.16.1.2", 64, "ip_hold", "port_output", P1),
    (32, P1, N1_MAC, "172.16.1.2", "172.16.0.2", 64, "ip_hold", "port_output", P0),
    (33, P0, N0_MAC, "172.16.0.2", "172.16.0.1", 64, "ip_input_local", "ip_input_local", None),
    (34, P1, N1_MAC, "172.16.1.2", "172.16.1.1", 64, "ip_input_local", "ip_input_local", None),
    # traceroute -N1: the first probe carries TTL 1 and dies at grout
    (35, P0, N0_MAC, "172.16.0.2", "16.1.0.1", 1, "ip_error_ttl_exceeded", "ip_error_ttl_exceeded", None),
    (36, P1, N1_MAC, "16.1.0.1", "16.0.0.1", 1, "ip_error_ttl_exceeded", "ip_error_ttl_exceeded", None),
    (37, P0, N0_MAC, "172.16.0.2", "172.16.1.2", 1, "ip_error_ttl_exceeded", "ip_error_ttl_exceeded", None),
    (38, P1, N1_MAC, "172.16.1.2", "172.16.0.2", 1, "ip_error_ttl_exceeded", "ip_error_ttl_exceeded", None),
]


def frames():
    fr = [S.frame(dst_mac=T.PORT_MAC[0] if iface == P0 else T.PORT_MAC[1], src_mac=smac, src=src, dst=dst, ttl=ttl,
                  proto=1, length=98)  # ICMP echo, ping's default 64-byte payload
          for _, iface, smac, src, dst, ttl, *_ in PINGS]
    return S.pack(fr, stride=128, iface=[p[1] for p in PINGS])


def check(out, v, resolved):
    for i, (line, _, _, _, _, ttl, before, after, egress) in enumerate(PINGS):
        want = after if resolved else before
        got = abi.EDGE_NAMES[v["edge"][i]]
        assert got == want, (f"ip_forward_test.sh:{line}", got, want)
        if want != "port_output":
            continue
        assert v["iface"][i] == egress  # the port behind iface_output
        peer = {P0: N0_MAC, P1: N1_MAC}[egress]
        if line == 29:
            peer = N1_MAC  # 16.1.0.1 learned behind nexthop 45: n1
        assert bytes(out[i][0:6]) == T.mac_bytes(peer)
        assert bytes(out[i][6:12]) == T.mac_bytes(T.PORT_MAC[0] if egress == P0 else T.PORT_MAC[1])
        assert out[i][22] == ttl - 1
        # the rewritten header still checksums to zero
        hdr = bytes(out[i][14:34])
        s = sum(int.from_bytes(hdr[k:k + 2], "big") for k in range(0, 20, 2))
        s = (s & 0xFFFF) + (s >> 16)
        assert (s + (s >> 16)) & 0xFFFF == 0xFFFF


@pytest.mark.parametrize("resolved", [False, True])
def test_smoke_ip_forward_oracle(resolved):
    t = smoke_topology(resolved)
    arr, meta = frames()
    out, v, _ = oracle.Oracle(t).process(arr, meta)
    check(out, v, resolved)


@pytest.mark.gpu
@pytest.mark.parametrize("resolved", [False, True])
def test_smoke_ip_forward_gpu(fastpath, resolved):
    from golden_util import run_gpu
    t = smoke_topology(resolved)
    arr, meta = frames()
    out, v, _ = run_gpu(fastpath, t, arr, meta)
    check(out, v, resolved)
    o_out, o_v, _ = oracle.Oracle(t).process(arr, meta)
    assert np.array_equal(v, o_v) and np.array_equal(out, o_out)
