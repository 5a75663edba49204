# SPDX-License-Identifier: BSD-3-Clause
"""Control-plane objects for the fast path, built with grout's semantics.

A Topology holds the iface table, the nexthop slots, the ECMP reta and the
routes exactly as grout's control plane would leave them for the datapath:

* add_port / add_vrf / add_vlan: struct iface (modules/infra/control/iface.h:
  20-35); VRF id 1 is the default VRF (gr_infra.h:51).
* add_address: addr4_add (modules/ip/control/address.c:60-115) -- one L3
  nexthop flagged LOCAL|LINK, REACHABLE, carrying the iface MAC, and a route
  on the address prefix (host bits masked by the FIB).
* add_nexthop: a gr_nexthop_info_l3 (gr_nexthop.h:93-105); a MAC makes it
  REACHABLE (l3_nexthop.c:244-250), no address makes it a LINK nexthop
  (l3_nexthop.c:233-238).
* add_group: GR_NH_T_GROUP with grout's weighted reta (group_reta_distribute,
  group_import_info: group_nexthop.c:27-56,101-166).
* add_route: gr_ip4_route_add_req (modules/ip/api/gr_ip4.h:47-56).
* IPv6: every VRF also gets a FIB6 (modules/ip6/control/route.c:103-125); an
  IPv6 nexthop address makes an AF_IP6 nexthop; add_address6 mirrors
  addr6_add (modules/ip6/control/address.c) and add_route6
  gr_ip6_route_add_req, a link-local prefix scoped to its iface.
* config_fullview / config_fullview6: fib_inject -4 / -6's route sets
  (smoke/fib_inject.c), ported in csrc/synth.c.

The same arrays feed the HIP library (grout_amd.fwd) and the test oracle.
"""
import ipaddress

import numpy as np

from . import abi


def ip4(s):
    """'a.b.c.d' -> host-order int."""
    return int(ipaddress.IPv4Address(s))


def ip6(s):
    """IPv6 text -> 16 bytes (network order)."""
    return ipaddress.IPv6Address(s).packed


def mac_bytes(m):
    if isinstance(m, (bytes, bytearray)):
        return bytes(m)
    return bytes(int(x, 16) for x in m.split(":"))


class Topology:
    def __init__(self, max_ifaces=1024, max_nexthops=1 << 17):
        self.max_ifaces = max_ifaces
        self.max_nexthops = max_nexthops
        self.ifaces = np.zeros(max_ifaces, dtype=abi.IFACE_DT)
        self.nh = np.zeros(max_nexthops + 1, dtype=abi.NH_DT)  # slot 0 = NULL
        self.n_nh = 0  # highest slot used
        self.reta = np.zeros(0, dtype=np.uint32)
        self.routes = []  # list of ROUTE_DT arrays
        self.fibs = {}  # vrf_id -> (max_routes, num_tbl8)
        self.routes6 = []  # list of ROUTE6_DT arrays
        self.fibs6 = {}  # vrf_id -> (max_routes, num_groups)

    # -- interfaces ---------------------------------------------------------
    def _iface(self, iface_id, itype, mode, flags, mtu, vrf_id, mac, **kw):
        if not 0 < iface_id < self.max_ifaces:
            raise ValueError("iface id")
        r = self.ifaces[iface_id]
        r["id"] = iface_id
        r["type"] = abi.IFACE_TYPE[itype]
        r["mode"] = abi.IFACE_MODE[mode] if isinstance(mode, str) else mode
        r["flags"] = flags
        r["mtu"] = mtu
        r["vrf_id"] = vrf_id
        if mac is not None:
            r["mac"] = np.frombuffer(mac_bytes(mac), np.uint8)
            r["mac_ok"] = 1
        else:
            r["mac"] = 0
            r["mac_ok"] = 0
        for k, v in kw.items():
            r[k] = v
        return iface_id

    def add_vrf(self, vrf_id=1, mac=None, max_routes=1 << 16, num_tbl8=0, max_routes6=1 << 16, num_groups6=0):
        """A VRF iface and its IPv4 and IPv6 FIBs (fib4_init, modules/ip/control/route.c:100-122)."""
        self._iface(vrf_id, "VRF", "VRF", abi.IFACE_F_UP, 1500, vrf_id, mac)
        self.fibs[vrf_id] = (max_routes, num_tbl8)
        self.fibs6[vrf_id] = (max_routes6, num_groups6)
        return vrf_id

    def add_port(self, iface_id, port_id, mac, vrf_id=1, mtu=1500, up=True, mode="VRF", flags=0):
        f = (abi.IFACE_F_UP if up else 0) | flags
        return self._iface(iface_id, "PORT", mode, f, mtu, vrf_id, mac, port_id=port_id)

    def add_vlan(self, iface_id, parent_id, vlan_id, mac=None, vrf_id=1, mtu=1500, up=True, flags=0):
        if mac is None:  # a VLAN set without a MAC takes its parent's (iface_vlan_set_eth_addr, modules/infra/control/vlan.c:180-192)
            p = self.ifaces[parent_id]
            mac = bytes(p["mac"]) if p["mac_ok"] else None
        f = (abi.IFACE_F_UP if up else 0) | flags
        return self._iface(iface_id, "VLAN", "VRF", f, mtu, vrf_id, mac,
                           vlan_id=vlan_id, parent_id=parent_id)

    def add_iface(self, iface_id, itype, mac=None, vrf_id=1, mode="VRF", mtu=1500, up=True, flags=0, **kw):
        f = (abi.IFACE_F_UP if up else 0) | flags
        return self._iface(iface_id, itype, mode, f, mtu, vrf_id, mac, **kw)

    def iface_mac(self, iface_id):
        r = self.ifaces[iface_id]
        return bytes(r["mac"]) if r["mac_ok"] else None

    # -- nexthops -----------------------------------------------------------
    def _slot(self, slot):
        if slot is None:
            slot = self.n_nh + 1
        if not 0 < slot <= self.max_nexthops:
            raise ValueError("nexthop slot")
        self.n_nh = max(self.n_nh, slot)
        return slot

    def add_nexthop(self, iface_id, ipv4=None, mac=None, nh_type="L3", state=None, flags=0,
                    vrf_id=None, slot=None):
        slot = self._slot(slot)
        r = self.nh[slot]
        r["type"] = abi.NH_T[nh_type]
        r["iface_id"] = iface_id
        r["vrf_id"] = vrf_id if vrf_id is not None else (self.ifaces[iface_id]["vrf_id"] if iface_id else 1)
        if nh_type == "L3":
            if ipv4 is None:
                r["af"] = abi.AF_UNSPEC
                flags |= abi.NH_F_LINK
            elif isinstance(ipv4, str) and ":" in ipv4:  # an IPv6 nexthop
                r["af"] = abi.AF_IP6
                r["ipv6"] = np.frombuffer(ip6(ipv4), np.uint8)
            else:
                r["af"] = abi.AF_IP4
                r["ipv4"] = ip4(ipv4) if isinstance(ipv4, str) else ipv4
            if mac is not None:
                r["mac"] = np.frombuffer(mac_bytes(mac), np.uint8)
                if state is None:
                    state = abi.NH_S["REACHABLE"]
        r["flags"] = flags
        r["state"] = state if state is not None else abi.NH_S["NEW"]
        return slot

    def add_address(self, iface_id, cidr):
        """addr4_add: LOCAL|LINK nexthop + route on the address prefix."""
        net = ipaddress.IPv4Interface(cidr)
        slot = self.add_nexthop(iface_id, str(net.ip), self.iface_mac(iface_id),
                                flags=abi.NH_F_LOCAL | abi.NH_F_LINK,
                                state=abi.NH_S["REACHABLE"])
        self.add_route(self.ifaces[iface_id]["vrf_id"], f"{net.ip}/{net.network.prefixlen}", slot)
        return slot

    def add_address6(self, iface_id, cidr):
        """addr6_add: LOCAL|LINK nexthop + route on the address prefix."""
        net = ipaddress.IPv6Interface(cidr)
        slot = self.add_nexthop(iface_id, str(net.ip), self.iface_mac(iface_id),
                                flags=abi.NH_F_LOCAL | abi.NH_F_LINK,
                                state=abi.NH_S["REACHABLE"])
        self.add_route6(self.ifaces[iface_id]["vrf_id"], f"{net.ip}/{net.network.prefixlen}", slot,
                        iface_id=iface_id)
        return slot

    def add_group(self, members, reta_size=None, slot=None, weights=None):
        """GR_NH_T_GROUP with the reta grout builds for it (group_import_info,
        modules/infra/control/group_nexthop.c:101-166): members ordered by
        weight, descending (:137-140; glibc's qsort keeps equal weights in
        order), reta_size = align32pow2(max/min weight x n_members) capped at
        MAX_NH_GROUP_RETA_SIZE 4096 (:142-154, nexthop.h:80), filled by
        group_reta_distribute (:27-56). `reta_size` overrides the size (the
        fill stays grout's); one member needs no reta (:131-135)."""
        slot = self._slot(slot)
        r = self.nh[slot]
        r["type"] = abi.NH_T["GROUP"]
        r["n_members"] = len(members)
        r["single"] = members[0] if len(members) == 1 else 0
        w = [max(1, x) for x in weights] if weights is not None else [1] * len(members)  # weight ?: 1 (:125)
        order = sorted(range(len(members)), key=lambda i: -w[i])
        mem, w = [members[i] for i in order], [w[i] for i in order]
        if reta_size is None:
            reta_size = min((w[0] // w[-1]) * len(mem), 4096) if mem else 1
            p = 1
            while p < reta_size:
                p *= 2
            reta_size = p
        if reta_size & (reta_size - 1):
            raise ValueError("reta size must be a power of two")
        r["reta_size"] = reta_size
        r["reta_off"] = len(self.reta)
        fill = []
        total = sum(w)
        for m, x in zip(mem, w):  # group_reta_distribute
            e = max((x * reta_size + total // 2) // total, 1)
            fill += [m] * min(e, reta_size - len(fill))
            if len(fill) >= reta_size:
                break
        fill += [mem[0] if mem else 0] * (reta_size - len(fill))
        self.reta = np.concatenate([self.reta, np.array(fill, dtype=np.uint32)])
        return slot

    # -- routes ---------------------------------------------------------------
    def add_route(self, vrf_id, cidr, nh_slot):
        net = ipaddress.IPv4Network(cidr, strict=False)
        a = np.zeros(1, dtype=abi.ROUTE_DT)
        a["ip"] = int(net.network_address)
        a["prefixlen"] = net.prefixlen
        a["vrf_id"] = vrf_id
        a["nh"] = nh_slot
        self.routes.append(a)

    def add_routes(self, arr):
        self.routes.append(np.ascontiguousarray(arr, dtype=abi.ROUTE_DT))

    def route_array(self):
        if not self.routes:
            return np.zeros(0, dtype=abi.ROUTE_DT)
        # np.concatenate normalises byte order: convert back to the C layout
        return np.concatenate(self.routes).astype(abi.ROUTE_DT)

    def add_route6(self, vrf_id, cidr, nh_slot, iface_id=0):
        net = ipaddress.IPv6Network(cidr, strict=False)
        a = np.zeros(1, dtype=abi.ROUTE6_DT)
        a["ip"] = np.frombuffer(net.network_address.packed, np.uint8)
        a["prefixlen"] = net.prefixlen
        a["vrf_id"] = vrf_id
        a["iface_id"] = iface_id
        a["nh"] = nh_slot
        self.routes6.append(a)

    def add_routes6(self, arr):
        self.routes6.append(np.ascontiguousarray(arr, dtype=abi.ROUTE6_DT))

    def route6_array(self):
        if not self.routes6:
            return np.zeros(0, dtype=abi.ROUTE6_DT)
        return np.concatenate(self.routes6).astype(abi.ROUTE6_DT)

    def live_ifaces(self):
        return self.ifaces[self.ifaces["id"] != 0]


# ---------------------------------------------------------------------------
# the BASELINE topologies
# ---------------------------------------------------------------------------
PORT_MAC = ["02:00:00:00:00:0%d" % p for p in range(4)]
SRC_MAC = "02:00:00:ff:ff:ff"
VRF_MAIN = 1
PORT_IFACE = [2, 3, 4, 5]  # p0..p3
N_FULLVIEW_NH = 2048


def base_ports(max_routes=1 << 16, num_tbl8=0, max_nexthops=1 << 17):
    t = Topology(max_nexthops=max_nexthops)
    t.add_vrf(VRF_MAIN, max_routes=max_routes, num_tbl8=num_tbl8)
    for p in range(4):
        t.add_port(PORT_IFACE[p], p, PORT_MAC[p])
    return t


def config_single_route():
    """smoke/ip_forward_test.sh:7-13 with nexthop 45 resolved (config 2)."""
    t = base_ports()
    t.add_address(PORT_IFACE[0], "172.16.0.1/24")
    t.add_address(PORT_IFACE[1], "172.16.1.1/24")
    gw = t.add_nexthop(PORT_IFACE[0], "172.16.0.2")  # 16.0.0.0/16 via 172.16.0.2 (unresolved)
    t.add_route(VRF_MAIN, "16.0.0.0/16", gw)
    nh45 = t.add_nexthop(PORT_IFACE[1], "172.16.1.2", "02:00:00:01:00:2d")
    t.add_route(VRF_MAIN, "16.1.0.0/16", nh45)
    return t


def fullview_nexthops(t, n_nh=N_FULLVIEW_NH):
    """nh j -> {p(1+(j-1)%3), 100.64.(j>>8).(j&255), 02:00:00:01:(j>>8):(j&255)}."""
    first = t.n_nh + 1
    for j in range(1, n_nh + 1):
        port = 1 + (j - 1) % 3
        t.add_nexthop(PORT_IFACE[port], f"100.64.{j >> 8}.{j & 255}",
                      "02:00:00:01:%02x:%02x" % (j >> 8, j & 255), slot=first + j - 1)
    return first


def config_fullview(count=1_000_000):
    """fib_inject -4 -n count over 2048 REACHABLE nexthops (configs 3-5)."""
    import ctypes
    t = base_ports(max_routes=count + 10)
    first = fullview_nexthops(t)
    routes = np.zeros(count, dtype=abi.ROUTE_DT)
    abi.check("gr_synth_fullview_routes",
              abi.host().gr_synth_fullview_routes(count, VRF_MAIN, first, N_FULLVIEW_NH,
                                                  routes.ctypes.data))
    t.add_routes(routes)
    t.add_address(PORT_IFACE[0], "172.16.0.1/24")
    del ctypes
    return t


# IPv6 full view: exactly fib_inject -6's route set (smoke/fib_inject.c:
# 38-47,136-179; smoke/fib6_fullview_manualtest.sh injects 200,000), over
# the same 2048 nexthops as the IPv4 view, made REACHABLE IPv6 nexthops
# instead of fib_inject's blackholes so that packets forward.
N_FULLVIEW6_NH = 2048
FULLVIEW6_ROUTES = 200_000


def fullview6_nexthops(t, n_nh=N_FULLVIEW6_NH):
    """nh j -> {p(1+(j-1)%3), 2001:db8:ffff::j, 02:00:00:06:(j>>8):(j&255)}."""
    first = t.n_nh + 1
    for j in range(1, n_nh + 1):
        port = 1 + (j - 1) % 3
        t.add_nexthop(PORT_IFACE[port], f"2001:db8:ffff::{j:x}", "02:00:00:06:%02x:%02x" % (j >> 8, j & 255),
                      slot=first + j - 1)
    return first


def fullview6_routes(count, vrf_id, first_nh, n_nh):
    """fib_inject -6 -n count: route i -> nexthop first_nh + i % n_nh."""
    r = np.zeros(count, dtype=abi.ROUTE6_DT)
    abi.check("gr_synth_fullview6_routes",
              abi.host().gr_synth_fullview6_routes(count, vrf_id, first_nh, n_nh, r.ctypes.data))
    return r


def config_fullview6(count=FULLVIEW6_ROUTES):
    """fib_inject -6 -n count over 2048 REACHABLE IPv6 nexthops (the IPv6 workload)."""
    t = base_ports(max_routes=1 << 10)
    t.fibs6[VRF_MAIN] = (count + 10, max(1 << 16, 4 * count))  # ~3-4 trie groups per deep route
    first = fullview6_nexthops(t)
    t.add_routes6(fullview6_routes(count, VRF_MAIN, first, N_FULLVIEW6_NH))
    t.add_address6(PORT_IFACE[0], "2001:db8::1/64")
    return t
