# SPDX-License-Identifier: BSD-3-Clause
"""The control-plane mirror (grout_amd/graph/gpu_fwd4_control.c) driven by
grout's own control sequences.

grout_amd/graph/gr_control_min.c restates how grout's control plane creates,
changes and destroys ifaces, nexthops, routes and addresses, and which
events it pushes (or, for GR_NH_ORIGIN_INTERNAL objects and nexthop state
changes, does not push: integration/grout-gpu_fwd4-control.patch adds the
internal channel the mirror needs there). The sequences below are grout's:

* addr4_add (modules/ip/control/address.c:60-132): an INTERNAL nexthop
  flagged LOCAL|LINK (no event, nexthop.c:341) and the connected route;
* route4_add via a gateway (route.c:336-385): a new STATIC nexthop;
* ARP learning (ip/control/nexthop.c:127-185): a LEARN nexthop and its
  INTERNAL /32 (no route event, route.c:258); a refresh (UPDATE event);
* nh4_resolve_cb (ip/control/nexthop.c:33-125) for a held packet to a
  connected host: a LEARN nexthop + /32, set PENDING without an event;
* l3_age (l3_nexthop.c:322-362): REACHABLE -> STALE without an event;
* the nexthop API (modules/infra/api/nexthop.c:29-78), groups with weights
  (group_nexthop.c), a member deleted out of its group without an event;
* addr4_delete, iface_destroy, nh_del.

CPU: after each step, what the mirror pushed (its shadow) equals the
topology grout's objects describe (grout_amd/topology.py, built with the
mirror's slots), and the mirror recorded no error; without the patch's
channel (the negative control) the mirror misses the address nexthops, the
connected routes and the learned /32s. GPU: whole graph walks on the state
the mirror loaded, against the oracle on that topology: packets to a
resolved connected host leave on port_output, packets to the router's
addresses reach ip_input_local with the address nexthop, nothing is dropped
stale; and a context that diverged is recovered by the mirror's replay."""
import ctypes
import ipaddress

import numpy as np
import pytest

import test_graph_walk as GW
from grout_amd import abi
from grout_amd import synth as S
from grout_amd import topology as T

P, U8, U16, U32, I = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_int

STATS_DT = np.dtype([("events", "<u8"), ("internal", "<u8"), ("commits", "<u8"), ("errors", "<u8"),
                     ("first_error", "<i4"), ("slots_used", "<u4"), ("reta_used", "<u4"), ("routes4", "<u4"),
                     ("routes6", "<u4"), ("pending", "<u4"), ("presync", "<u8"), ("unordered", "<u8"),
                     ("no_timer", "<u8")])
assert STATS_DT.itemsize == 80

ORIGIN_STATIC, ORIGIN_LINK, ORIGIN_LEARN, ORIGIN_INTERNAL = 4, 2, 3, 255
NH_F_NEIGH = 0x20
VRF = T.VRF_MAIN
PORTS = T.PORT_IFACE  # p0..p3: ifaces 2..5, DPDK ports 0..3
GW_MAC = "02:00:00:01:00:02"
NEIGH_MAC = "02:00:00:02:00:07"
HOST3_MAC = "02:00:00:03:00:09"
M100, M101 = "02:00:00:03:01:00", "02:00:00:03:01:01"

_set = False


def lib():
    global _set
    L = GW.lib()
    if not _set:
        sig = {
            "gc_begin": (I, []), "gc_end": (I, []),
            "gc_vrf_add": (I, [U16, U32, U32, U32, U32]),
            "gc_port_add": (I, [U16, U16, P, U16, U16, I, U16]),
            "gc_vlan_add": (I, [U16, U16, U16, P, U16, I]),
            "gc_iface_up": (I, [U16, I]), "gc_iface_mac": (I, [U16, P]), "gc_iface_del": (I, [U16]),
            "gc_addr4_add": (I, [U16, U32, U8]), "gc_addr4_del": (I, [U16, U32, U8]),
            "gc_addr6_add": (I, [U16, P, U8]), "gc_addr6_del": (I, [U16, P, U8]),
            "gc_route4_add": (I, [U16, U32, U8, U32, U32, U8, I]), "gc_route4_del": (I, [U16, U32, U8, I]),
            "gc_route6_add": (I, [U16, P, U8, P, U32, U8, I]), "gc_route6_del": (I, [U16, P, U8, I]),
            "gc_route4_add_many": (I, [U16, U32, U8, U32, U32, U8]),
            "gc_arp_many": (I, [U16, U32, U32, P]),
            "gc_arp": (I, [U16, U32, P]), "gc_ndp": (I, [U16, P, P]),
            "gc_resolve4": (I, [U16, U32]), "gc_age4": (I, [U16, U32, U32, U32]),
            "gc_nh_add_l3": (I, [U32, U16, U32, P, U8, I]), "gc_nh_add_type": (I, [U32, U8, U16, U8]),
            "gc_nh_add_group": (I, [U32, U32, P, P, U8, I]), "gc_nh_del": (I, [U32, I]),
            "gc_nh_del_l3": (I, [U16, U32, I]),
            "gc_slot4": (U32, [U16, U32]), "gc_slot6": (U32, [U16, U16, P]), "gc_slot_id": (U32, [U32]),
            "gc_slot_route4": (U32, [U16, U32, U8]), "gc_nh_count": (U32, []), "gc_events": (None, [P]),
            "gr_test_internal_events": (None, [I]),
            "gpu_fwd4_control_nh": (I, [U32, P]), "gpu_fwd4_control_iface": (I, [U16, P]),
            "gpu_fwd4_control_reta": (I, [U32, P, U32]), "gpu_fwd4_control_routes4": (I, [P, U32]),
            "gpu_fwd4_control_routes6": (I, [P, U32]), "gpu_fwd4_control_stats": (None, [P]),
            "gpu_fwd4_control_replay": (I, [U32]),
            "gc_arp_vrf_resize": (I, [U16, U16, U32, P, U32, U32]), "gc_attach": (I, [I]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _set = True
    return L


def be(ip):
    """An IPv4 address as the uint32 whose memory is network order (ip4_addr_t)."""
    return int.from_bytes(ipaddress.IPv4Address(ip).packed, "little")


def mac(m):
    return ctypes.create_string_buffer(T.mac_bytes(m), 6)


def ok(r):
    assert r >= 0, r
    return r


def stats():
    s = np.zeros(1, dtype=STATS_DT)
    lib().gpu_fwd4_control_stats(s.ctypes.data)
    return s[0]


# ---------------------------------------------------------------------------
# grout's control sequences
# ---------------------------------------------------------------------------
def build_base():
    """VRF 1, ports p0..p3 with an address each, a gateway route resolved by
    ARP, a learned neighbour, a weighted group and a blackhole through the
    nexthop API."""
    L = lib()
    ok(L.gc_vrf_add(VRF, 1 << 16, 0, 1 << 16, 0))
    for p, ifid in enumerate(PORTS):
        assert L.gc_port_add(ifid, p, mac(T.PORT_MAC[p]), VRF, 1500, 1, 0) == ifid
        ok(L.gc_addr4_add(ifid, be(f"172.16.{p}.1"), 24))
    ok(L.gc_route4_add(VRF, be("16.0.0.0"), 8, be("172.16.1.2"), 0, ORIGIN_STATIC, 0))
    ok(L.gc_route4_add(VRF, be("17.0.0.0"), 8, be("172.16.1.2"), 0, ORIGIN_STATIC, 0))  # the same nexthop
    ok(L.gc_arp(PORTS[1], be("172.16.1.2"), mac(GW_MAC)))  # the gateway answers: REACHABLE
    ok(L.gc_arp(PORTS[2], be("172.16.2.7"), mac(NEIGH_MAC)))  # a neighbour learned: LEARN + INTERNAL /32
    ok(L.gc_nh_add_l3(100, PORTS[3], be("172.16.3.20"), mac(M100), ORIGIN_STATIC, 0))
    ok(L.gc_nh_add_l3(101, PORTS[3], be("172.16.3.21"), mac(M101), ORIGIN_STATIC, 0))
    ids, w = (ctypes.c_uint32 * 2)(100, 101), (ctypes.c_uint32 * 2)(1, 3)
    ok(L.gc_nh_add_group(200, 2, ids, w, ORIGIN_STATIC, 0))
    ok(L.gc_route4_add(VRF, be("18.0.0.0"), 8, 0, 200, ORIGIN_STATIC, 0))
    ok(L.gc_nh_add_type(300, abi.NH_T["BLACKHOLE"], VRF, ORIGIN_STATIC))
    ok(L.gc_route4_add(VRF, be("19.0.0.0"), 8, 0, 300, ORIGIN_STATIC, 0))


class Want:
    """The topology grout's objects describe, at the mirror's slots."""

    def __init__(self):
        self.t = T.Topology()
        # a VRF's iface_get_eth_addr succeeds with its (zero) router MAC (vrf.c:366-370)
        self.t.add_vrf(VRF, mac="00:00:00:00:00:00")
        self.ports = set()

    def port(self, p, up=True):
        self.t.add_port(PORTS[p], p, T.PORT_MAC[p], up=up)
        self.ports.add(p)

    def address(self, p, cidr):
        L = lib()
        net = ipaddress.IPv4Interface(cidr)
        s = L.gc_slot4(VRF, be(str(net.ip)))
        assert s, cidr
        self.t.add_nexthop(PORTS[p], str(net.ip), T.PORT_MAC[p], flags=abi.NH_F_LOCAL | abi.NH_F_LINK,
                           state=abi.NH_S["REACHABLE"], slot=s)
        self.t.add_route(VRF, str(net.network), s)
        return s

    def l3(self, slot, p, ip, m=None, state=None, flags=0):
        assert slot
        self.t.add_nexthop(PORTS[p], ip, m, state=state, flags=flags, slot=slot)
        return slot

    def route(self, cidr, slot):
        self.t.add_route(VRF, cidr, slot)

    def drop_nh(self, slot):
        """A nexthop gone, with the routes naming it."""
        self.t.nh[slot] = 0
        r = self.t.route_array()
        self.t.routes = [r[r["nh"] != slot]]

    def drop_iface(self, p):
        self.t.ifaces[PORTS[p]] = 0


def want_base(w, gw_state="REACHABLE", neigh_state="REACHABLE", group=True):
    L = lib()
    for p in range(4):
        w.port(p)
        w.address(p, f"172.16.{p}.1/24")
    g = w.l3(L.gc_slot4(VRF, be("172.16.1.2")), 1, "172.16.1.2", GW_MAC, abi.NH_S[gw_state])
    w.route("16.0.0.0/8", g)
    w.route("17.0.0.0/8", g)
    n = w.l3(L.gc_slot4(VRF, be("172.16.2.7")), 2, "172.16.2.7", NEIGH_MAC, abi.NH_S[neigh_state], NH_F_NEIGH)
    w.route("172.16.2.7/32", n)
    a = w.l3(L.gc_slot_id(100), 3, "172.16.3.20", M100)
    b = w.l3(L.gc_slot_id(101), 3, "172.16.3.21", M101)
    if group:
        grp = L.gc_slot_id(200)
        w.t.add_group([a, b], weights=[1, 3], slot=grp)
        w.route("18.0.0.0/8", grp)
    bh = L.gc_slot_id(300)
    w.t.add_nexthop(0, nh_type="BLACKHOLE", vrf_id=VRF, slot=bh)
    w.route("19.0.0.0/8", bh)
    return dict(gw=g, neigh=n, m100=a, m101=b, bh=bh)


def check_shadow(w):
    """What the mirror pushed == the topology grout's objects describe."""
    L = lib()
    t = w.t
    st = stats()
    assert st["errors"] == 0, st
    # ifaces
    live = t.live_ifaces()
    for r in live:
        got = np.zeros(1, dtype=abi.IFACE_DT)
        assert L.gpu_fwd4_control_iface(int(r["id"]), got.ctypes.data) == 0, r["id"]
        for f in ("id", "type", "mode", "flags", "mtu", "vrf_id", "port_id", "vlan_id", "parent_id", "mac", "mac_ok"):
            assert np.array_equal(got[0][f], r[f]), (int(r["id"]), f, got[0][f], r[f])
    # nexthops: every slot the topology uses, and no other
    used = {i for i in range(1, t.n_nh + 1) if t.nh[i]["type"] != 0}
    assert st["slots_used"] == len(used), (st["slots_used"], sorted(used))
    for s in used:
        got = np.zeros(1, dtype=abi.NH_DT)
        assert L.gpu_fwd4_control_nh(s, got.ctypes.data) == 0, s
        g, e = got[0], t.nh[s]
        for f in ("type", "state", "flags", "af", "iface_id", "vrf_id", "ipv4", "mac", "ipv6", "n_members"):
            assert np.array_equal(g[f], e[f]), (s, f, g[f], e[f])
        if e["type"] == abi.NH_T["GROUP"]:
            if e["n_members"] == 1:
                assert g["single"] == e["single"], (s, g["single"], e["single"])
            elif e["n_members"] > 1:
                assert g["reta_size"] == e["reta_size"]
                rg = np.zeros(int(g["reta_size"]), dtype=np.uint32)
                assert L.gpu_fwd4_control_reta(int(g["reta_off"]), rg.ctypes.data, len(rg)) == 0
                re = t.reta[int(e["reta_off"]):int(e["reta_off"]) + int(e["reta_size"])]
                assert np.array_equal(rg, re), (s, rg, re)
    # routes
    n = L.gpu_fwd4_control_routes4(None, 0)
    got = np.zeros(n, dtype=abi.ROUTE_DT)
    L.gpu_fwd4_control_routes4(got.ctypes.data, n)
    want = t.route_array()
    key = lambda a: sorted(zip(a["vrf_id"].tolist(), a["ip"].tolist(), a["prefixlen"].tolist(), a["nh"].tolist()))
    assert key(got) == key(want)
    n = L.gpu_fwd4_control_routes6(None, 0)
    got = np.zeros(n, dtype=abi.ROUTE6_DT)
    L.gpu_fwd4_control_routes6(got.ctypes.data, n)
    want = t.route6_array()

    def key6(a):  # the scope iface only keys link-local prefixes (ip6.h:23-36)
        ll = (a["ip"][:, 0] == 0xFE) & ((a["ip"][:, 1] & 0xC0) == 0x80)
        return sorted(zip(a["vrf_id"].tolist(), [bytes(x) for x in a["ip"]], a["prefixlen"].tolist(),
                          np.where(ll, a["iface_id"], 0).tolist(), a["nh"].tolist()))
    assert key6(got) == key6(want)


@pytest.fixture
def control():
    """A fresh mirror and control plane (CPU: no module initialised)."""
    L = lib()
    if L.gh_hip_ctx():
        pytest.skip("a GPU module is initialised in this process: the GPU tests cover it")
    L.gr_test_internal_events(1)
    ok(L.gc_begin())
    yield L
    L.gr_test_internal_events(1)
    ok(L.gc_end())


def test_mirror_follows_grout_sequences(control):
    L = control
    build_base()
    w = Want()
    want_base(w)
    check_shadow(w)
    ev = np.zeros(2, dtype=np.uint64)
    L.gc_events(ev.ctypes.data)
    # the address nexthops (4 NEW), the connected routes' nexthops, the /32 of
    # the learned neighbour: INTERNAL objects, only on the patch's channel
    assert ev[1] >= 4 + 1, ev
    assert stats()["internal"] == ev[1]


def test_mirror_publishes_route_changes_in_batches(control):
    """Route events reach every context's RIB at once and are published in
    batches (gpu_fwd4_control.c, "publication"): when the control loop's turn
    ends, or every 4096 changes. A full view FRR installs in one burst then
    costs a few hundred commits, not one per route. grout's wait for the
    datapath before it frees a nexthop (nexthop_destroy's synchronize, after
    the pre-delete event the patch pushes) publishes first, so a route deleted
    with its nexthop is off every GPU before the synchronize starts."""
    L = control
    build_base()
    st0 = stats()
    assert st0["pending"] == 0
    # one turn: 10,000 /24s via nexthop 100 (4096 + 4096 published on the way, the rest at the turn's end)
    ok(L.gc_route4_add_many(VRF, be("20.0.0.0"), 24, 10_000, 100, ORIGIN_STATIC))
    st1 = stats()
    assert st1["commits"] - st0["commits"] == 3 and st1["pending"] == 0, (st0, st1)
    assert st1["routes4"] - st0["routes4"] == 10_000
    # a single route: published at its turn's end
    ok(L.gc_route4_add(VRF, be("21.0.0.0"), 8, 0, 101, ORIGIN_STATIC, 0))
    st2 = stats()
    assert st2["commits"] - st1["commits"] == 1 and st2["pending"] == 0
    # nexthop 100 deleted through the API: its 10,000 routes go (route events,
    # held), then nexthop_destroy's pre-delete publishes them before its
    # synchronize; nothing is left for the turn's end
    ok(L.gc_nh_del(100, 0))
    st3 = stats()
    assert st3["presync"] - st2["presync"] >= 1, (st2, st3)
    assert st3["pending"] == 0 and st3["routes4"] == st2["routes4"] - 10_000  # the group keeps its route


def test_mirror_vrf_resize_publishes_nexthops_first(control):
    """A VRF's FIBs resized (iface_reconfig with GR_VRF_SET_FIB, vrf.c:315-357:
    grout migrates its routes, the mirror refills new device FIBs and
    publishes them) in the same control-loop turn as a neighbour learned by
    ARP, whose L3 nexthop is still waiting for the next publication: the
    refill publishes the nexthops before the routes that may name them (slots
    are reused: a stale slot could carry a deleted neighbour's MAC). No
    publication is ever made with L3 nexthop changes pending (unordered 0)."""
    L = control
    build_base()
    w = Want()
    want_base(w)
    st0 = stats()
    ok(L.gc_arp_vrf_resize(VRF, PORTS[2], be("172.16.2.9"), mac(HOST3_MAC), 1 << 17, 1 << 17))
    st1 = stats()
    assert st1["errors"] == 0 and st1["unordered"] == 0, st1
    assert st1["commits"] - st0["commits"] >= 2 and st1["pending"] == 0, (st0, st1)  # the refill's v4 + v6
    h = w.l3(L.gc_slot4(VRF, be("172.16.2.9")), 2, "172.16.2.9", HOST3_MAC, abi.NH_S["REACHABLE"], NH_F_NEIGH)
    w.route("172.16.2.9/32", h)
    check_shadow(w)
    # an unchanged size is not a reconfiguration of the FIBs: nothing refilled
    ok(L.gc_arp_vrf_resize(VRF, PORTS[2], be("172.16.2.9"), None, 1 << 17, 0))
    assert stats()["commits"] == st1["commits"]


def test_mirror_timer_follows_the_event_base(control):
    """Route events before the module's init attaches the control thread's
    event base have no publication timer: each change is published at once,
    counted (no_timer). Once a base is attached the timer is made on it and
    the changes of one turn are published together again."""
    L = control
    build_base()
    ok(L.gc_attach(0))
    st0 = stats()
    ok(L.gc_route4_add_many(VRF, be("20.0.0.0"), 24, 10, 100, ORIGIN_STATIC))
    st1 = stats()
    assert st1["no_timer"] - st0["no_timer"] == 10 and st1["commits"] - st0["commits"] == 10, (st0, st1)
    ok(L.gc_attach(1))
    ok(L.gc_route4_add_many(VRF, be("21.0.0.0"), 24, 10, 100, ORIGIN_STATIC))
    st2 = stats()
    assert st2["no_timer"] == st1["no_timer"] and st2["commits"] - st1["commits"] == 1, (st1, st2)
    assert st2["errors"] == 0 and st2["unordered"] == 0


def test_mirror_without_the_patch_misses_internal_objects(control):
    """The negative control: grout as it is emits no event for INTERNAL
    nexthops and routes. The connected routes then name nexthops the mirror
    never saw (it refuses them: -ENOENT), and the learned neighbour's /32 and
    the router's addresses never reach the GPUs."""
    L = control
    L.gr_test_internal_events(0)
    build_base()
    st = stats()
    assert st["errors"] >= 4 and st["first_error"] == -2, st  # the 4 connected routes: -ENOENT
    assert L.gc_slot4(VRF, be("172.16.0.1")) == 0  # the address nexthop: never mirrored
    n = L.gpu_fwd4_control_routes4(None, 0)
    r = np.zeros(n, dtype=abi.ROUTE_DT)
    L.gpu_fwd4_control_routes4(r.ctypes.data, n)
    assert T.ip4("172.16.2.7") not in r["ip"].tolist()  # the learned /32
    assert not (r["prefixlen"] == 24).any()  # the connected routes


def test_mirror_state_changes_and_deletes(control):
    """Changes grout makes without a public event (ARP resolution, ageing,
    a group member removed with its nexthop) and every delete path; at the
    end nothing is left: no slot, no reta entry, no route."""
    L = control
    build_base()
    w = Want()
    sl = want_base(w)
    check_shadow(w)
    # l3_age: the learned neighbour goes STALE
    ok(L.gc_age4(VRF, be("172.16.2.7"), 1201, 0))
    w.t.nh[sl["neigh"]]["state"] = abi.NH_S["STALE"]
    check_shadow(w)
    # a packet held for an unresolved connected host: nh4_resolve_cb creates
    # a LEARN nexthop and its /32, PENDING; then the host answers
    ok(L.gc_resolve4(VRF, be("172.16.3.9")))
    h = L.gc_slot4(VRF, be("172.16.3.9"))
    w.l3(h, 3, "172.16.3.9", None, abi.NH_S["PENDING"], NH_F_NEIGH)
    w.route("172.16.3.9/32", h)
    check_shadow(w)
    ok(L.gc_arp(PORTS[3], be("172.16.3.9"), mac(HOST3_MAC)))
    w.t.nh[h]["state"] = abi.NH_S["REACHABLE"]
    w.t.nh[h]["mac"] = np.frombuffer(T.mac_bytes(HOST3_MAC), np.uint8)
    check_shadow(w)
    # a group member deleted: grout drops it from the group in place
    # (remove_group_member_cb, group_nexthop.c:58-81): one member left
    ok(L.gc_nh_del(101, 0))
    grp = L.gc_slot_id(200)
    w.t.nh[sl["m101"]] = 0
    g = w.t.nh[grp]
    g["n_members"], g["single"] = 1, sl["m100"]
    check_shadow(w)
    # the gateway nexthop deleted through the API: its routes go first
    # (nh_del: nexthop_routes_cleanup, then the references)
    ok(L.gc_nh_del_l3(PORTS[1], be("172.16.1.2"), 0))
    w.drop_nh(sl["gw"])
    check_shadow(w)
    # an address deleted: its nexthop and its connected route
    a0 = L.gc_slot4(VRF, be("172.16.0.1"))
    ok(L.gc_addr4_del(PORTS[0], be("172.16.0.1"), 24))
    w.drop_nh(a0)
    check_shadow(w)
    # an iface destroyed: its learned neighbours (nexthop_iface_cleanup) and
    # its addresses go with it
    a2 = L.gc_slot4(VRF, be("172.16.2.1"))
    ok(L.gc_iface_del(PORTS[2]))
    w.drop_nh(sl["neigh"])
    w.drop_nh(a2)
    w.drop_iface(2)
    check_shadow(w)
    got = np.zeros(1, dtype=abi.IFACE_DT)
    assert L.gpu_fwd4_control_iface(PORTS[2], got.ctypes.data) < 0
    # everything through grout's paths: the mirror ends empty
    ok(L.gc_end())
    st = stats()
    assert st["slots_used"] == 0 and st["reta_used"] == 0 and st["routes4"] == 0 and st["routes6"] == 0, st
    assert st["errors"] == 0, st
    assert L.gc_nh_count() == 0
    ok(L.gc_begin())  # for the fixture's gc_end


# ---------------------------------------------------------------------------
# IPv6: addr6_add, a gateway route resolved by NDP, learned neighbours (a
# global one and a link-local one, scoped to its iface)
# ---------------------------------------------------------------------------
GW6_MAC, N6_MAC, LL_MAC = "02:00:00:06:00:02", "02:00:00:06:00:07", "02:00:00:06:fe:07"


def ip6b(s):
    return ctypes.create_string_buffer(T.ip6(s), 16)


def build_v6():
    L = lib()
    ok(L.gc_addr6_add(PORTS[0], ip6b("2001:db8::1"), 64))
    ok(L.gc_addr6_add(PORTS[1], ip6b("2001:db8:1::1"), 64))
    ok(L.gc_addr6_add(PORTS[1], ip6b("fe80::1"), 64))
    ok(L.gc_route6_add(VRF, ip6b("2001:db8:100::"), 48, ip6b("2001:db8:1::2"), 0, ORIGIN_STATIC, 0))
    ok(L.gc_ndp(PORTS[1], ip6b("2001:db8:1::2"), mac(GW6_MAC)))
    ok(L.gc_ndp(PORTS[1], ip6b("2001:db8:1::7"), mac(N6_MAC)))
    ok(L.gc_ndp(PORTS[1], ip6b("fe80::7"), mac(LL_MAC)))


def want_v6(w):
    L = lib()
    sl = {}
    for p, cidr in ((0, "2001:db8::1/64"), (1, "2001:db8:1::1/64"), (1, "fe80::1/64")):
        net = ipaddress.IPv6Interface(cidr)
        s = L.gc_slot6(VRF, PORTS[p], ip6b(str(net.ip)))
        w.l3(s, p, str(net.ip), T.PORT_MAC[p], abi.NH_S["REACHABLE"], abi.NH_F_LOCAL | abi.NH_F_LINK)
        w.t.add_route6(VRF, str(net.network), s, iface_id=PORTS[p])
        sl[cidr] = s
    g = w.l3(L.gc_slot6(VRF, PORTS[1], ip6b("2001:db8:1::2")), 1, "2001:db8:1::2", GW6_MAC, abi.NH_S["REACHABLE"])
    w.t.add_route6(VRF, "2001:db8:100::/48", g)
    n = w.l3(L.gc_slot6(VRF, PORTS[1], ip6b("2001:db8:1::7")), 1, "2001:db8:1::7", N6_MAC, abi.NH_S["REACHABLE"],
             NH_F_NEIGH)
    w.t.add_route6(VRF, "2001:db8:1::7/128", n)
    ll = w.l3(L.gc_slot6(VRF, PORTS[1], ip6b("fe80::7")), 1, "fe80::7", LL_MAC, abi.NH_S["REACHABLE"], NH_F_NEIGH)
    w.t.add_route6(VRF, "fe80::7/128", ll, iface_id=PORTS[1])
    sl.update(gw6=g, n6=n, ll7=ll)
    return sl


def test_mirror_ipv6_sequences(control):
    L = control
    build_base()
    build_v6()
    w = Want()
    want_base(w)
    sl = want_v6(w)
    check_shadow(w)
    # the link-local neighbour is keyed by its iface: the same address on p0
    # is another nexthop (l3_nexthop.c:68-75), which does not exist
    assert L.gc_slot6(VRF, PORTS[0], ip6b("fe80::7")) == 0
    # an address deleted: its nexthop and its connected route
    ok(L.gc_addr6_del(PORTS[0], ip6b("2001:db8::1"), 64))
    w.t.nh[sl["2001:db8::1/64"]] = 0
    r6 = w.t.route6_array()
    w.t.routes6 = [r6[r6["nh"] != sl["2001:db8::1/64"]]]
    check_shadow(w)


# ---------------------------------------------------------------------------
# GPU: graph walks on the state the mirror loaded
# ---------------------------------------------------------------------------
CASES4 = [  # label, dst range (ingress p0)
    ("gw", "16.0.0.0", "17.255.255.255"),
    ("neigh", "172.16.2.7", "172.16.2.7"),
    ("conn", "172.16.3.9", "172.16.3.9"),
    ("self", "172.16.0.1", "172.16.0.1"),
    ("other_addr", "172.16.1.1", "172.16.1.1"),
    ("group", "18.0.0.0", "18.255.255.255"),
    ("blackhole", "19.0.0.0", "19.255.255.255"),
    ("noroute", "10.0.0.0", "10.255.255.255"),
]
CASES6 = [  # label, prefix (dst under it), ingress port
    ("gw6", "2001:db8:100::/48", 0),
    ("neigh6", "2001:db8:1::7/128", 0),
    ("self6", "2001:db8::1/128", 0),
    ("ll7", "fe80::7/128", 1),
]
PER_CASE = 96


def corpus():
    frs, mes, labs = [], [], []
    for k, (lab, lo, hi) in enumerate(CASES4):
        fr, me = S.stream(PER_CASE, 0xC70 + k, dst_range=(T.ip4(lo), T.ip4(hi)))
        frs.append(fr)
        mes.append(me)
        labs += [lab] * PER_CASE
    for k, (lab, cidr, p) in enumerate(CASES6):
        net = ipaddress.IPv6Network(cidr)
        r = np.zeros(1, dtype=abi.ROUTE6_DT)
        r["ip"] = np.frombuffer(net.network_address.packed, np.uint8)
        r["prefixlen"] = net.prefixlen
        fr, me = S.stream6(PER_CASE, 0xC80 + k, r, in_iface=PORTS[p], dst_mac=T.PORT_MAC[p])
        frs.append(fr)
        mes.append(me)
        labs += [lab] * PER_CASE
    # interleave the cases, as traffic would
    fr, me, labs = np.concatenate(frs), np.concatenate(mes), np.array(labs)
    order = np.random.default_rng(0xC7).permutation(len(me))
    return np.ascontiguousarray(fr[order]), np.ascontiguousarray(me[order]), labs[order].tolist()


def walk_check(w, fr, me, labs):
    stale0 = GW.walk_info()["stale"]
    got = GW.check_walk(w.t, fr, me, labs, loaded=True)
    assert GW.walk_info()["stale"] == stale0  # nothing dropped for a missing object
    labs = np.array(labs)
    return {lab: got[labs == lab] for lab in set(labs.tolist())}


def edges(g):
    return sorted({abi.EDGE_NAMES[e] for e in g["edge"]})


@pytest.fixture
def mirrored():
    """The walk graph with every context wiped, then loaded by the mirror from
    grout's control sequences only; at the end grout's paths remove it all."""
    from golden_util import fresh_fastpath_state
    L = lib()
    fp = GW.graph_ctx()
    fresh_fastpath_state(fp, T.Topology(), GW._gh.setdefault("state", {}))  # nothing from earlier tests
    L.gr_test_internal_events(1)
    ok(L.gc_begin())
    try:
        build_base()
        build_v6()
        yield L
    finally:
        r = L.gc_end()  # -EBUSY if the mirror held anything grout no longer has
        GW._gh["state"]["key"] = None  # the next walk test loads its own topology
        assert r == 0, r


@pytest.mark.gpu
def test_control_plane_walk(mirrored):
    """grout's objects reach every GPU through the mirror alone, and a graph
    walk over them takes grout's edges, bit-exact with the oracle: the
    router's addresses reach ip_input_local with the address nexthop, a
    resolved connected host (ARP-learned, its INTERNAL /32) leaves on
    port_output with its MAC, an unresolved one waits in ip_hold on the
    connected route's nexthop; then every change grout makes without a public
    event (ageing, resolution, a group member dropped) and the delete paths,
    each walked again. Nothing is dropped stale."""
    L = mirrored
    w = Want()
    sl = want_base(w)
    sl.update(want_v6(w))
    check_shadow(w)
    fr, me, labs = corpus()
    g = walk_check(w, fr, me, labs)
    addr = {p: L.gc_slot4(VRF, be(f"172.16.{p}.1")) for p in range(4)}
    assert edges(g["gw"]) == ["port_output"] and (g["gw"]["iface"] == PORTS[1]).all()
    assert edges(g["neigh"]) == ["port_output"] and (g["neigh"]["iface"] == PORTS[2]).all()
    assert edges(g["conn"]) == ["ip_hold"] and (g["conn"]["nh"] == addr[3]).all()
    assert edges(g["self"]) == ["ip_input_local"] and (g["self"]["nh"] == addr[0]).all()
    assert edges(g["other_addr"]) == ["ip_input_local"] and (g["other_addr"]["nh"] == addr[1]).all()
    assert edges(g["group"]) == ["port_output"] and (g["group"]["iface"] == PORTS[3]).all()
    assert edges(g["blackhole"]) == ["ip_blackhole"]
    assert edges(g["noroute"]) == ["ip_error_dest_unreach"]
    assert edges(g["gw6"]) == ["port_output"] and edges(g["neigh6"]) == ["port_output"]
    assert edges(g["self6"]) == ["ip6_input_local"] and (g["self6"]["nh"] == sl["2001:db8::1/64"]).all()
    assert edges(g["ll7"]) == ["port_output"] and (g["ll7"]["iface"] == PORTS[1]).all()
    # the neighbour ages out (l3_age: STALE, no public event): held
    ok(L.gc_age4(VRF, be("172.16.2.7"), 1201, 0))
    w.t.nh[sl["neigh"]]["state"] = abi.NH_S["STALE"]
    g = walk_check(w, fr, me, labs)
    assert edges(g["neigh"]) == ["ip_hold"] and (g["neigh"]["nh"] == sl["neigh"]).all()
    # the held packet for 172.16.3.9 is resolved (nh4_resolve_cb): a LEARN
    # nexthop and its /32, PENDING; then the host answers the ARP request
    ok(L.gc_resolve4(VRF, be("172.16.3.9")))
    h = w.l3(L.gc_slot4(VRF, be("172.16.3.9")), 3, "172.16.3.9", None, abi.NH_S["PENDING"], NH_F_NEIGH)
    w.route("172.16.3.9/32", h)
    g = walk_check(w, fr, me, labs)
    assert edges(g["conn"]) == ["ip_hold"] and (g["conn"]["nh"] == h).all()
    ok(L.gc_arp(PORTS[3], be("172.16.3.9"), mac(HOST3_MAC)))
    w.t.nh[h]["state"] = abi.NH_S["REACHABLE"]
    w.t.nh[h]["mac"] = np.frombuffer(T.mac_bytes(HOST3_MAC), np.uint8)
    g = walk_check(w, fr, me, labs)
    assert edges(g["conn"]) == ["port_output"] and (g["conn"]["iface"] == PORTS[3]).all()
    # a group member deleted: the group forwards on the one left
    ok(L.gc_nh_del(101, 0))
    w.t.nh[sl["m101"]] = 0
    grp = w.t.nh[L.gc_slot_id(200)]
    grp["n_members"], grp["single"] = 1, sl["m100"]
    g = walk_check(w, fr, me, labs)
    assert edges(g["group"]) == ["port_output"]
    # the gateway deleted (its routes first): no route
    ok(L.gc_nh_del_l3(PORTS[1], be("172.16.1.2"), 0))
    w.drop_nh(sl["gw"])
    g = walk_check(w, fr, me, labs)
    assert edges(g["gw"]) == ["ip_error_dest_unreach"]
    # the neighbour's iface destroyed: its nexthops and its address go
    a2 = addr[2]
    ok(L.gc_iface_del(PORTS[2]))
    w.drop_nh(sl["neigh"])
    w.drop_nh(a2)
    w.drop_iface(2)
    check_shadow(w)
    g = walk_check(w, fr, me, labs)
    assert edges(g["neigh"]) == ["ip_error_dest_unreach"]


@pytest.mark.gpu
def test_control_bulk_routes_walk(mirrored):
    """A burst of 60,000 routes in one control-loop turn (FRR installing a
    view; the VRF's FIB holds 65,536) reaches every GPU in 15 publications,
    not 60,000, and forwards bit-exact; deleting their nexthop takes them all
    off before grout's synchronize (the pre-delete publication), and nothing
    is dropped stale."""
    import time
    L = mirrored
    w = Want()
    sl = want_base(w)
    sl.update(want_v6(w))
    n = 60_000
    c0 = stats()["commits"]
    t0 = time.perf_counter()
    ok(L.gc_route4_add_many(VRF, be("20.0.0.0"), 24, n, 100, ORIGIN_STATIC))
    dt = time.perf_counter() - t0
    st = stats()
    assert st["commits"] - c0 == -(-n // 4096) and st["pending"] == 0 and st["errors"] == 0, st
    print(f"{n} routes in one turn: {dt:.3f} s ({n / dt / 1e6:.2f} M routes/s), "
          f"{int(st['commits'] - c0)} publications")
    r = np.zeros(n, dtype=abi.ROUTE_DT)
    r["ip"] = T.ip4("20.0.0.0") + 256 * np.arange(n, dtype=np.uint32)
    r["prefixlen"], r["vrf_id"], r["nh"] = 24, VRF, sl["m100"]
    w.t.add_routes(r)
    fr, me = S.stream(20_000, 0xB17, routes=r, in_iface=PORTS[0], dst_mac=T.PORT_MAC[0])
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    g = walk_check(w, fr, me, ["bulk"] * len(me))["bulk"]
    assert edges(g) == ["port_output"] and (g["iface"] == PORTS[3]).all()
    # an ARP storm: 2,000 neighbours learned in one turn (each a LEARN nexthop,
    # pushed at once, and its INTERNAL /32, published with the turn)
    s0 = stats()
    t0 = time.perf_counter()
    ok(L.gc_arp_many(PORTS[2], be("10.9.0.1"), 2000, mac(NEIGH_MAC)))
    dt = time.perf_counter() - t0
    s1 = stats()
    assert s1["slots_used"] - s0["slots_used"] == 2000 and s1["routes4"] - s0["routes4"] == 2000
    assert s1["commits"] - s0["commits"] == 1 and s1["errors"] == 0, (s0, s1)
    print(f"2000 neighbours in one turn: {dt:.3f} s ({dt / 2000 * 1e6:.0f} us each)")
    # their nexthop deleted through the API: the routes go first, published before the synchronize
    p0 = stats()["presync"]
    ok(L.gc_nh_del(100, 0))
    st = stats()
    assert st["presync"] > p0 and st["pending"] == 0
    w.drop_nh(sl["m100"])
    grp = w.t.nh[L.gc_slot_id(200)]
    grp["n_members"], grp["single"] = 1, sl["m101"]
    g = walk_check(w, fr, me, ["bulk"] * len(me))["bulk"]
    assert edges(g) == ["ip_error_dest_unreach"]


@pytest.mark.gpu
def test_control_vrf_resize_walk(mirrored):
    """The VRF's FIBs resized in the turn a neighbour is learned: the GPUs'
    new FIBs hold every route and the neighbour's nexthop is published with
    them; walks to it and to the base corpus forward bit-exact."""
    L = mirrored
    w = Want()
    sl = want_base(w)
    sl.update(want_v6(w))
    ok(L.gc_arp_vrf_resize(VRF, PORTS[2], be("172.16.2.9"), mac(HOST3_MAC), 1 << 17, 1 << 17))
    assert stats()["unordered"] == 0 and stats()["errors"] == 0
    h = w.l3(L.gc_slot4(VRF, be("172.16.2.9")), 2, "172.16.2.9", HOST3_MAC, abi.NH_S["REACHABLE"], NH_F_NEIGH)
    w.route("172.16.2.9/32", h)
    check_shadow(w)
    fr, me, labs = corpus()
    g = walk_check(w, fr, me, labs)
    assert edges(g["gw"]) == ["port_output"] and edges(g["group"]) == ["port_output"]
    r = np.zeros(1, dtype=abi.ROUTE_DT)
    r["ip"], r["prefixlen"], r["vrf_id"], r["nh"] = T.ip4("172.16.2.9"), 32, VRF, h
    fr, me = S.stream(4096, 0xB19, routes=r, in_iface=PORTS[0], dst_mac=T.PORT_MAC[0])
    fr, me = np.ascontiguousarray(fr), np.ascontiguousarray(me, dtype=abi.META_DT)
    g = walk_check(w, fr, me, ["host"] * len(me))["host"]
    assert edges(g) == ["port_output"] and (g["iface"] == PORTS[2]).all()


@pytest.mark.gpu
def test_control_replay_recovers_diverged_context(mirrored):
    """A context that loses the control plane's state (here its VRF's FIBs
    destroyed behind the mirror's back) fails the next replicated change and
    is marked diverged: its graphs punt to grout's CPU nodes. The mirror's
    replay rebuilds it from what it holds (ifaces, nexthops, reta, the FIBs,
    published) and resyncs it; the graph bound to it forwards bit-exact."""
    from grout_amd.fwd import FastPath
    L = mirrored
    assert L.gh_n_ctx() == 2
    w = Want()
    want_base(w)
    want_v6(w)
    h1 = FastPath.borrow(L.gh_ctx_at(1))
    k = L.gh_graph_create(3, 0)  # a worker graph on the least loaded context: 1
    assert k > 0 and L.gh_graph_gpu() == 1
    try:
        h1.fib_destroy(VRF)
        # grout adds a route: it fails on context 1 only
        ok(L.gc_route4_add(VRF, be("20.0.0.0"), 8, 0, 300, ORIGIN_STATIC, 0))
        w.route("20.0.0.0/8", L.gc_slot_id(300))
        assert stats()["errors"] > 0
        assert L.gpu_fwd4_diverged(0) == 0 and L.gpu_fwd4_diverged(1) == 1
        fr, me, labs = corpus()
        got, _, _, _ = GW.walk(fr, me)
        assert (got["edge"] == abi.EDGE["punt"]).all()  # iface_input_cpu: grout's CPU nodes
        assert L.gpu_fwd4_control_replay(1) == 0
        assert L.gpu_fwd4_diverged(1) == 0
        walk_check(w, fr, me, labs)
    finally:
        L.gpu_fwd4_resync(1)
        assert L.gh_graph_destroy() == 0
        L.gh_graph_use(0)
