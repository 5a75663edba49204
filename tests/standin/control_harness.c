// SPDX-License-Identifier: BSD-3-Clause
//
// control_harness.c -- test harness (not the product): grout's control
// sequences, replayed through the control-plane stand-in (gr_control_min.c)
// into the fast path's mirror (gpu_fwd4_control.c), for
// tests/test_control_mirror.py.
//
// Every call runs on a control thread of its own, as grout's API handlers and
// ARP/NDP callbacks run on its control thread, while the calling thread plays
// the worker: it walks the current graph and reports quiescent until the
// call returns (grout's rte_rcu_qsbr_synchronize in nexthop_destroy,
// iface_destroy and group_import_info waits for the workers). Without a
// module (CPU tests) there is no QSBR variable and the call runs directly.
#include "gpu_fwd4_control.h"
#include "gpu_fwd4_node.h"
#include "gr_control_min.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void gh_walk_idle(void); // walk_harness.c
int gh_inited(void);
void gh_objects_clear(void);
void gh_objects_restore(void);

struct call {
	int (*fn)(void *);
	void *arg;
	int ret;
	int done;
};

// One control call is one turn of grout's control loop: its timers (the
// mirror's publication) fire when it ends.
static int control_turn(int (*fn)(void *), void *arg) {
	const int r = fn(arg);
	gr_test_event_loop_turn();
	return r;
}

static void *control_thread(void *p) {
	struct call *c = p;
	gr_test_lcore_set(RTE_MAX_LCORE - 1); // not a worker's lcore
	c->ret = control_turn(c->fn, c->arg);
	__atomic_store_n(&c->done, 1, __ATOMIC_RELEASE);
	return NULL;
}

static int on_control(int (*fn)(void *), void *arg) {
	if (!gh_inited())
		return control_turn(fn, arg);
	struct call c = {.fn = fn, .arg = arg};
	pthread_t th;
	if (pthread_create(&th, NULL, control_thread, &c) != 0)
		return -EAGAIN;
	while (!__atomic_load_n(&c.done, __ATOMIC_ACQUIRE))
		gh_walk_idle();
	pthread_join(th, NULL);
	return c.ret;
}

#define MAC(p) (*(const struct rte_ether_addr *)(p))

// ---- begin / end -------------------------------------------------------------
// The harness's objects leave the node's registries; the mirror starts empty
// (the fast path contexts are wiped by the test first).
int gc_begin(void) {
	if (gh_inited())
		gh_objects_clear();
	gpu_fwd4_control_reset();
	gr_test_events_reset();
	// without the module (CPU tests) the mirror still gets the control
	// thread's event base, as the module's init passes it
	gpu_fwd4_control_attach(gr_test_event_base());
	return 0;
}

// Tests: the mirror's event base taken away (events before the module's
// init: no timer) or given back.
int gc_attach(int on) {
	gpu_fwd4_control_attach(on ? gr_test_event_base() : NULL);
	return 0;
}

static int do_reset(void *arg) {
	(void)arg;
	gr_test_control_reset();
	return 0;
}

// Every object destroyed through grout's paths (the mirror empties the
// contexts), then the harness's objects back. -EBUSY: the mirror still held
// a slot, a reta entry or a route when grout had nothing left.
int gc_end(void) {
	int r = on_control(do_reset, NULL);
	struct gpu_fwd4_control_stats st;
	gpu_fwd4_control_stats(&st);
	if (r == 0 && (st.slots_used || st.reta_used || st.routes4 || st.routes6))
		r = -EBUSY;
	gpu_fwd4_control_reset();
	if (gh_inited())
		gh_objects_restore();
	return r;
}

// ---- ifaces ------------------------------------------------------------------
struct a_iface {
	struct gr_iface conf;
	union {
		struct gr_iface_info_vrf vrf;
		struct gr_iface_info_port port;
		struct gr_iface_info_vlan vlan;
	} info;
	uint16_t id;
	int up;
	uint8_t mac[6];
};

static int do_iface_add(void *p) {
	struct a_iface *a = p;
	struct iface *i = iface_create(&a->conf, &a->info);
	return i != NULL ? i->id : -errno;
}

int gc_vrf_add(uint16_t id, uint32_t max_routes, uint32_t num_tbl8, uint32_t max_routes6, uint32_t num_tbl8_6) {
	struct a_iface a = {.conf = {.id = id, .type = GR_IFACE_TYPE_VRF, .mode = GR_IFACE_MODE_VRF,
				     .flags = GR_IFACE_F_UP, .mtu = 1500}};
	snprintf(a.conf.name, sizeof(a.conf.name), "vrf%u", id);
	a.info.vrf.ipv4 = (struct gr_iface_info_vrf_fib) {max_routes, num_tbl8};
	a.info.vrf.ipv6 = (struct gr_iface_info_vrf_fib) {max_routes6, num_tbl8_6};
	return on_control(do_iface_add, &a);
}

int gc_port_add(uint16_t id, uint16_t port_id, const uint8_t *mac, uint16_t vrf_id, uint16_t mtu, int up,
		uint16_t flags) {
	struct a_iface a = {.conf = {.id = id, .type = GR_IFACE_TYPE_PORT, .mode = GR_IFACE_MODE_VRF,
				     .flags = (uint16_t)((up ? GR_IFACE_F_UP : 0) | flags), .mtu = mtu,
				     .vrf_id = vrf_id}};
	snprintf(a.conf.name, sizeof(a.conf.name), "p%u", port_id);
	a.info.port.mac = MAC(mac);
	a.info.port.port_id = port_id;
	return on_control(do_iface_add, &a);
}

int gc_vlan_add(uint16_t id, uint16_t parent_id, uint16_t vlan_id, const uint8_t *mac, uint16_t vrf_id, int up) {
	struct a_iface a = {.conf = {.id = id, .type = GR_IFACE_TYPE_VLAN, .mode = GR_IFACE_MODE_VRF,
				     .flags = up ? GR_IFACE_F_UP : 0, .mtu = 1500, .vrf_id = vrf_id}};
	snprintf(a.conf.name, sizeof(a.conf.name), "v%u.%u", parent_id, vlan_id);
	a.info.vlan.parent_id = parent_id;
	a.info.vlan.vlan_id = vlan_id;
	if (mac != NULL)
		a.info.vlan.mac = MAC(mac);
	return on_control(do_iface_add, &a);
}

static int do_iface_up(void *p) {
	struct a_iface *a = p;
	return iface_set_up_down(iface_from_id_rw(a->id), a->up);
}

// One control-loop turn: a neighbour learned by ARP on `iface_id` (its L3
// nexthop waits for the next publication of the mirror), then the VRF's FIBs
// resized (grout migrates its routes; the mirror refills new device FIBs and
// publishes them). max_routes 0: that family unchanged.
struct a_vrf_resize {
	uint16_t vrf_id, iface_id;
	uint32_t ip_be;
	const uint8_t *mac;
	struct gr_iface_info_vrf_fib v4, v6;
};

static int do_arp_vrf_resize(void *p) {
	struct a_vrf_resize *a = p;
	int r = 0;
	if (a->mac != NULL)
		r = arp_probe_input(a->iface_id, a->ip_be, (const struct rte_ether_addr *)a->mac);
	if (r < 0)
		return r;
	return iface_vrf_reconfig_fib(iface_from_id_rw(a->vrf_id), &a->v4, &a->v6);
}

int gc_arp_vrf_resize(uint16_t vrf_id, uint16_t iface_id, uint32_t ip_be, const uint8_t *mac, uint32_t max_routes,
		      uint32_t max_routes6) {
	struct a_vrf_resize a = {.vrf_id = vrf_id, .iface_id = iface_id, .ip_be = ip_be, .mac = mac,
				 .v4 = {max_routes, 0}, .v6 = {max_routes6, 0}};
	return on_control(do_arp_vrf_resize, &a);
}

int gc_iface_up(uint16_t id, int up) {
	struct a_iface a = {.id = id, .up = up};
	return on_control(do_iface_up, &a);
}

static int do_iface_mac(void *p) {
	struct a_iface *a = p;
	return iface_set_eth_addr(iface_from_id_rw(a->id), &MAC(a->mac));
}

int gc_iface_mac(uint16_t id, const uint8_t *mac) {
	struct a_iface a = {.id = id};
	memcpy(a.mac, mac, 6);
	return on_control(do_iface_mac, &a);
}

static int do_iface_del(void *p) {
	struct a_iface *a = p;
	return iface_destroy(iface_from_id_rw(a->id));
}

int gc_iface_del(uint16_t id) {
	struct a_iface a = {.id = id};
	return on_control(do_iface_del, &a);
}

// ---- addresses, routes, neighbours ------------------------------------------
struct a_l3 {
	uint16_t vrf_id, iface_id;
	uint8_t ip[16], gw[16];
	uint8_t prefixlen;
	uint32_t nh_id;
	gr_nh_origin_t origin;
	int flag;
	uint8_t mac[6];
	uint32_t age, probes;
};

static ip4_addr_t v4(const uint8_t *b) {
	ip4_addr_t x;
	memcpy(&x, b, 4);
	return x;
}

static int do_addr4_add(void *p) {
	struct a_l3 *a = p;
	return addr4_add(a->iface_id, v4(a->ip), a->prefixlen, GR_NH_ORIGIN_LINK); // the API's origin (address.c:135)
}
static int do_addr4_del(void *p) {
	struct a_l3 *a = p;
	return addr4_delete(a->iface_id, v4(a->ip), a->prefixlen);
}
static int do_addr6_add(void *p) {
	struct a_l3 *a = p;
	return addr6_add(a->iface_id, a->ip, a->prefixlen, GR_NH_ORIGIN_LINK);
}
static int do_addr6_del(void *p) {
	struct a_l3 *a = p;
	return addr6_delete(a->iface_id, a->ip, a->prefixlen);
}
static int do_route4_add(void *p) {
	struct a_l3 *a = p;
	return route4_add(a->vrf_id, v4(a->ip), a->prefixlen, v4(a->gw), a->nh_id, a->origin, a->flag);
}
static int do_route4_del(void *p) {
	struct a_l3 *a = p;
	return route4_del(a->vrf_id, v4(a->ip), a->prefixlen, a->flag);
}
static int do_route6_add(void *p) {
	struct a_l3 *a = p;
	return route6_add(a->vrf_id, a->ip, a->prefixlen, a->gw, a->nh_id, a->origin, a->flag);
}
static int do_route6_del(void *p) {
	struct a_l3 *a = p;
	return route6_del(a->vrf_id, a->ip, a->prefixlen, a->flag);
}
static int do_arp(void *p) {
	struct a_l3 *a = p;
	return arp_probe_input(a->iface_id, v4(a->ip), &MAC(a->mac));
}
static int do_ndp(void *p) {
	struct a_l3 *a = p;
	return ndp_probe_input(a->iface_id, a->ip, &MAC(a->mac));
}
// a packet to ip held by ip_output on the nexthop its route gave (nh4_resolve_cb)
static int do_resolve4(void *p) {
	struct a_l3 *a = p;
	struct nexthop *nh = rib4_lookup(a->vrf_id, v4(a->ip));
	if (nh == NULL)
		return -errno;
	return nh4_resolve(nh, v4(a->ip)) != NULL ? 0 : -errno;
}
static int do_age4(void *p) {
	struct a_l3 *a = p;
	struct nexthop *nh = nh4_lookup(a->vrf_id, v4(a->ip));
	if (nh == NULL)
		return -errno;
	nexthop_l3_age(nh, a->age, a->probes);
	return 0;
}

#define IP4(a, x) memcpy((a).ip, &(x), 4)

int gc_addr4_add(uint16_t iface_id, uint32_t ip_be, uint8_t prefixlen) {
	struct a_l3 a = {.iface_id = iface_id, .prefixlen = prefixlen};
	IP4(a, ip_be);
	return on_control(do_addr4_add, &a);
}
int gc_addr4_del(uint16_t iface_id, uint32_t ip_be, uint8_t prefixlen) {
	struct a_l3 a = {.iface_id = iface_id, .prefixlen = prefixlen};
	IP4(a, ip_be);
	return on_control(do_addr4_del, &a);
}
int gc_addr6_add(uint16_t iface_id, const uint8_t *ip, uint8_t prefixlen) {
	struct a_l3 a = {.iface_id = iface_id, .prefixlen = prefixlen};
	memcpy(a.ip, ip, 16);
	return on_control(do_addr6_add, &a);
}
int gc_addr6_del(uint16_t iface_id, const uint8_t *ip, uint8_t prefixlen) {
	struct a_l3 a = {.iface_id = iface_id, .prefixlen = prefixlen};
	memcpy(a.ip, ip, 16);
	return on_control(do_addr6_del, &a);
}
int gc_route4_add(uint16_t vrf_id, uint32_t ip_be, uint8_t prefixlen, uint32_t gw_be, uint32_t nh_id, uint8_t origin,
		  int exist_ok) {
	struct a_l3 a = {.vrf_id = vrf_id, .prefixlen = prefixlen, .nh_id = nh_id, .origin = origin, .flag = exist_ok};
	IP4(a, ip_be);
	memcpy(a.gw, &gw_be, 4);
	return on_control(do_route4_add, &a);
}
// count routes of /prefixlen from ip (host order steps) via nexthop nh_id, in
// one control turn, as FRR's bulk installs reach grout
struct a_many {
	uint16_t vrf_id;
	uint32_t ip_host;
	uint8_t prefixlen;
	uint32_t count, nh_id;
	uint8_t origin;
};
static int do_route4_add_many(void *p) {
	const struct a_many *a = p;
	const uint32_t step = a->prefixlen ? 1u << (32 - a->prefixlen) : 0;
	for (uint32_t k = 0; k < a->count; k++) {
		const uint32_t ip = __builtin_bswap32(a->ip_host + k * step);
		const int r = route4_add(a->vrf_id, ip, a->prefixlen, 0, a->nh_id, a->origin, 0);
		if (r < 0)
			return r;
	}
	return 0;
}
int gc_route4_add_many(uint16_t vrf_id, uint32_t ip_be, uint8_t prefixlen, uint32_t count, uint32_t nh_id,
		       uint8_t origin) {
	struct a_many a = {.vrf_id = vrf_id, .ip_host = __builtin_bswap32(ip_be), .prefixlen = prefixlen,
			   .count = count, .nh_id = nh_id, .origin = origin};
	return on_control(do_route4_add_many, &a);
}

int gc_route4_del(uint16_t vrf_id, uint32_t ip_be, uint8_t prefixlen, int missing_ok) {
	struct a_l3 a = {.vrf_id = vrf_id, .prefixlen = prefixlen, .flag = missing_ok};
	IP4(a, ip_be);
	return on_control(do_route4_del, &a);
}
int gc_route6_add(uint16_t vrf_id, const uint8_t *ip, uint8_t prefixlen, const uint8_t *gw, uint32_t nh_id,
		  uint8_t origin, int exist_ok) {
	struct a_l3 a = {.vrf_id = vrf_id, .prefixlen = prefixlen, .nh_id = nh_id, .origin = origin, .flag = exist_ok};
	memcpy(a.ip, ip, 16);
	if (gw != NULL)
		memcpy(a.gw, gw, 16);
	return on_control(do_route6_add, &a);
}
int gc_route6_del(uint16_t vrf_id, const uint8_t *ip, uint8_t prefixlen, int missing_ok) {
	struct a_l3 a = {.vrf_id = vrf_id, .prefixlen = prefixlen, .flag = missing_ok};
	memcpy(a.ip, ip, 16);
	return on_control(do_route6_del, &a);
}
int gc_arp(uint16_t iface_id, uint32_t sip_be, const uint8_t *mac) {
	struct a_l3 a = {.iface_id = iface_id};
	IP4(a, sip_be);
	memcpy(a.mac, mac, 6);
	return on_control(do_arp, &a);
}
// count neighbours from sip (host-order steps) learned in one control turn,
// as an ARP storm reaches grout
struct a_arps {
	uint16_t iface_id;
	uint32_t ip_host, count;
	uint8_t mac[6];
};
static int do_arp_many(void *p) {
	const struct a_arps *a = p;
	for (uint32_t k = 0; k < a->count; k++) {
		const int r = arp_probe_input(a->iface_id, __builtin_bswap32(a->ip_host + k), &MAC(a->mac));
		if (r < 0)
			return r;
	}
	return 0;
}
int gc_arp_many(uint16_t iface_id, uint32_t sip_be, uint32_t count, const uint8_t *mac) {
	struct a_arps a = {.iface_id = iface_id, .ip_host = __builtin_bswap32(sip_be), .count = count};
	memcpy(a.mac, mac, 6);
	return on_control(do_arp_many, &a);
}

int gc_ndp(uint16_t iface_id, const uint8_t *ip, const uint8_t *mac) {
	struct a_l3 a = {.iface_id = iface_id};
	memcpy(a.ip, ip, 16);
	memcpy(a.mac, mac, 6);
	return on_control(do_ndp, &a);
}
int gc_resolve4(uint16_t vrf_id, uint32_t dst_be) {
	struct a_l3 a = {.vrf_id = vrf_id};
	IP4(a, dst_be);
	return on_control(do_resolve4, &a);
}
int gc_age4(uint16_t vrf_id, uint32_t ip_be, uint32_t reply_age_s, uint32_t probes) {
	struct a_l3 a = {.vrf_id = vrf_id, .age = reply_age_s, .probes = probes};
	IP4(a, ip_be);
	return on_control(do_age4, &a);
}

// ---- nexthops through the API (modules/infra/api/nexthop.c) ------------------
struct a_nh {
	struct gr_nexthop_base base;
	struct gr_nexthop_info_l3 l3;
	struct gr_nexthop_info_group *group;
	int flag;
};

static int do_nh_add(void *p) {
	struct a_nh *a = p;
	return nh_add(&a->base, a->base.type == GR_NH_T_GROUP ? (const void *)a->group : &a->l3, a->flag);
}
static int do_nh_del(void *p) {
	struct a_nh *a = p;
	return nh_del(&a->base, NULL, a->flag);
}

int gc_nh_add_l3(uint32_t nh_id, uint16_t iface_id, uint32_t ip_be, const uint8_t *mac, uint8_t origin, int exist_ok) {
	struct a_nh a = {.base = {.type = GR_NH_T_L3, .origin = origin, .iface_id = iface_id, .nh_id = nh_id},
			 .l3 = {.af = ip_be ? GR_AF_IP4 : GR_AF_UNSPEC, .ipv4 = ip_be}, .flag = exist_ok};
	if (mac != NULL)
		a.l3.mac = MAC(mac);
	return on_control(do_nh_add, &a);
}

// blackhole / reject nexthops (no info), in a VRF
int gc_nh_add_type(uint32_t nh_id, uint8_t type, uint16_t vrf_id, uint8_t origin) {
	struct a_nh a = {.base = {.type = type, .origin = origin, .vrf_id = vrf_id, .nh_id = nh_id}};
	return on_control(do_nh_add, &a);
}

int gc_nh_add_group(uint32_t nh_id, uint32_t n, const uint32_t *ids, const uint32_t *weights, uint8_t origin,
		    int exist_ok) {
	struct gr_nexthop_info_group *g = calloc(1, sizeof(*g) + n * sizeof(g->members[0]));
	if (g == NULL)
		return -ENOMEM;
	g->n_members = n;
	for (uint32_t i = 0; i < n; i++) {
		g->members[i].nh_id = ids[i];
		g->members[i].weight = weights != NULL ? weights[i] : 1;
	}
	struct a_nh a = {.base = {.type = GR_NH_T_GROUP, .origin = origin, .nh_id = nh_id}, .group = g,
			 .flag = exist_ok};
	int r = on_control(do_nh_add, &a);
	free(g);
	return r;
}

static int do_nh_del_l3(void *p) {
	struct a_nh *a = p;
	return nh_del(&a->base, &a->l3, a->flag);
}

// an L3 nexthop deleted through the API by its address (auto ids)
int gc_nh_del_l3(uint16_t iface_id, uint32_t ip_be, int missing_ok) {
	struct a_nh a = {.base = {.type = GR_NH_T_L3, .iface_id = iface_id}, .l3 = {.af = GR_AF_IP4, .ipv4 = ip_be},
			 .flag = missing_ok};
	return on_control(do_nh_del_l3, &a);
}

int gc_nh_del(uint32_t nh_id, int missing_ok) {
	struct a_nh a = {.base = {.nh_id = nh_id}, .flag = missing_ok};
	return on_control(do_nh_del, &a);
}

// ---- what the tests read back --------------------------------------------------
// The slot the mirror gave the nexthop grout knows by address / by id / as the
// route (vrf, ip, prefixlen) names it; 0 = none.
uint32_t gc_slot4(uint16_t vrf_id, uint32_t ip_be) {
	return gpu_fwd4_control_nh_slot(nh4_lookup(vrf_id, ip_be));
}
uint32_t gc_slot6(uint16_t vrf_id, uint16_t iface_id, const uint8_t *ip) {
	return gpu_fwd4_control_nh_slot(nh6_lookup(vrf_id, iface_id, ip));
}
uint32_t gc_slot_id(uint32_t nh_id) {
	return gpu_fwd4_control_nh_slot(nexthop_lookup_id(nh_id));
}
uint32_t gc_slot_route4(uint16_t vrf_id, uint32_t ip_be, uint8_t prefixlen) {
	return gpu_fwd4_control_nh_slot(rib4_lookup_exact(vrf_id, ip_be, prefixlen));
}
// nexthops in use in grout's pool
uint32_t gc_nh_count(void) {
	uint32_t n = 0, cap;
	const struct nexthop *p = gr_test_nh_base(&cap);
	for (uint32_t k = 0; k < cap; k++)
		n += p[k].ref_count != 0;
	return n;
}
void gc_events(uint64_t out[2]) {
	gr_test_events_count(&out[0], &out[1]);
}
