// SPDX-License-Identifier: BSD-3-Clause
//
// gr_control_min.c -- the control-plane stand-in behind gr_control_min.h: a
// restatement of how grout creates, changes and destroys the ifaces,
// nexthops, routes and addresses the fast path mirrors, and which events it
// pushes while doing so (test infrastructure; in grout these are grout's own
// files). Each function cites the grout code it restates. With
// integration/grout-gpu_fwd4-control.patch applied, every place where grout
// changes an object without an event pushes an internal one instead
// (event_push_internal); the stand-in does the same at the same places,
// marked "patch:".
#include "gr_control_min.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int errno_set(int e) {
	errno = e;
	return -e;
}

static void *errno_set_null(int e) {
	errno = e;
	return NULL;
}

static bool ether_is_zero(const struct rte_ether_addr *a) {
	static const uint8_t z[6];
	return memcmp(a->addr_bytes, z, 6) == 0;
}

static bool ip6_is_unspec(const uint8_t a[16]) {
	static const uint8_t z[16];
	return memcmp(a, z, 16) == 0;
}

static bool ip6_is_linklocal(const uint8_t a[16]) { // fe80::/10
	return a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
}

// addr6_linklocal_scope (modules/ip6/control/ip6.h:23-36)
static const uint8_t *ll_scope(const uint8_t ip[16], uint8_t tmp[16], uint16_t iface_id) {
	if (!ip6_is_linklocal(ip))
		return ip;
	memcpy(tmp, ip, 16);
	tmp[2] = (uint8_t)(iface_id >> 8);
	tmp[3] = (uint8_t)iface_id;
	return tmp;
}

static void rcu_sync(void) {
	if (gr_datapath_rcu() != NULL)
		rte_rcu_qsbr_synchronize(gr_datapath_rcu(), RTE_QSBR_THRID_INVALID);
}

// ---- libevent timers ---------------------------------------------------------
struct event {
	struct event_base *base;
	void (*cb)(int, short, void *);
	void *arg;
	int pending;
	struct event *next;
};
static struct event *timers;

struct event *event_new(struct event_base *base, evutil_socket_t fd, short what, event_callback_fn cb, void *arg) {
	(void)fd;
	(void)what;
	struct event *e = calloc(1, sizeof(*e));
	if (e == NULL)
		return NULL;
	e->base = base;
	e->cb = cb;
	e->arg = arg;
	e->next = timers;
	timers = e;
	return e;
}

int event_add(struct event *ev, const struct timeval *tv) {
	(void)tv;
	if (ev->base == NULL)
		return -1; // libevent: no event_base set
	ev->pending = 1;
	return 0;
}

int event_del(struct event *ev) {
	ev->pending = 0;
	return 0;
}

void event_free(struct event *ev) {
	for (struct event **p = &timers; *p != NULL; p = &(*p)->next)
		if (*p == ev) {
			*p = ev->next;
			break;
		}
	free(ev);
}

struct event_base *gr_test_event_base(void) {
	static char base; // opaque: only its address is used
	return (struct event_base *)&base;
}

void gr_test_event_loop_turn(void) {
	for (int round = 0; round < 16; round++) { // a callback may add a timer again
		int fired = 0;
		for (struct event *e = timers; e != NULL; e = e->next)
			if (e->pending) {
				e->pending = 0;
				e->cb(-1, 0x01 /* EV_TIMEOUT */, e->arg);
				fired = 1;
				break; // the list may have changed
			}
		if (!fired)
			return;
	}
}

// ---- events (main/event.c:25-67) -------------------------------------------
#define MAX_SUBS 128
static struct {
	uint32_t ev;
	event_sub_cb_t cb;
} subs[MAX_SUBS], isubs[MAX_SUBS];
static unsigned n_subs, n_isubs;
static uint64_t n_pub, n_int;

static void subscribe(unsigned *n, uint32_t ev, event_sub_cb_t cb, int internal) {
	if (*n == MAX_SUBS || cb == NULL)
		abort(); // grout: ABORT / assert
	if (internal) {
		isubs[*n].ev = ev;
		isubs[(*n)++].cb = cb;
	} else {
		subs[*n].ev = ev;
		subs[(*n)++].cb = cb;
	}
}

void event_subscribe(uint32_t ev_type, event_sub_cb_t callback) {
	subscribe(&n_subs, ev_type, callback, 0);
}

void event_subscribe_internal(uint32_t ev_type, event_sub_cb_t callback) {
	subscribe(&n_isubs, ev_type, callback, 1);
}

// From the control thread, subscribers are notified at once (event.c:54-67).
void event_push(uint32_t ev_type, const void *obj) {
	n_pub++;
	for (unsigned i = 0; i < n_subs; i++)
		if (subs[i].ev == ev_type)
			subs[i].cb(ev_type, obj);
}

static int internal_on = 1;

void gr_test_internal_events(int on) {
	internal_on = on;
}

void event_push_internal(uint32_t ev_type, const void *obj) {
	if (!internal_on) // grout without integration/grout-gpu_fwd4-control.patch
		return;
	n_int++;
	for (unsigned i = 0; i < n_isubs; i++)
		if (isubs[i].ev == ev_type)
			isubs[i].cb(ev_type, obj);
}

void gr_test_events_reset(void) {
	n_pub = n_int = 0;
}

void gr_test_events_count(uint64_t *pub, uint64_t *internal) {
	if (pub != NULL)
		*pub = n_pub;
	if (internal != NULL)
		*internal = n_int;
}

// ---- ifaces (modules/infra/control/iface.c, vrf.c, port.c, vlan.c) ---------
static struct iface ifs[GR_MAX_IFACES];
static bool if_used[GR_MAX_IFACES];
static const uint32_t max_routes_default = 1u << 16; // route.c:32, gr_config

static uint32_t fib4_auto_tbl8(uint32_t max_routes) { // route.c:38-41
	const uint32_t n = max_routes / 500;
	return n < 256 ? 256 : n;
}

struct iface *gr_test_iface_base(void) {
	return ifs;
}

struct iface *iface_from_id_rw(uint16_t id) {
	return id < GR_MAX_IFACES && if_used[id] ? &ifs[id] : NULL;
}

static struct iface *get_vrf_iface(uint16_t vrf_id) {
	struct iface *v = iface_from_id_rw(vrf_id);
	return v != NULL && v->type == GR_IFACE_TYPE_VRF ? v : NULL;
}

int iface_get_eth_addr(const struct iface *iface, struct rte_ether_addr *mac) { // iface.c:475-487
	if (iface == NULL)
		return errno_set(EINVAL);
	switch (iface->type) {
	case GR_IFACE_TYPE_VRF: // vrf.c:366-370
		*mac = iface_info_vrf(iface)->mac;
		return 0;
	case GR_IFACE_TYPE_PORT: // port.c:659-663
		*mac = iface_info_port(iface)->mac;
		return 0;
	case GR_IFACE_TYPE_VLAN: // vlan.c:174-178
		*mac = iface_info_vlan(iface)->mac;
		return 0;
	default:
		return errno_set(EOPNOTSUPP);
	}
}

// iface_create (iface.c:171-267) with the type inits of vrf.c:230-255 (the
// FIB sizes, defaults filled by fib4_init, route.c:100-122), port.c and
// vlan.c (an unset MAC is the parent's, vlan.c:180-192). The default VRF is
// created on demand, as vrf_incref does.
struct iface *iface_create(const struct gr_iface *conf, const void *api_info) {
	if (conf == NULL || conf->type == GR_IFACE_TYPE_UNDEF || conf->type > GR_IFACE_TYPE_VXLAN)
		return errno_set_null(EINVAL);
	uint16_t id = conf->id;
	if (id == 0)
		for (id = 1; id < GR_MAX_IFACES && if_used[id]; id++)
			;
	if (id == 0 || id >= GR_MAX_IFACES)
		return errno_set_null(ENOSPC);
	if (if_used[id])
		return errno_set_null(EEXIST);
	uint16_t vrf_id = conf->vrf_id;
	struct iface *vrf = NULL;
	if (conf->type == GR_IFACE_TYPE_VRF) {
		vrf_id = id;
	} else if (conf->mode == GR_IFACE_MODE_VRF) {
		if (vrf_id == GR_VRF_ID_UNDEF)
			vrf_id = GR_VRF_DEFAULT_ID;
		if ((vrf = get_vrf_iface(vrf_id)) == NULL) {
			if (vrf_id != GR_VRF_DEFAULT_ID || if_used[vrf_id])
				return errno_set_null(ENONET);
			struct gr_iface vc = {.id = vrf_id, .type = GR_IFACE_TYPE_VRF, .mode = GR_IFACE_MODE_VRF,
					      .flags = GR_IFACE_F_UP, .mtu = 1500};
			snprintf(vc.name, sizeof(vc.name), "main");
			if ((vrf = iface_create(&vc, NULL)) == NULL)
				return NULL;
		}
	}
	struct iface *i = &ifs[id];
	memset(i, 0, sizeof(*i));
	i->base = conf->base;
	i->id = id;
	i->vrf_id = vrf_id;
	if (i->mtu == 0)
		i->mtu = 1500; // iface.c:618-619
	if (i->flags & GR_IFACE_F_UP)
		i->state |= GR_IFACE_S_RUNNING;
	switch (conf->type) {
	case GR_IFACE_TYPE_VRF: {
		struct iface_info_vrf *v = iface_info_vrf(i);
		const struct gr_iface_info_vrf *a = api_info;
		if (a != NULL) {
			v->ipv4 = a->ipv4;
			v->ipv6 = a->ipv6;
			v->mac = a->mac;
		}
		if (v->ipv4.max_routes == 0)
			v->ipv4.max_routes = max_routes_default;
		if (v->ipv4.num_tbl8 == 0)
			v->ipv4.num_tbl8 = fib4_auto_tbl8(v->ipv4.max_routes);
		if (v->ipv6.max_routes == 0)
			v->ipv6.max_routes = max_routes_default;
		break;
	}
	case GR_IFACE_TYPE_PORT: {
		const struct gr_iface_info_port *a = api_info;
		if (a == NULL)
			return errno_set_null(EINVAL);
		iface_info_port(i)->mac = a->mac;
		iface_info_port(i)->port_id = a->port_id;
		break;
	}
	case GR_IFACE_TYPE_VLAN: {
		const struct gr_iface_info_vlan *a = api_info;
		const struct iface *parent = a != NULL ? iface_from_id_rw(a->parent_id) : NULL;
		if (parent == NULL)
			return errno_set_null(ENODEV);
		struct iface_info_vlan *v = iface_info_vlan(i);
		v->parent_id = a->parent_id;
		v->vlan_id = a->vlan_id;
		v->mac = a->mac;
		if (ether_is_zero(&v->mac) && iface_get_eth_addr(parent, &v->mac) < 0)
			return NULL;
		break;
	}
	default:
		break;
	}
	if (vrf != NULL)
		iface_info_vrf(vrf)->ref_count++;
	i->name = strdup(conf->name);
	if_used[id] = true;
	gr_iface_register(i); // ifaces[ifid] = iface (iface.c:262)
	event_push(GR_EVENT_IFACE_ADD, i);
	event_push(GR_EVENT_IFACE_POST_ADD, i);
	return i;
}

// iface_set_up_down, the generic path (iface.c:632-654)
// iface_reconfig (iface.c:325-420) of a VRF's FIB sizes (GR_VRF_SET_FIB,
// vrf.c:315-357): per address family a non-zero max_routes replaces the size
// (and resets num_tbl8 unless one is given too), a non-zero num_tbl8 replaces
// that; an unchanged family is skipped; fib4_reconfig / fib6_reconfig fill
// the defaults (route.c:740-748) and migrate the routes (the stand-in's RIB is
// a list: nothing to move). Then GR_EVENT_IFACE_POST_RECONFIG (iface.c:420).
int iface_vrf_reconfig_fib(struct iface *iface, const struct gr_iface_info_vrf_fib *v4,
			   const struct gr_iface_info_vrf_fib *v6) {
	if (iface == NULL || iface->type != GR_IFACE_TYPE_VRF)
		return errno_set(EINVAL);
	struct iface_info_vrf *vrf = iface_info_vrf(iface);
	const struct gr_iface_info_vrf_fib *api[2] = {v4, v6};
	struct gr_iface_info_vrf_fib *conf[2] = {&vrf->ipv4, &vrf->ipv6};
	for (int af = 0; af < 2; af++) {
		if (api[af] == NULL || (api[af]->max_routes == 0 && api[af]->num_tbl8 == 0))
			continue;
		const struct gr_iface_info_vrf_fib old = *conf[af];
		if (api[af]->max_routes) {
			conf[af]->max_routes = api[af]->max_routes;
			if (!api[af]->num_tbl8)
				conf[af]->num_tbl8 = 0;
		}
		if (api[af]->num_tbl8)
			conf[af]->num_tbl8 = api[af]->num_tbl8;
		if (conf[af]->max_routes == old.max_routes && conf[af]->num_tbl8 == old.num_tbl8)
			continue;
		if (!conf[af]->max_routes)
			conf[af]->max_routes = max_routes_default;
		if (af == 0 && !conf[af]->num_tbl8)
			conf[af]->num_tbl8 = fib4_auto_tbl8(conf[af]->max_routes);
	}
	event_push(GR_EVENT_IFACE_POST_RECONFIG, iface);
	return 0;
}

int iface_set_up_down(struct iface *iface, bool up) {
	if (iface == NULL)
		return errno_set(EINVAL);
	if (!(iface->flags & GR_IFACE_F_UP) && up) {
		iface->flags |= GR_IFACE_F_UP;
		iface->state |= GR_IFACE_S_RUNNING;
		event_push(GR_EVENT_IFACE_STATUS_UP, iface);
	} else if ((iface->flags & GR_IFACE_F_UP) && !up) {
		iface->flags &= (uint16_t)~GR_IFACE_F_UP;
		iface->state &= (uint16_t)~GR_IFACE_S_RUNNING;
		event_push(GR_EVENT_IFACE_STATUS_DOWN, iface);
	}
	return 0;
}

// iface_set_eth_addr (iface.c:506-523) with the type setters (port.c,
// vlan.c:180-200: zero means the parent's, vrf.c:372-376)
int iface_set_eth_addr(struct iface *iface, const struct rte_ether_addr *mac) {
	if (iface == NULL || mac == NULL)
		return errno_set(EINVAL);
	switch (iface->type) {
	case GR_IFACE_TYPE_VRF:
		iface_info_vrf(iface)->mac = *mac;
		break;
	case GR_IFACE_TYPE_PORT:
		iface_info_port(iface)->mac = *mac;
		break;
	case GR_IFACE_TYPE_VLAN: {
		struct rte_ether_addr next = *mac;
		if (ether_is_zero(&next)
		    && iface_get_eth_addr(iface_from_id_rw(iface_info_vlan(iface)->parent_id), &next) < 0)
			return -errno;
		iface_info_vlan(iface)->mac = next;
		break;
	}
	default:
		return errno_set(EOPNOTSUPP);
	}
	event_push(GR_EVENT_IFACE_MAC_CHANGE, iface);
	return 0;
}

static bool has_subinterfaces(uint16_t id) {
	for (uint16_t k = 1; k < GR_MAX_IFACES; k++)
		if (if_used[k] && ifs[k].type == GR_IFACE_TYPE_VLAN && iface_info_vlan(&ifs[k])->parent_id == id)
			return true;
	return false;
}

// iface_destroy (iface.c:690-725): PRE_REMOVE (grout's own subscribers drop
// the iface's nexthops and addresses, nexthop.c:475-491, address.c:257-279),
// STATUS_DOWN if it was up, out of ifaces[], synchronize, REMOVE, freed.
int iface_destroy(struct iface *iface) {
	if (iface == NULL || !if_used[iface->id] || iface != &ifs[iface->id])
		return errno_set(EINVAL);
	if (has_subinterfaces(iface->id))
		return errno_set(EBUSY);
	if (iface->type == GR_IFACE_TYPE_VRF && iface_info_vrf(iface)->ref_count != 0)
		return errno_set(EBUSY);
	event_push(GR_EVENT_IFACE_PRE_REMOVE, iface);
	if (iface->flags & GR_IFACE_F_UP) {
		iface->flags &= (uint16_t)~GR_IFACE_F_UP;
		event_push(GR_EVENT_IFACE_STATUS_DOWN, iface);
	}
	gr_iface_unregister(iface->id);
	rcu_sync();
	event_push(GR_EVENT_IFACE_REMOVE, iface);
	if (iface->type != GR_IFACE_TYPE_VRF && iface->mode == GR_IFACE_MODE_VRF) {
		struct iface *vrf = get_vrf_iface(iface->vrf_id);
		if (vrf != NULL && iface_info_vrf(vrf)->ref_count > 0)
			iface_info_vrf(vrf)->ref_count--;
	}
	free(iface->name);
	if_used[iface->id] = false;
	memset(iface, 0, sizeof(*iface));
	return 0;
}

// ---- nexthops (modules/infra/control/nexthop.c, l3_nexthop.c,
// group_nexthop.c) -----------------------------------------------------------
#define NH_POOL 8192 // gr_config.max_nexthops here
static struct nexthop nh_pool[NH_POOL];
static bool nh_busy[NH_POOL]; // taken from the pool
static bool nh_hashed[NH_POOL]; // in l3_hash (l3_import_info / l3_remove_references)
static uint8_t nh_ids[NH_POOL + 1]; // id_pool: ids 1..NH_POOL

struct nexthop *gr_test_nh_base(uint32_t *count) {
	if (count != NULL)
		*count = NH_POOL;
	return nh_pool;
}

static uint32_t pool_index(const struct nexthop *nh) {
	return (uint32_t)(nh - nh_pool);
}

void nexthop_iter(nh_iter_cb_t cb, void *priv) { // nexthop.c:426-444: ref_count != 0
	for (uint32_t k = 0; k < NH_POOL; k++)
		if (nh_busy[k] && nh_pool[k].ref_count != 0)
			cb(&nh_pool[k], priv);
}

struct nexthop *nexthop_lookup_id(uint32_t nh_id) { // nexthop.c:466-473
	if (nh_id == 0)
		return errno_set_null(ENOENT);
	for (uint32_t k = 0; k < NH_POOL; k++)
		if (nh_busy[k] && nh_pool[k].nh_id == nh_id)
			return &nh_pool[k];
	return errno_set_null(ENOENT);
}

// nexthop_id_put / nexthop_id_get (nexthop.c:91-132)
static void nexthop_id_put(struct nexthop *nh) {
	if (nh->nh_id == 0)
		return;
	if (nh->nh_id <= NH_POOL)
		nh_ids[nh->nh_id] = 0;
	nh->nh_id = 0;
}

static int nexthop_id_get(struct nexthop *nh) {
	if (nh->origin == GR_NH_ORIGIN_INTERNAL || nh->origin == GR_NH_ORIGIN_LEARN) {
		nh->nh_id = 0;
		return 0;
	}
	if (nh->nh_id == 0 && nh->origin == GR_NH_ORIGIN_LINK)
		return 0;
	if (nh->nh_id == 0) {
		for (uint32_t id = 1; id <= NH_POOL; id++)
			if (!nh_ids[id]) {
				nh_ids[id] = 1;
				nh->nh_id = id;
				return 0;
			}
		return errno_set(ENOSPC);
	}
	if (nh->nh_id <= NH_POOL) {
		if (nh_ids[nh->nh_id])
			return errno_set(EBUSY);
		nh_ids[nh->nh_id] = 1;
	}
	return 0;
}

// set_nexthop_key + the hash compare (l3_nexthop.c:51-87): af, vrf and the
// address, a link-local IPv6 address scoped to its iface
static bool l3_key_eq(const struct nexthop *nh, addr_family_t af, uint16_t vrf_id, uint16_t iface_id,
		      const void *addr) {
	const struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
	if (l3->af != af || nh->vrf_id != vrf_id)
		return false;
	if (af == GR_AF_IP4)
		return l3->ipv4 == *(const ip4_addr_t *)addr;
	uint8_t a[16], b[16];
	return memcmp(ll_scope(l3->ipv6, a, nh->iface_id), ll_scope(addr, b, iface_id), 16) == 0;
}

struct nexthop *nexthop_lookup_l3(addr_family_t af, uint16_t vrf_id, uint16_t iface_id, const void *addr) {
	if (af == GR_AF_UNSPEC) // l3_nexthop.c:89-101
		return NULL;
	for (uint32_t k = 0; k < NH_POOL; k++)
		if (nh_hashed[k] && l3_key_eq(&nh_pool[k], af, vrf_id, iface_id, addr))
			return &nh_pool[k];
	return errno_set_null(ENOENT);
}

struct nexthop *nexthop_lookup(const struct gr_nexthop_base *base, const void *info) { // nexthop.c:297-315
	struct nexthop *nh = NULL;
	if (base == NULL)
		return errno_set_null(EINVAL);
	if (base->nh_id != GR_NH_ID_UNSET)
		nh = nexthop_lookup_id(base->nh_id);
	if (nh == NULL && base->type == GR_NH_T_L3 && info != NULL) { // l3_lookup, l3_nexthop.c:103-113
		const struct gr_nexthop_info_l3 *l3 = info;
		const struct iface *iface = iface_from_id_rw(base->iface_id);
		nh = nexthop_lookup_l3(l3->af, iface != NULL ? iface->vrf_id : base->vrf_id, base->iface_id,
				       l3->af == GR_AF_IP4 ? (const void *)&l3->ipv4 : l3->ipv6);
	}
	return nh != NULL ? nh : errno_set_null(ENOENT);
}

// l3_import_info (l3_nexthop.c:216-282)
static int l3_import_info(struct nexthop *nh, const struct gr_nexthop_info_l3 *pub) {
	struct nexthop_info_l3 priv = *nexthop_info_l3(nh);
	priv.flags = pub->flags;
	switch (pub->af) {
	case GR_AF_IP4:
		if (pub->ipv4 == 0)
			return errno_set(EDESTADDRREQ);
		break;
	case GR_AF_IP6:
		if (ip6_is_unspec(pub->ipv6))
			return errno_set(EDESTADDRREQ);
		break;
	case GR_AF_UNSPEC:
		if (pub->ipv4 || !ip6_is_unspec(pub->ipv6))
			return errno_set(EINVAL);
		priv.flags |= GR_NH_F_LINK;
		break;
	default:
		return errno_set(ENOPROTOOPT);
	}
	if (!ether_is_zero(&pub->mac)) {
		if (pub->af == GR_AF_UNSPEC)
			return errno_set(EINVAL);
		priv.mac = pub->mac;
		priv.state = GR_NH_S_REACHABLE;
	}
	const bool has_new = pub->af != GR_AF_UNSPEC;
	if (has_new) {
		const struct nexthop *ex = nexthop_lookup_l3(pub->af, nh->vrf_id, nh->iface_id,
							     pub->af == GR_AF_IP4 ? (const void *)&pub->ipv4 : pub->ipv6);
		if (ex != NULL && ex != nh)
			return errno_set(EADDRINUSE);
	}
	memcpy(priv.ipv6, pub->ipv6, 16); // ipv6 encompasses ipv4
	priv.af = pub->af;
	priv.prefixlen = pub->prefixlen;
	nh_hashed[pool_index(nh)] = has_new;
	*nexthop_info_l3(nh) = priv;
	return 0;
}

static void nexthop_destroy(struct nexthop *nh);

void nexthop_incref(struct nexthop *nh) {
	nh->ref_count++;
}

void nexthop_decref(struct nexthop *nh) { // nexthop.c:521-526
	if (nh->ref_count == 0)
		abort();
	if (--nh->ref_count == 0)
		nexthop_destroy(nh);
}

// group_reta_distribute (group_nexthop.c:27-56)
static void group_reta_distribute(uint16_t n_members, uint16_t reta_size, struct nh_group_member *members,
				  struct nexthop **reta) {
	uint32_t total = 0;
	for (uint16_t i = 0; i < n_members; i++)
		total += members[i].weight;
	uint32_t idx = 0;
	for (uint16_t i = 0; i < n_members && idx < reta_size; i++) {
		uint32_t entries = (members[i].weight * reta_size + total / 2) / total;
		if (entries == 0 && members[i].weight > 0)
			entries = 1;
		for (uint32_t j = 0; j < entries && idx < reta_size; j++)
			reta[idx++] = members[i].nh;
	}
	while (idx < reta_size && n_members > 0)
		reta[idx++] = members[0].nh;
}

static int by_weight_desc(const void *a, const void *b) {
	return (int)((const struct nh_group_member *)b)->weight - (int)((const struct nh_group_member *)a)->weight;
}

static uint32_t align32pow2(uint32_t x) {
	uint32_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

// group_import_info (group_nexthop.c:101-186)
static int group_import_info(struct nexthop *nh, const struct gr_nexthop_info_group *group) {
	struct nexthop_info_group *pvt = nexthop_info_group(nh);
	struct nh_group_member *members = NULL, *tmp;
	struct nexthop **reta = NULL, **old_reta, *one = NULL;
	uint32_t reta_size = 0, n_tmp;
	if (group->n_members > 0 && (members = calloc(group->n_members, sizeof(*members))) == NULL)
		return errno_set(ENOMEM);
	for (uint32_t i = 0; i < group->n_members; i++) {
		struct nexthop *m = nexthop_lookup_id(group->members[i].nh_id);
		if (m == NULL) {
			free(members);
			return errno_set(ENOENT);
		}
		members[i].nh = m;
		members[i].weight = group->members[i].weight ? group->members[i].weight : 1;
	}
	if (group->n_members == 1) {
		one = members[0].nh;
		nexthop_incref(one);
	} else if (group->n_members > 1) {
		qsort(members, group->n_members, sizeof(members[0]), by_weight_desc);
		const uint32_t max_w = members[0].weight, min_w = members[group->n_members - 1].weight;
		reta_size = (max_w / min_w) * group->n_members;
		if (reta_size > MAX_NH_GROUP_RETA_SIZE)
			reta_size = MAX_NH_GROUP_RETA_SIZE;
		reta_size = align32pow2(reta_size);
		if ((reta = calloc(reta_size, sizeof(*reta))) == NULL) {
			free(members);
			return errno_set(ENOMEM);
		}
		for (uint32_t i = 0; i < group->n_members; i++)
			nexthop_incref(members[i].nh);
		group_reta_distribute((uint16_t)group->n_members, (uint16_t)reta_size, members, reta);
	}
	n_tmp = pvt->n_members;
	tmp = pvt->members;
	old_reta = pvt->reta;
	pvt->n_members = (uint16_t)group->n_members;
	pvt->members = members;
	pvt->nh = one;
	pvt->reta_size = (uint16_t)reta_size;
	pvt->reta = reta;
	rcu_sync();
	for (uint32_t i = 0; i < n_tmp; i++)
		nexthop_decref(tmp[i].nh);
	free(old_reta);
	free(tmp);
	return 0;
}

// remove_group_member_cb (group_nexthop.c:58-81)
static void remove_group_member_cb(struct nexthop *nh, void *deleted) {
	if (nh->type != GR_NH_T_GROUP)
		return;
	bool removed = false;
	struct nexthop_info_group *g = nexthop_info_group(nh);
	for (uint32_t i = 0; i < g->n_members; i++) {
		if (g->members[i].nh == deleted) {
			g->members[i].nh = g->members[g->n_members - 1].nh;
			g->members[i].weight = g->members[g->n_members - 1].weight;
			g->n_members--;
			removed = true;
		}
	}
	if (removed) {
		if (g->n_members == 1) {
			g->nh = g->members[0].nh;
		} else if (g->n_members > 1) {
			g->nh = NULL;
			group_reta_distribute(g->n_members, g->reta_size, g->members, g->reta);
		}
		event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch: no event in grout
	}
}

// nexthop_update (nexthop.c:347-395)
int nexthop_update(struct nexthop *nh, const struct gr_nexthop_base *base, const void *info) {
	struct gr_nexthop_base backup = nh->base;
	int ret;
	if (base->type < GR_NH_T_L3 || base->type > GR_NH_T_GROUP)
		return errno_set(ESOCKTNOSUPPORT);
	nexthop_id_put(nh);
	nh->base = *base;
	if ((ret = nexthop_id_get(nh)) < 0)
		return ret;
	if (nh->type == GR_NH_T_GROUP) {
		nh->vrf_id = GR_VRF_ID_UNDEF;
	} else if (nh->iface_id != GR_IFACE_ID_UNDEF) {
		const struct iface *iface = iface_from_id_rw(nh->iface_id);
		if (iface == NULL) {
			ret = errno_set(ENODEV);
			goto err;
		}
		nh->vrf_id = iface->vrf_id;
	} else if (nh->vrf_id != GR_VRF_ID_UNDEF && get_vrf_iface(nh->vrf_id) == NULL) {
		ret = errno_set(ENONET);
		goto err;
	}
	if (nh->type == GR_NH_T_L3 && (ret = l3_import_info(nh, info)) < 0)
		goto err;
	if (nh->type == GR_NH_T_GROUP && (ret = group_import_info(nh, info)) < 0)
		goto err;
	if (nh->ref_count > 0) {
		if (nh->origin != GR_NH_ORIGIN_INTERNAL)
			event_push(GR_EVENT_NEXTHOP_UPDATE, nh);
		else
			event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
	}
	return 0;
err:
	if (nh->ref_count == 0)
		nexthop_id_put(nh);
	nh->base = backup;
	return ret;
}

// nexthop_new (nexthop.c:317-345)
struct nexthop *nexthop_new(const struct gr_nexthop_base *base, const void *info) {
	if (base == NULL)
		return errno_set_null(EINVAL);
	uint32_t k = 0;
	while (k < NH_POOL && nh_busy[k])
		k++;
	if (k == NH_POOL)
		return errno_set_null(ENOBUFS); // rte_mempool_get
	struct nexthop *nh = &nh_pool[k];
	memset(nh, 0, sizeof(*nh));
	nh_busy[k] = true;
	int ret = nexthop_update(nh, base, info);
	if (ret < 0) {
		nh_busy[k] = false;
		nh_hashed[k] = false;
		return errno_set_null(-ret);
	}
	nexthop_incref(nh);
	if (nh->origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_NEXTHOP_NEW, nh);
	else
		event_push_internal(GR_EVENT_NEXTHOP_NEW, nh); // patch
	return nh;
}

// nexthop_destroy (nexthop.c:493-519): remove_references of every type
// (l3: out of the hash, group: out of every group), the id back, synchronize,
// DELETE, the type's free (group: members released), back to the pool.
static void nexthop_destroy(struct nexthop *nh) {
	nh_hashed[pool_index(nh)] = false;
	nexthop_iter(remove_group_member_cb, nh);
	nexthop_id_put(nh);
	event_push_internal(GR_EVENT_NEXTHOP_PRE_DELETE, nh); // patch
	rcu_sync();
	if (nh->origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_NEXTHOP_DELETE, nh);
	else
		event_push_internal(GR_EVENT_NEXTHOP_DELETE, nh); // patch
	if (nh->type == GR_NH_T_GROUP) { // group_free (group_nexthop.c:88-95)
		struct nexthop_info_group *g = nexthop_info_group(nh);
		for (uint32_t i = 0; i < g->n_members; i++) // the single member's too: members[0] == nh
			nexthop_decref(g->members[i].nh);
		free(g->members);
		free(g->reta);
	}
	nh_busy[pool_index(nh)] = false;
	memset(nh, 0, sizeof(*nh));
}

// nexthop_routes_cleanup (l3_nexthop.c:145-152): every address family
void nexthop_routes_cleanup(struct nexthop *nh) {
	rib4_cleanup(nh);
	rib6_cleanup(nh);
}

// l3_age (l3_nexthop.c:322-362), one nexthop: REACHABLE -> STALE after
// lifetime_reachable_sec (DEFAULT_LIFETIME_REACHABLE, 1200 s,
// modules/infra/control/nexthop.c:23), PENDING / STALE -> FAILED
// after max ucast + bcast probes (3 + 3).
void nexthop_l3_age(struct nexthop *nh, uint32_t reply_age_s, uint32_t probes) {
	struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
	switch (l3->state) {
	case GR_NH_S_PENDING:
	case GR_NH_S_STALE:
		if (probes >= 6) {
			l3->state = GR_NH_S_FAILED;
			event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
		}
		break;
	case GR_NH_S_REACHABLE:
		if (reply_age_s > 1200) {
			l3->state = GR_NH_S_STALE;
			event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
		}
		break;
	default:
		break;
	}
}

// nh_add / nh_del (modules/infra/api/nexthop.c:29-78)
int nh_add(const struct gr_nexthop_base *base, const void *info, bool exist_ok) {
	if (base->type != GR_NH_T_GROUP && base->vrf_id == GR_VRF_ID_UNDEF && base->iface_id == GR_IFACE_ID_UNDEF)
		return errno_set(EINVAL);
	struct nexthop *nh = nexthop_lookup(base, info);
	if (nh == NULL)
		return nexthop_new(base, info) == NULL ? -errno : 0;
	if (!exist_ok)
		return errno_set(EEXIST);
	return nexthop_update(nh, base, info);
}

int nh_del(const struct gr_nexthop_base *base, const void *info, bool missing_ok) {
	struct nexthop *nh = nexthop_lookup(base, info);
	if (nh == NULL)
		return missing_ok ? 0 : errno_set(ENOENT);
	if (nh->type == GR_NH_T_L3) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
		if ((l3->flags & NH_LOCAL_ADDR_FLAGS) == NH_LOCAL_ADDR_FLAGS || nh->origin == GR_NH_ORIGIN_LINK)
			return errno_set(EBUSY);
	}
	nexthop_routes_cleanup(nh);
	while (nh->ref_count > 0)
		nexthop_decref(nh);
	return 0;
}

// nexthop_iface_cleanup (nexthop.c:475-491), on GR_EVENT_IFACE_PRE_REMOVE
static void nh_cleanup_interface_cb(struct nexthop *nh, void *priv) {
	if (nh->iface_id != (uintptr_t)priv)
		return;
	if (nh->type == GR_NH_T_L3
	    && (nexthop_info_l3(nh)->flags & NH_LOCAL_ADDR_FLAGS) == NH_LOCAL_ADDR_FLAGS)
		return; // addresses are cleaned per address family
	nexthop_routes_cleanup(nh);
	while (nh->ref_count)
		nexthop_decref(nh);
}

static void nexthop_iface_cleanup(uint32_t ev, const void *obj) {
	(void)ev;
	nexthop_iter(nh_cleanup_interface_cb, (void *)(uintptr_t)((const struct iface *)obj)->id);
}

// ---- RIBs: rte_rib's exact-match store (the FIB is the fast path's) --------
struct rib_entry {
	uint16_t vrf_id;
	uint8_t af;
	uint8_t prefixlen;
	uint8_t ip[16]; // IPv4: host order in the first 4 bytes; IPv6 scoped; masked
	gr_nh_origin_t origin;
	struct nexthop *nh;
};
static struct rib_entry *rib;
static uint32_t rib_n, rib_cap;

static void mask16(uint8_t a[16], uint8_t plen) {
	for (int b = 0; b < 16; b++) {
		const int keep = (int)plen - 8 * b;
		a[b] &= keep >= 8 ? 0xff : keep <= 0 ? 0 : (uint8_t)(0xff << (8 - keep));
	}
}

static void rib_key4(uint8_t k[16], ip4_addr_t ip, uint8_t plen) {
	memset(k, 0, 16);
	const uint32_t h = __builtin_bswap32(ip);
	memcpy(k, &h, 4);
	const uint32_t m = plen ? h & (0xffffffffu << (32 - plen)) : 0;
	memcpy(k, &m, 4);
}

static struct rib_entry *rib_exact(uint16_t vrf_id, uint8_t af, const uint8_t k[16], uint8_t plen) {
	for (uint32_t i = 0; i < rib_n; i++)
		if (rib[i].vrf_id == vrf_id && rib[i].af == af && rib[i].prefixlen == plen && memcmp(rib[i].ip, k, 16) == 0)
			return &rib[i];
	return NULL;
}

static bool in_prefix4(const struct rib_entry *e, uint32_t host_ip) {
	uint32_t p;
	memcpy(&p, e->ip, 4);
	return e->prefixlen == 0 || ((host_ip ^ p) >> (32 - e->prefixlen)) == 0;
}

static bool in_prefix6(const struct rib_entry *e, const uint8_t a[16]) {
	uint8_t m[16];
	memcpy(m, a, 16);
	mask16(m, e->prefixlen);
	return memcmp(m, e->ip, 16) == 0;
}

static struct rib_entry *rib_add(void) {
	if (rib_n == rib_cap) {
		uint32_t cap = rib_cap ? rib_cap * 2 : 256;
		struct rib_entry *r = realloc(rib, cap * sizeof(*r));
		if (r == NULL)
			return NULL;
		rib = r;
		rib_cap = cap;
	}
	return &rib[rib_n++];
}

static void rib_remove(struct rib_entry *e) {
	*e = rib[--rib_n];
}

// ---- IPv4 (modules/ip/control/route.c) -------------------------------------
// rib4_insert_or_replace (route.c:212-275)
static int rib4_insert_or_replace(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, gr_nh_origin_t origin,
				  struct nexthop *nh, bool replace) {
	uint8_t k[16];
	if (get_vrf_iface(vrf_id) == NULL)
		return errno_set(ENONET);
	if (prefixlen > 32)
		return errno_set(EINVAL);
	rib_key4(k, ip, prefixlen);
	struct rib_entry *e = rib_exact(vrf_id, GR_AF_IP4, k, prefixlen);
	struct nexthop *existing = e != NULL ? e->nh : NULL;
	if (existing != NULL && !replace) {
		const bool equal = existing->vrf_id == nh->vrf_id && existing->iface_id == nh->iface_id
			&& existing->type == nh->type;
		return errno_set(equal ? EEXIST : EBUSY);
	}
	if (e == NULL && (e = rib_add()) == NULL)
		return errno_set(ENOMEM);
	*e = (struct rib_entry) {.vrf_id = vrf_id, .af = GR_AF_IP4, .prefixlen = prefixlen, .origin = origin, .nh = nh};
	memcpy(e->ip, k, 16);
	const struct route4_event ev = {.dest = {ip, prefixlen}, .vrf_id = vrf_id, .origin = origin, .nh = nh};
	if (origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_IP_ROUTE_ADD, &ev);
	else
		event_push_internal(GR_EVENT_IP_ROUTE_ADD, &ev); // patch
	nexthop_incref(nh);
	if (existing != NULL)
		nexthop_decref(existing);
	return 0;
}

int rib4_insert(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, gr_nh_origin_t origin, struct nexthop *nh) {
	return rib4_insert_or_replace(vrf_id, ip, prefixlen, origin, nh, false);
}

// rib4_delete (route.c:287-333)
int rib4_delete(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, gr_nh_type_t nh_type) {
	uint8_t k[16];
	if (get_vrf_iface(vrf_id) == NULL)
		return errno_set(ENONET);
	rib_key4(k, ip, prefixlen);
	struct rib_entry *e = rib_exact(vrf_id, GR_AF_IP4, k, prefixlen);
	if (e == NULL)
		return errno_set(ENOENT);
	struct nexthop *nh = e->nh;
	const gr_nh_origin_t origin = e->origin;
	if (nh->type != nh_type)
		return errno_set(EINVAL);
	rib_remove(e);
	const struct route4_event ev = {.dest = {ip, prefixlen}, .vrf_id = vrf_id, .origin = origin, .nh = nh};
	if (origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_IP_ROUTE_DEL, &ev);
	else
		event_push_internal(GR_EVENT_IP_ROUTE_DEL, &ev); // patch
	nexthop_decref(nh);
	return 0;
}

struct nexthop *rib4_lookup(uint16_t vrf_id, ip4_addr_t ip) { // route.c:169-185
	const uint32_t h = __builtin_bswap32(ip);
	struct rib_entry *best = NULL;
	for (uint32_t i = 0; i < rib_n; i++)
		if (rib[i].vrf_id == vrf_id && rib[i].af == GR_AF_IP4 && in_prefix4(&rib[i], h)
		    && (best == NULL || rib[i].prefixlen > best->prefixlen))
			best = &rib[i];
	return best != NULL ? best->nh : errno_set_null(ENETUNREACH);
}

struct nexthop *rib4_lookup_exact(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen) {
	uint8_t k[16];
	rib_key4(k, ip, prefixlen);
	struct rib_entry *e = rib_exact(vrf_id, GR_AF_IP4, k, prefixlen);
	return e != NULL ? e->nh : errno_set_null(ENETUNREACH);
}

// rib4_cleanup (route.c:531-579): collect, then delete each
static void rib_cleanup(struct nexthop *nh, uint8_t af) {
	uint32_t n = 0;
	struct rib_entry *todo = malloc((rib_n ? rib_n : 1) * sizeof(*todo));
	if (todo == NULL)
		return;
	for (uint32_t i = 0; i < rib_n; i++)
		if (rib[i].af == af && (nh == NULL || rib[i].nh == nh))
			todo[n++] = rib[i];
	for (uint32_t i = 0; i < n; i++) {
		if (af == GR_AF_IP4) {
			uint32_t h;
			memcpy(&h, todo[i].ip, 4);
			rib4_delete(todo[i].vrf_id, __builtin_bswap32(h), todo[i].prefixlen, todo[i].nh->type);
		} else {
			// a scoped link-local prefix: its scope is the iface in bytes 2-3
			uint8_t ip[16];
			memcpy(ip, todo[i].ip, 16);
			uint16_t scope = 0;
			if (ip6_is_linklocal(ip)) {
				scope = (uint16_t)(ip[2] << 8 | ip[3]);
				ip[2] = ip[3] = 0;
			}
			rib6_delete(todo[i].vrf_id, scope, ip, todo[i].prefixlen, todo[i].nh->type);
		}
	}
	free(todo);
}

void rib4_cleanup(struct nexthop *nh) {
	rib_cleanup(nh, GR_AF_IP4);
}

// route4_add / route4_del (route.c:336-399)
int route4_add(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, ip4_addr_t gw, uint32_t nh_id,
	       gr_nh_origin_t origin, bool exist_ok) {
	bool created = false;
	struct nexthop *nh;
	if (origin == GR_NH_ORIGIN_INTERNAL)
		return errno_set(EINVAL);
	if (nh_id != GR_NH_ID_UNSET) {
		if ((nh = nexthop_lookup_id(nh_id)) == NULL)
			return errno_set(ENOENT);
	} else {
		nh = nexthop_lookup_l3(GR_AF_IP4, vrf_id, GR_IFACE_ID_UNDEF, &gw);
		if (nh == NULL && (nh = rib4_lookup(vrf_id, gw)) == NULL)
			return errno_set(EHOSTUNREACH);
		if (nh->type != GR_NH_T_L3 || nexthop_info_l3(nh)->ipv4 != gw) {
			const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .iface_id = nh->iface_id,
							     .vrf_id = vrf_id, .origin = origin};
			const struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP4, .ipv4 = gw};
			if ((nh = nexthop_new(&base, &l3)) == NULL)
				return -errno;
			created = true;
		}
	}
	int ret = rib4_insert_or_replace(vrf_id, ip, prefixlen, origin, nh, exist_ok);
	if (ret < 0 && created)
		nexthop_decref(nh);
	return ret;
}

int route4_del(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, bool missing_ok) {
	struct nexthop *nh = rib4_lookup(vrf_id, ip);
	int ret = rib4_delete(vrf_id, ip, prefixlen, nh != NULL ? nh->type : GR_NH_T_L3);
	if ((ret == -ENOENT || ret == -ENONET) && missing_ok)
		ret = 0;
	return ret;
}

// ---- addresses (modules/ip/control/address.c, ip6/control/address.c) --------
#define MAX_ADDRS 16
static struct nexthop *addrs4[GR_MAX_IFACES][MAX_ADDRS];
static uint32_t n_addrs4[GR_MAX_IFACES];
static struct nexthop *addrs6[GR_MAX_IFACES][MAX_ADDRS];
static uint32_t n_addrs6[GR_MAX_IFACES];

// addr4_add (address.c:60-132)
int addr4_add(uint16_t iface_id, ip4_addr_t ip, uint16_t prefixlen, gr_nh_origin_t origin) {
	const struct iface *iface = iface_from_id_rw(iface_id);
	struct nexthop *nh;
	if (iface == NULL)
		return errno_set(ENODEV);
	if (iface->mode != GR_IFACE_MODE_VRF)
		return errno_set(EMEDIUMTYPE);
	for (uint32_t i = 0; i < n_addrs4[iface_id]; i++) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs4[iface_id][i]);
		if (ip == l3->ipv4 && prefixlen == l3->prefixlen)
			return errno_set(EEXIST);
	}
	if (nh4_lookup(iface->vrf_id, ip) != NULL)
		return errno_set(EADDRINUSE);
	if (n_addrs4[iface_id] == MAX_ADDRS)
		return errno_set(ENOSPC);
	const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .origin = GR_NH_ORIGIN_INTERNAL,
					     .iface_id = iface->id, .vrf_id = iface->vrf_id};
	struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP4, .ipv4 = ip, .prefixlen = (uint8_t)prefixlen,
					.flags = NH_LOCAL_ADDR_FLAGS, .state = GR_NH_S_REACHABLE};
	if (iface_get_eth_addr(iface, &l3.mac) < 0 && errno != EOPNOTSUPP)
		return -errno;
	if ((nh = nexthop_new(&base, &l3)) == NULL)
		return -errno;
	int ret = rib4_insert(iface->vrf_id, ip, (uint8_t)prefixlen, origin, nh);
	if (ret < 0) {
		nexthop_decref(nh);
		return ret;
	}
	addrs4[iface_id][n_addrs4[iface_id]++] = nh;
	const struct gr_ip4_ifaddr a = {.ip = ip, .prefixlen = (uint8_t)prefixlen, .iface_id = iface_id};
	event_push(GR_EVENT_IP_ADDR_ADD, &a);
	return 0;
}

// addr4_delete (address.c:145-190)
int addr4_delete(uint16_t iface_id, ip4_addr_t ip, uint16_t prefixlen) {
	if (iface_id >= GR_MAX_IFACES)
		return errno_set(ENODEV);
	uint32_t i = 0;
	struct nexthop *nh = NULL;
	for (; i < n_addrs4[iface_id]; i++) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs4[iface_id][i]);
		if (l3->ipv4 == ip && l3->prefixlen == prefixlen) {
			nh = addrs4[iface_id][i];
			break;
		}
	}
	if (nh == NULL)
		return errno_set(ENOENT);
	const struct gr_ip4_ifaddr a = {.ip = ip, .prefixlen = (uint8_t)prefixlen, .iface_id = iface_id};
	event_push(GR_EVENT_IP_ADDR_DEL, &a);
	nexthop_routes_cleanup(nh);
	while (nh->ref_count > 0)
		nexthop_decref(nh);
	memmove(&addrs4[iface_id][i], &addrs4[iface_id][i + 1], (n_addrs4[iface_id] - i - 1) * sizeof(nh));
	n_addrs4[iface_id]--;
	return 0;
}

// address.c:257-279 / ip6 address.c: an iface going away drops its addresses
static void addr_iface_cleanup(uint32_t ev, const void *obj) {
	(void)ev;
	const struct iface *iface = obj;
	while (n_addrs4[iface->id] > 0) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs4[iface->id][n_addrs4[iface->id] - 1]);
		addr4_delete(iface->id, l3->ipv4, l3->prefixlen);
	}
	while (n_addrs6[iface->id] > 0) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs6[iface->id][n_addrs6[iface->id] - 1]);
		uint8_t ip[16];
		memcpy(ip, l3->ipv6, 16);
		addr6_delete(iface->id, ip, l3->prefixlen);
	}
}

// ---- ARP (modules/ip/control/nexthop.c) -------------------------------------
// arp_probe_input_cb (nexthop.c:127-185), without the reply and the held
// packets' resubmission (datapath work)
int arp_probe_input(uint16_t iface_id, ip4_addr_t sip, const struct rte_ether_addr *sha) {
	const struct iface *iface = iface_from_id_rw(iface_id);
	if (iface == NULL)
		return errno_set(ENODEV);
	struct nexthop *nh = nh4_lookup(iface->vrf_id, sip);
	if (nh == NULL) {
		const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .origin = GR_NH_ORIGIN_LEARN,
						     .iface_id = iface->id, .vrf_id = iface->vrf_id};
		const struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP4, .ipv4 = sip, .mac = *sha,
						      .flags = GR_NH_F_NEIGH};
		if ((nh = nexthop_new(&base, &l3)) == NULL)
			return -errno;
		// an internal /32 route to reference the new nexthop (:169)
		if (rib4_insert(iface->vrf_id, sip, 32, GR_NH_ORIGIN_INTERNAL, nh) < 0)
			return -errno;
	} else {
		struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
		l3->state = GR_NH_S_REACHABLE;
		l3->ucast_probes = 0;
		l3->bcast_probes = 0;
		l3->mac = *sha;
		if (nh->origin != GR_NH_ORIGIN_INTERNAL)
			event_push(GR_EVENT_NEXTHOP_UPDATE, nh);
		else
			event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
	}
	return 0;
}

// nh4_resolve_cb (nexthop.c:33-125) for a held IPv4 packet to dst
struct nexthop *nh4_resolve(struct nexthop *nh, ip4_addr_t dst) {
	struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
	if ((l3->flags & GR_NH_F_LINK) && dst != l3->ipv4) {
		struct nexthop *remote = nh4_lookup(nh->vrf_id, dst);
		if (remote == NULL) {
			const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .origin = GR_NH_ORIGIN_LEARN,
							     .vrf_id = nh->vrf_id, .iface_id = nh->iface_id};
			const struct gr_nexthop_info_l3 info = {.af = GR_AF_IP4, .ipv4 = dst, .flags = GR_NH_F_NEIGH};
			if ((remote = nexthop_new(&base, &info)) == NULL)
				return NULL;
			if (rib4_insert(nh->vrf_id, dst, 32, GR_NH_ORIGIN_INTERNAL, remote) < 0) {
				nexthop_decref(remote);
				return NULL;
			}
		}
		nh = remote;
		l3 = nexthop_info_l3(remote);
	}
	if (l3->state != GR_NH_S_REACHABLE && l3->state != GR_NH_S_PENDING) {
		l3->state = GR_NH_S_PENDING; // after arp_output_request_solicit
		event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
	}
	return nh;
}

// ---- IPv6 (modules/ip6/control/route.c, address.c, nexthop.c) --------------
// rib6_insert_or_replace (route.c:229-297): the key is the scoped address
static int rib6_insert_or_replace(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen,
				  gr_nh_origin_t origin, struct nexthop *nh, bool replace) {
	uint8_t tmp[16], k[16];
	if (get_vrf_iface(vrf_id) == NULL)
		return errno_set(ENONET);
	if (prefixlen > 128)
		return errno_set(EINVAL);
	memcpy(k, ll_scope(ip, tmp, iface_id), 16);
	mask16(k, prefixlen);
	struct rib_entry *e = rib_exact(vrf_id, GR_AF_IP6, k, prefixlen);
	struct nexthop *existing = e != NULL ? e->nh : NULL;
	if (existing != NULL && !replace) {
		const bool equal = existing->vrf_id == nh->vrf_id && existing->iface_id == nh->iface_id
			&& existing->type == nh->type;
		return errno_set(equal ? EEXIST : EBUSY);
	}
	if (e == NULL && (e = rib_add()) == NULL)
		return errno_set(ENOMEM);
	*e = (struct rib_entry) {.vrf_id = vrf_id, .af = GR_AF_IP6, .prefixlen = prefixlen, .origin = origin, .nh = nh};
	memcpy(e->ip, k, 16);
	struct route6_event ev = {.vrf_id = vrf_id, .origin = origin, .nh = nh, .iface_id = iface_id};
	memcpy(ev.dest.ip, ip, 16);
	ev.dest.prefixlen = prefixlen;
	if (origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_IP6_ROUTE_ADD, &ev);
	else
		event_push_internal(GR_EVENT_IP6_ROUTE_ADD, &ev); // patch
	nexthop_incref(nh);
	if (existing != NULL)
		nexthop_decref(existing);
	return 0;
}

int rib6_insert(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen, gr_nh_origin_t origin,
		struct nexthop *nh) {
	return rib6_insert_or_replace(vrf_id, iface_id, ip, prefixlen, origin, nh, false);
}

// rib6_delete (route.c:310-360)
int rib6_delete(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen, gr_nh_type_t nh_type) {
	uint8_t tmp[16], k[16];
	if (get_vrf_iface(vrf_id) == NULL)
		return errno_set(ENONET);
	memcpy(k, ll_scope(ip, tmp, iface_id), 16);
	mask16(k, prefixlen);
	struct rib_entry *e = rib_exact(vrf_id, GR_AF_IP6, k, prefixlen);
	if (e == NULL)
		return errno_set(ENOENT);
	struct nexthop *nh = e->nh;
	const gr_nh_origin_t origin = e->origin;
	if (nh->type != nh_type)
		return errno_set(EINVAL);
	rib_remove(e);
	struct route6_event ev = {.vrf_id = vrf_id, .origin = origin, .nh = nh, .iface_id = iface_id};
	memcpy(ev.dest.ip, ip, 16);
	ev.dest.prefixlen = prefixlen;
	if (origin != GR_NH_ORIGIN_INTERNAL)
		event_push(GR_EVENT_IP6_ROUTE_DEL, &ev);
	else
		event_push_internal(GR_EVENT_IP6_ROUTE_DEL, &ev); // patch
	nexthop_decref(nh);
	return 0;
}

struct nexthop *rib6_lookup(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16]) {
	uint8_t tmp[16];
	const uint8_t *k = ll_scope(ip, tmp, iface_id);
	struct rib_entry *best = NULL;
	for (uint32_t i = 0; i < rib_n; i++)
		if (rib[i].vrf_id == vrf_id && rib[i].af == GR_AF_IP6 && in_prefix6(&rib[i], k)
		    && (best == NULL || rib[i].prefixlen > best->prefixlen))
			best = &rib[i];
	return best != NULL ? best->nh : errno_set_null(ENETUNREACH);
}

void rib6_cleanup(struct nexthop *nh) {
	rib_cleanup(nh, GR_AF_IP6);
}

// route6_add / route6_del (ip6 route.c:362-430)
int route6_add(uint16_t vrf_id, const uint8_t ip[16], uint8_t prefixlen, const uint8_t gw[16], uint32_t nh_id,
	       gr_nh_origin_t origin, bool exist_ok) {
	bool created = false;
	struct nexthop *nh;
	if (origin == GR_NH_ORIGIN_INTERNAL)
		return errno_set(EINVAL);
	if (nh_id != GR_NH_ID_UNSET) {
		if ((nh = nexthop_lookup_id(nh_id)) == NULL)
			return errno_set(ENOENT);
	} else {
		nh = nh6_lookup(vrf_id, GR_IFACE_ID_UNDEF, gw);
		if (nh == NULL && (nh = rib6_lookup(vrf_id, GR_IFACE_ID_UNDEF, gw)) == NULL)
			return errno_set(EHOSTUNREACH);
		if (nh->type != GR_NH_T_L3 || memcmp(nexthop_info_l3(nh)->ipv6, gw, 16) != 0) {
			const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .iface_id = nh->iface_id,
							     .vrf_id = vrf_id, .origin = origin};
			struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP6};
			memcpy(l3.ipv6, gw, 16);
			if ((nh = nexthop_new(&base, &l3)) == NULL)
				return -errno;
			created = true;
		}
	}
	int ret = rib6_insert_or_replace(vrf_id, GR_IFACE_ID_UNDEF, ip, prefixlen, origin, nh, exist_ok);
	if (ret < 0 && created)
		nexthop_decref(nh);
	return ret;
}

int route6_del(uint16_t vrf_id, const uint8_t ip[16], uint8_t prefixlen, bool missing_ok) {
	struct nexthop *nh = rib6_lookup(vrf_id, GR_IFACE_ID_UNDEF, ip);
	int ret = rib6_delete(vrf_id, GR_IFACE_ID_UNDEF, ip, prefixlen, nh != NULL ? nh->type : GR_NH_T_L3);
	if ((ret == -ENOENT || ret == -ENONET) && missing_ok)
		ret = 0;
	return ret;
}

// iface6_addr_add (modules/ip6/control/address.c:177-260), without the solicited-node multicast
// group join (multicast membership stays on the CPU, mcast6_addr_add)
int addr6_add(uint16_t iface_id, const uint8_t ip[16], uint16_t prefixlen, gr_nh_origin_t origin) {
	const struct iface *iface = iface_from_id_rw(iface_id);
	struct nexthop *nh;
	if (iface == NULL)
		return errno_set(ENODEV);
	if (iface->mode != GR_IFACE_MODE_VRF)
		return errno_set(EMEDIUMTYPE);
	for (uint32_t i = 0; i < n_addrs6[iface_id]; i++) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs6[iface_id][i]);
		if (prefixlen == l3->prefixlen && memcmp(l3->ipv6, ip, 16) == 0)
			return errno_set(EEXIST);
	}
	if (nh6_lookup(iface->vrf_id, iface->id, ip) != NULL)
		return errno_set(EADDRINUSE);
	if (n_addrs6[iface_id] == MAX_ADDRS)
		return errno_set(ENOSPC);
	const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .iface_id = iface->id, .vrf_id = iface->vrf_id,
					     .origin = GR_NH_ORIGIN_INTERNAL};
	struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP6, .prefixlen = (uint8_t)prefixlen,
					.flags = NH_LOCAL_ADDR_FLAGS, .state = GR_NH_S_REACHABLE};
	memcpy(l3.ipv6, ip, 16);
	if (iface_get_eth_addr(iface, &l3.mac) < 0 && errno != EOPNOTSUPP)
		return -errno;
	if ((nh = nexthop_new(&base, &l3)) == NULL)
		return -errno;
	int ret = rib6_insert(iface->vrf_id, iface->id, ip, (uint8_t)prefixlen, origin, nh);
	if (ret < 0)
		return ret;
	addrs6[iface_id][n_addrs6[iface_id]++] = nh;
	struct gr_ip6_ifaddr a = {.prefixlen = (uint8_t)prefixlen, .iface_id = iface_id};
	memcpy(a.ip, ip, 16);
	event_push(GR_EVENT_IP6_ADDR_ADD, &a);
	return 0;
}

int addr6_delete(uint16_t iface_id, const uint8_t ip[16], uint16_t prefixlen) {
	if (iface_id >= GR_MAX_IFACES)
		return errno_set(ENODEV);
	uint32_t i = 0;
	struct nexthop *nh = NULL;
	for (; i < n_addrs6[iface_id]; i++) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(addrs6[iface_id][i]);
		if (l3->prefixlen == prefixlen && memcmp(l3->ipv6, ip, 16) == 0) {
			nh = addrs6[iface_id][i];
			break;
		}
	}
	if (nh == NULL)
		return errno_set(ENOENT);
	struct gr_ip6_ifaddr a = {.prefixlen = (uint8_t)prefixlen, .iface_id = iface_id};
	memcpy(a.ip, ip, 16);
	event_push(GR_EVENT_IP6_ADDR_DEL, &a);
	nexthop_routes_cleanup(nh);
	while (nh->ref_count > 0)
		nexthop_decref(nh);
	memmove(&addrs6[iface_id][i], &addrs6[iface_id][i + 1], (n_addrs6[iface_id] - i - 1) * sizeof(nh));
	n_addrs6[iface_id]--;
	return 0;
}

// ndp_probe_input_cb (ip6 nexthop.c:180-240): learn or refresh a neighbour
int ndp_probe_input(uint16_t iface_id, const uint8_t ip[16], const struct rte_ether_addr *mac) {
	const struct iface *iface = iface_from_id_rw(iface_id);
	if (iface == NULL)
		return errno_set(ENODEV);
	if (ip6_is_unspec(ip) || ip[0] == 0xff)
		return errno_set(EINVAL);
	struct nexthop *nh = nh6_lookup(iface->vrf_id, iface->id, ip);
	if (nh == NULL) {
		const struct gr_nexthop_base base = {.type = GR_NH_T_L3, .iface_id = iface->id,
						     .vrf_id = iface->vrf_id, .origin = GR_NH_ORIGIN_LEARN};
		struct gr_nexthop_info_l3 l3 = {.af = GR_AF_IP6, .mac = *mac, .flags = GR_NH_F_NEIGH};
		memcpy(l3.ipv6, ip, 16);
		if ((nh = nexthop_new(&base, &l3)) == NULL)
			return -errno;
		if (rib6_insert(iface->vrf_id, iface->id, ip, 128, GR_NH_ORIGIN_INTERNAL, nh) < 0) {
			nexthop_decref(nh);
			return -errno;
		}
	} else {
		struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
		l3->state = GR_NH_S_REACHABLE;
		l3->ucast_probes = 0;
		l3->bcast_probes = 0;
		l3->mac = *mac;
		if (nh->origin != GR_NH_ORIGIN_INTERNAL)
			event_push(GR_EVENT_NEXTHOP_UPDATE, nh);
		else
			event_push_internal(GR_EVENT_NEXTHOP_UPDATE, nh); // patch
	}
	return 0;
}

// ---- reset (tests) ---------------------------------------------------------
static void drop_all_cb(struct nexthop *nh, void *priv) {
	(void)priv;
	nexthop_routes_cleanup(nh);
	while (nh->ref_count)
		nexthop_decref(nh);
}

void gr_test_control_reset(void) {
	// the addresses, every route (the VRFs still there), every nexthop, then
	// the ifaces: sub-interfaces first, VRFs last
	for (uint16_t id = 1; id < GR_MAX_IFACES; id++)
		if (if_used[id])
			addr_iface_cleanup(GR_EVENT_IFACE_PRE_REMOVE, &ifs[id]);
	rib4_cleanup(NULL);
	rib6_cleanup(NULL);
	for (uint32_t k = 0; k < NH_POOL; k++)
		if (nh_busy[k] && nh_pool[k].ref_count)
			drop_all_cb(&nh_pool[k], NULL);
	for (int pass = 0; pass < 3; pass++)
		for (uint16_t id = 1; id < GR_MAX_IFACES; id++) {
			if (!if_used[id])
				continue;
			const int t = ifs[id].type;
			if ((pass == 0 && t == GR_IFACE_TYPE_VLAN) || (pass == 1 && t != GR_IFACE_TYPE_VRF)
			    || pass == 2)
				iface_destroy(&ifs[id]);
		}
}

RTE_INIT(gr_control_min_init) {
	event_subscribe(GR_EVENT_IFACE_PRE_REMOVE, nexthop_iface_cleanup); // nexthop.c:592
	event_subscribe(GR_EVENT_IFACE_PRE_REMOVE, addr_iface_cleanup); // address.c:325
}
