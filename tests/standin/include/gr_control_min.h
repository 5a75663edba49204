// SPDX-License-Identifier: BSD-3-Clause
//
// gr_control_min.h -- a stand-in for the part of grout's control plane that
// creates, changes and destroys the objects the fast path mirrors, for the
// tests (gr_control_min.c restates it). Same names, argument meanings, event
// order and errors as grout:
//
//   events       main/event.{h,c} (event_subscribe / event_push), plus the
//                in-process channel integration/grout-gpu_fwd4-control.patch
//                adds (event_subscribe_internal / event_push_internal)
//   ifaces       modules/infra/control/iface.c:171-267 (iface_create),
//                :632-654 (iface_set_up_down), :506-523 (iface_set_eth_addr),
//                :690-725 (iface_destroy)
//   nexthops     modules/infra/control/nexthop.c:317-530, l3_nexthop.c
//                (import, lookup, ageing), group_nexthop.c
//   IPv4 / IPv6  modules/ip/control/route.c:212-400, address.c:60-200,
//                nexthop.c:33-185; modules/ip6/control/route.c:229-360,
//                address.c:180-290, nexthop.c:40-240
//   nexthop API  modules/infra/api/nexthop.c:29-78
//
// The RIBs are plain lists (the stand-in has no rte_fib): what matters here is
// which objects grout creates and which events (or none) it pushes, in which
// order, with which rte_rcu_qsbr_synchronize between them. Everything runs on
// the control thread.
#pragma once

#include "gr_datapath_min.h"

#ifdef __cplusplus
extern "C" {
#endif

// ---- events (main/event.h; gr_api.h:32 GR_MSG_TYPE) -------------------------
#define GR_MSG_TYPE(module, id) (((uint32_t)(0xffff & (module)) << 16) | (0xffff & (id)))
#define GR_INFRA_MODULE 0xacdc
#define GR_IP4_MODULE 0xf00d
#define GR_IP6_MODULE 0xfeed
enum { // gr_infra.h:257-266
	GR_EVENT_IFACE_ADD = GR_MSG_TYPE(GR_INFRA_MODULE, 0x1001),
	GR_EVENT_IFACE_POST_ADD,
	GR_EVENT_IFACE_PRE_REMOVE,
	GR_EVENT_IFACE_REMOVE,
	GR_EVENT_IFACE_POST_RECONFIG,
	GR_EVENT_IFACE_STATUS_UP,
	GR_EVENT_IFACE_STATUS_DOWN,
	GR_EVENT_IFACE_MAC_CHANGE,
};
enum { // gr_nexthop.h:135-139
	GR_EVENT_NEXTHOP_NEW = GR_MSG_TYPE(GR_INFRA_MODULE, 0x3001),
	GR_EVENT_NEXTHOP_DELETE,
	GR_EVENT_NEXTHOP_UPDATE,
};
enum { // gr_ip4.h:179-184
	GR_EVENT_IP_ADDR_ADD = GR_MSG_TYPE(GR_IP4_MODULE, 0x1001),
	GR_EVENT_IP_ADDR_DEL,
	GR_EVENT_IP_ROUTE_ADD,
	GR_EVENT_IP_ROUTE_DEL,
};
enum { // gr_ip6.h:219-224
	GR_EVENT_IP6_ADDR_ADD = GR_MSG_TYPE(GR_IP6_MODULE, 0x1001),
	GR_EVENT_IP6_ADDR_DEL,
	GR_EVENT_IP6_ROUTE_ADD,
	GR_EVENT_IP6_ROUTE_DEL,
};

typedef void (*event_sub_cb_t)(uint32_t ev_type, const void *obj);
void event_subscribe(uint32_t ev_type, event_sub_cb_t callback);
void event_push(uint32_t ev_type, const void *obj);
// The patch's in-process channel: changes grout publishes to no API client
// (GR_NH_ORIGIN_INTERNAL objects, nexthop state changes without an event),
// delivered only to callbacks registered with event_subscribe_internal.
void event_subscribe_internal(uint32_t ev_type, event_sub_cb_t callback);
void event_push_internal(uint32_t ev_type, const void *obj);
// nexthop_destroy pushes it on the internal channel before it waits for the
// datapath (the patch defines it in modules/infra/control/nexthop.h): a
// subscriber that holds FIB changes back publishes them first.
#define GR_EVENT_NEXTHOP_PRE_DELETE GR_MSG_TYPE(GR_INFRA_MODULE, 0x30ff)
// Tests: the event counters zeroed; events pushed (public, internal) since.
void gr_test_events_reset(void);
// Tests: 0 = grout without the patch (event_push_internal does nothing).
void gr_test_internal_events(int on);
void gr_test_events_count(uint64_t *pub, uint64_t *internal);

// ---- the control thread's event loop: libevent's timers (in grout, libevent
// itself on the event base modules get at init) -------------------------------
struct event;
struct timeval;
typedef int evutil_socket_t; // libevent's, on POSIX (event2/util.h)
typedef void (*event_callback_fn)(evutil_socket_t, short, void *); // event2/event.h
struct event *event_new(struct event_base *base, evutil_socket_t fd, short what, event_callback_fn cb, void *arg);
int event_add(struct event *ev, const struct timeval *tv);
int event_del(struct event *ev);
void event_free(struct event *ev);
#define evtimer_new(b, cb, arg) event_new((b), -1, 0, (cb), (arg))
#define evtimer_add(ev, tv) event_add((ev), (tv))
#define evtimer_del(ev) event_del(ev)
// Tests: one turn of the control thread's loop ends (each harness control
// call is one): every pending timer fires. Time is not modelled: a turn is
// taken to outlast any timer's delay.
void gr_test_event_loop_turn(void);
// The control thread's event base the harness gives modules at init (grout:
// its libevent base). An event made without one cannot be added (libevent's
// event_add: "event has no event_base set", -1).
struct event_base *gr_test_event_base(void);

// route4_event / route6_event (modules/ip/control/route.c:205-210,
// modules/ip6/control/route.c:222-227), moved into ip4.h / ip6.h by the
// patch so that a subscriber can read them; route6_event gains the scope
// iface of a link-local prefix (addr6_linklocal_scope, ip6.h:23-36).
struct ip4_net {
	ip4_addr_t ip;
	uint8_t prefixlen;
};
struct ip6_net {
	uint8_t ip[16];
	uint8_t prefixlen;
};
struct route4_event {
	struct ip4_net dest;
	uint16_t vrf_id;
	gr_nh_origin_t origin;
	const struct nexthop *nh;
};
struct route6_event {
	struct ip6_net dest;
	uint16_t vrf_id;
	gr_nh_origin_t origin;
	const struct nexthop *nh;
	uint16_t iface_id; // added by the patch: the scope of a link-local prefix
};

// struct gr_ip4_ifaddr / gr_ip6_ifaddr (gr_ip4.h, gr_ip6.h): the ADDR events' objects
struct gr_ip4_ifaddr {
	ip4_addr_t ip;
	uint8_t prefixlen;
	uint16_t iface_id;
};
struct gr_ip6_ifaddr {
	uint8_t ip[16];
	uint8_t prefixlen;
	uint16_t iface_id;
};

// ---- ifaces ------------------------------------------------------------------
// struct gr_iface (gr_infra.h:90-96), and the per-type API info the stand-in
// takes (gr_infra.h:105-153; a port's DPDK port id is given, grout gets it
// from the probed device).
struct gr_iface {
	union {
		struct __gr_iface_base base;
		struct {
			GR_IFACE_BASE_FIELDS
		};
	};
	char name[16];
};
struct gr_iface_info_vrf {
	struct gr_iface_info_vrf_fib ipv4;
	struct gr_iface_info_vrf_fib ipv6;
	struct rte_ether_addr mac;
};
struct gr_iface_info_port {
	struct rte_ether_addr mac;
	uint16_t port_id;
};
struct gr_iface_info_vlan {
	uint16_t parent_id;
	uint16_t vlan_id;
	struct rte_ether_addr mac; // zero: the parent's (vlan.c:174-192)
};

// conf->id != 0 asks for that id (the stand-in's way to lay out ids; grout
// allocates them). A VRF-mode iface with vrf_id UNDEF joins VRF 1, created
// on demand (gr_infra.h:81-84). NULL + errno on failure.
struct iface *iface_create(const struct gr_iface *conf, const void *api_info);
int iface_destroy(struct iface *);
int iface_set_up_down(struct iface *, bool up);
int iface_set_eth_addr(struct iface *, const struct rte_ether_addr *);
// iface_reconfig of a VRF's FIB sizes (GR_VRF_SET_FIB): NULL or zero sizes leave a family as it is.
int iface_vrf_reconfig_fib(struct iface *, const struct gr_iface_info_vrf_fib *v4,
			   const struct gr_iface_info_vrf_fib *v6);
int iface_get_eth_addr(const struct iface *, struct rte_ether_addr *);
struct iface *iface_from_id_rw(uint16_t id);
// The stand-in's iface storage (ids index it), for the harness's decoding.
struct iface *gr_test_iface_base(void);

// ---- nexthops ----------------------------------------------------------------
struct gr_nexthop_group_member {
	uint32_t nh_id;
	uint32_t weight;
};
struct gr_nexthop_info_group {
	uint32_t n_members;
	struct gr_nexthop_group_member members[];
};

struct nexthop *nexthop_new(const struct gr_nexthop_base *, const void *info);
int nexthop_update(struct nexthop *, const struct gr_nexthop_base *, const void *info);
void nexthop_incref(struct nexthop *);
void nexthop_decref(struct nexthop *);
struct nexthop *nexthop_lookup(const struct gr_nexthop_base *, const void *info);
struct nexthop *nexthop_lookup_id(uint32_t nh_id);
struct nexthop *nexthop_lookup_l3(addr_family_t af, uint16_t vrf_id, uint16_t iface_id, const void *addr);
void nexthop_routes_cleanup(struct nexthop *);
typedef void (*nh_iter_cb_t)(struct nexthop *nh, void *priv);
void nexthop_iter(nh_iter_cb_t, void *priv);
// l3_age (l3_nexthop.c:322-362) on one LEARN nexthop, as if its last reply
// were reply_age_s old and `probes` probes had been sent.
void nexthop_l3_age(struct nexthop *, uint32_t reply_age_s, uint32_t probes);
// nexthop API (modules/infra/api/nexthop.c:29-78): 0 or -errno.
int nh_add(const struct gr_nexthop_base *, const void *info, bool exist_ok);
int nh_del(const struct gr_nexthop_base *, const void *info, bool missing_ok);
// The stand-in's nexthop storage (grout: the rte_mempool), for decoding.
struct nexthop *gr_test_nh_base(uint32_t *count);

static inline struct nexthop *nh4_lookup(uint16_t vrf_id, ip4_addr_t ip) { // ip4.h:21-24
	return nexthop_lookup_l3(GR_AF_IP4, vrf_id, GR_IFACE_ID_UNDEF, &ip);
}
static inline struct nexthop *nh6_lookup(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16]) {
	return nexthop_lookup_l3(GR_AF_IP6, vrf_id, iface_id, ip);
}

// ---- IPv4 --------------------------------------------------------------------
int rib4_insert(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, gr_nh_origin_t origin, struct nexthop *nh);
int rib4_delete(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, gr_nh_type_t nh_type);
struct nexthop *rib4_lookup(uint16_t vrf_id, ip4_addr_t ip);
struct nexthop *rib4_lookup_exact(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen);
void rib4_cleanup(struct nexthop *);
// route4_add / route4_del API handlers (route.c:336-399): gw 0 with nh_id.
int route4_add(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, ip4_addr_t gw, uint32_t nh_id,
	       gr_nh_origin_t origin, bool exist_ok);
int route4_del(uint16_t vrf_id, ip4_addr_t ip, uint8_t prefixlen, bool missing_ok);
int addr4_add(uint16_t iface_id, ip4_addr_t ip, uint16_t prefixlen, gr_nh_origin_t origin);
int addr4_delete(uint16_t iface_id, ip4_addr_t ip, uint16_t prefixlen);
// The control-thread part of arp_probe_input_cb (ip/control/nexthop.c:127-185):
// an ARP packet from (sip, sha) received on iface.
int arp_probe_input(uint16_t iface_id, ip4_addr_t sip, const struct rte_ether_addr *sha);
// nh4_resolve_cb (ip/control/nexthop.c:33-125) for a packet to dst that
// ip_output held on nexthop nh: the nexthop the packet now waits on (a LEARN
// nexthop + its INTERNAL /32 for a connected destination).
struct nexthop *nh4_resolve(struct nexthop *nh, ip4_addr_t dst);

// ---- IPv6 --------------------------------------------------------------------
int rib6_insert(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen, gr_nh_origin_t origin,
		struct nexthop *nh);
int rib6_delete(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen, gr_nh_type_t nh_type);
struct nexthop *rib6_lookup(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16]);
void rib6_cleanup(struct nexthop *);
int route6_add(uint16_t vrf_id, const uint8_t ip[16], uint8_t prefixlen, const uint8_t gw[16], uint32_t nh_id,
	       gr_nh_origin_t origin, bool exist_ok);
int route6_del(uint16_t vrf_id, const uint8_t ip[16], uint8_t prefixlen, bool missing_ok);
int addr6_add(uint16_t iface_id, const uint8_t ip[16], uint16_t prefixlen, gr_nh_origin_t origin);
int addr6_delete(uint16_t iface_id, const uint8_t ip[16], uint16_t prefixlen);
// The control-thread part of ndp_probe_input_cb (ip6/control/nexthop.c:150-240)
// for a neighbour advertisement / solicitation carrying a link-layer address.
int ndp_probe_input(uint16_t iface_id, const uint8_t ip[16], const struct rte_ether_addr *mac);

// Tests: destroy every object (ifaces, nexthops, routes) in grout's order.
void gr_test_control_reset(void);

#ifdef __cplusplus
}
#endif
