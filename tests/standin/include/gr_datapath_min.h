// SPDX-License-Identifier: BSD-3-Clause
//
// gr_datapath_min.h -- a stand-in for the part of grout's own datapath and
// module surface that a grout node uses, on top of rte_graph_min.h:
//
//   mbuf private data       modules/infra/datapath/mbuf.h:27-41 (layout:
//                           trace head, iface, then the node's fields),
//                           rxtx.h:45-48, eth.h:14-36, l3.h:9
//   node registration       modules/infra/control/graph.h:31-85
//                           (GR_NODE_CTX_TYPE, gr_node_info, GR_NODE_REGISTER,
//                           GR_DROP_REGISTER), gr_node_attach_parent
//                           (graph.c:35-63), the registration walk of
//                           graph_init (graph.c:652-688)
//   modules                 main/module.h:43-49 (struct module, module_register)
//
// The objects grout's nodes dereference (struct iface, struct nexthop) have
// grout's layout: the public base fields, then per-type info
// (modules/infra/control/iface.h:20-35, nexthop.h:22-96). Nothing in the
// datapath node reads more than the base fields and the L3 info; the control
// plane stand-in (gr_control_min.h) and the mirror (gpu_fwd4_control.c) use
// the rest. Everything here is written for this repo; in grout the node
// includes grout's real headers instead.
#pragma once

#include "rte_graph_min.h"
#include "rte_rcu_min.h"

#include <grout_hip.h>
#include <stdalign.h>
#include <stdbool.h>
#include <sys/queue.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- objects ---------------------------------------------------------------
// gr_iface_type_t / gr_iface_flags_t / gr_iface_mode_t (gr_infra.h:18-62),
// gr_nh_* (gr_nexthop.h:12-82) and addr_family_t (gr_net_types.h): grout's
// values.
typedef uint8_t gr_iface_type_t; // grout: enum : uint8_t (C23)
enum {
	GR_IFACE_TYPE_UNDEF = 0,
	GR_IFACE_TYPE_VRF,
	GR_IFACE_TYPE_PORT,
	GR_IFACE_TYPE_VLAN,
	GR_IFACE_TYPE_IPIP,
	GR_IFACE_TYPE_BOND,
	GR_IFACE_TYPE_BRIDGE,
	GR_IFACE_TYPE_VXLAN,
};
typedef uint8_t gr_iface_mode_t;
#define GR_IFACE_MODE_VRF GR_HIP_IFACE_MODE_VRF
#define GR_IFACE_MODE_XC GR_HIP_IFACE_MODE_XC
#define GR_IFACE_F_UP GR_HIP_IFACE_F_UP
#define GR_IFACE_F_SNAT_STATIC GR_HIP_IFACE_F_SNAT_STATIC
#define GR_IFACE_F_SNAT_DYNAMIC GR_HIP_IFACE_F_SNAT_DYNAMIC
#define GR_IFACE_S_RUNNING 0x0001

// GR_IFACE_ID_UNDEF, GR_VRF_DEFAULT_ID, GR_VRF_ID_UNDEF (gr_infra.h:48-53)
#define GR_IFACE_ID_UNDEF 0
#define GR_VRF_DEFAULT_ID 1
#define GR_VRF_ID_UNDEF GR_IFACE_ID_UNDEF
typedef uint8_t addr_family_t;
#define GR_AF_UNSPEC GR_HIP_AF_UNSPEC
#define GR_AF_IP4 GR_HIP_AF_IP4
#define GR_AF_IP6 GR_HIP_AF_IP6
typedef uint8_t gr_nh_type_t;
#define GR_NH_T_L3 GR_HIP_NH_T_L3
#define GR_NH_T_BLACKHOLE GR_HIP_NH_T_BLACKHOLE
#define GR_NH_T_REJECT GR_HIP_NH_T_REJECT
#define GR_NH_T_GROUP GR_HIP_NH_T_GROUP
typedef uint8_t gr_nh_state_t;
#define GR_NH_S_NEW GR_HIP_NH_S_NEW
#define GR_NH_S_PENDING GR_HIP_NH_S_PENDING
#define GR_NH_S_REACHABLE GR_HIP_NH_S_REACHABLE
#define GR_NH_S_STALE GR_HIP_NH_S_STALE
#define GR_NH_S_FAILED GR_HIP_NH_S_FAILED
typedef uint8_t gr_nh_flags_t;
#define GR_NH_F_LOCAL GR_HIP_NH_F_LOCAL
#define GR_NH_F_GATEWAY GR_HIP_NH_F_GATEWAY
#define GR_NH_F_LINK GR_HIP_NH_F_LINK
#define GR_NH_F_MCAST GR_HIP_NH_F_MCAST
#define GR_NH_F_NEIGH 0x20
#define NH_LOCAL_ADDR_FLAGS (GR_NH_F_LOCAL | GR_NH_F_LINK) // nexthop.h:185
typedef uint8_t gr_nh_origin_t;
#define GR_NH_ORIGIN_UNSPEC 0
#define GR_NH_ORIGIN_LINK 2
#define GR_NH_ORIGIN_LEARN 3
#define GR_NH_ORIGIN_STATIC 4
#define GR_NH_ORIGIN_ZEBRA 11
#define GR_NH_ORIGIN_BGP 186
#define GR_NH_ORIGIN_INTERNAL 255
#define GR_NH_ID_UNSET 0
typedef uint32_t ip4_addr_t; // network order

// __gr_iface_base (gr_infra.h:73-87)
#define GR_IFACE_BASE_FIELDS                                                                       \
	uint16_t id;                                                                               \
	gr_iface_type_t type;                                                                      \
	gr_iface_mode_t mode;                                                                      \
	uint16_t flags;                                                                            \
	uint16_t state;                                                                            \
	uint16_t mtu;                                                                              \
	uint16_t vrf_id;                                                                           \
	uint16_t domain_id;                                                                        \
	uint32_t speed;
struct __gr_iface_base {
	GR_IFACE_BASE_FIELDS
};

#define GR_IFACE_INFO_SIZE 64
struct iface {
	union { // BASE(__gr_iface_base)
		struct __gr_iface_base base;
		struct {
			GR_IFACE_BASE_FIELDS
		};
	};
	char *name;
	alignas(void *) uint8_t info[GR_IFACE_INFO_SIZE]; // grout: sized by type
};

// Per-type iface info (GR_IFACE_INFO, iface.h:37-42): vrf.h:10-16,
// port.h:17-30, vlan.h:10 over gr_infra.h:105-153.
struct gr_iface_info_vrf_fib {
	uint32_t max_routes; // 0 = default
	uint32_t num_tbl8; // 0 = auto
};
struct iface_info_vrf {
	struct gr_iface_info_vrf_fib ipv4;
	struct gr_iface_info_vrf_fib ipv6;
	struct rte_ether_addr mac;
	uint16_t ref_count;
};
struct iface_info_port {
	uint16_t n_rxq, n_txq, rxq_size, txq_size;
	struct rte_ether_addr mac;
	uint16_t port_id;
};
struct iface_info_vlan {
	uint16_t parent_id;
	uint16_t vlan_id;
	struct rte_ether_addr mac;
};
#define GR_IFACE_INFO_GETTER(type_name)                                                            \
	static inline struct type_name *type_name(const struct iface *iface) {                     \
		_Static_assert(sizeof(struct type_name) <= GR_IFACE_INFO_SIZE, #type_name);        \
		return (struct type_name *)iface->info;                                            \
	}
GR_IFACE_INFO_GETTER(iface_info_vrf)
GR_IFACE_INFO_GETTER(iface_info_port)
GR_IFACE_INFO_GETTER(iface_info_vlan)

// struct gr_nexthop_base (gr_nexthop.h:84-90)
#define GR_NEXTHOP_BASE_FIELDS                                                                     \
	gr_nh_type_t type;                                                                         \
	gr_nh_origin_t origin;                                                                     \
	uint16_t iface_id;                                                                         \
	uint16_t vrf_id;                                                                           \
	uint32_t nh_id;
struct gr_nexthop_base {
	GR_NEXTHOP_BASE_FIELDS
};

// struct gr_nexthop_info_l3 (gr_nexthop.h:93-105)
#define GR_NEXTHOP_INFO_L3_FIELDS                                                                  \
	gr_nh_state_t state;                                                                       \
	gr_nh_flags_t flags;                                                                       \
	addr_family_t af;                                                                          \
	uint8_t prefixlen;                                                                         \
	union {                                                                                    \
		ip4_addr_t ipv4;                                                                   \
		uint8_t ipv6[16];                                                                  \
	};                                                                                         \
	struct rte_ether_addr mac;
struct gr_nexthop_info_l3 {
	GR_NEXTHOP_INFO_L3_FIELDS
};

// struct nexthop (nexthop.h:22-31): two cache lines
struct nexthop {
	union { // BASE(gr_nexthop_base)
		struct gr_nexthop_base base;
		struct {
			GR_NEXTHOP_BASE_FIELDS
		};
	};
	uint32_t ref_count; // number of routes referencing this nexthop
	alignas(void *) uint8_t info[128 - sizeof(struct gr_nexthop_base) - sizeof(uint32_t)];
};

// GR_NH_TYPE_INFO(GR_NH_T_L3, nexthop_info_l3, ...) (nexthop.h:43-56)
struct nexthop_info_l3 {
	union { // BASE(gr_nexthop_info_l3)
		struct gr_nexthop_info_l3 base;
		struct {
			GR_NEXTHOP_INFO_L3_FIELDS
		};
	};
	uint64_t last_reply;
	uint64_t last_request;
	uint8_t ucast_probes;
	uint8_t bcast_probes;
	uint16_t held_pkts;
};

// GR_NH_TYPE_INFO(GR_NH_T_GROUP, nexthop_info_group, ...) (nexthop.h:75-87)
struct nh_group_member {
	struct nexthop *nh;
	uint32_t weight;
};
#define MAX_NH_GROUP_RETA_SIZE 4096
struct nexthop_info_group {
	uint16_t n_members;
	uint16_t reta_size; // a power of two
	struct nexthop *nh; // shortcut when there is a single nexthop in the group
	struct nh_group_member *members;
	struct nexthop **reta;
};

static inline struct nexthop_info_l3 *nexthop_info_l3(const struct nexthop *nh) {
	_Static_assert(sizeof(struct nexthop_info_l3) <= sizeof(((struct nexthop *)0)->info), "l3 info");
	return (struct nexthop_info_l3 *)nh->info;
}

static inline struct nexthop_info_group *nexthop_info_group(const struct nexthop *nh) {
	_Static_assert(sizeof(struct nexthop_info_group) <= sizeof(((struct nexthop *)0)->info), "group info");
	return (struct nexthop_info_group *)nh->info;
}

// grout's iface registry (iface.c:459-466: ifaces[id], cleared by
// iface_destroy before its RCU synchronisation, :710-712). The nexthop
// objects the fast path names by slot are the node's own registry
// (gpu_fwd4_nh_obj_set), not grout's.
#define GR_MAX_IFACES 1024
const struct iface *iface_from_id(uint16_t id);
void gr_iface_register(struct iface *);
void gr_iface_unregister(uint16_t id);

// ---- lcores, RCU, per-lcore iface counters ---------------------------------
#define RTE_MAX_LCORE 128
// The calling thread's lcore id (DPDK rte_lcore_id()); the stand-in's threads
// set theirs with gr_test_lcore_set (default 0).
unsigned rte_lcore_id(void);
void gr_test_lcore_set(unsigned lcore_id);

// The datapath's QSBR variable (main_loop.c:534-536, created by the "rcu"
// module, :538-543): every worker registers its lcore id as a reader
// (:408); the datapath hooks' modules register theirs above (sized in by
// integration/grout-gpu_fwd4-datapath.patch, see "datapath hooks" below).
struct rte_rcu_qsbr *gr_datapath_rcu(void);

// struct iface_stats and its per-lcore table (iface.h:105-119)
struct iface_stats {
	uint64_t rx_packets;
	uint64_t rx_bytes;
	uint64_t tx_packets;
	uint64_t tx_bytes;
	uint64_t cp_rx_packets;
	uint64_t cp_rx_bytes;
	uint64_t cp_tx_packets;
	uint64_t cp_tx_bytes;
} __attribute__((aligned(64)));

extern struct iface_stats (*iface_stats)[RTE_MAX_LCORE];
static inline struct iface_stats *iface_get_stats(uint16_t lcore_id, uint16_t ifid) {
	return &iface_stats[ifid][lcore_id];
}

// ---- mbuf private data -----------------------------------------------------
struct gr_trace_item;
STAILQ_HEAD(gr_trace_head, gr_trace_item);

#define GR_MBUF_PRIV_MAX_SIZE 64

#define GR_MBUF_PRIV_DATA_TYPE(type_name, fields)                                                  \
	struct type_name {                                                                         \
		struct gr_trace_head traces;                                                       \
		const struct iface *iface;                                                         \
		struct fields;                                                                     \
	};                                                                                         \
	static inline struct type_name *type_name(struct rte_mbuf *m) {                            \
		_Static_assert(sizeof(struct type_name) <= GR_MBUF_PRIV_MAX_SIZE, #type_name);     \
		return (struct type_name *)rte_mbuf_to_priv(m);                                    \
	}

typedef enum {
	ETH_DOMAIN_UNKNOWN = 0,
	ETH_DOMAIN_LOOPBACK,
	ETH_DOMAIN_LOCAL,
	ETH_DOMAIN_BROADCAST,
	ETH_DOMAIN_MULTICAST,
	ETH_DOMAIN_OTHER,
} eth_domain_t;

struct l3_addr { // gr_net_types.h: an address family and an IPv4/IPv6 address
	addr_family_t af;
	union {
		ip4_addr_t ipv4;
		uint8_t ipv6[16];
	};
};

GR_MBUF_PRIV_DATA_TYPE(mbuf_data, {});
GR_MBUF_PRIV_DATA_TYPE(iface_mbuf_data, {
	uint16_t vlan_id;
	struct l3_addr vtep;
});
GR_MBUF_PRIV_DATA_TYPE(eth_input_mbuf_data, {
	eth_domain_t domain;
	const struct nexthop *nh;
});
GR_MBUF_PRIV_DATA_TYPE(l3_mbuf_data, { const struct nexthop *nh; });
GR_MBUF_PRIV_DATA_TYPE(eth_output_mbuf_data, {
	struct rte_ether_addr dst;
	rte_be16_t ether_type;
	struct l3_addr vtep;
});

// ---- conntrack and NAT (modules/policy: conntrack.h:24-67,
// nat_datapath.h:48-67). Stand-ins for the tests: a connection table and a
// static SNAT table filled by the harness (walk_harness.c), with grout's
// signatures and private data; in grout the nodes use the real ones.
typedef enum {
	CONN_FLOW_FWD = 0,
	CONN_FLOW_REV,
} conn_flow_t;

struct conn_key {
	uint16_t iface_id;
	addr_family_t af;
	uint8_t proto;
	ip4_addr_t src;
	ip4_addr_t dst;
	rte_be16_t src_id;
	rte_be16_t dst_id;
};

struct conn {
	struct conn_key fwd_key;
	struct conn_key rev_key;
};

GR_MBUF_PRIV_DATA_TYPE(conn_mbuf_data, {
	struct conn *conn;
	conn_flow_t flow;
});

bool gr_conn_parse_key(const struct iface *, const addr_family_t, const struct rte_mbuf *, struct conn_key *);
struct conn *gr_conn_lookup(const struct conn_key *, conn_flow_t *);

typedef enum {
	NAT_VERDICT_CONTINUE,
	NAT_VERDICT_FINAL,
	NAT_VERDICT_DROP,
} nat_verdict_t;

// grout's snat44_process is static inline (nat_datapath.h:57): so is this,
// over the stand-in's static rules
nat_verdict_t gr_standin_snat44_process(const struct iface *, struct rte_mbuf *);
static inline nat_verdict_t snat44_process(const struct iface *iface, struct rte_mbuf *mbuf) {
	return gr_standin_snat44_process(iface, mbuf);
}

// Test tables behind the stand-ins (0 or -ENOSPC).
int gr_test_conn_add(const struct conn_key *fwd, const struct conn_key *rev, struct conn **out);
int gr_test_snat44_static_add(uint16_t iface_id, ip4_addr_t from, ip4_addr_t to);
void gr_test_policy_clear(void);

static inline bool gr_mbuf_is_traced(struct rte_mbuf *m) {
	return !STAILQ_EMPTY(&mbuf_data(m)->traces);
}

// ---- nodes -----------------------------------------------------------------
#define GR_NODE_CTX_TYPE(type_name, fields)                                                        \
	struct type_name fields;                                                                   \
	static inline struct type_name *type_name(struct rte_node *node) {                         \
		_Static_assert(sizeof(struct type_name) <= RTE_NODE_CTX_SZ, #type_name);           \
		return (struct type_name *)node->ctx;                                              \
	}

typedef void (*gr_node_register_cb_t)(void);

typedef enum {
	GR_NODE_T_CONTROL = 1 << 0,
	GR_NODE_T_L1 = 1 << 1,
	GR_NODE_T_L2 = 1 << 2,
	GR_NODE_T_L3 = 1 << 3,
	GR_NODE_T_L4 = 1 << 4,
} gr_node_type_t;

struct gr_node_info {
	struct rte_node_register *node;
	gr_node_type_t type;
	gr_node_register_cb_t register_callback;
	gr_node_register_cb_t unregister_callback;
	STAILQ_ENTRY(gr_node_info) next;
};

STAILQ_HEAD(node_infos, gr_node_info);
extern struct node_infos node_infos;

#define GR_NODE_REGISTER(info)                                                                     \
	RTE_INIT(gr_node_register_##info) {                                                        \
		STAILQ_INSERT_TAIL(&node_infos, &info, next);                                      \
	}

uint16_t drop_packets(struct rte_graph *, struct rte_node *, void **, uint16_t);

#define GR_DROP_REGISTER(node_name)                                                                \
	static struct rte_node_register drop_node_##node_name = {                                  \
		.name = #node_name,                                                                \
		.process = drop_packets,                                                           \
	};                                                                                         \
	static struct gr_node_info drop_info_##node_name = {                                       \
		.node = &drop_node_##node_name,                                                    \
	};                                                                                         \
	RTE_INIT(gr_drop_register_##node_name) {                                                   \
		STAILQ_INSERT_TAIL(&node_infos, &drop_info_##node_name, next);                     \
	}

// Add `node` as a next node of `parent`; returns the new edge (graph.c:35-63).
// Aborts when the parent does not exist, as grout does.
rte_edge_t gr_node_attach_parent(const char *parent, const char *node);

// graph_init's registration pass (graph.c:652-688): register every node of
// node_infos with rte_graph, then run their register callbacks. 0 or -errno.
int gr_nodes_register(void);

// ---- datapath hooks ----------------------------------------------------------
// What integration/grout-gpu_fwd4-datapath.patch adds to grout's
// modules/infra/datapath/datapath.h and main_loop.c: a module whose nodes hold
// packets across graph walks, or count for nodes that do not run themselves,
// registers hooks (at constructor time, before the "rcu" module's init) that
// gr_datapath_loop calls. Without such a module grout runs as before.
typedef void (*gr_node_stats_cb_t)(void *cookie, uint32_t node_id, uint64_t packets, uint64_t calls);

struct gr_datapath_hooks {
	const char *name;
	// QSBR reader ids the module's nodes use above the workers' lcore ids;
	// rcu_base, the first of them, is set by gr_datapath_hooks_register
	uint32_t rcu_readers;
	uint32_t rcu_base;
	// the worker is about to leave `graph` (reconfiguration, shutdown): hand
	// back through the graph what its nodes hold. Returns the mbufs that went
	// to a drop node instead (counted there), or -errno.
	int (*graph_leave)(struct rte_graph *graph);
	// the housekeeping tick, after rte_graph's own counters: cb once per node
	// with what it counted since the last tick
	int (*stats_flush)(const struct rte_graph *graph, unsigned lcore_id, gr_node_stats_cb_t cb, void *cookie);
	// what the module's nodes still hold in `graph` (packets accumulating or
	// on a device, and QSBR readers of theirs online), read at the
	// housekeeping tick: while it is not 0 the worker neither sleeps nor
	// blocks on RX interrupts
	uint64_t (*holding)(const struct rte_graph *graph);
	STAILQ_ENTRY(gr_datapath_hooks) next;
};

void gr_datapath_hooks_register(struct gr_datapath_hooks *);
// The QSBR reader ids the hooks registered (the patched rcu_init sizes its
// variable for RTE_MAX_LCORE + this).
uint32_t gr_datapath_hooks_readers(void);
// What the patched gr_datapath_loop does, for the harness's worker loop:
// every hook's graph_leave (the sum of their returns, the first -errno wins),
// every hook's stats_flush.
int gr_datapath_hooks_graph_leave(struct rte_graph *graph);
void gr_datapath_hooks_stats_flush(const struct rte_graph *graph, unsigned lcore_id, gr_node_stats_cb_t cb,
				   void *cookie);
// every hook's holding, summed (the patched loop's `held`)
uint64_t gr_datapath_hooks_holding(const struct rte_graph *graph);

// ---- modules ---------------------------------------------------------------
struct event_base;

struct module {
	const char *name;
	const char *depends_on;
	void (*init)(struct event_base *);
	void (*fini)(struct event_base *);
	STAILQ_ENTRY(module) next;
};

void module_register(struct module *);
// Run the registered modules' init (dependencies first) / fini (reverse).
int gr_modules_init(struct event_base *);
void gr_modules_fini(struct event_base *);

#ifdef __cplusplus
}
#endif
