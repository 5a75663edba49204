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
// The objects grout's nodes dereference (struct iface, struct nexthop) are
// reduced to what the GPU node needs to hand packets back: an id and a
// nexthop slot. Everything here is written for this repo; in grout the node
// includes grout's real headers instead.
#pragma once

#include "rte_graph_min.h"
#include "rte_rcu_min.h"

#include <grout_hip.h>
#include <stdbool.h>
#include <sys/queue.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- objects ---------------------------------------------------------------
// gr_iface_type_t / gr_iface_flags_t (gr_infra.h:18-38), gr_nh_* and
// addr_family_t (gr_nexthop.h:12-40, gr_net_types.h): grout's values.
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
#define GR_IFACE_F_UP GR_HIP_IFACE_F_UP
#define GR_IFACE_F_SNAT_STATIC GR_HIP_IFACE_F_SNAT_STATIC
#define GR_IFACE_F_SNAT_DYNAMIC GR_HIP_IFACE_F_SNAT_DYNAMIC
typedef uint8_t addr_family_t;
#define GR_AF_UNSPEC GR_HIP_AF_UNSPEC
#define GR_AF_IP4 GR_HIP_AF_IP4
#define GR_AF_IP6 GR_HIP_AF_IP6
typedef uint8_t gr_nh_type_t;
#define GR_NH_T_L3 GR_HIP_NH_T_L3
#define GR_NH_S_REACHABLE GR_HIP_NH_S_REACHABLE
#define GR_NH_F_LOCAL GR_HIP_NH_F_LOCAL
#define GR_NH_F_LINK GR_HIP_NH_F_LINK
typedef uint32_t ip4_addr_t; // network order

struct iface {
	uint16_t id;
	gr_iface_type_t type;
	uint8_t mode;
	uint16_t flags;
	uint16_t mtu;
	uint16_t vrf_id;
};

// nexthop_info_l3 (nexthop.h:41-54 over gr_nexthop.h:93-105)
struct nexthop_info_l3 {
	uint8_t state;
	uint8_t flags;
	addr_family_t af;
	ip4_addr_t ipv4;
	uint8_t ipv6[16];
	struct rte_ether_addr mac;
};

struct nexthop {
	uint32_t slot; // the dense index the device FIB holds
	gr_nh_type_t type;
	uint16_t iface_id;
	uint16_t vrf_id;
	struct nexthop_info_l3 l3;
};

static inline const struct nexthop_info_l3 *nexthop_info_l3(const struct nexthop *nh) {
	return &nh->l3;
}

// grout's iface registry (iface.c:459-466: ifaces[id], cleared by
// iface_destroy before its RCU synchronisation, :710-712). The nexthop
// objects the fast path names by slot are the node's own registry
// (gpu_fwd4_nh_obj_set), not grout's.
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
// (:408); the fast path's node registers GPU_FWD4_RCU_READERS more
// (gpu_fwd4_node.h, sized in by integration/grout-gpu_fwd4-datapath.patch).
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

nat_verdict_t snat44_process(const struct iface *, struct rte_mbuf *);

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
