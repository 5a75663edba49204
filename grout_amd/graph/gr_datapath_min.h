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
//   modules                 main/module.h:45-53 (struct module, module_register)
//
// The objects grout's nodes dereference (struct iface, struct nexthop) are
// reduced to what the GPU node needs to hand packets back: an id and a
// nexthop slot. Everything here is written for this repo; in grout the node
// includes grout's real headers instead.
#pragma once

#include "rte_graph_min.h"

#include <stdbool.h>
#include <sys/queue.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- objects ---------------------------------------------------------------
struct iface {
	uint16_t id;
	uint16_t vrf_id;
};

struct nexthop {
	uint32_t slot; // the dense index the device FIB holds
};

// Registries the control plane fills (grout: iface.c / nexthop.c pools).
const struct iface *iface_from_id(uint16_t id);
void gr_iface_register(struct iface *);
const struct nexthop *gr_nexthop_from_slot(uint32_t slot);
void gr_nexthop_register(struct nexthop *);

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
	uint8_t family;
	uint8_t addr[16];
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
