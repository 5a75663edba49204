// SPDX-License-Identifier: BSD-3-Clause
//
// rte_graph_min.h -- a stand-in for the part of DPDK's rte_graph / rte_mbuf
// API that grout's datapath nodes use, so that the fast path's rte_graph
// node (gpu_fwd4_node.c) is compiled and walked here, where DPDK is not
// installed. It is not DPDK: only the names, argument
// meanings and return conventions of the calls below follow DPDK 25.11
// (lib/graph: rte_graph.h, rte_graph_worker_common.h; lib/mbuf: rte_mbuf.h),
// which grout pins (subprojects/dpdk-25.11.wrap). Against a real DPDK build
// the node source includes <rte_graph_worker.h> / <rte_mbuf.h> instead.
//
// Semantics kept from rte_graph (what grout's nodes rely on):
//   * nodes are registered process-wide (RTE_NODE_REGISTER / constructor),
//     each with a process() callback and named next nodes (edges); edges can
//     be appended later (rte_node_edge_update, grout's gr_node_attach_parent);
//   * a graph instantiates the nodes matching its patterns plus every node
//     reachable through edges, and fails if an edge names no node;
//   * rte_graph_walk() calls every source node, then every node holding
//     objects, in the order they became pending, until none is left;
//   * process(graph, node, node->objs, node->idx) runs on the node's own
//     object array, which is empty again afterwards; rte_node_enqueue_x1 /
//     rte_node_enqueue / rte_node_next_stream_move hand objects to the next
//     node (a node does not enqueue to itself, as in DPDK); per-node
//     counters count process() calls, the objects handed in (DPDK's objs /
//     calls) and the return values.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- rte_mbuf (the fields grout's fast-path nodes touch) -------------------
#define RTE_PKTMBUF_HEADROOM 128
#define RTE_MBUF_F_RX_VLAN (1ULL << 0)
#define RTE_MBUF_F_RX_IP_CKSUM_UNKNOWN 0
#define RTE_MBUF_F_RX_IP_CKSUM_BAD (1ULL << 4)
#define RTE_MBUF_F_RX_IP_CKSUM_GOOD (1ULL << 7)
#define RTE_MBUF_F_RX_IP_CKSUM_NONE ((1ULL << 4) | (1ULL << 7))
#define RTE_MBUF_F_RX_IP_CKSUM_MASK ((1ULL << 4) | (1ULL << 7))
#define RTE_PTYPE_L3_IPV4 0x00000010
#define RTE_PTYPE_L3_IPV6 0x00000040

struct rte_mempool;

struct rte_mbuf {
	void *buf_addr;
	uint64_t buf_iova;
	uint16_t data_off;
	uint16_t refcnt;
	uint16_t nb_segs;
	uint16_t port;
	uint64_t ol_flags;
	uint32_t packet_type;
	uint32_t pkt_len;
	uint16_t data_len;
	uint16_t vlan_tci;
	union {
		uint32_t rss;
	} hash;
	uint16_t vlan_tci_outer;
	uint16_t buf_len;
	uint32_t _pad0;
	struct rte_mempool *pool;
	struct rte_mbuf *next;
	uint64_t _rest[7]; // the second cache line of DPDK's mbuf
} __attribute__((aligned(64)));

_Static_assert(sizeof(struct rte_mbuf) == 128, "rte_mbuf is two cache lines");

#define rte_pktmbuf_mtod(m, t) ((t)((char *)(m)->buf_addr + (m)->data_off))
// rte_prefetch.h: into every cache level
static inline void rte_prefetch0(const volatile void *p) {
	__builtin_prefetch((const void *)p, 0, 3);
}
// rte_prefetch.h: into every cache level, for a write
static inline void rte_prefetch0_write(const void *p) {
	__builtin_prefetch(p, 1, 3);
}
// DPDK puts the mbuf back in m->pool; the stand-in's mbufs belong to the harness
static inline void rte_pktmbuf_free(struct rte_mbuf *m) {
	(void)m;
}
#define rte_pktmbuf_pkt_len(m) ((m)->pkt_len)
#define rte_pktmbuf_data_len(m) ((m)->data_len)

// grout's pools are created with a 64-byte private area (mempool.c:97)
static inline void *rte_mbuf_to_priv(struct rte_mbuf *m) {
	return (char *)m + sizeof(struct rte_mbuf);
}
#define rte_pktmbuf_mtod_offset(m, t, o) ((t)((char *)(m)->buf_addr + (m)->data_off + (o)))

// ---- lib/net (the headers the CPU continuation nodes read) -----------------
typedef uint16_t rte_be16_t;
typedef uint32_t rte_be32_t;
#define RTE_BE16(v) ((rte_be16_t)((((v) & 0xffu) << 8) | (((v) >> 8) & 0xffu)))
#define rte_be_to_cpu_16(v) RTE_BE16(v)
#define rte_cpu_to_be_16(v) RTE_BE16(v)
#define RTE_ETHER_TYPE_IPV4 0x0800
#define RTE_IPV4_HDR_DF_FLAG (1 << 14)
#define RTE_IPV4_HDR_OFFSET_MASK 0x1fff

struct rte_ether_addr {
	uint8_t addr_bytes[6];
} __attribute__((aligned(2)));

struct rte_ipv4_hdr {
	uint8_t version_ihl;
	uint8_t type_of_service;
	rte_be16_t total_length;
	rte_be16_t packet_id;
	rte_be16_t fragment_offset;
	uint8_t time_to_live;
	uint8_t next_proto_id;
	rte_be16_t hdr_checksum;
	rte_be32_t src_addr;
	rte_be32_t dst_addr;
} __attribute__((packed));

struct rte_udp_hdr {
	rte_be16_t src_port;
	rte_be16_t dst_port;
	rte_be16_t dgram_len;
	rte_be16_t dgram_cksum;
} __attribute__((packed));

static inline uint8_t rte_ipv4_hdr_len(const struct rte_ipv4_hdr *ip) {
	return (uint8_t)((ip->version_ihl & 0xf) * 4);
}

// ---- rte_graph --------------------------------------------------------------
#define RTE_GRAPH_BURST_SIZE 256
#define RTE_NODE_NAMESIZE 64
#define RTE_GRAPH_NAMESIZE 64
#define RTE_NODE_CTX_SZ 16
#define RTE_NODE_SOURCE_F (1ULL << 0)

typedef uint32_t rte_node_t;
typedef uint16_t rte_edge_t;
typedef uint16_t rte_graph_t;
#define RTE_NODE_ID_INVALID UINT32_MAX
#define RTE_EDGE_ID_INVALID UINT16_MAX
#define RTE_GRAPH_ID_INVALID UINT16_MAX

struct rte_graph;
struct rte_node;

typedef uint16_t (*rte_node_process_t)(struct rte_graph *graph, struct rte_node *node, void **objs,
				       uint16_t nb_objs);
typedef int (*rte_node_init_t)(const struct rte_graph *graph, struct rte_node *node);
typedef void (*rte_node_fini_t)(const struct rte_graph *graph, struct rte_node *node);

struct rte_node_register {
	char name[RTE_NODE_NAMESIZE];
	uint64_t flags;
	rte_node_process_t process;
	rte_node_init_t init;
	rte_node_fini_t fini;
	rte_node_t id; // set by __rte_node_register
	rte_node_t parent_id;
	rte_edge_t nb_edges;
	const char *next_nodes[];
};

// A node instance inside one graph (what process() receives).
struct rte_node {
	uint8_t ctx[RTE_NODE_CTX_SZ] __attribute__((aligned(16)));
	void *ctx_ptr;
	char name[RTE_NODE_NAMESIZE];
	rte_node_t id;
	rte_edge_t nb_edges;
	uint16_t idx; // objects held
	uint16_t size; // capacity of objs
	uint16_t pending; // in the graph's pending list
	void **objs;
	rte_node_process_t process;
	struct rte_node **nodes; // [nb_edges]: next node instances by edge
	uint64_t total_objs, total_calls, total_packets; // packets = process() returns (DPDK's objs)
	uint32_t max_idx; // most objects the node ever held (its stream's high-water mark)
};

struct rte_graph_param {
	int socket_id;
	uint16_t nb_node_patterns;
	const char **node_patterns;
};

// The fields of DPDK's struct rte_graph a node's init may read (the graph
// of a grout worker is named "gr-%04x" after (cpu_id << 1) | index,
// graph.c:118-119, and created on the worker's NUMA socket, :134-135).
struct rte_graph_priv;
struct rte_graph {
	char name[RTE_GRAPH_NAMESIZE];
	rte_graph_t id;
	int socket;
	struct rte_graph_priv *priv; // the stand-in runtime's own state
};

rte_node_t __rte_node_register(const struct rte_node_register *reg);
#define RTE_NODE_REGISTER(node)                                                                    \
	__attribute__((constructor)) static void rte_node_register_##node(void) {                  \
		node.id = __rte_node_register(&node);                                                  \
	}

rte_node_t rte_node_from_name(const char *name);
const char *rte_node_id_to_name(rte_node_t id);
rte_node_t rte_node_max_count(void);
// Append (from == RTE_EDGE_ID_INVALID) or overwrite edges from index `from`;
// returns the number of edges of the node after the update.
rte_edge_t rte_node_edge_update(rte_node_t id, rte_edge_t from, const char **next_nodes, uint16_t nb_edges);
rte_edge_t rte_node_edge_count(rte_node_t id);
// names[] (rte_node_edge_count entries, or NULL to count): the edge names.
rte_edge_t rte_node_edge_get(rte_node_t id, char *next_nodes[]);

rte_graph_t rte_graph_create(const char *name, struct rte_graph_param *prm);
int rte_graph_destroy(rte_graph_t id);
struct rte_graph *rte_graph_lookup(const char *name);
// DPDK's rte_graph_walk, rte_node_enqueue and rte_node_enqueue_x1 are static
// inline (rte_graph_worker.h, rte_graph_worker_common.h): so are these, over
// the stand-in's walk and enqueue
void rte_standin_graph_walk(struct rte_graph *graph);
static inline void rte_graph_walk(struct rte_graph *graph) {
	rte_standin_graph_walk(graph);
}
// The instance of node `name` in `graph` (NULL if absent); for counters.
struct rte_node *rte_graph_node_get_by_name(const char *graph, const char *name);

// Worker API (rte_graph_worker_common.h)
void rte_standin_node_enqueue_x1(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void *obj);
void rte_standin_node_enqueue(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void **objs,
			      uint16_t nb_objs);
static inline void rte_node_enqueue_x1(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void *obj) {
	rte_standin_node_enqueue_x1(graph, node, next, obj);
}
static inline void rte_node_enqueue(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void **objs,
				    uint16_t nb_objs) {
	rte_standin_node_enqueue(graph, node, next, objs, nb_objs);
}
void rte_node_next_stream_move(struct rte_graph *graph, struct rte_node *src, rte_edge_t next);

#define RTE_INIT(fn)                                                                               \
	__attribute__((constructor)) static void fn(void)

#ifdef __cplusplus
}
#endif
