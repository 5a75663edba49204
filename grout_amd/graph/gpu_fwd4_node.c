// SPDX-License-Identifier: BSD-3-Clause
//
// gpu_fwd4_node.c -- the grout node that puts the MI355X fast path into
// grout's graph. It is registered as "iface_input", so
// port_rx's IFACE_INPUT edge (modules/infra/datapath/port_rx.c:17-20) lands
// on it, and its next nodes are the verdict edges of enum gr_hip_edge (the
// terminal edges of iface_input .. iface_output) in
// enum order. grout's stock iface_input stays registered as
// "iface_input_cpu", the PUNT target.
//
// Per graph (one per worker, worker.c) the node keeps a walk: the mbufs of
// successive RX bursts accumulate until a batch is full, an RX burst comes
// back short (the queue drained: latency matters more than batching) or the
// oldest packet has waited max_delay; then gr_hip_node_process() stages
// their header lines, forwards them on the GPU and hands them back, and each
// mbuf is enqueued on its verdict's edge with grout's private data for that
// edge. A source node, "gpu_fwd4_flush", flushes a walk whose packets have
// waited max_delay when no new burst arrives (rte_graph calls a node only
// when it holds objects).
//
// Built here against the rte_graph / grout stand-ins (rte_graph_min.h,
// gr_datapath_min.h); in grout it includes <gr_graph.h>, <gr_mbuf.h>,
// <gr_module.h> and the DPDK headers instead, with no other change.
#include "gpu_fwd4_node.h"

#include "gr_datapath_min.h"

#include <errno.h>
#include <stdlib.h>
#include <time.h>

static struct gpu_fwd4_conf conf = {
	.dev = 0,
	.max_ifaces = 1024,
	.max_nexthops = 1u << 17,
	.batch = 1u << 16,
	.rx_burst = 64,
	.max_delay_ns = 50000,
};
static gr_hip_ctx_t *hip_ctx;

int gpu_fwd4_configure(const struct gpu_fwd4_conf *c) {
	if (c == NULL || c->batch == 0 || c->rx_burst == 0 || hip_ctx != NULL)
		return -EINVAL;
	conf = *c;
	return 0;
}

gr_hip_ctx_t *gpu_fwd4_hip_ctx(void) {
	return hip_ctx;
}

// ---- module: one fast-path context per process (one GPU) -------------------
static void gpu_init(struct event_base *ev) {
	(void)ev;
	if (gr_hip_init(conf.dev, conf.max_ifaces, conf.max_nexthops, &hip_ctx) < 0)
		hip_ctx = NULL; // the node's init fails, so does graph creation
}

static void gpu_fini(struct event_base *ev) {
	(void)ev;
	if (hip_ctx != NULL)
		gr_hip_fini(hip_ctx);
	hip_ctx = NULL;
}

static struct module gpu_module = {
	.name = "gpu_fwd4",
	.init = gpu_init,
	.fini = gpu_fini,
};

RTE_INIT(gpu_module_init) {
	module_register(&gpu_module);
}

// ---- per-graph walk state ----------------------------------------------------
struct gpu_walk {
	const struct rte_graph *graph;
	gr_hip_queue_t *q;
	uint32_t n, cap;
	uint64_t first_ns; // arrival of the oldest held packet, 0 = none
	struct rte_mbuf **mbufs;
	struct gr_hip_mbuf *v;
	struct gr_hip_node_stats stats;
	uint64_t gpu_errors; // batches punted because the GPU call failed
};

#define MAX_WALKS 64
static struct gpu_walk *walks[MAX_WALKS];

static struct gpu_walk *walk_of(const struct rte_graph *g) {
	for (int i = 0; i < MAX_WALKS; i++)
		if (walks[i] != NULL && walks[i]->graph == g)
			return walks[i];
	return NULL;
}

GR_NODE_CTX_TYPE(gpu_fwd4_ctx, { struct gpu_walk *w; });

static uint64_t now_ns(void) {
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static uint8_t ck_status(uint64_t ol_flags) {
	switch (ol_flags & RTE_MBUF_F_RX_IP_CKSUM_MASK) {
	case RTE_MBUF_F_RX_IP_CKSUM_GOOD:
		return GR_HIP_CKSUM_GOOD;
	case RTE_MBUF_F_RX_IP_CKSUM_BAD:
		return GR_HIP_CKSUM_BAD;
	default: // UNKNOWN or NONE: ip_input verifies in software (ip_input.c:80-92)
		return GR_HIP_CKSUM_UNKNOWN;
	}
}

// The private data grout's chain leaves for the node behind `edge`: the iface
// everywhere; iface_input's vlan_id before eth_input; eth_input's domain and
// pre-resolved nexthop (NULL), then ip_input's / ip6_input's l3 nexthop over
// them (l3.h:9 shares the bytes, ip_input.c:156); iface_output's vlan_id for
// port_output / port_tx (iface_output.c:81-86, port_tx.c:84-118).
static void hand_back(struct rte_mbuf *m, const struct gr_hip_mbuf *v) {
	m->data_off = v->data_off; // frame bytes were rewritten in place
	m->data_len = v->data_len;
	m->pkt_len = v->pkt_len;
	m->packet_type = v->packet_type;
	const uint8_t *f = v->frame;
	const int ip6 = f[12] == 0x86 && f[13] == 0xdd;
	mbuf_data(m)->iface = iface_from_id(v->iface);
	switch (gr_hip_edge_node(v->edge, v->nh, ip6)) {
	case GR_HIP_NODE_IFACE_INPUT:
	case GR_HIP_NODE_IFACE_OUTPUT:
		iface_mbuf_data(m)->vlan_id = v->vlan_id;
		break;
	case GR_HIP_NODE_ETH_OUTPUT:
		if (v->nh)
			l3_mbuf_data(m)->nh = gr_nexthop_from_slot(v->nh);
		break;
	default: {
		struct eth_input_mbuf_data *e = eth_input_mbuf_data(m);
		e->domain = (eth_domain_t)v->domain;
		e->nh = NULL;
		if (v->nh)
			l3_mbuf_data(m)->nh = gr_nexthop_from_slot(v->nh);
		break;
	}
	}
}

static void flush(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	if (w->n == 0)
		return;
	const int r = gr_hip_node_process(w->q, w->v, w->n, conf.rx_burst, &w->stats);
	if (r < 0) {
		// the GPU could not take them (mbufs untouched): grout's CPU nodes do
		w->gpu_errors++;
		for (uint32_t i = 0; i < w->n; i++)
			rte_node_enqueue_x1(graph, node, GR_HIP_E_PUNT, w->mbufs[i]);
	} else {
		// r > 0: a kernel gave up; the packets it did not reach come back
		// as PUNT with their frames untouched, the others forwarded as usual
		if (r > 0)
			w->gpu_errors++;
		for (uint32_t i = 0; i < w->n; i++) {
			if (w->v[i].edge != GR_HIP_E_PUNT)
				hand_back(w->mbufs[i], &w->v[i]);
			rte_node_enqueue_x1(graph, node, w->v[i].edge, w->mbufs[i]);
		}
	}
	w->n = 0;
	w->first_ns = 0;
}

static uint16_t gpu_fwd4_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	struct gpu_walk *w = gpu_fwd4_ctx(node)->w;
	uint8_t walk = GR_HIP_MBUF_F_WALK; // this call is one graph walk's iface_input stream
	for (uint16_t i = 0; i < nb_objs; i++) {
		struct rte_mbuf *m = objs[i];
		if (m->nb_segs > 1 || gr_mbuf_is_traced(m)) { // grout's CPU nodes
			rte_node_enqueue_x1(graph, node, GR_HIP_E_PUNT, m);
			continue;
		}
		if (w->n == w->cap)
			flush(graph, node, w);
		const struct iface_mbuf_data *d = iface_mbuf_data(m);
		w->mbufs[w->n] = m;
		w->v[w->n++] = (struct gr_hip_mbuf) {
			.frame = rte_pktmbuf_mtod(m, void *),
			.pkt_len = rte_pktmbuf_pkt_len(m),
			.data_len = m->data_len,
			.data_off = m->data_off,
			.packet_type = m->packet_type,
			.rss = m->hash.rss,
			.iface = d->iface != NULL ? d->iface->id : 0,
			.vlan_id = d->vlan_id,
			.ck = ck_status(m->ol_flags),
			.flags = walk,
		};
		walk = 0;
	}
	if (w->n == 0)
		return nb_objs;
	const uint64_t t = now_ns();
	if (w->first_ns == 0)
		w->first_ns = t;
	if (w->n >= conf.batch || nb_objs < conf.rx_burst || t - w->first_ns >= conf.max_delay_ns)
		flush(graph, node, w);
	return nb_objs;
}

static int gpu_fwd4_init(const struct rte_graph *graph, struct rte_node *node) {
	if (hip_ctx == NULL)
		return -ENODEV;
	int slot = 0;
	while (slot < MAX_WALKS && walks[slot] != NULL)
		slot++;
	if (slot == MAX_WALKS)
		return -ENOSPC;
	struct gpu_walk *w = calloc(1, sizeof(*w));
	if (w == NULL)
		return -ENOMEM;
	w->graph = graph;
	w->cap = conf.batch + RTE_GRAPH_BURST_SIZE;
	w->mbufs = calloc(w->cap, sizeof(*w->mbufs));
	w->v = calloc(w->cap, sizeof(*w->v));
	int r = (w->mbufs == NULL || w->v == NULL) ? -ENOMEM : gr_hip_queue_create(hip_ctx, NULL, &w->q);
	if (r < 0) {
		free(w->mbufs);
		free(w->v);
		free(w);
		return r;
	}
	walks[slot] = w;
	gpu_fwd4_ctx(node)->w = w;
	return 0;
}

static void gpu_fwd4_fini(const struct rte_graph *graph, struct rte_node *node) {
	(void)node;
	for (int i = 0; i < MAX_WALKS; i++) {
		struct gpu_walk *w = walks[i];
		if (w == NULL || w->graph != graph)
			continue;
		gr_hip_queue_destroy(w->q);
		free(w->mbufs);
		free(w->v);
		free(w);
		walks[i] = NULL;
	}
}

// next_nodes in enum gr_hip_edge order (include/grout_hip.h)
#define GPU_FWD4_EDGES                                                                             \
	[GR_HIP_E_PUNT] = "iface_input_cpu",                                                       \
	[GR_HIP_E_IFACE_MODE_UNKNOWN] = "iface_mode_unknown",                                      \
	[GR_HIP_E_IFACE_INPUT_ADMIN_DOWN] = "iface_input_admin_down",                              \
	[GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN] = "iface_input_unknown_vlan",                          \
	[GR_HIP_E_XCONNECT] = "xconnect",                                                          \
	[GR_HIP_E_BRIDGE_INPUT] = "bridge_input",                                                  \
	[GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE] = "eth_input_unknown_type",                              \
	[GR_HIP_E_ETH_INPUT_INVALID_IFACE] = "eth_input_invalid_iface",                            \
	[GR_HIP_E_SNAP_INPUT] = "snap_input",                                                      \
	[GR_HIP_E_ARP_INPUT] = "arp_input",                                                        \
	[GR_HIP_E_IP6_INPUT] = "ip6_input",                                                        \
	[GR_HIP_E_LACP_INPUT] = "lacp_input",                                                      \
	[GR_HIP_E_IP_INPUT_LOCAL] = "ip_input_local",                                              \
	[GR_HIP_E_IP_INPUT_LOCAL_CT] = "ip_input_local_ct",                                        \
	[GR_HIP_E_IP_ERROR_DEST_UNREACH] = "ip_error_dest_unreach",                                \
	[GR_HIP_E_IP_INPUT_BAD_CHECKSUM] = "ip_input_bad_checksum",                                \
	[GR_HIP_E_IP_INPUT_BAD_ADDRESS] = "ip_input_bad_address",                                  \
	[GR_HIP_E_IP_INPUT_BAD_LENGTH] = "ip_input_bad_length",                                    \
	[GR_HIP_E_IP_INPUT_BAD_VERSION] = "ip_input_bad_version",                                  \
	[GR_HIP_E_IP_INPUT_OTHER_HOST] = "ip_input_other_host",                                    \
	[GR_HIP_E_IP_BLACKHOLE] = "ip_blackhole",                                                  \
	[GR_HIP_E_DNAT44_STATIC] = "dnat44_static",                                                \
	[GR_HIP_E_IP_ERROR_TTL_EXCEEDED] = "ip_error_ttl_exceeded",                                \
	[GR_HIP_E_IP_HOLD] = "ip_hold",                                                            \
	[GR_HIP_E_IP_OUTPUT_ERROR] = "ip_output_error",                                            \
	[GR_HIP_E_IP_FRAGMENT] = "ip_fragment",                                                    \
	[GR_HIP_E_IP_ERROR_FRAG_NEEDED] = "ip_error_frag_needed",                                  \
	[GR_HIP_E_SR6_OUTPUT] = "sr6_output",                                                      \
	[GR_HIP_E_XVRF] = "xvrf",                                                                  \
	[GR_HIP_E_IPIP_OUTPUT] = "ipip_output",                                                    \
	[GR_HIP_E_IP_OUTPUT_SNAT] = "ip_output_snat",                                              \
	[GR_HIP_E_ETH_OUTPUT_NO_MAC] = "eth_output_no_mac",                                        \
	[GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE] = "iface_output_inval_type",                            \
	[GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN] = "iface_output_admin_down",                            \
	[GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT] = "iface_output_vlan_no_parent",                    \
	[GR_HIP_E_BOND_OUTPUT] = "bond_output",                                                    \
	[GR_HIP_E_VXLAN_OUTPUT] = "vxlan_output",                                                  \
	[GR_HIP_E_PORT_OUTPUT] = "port_output",                                                    \
	[GR_HIP_E_IP6_INPUT_LOCAL] = "ip6_input_local",                                            \
	[GR_HIP_E_IP6_ERROR_DEST_UNREACH] = "ip6_error_dest_unreach",                              \
	[GR_HIP_E_IP6_INPUT_NOT_MEMBER] = "ip6_input_not_member",                                  \
	[GR_HIP_E_IP6_INPUT_OTHER_HOST] = "ip6_input_other_host",                                  \
	[GR_HIP_E_IP6_INPUT_BAD_VERSION] = "ip6_input_bad_version",                                \
	[GR_HIP_E_IP6_INPUT_BAD_ADDR] = "ip6_input_bad_addr",                                      \
	[GR_HIP_E_IP6_INPUT_BAD_LENGTH] = "ip6_input_bad_length",                                  \
	[GR_HIP_E_IP6_BLACKHOLE] = "ip6_blackhole",                                                \
	[GR_HIP_E_SR6_LOCAL] = "sr6_local",                                                        \
	[GR_HIP_E_IP6_ERROR_TTL_EXCEEDED] = "ip6_error_ttl_exceeded",                              \
	[GR_HIP_E_IP6_HOLD] = "ip6_hold",                                                          \
	[GR_HIP_E_IP6_OUTPUT_ERROR] = "ip6_output_error",                                          \
	[GR_HIP_E_IP6_OUTPUT_TOO_BIG] = "ip6_output_too_big",

static struct rte_node_register gpu_fwd4_node = {
	.name = "iface_input",
	.process = gpu_fwd4_process,
	.init = gpu_fwd4_init,
	.fini = gpu_fwd4_fini,
	.nb_edges = GR_HIP_E_COUNT,
	.next_nodes = {GPU_FWD4_EDGES},
};

static struct gr_node_info gpu_fwd4_info = {
	.node = &gpu_fwd4_node,
	.type = GR_NODE_T_L2,
};

GR_NODE_REGISTER(gpu_fwd4_info);

// ---- the age flush (source node) -------------------------------------------
GR_NODE_CTX_TYPE(gpu_flush_ctx, { struct gpu_walk *w; struct rte_node *fwd; });

static uint16_t gpu_flush_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	(void)objs;
	(void)nb_objs;
	struct gpu_flush_ctx *c = gpu_flush_ctx(node);
	if (c->w == NULL && (c->w = walk_of(graph)) == NULL)
		return 0;
	struct gpu_walk *w = c->w;
	if (w->n == 0 || now_ns() - w->first_ns < conf.max_delay_ns)
		return 0;
	const uint32_t n = w->n;
	flush(graph, node, w); // same edges as iface_input, same order
	return (uint16_t)(n > UINT16_MAX ? UINT16_MAX : n);
}

static struct rte_node_register gpu_flush_node = {
	.name = "gpu_fwd4_flush",
	.flags = RTE_NODE_SOURCE_F,
	.process = gpu_flush_process,
	.nb_edges = GR_HIP_E_COUNT,
	.next_nodes = {GPU_FWD4_EDGES},
};

static struct gr_node_info gpu_flush_info = {
	.node = &gpu_flush_node,
	.type = GR_NODE_T_L2,
};

GR_NODE_REGISTER(gpu_flush_info);

int gpu_fwd4_node_stats(const struct rte_graph *graph, struct gr_hip_node_stats *stats, uint64_t *gpu_errors) {
	struct gpu_walk *w = walk_of(graph);
	if (w == NULL)
		return -ENOENT;
	if (stats != NULL)
		*stats = w->stats;
	if (gpu_errors != NULL)
		*gpu_errors = w->gpu_errors;
	return 0;
}

int gpu_fwd4_queue_stats(const struct rte_graph *graph, struct gr_hip_iface_stats *stats, uint32_t max_ifaces,
			 int reset) {
	struct gpu_walk *w = walk_of(graph);
	if (w == NULL)
		return -ENOENT;
	return gr_hip_queue_stats(w->q, stats, max_ifaces, reset);
}
