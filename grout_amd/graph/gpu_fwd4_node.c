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
// The module opens one fast-path context per configured GPU (all visible
// ones by default). Each worker graph binds to one of them at creation,
// NUMA-aware (pick_gpu); the control plane applies every change to all of
// them (gpu_fwd4_iface_set ... below, FANOUT).
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
#include <string.h>
#include <time.h>

static struct gpu_fwd4_conf conf = {
	.n_devs = 0, // every visible device
	.max_ifaces = 1024,
	.max_nexthops = 1u << 17,
	.batch = 1u << 16,
	.rx_burst = 64,
	.max_delay_ns = 50000,
};

// One fast-path context per GPU; the worker graphs are spread over them.
static struct {
	gr_hip_ctx_t *ctx;
	int dev;
	int numa; // the device's NUMA node
	uint32_t graphs; // worker graphs bound to it
} gpus[GPU_FWD4_MAX_DEVS];
static uint32_t n_gpus;

int gpu_fwd4_configure(const struct gpu_fwd4_conf *c) {
	if (c == NULL || c->batch == 0 || c->rx_burst == 0 || c->n_devs > GPU_FWD4_MAX_DEVS || n_gpus != 0)
		return -EINVAL;
	conf = *c;
	return 0;
}

gr_hip_ctx_t *gpu_fwd4_hip_ctx(void) {
	return n_gpus ? gpus[0].ctx : NULL;
}

uint32_t gpu_fwd4_n_ctx(void) {
	return n_gpus;
}

gr_hip_ctx_t *gpu_fwd4_ctx_at(uint32_t i) {
	return i < n_gpus ? gpus[i].ctx : NULL;
}

// ---- module: one fast-path context per configured device -------------------
static void gpu_fini(struct event_base *ev);

static void gpu_init(struct event_base *ev) {
	(void)ev;
	int devs[GPU_FWD4_MAX_DEVS];
	uint32_t n = conf.n_devs;
	if (n == 0) { // every visible device
		const int count = gr_hip_device_count();
		n = count > 0 ? (uint32_t)count : 0;
		if (n > GPU_FWD4_MAX_DEVS)
			n = GPU_FWD4_MAX_DEVS;
		for (uint32_t i = 0; i < n; i++)
			devs[i] = (int)i;
	} else {
		memcpy(devs, conf.devs, n * sizeof(devs[0]));
	}
	for (uint32_t i = 0; i < n; i++) {
		gr_hip_ctx_t *c = NULL;
		if (gr_hip_init(devs[i], conf.max_ifaces, conf.max_nexthops, &c) < 0) {
			gpu_fini(NULL); // all or nothing: the nodes' init then fails
			return;
		}
		const int numa = gr_hip_device_numa_node(devs[i]);
		gpus[n_gpus].ctx = c;
		gpus[n_gpus].dev = devs[i];
		gpus[n_gpus].numa = numa < 0 ? 0 : numa;
		gpus[n_gpus].graphs = 0;
		n_gpus++;
	}
}

static void gpu_fini(struct event_base *ev) {
	(void)ev;
	while (n_gpus > 0)
		gr_hip_fini(gpus[--n_gpus].ctx);
}

static struct module gpu_module = {
	.name = "gpu_fwd4",
	.init = gpu_init,
	.fini = gpu_fini,
};

RTE_INIT(gpu_module_init) {
	module_register(&gpu_module);
}

// The GPU a worker graph runs on: one on the graph's NUMA socket (any GPU if
// none is), the one with the fewest graphs, lowest first -- the policy of
// grout's RX queue distribution over workers (worker.c:424-481): round robin
// over the CPUs of the port's socket.
static int pick_gpu(const struct rte_graph *graph) {
	int best = -1;
	for (int pass = 0; pass < 2 && best < 0; pass++) {
		for (uint32_t i = 0; i < n_gpus; i++) {
			if (pass == 0 && gpus[i].numa != graph->socket)
				continue;
			if (best < 0 || gpus[i].graphs < gpus[best].graphs)
				best = (int)i;
		}
	}
	return best;
}

// ---- per-graph walk state ----------------------------------------------------
struct gpu_walk {
	const struct rte_graph *graph;
	int gpu; // index in gpus[]
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
	if (n_gpus == 0)
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
	w->gpu = pick_gpu(graph);
	w->cap = conf.batch + RTE_GRAPH_BURST_SIZE;
	w->mbufs = calloc(w->cap, sizeof(*w->mbufs));
	w->v = calloc(w->cap, sizeof(*w->v));
	int r = (w->mbufs == NULL || w->v == NULL) ? -ENOMEM : gr_hip_queue_create(gpus[w->gpu].ctx, NULL, &w->q);
	if (r < 0) {
		free(w->mbufs);
		free(w->v);
		free(w);
		return r;
	}
	gpus[w->gpu].graphs++;
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
		if ((uint32_t)w->gpu < n_gpus && gpus[w->gpu].graphs > 0)
			gpus[w->gpu].graphs--;
		free(w->mbufs);
		free(w->v);
		free(w);
		walks[i] = NULL;
	}
}

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

int gpu_fwd4_graph_gpu(const struct rte_graph *graph) {
	struct gpu_walk *w = walk_of(graph);
	return w == NULL ? -ENOENT : w->gpu;
}

// ---- control plane: every change goes to every GPU's context ---------------
// (grout's control thread calls these from its event handlers, INTEGRATION.md
// §3; each context is updated under its own quiesce, so a GPU's in-flight
// walks see the old or the new state, never a mix.) The first error is
// returned; the other contexts still get the change.
#define FANOUT(call)                                                                               \
	do {                                                                                       \
		int ret__ = n_gpus ? 0 : -ENODEV;                                                  \
		for (uint32_t i = 0; i < n_gpus; i++) {                                            \
			gr_hip_ctx_t *ctx = gpus[i].ctx;                                           \
			const int r__ = (call);                                                    \
			if (r__ < 0 && ret__ == 0)                                                 \
				ret__ = r__;                                                       \
		}                                                                                  \
		return ret__;                                                                      \
	} while (0)

int gpu_fwd4_iface_set(const struct gr_hip_iface *ifaces, uint32_t n) {
	FANOUT(gr_hip_iface_set(ctx, ifaces, n));
}
int gpu_fwd4_iface_del(uint16_t iface_id) {
	FANOUT(gr_hip_iface_del(ctx, iface_id));
}
int gpu_fwd4_nh_set(uint32_t first_slot, const struct gr_hip_nh *nh, uint32_t n) {
	FANOUT(gr_hip_nh_set(ctx, first_slot, nh, n));
}
int gpu_fwd4_reta_set(uint32_t first, const uint32_t *slots, uint32_t n) {
	FANOUT(gr_hip_reta_set(ctx, first, slots, n));
}
int gpu_fwd4_fib4_create(uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8) {
	FANOUT(gr_hip_fib4_create(ctx, vrf_id, max_routes, num_tbl8));
}
int gpu_fwd4_fib4_destroy(uint16_t vrf_id) {
	FANOUT(gr_hip_fib4_destroy(ctx, vrf_id));
}
int gpu_fwd4_route4_add(const struct gr_hip_route4 *routes, uint32_t n, int replace) {
	FANOUT(gr_hip_route4_add(ctx, routes, n, replace));
}
int gpu_fwd4_route4_del(uint16_t vrf_id, uint32_t ip, uint8_t prefixlen) {
	FANOUT(gr_hip_route4_del(ctx, vrf_id, ip, prefixlen));
}
int gpu_fwd4_fib4_commit(uint16_t vrf_id) {
	FANOUT(gr_hip_fib4_commit(ctx, vrf_id));
}
int gpu_fwd4_fib6_create(uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8) {
	FANOUT(gr_hip_fib6_create(ctx, vrf_id, max_routes, num_tbl8));
}
int gpu_fwd4_fib6_destroy(uint16_t vrf_id) {
	FANOUT(gr_hip_fib6_destroy(ctx, vrf_id));
}
int gpu_fwd4_route6_add(const struct gr_hip_route6 *routes, uint32_t n, int replace) {
	FANOUT(gr_hip_route6_add(ctx, routes, n, replace));
}
int gpu_fwd4_route6_del(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen) {
	FANOUT(gr_hip_route6_del(ctx, vrf_id, iface_id, ip, prefixlen));
}
int gpu_fwd4_fib6_commit(uint16_t vrf_id) {
	FANOUT(gr_hip_fib6_commit(ctx, vrf_id));
}
int gpu_fwd4_edges_set(int table, uint16_t key, uint8_t edge) {
	switch (table) {
	case GR_HIP_EDGES_ETH_TYPE:
		FANOUT(gr_hip_edges_eth_type(ctx, key, edge));
	case GR_HIP_EDGES_IFACE_MODE:
		FANOUT(gr_hip_edges_iface_mode(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP_INPUT_NH_TYPE:
		FANOUT(gr_hip_edges_ip_input_nh_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP_OUTPUT_NH_TYPE:
		FANOUT(gr_hip_edges_ip_output_nh_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP_OUTPUT_IFACE_TYPE:
		FANOUT(gr_hip_edges_ip_output_iface_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IFACE_OUTPUT_TYPE:
		FANOUT(gr_hip_edges_iface_output_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP6_INPUT_NH_TYPE:
		FANOUT(gr_hip_edges_ip6_input_nh_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP6_OUTPUT_NH_TYPE:
		FANOUT(gr_hip_edges_ip6_output_nh_type(ctx, (uint8_t)key, edge));
	case GR_HIP_EDGES_IP6_OUTPUT_IFACE_TYPE:
		FANOUT(gr_hip_edges_ip6_output_iface_type(ctx, (uint8_t)key, edge));
	default:
		return -EINVAL;
	}
}
int gpu_fwd4_tune(const char *key, int value) {
	FANOUT(gr_hip_tune(ctx, key, value));
}
int gpu_fwd4_host_register(void *ptr, size_t bytes) {
	FANOUT(gr_hip_host_register(ctx, ptr, bytes));
}
int gpu_fwd4_host_unregister(void *ptr) {
	FANOUT(gr_hip_host_unregister(ctx, ptr));
}
