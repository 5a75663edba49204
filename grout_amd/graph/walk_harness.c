// SPDX-License-Identifier: BSD-3-Clause
//
// walk_harness.c -- test harness (not the product): a graph around the fast
// path's grout node, for tests/test_graph_walk.py.
//
//   port_rx (source, stand-in for port_rx.c:281-316: bursts of rx_burst
//   mbufs from an injected array, iface / vlan_id in the private data)
//     -> iface_input (gpu_fwd4_node.c) -> one recorder node per verdict edge
//   gpu_fwd4_flush (source) -> the same recorder nodes
//
// Recorder nodes stand in for grout's next nodes (ip_hold, port_output, the
// drop nodes ...): they note which edge each mbuf arrived on, in order.
// mbufs are built like grout's pool (mempool.c:57-100): 128-byte rte_mbuf,
// 64-byte private area, 2048-byte data room, frame at headroom 128.
#include "gpu_fwd4_node.h"
#include "gr_datapath_min.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>

#define GH_PRIV 64
#define GH_ROOM 2048
#define GH_MBUF_SZ (sizeof(struct rte_mbuf) + GH_PRIV + GH_ROOM)

struct gh_mbuf_out { // per injected mbuf, in injection order
	uint32_t pkt_len;
	uint16_t data_len;
	uint16_t data_off;
	uint32_t packet_type;
	uint16_t iface; // mbuf_data(m)->iface->id (0 = NULL)
	uint16_t vlan_id; // iface_mbuf_data(m)->vlan_id
	uint8_t edge; // the recorder node it reached (edge index of iface_input), 0xff = none
	uint8_t domain; // eth_input_mbuf_data(m)->domain (low byte)
	uint16_t _pad;
	uint32_t nh; // l3_mbuf_data(m)->nh->slot (0 = NULL)
	uint32_t seq; // arrival order over all recorders
	uint32_t eth_nh; // eth_input_mbuf_data(m)->nh->slot (0 = NULL)
};

static struct {
	uint8_t *mem;
	uint32_t n, next_rx, recorded;
	uint32_t rx_burst;
	const struct gr_hip_pkt_meta *meta_in;
	uint8_t *edge_of; // [n]
	uint32_t *seq_of; // [n]
	struct iface *ifaces;
	struct nexthop *nhs;
	uint32_t max_ifaces, max_nh;
	rte_graph_t gid;
	struct rte_graph *graph;
	char name[RTE_GRAPH_NAMESIZE];
	int inited;
	int pin; // register the mbuf memory with the fast path (frames by address)
	void *pinned; // what is registered now
} H = {.gid = RTE_GRAPH_ID_INVALID, .pin = 1};

// Whether gh_load registers its mbuf memory with gr_hip_host_register (grout:
// the mempools' memory), so that the node hands frames over by address.
void gh_set_pin(int on) {
	H.pin = on;
}

static void unpin(void) {
	if (H.pinned != NULL && gpu_fwd4_hip_ctx() != NULL)
		gr_hip_host_unregister(gpu_fwd4_hip_ctx(), H.pinned);
	H.pinned = NULL;
}

static struct rte_mbuf *mbuf_at(uint32_t i) {
	return (struct rte_mbuf *)(H.mem + (size_t)i * GH_MBUF_SZ);
}

static uint16_t port_rx_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	(void)objs;
	(void)nb;
	uint32_t k = 0;
	void *burst[RTE_GRAPH_BURST_SIZE];
	while (k < H.rx_burst && H.next_rx < H.n) {
		const uint32_t i = H.next_rx++;
		struct rte_mbuf *m = mbuf_at(i);
		const struct gr_hip_pkt_meta *pm = &H.meta_in[i];
		struct iface_mbuf_data *d = iface_mbuf_data(m);
		d->iface = iface_from_id(pm->iface);
		d->vlan_id = pm->vlan_ck & 0xfff;
		burst[k++] = m;
	}
	rte_node_enqueue(graph, node, 0, burst, (uint16_t)k);
	return (uint16_t)k;
}

static struct rte_node_register port_rx_node = {
	.name = "port_rx",
	.flags = RTE_NODE_SOURCE_F,
	.process = port_rx_process,
	.nb_edges = 1,
	.next_nodes = {"iface_input"},
};

// a recorder's ctx holds the edge index it stands for
static uint16_t recorder_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	(void)graph;
	const uint8_t edge = node->ctx[0];
	for (uint16_t k = 0; k < nb; k++) {
		const size_t off = (uint8_t *)objs[k] - H.mem;
		const uint32_t i = (uint32_t)(off / GH_MBUF_SZ);
		if (i < H.n) {
			H.edge_of[i] = edge;
			H.seq_of[i] = H.recorded++;
		}
	}
	return nb;
}

static int recorder_init(const struct rte_graph *graph, struct rte_node *node) {
	(void)graph;
	// the recorder for edge e is named after edge e of iface_input
	rte_node_t fwd = rte_node_from_name("iface_input");
	rte_edge_t n = rte_node_edge_count(fwd);
	char **names = calloc(n, sizeof(char *));
	if (names == NULL)
		return -ENOMEM;
	rte_node_edge_get(fwd, names);
	node->ctx[0] = 0xff;
	for (rte_edge_t e = 0; e < n; e++)
		if (strcmp(names[e], node->name) == 0)
			node->ctx[0] = (uint8_t)e;
	free(names);
	return 0;
}

static int register_recorders(void) {
	rte_node_t fwd = rte_node_from_name("iface_input");
	if (fwd == RTE_NODE_ID_INVALID)
		return -ENOENT;
	rte_edge_t n = rte_node_edge_count(fwd);
	char **names = calloc(n, sizeof(char *));
	if (names == NULL)
		return -ENOMEM;
	rte_node_edge_get(fwd, names);
	for (rte_edge_t e = 0; e < n; e++) {
		if (rte_node_from_name(names[e]) != RTE_NODE_ID_INVALID)
			continue;
		struct rte_node_register *r = calloc(1, sizeof(*r));
		if (r == NULL)
			break;
		snprintf(r->name, sizeof(r->name), "%s", names[e]);
		r->process = recorder_process;
		r->init = recorder_init;
		if (__rte_node_register(r) == RTE_NODE_ID_INVALID)
			break;
	}
	free(names);
	return 0;
}

// Register the graph's nodes (port_rx, grout's node infos, the recorders)
// without touching the GPU. Idempotent.
int gh_register(void) {
	static int done;
	if (done)
		return 0;
	if (__rte_node_register(&port_rx_node) == RTE_NODE_ID_INVALID)
		return -EEXIST;
	int r;
	if ((r = gr_nodes_register()) < 0 || (r = register_recorders()) < 0)
		return r;
	done = 1;
	return 0;
}

int gh_init(int dev, uint32_t max_ifaces, uint32_t max_nh, uint32_t batch, uint32_t rx_burst,
	    uint64_t max_delay_ns) {
	if (H.inited)
		return -EALREADY;
	struct gpu_fwd4_conf c = {dev, max_ifaces, max_nh, batch, rx_burst, max_delay_ns};
	int r = gpu_fwd4_configure(&c);
	if (r < 0)
		return r;
	H.rx_burst = rx_burst > RTE_GRAPH_BURST_SIZE ? RTE_GRAPH_BURST_SIZE : rx_burst;
	H.max_ifaces = max_ifaces;
	H.max_nh = max_nh;
	H.ifaces = calloc(max_ifaces, sizeof(*H.ifaces));
	H.nhs = calloc((size_t)max_nh + 1, sizeof(*H.nhs));
	if (H.ifaces == NULL || H.nhs == NULL)
		return -ENOMEM;
	for (uint32_t i = 1; i < max_ifaces; i++) { // grout's iface / nexthop objects
		H.ifaces[i].id = (uint16_t)i;
		gr_iface_register(&H.ifaces[i]);
	}
	for (uint32_t s = 1; s <= max_nh; s++) {
		H.nhs[s].slot = s;
		gr_nexthop_register(&H.nhs[s]);
	}
	if ((r = gh_register()) < 0)
		return r;
	if ((r = gr_modules_init(NULL)) < 0)
		return r;
	H.inited = 1;
	return gpu_fwd4_hip_ctx() != NULL ? 0 : -ENODEV;
}

void *gh_hip_ctx(void) {
	return gpu_fwd4_hip_ctx();
}

// The graph of one worker: what worker_graph_new would select.
int gh_graph_create(const char *name) {
	const char *patterns[] = {"port_rx", "gpu_fwd4_flush"};
	struct rte_graph_param prm = {.socket_id = 0, .nb_node_patterns = 2, .node_patterns = patterns};
	H.gid = rte_graph_create(name, &prm);
	if (H.gid == RTE_GRAPH_ID_INVALID)
		return -EINVAL;
	H.graph = rte_graph_lookup(name);
	snprintf(H.name, sizeof(H.name), "%s", name);
	return 0;
}

int gh_graph_destroy(void) {
	if (H.gid == RTE_GRAPH_ID_INVALID)
		return -ENOENT;
	int r = rte_graph_destroy(H.gid);
	H.gid = RTE_GRAPH_ID_INVALID;
	H.graph = NULL;
	return r;
}

int gh_load(const uint8_t *frames, uint32_t stride, const struct gr_hip_pkt_meta *meta, uint32_t n) {
	if (stride > GH_ROOM - RTE_PKTMBUF_HEADROOM)
		return -EINVAL;
	unpin();
	free(H.mem);
	free(H.edge_of);
	free(H.seq_of);
	H.mem = calloc(n ? n : 1, GH_MBUF_SZ);
	H.edge_of = malloc(n ? n : 1);
	H.seq_of = calloc(n ? n : 1, sizeof(uint32_t));
	if (H.mem == NULL || H.edge_of == NULL || H.seq_of == NULL)
		return -ENOMEM;
	memset(H.edge_of, 0xff, n);
	for (uint32_t i = 0; i < n; i++) {
		struct rte_mbuf *m = mbuf_at(i);
		m->buf_addr = (uint8_t *)m + sizeof(struct rte_mbuf) + GH_PRIV;
		m->buf_len = GH_ROOM;
		m->data_off = RTE_PKTMBUF_HEADROOM;
		m->nb_segs = 1;
		m->refcnt = 1;
		m->pkt_len = meta[i].pkt_len;
		m->data_len = meta[i].pkt_len;
		m->hash.rss = meta[i].rss;
		const uint32_t ck = (meta[i].vlan_ck >> 12) & 3;
		m->ol_flags = ck == GR_HIP_CKSUM_BAD ? RTE_MBUF_F_RX_IP_CKSUM_BAD
			: ck == GR_HIP_CKSUM_GOOD    ? RTE_MBUF_F_RX_IP_CKSUM_GOOD
						     : RTE_MBUF_F_RX_IP_CKSUM_UNKNOWN;
		memcpy(rte_pktmbuf_mtod(m, uint8_t *), frames + (size_t)i * stride, stride);
	}
	H.n = n;
	H.next_rx = 0;
	H.recorded = 0;
	H.meta_in = meta;
	if (H.pin && n && gpu_fwd4_hip_ctx() != NULL) {
		int r = gr_hip_host_register(gpu_fwd4_hip_ctx(), H.mem, (size_t)n * GH_MBUF_SZ);
		if (r < 0)
			return r;
		H.pinned = H.mem;
	}
	return 0;
}

// Walk until every injected mbuf reached a recorder, at most max_walks
// times. Returns the number of walks, or -ETIMEDOUT.
int gh_run(uint32_t max_walks) {
	if (H.graph == NULL)
		return -ENOENT;
	for (uint32_t w = 1; w <= max_walks; w++) {
		rte_graph_walk(H.graph);
		if (H.recorded == H.n && H.next_rx == H.n)
			return (int)w;
	}
	return -ETIMEDOUT;
}

// The private area is a union of the nodes' views: a pointer field may hold
// another view's bytes, so decode without dereferencing. 0 = NULL,
// 0xffffffff = not one of the registered objects.
static uint32_t slot_of(const struct nexthop *nh) {
	if (nh == NULL)
		return 0;
	if (nh < H.nhs + 1 || nh > H.nhs + H.max_nh)
		return 0xffffffffu;
	return (uint32_t)(nh - H.nhs);
}

static uint32_t iface_id_of(const struct iface *i) {
	if (i == NULL)
		return 0;
	if (i < H.ifaces + 1 || i >= H.ifaces + H.max_ifaces)
		return 0xffff;
	return (uint32_t)(i - H.ifaces);
}

int gh_results(struct gh_mbuf_out *out, uint8_t *lines) {
	for (uint32_t i = 0; i < H.n; i++) {
		struct rte_mbuf *m = mbuf_at(i);
		struct gh_mbuf_out *o = &out[i];
		memset(o, 0, sizeof(*o));
		o->pkt_len = m->pkt_len;
		o->data_len = m->data_len;
		o->data_off = m->data_off;
		o->packet_type = m->packet_type;
		o->iface = (uint16_t)iface_id_of(mbuf_data(m)->iface);
		o->vlan_id = iface_mbuf_data(m)->vlan_id;
		o->edge = H.edge_of[i];
		o->domain = (uint8_t)eth_input_mbuf_data(m)->domain;
		o->nh = slot_of(l3_mbuf_data(m)->nh);
		o->eth_nh = slot_of(eth_input_mbuf_data(m)->nh);
		o->seq = H.seq_of[i];
		// the frame as port_rx delivered it: header line at the RX position
		memcpy(lines + (size_t)i * GR_HIP_LINE, (uint8_t *)m->buf_addr + RTE_PKTMBUF_HEADROOM, GR_HIP_LINE);
	}
	return (int)H.n;
}

int gh_node_stats(struct gr_hip_node_stats *stats, uint64_t *gpu_errors) {
	return H.graph ? gpu_fwd4_node_stats(H.graph, stats, gpu_errors) : -ENOENT;
}

int gh_queue_stats(struct gr_hip_iface_stats *stats, uint32_t max_ifaces, int reset) {
	return H.graph ? gpu_fwd4_queue_stats(H.graph, stats, max_ifaces, reset) : -ENOENT;
}

// rte_graph's own counters of a node of the graph (objs, calls, packets).
int gh_rte_node_counters(const char *node, uint64_t out[3]) {
	struct rte_node *n = H.graph ? rte_graph_node_get_by_name(H.name, node) : NULL;
	if (n == NULL)
		return -ENOENT;
	out[0] = n->total_objs;
	out[1] = n->total_calls;
	out[2] = n->total_packets;
	return 0;
}

void gh_fini(void) {
	unpin();
	gh_graph_destroy();
	gr_modules_fini(NULL);
	free(H.mem);
	free(H.edge_of);
	free(H.seq_of);
	H.mem = NULL;
	H.edge_of = NULL;
	H.seq_of = NULL;
	H.n = 0;
}
