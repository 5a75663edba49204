// SPDX-License-Identifier: BSD-3-Clause
//
// walk_harness.c -- test harness (not the product): worker graphs around the
// fast path's grout node, for tests/test_graph_walk.py.
//
//   port_rx (source, stand-in for port_rx.c:281-316: bursts of rx_burst
//   mbufs from an injected array, iface / vlan_id in the private data)
//     -> iface_input (gpu_fwd4_node.c) -> grout's next nodes
//   gpu_fwd4_flush (source) -> the same next nodes
//
// Every node of the graph carries a grout node name: the fast path's two
// nodes, the two CPU continuation nodes (gpu_fwd4_cpu_nodes.c:
// ip_input_local_ct, ip_output_snat), and recorders standing in for the rest
// of grout's nodes under their own names (ip_hold, port_output, eth_output,
// dnat44_dynamic, the drop nodes ... and iface_input_cpu, grout's iface_input
// renamed by integration/grout-iface_input_cpu.patch). A recorder notes
// which node each mbuf reached, in order, and keeps the mbuf.
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
#define GH_MAX_GRAPHS 8
#define GH_MAX_RECORDERS 128

struct gh_mbuf_out { // per injected mbuf, in injection order
	uint32_t pkt_len;
	uint16_t data_len;
	uint16_t data_off;
	uint32_t packet_type;
	uint16_t iface; // mbuf_data(m)->iface->id (0 = NULL)
	uint16_t vlan_id; // iface_mbuf_data(m)->vlan_id
	uint8_t edge; // the recorder it reached (gh_recorder_name), 0xff = none
	uint8_t domain; // eth_input_mbuf_data(m)->domain (low byte)
	uint16_t conn; // conn_mbuf_data(m)->conn as a table index + 1 (0 = none)
	uint32_t nh; // l3_mbuf_data(m)->nh->slot (0 = NULL)
	uint32_t seq; // arrival order over all recorders
	uint32_t eth_nh; // eth_input_mbuf_data(m)->nh->slot (0 = NULL)
	uint8_t eth_dst[6]; // eth_output_mbuf_data(m)->dst
	uint16_t eth_type; // eth_output_mbuf_data(m)->ether_type (as stored)
	uint8_t vtep_af; // eth_output_mbuf_data(m)->vtep.af
	uint8_t flow; // conn_mbuf_data(m)->flow
	uint16_t _pad;
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
	struct {
		rte_graph_t gid;
		struct rte_graph *graph;
		char name[RTE_GRAPH_NAMESIZE];
	} graphs[GH_MAX_GRAPHS];
	int cur; // the graph gh_run / gh_results / stats use
	char *recorders[GH_MAX_RECORDERS]; // recorder id -> node name
	uint32_t n_recorders;
	int inited;
	int pin; // register the mbuf memory with the fast path (frames by address)
	void *pinned; // what is registered now
} H = {.cur = -1, .pin = 1};

// Whether gh_load registers its mbuf memory with gr_hip_host_register (grout:
// the mempools' memory), so that the node hands frames over by address.
void gh_set_pin(int on) {
	H.pin = on;
}

static void unpin(void) {
	if (H.pinned != NULL && gpu_fwd4_n_ctx() != 0)
		gpu_fwd4_host_unregister(H.pinned);
	H.pinned = NULL;
}

static struct rte_mbuf *mbuf_at(uint32_t i) {
	return (struct rte_mbuf *)(H.mem + (size_t)i * GH_MBUF_SZ);
}

// Whether port_rx leaves each mbuf and frame in the CPU's caches, as a PMD
// does on a real RX: it writes the mbuf fields from the RX descriptor, and
// the NIC's DMA lands the frame in the LLC (DDIO). Off: both stay where
// gh_load left them (cold for large loads).
static int rx_touch;

void gh_set_rx_touch(int on) {
	rx_touch = on;
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
		if (rx_touch) {
			m->pkt_len = pm->pkt_len; // the PMD's descriptor fields
			m->data_len = pm->pkt_len;
			m->hash.rss = pm->rss;
			__builtin_prefetch(rte_pktmbuf_mtod(m, void *), 0, 1); // DDIO: the frame in the LLC
		}
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

// a recorder's ctx holds its recorder id
static uint16_t recorder_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	(void)graph;
	const uint8_t id = node->ctx[0];
	for (uint16_t k = 0; k < nb; k++) {
		const size_t off = (uint8_t *)objs[k] - H.mem;
		const uint32_t i = (uint32_t)(off / GH_MBUF_SZ);
		if (i < H.n) {
			H.edge_of[i] = id;
			H.seq_of[i] = H.recorded++;
		}
	}
	return nb;
}

static int recorder_init(const struct rte_graph *graph, struct rte_node *node) {
	(void)graph;
	node->ctx[0] = 0xff;
	for (uint32_t r = 0; r < H.n_recorders; r++)
		if (strcmp(H.recorders[r], node->name) == 0)
			node->ctx[0] = (uint8_t)r;
	return 0;
}

static int add_recorder(const char *name) {
	if (rte_node_from_name(name) != RTE_NODE_ID_INVALID)
		return 0;
	if (H.n_recorders == GH_MAX_RECORDERS)
		return -ENOSPC;
	struct rte_node_register *r = calloc(1, sizeof(*r));
	if (r == NULL)
		return -ENOMEM;
	snprintf(r->name, sizeof(r->name), "%s", name);
	r->process = recorder_process;
	r->init = recorder_init;
	if (__rte_node_register(r) == RTE_NODE_ID_INVALID)
		return -EINVAL;
	H.recorders[H.n_recorders++] = strdup(name);
	return 0;
}

// Recorders for every next node no registered node provides, reachable from
// the fast path's node: the ones named after its edges first (recorder id ==
// edge), then those behind the CPU continuation nodes.
static int register_recorders(void) {
	const char *roots[] = {"iface_input", "ip_input_local_ct", "ip_output_snat"};
	for (unsigned k = 0; k < sizeof(roots) / sizeof(roots[0]); k++) {
		rte_node_t id = rte_node_from_name(roots[k]);
		if (id == RTE_NODE_ID_INVALID)
			return -ENOENT;
		rte_edge_t n = rte_node_edge_count(id);
		char **names = calloc(n, sizeof(char *));
		if (names == NULL)
			return -ENOMEM;
		rte_node_edge_get(id, names);
		for (rte_edge_t e = 0; e < n; e++) {
			if (k == 0 && rte_node_from_name(names[e]) != RTE_NODE_ID_INVALID && H.n_recorders == e) {
				// a real node at this edge (the CPU continuation nodes): keep
				// recorder ids equal to edge ids with a placeholder
				H.recorders[H.n_recorders++] = strdup(names[e]);
				continue;
			}
			int r = add_recorder(names[e]);
			if (r < 0) {
				free(names);
				return r;
			}
		}
		free(names);
	}
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

const char *gh_recorder_name(uint32_t id) {
	return id < H.n_recorders ? H.recorders[id] : NULL;
}

// devs[n_devs]: the GPUs the module opens (n_devs 0: all).
int gh_init(const int *devs, uint32_t n_devs, uint32_t max_ifaces, uint32_t max_nh, uint32_t batch,
	    uint32_t rx_burst, uint64_t max_delay_ns) {
	if (H.inited)
		return -EALREADY;
	struct gpu_fwd4_conf c = {.n_devs = n_devs, .max_ifaces = max_ifaces, .max_nexthops = max_nh,
				  .batch = batch, .rx_burst = rx_burst, .max_delay_ns = max_delay_ns};
	if (n_devs > GPU_FWD4_MAX_DEVS)
		return -EINVAL;
	for (uint32_t i = 0; i < n_devs; i++)
		c.devs[i] = devs[i];
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
	return gpu_fwd4_n_ctx() != 0 ? 0 : -ENODEV;
}

void *gh_hip_ctx(void) {
	return gpu_fwd4_hip_ctx();
}

void *gh_ctx_at(uint32_t i) {
	return gpu_fwd4_ctx_at(i);
}

uint32_t gh_n_ctx(void) {
	return gpu_fwd4_n_ctx();
}

// grout's control plane objects the CPU continuation nodes read (the type,
// flags and L3 nexthop info the GPU mirrors hold as well).
int gh_set_objects(const struct gr_hip_iface *ifs, uint32_t n_if, const struct gr_hip_nh *nhs, uint32_t first,
		   uint32_t n_nh) {
	if (H.ifaces == NULL)
		return -ENODEV;
	for (uint32_t k = 0; k < n_if; k++) {
		const struct gr_hip_iface *s = &ifs[k];
		if (s->id == 0 || s->id >= H.max_ifaces)
			return -EINVAL;
		struct iface *d = &H.ifaces[s->id];
		d->type = s->type;
		d->mode = s->mode;
		d->flags = s->flags;
		d->mtu = s->mtu;
		d->vrf_id = s->vrf_id;
	}
	for (uint32_t k = 0; k < n_nh; k++) {
		const uint32_t slot = first + k;
		if (slot == 0 || slot > H.max_nh)
			return -EINVAL;
		const struct gr_hip_nh *s = &nhs[k];
		struct nexthop *d = &H.nhs[slot];
		d->type = s->type;
		d->iface_id = s->iface_id;
		d->vrf_id = s->vrf_id;
		d->l3.state = s->state;
		d->l3.flags = s->flags;
		d->l3.af = s->af;
		d->l3.ipv4 = s->ipv4;
		memcpy(d->l3.ipv6, s->ipv6, 16);
		memcpy(d->l3.mac.addr_bytes, s->mac, 6);
	}
	return 0;
}

// The conntrack / SNAT stand-ins' tables (gr_datapath_min.h).
int gh_conn_add(const struct conn_key *fwd, const struct conn_key *rev) {
	return gr_test_conn_add(fwd, rev, NULL);
}

int gh_snat44_static_add(uint16_t iface_id, uint32_t from, uint32_t to) {
	return gr_test_snat44_static_add(iface_id, from, to);
}

void gh_policy_clear(void) {
	gr_test_policy_clear();
}

// One worker's graph: what worker_graph_new selects (graph.c:93-145), named
// after the worker's CPU like grout's ("gr-%04x", (cpu << 1) | index) and
// created on `socket`. It becomes the current graph.
int gh_graph_create(unsigned cpu, int socket) {
	int k = 0;
	while (k < GH_MAX_GRAPHS && H.graphs[k].graph != NULL)
		k++;
	if (k == GH_MAX_GRAPHS)
		return -ENOSPC;
	char name[RTE_GRAPH_NAMESIZE];
	snprintf(name, sizeof(name), "gr-%04x", (cpu << 1) & 0xffff);
	const char *patterns[] = {"port_rx", "gpu_fwd4_flush"};
	struct rte_graph_param prm = {.socket_id = socket, .nb_node_patterns = 2, .node_patterns = patterns};
	rte_graph_t gid = rte_graph_create(name, &prm);
	if (gid == RTE_GRAPH_ID_INVALID)
		return -EINVAL;
	H.graphs[k].gid = gid;
	H.graphs[k].graph = rte_graph_lookup(name);
	snprintf(H.graphs[k].name, sizeof(H.graphs[k].name), "%s", name);
	H.cur = k;
	return k;
}

int gh_graph_use(int k) {
	if (k < 0 || k >= GH_MAX_GRAPHS || H.graphs[k].graph == NULL)
		return -ENOENT;
	H.cur = k;
	return 0;
}

// The GPU context index the current graph's node runs on.
int gh_graph_gpu(void) {
	return H.cur >= 0 ? gpu_fwd4_graph_gpu(H.graphs[H.cur].graph) : -ENOENT;
}

static struct rte_graph *cur_graph(void) {
	return H.cur >= 0 ? H.graphs[H.cur].graph : NULL;
}

int gh_graph_destroy(void) {
	if (H.cur < 0 || H.graphs[H.cur].graph == NULL)
		return -ENOENT;
	int r = rte_graph_destroy(H.graphs[H.cur].gid);
	H.graphs[H.cur].graph = NULL;
	H.cur = -1;
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
	if (H.pin && n && gpu_fwd4_n_ctx() != 0) {
		int r = gpu_fwd4_host_register(H.mem, (size_t)n * GH_MBUF_SZ);
		if (r < 0)
			return r;
		H.pinned = H.mem;
	}
	return 0;
}

// Walk the current graph until every injected mbuf reached a recorder, at
// most max_walks times. Returns the number of walks, or -ETIMEDOUT.
int gh_run(uint32_t max_walks) {
	struct rte_graph *g = cur_graph();
	if (g == NULL)
		return -ENOENT;
	for (uint32_t w = 1; w <= max_walks; w++) {
		rte_graph_walk(g);
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

uint32_t gr_test_conn_index(const struct conn *c); // gr_datapath_min.c

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
		const struct eth_output_mbuf_data *e = eth_output_mbuf_data(m);
		memcpy(o->eth_dst, e->dst.addr_bytes, 6);
		o->eth_type = e->ether_type;
		o->vtep_af = e->vtep.af;
		const struct conn_mbuf_data *cd = conn_mbuf_data(m);
		o->conn = (uint16_t)gr_test_conn_index(cd->conn);
		o->flow = (uint8_t)cd->flow;
		// the frame as port_rx delivered it: header line at the RX position
		memcpy(lines + (size_t)i * GR_HIP_LINE, (uint8_t *)m->buf_addr + RTE_PKTMBUF_HEADROOM, GR_HIP_LINE);
	}
	return (int)H.n;
}

int gh_node_stats(struct gr_hip_node_stats *stats, uint64_t *gpu_errors) {
	struct rte_graph *g = cur_graph();
	return g ? gpu_fwd4_node_stats(g, stats, gpu_errors) : -ENOENT;
}

int gh_queue_stats(struct gr_hip_iface_stats *stats, uint32_t max_ifaces, int reset) {
	struct rte_graph *g = cur_graph();
	return g ? gpu_fwd4_queue_stats(g, stats, max_ifaces, reset) : -ENOENT;
}

// rte_graph's own counters of a node of the current graph (objs, calls, packets).
int gh_rte_node_counters(const char *node, uint64_t out[3]) {
	struct rte_node *n = H.cur >= 0 ? rte_graph_node_get_by_name(H.graphs[H.cur].name, node) : NULL;
	if (n == NULL)
		return -ENOENT;
	out[0] = n->total_objs;
	out[1] = n->total_calls;
	out[2] = n->total_packets;
	return 0;
}

void gh_fini(void) {
	unpin();
	for (int k = 0; k < GH_MAX_GRAPHS; k++) {
		if (H.graphs[k].graph != NULL) {
			rte_graph_destroy(H.graphs[k].gid);
			H.graphs[k].graph = NULL;
		}
	}
	H.cur = -1;
	gr_modules_fini(NULL);
	free(H.mem);
	free(H.edge_of);
	free(H.seq_of);
	H.mem = NULL;
	H.edge_of = NULL;
	H.seq_of = NULL;
	H.n = 0;
}
