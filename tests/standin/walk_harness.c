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
#define _GNU_SOURCE // pthread_setaffinity_np, CPU_SET

#include "gpu_fwd4_control.h"
#include "gpu_fwd4_node.h"
#include "gr_control_min.h"
#include "gr_datapath_min.h"

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <sys/mman.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#define GH_PRIV 64
#define GH_ROOM 2048
#define GH_MBUF_SZ (sizeof(struct rte_mbuf) + GH_PRIV + GH_ROOM)
#define GH_MAX_GRAPHS 40
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
	uint8_t *mem; // the mbufs (mbuf_mem_alloc)
	void *mem_map;
	size_t mem_len;
	uint32_t n, next_rx, recorded;
	uint32_t rx_burst;
	const struct gr_hip_pkt_meta *meta_in;
	uint8_t *edge_of; // [n]
	uint32_t *seq_of; // [n]
	struct iface *ifaces;
	struct nexthop *nhs;
	uint32_t max_ifaces, max_nh;
	struct {
		_Alignas(128) rte_graph_t gid; // each worker's on lines of its own
		struct rte_graph *graph;
		char name[RTE_GRAPH_NAMESIZE];
		// the worker's node statistics as grout's housekeeping keeps them
		// (struct worker_stats node_stats, main_loop.c:40-66), by node id,
		// and the rte_graph counters already folded in
		uint64_t *w_packets, *w_batches, *prev_packets, *prev_calls;
		// workers mode (gh_workers_run): this graph's share of the injected
		// mbufs [rx_next, rx_end) and what reached its recorders
		uint32_t rx_next, rx_end;
		uint64_t recorded;
		// recycle mode: the worker's mempool, a stack of free mbuf indices;
		// rx_next .. rx_end count the passes over its share rx_start + [0, share)
		uint32_t *free_mb, n_free;
		uint32_t rx_start, share;
		// latency mode: the worker's histogram of TSC cycles from port_rx to a recorder
		uint64_t *lat;
	} graphs[GH_MAX_GRAPHS];
	const uint8_t *frames_in; // gh_load's stream (recycle mode refills the mbufs from it)
	uint32_t stride_in;
	uint32_t recycle; // workers mode: mbufs per worker's pool (0: every packet its own mbuf)
	uint32_t passes; // recycle mode: times each worker goes over its share of the stream
	int workers; // gh_workers_run is walking every graph from its own thread
	uint32_t wk0; // gh_workers_run's worker k walks graph slot wk0 + k
	int lcores[GH_MAX_GRAPHS], n_lcores; // workers mode: worker k pinned to lcores[k] (k < n_lcores)
	uint32_t loop; // walks since the last housekeeping tick (main_loop.c:461)
	uint8_t *if_dead, *nh_dead; // objects the RCU test's control thread freed
	uint32_t freed_reads; // grout nodes behind the edges read a freed object
	uint32_t rec_ip_hold; // recorder id of ip_hold (reads l3_mbuf_data.nh, ip_hold.c:25)
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

// Measurement: port_rx hands its bursts straight to port_output, past the
// node (the harness's own cost per packet, without the fast path).
static int null_node;

void gh_set_null_node(int on) {
	null_node = on;
}

// Workers mode: each worker's packets through a pool of `pool` mbufs of its
// own, refilled from the loaded stream as they come back from the recorders
// (a mempool and its per-lcore cache), instead of one mbuf per packet, going
// `passes` times over its share of the stream. pool 0: off.
void gh_set_recycle(uint32_t pool, uint32_t passes) {
	H.recycle = pool;
	H.passes = passes ? passes : 1;
}

// Workers mode: worker k walks graph slot slot0 + k (e.g. the chain graphs
// created after the GPU node's).
int gh_workers_first(uint32_t slot0) {
	if (slot0 >= GH_MAX_GRAPHS)
		return -EINVAL;
	H.wk0 = slot0;
	return 0;
}

// Workers mode: worker k pinned to cpus[k], as grout pins each worker to its
// lcore. n 0: the scheduler places them.
int gh_set_lcores(const int *cpus, int n) {
	if (n < 0 || n > GH_MAX_GRAPHS)
		return -EINVAL;
	for (int k = 0; k < n; k++) {
		if (cpus[k] < 0 || cpus[k] >= CPU_SETSIZE)
			return -EINVAL;
		H.lcores[k] = cpus[k];
	}
	H.n_lcores = n;
	return 0;
}

// ---- latency: each packet's time from port_rx to the recorder behind its edge
// Workers mode with gh_set_latency(1): port_rx stamps every mbuf of a burst
// with one TSC read (in the mbuf's second cache line, where DPDK keeps its
// dynamic fields, e.g. the RX timestamp), the recorders read the TSC once per
// call and count each packet's cycles in the worker's log histogram:
// GH_LAT_SUB buckets per power of two. Off by default: the throughput runs
// pay none of it.
#define GH_LAT_SUB 16
#define GH_LAT_BUCKETS (64 * GH_LAT_SUB)
static int lat_on;
static double tsc_per_ns; // measured over the last gh_workers_run

static inline uint64_t tsc(void) {
	return __builtin_ia32_rdtsc();
}

static inline unsigned lat_bucket(uint64_t d) {
	if (d < GH_LAT_SUB)
		return (unsigned)d;
	const unsigned e = 63u - (unsigned)__builtin_clzll(d); // >= 4
	return e * GH_LAT_SUB + (unsigned)((d >> (e - 4)) & (GH_LAT_SUB - 1));
}

void gh_set_latency(int on) {
	lat_on = on;
}

// The bucket's lower edge, in cycles (for the test's percentiles).
uint64_t gh_lat_bucket_floor(uint32_t b) {
	if (b < GH_LAT_SUB)
		return b;
	const unsigned e = b / GH_LAT_SUB, f = b % GH_LAT_SUB;
	return (1ull << e) | ((uint64_t)f << (e - 4));
}

static uint16_t port_rx_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	(void)objs;
	(void)nb;
	uint32_t k = 0;
	void *burst[RTE_GRAPH_BURST_SIZE];
	const uint64_t stamp = lat_on ? tsc() : 0;
	// workers mode: each graph polls its own part of the mbufs (its RX queue)
	uint32_t *next = &H.next_rx, end = H.n;
	if (H.workers && node->ctx[0] != 0) {
		next = &H.graphs[node->ctx[0] - 1].rx_next;
		end = H.graphs[node->ctx[0] - 1].rx_end;
	}
	if (H.workers && H.recycle && node->ctx[0] != 0) {
		// recycle mode: each packet of the worker's share of the stream into
		// an mbuf of its pool, as a PMD refills its RX ring from a mempool
		// (the NIC's DMA writes the frame, DDIO lands it in the LLC)
		__typeof__(&H.graphs[0]) G = &H.graphs[node->ctx[0] - 1];
		while (k < H.rx_burst && G->rx_next < G->rx_end && G->n_free > 0) {
			const uint32_t i = G->rx_start + (G->rx_next++ - G->rx_start) % G->share;
			struct rte_mbuf *m = mbuf_at(G->free_mb[--G->n_free]);
			const struct gr_hip_pkt_meta *pm = &H.meta_in[i];
			m->data_off = RTE_PKTMBUF_HEADROOM;
			m->pkt_len = pm->pkt_len;
			m->data_len = pm->pkt_len;
			m->packet_type = 0;
			m->hash.rss = pm->rss;
			const uint32_t ck = (pm->vlan_ck >> 12) & 3;
			m->ol_flags = ck == GR_HIP_CKSUM_BAD ? RTE_MBUF_F_RX_IP_CKSUM_BAD
				: ck == GR_HIP_CKSUM_GOOD    ? RTE_MBUF_F_RX_IP_CKSUM_GOOD
							     : RTE_MBUF_F_RX_IP_CKSUM_UNKNOWN;
			memcpy(rte_pktmbuf_mtod(m, uint8_t *), H.frames_in + (size_t)i * H.stride_in, H.stride_in);
			struct iface_mbuf_data *d = iface_mbuf_data(m);
			d->iface = iface_from_id(pm->iface);
			d->vlan_id = pm->vlan_ck & 0xfff;
			if (lat_on)
				m->_rest[0] = stamp;
			burst[k++] = m;
		}
		rte_node_enqueue(graph, node, null_node ? 1 : 0, burst, (uint16_t)k);
		return (uint16_t)k;
	}
	while (k < H.rx_burst && *next < end) {
		const uint32_t i = (*next)++;
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
		if (lat_on)
			m->_rest[0] = stamp;
		burst[k++] = m;
	}
	rte_node_enqueue(graph, node, null_node ? 1 : 0, burst, (uint16_t)k);
	return (uint16_t)k;
}

// ctx[0]: the harness slot of the node's graph + 1 (0: not one of them)
static int graph_slot_init(const struct rte_graph *graph, struct rte_node *node) {
	node->ctx[0] = 0;
	for (int k = 0; k < GH_MAX_GRAPHS; k++)
		if (strcmp(graph->name, H.graphs[k].name) == 0)
			node->ctx[0] = (uint8_t)(k + 1);
	return 0;
}

static struct rte_node_register port_rx_node = {
	.name = "port_rx",
	.flags = RTE_NODE_SOURCE_F,
	.init = graph_slot_init,
	.process = port_rx_process,
	.nb_edges = 2,
	.next_nodes = {"iface_input", "port_output"},
};

// ---- grout's CPU chain in the same harness (like-for-like measurement) -----
// A "chain" graph (gh_graph_create_chain) is the GPU node's worker graph with
// grout's own node chain in its place: port_rx_chain (port_rx's code, the same
// mempools, lcores and recorders) hands its bursts to cpu_chain, which runs
// the oracle's restatement of grout's nodes iface_input .. iface_output
// (or_walk_frames, reached through the pointer gh_set_chain is given: this
// library links nothing of the oracle) on the mbufs in place, writes grout's
// mbuf fields and private data for each packet's edge as grout's nodes leave
// them, and enqueues runs of one edge on the same edges as the GPU node.
// Test infrastructure only (tests/perf_node_chain.py).
typedef int (*gh_chain_fn)(const void *topo, uint8_t *const *frames, uint32_t readable,
			   const struct gr_hip_pkt_meta *meta, uint16_t n, struct gr_hip_mbuf *mo);
static gh_chain_fn chain_fn;
static const void *chain_topo;

void gh_set_chain(void *fn, const void *topo) {
	chain_fn = (gh_chain_fn)fn;
	chain_topo = topo;
}

#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wmaybe-uninitialized" // frames / meta: filled for every i < nb
static uint16_t cpu_chain_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	uint8_t *frames[RTE_GRAPH_BURST_SIZE];
	struct gr_hip_pkt_meta meta[RTE_GRAPH_BURST_SIZE];
	struct gr_hip_mbuf mo[RTE_GRAPH_BURST_SIZE];
	uint8_t edge[RTE_GRAPH_BURST_SIZE];
	if (nb == 0)
		return 0;
	if (chain_fn == NULL) {
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, objs, nb);
		return nb;
	}
	for (uint16_t i = 0; i < nb; i++) { // what grout's nodes read of each mbuf
		struct rte_mbuf *m = objs[i];
		const struct iface_mbuf_data *d = iface_mbuf_data(m);
		const uint64_t ck = m->ol_flags & RTE_MBUF_F_RX_IP_CKSUM_MASK;
		frames[i] = rte_pktmbuf_mtod(m, uint8_t *);
		meta[i].iface = d->iface != NULL ? d->iface->id : 0;
		meta[i].pkt_len = (uint16_t)m->pkt_len;
		meta[i].rss = m->hash.rss;
		meta[i].vlan_ck = (uint16_t)((d->vlan_id & 0xfff)
			| ((ck == RTE_MBUF_F_RX_IP_CKSUM_GOOD ? GR_HIP_CKSUM_GOOD
			    : ck == RTE_MBUF_F_RX_IP_CKSUM_BAD ? GR_HIP_CKSUM_BAD : GR_HIP_CKSUM_UNKNOWN) << 12));
	}
	chain_fn(chain_topo, frames, GH_ROOM - RTE_PKTMBUF_HEADROOM, meta, nb, mo);
	for (uint16_t i = 0; i < nb; i++) { // grout's mbuf fields and private data at the edge
		struct rte_mbuf *m = objs[i];
		const struct gr_hip_mbuf *o = &mo[i];
		edge[i] = o->edge;
		if (o->edge == GR_HIP_E_PUNT)
			continue;
		m->data_off = (uint16_t)(m->data_off + o->data_off - RTE_PKTMBUF_HEADROOM);
		m->data_len = o->data_len;
		m->pkt_len = o->pkt_len;
		m->packet_type = o->packet_type;
		struct iface_mbuf_data *d = iface_mbuf_data(m);
		d->iface = iface_from_id(o->iface);
		if (o->edge == GR_HIP_E_PORT_OUTPUT)
			d->vlan_id = o->vlan_id; // iface_output's, for port_tx
		else if (o->nh != 0)
			l3_mbuf_data(m)->nh = o->nh <= H.max_nh ? &H.nhs[o->nh] : NULL;
		else
			eth_input_mbuf_data(m)->domain = o->domain;
	}
	for (uint16_t i = 1, run = 0; i <= nb; i++) {
		if (i == nb || edge[i] != edge[run]) {
			rte_node_enqueue(graph, node, edge[run], &objs[run], (uint16_t)(i - run));
			run = i;
		}
	}
	return nb;
}

#pragma GCC diagnostic pop

static struct rte_node_register cpu_chain_node = {
	.name = "cpu_chain",
	.process = cpu_chain_process,
	.nb_edges = GR_HIP_E_COUNT,
	.next_nodes = {GPU_FWD4_EDGES},
};

static struct rte_node_register port_rx_chain_node = {
	.name = "port_rx_chain",
	.flags = RTE_NODE_SOURCE_F,
	.init = graph_slot_init,
	.process = port_rx_process,
	.nb_edges = 2,
	.next_nodes = {"cpu_chain", "port_output"},
};

// a recorder's ctx holds its recorder id
static uint16_t recorder_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb) {
	(void)graph;
	const uint8_t id = node->ctx[0];
	if (H.workers) { // a rate measurement: grout's node behind the edge takes the mbufs, no record
		if (node->ctx[1] != 0) {
			__typeof__(&H.graphs[0]) G = &H.graphs[node->ctx[1] - 1];
			G->recorded += nb;
			if (lat_on && G->lat != NULL) {
				const uint64_t now = tsc();
				for (uint16_t k = 0; k < nb; k++)
					G->lat[lat_bucket(now - ((struct rte_mbuf *)objs[k])->_rest[0])]++;
			}
			if (H.recycle) // back to the worker's mempool (port_tx's completion, a drop node's free)
				for (uint16_t k = 0; k < nb; k++)
					G->free_mb[G->n_free++] = (uint32_t)(((uint8_t *)objs[k] - H.mem) / GH_MBUF_SZ);
		}
		return nb;
	}
	for (uint16_t k = 0; k < nb; k++) {
		const size_t off = (uint8_t *)objs[k] - H.mem;
		const uint32_t i = (uint32_t)(off / GH_MBUF_SZ);
		struct rte_mbuf *m = objs[k];
		// what grout's node here would dereference: the iface everywhere,
		// ip_hold's nexthop; neither may have been freed (RCU)
		const struct iface *ifp = mbuf_data(m)->iface;
		if (ifp != NULL && ifp >= H.ifaces && ifp < H.ifaces + H.max_ifaces && H.if_dead[ifp - H.ifaces])
			__atomic_fetch_add(&H.freed_reads, 1, __ATOMIC_RELAXED);
		if (id == H.rec_ip_hold) {
			const struct nexthop *nh = l3_mbuf_data(m)->nh;
			if (nh != NULL && nh >= H.nhs && nh <= H.nhs + H.max_nh && H.nh_dead[nh - H.nhs])
				__atomic_fetch_add(&H.freed_reads, 1, __ATOMIC_RELAXED);
		}
		if (i < H.n) {
			H.edge_of[i] = id;
			__atomic_store_n(&H.seq_of[i], __atomic_fetch_add(&H.recorded, 1, __ATOMIC_ACQ_REL), __ATOMIC_RELAXED);
		}
	}
	return nb;
}

static int recorder_init(const struct rte_graph *graph, struct rte_node *node) {
	graph_slot_init(graph, node);
	node->ctx[1] = node->ctx[0];
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
	H.rec_ip_hold = GR_HIP_E_IP_HOLD;
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

// grout's nodes the fast path replaces: they stay in every worker graph
// (graph_init puts every registered node in base_node_names, graph.c:652-688;
// worker_graph_new selects them all, :130), idle, and grout's statistics
// report them under their names (gpu_fwd4_stats_flush). Stand-ins here.
static const char *const replaced[] = {"eth_input", "ip_input", "ip_forward", "ip_output", "eth_output",
				       "iface_output", "ip6_input", "ip6_forward", "ip6_output"};
#define N_REPLACED (sizeof(replaced) / sizeof(replaced[0]))

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
	// the chain graphs' nodes (after the recorders: cpu_chain's edges are theirs)
	if (__rte_node_register(&cpu_chain_node) == RTE_NODE_ID_INVALID
	    || __rte_node_register(&port_rx_chain_node) == RTE_NODE_ID_INVALID)
		return -EEXIST;
	for (unsigned k = 0; k < N_REPLACED; k++)
		if ((r = add_recorder(replaced[k])) < 0)
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
	H.if_dead = calloc(max_ifaces, 1);
	H.nh_dead = calloc((size_t)max_nh + 1, 1);
	if (H.ifaces == NULL || H.nhs == NULL || H.if_dead == NULL || H.nh_dead == NULL)
		return -ENOMEM;
	if ((r = gh_register()) < 0)
		return r;
	if ((r = gr_modules_init(gr_test_event_base())) < 0)
		return r;
	// grout's iface / nexthop objects, in grout's iface table and in the
	// node's registries (the control plane's object events)
	for (uint32_t i = 1; i < max_ifaces; i++) {
		H.ifaces[i].id = (uint16_t)i;
		gr_iface_register(&H.ifaces[i]);
		if ((r = gpu_fwd4_iface_obj_set((uint16_t)i, &H.ifaces[i])) < 0)
			return r;
	}
	for (uint32_t s = 1; s <= max_nh; s++) {
		if ((r = gpu_fwd4_nh_obj_set(s, &H.nhs[s])) < 0)
			return r;
	}
	// this thread is the worker of every graph: lcore 0, a QSBR reader
	// online from its first graph on (main_loop.c:408,441)
	gr_test_lcore_set(0);
	if (gr_datapath_rcu() == NULL || rte_rcu_qsbr_thread_register(gr_datapath_rcu(), 0) < 0)
		return -ENODEV;
	rte_rcu_qsbr_thread_online(gr_datapath_rcu(), 0);
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
		struct nexthop_info_l3 *l3 = nexthop_info_l3(d);
		d->type = s->type;
		d->iface_id = s->iface_id;
		d->vrf_id = s->vrf_id;
		l3->state = s->state;
		l3->flags = s->flags;
		l3->af = s->af;
		if (s->af == GR_AF_IP6)
			memcpy(l3->ipv6, s->ipv6, 16);
		else
			l3->ipv4 = s->ipv4;
		memcpy(l3->mac.addr_bytes, s->mac, 6);
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
static int graph_create(unsigned cpu, unsigned index, int socket);
static int graph_chain; // the next graph_create makes a chain graph

int gh_graph_create(unsigned cpu, int socket) {
	return graph_create(cpu, 0, socket);
}

// A worker graph with grout's CPU chain in place of the GPU node (see
// cpu_chain above); the other index of the worker's names.
int gh_graph_create_chain(unsigned cpu, int socket) {
	graph_chain = 1;
	const int k = graph_create(cpu, 1, socket);
	graph_chain = 0;
	return k;
}

// grout names a worker's graphs "gr-%04x" with (cpu << 1) | index, the index
// alternating at each reconfiguration (worker_graph_reload, graph.c:263-290)
static int graph_create(unsigned cpu, unsigned index, int socket) {
	int k = 0;
	while (k < GH_MAX_GRAPHS && H.graphs[k].graph != NULL)
		k++;
	if (k == GH_MAX_GRAPHS)
		return -ENOSPC;
	char name[RTE_GRAPH_NAMESIZE];
	snprintf(name, sizeof(name), "gr-%04x", ((cpu << 1) | (index & 1)) & 0xffff);
	const char *patterns[2 + N_REPLACED] = {graph_chain ? "port_rx_chain" : "port_rx",
						graph_chain ? "cpu_chain" : "gpu_fwd4_flush"};
	for (unsigned i = 0; i < N_REPLACED; i++)
		patterns[2 + i] = replaced[i];
	struct rte_graph_param prm = {
		.socket_id = socket, .nb_node_patterns = 2 + N_REPLACED, .node_patterns = patterns};
	snprintf(H.graphs[k].name, sizeof(H.graphs[k].name), "%s", name); // the nodes' init look it up
	rte_graph_t gid = rte_graph_create(name, &prm);
	if (gid == RTE_GRAPH_ID_INVALID) {
		H.graphs[k].name[0] = 0;
		return -EINVAL;
	}
	H.graphs[k].gid = gid;
	H.graphs[k].graph = rte_graph_lookup(name);
	const size_t nn = rte_node_max_count() + 1;
	H.graphs[k].w_packets = calloc(nn, sizeof(uint64_t));
	H.graphs[k].w_batches = calloc(nn, sizeof(uint64_t));
	H.graphs[k].prev_packets = calloc(nn, sizeof(uint64_t));
	H.graphs[k].prev_calls = calloc(nn, sizeof(uint64_t));
	if (H.graphs[k].w_packets == NULL || H.graphs[k].w_batches == NULL || H.graphs[k].prev_packets == NULL
	    || H.graphs[k].prev_calls == NULL)
		return -ENOMEM;
	H.cur = k;
	return k;
}

static void graph_stats_free(int k) {
	H.graphs[k].name[0] = 0;
	free(H.graphs[k].w_packets);
	free(H.graphs[k].w_batches);
	free(H.graphs[k].prev_packets);
	free(H.graphs[k].prev_calls);
	H.graphs[k].w_packets = H.graphs[k].w_batches = H.graphs[k].prev_packets = H.graphs[k].prev_calls = NULL;
}

// port_rx's burst (1..256), and the node's (gpu_fwd4_set_rx_burst).
int gh_set_rx_burst(uint32_t rx_burst) {
	int r = gpu_fwd4_set_rx_burst(rx_burst);
	if (r == 0)
		H.rx_burst = rx_burst;
	return r;
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
	graph_stats_free(H.cur);
	H.cur = -1;
	return r;
}

// The mbufs' memory. DPDK's mempools live in hugepages (EAL), so the
// stand-in's mbufs are on transparent huge pages: 2 MiB aligned, madvised,
// zeroed (a page per mbuf would add a TLB miss per packet no grout worker
// has).
static void mbuf_mem_free(void) {
	if (H.mem_map != NULL)
		munmap(H.mem_map, H.mem_len);
	H.mem_map = NULL;
	H.mem = NULL;
	H.mem_len = 0;
}

static int mbuf_mem_alloc(size_t bytes) {
	const size_t huge = (size_t)2 << 20;
	const size_t len = ((bytes + huge - 1) & ~(huge - 1)) + huge;
	void *p = mmap(NULL, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (p == MAP_FAILED)
		return -ENOMEM;
	uint8_t *a = (uint8_t *)(((uintptr_t)p + huge - 1) & ~(uintptr_t)(huge - 1));
	(void)madvise(a, len - (size_t)(a - (uint8_t *)p), MADV_HUGEPAGE); // best effort
	H.mem_map = p;
	H.mem_len = len;
	H.mem = a;
	return 0;
}

int gh_load(const uint8_t *frames, uint32_t stride, const struct gr_hip_pkt_meta *meta, uint32_t n) {
	if (stride > GH_ROOM - RTE_PKTMBUF_HEADROOM)
		return -EINVAL;
	unpin();
	mbuf_mem_free();
	free(H.edge_of);
	free(H.seq_of);
	H.edge_of = malloc(n ? n : 1);
	H.seq_of = calloc(n ? n : 1, sizeof(uint32_t));
	if (mbuf_mem_alloc((size_t)(n ? n : 1) * GH_MBUF_SZ) < 0 || H.edge_of == NULL || H.seq_of == NULL)
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
	H.frames_in = frames; // the caller keeps it while it walks (recycle mode)
	H.stride_in = stride;
	if (H.pin && n && gpu_fwd4_n_ctx() != 0) {
		int r = gpu_fwd4_host_register(H.mem, (size_t)n * GH_MBUF_SZ);
		if (r < 0)
			return r;
		H.pinned = H.mem;
	}
	return 0;
}

// grout's housekeeping tick for the current graph, as main_loop.c does it
// every 256 walks (:461-475) with integration/grout-gpu_fwd4-datapath.patch:
// the QSBR quiescent report, rte_graph's per-node counters folded into the
// worker's node statistics (node_stats_callback, :40-66: packets = DPDK's
// objs, the sum of process() returns; batches = calls), then every datapath
// hook's stats_flush (the fast path module's: its counters for the nodes it
// replaced and for the ifaces).
static uint64_t window_count; // the tick's ctx.last_count: packets any node counted in the window

static void gpu_node_stat(void *cookie, uint32_t node_id, uint64_t packets, uint64_t calls) {
	const int k = (int)(intptr_t)cookie;
	H.graphs[k].w_packets[node_id] += packets;
	H.graphs[k].w_batches[node_id] += calls;
	window_count += packets; // hook_node_stats: ctx->last_count += packets
}

// Returns what grout's tick finds in ctx.last_count: the packets the graph's
// nodes (and the hooks, for the nodes they replaced) counted in the window.
static uint64_t housekeeping(int k) {
	rte_rcu_qsbr_quiescent(gr_datapath_rcu(), rte_lcore_id());
	window_count = 0;
	const rte_node_t nn = rte_node_max_count();
	for (rte_node_t id = 0; id < nn; id++) {
		struct rte_node *n = rte_graph_node_get_by_name(H.graphs[k].name, rte_node_id_to_name(id));
		if (n == NULL)
			continue;
		H.graphs[k].w_packets[id] += n->total_packets - H.graphs[k].prev_packets[id];
		H.graphs[k].w_batches[id] += n->total_calls - H.graphs[k].prev_calls[id];
		window_count += n->total_packets - H.graphs[k].prev_packets[id];
		H.graphs[k].prev_packets[id] = n->total_packets;
		H.graphs[k].prev_calls[id] = n->total_calls;
	}
	gr_datapath_hooks_stats_flush(H.graphs[k].graph, rte_lcore_id(), gpu_node_stat, (void *)(intptr_t)k);
	return window_count;
}

static void walk_once(int k) {
	rte_graph_walk(H.graphs[k].graph);
	if (++H.loop == 256) { // HOUSEKEEPING_INTERVAL
		H.loop = 0;
		housekeeping(k);
	}
}

// The worker while grout's control thread works (control_harness.c): one
// walk of the current graph (nothing injected is left: the flush node runs,
// the QSBR readers of the batches handed back go offline) and a quiescent
// report, as gr_datapath_loop does between bursts (main_loop.c:441-464).
void gh_walk_idle(void) {
	if (H.cur >= 0 && H.graphs[H.cur].graph != NULL)
		walk_once(H.cur);
	if (H.inited && gr_datapath_rcu() != NULL)
		rte_rcu_qsbr_quiescent(gr_datapath_rcu(), rte_lcore_id());
}

int gh_inited(void) {
	return H.inited;
}

// The harness's own objects out of grout's iface table and the node's
// registries (a test that builds its objects through grout's control plane
// instead, control_harness.c), and back.
void gh_objects_clear(void) {
	for (uint32_t i = 1; i < H.max_ifaces; i++) {
		gr_iface_unregister((uint16_t)i);
		gpu_fwd4_iface_obj_set((uint16_t)i, NULL);
	}
	for (uint32_t s = 1; s <= H.max_nh; s++)
		gpu_fwd4_nh_obj_set(s, NULL);
}

void gh_objects_restore(void) {
	for (uint32_t i = 1; i < H.max_ifaces; i++) {
		gr_iface_register(&H.ifaces[i]);
		gpu_fwd4_iface_obj_set((uint16_t)i, &H.ifaces[i]);
	}
	for (uint32_t s = 1; s <= H.max_nh; s++)
		gpu_fwd4_nh_obj_set(s, &H.nhs[s]);
}

// Walk the current graph until every injected mbuf reached a recorder, at
// most max_walks times, the way gr_datapath_loop does (housekeeping every
// 256 walks), then one housekeeping tick so that the statistics are whole.
// Returns the number of walks, or -ETIMEDOUT.
int gh_run(uint32_t max_walks) {
	struct rte_graph *g = cur_graph();
	if (g == NULL)
		return -ENOENT;
	for (uint32_t w = 1; w <= max_walks; w++) {
		walk_once(H.cur);
		if (__atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE) == H.n && H.next_rx == H.n) {
			housekeeping(H.cur);
			return (int)w;
		}
	}
	return -ETIMEDOUT;
}

// The worker's node statistics of the current graph for node `name`, as
// worker_dump_stats reports them (worker.c:502-560): out[0] packets,
// out[1] batches.
int gh_worker_stats(const char *name, uint64_t out[2]) {
	if (H.cur < 0)
		return -ENOENT;
	const rte_node_t id = rte_node_from_name(name);
	if (id == RTE_NODE_ID_INVALID || rte_graph_node_get_by_name(H.graphs[H.cur].name, name) == NULL)
		return -ENOENT;
	out[0] = H.graphs[H.cur].w_packets[id];
	out[1] = H.graphs[H.cur].w_batches[id];
	return 0;
}

// `grcli interface stats` for iface `id`: the per-lcore counters summed the
// way iface_stats_get does (modules/infra/api/stats.c:197-222).
int gh_iface_stats(uint16_t id, struct gr_hip_iface_stats *out) {
	if (id >= H.max_ifaces || out == NULL)
		return -EINVAL;
	memset(out, 0, sizeof(*out));
	for (int l = 0; l < RTE_MAX_LCORE; l++) {
		const struct iface_stats *st = iface_get_stats((uint16_t)l, id);
		out->rx_packets += st->rx_packets;
		out->rx_bytes += st->rx_bytes;
		out->tx_packets += st->tx_packets;
		out->tx_bytes += st->tx_bytes;
	}
	return 0;
}

// Zero the grout-side statistics (iface_stats of every lcore, the current
// graph's worker node statistics).
void gh_stats_reset(void) {
	for (uint32_t i = 0; i < H.max_ifaces; i++)
		for (int l = 0; l < RTE_MAX_LCORE; l++)
			memset(iface_get_stats((uint16_t)l, (uint16_t)i), 0, sizeof(struct iface_stats));
	if (H.cur >= 0) {
		const size_t nn = rte_node_max_count() + 1;
		memset(H.graphs[H.cur].w_packets, 0, nn * sizeof(uint64_t));
		memset(H.graphs[H.cur].w_batches, 0, nn * sizeof(uint64_t));
	}
}

int gh_walk_info(struct gpu_fwd4_walk_info *info) {
	struct rte_graph *g = cur_graph();
	return g ? gpu_fwd4_walk_info(g, info) : -ENOENT;
}

// gpu_fwd4_node_stats of graph slot k.
int gh_node_stats_at(int k, struct gr_hip_node_stats *stats, uint64_t *gpu_errors) {
	if (k < 0 || k >= GH_MAX_GRAPHS || H.graphs[k].graph == NULL)
		return -ENOENT;
	return gpu_fwd4_node_stats(H.graphs[k].graph, stats, gpu_errors);
}

// The same for graph slot k (workers mode: worker k's graph).
int gh_walk_info_at(int k, struct gpu_fwd4_walk_info *info) {
	if (k < 0 || k >= GH_MAX_GRAPHS || H.graphs[k].graph == NULL)
		return -ENOENT;
	return gpu_fwd4_walk_info(H.graphs[k].graph, info);
}

// ---- RCU: grout deletes an object a batch on the GPU names -----------------
struct gh_rcu_result {
	uint32_t sync_before_handback; // synchronize had returned before the hand-back
	uint32_t recorded_at_sync; // mbufs through grout's nodes when synchronize returned
	uint32_t freed_reads; // grout's nodes read a freed object
	uint32_t recorded;
	uint64_t stale; // dropped by the node: the object was gone at hand-back
	uint64_t sync_us; // synchronize's wait
	uint32_t walks;
	uint32_t sync_done;
};

static struct {
	uint32_t slot;
	uint16_t iface_id;
	uint32_t done, recorded_at_sync;
	uint64_t sync_us;
} R;

static uint64_t mono_us(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000u + (uint64_t)t.tv_nsec / 1000u;
}

// The control thread: iface_destroy / nexthop_destroy as grout orders them
// (iface.c:702-725, nexthop.c:493-518): the iface leaves grout's table, the
// nexthop its id pool; rte_rcu_qsbr_synchronize; then the events that follow
// it (GR_EVENT_IFACE_REMOVE / NEXTHOP_DELETE: the node's registries), and the
// objects are freed (marked dead here).
static void *rcu_control(void *arg) {
	(void)arg;
	if (R.iface_id)
		gr_iface_unregister(R.iface_id);
	const uint64_t t0 = mono_us();
	rte_rcu_qsbr_synchronize(gr_datapath_rcu(), RTE_QSBR_THRID_INVALID);
	R.sync_us = mono_us() - t0;
	R.recorded_at_sync = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE);
	if (R.iface_id)
		gpu_fwd4_iface_obj_set(R.iface_id, NULL);
	if (R.slot)
		gpu_fwd4_nh_obj_set(R.slot, NULL);
	if (R.iface_id)
		H.if_dead[R.iface_id] = 1;
	if (R.slot)
		H.nh_dead[R.slot] = 1;
	__atomic_store_n(&R.done, 1, __ATOMIC_RELEASE);
	return NULL;
}

// With the injected stream loaded (gh_load), walk until a batch is on the
// GPU, then delete nexthop `slot` and iface `iface_id` (0: none) from a
// control thread while the worker goes on: it reports quiescent, waits
// hold_ms, then walks until every mbuf is through and the control thread
// is done. Afterwards the objects are registered again.
int gh_rcu_delete_test(uint32_t slot, uint16_t iface_id, uint32_t hold_ms, struct gh_rcu_result *res) {
	if (H.cur < 0 || res == NULL || slot > H.max_nh || iface_id >= H.max_ifaces)
		return -EINVAL;
	memset(res, 0, sizeof(*res));
	memset(&R, 0, sizeof(R));
	R.slot = slot;
	R.iface_id = iface_id;
	H.freed_reads = 0;
	struct gpu_fwd4_walk_info info;
	struct gpu_fwd4_walk_info info0;
	gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info0);
	uint32_t w = 0;
	for (;;) { // until the stream's first batch is on the GPU
		walk_once(H.cur);
		w++;
		gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info);
		if (info.in_flight && info.batches > info0.batches)
			break;
		if (H.recorded == H.n || w > 1000000)
			return -EAGAIN;
	}
	pthread_t th;
	struct rte_rcu_qsbr *v = gr_datapath_rcu();
	const uint64_t tok0 = __atomic_load_n(&v->token, __ATOMIC_ACQUIRE);
	if (pthread_create(&th, NULL, rcu_control, NULL) != 0)
		return -EAGAIN;
	// the worker's housekeeping, once the control thread's synchronize has
	// started (a quiescent state reported before its token would not count)
	for (const uint64_t t_max = mono_us() + 1000000u;
	     __atomic_load_n(&v->token, __ATOMIC_ACQUIRE) == tok0 && mono_us() < t_max;)
		sched_yield();
	rte_rcu_qsbr_quiescent(v, rte_lcore_id());
	usleep(hold_ms * 1000u);
	res->sync_before_handback = __atomic_load_n(&R.done, __ATOMIC_ACQUIRE);
	const uint64_t t_end = mono_us() + 5000000u;
	while (mono_us() < t_end) {
		walk_once(H.cur);
		w++;
		if (__atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE) == H.n && __atomic_load_n(&R.done, __ATOMIC_ACQUIRE))
			break;
	}
	housekeeping(H.cur);
	pthread_join(th, NULL);
	gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info);
	res->recorded_at_sync = R.recorded_at_sync;
	res->freed_reads = H.freed_reads;
	res->recorded = H.recorded;
	res->stale = info.stale - info0.stale;
	res->sync_us = R.sync_us;
	res->walks = w;
	res->sync_done = R.done;
	// the objects come back for the next tests
	if (iface_id) {
		H.if_dead[iface_id] = 0;
		gr_iface_register(&H.ifaces[iface_id]);
		gpu_fwd4_iface_obj_set(iface_id, &H.ifaces[iface_id]);
	}
	if (slot) {
		H.nh_dead[slot] = 0;
		gpu_fwd4_nh_obj_set(slot, &H.nhs[slot]);
	}
	return 0;
}

// ---- grout's worker loop when RX goes quiet -----------------------------------
// gr_datapath_loop's housekeeping (main_loop.c:461-527) with the datapath
// patch: every 256 walks the tick folds the counters (ctx.last_count) and
// sums what the hooks hold; a window with neither counts as idle. Micro-sleep
// mode (max_sleep_us > 0, no adaptive IRQ): each idle window sleeps 1 us
// longer, up to max_sleep_us (port.c:833-878 sets it). Adaptive-IRQ mode:
// after two idle windows the worker arms its RX interrupts and, with no RX
// pending, takes its QSBR reader offline and blocks (adaptive_irq_wait,
// :202-314); here the block is a wait of block_ms on a control thread that
// runs rte_rcu_qsbr_synchronize meanwhile (grout's route or nexthop delete,
// route.c:764), and the test ends. The loaded stream is one burst followed by
// silence: port_rx delivers it, then nothing.
struct gh_loop_result {
	uint32_t walks; // graph walks
	uint32_t windows; // housekeeping ticks
	uint32_t sleeps; // micro-sleeps taken
	uint32_t sleeps_held; // ... of them while a hook held packets (counted with ignore_holding)
	uint32_t busy_held; // ticks busy only because a hook held packets
	uint32_t blocked; // the adaptive-IRQ stand-in blocked
	uint32_t recorded_at_block; // mbufs through grout's nodes when the worker blocked (or stopped)
	uint64_t held_at_block; // what the hooks held then
	uint32_t readers_online_at_block; // the node's QSBR readers online then
	uint32_t sync_returned; // the control thread's synchronize returned while the worker was blocked
	uint64_t sync_us;
	uint64_t elapsed_us;
	uint32_t recorded; // at the end
};

static struct {
	volatile int done;
	uint64_t us;
} LS;

static void *loop_sync(void *arg) {
	(void)arg;
	const uint64_t t0 = mono_us();
	rte_rcu_qsbr_synchronize(gr_datapath_rcu(), RTE_QSBR_THRID_INVALID);
	LS.us = mono_us() - t0;
	__atomic_store_n(&LS.done, 1, __ATOMIC_RELEASE);
	return NULL;
}

// ignore_holding: the loop as grout runs it without the holding hook (for the
// test that shows what goes wrong then). idle_windows: micro-sleep mode stops
// after that many idle ticks in a row once everything is through.
int gh_loop_test(uint32_t max_sleep_us, int adaptive_irq, int ignore_holding, uint32_t block_ms,
		 uint32_t idle_windows, uint32_t max_walks, struct gh_loop_result *res) {
	struct rte_graph *g = cur_graph();
	if (g == NULL || res == NULL)
		return -ENOENT;
	memset(res, 0, sizeof(*res));
	const uint64_t t0 = mono_us();
	uint32_t loop = 0, sleep = 0, airq_empty = 0, idle_run = 0;
	struct rte_rcu_qsbr *v = gr_datapath_rcu();
	for (uint32_t w = 0; w < max_walks; w++) {
		rte_graph_walk(g);
		res->walks++;
		if (++loop < 256)
			continue;
		loop = 0;
		res->windows++;
		const uint64_t last_count = housekeeping(H.cur);
		const uint64_t hold = gr_datapath_hooks_holding(g);
		const uint64_t held = ignore_holding ? 0 : hold;
		if (last_count == 0 && hold && !ignore_holding)
			res->busy_held++;
		if (adaptive_irq) {
			if (last_count == 0 && held == 0 && ++airq_empty >= 2) { // ADAPTIVE_IRQ_EMPTY_WINDOWS
				airq_empty = 0;
				if (H.next_rx < H.n) // rte_eth_rx_queue_count() > 0: poll on
					continue;
				// rte_rcu_qsbr_thread_offline, then the epoll wait
				struct gpu_fwd4_walk_info info;
				gpu_fwd4_walk_info(g, &info);
				res->blocked = 1;
				res->recorded_at_block = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE);
				res->held_at_block = hold;
				res->readers_online_at_block = info.readers_online;
				rte_rcu_qsbr_thread_offline(v, rte_lcore_id());
				memset(&LS, 0, sizeof(LS));
				pthread_t th;
				if (pthread_create(&th, NULL, loop_sync, NULL) != 0)
					return -EAGAIN;
				for (const uint64_t t_end = mono_us() + (uint64_t)block_ms * 1000u;
				     !__atomic_load_n(&LS.done, __ATOMIC_ACQUIRE) && mono_us() < t_end;)
					usleep(100);
				res->sync_returned = __atomic_load_n(&LS.done, __ATOMIC_ACQUIRE);
				res->sync_us = LS.us;
				// the wakeup (a reconfig kick here): back online, and the
				// node's readers (if any were left online) are released by
				// walks until the synchronize is through
				rte_rcu_qsbr_thread_online(v, rte_lcore_id());
				for (const uint64_t t_end = mono_us() + 5000000u;
				     !__atomic_load_n(&LS.done, __ATOMIC_ACQUIRE) && mono_us() < t_end;) {
					rte_graph_walk(g);
					rte_rcu_qsbr_quiescent(v, rte_lcore_id());
				}
				pthread_join(th, NULL);
				break;
			}
			if (last_count || held)
				airq_empty = 0;
		} else {
			if (last_count == 0 && held == 0 && max_sleep_us > 0) {
				sleep = sleep >= max_sleep_us ? max_sleep_us : sleep + 1;
				usleep(sleep);
				res->sleeps++;
				if (hold)
					res->sleeps_held++;
			} else {
				sleep = 0;
			}
			const int through = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE) == H.n && H.next_rx == H.n;
			idle_run = through && last_count == 0 && held == 0 ? idle_run + 1 : 0;
			if (idle_run >= idle_windows) {
				struct gpu_fwd4_walk_info info;
				gpu_fwd4_walk_info(g, &info);
				res->recorded_at_block = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE);
				res->held_at_block = hold;
				res->readers_online_at_block = info.readers_online;
				break;
			}
		}
	}
	res->elapsed_us = mono_us() - t0;
	res->recorded = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE);
	return 0;
}

// ---- a control plane churning while the worker forwards --------------------
struct gh_churn_result {
	uint32_t cycles; // delete / re-add cycles of nexthop a
	uint32_t commits;
	uint32_t freed_reads; // grout's nodes read a freed object
	uint32_t recorded;
	uint64_t stale; // dropped by the node: the object was gone at hand-back
	uint32_t walks;
	uint32_t err; // a control call failed
	// where the race window was: walks that ended with a batch on the GPU
	// between the move of the route (published) and the registry clear, and
	// between the clear and the nexthop's return
	uint32_t inflight_moved;
	uint32_t inflight_cleared;
};

static struct {
	struct gr_hip_route4 rt;
	uint32_t a, b, gap_us;
	volatile int stop, done;
	int phase; // 1: route moved and published, 2: registry entry cleared, 0: otherwise
	uint32_t cycles, commits, err;
} C;

static int route_to(uint32_t slot) {
	C.rt.nh = slot;
	int r = gpu_fwd4_route4_add(&C.rt, 1, 1);
	if (r == 0)
		r = gpu_fwd4_fib4_commit(C.rt.vrf_id);
	C.commits += r == 0;
	return r;
}

// nexthop_destroy as grout orders it, over and over: the routes leave the
// nexthop first (nexthop_routes_cleanup: here the route moves to b and is
// published), then rte_rcu_qsbr_synchronize, then NEXTHOP_DELETE clears the
// registry and the object is freed (dead); then it comes back (NEXTHOP_NEW)
// and the route returns to it.
static void *churn_control(void *arg) {
	(void)arg;
	while (!C.stop) {
		if (route_to(C.b) < 0)
			C.err++;
		__atomic_store_n(&C.phase, 1, __ATOMIC_RELEASE);
		rte_rcu_qsbr_synchronize(gr_datapath_rcu(), RTE_QSBR_THRID_INVALID);
		gpu_fwd4_nh_obj_set(C.a, NULL);
		__atomic_store_n(&H.nh_dead[C.a], 1, __ATOMIC_RELEASE);
		__atomic_store_n(&C.phase, 2, __ATOMIC_RELEASE);
		usleep(C.gap_us);
		__atomic_store_n(&C.phase, 0, __ATOMIC_RELEASE);
		__atomic_store_n(&H.nh_dead[C.a], 0, __ATOMIC_RELEASE);
		gpu_fwd4_nh_obj_set(C.a, &H.nhs[C.a]);
		if (route_to(C.a) < 0)
			C.err++;
		C.cycles++;
		usleep(C.gap_us);
	}
	__atomic_store_n(&C.done, 1, __ATOMIC_RELEASE);
	return NULL;
}

// Another worker's load on the graph's GPU during gh_churn_test: batches of
// gpu_load zeroed packets (each a whole-GPU kernel, as the ring kernel is
// persistent: ~0.1 ms at 2^22) submitted back to back on a queue of their
// own, so that the node's batches wait behind them and stay on the GPU
// across a publication and the synchronize after it, the window an RCU
// reader must cover. 0: none.
static uint32_t gpu_load;

void gh_set_gpu_load(uint32_t n) {
	gpu_load = n;
}

static void *gpu_load_thread(void *arg) {
	gr_hip_ctx_t *ctx = arg;
	gr_hip_queue_t *q = NULL;
	struct gr_hip_batch b;
	if (gr_hip_queue_create(ctx, NULL, &q) < 0)
		return NULL;
	if (gr_hip_batch_alloc(ctx, gpu_load, GR_HIP_LINE, &b) == 0) {
		while (!C.stop) {
			if (gr_hip_fwd4_submit(q, &b) < 0 || gr_hip_fwd4_submit(q, &b) < 0)
				break;
			gr_hip_queue_sync(q);
		}
		gr_hip_queue_sync(q);
		gr_hip_batch_free(ctx, &b);
	}
	gr_hip_queue_destroy(q);
	return NULL;
}

// With the injected stream loaded (gh_load) and route (ip, prefixlen, vrf)
// on nexthop a, walk the whole stream while a control thread cycles nexthop
// a out and back (churn_control), gap_us between steps. The worker reports
// quiescent every 256 walks as grout does, and also after every walk with
// quiesce_each (a worker may: QSBR allows it, main_loop.c:462-463 expects
// it once workers reclaim; the worst case for a reader held across walks).
int gh_churn_test(uint32_t ip_be, uint8_t prefixlen, uint16_t vrf_id, uint32_t a, uint32_t b, uint32_t gap_us,
		  uint32_t quiesce_each, struct gh_churn_result *res) {
	if (H.cur < 0 || res == NULL || a == 0 || b == 0 || a > H.max_nh || b > H.max_nh)
		return -EINVAL;
	memset(res, 0, sizeof(*res));
	memset(&C, 0, sizeof(C));
	C.rt = (struct gr_hip_route4) {.ip = ip_be, .prefixlen = prefixlen, .vrf_id = vrf_id, .nh = a};
	C.a = a;
	C.b = b;
	C.gap_us = gap_us;
	H.freed_reads = 0;
	struct gpu_fwd4_walk_info info0, info;
	gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info0);
	pthread_t th, lt;
	const int loaded = gpu_load != 0
		&& pthread_create(&lt, NULL, gpu_load_thread, gpu_fwd4_ctx_at((uint32_t)gpu_fwd4_graph_gpu(H.graphs[H.cur].graph)))
			== 0;
	if (pthread_create(&th, NULL, churn_control, NULL) != 0) {
		C.stop = 1;
		if (loaded)
			pthread_join(lt, NULL);
		return -EAGAIN;
	}
	uint32_t w = 0;
	const uint64_t t_end = mono_us() + 20000000u;
	// the worker walks until the stream is through and the control thread
	// has stopped: a synchronize under way waits for the node's readers,
	// which go offline only as the worker walks
	while (mono_us() < t_end && !__atomic_load_n(&C.done, __ATOMIC_ACQUIRE)) {
		walk_once(H.cur);
		w++;
		const int ph = __atomic_load_n(&C.phase, __ATOMIC_ACQUIRE);
		if (ph != 0) {
			gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info);
			if (info.in_flight)
				*(ph == 1 ? &res->inflight_moved : &res->inflight_cleared) += 1;
		}
		if (quiesce_each)
			rte_rcu_qsbr_quiescent(gr_datapath_rcu(), rte_lcore_id());
		if (__atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE) == H.n && H.next_rx == H.n)
			C.stop = 1;
	}
	C.stop = 1;
	if (!__atomic_load_n(&C.done, __ATOMIC_ACQUIRE)) { // the deadline: readers released, the thread can end
		gpu_fwd4_rcu_readers(0);
		for (uint32_t k = 0; k < 4; k++)
			walk_once(H.cur);
		C.err++;
	}
	pthread_join(th, NULL);
	if (loaded)
		pthread_join(lt, NULL);
	housekeeping(H.cur);
	gpu_fwd4_walk_info(H.graphs[H.cur].graph, &info);
	res->cycles = C.cycles;
	res->commits = C.commits;
	res->freed_reads = H.freed_reads;
	res->recorded = H.recorded;
	res->stale = info.stale - info0.stale;
	res->walks = w;
	res->err = C.err;
	H.nh_dead[a] = 0;
	gpu_fwd4_nh_obj_set(a, &H.nhs[a]);
	return 0;
}

// The private area is a union of the nodes' views: a pointer field may hold
// another view's bytes, so decode without dereferencing. 0 = NULL,
// 0xffffffff = not one of the registered objects.
static uint32_t slot_of(const struct nexthop *nh) {
	if (nh == NULL)
		return 0;
	if (nh < H.nhs + 1 || nh > H.nhs + H.max_nh) {
		// grout's nexthops (the control-plane stand-in's pool): the slot the
		// mirror gave them, looked up by address
		const uint32_t s = gpu_fwd4_control_nh_slot(nh);
		return s != 0 ? s : 0xffffffffu;
	}
	return (uint32_t)(nh - H.nhs);
}

static uint32_t iface_id_of(const struct iface *i) {
	if (i == NULL)
		return 0;
	const struct iface *c = gr_test_iface_base(); // grout's ifaces (control-plane stand-in)
	if (i >= c + 1 && i < c + GR_MAX_IFACES)
		return (uint32_t)(i - c);
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

// rte_graph's own counters of a node of the current graph (objects handed
// in, calls, process() returns, the stream's high-water mark).
int gh_rte_node_counters(const char *node, uint64_t out[4]) {
	struct rte_node *n = H.cur >= 0 ? rte_graph_node_get_by_name(H.graphs[H.cur].name, node) : NULL;
	if (n == NULL)
		return -ENOENT;
	out[0] = n->total_objs;
	out[1] = n->total_calls;
	out[2] = n->total_packets;
	out[3] = n->max_idx;
	return 0;
}

void gh_fini(void) {
	unpin();
	for (int k = 0; k < GH_MAX_GRAPHS; k++) {
		if (H.graphs[k].graph != NULL) {
			rte_graph_destroy(H.graphs[k].gid);
			H.graphs[k].graph = NULL;
			graph_stats_free(k);
		}
	}
	if (gr_datapath_rcu() != NULL)
		rte_rcu_qsbr_thread_unregister(gr_datapath_rcu(), 0);
	H.cur = -1;
	gr_modules_fini(gr_test_event_base());
	mbuf_mem_free();
	free(H.edge_of);
	free(H.seq_of);
	H.edge_of = NULL;
	H.seq_of = NULL;
	H.n = 0;
}

// ---- a graph reload while the node holds batches ---------------------------
struct gh_reload_result {
	uint32_t held; // mbufs the node held when the worker left the graph
	uint32_t in_flight; // batches it had on the GPU
	int32_t left; // the graph_leave hooks' return: mbufs the drain sent to grout's CPU nodes (-1: not called)
	uint32_t recorded; // mbufs through grout's nodes when the old graph was destroyed
	uint64_t fini_freed; // mbufs the old graph's fini freed
	int32_t graph; // the new current graph
	uint32_t rx; // mbufs port_rx had delivered by then
	uint32_t readers_online; // the node's QSBR readers online after the drain
	uint32_t held_after; // mbufs the node held after it
	uint32_t in_flight_after;
	uint32_t _pad;
};

// grout's reconfiguration of a worker (worker_graph_reload, graph.c:263-290;
// gr_datapath_loop, main_loop.c:466-470): the worker walks its graph
// `walks` times, leaves it at a housekeeping tick (with the datapath patch:
// the graph_leave hooks first, the node's gpu_fwd4_drain, when `drain`), the control plane creates the new
// graph (the other name index) and destroys the old one. The new graph is
// the current one afterwards; port_rx goes on with the injected stream.
int gh_reload_test(uint32_t walks, int drain, struct gh_reload_result *res) {
	if (H.cur < 0 || res == NULL)
		return -ENOENT;
	memset(res, 0, sizeof(*res));
	const int k = H.cur;
	for (uint32_t i = 0; i < walks; i++)
		walk_once(k);
	struct gpu_fwd4_walk_info info;
	gpu_fwd4_walk_info(H.graphs[k].graph, &info);
	res->held = info.held;
	res->in_flight = info.in_flight;
	res->left = drain ? gr_datapath_hooks_graph_leave(H.graphs[k].graph) : -1;
	gpu_fwd4_walk_info(H.graphs[k].graph, &info);
	res->readers_online = info.readers_online;
	res->held_after = info.held;
	res->in_flight_after = info.in_flight;
	housekeeping(k);
	res->recorded = __atomic_load_n(&H.recorded, __ATOMIC_ACQUIRE);
	res->rx = H.next_rx;
	unsigned index = 0;
	sscanf(H.graphs[k].name, "gr-%x", &index);
	const int nk = graph_create(index >> 1, (index & 1) ^ 1, 0);
	if (nk < 0)
		return nk;
	const uint64_t f0 = gpu_fwd4_fini_freed();
	int r = rte_graph_destroy(H.graphs[k].gid);
	H.graphs[k].graph = NULL;
	graph_stats_free(k);
	res->fini_freed = gpu_fwd4_fini_freed() - f0;
	H.cur = nk;
	res->graph = nk;
	return r;
}

// ---- several workers, one graph each, on one GPU ----------------------------
struct gh_workers_arg {
	int k; // graph slot
	int cpu; // -1: not pinned
	pthread_barrier_t *bar;
	uint64_t walks;
	int err;
};

static void *worker_thread(void *p) {
	struct gh_workers_arg *a = p;
	struct rte_graph *g = H.graphs[a->k].graph;
	if (a->cpu >= 0) { // grout's worker on its lcore (worker.c: the thread's affinity)
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(a->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	pthread_barrier_wait(a->bar);
	uint64_t w = 0;
	const uint64_t want = H.graphs[a->k].rx_end - (H.graphs[a->k].rx_next);
	for (uint32_t loop = 0; H.graphs[a->k].recorded < want; w++) {
		rte_graph_walk(g);
		if (++loop == 256) { // grout's housekeeping tick: the node's statistics fold
			loop = 0;
			gr_datapath_hooks_stats_flush(g, (unsigned)a->k, NULL, NULL); // its own lcore's iface_stats
		}
		if (w > (1ull << 32)) {
			a->err = -ETIMEDOUT;
			break;
		}
	}
	a->walks = w;
	pthread_barrier_wait(a->bar);
	return NULL;
}

// gr_datapath_loop on `threads` workers at once (worker.c: one graph per
// worker): graph slots 0 .. threads-1 (gh_graph_create'd), each polling its
// own contiguous share of the injected mbufs, each walked from its own
// pthread until everything it received is through its node and handed to
// the recorders behind (which only count in this mode). Returns 0 and the
// wall time from the start barrier to the last worker's end, or -errno.
int gh_workers_run(uint32_t threads, double *seconds, uint64_t *walks) {
	if (threads == 0 || H.wk0 + threads > GH_MAX_GRAPHS || H.n == 0)
		return -EINVAL;
	for (uint32_t k = 0; k < threads; k++)
		if (H.graphs[H.wk0 + k].graph == NULL)
			return -ENOENT;
	pthread_t th[GH_MAX_GRAPHS];
	struct gh_workers_arg args[GH_MAX_GRAPHS];
	if (H.recycle && ((uint64_t)H.recycle * threads > H.n || (uint64_t)H.n * H.passes > UINT32_MAX))
		return -EINVAL; // the pools are carved out of the loaded mbufs
	pthread_barrier_t bar;
	for (uint32_t k = 0; k < threads; k++) {
		H.graphs[H.wk0 + k].rx_next = (uint32_t)((uint64_t)H.n * k / threads);
		H.graphs[H.wk0 + k].rx_end = (uint32_t)((uint64_t)H.n * (k + 1) / threads);
		H.graphs[H.wk0 + k].recorded = 0;
		if (H.recycle) {
			H.graphs[H.wk0 + k].free_mb = malloc(H.recycle * sizeof(uint32_t));
			if (H.graphs[H.wk0 + k].free_mb == NULL) {
				for (uint32_t j = 0; j < k; j++) {
					free(H.graphs[H.wk0 + j].free_mb);
					H.graphs[H.wk0 + j].free_mb = NULL;
				}
				return -ENOMEM;
			}
			for (uint32_t j = 0; j < H.recycle; j++) // popped from the top: lowest index first
				H.graphs[H.wk0 + k].free_mb[j] = k * H.recycle + (H.recycle - 1 - j);
			H.graphs[H.wk0 + k].n_free = H.recycle;
			H.graphs[H.wk0 + k].rx_start = H.graphs[H.wk0 + k].rx_next;
			H.graphs[H.wk0 + k].share = H.graphs[H.wk0 + k].rx_end - H.graphs[H.wk0 + k].rx_next;
			H.graphs[H.wk0 + k].rx_end = H.graphs[H.wk0 + k].rx_next + H.graphs[H.wk0 + k].share * H.passes;
		}
		args[k] = (struct gh_workers_arg) {.k = (int)(H.wk0 + k), .cpu = -1, .bar = &bar};
	}
	for (uint32_t k = 0; k < threads && (int)k < H.n_lcores; k++)
		args[k].cpu = H.lcores[k];
	for (int g = 0; g < GH_MAX_GRAPHS; g++) { // this run's histograms only
		free(H.graphs[g].lat);
		H.graphs[g].lat = NULL;
	}
	for (uint32_t k = 0; k < threads && lat_on; k++)
		H.graphs[H.wk0 + k].lat = calloc(GH_LAT_BUCKETS, sizeof(uint64_t));
	pthread_barrier_init(&bar, NULL, threads + 1);
	H.workers = 1;
	for (uint32_t k = 0; k < threads; k++)
		pthread_create(&th[k], NULL, worker_thread, &args[k]);
	struct timespec a, b;
	pthread_barrier_wait(&bar);
	clock_gettime(CLOCK_MONOTONIC, &a);
	const uint64_t tsc_a = tsc();
	pthread_barrier_wait(&bar);
	const uint64_t tsc_b = tsc();
	clock_gettime(CLOCK_MONOTONIC, &b);
	int err = 0;
	uint64_t w = 0;
	for (uint32_t k = 0; k < threads; k++) {
		pthread_join(th[k], NULL);
		w += args[k].walks;
		if (args[k].err && !err)
			err = args[k].err;
	}
	H.workers = 0;
	pthread_barrier_destroy(&bar);
	for (uint32_t k = 0; k < threads; k++) {
		free(H.graphs[H.wk0 + k].free_mb);
		H.graphs[H.wk0 + k].free_mb = NULL;
		H.graphs[H.wk0 + k].n_free = 0;
	}
	*seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
	if (*seconds > 0)
		tsc_per_ns = (double)(tsc_b - tsc_a) / (*seconds * 1e9);
	if (walks != NULL)
		*walks = w;
	return err;
}

// Latency mode: the last gh_workers_run's histogram, summed over its workers
// (GH_LAT_BUCKETS counts of TSC cycles, gh_lat_bucket_floor gives each
// bucket's lower edge), and the TSC's rate over that run (cycles per ns).
int gh_latency(uint64_t *hist, uint32_t n, double *cycles_per_ns) {
	if (hist == NULL || n < GH_LAT_BUCKETS)
		return -EINVAL;
	memset(hist, 0, GH_LAT_BUCKETS * sizeof(uint64_t));
	for (int k = 0; k < GH_MAX_GRAPHS; k++)
		for (uint32_t b = 0; H.graphs[k].lat != NULL && b < GH_LAT_BUCKETS; b++)
			hist[b] += H.graphs[k].lat[b];
	if (cycles_per_ns != NULL)
		*cycles_per_ns = tsc_per_ns;
	return GH_LAT_BUCKETS;
}
