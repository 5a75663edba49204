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
// back short or a whole graph walk brings none (the queues drained: latency
// matters more than batching), or the oldest packet has waited max_delay.
// Each process() call's mbufs are staged as they arrive (gr_hip_node_append:
// header line and metadata into the queue's pinned walk slot while the
// frames are in cache), the batch is sent to the GPU at the flush
// (gr_hip_node_send), and once the GPU is done
// the batch is handed back (gr_hip_node_finish): each mbuf is enqueued on
// its verdict's edge with grout's private data for that edge. Batches are
// pipelined two deep ("depth" 2, the default): while the GPU forwards one,
// the worker accumulates and stages the next, and hands the one before back
// as soon as it is done; deeper (up to GR_HIP_NODE_DEPTH), depth - 1 batches
// are on the GPU while the next accumulates, so that a worker whose batches
// take longer on the GPU than to fill (small batches under a latency budget,
// many workers) keeps filling. Batches leave in the order they arrived. A source
// node, "gpu_fwd4_flush", runs every graph walk: it hands back a batch whose
// GPU work has completed, and flushes the batch held when the walk before
// brought no packet or its oldest packet has waited max_delay (rte_graph
// calls a node only when it holds objects).
//
// RCU. A batch's mbufs stay with the node across graph walks (accumulation,
// then the GPU), and grout's worker reports a QSBR quiescent state every 256
// walks whatever the node holds (main_loop.c:461-464). So each batch holds a
// QSBR reader of its own: one of the graph's GPU_FWD4_RCU_PER_GRAPH reader
// ids goes online when the batch takes its first mbuf (before the GPU reads
// any mirror for it) and offline at the start of the graph walk after the
// one that handed the batch back, once grout's nodes behind the edges have
// processed it. rte_rcu_qsbr_synchronize() in grout's control plane
// (nexthop_destroy, nexthop.c:505; iface_destroy, iface.c:712) therefore
// returns only after every batch that may name the object it frees is
// handed back. The hand-back turns the verdict's iface id and nexthop slot
// into pointers through the node's own registries (gpu_fwd4_iface_obj_set /
// _nh_obj_set), which the control plane clears only after that
// synchronisation, never through grout's iface_from_id, which is cleared
// before it.
//
// Stream limits. rte_graph holds a node's input stream in uint16_t-sized
// arrays; the node therefore hands at most one batch back per process() call
// (all those on the GPU only on the way out: a drain leaving the graph, a GPU
// marked diverged, GR_HIP_NODE_DEPTH x GPU_FWD4_BATCH_MAX < UINT16_MAX) and
// batches are at most GPU_FWD4_BATCH_MAX packets.
//
// It includes grout's and DPDK's headers by their names and builds unchanged
// in grout (modules/gpu, integration/grout-gpu_module-build.patch) and here,
// where the include path leads those names to the test stand-ins
// (tests/standin/include).
#include "gpu_fwd4_node.h"
#include "gpu_fwd4_control.h"

#include "datapath.h"
#include "eth.h"
#include "graph.h"
#include "iface.h"
#include "l3.h"
#include "mbuf.h"
#include "module.h"
#include "rcu.h"
#include "rxtx.h"

#include <rte_common.h>
#include <rte_graph.h>
#include <rte_graph_worker.h>
#include <rte_mbuf.h>
#include <rte_rcu_qsbr.h>

#include <errno.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static struct gpu_fwd4_conf conf = {
	.n_devs = 0, // every visible device
	.max_ifaces = 1024,
	.max_nexthops = 1u << 17,
	.batch = GPU_FWD4_BATCH_MAX,
	.rx_burst = 64,
	.max_delay_ns = 50000,
	.depth = 0, // from the latency budget (depth_now)
};

// One fast-path context per GPU; the worker graphs are spread over them.
static struct {
	gr_hip_ctx_t *ctx;
	int dev;
	int numa; // the device's NUMA node
	uint32_t graphs; // worker graphs bound to it
	int diverged; // a control call failed here only: its graphs punt (FANOUT)
} gpus[GPU_FWD4_MAX_DEVS];
static uint32_t n_gpus;

int gpu_fwd4_configure(const struct gpu_fwd4_conf *c) {
	if (c == NULL || c->batch == 0 || c->rx_burst == 0 || c->n_devs > GPU_FWD4_MAX_DEVS || n_gpus != 0
	    || c->depth > GR_HIP_NODE_DEPTH)
		return -EINVAL;
	conf = *c;
	if (conf.batch > GPU_FWD4_BATCH_MAX)
		conf.batch = GPU_FWD4_BATCH_MAX;
	return 0;
}

void gpu_fwd4_conf_get(struct gpu_fwd4_conf *c) {
	if (c != NULL)
		*c = conf;
}

// Budgets up to this get the deepest pipeline when conf.depth is 0 (DESIGN.md
// §6.3: at 50 us, 1.2-2.3x depth 2 at 8 and 16 workers; at 100 us little
// gain and a p99 past the budget at 16 workers)
#define DEPTH_AUTO_BUDGET_NS 75000

// The depth in effect: conf's, or with conf.depth 0 (the default) 2, and
// GR_HIP_NODE_DEPTH under a latency budget of DEPTH_AUTO_BUDGET_NS or less.
static uint32_t depth_now(void) {
	if (conf.depth != 0)
		return conf.depth;
	const uint64_t b = conf.latency_budget_ns;
	return b != 0 && b <= DEPTH_AUTO_BUDGET_NS ? GR_HIP_NODE_DEPTH : 2;
}

// More than one batch per graph on the GPU: a queue's one-ring batches run
// on its rings in turn, not one after the other on its first ("resident_rotate").
static void rotate_sync(void) {
	for (uint32_t i = 0; i < n_gpus; i++)
		gr_hip_tune(gpus[i].ctx, "resident_rotate", depth_now() > 2);
}

int gpu_fwd4_set_depth(uint32_t depth) {
	if (depth > GR_HIP_NODE_DEPTH)
		return -EINVAL;
	conf.depth = depth; // a graph's next flush switches (finishing what is in flight first)
	rotate_sync();
	return 0;
}

int gpu_fwd4_set_launch_per_batch(int on) {
	conf.launch_per_batch = on ? 1 : 0;
	for (uint32_t i = 0; i < n_gpus; i++)
		gr_hip_tune(gpus[i].ctx, "resident", on ? 0 : 1);
	return 0;
}

int gpu_fwd4_set_rx_burst(uint32_t rx_burst) {
	if (rx_burst == 0 || rx_burst > RTE_GRAPH_BURST_SIZE)
		return -EINVAL;
	conf.rx_burst = rx_burst;
	return 0;
}

int gpu_fwd4_set_batch(uint32_t batch, uint64_t max_delay_ns) {
	if (batch == 0)
		return -EINVAL;
	conf.batch = batch > GPU_FWD4_BATCH_MAX ? GPU_FWD4_BATCH_MAX : batch;
	conf.max_delay_ns = max_delay_ns;
	return 0;
}

// ---- the grout objects verdicts name (see "RCU" above) ---------------------
// (object pointers kept as const void *: the one table allocator serves both)
static const void **if_obj;
static uint32_t if_obj_n;
static const void **nh_obj;
static uint32_t nh_obj_n;

// Allocated at the first set, from the control thread; the size is published
// after the table (release), and the workers read it first (acquire).
static int obj_table(const void ***t, uint32_t *n, uint32_t want) {
	if (*t == NULL) {
		if ((*t = calloc(want, sizeof(void *))) == NULL)
			return -ENOMEM;
		__atomic_store_n(n, want, __ATOMIC_RELEASE);
	}
	return 0;
}

int gpu_fwd4_iface_obj_set(uint16_t id, const struct iface *i) {
	int r = obj_table(&if_obj, &if_obj_n, conf.max_ifaces);
	if (r < 0)
		return r;
	if (id == 0 || id >= if_obj_n)
		return -EINVAL;
	__atomic_store_n(&if_obj[id], i, __ATOMIC_RELEASE);
	return 0;
}

int gpu_fwd4_nh_obj_set(uint32_t slot, const struct nexthop *nh) {
	int r = obj_table(&nh_obj, &nh_obj_n, conf.max_nexthops + 1);
	if (r < 0)
		return r;
	if (slot == 0 || slot >= nh_obj_n)
		return -EINVAL;
	__atomic_store_n(&nh_obj[slot], nh, __ATOMIC_RELEASE);
	return 0;
}

const struct iface *gpu_fwd4_iface_obj(uint16_t id) {
	return id < __atomic_load_n(&if_obj_n, __ATOMIC_ACQUIRE) ? (const struct iface *)__atomic_load_n(&if_obj[id], __ATOMIC_ACQUIRE)
								  : NULL;
}

const struct nexthop *gpu_fwd4_nh_obj(uint32_t slot) {
	return slot < __atomic_load_n(&nh_obj_n, __ATOMIC_ACQUIRE)
		? (const struct nexthop *)__atomic_load_n(&nh_obj[slot], __ATOMIC_ACQUIRE)
		: NULL;
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
	gpu_fwd4_control_attach(ev); // the mirror's publication timer
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
		gr_hip_tune(c, "resident", conf.launch_per_batch ? 0 : 1);
		gr_hip_tune(c, "resident_rotate", depth_now() > 2); // (rotate_sync)
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
	while (n_gpus > 0) {
		gr_hip_fini(gpus[--n_gpus].ctx);
		gpus[n_gpus].diverged = 0;
	}
	free(if_obj);
	free(nh_obj);
	if_obj = NULL;
	nh_obj = NULL;
	if_obj_n = nh_obj_n = 0;
}

static struct module gpu_module = {
	.name = "gpu_fwd4",
	.depends_on = "rcu", // the graphs' QSBR readers (main_loop.c:538-552)
	.init = gpu_init,
	.fini = gpu_fini,
};

// grout's worker loop calls these (datapath.h's hooks, which
// integration/grout-gpu_fwd4-datapath.patch adds to main_loop.c): the drain
// before a worker leaves its graph, the statistics fold at each housekeeping
// tick, and the QSBR reader ids of the node's batches (see "RCU" above),
// which the rcu module's init sizes in.
static struct gr_datapath_hooks gpu_hooks = {
	.name = "gpu_fwd4",
	.rcu_readers = GPU_FWD4_RCU_READERS,
	.graph_leave = gpu_fwd4_drain,
	.stats_flush = gpu_fwd4_stats_flush,
	.holding = gpu_fwd4_holding,
};

RTE_INIT(gpu_module_init) {
	module_register(&gpu_module);
	gr_datapath_hooks_register(&gpu_hooks); // before the rcu module's init reads the readers
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
// A graph walk is one process() call (its first mbuf carries
// GR_HIP_MBUF_F_WALK): up to vector_max = 256 packets (graph.c:612-650).
// The node splits a longer call (several RX queues and other nodes feeding
// it more) at RTE_GRAPH_BURST_SIZE.
#define WALK_SPLIT RTE_GRAPH_BURST_SIZE

// Batch buffers per graph: the library's walk slots (conf.depth of them in use)
#define WALK_BUFS GR_HIP_NODE_DEPTH
_Static_assert(GPU_FWD4_RCU_PER_GRAPH >= 2 * WALK_BUFS, "a reader per batch held, and per batch handed back in a walk");
_Static_assert((uint64_t)WALK_BUFS * GPU_FWD4_BATCH_MAX + RTE_GRAPH_BURST_SIZE <= UINT16_MAX,
	       "every batch handed back in one walk fits rte_graph's stream");

enum { RD_FREE = 0, RD_HELD, RD_RELEASE };

struct gpu_walk {
	uint64_t prof_ns[GPU_FWD4_PROF_COUNT]; // gpu_fwd4_prof's clocks, this worker's
	const struct rte_graph *graph;
	int slot; // index in walks[]: its QSBR reader ids
	int gpu; // index in gpus[]
	gr_hip_queue_t *q;
	uint32_t n, cap; // the batch accumulating, in buffer `cur`
	uint64_t first_ns; // arrival of the oldest held packet, 0 = none
	// batch buffers, a ring: the npend batches on the GPU (sent, oldest in
	// `head`) and after them the one accumulating, cur = (head + npend) % WALK_BUFS
	uint32_t cur, head, npend;
	struct rte_mbuf **mbufs[WALK_BUFS];
	uint8_t *edges[WALK_BUFS]; // each mbuf's edge, as the one-pass hand-back leaves it
	uint32_t pend_n[WALK_BUFS]; // a batch on the GPU: its size,
	uint64_t pend_ns[WALK_BUFS]; // when it was sent,
	uint64_t pend_first_ns[WALK_BUFS]; // and when its oldest packet arrived
	uint64_t gpu_ns; // how long the last batches took to come back (a moving average), 0: none yet
	// QSBR readers (see "RCU" above): rd[k] is the reader buffer k's batch
	// holds (-1: none), rstate the state of each of the graph's readers
	int8_t rd[WALK_BUFS];
	uint8_t rstate[GPU_FWD4_RCU_PER_GRAPH];
	struct gr_hip_node_stats stats;
	struct gr_hip_node_stats flushed; // what gpu_fwd4_stats_flush reported already
	uint32_t node_id[GR_HIP_NODE_COUNT]; // rte_graph ids of the replaced nodes
	struct gr_hip_iface_stats *ifs; // gpu_fwd4_stats_flush's buffer [conf.max_ifaces]
	struct gr_hip_mbuf_layout lay; // where the hand-back writes in grout's mbufs
	uint64_t gpu_errors; // batches punted because the GPU call failed
	uint64_t append_errors; // graph walks punted because they could not be staged
	uint64_t batches, max_batch, stale;
	int rx_seen; // the node took packets since the flush node last ran
	int draining; // gpu_fwd4_drain: DRAIN_HAND_BACK or DRAIN_LEAVE (0: not draining)
	uint64_t handed; // batches handed back (delivered onto their edges)
	uint64_t drain_punted; // mbufs a drain in DRAIN_LEAVE mode sent to grout's CPU nodes
	// mbufs of a batch the GPU would neither finish nor give up (the fast
	// path's -EDEADLK: its resident kernel did not leave): never handed on,
	// since the GPU may still rewrite their frames; the GPU is marked diverged
	uint64_t stranded;
	// latency budget (conf.latency_budget_ns): the batch cap in effect, the
	// arrival of the oldest packet of the batch on the GPU, and what the
	// batches' oldest packets took, arrival to hand-back (a moving average)
	uint32_t lcap;
	uint64_t rtt_ns; // the batches' round trips, send to back (a moving average of those sampled)
	uint64_t lat_ns;
	uint64_t over_budget;
};

// gpu_fwd4_drain's modes: hand every batch back within the walk (the held one
// sent and waited for at once), or leave the GPU: the batch on it handed back,
// what is held or arrives sent to grout's CPU nodes (PUNT), untouched.
enum { DRAIN_HAND_BACK = 1, DRAIN_LEAVE = 2 };

static uint64_t now_ns(void) {
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// Where the workers' time goes (gpu_fwd4_prof): accumulated only while on,
// each worker's in its own gpu_walk (no line shared between workers),
// summed over the graphs when read.
static int prof_on;

#define PROF_T0() const uint64_t prof_t0__ = prof_on ? now_ns() : 0
#define PROF_ADD(k)                                                                                \
	do {                                                                                       \
		if (prof_on)                                                                       \
			w->prof_ns[k] += now_ns() - prof_t0__;                                     \
	} while (0)

static struct gpu_walk *walks[GPU_FWD4_MAX_GRAPHS];

void gpu_fwd4_prof(int on, uint64_t *out) {
	if (out != NULL)
		memset(out, 0, GPU_FWD4_PROF_COUNT * sizeof(uint64_t));
	for (int i = 0; i < GPU_FWD4_MAX_GRAPHS; i++) {
		if (walks[i] == NULL)
			continue;
		for (int k = 0; out != NULL && k < GPU_FWD4_PROF_COUNT; k++)
			out[k] += walks[i]->prof_ns[k];
		memset(walks[i]->prof_ns, 0, sizeof(walks[i]->prof_ns));
	}
	prof_on = on;
}

static struct gpu_walk *walk_of(const struct rte_graph *g) {
	for (int i = 0; i < GPU_FWD4_MAX_GRAPHS; i++)
		if (walks[i] != NULL && walks[i]->graph == g)
			return walks[i];
	return NULL;
}

int gpu_fwd4_set_latency_budget(uint64_t budget_ns) {
	conf.latency_budget_ns = budget_ns; // each graph's cap restarts at its next batch
	for (int i = 0; i < GPU_FWD4_MAX_GRAPHS; i++)
		if (walks[i] != NULL)
			walks[i]->lcap = 0;
	rotate_sync(); // the depth may follow the budget
	return 0;
}

GR_NODE_CTX_TYPE(gpu_fwd4_ctx, { struct gpu_walk *w; });

// ---- RCU: one QSBR reader per batch, from its first mbuf to the walk after
// its hand-back
static int rcu_on = 1;

void gpu_fwd4_rcu_readers(int on) {
	rcu_on = on;
}

static unsigned reader_id(const struct gpu_walk *w, int r) {
	return gpu_hooks.rcu_base + (unsigned)w->slot * GPU_FWD4_RCU_PER_GRAPH + (unsigned)r;
}

// Buffer k's batch takes its first mbuf: a free reader goes online for it.
static void reader_hold(struct gpu_walk *w, uint32_t k) {
	if (w->rd[k] >= 0)
		return;
	for (int r = 0; r < GPU_FWD4_RCU_PER_GRAPH; r++) {
		if (w->rstate[r] != RD_FREE)
			continue;
		w->rstate[r] = RD_HELD;
		w->rd[k] = (int8_t)r;
		if (rcu_on)
			rte_rcu_qsbr_thread_online(gr_datapath_rcu(), reader_id(w, r));
		return;
	}
	// not reached: WALK_BUFS batches held + as many released per walk at most
}

// Buffer k's batch was handed back: its reader goes offline at the next walk.
static void reader_handed_back(struct gpu_walk *w, uint32_t k) {
	if (w->rd[k] < 0)
		return;
	w->rstate[w->rd[k]] = RD_RELEASE;
	w->rd[k] = -1;
}

// A graph walk starts (the flush source node runs first): the batches handed
// back in earlier walks have been through grout's nodes behind the edges.
static void readers_release(struct gpu_walk *w) {
	for (int r = 0; r < GPU_FWD4_RCU_PER_GRAPH; r++) {
		if (w->rstate[r] != RD_RELEASE)
			continue;
		w->rstate[r] = RD_FREE;
		rte_rcu_qsbr_thread_offline(gr_datapath_rcu(), reader_id(w, r));
	}
}

// Where the one-pass hand-back (gr_hip_node_finish_mbufs) writes grout's
// mbuf fields and the private data grout's chain leaves for the node behind
// each edge: the iface everywhere; iface_input's vlan_id before eth_input;
// eth_input's domain and pre-resolved nexthop (NULL), then ip_input's /
// ip6_input's l3 nexthop over them (l3.h:9 shares the bytes, ip_input.c:156);
// iface_output's vlan_id for port_output / port_tx (iface_output.c:81-86,
// port_tx.c:84-118). The verdict's iface id and nexthop slot become pointers
// through the node's registries (see "RCU" above); a packet whose object is
// no longer registered (the control plane broke the RCU contract) keeps its
// mbuf as it was and goes to ip_output_error, counted.
static void layout_init(struct gr_hip_mbuf_layout *l) {
	memset(l, 0, sizeof(*l));
	l->data_off = offsetof(struct rte_mbuf, data_off);
	l->data_len = offsetof(struct rte_mbuf, data_len);
	l->pkt_len = offsetof(struct rte_mbuf, pkt_len);
	l->packet_type = offsetof(struct rte_mbuf, packet_type);
	l->priv = sizeof(struct rte_mbuf); // rte_mbuf_to_priv
	l->priv_iface = offsetof(struct mbuf_data, iface);
	l->priv_vlan_id = offsetof(struct iface_mbuf_data, vlan_id);
	l->priv_domain = offsetof(struct eth_input_mbuf_data, domain);
	l->priv_eth_nh = offsetof(struct eth_input_mbuf_data, nh);
	l->priv_l3_nh = offsetof(struct l3_mbuf_data, nh);
	// what the staging reads (gr_hip_node_append_mbufs): the frame at
	// rte_pktmbuf_mtod, hash.rss, the ingress iface's id, and the checksum
	// status ip_input tests (UNKNOWN or NONE: verified in software,
	// ip_input.c:80-92)
	l->buf_addr = offsetof(struct rte_mbuf, buf_addr);
	l->ol_flags = offsetof(struct rte_mbuf, ol_flags);
	l->rss = offsetof(struct rte_mbuf, hash.rss);
	l->iface_id = offsetof(struct iface, id);
	l->ck_mask = RTE_MBUF_F_RX_IP_CKSUM_MASK;
	l->ck_good = RTE_MBUF_F_RX_IP_CKSUM_GOOD;
	l->ck_bad = RTE_MBUF_F_RX_IP_CKSUM_BAD;
}
_Static_assert(sizeof(((struct rte_mbuf *)0)->data_off) == 2 && sizeof(((struct rte_mbuf *)0)->data_len) == 2
		       && sizeof(((struct rte_mbuf *)0)->pkt_len) == 4 && sizeof(((struct rte_mbuf *)0)->packet_type) == 4
		       && sizeof(eth_domain_t) == 4 && sizeof(((struct rte_mbuf *)0)->buf_addr) == 8
		       && sizeof(((struct rte_mbuf *)0)->ol_flags) == 8 && sizeof(((struct rte_mbuf *)0)->hash.rss) == 4
		       && sizeof(((struct iface *)0)->id) == 2,
	       "the widths gr_hip_mbuf_layout names");

// The registries as they are now (allocated once, at their first set).
static const struct gr_hip_mbuf_layout *layout_now(struct gpu_walk *w) {
	w->lay.n_ifaces = __atomic_load_n(&if_obj_n, __ATOMIC_ACQUIRE);
	w->lay.ifaces = if_obj;
	w->lay.n_nh = __atomic_load_n(&nh_obj_n, __ATOMIC_ACQUIRE);
	w->lay.nh = nh_obj;
	return &w->lay;
}

// Hand the GPU's oldest batch back onto buffer k's mbufs (one pass: frames,
// mbuf fields, private data) and return the finish's result.
static int hand_back(struct gpu_walk *w, uint32_t k) {
	uint32_t stale = 0;
	const int r = gr_hip_node_finish_mbufs(w->q, (void *const *)w->mbufs[k], layout_now(w), w->edges[k], &stale,
					       &w->stats);
	w->stale += stale;
	return r;
}

// Enqueue batch buffer k (n mbufs) on their edges; r: what the GPU call
// returned (< 0: the GPU could not take them, mbufs untouched: grout's CPU
// nodes do; > 0: a kernel gave up, the packets it did not reach come back as
// PUNT with their frames untouched, the others are forwarded as usual).
static void deliver(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w, uint32_t k, uint32_t n,
		    int r) {
	PROF_T0();
	struct rte_mbuf **mb = w->mbufs[k];
	if (r != 0)
		w->gpu_errors++;
	if (r < 0) {
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, (void **)mb, (uint16_t)n);
	} else {
		// runs of one edge go in one rte_node_enqueue (a forwarded stream is
		// mostly one run to port_output); a batch is at most
		// GPU_FWD4_BATCH_MAX < UINT16_MAX
		const uint8_t *e = w->edges[k];
		uint32_t run = 0;
		for (uint32_t i = 1; i <= n; i++) {
			if (i == n || e[i] != e[run]) {
				rte_node_enqueue(graph, node, e[run], (void **)&mb[run], (uint16_t)(i - run));
				run = i;
			}
		}
	}
	reader_handed_back(w, k);
	w->handed++;
	PROF_ADD(GPU_FWD4_PROF_DELIVER);
}

// The oldest batch on the GPU is done (or the poll failed: finish_oldest
// reports it): polled like a worker polls its RX queues, the time it took
// noted for reap's first poll.
static void poll_until_ready(struct gpu_walk *w) {
	if (w->npend == 0)
		return;
	PROF_T0();
	int polls = 0;
	for (int ready = 0; !ready; polls++)
		if (gr_hip_node_pending(w->q, &ready) <= 0) // an error, or nothing in flight after all
			break;
	PROF_ADD(GPU_FWD4_PROF_POLL);
	const uint64_t waited = now_ns() - w->pend_ns[w->head];
	w->gpu_ns = w->gpu_ns ? (w->gpu_ns * 7 + waited) / 8 : waited;
	if (polls > 1) // it came back just now: its round trip (else it was back before: no sample)
		w->rtt_ns = w->rtt_ns ? (w->rtt_ns * 7 + waited) / 8 : waited;
}

// What the batch accumulating may hold, and how long its oldest packet may
// wait before it is sent: conf's, or under a latency budget the graph's cap
// and the budget less the GPU's round trip (a quarter of the budget at least;
// the round trip sampled when a batch comes back while polled, not when the
// next batch's fill outlasted it).
static uint32_t batch_cap(struct gpu_walk *w) {
	if (conf.latency_budget_ns == 0)
		return conf.batch;
	if (w->lcap == 0 || w->lcap > conf.batch)
		w->lcap = conf.batch < 1024 ? conf.batch : 1024;
	return w->lcap;
}

static uint64_t hold_max(const struct gpu_walk *w) {
	const uint64_t b = conf.latency_budget_ns;
	if (b == 0)
		return conf.max_delay_ns;
	const uint64_t h = w->rtt_ns + b / 4 < b ? b - w->rtt_ns : b / 4;
	return h < conf.max_delay_ns ? h : conf.max_delay_ns;
}

// A batch came back: its oldest packet took `lat` from its arrival. Under a
// budget the cap follows the moving average of those times: down by an eighth
// while it is above 17/20 of the budget, up by an eighth (64 at least) while it
// is below 13/20 and full batches come back. One late batch (a host stall,
// another worker's burst on the GPU) moves it little: every worker keeps
// batches of about the same size, and the slowest one sets the pace.
static void budget_update(struct gpu_walk *w, uint64_t lat, uint32_t n) {
	w->lat_ns = w->lat_ns ? (w->lat_ns * 7 + lat) / 8 : lat;
	const uint64_t b = conf.latency_budget_ns;
	if (b == 0)
		return;
	if (lat > b)
		w->over_budget++;
	const uint32_t cap = batch_cap(w), step = cap / 8 > 64 ? cap / 8 : 64;
	if (w->lat_ns * 20 > b * 17)
		w->lcap = cap > step + 64 ? cap - step : 64;
	else if (w->lat_ns * 20 < b * 13 && n >= cap - cap / 8)
		w->lcap = cap + step < conf.batch ? cap + step : conf.batch;
}

// Wait for the oldest batch on the GPU and hand it back. Returns its size.
// The fast path bounds the wait: past the batch's deadline it retires what
// the GPU did not run, and the hand-back punts those packets, untouched, to
// grout's CPU nodes (counted in gpu_errors). Only when the GPU would not let
// go of the batch (-EDEADLK) are its mbufs kept: stranded, never handed on,
// and the GPU marked diverged (its graphs punt from then on).
static uint32_t finish_oldest(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	if (w->npend == 0)
		return 0;
	const uint32_t k = w->head, n = w->pend_n[k];
	PROF_T0();
	const int r = hand_back(w, k); // the library's oldest walk: buffer k's
	PROF_ADD(GPU_FWD4_PROF_FINISH);
	w->head = (k + 1) % WALK_BUFS;
	w->npend--;
	budget_update(w, now_ns() - w->pend_first_ns[k], n);
	if (r == -EDEADLK) {
		w->stranded += n;
		w->gpu_errors++;
		reader_handed_back(w, k);
		__atomic_store_n(&gpus[w->gpu].diverged, 1, __ATOMIC_RELEASE);
		return 0;
	}
	deliver(graph, node, w, k, n, r);
	return n;
}

// Every batch on the GPU, oldest first (leaving the graph, a GPU diverged).
static uint32_t finish_all(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	uint32_t n = 0;
	while (w->npend != 0)
		n += finish_oldest(graph, node, w);
	return n;
}

static void started(struct gpu_walk *w, uint32_t n) {
	w->batches++;
	if (n > w->max_batch)
		w->max_batch = n;
}

// Send the accumulated batch; returns the mbufs handed back meanwhile: one
// batch at most (the accumulated one when synchronous, else the oldest on the
// GPU once depth - 1 are there, or once it is done), two only when the GPU
// refuses this one (both then go to grout's CPU nodes and the walk's edges
// hold at most three batches: still under rte_graph's stream limit).
static uint32_t flush(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	if (w->n == 0)
		return 0;
	const uint32_t k = w->cur, n = w->n;
	const uint64_t first = w->first_ns;
	w->n = 0;
	w->first_ns = 0;
	if (gpus[w->gpu].diverged) { // not to this GPU: grout's CPU nodes, after the batches before
		const uint32_t d = finish_all(graph, node, w);
		gr_hip_node_discard(w->q);
		deliver(graph, node, w, k, n, -ESTALE);
		w->cur = (w->head + w->npend) % WALK_BUFS;
		return d + n;
	}
	const uint32_t depth = depth_now();
	if ((depth < 2 || w->draining) && w->npend == 0) { // synchronous
		started(w, n);
		int r = gr_hip_node_send(w->q, NULL, n, WALK_SPLIT);
		if (r == 0)
			r = hand_back(w, k);
		if (r == -EDEADLK) { // stranded: see finish_oldest
			w->stranded += n;
			w->gpu_errors++;
			reader_handed_back(w, k);
			__atomic_store_n(&gpus[w->gpu].diverged, 1, __ATOMIC_RELEASE);
			return 0;
		}
		deliver(graph, node, w, k, n, r);
		return n;
	}
	// send this batch (staged as it arrived, gpu_fwd4_process) while the
	// ones before may still be on the GPU; with depth - 1 of them there (one
	// for depth 1 and during a drain), hand the oldest back, waiting for it,
	// else only if it is done: batches leave in arrival order
	PROF_T0();
	const int r = gr_hip_node_send(w->q, NULL, n, WALK_SPLIT);
	PROF_ADD(GPU_FWD4_PROF_START);
	const uint32_t room = depth > 2 && !w->draining ? depth - 1 : 1;
	uint32_t delivered = 0;
	if (r < 0 || w->npend >= room) {
		poll_until_ready(w); // a worker polls; a blocking wait would sleep on the GPU's interrupt
		delivered = finish_oldest(graph, node, w);
	} else if (w->npend != 0) {
		int ready = 0;
		if (gr_hip_node_pending(w->q, &ready) > 0 && ready)
			delivered = finish_oldest(graph, node, w);
	}
	if (r < 0) { // the GPU did not take it: grout's CPU nodes do, after the batches before
		delivered += finish_all(graph, node, w);
		deliver(graph, node, w, k, n, r);
		w->cur = (w->head + w->npend) % WALK_BUFS;
		return delivered + n;
	}
	started(w, n);
	w->pend_n[k] = n;
	w->pend_ns[k] = now_ns();
	w->pend_first_ns[k] = first ? first : w->pend_ns[k];
	w->npend++;
	w->cur = (w->head + w->npend) % WALK_BUFS;
	return delivered;
}

// A batch spends at least this long on the GPU (PCIe both ways, the kernel's
// tile latency: ~12 us for 64 packets resident): no poll before.
// With a launch per batch, nor before 3/4 of what the last batches took: each
// poll is then a runtime call (hipEventQuery), whose locks every worker of the
// process shares; with the resident kernel a poll is a load of a done word.
#define REAP_MIN_NS 10000

// The oldest batch on the GPU is done: hand it back now (a poll, no wait).
static uint32_t reap(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	int ready = 0;
	if (w->npend == 0)
		return 0;
	const uint64_t t = now_ns(), waited = t - w->pend_ns[w->head];
	if (waited < REAP_MIN_NS || (conf.launch_per_batch && waited < w->gpu_ns / 4 * 3))
		return 0;
	PROF_T0();
	const int r = gr_hip_node_pending(w->q, &ready);
	PROF_ADD(GPU_FWD4_PROF_POLL);
	if (r < 0) // past its deadline, or the GPU failed: the finish decides (bounded)
		return finish_oldest(graph, node, w);
	if (!ready)
		return 0;
	w->gpu_ns = w->gpu_ns ? (w->gpu_ns * 7 + waited) / 8 : waited; // an upper bound: polled late
	w->rtt_ns = w->rtt_ns ? (w->rtt_ns * 7 + waited) / 8 : waited;
	return finish_oldest(graph, node, w);
}

// gpu_fwd4_drain past its bound (DRAIN_LEAVE): the batches on the GPU are
// waited for and handed back; the held one (staged, not sent: its frames and
// mbufs untouched) goes to grout's CPU nodes, after them in arrival order.
// Returns the mbufs handed back or sent on.
static uint32_t leave(struct rte_graph *graph, struct rte_node *node, struct gpu_walk *w) {
	uint32_t n = finish_all(graph, node, w);
	if (w->n != 0) {
		const uint32_t k = w->cur, held = w->n;
		gr_hip_node_discard(w->q);
		w->n = 0;
		w->first_ns = 0;
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, (void **)w->mbufs[k], (uint16_t)held);
		reader_handed_back(w, k);
		w->drain_punted += held;
		n += held;
	}
	return n;
}

static uint16_t gpu_fwd4_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	struct gpu_walk *w = gpu_fwd4_ctx(node)->w;
	PROF_T0();
	if (w->draining == DRAIN_LEAVE) { // the worker leaves the graph: nothing more for the GPU
		leave(graph, node, w);
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, objs, nb_objs);
		w->drain_punted += nb_objs;
		return nb_objs;
	}
	if (gpus[w->gpu].diverged) { // this GPU's mirrors are out of step: grout's CPU nodes
		if (w->n != 0)
			flush(graph, node, w); // the packets held first (punted too)
		else
			reap(graph, node, w);
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, objs, nb_objs);
		return nb_objs;
	}
	const uint32_t n0 = w->n; // this call is one graph walk's iface_input stream
	w->rx_seen = 1;
	// software pipeline over the burst (as DPDK's l3fwd does): each mbuf
	// PF_MBUF ahead, its frame PF_FRAME ahead, so that their misses overlap
	// and the staging below finds the frames in cache
	enum { PF_MBUF = 8, PF_FRAME = 4 };
	for (uint16_t i = 0; i < nb_objs && i < PF_MBUF; i++)
		rte_prefetch0(objs[i]);
	for (uint16_t i = 0; i < nb_objs && i < PF_FRAME; i++)
		rte_prefetch0(rte_pktmbuf_mtod((struct rte_mbuf *)objs[i], void *));
	for (uint16_t i = 0; i < nb_objs; i++) {
		struct rte_mbuf *m = objs[i];
		if (i + PF_MBUF < nb_objs)
			rte_prefetch0(objs[i + PF_MBUF]);
		if (i + PF_FRAME < nb_objs)
			rte_prefetch0(rte_pktmbuf_mtod((struct rte_mbuf *)objs[i + PF_FRAME], void *));
		// grout's CPU nodes: multi-segment or traced mbufs; and, never in
		// practice (a batch starts below conf.batch and a call brings at
		// most RTE_GRAPH_BURST_SIZE), a full buffer
		if (m->nb_segs > 1 || gr_mbuf_is_traced(m) || w->n == w->cap) {
			rte_node_enqueue_x1(graph, node, GR_HIP_E_PUNT, m);
			continue;
		}
		if (w->n == 0)
			reader_hold(w, w->cur); // before the GPU reads any mirror for this batch
		w->mbufs[w->cur][w->n++] = m;
	}
	// stage this walk now, while its mbufs and frames are in cache: the
	// library reads each mbuf through the layout (frame, lengths, private
	// data) and stages its header line and metadata in one pass. A walk that
	// cannot be staged (no pinned memory for the slot ...; the append leaves
	// the slot as it was) goes to grout's CPU nodes now, untouched and
	// counted; the walks before it stay in the batch.
	if (w->n > n0
	    && gr_hip_node_append_mbufs(w->q, (void *const *)&w->mbufs[w->cur][n0], w->n - n0, &w->lay, WALK_SPLIT) < 0) {
		rte_node_enqueue(graph, node, GR_HIP_E_PUNT, (void **)&w->mbufs[w->cur][n0], (uint16_t)(w->n - n0));
		w->append_errors++;
		w->n = n0;
		if (n0 == 0)
			reader_handed_back(w, w->cur); // the batch this walk would have started
	}
	PROF_ADD(GPU_FWD4_PROF_ACCUMULATE);
	if (w->n == 0) {
		reap(graph, node, w);
		return nb_objs;
	}
	const uint64_t t = now_ns();
	if (w->first_ns == 0)
		w->first_ns = t;
	if (w->draining || w->n >= batch_cap(w) || nb_objs < conf.rx_burst || t - w->first_ns >= hold_max(w))
		flush(graph, node, w);
	else
		reap(graph, node, w);
	return nb_objs;
}

static void walk_free(struct gpu_walk *w) {
	for (int k = 0; k < WALK_BUFS; k++) {
		free(w->mbufs[k]);
		free(w->edges[k]);
	}
	free(w->ifs);
	free(w);
}

// rte_graph ids of the replaced nodes, by enum gr_hip_node
static const char *const replaced_names[GR_HIP_NODE_COUNT] = {
	[GR_HIP_NODE_IFACE_INPUT] = "iface_input",
	[GR_HIP_NODE_ETH_INPUT] = "eth_input",
	[GR_HIP_NODE_IP_INPUT] = "ip_input",
	[GR_HIP_NODE_IP_FORWARD] = "ip_forward",
	[GR_HIP_NODE_IP_OUTPUT] = "ip_output",
	[GR_HIP_NODE_ETH_OUTPUT] = "eth_output",
	[GR_HIP_NODE_IFACE_OUTPUT] = "iface_output",
	[GR_HIP_NODE_IP6_INPUT] = "ip6_input",
	[GR_HIP_NODE_IP6_FORWARD] = "ip6_forward",
	[GR_HIP_NODE_IP6_OUTPUT] = "ip6_output",
};

static int gpu_fwd4_init(const struct rte_graph *graph, struct rte_node *node) {
	if (n_gpus == 0)
		return -ENODEV;
	if (gr_datapath_rcu() == NULL)
		return -ENODEV;
	int slot = 0;
	while (slot < GPU_FWD4_MAX_GRAPHS && walks[slot] != NULL)
		slot++;
	if (slot == GPU_FWD4_MAX_GRAPHS)
		return -ENOSPC;
	// the worker's own lines (grout: rte_zmalloc, cache-aligned): no line the
	// walk writes shared with another worker's
	const size_t wsz = (sizeof(struct gpu_walk) + 127) / 128 * 128;
	struct gpu_walk *w = aligned_alloc(128, wsz);
	if (w == NULL)
		return -ENOMEM;
	memset(w, 0, wsz);
	w->graph = graph;
	w->slot = slot;
	w->gpu = pick_gpu(graph);
	w->cap = GPU_FWD4_BATCH_MAX + RTE_GRAPH_BURST_SIZE; // any batch set_batch allows
	int r = 0;
	for (int k = 0; k < WALK_BUFS; k++) {
		w->rd[k] = -1;
		w->mbufs[k] = calloc(w->cap, sizeof(*w->mbufs[k]));
		w->edges[k] = calloc(w->cap, 1);
		if (w->mbufs[k] == NULL || w->edges[k] == NULL)
			r = -ENOMEM;
	}
	layout_init(&w->lay);
	if ((w->ifs = calloc(conf.max_ifaces, sizeof(*w->ifs))) == NULL)
		r = -ENOMEM;
	for (int k = 0; k < GR_HIP_NODE_COUNT; k++)
		w->node_id[k] = rte_node_from_name(replaced_names[k]);
	if (r == 0)
		r = gr_hip_queue_create(gpus[w->gpu].ctx, NULL, &w->q);
	for (int i = 0; r == 0 && i < GPU_FWD4_RCU_PER_GRAPH; i++)
		r = rte_rcu_qsbr_thread_register(gr_datapath_rcu(), reader_id(w, i)); // offline until a batch holds it
	if (r < 0) {
		if (w->q != NULL)
			gr_hip_queue_destroy(w->q);
		walk_free(w);
		return r;
	}
	gpus[w->gpu].graphs++;
	walks[slot] = w;
	gpu_fwd4_ctx(node)->w = w;
	return 0;
}

// mbufs a graph still held when it was destroyed (not drained first)
static uint64_t fini_freed;

uint64_t gpu_fwd4_fini_freed(void) {
	return __atomic_load_n(&fini_freed, __ATOMIC_RELAXED);
}

// Batches a drain may hand back: -1 = those the node holds when it starts +
// DRAIN_EXTRA (what RX brings during its walks), else this many
// (gpu_fwd4_set_drain_bound).
#define DRAIN_EXTRA 2
static int32_t drain_bound = -1;

int gpu_fwd4_set_drain_bound(int32_t batches) {
	drain_bound = batches < 0 ? -1 : batches;
	return 0;
}

// Leaving a graph (grout's worker before it switches to a new graph or shuts
// down: the graph_leave hook, main_loop.c:466-470 with
// integration/grout-gpu_fwd4-datapath.patch). grout itself holds no packet
// across graph walks; the node holds up to `depth` batches. Walks of the graph in
// DRAIN_HAND_BACK mode hand the batches on the GPU back (waiting for them) and
// send the held one, and whatever RX brings meanwhile, synchronously: one walk
// normally leaves nothing held. The walks are bounded by batches handed back,
// not by walks: once the batches held at the start and DRAIN_EXTRA more are
// back (gpu_fwd4_set_drain_bound), one walk in DRAIN_LEAVE mode hands back the batches on the GPU and sends
// what is still held, and what RX brings in that walk, to grout's CPU nodes
// (PUNT, untouched: forwarded by iface_input_cpu, counted there). Every
// hand-back went through grout's nodes within its walk, so the batches' QSBR
// readers go offline here. Returns the mbufs sent to grout's CPU nodes in
// DRAIN_LEAVE mode (0 normally), or -ENOENT.
int gpu_fwd4_drain(struct rte_graph *graph) {
	struct gpu_walk *w = walk_of(graph);
	if (w == NULL)
		return -ENOENT;
	const uint64_t h0 = w->handed, p0 = w->drain_punted;
	const uint64_t bound = drain_bound >= 0 ? (uint64_t)drain_bound : (w->n != 0) + (uint64_t)w->npend + DRAIN_EXTRA;
	w->draining = DRAIN_HAND_BACK;
	while ((w->n != 0 || w->npend != 0) && w->handed - h0 < bound)
		rte_graph_walk(graph);
	if (w->n != 0 || w->npend != 0) {
		w->draining = DRAIN_LEAVE;
		rte_graph_walk(graph);
	}
	w->draining = 0;
	readers_release(w);
	return (int)(w->drain_punted - p0);
}

static void gpu_fwd4_fini(const struct rte_graph *graph, struct rte_node *node) {
	(void)node;
	for (int i = 0; i < GPU_FWD4_MAX_GRAPHS; i++) {
		struct gpu_walk *w = walks[i];
		if (w == NULL || w->graph != graph)
			continue;
		// a graph destroyed without gpu_fwd4_drain: its mbufs go back to the
		// pool, counted (gpu_fwd4_fini_freed). A batch on the GPU is
		// dropped from the queue only once the GPU is done with its frames
		// (gr_hip_node_finish waits before it refuses a batch appended from
		// the mbufs)
		// (a GPU that would not let go of it, -EDEADLK: its mbufs stay
		// stranded, never freed, since the GPU may still write their frames)
		uint64_t freed = w->n;
		for (; w->npend != 0; w->npend--, w->head = (w->head + 1) % WALK_BUFS) { // oldest first
			const uint32_t k = w->head;
			if (gr_hip_node_finish(w->q, NULL, NULL, NULL) == -EDEADLK) {
				w->stranded += w->pend_n[k];
				continue;
			}
			for (uint32_t j = 0; j < w->pend_n[k]; j++)
				rte_pktmbuf_free(w->mbufs[k][j]);
			freed += w->pend_n[k];
		}
		for (uint32_t j = 0; j < w->n; j++) // held, never sent
			rte_pktmbuf_free(w->mbufs[w->cur][j]);
		__atomic_fetch_add(&fini_freed, freed, __ATOMIC_RELAXED);
		gr_hip_queue_destroy(w->q);
		for (int k = 0; k < GPU_FWD4_RCU_PER_GRAPH; k++) { // offline, then gone (rte_rcu_qsbr.h)
			if (w->rstate[k] != RD_FREE)
				rte_rcu_qsbr_thread_offline(gr_datapath_rcu(), reader_id(w, k));
			rte_rcu_qsbr_thread_unregister(gr_datapath_rcu(), reader_id(w, k));
		}
		if ((uint32_t)w->gpu < n_gpus && gpus[w->gpu].graphs > 0)
			gpus[w->gpu].graphs--;
		walks[i] = NULL;
		walk_free(w);
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
	PROF_T0();
	struct gpu_walk *w = c->w;
	// a new graph walk: what was handed back in the walks before has been
	// through grout's nodes, those batches' QSBR readers go offline
	readers_release(w);
	if (w->draining == DRAIN_LEAVE) {
		const uint32_t n = leave(graph, node, w);
		return (uint16_t)(n > UINT16_MAX ? UINT16_MAX : n);
	}
	// same edges as iface_input, same order; one batch handed back at most
	// (flush() hands back one more at most, and none is after these)
	const uint64_t t = now_ns();
	uint32_t n = 0;
	// (conf's delay, also under a latency budget: the oldest batch on the GPU is
	// reaped as soon as it is back, and a wait here would stall RX)
	if (w->npend != 0 && (w->draining || t - w->pend_ns[w->head] >= conf.max_delay_ns))
		n = finish_oldest(graph, node, w); // waited long enough (or leaving the graph): wait for the GPU
	else
		n = reap(graph, node, w);
	// a whole graph walk brought the node nothing: the RX queues drained,
	// latency wins over batching (as for a short burst); else max_delay
	const int idle = !w->rx_seen;
	w->rx_seen = 0;
	if (w->n != 0 && (w->draining || idle || t - w->first_ns >= hold_max(w)))
		n += flush(graph, node, w); // pipelined: a later walk of the graph hands it back
	PROF_ADD(GPU_FWD4_PROF_FLUSH_NODE);
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
	return gr_hip_node_iface_stats(w->q, stats, max_ifaces, reset);
}

int gpu_fwd4_stats_flush(const struct rte_graph *graph, unsigned lcore_id, gpu_fwd4_node_stat_cb cb, void *cookie) {
	struct gpu_walk *w = walk_of(graph);
	if (w == NULL)
		return -ENOENT;
	uint64_t total = 0;
	// iface_input is the node itself: rte_graph counts it
	for (int k = GR_HIP_NODE_IFACE_INPUT + 1; k < GR_HIP_NODE_COUNT; k++) {
		const uint64_t p = w->stats.packets[k] - w->flushed.packets[k];
		const uint64_t c = w->stats.calls[k] - w->flushed.calls[k];
		if ((p || c) && cb != NULL && w->node_id[k] != RTE_NODE_ID_INVALID)
			cb(cookie, w->node_id[k], p, c);
		total += p;
	}
	w->flushed = w->stats;
	if (gr_hip_node_iface_stats(w->q, w->ifs, conf.max_ifaces, 1) == 0) {
		for (uint32_t i = 1; i < conf.max_ifaces; i++) {
			const struct gr_hip_iface_stats *d = &w->ifs[i];
			if ((d->rx_packets | d->tx_packets) == 0)
				continue;
			struct iface_stats *st = iface_get_stats((uint16_t)lcore_id, (uint16_t)i);
			st->rx_packets += d->rx_packets;
			st->rx_bytes += d->rx_bytes;
			st->tx_packets += d->tx_packets;
			st->tx_bytes += d->tx_bytes;
		}
	}
	return (int)(total > INT32_MAX ? INT32_MAX : total);
}

int gpu_fwd4_walk_info(const struct rte_graph *graph, struct gpu_fwd4_walk_info *info) {
	struct gpu_walk *w = walk_of(graph);
	if (w == NULL || info == NULL)
		return -ENOENT;
	memset(info, 0, sizeof(*info));
	info->held = w->n;
	info->in_flight = w->npend;
	info->batches = w->batches;
	info->max_batch = w->max_batch;
	info->stale = w->stale;
	for (int r = 0; r < GPU_FWD4_RCU_PER_GRAPH; r++)
		info->readers_online += w->rstate[r] != RD_FREE;
	info->diverged = gpus[w->gpu].diverged;
	info->append_errors = w->append_errors;
	info->handed = w->handed;
	info->drain_punted = w->drain_punted;
	info->stranded = w->stranded;
	info->batch_cap = batch_cap(w);
	info->lat_ns = w->lat_ns;
	info->over_budget = w->over_budget;
	info->depth = depth_now();
	return 0;
}

uint64_t gpu_fwd4_holding(const struct rte_graph *graph) {
	const struct gpu_walk *w = walk_of(graph);
	if (w == NULL)
		return 0;
	uint64_t held = w->n;
	for (uint32_t i = 0; i < w->npend; i++)
		held += w->pend_n[(w->head + i) % WALK_BUFS];
	for (int r = 0; r < GPU_FWD4_RCU_PER_GRAPH; r++)
		held += w->rstate[r] != RD_FREE; // offline at the next walk's flush node
	return held;
}

int gpu_fwd4_graph_gpu(const struct rte_graph *graph) {
	struct gpu_walk *w = walk_of(graph);
	return w == NULL ? -ENOENT : w->gpu;
}

// ---- control plane: every change goes to every GPU's context ---------------
// (grout's control thread calls these from its event handlers, INTEGRATION.md
// §4; each context is updated under its own quiesce, so a GPU's in-flight
// walks see the old or the new state, never a mix.) The first error is
// returned; the other contexts still get the change. A context where the
// call failed while it succeeded elsewhere, or failed differently, is marked
// diverged (see gpu_fwd4_node.h).
static void mark_diverged(const int *rs) {
	int ok = 0;
	for (uint32_t i = 0; i < n_gpus; i++)
		ok |= rs[i] >= 0;
	for (uint32_t i = 0; i < n_gpus; i++)
		if (rs[i] < 0 && (ok || rs[i] != rs[0]))
			__atomic_store_n(&gpus[i].diverged, 1, __ATOMIC_RELEASE);
}

#define FANOUT(call)                                                                               \
	do {                                                                                       \
		int ret__ = n_gpus ? 0 : -ENODEV;                                                  \
		int rs__[GPU_FWD4_MAX_DEVS];                                                       \
		for (uint32_t i = 0; i < n_gpus; i++) {                                            \
			gr_hip_ctx_t *ctx = gpus[i].ctx;                                           \
			rs__[i] = (call);                                                          \
			if (rs__[i] < 0 && ret__ == 0)                                             \
				ret__ = rs__[i];                                                   \
		}                                                                                  \
		if (ret__ < 0)                                                                     \
			mark_diverged(rs__);                                                       \
		return ret__;                                                                      \
	} while (0)

int gpu_fwd4_diverged(uint32_t i) {
	return i < n_gpus ? __atomic_load_n(&gpus[i].diverged, __ATOMIC_ACQUIRE) : -ENOENT;
}

int gpu_fwd4_resync(uint32_t i) {
	if (i >= n_gpus)
		return -ENOENT;
	__atomic_store_n(&gpus[i].diverged, 0, __ATOMIC_RELEASE);
	return 0;
}

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
