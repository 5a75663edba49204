// SPDX-License-Identifier: BSD-3-Clause
//
// graph_selftest.c -- test harness (not the product): checks the rte_graph
// stand-in's semantics that grout's nodes rely on, with toy nodes and no GPU
// (tests/test_graph_walk.py, CPU). Returns 0, or minus the failing line.
#include "gr_datapath_min.h"

#include <stdint.h>
#include <stdlib.h>

#define CHECK(c)                                                                                   \
	do {                                                                                       \
		if (!(c))                                                                          \
			return -__LINE__;                                                          \
	} while (0)

#define ST_TOTAL 1000
#define ST_BURST 64

static uint32_t st_next; // objects emitted by the source
static uintptr_t st_seen[4 * ST_TOTAL];
static uint32_t st_n_seen;

static uint16_t st_src(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	(void)objs;
	(void)nb;
	void *burst[ST_BURST];
	uint16_t k = 0;
	while (k < ST_BURST && st_next < ST_TOTAL)
		burst[k++] = (void *)(uintptr_t)(++st_next);
	rte_node_enqueue(g, n, 0, burst, k);
	return k;
}

static uint16_t st_split(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	for (uint16_t i = 0; i < nb; i++) {
		uintptr_t v = (uintptr_t)objs[i];
		rte_node_enqueue_x1(g, n, (rte_edge_t)(v & 1), objs[i]); // 0: even, 1: odd
	}
	return nb;
}

static uint16_t st_even(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	if (objs != n->objs || nb != n->idx)
		return 0; // process() runs on the node's own array (checked below)
	rte_node_next_stream_move(g, n, 0); // DPDK's "everything to one edge"
	return nb;
}

static uint16_t st_odd(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	for (uint16_t i = 0; i < nb; i++) // tagged, to the sink through st_tag
		rte_node_enqueue_x1(g, n, 0, (void *)((uintptr_t)objs[i] + 10000));
	return nb / 2; // counted as the node's packets
}

static uint16_t st_tag(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	rte_node_enqueue(g, n, 0, objs, nb);
	return nb;
}

static uint16_t st_sink(struct rte_graph *g, struct rte_node *n, void **objs, uint16_t nb) {
	(void)g;
	(void)n;
	for (uint16_t i = 0; i < nb && st_n_seen < 4 * ST_TOTAL; i++)
		st_seen[st_n_seen++] = (uintptr_t)objs[i];
	return nb;
}

static struct rte_node_register st_src_node = {
	.name = "st_src", .flags = RTE_NODE_SOURCE_F, .process = st_src, .nb_edges = 1, .next_nodes = {"st_split"}};
static struct rte_node_register st_split_node = {
	.name = "st_split", .process = st_split, .nb_edges = 2, .next_nodes = {"st_even", "st_odd"}};
static struct rte_node_register st_even_node = {
	.name = "st_even", .process = st_even, .nb_edges = 1, .next_nodes = {"st_sink"}};
static struct rte_node_register st_odd_node = {
	.name = "st_odd", .process = st_odd, .nb_edges = 1, .next_nodes = {"st_tag"}};
static struct rte_node_register st_tag_node = {
	.name = "st_tag", .process = st_tag, .nb_edges = 1, .next_nodes = {"st_sink"}};
static struct rte_node_register st_sink_node = {.name = "st_sink", .process = st_sink};
static struct rte_node_register st_bad_node = {
	.name = "st_bad", .process = st_sink, .nb_edges = 1, .next_nodes = {"st_missing"}};

static struct gr_node_info st_infos[] = {
	{.node = &st_src_node, .type = GR_NODE_T_L1},   {.node = &st_split_node, .type = GR_NODE_T_L2},
	{.node = &st_even_node, .type = GR_NODE_T_L2},  {.node = &st_odd_node, .type = GR_NODE_T_L2},   {.node = &st_tag_node, .type = GR_NODE_T_L2},
	{.node = &st_sink_node, .type = GR_NODE_T_L2}, {.node = &st_bad_node, .type = GR_NODE_T_L2},
};

int gh_graph_selftest(void) {
	static int registered;
	if (!registered) {
		for (size_t i = 0; i < sizeof(st_infos) / sizeof(st_infos[0]); i++)
			STAILQ_INSERT_TAIL(&node_infos, &st_infos[i], next);
		CHECK(gr_nodes_register() == 0);
		registered = 1;
	}
	// dynamic edges (gr_node_attach_parent): appended once, found again after
	rte_edge_t e = gr_node_attach_parent("st_split", "st_sink");
	CHECK(e == 2);
	CHECK(gr_node_attach_parent("st_split", "st_sink") == 2);
	CHECK(rte_node_edge_count(rte_node_from_name("st_split")) == 3);

	// a graph whose edge names no node is refused
	const char *bad[] = {"st_bad"};
	struct rte_graph_param pb = {.nb_node_patterns = 1, .node_patterns = bad};
	CHECK(rte_graph_create("st_bad_graph", &pb) == RTE_GRAPH_ID_INVALID);
	const char *none[] = {"no_such_node*"};
	struct rte_graph_param pn = {.nb_node_patterns = 1, .node_patterns = none};
	CHECK(rte_graph_create("st_none", &pn) == RTE_GRAPH_ID_INVALID);

	// the source pulls in every node reachable from it
	const char *pat[] = {"st_src"};
	struct rte_graph_param p = {.nb_node_patterns = 1, .node_patterns = pat};
	rte_graph_t id = rte_graph_create("st", &p);
	CHECK(id != RTE_GRAPH_ID_INVALID);
	CHECK(rte_graph_create("st", &p) == RTE_GRAPH_ID_INVALID); // names are unique
	struct rte_graph *g = rte_graph_lookup("st");
	CHECK(g != NULL && rte_graph_node_get_by_name("st", "st_sink") != NULL);
	CHECK(rte_graph_node_get_by_name("st", "st_bad") == NULL);

	st_next = 0;
	st_n_seen = 0;
	int walks = 0;
	while (st_next < ST_TOTAL && walks < 100) {
		rte_graph_walk(g);
		walks++;
	}
	CHECK(walks == (ST_TOTAL + ST_BURST - 1) / ST_BURST);
	CHECK(st_n_seen == ST_TOTAL); // every object reached the sink exactly once
	uint32_t even = 0, odd = 0;
	for (uint32_t i = 0; i < st_n_seen; i++) {
		if (st_seen[i] < 10000) {
			CHECK((st_seen[i] & 1) == 0);
			even++;
		} else {
			CHECK(((st_seen[i] - 10000) & 1) == 1);
			odd++;
		}
	}
	CHECK(even == ST_TOTAL / 2 && odd == ST_TOTAL / 2);
	// within a walk the pending nodes run in the order they became pending:
	// st_even (pending before st_odd) reaches the sink first, st_tag last
	CHECK(st_seen[0] == 2 && st_seen[ST_BURST / 2 - 1] == ST_BURST && st_seen[ST_BURST / 2] == 10001);

	const struct rte_node *src = rte_graph_node_get_by_name("st", "st_src");
	const struct rte_node *split = rte_graph_node_get_by_name("st", "st_split");
	const struct rte_node *oddn = rte_graph_node_get_by_name("st", "st_odd");
	const struct rte_node *evenn = rte_graph_node_get_by_name("st", "st_even");
	CHECK(src->total_calls == (uint64_t)walks && src->total_packets == ST_TOTAL);
	CHECK(split->total_calls == (uint64_t)walks && split->total_objs == ST_TOTAL);
	CHECK(evenn->total_packets == ST_TOTAL / 2); // it saw its own array every time
	CHECK(oddn->total_calls == (uint64_t)walks && oddn->total_objs == ST_TOTAL / 2);
	CHECK(oddn->total_packets == ST_TOTAL / 4);
	CHECK(rte_graph_destroy(id) == 0 && rte_graph_lookup("st") == NULL);
	return 0;
}

// ---- the QSBR stand-in (rte_rcu_min.c) -------------------------------------
#include <pthread.h>
#include <unistd.h>

static struct rte_rcu_qsbr *rs_v;
static volatile int rs_done;

static void *rs_sync(void *arg) {
	(void)arg;
	rte_rcu_qsbr_synchronize(rs_v, RTE_QSBR_THRID_INVALID);
	__atomic_store_n(&rs_done, 1, __ATOMIC_RELEASE);
	return NULL;
}

int gh_rcu_selftest(void) {
	const uint32_t n = 8;
	rs_v = aligned_alloc(64, (rte_rcu_qsbr_get_memsize(n) + 63) & ~(size_t)63);
	CHECK(rs_v != NULL && rte_rcu_qsbr_init(rs_v, n) == 0);
	CHECK(rte_rcu_qsbr_thread_register(rs_v, n) < 0); // ids below max_threads
	// registered readers start offline: nothing to wait for
	CHECK(rte_rcu_qsbr_thread_register(rs_v, 1) == 0 && rte_rcu_qsbr_thread_register(rs_v, 2) == 0);
	CHECK(rs_v->num_threads == 2);
	uint64_t t = rte_rcu_qsbr_start(rs_v);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 1);
	// an online reader holds a writer until it reports quiescent after it started
	rte_rcu_qsbr_thread_online(rs_v, 1);
	t = rte_rcu_qsbr_start(rs_v);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 0);
	rte_rcu_qsbr_quiescent(rs_v, 1);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 1);
	// ... or goes offline
	t = rte_rcu_qsbr_start(rs_v);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 0);
	rte_rcu_qsbr_thread_offline(rs_v, 1);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 1);
	// a reader coming online after the writer started holds nothing older
	t = rte_rcu_qsbr_start(rs_v);
	rte_rcu_qsbr_thread_online(rs_v, 2);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 1);
	// a reader that reported before the token is waited for
	rte_rcu_qsbr_quiescent(rs_v, 2);
	t = rte_rcu_qsbr_start(rs_v);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 0);
	// synchronize blocks until then, from another thread
	rs_done = 0;
	pthread_t th;
	CHECK(pthread_create(&th, NULL, rs_sync, NULL) == 0);
	usleep(20000);
	const int early = __atomic_load_n(&rs_done, __ATOMIC_ACQUIRE);
	rte_rcu_qsbr_quiescent(rs_v, 2);
	pthread_join(th, NULL);
	CHECK(early == 0 && rs_done == 1);
	// unregistered readers are not waited for, even when they were online
	t = rte_rcu_qsbr_start(rs_v);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 0);
	CHECK(rte_rcu_qsbr_thread_unregister(rs_v, 2) == 0 && rs_v->num_threads == 1);
	CHECK(rte_rcu_qsbr_check(rs_v, t, false) == 1);
	// synchronize from a reader reports its own quiescent state first
	rte_rcu_qsbr_thread_online(rs_v, 1);
	rte_rcu_qsbr_synchronize(rs_v, 1);
	free(rs_v);
	rs_v = NULL;
	return 0;
}
