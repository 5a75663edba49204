// SPDX-License-Identifier: BSD-3-Clause
//
// rte_graph_min.c -- the graph runtime behind rte_graph_min.h: a process-wide
// node registry, graphs built from name patterns, and the walk. See the
// header for which rte_graph semantics are kept.
#include "rte_graph_min.h"

#include <errno.h>
#include <fnmatch.h>
#include <stdio.h>
#include <stdlib.h>

#define MAX_NODES 1024
#define MAX_GRAPHS 64

struct node_def {
	char name[RTE_NODE_NAMESIZE];
	uint64_t flags;
	rte_node_process_t process;
	rte_node_init_t init;
	rte_node_fini_t fini;
	char **edges; // names
	rte_edge_t nb_edges;
};

// A graph's memory is its worker's alone (DPDK allocates each graph in one
// cache-aligned memzone, graph_populate.c): every allocation of a graph on
// whole 128-byte line pairs, so that no line a walk writes (node counters,
// object arrays, the pending list) is shared with another worker's graph.
#define GRAPH_LINE 128

static void *graph_zalloc(size_t n) {
	const size_t sz = (n + GRAPH_LINE - 1) / GRAPH_LINE * GRAPH_LINE;
	void *p = aligned_alloc(GRAPH_LINE, sz ? sz : GRAPH_LINE);
	if (p != NULL)
		memset(p, 0, sz ? sz : GRAPH_LINE);
	return p;
}

static struct node_def defs[MAX_NODES];
static rte_node_t n_defs;

struct rte_graph_priv {
	uint32_t n_nodes;
	struct rte_node **nodes; // instances, by position
	int32_t *inst_of; // [MAX_NODES]: node id -> position, -1 if absent
	struct rte_node **pending; // FIFO of nodes holding objects
	uint32_t pend_head, pend_tail, pend_cap;
};

static struct rte_graph *graphs[MAX_GRAPHS];

rte_node_t __rte_node_register(const struct rte_node_register *reg) {
	if (reg == NULL || reg->name[0] == '\0' || reg->process == NULL || n_defs >= MAX_NODES)
		return RTE_NODE_ID_INVALID;
	if (rte_node_from_name(reg->name) != RTE_NODE_ID_INVALID)
		return RTE_NODE_ID_INVALID; // duplicate name (DPDK: EEXIST)
	struct node_def *d = &defs[n_defs];
	memset(d, 0, sizeof(*d));
	snprintf(d->name, sizeof(d->name), "%s", reg->name);
	d->flags = reg->flags;
	d->process = reg->process;
	d->init = reg->init;
	d->fini = reg->fini;
	if (reg->nb_edges) {
		d->edges = calloc(reg->nb_edges, sizeof(char *));
		if (d->edges == NULL)
			return RTE_NODE_ID_INVALID;
		for (rte_edge_t e = 0; e < reg->nb_edges; e++)
			d->edges[e] = strdup(reg->next_nodes[e] ? reg->next_nodes[e] : "");
		d->nb_edges = reg->nb_edges;
	}
	return n_defs++;
}

rte_node_t rte_node_from_name(const char *name) {
	for (rte_node_t i = 0; i < n_defs; i++)
		if (strcmp(defs[i].name, name) == 0)
			return i;
	return RTE_NODE_ID_INVALID;
}

const char *rte_node_id_to_name(rte_node_t id) {
	return id < n_defs ? defs[id].name : NULL;
}

rte_node_t rte_node_max_count(void) {
	return n_defs;
}

rte_edge_t rte_node_edge_update(rte_node_t id, rte_edge_t from, const char **next_nodes, uint16_t nb_edges) {
	if (id >= n_defs)
		return RTE_EDGE_ID_INVALID;
	struct node_def *d = &defs[id];
	if (from == RTE_EDGE_ID_INVALID)
		from = d->nb_edges;
	if (from > d->nb_edges)
		return RTE_EDGE_ID_INVALID;
	uint32_t need = (uint32_t)from + nb_edges;
	if (need > d->nb_edges) {
		char **e = realloc(d->edges, need * sizeof(char *));
		if (e == NULL)
			return RTE_EDGE_ID_INVALID;
		for (uint32_t i = d->nb_edges; i < need; i++)
			e[i] = NULL;
		d->edges = e;
	}
	for (uint16_t i = 0; i < nb_edges; i++) {
		free(d->edges[from + i]);
		d->edges[from + i] = strdup(next_nodes[i]);
	}
	if (need > d->nb_edges)
		d->nb_edges = (rte_edge_t)need;
	return d->nb_edges;
}

rte_edge_t rte_node_edge_count(rte_node_t id) {
	return id < n_defs ? defs[id].nb_edges : RTE_EDGE_ID_INVALID;
}

rte_edge_t rte_node_edge_get(rte_node_t id, char *next_nodes[]) {
	if (id >= n_defs)
		return RTE_EDGE_ID_INVALID;
	if (next_nodes != NULL)
		for (rte_edge_t e = 0; e < defs[id].nb_edges; e++)
			next_nodes[e] = defs[id].edges[e];
	return defs[id].nb_edges;
}

static void graph_free(struct rte_graph *g) {
	if (g == NULL)
		return;
	for (uint32_t i = 0; i < g->priv->n_nodes; i++) {
		struct rte_node *n = g->priv->nodes[i];
		if (n == NULL)
			continue;
		free(n->objs);
		free(n->nodes);
		free(n);
	}
	free(g->priv->nodes);
	free(g->priv->inst_of);
	free(g->priv->pending);
	free(g->priv);
	free(g);
}

static int add_node(struct rte_graph *g, rte_node_t id) {
	if (g->priv->inst_of[id] >= 0)
		return 0;
	struct rte_node *n = graph_zalloc(sizeof(*n));
	if (n == NULL)
		return -ENOMEM;
	g->priv->inst_of[id] = (int32_t)g->priv->n_nodes;
	g->priv->nodes[g->priv->n_nodes++] = n;
	const struct node_def *d = &defs[id];
	snprintf(n->name, sizeof(n->name), "%s", d->name);
	n->id = id;
	n->process = d->process;
	n->size = RTE_GRAPH_BURST_SIZE;
	n->objs = graph_zalloc(n->size * sizeof(void *));
	if (n->objs == NULL)
		return -ENOMEM;
	for (rte_edge_t e = 0; e < d->nb_edges; e++) { // every reachable node joins
		rte_node_t nx = rte_node_from_name(d->edges[e]);
		if (nx == RTE_NODE_ID_INVALID)
			return -ENOENT;
		int r = add_node(g, nx);
		if (r < 0)
			return r;
	}
	return 0;
}

rte_graph_t rte_graph_create(const char *name, struct rte_graph_param *prm) {
	if (name == NULL || prm == NULL || rte_graph_lookup(name) != NULL)
		return RTE_GRAPH_ID_INVALID;
	rte_graph_t id = 0;
	while (id < MAX_GRAPHS && graphs[id] != NULL)
		id++;
	if (id == MAX_GRAPHS)
		return RTE_GRAPH_ID_INVALID;
	struct rte_graph *g = graph_zalloc(sizeof(*g));
	if (g == NULL)
		return RTE_GRAPH_ID_INVALID;
	if ((g->priv = graph_zalloc(sizeof(*g->priv))) == NULL) {
		free(g);
		return RTE_GRAPH_ID_INVALID;
	}
	snprintf(g->name, sizeof(g->name), "%s", name);
	g->id = id;
	g->socket = prm->socket_id;
	g->priv->nodes = graph_zalloc(MAX_NODES * sizeof(*g->priv->nodes));
	g->priv->inst_of = graph_zalloc(MAX_NODES * sizeof(*g->priv->inst_of));
	g->priv->pend_cap = MAX_NODES + 1;
	g->priv->pending = graph_zalloc(g->priv->pend_cap * sizeof(*g->priv->pending));
	if (g->priv->nodes == NULL || g->priv->inst_of == NULL || g->priv->pending == NULL)
		goto fail;
	for (uint32_t i = 0; i < MAX_NODES; i++)
		g->priv->inst_of[i] = -1;
	for (uint16_t p = 0; p < prm->nb_node_patterns; p++) {
		int matched = 0;
		for (rte_node_t i = 0; i < n_defs; i++) {
			if (fnmatch(prm->node_patterns[p], defs[i].name, 0) != 0)
				continue;
			matched = 1;
			if (add_node(g, i) < 0)
				goto fail;
		}
		if (!matched)
			goto fail; // DPDK: a pattern must select at least one node
	}
	// resolve edges to instances, then init
	for (uint32_t i = 0; i < g->priv->n_nodes; i++) {
		struct rte_node *n = g->priv->nodes[i];
		const struct node_def *d = &defs[n->id];
		n->nb_edges = d->nb_edges;
		n->nodes = graph_zalloc((d->nb_edges ? d->nb_edges : 1) * sizeof(*n->nodes));
		if (n->nodes == NULL)
			goto fail;
		for (rte_edge_t e = 0; e < d->nb_edges; e++)
			n->nodes[e] = g->priv->nodes[g->priv->inst_of[rte_node_from_name(d->edges[e])]];
	}
	for (uint32_t i = 0; i < g->priv->n_nodes; i++) {
		struct rte_node *n = g->priv->nodes[i];
		if (defs[n->id].init != NULL && defs[n->id].init(g, n) < 0)
			goto fail;
	}
	graphs[id] = g;
	return id;
fail:
	graph_free(g);
	return RTE_GRAPH_ID_INVALID;
}

int rte_graph_destroy(rte_graph_t id) {
	if (id >= MAX_GRAPHS || graphs[id] == NULL)
		return -ENOENT;
	struct rte_graph *g = graphs[id];
	for (uint32_t i = 0; i < g->priv->n_nodes; i++)
		if (defs[g->priv->nodes[i]->id].fini != NULL)
			defs[g->priv->nodes[i]->id].fini(g, g->priv->nodes[i]);
	graphs[id] = NULL;
	graph_free(g);
	return 0;
}

struct rte_graph *rte_graph_lookup(const char *name) {
	for (int i = 0; i < MAX_GRAPHS; i++)
		if (graphs[i] != NULL && strcmp(graphs[i]->name, name) == 0)
			return graphs[i];
	return NULL;
}

struct rte_node *rte_graph_node_get_by_name(const char *graph, const char *name) {
	struct rte_graph *g = rte_graph_lookup(graph);
	rte_node_t id = rte_node_from_name(name);
	if (g == NULL || id == RTE_NODE_ID_INVALID || g->priv->inst_of[id] < 0)
		return NULL;
	return g->priv->nodes[g->priv->inst_of[id]];
}

static void make_pending(struct rte_graph *g, struct rte_node *n) {
	if (n->pending)
		return;
	n->pending = 1;
	g->priv->pending[g->priv->pend_tail] = n;
	g->priv->pend_tail = (g->priv->pend_tail + 1) % g->priv->pend_cap;
}

// A node's stream holds at most UINT16_MAX objects (struct rte_node size /
// idx are uint16_t; DPDK's __rte_node_stream_alloc_size grows the stream to
// at most that and verifies it is not already there): more aborts.
static int grow(struct rte_node *n, uint32_t need) {
	if (need <= n->size)
		return 0;
	if (need > UINT16_MAX)
		return -ENOSPC;
	uint32_t sz = n->size;
	while (sz < need)
		sz *= 2;
	if (sz > UINT16_MAX)
		sz = UINT16_MAX;
	void **o = graph_zalloc(sz * sizeof(void *));
	if (o == NULL)
		return -ENOMEM;
	memcpy(o, n->objs, n->idx * sizeof(void *));
	free(n->objs);
	n->objs = o;
	n->size = (uint16_t)sz;
	return 0;
}

static void enqueue(struct rte_graph *g, struct rte_node *node, rte_edge_t next, void **objs, uint16_t nb) {
	if (next >= node->nb_edges || node->nodes[next] == node) {
		fprintf(stderr, "rte_graph_min: %s: bad edge %u (%u edges)\n", node->name, next, node->nb_edges);
		abort(); // a programming error, as DPDK's RTE_ASSERT
	}
	struct rte_node *to = node->nodes[next];
	if (grow(to, (uint32_t)to->idx + nb) < 0) {
		fprintf(stderr, "rte_graph_min: %s: cannot hold %u objects\n", to->name, to->idx + nb);
		abort();
	}
	memcpy(&to->objs[to->idx], objs, nb * sizeof(void *));
	to->idx += nb;
	if (to->idx > to->max_idx)
		to->max_idx = to->idx;
	make_pending(g, to);
}

void rte_standin_node_enqueue_x1(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void *obj) {
	enqueue(graph, node, next, &obj, 1);
}

void rte_standin_node_enqueue(struct rte_graph *graph, struct rte_node *node, rte_edge_t next, void **objs,
		      uint16_t nb_objs) {
	if (nb_objs)
		enqueue(graph, node, next, objs, nb_objs);
}

// DPDK swaps the object arrays when the destination is empty; copying is
// equivalent for the caller (the source keeps no objects afterwards).
void rte_node_next_stream_move(struct rte_graph *graph, struct rte_node *src, rte_edge_t next) {
	uint16_t nb = src->idx;
	src->idx = 0;
	if (nb)
		enqueue(graph, src, next, src->objs, nb);
}

static void run(struct rte_graph *g, struct rte_node *n) {
	const uint16_t nb = n->idx;
	const uint16_t ret = n->process(g, n, n->objs, nb);
	n->idx = 0; // whatever process() did not move is consumed
	n->total_calls++;
	n->total_objs += nb;
	n->total_packets += ret;
}

void rte_standin_graph_walk(struct rte_graph *g) {
	for (uint32_t i = 0; i < g->priv->n_nodes; i++) { // sources first
		struct rte_node *n = g->priv->nodes[i];
		if (defs[n->id].flags & RTE_NODE_SOURCE_F) {
			uint16_t ret = n->process(g, n, NULL, 0);
			n->total_calls++;
			n->total_packets += ret;
		}
	}
	while (g->priv->pend_head != g->priv->pend_tail) {
		struct rte_node *n = g->priv->pending[g->priv->pend_head];
		g->priv->pend_head = (g->priv->pend_head + 1) % g->priv->pend_cap;
		n->pending = 0;
		if (n->idx)
			run(g, n);
	}
}
