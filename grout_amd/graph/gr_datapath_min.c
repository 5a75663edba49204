// SPDX-License-Identifier: BSD-3-Clause
//
// gr_datapath_min.c -- the grout-side registries behind gr_datapath_min.h:
// node infos and their registration pass, parent attachment, the drop
// node's process(), modules, and the iface / nexthop lookups.
#include "gr_datapath_min.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>

struct node_infos node_infos = STAILQ_HEAD_INITIALIZER(node_infos);

#define MAX_IFACES 1024
#define MAX_SLOTS (1u << 17)

static const struct iface *ifaces[MAX_IFACES];
static const struct nexthop **nexthops;

const struct iface *iface_from_id(uint16_t id) {
	return id < MAX_IFACES ? ifaces[id] : NULL;
}

void gr_iface_register(struct iface *i) {
	if (i != NULL && i->id < MAX_IFACES)
		ifaces[i->id] = i;
}

const struct nexthop *gr_nexthop_from_slot(uint32_t slot) {
	return (slot < MAX_SLOTS && nexthops != NULL) ? nexthops[slot] : NULL;
}

void gr_nexthop_register(struct nexthop *nh) {
	if (nh == NULL || nh->slot >= MAX_SLOTS)
		return;
	if (nexthops == NULL && (nexthops = calloc(MAX_SLOTS, sizeof(*nexthops))) == NULL)
		return;
	nexthops[nh->slot] = nh;
}

rte_edge_t gr_node_attach_parent(const char *parent, const char *node) {
	rte_node_t id = rte_node_from_name(parent);
	if (id == RTE_NODE_ID_INVALID) {
		fprintf(stderr, "'%s' parent node not found\n", parent);
		abort(); // grout: ABORT()
	}
	// already an edge: return it (rte_node_edge_update appends duplicates)
	rte_edge_t n = rte_node_edge_count(id);
	char **names = calloc(n ? n : 1, sizeof(char *));
	if (names == NULL)
		abort();
	rte_node_edge_get(id, names);
	for (rte_edge_t e = 0; e < n; e++)
		if (strcmp(names[e], node) == 0) {
			free(names);
			return e;
		}
	free(names);
	if (rte_node_edge_update(id, RTE_EDGE_ID_INVALID, &node, 1) == RTE_EDGE_ID_INVALID) {
		fprintf(stderr, "rte_node_edge_update(%s -> %s) failed\n", parent, node);
		abort();
	}
	return n;
}

// grout frees the mbufs (drop.c:13-30); the stand-in has no mempool to
// return them to, so its callers own them.
uint16_t drop_packets(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	(void)graph;
	(void)node;
	(void)objs;
	return nb_objs;
}

int gr_nodes_register(void) {
	struct gr_node_info *info;
	STAILQ_FOREACH(info, &node_infos, next) {
		if (rte_node_from_name(info->node->name) != RTE_NODE_ID_INVALID)
			continue; // registered by an earlier pass
		rte_node_t id = __rte_node_register(info->node);
		if (id == RTE_NODE_ID_INVALID)
			return -EINVAL;
		info->node->id = id;
	}
	STAILQ_FOREACH(info, &node_infos, next)
		if (info->register_callback != NULL)
			info->register_callback();
	return 0;
}

// ---- modules ---------------------------------------------------------------
STAILQ_HEAD(modules, module);
static struct modules modules = STAILQ_HEAD_INITIALIZER(modules);
#define MAX_MODULES 64
static struct module *inited[MAX_MODULES];
static int n_inited;

void module_register(struct module *m) {
	STAILQ_INSERT_TAIL(&modules, m, next);
}

static int is_inited(const char *name) {
	for (int i = 0; i < n_inited; i++)
		if (strcmp(inited[i]->name, name) == 0)
			return 1;
	return 0;
}

// Dependencies first (grout: modules_init, main/module.c): repeat passes over
// the modules whose dependency is initialised; a cycle or a missing
// dependency leaves modules behind and fails.
int gr_modules_init(struct event_base *ev) {
	int total = 0, progress = 1;
	struct module *m;
	STAILQ_FOREACH(m, &modules, next)
		total++;
	while (n_inited < total && progress) {
		progress = 0;
		STAILQ_FOREACH(m, &modules, next) {
			if (is_inited(m->name) || (m->depends_on != NULL && !is_inited(m->depends_on)))
				continue;
			if (n_inited == MAX_MODULES)
				return -ENOSPC;
			if (m->init != NULL)
				m->init(ev);
			inited[n_inited++] = m;
			progress = 1;
		}
	}
	return n_inited == total ? 0 : -ENOENT;
}

void gr_modules_fini(struct event_base *ev) {
	while (n_inited > 0) {
		struct module *m = inited[--n_inited];
		if (m->fini != NULL)
			m->fini(ev);
	}
}
