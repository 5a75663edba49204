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

// ---- lcores, RCU, iface counters -------------------------------------------
static __thread unsigned lcore_of_thread;

unsigned rte_lcore_id(void) {
	return lcore_of_thread;
}

void gr_test_lcore_set(unsigned lcore_id) {
	lcore_of_thread = lcore_id;
}

static struct iface_stats iface_stats_mem[MAX_IFACES][RTE_MAX_LCORE];
struct iface_stats (*iface_stats)[RTE_MAX_LCORE] = iface_stats_mem;

static struct rte_rcu_qsbr *rcu;

struct rte_rcu_qsbr *gr_datapath_rcu(void) {
	return rcu;
}

// ---- datapath hooks (the datapath patch's main_loop.c) -----------------------
static STAILQ_HEAD(, gr_datapath_hooks) hooks = STAILQ_HEAD_INITIALIZER(hooks);
static uint32_t hooks_readers;

void gr_datapath_hooks_register(struct gr_datapath_hooks *h) {
	h->rcu_base = RTE_MAX_LCORE + hooks_readers;
	hooks_readers += h->rcu_readers;
	STAILQ_INSERT_TAIL(&hooks, h, next);
}

uint32_t gr_datapath_hooks_readers(void) {
	return hooks_readers;
}

int gr_datapath_hooks_graph_leave(struct rte_graph *graph) {
	struct gr_datapath_hooks *h;
	int ret = 0;
	STAILQ_FOREACH(h, &hooks, next) {
		const int n = h->graph_leave != NULL ? h->graph_leave(graph) : 0;
		if (n < 0 && ret >= 0)
			ret = n;
		else if (n > 0 && ret >= 0)
			ret += n;
	}
	return ret;
}

void gr_datapath_hooks_stats_flush(const struct rte_graph *graph, unsigned lcore_id, gr_node_stats_cb_t cb,
				   void *cookie) {
	struct gr_datapath_hooks *h;
	STAILQ_FOREACH(h, &hooks, next)
		if (h->stats_flush != NULL)
			h->stats_flush(graph, lcore_id, cb, cookie);
}

uint64_t gr_datapath_hooks_holding(const struct rte_graph *graph) {
	struct gr_datapath_hooks *h;
	uint64_t held = 0;
	STAILQ_FOREACH(h, &hooks, next)
		if (h->holding != NULL)
			held += h->holding(graph);
	return held;
}

// grout's rcu module (main_loop.c:538-552) as the integration patch sizes
// it: the workers' lcore ids, then the hooks' readers.
static void rcu_init(struct event_base *ev) {
	(void)ev;
	const uint32_t n = RTE_MAX_LCORE + hooks_readers;
	rcu = aligned_alloc(64, (rte_rcu_qsbr_get_memsize(n) + 63) & ~(size_t)63);
	if (rcu == NULL || rte_rcu_qsbr_init(rcu, n) < 0)
		abort(); // grout: ABORT("rte_zmalloc(rcu)")
}

static void rcu_fini(struct event_base *ev) {
	(void)ev;
	free(rcu);
	rcu = NULL;
}

static struct module rcu_module = {
	.name = "rcu",
	.init = rcu_init,
	.fini = rcu_fini,
};

RTE_INIT(rcu_module_init) {
	module_register(&rcu_module);
}

static const struct iface *ifaces[MAX_IFACES];

const struct iface *iface_from_id(uint16_t id) {
	return id < MAX_IFACES ? __atomic_load_n(&ifaces[id], __ATOMIC_ACQUIRE) : NULL;
}

void gr_iface_register(struct iface *i) {
	if (i != NULL && i->id < MAX_IFACES)
		__atomic_store_n(&ifaces[i->id], i, __ATOMIC_RELEASE);
}

void gr_iface_unregister(uint16_t id) {
	if (id < MAX_IFACES)
		__atomic_store_n(&ifaces[id], NULL, __ATOMIC_RELEASE);
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

// ---- conntrack / NAT stand-ins (tests) -------------------------------------
#define MAX_CONNS 64
#define MAX_SNAT 64

static struct conn conns[MAX_CONNS];
static uint32_t n_conns;
static struct {
	uint16_t iface_id;
	ip4_addr_t from, to;
} snat_rules[MAX_SNAT];
static uint32_t n_snat;

void gr_test_policy_clear(void) {
	n_conns = 0;
	n_snat = 0;
}

int gr_test_conn_add(const struct conn_key *fwd, const struct conn_key *rev, struct conn **out) {
	if (n_conns == MAX_CONNS)
		return -ENOSPC;
	struct conn *c = &conns[n_conns++];
	c->fwd_key = *fwd;
	c->rev_key = *rev;
	if (out != NULL)
		*out = c;
	return 0;
}

int gr_test_snat44_static_add(uint16_t iface_id, ip4_addr_t from, ip4_addr_t to) {
	if (n_snat == MAX_SNAT)
		return -ENOSPC;
	snat_rules[n_snat].iface_id = iface_id;
	snat_rules[n_snat].from = from;
	snat_rules[n_snat].to = to;
	n_snat++;
	return 0;
}

// The key of an IPv4 packet's first fragment: iface, protocol, addresses
// and UDP ports (grout's gr_conn_parse_key also reads TCP ports and ICMP ids).
bool gr_conn_parse_key(const struct iface *iface, const addr_family_t af, const struct rte_mbuf *m,
		       struct conn_key *key) {
	const struct rte_ipv4_hdr *ip = rte_pktmbuf_mtod(m, const struct rte_ipv4_hdr *);
	if (af != GR_AF_IP4 || (rte_be_to_cpu_16(ip->fragment_offset) & RTE_IPV4_HDR_OFFSET_MASK) != 0)
		return false;
	memset(key, 0, sizeof(*key));
	key->iface_id = iface->id;
	key->af = af;
	key->proto = ip->next_proto_id;
	key->src = ip->src_addr;
	key->dst = ip->dst_addr;
	if (ip->next_proto_id == 17) { // IPPROTO_UDP
		const struct rte_udp_hdr *udp = rte_pktmbuf_mtod_offset(m, const struct rte_udp_hdr *,
									  rte_ipv4_hdr_len(ip));
		key->src_id = udp->src_port;
		key->dst_id = udp->dst_port;
	}
	return true;
}

static bool key_eq(const struct conn_key *a, const struct conn_key *b) {
	return a->iface_id == b->iface_id && a->af == b->af && a->proto == b->proto && a->src == b->src
		&& a->dst == b->dst && a->src_id == b->src_id && a->dst_id == b->dst_id;
}

struct conn *gr_conn_lookup(const struct conn_key *key, conn_flow_t *flow) {
	for (uint32_t i = 0; i < n_conns; i++) {
		if (key_eq(&conns[i].fwd_key, key)) {
			*flow = CONN_FLOW_FWD;
			return &conns[i];
		}
		if (key_eq(&conns[i].rev_key, key)) {
			*flow = CONN_FLOW_REV;
			return &conns[i];
		}
	}
	return NULL;
}

// One's-complement update of a checksum for a changed 32-bit field (RFC 1624
// eqn. 3, what grout's fixup_checksum_32 computes).
static rte_be16_t cksum_update32(rte_be16_t cksum, uint32_t from, uint32_t to) {
	uint32_t sum = (uint16_t)~cksum;
	sum += (uint16_t)~from + (uint16_t)~(from >> 16);
	sum += (to & 0xffff) + (to >> 16);
	sum = (sum & 0xffff) + (sum >> 16);
	sum = (sum & 0xffff) + (sum >> 16);
	return (rte_be16_t)~sum;
}

// snat44_process with static rules only: a packet whose source has a rule
// on the egress iface gets the translated source, its IPv4 checksum and a
// non-zero UDP checksum updated (FINAL); anything else CONTINUEs.
nat_verdict_t gr_standin_snat44_process(const struct iface *iface, struct rte_mbuf *m) {
	if (!(iface->flags & GR_IFACE_F_SNAT_STATIC))
		return NAT_VERDICT_CONTINUE;
	struct rte_ipv4_hdr *ip = rte_pktmbuf_mtod(m, struct rte_ipv4_hdr *);
	for (uint32_t i = 0; i < n_snat; i++) {
		if (snat_rules[i].iface_id != iface->id || snat_rules[i].from != ip->src_addr)
			continue;
		const ip4_addr_t to = snat_rules[i].to;
		ip->hdr_checksum = cksum_update32(ip->hdr_checksum, ip->src_addr, to);
		if ((rte_be_to_cpu_16(ip->fragment_offset) & RTE_IPV4_HDR_OFFSET_MASK) == 0 && ip->next_proto_id == 17) {
			struct rte_udp_hdr *udp = rte_pktmbuf_mtod_offset(m, struct rte_udp_hdr *, rte_ipv4_hdr_len(ip));
			if (udp->dgram_cksum != 0) {
				udp->dgram_cksum = cksum_update32(udp->dgram_cksum, ip->src_addr, to);
				if (udp->dgram_cksum == 0)
					udp->dgram_cksum = 0xffff;
			}
		}
		ip->src_addr = to;
		return NAT_VERDICT_FINAL;
	}
	return NAT_VERDICT_CONTINUE;
}

// A connection's table index + 1 (0: not one of the stand-in's connections),
// for the harness to decode conn_mbuf_data without dereferencing it.
uint32_t gr_test_conn_index(const struct conn *c) {
	if (c < conns || c >= conns + n_conns)
		return 0;
	return (uint32_t)(c - conns) + 1;
}
