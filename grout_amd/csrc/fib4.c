// SPDX-License-Identifier: BSD-3-Clause
//
// fib4.c -- RIB trie + DIR24_8-equivalent painter (see fib4.h).
//
// Every change (add, replace, delete) re-paints only the table entries under
// the changed prefix: walking the trie below it, each /24 slot gets either a
// direct entry (no more-specific route inside it) or a tbl8 group painted
// from the trie down to /32. Empty groups are returned to a free list. The
// result equals a from-scratch longest-prefix-match build, which is what
// DPDK's dir24_8 maintains incrementally for grout (rte_fib_add,
// modules/ip/control/route.c:243,689).
#include "fib4.h"

#include <errno.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

#define NIL 0u // child == 0: no child (node 0 is the root, never a child)
#define NONE UINT32_MAX // "no node" for the painters, which may start at the root
#define DIRTY_CAP 4096 // tbl24 ranges tracked before the closest ones are merged

struct node {
	uint32_t child[2];
	uint32_t nh; // route on this exact prefix (0 = none)
	uint32_t n_routes; // routes in this subtree (this node included)
};

struct gr_fib4 {
	uint32_t max_routes, num_tbl8;
	struct node *nodes;
	uint32_t n_nodes, cap_nodes;
	uint32_t *free_nodes;
	uint32_t n_free_nodes, cap_free_nodes;
	uint32_t n_routes;
	uint32_t *tbl24; // GR_FIB4_TBL24_ENTRIES
	uint32_t *tbl8; // num_tbl8 * 256
	uint32_t *tbl8_free; // stack of free group indexes
	uint32_t tbl8_nfree;
	struct gr_fib4_range *dirty; // tbl24 index ranges touched, DIRTY_CAP at most
	uint32_t n_dirty;
	uint8_t *tbl8_dirty; // per group
	uint32_t *dirty_groups;
	uint32_t n_dirty_groups;
};

static uint32_t node_alloc(struct gr_fib4 *f) {
	if (f->n_free_nodes)
		return f->free_nodes[--f->n_free_nodes];
	if (f->n_nodes == f->cap_nodes) {
		uint32_t cap = f->cap_nodes ? f->cap_nodes * 2 : 1024;
		struct node *n = realloc(f->nodes, (size_t)cap * sizeof(*n));
		if (n == NULL)
			return NIL;
		f->nodes = n;
		f->cap_nodes = cap;
	}
	uint32_t i = f->n_nodes++;
	memset(&f->nodes[i], 0, sizeof(f->nodes[i]));
	return i;
}

static void node_release(struct gr_fib4 *f, uint32_t i) {
	if (f->n_free_nodes == f->cap_free_nodes) {
		uint32_t cap = f->cap_free_nodes ? f->cap_free_nodes * 2 : 1024;
		uint32_t *p = realloc(f->free_nodes, (size_t)cap * sizeof(*p));
		if (p == NULL)
			return; // leak the node slot, harmless
		f->free_nodes = p;
		f->cap_free_nodes = cap;
	}
	memset(&f->nodes[i], 0, sizeof(f->nodes[i]));
	f->free_nodes[f->n_free_nodes++] = i;
}

struct gr_fib4 *gr_fib4_new(uint32_t max_routes, uint32_t num_tbl8) {
	if (num_tbl8 == 0 || num_tbl8 > (GR_FIB4_EXT >> 8))
		return NULL;
	struct gr_fib4 *f = calloc(1, sizeof(*f));
	if (f == NULL)
		return NULL;
	f->max_routes = max_routes ? max_routes : UINT32_MAX;
	f->num_tbl8 = num_tbl8;
	f->tbl24 = calloc(GR_FIB4_TBL24_ENTRIES, sizeof(uint32_t));
	f->tbl8 = calloc((size_t)num_tbl8 * 256, sizeof(uint32_t));
	f->tbl8_free = malloc((size_t)num_tbl8 * sizeof(uint32_t));
	f->tbl8_dirty = calloc(num_tbl8, 1);
	f->dirty_groups = malloc((size_t)num_tbl8 * sizeof(uint32_t));
	f->dirty = malloc(DIRTY_CAP * sizeof(*f->dirty));
	if (!f->tbl24 || !f->tbl8 || !f->tbl8_free || !f->tbl8_dirty || !f->dirty_groups || !f->dirty
	    || node_alloc(f) != 0) {
		gr_fib4_free(f);
		return NULL;
	}
	for (uint32_t g = 0; g < num_tbl8; g++) // pop lowest indexes first
		f->tbl8_free[g] = num_tbl8 - 1 - g;
	f->tbl8_nfree = num_tbl8;
	return f;
}

void gr_fib4_free(struct gr_fib4 *f) {
	if (f == NULL)
		return;
	free(f->nodes);
	free(f->free_nodes);
	free(f->tbl24);
	free(f->tbl8);
	free(f->tbl8_free);
	free(f->tbl8_dirty);
	free(f->dirty_groups);
	free(f->dirty);
	free(f);
}

static uint32_t mask_of(uint8_t len) {
	return len == 0 ? 0 : ~0u << (32 - len);
}

static int range_cmp(const void *a, const void *b) {
	const struct gr_fib4_range *x = a, *y = b;
	return x->lo < y->lo ? -1 : x->lo > y->lo;
}

// Sort the dirty ranges and merge those less than `gap` entries apart
// (gap 0: overlapping or adjacent ones only).
static void dirty_merge(struct gr_fib4 *f, uint32_t gap) {
	if (f->n_dirty < 2)
		return;
	qsort(f->dirty, f->n_dirty, sizeof(*f->dirty), range_cmp);
	uint32_t n = 0;
	for (uint32_t i = 1; i < f->n_dirty; i++) {
		struct gr_fib4_range *r = &f->dirty[n];
		if ((uint64_t)f->dirty[i].lo <= (uint64_t)r->hi + gap) {
			if (f->dirty[i].hi > r->hi)
				r->hi = f->dirty[i].hi;
		} else {
			f->dirty[++n] = f->dirty[i];
		}
	}
	f->n_dirty = n + 1;
}

// A painter wrote tbl24[lo, hi). Painting walks addresses upwards, so a
// range usually extends the last one; a full list is merged, exactly first,
// then over gaps 4x wider each pass until half of it is free again.
static void mark_tbl24(struct gr_fib4 *f, uint32_t lo, uint32_t hi) {
	if (f->n_dirty) {
		struct gr_fib4_range *r = &f->dirty[f->n_dirty - 1];
		if (lo <= r->hi && hi >= r->lo) {
			if (lo < r->lo)
				r->lo = lo;
			if (hi > r->hi)
				r->hi = hi;
			return;
		}
	}
	if (f->n_dirty == DIRTY_CAP) {
		uint32_t gap = 0;
		dirty_merge(f, gap);
		while (f->n_dirty > DIRTY_CAP / 2) {
			gap = gap ? gap * 4 : 16;
			dirty_merge(f, gap);
		}
	}
	f->dirty[f->n_dirty].lo = lo;
	f->dirty[f->n_dirty].hi = hi;
	f->n_dirty++;
}

static void mark_group(struct gr_fib4 *f, uint32_t g) {
	if (!f->tbl8_dirty[g]) {
		f->tbl8_dirty[g] = 1;
		f->dirty_groups[f->n_dirty_groups++] = g;
	}
}

// Paint tbl8 group g for the subtree `n` at depth `d` (24 < d <= 32)
// covering addresses [base, base + 2^(32-d)) of the /24 it belongs to.
static void paint8(struct gr_fib4 *f, uint32_t g, uint32_t n, uint8_t d, uint32_t base, uint32_t inh) {
	uint32_t *t = &f->tbl8[(size_t)g * 256];
	uint32_t lo = base & 0xff, cnt = 1u << (32 - d);
	if (n == NONE) {
		for (uint32_t i = 0; i < cnt; i++)
			t[lo + i] = inh;
		return;
	}
	const struct node *nd = &f->nodes[n];
	if (nd->nh)
		inh = nd->nh;
	if (d == 32 || nd->n_routes == (nd->nh != 0)) {
		for (uint32_t i = 0; i < cnt; i++)
			t[lo + i] = inh;
		return;
	}
	uint32_t c0 = nd->child[0] ? nd->child[0] : NONE, c1 = nd->child[1] ? nd->child[1] : NONE;
	paint8(f, g, c0, (uint8_t)(d + 1), base, inh);
	paint8(f, g, c1, (uint8_t)(d + 1), base | (1u << (31 - d)), inh);
}

static void group_release(struct gr_fib4 *f, uint32_t e) {
	if (e & GR_FIB4_EXT)
		f->tbl8_free[f->tbl8_nfree++] = e & ~GR_FIB4_EXT;
}

// Paint the tbl24 range of the subtree `n` at depth d (<= 24) covering
// [base, base + 2^(32-d)), with `inh` the nexthop inherited from above.
// Returns -ENOSPC if a tbl8 group was needed and none was free.
static int paint24(struct gr_fib4 *f, uint32_t n, uint8_t d, uint32_t base, uint32_t inh) {
	uint32_t lo = base >> 8, cnt = 1u << (24 - d);
	if (n != NONE && f->nodes[n].nh)
		inh = f->nodes[n].nh;
	bool leafish = n == NONE || f->nodes[n].n_routes == (f->nodes[n].nh != 0);
	if (leafish) { // nothing more specific below: flat range
		for (uint32_t i = 0; i < cnt; i++) {
			group_release(f, f->tbl24[lo + i]);
			f->tbl24[lo + i] = inh;
		}
		mark_tbl24(f, lo, lo + cnt);
		return 0;
	}
	const struct node *nd = &f->nodes[n];
	if (d < 24) {
		uint32_t c0 = nd->child[0] ? nd->child[0] : NONE, c1 = nd->child[1] ? nd->child[1] : NONE;
		int r = paint24(f, c0, (uint8_t)(d + 1), base, inh);
		if (r == 0)
			r = paint24(f, c1, (uint8_t)(d + 1), base | (1u << (31 - d)), inh);
		return r;
	}
	// d == 24 with more-specific routes below: needs a tbl8 group
	uint32_t e = f->tbl24[lo], g;
	if (e & GR_FIB4_EXT) {
		g = e & ~GR_FIB4_EXT;
	} else {
		if (f->tbl8_nfree == 0)
			return -ENOSPC;
		g = f->tbl8_free[--f->tbl8_nfree];
		f->tbl24[lo] = GR_FIB4_EXT | g;
		mark_tbl24(f, lo, lo + 1);
	}
	paint8(f, g, nd->child[0] ? nd->child[0] : NONE, 25, base, inh);
	paint8(f, g, nd->child[1] ? nd->child[1] : NONE, 25, base | 0x80, inh);
	mark_group(f, g);
	return 0;
}

// Re-paint everything under prefix (ip, len): find the deepest existing node
// on the path for the inherited nexthop, then paint.
static int repaint(struct gr_fib4 *f, uint32_t ip, uint8_t len) {
	uint32_t inh = 0, n = 0; // root
	uint8_t top = len < 24 ? len : 24;
	// walk down to depth `top` (the painting root)
	for (uint8_t d = 0; d < top; d++) {
		if (f->nodes[n].nh)
			inh = f->nodes[n].nh;
		n = f->nodes[n].child[(ip >> (31 - d)) & 1];
		if (n == NIL) { // path ends above: the range is flat under inh
			n = NONE;
			break;
		}
	}
	return paint24(f, n, top, ip & mask_of(top), inh);
}

static void recount(struct gr_fib4 *f, const uint32_t *path, int depth) {
	for (int i = depth; i >= 0; i--) {
		struct node *nd = &f->nodes[path[i]];
		uint32_t c = nd->nh != 0;
		if (nd->child[0])
			c += f->nodes[nd->child[0]].n_routes;
		if (nd->child[1])
			c += f->nodes[nd->child[1]].n_routes;
		nd->n_routes = c;
	}
}

int gr_fib4_add(struct gr_fib4 *f, uint32_t ip, uint8_t len, uint32_t nh, int replace) {
	if (len > 32 || nh == 0 || (nh & GR_FIB4_EXT))
		return -EINVAL;
	ip &= mask_of(len);
	uint32_t path[33];
	uint32_t n = 0;
	path[0] = 0;
	for (uint8_t d = 0; d < len; d++) {
		uint32_t b = (ip >> (31 - d)) & 1;
		uint32_t c = f->nodes[n].child[b];
		if (c == NIL) {
			c = node_alloc(f);
			if (c == NIL)
				return -ENOMEM;
			f->nodes[n].child[b] = c; // f->nodes may have moved: re-index
		}
		n = c;
		path[d + 1] = n;
	}
	uint32_t old = f->nodes[n].nh;
	if (old != 0 && !replace) {
		recount(f, path, len); // drop nothing, but keep counts right
		return -EEXIST;
	}
	if (old == 0 && f->n_routes >= f->max_routes) {
		recount(f, path, len);
		gr_fib4_del(f, ip, len); // prune the empty path
		return -ENOSPC;
	}
	f->nodes[n].nh = nh;
	recount(f, path, len);
	if (old == 0)
		f->n_routes++;
	int r = repaint(f, ip, len);
	if (r < 0) { // out of tbl8 groups: undo (like rte_fib_add failing)
		if (old == 0)
			gr_fib4_del(f, ip, len);
		else {
			f->nodes[n].nh = old;
			repaint(f, ip, len);
		}
	}
	return r;
}

int gr_fib4_del(struct gr_fib4 *f, uint32_t ip, uint8_t len) {
	if (len > 32)
		return -EINVAL;
	ip &= mask_of(len);
	uint32_t path[33];
	uint32_t n = 0;
	path[0] = 0;
	for (uint8_t d = 0; d < len; d++) {
		n = f->nodes[n].child[(ip >> (31 - d)) & 1];
		if (n == NIL)
			return -ENOENT;
		path[d + 1] = n;
	}
	bool had = f->nodes[n].nh != 0;
	f->nodes[n].nh = 0;
	recount(f, path, len);
	// prune empty branch
	for (int d = len; d > 0; d--) {
		struct node *nd = &f->nodes[path[d]];
		if (nd->n_routes || nd->child[0] || nd->child[1])
			break;
		uint32_t b = (ip >> (32 - d)) & 1;
		f->nodes[path[d - 1]].child[b] = NIL;
		node_release(f, path[d]);
	}
	if (!had)
		return -ENOENT;
	f->n_routes--;
	return repaint(f, ip, len);
}

uint32_t gr_fib4_lookup(const struct gr_fib4 *f, uint32_t ip) {
	uint32_t e = f->tbl24[ip >> 8];
	if (e & GR_FIB4_EXT)
		e = f->tbl8[(size_t)(e & ~GR_FIB4_EXT) * 256 + (ip & 0xff)];
	return e;
}

uint32_t gr_fib4_get(const struct gr_fib4 *f, uint32_t ip, uint8_t len) {
	if (len > 32)
		return 0;
	uint32_t n = 0;
	for (uint8_t d = 0; d < len; d++) {
		n = f->nodes[n].child[(ip >> (31 - d)) & 1];
		if (n == NIL)
			return 0;
	}
	return f->nodes[n].nh;
}

const uint32_t *gr_fib4_tbl24(const struct gr_fib4 *f) {
	return f->tbl24;
}
const uint32_t *gr_fib4_tbl8(const struct gr_fib4 *f) {
	return f->tbl8;
}
uint32_t gr_fib4_num_tbl8(const struct gr_fib4 *f) {
	return f->num_tbl8;
}
uint32_t gr_fib4_tbl8_used(const struct gr_fib4 *f) {
	return f->num_tbl8 - f->tbl8_nfree;
}
uint32_t gr_fib4_n_routes(const struct gr_fib4 *f) {
	return f->n_routes;
}

int gr_fib4_dirty_tbl24(struct gr_fib4 *f, struct gr_fib4_range *ranges, uint32_t max) {
	dirty_merge(f, 0);
	if (f->n_dirty > max)
		return -1;
	memcpy(ranges, f->dirty, (size_t)f->n_dirty * sizeof(*ranges));
	return (int)f->n_dirty;
}

int gr_fib4_dirty_tbl8(struct gr_fib4 *f, uint32_t *groups, uint32_t max) {
	if (f->n_dirty_groups > max)
		return -1;
	memcpy(groups, f->dirty_groups, (size_t)f->n_dirty_groups * sizeof(*groups));
	return (int)f->n_dirty_groups;
}

void gr_fib4_dirty_clear(struct gr_fib4 *f) {
	for (uint32_t i = 0; i < f->n_dirty_groups; i++)
		f->tbl8_dirty[f->dirty_groups[i]] = 0;
	f->n_dirty_groups = 0;
	f->n_dirty = 0;
}
