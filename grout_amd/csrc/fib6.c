// SPDX-License-Identifier: BSD-3-Clause
//
// fib6.c -- the IPv6 RIB of one VRF and the multibit trie the kernel walks
// (see fib6.h), kept up to date route by route.
//
// The RIB is an exact-prefix hash (rib6_insert_or_replace / rib6_delete
// semantics of modules/ip6/control/route.c:229-345: one nexthop per (prefix,
// length), replace on request).
//
// Three layers, each updated incrementally, the way grout changes its
// rte_fib6 one route at a time (rte_fib6_add / rte_fib6_delete,
// modules/ip6/control/route.c:229-345):
//
//   1. the plain trie: a first level of 2^16 entries (address bytes 0-1) and
//      nodes of 256 entries per further byte, every entry a leaf (the
//      nexthop of the longest matching prefix, with that prefix's length) or
//      a child node. A route add paints the entries its prefix covers whose
//      leaf is not longer, a delete repaints the entries it painted with the
//      next longest covering route (DIR24_8's rule, byte by byte); both mark
//      the nodes they touch and their ancestors dirty. A node whose entries
//      all hold one leaf folds back into its parent.
//   2. compression, recomputed bottom-up for the dirty nodes only: a node
//      whose entries all hold one leaf is that leaf; all but one, a skip
//      ("the next bytes equal this key: continue, else this leaf"), merging
//      a child's skip of the same miss leaf (up to 7 key bytes).
//   3. the device image (top, 1 KiB group slots, 16-byte skip nodes),
//      materialised top-down along the dirty paths only, clean subtrees
//      keeping their slots: a node becomes a group slot, a skip node, or a
//      wide group of 256 consecutive slots indexed by two bytes when it holds
//      at least GR_FIB6_WIDE_MIN child groups and no skip (its children then
//      are its rows), or when it is a one-byte skip over a child heading at
//      least GR_FIB6_SKIP_WIDE_MIN groups. A wide group's rows keep one entry
//      per 2^s of the second byte when its children's entries only change at
//      multiples of 2^s there (their granularity: prefixes that end inside
//      that byte, as fib_inject's /42, /44 and /46 do): 2^(8-s) slots instead
//      of 256, so that a route's entry shares its lines with its neighbours'
//      instead of owning one. Every write compares, and the
//      slots, skips and first-level entries that changed form the dirty
//      lists a commit uploads (gr_fib6_dirty).
#include "fib6.h"

#include <errno.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

struct rib6_ent {
	uint8_t ip[16];
	uint8_t len;
	uint8_t used; // 0 free, 1 live, 2 deleted (tombstone)
	uint8_t _pad[2];
	uint32_t nh;
};

#define NO_NODE UINT32_MAX
#define REF 0x80000000u // a plain entry holding a child node (index in bits 0-30)

enum { CK_LEAF, CK_SKIP, CK_GROUP }; // compressed kind
enum { R_NONE, R_STANDALONE, R_ROWS, R_MERGED, R_RANGE }; // how the image holds a node
enum { OBJ_NONE, OBJ_SLOT, OBJ_RUN, OBJ_SKIP }; // what it owns in the image

struct node {
	uint32_t ent[GR_FIB6_GROUP]; // plain: leaf nexthop (bit 31 clear) or REF | child
	uint8_t dep[GR_FIB6_GROUP]; // the leaf's prefix length
	uint32_t parent; // NO_NODE: a first-level entry's child
	uint32_t pslot; // index in the parent (first-level index when parent is NO_NODE)
	uint8_t pos; // address byte its entries are indexed by (2..15)
	uint8_t dirty; // touched (or below a touched node) since the last build
	uint8_t live;
	// compression (layer 2)
	uint8_t ckind;
	uint8_t sk_n; // CK_SKIP: key bytes
	uint8_t sk_key[7];
	uint8_t role, obj;
	uint8_t gran; // its entries change only at multiples of 2^gran (0..8): a row may keep 1 per 2^gran
	uint8_t run_c; // OBJ_RUN: the run's size, 2^run_c slots
	uint8_t row_s; // R_ROWS: the shift of the wide group holding its row
	// range shape (leaves only, one run of rs_in over [rs_lo, rs_hi], rs_miss
	// elsewhere): a parent range group holds it in one 8-byte entry
	uint8_t rs_ok, rs_lo, rs_hi;
	uint32_t rs_in, rs_miss;
	uint16_t n_grp_ch, n_skip_ch; // children of kind CK_GROUP / CK_SKIP
	uint32_t cval; // CK_LEAF: the leaf; CK_SKIP: the miss leaf
	uint32_t chain; // CK_SKIP: past the key, a leaf or REF | node (the chain's end)
	uint32_t merged; // CK_SKIP: the child whose skip this one absorbed, or NO_NODE
	uint32_t cgroups; // group-kind nodes in its compressed subtree (saturating)
	// the device image (layer 3)
	uint32_t obj_idx; // slot, first slot of a run, or skip index
	uint32_t enc; // R_STANDALONE: the entry that stands for it
	uint32_t row_at; // R_ROWS: the first entry of its row in the groups array
};

struct u32vec {
	uint32_t *v;
	uint32_t n, cap;
};

static int vpush(struct u32vec *a, uint32_t x) {
	if (a->n == a->cap) {
		uint32_t c = a->cap ? 2 * a->cap : 256;
		uint32_t *v = realloc(a->v, (size_t)c * sizeof(*v));
		if (v == NULL)
			return -ENOMEM;
		a->v = v;
		a->cap = c;
	}
	a->v[a->n++] = x;
	return 0;
}

struct gr_fib6 {
	struct rib6_ent *ht;
	uint32_t cap; // power of two
	uint32_t n_routes, n_tomb, max_routes;
	uint32_t max_slot;
	// plain trie
	uint32_t ptop[GR_FIB6_TOP];
	uint8_t ptop_dep[GR_FIB6_TOP];
	struct node *nodes;
	uint32_t n_nodes_cap, n_nodes_hw, n_nodes_live;
	struct u32vec node_free;
	struct u32vec dirty_nodes[16]; // by position
	struct u32vec dirty_ptop; // first-level entries touched
	uint8_t *ptop_dirty; // GR_FIB6_TOP flags
	// the device image: top, group slots, skips (fib6.h encoding)
	uint32_t top[GR_FIB6_TOP];
	uint32_t *groups; // max_groups * GR_FIB6_GROUP
	struct gr_fib6_skip *skips; // max_groups
	uint32_t max_groups, slot_hw, slots_live, skip_hw, skips_live;
	struct u32vec slot_free, skip_free;
	struct u32vec run_free[9]; // free runs of 2^c slots, c = 1..8
	// what the builds since the last gr_fib6_dirty_clear changed in the image
	uint8_t *slot_dirty, *skip_dirty, *top_dirty;
	struct u32vec d_slots, d_skips, d_top;
	bool all_dirty; // everything (no upload yet)
	uint64_t generation;
	uint32_t marks; // image writes of the current build
};

static void mask6(uint8_t out[16], const uint8_t ip[16], uint8_t len) {
	for (int i = 0; i < 16; i++) {
		int bits = (int)len - 8 * i;
		uint8_t m = bits >= 8 ? 0xff : bits <= 0 ? 0 : (uint8_t)(0xff << (8 - bits));
		out[i] = ip[i] & m;
	}
}

static uint32_t hash6(const uint8_t ip[16], uint8_t len) {
	uint64_t a, b;
	memcpy(&a, ip, 8);
	memcpy(&b, ip + 8, 8);
	uint64_t h = (a * 0x9e3779b97f4a7c15ull) ^ (b + 0x632be59bd9b4e019ull + len);
	h ^= h >> 29;
	h *= 0xbf58476d1ce4e5b9ull;
	h ^= h >> 32;
	return (uint32_t)h;
}

// Slot of (ip, len): live entry, or the first free/tombstone slot when absent.
static struct rib6_ent *ht_find(const gr_fib6_t *f, const uint8_t ip[16], uint8_t len, bool *found) {
	uint32_t m = f->cap - 1, i = hash6(ip, len) & m;
	struct rib6_ent *first_free = NULL;
	for (uint32_t probe = 0; probe < f->cap; probe++, i = (i + 1) & m) {
		struct rib6_ent *e = &f->ht[i];
		if (e->used == 0) {
			*found = false;
			return first_free ? first_free : e;
		}
		if (e->used == 2) {
			if (!first_free)
				first_free = e;
			continue;
		}
		if (e->len == len && memcmp(e->ip, ip, 16) == 0) {
			*found = true;
			return e;
		}
	}
	*found = false;
	return first_free;
}

gr_fib6_t *gr_fib6_new(uint32_t max_routes, uint32_t max_groups) {
	if (max_routes == 0 || max_routes > (1u << 28))
		return NULL;
	if (max_groups == 0)
		max_groups = 1u << 16;
	if (max_groups > GR_FIB6_WIDE_IDX)
		return NULL;
	gr_fib6_t *f = calloc(1, sizeof(*f));
	if (f == NULL)
		return NULL;
	uint32_t cap = 16;
	while (cap < 2 * max_routes)
		cap <<= 1;
	f->cap = cap;
	f->max_routes = max_routes;
	f->max_groups = max_groups;
	f->ht = calloc(cap, sizeof(*f->ht));
	// zeroed on demand by the OS: only the slots in use are ever touched
	f->groups = calloc((size_t)max_groups * GR_FIB6_GROUP, sizeof(uint32_t));
	f->skips = calloc(max_groups, sizeof(*f->skips));
	f->slot_dirty = calloc(max_groups, 1);
	f->skip_dirty = calloc(max_groups, 1);
	f->top_dirty = calloc(GR_FIB6_TOP, 1);
	f->ptop_dirty = calloc(GR_FIB6_TOP, 1);
	f->all_dirty = true;
	if (!f->ht || !f->groups || !f->skips || !f->slot_dirty || !f->skip_dirty || !f->top_dirty || !f->ptop_dirty) {
		gr_fib6_free(f);
		return NULL;
	}
	return f;
}

void gr_fib6_free(gr_fib6_t *f) {
	if (f == NULL)
		return;
	free(f->ht);
	free(f->nodes);
	free(f->node_free.v);
	for (int i = 0; i < 16; i++)
		free(f->dirty_nodes[i].v);
	free(f->dirty_ptop.v);
	free(f->ptop_dirty);
	free(f->groups);
	free(f->skips);
	free(f->slot_free.v);
	for (int c = 0; c < 9; c++)
		free(f->run_free[c].v);
	free(f->skip_free.v);
	free(f->slot_dirty);
	free(f->skip_dirty);
	free(f->top_dirty);
	free(f->d_slots.v);
	free(f->d_skips.v);
	free(f->d_top.v);
	free(f);
}

static int ht_rehash(gr_fib6_t *f) { // drop tombstones
	struct rib6_ent *old = f->ht;
	f->ht = calloc(f->cap, sizeof(*f->ht));
	if (f->ht == NULL) {
		f->ht = old;
		return -ENOMEM;
	}
	for (uint32_t i = 0; i < f->cap; i++) {
		if (old[i].used != 1)
			continue;
		bool found;
		struct rib6_ent *e = ht_find(f, old[i].ip, old[i].len, &found);
		*e = old[i];
	}
	f->n_tomb = 0;
	free(old);
	return 0;
}

// ---- layer 1: the plain trie -----------------------------------------------

// Mark node n and its ancestors dirty, and the first-level entry above them.
static int touch(gr_fib6_t *f, uint32_t n) {
	while (n != NO_NODE) {
		struct node *x = &f->nodes[n];
		if (x->dirty)
			return 0; // its ancestors are already
		x->dirty = 1;
		if (vpush(&f->dirty_nodes[x->pos], n) < 0)
			return -ENOMEM;
		if (x->parent == NO_NODE) {
			n = x->pslot;
			break;
		}
		n = x->parent;
	}
	if (!f->ptop_dirty[n]) {
		f->ptop_dirty[n] = 1;
		if (vpush(&f->dirty_ptop, n) < 0)
			return -ENOMEM;
	}
	return 0;
}

static int touch_top(gr_fib6_t *f, uint32_t t) {
	if (f->ptop_dirty[t])
		return 0;
	f->ptop_dirty[t] = 1;
	return vpush(&f->dirty_ptop, t);
}

// A node under entry (parent, pslot) at position pos, every entry the leaf
// (nh, dep) it replaces. Returns its index or NO_NODE.
static uint32_t node_new(gr_fib6_t *f, uint32_t parent, uint32_t pslot, uint8_t pos, uint32_t nh, uint8_t dep) {
	uint32_t n;
	if (f->node_free.n) {
		n = f->node_free.v[--f->node_free.n];
	} else {
		if (f->n_nodes_hw == f->n_nodes_cap) {
			uint32_t c = f->n_nodes_cap ? 2 * f->n_nodes_cap : 1024;
			if (c > REF)
				return NO_NODE;
			struct node *v = realloc(f->nodes, (size_t)c * sizeof(*v));
			if (v == NULL)
				return NO_NODE;
			f->nodes = v;
			f->n_nodes_cap = c;
		}
		n = f->n_nodes_hw++;
	}
	struct node *x = &f->nodes[n];
	memset(x, 0, sizeof(*x));
	for (int i = 0; i < GR_FIB6_GROUP; i++)
		x->ent[i] = nh;
	memset(x->dep, dep, sizeof(x->dep));
	x->parent = parent;
	x->pslot = pslot;
	x->pos = pos;
	x->live = 1;
	x->ckind = CK_LEAF;
	x->cval = nh;
	x->merged = NO_NODE;
	f->n_nodes_live++;
	return n;
}

// Paint (nh, len) into entry i of node n when its leaf is not longer; into
// every entry of a child node the same way (DIR24_8's rule).
static int paint_entry(gr_fib6_t *f, uint32_t n, int i, uint8_t len, uint32_t nh) {
	struct node *x = &f->nodes[n];
	if (x->ent[i] & REF) {
		const uint32_t c = x->ent[i] & ~REF;
		for (int j = 0; j < GR_FIB6_GROUP; j++) {
			int r = paint_entry(f, c, j, len, nh);
			if (r < 0)
				return r;
		}
		return 0;
	}
	if (x->dep[i] > len || (x->dep[i] == len && x->ent[i] == nh))
		return 0;
	x->ent[i] = nh;
	x->dep[i] = len;
	return touch(f, n);
}

// Repaint, under entry i of node n, the leaves painted by a prefix of length
// len with (nh, dep) (a delete: the next longest covering route).
static int unpaint_entry(gr_fib6_t *f, uint32_t n, int i, uint8_t len, uint32_t nh, uint8_t dep) {
	struct node *x = &f->nodes[n];
	if (x->ent[i] & REF) {
		const uint32_t c = x->ent[i] & ~REF;
		for (int j = 0; j < GR_FIB6_GROUP; j++) {
			int r = unpaint_entry(f, c, j, len, nh, dep);
			if (r < 0)
				return r;
		}
		return 0;
	}
	if (x->dep[i] != len)
		return 0;
	x->ent[i] = nh;
	x->dep[i] = dep;
	return touch(f, n);
}

// The same at the first level.
static int paint_top(gr_fib6_t *f, uint32_t t, uint8_t len, uint32_t nh, bool del, uint32_t rnh, uint8_t rdep) {
	if (f->ptop[t] & REF) {
		const uint32_t c = f->ptop[t] & ~REF;
		for (int j = 0; j < GR_FIB6_GROUP; j++) {
			int r = del ? unpaint_entry(f, c, j, len, rnh, rdep) : paint_entry(f, c, j, len, nh);
			if (r < 0)
				return r;
		}
		return 0;
	}
	if (del) {
		if (f->ptop_dep[t] != len)
			return 0;
		f->ptop[t] = rnh;
		f->ptop_dep[t] = rdep;
	} else {
		if (f->ptop_dep[t] > len || (f->ptop_dep[t] == len && f->ptop[t] == nh))
			return 0;
		f->ptop[t] = nh;
		f->ptop_dep[t] = len;
	}
	return touch_top(f, t);
}

// Apply a route add (del false) or delete (del true, replaced by (rnh,
// rdep)) of ip/len to the plain trie.
static int apply(gr_fib6_t *f, const uint8_t ip[16], uint8_t len, uint32_t nh, bool del, uint32_t rnh, uint8_t rdep) {
	if (len <= 16) {
		const uint32_t base = ((uint32_t)ip[0] << 8) | ip[1], cnt = 1u << (16 - len);
		for (uint32_t t = base; t < base + cnt; t++) {
			int r = paint_top(f, t, len, nh, del, rnh, rdep);
			if (r < 0)
				return r;
		}
		return 0;
	}
	// down to the node of the prefix's last byte, creating nodes on the way
	// (a delete too: a leaf folded from several prefixes of one length and
	// nexthop unfolds, and only this prefix's range is repainted)
	const uint32_t t = ((uint32_t)ip[0] << 8) | ip[1];
	if (!(f->ptop[t] & REF)) {
		const uint32_t c = node_new(f, NO_NODE, t, 2, f->ptop[t], f->ptop_dep[t]);
		if (c == NO_NODE)
			return -ENOMEM;
		f->ptop[t] = REF | c;
		int r = touch(f, c);
		if (r < 0)
			return r;
	}
	uint32_t n = f->ptop[t] & ~REF;
	unsigned b = 2;
	while (len > 8 * (b + 1)) { // the prefix goes past this node's byte
		struct node *x = &f->nodes[n];
		const uint32_t i = ip[b];
		if (!(x->ent[i] & REF)) {
			const uint32_t c = node_new(f, n, i, (uint8_t)(b + 1), x->ent[i], x->dep[i]);
			if (c == NO_NODE)
				return -ENOMEM;
			x = &f->nodes[n]; // node_new may have moved the array
			x->ent[i] = REF | c;
			int r = touch(f, c);
			if (r < 0)
				return r;
		}
		n = f->nodes[n].ent[i] & ~REF;
		b++;
	}
	const unsigned k = len - 8 * b; // 1..8 bits of byte b
	const uint32_t base = ip[b] & (0xff00u >> k) & 0xff, cnt = 1u << (8 - k);
	for (uint32_t i = base; i < base + cnt; i++) {
		int r = del ? unpaint_entry(f, n, (int)i, len, rnh, rdep) : paint_entry(f, n, (int)i, len, nh);
		if (r < 0)
			return r;
	}
	return 0;
}

// The longest route covering ip with a prefix shorter than len: (nh, length),
// (0, 0) when none.
static void covering(const gr_fib6_t *f, const uint8_t ip[16], uint8_t len, uint32_t *nh, uint8_t *dep) {
	for (int l = (int)len - 1; l >= 0; l--) {
		uint8_t key[16];
		mask6(key, ip, (uint8_t)l);
		bool found;
		const struct rib6_ent *e = ht_find(f, key, (uint8_t)l, &found);
		if (found) {
			*nh = e->nh;
			*dep = (uint8_t)l;
			return;
		}
	}
	*nh = 0;
	*dep = 0;
}

int gr_fib6_add(gr_fib6_t *f, const uint8_t ip[16], uint8_t len, uint32_t nh, int replace) {
	if (f == NULL || ip == NULL || len > 128 || nh == 0 || nh >= GR_FIB6_EXT)
		return -EINVAL;
	uint8_t key[16];
	mask6(key, ip, len);
	bool found;
	struct rib6_ent *e = ht_find(f, key, len, &found);
	if (found) {
		if (!replace)
			return -EEXIST;
		if (e->nh == nh)
			return 0;
		e->nh = nh;
	} else {
		if (f->n_routes >= f->max_routes || e == NULL)
			return -ENOSPC;
		if (e->used == 2)
			f->n_tomb--;
		memcpy(e->ip, key, 16);
		e->len = len;
		e->nh = nh;
		e->used = 1;
		f->n_routes++;
	}
	if (nh > f->max_slot)
		f->max_slot = nh;
	return apply(f, key, len, nh, false, 0, 0);
}

int gr_fib6_del(gr_fib6_t *f, const uint8_t ip[16], uint8_t len) {
	if (f == NULL || ip == NULL || len > 128)
		return -EINVAL;
	uint8_t key[16];
	mask6(key, ip, len);
	bool found;
	struct rib6_ent *e = ht_find(f, key, len, &found);
	if (!found)
		return -ENOENT;
	e->used = 2;
	f->n_routes--;
	f->n_tomb++;
	if (f->n_tomb > f->cap / 4)
		(void)ht_rehash(f); // a failed rehash only costs probe length
	uint32_t rnh;
	uint8_t rdep;
	covering(f, key, len, &rnh, &rdep);
	return apply(f, key, len, 0, true, rnh, rdep);
}

// ---- layer 3 storage: slots, runs of 256 slots, skips ----------------------

static int mark_slot(gr_fib6_t *f, uint32_t s) {
	f->marks++;
	if (f->slot_dirty[s])
		return 0;
	f->slot_dirty[s] = 1;
	return vpush(&f->d_slots, s);
}

static int mark_skip(gr_fib6_t *f, uint32_t k) {
	f->marks++;
	if (f->skip_dirty[k])
		return 0;
	f->skip_dirty[k] = 1;
	return vpush(&f->d_skips, k);
}

static int put_top(gr_fib6_t *f, uint32_t t, uint32_t v) {
	if (f->top[t] == v)
		return 0;
	f->top[t] = v;
	f->marks++;
	if (f->top_dirty[t])
		return 0;
	f->top_dirty[t] = 1;
	return vpush(&f->d_top, t);
}

static inline int put(gr_fib6_t *f, uint32_t s, int i, uint32_t v) {
	uint32_t *p = &f->groups[(size_t)s * GR_FIB6_GROUP + i];
	if (*p == v)
		return 0;
	*p = v;
	return mark_slot(f, s);
}

// A free run of 2^c slots (c = 1..8), splitting a larger free one if need
// be (its other halves go back to their classes); -ENOSPC when none.
static int run_pop(gr_fib6_t *f, unsigned c, uint32_t *w) {
	unsigned k = c;
	while (k <= 8 && f->run_free[k].n == 0)
		k++;
	if (k > 8)
		return -ENOSPC;
	const uint32_t x = f->run_free[k].v[--f->run_free[k].n];
	for (unsigned j = k; j > c; j--)
		if (vpush(&f->run_free[j - 1], x + (1u << (j - 1))) < 0)
			return -ENOMEM;
	*w = x;
	return 0;
}

// A new slot: written whole this build, whatever the image held there.
static int slot_alloc(gr_fib6_t *f, uint32_t *s) {
	if (f->slot_free.n) {
		*s = f->slot_free.v[--f->slot_free.n];
	} else if (f->slot_hw < f->max_groups) {
		*s = f->slot_hw++;
	} else {
		uint32_t w; // break the smallest free run into single slots
		int r = run_pop(f, 1, &w);
		if (r < 0)
			return r;
		if ((r = vpush(&f->slot_free, w + 1)) < 0)
			return r;
		*s = w;
	}
	f->slots_live++;
	return mark_slot(f, *s);
}

static void slot_free(gr_fib6_t *f, uint32_t s) {
	memset(f->groups + (size_t)s * GR_FIB6_GROUP, 0, GR_FIB6_GROUP * sizeof(uint32_t));
	f->slots_live--;
	(void)vpush(&f->slot_free, s); // a failed push only leaks the slot
}

static bool run_available(const gr_fib6_t *f, unsigned c) {
	for (unsigned k = c; k <= 8; k++)
		if (f->run_free[k].n)
			return true;
	return f->slot_hw + (1u << c) <= f->max_groups;
}

// A run of 2^c consecutive slots (c = 1..8), every slot marked written.
static int run_alloc(gr_fib6_t *f, unsigned c, uint32_t *w) {
	const uint32_t len = 1u << c;
	if (run_pop(f, c, w) == 0) {
		// from a free run
	} else if (f->slot_hw + len <= f->max_groups) {
		*w = f->slot_hw;
		f->slot_hw += len;
	} else {
		return -ENOSPC;
	}
	f->slots_live += len;
	for (uint32_t k = 0; k < len; k++) {
		int r = mark_slot(f, *w + k);
		if (r < 0)
			return r;
	}
	return 0;
}

static void run_free(gr_fib6_t *f, uint32_t w, unsigned c) {
	const uint32_t len = 1u << c;
	memset(f->groups + (size_t)w * GR_FIB6_GROUP, 0, (size_t)len * GR_FIB6_GROUP * sizeof(uint32_t));
	f->slots_live -= len;
	(void)vpush(&f->run_free[c], w);
}

static int skip_alloc(gr_fib6_t *f, uint32_t *k) {
	if (f->skip_free.n)
		*k = f->skip_free.v[--f->skip_free.n];
	else if (f->skip_hw < f->max_groups)
		*k = f->skip_hw++;
	else
		return -ENOSPC;
	f->skips_live++;
	return mark_skip(f, *k);
}

static void skip_free(gr_fib6_t *f, uint32_t k) {
	memset(&f->skips[k], 0, sizeof(f->skips[k]));
	f->skips_live--;
	(void)vpush(&f->skip_free, k);
}

// Give back what node x owns in the image.
static void release(gr_fib6_t *f, struct node *x) {
	switch (x->obj) {
	case OBJ_SLOT:
		slot_free(f, x->obj_idx);
		break;
	case OBJ_RUN:
		run_free(f, x->obj_idx, x->run_c);
		break;
	case OBJ_SKIP:
		skip_free(f, x->obj_idx);
		break;
	}
	x->obj = OBJ_NONE;
}

// ---- layer 2: compression, bottom-up over the dirty nodes ------------------

// The compressed value of entry i of node x: a leaf, or a child node that
// compresses to a leaf, or REF | child.
static inline uint32_t cvalue(const gr_fib6_t *f, const struct node *x, int i) {
	const uint32_t e = x->ent[i];
	if (!(e & REF))
		return e;
	const struct node *c = &f->nodes[e & ~REF];
	return c->ckind == CK_LEAF ? c->cval : e;
}

#define CGROUPS_MAX 0x3fffffffu

static void compress_node(gr_fib6_t *f, struct node *x) {
	uint32_t v0 = cvalue(f, x, 0), v1 = cvalue(f, x, 1), v2 = cvalue(f, x, 2);
	// the leaf most entries hold: one of the first three
	const uint32_t d = v0 == v1 || v0 == v2 ? v0 : v1;
	uint32_t n_grp = 0, n_skip = 0, groups = 0;
	int x_exc = -1, n_exc = 0;
	for (int i = 0; i < GR_FIB6_GROUP; i++) {
		const uint32_t e = x->ent[i];
		if (e & REF) {
			const struct node *c = &f->nodes[e & ~REF];
			n_grp += c->ckind == CK_GROUP;
			n_skip += c->ckind == CK_SKIP;
			groups += c->cgroups;
			if (groups > CGROUPS_MAX)
				groups = CGROUPS_MAX;
		}
		if (cvalue(f, x, i) != d) {
			x_exc = i;
			n_exc++;
		}
	}
	x->n_grp_ch = (uint16_t)n_grp;
	x->n_skip_ch = (uint16_t)n_skip;
	x->merged = NO_NODE;
	// granularity: the entries (as the image holds them: leaves, or a child
	// each) change only at multiples of 2^gran
	unsigned gran = 8;
	for (int i = 1; i < GR_FIB6_GROUP && gran; i++)
		if (x->ent[i] != x->ent[i - 1] || (x->ent[i] & REF)) {
			const unsigned tz = (unsigned)__builtin_ctz((unsigned)i);
			if (tz < gran)
				gran = tz;
		}
	if (x->ent[0] & REF)
		gran = 0;
	x->gran = (uint8_t)gran;
	// range shape: leaves that fit a range group's entry, V0 .. V1 .. V0
	// (at most two changes, the outer values equal), or V0 .. V1
	x->rs_ok = 0;
	{
		int nch = 0, ch[2] = {0, 0};
		bool ok = true;
		for (int i = 0; i < GR_FIB6_GROUP && ok; i++) {
			const uint32_t e = x->ent[i];
			ok = !(e & REF) && e <= GR_FIB6_RANGE_LEAF;
			if (ok && i && e != x->ent[i - 1]) {
				if (nch == 2)
					ok = false;
				else
					ch[nch++] = i;
			}
		}
		if (ok && nch == 2 && x->ent[0] != x->ent[GR_FIB6_GROUP - 1])
			ok = false;
		if (ok) {
			x->rs_ok = 1;
			x->rs_miss = x->ent[0];
			x->rs_in = nch ? x->ent[ch[0]] : x->ent[0];
			x->rs_lo = (uint8_t)(nch ? ch[0] : 0);
			x->rs_hi = (uint8_t)(nch == 2 ? ch[1] - 1 : 255);
		}
	}
	if ((d & REF) || n_exc > 1) {
		x->ckind = CK_GROUP;
		x->cgroups = groups + 1 > CGROUPS_MAX ? CGROUPS_MAX : groups + 1;
		return;
	}
	if (n_exc == 0) { // every entry the same leaf
		x->ckind = CK_LEAF;
		x->cval = d;
		x->cgroups = 0;
		return;
	}
	x->ckind = CK_SKIP;
	x->cval = d;
	x->sk_key[0] = (uint8_t)x_exc;
	x->sk_n = 1;
	const uint32_t e = cvalue(f, x, x_exc);
	x->chain = e;
	x->cgroups = 0;
	if (e & REF) {
		const uint32_t ci = e & ~REF;
		const struct node *c = &f->nodes[ci];
		if (c->ckind == CK_SKIP && c->cval == d && c->sk_n < 7) { // prepend x to the child's key
			memcpy(x->sk_key + 1, c->sk_key, c->sk_n);
			x->sk_n = (uint8_t)(c->sk_n + 1);
			x->chain = c->chain;
			x->merged = ci;
		}
		if (x->chain & REF)
			x->cgroups = f->nodes[x->chain & ~REF].cgroups;
	}
}

// A node whose entries all hold one leaf (same nexthop, same prefix length)
// folds into its parent's entry.
static bool fold(gr_fib6_t *f, uint32_t n) {
	struct node *x = &f->nodes[n];
	const uint32_t e0 = x->ent[0];
	const uint8_t d0 = x->dep[0];
	if (e0 & REF)
		return false;
	for (int i = 1; i < GR_FIB6_GROUP; i++)
		if (x->ent[i] != e0 || x->dep[i] != d0)
			return false;
	if (x->parent == NO_NODE) {
		f->ptop[x->pslot] = e0;
		f->ptop_dep[x->pslot] = d0;
	} else {
		struct node *p = &f->nodes[x->parent];
		p->ent[x->pslot] = e0;
		p->dep[x->pslot] = d0;
	}
	release(f, x);
	x->live = 0;
	f->n_nodes_live--;
	(void)vpush(&f->node_free, n);
	return true;
}

// ---- layer 3: materialisation, top-down along the dirty paths --------------

static int standalone(gr_fib6_t *f, uint32_t n, uint32_t *enc);

// The entry standing for plain entry e of a node at position pos - 1, i.e.
// at position pos.
static int entry_enc(gr_fib6_t *f, uint32_t e, uint32_t *enc) {
	if (!(e & REF)) {
		*enc = e;
		return 0;
	}
	return standalone(f, e & ~REF, enc);
}

static inline int put_at(gr_fib6_t *f, uint32_t e, uint32_t v) {
	return put(f, e / GR_FIB6_GROUP, (int)(e % GR_FIB6_GROUP), v);
}

// Node n's entries as they stand at its position, one per 2^sh (sh <= its
// granularity), from entry e of the groups array on (a group slot's content
// with sh 0, or a row of its parent's wide group).
static int rows_of(gr_fib6_t *f, uint32_t n, uint32_t e, unsigned sh) {
	for (uint32_t j = 0; j < ((uint32_t)GR_FIB6_GROUP >> sh); j++) {
		uint32_t v;
		int r = entry_enc(f, f->nodes[n].ent[j << sh], &v);
		if (r < 0)
			return r;
		if ((r = put_at(f, e + j, v)) < 0)
			return r;
	}
	return 0;
}

static int fill_row(gr_fib6_t *f, uint32_t e, unsigned sh, uint32_t leaf) {
	for (uint32_t j = 0; j < ((uint32_t)GR_FIB6_GROUP >> sh); j++) {
		int r = put_at(f, e + j, leaf);
		if (r < 0)
			return r;
	}
	return 0;
}

// Child node c becomes the row at entry e of a wide group of shift sh.
static int as_row(gr_fib6_t *f, uint32_t c, uint32_t e, unsigned sh) {
	struct node *x = &f->nodes[c];
	if (!x->dirty && x->role == R_ROWS && x->row_at == e && x->row_s == sh && !f->slot_dirty[e / GR_FIB6_GROUP])
		return 0; // unchanged (a slot written since the last upload may be a new run)
	release(f, x);
	x->role = R_ROWS;
	x->row_at = e;
	x->row_s = (uint8_t)sh;
	return rows_of(f, c, e, sh);
}

// Node x owns a slot, a skip node or a run of 2^c slots (OBJ_RUN).
static int own(gr_fib6_t *f, struct node *x, int obj, unsigned c, uint32_t *idx) {
	if (x->obj == obj && (obj != OBJ_RUN || x->run_c == c)) {
		*idx = x->obj_idx;
		return 0;
	}
	release(f, x);
	int r = obj == OBJ_SLOT ? slot_alloc(f, idx) : obj == OBJ_RUN ? run_alloc(f, c, idx) : skip_alloc(f, idx);
	if (r < 0)
		return r;
	x->obj = (uint8_t)obj;
	x->obj_idx = *idx;
	x->run_c = (uint8_t)(obj == OBJ_RUN ? c : 0);
	return 0;
}

// A wide entry: run w of shift sh.
static inline uint32_t wide_enc(uint32_t w, unsigned sh) {
	return GR_FIB6_EXT | GR_FIB6_WIDE | ((uint32_t)sh << GR_FIB6_WIDE_SHIFT) | w;
}

// The shift of node x as a wide group: the coarsest granularity all its child
// groups share (its leaf rows are constant, any shift suits them).
static unsigned wide_shift(const gr_fib6_t *f, const struct node *x) {
#ifdef FIB6_NO_NARROW // measurement builds (A/B)
	return 0;
#endif
	unsigned sh = 8;
	for (int k = 0; k < GR_FIB6_GROUP && sh; k++) {
		const uint32_t e = x->ent[k];
		if ((e & REF) && f->nodes[e & ~REF].ckind == CK_GROUP && f->nodes[e & ~REF].gran < sh)
			sh = f->nodes[e & ~REF].gran;
	}
	return sh == 8 ? 0 : sh; // (no child group: not a wide candidate)
}

// Node x as a range group: a group of leaves and children of range shape,
// one of them at least (fib6.h).
static bool range_ok(const gr_fib6_t *f, const struct node *x) {
#ifdef FIB6_NO_RANGE // measurement builds (A/B)
	return false;
#endif
	if (x->ckind != CK_GROUP || x->pos > 14)
		return false;
	int kids = 0;
	for (int k = 0; k < GR_FIB6_GROUP; k++) {
		const uint32_t e = x->ent[k];
		if (!(e & REF)) {
			if (e > GR_FIB6_RANGE_LEAF)
				return false;
			continue;
		}
		const struct node *c = &f->nodes[e & ~REF];
		if (c->ckind == CK_LEAF ? c->cval > GR_FIB6_RANGE_LEAF : !c->rs_ok)
			return false;
		kids += c->ckind != CK_LEAF;
	}
	return kids > 0;
}

// The entry that stands for node n at its position, its image written.
static int standalone(gr_fib6_t *f, uint32_t n, uint32_t *enc) {
	struct node *x = &f->nodes[n];
	if (!x->dirty && x->role == R_STANDALONE) {
		*enc = x->enc;
		return 0;
	}
	const unsigned b = x->pos;
	uint32_t idx, v;
	int r = 0;
	if (x->ckind == CK_LEAF) {
		release(f, x);
		v = x->cval;
	} else if (x->ckind == CK_SKIP) {
		const bool heavy = (x->chain & REF) && f->nodes[x->chain & ~REF].ckind == CK_GROUP
			&& f->nodes[x->chain & ~REF].cgroups >= GR_FIB6_SKIP_WIDE_MIN;
#ifdef FIB6_NO_NARROW
		const unsigned sh = 0, rc = 8;
#else
		const unsigned sh = heavy ? f->nodes[x->chain & ~REF].gran : 0, rc = 8 - sh;
#endif
		if (x->sk_n == 1 && b <= 14 && heavy
		    && ((x->obj == OBJ_RUN && x->run_c == rc) || run_available(f, rc))) {
			// a one-byte skip over a heavy subtree: one wide group, row key =
			// the child's entries, every other row the miss leaf
			if ((r = own(f, x, OBJ_RUN, rc, &idx)) < 0)
				return r;
			x = &f->nodes[n];
			const uint32_t key = x->sk_key[0], miss = x->cval, c = x->chain & ~REF;
			const uint32_t e0 = idx * GR_FIB6_GROUP, rl = GR_FIB6_GROUP >> sh;
			for (uint32_t k = 0; k < GR_FIB6_GROUP && r == 0; k++)
				r = k == key ? as_row(f, c, e0 + k * rl, sh) : fill_row(f, e0 + k * rl, sh, miss);
			if (r < 0)
				return r;
			v = wide_enc(idx, sh);
		} else {
			if ((r = own(f, x, OBJ_SKIP, 0, &idx)) < 0)
				return r;
			uint32_t child;
			if ((r = entry_enc(f, f->nodes[n].chain, &child)) < 0)
				return r;
			x = &f->nodes[n];
			struct gr_fib6_skip k;
			memset(&k, 0, sizeof(k));
			memcpy(k.key, x->sk_key, x->sk_n);
			k.n = x->sk_n;
			k.child = child;
			k.miss = x->cval;
			if (memcmp(&f->skips[idx], &k, sizeof(k)) != 0) {
				f->skips[idx] = k;
				if ((r = mark_skip(f, idx)) < 0)
					return r;
			}
			v = GR_FIB6_EXT | GR_FIB6_SKIP | idx;
			// the nodes whose skips this one absorbed own nothing
			for (uint32_t m = x->merged; m != NO_NODE;) {
				struct node *y = &f->nodes[m];
				release(f, y);
				y->role = R_MERGED;
				m = y->ckind == CK_SKIP ? y->merged : NO_NODE;
			}
		}
	} else if (range_ok(f, x) && ((x->obj == OBJ_RUN && x->run_c == 1) || run_available(f, 1))) {
		// range group: each entry folds a leaf, or a child's run and miss
		if ((r = own(f, x, OBJ_RUN, 1, &idx)) < 0)
			return r;
		const uint32_t e0 = idx * GR_FIB6_GROUP;
		for (uint32_t k = 0; k < GR_FIB6_GROUP && r == 0; k++) {
			const uint32_t e = f->nodes[n].ent[k];
			uint32_t in = e, miss = e, lo = 0, hi = 255;
			if (e & REF) {
				struct node *c = &f->nodes[e & ~REF];
				if (c->ckind == CK_LEAF) {
					in = miss = c->cval;
				} else {
					in = c->rs_in;
					miss = c->rs_miss;
					lo = c->rs_lo;
					hi = c->rs_hi;
				}
				release(f, c); // held in this entry, it owns nothing
				c->role = R_RANGE;
			}
			r = put_at(f, e0 + 2 * k, in | lo << 24);
			if (r == 0)
				r = put_at(f, e0 + 2 * k + 1, miss | hi << 24);
		}
		if (r < 0)
			return r;
		x = &f->nodes[n];
		v = GR_FIB6_EXT | GR_FIB6_RANGE | idx;
	} else if (b <= 14 && x->n_skip_ch == 0 && x->n_grp_ch >= GR_FIB6_WIDE_MIN
		   && ((x->obj == OBJ_RUN && x->run_c == 8 - wide_shift(f, x)) || run_available(f, 8 - wide_shift(f, x)))) {
		// wide: entry (k, y) = entry y of child k, or the leaf at k repeated;
		// one per 2^sh of y when every child group allows it
		const unsigned sh = wide_shift(f, x), rc = 8 - sh;
		if ((r = own(f, x, OBJ_RUN, rc, &idx)) < 0)
			return r;
		const uint32_t e0 = idx * GR_FIB6_GROUP, rl = GR_FIB6_GROUP >> sh;
		for (uint32_t k = 0; k < GR_FIB6_GROUP && r == 0; k++) {
			const uint32_t e = f->nodes[n].ent[k];
			if ((e & REF) && f->nodes[e & ~REF].ckind == CK_GROUP)
				r = as_row(f, e & ~REF, e0 + k * rl, sh);
			else
				r = fill_row(f, e0 + k * rl, sh, (e & REF) ? f->nodes[e & ~REF].cval : e);
		}
		if (r < 0)
			return r;
		v = wide_enc(idx, sh);
	} else {
		if ((r = own(f, x, OBJ_SLOT, 0, &idx)) < 0)
			return r;
		if ((r = rows_of(f, n, idx * GR_FIB6_GROUP, 0)) < 0)
			return r;
		v = GR_FIB6_EXT | idx;
	}
	x = &f->nodes[n];
	x->role = R_STANDALONE;
	x->enc = v;
	*enc = v;
	return 0;
}

// A build that stopped part way (no room for a group, a run or a skip, or no
// memory) has materialised some of the dirty paths and not others, and the
// nodes it re-owned may have left slots that entries it did not rewrite still
// name. Nothing of it is published (the commit fails), and the next build
// redoes all of it: every live node and every first-level entry dirty, the
// whole image to upload. Routes deleted meanwhile free the room it lacked.
static int dirty_all(gr_fib6_t *f) {
	for (uint32_t n = 0; n < f->n_nodes_hw; n++) {
		struct node *x = &f->nodes[n];
		if (!x->live || x->dirty)
			continue;
		x->dirty = 1;
		if (vpush(&f->dirty_nodes[x->pos], n) < 0)
			return -ENOMEM;
	}
	for (uint32_t t = 0; t < GR_FIB6_TOP; t++)
		if (touch_top(f, t) < 0)
			return -ENOMEM;
	f->all_dirty = true;
	return 0;
}

int gr_fib6_build(gr_fib6_t *f) {
	if (f == NULL)
		return -EINVAL;
	const uint32_t marks0 = f->marks;
	int r = 0;
	// layer 2: deepest first; nodes that fold away leave their parent dirty
	for (int pos = 15; pos >= 2; pos--) {
		struct u32vec *dl = &f->dirty_nodes[pos];
		for (uint32_t k = 0; k < dl->n; k++) {
			const uint32_t n = dl->v[k];
			if (!f->nodes[n].live || fold(f, n))
				continue;
			compress_node(f, &f->nodes[n]);
		}
	}
	// layer 3: from the first-level entries above dirty nodes
	for (uint32_t k = 0; k < f->dirty_ptop.n && r == 0; k++) {
		const uint32_t t = f->dirty_ptop.v[k];
		uint32_t v;
		r = entry_enc(f, f->ptop[t], &v);
		if (r == 0)
			r = put_top(f, t, v);
	}
	if (r < 0) { // keep everything dirty: the next build starts over
		const int e = dirty_all(f);
		return e < 0 ? e : r;
	}
	for (int pos = 2; pos < 16; pos++) {
		struct u32vec *dl = &f->dirty_nodes[pos];
		for (uint32_t k = 0; k < dl->n; k++)
			f->nodes[dl->v[k]].dirty = 0;
		dl->n = 0;
	}
	for (uint32_t k = 0; k < f->dirty_ptop.n; k++)
		f->ptop_dirty[f->dirty_ptop.v[k]] = 0;
	f->dirty_ptop.n = 0;
	if (f->marks != marks0)
		f->generation++;
	return r;
}

// ---- lookups and accessors ---------------------------------------------------

uint32_t gr_fib6_lookup(const gr_fib6_t *f, const uint8_t ip[16]) {
	uint32_t ent = f->top[((uint32_t)ip[0] << 8) | ip[1]];
	int b = 2;
	while (b < 16 && (ent & GR_FIB6_EXT)) {
		if ((ent & GR_FIB6_RANGE) == GR_FIB6_RANGE) {
			const uint32_t *q = f->groups + (size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP + 2 * ip[b];
			const uint32_t y = ip[b + 1];
			ent = y >= (q[0] >> 24) && y <= (q[1] >> 24) ? q[0] & GR_FIB6_RANGE_LEAF : q[1] & GR_FIB6_RANGE_LEAF;
			b += 2;
		} else if (ent & GR_FIB6_SKIP) {
			const struct gr_fib6_skip *k = &f->skips[ent & GR_FIB6_IDX];
			const bool match = b + k->n <= 16 && memcmp(ip + b, k->key, k->n) == 0;
			ent = match ? k->child : k->miss;
			b += k->n;
		} else if (ent & GR_FIB6_WIDE) {
			const unsigned sh = (ent >> GR_FIB6_WIDE_SHIFT) & 7;
			ent = f->groups[(size_t)(ent & GR_FIB6_WIDE_IDX) * GR_FIB6_GROUP + ((uint32_t)ip[b] << (8 - sh))
					+ (ip[b + 1] >> sh)];
			b += 2;
		} else {
			ent = f->groups[(size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP + ip[b++]];
		}
	}
	return ent & GR_FIB6_EXT ? 0 : ent;
}

uint32_t gr_fib6_lookup_rib(const gr_fib6_t *f, const uint8_t ip[16]) {
	for (int len = 128; len >= 0; len--) {
		uint8_t key[16];
		mask6(key, ip, (uint8_t)len);
		bool found;
		const struct rib6_ent *e = ht_find(f, key, (uint8_t)len, &found);
		if (found)
			return e->nh;
	}
	return 0;
}

const uint32_t *gr_fib6_top(const gr_fib6_t *f) {
	return f->top;
}
const uint32_t *gr_fib6_groups(const gr_fib6_t *f) {
	return f->groups;
}
uint32_t gr_fib6_groups_used(const gr_fib6_t *f) {
	return f->slot_hw;
}
uint32_t gr_fib6_groups_live(const gr_fib6_t *f) {
	return f->slots_live;
}
const struct gr_fib6_skip *gr_fib6_skips(const gr_fib6_t *f) {
	return f->skips;
}
uint32_t gr_fib6_skips_used(const gr_fib6_t *f) {
	return f->skip_hw;
}
uint32_t gr_fib6_groups_painted(const gr_fib6_t *f) {
	return f->n_nodes_live;
}
uint32_t gr_fib6_max_groups(const gr_fib6_t *f) {
	return f->max_groups;
}
uint32_t gr_fib6_n_routes(const gr_fib6_t *f) {
	return f->n_routes;
}
uint32_t gr_fib6_max_slot(const gr_fib6_t *f) {
	return f->max_slot;
}
uint64_t gr_fib6_generation(const gr_fib6_t *f) {
	return f->generation;
}

int gr_fib6_dirty(const gr_fib6_t *f, int kind, const uint32_t **list, uint32_t *n) {
	if (f == NULL || list == NULL || n == NULL)
		return -EINVAL;
	const struct u32vec *v = kind == GR_FIB6_DIRTY_TOP ? &f->d_top
		: kind == GR_FIB6_DIRTY_SLOTS             ? &f->d_slots
		: kind == GR_FIB6_DIRTY_SKIPS             ? &f->d_skips
							  : NULL;
	if (v == NULL)
		return -EINVAL;
	*list = v->v;
	*n = v->n;
	return f->all_dirty ? 1 : 0;
}

void gr_fib6_dirty_clear(gr_fib6_t *f) {
	for (uint32_t k = 0; k < f->d_top.n; k++)
		f->top_dirty[f->d_top.v[k]] = 0;
	for (uint32_t k = 0; k < f->d_slots.n; k++)
		f->slot_dirty[f->d_slots.v[k]] = 0;
	for (uint32_t k = 0; k < f->d_skips.n; k++)
		f->skip_dirty[f->d_skips.v[k]] = 0;
	f->d_top.n = f->d_slots.n = f->d_skips.n = 0;
	f->all_dirty = false;
}
