// SPDX-License-Identifier: BSD-3-Clause
//
// fib6.c -- the IPv6 RIB of one VRF and the multibit trie the kernel walks
// (see fib6.h). The RIB is an exact-prefix hash (rib6_insert_or_replace /
// rib6_delete semantics of modules/ip6/control/route.c:229-345: one nexthop
// per (prefix, length), replace on request). The trie is repainted from the
// RIB on commit, routes in ascending prefix length so that a longer prefix
// always overwrites a shorter one: a route ending in the first level paints
// its 2^(16-len) entries; a longer route walks (creating groups, each
// initialised with the entry it replaces, so shorter prefixes stay visible
// below it) to the group of its last byte and paints 2^(8-k) entries there.
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

struct gr_fib6 {
	struct rib6_ent *ht;
	uint32_t cap; // power of two
	uint32_t n_routes, n_tomb, max_routes;
	uint32_t *top; // GR_FIB6_TOP
	uint32_t *groups; // max_groups * GR_FIB6_GROUP
	uint32_t max_groups, n_groups, n_painted;
	struct gr_fib6_skip *skips; // max_groups: each replaces at least one group
	uint32_t n_skips;
	uint32_t *remap; // max_groups, compaction scratch
	uint8_t *live; // max_groups
	uint32_t max_slot;
	bool dirty;
	uint64_t generation;
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
	if (max_groups > GR_FIB6_IDX)
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
	f->top = calloc(GR_FIB6_TOP, sizeof(uint32_t));
	f->groups = malloc((size_t)max_groups * GR_FIB6_GROUP * sizeof(uint32_t));
	f->skips = malloc((size_t)max_groups * sizeof(*f->skips));
	f->remap = malloc((size_t)max_groups * sizeof(uint32_t));
	f->live = malloc(max_groups);
	if (!f->ht || !f->top || !f->groups || !f->skips || !f->remap || !f->live) {
		gr_fib6_free(f);
		return NULL;
	}
	return f;
}

void gr_fib6_free(gr_fib6_t *f) {
	if (f == NULL)
		return;
	free(f->ht);
	free(f->top);
	free(f->groups);
	free(f->skips);
	free(f->remap);
	free(f->live);
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
		if (e->nh != nh) {
			e->nh = nh;
			f->dirty = true;
		}
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
		f->dirty = true;
	}
	if (nh > f->max_slot)
		f->max_slot = nh;
	return 0;
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
	f->dirty = true;
	if (f->n_tomb > f->cap / 4)
		(void)ht_rehash(f); // a failed rehash only costs probe length
	return 0;
}

static int paint(gr_fib6_t *f, const struct rib6_ent *r) {
	const uint8_t *ip = r->ip;
	if (r->len <= 16) {
		uint32_t base = ((uint32_t)ip[0] << 8) | ip[1];
		uint32_t cnt = 1u << (16 - r->len);
		for (uint32_t i = 0; i < cnt; i++)
			f->top[base + i] = r->nh; // ascending order: never a group yet
		return 0;
	}
	uint32_t *e = &f->top[((uint32_t)ip[0] << 8) | ip[1]];
	unsigned consumed = 16, b = 2;
	for (;;) {
		if (!(*e & GR_FIB6_EXT)) {
			if (f->n_groups >= f->max_groups)
				return -ENOSPC;
			uint32_t g = f->n_groups++;
			uint32_t *grp = f->groups + (size_t)g * GR_FIB6_GROUP;
			for (int i = 0; i < GR_FIB6_GROUP; i++)
				grp[i] = *e;
			*e = GR_FIB6_EXT | g;
		}
		uint32_t *grp = f->groups + (size_t)(*e & ~GR_FIB6_EXT) * GR_FIB6_GROUP;
		if (r->len <= consumed + 8) {
			unsigned nb = r->len - consumed;
			uint32_t base = ip[b], cnt = 1u << (8 - nb);
			for (uint32_t i = 0; i < cnt; i++)
				grp[base + i] = r->nh;
			return 0;
		}
		e = &grp[ip[b]];
		b++;
		consumed += 8;
	}
}

// Path compression (bottom-up): a group whose entries all hold one leaf D
// but for one index x becomes a skip node {key x, child = entry x, miss D};
// a skip whose child is a skip with the same miss and room in its key
// absorbs it. Returns the entry that replaces `ent`.
static uint32_t compress(gr_fib6_t *f, uint32_t ent) {
	if (!(ent & GR_FIB6_EXT) || (ent & GR_FIB6_SKIP))
		return ent;
	uint32_t *grp = f->groups + (size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP;
	for (int i = 0; i < GR_FIB6_GROUP; i++)
		grp[i] = compress(f, grp[i]);
	// the leaf most entries hold: one of the first three
	uint32_t d = grp[0] == grp[1] || grp[0] == grp[2] ? grp[0] : grp[1];
	if (d & GR_FIB6_EXT)
		return ent;
	int x = -1;
	for (int i = 0; i < GR_FIB6_GROUP; i++) {
		if (grp[i] == d)
			continue;
		if (x >= 0)
			return ent; // two paths leave this group
		x = i;
	}
	if (x < 0)
		return d; // every entry the same leaf
	const uint32_t child = grp[x];
	if ((child & GR_FIB6_SKIP) && (child & GR_FIB6_EXT)) {
		struct gr_fib6_skip *k = &f->skips[child & GR_FIB6_IDX];
		if (k->miss == d && k->n < 7) { // prepend x to the child's key
			memmove(k->key + 1, k->key, k->n);
			k->key[0] = (uint8_t)x;
			k->n++;
			return child;
		}
	}
	struct gr_fib6_skip *k = &f->skips[f->n_skips];
	memset(k, 0, sizeof(*k));
	k->key[0] = (uint8_t)x;
	k->n = 1;
	k->child = child;
	k->miss = d;
	return GR_FIB6_EXT | GR_FIB6_SKIP | f->n_skips++;
}

static void mark(gr_fib6_t *f, uint32_t ent) {
	if (!(ent & GR_FIB6_EXT))
		return;
	if (ent & GR_FIB6_SKIP) {
		mark(f, f->skips[ent & GR_FIB6_IDX].child);
		return;
	}
	const uint32_t g = ent & GR_FIB6_IDX, slots = (ent & GR_FIB6_WIDE) ? GR_FIB6_GROUP : 1;
	for (uint32_t s = 0; s < slots; s++)
		f->live[g + s] = 1;
	for (uint32_t i = 0; i < slots * GR_FIB6_GROUP; i++)
		mark(f, f->groups[(size_t)g * GR_FIB6_GROUP + i]);
}

static uint32_t relink(const gr_fib6_t *f, uint32_t ent) {
	// a wide group's slots stay consecutive: all live, packed in order
	if ((ent & GR_FIB6_EXT) && !(ent & GR_FIB6_SKIP))
		return (ent & (GR_FIB6_EXT | GR_FIB6_WIDE)) | f->remap[ent & GR_FIB6_IDX];
	return ent;
}

// Group slots in the subtree of `ent`, counting stops at `cap`.
static uint32_t subtree_groups(const gr_fib6_t *f, uint32_t ent, uint32_t cap) {
	if (!(ent & GR_FIB6_EXT))
		return 0;
	if (ent & GR_FIB6_SKIP)
		return subtree_groups(f, f->skips[ent & GR_FIB6_IDX].child, cap);
	const uint32_t slots = (ent & GR_FIB6_WIDE) ? GR_FIB6_GROUP : 1;
	uint32_t n = slots;
	const uint32_t *e = f->groups + (size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP;
	for (uint32_t i = 0; i < slots * GR_FIB6_GROUP && n < cap; i++)
		n += subtree_groups(f, e[i], cap - n);
	return n;
}

// Level compression (top-down, entries at byte b): a group whose entries
// hold at least GR_FIB6_WIDE_MIN child groups and no skip node, at b <= 14,
// becomes a wide group: entry (x, y) = entry y of child x, or the group's
// own leaf at x repeated; so does a one-byte skip whose child group heads at
// least GR_FIB6_SKIP_WIDE_MIN groups. Stops quietly when the group capacity
// runs out.
static uint32_t widen(gr_fib6_t *f, uint32_t ent, unsigned b) {
	if (!(ent & GR_FIB6_EXT) || b >= 16)
		return ent;
	if (ent & GR_FIB6_SKIP) {
		struct gr_fib6_skip *k = &f->skips[ent & GR_FIB6_IDX];
		// a one-byte skip over a heavy subtree becomes a wide group: row
		// key = the child group, every other row the miss leaf (the skip's
		// test and the child's gather in one gather)
		if (k->n == 1 && b <= 14 && (k->child & GR_FIB6_EXT) && !(k->child & (GR_FIB6_SKIP | GR_FIB6_WIDE))
		    && f->n_groups + GR_FIB6_GROUP <= f->max_groups
		    && subtree_groups(f, k->child, GR_FIB6_SKIP_WIDE_MIN) >= GR_FIB6_SKIP_WIDE_MIN) {
			const uint32_t w = f->n_groups;
			f->n_groups += GR_FIB6_GROUP;
			uint32_t *W = f->groups + (size_t)w * GR_FIB6_GROUP;
			for (uint32_t i = 0; i < GR_FIB6_GROUP * GR_FIB6_GROUP; i++)
				W[i] = k->miss;
			uint32_t *row = W + (size_t)k->key[0] * GR_FIB6_GROUP;
			memcpy(row, f->groups + (size_t)(k->child & GR_FIB6_IDX) * GR_FIB6_GROUP, GR_FIB6_GROUP * sizeof(uint32_t));
			for (uint32_t i = 0; i < GR_FIB6_GROUP; i++)
				row[i] = widen(f, row[i], b + 2);
			return GR_FIB6_EXT | GR_FIB6_WIDE | w;
		}
		k->child = widen(f, k->child, b + k->n);
		return ent;
	}
	const uint32_t g = ent & GR_FIB6_IDX;
	uint32_t n_grp = 0, n_skip = 0;
	for (int i = 0; i < GR_FIB6_GROUP; i++) {
		const uint32_t e = f->groups[(size_t)g * GR_FIB6_GROUP + i];
		if (e & GR_FIB6_EXT)
			*((e & GR_FIB6_SKIP) ? &n_skip : &n_grp) += 1;
	}
	if (b <= 14 && n_skip == 0 && n_grp >= GR_FIB6_WIDE_MIN && f->n_groups + GR_FIB6_GROUP <= f->max_groups) {
		const uint32_t w = f->n_groups;
		f->n_groups += GR_FIB6_GROUP;
		const uint32_t *grp = f->groups + (size_t)g * GR_FIB6_GROUP;
		uint32_t *W = f->groups + (size_t)w * GR_FIB6_GROUP;
		for (int x = 0; x < GR_FIB6_GROUP; x++) {
			uint32_t *row = W + (size_t)x * GR_FIB6_GROUP;
			if (grp[x] & GR_FIB6_EXT)
				memcpy(row, f->groups + (size_t)(grp[x] & GR_FIB6_IDX) * GR_FIB6_GROUP,
				       GR_FIB6_GROUP * sizeof(uint32_t));
			else
				for (int y = 0; y < GR_FIB6_GROUP; y++)
					row[y] = grp[x];
		}
		for (uint32_t i = 0; i < GR_FIB6_GROUP * GR_FIB6_GROUP; i++)
			W[i] = widen(f, W[i], b + 2);
		return GR_FIB6_EXT | GR_FIB6_WIDE | w;
	}
	for (int i = 0; i < GR_FIB6_GROUP; i++) {
		uint32_t *e = &f->groups[(size_t)g * GR_FIB6_GROUP + i];
		*e = widen(f, *e, b + 1);
	}
	return ent;
}

// Pack the groups still referenced to the front.
static void pack(gr_fib6_t *f) {
	memset(f->live, 0, f->n_groups);
	for (uint32_t i = 0; i < GR_FIB6_TOP; i++)
		mark(f, f->top[i]);
	uint32_t n = 0;
	for (uint32_t g = 0; g < f->n_groups; g++)
		f->remap[g] = f->live[g] ? n++ : UINT32_MAX;
	for (uint32_t i = 0; i < GR_FIB6_TOP; i++)
		f->top[i] = relink(f, f->top[i]);
	for (uint32_t k = 0; k < f->n_skips; k++)
		f->skips[k].child = relink(f, f->skips[k].child);
	for (uint32_t g = 0; g < f->n_groups; g++) {
		if (!f->live[g])
			continue;
		uint32_t *src = f->groups + (size_t)g * GR_FIB6_GROUP;
		uint32_t *dst = f->groups + (size_t)f->remap[g] * GR_FIB6_GROUP; // never above src
		for (int i = 0; i < GR_FIB6_GROUP; i++)
			dst[i] = relink(f, src[i]);
	}
	f->n_groups = n;
}

// Path-compress, pack, level-compress, pack again.
static void compress_all(gr_fib6_t *f) {
	f->n_painted = f->n_groups;
	f->n_skips = 0;
	for (uint32_t i = 0; i < GR_FIB6_TOP; i++)
		f->top[i] = compress(f, f->top[i]);
	pack(f);
	for (uint32_t i = 0; i < GR_FIB6_TOP; i++)
		f->top[i] = widen(f, f->top[i], 2);
	pack(f);
}

int gr_fib6_build(gr_fib6_t *f) {
	if (f == NULL)
		return -EINVAL;
	if (!f->dirty)
		return 0;
	// counting sort of the live routes by prefix length
	uint32_t count[130] = {0};
	for (uint32_t i = 0; i < f->cap; i++)
		if (f->ht[i].used == 1)
			count[f->ht[i].len + 1]++;
	for (int l = 1; l < 130; l++)
		count[l] += count[l - 1];
	const struct rib6_ent **order = malloc((size_t)(f->n_routes ? f->n_routes : 1) * sizeof(*order));
	if (order == NULL)
		return -ENOMEM;
	for (uint32_t i = 0; i < f->cap; i++)
		if (f->ht[i].used == 1)
			order[count[f->ht[i].len]++] = &f->ht[i];
	memset(f->top, 0, GR_FIB6_TOP * sizeof(uint32_t));
	f->n_groups = 0;
	int ret = 0;
	for (uint32_t i = 0; i < f->n_routes && ret == 0; i++)
		ret = paint(f, order[i]);
	free(order);
	if (ret < 0)
		return ret;
	compress_all(f);
	f->dirty = false;
	f->generation++;
	return 0;
}

uint32_t gr_fib6_lookup(const gr_fib6_t *f, const uint8_t ip[16]) {
	uint32_t ent = f->top[((uint32_t)ip[0] << 8) | ip[1]];
	int b = 2;
	while (b < 16 && (ent & GR_FIB6_EXT)) {
		if (ent & GR_FIB6_SKIP) {
			const struct gr_fib6_skip *k = &f->skips[ent & GR_FIB6_IDX];
			const bool match = b + k->n <= 16 && memcmp(ip + b, k->key, k->n) == 0;
			ent = match ? k->child : k->miss;
			b += k->n;
		} else if (ent & GR_FIB6_WIDE) {
			ent = f->groups[(size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP + ((uint32_t)ip[b] << 8) + ip[b + 1]];
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
	return f->n_groups;
}
const struct gr_fib6_skip *gr_fib6_skips(const gr_fib6_t *f) {
	return f->skips;
}
uint32_t gr_fib6_skips_used(const gr_fib6_t *f) {
	return f->n_skips;
}
uint32_t gr_fib6_groups_painted(const gr_fib6_t *f) {
	return f->n_painted;
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

static int cmp_u32(const void *a, const void *b) {
	const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
	return x < y ? -1 : x > y;
}

static int cmp_run(const void *a, const void *b) { // (count, key) pairs: count descending, key ascending
	const uint32_t *x = a, *y = b;
	if (x[0] != y[0])
		return x[0] > y[0] ? -1 : 1;
	return x[1] < y[1] ? -1 : x[1] > y[1];
}

int gr_fib6_shortcuts(const gr_fib6_t *f, uint32_t *keys, uint32_t *ents, uint32_t max) {
	if (f == NULL || (max && (keys == NULL || ents == NULL)))
		return -EINVAL;
	uint32_t n = 0;
	uint32_t *k = malloc((size_t)(f->n_routes ? f->n_routes : 1) * sizeof(*k));
	if (k == NULL)
		return -ENOMEM;
	for (uint32_t i = 0; i < f->cap; i++) {
		const struct rib6_ent *r = &f->ht[i];
		if (r->used == 1 && r->len >= 32)
			k[n++] = (uint32_t)r->ip[0] | (uint32_t)r->ip[1] << 8 | (uint32_t)r->ip[2] << 16 | (uint32_t)r->ip[3] << 24;
	}
	qsort(k, n, sizeof(*k), cmp_u32);
	// (routes under the /32, key), busiest first
	uint32_t *runs = malloc((size_t)(n ? n : 1) * 2 * sizeof(*runs));
	if (runs == NULL) {
		free(k);
		return -ENOMEM;
	}
	uint32_t nr = 0;
	for (uint32_t i = 0; i < n;) {
		uint32_t j = i;
		while (j < n && k[j] == k[i])
			j++;
		runs[2 * nr] = j - i;
		runs[2 * nr + 1] = k[i];
		nr++;
		i = j;
	}
	qsort(runs, nr, 2 * sizeof(*runs), cmp_run);
	uint32_t out = 0;
	for (uint32_t i = 0; i < nr && out < max; i++) {
		const uint32_t key = runs[2 * i + 1];
		const uint8_t ip[4] = {key & 0xff, (key >> 8) & 0xff, (key >> 16) & 0xff, key >> 24};
		uint32_t ent = f->top[((uint32_t)ip[0] << 8) | ip[1]];
		int b = 2;
		bool ok = true;
		while (b < 4 && (ent & GR_FIB6_EXT)) {
			if (ent & GR_FIB6_SKIP) {
				const struct gr_fib6_skip *s = &f->skips[ent & GR_FIB6_IDX];
				if (b + s->n > 4) { // compares bytes past the key
					ok = false;
					break;
				}
				ent = memcmp(ip + b, s->key, s->n) == 0 ? s->child : s->miss;
				b += s->n;
			} else if (ent & GR_FIB6_WIDE) {
				if (b != 2) { // bytes 3 and 4
					ok = false;
					break;
				}
				ent = f->groups[(size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP + ((uint32_t)ip[2] << 8) + ip[3]];
				b = 4;
			} else {
				ent = f->groups[(size_t)(ent & GR_FIB6_IDX) * GR_FIB6_GROUP + ip[b++]];
			}
		}
		if (!ok || ent == 0)
			continue;
		keys[out] = key;
		ents[out] = ent;
		out++;
	}
	free(runs);
	free(k);
	return (int)out;
}
