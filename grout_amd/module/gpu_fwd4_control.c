// SPDX-License-Identifier: BSD-3-Clause
//
// gpu_fwd4_control.c -- the fast path module's control-plane mirror
// (gpu_fwd4_control.h). grout's control thread calls the
// handlers below from its event dispatch; they convert grout's objects into
// the flat device mirrors of include/grout_hip.h and apply them to every GPU
// context through the node module's replicated calls (gpu_fwd4_*). The
// mirror also keeps what it pushed (a shadow), which serves the slot and
// reta bookkeeping, the tests, and the replay into a context that diverged.
//
// It includes grout's headers by their names (ip4.h / ip6.h / event.h / nexthop.h
// with integration/grout-gpu_fwd4-control.patch applied); here the include path
// leads them to the test stand-ins (tests/standin/include).
#include "gpu_fwd4_control.h"

#include "gpu_fwd4_node.h"

#include "event.h"
#include "iface.h"
#include "ip4.h"
#include "ip6.h"
#include "nexthop.h"
#include "port.h"
#include "vlan.h"
#include "vrf.h"

#include <event2/event.h>
#include <rte_common.h>
#include <rte_ether.h>

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

// ---- a small open-addressing hash: fixed-size keys -> uint32 ---------------
struct ht {
	uint32_t cap; // power of two, 0 = not allocated
	uint32_t n;
	uint32_t key_len;
	uint8_t *keys;
	uint32_t *vals;
	uint8_t *used;
};

static uint64_t ht_hash(const void *k, uint32_t len) {
	uint64_t h = 0xcbf29ce484222325ull; // FNV-1a, then a final mix
	for (uint32_t i = 0; i < len; i++)
		h = (h ^ ((const uint8_t *)k)[i]) * 0x100000001b3ull;
	h ^= h >> 33;
	h *= 0xff51afd7ed558ccdull;
	return h ^ (h >> 33);
}

static int ht_alloc(struct ht *t, uint32_t cap, uint32_t key_len) {
	struct ht n = {.cap = cap, .key_len = key_len};
	n.keys = calloc(cap, key_len);
	n.vals = calloc(cap, sizeof(uint32_t));
	n.used = calloc(cap, 1);
	if (n.keys == NULL || n.vals == NULL || n.used == NULL) {
		free(n.keys);
		free(n.vals);
		free(n.used);
		return -ENOMEM;
	}
	*t = n;
	return 0;
}

static void ht_free(struct ht *t) {
	free(t->keys);
	free(t->vals);
	free(t->used);
	memset(t, 0, sizeof(*t));
}

static int64_t ht_slot(const struct ht *t, const void *key) {
	if (t->cap == 0)
		return -1;
	for (uint32_t i = (uint32_t)ht_hash(key, t->key_len) & (t->cap - 1);; i = (i + 1) & (t->cap - 1)) {
		if (!t->used[i])
			return -1;
		if (memcmp(t->keys + (size_t)i * t->key_len, key, t->key_len) == 0)
			return i;
	}
}

static uint32_t *ht_find(const struct ht *t, const void *key) {
	const int64_t i = ht_slot(t, key);
	return i < 0 ? NULL : &t->vals[i];
}

static int ht_put(struct ht *t, const void *key, uint32_t val, uint32_t key_len) {
	uint32_t *v = ht_find(t, key);
	if (v != NULL) {
		*v = val;
		return 0;
	}
	if (t->cap == 0 || 2 * (t->n + 1) > t->cap) { // grow: load <= 1/2
		struct ht g;
		int r = ht_alloc(&g, t->cap ? 2 * t->cap : 64, key_len);
		if (r < 0)
			return r;
		for (uint32_t i = 0; i < t->cap; i++)
			if (t->used[i])
				ht_put(&g, t->keys + (size_t)i * key_len, t->vals[i], key_len);
		ht_free(t);
		*t = g;
	}
	uint32_t i = (uint32_t)ht_hash(key, key_len) & (t->cap - 1);
	while (t->used[i])
		i = (i + 1) & (t->cap - 1);
	t->used[i] = 1;
	memcpy(t->keys + (size_t)i * key_len, key, key_len);
	t->vals[i] = val;
	t->n++;
	return 0;
}

static void ht_del(struct ht *t, const void *key) { // linear probing: backward shift
	int64_t s = ht_slot(t, key);
	if (s < 0)
		return;
	uint32_t i = (uint32_t)s;
	t->used[i] = 0;
	t->n--;
	for (uint32_t j = (i + 1) & (t->cap - 1); t->used[j]; j = (j + 1) & (t->cap - 1)) {
		const uint32_t h = (uint32_t)ht_hash(t->keys + (size_t)j * t->key_len, t->key_len) & (t->cap - 1);
		// entry j may move to the hole i if its home h is not in (i, j]
		if (i <= j ? (h > i && h <= j) : (h > i || h <= j))
			continue;
		memcpy(t->keys + (size_t)i * t->key_len, t->keys + (size_t)j * t->key_len, t->key_len);
		t->vals[i] = t->vals[j];
		t->used[i] = 1;
		t->used[j] = 0;
		i = j;
	}
}

// ---- the mirror's state ----------------------------------------------------
struct route4_key {
	uint32_t ip; // network order, masked
	uint16_t vrf_id;
	uint8_t prefixlen;
	uint8_t _pad;
};
struct route6_key {
	uint8_t ip[16]; // masked
	uint16_t vrf_id;
	uint16_t iface_id; // scope of a link-local prefix, else 0
	uint8_t prefixlen;
	uint8_t _pad[3];
};
struct fib_conf {
	uint8_t on4, on6;
	struct gr_iface_info_vrf_fib v4, v6;
};

static struct {
	int ready;
	uint32_t max_nh, max_ifaces;
	struct ht slots; // struct nexthop * -> slot
	uint32_t *free_slots, n_free, next_slot; // slot allocator: recycled, then fresh
	struct gr_hip_nh *nh; // [max_nh + 1] what each slot holds
	struct gr_hip_iface *ifs; // [max_ifaces]
	uint8_t *if_live, *if_seen, *if_removing;
	uint32_t *reta; // [reta_top]
	uint32_t reta_top, reta_cap, reta_used;
	struct {
		uint32_t off, len;
	} *holes; // free reta ranges, by offset
	uint32_t n_holes, holes_cap;
	struct gr_hip_route4 *r4;
	uint32_t n_r4, cap_r4;
	struct ht k4; // route4_key -> index in r4
	struct gr_hip_route6 *r6;
	uint32_t n_r6, cap_r6;
	struct ht k6;
	struct fib_conf *fibs; // [max_ifaces] by VRF id
	// route changes applied to every context's RIB and not yet published
	// (see "publication" below)
	uint8_t *dirty4, *dirty6; // [max_ifaces] by VRF id
	uint32_t *nh_dirty, n_nh_dirty; // L3 nexthop slots whose mirror waits for the publication
	uint8_t *nh_is_dirty; // [max_nh + 1]
	uint32_t pending;
	struct event *flush_ev;
	int flush_armed;
	struct gpu_fwd4_control_stats st;
} M;

static struct event_base *ev_base; // the control thread's (gpu_fwd4_control_attach)
static void publish_cb(int fd, short what, void *arg);

static void note(int r) {
	// no GPU context at all (CPU tests): the shadow alone is kept
	if (r >= 0 || (r == -ENODEV && gpu_fwd4_n_ctx() == 0))
		return;
	if (M.st.errors++ == 0)
		M.st.first_error = r;
}

static int ready(void) {
	if (M.ready)
		return 0;
	struct gpu_fwd4_conf c;
	gpu_fwd4_conf_get(&c);
	M.max_nh = c.max_nexthops;
	M.max_ifaces = c.max_ifaces;
	M.free_slots = calloc(M.max_nh + 1, sizeof(uint32_t));
	M.nh = calloc(M.max_nh + 1, sizeof(*M.nh));
	M.ifs = calloc(M.max_ifaces, sizeof(*M.ifs));
	M.if_live = calloc(M.max_ifaces, 1);
	M.if_seen = calloc(M.max_ifaces, 1);
	M.if_removing = calloc(M.max_ifaces, 1);
	M.fibs = calloc(M.max_ifaces, sizeof(*M.fibs));
	M.dirty4 = calloc(M.max_ifaces, 1);
	M.dirty6 = calloc(M.max_ifaces, 1);
	M.nh_dirty = calloc(M.max_nh + 1, sizeof(uint32_t));
	M.nh_is_dirty = calloc(M.max_nh + 1, 1);
	if (M.free_slots == NULL || M.nh == NULL || M.ifs == NULL || M.if_live == NULL || M.if_seen == NULL
	    || M.if_removing == NULL || M.fibs == NULL || M.dirty4 == NULL || M.dirty6 == NULL || M.nh_dirty == NULL
	    || M.nh_is_dirty == NULL) {
		gpu_fwd4_control_reset();
		return -ENOMEM;
	}
	M.next_slot = 1;
	M.ready = 1;
	return 0;
}

void gpu_fwd4_control_reset(void) {
	ht_free(&M.slots);
	ht_free(&M.k4);
	ht_free(&M.k6);
	free(M.free_slots);
	free(M.nh);
	free(M.ifs);
	free(M.if_live);
	free(M.if_seen);
	free(M.if_removing);
	free(M.reta);
	free(M.holes);
	free(M.r4);
	free(M.r6);
	free(M.fibs);
	free(M.dirty4);
	free(M.dirty6);
	free(M.nh_dirty);
	free(M.nh_is_dirty);
	if (M.flush_ev != NULL)
		event_free(M.flush_ev);
	memset(&M, 0, sizeof(M));
}

// The publication timer lives on the control thread's event base: created
// here when the module's init passes it (and on first use after a reset),
// rebuilt when the base changes. With no base (events before the module's
// init) every change is published at once, counted in no_timer.
void gpu_fwd4_control_attach(struct event_base *ev) {
	if (ev == ev_base && (M.flush_ev != NULL || ev == NULL))
		return;
	if (M.flush_ev != NULL) { // on the old loop: publish what it waited for, then move
		gpu_fwd4_control_flush();
		event_free(M.flush_ev);
		M.flush_ev = NULL;
	}
	ev_base = ev;
	if (ev != NULL)
		M.flush_ev = evtimer_new(ev, publish_cb, NULL);
}

// ---- nexthop slots ---------------------------------------------------------
uint32_t gpu_fwd4_control_nh_slot(const struct nexthop *nh) {
	const uint32_t *s = nh != NULL ? ht_find(&M.slots, &nh) : NULL;
	return s != NULL ? *s : 0;
}

static uint32_t slot_get(const struct nexthop *nh) {
	uint32_t s = gpu_fwd4_control_nh_slot(nh);
	if (s != 0)
		return s;
	if (M.n_free > 0)
		s = M.free_slots[--M.n_free];
	else if (M.next_slot <= M.max_nh)
		s = M.next_slot++;
	else
		return 0;
	if (ht_put(&M.slots, &nh, s, sizeof(nh)) < 0) {
		M.free_slots[M.n_free++] = s;
		return 0;
	}
	M.st.slots_used++;
	return s;
}

static void slot_put(const struct nexthop *nh, uint32_t s) {
	ht_del(&M.slots, &nh);
	M.free_slots[M.n_free++] = s;
	M.st.slots_used--;
}

// ---- reta ranges: first fit over the holes, else the top -------------------
static int reta_alloc(uint32_t len, uint32_t *off) {
	for (uint32_t i = 0; i < M.n_holes; i++) {
		if (M.holes[i].len < len)
			continue;
		*off = M.holes[i].off;
		M.holes[i].off += len;
		M.holes[i].len -= len;
		if (M.holes[i].len == 0) {
			memmove(&M.holes[i], &M.holes[i + 1], (M.n_holes - i - 1) * sizeof(M.holes[0]));
			M.n_holes--;
		}
		M.reta_used += len;
		return 0;
	}
	if (M.reta_top + len > M.reta_cap) {
		uint32_t cap = M.reta_cap ? M.reta_cap : 4096;
		while (cap < M.reta_top + len)
			cap *= 2;
		uint32_t *r = realloc(M.reta, cap * sizeof(uint32_t));
		if (r == NULL)
			return -ENOMEM;
		memset(r + M.reta_cap, 0, (cap - M.reta_cap) * sizeof(uint32_t));
		M.reta = r;
		M.reta_cap = cap;
	}
	*off = M.reta_top;
	M.reta_top += len;
	M.reta_used += len;
	return 0;
}

static void reta_free(uint32_t off, uint32_t len) {
	if (len == 0)
		return;
	M.reta_used -= len;
	if (M.n_holes == M.holes_cap) {
		uint32_t cap = M.holes_cap ? 2 * M.holes_cap : 16;
		void *h = realloc(M.holes, cap * sizeof(M.holes[0]));
		if (h == NULL)
			return; // the range is lost to reuse, nothing worse
		M.holes = h;
		M.holes_cap = cap;
	}
	uint32_t i = 0;
	while (i < M.n_holes && M.holes[i].off < off)
		i++;
	memmove(&M.holes[i + 1], &M.holes[i], (M.n_holes - i) * sizeof(M.holes[0]));
	M.holes[i].off = off;
	M.holes[i].len = len;
	M.n_holes++;
	if (i + 1 < M.n_holes && M.holes[i].off + M.holes[i].len == M.holes[i + 1].off) { // merge right
		M.holes[i].len += M.holes[i + 1].len;
		memmove(&M.holes[i + 1], &M.holes[i + 2], (M.n_holes - i - 2) * sizeof(M.holes[0]));
		M.n_holes--;
	}
	if (i > 0 && M.holes[i - 1].off + M.holes[i - 1].len == M.holes[i].off) { // merge left
		M.holes[i - 1].len += M.holes[i].len;
		memmove(&M.holes[i], &M.holes[i + 1], (M.n_holes - i - 1) * sizeof(M.holes[0]));
		M.n_holes--;
	}
}

// ---- nexthops ----------------------------------------------------------------
// struct nexthop (nexthop.h:22-96) -> struct gr_hip_nh. A group's reta
// (struct nexthop *[reta_size], group_nexthop.c:27-56) becomes slots in a
// range of the contexts' reta table; the range is kept while the size is.
static void nh_changed(uint32_t slot);
static void nh_flush(void);

static int push_nh(uint32_t slot, const struct nexthop *nh) {
	if (nh->type != GR_NH_T_L3)
		nh_flush(); // the slots a group or a type nexthop may name are on every GPU first
	struct gr_hip_nh o;
	memset(&o, 0, sizeof(o));
	o.type = nh->type;
	o.iface_id = nh->iface_id;
	o.vrf_id = nh->vrf_id;
	const struct gr_hip_nh old = M.nh[slot];
	uint32_t new_off = 0, new_len = 0;
	int r = 0;
	if (nh->type == GR_NH_T_L3) {
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
		o.state = l3->state;
		o.flags = l3->flags;
		o.af = l3->af;
		if (l3->af == GR_AF_IP4)
			o.ipv4 = l3->ipv4;
		else if (l3->af == GR_AF_IP6)
			memcpy(o.ipv6, l3->ipv6, 16);
		memcpy(o.mac, l3->mac.addr_bytes, 6);
	} else if (nh->type == GR_NH_T_GROUP) {
		const struct nexthop_info_group *g = nexthop_info_group(nh);
		o.n_members = g->n_members;
		o.reta_size = g->reta_size;
		if (g->n_members == 1) // nexthop_group_get_nh's shortcut (nexthop.h:89-96)
			o.single = gpu_fwd4_control_nh_slot(g->nh);
		if (g->n_members > 1 && g->reta_size > 0) {
			const int keep = old.type == GR_NH_T_GROUP && old.n_members > 1 && old.reta_size == g->reta_size;
			if (keep) {
				new_off = old.reta_off;
			} else if ((r = reta_alloc(g->reta_size, &new_off)) < 0) {
				return r;
			}
			new_len = g->reta_size;
			for (uint32_t i = 0; i < g->reta_size; i++)
				M.reta[new_off + i] = gpu_fwd4_control_nh_slot(g->reta[i]);
			note(r = gpu_fwd4_reta_set(new_off, &M.reta[new_off], g->reta_size));
			o.reta_off = new_off;
		}
	}
	M.nh[slot] = o;
	if (nh->type == GR_NH_T_L3)
		nh_changed(slot); // published before any route or group naming it (see "publication")
	else
		note(r = gpu_fwd4_nh_set(slot, &o, 1));
	// the old range goes once the nexthop no longer names it
	if (old.type == GR_NH_T_GROUP && old.n_members > 1 && old.reta_size > 0
	    && !(new_len == old.reta_size && new_off == old.reta_off))
		reta_free(old.reta_off, old.reta_size);
	return r;
}

static void on_nexthop(uint32_t ev, const void *obj) {
	const struct nexthop *nh = obj;
	uint32_t slot;
	switch (ev) {
	case GR_EVENT_NEXTHOP_NEW:
	case GR_EVENT_NEXTHOP_UPDATE:
		if ((slot = slot_get(nh)) == 0) {
			note(-ENOSPC);
			return;
		}
		// the registry first: a packet may name the slot once the GPU has it
		note(gpu_fwd4_nh_obj_set(slot, nh));
		push_nh(slot, nh);
		break;
	case GR_EVENT_NEXTHOP_DELETE: // after grout's synchronize (nexthop.c:505-513)
		if ((slot = gpu_fwd4_control_nh_slot(nh)) == 0)
			return;
		const struct gr_hip_nh old = M.nh[slot];
		memset(&M.nh[slot], 0, sizeof(M.nh[slot]));
		nh_changed(slot); // no route names it since grout's synchronize
		note(gpu_fwd4_nh_obj_set(slot, NULL));
		if (old.type == GR_NH_T_GROUP && old.n_members > 1)
			reta_free(old.reta_off, old.reta_size);
		slot_put(nh, slot);
		break;
	}
}

// ---- routes ------------------------------------------------------------------
static uint32_t mask4(uint32_t ip_be, uint8_t plen) {
	const uint32_t h = __builtin_bswap32(ip_be);
	return __builtin_bswap32(plen ? h & (0xffffffffu << (32 - plen)) : 0);
}

// A publication while L3 nexthop changes still wait for theirs may put on the
// GPUs a route naming a slot whose mirror is stale (slots are reused): every
// caller flushes the nexthops first (nh_flush), counted here if one did not.
static void commit_check(void) {
	if (M.n_nh_dirty != 0)
		M.st.unordered++;
}

static void commit4(uint16_t vrf_id) {
	commit_check();
	note(gpu_fwd4_fib4_commit(vrf_id));
	M.st.commits++;
	M.dirty4[vrf_id] = 0;
}

static void commit6(uint16_t vrf_id) {
	commit_check();
	note(gpu_fwd4_fib6_commit(vrf_id));
	M.st.commits++;
	M.dirty6[vrf_id] = 0;
}

// ---- publication -------------------------------------------------------------
// Each route event reaches every context's RIB at once; publishing it (a
// commit: the changed tbl24 ranges / trie paths uploaded into the unpublished
// copy and the copies flipped) waits until the control thread's
// event loop comes round (a timer of PUBLISH_DELAY_US), PUBLISH_BATCH changes
// have gathered, or grout is about to wait for the datapath before freeing a
// nexthop (GR_EVENT_NEXTHOP_PRE_DELETE, pushed by nexthop_destroy before its
// rte_rcu_qsbr_synchronize; an iface's removal destroys its nexthops the same
// way). So a full view loaded by FRR is published in a few hundred commits, not
// one per route, and a deleted route is still off every GPU before grout's
// synchronize for its nexthop starts: no batch started after it can name the
// nexthop's slot, which the slot's next owner may reuse.
#define PUBLISH_BATCH 4096
#define PUBLISH_DELAY_US 200

static int cmp_u32(const void *a, const void *b) {
	const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
	return x < y ? -1 : x > y;
}

// The L3 nexthops changed since the last publication onto every GPU, one
// call per run of consecutive slots (a burst of learned neighbours takes
// consecutive slots).
static void nh_flush(void) {
	if (M.n_nh_dirty == 0)
		return;
	qsort(M.nh_dirty, M.n_nh_dirty, sizeof(uint32_t), cmp_u32);
	for (uint32_t i = 0, j; i < M.n_nh_dirty; i = j) {
		for (j = i + 1; j < M.n_nh_dirty && M.nh_dirty[j] == M.nh_dirty[j - 1] + 1; j++)
			;
		note(gpu_fwd4_nh_set(M.nh_dirty[i], &M.nh[M.nh_dirty[i]], j - i));
	}
	for (uint32_t i = 0; i < M.n_nh_dirty; i++)
		M.nh_is_dirty[M.nh_dirty[i]] = 0;
	M.n_nh_dirty = 0;
}

void gpu_fwd4_control_flush(void) {
	if (M.flush_armed) {
		evtimer_del(M.flush_ev);
		M.flush_armed = 0;
	}
	if (M.pending == 0)
		return;
	nh_flush(); // before the routes that may name them
	for (uint32_t v = 0; v < M.max_ifaces; v++) {
		if (M.dirty4[v])
			commit4((uint16_t)v);
		if (M.dirty6[v])
			commit6((uint16_t)v);
	}
	M.pending = 0;
}

static void publish_cb(int fd, short what, void *arg) {
	(void)fd;
	(void)what;
	(void)arg;
	M.flush_armed = 0;
	gpu_fwd4_control_flush();
}

static void publish_later(void) {
	if (++M.pending >= PUBLISH_BATCH) {
		gpu_fwd4_control_flush();
		return;
	}
	if (M.flush_armed)
		return;
	if (M.flush_ev == NULL && ev_base != NULL)
		M.flush_ev = evtimer_new(ev_base, publish_cb, NULL);
	const struct timeval tv = {.tv_sec = 0, .tv_usec = PUBLISH_DELAY_US};
	if (M.flush_ev == NULL || evtimer_add(M.flush_ev, &tv) < 0) {
		M.st.no_timer++;
		gpu_fwd4_control_flush(); // no timer: publish now
		return;
	}
	M.flush_armed = 1;
}

static void route_changed(uint16_t vrf_id, int ip6) {
	(ip6 ? M.dirty6 : M.dirty4)[vrf_id] = 1;
	publish_later();
}

static void nh_changed(uint32_t slot) {
	if (!M.nh_is_dirty[slot]) {
		M.nh_is_dirty[slot] = 1;
		M.nh_dirty[M.n_nh_dirty++] = slot;
	}
	publish_later();
}

static void shadow_route4(const struct gr_hip_route4 *rt, int add) {
	const struct route4_key k = {.ip = rt->ip, .vrf_id = rt->vrf_id, .prefixlen = rt->prefixlen};
	uint32_t *idx = ht_find(&M.k4, &k);
	if (add) {
		if (idx != NULL) {
			M.r4[*idx] = *rt;
			return;
		}
		if (M.n_r4 == M.cap_r4) {
			const uint32_t cap = M.cap_r4 ? 2 * M.cap_r4 : 1024;
			void *p = realloc(M.r4, cap * sizeof(*M.r4));
			if (p == NULL) {
				note(-ENOMEM);
				return;
			}
			M.r4 = p;
			M.cap_r4 = cap;
		}
		if (ht_put(&M.k4, &k, M.n_r4, sizeof(k)) < 0) {
			note(-ENOMEM);
			return;
		}
		M.r4[M.n_r4++] = *rt;
	} else if (idx != NULL) {
		const uint32_t i = *idx;
		ht_del(&M.k4, &k);
		if (i != --M.n_r4) { // the last route fills the hole
			M.r4[i] = M.r4[M.n_r4];
			const struct gr_hip_route4 *m = &M.r4[i];
			const struct route4_key mk = {.ip = m->ip, .vrf_id = m->vrf_id, .prefixlen = m->prefixlen};
			*ht_find(&M.k4, &mk) = i;
		}
	}
	M.st.routes4 = M.n_r4;
}

// GR_EVENT_IP_ROUTE_ADD / _DEL: struct route4_event (route.c:205-210)
static void on_route4(uint32_t ev, const void *obj) {
	const struct route4_event *r = obj;
	struct gr_hip_route4 rt = {.ip = mask4(r->dest.ip, r->dest.prefixlen), .prefixlen = r->dest.prefixlen,
				   .vrf_id = r->vrf_id};
	if (ev == GR_EVENT_IP_ROUTE_ADD) {
		if ((rt.nh = gpu_fwd4_control_nh_slot(r->nh)) == 0) {
			note(-ENOENT); // a nexthop that never had an event: cannot happen with the patch
			return;
		}
		note(gpu_fwd4_route4_add(&rt, 1, 1));
		shadow_route4(&rt, 1);
	} else {
		note(gpu_fwd4_route4_del(rt.vrf_id, rt.ip, rt.prefixlen));
		shadow_route4(&rt, 0);
	}
	route_changed(r->vrf_id, 0);
}

static bool ip6_is_linklocal(const uint8_t a[16]) {
	return a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
}

static void mask6(uint8_t a[16], uint8_t plen) {
	for (int b = 0; b < 16; b++) {
		const int keep = (int)plen - 8 * b;
		a[b] &= keep >= 8 ? 0xff : keep <= 0 ? 0 : (uint8_t)(0xff << (8 - keep));
	}
}

static struct route6_key key6(const struct gr_hip_route6 *rt) {
	struct route6_key k;
	memset(&k, 0, sizeof(k));
	memcpy(k.ip, rt->ip, 16);
	k.vrf_id = rt->vrf_id;
	k.iface_id = rt->iface_id;
	k.prefixlen = rt->prefixlen;
	return k;
}

static void shadow_route6(const struct gr_hip_route6 *rt, int add) {
	const struct route6_key k = key6(rt);
	uint32_t *idx = ht_find(&M.k6, &k);
	if (add) {
		if (idx != NULL) {
			M.r6[*idx] = *rt;
			return;
		}
		if (M.n_r6 == M.cap_r6) {
			const uint32_t cap = M.cap_r6 ? 2 * M.cap_r6 : 1024;
			void *p = realloc(M.r6, cap * sizeof(*M.r6));
			if (p == NULL) {
				note(-ENOMEM);
				return;
			}
			M.r6 = p;
			M.cap_r6 = cap;
		}
		if (ht_put(&M.k6, &k, M.n_r6, sizeof(k)) < 0) {
			note(-ENOMEM);
			return;
		}
		M.r6[M.n_r6++] = *rt;
	} else if (idx != NULL) {
		const uint32_t i = *idx;
		ht_del(&M.k6, &k);
		if (i != --M.n_r6) {
			M.r6[i] = M.r6[M.n_r6];
			const struct route6_key mk = key6(&M.r6[i]);
			*ht_find(&M.k6, &mk) = i;
		}
	}
	M.st.routes6 = M.n_r6;
}

// GR_EVENT_IP6_ROUTE_ADD / _DEL: struct route6_event (ip6 route.c:222-227)
// with the scope iface the patch adds to it
static void on_route6(uint32_t ev, const void *obj) {
	const struct route6_event *r = obj;
	struct gr_hip_route6 rt;
	memset(&rt, 0, sizeof(rt));
	memcpy(rt.ip, r->dest.ip, 16);
	mask6(rt.ip, r->dest.prefixlen);
	rt.prefixlen = r->dest.prefixlen;
	rt.vrf_id = r->vrf_id;
	rt.iface_id = ip6_is_linklocal(r->dest.ip) ? r->iface_id : 0;
	if (ev == GR_EVENT_IP6_ROUTE_ADD) {
		if ((rt.nh = gpu_fwd4_control_nh_slot(r->nh)) == 0) {
			note(-ENOENT);
			return;
		}
		note(gpu_fwd4_route6_add(&rt, 1, 1));
		shadow_route6(&rt, 1);
	} else {
		note(gpu_fwd4_route6_del(rt.vrf_id, rt.iface_id, rt.ip, rt.prefixlen));
		shadow_route6(&rt, 0);
	}
	route_changed(r->vrf_id, 1);
}

// ---- ifaces ------------------------------------------------------------------
// struct iface (iface.h:20-35 + the type info) -> struct gr_hip_iface
static void iface_to_hip(const struct iface *i, struct gr_hip_iface *o) {
	memset(o, 0, sizeof(*o));
	o->id = i->id;
	o->type = i->type;
	o->mode = i->mode;
	o->flags = i->flags;
	o->mtu = i->mtu;
	o->vrf_id = i->vrf_id;
	if (i->type == GR_IFACE_TYPE_PORT)
		o->port_id = iface_info_port(i)->port_id;
	if (i->type == GR_IFACE_TYPE_VLAN) {
		o->vlan_id = iface_info_vlan(i)->vlan_id;
		o->parent_id = iface_info_vlan(i)->parent_id;
	}
	struct rte_ether_addr mac;
	if (iface_get_eth_addr(i, &mac) == 0) { // iface.c:475-487
		memcpy(o->mac, mac.addr_bytes, 6);
		o->mac_ok = 1;
	}
}

// A VRF's FIBs, sized as grout sized its own (vrf.c:230-255, route.c:100-122)
static void fib_create(uint16_t vrf_id, const struct iface_info_vrf *v) {
	struct fib_conf *f = &M.fibs[vrf_id];
	note(gpu_fwd4_fib4_create(vrf_id, v->ipv4.max_routes, v->ipv4.num_tbl8));
	note(gpu_fwd4_fib6_create(vrf_id, v->ipv6.max_routes, v->ipv6.num_tbl8));
	f->on4 = f->on6 = 1;
	f->v4 = v->ipv4;
	f->v6 = v->ipv6;
}

static void fib_destroy(uint16_t vrf_id) {
	struct fib_conf *f = &M.fibs[vrf_id];
	M.dirty4[vrf_id] = M.dirty6[vrf_id] = 0; // nothing left to publish there
	if (f->on4)
		note(gpu_fwd4_fib4_destroy(vrf_id));
	if (f->on6)
		note(gpu_fwd4_fib6_destroy(vrf_id));
	memset(f, 0, sizeof(*f));
}

// Every route of a VRF again, into its (re-created) FIBs, and published:
// the L3 nexthops waiting for the next publication first, as for any other
// (the routes may name their slots).
static void fib_refill(uint16_t vrf_id) {
	nh_flush();
	for (uint32_t i = 0; i < M.n_r4; i++)
		if (M.r4[i].vrf_id == vrf_id)
			note(gpu_fwd4_route4_add(&M.r4[i], 1, 1));
	for (uint32_t i = 0; i < M.n_r6; i++)
		if (M.r6[i].vrf_id == vrf_id)
			note(gpu_fwd4_route6_add(&M.r6[i], 1, 1));
	commit4(vrf_id);
	commit6(vrf_id);
}

static void push_iface(const struct iface *i) {
	struct gr_hip_iface o;
	iface_to_hip(i, &o);
	note(gpu_fwd4_iface_set(&o, 1));
	M.ifs[i->id] = o;
	M.if_live[i->id] = M.if_seen[i->id] = 1;
}

static void on_iface(uint32_t ev, const void *obj) {
	const struct iface *i = obj;
	if (i->id == 0 || i->id >= M.max_ifaces)
		return;
	switch (ev) {
	case GR_EVENT_IFACE_POST_ADD:
		M.if_removing[i->id] = 0;
		note(gpu_fwd4_iface_obj_set(i->id, i)); // before any packet can name it
		if (i->type == GR_IFACE_TYPE_VRF)
			fib_create(i->id, iface_info_vrf(i));
		push_iface(i);
		break;
	case GR_EVENT_IFACE_POST_RECONFIG:
		if (i->type == GR_IFACE_TYPE_VRF) { // new FIB sizes: grout migrates the routes (route.c:717-752)
			const struct iface_info_vrf *v = iface_info_vrf(i);
			const struct fib_conf *f = &M.fibs[i->id];
			if (memcmp(&f->v4, &v->ipv4, sizeof(f->v4)) != 0 || memcmp(&f->v6, &v->ipv6, sizeof(f->v6)) != 0) {
				fib_destroy(i->id);
				fib_create(i->id, v);
				fib_refill(i->id);
			}
		}
		// fallthrough
	case GR_EVENT_IFACE_STATUS_UP:
	case GR_EVENT_IFACE_STATUS_DOWN:
	case GR_EVENT_IFACE_MAC_CHANGE:
		if (!M.if_removing[i->id]) // iface_destroy's STATUS_DOWN comes after PRE_REMOVE
			push_iface(i);
		break;
	case GR_EVENT_IFACE_PRE_REMOVE: // the iface leaves the GPUs with grout's ifaces[] (iface.c:702-712)
		M.st.presync += M.pending != 0;
		gpu_fwd4_control_flush(); // before grout's synchronize (see "publication")
		M.if_removing[i->id] = 1;
		M.if_live[i->id] = 0;
		memset(&M.ifs[i->id], 0, sizeof(M.ifs[i->id]));
		note(gpu_fwd4_iface_del(i->id));
		break;
	case GR_EVENT_IFACE_REMOVE: // after grout's synchronize (iface.c:712-719)
		note(gpu_fwd4_iface_obj_set(i->id, NULL));
		if (i->type == GR_IFACE_TYPE_VRF)
			fib_destroy(i->id);
		M.if_removing[i->id] = 0;
		break;
	}
}

// ---- dispatch ----------------------------------------------------------------
static void dispatch(uint32_t ev, const void *obj) {
	if (ready() < 0) {
		note(-ENOMEM);
		return;
	}
	switch (ev) {
	case GR_EVENT_NEXTHOP_NEW:
	case GR_EVENT_NEXTHOP_UPDATE:
	case GR_EVENT_NEXTHOP_DELETE:
		on_nexthop(ev, obj);
		break;
	case GR_EVENT_NEXTHOP_PRE_DELETE: // grout waits for the datapath next: publish first
		M.st.presync += M.pending != 0;
		gpu_fwd4_control_flush();
		break;
	case GR_EVENT_IP_ROUTE_ADD:
	case GR_EVENT_IP_ROUTE_DEL:
		on_route4(ev, obj);
		break;
	case GR_EVENT_IP6_ROUTE_ADD:
	case GR_EVENT_IP6_ROUTE_DEL:
		on_route6(ev, obj);
		break;
	default:
		on_iface(ev, obj);
		break;
	}
}

static void on_event(uint32_t ev, const void *obj) {
	M.st.events++;
	dispatch(ev, obj);
}

static void on_internal_event(uint32_t ev, const void *obj) {
	M.st.internal++;
	dispatch(ev, obj);
}

// grout: RTE_INIT in the module's control file, as its own modules subscribe
// (e.g. modules/infra/control/nexthop.c:588-595)
RTE_INIT(gpu_fwd4_control_init) {
	static const uint32_t iface_evs[] = {GR_EVENT_IFACE_POST_ADD,    GR_EVENT_IFACE_POST_RECONFIG,
					     GR_EVENT_IFACE_STATUS_UP,   GR_EVENT_IFACE_STATUS_DOWN,
					     GR_EVENT_IFACE_MAC_CHANGE,  GR_EVENT_IFACE_PRE_REMOVE,
					     GR_EVENT_IFACE_REMOVE};
	static const uint32_t obj_evs[] = {GR_EVENT_NEXTHOP_NEW,   GR_EVENT_NEXTHOP_UPDATE, GR_EVENT_NEXTHOP_DELETE,
					   GR_EVENT_IP_ROUTE_ADD,  GR_EVENT_IP_ROUTE_DEL,   GR_EVENT_IP6_ROUTE_ADD,
					   GR_EVENT_IP6_ROUTE_DEL};
	for (unsigned k = 0; k < sizeof(iface_evs) / sizeof(iface_evs[0]); k++)
		event_subscribe(iface_evs[k], on_event);
	for (unsigned k = 0; k < sizeof(obj_evs) / sizeof(obj_evs[0]); k++) {
		event_subscribe(obj_evs[k], on_event);
		event_subscribe_internal(obj_evs[k], on_internal_event);
	}
	event_subscribe_internal(GR_EVENT_NEXTHOP_PRE_DELETE, on_internal_event);
}

// ---- queries -------------------------------------------------------------------
int gpu_fwd4_control_nh(uint32_t slot, struct gr_hip_nh *out) {
	if (!M.ready || slot == 0 || slot > M.max_nh || out == NULL)
		return -EINVAL;
	*out = M.nh[slot];
	return M.nh[slot].type != 0 ? 0 : -ENOENT;
}

int gpu_fwd4_control_iface(uint16_t id, struct gr_hip_iface *out) {
	if (!M.ready || id >= M.max_ifaces || out == NULL)
		return -EINVAL;
	*out = M.ifs[id];
	return M.if_live[id] ? 0 : -ENOENT;
}

int gpu_fwd4_control_reta(uint32_t first, uint32_t *slots, uint32_t n) {
	if ((uint64_t)first + n > M.reta_top || (slots == NULL && n))
		return -EINVAL;
	memcpy(slots, M.reta + first, n * sizeof(uint32_t));
	return 0;
}

int gpu_fwd4_control_routes4(struct gr_hip_route4 *out, uint32_t max) {
	if (out != NULL)
		memcpy(out, M.r4, (max < M.n_r4 ? max : M.n_r4) * sizeof(*out));
	return (int)M.n_r4;
}

int gpu_fwd4_control_routes6(struct gr_hip_route6 *out, uint32_t max) {
	if (out != NULL)
		memcpy(out, M.r6, (max < M.n_r6 ? max : M.n_r6) * sizeof(*out));
	return (int)M.n_r6;
}

void gpu_fwd4_control_stats(struct gpu_fwd4_control_stats *st) {
	if (st != NULL) {
		*st = M.st;
		st->pending = M.pending;
	}
}

// ---- replay into one context -------------------------------------------------
int gpu_fwd4_control_replay(uint32_t i) {
	gr_hip_ctx_t *ctx = gpu_fwd4_ctx_at(i);
	int r = 0, e;
	if (ctx == NULL)
		return -ENOENT;
	if (!M.ready)
		return gpu_fwd4_resync(i);
#define REPLAY(call)                                                                               \
	do {                                                                                       \
		if ((e = (call)) < 0 && r == 0)                                                    \
			r = e;                                                                     \
	} while (0)
	for (uint32_t id = 1; id < M.max_ifaces; id++) {
		if (M.if_live[id])
			REPLAY(gr_hip_iface_set(ctx, &M.ifs[id], 1));
		else if (M.if_seen[id])
			REPLAY(gr_hip_iface_del(ctx, (uint16_t)id));
	}
	if (M.reta_top)
		REPLAY(gr_hip_reta_set(ctx, 0, M.reta, M.reta_top));
	if (M.next_slot > 1)
		REPLAY(gr_hip_nh_set(ctx, 1, &M.nh[1], M.next_slot - 1));
	for (uint32_t v = 1; v < M.max_ifaces; v++) {
		const struct fib_conf *f = &M.fibs[v];
		if (!f->on4)
			continue;
		gr_hip_fib4_destroy(ctx, (uint16_t)v); // whatever it held
		gr_hip_fib6_destroy(ctx, (uint16_t)v);
		REPLAY(gr_hip_fib4_create(ctx, (uint16_t)v, f->v4.max_routes, f->v4.num_tbl8));
		REPLAY(gr_hip_fib6_create(ctx, (uint16_t)v, f->v6.max_routes, f->v6.num_tbl8));
		for (uint32_t k = 0; k < M.n_r4; k++)
			if (M.r4[k].vrf_id == v)
				REPLAY(gr_hip_route4_add(ctx, &M.r4[k], 1, 1));
		for (uint32_t k = 0; k < M.n_r6; k++)
			if (M.r6[k].vrf_id == v)
				REPLAY(gr_hip_route6_add(ctx, &M.r6[k], 1, 1));
		REPLAY(gr_hip_fib4_commit(ctx, (uint16_t)v));
		REPLAY(gr_hip_fib6_commit(ctx, (uint16_t)v));
	}
#undef REPLAY
	return r < 0 ? r : gpu_fwd4_resync(i);
}
