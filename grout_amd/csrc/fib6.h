// SPDX-License-Identifier: BSD-3-Clause
//
// fib6.h -- host side of the device IPv6 FIB: the RIB of one VRF and the
// multibit trie painted from it. Not a public header.
//
// grout keeps IPv6 routes in rte_rib6 and looks them up in an rte_fib6 TRIE
// (modules/ip6/control/route.c:66-98,151-173). The device table here is a
// multibit trie: a first level of 2^16 entries indexed by address bytes 0-1,
// then groups of 256 entries indexed by each further byte, path-compressed:
// a group whose 256 entries all hold one leaf but for one index becomes a
// skip node ("bytes b..b+n-1 equal key: continue with child, else the leaf
// miss"), and consecutive skips merge (up to 7 key bytes); level-compressed:
// a group whose entries are mostly child groups (and no skip), or a one-byte
// skip over a heavy subtree with its child group, becomes one wide group of
// 65536 entries indexed by two bytes, 256 consecutive group slots, one
// dependent gather instead of two on its paths; when its children's entries
// only change at multiples of 2^s in byte b + 1 (their prefixes end in the
// top 8 - s bits of that byte), its rows keep one entry per 2^s: 2^(8-s)
// slots in all, entry (x, y) at x * 2^(8-s) + (y >> s). Entry encoding
// (u32): bit 31 clear = the nexthop slot of the longest matching prefix (0 =
// no route, the FIB default_nh, modules/ip6/control/route.c:68); bits 31 and 30 = skip node
// index in bits 0-28; bits 31 and 29 = wide group, its first slot in bits
// 0-25 and s in bits 26-28; bits 31, 30 and 29 = range group (below), its
// first slot in bits 0-28; bit 31 alone = group index in bits 0-28.
//
// Range group: a node at byte b whose children each hold one run of a leaf
// in byte b + 1 and another leaf around it (a prefix that ends inside byte
// b + 1, as fib_inject's /42, /44 and /46 do under their /40s), folded
// into 256 8-byte entries over two slots: entry x = {in | lo << 24, miss |
// hi << 24}, the leaf is in when lo <= byte b + 1 <= hi, else miss (a
// leaf entry of the node: in = miss). One gather ends the walk, and a
// route's entry shares its line with 15 neighbours instead of owning one.
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_FIB6_EXT 0x80000000u
#define GR_FIB6_SKIP 0x40000000u
#define GR_FIB6_WIDE 0x20000000u
#define GR_FIB6_IDX 0x1fffffffu
#define GR_FIB6_WIDE_SHIFT 26 // bits 26-28 of a wide entry: s
#define GR_FIB6_WIDE_IDX 0x03ffffffu // its first slot
#define GR_FIB6_RANGE (GR_FIB6_SKIP | GR_FIB6_WIDE) // both bits: a range group
#define GR_FIB6_RANGE_LEAF 0x00ffffffu // the leaves a range group can hold
#define GR_FIB6_WIDE_MIN 64 // child groups (of 256 entries) that make a group wide
#define GR_FIB6_SKIP_WIDE_MIN 16 // groups under a one-byte skip's child that make the pair wide

struct gr_fib6_skip { // 16 bytes, as the kernel loads it
	uint8_t key[7];
	uint8_t n; // key bytes, 1..7
	uint32_t child; // entry when they match (depth + n)
	uint32_t miss; // leaf when they do not
};
#define GR_FIB6_TOP 65536
#define GR_FIB6_GROUP 256

typedef struct gr_fib6 gr_fib6_t;

gr_fib6_t *gr_fib6_new(uint32_t max_routes, uint32_t max_groups);
void gr_fib6_free(gr_fib6_t *);

// ip: the (already scoped) prefix; host bits are masked. 0, -EEXIST, -ENOSPC.
int gr_fib6_add(gr_fib6_t *, const uint8_t ip[16], uint8_t prefixlen, uint32_t nh, int replace);
// 0 or -ENOENT.
int gr_fib6_del(gr_fib6_t *, const uint8_t ip[16], uint8_t prefixlen);
// Routes are painted into the plain trie as they are added and deleted; a
// build brings the image (the tables the kernel walks) up to date along the
// changed paths only: 0, -ENOSPC (no group slot left) or -ENOMEM.
int gr_fib6_build(gr_fib6_t *);
// Longest-prefix match through the painted trie (as the kernel walks it).
uint32_t gr_fib6_lookup(const gr_fib6_t *, const uint8_t ip[16]);
// Longest-prefix match through the RIB (truth for tests).
uint32_t gr_fib6_lookup_rib(const gr_fib6_t *, const uint8_t ip[16]);

const uint32_t *gr_fib6_top(const gr_fib6_t *);
const uint32_t *gr_fib6_groups(const gr_fib6_t *);
uint32_t gr_fib6_groups_used(const gr_fib6_t *);
const struct gr_fib6_skip *gr_fib6_skips(const gr_fib6_t *);
uint32_t gr_fib6_skips_used(const gr_fib6_t *);
// Nodes of the plain (uncompressed) trie.
uint32_t gr_fib6_groups_painted(const gr_fib6_t *);
uint32_t gr_fib6_max_groups(const gr_fib6_t *);
uint32_t gr_fib6_n_routes(const gr_fib6_t *);
uint32_t gr_fib6_max_slot(const gr_fib6_t *);
// Build generation: bumps on every repaint that changed the tables.
uint64_t gr_fib6_generation(const gr_fib6_t *);

// Slots in use (gr_fib6_groups_used is the high-water mark the image spans).
uint32_t gr_fib6_groups_live(const gr_fib6_t *);

// What the builds since the last gr_fib6_dirty_clear changed in the image:
// first-level indexes, group slots (1 KiB each) or skip nodes, in no
// particular order (a slot or skip once). Returns 1 when everything is to be
// taken as changed (no clear yet: the first upload), 0, or -EINVAL. A commit
// uploads them to the device copy it writes, then clears.
enum { GR_FIB6_DIRTY_TOP, GR_FIB6_DIRTY_SLOTS, GR_FIB6_DIRTY_SKIPS };
int gr_fib6_dirty(const gr_fib6_t *, int kind, const uint32_t **list, uint32_t *n);
void gr_fib6_dirty_clear(gr_fib6_t *);

#ifdef __cplusplus
}
#endif
