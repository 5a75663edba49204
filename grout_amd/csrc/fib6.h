// SPDX-License-Identifier: BSD-3-Clause
//
// fib6.h -- host side of the device IPv6 FIB: the RIB of one VRF and the
// multibit trie painted from it. Not a public header.
//
// grout keeps IPv6 routes in rte_rib6 and looks them up in an rte_fib6 TRIE
// (modules/ip6/control/route.c:66-98,151-173). The device table here is a
// multibit trie: a first level of 2^16 entries indexed by address bytes 0-1,
// then groups of 256 entries indexed by each further byte. Entry encoding
// (u32): bit 31 set = group index in bits 0-30, else the nexthop slot of the
// longest matching prefix (0 = no route, the FIB default_nh, route.c:80).
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_FIB6_EXT 0x80000000u
#define GR_FIB6_TOP 65536
#define GR_FIB6_GROUP 256

typedef struct gr_fib6 gr_fib6_t;

gr_fib6_t *gr_fib6_new(uint32_t max_routes, uint32_t max_groups);
void gr_fib6_free(gr_fib6_t *);

// ip: the (already scoped) prefix; host bits are masked. 0, -EEXIST, -ENOSPC.
int gr_fib6_add(gr_fib6_t *, const uint8_t ip[16], uint8_t prefixlen, uint32_t nh, int replace);
// 0 or -ENOENT.
int gr_fib6_del(gr_fib6_t *, const uint8_t ip[16], uint8_t prefixlen);
// Repaint the trie if routes changed since the last build: 0 or -ENOSPC.
int gr_fib6_build(gr_fib6_t *);
// Longest-prefix match through the painted trie (as the kernel walks it).
uint32_t gr_fib6_lookup(const gr_fib6_t *, const uint8_t ip[16]);
// Longest-prefix match through the RIB (truth for tests).
uint32_t gr_fib6_lookup_rib(const gr_fib6_t *, const uint8_t ip[16]);

const uint32_t *gr_fib6_top(const gr_fib6_t *);
const uint32_t *gr_fib6_groups(const gr_fib6_t *);
uint32_t gr_fib6_groups_used(const gr_fib6_t *);
uint32_t gr_fib6_max_groups(const gr_fib6_t *);
uint32_t gr_fib6_n_routes(const gr_fib6_t *);
uint32_t gr_fib6_max_slot(const gr_fib6_t *);
// Build generation: bumps on every repaint that changed the tables.
uint64_t gr_fib6_generation(const gr_fib6_t *);

#ifdef __cplusplus
}
#endif
