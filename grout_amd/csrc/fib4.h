// SPDX-License-Identifier: BSD-3-Clause
//
// fib4.h -- host side of the device FIB: a binary-trie RIB and the DIR24_8-
// equivalent tables (4-byte entries) it paints incrementally.
//
// Replaces DPDK rte_fib/rte_rib as created by grout's create_fib
// (modules/ip/control/route.c:63-98) and updated by rte_fib_add /
// rte_fib_delete in rib4_insert_or_replace / rib4_delete (modules/ip/control/route.c:212-330).
//
// Table encoding (the layout the HIP kernel walks):
//   tbl24[ip >> 8]:  0            no route
//                    bit31 == 0   nexthop slot (1 .. 2^24-1)
//                    bit31 == 1   tbl8 group index in bits 0..30
//   tbl8[group * 256 + (ip & 0xff)]: nexthop slot, 0 = no route
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_FIB4_TBL24_ENTRIES (1u << 24)
#define GR_FIB4_EXT 0x80000000u

struct gr_fib4;

struct gr_fib4 *gr_fib4_new(uint32_t max_routes, uint32_t num_tbl8);
void gr_fib4_free(struct gr_fib4 *);

// ip in host byte order. Returns 0, -EEXIST (exists and !replace), -ENOSPC
// (max_routes or tbl8 groups exhausted), -ENOMEM, -EINVAL.
int gr_fib4_add(struct gr_fib4 *, uint32_t ip, uint8_t prefixlen, uint32_t nh, int replace);
int gr_fib4_del(struct gr_fib4 *, uint32_t ip, uint8_t prefixlen);
uint32_t gr_fib4_lookup(const struct gr_fib4 *, uint32_t ip);
// Exact-prefix RIB lookup (rte_rib_lookup_exact); 0 if absent.
uint32_t gr_fib4_get(const struct gr_fib4 *, uint32_t ip, uint8_t prefixlen);

const uint32_t *gr_fib4_tbl24(const struct gr_fib4 *);
const uint32_t *gr_fib4_tbl8(const struct gr_fib4 *);
uint32_t gr_fib4_num_tbl8(const struct gr_fib4 *);
uint32_t gr_fib4_tbl8_used(const struct gr_fib4 *);
uint32_t gr_fib4_n_routes(const struct gr_fib4 *);

// Dirty tracking for the device upload, since the last gr_fib4_dirty_clear:
// the tbl24 index ranges [lo, hi) painted, sorted and disjoint (at most 4096
// are kept: past that the closest ones are merged, so a range may cover
// unchanged entries), and the tbl8 groups painted. Each returns the number
// written (at most `max`; -1 if more: upload everything).
struct gr_fib4_range {
	uint32_t lo, hi;
};
int gr_fib4_dirty_tbl24(struct gr_fib4 *, struct gr_fib4_range *ranges, uint32_t max);
int gr_fib4_dirty_tbl8(struct gr_fib4 *, uint32_t *groups, uint32_t max);
void gr_fib4_dirty_clear(struct gr_fib4 *);

#ifdef __cplusplus
}
#endif
