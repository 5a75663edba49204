// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_dev.h -- device helpers shared by the forwarding kernels
// (fwd4_ring.hip): table views, counter aggregation,
// vector loads and stores. Not a public header.
#pragma once

#include <hip/hip_runtime.h>

#include "fwd4_kernel.h"

#define CHAIN GR_HIP_EDGE_CHAIN

// Table pointers reached through fwd4_tables are generic to the compiler;
// reading them as global (address space 1) gives global_load instead of
// flat_load, which would force vmcnt(0) + lgkmcnt(0) at every use.
#define GR_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const T *p) {
	return *(const GR_GLOBAL T *)p;
}

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
// two dwords at a dword-aligned address (one global_load_dwordx2)
typedef uint32_t u2a __attribute__((ext_vector_type(2), aligned(4)));

__device__ __forceinline__ uint4 gld4(const void *p) {
	const u4v v = *(const GR_GLOBAL u4v *)p;
	return uint4{v.x, v.y, v.z, v.w};
}

// What the chain reads: table pointers (loaded once per workgroup from the
// device-resident fwd4_tables) and the ether type table, copied into LDS.
// A field of the launch's table block, through the scalar cache (the block
// is uniform and read-only for the kernel's life).
template <typename X>
__device__ __forceinline__ X tload(const X *p) {
	return *(const __attribute__((address_space(4))) X *)p;
}

// What the node chain keeps at hand; the tables only cold paths use (slow
// adjacencies, ECMP retas, the VLAN table, the global fast adjacencies past
// the LDS copies) are read from the table block T where they are used, so
// that the kernel's SGPRs (106, all taken) are not held for them.
struct kctx {
	const fwd4_tables *T;
	const fwd4_rx *rx;
	uint32_t max_ifaces, max_nh, readable;
	const fwd4_edges *edges; // LDS copy
	uint32_t ip4_edge; // eth_input edges of ether types IPv4 / IPv6 (wave-uniform)
	uint32_t ip6_edge;
	const fwd4_rx6 *rx6;
	gr_hip_iface_stats *stats;
	const __attribute__((address_space(3))) u4v *nhf6_lds; // slots 1..nhf6_n staged in LDS
	uint32_t nhf6_n;
	const uint32_t *top6; // the trie whose first-level entries FWD4_TOP6_BASE.. are staged
	const __attribute__((address_space(3))) uint32_t *top6_lds;
	uint32_t top6_n;
};

struct rxv {
	uint32_t id, e_in, flags, mac_lo, mac_hi;
	const uint32_t *tbl24, *tbl8;
};

__device__ __forceinline__ rxv unpack_rx(uint4 a, uint4 b) {
	rxv r;
	r.id = a.x & 0xffff;
	r.e_in = (a.x >> 16) & 0xff;
	r.flags = a.x >> 24;
	r.mac_lo = a.y;
	r.mac_hi = a.z & 0xffff;
	r.tbl24 = reinterpret_cast<const uint32_t *>(((uint64_t)b.y << 32) | b.x);
	r.tbl8 = reinterpret_cast<const uint32_t *>(((uint64_t)b.w << 32) | b.z);
	return r;
}

// The RX view of an iface (iface_from_id, iface.c:459-466 + get_fib).
__device__ __forceinline__ rxv load_rx(const kctx &P, uint32_t id) {
	rxv r;
	r.id = 0;
	if (id == 0 || id >= P.max_ifaces)
		return r;
	const uint4 *p = reinterpret_cast<const uint4 *>(P.rx + id);
	return unpack_rx(gld4(p), gld4(p + 1));
}

struct adjv {
	uint32_t type, e_in, flags, e_pre, e_mid, e_post, oif, mtu, post_iface, ipv4, tx_if, tx_par;
	uint32_t dmac_lo, dmac_hi, smac_lo, smac_hi; // bytes 0-3 / 4-5
	uint32_t n_members, reta_size, reta_off, single;
};

__device__ __forceinline__ adjv unpack_adj(uint4 a, uint4 b, uint4 c) {
	adjv r;
	r.type = a.x & 0xff;
	r.e_in = (a.x >> 8) & 0xff;
	r.flags = (a.x >> 16) & 0xff;
	r.e_pre = a.x >> 24;
	r.e_mid = a.y & 0xff;
	r.e_post = (a.y >> 8) & 0xff;
	r.oif = a.y >> 16;
	r.mtu = a.z & 0xffff;
	r.post_iface = a.z >> 16;
	r.ipv4 = a.w;
	r.tx_if = b.x & 0xffff;
	r.tx_par = b.x >> 16;
	r.dmac_lo = b.y; // bytes 20-23
	r.dmac_hi = b.z & 0xffff; // 24-25
	r.smac_lo = (b.z >> 16) | (b.w << 16); // 26-29
	r.smac_hi = b.w >> 16; // 30-31
	r.n_members = c.x & 0xffff;
	r.reta_size = c.x >> 16;
	r.reta_off = c.y;
	r.single = c.z;
	return r;
}

__device__ __forceinline__ adjv load_adj(const kctx &P, uint32_t slot) {
	const uint4 *p = reinterpret_cast<const uint4 *>(tload(&P.T->adj) + slot);
	return unpack_adj(gld4(p), gld4(p + 1), gld4(p + 2));
}

// VLAN sub-interface demux, vlan_get_iface (vlan.c:27-34): open addressing
// on (parent << 16 | vlan) + 1.
__device__ __forceinline__ uint32_t vlan_lookup(const kctx &P, uint32_t parent, uint32_t vid) {
	const uint32_t *keys = tload(&P.T->vlan_keys);
	if (keys == nullptr)
		return 0;
	const uint16_t *vals = tload(&P.T->vlan_vals);
	const uint32_t mask = tload(&P.T->vlan_mask);
	uint32_t key = ((parent << 16) | vid) + 1;
	uint32_t h = (key * 0x9e3779b1u) & mask;
	for (uint32_t i = 0; i <= mask; i++) {
		uint32_t k = gld(keys + h);
		if (k == key)
			return gld(vals + h);
		if (k == 0)
			return 0;
		h = (h + 1) & mask;
	}
	return 0;
}

// Add to the counters of (kind, iface) in this workgroup's global shard.
__device__ __forceinline__ void shard_add(gr_hip_iface_stats *stats, uint32_t max_ifaces, uint32_t kind, uint32_t iface,
					  unsigned long long pkts, unsigned long long bytes) {
	gr_hip_iface_stats *st = stats + (size_t)(blockIdx.x % FWD4_STAT_SHARDS) * max_ifaces + iface;
	GR_GLOBAL unsigned long long *c = (GR_GLOBAL unsigned long long *)(kind ? &st->tx_packets : &st->rx_packets);
	__hip_atomic_fetch_add(c, pkts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__hip_atomic_fetch_add(c + 1, bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct stat_slot {
	uint32_t key; // ((kind << 16) | iface) + 1, 0 = free
	uint32_t pkts;
	unsigned long long bytes;
};

// One lane (the wave leader of a key) adds a wave's contribution to the
// workgroup's LDS slots: direct-mapped on (iface, kind), claimed once with a
// compare-and-swap, then fire-and-forget LDS atomics. A slot already owned
// by another key (two ifaces 32 apart) sends the update to the global shard.
__device__ __forceinline__ void slot_add(stat_slot *slots, const kctx &P, uint32_t key, uint32_t pkts, uint32_t bytes) {
	const uint32_t kind = (key - 1) >> 16, iface = (key - 1) & 0xffff;
	stat_slot *sl = &slots[(iface * 2 + kind) & (FWD4_STAT_SLOTS - 1)];
	uint32_t cur = sl->key;
	if (cur != key && cur == 0)
		cur = atomicCAS(&sl->key, 0u, key) == 0 ? key : sl->key;
	if (cur == key) {
		atomicAdd(&sl->pkts, pkts);
		atomicAdd(&sl->bytes, (unsigned long long)bytes);
		return;
	}
	shard_add(P.stats, P.max_ifaces, kind, iface, pkts, bytes);
}

// Sum of v over the wave with DPP (no LDS): quad, half-row and row steps,
// then row broadcasts; lane 63 ends with the total.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
	v += __builtin_amdgcn_update_dpp(0u, v, 0xb1, 0xf, 0xf, false); // quad_perm [1,0,3,2]
	v += __builtin_amdgcn_update_dpp(0u, v, 0x4e, 0xf, 0xf, false); // quad_perm [2,3,0,1]
	v += __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xf, 0xf, false); // row_half_mirror
	v += __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xf, 0xf, false); // row_mirror
	v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); // row_bcast:15
	v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); // row_bcast:31
	return __builtin_amdgcn_readlane(v, 63);
}

// Wave-aggregate one counter key per lane (0 = nothing) into the LDS slots.
// Every lane of the wave must call it (converged).
__device__ __forceinline__ void wave_count(stat_slot *slots, const kctx &P, uint32_t key, uint32_t len) {
	for (;;) {
		unsigned long long act = __ballot(key != 0);
		if (act == 0)
			break;
		const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1;
		const uint32_t k = __builtin_amdgcn_readlane(key, lead);
		const bool same = key == k;
		const uint32_t cnt = (uint32_t)__popcll(__ballot(same));
		const uint32_t b = wave_sum(same ? len : 0u);
		if ((threadIdx.x & 63) == lead)
			slot_add(slots, P, k, cnt, b);
		if (same)
			key = 0;
	}
}

// l2l3_edges[ether_type] (eth_input.c:26,60): IPv4 from a register, the
// other registered types from the LDS table.
__device__ __forceinline__ uint32_t eth_type_edge(const kctx &P, uint32_t type_raw) {
	if (type_raw == 0x0008u) // RTE_BE16(RTE_ETHER_TYPE_IPV4)
		return P.ip4_edge;
	if (type_raw == 0xdd86u) // RTE_BE16(RTE_ETHER_TYPE_IPV6)
		return P.ip6_edge;
	uint32_t e = GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE;
	const fwd4_edges &E = *P.edges;
	for (uint32_t i = 0; i < E.n_eth_types; i++)
		if (E.eth_type_be[i] == type_raw)
			e = E.eth_type_edge[i];
	return e;
}

// Edge of one ether type (raw big-endian value), computed once per wave from
// the LDS table.
__device__ __forceinline__ uint32_t type_edge_of(const fwd4_edges &E, uint32_t type_raw) {
	uint32_t e = GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE;
	for (uint32_t i = 0; i < E.n_eth_types; i++)
		if (E.eth_type_be[i] == type_raw)
			e = E.eth_type_edge[i];
	return __builtin_amdgcn_readfirstlane(e);
}

__device__ __forceinline__ uint32_t lo16(uint32_t x) {
	return x & 0xffff;
}
__device__ __forceinline__ uint32_t hi16(uint32_t x) {
	return x >> 16;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
	return ((x & 0xff) << 8) | ((x >> 8) & 0xff);
}

struct result {
	uint32_t edge, domain, iface, nh;
	uint32_t rx_if, rx_par, tx_if, tx_par; // counter keys (0 = none)
};


template <bool NT>
__device__ __forceinline__ u4v ld16(const uint8_t *p) {
	const u4v *q = reinterpret_cast<const u4v *>(p);
	if (NT)
		return __builtin_nontemporal_load(q);
	return *q;
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, u4v v) {
	u4v *q = reinterpret_cast<u4v *>(p);
	if (NT)
		__builtin_nontemporal_store(v, q);
	else
		*q = v;
}

