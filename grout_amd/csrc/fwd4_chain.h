// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_chain.h -- the node chain split at its dependent loads, for kernels
// that keep a tile's header lines in an LDS image (fwd4_ring.hip):
// chain_head (iface_input .. ip_input checks), chain_fib
// (fib4_lookup), chain_tail (adjacency .. iface_output, rewriting the row).
// Not a public header.
//
// LDS image of a 64-packet tile: row r (64 bytes) = packet r, its 16-byte
// chunk j at slot j ^ ((r >> 2) & 3) -- conflict-free both for the
// 4-lanes-per-row coalesced fill/drain and for one-row-per-lane reads.
#pragma once

#include "fib6.h" // the trie entry encoding chain_fib6 walks
#include "fwd4_dev.h"

// Kernel-wide view of the tables (read once per wave from fwd4_tables).
__device__ __forceinline__ kctx make_kctx(const fwd4_params &A, const fwd4_edges *edges) {
	const fwd4_tables *T = A.T;
	kctx P;
	P.T = T;
	P.rx = T->rx;
	P.max_ifaces = T->max_ifaces;
	P.max_nh = T->max_nh;
	P.readable = A.readable;
	P.edges = edges;
	P.stats = A.stats;
	P.ip4_edge = type_edge_of(*edges, 0x0008u);
	P.ip6_edge = type_edge_of(*edges, 0xdd86u);
	P.rx6 = T->rx6;
	P.nhf6_lds = nullptr; // set by the kernel that stages them
	P.nhf6_n = 0;
	P.top6 = nullptr;
	P.top6_lds = nullptr;
	P.top6_n = 0;
	return P;
}

// Byte offset of 16-byte chunk j of row r in a wave's LDS image.
__device__ __forceinline__ uint32_t row_off(uint32_t r, uint32_t j) {
	return r * 64 + ((j ^ ((r >> 2) & 3)) << 4);
}

__device__ __forceinline__ u4v lds_get(const uint8_t *R, uint32_t r, uint32_t j) {
	return *reinterpret_cast<const u4v *>(R + row_off(r, j));
}

__device__ __forceinline__ void lds_put(uint8_t *R, uint32_t r, uint32_t j, u4v v) {
	*reinterpret_cast<u4v *>(R + row_off(r, j)) = v;
}

__device__ __forceinline__ void compiler_fence() {
	asm volatile("" ::: "memory");
}

// RX view of a wave-uniform iface id through the scalar cache.
__device__ __forceinline__ rxv load_rx_scalar(const kctx &P, uint32_t id) {
	rxv r;
	r.id = 0;
	if (id == 0 || id >= P.max_ifaces)
		return r;
	typedef uint32_t u8s __attribute__((ext_vector_type(8)));
	u8s v;
	// the address is wave-uniform; say so, so that it is always in SGPRs
	const uint64_t a = reinterpret_cast<uint64_t>(P.rx + id);
	const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)), lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
	const uint64_t p = ((uint64_t)hi << 32) | lo;
	asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
	return unpack_rx(uint4{v[0], v[1], v[2], v[3]}, uint4{v[4], v[5], v[6], v[7]});
}

#define HEAD_DONE 0 // the packet left the chain, r.edge set
#define HEAD_IN4 1 // the packet left the chain in ip_input, r.edge set
#define HEAD_IP4 4 // continue to the IPv4 FIB lookup: dst, data_len set
#define HEAD_IP6 6 // continue into ip6_input (chain6): data_len set

// iface_input -> eth_input -> ip_input up to the FIB lookup, for the packet
// in row `row` of R. Returns HEAD_*; dst is the IPv4 destination in network
// order as stored.
__device__ __forceinline__ int chain_head(const kctx &P, const uint8_t *R, uint32_t row, const gr_hip_pkt_meta &m,
					  rxv &rx, result &r, uint32_t &dst, uint32_t &data_len, const uint8_t *frame) {
	// ---- iface_input (iface_input.c:52-112)
	if (rx.id == 0)
		return HEAD_DONE; // PUNT
	const uint32_t vlan = m.vlan_ck & 0xfff;
	if (vlan != 0 && (rx.flags & FWD4_RX_VLAN_DEMUX)) { // :74-86
		rxv v = load_rx(P, vlan_lookup(P, rx.id, vlan));
		if (v.id == 0) {
			r.edge = GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN;
			return HEAD_DONE;
		}
		rx = v;
	}
	r.iface = rx.id;
	if (rx.e_in != CHAIN) { // admin down :88-91, or the mode edge :97
		r.edge = rx.e_in;
		if (rx.e_in != GR_HIP_E_IFACE_INPUT_ADMIN_DOWN) {
			r.rx_if = rx.id;
			r.rx_par = m.iface != rx.id ? m.iface : 0;
		}
		return HEAD_DONE;
	}
	r.rx_if = rx.id; // IFACE_STATS_INC :93-95
	r.rx_par = m.iface != rx.id ? m.iface : 0;

	// ---- eth_input (eth_input.c:35-88)
	const u4v c0 = lds_get(R, row, 0);
	const uint32_t type_raw = lo16(c0.w);
	const uint32_t type = bswap16(type_raw);
	if (type < 1536 || type == 0x8870) { // snap.h:11-12
		r.edge = GR_HIP_E_SNAP_INPUT;
		return HEAD_DONE;
	}
	if (!(rx.flags & FWD4_RX_MAC_OK)) {
		r.edge = GR_HIP_E_ETH_INPUT_INVALID_IFACE;
		return HEAD_DONE;
	}
	if (c0.x & 1) {
		bool bc = c0.x == 0xffffffffu && lo16(c0.y) == 0xffff;
		r.domain = bc ? GR_HIP_ETH_DOMAIN_BROADCAST : GR_HIP_ETH_DOMAIN_MULTICAST;
	} else if (c0.x == rx.mac_lo && lo16(c0.y) == rx.mac_hi) {
		r.domain = GR_HIP_ETH_DOMAIN_LOCAL;
	} else {
		r.domain = GR_HIP_ETH_DOMAIN_OTHER;
	}
	data_len = m.pkt_len >= 14 ? m.pkt_len - 14u : m.pkt_len;
	const uint32_t e = eth_type_edge(P, type_raw);
	if (e == GR_HIP_EDGE_CHAIN6)
		return HEAD_IP6;
	if (e != CHAIN) {
		r.edge = e;
		return HEAD_DONE;
	}

	// ---- ip_input (ip_input.c:58-187)
	const uint32_t vihl = (c0.w >> 16) & 0xff;
	const uint32_t ihl = vihl & 0xf;
	if (data_len < 20) { // (1)
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return HEAD_IN4;
	}
	const u4v c1 = lds_get(R, row, 1);
	const u4v c2 = lds_get(R, row, 2);
	const uint32_t ck = (m.vlan_ck >> 12) & 3;
	if (ck == GR_HIP_CKSUM_UNKNOWN) { // (2) rte_ipv4_cksum over ihl*4 bytes
		const uint32_t hl = ihl * 4;
		if (14 + hl > P.readable) {
			r.edge = GR_HIP_E_PUNT;
			r.rx_if = r.rx_par = 0;
			r.domain = 0;
			r.iface = m.iface;
			return HEAD_IN4;
		}
		uint32_t sum = 0;
		if (ihl != 0) {
			const u4v c3 = lds_get(R, row, 3);
			const uint32_t w[12] = {c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
			sum = hi16(c0.w);
#pragma unroll
			for (uint32_t j = 4; j < 16; j++) {
				uint32_t v = w[j - 4];
				uint32_t full = lo16(v) + hi16(v);
				sum += (j <= 2 + ihl) ? full : (j == 3 + ihl ? lo16(v) : 0u);
			}
			if (ihl > 12) { // options reach past the line: bytes 64..73
				uint4 x = gld4(frame + 64);
				uint32_t xw[3] = {x.x, x.y, x.z};
#pragma unroll
				for (uint32_t j = 16; j < 19; j++) {
					uint32_t v = xw[j - 16];
					uint32_t full = lo16(v) + hi16(v);
					sum += (j <= 2 + ihl) ? full : (j == 3 + ihl ? lo16(v) : 0u);
				}
			}
		}
		sum = (sum & 0xffff) + (sum >> 16);
		sum = (sum & 0xffff) + (sum >> 16);
		if (sum != 0xffff) {
			r.edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
			return HEAD_IN4;
		}
	} else if (ck == GR_HIP_CKSUM_BAD) {
		r.edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
		return HEAD_IN4;
	}
	dst = hi16(c1.w) | (lo16(c2.x) << 16);
	if (dst == 0) {
		r.edge = GR_HIP_E_IP_INPUT_BAD_ADDRESS;
		return HEAD_IN4;
	}
	if ((vihl >> 4) != 4) { // (3)
		r.edge = GR_HIP_E_IP_INPUT_BAD_VERSION;
		return HEAD_IN4;
	}
	if (ihl * 4 < 20) { // (4)
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return HEAD_IN4;
	}
	if (bswap16(lo16(c1.x)) < 20) { // (5)
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return HEAD_IN4;
	}
	if (r.domain != GR_HIP_ETH_DOMAIN_LOCAL) {
		bool mc = r.domain == GR_HIP_ETH_DOMAIN_BROADCAST || r.domain == GR_HIP_ETH_DOMAIN_MULTICAST;
		r.edge = mc ? GR_HIP_E_IP_INPUT_LOCAL : GR_HIP_E_IP_INPUT_OTHER_HOST;
		return HEAD_IN4;
	}
	const uint32_t d0 = dst & 0xff;
	if (dst == 0xffffffffu || (d0 >= 224 && d0 <= 239)) {
		r.edge = GR_HIP_E_IP_INPUT_LOCAL;
		return HEAD_IN4;
	}
	return HEAD_IP4;
}

// fib4_lookup (modules/ip/control/route.c:147-167) in the iface's VRF table.
__device__ __forceinline__ uint32_t chain_fib(const rxv &rx, uint32_t dst) {
	if (rx.tbl24 == nullptr)
		return 0;
	const uint32_t ip = __builtin_bswap32(dst);
	if (rx.flags & FWD4_RX_FIB24W2) {
		uint32_t ent = gld(reinterpret_cast<const uint16_t *>(rx.tbl24) + (ip >> 8));
		if (ent & 0x8000u)
			ent = gld(reinterpret_cast<const uint16_t *>(rx.tbl8) + (size_t)(ent & 0x7fffu) * 256 + (ip & 0xff));
		return ent;
	}
	if (rx.flags & FWD4_RX_FIB16) {
		uint32_t ent = gld(rx.tbl24 + (ip >> 16));
		if (ent & 0x80000000u) {
			const uint16_t *chunks = reinterpret_cast<const uint16_t *>(rx.tbl24 + 65536);
			ent = gld(chunks + (size_t)(ent & 0x7fffffffu) * 256 + ((ip >> 8) & 0xff));
		}
		if (ent & 0x8000u)
			ent = gld(reinterpret_cast<const uint16_t *>(rx.tbl8) + (size_t)(ent & 0x7fffu) * 256 + (ip & 0xff));
		return ent;
	}
	uint32_t ent = gld(rx.tbl24 + (ip >> 8));
	if (ent & 0x80000000u)
		ent = gld(rx.tbl8 + (size_t)(ent & 0x7fffffffu) * 256 + (ip & 0xff));
	return ent;
}

// From the adjacency (its first 32 bytes in a, b) to the verdict:
// group resolution, ip_input's nexthop checks, ip_forward, ip_output,
// eth_output, iface_output. Rewrites row `row` of R.
__device__ __forceinline__ void chain_tail(const kctx &P, uint8_t *R, uint32_t row, const gr_hip_pkt_meta &m,
					  uint32_t rx_flags, result &r, uint32_t dst, uint32_t data_len, uint32_t slot,
					  uint4 a, uint4 b) {
	adjv A = unpack_adj(a, b, uint4{0, 0, 0, 0});
	if (A.type == GR_HIP_NH_T_GROUP) { // nexthop_group_get_nh, nexthop.h:89-96
		const uint4 c = gld4(reinterpret_cast<const uint4 *>(tload(&P.T->adj) + slot) + 2);
		const uint32_t n_members = c.x & 0xffff, reta_size = c.x >> 16;
		if (n_members == 1) {
			slot = c.z;
		} else if (n_members == 0) {
			slot = 0;
		} else {
			uint32_t i = c.y + (m.rss & (reta_size - 1));
			slot = i < tload(&P.T->reta_cap) ? gld(tload(&P.T->reta) + i) : 0;
		}
		if (slot == 0 || slot > P.max_nh) {
			r.edge = GR_HIP_E_IP_ERROR_DEST_UNREACH;
			return;
		}
		A = load_adj(P, slot);
	}
	r.nh = slot;
	if (A.e_in != CHAIN) {
		r.edge = A.e_in;
		return;
	}
	if ((A.flags & FWD4_ADJ_LOCAL) && dst == A.ipv4) {
		r.edge = (rx_flags & FWD4_RX_SNAT_DYN) ? GR_HIP_E_IP_INPUT_LOCAL_CT : GR_HIP_E_IP_INPUT_LOCAL;
		return;
	}

	// ---- ip_forward (ip_forward.c:21-33)
	u4v c1 = lds_get(R, row, 1); // bytes 16-31: w5 = c1.y (ttl), w6 = c1.z (cksum)
	const uint32_t ttl = (c1.y >> 16) & 0xff;
	if (ttl <= 1) {
		r.edge = GR_HIP_E_IP_ERROR_TTL_EXCEEDED;
		return;
	}
	c1.y = (c1.y & 0xff00ffffu) | ((ttl - 1) << 16);
	uint32_t ck = lo16(c1.z) + 1;
	ck += ck >= 0xffff;
	c1.z = (c1.z & 0xffff0000u) | (ck & 0xffff);
	lds_put(R, row, 1, c1);

	// ---- ip_output (ip_output.c:79-138)
	if (A.e_pre != CHAIN) {
		r.edge = A.e_pre;
		return;
	}
	r.iface = A.oif;
	if (data_len > A.mtu) {
		r.edge = (c1.y & 0x40) ? GR_HIP_E_IP_ERROR_FRAG_NEEDED : GR_HIP_E_IP_FRAGMENT;
		return;
	}
	if (A.e_mid != CHAIN) {
		r.edge = A.e_mid;
		return;
	}
	if ((A.flags & FWD4_ADJ_LINK) && dst != A.ipv4) {
		r.edge = GR_HIP_E_IP_HOLD;
		return;
	}

	// ---- eth_output (eth_output.c:43-62) + iface_output (iface_output.c:75-108)
	u4v c0 = lds_get(R, row, 0);
	c0.x = A.dmac_lo;
	c0.y = (c0.y & 0xffff0000u) | A.dmac_hi;
	r.edge = A.e_post;
	if (A.e_post != GR_HIP_E_ETH_OUTPUT_NO_MAC) {
		c0.y = lo16(c0.y) | (A.smac_lo << 16);
		c0.z = (A.smac_lo >> 16) | (A.smac_hi << 16);
		c0.w = (c0.w & 0xffff0000u) | 0x0008u;
		r.iface = A.post_iface;
		r.tx_if = A.tx_if;
		r.tx_par = A.tx_par;
	}
	lds_put(R, row, 0, c0);
}


// The plain forward of a fast adjacency f (fwd4_nhf as 4 words): the same
// steps and results as chain_tail for such a nexthop -- ip_forward
// (ip_forward.c:21-33), the MTU/DF check (ip_output.c:99-106), eth_output
// (eth_output.c:43-62) and iface_output to port_output.
__device__ __forceinline__ void fast_tail(uint8_t *R, uint32_t row, result &r, uint32_t data_len, uint32_t slot,
					  uint4 f) {
	r.nh = slot;
	u4v c1 = lds_get(R, row, 1);
	const uint32_t ttl = (c1.y >> 16) & 0xff;
	if (ttl <= 1) {
		r.edge = GR_HIP_E_IP_ERROR_TTL_EXCEEDED;
		return;
	}
	c1.y = (c1.y & 0xff00ffffu) | ((ttl - 1) << 16);
	uint32_t ck = lo16(c1.z) + 1;
	ck += ck >= 0xffff;
	c1.z = (c1.z & 0xffff0000u) | (ck & 0xffff);
	lds_put(R, row, 1, c1);
	const uint32_t oif = f.y >> 16;
	r.iface = oif;
	if (data_len > (f.w >> 16)) {
		r.edge = (c1.y & 0x40) ? GR_HIP_E_IP_ERROR_FRAG_NEEDED : GR_HIP_E_IP_FRAGMENT;
		return;
	}
	u4v c0 = lds_get(R, row, 0);
	c0.x = f.x;
	c0.y = (f.y & 0xffff) | (f.z << 16);
	c0.z = (f.z >> 16) | (f.w << 16);
	c0.w = (c0.w & 0xffff0000u) | 0x0008u;
	lds_put(R, row, 0, c0);
	r.edge = GR_HIP_E_PORT_OUTPUT;
	r.tx_if = oif;
}

// ---- IPv6: ip6_input -> ip6_forward -> ip6_output -> eth_output -> iface_output

// 32-bit word of the header line at byte offset 4 * k + 2 (the IPv6
// addresses start at 22 and 38): from the 16 little-endian line words.
__device__ __forceinline__ uint32_t word_at2(const uint32_t (&w)[16], int k) {
	return (w[k] >> 16) | (w[k + 1] << 16);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&a)[4], int i) {
	return (a[i >> 2] >> (8 * (i & 3))) & 0xff;
}

// The FIB6 view of RX iface `id` (its VRF's trie): through the scalar cache
// when the active lanes share the iface (a tile from one RX queue), as the
// IPv4 RX view is, since the trie walk's first gather waits for it.
__device__ __forceinline__ fwd4_rx6 load_rx6(const kctx &P, uint32_t id) {
	const uint32_t id0 = __builtin_amdgcn_readfirstlane(id);
	if (__ballot(id != id0) == 0) {
		typedef uint32_t u4s __attribute__((ext_vector_type(4)));
		typedef uint32_t u2s __attribute__((ext_vector_type(2)));
		const uint64_t a = reinterpret_cast<uint64_t>(P.rx6 + id0);
		const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)), lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
		const uint64_t p = ((uint64_t)hi << 32) | lo;
		u4s x;
		u2s y;
		asm volatile("s_load_dwordx4 %0, %2, 0x0\n\ts_load_dwordx2 %1, %2, 0x10\n\ts_waitcnt lgkmcnt(0)"
			     : "=&s"(x), "=&s"(y)
			     : "s"(p)
			     : "memory");
		fwd4_rx6 v;
		v.top = reinterpret_cast<const uint32_t *>(((uint64_t)x[1] << 32) | x[0]);
		v.groups = reinterpret_cast<const uint32_t *>(((uint64_t)x[3] << 32) | x[2]);
		v.skips = reinterpret_cast<const uint4 *>(((uint64_t)y[1] << 32) | y[0]);
		return v;
	}
	return fwd4_rx6{gld(&P.rx6[id].top), gld(&P.rx6[id].groups), gld(&P.rx6[id].skips)};
}

// rte_fib6_lookup (modules/ip6/control/route.c:150-173) in the fib6.h trie of the iface's VRF:
// key = dst with link-local addresses scoped to the ingress iface
// (addr6_linklocal_scope, ip6.h:23-36). chain6 runs it in two parts: the
// first level and the gather of the level after it before ip6_input's checks
// (fib6_first), so that they run while that gather is in flight, the rest
// after them (fib6_rest); a packet the checks stop discards the gather.

// Slot offset in the groups array of the element of entry `ent` (range, wide
// or plain group) for key byte b (and b + 1 for wide and range groups).
__device__ __forceinline__ size_t fib6_group_off(uint32_t ent, const uint32_t (&key)[4], int b) {
	const uint32_t kind = ent & GR_FIB6_RANGE;
	const uint32_t x = byte_of(key, b), y = b < 15 ? byte_of(key, b + 1) : 0;
	const uint32_t sh = (ent >> GR_FIB6_WIDE_SHIFT) & 7;
	return kind == GR_FIB6_RANGE ? (size_t)(ent & GR_FIB6_IDX) * 256 + 2 * x
	       : kind == GR_FIB6_WIDE ? (size_t)(ent & GR_FIB6_WIDE_IDX) * 256 + (x << (8 - sh)) + (y >> sh)
				      : (size_t)(ent & GR_FIB6_IDX) * 256 + x;
}

// The entry the gathered element q gives for entry `ent` of a range, wide or
// plain group at key byte b; b moves past the bytes it used.
__device__ __forceinline__ uint32_t fib6_group_next(uint32_t ent, u2a q, const uint32_t (&key)[4], int &b) {
	const uint32_t kind = ent & GR_FIB6_RANGE;
	const uint32_t y = b < 15 ? byte_of(key, b + 1) : 0;
	b += kind == 0 ? 1 : 2;
	return kind == GR_FIB6_RANGE ? (y >= (q.x >> 24) && y <= (q.y >> 24) ? q.x : q.y) & GR_FIB6_RANGE_LEAF : q.x;
}

// The scoped key and the first level's entry for it: from LDS where the
// launch staged it (2000::/4 of the only IPv6 VRF), else one gather. 0 (no
// route) without a trie.
__device__ __forceinline__ uint32_t fib6_first(const kctx &P, const fwd4_rx6 &v, const uint32_t (&dst)[4],
					       uint32_t iface_id, uint32_t (&key)[4]) {
	for (int i = 0; i < 4; i++)
		key[i] = dst[i];
	if (v.top == nullptr)
		return 0;
	if ((key[0] & 0xff) == 0xfe && (key[0] & 0xc000) == 0x8000)
		key[0] = (key[0] & 0xffff) | ((iface_id >> 8) << 16) | ((iface_id & 0xff) << 24);
	const uint32_t idx = (byte_of(key, 0) << 8) | byte_of(key, 1);
	const uint32_t k6 = idx - FWD4_TOP6_BASE;
	return v.top == P.top6 && k6 < P.top6_n ? P.top6_lds[k6] : gld(v.top + idx);
}

// The walk from entry `ent` at key byte b to the leaf: the nexthop slot, 0 =
// no route.
__device__ __forceinline__ uint32_t fib6_rest(const fwd4_rx6 &v, const uint32_t (&key)[4], uint32_t ent, int b) {
	while (b < 16 && (ent & 0x80000000u)) {
		if ((ent & GR_FIB6_RANGE) == GR_FIB6_SKIP) { // skip node: key bytes 0-6, n in byte 7
			const uint4 k = gld4(v.skips + (ent & GR_FIB6_IDX));
			const int n = k.y >> 24;
			bool match = b + n <= 16;
			for (int i = 0; i < n && match; i++)
				match = byte_of(key, b + i) == ((i < 4 ? k.x >> (8 * i) : k.y >> (8 * (i - 4))) & 0xff);
			ent = match ? k.z : k.w;
			b += n;
			continue;
		}
		// the three group kinds in one gather, so that a wave whose lanes sit
		// in different kinds issues one load per level, not one per kind
		// (each behind the one before); the 8 bytes at a 4-byte entry read
		// the next entry too (the groups are followed by the skip nodes)
		//   range group: entry {in | lo << 24, miss | hi << 24} by byte b
		//   wide group: byte b and the top 8 - s bits of byte b + 1 (b <= 14)
		//   plain group: byte b
		const u2a q = *(const GR_GLOBAL u2a *)(v.groups + fib6_group_off(ent, key, b));
		ent = fib6_group_next(ent, q, key, b);
	}
	return (ent & 0x80000000u) ? 0 : ent;
}

// From ip6_input (ip6_input.c:58-145) to iface_output for an IPv6 packet in
// row `row` of R, eth_input done (domain in r, data_len = the mbuf's after
// its adj). Rewrites the hop limit and the L2 header in R.
__device__ __forceinline__ void chain6(const kctx &P, uint8_t *R, uint32_t row, const gr_hip_pkt_meta &m,
				       const rxv &rx, result &r, uint32_t data_len) {
	if (data_len < 40) { // ip6_input.c:63-70
		r.edge = GR_HIP_E_IP6_INPUT_BAD_LENGTH;
		return;
	}
	uint32_t w[16];
#pragma unroll
	for (int k = 0; k < 4; k++) {
		const u4v c = lds_get(R, row, k);
		w[4 * k] = c.x;
		w[4 * k + 1] = c.y;
		w[4 * k + 2] = c.z;
		w[4 * k + 3] = c.w;
	}
	// IPv6 header at byte 14: version 14, hop limit 21, src 22-37, dst 38-53
	if ((((w[3] >> 16) & 0xff) & 0xf0) != 0x60) { // rte_ipv6_check_version, ip6_input.c:72-75
		r.edge = GR_HIP_E_IP6_INPUT_BAD_VERSION;
		return;
	}
	const uint32_t dst[4] = {word_at2(w, 9), word_at2(w, 10), word_at2(w, 11), word_at2(w, 12)};
	// the trie walk's first level and the gather after it, in flight under
	// the address checks below, which may discard them (they are
	// ip6_input.c:77-120)
	const fwd4_rx6 v6 = load_rx6(P, rx.id);
	uint32_t key[4];
	uint32_t ent = fib6_first(P, v6, dst, rx.id, key);
	int kb = 2; // the key byte ent indexes with
	const bool pend = (ent & 0x80000000u) && (ent & GR_FIB6_RANGE) != GR_FIB6_SKIP;
	u2a q = {0, 0};
	if (pend)
		q = *(const GR_GLOBAL u2a *)(v6.groups + fib6_group_off(ent, key, kb));
	const uint32_t src0 = (w[5] >> 16) & 0xff;
	if (src0 == 0xff || (dst[0] | dst[1] | dst[2] | dst[3]) == 0) { // mcast src, unspec dst, ip6_input.c:77-81
		r.edge = GR_HIP_E_IP6_INPUT_BAD_ADDR;
		return;
	}
	if ((dst[0] & 0xff) == 0xff) { // ip6_input.c:83-103
		const uint32_t scope = (dst[0] >> 8) & 0xf; // rte_ipv6_mc_scope
		if (scope <= 1) { // RTE_IPV6_MC_SCOPE_NONE / _IFACELOCAL
			r.edge = GR_HIP_E_IP6_INPUT_BAD_ADDR;
		} else { // mcast6_get_member: group membership lives on the CPU
			r.edge = GR_HIP_E_PUNT;
			r.rx_if = r.rx_par = 0;
			r.domain = 0;
			r.iface = m.iface;
		}
		return;
	}
	if (r.domain != GR_HIP_ETH_DOMAIN_LOCAL) { // ip6_input.c:105-120 (LOOPBACK never from a port)
		const bool mc = r.domain == GR_HIP_ETH_DOMAIN_BROADCAST || r.domain == GR_HIP_ETH_DOMAIN_MULTICAST;
		r.edge = mc ? GR_HIP_E_IP6_INPUT_LOCAL : GR_HIP_E_IP6_INPUT_OTHER_HOST;
		return;
	}
	if (pend) // ip6_input.c:124-131
		ent = fib6_group_next(ent, q, key, kb);
	uint32_t slot = fib6_rest(v6, key, ent, kb);
	if (slot == 0 || slot > P.max_nh) {
		r.edge = GR_HIP_E_IP6_ERROR_DEST_UNREACH;
		return;
	}
	{
		// fast adjacency (make_nhf6: L3, no LOCAL/LINK flag, every edge chains to
		// port_output of a port): ip6_forward, ip6_output, eth_output and
		// iface_output on its MACs, oif and MTU alone -- the same steps and
		// results as below for such a nexthop
		uint4 f;
		if (slot <= P.nhf6_n) {
			const u4v v = P.nhf6_lds[slot - 1];
			f = uint4{v.x, v.y, v.z, v.w};
		} else {
			f = gld4(tload(&P.T->nhf6) + slot);
		}
		if (f.w >> 16) {
			r.nh = slot;
			const uint32_t hop = (w[5] >> 8) & 0xff;
			if (hop <= 1) { // ip6_forward.c:25-30
				r.edge = GR_HIP_E_IP6_ERROR_TTL_EXCEEDED;
				return;
			}
			u4v c1 = lds_get(R, row, 1);
			c1.y = (c1.y & 0xffff00ffu) | ((hop - 1) << 8);
			lds_put(R, row, 1, c1);
			if (data_len > (f.w >> 16)) { // ip6_output.c:97-100
				r.edge = GR_HIP_E_IP6_OUTPUT_TOO_BIG;
				return;
			}
			const uint32_t oif = f.y >> 16;
			u4v c0 = lds_get(R, row, 0);
			c0.x = f.x;
			c0.y = (f.y & 0xffff) | (f.z << 16);
			c0.z = (f.z >> 16) | (f.w << 16);
			c0.w = (c0.w & 0xffff0000u) | 0xdd86u;
			lds_put(R, row, 0, c0);
			r.iface = oif;
			r.edge = GR_HIP_E_PORT_OUTPUT;
			r.tx_if = oif;
			return;
		}
	}
	const fwd4_adj6 *adj6 = tload(&P.T->adj6);
	const uint4 *ap = reinterpret_cast<const uint4 *>(adj6 + slot);
	uint4 a = gld4(ap), b = gld4(ap + 1), c = gld4(ap + 2);
	if ((a.x & 0xff) == GR_HIP_NH_T_GROUP) { // nexthop_group_get_nh, nexthop.h:89-96
		const uint4 g = gld4(reinterpret_cast<const uint4 *>(tload(&P.T->adj) + slot) + 2);
		const uint32_t n_members = g.x & 0xffff, reta_size = g.x >> 16;
		if (n_members == 1) {
			slot = g.z;
		} else if (n_members == 0) {
			slot = 0;
		} else {
			const uint32_t i = g.y + (m.rss & (reta_size - 1));
			slot = i < tload(&P.T->reta_cap) ? gld(tload(&P.T->reta) + i) : 0;
		}
		if (slot == 0 || slot > P.max_nh) {
			r.edge = GR_HIP_E_IP6_ERROR_DEST_UNREACH;
			return;
		}
		ap = reinterpret_cast<const uint4 *>(adj6 + slot);
		a = gld4(ap);
		b = gld4(ap + 1);
		c = gld4(ap + 2);
	}
	r.nh = slot; // l3_mbuf_data(mbuf)->nh, ip6_input.c:151-153
	const uint32_t e_in = (a.x >> 8) & 0xff, flags = (a.x >> 16) & 0xff;
	if (e_in != CHAIN) { // nh_type_edges, ip6_input.c:133-135
		r.edge = e_in;
		return;
	}
	const bool is_nh = dst[0] == b.w && dst[1] == c.x && dst[2] == c.y && dst[3] == c.z;
	if ((flags & FWD4_ADJ_LOCAL) && is_nh) { // ip6_input.c:139-144
		r.edge = GR_HIP_E_IP6_INPUT_LOCAL;
		return;
	}

	// ---- ip6_forward (ip6_forward.c:25-30)
	const uint32_t hop = (w[5] >> 8) & 0xff;
	if (hop <= 1) {
		r.edge = GR_HIP_E_IP6_ERROR_TTL_EXCEEDED;
		return;
	}
	u4v c1 = lds_get(R, row, 1);
	c1.y = (c1.y & 0xffff00ffu) | ((hop - 1) << 8);
	lds_put(R, row, 1, c1);

	// ---- ip6_output (ip6_output.c:75-134), adjacency resolved ahead of time
	const uint32_t e_pre = a.x >> 24, e_mid = a.y & 0xff, e_post = (a.y >> 8) & 0xff;
	if (e_pre != CHAIN) { // nh type edge ip6_output.c:83-85, no iface :92-95
		r.edge = e_pre;
		return;
	}
	if (data_len > (a.z & 0xffff)) { // rte_pktmbuf_pkt_len > mtu, ip6_output.c:97-100
		r.edge = GR_HIP_E_IP6_OUTPUT_TOO_BIG;
		return;
	}
	r.iface = a.y >> 16; // mbuf_data(mbuf)->iface = iface, ip6_output.c:105
	if (e_mid != CHAIN) { // iface type edge ip6_output.c:104-107, state :111-117
		r.edge = e_mid;
		return;
	}
	if ((flags & FWD4_ADJ_LINK) && !is_nh) { // ip6_output.c:111-117
		r.edge = GR_HIP_E_IP6_HOLD;
		return;
	}

	// ---- eth_output (eth_output.c:43-62) + iface_output (iface_output.c:75-108)
	u4v c0 = lds_get(R, row, 0);
	c0.x = b.x; // dst MAC 0-3
	c0.y = (c0.y & 0xffff0000u) | (b.y & 0xffff); // dst MAC 4-5
	r.edge = e_post;
	if (e_post != GR_HIP_E_ETH_OUTPUT_NO_MAC) {
		c0.y = b.y; // dst MAC 4-5, src MAC 0-1
		c0.z = b.z; // src MAC 2-5
		c0.w = (c0.w & 0xffff0000u) | 0xdd86u; // RTE_BE16(RTE_ETHER_TYPE_IPV6)
		r.iface = a.z >> 16;
		r.tx_if = a.w & 0xffff;
		r.tx_par = a.w >> 16;
	}
	lds_put(R, row, 0, c0);
}

// ---- eth_output's per-walk source-MAC cache (eth_output.c:37-59)
//
// eth_output looks the source MAC up only when the packet's iface differs
// from the last one it looked up in this graph walk (last_iface_id, which a
// failed lookup leaves unchanged); a failed lookup (eth_output_no_mac)
// zeroes the cached MAC. So a packet of the cached iface that follows a
// no-MAC packet in the same walk leaves with source MAC 00:00:00:00:00:00.
// Walks lie inside a 64-packet tile (GR_HIP_META_WALK): a wave resolves its
// tile's walks after the chain, only when one of its packets is no-MAC.
//
// eth_output's stream in a walk is rte_graph's order: the IPv4 packets that
// reached it (in RX order), then the IPv6 ones -- or the other way round when
// ip6_input received a packet before ip_input did (the walk's pending queue
// runs ip6_input -> ip6_forward -> ip6_output first).

// The packet went through eth_output to an iface_output edge.
__device__ __forceinline__ bool past_eth_output(uint32_t edge, uint32_t nh) {
	return (edge >= GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE && edge <= GR_HIP_E_PORT_OUTPUT)
		|| (edge == GR_HIP_E_BRIDGE_INPUT && nh != 0);
}

// fam: 1 = the packet entered ip_input, 2 = ip6_input, 0 = neither.
// Returns whether lane's row must get a zero source MAC. Wave-converged.
__device__ bool eth_output_walks(const kctx &P, uint32_t lane, bool live, bool walk_bit, uint32_t fam, const result &r) {
	static_assert(GR_HIP_E_PORT_OUTPUT - GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE == 5, "iface_output edges");
	const bool nomac = live && r.edge == GR_HIP_E_ETH_OUTPUT_NO_MAC;
	const bool out = live && past_eth_output(r.edge, r.nh);
	uint32_t eo = 0; // priv->iface at eth_output: the nexthop's iface (ip_output.c:91-97)
	if (nomac)
		eo = r.iface;
	else if (out)
		eo = fam == 2 ? gld(&tload(&P.T->adj6)[r.nh].oif) : gld(&tload(&P.T->adj)[r.nh].oif);
	const uint64_t E = __ballot(nomac || out), N = __ballot(nomac);
	const uint64_t F4 = __ballot(live && fam == 1), F6 = __ballot(live && fam == 2);
	uint64_t starts = __ballot(live && walk_bit) | 1;
	uint64_t zero = 0;
	while (starts) {
		const uint32_t b = (uint32_t)__builtin_ctzll(starts);
		starts &= starts - 1;
		const uint32_t e = starts ? (uint32_t)__builtin_ctzll(starts) : 64;
		const uint64_t w = (e == 64 ? ~0ull : (1ull << e) - 1) & ~((1ull << b) - 1);
		if ((E & N & w) == 0)
			continue; // no failed lookup in this walk: every packet has its iface's MAC
		const uint64_t f4 = F4 & w, f6 = F6 & w;
		const bool six_first = f6 != 0 && (f4 == 0 || __builtin_ctzll(f6) < __builtin_ctzll(f4));
		uint32_t last = GR_HIP_IFACE_ID_UNDEF;
		bool cleared = false; // the cached source MAC was zeroed
		for (int pass = 0; pass < 2; pass++) {
			uint64_t s = E & ((pass == 0) == six_first ? f6 : f4);
			while (s) {
				const uint32_t i = (uint32_t)__builtin_ctzll(s);
				s &= s - 1;
				const uint32_t ifc = __builtin_amdgcn_readlane(eo, i);
				if (ifc != last) {
					if ((N >> i) & 1) { // iface_get_eth_addr failed: src_mac zeroed, last kept
						cleared = true;
						continue;
					}
					last = ifc;
					cleared = false;
				} else if (cleared) {
					zero |= 1ull << i;
				}
			}
		}
	}
	return (zero >> lane) & 1;
}
