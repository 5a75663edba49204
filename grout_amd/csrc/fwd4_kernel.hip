// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_kernel.hip -- the fused IPv4 forwarding kernel for gfx950 (MI355X).
//
// One lane per packet. A 256-thread workgroup (4 wave64s) owns a tile of 256
// packets: their 64-byte header lines are staged into LDS with coalesced
// 16-byte loads (4 lanes per line), each lane then walks its packet through
//   iface_input (iface_input.c:52-112) -> eth_input (eth_input.c:35-88)
//   -> ip_input (ip_input.c:47-197) with the DIR24_8 lookup of fib4_lookup
//      (route.c:147-167) and group resolution (nexthop.h:89-96)
//   -> ip_forward (ip_forward.c:14-41) -> ip_output (ip_output.c:122-223)
//   -> eth_output (eth_output.c:28-77) -> iface_output (iface_output.c:198-255)
// entirely in registers, and the rewritten lines leave through LDS with
// coalesced 16-byte stores. Per-iface rx/tx counters are reduced per wave
// (ballot), per workgroup (LDS slot table) and flushed once per workgroup to
// a sharded global table. The grid is persistent (<= 8 workgroups per CU) and
// strides over tiles. No MFMA: this is HBM-bound integer work.
#include "fwd4_dev.h"

// The node chain for one packet. w[] is the 64-byte line (little-endian
// words: byte j is (w[j/4] >> 8*(j%4)) & 0xff), modified in place.
__device__ __forceinline__ result process(const kctx &P, uint32_t (&w)[16], const gr_hip_pkt_meta &m, const uint8_t *frame) {
	result r = {GR_HIP_E_PUNT, 0, m.iface, 0, 0, 0, 0, 0};

	// ---- iface_input (iface_input.c:52-112)
	rxv rx = load_rx(P, m.iface);
	if (rx.id == 0)
		return r; // port_rx always sets a valid iface: not grout's case, punt
	const uint32_t vlan = m.vlan_ck & 0xfff;
	if (vlan != 0 && (rx.flags & FWD4_RX_VLAN_DEMUX)) { // :74-86
		rxv v = load_rx(P, vlan_lookup(P, rx.id, vlan));
		if (v.id == 0) {
			r.edge = GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN;
			return r;
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
		return r;
	}
	r.rx_if = rx.id; // IFACE_STATS_INC :93-95
	r.rx_par = m.iface != rx.id ? m.iface : 0;

	// ---- eth_input (eth_input.c:35-88)
	const uint32_t type_raw = lo16(w[3]); // as stored (big endian)
	const uint32_t type = bswap16(type_raw);
	if (type < 1536 || type == 0x8870) { // snap.h:11-12
		r.edge = GR_HIP_E_SNAP_INPUT;
		return r;
	}
	if (!(rx.flags & FWD4_RX_MAC_OK)) { // iface_get_eth_addr() < 0
		r.edge = GR_HIP_E_ETH_INPUT_INVALID_IFACE;
		return r;
	}
	if (w[0] & 1) { // rte_is_multicast_ether_addr
		bool bc = w[0] == 0xffffffffu && lo16(w[1]) == 0xffff;
		r.domain = bc ? GR_HIP_ETH_DOMAIN_BROADCAST : GR_HIP_ETH_DOMAIN_MULTICAST;
	} else if (w[0] == rx.mac_lo && lo16(w[1]) == rx.mac_hi) {
		r.domain = GR_HIP_ETH_DOMAIN_LOCAL;
	} else {
		r.domain = GR_HIP_ETH_DOMAIN_OTHER;
	}
	const uint32_t data_len = m.pkt_len >= 14 ? m.pkt_len - 14u : m.pkt_len; // rte_pktmbuf_adj
	const uint32_t e = eth_type_edge(P, type_raw); // l2l3_edges[ether_type]
	if (e != CHAIN) {
		r.edge = e;
		return r;
	}

	// ---- ip_input (ip_input.c:58-187); the IPv4 header starts at byte 14
	const uint32_t vihl = (w[3] >> 16) & 0xff;
	const uint32_t ihl = vihl & 0xf;
	if (data_len < 20) { // (1) :70-77
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return r;
	}
	const uint32_t ck = (m.vlan_ck >> 12) & 3;
	if (ck == GR_HIP_CKSUM_UNKNOWN) { // (2) :80-88, rte_ipv4_cksum
		const uint32_t hl = ihl * 4;
		if (14 + hl > P.readable) {
			r.edge = GR_HIP_E_PUNT; // header bytes not present: CPU path
			r.rx_if = r.rx_par = 0;
			r.domain = 0;
			r.iface = m.iface;
			return r;
		}
		// rte_raw_cksum over hl bytes: 16-bit LE words at offsets 14, 16, ...
		uint32_t sum = 0;
		if (ihl != 0) {
			sum = hi16(w[3]);
#pragma unroll
			for (uint32_t j = 4; j < 16; j++) {
				uint32_t full = lo16(w[j]) + hi16(w[j]);
				sum += (j <= 2 + ihl) ? full : (j == 3 + ihl ? lo16(w[j]) : 0u);
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
		if (sum != 0xffff) { // (uint16_t)~sum != 0
			r.edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
			return r;
		}
	} else if (ck == GR_HIP_CKSUM_BAD) { // :89-91
		r.edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
		return r;
	}
	const uint32_t dst = hi16(w[7]) | (lo16(w[8]) << 16); // network order, as stored
	if (dst == 0) { // :94-97
		r.edge = GR_HIP_E_IP_INPUT_BAD_ADDRESS;
		return r;
	}
	if ((vihl >> 4) != 4) { // (3) :102-105
		r.edge = GR_HIP_E_IP_INPUT_BAD_VERSION;
		return r;
	}
	if (ihl * 4 < 20) { // (4) :109-112
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return r;
	}
	if (bswap16(lo16(w[4])) < 20) { // (5) :117-120
		r.edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
		return r;
	}
	if (r.domain != GR_HIP_ETH_DOMAIN_LOCAL) { // :122-137 (LOOPBACK never from a port)
		bool mc = r.domain == GR_HIP_ETH_DOMAIN_BROADCAST || r.domain == GR_HIP_ETH_DOMAIN_MULTICAST;
		r.edge = mc ? GR_HIP_E_IP_INPUT_LOCAL : GR_HIP_E_IP_INPUT_OTHER_HOST;
		return r;
	}
	const uint32_t d0 = dst & 0xff;
	if (dst == 0xffffffffu || (d0 >= 224 && d0 <= 239)) { // :139-142
		r.edge = GR_HIP_E_IP_INPUT_LOCAL;
		return r;
	}
	// fib4_lookup (route.c:147-167): DIR24_8 of the iface's VRF
	uint32_t slot = 0;
	if (rx.tbl24 != nullptr) {
		const uint32_t ip = __builtin_bswap32(dst);
		if (rx.flags & FWD4_RX_FIB16) { // DIR-16-8-8, 2-byte entries, bit15 = tbl8 group
			uint32_t ent = gld(rx.tbl24 + (ip >> 16)); // top: bit31 = chunk of 256 /24 entries
			if (ent & 0x80000000u) {
				const uint16_t *chunks = reinterpret_cast<const uint16_t *>(rx.tbl24 + 65536);
				ent = gld(chunks + (size_t)(ent & 0x7fffffffu) * 256 + ((ip >> 8) & 0xff));
			}
			if (ent & 0x8000u)
				ent = gld(reinterpret_cast<const uint16_t *>(rx.tbl8) + (size_t)(ent & 0x7fffu) * 256 + (ip & 0xff));
			slot = ent;
		} else {
			uint32_t ent = gld(rx.tbl24 + (ip >> 8));
			if (ent & 0x80000000u)
				ent = gld(rx.tbl8 + (size_t)(ent & 0x7fffffffu) * 256 + (ip & 0xff));
			slot = ent;
		}
	}
	if (slot == 0 || slot > P.max_nh) {
		r.edge = GR_HIP_E_IP_ERROR_DEST_UNREACH; // NO_ROUTE :150-153
		return r;
	}
	adjv a = load_adj(P, slot);
	if (a.type == GR_HIP_NH_T_GROUP) { // nexthop_group_get_nh, nexthop.h:89-96
		if (a.n_members == 1) {
			slot = a.single;
		} else if (a.n_members == 0) {
			slot = 0;
		} else {
			uint32_t i = a.reta_off + (m.rss & (a.reta_size - 1));
			slot = i < P.reta_cap ? gld(P.reta + i) : 0;
		}
		if (slot == 0 || slot > P.max_nh) {
			r.edge = GR_HIP_E_IP_ERROR_DEST_UNREACH;
			return r;
		}
		a = load_adj(P, slot);
	}
	r.nh = slot; // l3_mbuf_data(mbuf)->nh :156
	if (a.e_in != CHAIN) { // nh_type_edges :158-160
		r.edge = a.e_in;
		return r;
	}
	if ((a.flags & FWD4_ADJ_LOCAL) && dst == a.ipv4) { // :166-187
		r.edge = (rx.flags & FWD4_RX_SNAT_DYN) ? GR_HIP_E_IP_INPUT_LOCAL_CT : GR_HIP_E_IP_INPUT_LOCAL;
		return r;
	}

	// ---- ip_forward (ip_forward.c:21-33)
	const uint32_t ttl = (w[5] >> 16) & 0xff;
	if (ttl <= 1) {
		r.edge = GR_HIP_E_IP_ERROR_TTL_EXCEEDED;
		return r;
	}
	w[5] = (w[5] & 0xff00ffffu) | ((ttl - 1) << 16);
	uint32_t c = lo16(w[6]) + 1; // host-order u16 + RTE_BE16(0x0100)
	c += c >= 0xffff;
	w[6] = (w[6] & 0xffff0000u) | (c & 0xffff);

	// ---- ip_output (ip_output.c:135-213), adjacency resolved ahead of time
	if (a.e_pre != CHAIN) { // nh type edge :147-149, no iface :151-155
		r.edge = a.e_pre;
		return r;
	}
	r.iface = a.oif; // :157
	if (data_len > a.mtu) { // :159-166, DF = BE 0x4000 -> byte 20 & 0x40
		r.edge = (w[5] & 0x40) ? GR_HIP_E_IP_ERROR_FRAG_NEEDED : GR_HIP_E_IP_FRAGMENT;
		return r;
	}
	if (a.e_mid != CHAIN) { // SNAT :172-179, iface type edge :170,181, state :186
		r.edge = a.e_mid;
		return r;
	}
	if ((a.flags & FWD4_ADJ_LINK) && dst != a.ipv4) { // :187
		r.edge = GR_HIP_E_IP_HOLD;
		return r;
	}

	// ---- eth_output (eth_output.c:297-316) + iface_output (iface_output.c:213-246)
	w[0] = a.dmac_lo;
	w[1] = (w[1] & 0xffff0000u) | a.dmac_hi;
	r.edge = a.e_post;
	if (a.e_post == GR_HIP_E_ETH_OUTPUT_NO_MAC)
		return r;
	w[1] = lo16(w[1]) | (a.smac_lo << 16);
	w[2] = (a.smac_lo >> 16) | (a.smac_hi << 16);
	w[3] = (w[3] & 0xffff0000u) | 0x0008u; // RTE_BE16(RTE_ETHER_TYPE_IPV4)
	r.iface = a.post_iface;
	r.tx_if = a.tx_if;
	r.tx_par = a.tx_par;
	return r;
}

// STATS: per-iface counters. NT: nontemporal loads and stores of the streamed
// lines, metadata and verdicts (keeps L2 for the FIB gathers). TILE: packets
// per workgroup = threads per workgroup (64: one wave, 256: four waves).
template <bool STATS, bool NT, int TILE>
__global__ void __launch_bounds__(TILE) gr_fwd4_kernel(const fwd4_params A) {
	__shared__ __attribute__((aligned(16))) uint8_t lines[TILE * FWD4_ROW];
	__shared__ stat_slot slots[FWD4_STAT_SLOTS];
	__shared__ fwd4_edges edges;
	const uint32_t tid = threadIdx.x;
	const fwd4_tables *T = A.T;

	for (uint32_t i = tid; i < sizeof(fwd4_edges); i += TILE)
		reinterpret_cast<uint8_t *>(&edges)[i] = reinterpret_cast<const uint8_t *>(&T->edges)[i];
	if (STATS && tid < FWD4_STAT_SLOTS) {
		slots[tid].key = 0;
		slots[tid].pkts = 0;
		slots[tid].bytes = 0;
	}
	kctx P;
	P.rx = T->rx;
	P.adj = T->adj;
	P.reta = T->reta;
	P.vlan_keys = T->vlan_keys;
	P.vlan_vals = T->vlan_vals;
	P.reta_cap = T->reta_cap;
	P.vlan_mask = T->vlan_mask;
	P.max_ifaces = T->max_ifaces;
	P.max_nh = T->max_nh;
	P.readable = A.readable;
	P.edges = &edges;
	P.stats = A.stats;
	__syncthreads();
	P.ip4_edge = ip4_edge_of(edges);

	const uint32_t n_tiles = (A.n + TILE - 1) / TILE;
	for (uint32_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
		const uint32_t base = tile * TILE;
		const uint32_t cnt = min((uint32_t)TILE, A.n - base);
		const bool live = tid < cnt;
		gr_hip_pkt_meta m = {0, 0, 0, 0};
		if (live) {
			u2v mm;
			const u2v *mp = reinterpret_cast<const u2v *>(A.meta + base + tid);
			if (NT)
				mm = __builtin_nontemporal_load(mp);
			else
				mm = *mp;
			m.iface = mm.x & 0xffff;
			m.vlan_ck = mm.x >> 16;
			m.pkt_len = mm.y & 0xffff;
			m.rss = mm.y >> 16;
		}
		// stage: 4 lanes per 64-byte line, 16 bytes each (coalesced)
#pragma unroll
		for (uint32_t k = 0; k < 4; k++) {
			uint32_t c = k * TILE + tid;
			uint32_t p = c >> 2, part = c & 3;
			if (p < cnt)
				*reinterpret_cast<u4v *>(&lines[p * FWD4_ROW + part * 16]) =
					ld16<NT>(A.in + (size_t)(base + p) * A.in_stride + part * 16);
		}
		__syncthreads();

		result r = {0, 0, 0, 0, 0, 0, 0, 0};
		if (live) {
			uint32_t w[16];
			u4v *row = reinterpret_cast<u4v *>(&lines[tid * FWD4_ROW]);
#pragma unroll
			for (int k = 0; k < 4; k++) {
				u4v x = row[k];
				w[4 * k] = x.x;
				w[4 * k + 1] = x.y;
				w[4 * k + 2] = x.z;
				w[4 * k + 3] = x.w;
			}
			const uint8_t *frame = A.in + (size_t)(base + tid) * A.in_stride;
			r = process(P, w, m, frame);
#pragma unroll
			for (int k = 0; k < 4; k++)
				row[k] = u4v{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
			u2v vv = u2v{r.edge | (r.domain << 8) | (r.iface << 16), r.nh};
			u2v *vp = reinterpret_cast<u2v *>(A.verdicts + base + tid);
			if (NT)
				__builtin_nontemporal_store(vv, vp);
			else
				*vp = vv;
		}
		// counter keys, packed: rx | rx_par << 16, tx | tx_par << 16
		const uint32_t rxk = r.rx_if | (r.rx_par << 16), txk = r.tx_if | (r.tx_par << 16);
		const uint32_t len = m.pkt_len;
		__syncthreads();
#pragma unroll
		for (uint32_t k = 0; k < 4; k++) {
			uint32_t c = k * TILE + tid;
			uint32_t p = c >> 2, part = c & 3;
			if (p < cnt)
				st16<NT>(A.out + (size_t)(base + p) * A.out_stride + part * 16,
					 *reinterpret_cast<const u4v *>(&lines[p * FWD4_ROW + part * 16]));
		}
		if (STATS) { // every lane of the wave takes part in the ballots
			wave_count(slots, P, (rxk & 0xffff) ? (rxk & 0xffff) + 1 : 0, len);
			wave_count(slots, P, (rxk >> 16) ? (rxk >> 16) + 1 : 0, len);
			wave_count(slots, P, (txk & 0xffff) ? ((txk & 0xffff) | 0x10000u) + 1 : 0, len);
			wave_count(slots, P, (txk >> 16) ? ((txk >> 16) | 0x10000u) + 1 : 0, len);
		}
		if (tile + gridDim.x < n_tiles)
			__syncthreads(); // the next tile reuses the LDS rows
	}

	if (STATS) {
		__syncthreads();
		if (tid < FWD4_STAT_SLOTS && slots[tid].key != 0) {
			const uint32_t key = slots[tid].key - 1;
			shard_add(A.stats, P.max_ifaces, key >> 16, key & 0xffff, slots[tid].pkts, slots[tid].bytes);
		}
	}
}

typedef void (*fwd4_kfn)(const fwd4_params);
#define KV(v) gr_fwd4_kernel<((v) & 1) != 0, ((v) & 2) != 0, ((v) & 4) ? 64 : 256>
static const fwd4_kfn kernels[8] = {KV(0), KV(1), KV(2), KV(3), KV(4), KV(5), KV(6), KV(7)};

static uint32_t tile_of(int variant) {
	return (variant & FWD4_V_TILE64) ? 64 : 256;
}

// variant: FWD4_V_* bits (counters, nontemporal streams, 64-packet tiles).
extern "C" hipError_t gr_fwd4_launch(const fwd4_params *A, uint32_t grid, hipStream_t s, int variant) {
	hipLaunchKernelGGL(kernels[variant & 7], dim3(grid), dim3(tile_of(variant)), 0, s, *A);
	return hipGetLastError();
}

extern "C" uint32_t gr_fwd4_tile(int variant) {
	return tile_of(variant);
}

// Resident workgroups per CU of a variant.
extern "C" int gr_fwd4_occupancy(int variant) {
	int b = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernels[variant & 7], (int)tile_of(variant), 0) != hipSuccess) {
		(void)hipGetLastError();
		return 0;
	}
	return b;
}
