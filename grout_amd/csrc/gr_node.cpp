// SPDX-License-Identifier: BSD-3-Clause
//
// gr_node.cpp -- the host half of the rte_graph node that hands packets to
// the fast path and back (include/grout_hip.h, "rte_graph node shim").
//
// Staging copies each mbuf's header line and metadata out; the hand-back
// puts each mbuf in the state grout's CPU chain leaves it at the verdict's
// edge. Which node a packet stopped in decides the mbuf fields:
//
//   node              data_off      packet_type  vlan_id                frame bytes
//   iface_input       +0            -            0 if VLAN-demuxed      -
//   eth_input         +0 / +14 (1)  -            0 if demuxed           -
//   ip(6)_input       +14           -            0 if demuxed           -
//   ip(6)_forward     +14           -            0 if demuxed           -
//   ip(6)_output      +14           L3_IPV4/6    0 if demuxed           TTL + checksum / hop limit
//   eth_output        +0 (2)        L3_IPV4/6    0                      + dst MAC
//   iface_output      +0 (2)        L3_IPV4/6    egress VLAN tag or 0   + bytes 6-13
//
// An IPv4 packet walks iface_input, eth_input, ip_input, ip_forward,
// ip_output, eth_output, iface_output; an IPv6 packet the ip6_* nodes in the
// middle (ip6_input.c, ip6_forward.c, ip6_output.c).
//
// (1) snap_input and eth_input_invalid_iface leave eth_input before its
//     rte_pktmbuf_adj(14) (eth_input.c:55-66 vs :80); adj is a no-op on a
//     frame shorter than 14 bytes (DPDK rte_pktmbuf_adj).
// (2) eth_output's gr_mbuf_prepend(14) (eth_output.c:43, mbuf.h:89-106)
//     undoes the adj: net data_off unchanged vs RX.
// vlan_id: iface_input clears it when it demuxes a tagged packet to a VLAN
// sub-interface (iface_input.c:74-86), eth_output clears it
// (eth_output.c:71), iface_output sets the egress VLAN's id
// (iface_output.c:81-86).
#include "gr_node_priv.h"

#include <errno.h>
#include <stddef.h>
#include <string.h>

static_assert(sizeof(struct gr_hip_mbuf) == 40 && offsetof(struct gr_hip_mbuf, nh) == 32, "gr_hip_mbuf layout");
static_assert(sizeof(struct gr_hip_node_stats) == 16 * GR_HIP_NODE_COUNT, "gr_hip_node_stats layout");

static inline int edge_node(uint8_t edge, uint32_t nh, int ip6) {
	switch (edge) {
	case GR_HIP_E_PUNT:
		return -1;
	case GR_HIP_E_IFACE_MODE_UNKNOWN:
	case GR_HIP_E_IFACE_INPUT_ADMIN_DOWN:
	case GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN:
	case GR_HIP_E_XCONNECT:
		return GR_HIP_NODE_IFACE_INPUT;
	case GR_HIP_E_BRIDGE_INPUT: // an iface_input mode edge and an iface_output type edge
		return nh ? GR_HIP_NODE_IFACE_OUTPUT : GR_HIP_NODE_IFACE_INPUT;
	case GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE:
	case GR_HIP_E_ETH_INPUT_INVALID_IFACE:
	case GR_HIP_E_SNAP_INPUT:
	case GR_HIP_E_ARP_INPUT:
	case GR_HIP_E_IP6_INPUT:
	case GR_HIP_E_LACP_INPUT:
		return GR_HIP_NODE_ETH_INPUT;
	case GR_HIP_E_IP_INPUT_LOCAL:
	case GR_HIP_E_IP_INPUT_LOCAL_CT:
	case GR_HIP_E_IP_ERROR_DEST_UNREACH:
	case GR_HIP_E_IP_INPUT_BAD_CHECKSUM:
	case GR_HIP_E_IP_INPUT_BAD_ADDRESS:
	case GR_HIP_E_IP_INPUT_BAD_LENGTH:
	case GR_HIP_E_IP_INPUT_BAD_VERSION:
	case GR_HIP_E_IP_INPUT_OTHER_HOST:
	case GR_HIP_E_IP_BLACKHOLE:
	case GR_HIP_E_DNAT44_STATIC:
		return GR_HIP_NODE_IP_INPUT;
	case GR_HIP_E_IP_ERROR_TTL_EXCEEDED:
		return GR_HIP_NODE_IP_FORWARD;
	case GR_HIP_E_IP_HOLD:
	case GR_HIP_E_IP_OUTPUT_ERROR:
	case GR_HIP_E_IP_FRAGMENT:
	case GR_HIP_E_IP_ERROR_FRAG_NEEDED:
	case GR_HIP_E_IPIP_OUTPUT:
	case GR_HIP_E_IP_OUTPUT_SNAT:
		return GR_HIP_NODE_IP_OUTPUT;
	case GR_HIP_E_SR6_OUTPUT: // nh type edge of both ip_output and ip6_output
	case GR_HIP_E_XVRF: // iface type edge of both
		return ip6 ? GR_HIP_NODE_IP6_OUTPUT : GR_HIP_NODE_IP_OUTPUT;
	case GR_HIP_E_IP6_INPUT_LOCAL:
	case GR_HIP_E_IP6_ERROR_DEST_UNREACH:
	case GR_HIP_E_IP6_INPUT_NOT_MEMBER:
	case GR_HIP_E_IP6_INPUT_OTHER_HOST:
	case GR_HIP_E_IP6_INPUT_BAD_VERSION:
	case GR_HIP_E_IP6_INPUT_BAD_ADDR:
	case GR_HIP_E_IP6_INPUT_BAD_LENGTH:
	case GR_HIP_E_IP6_BLACKHOLE:
	case GR_HIP_E_SR6_LOCAL:
		return GR_HIP_NODE_IP6_INPUT;
	case GR_HIP_E_IP6_ERROR_TTL_EXCEEDED:
		return GR_HIP_NODE_IP6_FORWARD;
	case GR_HIP_E_IP6_HOLD:
	case GR_HIP_E_IP6_OUTPUT_ERROR:
	case GR_HIP_E_IP6_OUTPUT_TOO_BIG:
		return GR_HIP_NODE_IP6_OUTPUT;
	case GR_HIP_E_ETH_OUTPUT_NO_MAC:
		return GR_HIP_NODE_ETH_OUTPUT;
	case GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE:
	case GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN:
	case GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT:
	case GR_HIP_E_BOND_OUTPUT:
	case GR_HIP_E_VXLAN_OUTPUT:
	case GR_HIP_E_PORT_OUTPUT:
		return GR_HIP_NODE_IFACE_OUTPUT;
	default:
		return -EINVAL;
	}
}

extern "C" int gr_hip_edge_node(uint8_t edge, uint32_t nh, int ip6) {
	return edge_node(edge, nh, ip6);
}

// Walk boundaries of the node's mbufs (include/grout_hip.h,
// gr_hip_node_layout): a walk starts at m[0], at GR_HIP_MBUF_F_WALK, and
// `burst` mbufs after the previous start. grout's walks hold at most
// RTE_GRAPH_BURST_SIZE = 256 packets (rx_burst_max / vector_max,
// modules/infra/control/graph.c:612-650, checked at :619); 64 by default
// (:88-91).
#define WALK_MAX 256
static inline uint32_t walk_burst(uint32_t burst) {
	return burst == 0 ? 64 : burst > WALK_MAX ? WALK_MAX : burst;
}

static inline bool walk_start(const struct gr_hip_mbuf *m, uint32_t i, uint32_t start, uint32_t burst) {
	return i == 0 || (m[i].flags & GR_HIP_MBUF_F_WALK) || i - start == burst;
}

// The walks of m (m[0] starts one) placed from slot p on; returns the first
// slot past them.
extern "C" uint64_t gr_node_layout_from(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, uint64_t p,
					uint32_t *pos) {
	burst = walk_burst(burst);
	for (uint32_t i = 0; i < n;) {
		// this walk: [i, e)
		uint32_t e = i + 1;
		while (e < n && !walk_start(m, e, i, burst))
			e++;
		const uint32_t len = e - i;
		// a walk that fits a tile never straddles one (the kernel resolves
		// eth_output's cache inside a tile); a longer one starts on a tile
		// (the hand-back resolves it, eth_output_walk)
		if ((p & 63) + len > 64)
			p = (p + 63) & ~63ull;
		for (uint32_t k = i; k < e; k++)
			pos[k] = (uint32_t)p++;
		i = e;
	}
	return p;
}

extern "C" int gr_hip_node_layout(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, uint32_t *pos) {
	if (n && (m == nullptr || pos == nullptr))
		return -EINVAL;
	const uint64_t p = gr_node_layout_from(m, n, burst, 0, pos);
	if (p > INT32_MAX)
		return -E2BIG;
	return (int)p;
}

extern "C" int gr_node_stage_from(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, const uint32_t *pos,
				  uint32_t next, void *lines, struct gr_hip_pkt_meta *meta) {
	burst = walk_burst(burst);
	uint8_t *L = static_cast<uint8_t *>(lines);
	constexpr uint32_t AHEAD = 16; // frames in flight: staging is bound by their cache misses
	for (uint32_t i = 0; i < n && i < AHEAD && L != nullptr; i++)
		__builtin_prefetch(m[i].frame, 0, 0);
	uint32_t start = 0; // next: first slot not yet written
	for (uint32_t i = 0; i < n; i++) {
		if (i + AHEAD < n && L != nullptr)
			__builtin_prefetch(m[i + AHEAD].frame, 0, 0);
		const uint32_t at = pos != nullptr ? pos[i] : next;
		for (; next < at; next++) { // a pad slot: punted by the kernel, counted nowhere
			meta[next] = gr_hip_pkt_meta{0, 0, 0, 0};
			if (L != nullptr)
				memset(L + (size_t)next * GR_HIP_LINE, 0, GR_HIP_LINE);
		}
		next = at + 1;
		// 64 bytes whatever data_len says: grout's nodes read the Ethernet and
		// IPv4 headers from the data room without a length check (eth_input.c
		// reads 14 bytes of a shorter frame), and an mbuf's data room always
		// holds 64 bytes past data_off (mempool.c:66-68)
		if (m[i].frame == nullptr)
			return -EINVAL;
		if (L != nullptr) // NULL: metadata only (the GPU reads the frames itself)
			memcpy(L + (size_t)at * GR_HIP_LINE, m[i].frame, GR_HIP_LINE);
		uint16_t vc = (uint16_t)((m[i].vlan_id & 0xfff) | ((m[i].ck & 3) << 12));
		if (walk_start(m, i, start, burst)) {
			start = i;
			vc |= GR_HIP_META_WALK;
		}
		meta[at].iface = m[i].iface;
		meta[at].vlan_ck = vc;
		meta[at].pkt_len = (uint16_t)(m[i].pkt_len > 0xffff ? 0xffff : m[i].pkt_len);
		meta[at].rss = (uint16_t)m[i].rss;
	}
	return 0;
}

// Where a walk of n mbufs appended at slot p ends: cut every `burst` mbufs,
// each piece placed as gr_node_layout_from places a walk.
extern "C" uint64_t gr_node_walk_end(uint64_t p, uint32_t n, uint32_t burst) {
	burst = walk_burst(burst);
	for (uint32_t i = 0; i < n; i += burst) {
		const uint32_t len = n - i < burst ? n - i : burst;
		if ((p & 63) + len > 64)
			p = (p + 63) & ~63ull;
		p += len;
	}
	return p;
}

template <typename T> static inline T get(const uint8_t *base, uint16_t off) {
	T v;
	memcpy(&v, base + off, sizeof(v));
	return v;
}

extern "C" void *gr_node_frame(const void *mbuf, const struct gr_hip_mbuf_layout *lay) {
	const uint8_t *mb = static_cast<const uint8_t *>(mbuf);
	return get<uint8_t *>(mb, lay->buf_addr) + get<uint16_t>(mb, lay->data_off);
}

// gr_hip_node_append_mbufs' one pass over a walk's mbufs (mbufs[0] starts
// it): each mbuf read through the layout (what the grout node used to put in
// a view: rte_pktmbuf_mtod, pkt_len, hash.rss, iface_mbuf_data's iface id and
// vlan_id, the checksum status), placed from slot p (pos[i]; pads zeroed) as
// gr_node_layout_from places it, and its header line (lines NULL: none) and
// metadata staged as gr_node_stage_from stages them. No view is written: the
// hand-back reads the mbufs again (gr_node_direct.meta). Returns the first
// slot past the walk.
extern "C" uint64_t gr_node_stage_mbufs(void *const *mbufs, uint32_t n, const struct gr_hip_mbuf_layout *lay,
					uint32_t burst, uint64_t p, uint32_t *pos, void *lines,
					struct gr_hip_pkt_meta *meta) {
	burst = walk_burst(burst);
	const struct gr_hip_mbuf_layout &L = *lay;
	uint8_t *lb = static_cast<uint8_t *>(lines);
	for (uint32_t i = 0; i < n; i++) {
		const bool start = i % burst == 0;
		if (start) {
			const uint32_t len = n - i < burst ? n - i : burst;
			if ((p & 63) + len > 64) { // pad to the next tile: punted by the kernel, counted nowhere
				for (const uint64_t e = (p + 63) & ~63ull; p < e; p++) {
					meta[p] = gr_hip_pkt_meta{0, 0, 0, 0};
					if (lb != nullptr)
						memset(lb + (size_t)p * GR_HIP_LINE, 0, GR_HIP_LINE);
				}
			}
		}
		const uint8_t *mb = static_cast<const uint8_t *>(mbufs[i]);
		const uint8_t *priv = mb + L.priv;
		const uint8_t *ifp = get<const uint8_t *>(priv, L.priv_iface);
		const uint64_t ck = get<uint64_t>(mb, L.ol_flags) & L.ck_mask;
		const uint32_t pkt_len = get<uint32_t>(mb, L.pkt_len);
		const uint8_t st = ck == L.ck_good ? GR_HIP_CKSUM_GOOD : ck == L.ck_bad ? GR_HIP_CKSUM_BAD : GR_HIP_CKSUM_UNKNOWN;
		pos[i] = (uint32_t)p;
		// 64 bytes whatever data_len says (gr_node_stage_from)
		if (lb != nullptr)
			memcpy(lb + (size_t)p * GR_HIP_LINE, gr_node_frame(mb, lay), GR_HIP_LINE);
		meta[p].iface = ifp != nullptr ? get<uint16_t>(ifp, L.iface_id) : 0;
		meta[p].vlan_ck = (uint16_t)((get<uint16_t>(priv, L.priv_vlan_id) & 0xfff) | (st << 12)
					     | (start ? GR_HIP_META_WALK : 0));
		meta[p].pkt_len = (uint16_t)(pkt_len > 0xffff ? 0xffff : pkt_len);
		meta[p].rss = (uint16_t)get<uint32_t>(mb, L.rss);
		p++;
	}
	return p;
}

extern "C" int gr_hip_node_stage(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, const uint32_t *pos,
				 void *lines, struct gr_hip_pkt_meta *meta) {
	if (n && (m == nullptr || meta == nullptr))
		return -EINVAL;
	return gr_node_stage_from(m, n, burst, pos, 0, lines, meta);
}

// The VLAN sub-interface of (parent, vlan_id) in the host image of the
// context's VLAN table (0: none), vlan_get_iface (iface_input.c:76).
static inline uint16_t vlan_sub(const struct gr_node_vlans *vl, uint16_t parent, uint16_t vlan_id) {
	if (vl == nullptr || vl->cap == 0)
		return 0;
	const uint32_t key = (((uint32_t)parent << 16) | vlan_id) + 1;
	for (uint32_t h = (key * 0x9e3779b1u) & (vl->cap - 1);; h = (h + 1) & (vl->cap - 1)) {
		if (vl->keys[h] == key)
			return vl->vals[h];
		if (vl->keys[h] == 0)
			return 0;
	}
}

// eth_output's per-walk source-MAC cache (eth_output.c:37-59) over a walk
// [a, e) longer than a tile, which the kernel resolved tile by tile: replay
// it over the whole walk and set each forwarded packet's source MAC (bytes
// 6-11 of its frame, already handed back) to the cached MAC: its iface's, or
// zero after a failed lookup of another iface (eth_output_no_mac). eth_output
// takes ip_output's packets, then ip6_output's, or the other way round when
// an IPv6 packet reached ip6_input first (rte_graph's pending queue), as the
// kernel's eth_output_walks does inside a tile.
static void eth_output_walk(uint8_t *const *wf, uint32_t a, uint32_t e, const uint32_t *pos,
			    const struct gr_hip_verdict *verdicts, const int8_t *fam, const struct gr_hip_iface *ifaces,
			    uint32_t n_ifaces, const struct gr_hip_nh *nh, uint32_t n_nh) {
	int32_t first4 = -1, first6 = -1;
	for (uint32_t i = a; i < e; i++) {
		if (fam[i - a] == 1 && first4 < 0)
			first4 = (int32_t)i;
		if (fam[i - a] == 2 && first6 < 0)
			first6 = (int32_t)i;
	}
	const bool six_first = first6 >= 0 && (first4 < 0 || first6 < first4);
	uint32_t last = GR_HIP_IFACE_ID_UNDEF;
	bool cleared = false; // the cached source MAC was zeroed
	for (int pass = 0; pass < 2; pass++) {
		const int8_t f = (pass == 0) == six_first ? 2 : 1;
		for (uint32_t i = a; i < e; i++) {
			if (fam[i - a] != f)
				continue;
			const struct gr_hip_verdict &v = verdicts[pos != nullptr ? pos[i] : i];
			const bool nomac = v.edge == GR_HIP_E_ETH_OUTPUT_NO_MAC;
			const int node = edge_node(v.edge, v.nh, f == 2);
			if (!nomac && node != GR_HIP_NODE_IFACE_OUTPUT)
				continue; // never reached eth_output
			// priv->iface at eth_output: the nexthop's iface (ip_output.c:91-97)
			const uint32_t eo = nomac ? v.iface : (v.nh < n_nh && nh != nullptr ? nh[v.nh].iface_id : 0);
			if (eo != last) {
				if (nomac) { // iface_get_eth_addr failed: src_mac zeroed, last kept
					cleared = true;
					continue;
				}
				last = eo;
				cleared = false;
			}
			if (nomac)
				continue;
			uint8_t *src = wf[i - a] + 6; // the walk's frames, wf[0] = packet a's
			if (cleared)
				memset(src, 0, 6);
			else if (eo < n_ifaces && ifaces != nullptr)
				memcpy(src, ifaces[eo].mac, 6);
		}
	}
}

static inline void count(struct gr_hip_iface_stats *st, uint32_t n_st, uint32_t id, bool tx, uint32_t len) {
	if (id == 0 || id >= n_st)
		return;
	if (tx) {
		st[id].tx_packets++;
		st[id].tx_bytes += len;
	} else {
		st[id].rx_packets++;
		st[id].rx_bytes += len;
	}
}

// The hand-back's prefetch distance and locality (measurement builds
// override them: tools/apply_cost.py).
#ifndef GR_NODE_APPLY_AHEAD
#define GR_NODE_APPLY_AHEAD 16
#endif
#ifndef GR_NODE_APPLY_PF_LOC
#define GR_NODE_APPLY_PF_LOC 0
#endif

static inline void prefetch_for_apply(const struct gr_hip_mbuf *m, uint32_t i, const struct gr_node_direct *d) {
	if (m != nullptr) // else the frame's address is in the mbuf's first line, prefetched below
		__builtin_prefetch(m[i].frame, 1, GR_NODE_APPLY_PF_LOC);
	if (d != nullptr) {
		const uint8_t *mb = static_cast<const uint8_t *>(d->mbufs[i]);
		__builtin_prefetch(mb, 1, GR_NODE_APPLY_PF_LOC); // data_off .. packet_type: the mbuf's first line
		__builtin_prefetch(mb + d->lay->priv, 1, GR_NODE_APPLY_PF_LOC); // the private data
	}
}

template <typename T> static inline void put(uint8_t *base, uint16_t off, T v) {
	memcpy(base + off, &v, sizeof(v));
}

static inline const void *reg_get(const void *const *reg, uint32_t n, uint32_t id) {
	return id < n && reg != nullptr ? __atomic_load_n(&reg[id], __ATOMIC_ACQUIRE) : nullptr;
}

// The view of mbuf i as the grout node used to build it (gr_node_stage_mbufs
// staged the same fields), read before the hand-back writes the mbuf.
static inline void view_of_mbuf(const struct gr_node_direct *d, uint32_t i, uint32_t at, struct gr_hip_mbuf &b) {
	const struct gr_hip_mbuf_layout &L = *d->lay;
	const uint8_t *mb = static_cast<const uint8_t *>(d->mbufs[i]);
	const uint16_t off = get<uint16_t>(mb, L.data_off);
	b.frame = get<uint8_t *>(mb, L.buf_addr) + off;
	b.pkt_len = get<uint32_t>(mb, L.pkt_len);
	b.data_len = get<uint16_t>(mb, L.data_len);
	b.data_off = off;
	b.packet_type = get<uint32_t>(mb, L.packet_type);
	b.rss = d->meta[at].rss;
	b.iface = d->meta[at].iface;
	b.vlan_id = get<uint16_t>(mb + L.priv, L.priv_vlan_id);
	b.ck = (uint8_t)((d->meta[at].vlan_ck >> 12) & 3);
	b.edge = 0;
	b.domain = 0;
	b.flags = (d->meta[at].vlan_ck & GR_HIP_META_WALK) ? GR_HIP_MBUF_F_WALK : 0;
	b.nh = 0;
}

// One packet's hand-back onto its mbuf (the grout node's private data for
// the node behind its edge); returns the edge.
static inline uint8_t to_mbuf(struct gr_node_direct *d, uint32_t i, const struct gr_hip_mbuf &b,
			      const struct gr_hip_verdict &v, int node) {
	if (v.edge == GR_HIP_E_PUNT)
		return GR_HIP_E_PUNT; // grout's CPU iface_input takes it as port_rx left it
	const struct gr_hip_mbuf_layout &L = *d->lay;
	const void *ifp = reg_get(L.ifaces, L.n_ifaces, v.iface);
	const void *nhp = nullptr;
	if ((ifp == nullptr && v.iface != 0)
	    || (node != GR_HIP_NODE_IFACE_INPUT && node != GR_HIP_NODE_IFACE_OUTPUT && v.nh != 0
		&& (nhp = reg_get(L.nh, L.n_nh, v.nh)) == nullptr)) {
		d->stale++; // an object grout freed: the mbuf stays as it was, a drop node takes it
		return GR_HIP_E_IP_OUTPUT_ERROR;
	}
	uint8_t *mb = static_cast<uint8_t *>(d->mbufs[i]);
	put<uint16_t>(mb, L.data_off, b.data_off);
	put<uint16_t>(mb, L.data_len, b.data_len);
	put<uint32_t>(mb, L.pkt_len, b.pkt_len);
	put<uint32_t>(mb, L.packet_type, b.packet_type);
	uint8_t *priv = mb + L.priv;
	put<const void *>(priv, L.priv_iface, ifp);
	switch (node) {
	case GR_HIP_NODE_IFACE_INPUT:
	case GR_HIP_NODE_IFACE_OUTPUT:
		put<uint16_t>(priv, L.priv_vlan_id, b.vlan_id);
		break;
	case GR_HIP_NODE_ETH_OUTPUT:
		if (v.nh)
			put<const void *>(priv, L.priv_l3_nh, nhp);
		break;
	default:
		put<uint32_t>(priv, L.priv_domain, b.domain);
		put<const void *>(priv, L.priv_eth_nh, nullptr);
		if (v.nh)
			put<const void *>(priv, L.priv_l3_nh, nhp);
		break;
	}
	return v.edge;
}

// The hand-back onto the mbufs of the packet a forwarding plane sees most:
// forwarded to port_output, untagged on ingress (line: its rewritten header
// line, or its frame when the GPU rewrote it in place). It is
// the general loop below specialised for that case (depth 6 of either
// family: no adj, iface_output's VLAN tag from the nexthop's iface, rx / tx
// counted where grout counts them, the mbuf and private data as to_mbuf
// writes them); returns false for any other packet, untouched.
static inline bool port_output_fast(struct gr_node_direct *d, uint32_t i, const struct gr_hip_mbuf &b,
				    const struct gr_hip_verdict &v, const uint8_t *line, const struct gr_hip_iface *ifaces,
				    uint32_t n_ifaces, const struct gr_hip_nh *nh, uint32_t n_nh,
				    struct gr_hip_iface_stats *ifst, uint32_t n_ifst, bool &ip6) {
	if (v.edge != GR_HIP_E_PORT_OUTPUT || b.vlan_id != 0 || v.nh == 0 || v.nh >= n_nh || nh == nullptr)
		return false;
	ip6 = line[12] == 0x86 && line[13] == 0xdd; // RTE_ETHER_TYPE_IPV6
	const struct gr_hip_mbuf_layout &L = *d->lay;
	const void *ifp = reg_get(L.ifaces, L.n_ifaces, v.iface);
	const uint16_t oif = nh[v.nh].iface_id;
	if (ifst != nullptr) {
		count(ifst, n_ifst, b.iface, false, b.pkt_len);
		count(ifst, n_ifst, oif, true, b.pkt_len);
		if (v.iface != oif)
			count(ifst, n_ifst, v.iface, true, b.pkt_len);
	}
	if (ifp == nullptr && v.iface != 0) {
		d->stale++; // see to_mbuf
		d->edges[i] = GR_HIP_E_IP_OUTPUT_ERROR;
		return true;
	}
	uint8_t *fr = static_cast<uint8_t *>(b.frame);
	if (line != fr) { // else the GPU rewrote the frame in place (frames by address)
		const uint32_t len = b.data_len < 26 ? b.data_len : 26; // bytes 0-25: see the general loop
		if (len >= 16) {
			memcpy(fr, line, 16);
			memcpy(fr + len - 16, line + len - 16, 16);
		} else {
			memcpy(fr, line, len);
		}
	}
	uint16_t vid = 0;
	if (oif < n_ifaces && ifaces != nullptr && ifaces[oif].id == oif && ifaces[oif].type == GR_HIP_IFACE_TYPE_VLAN)
		vid = ifaces[oif].vlan_id;
	uint8_t *mb = static_cast<uint8_t *>(d->mbufs[i]);
	if (d->meta == nullptr) { // the view's lengths (read from this mbuf otherwise: unchanged)
		put<uint16_t>(mb, L.data_off, b.data_off); // eth_output's prepend undid ip_input's adj
		put<uint16_t>(mb, L.data_len, b.data_len);
		put<uint32_t>(mb, L.pkt_len, b.pkt_len);
	}
	put<uint32_t>(mb, L.packet_type, ip6 ? GR_HIP_PTYPE_L3_IPV6 : GR_HIP_PTYPE_L3_IPV4);
	uint8_t *priv = mb + L.priv;
	put<const void *>(priv, L.priv_iface, ifp);
	put<uint16_t>(priv, L.priv_vlan_id, vid);
	d->edges[i] = GR_HIP_E_PORT_OUTPUT;
	return true;
}

extern "C" int gr_hip_node_apply(
	struct gr_hip_mbuf *m,
	uint32_t n,
	uint32_t burst,
	const uint32_t *pos,
	const void *lines,
	uint32_t line_stride,
	const struct gr_hip_verdict *verdicts,
	const struct gr_hip_iface *ifaces,
	uint32_t n_ifaces,
	const struct gr_hip_nh *nh,
	uint32_t n_nh,
	struct gr_hip_node_stats *stats
) {
	return gr_node_apply_ex(m, n, burst, pos, lines, line_stride, verdicts, ifaces, n_ifaces, nh, n_nh, stats,
				nullptr, nullptr, 0, nullptr);
}

extern "C" int gr_node_apply_ex(
	struct gr_hip_mbuf *m,
	uint32_t n,
	uint32_t burst,
	const uint32_t *pos,
	const void *lines,
	uint32_t line_stride,
	const struct gr_hip_verdict *verdicts,
	const struct gr_hip_iface *ifaces,
	uint32_t n_ifaces,
	const struct gr_hip_nh *nh,
	uint32_t n_nh,
	struct gr_hip_node_stats *stats,
	const struct gr_node_vlans *vlans,
	struct gr_hip_iface_stats *ifst,
	uint32_t n_ifst,
	struct gr_node_direct *direct
) {
	if (n == 0)
		return 0;
	if (direct != nullptr && (direct->mbufs == nullptr || direct->lay == nullptr || direct->edges == nullptr))
		return -EINVAL;
	const bool own = direct != nullptr && direct->meta != nullptr; // no views: read from the mbufs
	if ((m == nullptr && !own) || (own && pos == nullptr) || verdicts == nullptr
	    || (lines != nullptr && line_stride < GR_HIP_PREFIX))
		return -EINVAL;
	burst = walk_burst(burst);
	const uint8_t *L = static_cast<const uint8_t *>(lines);
	// the nodes an IPv4 / IPv6 packet walks, in order
	static const int path4[] = {GR_HIP_NODE_IFACE_INPUT, GR_HIP_NODE_ETH_INPUT, GR_HIP_NODE_IP_INPUT,
				    GR_HIP_NODE_IP_FORWARD, GR_HIP_NODE_IP_OUTPUT, GR_HIP_NODE_ETH_OUTPUT,
				    GR_HIP_NODE_IFACE_OUTPUT};
	static const int path6[] = {GR_HIP_NODE_IFACE_INPUT, GR_HIP_NODE_ETH_INPUT, GR_HIP_NODE_IP6_INPUT,
				    GR_HIP_NODE_IP6_FORWARD, GR_HIP_NODE_IP6_OUTPUT, GR_HIP_NODE_ETH_OUTPUT,
				    GR_HIP_NODE_IFACE_OUTPUT};
	// position of each node on a packet's path (-1: not on it), per family
	static const int8_t depth_of[2][GR_HIP_NODE_COUNT] = {
		{0, 1, 2, 3, 4, 5, 6, -1, -1, -1}, // IPv4: path4
		{0, 1, -1, -1, -1, 5, 6, 2, 3, 4}, // IPv6: path6
	};
	static_assert(GR_HIP_NODE_COUNT == 10 && GR_HIP_NODE_IP6_INPUT == 7, "node order");
	uint32_t ended[2][7] = {}; // packets of the walk that stopped at depth d, per family
	uint32_t reach[GR_HIP_NODE_COUNT] = {};
	uint32_t start = 0; // first mbuf of the current graph walk
	int8_t fam[WALK_MAX]; // per packet of the walk: 1 = entered ip_input, 2 = ip6_input, 0 = neither
	uint8_t *wf[WALK_MAX]; // per packet of the walk: its frame (eth_output_walk)
	bool walk_nomac = false; // the walk holds an eth_output_no_mac packet
	// frames read (the ether type) and written back: prefetch them, the loop
	// is bound by their cache misses
	constexpr uint32_t AHEAD = GR_NODE_APPLY_AHEAD;
	for (uint32_t i = 0; i < n && i < AHEAD; i++)
		prefetch_for_apply(m, i, direct);
	for (uint32_t i = 0; i < n; i++) {
		if (i + AHEAD < n)
			prefetch_for_apply(m, i + AHEAD, direct);
		const uint32_t at = pos != nullptr ? pos[i] : i;
		const struct gr_hip_verdict &v = verdicts[at];
		// direct: the view is only read (own: built from the mbuf before the
		// hand-back writes it), the mbuf gets the result below
		struct gr_hip_mbuf copy;
		if (own)
			view_of_mbuf(direct, i, at, copy);
		else if (direct != nullptr)
			copy = m[i];
		struct gr_hip_mbuf &b = direct != nullptr ? copy : m[i];
		if (i - start < WALK_MAX)
			wf[i - start] = static_cast<uint8_t *>(b.frame);
		bool fast6;
		if (direct != nullptr
		    && port_output_fast(direct, i, b, v,
					L != nullptr ? L + (size_t)at * line_stride : static_cast<const uint8_t *>(b.frame),
					ifaces, n_ifaces, nh, n_nh, ifst, n_ifst, fast6)) {
			if (i - start < WALK_MAX)
				fam[i - start] = fast6 ? 2 : 1;
			ended[fast6][6]++;
			goto walk_end;
		}
		{
		const uint32_t len0 = b.pkt_len; // as iface_input / iface_output count it
		const uint16_t iface0 = b.iface, vlan0 = b.vlan_id; // as port_rx left them
		// lines NULL: the GPU rewrote the frames in place already
		const uint8_t *line = L != nullptr ? L + (size_t)at * line_stride : static_cast<const uint8_t *>(b.frame);
		const bool ip6 = line[12] == 0x86 && line[13] == 0xdd; // RTE_ETHER_TYPE_IPV6
		const int node = edge_node(v.edge, v.nh, ip6);
		if (node < -1)
			return -EINVAL;
		b.edge = v.edge;
		if (i - start < WALK_MAX)
			fam[i - start] = 0;
		walk_nomac |= v.edge == GR_HIP_E_ETH_OUTPUT_NO_MAC;
		if (node >= 0) {
			const int depth = depth_of[ip6][node]; // position of `node` on the packet's path
			if (depth < 0)
				return -EINVAL;
			if (depth >= 2 && i - start < WALK_MAX)
				fam[i - start] = ip6 ? 2 : 1;
			ended[ip6][depth]++;
			// VLAN demux in iface_input: the tag was consumed
			const bool demuxed = b.vlan_id != 0 && v.edge != GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN && b.iface < n_ifaces
				&& ifaces != nullptr && ifaces[b.iface].id == b.iface
				&& ifaces[b.iface].mode == GR_HIP_IFACE_MODE_VRF;
			// depth: 0 iface_input, 1 eth_input, 2 ip(6)_input, 3 ip(6)_forward,
			// 4 ip(6)_output, 5 eth_output, 6 iface_output
			const bool adj = depth >= 2
				|| (depth == 1 && v.edge != GR_HIP_E_SNAP_INPUT && v.edge != GR_HIP_E_ETH_INPUT_INVALID_IFACE);
			if (adj && depth < 5 && b.data_len >= 14) { // rte_pktmbuf_adj(14)
				b.data_off += 14;
				b.data_len -= 14;
				b.pkt_len -= 14;
			}
			if (depth >= 4) {
				b.packet_type = ip6 ? GR_HIP_PTYPE_L3_IPV6 : GR_HIP_PTYPE_L3_IPV4;
				// the chain rewrote nothing past byte 25 (L2 0-13, TTL 22 and
				// checksum 24-25, or the hop limit 21)
				uint32_t len = b.data_len + (depth < 5 ? 14u : 0u);
				if (len > 26)
					len = 26;
				uint8_t *fr = static_cast<uint8_t *>(b.frame);
				if (L != nullptr && len >= 16) { // two overlapping 16-byte moves, no call
					memcpy(fr, line, 16);
					memcpy(fr + len - 16, line + len - 16, 16);
				} else if (L != nullptr) {
					memcpy(fr, line, len);
				}
			}
			if (depth <= 4) {
				if (demuxed)
					b.vlan_id = 0;
			} else if (depth == 5) {
				b.vlan_id = 0;
			} else {
				uint16_t vid = 0;
				if (v.nh && v.nh < n_nh && nh != nullptr) {
					uint16_t oif = nh[v.nh].iface_id;
					if (oif < n_ifaces && ifaces != nullptr && ifaces[oif].id == oif
					    && ifaces[oif].type == GR_HIP_IFACE_TYPE_VLAN)
						vid = ifaces[oif].vlan_id;
				}
				b.vlan_id = vid;
			}
			// per-iface counters where grout counts them (rxtx.h:84-117):
			// iface_input past its admin-down and unknown-VLAN drops
			// (iface_input.c:93-95), iface_output past its no-parent and
			// admin-down drops (iface_output.c:103-105)
			if (ifst != nullptr) {
				if (v.edge != GR_HIP_E_IFACE_INPUT_ADMIN_DOWN && v.edge != GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN) {
					const uint16_t self = demuxed ? vlan_sub(vlans, iface0, vlan0) : b.iface;
					count(ifst, n_ifst, self, false, len0);
					if (demuxed)
						count(ifst, n_ifst, iface0, false, len0);
				}
				if (depth == 6 && v.edge != GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN
				    && v.edge != GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT && v.nh && v.nh < n_nh && nh != nullptr) {
					const uint16_t oif = nh[v.nh].iface_id;
					count(ifst, n_ifst, oif, true, len0);
					if (v.iface != oif)
						count(ifst, n_ifst, v.iface, true, len0);
				}
			}
			b.iface = v.iface;
			b.domain = v.domain;
			b.nh = v.nh;
		}
		if (direct != nullptr)
			direct->edges[i] = to_mbuf(direct, i, b, v, node);
		}
	walk_end:
		if (i + 1 == n
		    || (own ? (direct->meta[pos[i + 1]].vlan_ck & GR_HIP_META_WALK) != 0 || i + 1 - start == burst
			    : walk_start(m, i + 1, start, burst))) { // this graph walk ends here
			if (walk_nomac && i + 1 - start > 64)
				eth_output_walk(wf, start, i + 1, pos, verdicts, fam, ifaces, n_ifaces, nh, n_nh);
			walk_nomac = false;
			start = i + 1;
			if (stats == nullptr)
				continue;
			// a packet that stopped at depth d passed every node before it
			uint32_t sent[2] = {0, 0}; // what ip_output / ip6_output enqueued to eth_output
			for (int f = 0; f < 2; f++) {
				const int *path = f ? path6 : path4;
				uint32_t from = 0;
				for (int d = 6; d >= 0; d--) {
					from += ended[f][d];
					reach[path[d]] += from;
					if (d == 5)
						sent[f] = from;
					ended[f][d] = 0;
				}
			}
			for (int k = 0; k < GR_HIP_NODE_COUNT; k++) {
				// ip_output / ip6_output return only what they sent to eth_output
				uint32_t ret = reach[k];
				if (k == GR_HIP_NODE_IP_OUTPUT)
					ret = sent[0];
				else if (k == GR_HIP_NODE_IP6_OUTPUT)
					ret = sent[1];
				stats->packets[k] += ret;
				stats->calls[k] += reach[k] != 0;
				reach[k] = 0;
			}
		}
	}
	return 0;
}
