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
//   ip_input          +14           -            0 if demuxed           -
//   ip_forward        +14           -            0 if demuxed           -
//   ip_output         +14           L3_IPV4      0 if demuxed           TTL, checksum
//   eth_output        +0 (2)        L3_IPV4      0                      + dst MAC
//   iface_output      +0 (2)        L3_IPV4      egress VLAN tag or 0   bytes 0-13, TTL, checksum
//
// (1) snap_input and eth_input_invalid_iface leave eth_input before its
//     rte_pktmbuf_adj(14) (eth_input.c:49-59 vs :80); adj is a no-op on a
//     frame shorter than 14 bytes (DPDK rte_pktmbuf_adj).
// (2) eth_output's gr_mbuf_prepend(14) (eth_output.c:305, mbuf.h:89-106)
//     undoes the adj: net data_off unchanged vs RX.
// vlan_id: iface_input clears it when it demuxes a tagged packet to a VLAN
// sub-interface (iface_input.c:74-86), eth_output clears it
// (eth_output.c:325), iface_output sets the egress VLAN's id
// (iface_output.c:219-224).
#include "../../include/grout_hip.h"

#include <errno.h>
#include <stddef.h>
#include <string.h>

static_assert(sizeof(struct gr_hip_mbuf) == 40 && offsetof(struct gr_hip_mbuf, nh) == 32, "gr_hip_mbuf layout");
static_assert(sizeof(struct gr_hip_node_stats) == 16 * GR_HIP_NODE_COUNT, "gr_hip_node_stats layout");

extern "C" int gr_hip_edge_node(uint8_t edge, uint32_t nh) {
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
	case GR_HIP_E_SR6_OUTPUT:
	case GR_HIP_E_XVRF:
	case GR_HIP_E_IPIP_OUTPUT:
	case GR_HIP_E_IP_OUTPUT_SNAT:
		return GR_HIP_NODE_IP_OUTPUT;
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

extern "C" int gr_hip_node_stage(const struct gr_hip_mbuf *m, uint32_t n, void *lines, struct gr_hip_pkt_meta *meta) {
	if (n && (m == nullptr || lines == nullptr || meta == nullptr))
		return -EINVAL;
	uint8_t *L = static_cast<uint8_t *>(lines);
	for (uint32_t i = 0; i < n; i++) {
		// 64 bytes whatever data_len says: grout's nodes read the Ethernet and
		// IPv4 headers from the data room without a length check (eth_input.c
		// reads 14 bytes of a shorter frame), and an mbuf's data room always
		// holds 64 bytes past data_off (mempool.c:66-68)
		if (m[i].frame == nullptr)
			return -EINVAL;
		memcpy(L + (size_t)i * GR_HIP_LINE, m[i].frame, GR_HIP_LINE);
		meta[i].iface = m[i].iface;
		meta[i].vlan_ck = (uint16_t)((m[i].vlan_id & 0xfff) | ((m[i].ck & 3) << 12));
		meta[i].pkt_len = (uint16_t)(m[i].pkt_len > 0xffff ? 0xffff : m[i].pkt_len);
		meta[i].rss = (uint16_t)m[i].rss;
	}
	return 0;
}

extern "C" int gr_hip_node_apply(
	struct gr_hip_mbuf *m,
	uint32_t n,
	const void *lines,
	uint32_t line_stride,
	const struct gr_hip_verdict *verdicts,
	const struct gr_hip_iface *ifaces,
	uint32_t n_ifaces,
	const struct gr_hip_nh *nh,
	uint32_t n_nh,
	uint32_t burst,
	struct gr_hip_node_stats *stats
) {
	if (n == 0)
		return 0;
	if (m == nullptr || lines == nullptr || verdicts == nullptr || line_stride < GR_HIP_LINE)
		return -EINVAL;
	if (burst == 0)
		burst = 64;
	const uint8_t *L = static_cast<const uint8_t *>(lines);
	uint32_t reach[GR_HIP_NODE_COUNT] = {};
	for (uint32_t i = 0; i < n; i++) {
		struct gr_hip_mbuf &b = m[i];
		const struct gr_hip_verdict &v = verdicts[i];
		const int node = gr_hip_edge_node(v.edge, v.nh);
		if (node < -1)
			return -EINVAL;
		b.edge = v.edge;
		if (node >= 0) {
			for (int k = 0; k <= node; k++)
				reach[k]++;
			// VLAN demux in iface_input: the tag was consumed
			const bool demuxed = b.vlan_id != 0 && v.edge != GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN && b.iface < n_ifaces
				&& ifaces != nullptr && ifaces[b.iface].id == b.iface
				&& ifaces[b.iface].mode == GR_HIP_IFACE_MODE_VRF;
			const bool adj = node >= GR_HIP_NODE_IP_INPUT
				|| (node == GR_HIP_NODE_ETH_INPUT && v.edge != GR_HIP_E_SNAP_INPUT
				    && v.edge != GR_HIP_E_ETH_INPUT_INVALID_IFACE);
			if (adj && node < GR_HIP_NODE_ETH_OUTPUT && b.data_len >= 14) { // rte_pktmbuf_adj(14)
				b.data_off += 14;
				b.data_len -= 14;
				b.pkt_len -= 14;
			}
			if (node >= GR_HIP_NODE_IP_OUTPUT) {
				b.packet_type = GR_HIP_PTYPE_L3_IPV4;
				// the chain rewrote nothing past byte 25 (TTL 22, checksum 24-25, L2 0-13)
				uint32_t len = b.data_len + (node < GR_HIP_NODE_ETH_OUTPUT ? 14u : 0u);
				if (len > 26)
					len = 26;
				memcpy(b.frame, L + (size_t)i * line_stride, len);
			}
			if (node <= GR_HIP_NODE_IP_OUTPUT) {
				if (demuxed)
					b.vlan_id = 0;
			} else if (node == GR_HIP_NODE_ETH_OUTPUT) {
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
			b.iface = v.iface;
			b.domain = v.domain;
			b.nh = v.nh;
		}
		if (stats != nullptr && ((i + 1) % burst == 0 || i + 1 == n)) {
			for (int k = 0; k < GR_HIP_NODE_COUNT; k++) {
				// ip_output returns only what it sent to eth_output
				const uint32_t ret = k == GR_HIP_NODE_IP_OUTPUT ? reach[GR_HIP_NODE_ETH_OUTPUT] : reach[k];
				stats->packets[k] += ret;
				stats->calls[k] += reach[k] != 0;
				reach[k] = 0;
			}
		}
	}
	return 0;
}
