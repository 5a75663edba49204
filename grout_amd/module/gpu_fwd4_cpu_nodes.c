// SPDX-License-Identifier: BSD-3-Clause
//
// gpu_fwd4_cpu_nodes.c -- the two grout nodes that continue, on the CPU, the
// work the fast path hands back at the exact point where grout's own node
// would call into state the GPU does not hold (conntrack, NAT tables):
//
//   ip_input_local_ct  the end of ip_input for a packet to a local address
//                      received on an iface with GR_IFACE_F_SNAT_DYNAMIC
//                      (modules/ip/datapath/ip_input.c:166-187): a conntrack
//                      hit goes to dnat44_dynamic with the connection in the
//                      private data, anything else to ip_input_local;
//   ip_output_snat     ip_output from its SNAT hook on, for a packet leaving
//                      through an iface with GR_IFACE_F_SNAT_STATIC / _DYNAMIC
//                      (ip_output.c:108-153): snat44_process, then the iface
//                      type edge, the HOLD check and eth_output's private data.
//
// Both receive mbufs in the state grout's chain leaves them there (the GPU
// node's hand-back: data_off past the Ethernet header, the ingress iface or
// the egress iface in mbuf_data, l3_mbuf_data.nh, TTL and checksum already
// rewritten by ip_forward). grout's and DPDK's headers by their names (the
// test stand-ins here, tests/standin/include).
#include "gpu_fwd4_node.h"

#include "conntrack.h"
#include "eth.h"
#include "graph.h"
#include "iface.h"
#include "l3.h"
#include "mbuf.h"
#include "nat_datapath.h"
#include "nexthop.h"

#include <rte_byteorder.h>
#include <rte_ether.h>
#include <rte_graph_worker.h>
#include <rte_ip.h>
#include <rte_mbuf.h>

#include <string.h>

// ---- ip_input_local_ct ------------------------------------------------------
enum {
	LOCAL_CT_LOCAL = 0,
	LOCAL_CT_DNAT44_DYNAMIC,
	LOCAL_CT_NB_EDGES,
};

static uint16_t
ip_input_local_ct_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	for (uint16_t i = 0; i < nb_objs; i++) {
		struct rte_mbuf *m = objs[i];
		const struct iface *iface = mbuf_data(m)->iface; // ingress (eth_input_mbuf_data.iface)
		rte_edge_t edge = LOCAL_CT_LOCAL;
		conn_flow_t flow = CONN_FLOW_REV;
		struct conn_key key;
		struct conn *conn;
		// ip_input.c:170-185 (returning fragments go to LOCAL: no reassembly)
		if (gr_conn_parse_key(iface, GR_AF_IP4, m, &key) && (conn = gr_conn_lookup(&key, &flow)) != NULL) {
			struct conn_mbuf_data *cd = conn_mbuf_data(m);
			cd->conn = conn;
			cd->flow = flow;
			edge = LOCAL_CT_DNAT44_DYNAMIC;
		}
		rte_node_enqueue_x1(graph, node, edge, m);
	}
	return nb_objs; // ip_input's return value (ip_input.c:196)
}

static struct rte_node_register ip_input_local_ct_node = {
	.name = "ip_input_local_ct",
	.process = ip_input_local_ct_process,
	.nb_edges = LOCAL_CT_NB_EDGES,
	.next_nodes = {
		[LOCAL_CT_LOCAL] = "ip_input_local",
		[LOCAL_CT_DNAT44_DYNAMIC] = "dnat44_dynamic",
	},
};

static struct gr_node_info ip_input_local_ct_info = {
	.node = &ip_input_local_ct_node,
	.type = GR_NODE_T_L3,
};

GR_NODE_REGISTER(ip_input_local_ct_info);

// ---- ip_output_snat -----------------------------------------------------------
// Edges: the fast path's verdict edges by enum gr_hip_edge value (the iface
// type edges registered with ip_output_register_interface_type land there,
// e.g. xvrf and ipip_output, and so does ip_hold), then eth_output and
// ip_output_drop.
enum {
	SNAT_ETH_OUTPUT = GR_HIP_E_COUNT,
	SNAT_DROP,
	SNAT_NB_EDGES,
};

static uint16_t ip_output_snat_process(struct rte_graph *graph, struct rte_node *node, void **objs, uint16_t nb_objs) {
	gr_hip_ctx_t *ctx = gpu_fwd4_hip_ctx();
	uint16_t sent = 0;
	for (uint16_t i = 0; i < nb_objs; i++) {
		struct rte_mbuf *m = objs[i];
		const struct rte_ipv4_hdr *ip = rte_pktmbuf_mtod(m, const struct rte_ipv4_hdr *);
		const struct nexthop *nh = l3_mbuf_data(m)->nh;
		const struct iface *iface = mbuf_data(m)->iface; // set by ip_output (ip_output.c:97)
		// the iface type edge ip_output computed before its SNAT hook
		// (ip_output.c:110), from the registrations the fast path mirrors
		const int t = ctx != NULL ? gr_hip_edges_get(ctx, GR_HIP_EDGES_IP_OUTPUT_IFACE_TYPE, iface->type) : -1;
		rte_edge_t edge = t == GR_HIP_EDGE_CHAIN ? SNAT_ETH_OUTPUT : t >= 0 && t < GR_HIP_E_COUNT ? (rte_edge_t)t
											  : GR_HIP_E_IP_OUTPUT_ERROR;
		if (snat44_process(iface, m) == NAT_VERDICT_DROP) // ip_output.c:112-119
			edge = SNAT_DROP;
		if (edge != SNAT_ETH_OUTPUT) // :121-122
			goto next;
		const struct nexthop_info_l3 *l3 = nexthop_info_l3(nh);
		if (l3->state != GR_NH_S_REACHABLE || ((l3->flags & GR_NH_F_LINK) && ip->dst_addr != l3->ipv4)) {
			edge = GR_HIP_E_IP_HOLD; // :124-138
			goto next;
		}
		struct eth_output_mbuf_data *eth_data = eth_output_mbuf_data(m); // :140-152
		eth_data->dst = l3->mac;
		eth_data->ether_type = RTE_BE16(RTE_ETHER_TYPE_IPV4);
		if (iface->type == GR_IFACE_TYPE_VXLAN) {
			eth_data->vtep.af = l3->af;
			if (l3->af == GR_AF_IP4)
				eth_data->vtep.ipv4 = l3->ipv4;
			else
				memcpy(eth_data->vtep.ipv6, l3->ipv6, 16);
		} else {
			eth_data->vtep.af = GR_AF_UNSPEC;
		}
		sent++;
next:
		rte_node_enqueue_x1(graph, node, edge, m);
	}
	return sent; // ip_output counts what it sent to eth_output (:153,162)
}

static struct rte_node_register ip_output_snat_node = {
	.name = "ip_output_snat",
	.process = ip_output_snat_process,
	.nb_edges = SNAT_NB_EDGES,
	.next_nodes = {
		GPU_FWD4_EDGES
		[SNAT_ETH_OUTPUT] = "eth_output",
		[SNAT_DROP] = "ip_output_drop",
	},
};

static struct gr_node_info ip_output_snat_info = {
	.node = &ip_output_snat_node,
	.type = GR_NODE_T_L3,
};

GR_NODE_REGISTER(ip_output_snat_info);
