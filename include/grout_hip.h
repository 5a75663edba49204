// SPDX-License-Identifier: BSD-3-Clause
//
// grout_hip.h -- C ABI of the MI355X-native IPv4 forwarding fast path.
//
// This is the only interface host C code (grout's datapath, a DPDK worker, or a
// ctypes test) uses to reach the GPU. Plain pointers and sizes, no C++ or torch
// types, never throws, never exits: every entry point returns 0 or -errno, the
// convention of grout's control plane (e.g. modules/ip/control/route.c:58,157).
//
// What it replaces in the reference (DPDK/grout, paths relative to its root):
//   * the per-burst walk  iface_input -> eth_input -> ip_input (+ fib4_lookup)
//     -> ip_forward -> ip_output -> eth_output -> iface_output
//     (modules/infra/datapath/iface_input.c:52-112, eth_input.c:35-88,
//      modules/ip/datapath/ip_input.c:47-197, modules/ip/control/route.c:147-167,
//      modules/ip/datapath/ip_forward.c:14-41, ip_output.c:63-163,
//      modules/infra/datapath/eth_output.c:27-77, iface_output.c:60-117)
//     is gr_hip_fwd4_submit(): one fused HIP kernel, one lane per packet.
//   * the DIR24_8 FIB that modules/ip/control/route.c:63-98 creates through
//     DPDK rte_fib, and the rte_fib_add() calls of rib4_insert_or_replace
//     (modules/ip/control/route.c:212-275), are the
//     gr_hip_route4_* / gr_hip_fib4_commit entry points (device-resident tables).
//   * the nexthop / iface objects the nodes dereference (nexthop.h:22-54,
//     iface.h:20-35) are mirrored with gr_hip_nh_set / gr_hip_iface_set
//     (hook: GR_EVENT_NEXTHOP_UPDATE, modules/infra/control/nexthop.c:386).
//   * the dynamic edge registrations (gr_eth_input_add_type eth_input.c:26,
//     ip_input_register_nexthop_type ip_input.c:36, ip_output_register_*
//     ip_output.c:34,46, iface_input_mode_register iface_input.c:22,
//     iface_output_type_register iface_output.c:25) are gr_hip_edges_*.
//
// Every per-packet output ("verdict") names the grout node the packet must be
// handed to next, i.e. one of the next_nodes of the replaced sub-graph
// (SURVEY.md Appendix A), together with the mbuf private data grout would have
// left for that node.
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_HIP_ABI_VERSION 3

// ---------------------------------------------------------------------------
// Values mirrored from grout's public API (identical numbering).
// ---------------------------------------------------------------------------

// gr_iface_type_t, modules/infra/api/gr_infra.h:18-28
enum {
	GR_HIP_IFACE_TYPE_UNDEF = 0,
	GR_HIP_IFACE_TYPE_VRF,
	GR_HIP_IFACE_TYPE_PORT,
	GR_HIP_IFACE_TYPE_VLAN,
	GR_HIP_IFACE_TYPE_IPIP,
	GR_HIP_IFACE_TYPE_BOND,
	GR_HIP_IFACE_TYPE_BRIDGE,
	GR_HIP_IFACE_TYPE_VXLAN,
	GR_HIP_IFACE_TYPE_COUNT,
};

// gr_iface_flags_t, gr_infra.h:31-38
#define GR_HIP_IFACE_F_UP 0x0001
#define GR_HIP_IFACE_F_PROMISC 0x0002
#define GR_HIP_IFACE_F_PACKET_TRACE 0x0004
#define GR_HIP_IFACE_F_SNAT_STATIC 0x0008
#define GR_HIP_IFACE_F_SNAT_DYNAMIC 0x0010

// gr_iface_mode_t, gr_infra.h:56-62
enum {
	GR_HIP_IFACE_MODE_VRF = 0,
	GR_HIP_IFACE_MODE_XC,
	GR_HIP_IFACE_MODE_BOND,
	GR_HIP_IFACE_MODE_BRIDGE,
	GR_HIP_IFACE_MODE_COUNT,
};

// gr_nh_state_t / gr_nh_flags_t / gr_nh_type_t, modules/infra/api/gr_nexthop.h:12-40
enum {
	GR_HIP_NH_S_NEW = 0,
	GR_HIP_NH_S_PENDING,
	GR_HIP_NH_S_REACHABLE,
	GR_HIP_NH_S_STALE,
	GR_HIP_NH_S_FAILED,
};
#define GR_HIP_NH_F_LOCAL 0x01
#define GR_HIP_NH_F_GATEWAY 0x02
#define GR_HIP_NH_F_LINK 0x04
#define GR_HIP_NH_F_MCAST 0x08
enum {
	GR_HIP_NH_T_L3 = 1,
	GR_HIP_NH_T_SR6_OUTPUT,
	GR_HIP_NH_T_SR6_LOCAL,
	GR_HIP_NH_T_DNAT,
	GR_HIP_NH_T_BLACKHOLE,
	GR_HIP_NH_T_REJECT,
	GR_HIP_NH_T_GROUP,
	GR_HIP_NH_T_COUNT,
};

// eth_domain_t, modules/infra/datapath/eth.h:14-21
enum {
	GR_HIP_ETH_DOMAIN_UNKNOWN = 0,
	GR_HIP_ETH_DOMAIN_LOOPBACK,
	GR_HIP_ETH_DOMAIN_LOCAL,
	GR_HIP_ETH_DOMAIN_BROADCAST,
	GR_HIP_ETH_DOMAIN_MULTICAST,
	GR_HIP_ETH_DOMAIN_OTHER,
};

// addr_family_t (api/gr_net_types.h): GR_AF_UNSPEC / GR_AF_IP4 / GR_AF_IP6
#define GR_HIP_AF_UNSPEC 0
#define GR_HIP_AF_IP4 1
#define GR_HIP_AF_IP6 2

// RTE_MBUF_F_RX_IP_CKSUM_* status reduced to what ip_input.c:80-92 tests.
#define GR_HIP_CKSUM_UNKNOWN 0 // UNKNOWN or NONE: verify in software
#define GR_HIP_CKSUM_BAD 1
#define GR_HIP_CKSUM_GOOD 2

#define GR_HIP_IFACE_ID_UNDEF 0 // gr_infra.h:48
#define GR_HIP_MAX_IFACES 1024 // default GROUT_MAX_IFACES, main/config.c:277
#define GR_HIP_MAX_NEXTHOPS ((1u << 24) - 1) // nh slot must fit 24 bits
#define GR_HIP_MAX_NH_GROUP_RETA 4096 // MAX_NH_GROUP_RETA_SIZE, nexthop.h:80

// ---------------------------------------------------------------------------
// Terminal edges: the next node of the replaced sub-graph a packet goes to.
// Each value is named after the grout node.
// ---------------------------------------------------------------------------
enum gr_hip_edge {
	GR_HIP_E_PUNT = 0, // not handled on the GPU: run grout's CPU iface_input
	// iface_input (iface_input.c:13-18, mode edges :20-28)
	GR_HIP_E_IFACE_MODE_UNKNOWN, // "iface_mode_unknown" (drop)
	GR_HIP_E_IFACE_INPUT_ADMIN_DOWN, // "iface_input_admin_down" (drop)
	GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN, // "iface_input_unknown_vlan" (drop)
	GR_HIP_E_XCONNECT, // "xconnect" (mode XC)
	GR_HIP_E_BRIDGE_INPUT, // "bridge_input" (mode BRIDGE; iface_output BRIDGE)
	// eth_input (eth_input.c:17-22, l2l3 edges :24-32)
	GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE, // "eth_input_unknown_type" (drop)
	GR_HIP_E_ETH_INPUT_INVALID_IFACE, // "eth_input_invalid_iface" (drop)
	GR_HIP_E_SNAP_INPUT, // "snap_input"
	GR_HIP_E_ARP_INPUT, // "arp_input"
	GR_HIP_E_IP6_INPUT, // "ip6_input"
	GR_HIP_E_LACP_INPUT, // "lacp_input"
	// ip_input (ip_input.c:20-32, nh type edges :34-44)
	GR_HIP_E_IP_INPUT_LOCAL, // "ip_input_local"
	GR_HIP_E_IP_INPUT_LOCAL_CT, // local dst on a SNAT_DYNAMIC iface: grout's
	                            // conntrack picks "ip_input_local" or
	                            // "dnat44_dynamic" (ip_input.c:170-185)
	GR_HIP_E_IP_ERROR_DEST_UNREACH, // "ip_error_dest_unreach"
	GR_HIP_E_IP_INPUT_BAD_CHECKSUM, // "ip_input_bad_checksum" (drop)
	GR_HIP_E_IP_INPUT_BAD_ADDRESS, // "ip_input_bad_address" (drop)
	GR_HIP_E_IP_INPUT_BAD_LENGTH, // "ip_input_bad_length" (drop)
	GR_HIP_E_IP_INPUT_BAD_VERSION, // "ip_input_bad_version" (drop)
	GR_HIP_E_IP_INPUT_OTHER_HOST, // "ip_input_other_host" (drop)
	GR_HIP_E_IP_BLACKHOLE, // "ip_blackhole" (drop)
	GR_HIP_E_DNAT44_STATIC, // "dnat44_static"
	// ip_forward (ip_forward.c:7-11)
	GR_HIP_E_IP_ERROR_TTL_EXCEEDED, // "ip_error_ttl_exceeded"
	// ip_output (ip_output.c:21-30, type edges :32-54)
	GR_HIP_E_IP_HOLD, // "ip_hold"
	GR_HIP_E_IP_OUTPUT_ERROR, // "ip_output_error" (drop)
	GR_HIP_E_IP_FRAGMENT, // "ip_fragment"
	GR_HIP_E_IP_ERROR_FRAG_NEEDED, // "ip_error_frag_needed"
	GR_HIP_E_SR6_OUTPUT, // "sr6_output"
	GR_HIP_E_XVRF, // "xvrf"
	GR_HIP_E_IPIP_OUTPUT, // "ipip_output"
	GR_HIP_E_IP_OUTPUT_SNAT, // egress iface has SNAT flags: grout's
	                         // snat44_process (nat_datapath.h:57-67) then the
	                         // rest of ip_output run on the CPU
	// eth_output (eth_output.c:14-19)
	GR_HIP_E_ETH_OUTPUT_NO_MAC, // "eth_output_no_mac" (drop)
	// iface_output (iface_output.c:16-21, type edges :23-33)
	GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE, // "iface_output_inval_type" (drop)
	GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN, // "iface_output_admin_down" (drop)
	GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT, // "iface_output_vlan_no_parent" (drop)
	GR_HIP_E_BOND_OUTPUT, // "bond_output"
	GR_HIP_E_VXLAN_OUTPUT, // "vxlan_output"
	GR_HIP_E_PORT_OUTPUT, // "port_output": the forwarded case
	// ip6_input (ip6_input.c:19-29, nh type edges :32-42,163-164)
	GR_HIP_E_IP6_INPUT_LOCAL, // "ip6_input_local"
	GR_HIP_E_IP6_ERROR_DEST_UNREACH, // "ip6_error_dest_unreach"
	GR_HIP_E_IP6_INPUT_NOT_MEMBER, // "ip6_input_not_member" (drop)
	GR_HIP_E_IP6_INPUT_OTHER_HOST, // "ip6_input_other_host" (drop)
	GR_HIP_E_IP6_INPUT_BAD_VERSION, // "ip6_input_bad_version" (drop)
	GR_HIP_E_IP6_INPUT_BAD_ADDR, // "ip6_input_bad_addr" (drop)
	GR_HIP_E_IP6_INPUT_BAD_LENGTH, // "ip6_input_bad_length" (drop)
	GR_HIP_E_IP6_BLACKHOLE, // "ip6_blackhole" (drop)
	GR_HIP_E_SR6_LOCAL, // "sr6_local" (srv6_local.c:481)
	// ip6_forward (ip6_forward.c:7-11)
	GR_HIP_E_IP6_ERROR_TTL_EXCEEDED, // "ip6_error_ttl_exceeded"
	// ip6_output (ip6_output.c:19-26, type edges :28-50)
	GR_HIP_E_IP6_HOLD, // "ip6_hold"
	GR_HIP_E_IP6_OUTPUT_ERROR, // "ip6_output_error" (drop)
	GR_HIP_E_IP6_OUTPUT_TOO_BIG, // "ip6_output_too_big" (drop)
	GR_HIP_E_COUNT,
};
// Registration value meaning "the next node of the chain" (eth_input for an
// iface mode, ip_input for an ether type, ip_forward for an ip_input nexthop
// type, eth_output for an ip_output type): never appears in a verdict.
#define GR_HIP_EDGE_CHAIN 0xff
// eth_input type edge value: continue into ip6_input on the GPU (the default
// for RTE_ETHER_TYPE_IPV6; GR_HIP_E_IP6_INPUT hands IPv6 to grout's CPU nodes)
#define GR_HIP_EDGE_CHAIN6 0xfe

// ---------------------------------------------------------------------------
// Control-plane mirrors (host -> device).
// ---------------------------------------------------------------------------

// Device mirror of struct iface (iface.h:20-35 + __gr_iface_base
// gr_infra.h:73-87 + the per-type info the datapath reads). 32 bytes.
struct gr_hip_iface {
	uint16_t id; // == index in the table; 0 = slot unused
	uint8_t type; // GR_HIP_IFACE_TYPE_*
	uint8_t mode; // GR_HIP_IFACE_MODE_*
	uint16_t flags; // GR_HIP_IFACE_F_*
	uint16_t mtu; // iface->mtu (default 1500, iface.c:618)
	uint16_t vrf_id; // L3 domain (GR_IFACE_MODE_VRF)
	uint16_t port_id; // PORT: iface_info_port(iface)->port_id (port.h:17-30)
	uint16_t vlan_id; // VLAN: iface_info_vlan(iface)->vlan_id
	uint16_t parent_id; // VLAN: iface_info_vlan(iface)->parent_id
	uint8_t mac[6]; // result of iface_get_eth_addr() (iface.c:475-487)
	uint8_t mac_ok; // 1 if iface_get_eth_addr() succeeded
	uint8_t _pad0;
	uint32_t _pad1[2];
};

// Device mirror of struct nexthop (nexthop.h:22-31) with the L3 info
// (nexthop.h:41-54, gr_nexthop.h:93-105) or the group info (nexthop.h:80-96).
// 32 bytes. A nexthop is identified by its slot index (1..); slot 0 is "no
// nexthop" (NULL), like the FIB value 0 in modules/ip/control/route.c:65,156.
struct gr_hip_nh {
	uint8_t type; // GR_HIP_NH_T_*
	uint8_t state; // GR_HIP_NH_S_* (L3)
	uint8_t flags; // GR_HIP_NH_F_* (L3)
	uint8_t af; // GR_HIP_AF_* (L3)
	uint16_t iface_id;
	uint16_t vrf_id;
	uint32_t ipv4; // network byte order, as ip4_addr_t
	uint8_t mac[6]; // L3
	uint16_t reta_size; // GROUP: power of two
	uint32_t reta_off; // GROUP: first slot of its reta in the reta table
	uint32_t single; // GROUP: nhg->nh shortcut used when n_members == 1
	uint16_t n_members; // GROUP
	uint16_t _pad0;
	uint8_t ipv6[16]; // L3, af GR_HIP_AF_IP6 (gr_nexthop.h:98-102)
};

// One IPv4 route, as gr_ip4_route_add_req (modules/ip/api/gr_ip4.h:47-56).
struct gr_hip_route4 {
	uint32_t ip; // network byte order; host bits are ignored (masked)
	uint8_t prefixlen; // 0..32
	uint8_t _pad0;
	uint16_t vrf_id;
	uint32_t nh; // nexthop slot (1..)
};

// One IPv6 route, as gr_ip6_route_add_req (modules/ip6/api/gr_ip6.h). A
// link-local prefix (fe80::/10) is scoped to iface_id like
// addr6_linklocal_scope (modules/ip6/control/ip6.h:23-36).
struct gr_hip_route6 {
	uint8_t ip[16]; // host bits are ignored (masked)
	uint8_t prefixlen; // 0..128
	uint8_t _pad0;
	uint16_t vrf_id;
	uint16_t iface_id; // scope of link-local prefixes, else ignored
	uint16_t _pad1;
	uint32_t nh; // nexthop slot (1..)
};

// ---------------------------------------------------------------------------
// Per-packet data exchanged with the kernel.
// ---------------------------------------------------------------------------

// Input metadata, 8 bytes per packet: what port_rx leaves in the mbuf and its
// private data (port_rx.c:281-316, rxtx.h:45-48) and what ip_input reads
// from rte_mbuf (ip_input.c:70-92,147).
struct gr_hip_pkt_meta {
	uint16_t iface; // iface_mbuf_data.iface (RX port iface id)
	uint16_t vlan_ck; // bits 0-11: iface_mbuf_data.vlan_id;
	                  // bits 12-13: GR_HIP_CKSUM_* from ol_flags;
	                  // bit 14: GR_HIP_META_WALK
	uint16_t pkt_len; // rte_pktmbuf_pkt_len == data_len (single segment)
	uint16_t rss; // low 16 bits of m->hash.rss (reta_size <= 4096)
};
// Graph walks. grout runs the nodes of one rte_graph_walk over at most 64
// packets (graph.c:88-91: vector_max 64, each RX queue's burst a share of
// it), and eth_output keeps a per-walk cache of the last source MAC it
// looked up (eth_output.c:37-59): after an eth_output_no_mac packet the next
// packet of the cached iface in the same walk leaves with source MAC
// 00:00:00:00:00:00. A batch is therefore cut into walks: one starts at
// packet 0, at every multiple of 64 and at every packet whose metadata has
// this bit. The rte_graph node (gr_hip_node_process) sets it at the start
// of each walk and pads so that no walk straddles a multiple of 64.
#define GR_HIP_META_WALK 0x4000

// Output verdict, 8 bytes per packet.
struct gr_hip_verdict {
	uint8_t edge; // enum gr_hip_edge
	uint8_t domain; // eth_input_mbuf_data.domain as left by eth_input
	uint16_t iface; // mbuf_data(m)->iface at that edge (ingress iface
	                // before ip_output, egress after it, the port after
	                // iface_output)
	uint32_t nh; // l3_mbuf_data.nh slot (0 = NULL)
};

#define GR_HIP_LINE 64 // bytes of frame header staged per packet

// A batch of packets, device-resident.
//   frame i:   in_frames + i * in_stride   (Ethernet header at offset 0; the
//              whole pkt_len bytes are readable, in_stride >= 64, % 16 == 0)
//   output i:  out_lines + i * out_stride  (the first 64 bytes of the frame as
//              grout leaves them at the verdict's edge; out_lines may equal
//              in_frames with out_stride == in_stride for in-place rewrite)
struct gr_hip_batch {
	const void *in_frames;
	void *out_lines;
	const struct gr_hip_pkt_meta *meta;
	struct gr_hip_verdict *verdicts;
	uint32_t n;
	uint32_t in_stride;
	uint32_t out_stride;
	uint32_t flags; // GR_HIP_BATCH_F_*
};
// Only the first 64 bytes of each frame are present (header-only staging from
// host mbufs): packets whose IPv4 header does not fit get GR_HIP_E_PUNT.
#define GR_HIP_BATCH_F_LINES_ONLY 0x1
// in_frames is an array of n frame addresses (uint64_t, device-accessible:
// device memory, or host memory pinned with gr_hip_host_register, 16-byte
// aligned frames), in_stride is ignored; out_lines NULL rewrites each frame's
// first 64 bytes in place (the bytes grout's chain changes, and the others
// as they were), else lines go to out_lines as usual.
#define GR_HIP_BATCH_F_FRAME_PTRS 0x2
// out_lines receives only the first 32 bytes of each output line, out_stride
// 32: every byte the path can change lies there (Ethernet header 0-13, IPv4
// TTL 22 and checksum 24-25, IPv6 hop limit 21); bytes 32-63 of every frame
// leave as they came. Not with in-place rewrite (out_lines NULL).
#define GR_HIP_BATCH_F_PREFIX32 0x4
#define GR_HIP_PREFIX 32

// Per-iface counters of one queue (iface.h:105-119 subset the path touches).
struct gr_hip_iface_stats {
	uint64_t rx_packets;
	uint64_t rx_bytes;
	uint64_t tx_packets;
	uint64_t tx_bytes;
};

// ---------------------------------------------------------------------------
// Entry points. All return 0 or -errno unless stated otherwise.
// ---------------------------------------------------------------------------
typedef struct gr_hip_ctx gr_hip_ctx_t;
typedef struct gr_hip_queue gr_hip_queue_t;

// Library / device lifetime. dev = HIP device ordinal.
int gr_hip_abi_version(void);
// Visible HIP devices (-ENODEV without a GPU), and the NUMA node of a device
// (from its PCI function in sysfs; 0 when the host reports none): the
// grout node maps worker graphs to devices on their socket, as grout maps
// RX queues to workers (modules/infra/control/worker.c:424-481).
int gr_hip_device_count(void);
int gr_hip_device_numa_node(int dev);
int gr_hip_init(int dev, uint32_t max_ifaces, uint32_t max_nexthops, gr_hip_ctx_t **out);
int gr_hip_fini(gr_hip_ctx_t *ctx);
const char *gr_hip_strerror(int err);

// Edge registrations (defaults = grout's default module set, applied by init).
int gr_hip_edges_eth_type(gr_hip_ctx_t *, uint16_t be_ether_type, uint8_t edge);
int gr_hip_edges_iface_mode(gr_hip_ctx_t *, uint8_t mode, uint8_t edge);
int gr_hip_edges_ip_input_nh_type(gr_hip_ctx_t *, uint8_t nh_type, uint8_t edge);
int gr_hip_edges_ip_output_nh_type(gr_hip_ctx_t *, uint8_t nh_type, uint8_t edge);
int gr_hip_edges_ip_output_iface_type(gr_hip_ctx_t *, uint8_t iface_type, uint8_t edge);
int gr_hip_edges_iface_output_type(gr_hip_ctx_t *, uint8_t iface_type, uint8_t edge);
int gr_hip_edges_ip6_input_nh_type(gr_hip_ctx_t *, uint8_t nh_type, uint8_t edge); // ip6_input.c:34
int gr_hip_edges_ip6_output_nh_type(gr_hip_ctx_t *, uint8_t nh_type, uint8_t edge); // ip6_output.c:42
int gr_hip_edges_ip6_output_iface_type(gr_hip_ctx_t *, uint8_t iface_type, uint8_t edge); // ip6_output.c:30
// The edge registered for `key` in one of the tables above (a grout node
// that continues a replaced node's work reads it, e.g. ip_output_snat):
// an enum gr_hip_edge value, GR_HIP_EDGE_CHAIN or GR_HIP_EDGE_CHAIN6.
enum {
	GR_HIP_EDGES_ETH_TYPE = 0, // key: raw big-endian ether type
	GR_HIP_EDGES_IFACE_MODE,
	GR_HIP_EDGES_IP_INPUT_NH_TYPE,
	GR_HIP_EDGES_IP_OUTPUT_NH_TYPE,
	GR_HIP_EDGES_IP_OUTPUT_IFACE_TYPE,
	GR_HIP_EDGES_IFACE_OUTPUT_TYPE,
	GR_HIP_EDGES_IP6_INPUT_NH_TYPE,
	GR_HIP_EDGES_IP6_OUTPUT_NH_TYPE,
	GR_HIP_EDGES_IP6_OUTPUT_IFACE_TYPE,
};
int gr_hip_edges_get(gr_hip_ctx_t *, int table, uint16_t key);

// Object mirrors. Changes become visible to submits issued after the call.
int gr_hip_iface_set(gr_hip_ctx_t *, const struct gr_hip_iface *ifaces, uint32_t n);
int gr_hip_iface_del(gr_hip_ctx_t *, uint16_t iface_id);
int gr_hip_nh_set(gr_hip_ctx_t *, uint32_t first_slot, const struct gr_hip_nh *nh, uint32_t n);
int gr_hip_reta_set(gr_hip_ctx_t *, uint32_t first, const uint32_t *slots, uint32_t n);

// RIB + device FIB (DIR24_8-equivalent; 2-byte entries while slots fit 15
// bits). Routes are staged in the host RIB (adds and deletes never touch the
// device or hold submitters). gr_hip_fib4_commit() publishes them: it writes
// the VRF's unpublished device copy and flips the view generation, the
// analogue of grout's RCU-protected rte_fib (modules/ip/control/route.c:87-95,
// 764). It never waits for submitted launches and returns once the upload is
// enqueued: launches already submitted finish on the old table, every submit
// after the call runs on the new one (its stream waits for the upload), and
// each launch reads one table from first packet to last. Thread-safe against
// concurrent submits on any queue.
int gr_hip_fib4_create(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8);
int gr_hip_fib4_destroy(gr_hip_ctx_t *, uint16_t vrf_id);
int gr_hip_route4_add(gr_hip_ctx_t *, const struct gr_hip_route4 *routes, uint32_t n, int replace);
int gr_hip_route4_del(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t ip, uint8_t prefixlen);
int gr_hip_fib4_commit(gr_hip_ctx_t *, uint16_t vrf_id);
// Host-side lookup in the committed tables (control-plane helper, modules/ip/control/route.c:169-185).
int gr_hip_fib4_lookup_host(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t ip_be, uint32_t *nh);
// Device table geometry: tbl8 groups in use, bytes of device memory.
int gr_hip_fib4_info(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t *n_routes, uint32_t *tbl8_used, uint64_t *dev_bytes);

// IPv6 FIB per VRF (create_fib6 / rib6_insert_or_replace / rib6_delete,
// modules/ip6/control/route.c:66-98,230-345). A multibit trie: a 2^16-entry
// first level indexed by the first two address bytes, then 256-entry groups
// per further byte (num_tbl8 of them; 0 = 1 << 16). fib6_lookup
// (modules/ip6/control/route.c:151-173) walks it; link-local destinations are scoped to the
// ingress iface first.
int gr_hip_fib6_create(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8);
int gr_hip_fib6_destroy(gr_hip_ctx_t *, uint16_t vrf_id);
int gr_hip_route6_add(gr_hip_ctx_t *, const struct gr_hip_route6 *routes, uint32_t n, int replace);
int gr_hip_route6_del(gr_hip_ctx_t *, uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen);
// Publishes like gr_hip_fib4_commit (the repainted trie, whole, into the
// unpublished copy).
int gr_hip_fib6_commit(gr_hip_ctx_t *, uint16_t vrf_id);
// Host lookup in the committed tables (tests / control plane), scoped like fib6_lookup.
int gr_hip_fib6_lookup_host(gr_hip_ctx_t *, uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint32_t *nh);
int gr_hip_fib6_info(gr_hip_ctx_t *, uint16_t vrf_id, uint32_t *n_routes, uint32_t *groups_used, uint64_t *dev_bytes);

// Queues: one per RX queue / worker; each owns a HIP stream. stream == NULL
// creates a private non-blocking stream, else the given hipStream_t is used.
int gr_hip_queue_create(gr_hip_ctx_t *, void *stream, gr_hip_queue_t **out);
int gr_hip_queue_destroy(gr_hip_queue_t *);
void *gr_hip_queue_stream(gr_hip_queue_t *);

// Device-resident fast path: enqueue the fused kernel on the queue's stream.
int gr_hip_fwd4_submit(gr_hip_queue_t *, const struct gr_hip_batch *);
// Wait until everything submitted on the queue is done. -ETIMEDOUT if a
// kernel gave up a ring wait since the last sync (its workgroup stopped
// early, so that batch's results are incomplete); the grid still drained.
int gr_hip_queue_sync(gr_hip_queue_t *);
// Device time in ms of the last `n` timed submits (HIP events around each
// timed launch, ring of 64; see "time_every"). Returns the sum; *count
// receives how many were measured.
int gr_hip_queue_kernel_ms(gr_hip_queue_t *, uint32_t n, float *ms, uint32_t *count);

// Tuning knobs, for measurements (A/B in one process). Keys:
//   "ring"      geometry of the ring kernel (loaders / storers / slots /
//               tiles in flight), 0..11; default 2;
//               12..14: geometry 2 with the 4-byte tbl24 gathers of 16 / 32
//               / 64 lanes through the scalar cache (measured slower,
//               DESIGN.md §6.1)
//   "stats"     1 = per-iface counters (default; grout always counts), 0 = off
//   "nt"        1 = nontemporal loads / stores of the streamed data (default)
//   "wg_per_cu" 0 = default grid (2 workgroups per CU, fewer if LDS
//               limits), N = N workgroups per CU
//   "fib_format" device FIB layout while every nexthop slot and tbl8 group
//               fits 15 bits: 2 = DIR24_8 with 2-byte entries (default),
//               1 = DIR-16-8-8 with 2-byte entries, 0 = DIR24_8 with 4-byte
//               entries (always used when 15 bits do not fit); applies from
//               the next gr_hip_fib4_commit ("fib16": 1 -> 1, 0 -> 0)
//   "host_direct" 1 = gr_hip_fwd4_host on pinned (hipHostMalloc'd or
//               registered) buffers runs the kernel on them directly, its
//               loads and stores crossing PCIe (default); 0 = always staged
//               chunk copies (pageable buffers always take that path)
//   "node_ptrs"  1 = gr_hip_node_process hands registered frames over by
//               address, 0 = stage header lines (default: faster from one
//               worker thread up, and much faster with several)
//   "time_every" N: only every N-th submit of a queue gets the HIP event
//               pair that gr_hip_queue_kernel_ms reads (default 1: all);
//               each pair costs ~7 us of stream time per launch. Setting
//               it restarts every queue's count: its submits 0, N, 2N ...
//               from then on are timed
//   "untimed"   1 = no events at all
//   "spin_max"  polls before a ring wait gives up (0 = default, ~0.4 s):
//               for tests of the give-up path
//   "fail_appends" N: the next N gr_hip_node_append calls fail with -ENOMEM
//               (the slot left as it was): for tests of the node's path
//   "alloc_contig" 1 = the large device arrays allocated from then on (FIB
//               tables, gr_hip_batch_alloc's buffers and gr_hip_batch_place's
//               candidates) are asked for physically contiguous first
//               (hipDeviceMallocContiguous: large fragments, fast address
//               translation for the kernel's streams and gathers), hipMalloc
//               when that fails (default); 0 = hipMalloc always
//   "tile_order" 0 = workgroup b takes 64-packet tiles b, b + G, b + 2G ...
//               (default), 1 = one contiguous run of tiles per workgroup,
//               2 = one region per XCD, its workgroups interleaved in it,
//               3 = runs of "tile_run" tiles (default 16), run j of
//               workgroup b being run j * G + b
//   "resident"  1 = node batches (gr_hip_node_send) go to the context's
//               resident kernel: one long-lived launch whose workgroups take
//               batches from per-queue descriptor rings in pinned host memory,
//               completion polled as a memory word (no launch, no runtime call,
//               no hardware queue per batch); per-iface counters are then the
//               hand-back's. 0 = one launch per batch (default; the grout
//               module turns it on unless gpu_fwd4_conf.launch_per_batch)
//   "resident_wgs" rings (workgroups) per queue, 1..8: a batch is split over
//               up to that many, "resident_tiles" tiles each (default 8;
//               queues taking their rings from then on)
//   "resident_tiles" 64-packet tiles per workgroup a batch is split into
//               (default 8)
//   "resident_split" at most this many of a queue's rings per batch, from the
//               next batch on (default 0: all of them)
//   "resident_budget" workgroups the batches of all busy queues (queues with
//               resident batches in flight) are split over together: a batch
//               takes at most budget / busy rings, at least 1 (default 32: a
//               lone worker's batch up to its 8 rings, 8 busy workers' 4 each,
//               16 busy workers' 2); 0 = no cap. "resident_busy" (read): busy
//               queues now
//   "resident_rings" rings in all (default 256: 32 queues; before the first
//               resident batch only; "resident_ring_count" reads it); the
//               workgroups of rings no queue holds leave at once
//   "resident_nap" a queue's helper rings (all but its first: they poll a
//               wake word in device memory that the first ring's workgroup
//               writes) back off their idle polls up to this many s_sleep(8)
//               between reads (default 16; the next launch)
//   "resident_ms" the kernel leaves once no ring has finished a batch for this
//               long; the next batch launches it again (default 50)
//   "resident_launches" (read) resident launches so far
//   "resident_rotate" 1 = a batch of k rings posted while other batches of
//               its queue are in flight runs on the queue's helper rings
//               h .. h + k - 1, h in turn, its first ring only waking them
//               (default 0; the
//               grout module sets it when more than one batch per graph is on
//               the GPU); "resident_rotating" (read) the setting
//   "resident_wait_ms" a resident batch not done this long after its post
//               (default 500) is cancelled: the kernel is stopped, what it did
//               not start is retired and handed back as not reached (the node
//               punts it); a kernel that does not leave makes the context's
//               resident path dead (-EDEADLK, nothing of the batch reused)
//   "resident_reserve_cu" CUs no ring may take (default 16; before the first
//               resident batch): a queue finds rings only while every ring
//               held on the device, over all contexts, fits the other CUs at
//               the kernel's occupancy, else it launches per batch
//   "resident_cap" / "resident_held" (read) those rings: the device's cap,
//               and what the queues of every context hold
//   "resident_cancels" (read) batches cancelled past their deadline
//   "resident_dead" (read) 1 once a kernel would not leave
//   "resident_hold" tests: 1 = the kernel leaves and is not launched again
//               (its batches reach their deadline), 0 = back to normal
//   "stage_min_tiles" the fast adjacencies (and IPv6 first-level slice) are
//               staged in each workgroup's LDS only when the launch gives every
//               workgroup at least this many 64-packet tiles (default 4);
//               smaller launches read them from the global tables
//   "fib_format_of" (read) the format VRF `value`'s FIB is on the device in
//   "occupancy" (read) resident workgroups per CU of the current variant
//   "host_path_last" (read) GR_HIP_HOST_PATH_* of the last gr_hip_fwd4_host(_ex)
//   "sync_check" debugging: the host path waits after every step it enqueues
//       and names a failing step on stderr (-EIO)
//   "stats_copy" measurement only: counters read by a copy and reset by a
//       memset, as before round 6 (tools/stats_read_probe.py)
//   "commit_us_stage" / "commit_us_enqueue" / "commit_us_publish" (read) the last
//       gr_hip_fib4_commit's phases in microseconds: host staging, the
//       enqueue under the shared lock, the flip under the exclusive lock
// Returns 0 (or the value read), -EINVAL, or -ENOENT for an unknown key.
int gr_hip_tune(gr_hip_ctx_t *, const char *key, int value);

// Host-memory path (header-only staging): `n` 64-byte header lines and
// metadata in host memory in, lines and verdicts back to host memory. On
// pinned buffers the kernel reads and writes them over PCIe itself
// ("host_direct"); otherwise chunks are copied through the queue's device
// staging on 3 streams. Completes before return. On -ETIMEDOUT (a kernel
// gave up, see gr_hip_queue_sync) every 64-packet tile was either processed
// whole or not at all: the verdicts of the packets it did not reach are
// left as they were (the staged path fills them with 0xff bytes).
int gr_hip_fwd4_host(
	gr_hip_queue_t *,
	const void *lines,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	struct gr_hip_verdict *verdicts
);
// Which of the three ways the last call took (gr_hip_tune "host_path_last"):
// every buffer device-accessible pinned memory and "host_direct" on (the
// kernel over PCIe), pinned with "host_direct" off (runtime copies through
// device staging), or any buffer pageable (the CPU copies it through the
// queue's own pinned buffers: pageable pointers never reach the runtime).
#define GR_HIP_HOST_PATH_DIRECT 0
#define GR_HIP_HOST_PATH_STAGED 1
#define GR_HIP_HOST_PATH_PAGEABLE 2
// The same with the output stride chosen: GR_HIP_LINE (64, whole lines, as
// gr_hip_fwd4_host) or GR_HIP_PREFIX (32: packed prefixes holding every byte
// the path changes, GR_HIP_BATCH_F_PREFIX32; less PCIe traffic back).
int gr_hip_fwd4_host_ex(
	gr_hip_queue_t *,
	const void *lines,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *verdicts
);

// Per-iface counters accumulated by the queue's kernels (rx in iface_input,
// tx in iface_output). `stats` receives max_ifaces entries.
int gr_hip_queue_stats(gr_hip_queue_t *, struct gr_hip_iface_stats *stats, uint32_t max_ifaces, int reset);
// The same counters before they are summed: `stats` receives 64 shards of
// `w` ifaces ([shard][w]; a workgroup b of a launch counts into shard b % 64).
// Returns the number of shards. Diagnostics (which workgroups counted what);
// grout's counters need only gr_hip_queue_stats / gr_hip_node_iface_stats.
// Both read the device counters at the memory side (one agent-scope atomic
// per counter, reset by exchange), never with a plain copy or memset.
int gr_hip_queue_stats_shards(gr_hip_queue_t *, struct gr_hip_iface_stats *stats, uint32_t w, int reset);

// Device / pinned host memory helpers for C callers without a framework
// allocator (pinned buffers make gr_hip_fwd4_host copies asynchronous).
int gr_hip_host_alloc(gr_hip_ctx_t *, size_t bytes, void **ptr);
int gr_hip_host_free(gr_hip_ctx_t *, void *ptr);
int gr_hip_dev_alloc(gr_hip_ctx_t *, size_t bytes, void **dptr);
int gr_hip_dev_free(gr_hip_ctx_t *, void *dptr);
int gr_hip_memcpy_h2d(gr_hip_ctx_t *, void *dst, const void *src, size_t bytes);
int gr_hip_memcpy_d2h(gr_hip_ctx_t *, void *dst, const void *src, size_t bytes);
// Device buffers of a batch of `n` packets for gr_hip_fwd4_submit: frames
// (n * in_stride bytes), output lines (n * 64), metadata and verdicts, all
// zeroed; fills *b (flags 0, out_stride 64). Free with gr_hip_batch_free.
int gr_hip_batch_alloc(gr_hip_ctx_t *, uint32_t n, uint32_t in_stride, struct gr_hip_batch *b);
// Which HBM pages back the frames and the output lines changes the kernel's
// time by up to ~15 %: some regions of an allocation translate slowly (the
// L1 TLB sits at its in-flight limit). With the batch's
// frames and metadata in place, this allocates `candidates` more output-line
// buffers (plain and, with "alloc_contig", physically contiguous in turn), times each
// (and the current one) over the batch on a private queue without counters
// and keeps the fastest; then `candidates` more frame buffers, each holding a
// copy of the frames, timed against the lines kept, and keeps the fastest
// of those and the current one. The rest are freed. `b` must come from
// gr_hip_batch_alloc; in_frames and out_lines may change (the frames keep
// their content), output lines and verdicts are overwritten (with the
// batch's results). On error the batch is left as it was.
int gr_hip_batch_place(gr_hip_ctx_t *, struct gr_hip_batch *b, uint32_t candidates);
int gr_hip_batch_free(gr_hip_ctx_t *, struct gr_hip_batch *b);
// Pin and map caller memory for the GPU (grout: the mbuf pools' memory), so
// that frames in it can be handed over by address (GR_HIP_BATCH_F_FRAME_PTRS,
// gr_hip_node_process). Memory already pinned is recorded as it is.
// -EEXIST if the range overlaps a registered one.
int gr_hip_host_register(gr_hip_ctx_t *, void *ptr, size_t bytes);
int gr_hip_host_unregister(gr_hip_ctx_t *, void *ptr);
// The device address of host address `ptr` in a registered range (-ENOENT).
int gr_hip_host_dev_addr(gr_hip_ctx_t *, const void *ptr, uint64_t *dev);

// ---------------------------------------------------------------------------
// rte_graph node shim: mbuf staging and hand-back
// ---------------------------------------------------------------------------
//
// What the grout node that replaces iface_input copies
// between each rte_mbuf (+ its 64-byte private area, mbuf.h:29-41) and the
// fast path. After gr_hip_node_apply() the mbuf is exactly as grout's CPU
// chain would have left it at `edge`: frame bytes (the L2 rewrite, TTL and
// checksum), data_off / data_len / pkt_len (eth_input's adj(14), undone by
// eth_output's prepend), packet_type (ip_output.c:85) and the private data
// the next node reads (iface, vlan_id, eth_input domain, l3 nexthop).
struct gr_hip_mbuf {
	void *frame; // in: rte_pktmbuf_mtod(m) as port_rx delivered it (64 bytes readable)
	uint32_t pkt_len; // in/out
	uint16_t data_len; // in/out
	uint16_t data_off; // in/out
	uint32_t packet_type; // in/out: RTE_PTYPE_L3_IPV4 / _IPV6 set by ip_output / ip6_output
	uint32_t rss; // in: m->hash.rss
	uint16_t iface; // in/out: iface_mbuf_data.iface (by id)
	uint16_t vlan_id; // in/out: iface_mbuf_data.vlan_id
	uint8_t ck; // in: GR_HIP_CKSUM_* from ol_flags
	uint8_t edge; // out: enum gr_hip_edge, the next node
	uint8_t domain; // out: eth_input_mbuf_data.domain
	uint8_t flags; // in: GR_HIP_MBUF_F_*
	uint32_t nh; // out: l3_mbuf_data.nh as a nexthop slot (0 = NULL)
};
// This mbuf starts a graph walk: the node sets it on the first mbuf of each
// process() call (one rte_graph_walk's iface_input stream).
#define GR_HIP_MBUF_F_WALK 0x01

#define GR_HIP_PTYPE_L3_IPV4 0x10 // RTE_PTYPE_L3_IPV4 (rte_mbuf_ptype.h)
#define GR_HIP_PTYPE_L3_IPV6 0x40 // RTE_PTYPE_L3_IPV6 (rte_mbuf_ptype.h)

// The nodes the fast path replaces, for per-node statistics.
enum gr_hip_node {
	GR_HIP_NODE_IFACE_INPUT = 0,
	GR_HIP_NODE_ETH_INPUT,
	GR_HIP_NODE_IP_INPUT,
	GR_HIP_NODE_IP_FORWARD,
	GR_HIP_NODE_IP_OUTPUT,
	GR_HIP_NODE_ETH_OUTPUT,
	GR_HIP_NODE_IFACE_OUTPUT,
	GR_HIP_NODE_IP6_INPUT,
	GR_HIP_NODE_IP6_FORWARD,
	GR_HIP_NODE_IP6_OUTPUT,
	GR_HIP_NODE_COUNT,
};

// rte_graph node counters as grout collects them (main_loop.c:40-66):
// packets = sum of process() return values, calls = process() invocations,
// one per node per graph walk that reaches it. Every node returns nb_objs
// except ip_output and ip6_output, which return only what they sent to
// eth_output (ip_output.c:153,162, ip6_output.c:144).
struct gr_hip_node_stats {
	uint64_t packets[GR_HIP_NODE_COUNT];
	uint64_t calls[GR_HIP_NODE_COUNT];
};

// The last node of the fast path a packet with this verdict went through
// (-1 for GR_HIP_E_PUNT, which grout's CPU iface_input takes instead); ip6:
// the packet is IPv6 (the eth_output / iface_output edges are shared).
int gr_hip_edge_node(uint8_t edge, uint32_t nh, int ip6);

// Graph walks of n mbufs: one starts at m[0], at every mbuf with
// GR_HIP_MBUF_F_WALK, and `burst` (1..256, grout's rx_burst_max /
// vector_max limit RTE_GRAPH_BURST_SIZE, graph.c:612-650; 0 = 64) mbufs
// after the previous start. The staged layout puts mbuf i at pos[i],
// padding so that no walk of up to 64 packets straddles a multiple of 64
// (the kernel resolves eth_output's per-walk cache inside a 64-packet tile,
// see GR_HIP_META_WALK) and a longer walk starts on one (the hand-back
// resolves the cache over the whole walk). Returns the number of staged
// slots (>= n), or -errno.
int gr_hip_node_layout(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, uint32_t *pos);

// Stage n mbufs: the first 64 bytes at each frame (read whatever data_len
// says, as grout's nodes do: an mbuf's data room always has them) into
// lines[pos[i] * 64] (lines NULL: skipped), and their metadata, with
// GR_HIP_META_WALK at each walk start. pos NULL: pos[i] = i. Slots the
// layout leaves free get metadata with iface 0 (the kernel punts them, they
// count nowhere) and zeroed lines.
int gr_hip_node_stage(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, const uint32_t *pos, void *lines,
		      struct gr_hip_pkt_meta *meta);

// Hand back: apply the fast path's verdicts and rewritten header lines
// (slot pos[i], line_stride apart, >= 32: only the first 26 bytes of a line
// are written back, so packed 32-byte prefixes do; lines NULL: the frames
// were rewritten in place) to the mbufs. ifaces[id] / nh[slot] are the mirrors pushed with
// gr_hip_iface_set / gr_hip_nh_set (the egress VLAN tag and the ingress VLAN
// demux are read from them). stats (optional) accumulates the per-node
// counters of the graph walks (as gr_hip_node_layout cuts them).
int gr_hip_node_apply(
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
);

// The node's whole walk on a queue: stage, forward on the GPU, apply with the
// context's mirrors. When every frame lies in memory registered with
// gr_hip_host_register (and is 16-byte aligned), the GPU reads and rewrites
// the frames in place over PCIe and only 8-byte frame addresses and metadata
// are staged when "node_ptrs" is on (default off); otherwise header lines are
// staged through gr_hip_fwd4_host. Returns the number of mbufs handed back as
// GR_HIP_E_PUNT, untouched, because a kernel gave up before reaching them
// (0 normally; the others are handed back as usual), or -errno with every
// mbuf untouched.
int gr_hip_node_process(gr_hip_queue_t *, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst,
			struct gr_hip_node_stats *stats);

// The same walk in two halves, so that the GPU forwards one walk while the
// CPU stages the next (and the node hands back the one before): start lays
// out and stages the mbufs and enqueues the GPU work without waiting; finish
// waits for the OLDEST walk started on the queue and hands it back, with the
// return value of gr_hip_node_process. Up to GR_HIP_NODE_DEPTH walks per
// queue are in flight (start returns -EBUSY beyond); their mbufs belong to
// the queue until their finish, which reports them in *m / *n. Walks finish
// in start order. gr_hip_node_process is start + finish and returns -EBUSY
// while walks are in flight.
// (4: the grout node keeps up to depth - 1 batches on the GPU while it
// accumulates the next, gpu_fwd4_conf.depth; a walk slot's pinned staging
// is allocated at its first use)
#define GR_HIP_NODE_DEPTH 4
int gr_hip_node_start(gr_hip_queue_t *, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst);
int gr_hip_node_finish(gr_hip_queue_t *, struct gr_hip_mbuf **m, uint32_t *n, struct gr_hip_node_stats *stats);
// The start half fused with the node's own pass over its mbufs, so that each
// rte_mbuf is touched once: the node appends each rte_graph walk's views as
// the walk brings them (gr_hip_node_append lays them out and stages their
// header lines and metadata into the queue's open walk slot at once, while
// the frames are in cache), then sends what it appended (gr_hip_node_send,
// with m / n = every view appended since the last send, in order: the same
// pointer the appends read, kept until finish). The layout and the staged
// bytes are gr_hip_node_start's for the same views, and the walk finishes
// the same way. Each append after the first of a slot must start with a
// GR_HIP_MBUF_F_WALK view (-EINVAL otherwise). append returns the slots
// staged so far, -EBUSY while GR_HIP_NODE_DEPTH walks are in flight; send
// returns 0, or -EINVAL when m / n are not what was appended (the appended
// walk is dropped, the views untouched). gr_hip_node_discard drops what was
// appended and not sent (a walk that will not go to the GPU).
int gr_hip_node_append(gr_hip_queue_t *, const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst);
// Where the hand-back writes in the caller's own mbufs, so that the finish
// sets them directly instead of the views (one pass over the batch, not
// two): byte offsets of the fields grout's nodes read in struct rte_mbuf
// (DPDK rte_mbuf_core.h: data_off and data_len uint16_t, pkt_len and
// packet_type uint32_t) and in its private area (grout mbuf.h:29-41,
// rxtx.h:45-48, eth.h:23-36, l3.h:9: iface a pointer, vlan_id uint16_t,
// domain a 32-bit enum, the nexthops pointers), and the caller's registries
// that turn a verdict's iface id / nexthop slot into the object pointer the
// private data holds (read with acquire loads; NULL = no longer registered).
// No DPDK type crosses the ABI.
struct gr_hip_mbuf_layout {
	uint16_t data_off, data_len, pkt_len, packet_type; // in struct rte_mbuf
	uint16_t priv; // the private area: (char *)m + priv (rte_mbuf_to_priv)
	uint16_t priv_iface; // mbuf_data.iface
	uint16_t priv_vlan_id; // iface_mbuf_data.vlan_id
	uint16_t priv_domain; // eth_input_mbuf_data.domain
	uint16_t priv_eth_nh; // eth_input_mbuf_data.nh
	uint16_t priv_l3_nh; // l3_mbuf_data.nh
	uint32_t n_ifaces, n_nh; // registry sizes
	const void *const *ifaces; // iface id -> object
	const void *const *nh; // nexthop slot -> object
	// read by gr_hip_node_append_mbufs (staging straight from the mbufs):
	uint16_t buf_addr; // in struct rte_mbuf (void *): the frame is buf_addr + data_off
	uint16_t ol_flags; // in struct rte_mbuf (uint64_t)
	uint16_t rss; // hash.rss in struct rte_mbuf (uint32_t)
	uint16_t iface_id; // the id (uint16_t) inside the object mbuf_data.iface points to
	// RTE_MBUF_F_RX_IP_CKSUM_MASK, _GOOD and _BAD (rte_mbuf_core.h): ol_flags
	// & ck_mask equal to ck_good / ck_bad is GR_HIP_CKSUM_GOOD / _BAD, anything
	// else GR_HIP_CKSUM_UNKNOWN (ip_input.c:80-92 verifies in software)
	uint64_t ck_mask, ck_good, ck_bad;
};
// gr_hip_node_append without views: the node passes one rte_graph walk's
// mbufs (mbufs[0] starts it; it is cut every `burst` mbufs) and the library
// reads each one through the layout (single segment; the frame at buf_addr +
// data_off, pkt_len, rss, the checksum status, the iface id and vlan_id from
// the private data) while it lays the walk out and stages its header line
// and metadata, in one pass. The appends of one batch pass consecutive parts
// of one mbufs array, with one layout (-EINVAL otherwise; a slot holds walks
// appended one way only). The next gr_hip_node_send then takes m == NULL and
// n = every mbuf appended since the last send, and the batch is handed back
// with gr_hip_node_finish_mbufs on that array (kept until then): the
// hand-back reads each mbuf's fields again through the layout before it
// writes them (gr_hip_node_finish drops such a batch with -EINVAL, after
// waiting for its GPU work: the caller may free the mbufs then).
// Returns as gr_hip_node_append.
int gr_hip_node_append_mbufs(gr_hip_queue_t *, void *const *mbufs, uint32_t n,
			     const struct gr_hip_mbuf_layout *layout, uint32_t burst);
// gr_hip_node_finish handing the oldest walk back straight onto its mbufs:
// mbufs[i] is the mbuf of view i (the views sent; they are read, not
// written). Each mbuf gets what gr_hip_node_apply gives its view, in its own
// fields and private data for the node behind its edge (the iface
// everywhere; vlan_id before eth_input and past iface_output; eth_input's
// domain and a NULL nexthop, ip_input's l3 nexthop over them), and
// edges[i] its edge. A packet whose iface or nexthop is no longer in the
// registries keeps its mbuf fields and private data and goes to
// GR_HIP_E_IP_OUTPUT_ERROR, counted in *stale; GR_HIP_E_PUNT: untouched.
// Returns as gr_hip_node_finish (edges not written on -errno).
int gr_hip_node_finish_mbufs(gr_hip_queue_t *, void *const *mbufs, const struct gr_hip_mbuf_layout *layout,
			     uint8_t *edges, uint32_t *stale, struct gr_hip_node_stats *stats);
int gr_hip_node_send(gr_hip_queue_t *, struct gr_hip_mbuf *m, uint32_t n, uint32_t burst);
int gr_hip_node_discard(gr_hip_queue_t *);
// Walks in flight on the queue; *ready (optional) = 1 when the oldest one's
// GPU work has completed (its finish will not wait).
int gr_hip_node_pending(gr_hip_queue_t *, int *ready);
// Per-iface rx / tx counters of the queue's node walks since the last reset,
// where grout counts them: rx in iface_input past its admin-down and
// unknown-VLAN drops (the VLAN sub-interface and its parent), tx in
// iface_output past its no-parent and admin-down drops (the egress iface and
// a VLAN's parent) (modules/infra/datapath/iface_input.c:93-95,
// iface_output.c:103-105, rxtx.h:84-117). The kernels count them (the
// "stats" knob, default on; with it off the hand-back counts them on the
// host): this call folds in a copy of the queue's device counters taken
// behind the walks launched so far, without waiting for it while walks are
// in flight (it lands by a later call), and waiting for it when none is, so
// that the counts are then exact. The grout node folds the result into
// grout's per-lcore iface_stats at its housekeeping tick
// (gpu_fwd4_stats_flush). Call from the thread that drives the queue's
// walks. `stats` receives max_ifaces entries, indexed by iface id.
int gr_hip_node_iface_stats(gr_hip_queue_t *, struct gr_hip_iface_stats *stats, uint32_t max_ifaces, int reset);

// Measurement: nanoseconds gr_hip_node_start (append + send) and
// gr_hip_node_finish spent in each part, summed over every queue of the
// process since the last reset, while the clocks run (the "node_prof" knob
// of gr_hip_tune, process-wide, default off: each clock read costs tens of
// nanoseconds per append). out[k] for k < n; returns
// GR_HIP_NODE_PROF_COUNT.
enum {
	GR_HIP_NODE_PROF_LAYOUT, // (unused: the layout is part of the staging)
	GR_HIP_NODE_PROF_PREP, // verdicts filled
	GR_HIP_NODE_PROF_LOCK, // the context lock, shared
	GR_HIP_NODE_PROF_STAGE, // layout + staging (gr_hip_node_append), buffers grown
	GR_HIP_NODE_PROF_LAUNCH, // the kernel launch (host_direct)
	GR_HIP_NODE_PROF_RECORD, // the walk's completion event
	GR_HIP_NODE_PROF_FIN_WAIT, // finish: the wait for the walk's GPU work and its error check
	GR_HIP_NODE_PROF_FIN_SCAN, // finish: the pass for packets a kernel that gave up left
	GR_HIP_NODE_PROF_FIN_APPLY, // finish: the context lock and the hand-back onto the views
	GR_HIP_NODE_PROF_COUNT,
};
int gr_hip_node_prof(uint64_t *out, uint32_t n, int reset);

#ifdef __cplusplus
}
#endif
