// SPDX-License-Identifier: BSD-3-Clause
//
// gpu_fwd4_node.h -- configuration and counters of the fast path's grout node
// (gpu_fwd4_node.c). The control plane mirrors its objects into the context
// returned by gpu_fwd4_hip_ctx() with the gr_hip_* calls.
#pragma once

#include <grout_hip.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct rte_graph;

// next_nodes in enum gr_hip_edge order (include/grout_hip.h)
#define GPU_FWD4_EDGES                                                                             \
	[GR_HIP_E_PUNT] = "iface_input_cpu",                                                       \
	[GR_HIP_E_IFACE_MODE_UNKNOWN] = "iface_mode_unknown",                                      \
	[GR_HIP_E_IFACE_INPUT_ADMIN_DOWN] = "iface_input_admin_down",                              \
	[GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN] = "iface_input_unknown_vlan",                          \
	[GR_HIP_E_XCONNECT] = "xconnect",                                                          \
	[GR_HIP_E_BRIDGE_INPUT] = "bridge_input",                                                  \
	[GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE] = "eth_input_unknown_type",                              \
	[GR_HIP_E_ETH_INPUT_INVALID_IFACE] = "eth_input_invalid_iface",                            \
	[GR_HIP_E_SNAP_INPUT] = "snap_input",                                                      \
	[GR_HIP_E_ARP_INPUT] = "arp_input",                                                        \
	[GR_HIP_E_IP6_INPUT] = "ip6_input",                                                        \
	[GR_HIP_E_LACP_INPUT] = "lacp_input",                                                      \
	[GR_HIP_E_IP_INPUT_LOCAL] = "ip_input_local",                                              \
	[GR_HIP_E_IP_INPUT_LOCAL_CT] = "ip_input_local_ct",                                        \
	[GR_HIP_E_IP_ERROR_DEST_UNREACH] = "ip_error_dest_unreach",                                \
	[GR_HIP_E_IP_INPUT_BAD_CHECKSUM] = "ip_input_bad_checksum",                                \
	[GR_HIP_E_IP_INPUT_BAD_ADDRESS] = "ip_input_bad_address",                                  \
	[GR_HIP_E_IP_INPUT_BAD_LENGTH] = "ip_input_bad_length",                                    \
	[GR_HIP_E_IP_INPUT_BAD_VERSION] = "ip_input_bad_version",                                  \
	[GR_HIP_E_IP_INPUT_OTHER_HOST] = "ip_input_other_host",                                    \
	[GR_HIP_E_IP_BLACKHOLE] = "ip_blackhole",                                                  \
	[GR_HIP_E_DNAT44_STATIC] = "dnat44_static",                                                \
	[GR_HIP_E_IP_ERROR_TTL_EXCEEDED] = "ip_error_ttl_exceeded",                                \
	[GR_HIP_E_IP_HOLD] = "ip_hold",                                                            \
	[GR_HIP_E_IP_OUTPUT_ERROR] = "ip_output_error",                                            \
	[GR_HIP_E_IP_FRAGMENT] = "ip_fragment",                                                    \
	[GR_HIP_E_IP_ERROR_FRAG_NEEDED] = "ip_error_frag_needed",                                  \
	[GR_HIP_E_SR6_OUTPUT] = "sr6_output",                                                      \
	[GR_HIP_E_XVRF] = "xvrf",                                                                  \
	[GR_HIP_E_IPIP_OUTPUT] = "ipip_output",                                                    \
	[GR_HIP_E_IP_OUTPUT_SNAT] = "ip_output_snat",                                              \
	[GR_HIP_E_ETH_OUTPUT_NO_MAC] = "eth_output_no_mac",                                        \
	[GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE] = "iface_output_inval_type",                            \
	[GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN] = "iface_output_admin_down",                            \
	[GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT] = "iface_output_vlan_no_parent",                    \
	[GR_HIP_E_BOND_OUTPUT] = "bond_output",                                                    \
	[GR_HIP_E_VXLAN_OUTPUT] = "vxlan_output",                                                  \
	[GR_HIP_E_PORT_OUTPUT] = "port_output",                                                    \
	[GR_HIP_E_IP6_INPUT_LOCAL] = "ip6_input_local",                                            \
	[GR_HIP_E_IP6_ERROR_DEST_UNREACH] = "ip6_error_dest_unreach",                              \
	[GR_HIP_E_IP6_INPUT_NOT_MEMBER] = "ip6_input_not_member",                                  \
	[GR_HIP_E_IP6_INPUT_OTHER_HOST] = "ip6_input_other_host",                                  \
	[GR_HIP_E_IP6_INPUT_BAD_VERSION] = "ip6_input_bad_version",                                \
	[GR_HIP_E_IP6_INPUT_BAD_ADDR] = "ip6_input_bad_addr",                                      \
	[GR_HIP_E_IP6_INPUT_BAD_LENGTH] = "ip6_input_bad_length",                                  \
	[GR_HIP_E_IP6_BLACKHOLE] = "ip6_blackhole",                                                \
	[GR_HIP_E_SR6_LOCAL] = "sr6_local",                                                        \
	[GR_HIP_E_IP6_ERROR_TTL_EXCEEDED] = "ip6_error_ttl_exceeded",                              \
	[GR_HIP_E_IP6_HOLD] = "ip6_hold",                                                          \
	[GR_HIP_E_IP6_OUTPUT_ERROR] = "ip6_output_error",                                          \
	[GR_HIP_E_IP6_OUTPUT_TOO_BIG] = "ip6_output_too_big",


#define GPU_FWD4_MAX_DEVS 16

struct gpu_fwd4_conf {
	uint32_t n_devs; // GPUs the module opens, 0 = every visible device
	int devs[GPU_FWD4_MAX_DEVS]; // their HIP ordinals (the same one twice: two contexts)
	uint32_t max_ifaces; // gr_hip_init sizes (grout: gr_config)
	uint32_t max_nexthops;
	uint32_t batch; // packets accumulated before a GPU walk
	uint32_t rx_burst; // port_rx burst size: a shorter burst flushes
	uint64_t max_delay_ns; // a held packet never waits longer (flush node)
	uint32_t depth; // batches in flight per graph: 1 = each waited for, 2 = pipelined (0: 2)
};

// Before module init (grout: from its configuration). 0 or -EINVAL.
int gpu_fwd4_configure(const struct gpu_fwd4_conf *);
// Batches in flight per graph (1 or 2), at any time. 0 or -EINVAL.
int gpu_fwd4_set_depth(uint32_t depth);
// Measurement: nanoseconds the node spent, per phase, since the last call
// (then reset); on = 0 stops accumulating. out: GPU_FWD4_PROF_COUNT values.
enum {
	GPU_FWD4_PROF_ACCUMULATE, // process(): mbufs into the batch's gr_hip_mbuf views
	GPU_FWD4_PROF_START, // gr_hip_node_start: layout, staging, launch
	GPU_FWD4_PROF_FINISH, // gr_hip_node_finish: wait for the GPU, hand-back onto the views
	GPU_FWD4_PROF_DELIVER, // the views onto the rte_mbufs + private data, enqueues
	GPU_FWD4_PROF_COUNT,
};
void gpu_fwd4_prof(int on, uint64_t *out);
// The module's fast-path contexts, one per GPU (NULL before init or on
// failure); gpu_fwd4_hip_ctx() is the first.
gr_hip_ctx_t *gpu_fwd4_hip_ctx(void);
uint32_t gpu_fwd4_n_ctx(void);
gr_hip_ctx_t *gpu_fwd4_ctx_at(uint32_t i);
// The context index a worker graph runs on (-ENOENT: not a graph of ours).
int gpu_fwd4_graph_gpu(const struct rte_graph *);
// What rte_graph would have counted for the replaced nodes, and batches the
// GPU refused (punted whole to grout's CPU nodes). 0 or -ENOENT.
int gpu_fwd4_node_stats(const struct rte_graph *, struct gr_hip_node_stats *, uint64_t *gpu_errors);
// The per-iface rx/tx counters of the graph's queue (gr_hip_queue_stats).
int gpu_fwd4_queue_stats(const struct rte_graph *, struct gr_hip_iface_stats *, uint32_t max_ifaces, int reset);

// Control plane, replicated to every context: the gr_hip_* call of the same
// name on each GPU. 0, or the first -errno (the others are still updated).
int gpu_fwd4_iface_set(const struct gr_hip_iface *, uint32_t n);
int gpu_fwd4_iface_del(uint16_t iface_id);
int gpu_fwd4_nh_set(uint32_t first_slot, const struct gr_hip_nh *, uint32_t n);
int gpu_fwd4_reta_set(uint32_t first, const uint32_t *slots, uint32_t n);
int gpu_fwd4_fib4_create(uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8);
int gpu_fwd4_fib4_destroy(uint16_t vrf_id);
int gpu_fwd4_route4_add(const struct gr_hip_route4 *, uint32_t n, int replace);
int gpu_fwd4_route4_del(uint16_t vrf_id, uint32_t ip, uint8_t prefixlen);
int gpu_fwd4_fib4_commit(uint16_t vrf_id);
int gpu_fwd4_fib6_create(uint16_t vrf_id, uint32_t max_routes, uint32_t num_tbl8);
int gpu_fwd4_fib6_destroy(uint16_t vrf_id);
int gpu_fwd4_route6_add(const struct gr_hip_route6 *, uint32_t n, int replace);
int gpu_fwd4_route6_del(uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen);
int gpu_fwd4_fib6_commit(uint16_t vrf_id);
int gpu_fwd4_edges_set(int table, uint16_t key, uint8_t edge); // table: GR_HIP_EDGES_*
int gpu_fwd4_tune(const char *key, int value);
int gpu_fwd4_host_register(void *ptr, size_t bytes); // grout: each mempool's memory
int gpu_fwd4_host_unregister(void *ptr);

#ifdef __cplusplus
}
#endif
