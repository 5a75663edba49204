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
struct iface;
struct nexthop;

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
#define GPU_FWD4_MAX_GRAPHS 64 // worker graphs (one per worker, worker.c)

// Largest batch a graph accumulates. The node hands at most one batch back
// per process() call (the node's, and its flush source node's), so one graph
// walk enqueues at most 2 x GPU_FWD4_BATCH_MAX mbufs plus a few bursts of
// punts on any one edge (every batch the graph holds, GR_HIP_NODE_DEPTH of
// them, only on the way out: a drain leaving the graph, a GPU marked
// diverged): under rte_graph's limit of what a node stream can
// hold (struct rte_node size / idx are uint16_t, DPDK
// __rte_node_stream_alloc_size verifies the size), with room to spare.
// Batches of 16k packets forward as fast as 64k ones.
#define GPU_FWD4_BATCH_MAX 15360

// QSBR readers of the node (see gpu_fwd4_node.c, "RCU"): each graph holds
// GPU_FWD4_RCU_PER_GRAPH reader ids, above the workers' lcore ids. The module
// asks for GPU_FWD4_RCU_READERS of them through its datapath hooks, and grout's
// rcu module sizes its QSBR variable for them
// (integration/grout-gpu_fwd4-datapath.patch).
#define GPU_FWD4_RCU_PER_GRAPH 8 // 2 x GR_HIP_NODE_DEPTH: batches held, batches handed back in a walk
#define GPU_FWD4_RCU_READERS (GPU_FWD4_MAX_GRAPHS * GPU_FWD4_RCU_PER_GRAPH)

struct gpu_fwd4_conf {
	uint32_t n_devs; // GPUs the module opens, 0 = every visible device
	int devs[GPU_FWD4_MAX_DEVS]; // their HIP ordinals (the same one twice: two contexts)
	uint32_t max_ifaces; // gr_hip_init sizes (grout: gr_config)
	uint32_t max_nexthops;
	uint32_t batch; // packets accumulated before a GPU walk (at most GPU_FWD4_BATCH_MAX)
	uint32_t rx_burst; // port_rx burst size (1..256): a shorter burst flushes
	uint64_t max_delay_ns; // a held packet never waits longer (flush node)
	// batches in flight per graph (1 .. GR_HIP_NODE_DEPTH): 1 = each waited
	// for, 2 = one on the GPU while the next accumulates, d = d - 1 on the
	// GPU while the next accumulates; 0 (the default): 2, and
	// GR_HIP_NODE_DEPTH under a latency budget of 75 us or less
	uint32_t depth;
	// 0 (the default): each GPU's batches go to its resident kernel (gr_hip
	// knob "resident": descriptor rings, no launch per batch); 1: one launch
	// per batch
	uint32_t launch_per_batch;
	// 0 (the default): batches of `batch` packets, held `max_delay_ns` at
	// most. Otherwise a latency budget for a packet from its arrival at the
	// node to its hand-back onto its edge: each graph sizes its batches so
	// that its batches' oldest packets come back within it (a batch cap that
	// follows the moving average of those times: an eighth down while it is
	// above 17/20 of the budget, an eighth up while below 13/20 of it), and
	// holds a packet at most the budget less the GPU's measured round trip
	// (a quarter of the budget at least)
	uint64_t latency_budget_ns;
};

// Before module init (grout: from its configuration). A batch above
// GPU_FWD4_BATCH_MAX is clamped to it. 0 or -EINVAL.
int gpu_fwd4_configure(const struct gpu_fwd4_conf *);
// The configuration in effect (batch clamped).
void gpu_fwd4_conf_get(struct gpu_fwd4_conf *);
// Batches in flight per graph (1 .. GR_HIP_NODE_DEPTH; 0: from the latency
// budget, gpu_fwd4_conf.depth), at any time. 0 or -EINVAL.
int gpu_fwd4_set_depth(uint32_t depth);
// 1: one launch per batch; 0: batches posted to the resident kernel (the
// default, gpu_fwd4_conf.launch_per_batch), on every GPU from the next batch
int gpu_fwd4_set_launch_per_batch(int on);
// Batch size and maximum hold time at any time (the next batch of each graph
// takes them; the batch is clamped to GPU_FWD4_BATCH_MAX). 0 or -EINVAL.
int gpu_fwd4_set_batch(uint32_t batch, uint64_t max_delay_ns);
// The latency budget (gpu_fwd4_conf.latency_budget_ns; 0: off), at any time.
int gpu_fwd4_set_latency_budget(uint64_t budget_ns);
// The RX burst (grout's rx_burst_max, graph.c:612-650: 1..256): a shorter
// burst means the RX queue drained, and the node flushes. 0 or -EINVAL.
int gpu_fwd4_set_rx_burst(uint32_t rx_burst);
// Measurement: nanoseconds the node spent, per phase, since the last call
// (then reset); on = 0 stops accumulating. out: GPU_FWD4_PROF_COUNT values.
enum {
	GPU_FWD4_PROF_ACCUMULATE, // process(): mbufs into the batch's gr_hip_mbuf views, staged (gr_hip_node_append)
	GPU_FWD4_PROF_START, // gr_hip_node_send: launch
	GPU_FWD4_PROF_FINISH, // gr_hip_node_finish: wait for the GPU, hand-back onto the views
	GPU_FWD4_PROF_DELIVER, // the views onto the rte_mbufs + private data, enqueues
	GPU_FWD4_PROF_POLL, // the completion poll of the oldest batch on the GPU (gr_hip_node_pending)
	GPU_FWD4_PROF_FLUSH_NODE, // the flush source node's whole call (its hand-backs and flushes included)
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
// The per-iface rx/tx counters of the graph's hand-backs not yet folded into
// grout's iface_stats by gpu_fwd4_stats_flush (gr_hip_node_iface_stats).
int gpu_fwd4_queue_stats(const struct rte_graph *, struct gr_hip_iface_stats *, uint32_t max_ifaces, int reset);

// grout's housekeeping tick (gr_datapath_loop, main_loop.c:461-475, through
// the stats_flush hook integration/grout-gpu_fwd4-datapath.patch adds, which
// the module registers): fold what the fast path
// counted for this worker's graph since the last tick into grout's own
// statistics, so that `grcli stats` and `grcli interface stats` read as with
// grout's CPU nodes:
//   * per replaced node (eth_input, ip_input, ip_forward, ip_output,
//     eth_output, iface_output, ip6_input, ip6_forward, ip6_output; the
//     node itself runs as "iface_input" and rte_graph counts it):
//     cb(cookie, node id, packets, calls) with what rte_graph would have
//     counted (process() returns, ip_output's rule; one call per graph walk
//     reaching the node), which the patch adds into the worker's
//     node_stats as node_stats_callback does (main_loop.c:40-66);
//   * per iface: rx / tx packets and bytes added into
//     iface_get_stats(lcore_id, iface) (iface.h:115-118), as
//     IFACE_STATS_FLUSH does (rxtx.h:107-117).
// Returns the packets reported to cb, or -ENOENT.
typedef void (*gpu_fwd4_node_stat_cb)(void *cookie, uint32_t node_id, uint64_t packets, uint64_t calls);
int gpu_fwd4_stats_flush(const struct rte_graph *, unsigned lcore_id, gpu_fwd4_node_stat_cb cb, void *cookie);

// The worker leaves its graph (reconfiguration or shutdown): before it does,
// grout's gr_datapath_loop calls this on the graph (the graph_leave hook the
// module registers, main_loop.c:466-470 with
// integration/grout-gpu_fwd4-datapath.patch). The node holds up to two
// batches across graph walks, grout nothing: walks of the graph hand them
// back through grout's nodes (the batches on the GPU waited for, the held one
// sent at once), bounded by batches handed back (those held at the start +
// 2, or gpu_fwd4_set_drain_bound's); past the bound the held mbufs,
// and those RX brings in the last walk, go to grout's CPU nodes (PUNT). The
// node then holds nothing and its QSBR readers are offline. Returns the mbufs
// sent to grout's CPU nodes that way (0 normally), or -ENOENT for a graph
// without the node.
int gpu_fwd4_drain(struct rte_graph *);
// Batches a drain may hand back before it sends the rest to grout's CPU
// nodes: -1 (the default) = those held when it starts + 2; tests set 0 to
// take that way at once. 0.
int gpu_fwd4_set_drain_bound(int32_t batches);
// grout's housekeeping tick asks every datapath hook what it holds (the
// holding hook integration/grout-gpu_fwd4-datapath.patch adds): the mbufs the
// node holds in `graph` (accumulating, and the batches on the GPU) plus its
// QSBR readers still online (they go offline at the next walk). While it is
// not 0, grout's worker neither micro-sleeps nor blocks on its RX interrupts
// (main_loop.c:478-508): the flush node's walks hand the batches back, and
// the readers go offline, before the worker idles. 0 for another graph.
uint64_t gpu_fwd4_holding(const struct rte_graph *);
// mbufs freed by the node's fini because a graph was destroyed while it held
// them (not drained first): counted, never silently.
uint64_t gpu_fwd4_fini_freed(void);

// Per-graph walk state, for tests and measurements.
struct gpu_fwd4_walk_info {
	uint32_t held; // mbufs accumulating
	uint32_t in_flight; // batches started and not handed back
	uint64_t batches; // batches started
	uint64_t max_batch; // largest batch started
	uint64_t stale; // packets whose iface / nexthop was gone at hand-back (dropped)
	uint32_t readers_online; // the graph's QSBR readers online
	int diverged; // its GPU's mirrors are out of step: everything goes to grout's CPU nodes
	uint64_t append_errors; // graph walks that could not be staged, punted to grout's CPU nodes
	uint64_t handed; // batches handed back onto their edges
	uint64_t drain_punted; // mbufs drains sent to grout's CPU nodes (DRAIN_LEAVE)
	uint64_t stranded; // mbufs of batches the GPU would not let go of (never handed on)
	uint32_t batch_cap; // the batch size in effect (latency budget: the graph's cap)
	uint64_t lat_ns; // moving average of the batches' oldest packet, arrival to hand-back
	uint64_t over_budget; // batches whose oldest packet came back past the latency budget
	uint32_t depth; // the depth in effect (gpu_fwd4_conf.depth, or the one the budget picked)
};
int gpu_fwd4_walk_info(const struct rte_graph *, struct gpu_fwd4_walk_info *);
// Tests only: 0 = the node takes no QSBR reader (round 2's behaviour, to
// show the RCU test fails without them); 1 = default.
void gpu_fwd4_rcu_readers(int on);

// The grout objects a verdict names, by id / nexthop slot, as the node hands
// packets back (iface in mbuf_data, l3_mbuf_data.nh). Set them from the
// control plane's object events (GR_EVENT_IFACE_POST_ADD, NEXTHOP_NEW) and
// clear them (NULL) only from the events grout pushes after its
// rte_rcu_qsbr_synchronize (GR_EVENT_IFACE_REMOVE, iface.c:710-719;
// GR_EVENT_NEXTHOP_DELETE, nexthop.c:505-514): grout itself clears
// ifaces[id] before it synchronises, and a batch still on the GPU may name
// the object. 0 or -EINVAL / -ENOMEM.
int gpu_fwd4_iface_obj_set(uint16_t iface_id, const struct iface *);
int gpu_fwd4_nh_obj_set(uint32_t slot, const struct nexthop *);
const struct iface *gpu_fwd4_iface_obj(uint16_t iface_id);
const struct nexthop *gpu_fwd4_nh_obj(uint32_t slot);

// Control plane, replicated to every context: the gr_hip_* call of the same
// name on each GPU. 0, or the first -errno (the others are still updated).
// A context on which a call fails while it succeeds on another (or fails
// differently) no longer holds the same state: it is marked diverged, and
// the graphs bound to it hand every packet to grout's CPU nodes (PUNT)
// until the control plane has replayed its state into that context and
// calls gpu_fwd4_resync(i).
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
// 1 if context i is diverged, 0 if not, -ENOENT.
int gpu_fwd4_diverged(uint32_t i);
// Context i holds the control plane's state again (replayed with the
// gr_hip_* calls on gpu_fwd4_ctx_at(i)): its graphs use the GPU again.
int gpu_fwd4_resync(uint32_t i);

#ifdef __cplusplus
}
#endif
