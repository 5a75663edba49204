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

struct gpu_fwd4_conf {
	int dev; // HIP device of this process
	uint32_t max_ifaces; // gr_hip_init sizes (grout: gr_config)
	uint32_t max_nexthops;
	uint32_t batch; // packets accumulated before a GPU walk
	uint32_t rx_burst; // port_rx burst size: a shorter burst flushes
	uint64_t max_delay_ns; // a held packet never waits longer (flush node)
};

// Before module init (grout: from its configuration). 0 or -EINVAL.
int gpu_fwd4_configure(const struct gpu_fwd4_conf *);
// The fast-path context of the module (NULL before init or on failure).
gr_hip_ctx_t *gpu_fwd4_hip_ctx(void);
// What rte_graph would have counted for the replaced nodes, and batches the
// GPU refused (punted whole to grout's CPU nodes). 0 or -ENOENT.
int gpu_fwd4_node_stats(const struct rte_graph *, struct gr_hip_node_stats *, uint64_t *gpu_errors);
// The per-iface rx/tx counters of the graph's queue (gr_hip_queue_stats).
int gpu_fwd4_queue_stats(const struct rte_graph *, struct gr_hip_iface_stats *, uint32_t max_ifaces, int reset);

#ifdef __cplusplus
}
#endif
