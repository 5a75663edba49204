// SPDX-License-Identifier: BSD-3-Clause
//
// gr_node_priv.h -- what gr_hip.cpp and gr_node.cpp share beyond the C ABI:
// the node's staging continued across appends, and its hand-back with the
// context's VLAN table and per-iface counters.
#pragma once

#include "../../include/grout_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

// Host image of the context's VLAN sub-interface table (open addressing,
// key ((parent << 16) | vlan_id) + 1, 0 = empty), the one the kernel probes.
struct gr_node_vlans {
	const uint32_t *keys;
	const uint16_t *vals;
	uint32_t cap; // power of two, or 0
};

// gr_hip_node_layout continuing at slot p (m[0] starts a walk); returns the
// first slot past the walks.
uint64_t gr_node_layout_from(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, uint64_t p, uint32_t *pos);
// gr_hip_node_stage continuing at slot `next` (the first one not yet
// written: pad slots from there up to pos[0] are zeroed).
int gr_node_stage_from(const struct gr_hip_mbuf *m, uint32_t n, uint32_t burst, const uint32_t *pos, uint32_t next,
		       void *lines, struct gr_hip_pkt_meta *meta);

// Where a walk of n mbufs appended at slot p ends (cut every `burst`).
uint64_t gr_node_walk_end(uint64_t p, uint32_t n, uint32_t burst);
// gr_hip_node_append_mbufs' pass: slots pos[], lines and metadata of one
// walk's mbufs from slot p on; returns the first slot past the walk.
uint64_t gr_node_stage_mbufs(void *const *mbufs, uint32_t n, const struct gr_hip_mbuf_layout *lay, uint32_t burst,
			     uint64_t p, uint32_t *pos, void *lines, struct gr_hip_pkt_meta *meta);
// rte_pktmbuf_mtod of an mbuf, through the layout.
void *gr_node_frame(const void *mbuf, const struct gr_hip_mbuf_layout *lay);

// The hand-back straight onto the caller's mbufs (gr_hip_node_finish_mbufs):
// the views are read, not written; edges[i] and *stale are the outputs.
// meta non-NULL: no views (the walk was appended from the mbufs): each
// packet's view is read from its mbuf through lay before the hand-back
// writes it, with its iface id and walk start from meta[pos[i]].
struct gr_node_direct {
	void *const *mbufs;
	const struct gr_hip_mbuf_layout *lay;
	uint8_t *edges;
	uint32_t stale;
	const struct gr_hip_pkt_meta *meta;
};

// gr_hip_node_apply, also adding each packet's rx / tx to ifst[iface id]
// (n_ifst entries) where grout's iface_input / iface_output count them;
// direct (optional): onto the mbufs instead of the views.
int gr_node_apply_ex(
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
);

#ifdef __cplusplus
}
#endif
