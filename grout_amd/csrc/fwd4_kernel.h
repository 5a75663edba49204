// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_kernel.h -- device-side layout shared by the kernel and the C-ABI
// implementation (gr_hip.hip). Not a public header.
#pragma once

#include "../../include/grout_hip.h"

#include <stdint.h>

#define FWD4_BLOCK 256 // packets per tile = threads per block (4 waves)
#define FWD4_ROW 80 // LDS bytes per staged 64-byte line (+16: no bank conflicts)
#define FWD4_STAT_SLOTS 32 // per-block iface counter slots (LDS)
#define FWD4_STAT_SHARDS 64 // global counter shards (block % shards)
#define FWD4_MAX_ETH_TYPES 16

struct fwd4_fib { // one per VRF id
	const uint32_t *tbl24; // NULL: no FIB for this VRF
	const uint32_t *tbl8;
};

struct fwd4_edges {
	uint16_t eth_type_be[FWD4_MAX_ETH_TYPES]; // registered types (raw BE value)
	uint8_t eth_type_edge[FWD4_MAX_ETH_TYPES];
	uint8_t n_eth_types;
	uint8_t mode[GR_HIP_IFACE_MODE_COUNT]; // iface_input mode -> edge
	uint8_t in_nh[8]; // ip_input nh type -> edge (GR_HIP_EDGE_CHAIN = ip_forward)
	uint8_t out_nh[8]; // ip_output nh type -> edge (CHAIN = eth_output)
	uint8_t out_iface[8]; // ip_output iface type -> edge
	uint8_t iout_type[8]; // iface_output iface type -> edge
};

// Device-resident per-context tables (updated by the control plane under
// quiesce, read by every launch through one pointer: scalar loads).
struct fwd4_tables {
	const struct gr_hip_iface *ifaces;
	const struct gr_hip_nh *nh;
	const uint32_t *reta;
	const struct fwd4_fib *fibs;
	const uint32_t *vlan_keys; // (parent << 16 | vlan_id) + 1, 0 = empty
	const uint16_t *vlan_vals;
	uint32_t reta_cap;
	uint32_t vlan_mask; // capacity - 1
	uint32_t max_ifaces;
	uint32_t max_nh;
	struct fwd4_edges edges;
};

// Per-launch kernel arguments.
struct fwd4_params {
	const uint8_t *in;
	uint8_t *out;
	const struct gr_hip_pkt_meta *meta;
	struct gr_hip_verdict *verdicts;
	struct gr_hip_iface_stats *stats; // [FWD4_STAT_SHARDS][max_ifaces]
	const struct fwd4_tables *T;
	uint32_t n;
	uint32_t in_stride;
	uint32_t out_stride;
	uint32_t readable; // frame bytes present per packet (64 or in_stride)
};

// Kernel variants (gr_hip_tune "staging"): how header lines move between
// HBM and registers.
enum {
	FWD4_STAGE_LDS = 0, // coalesced 16 B/lane loads -> LDS -> per-lane rows
	FWD4_STAGE_DIRECT = 1, // each lane loads / stores its own 64 B line
};
