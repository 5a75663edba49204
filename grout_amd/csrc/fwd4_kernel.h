// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_kernel.h -- device-side layout shared by the forwarding kernel
// (fwd4_ring.hip) and the C-ABI implementation (gr_hip.cpp). Not a public
// header.
#pragma once

#include "../../include/grout_hip.h"

#include <stdint.h>

#define FWD4_STAT_SLOTS 32 // per-block iface counter slots (LDS)
#define FWD4_STAT_SHARDS 64 // global counter shards (block % shards)
#define FWD4_MAX_ETH_TYPES 16

struct fwd4_edges {
	uint16_t eth_type_be[FWD4_MAX_ETH_TYPES]; // registered types (raw BE value)
	uint8_t eth_type_edge[FWD4_MAX_ETH_TYPES];
	uint8_t n_eth_types;
	uint8_t mode[GR_HIP_IFACE_MODE_COUNT]; // iface_input mode -> edge
	uint8_t in_nh[8]; // ip_input nh type -> edge (GR_HIP_EDGE_CHAIN = ip_forward)
	uint8_t out_nh[8]; // ip_output nh type -> edge (CHAIN = eth_output)
	uint8_t out_iface[8]; // ip_output iface type -> edge
	uint8_t iout_type[8]; // iface_output iface type -> edge
	uint8_t in6_nh[8]; // ip6_input nh type -> edge (CHAIN = ip6_forward)
	uint8_t out6_nh[8]; // ip6_output nh type -> edge (CHAIN = eth_output)
	uint8_t out6_iface[8]; // ip6_output iface type -> edge
};

// Per-iface RX view, 32 bytes: what iface_input and eth_input need from an
// ingress iface, and the FIB of its VRF (get_fib, modules/ip/control/route.c:51-61), resolved
// by the control plane when ifaces, VRFs or edge registrations change.
#define FWD4_RX_MAC_OK 0x01 // iface_get_eth_addr() succeeds
#define FWD4_RX_SNAT_DYN 0x02 // GR_IFACE_F_SNAT_DYNAMIC
#define FWD4_RX_VLAN_DEMUX 0x04 // mode VRF: tagged packets look up a sub-iface
#define FWD4_RX_FIB16 0x08 // DIR-16-8-8 FIB: tbl24 points at top[65536] (u32,
                           // bit31 = chunk) followed by 2-byte /24 chunks;
                           // tbl8 has 2-byte entries (bit15 = tbl8 group)
#define FWD4_RX_FIB24W2 0x10 // DIR24_8 with 2-byte entries: tbl24 points at
                             // u16[2^24] (bit15 = tbl8 group), tbl8 as FIB16
struct fwd4_rx {
	uint16_t id; // 0: no such iface
	uint8_t e_in; // iface_input edge: ADMIN_DOWN, mode edge or CHAIN (eth_input)
	uint8_t flags; // FWD4_RX_*
	uint8_t mac[6];
	uint8_t _pad[6];
	const uint32_t *tbl24; // NULL: no FIB (no route)
	const uint32_t *tbl8;
};

// Per-iface IPv6 view, 16 bytes: the FIB6 of the iface's VRF (get_fib6,
// modules/ip6/control/route.c:54-64). NULL: no IPv6 FIB (no route).
struct fwd4_rx6 {
	const uint32_t *top; // [65536] (fib6.h encoding)
	const uint32_t *groups; // [n][256]
	const uint4 *skips; // struct gr_fib6_skip [n]
};

// Per-nexthop adjacency, 64 bytes: the nexthop fields ip_input reads plus
// the outcome of ip_output -> eth_output -> iface_output for that nexthop,
// precomputed from the iface mirror (everything but the packet-dependent
// MTU/DF and LINK destination checks). Recomputed on nexthop, iface and
// edge-registration changes.
#define FWD4_ADJ_LOCAL 0x01 // L3 nexthop flagged LOCAL (ip_input.c:166-168)
#define FWD4_ADJ_LINK 0x02 // flagged LINK (ip_output.c:126-127)
struct fwd4_adj {
	uint8_t type; // GR_HIP_NH_T_*
	uint8_t e_in; // ip_input nh type edge (CHAIN = ip_forward)
	uint8_t flags; // FWD4_ADJ_*
	uint8_t e_pre; // ip_output before the MTU check (nh type edge, ERROR) or CHAIN
	uint8_t e_mid; // after it: SNAT, iface type edge, HOLD (state) or CHAIN
	uint8_t e_post; // eth_output / iface_output outcome
	uint16_t oif; // mbuf_data(m)->iface set by ip_output
	uint16_t mtu; // of oif
	uint16_t post_iface; // priv iface at e_post
	uint32_t ipv4; // network order
	uint16_t tx_if, tx_par; // iface_output counter keys (0 = not counted)
	uint8_t dmac[6]; // nexthop MAC
	uint8_t smac[6]; // oif MAC
	uint16_t n_members; // GROUP
	uint16_t reta_size;
	uint32_t reta_off;
	uint32_t single;
	uint32_t _pad[5];
};

// Per-nexthop IPv6 adjacency, 64 bytes: fwd4_adj for the ip6_input /
// ip6_output edge tables (ip6_input.c:133-144, ip6_output.c:75-134). e_pre
// is the nh type edge or ERROR (before the MTU check, iface = ingress),
// e_mid the iface type edge or HOLD by state (after it, iface = oif).
struct fwd4_adj6 {
	uint8_t type;
	uint8_t e_in;
	uint8_t flags; // FWD4_ADJ_LOCAL / FWD4_ADJ_LINK
	uint8_t e_pre;
	uint8_t e_mid;
	uint8_t e_post;
	uint16_t oif;
	uint16_t mtu;
	uint16_t post_iface;
	uint16_t tx_if, tx_par;
	uint8_t dmac[6];
	uint8_t smac[6];
	uint8_t ipv6[16];
	uint32_t _pad[5];
};

// Fast adjacency, 16 bytes: a nexthop whose packets take the plain forward
// (L3, no LOCAL/LINK flag, ip_output/eth_output/iface_output all chain to
// port_output of a port oif: post_iface = tx iface = oif, no parent) needs
// only its MACs, oif and MTU. mtu == 0: not plain, read the fwd4_adj. The
// IPv6 chain has its own table (nhf6, plain by fwd4_adj6's edges).
struct fwd4_nhf {
	uint8_t dmac[6];
	uint16_t oif;
	uint8_t smac[6];
	uint16_t mtu;
};

// Device-resident per-context tables (updated by the control plane under
// quiesce, read by every launch through one pointer).
struct fwd4_tables {
	const struct fwd4_rx *rx; // [max_ifaces]
	const struct fwd4_adj *adj; // [max_nh + 1]
	const struct fwd4_nhf *nhf; // [max_nh + 1]
	const struct fwd4_rx6 *rx6; // [max_ifaces]
	const struct fwd4_adj6 *adj6; // [max_nh + 1]
	const struct fwd4_nhf *nhf6; // [max_nh + 1] fast adjacencies of the IPv6 chain
	const uint32_t *reta;
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
	uint32_t nhf_lds; // fwd4_ring.hip: fast adjacencies 1..nhf_lds staged in LDS
	uint32_t nhf6_lds; // and IPv6 fast adjacencies 1..nhf6_lds after them
	// and the first-level FIB6 entries [FWD4_TOP6_BASE, FWD4_TOP6_BASE + top6_lds)
	// of top6 (4 bytes each) after those: the trie of the only VRF with IPv6
	// routes (NULL, 0: none staged)
	const uint32_t *top6;
	uint32_t top6_lds;
	uint32_t chunk; // fwd4_ring.hip: 0 = workgroup b takes tiles b, b + G, ...;
	                // else the contiguous tiles [b * chunk, (b + 1) * chunk)
	uint32_t order; // 2: XCD x (= b % 8) takes region [x * chunk, (x + 1) * chunk),
	                // its workgroups interleaved in it (grid % 8 == 0);
	                // 3: runs of `chunk` tiles, run j of workgroup b = run j * G + b
	uint32_t spin_max; // polls before a ring wait gives up (0 = RING_SPIN_MAX)
	uint32_t *err; // set to 1 when a workgroup gave up (host-mapped; may be NULL)
	// the resident kernel (gr_fwd4_resident): the workgroup's index and count in
	// the tile order (wgs 0: blockIdx / gridDim), and whether `in` holds frame
	// addresses (GR_HIP_BATCH_F_FRAME_PTRS)
	uint32_t wg0, wgs;
	uint32_t ptrs;
	uint32_t _pad;
};

// The resident kernel's batches: ring r of a context holds `ndesc`
// descriptors in pinned host memory; the host writes A, then `seq` (release);
// the kernel's workgroup r takes them in seq order (1, 2, ...), runs each,
// and stores its seq into done[r * stride] (release, system scope). A batch
// split over k rings of a queue is posted to its helpers (rings r+1 .. r+k-1)
// first, then to its first ring r, whose descriptor names the helpers' seqs:
// the first ring's workgroup wakes them through device memory (wake[]), so
// that only first rings poll host memory.
struct __attribute__((aligned(64))) fwd4_res_desc {
	uint64_t seq;
	uint64_t helper_seq[7]; // first ring: the seq of this batch on ring r + 1 + j, j < A.wgs - 1
	struct fwd4_params A;
};

struct fwd4_res_params {
	struct fwd4_res_desc *descs; // [rings][ndesc], host memory
	uint64_t *done; // [rings * stride], host memory
	uint64_t *exited; // [rings * stride], host memory: launch_id once ring r's workgroup has left
	uint32_t *stop; // host memory: nonzero = every workgroup leaves after its batch
	uint64_t *wake; // [rings * stride], device memory: the last helper seq a first ring woke ring r for
	uint64_t *active; // device memory: s_memrealtime when a workgroup last finished a batch
	const uint32_t *taken; // host memory [rings]: 0 = no queue holds ring r (its workgroup leaves at
	                       // once), 1 = a queue's first ring, 2 = one of its helpers (polls backed off)
	uint64_t lifetime; // s_memrealtime ticks (100 MHz): a first ring idle past it, with no batch
	                   // finished anywhere for as long (*active), sets *stop
	uint64_t launch_id;
	uint32_t ndesc;
	uint32_t stride; // uint64_t per ring in done / exited
	uint32_t nap_max; // helper rings' idle polls (device memory) back off up to this many s_sleep(8)
	uint32_t _pad;
};

// First-level FIB6 entries a launch may stage in LDS: 2000::/4 (index =
// address bytes 0-1), where every global unicast allocation lies today.
#define FWD4_TOP6_BASE 0x2000u
#define FWD4_TOP6_MAX 4096u

// Kernel variants (bit mask, gr_hip_tune): counters, nontemporal loads and
// stores of the streamed data.
#define FWD4_V_STATS 0x1
#define FWD4_V_NT 0x2 // nontemporal loads and stores of the streamed data
#define FWD4_V_PTRS 0x4 // A.in is an array of frame addresses (GR_HIP_BATCH_F_FRAME_PTRS)
