// SPDX-License-Identifier: BSD-3-Clause
//
// oracle.h -- TEST INFRASTRUCTURE ONLY. Not part of the product.
//
// A CPU restatement, in plain C, of grout's IPv4 forwarding node chain:
// iface_input -> eth_input -> ip_input (+ fib4_lookup) -> ip_forward ->
// ip_output -> eth_output -> iface_output, run through a minimal rte_graph-like
// burst walk (bursts of 64, modules/infra/control/graph.c:88-91). Every
// function in oracle.c cites the reference file:line it follows.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library, and only as the checker / CPU baseline. The product
// (grout_amd/) never links or calls it.
//
// Parity pinning: the reference cannot be built here (DPDK >= 25.11 is fetched
// over the network). The restatement is pinned by the
// known-answer cases of the reference's only hot-path unit test
// (modules/ip/datapath/ip_input.c:302-383, restated in tests/test_oracle_kat.py),
// by hand-derived cases of ip_forward's checksum arithmetic, and by a
// brute-force longest-prefix match cross-check of both of its LPMs. FIB parity
// against DPDK's rte_fib itself is therefore partial (no reference test pins it).
#pragma once

#include "../include/grout_hip.h"

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_topo or_topo_t;

or_topo_t *or_topo_new(uint32_t max_ifaces, uint32_t max_nexthops);
void or_topo_free(or_topo_t *);

// Same registration surface as grout (eth_input.c:26, ip_input.c:36, ...);
// or_topo_new() applies grout's default module set.
int or_edge_eth_type(or_topo_t *, uint16_t be_type, uint8_t edge);
int or_edge_iface_mode(or_topo_t *, uint8_t mode, uint8_t edge);
int or_edge_ip_input_nh_type(or_topo_t *, uint8_t nh_type, uint8_t edge);
int or_edge_ip_output_nh_type(or_topo_t *, uint8_t nh_type, uint8_t edge);
int or_edge_ip_output_iface_type(or_topo_t *, uint8_t iface_type, uint8_t edge);
int or_edge_iface_output_type(or_topo_t *, uint8_t iface_type, uint8_t edge);

int or_iface_set(or_topo_t *, const struct gr_hip_iface *, uint32_t n);
int or_nh_set(or_topo_t *, uint32_t first_slot, const struct gr_hip_nh *, uint32_t n);
int or_reta_set(or_topo_t *, uint32_t first, const uint32_t *slots, uint32_t n);

// RIB: per-VRF exact-prefix hash tables (one per prefix length).
int or_fib_create(or_topo_t *, uint16_t vrf_id, uint32_t num_tbl8);
int or_route_add(or_topo_t *, const struct gr_hip_route4 *, uint32_t n, int replace);
int or_route_del(or_topo_t *, uint16_t vrf_id, uint32_t ip_be, uint8_t prefixlen);
// Build the DIR24_8 restatement (DPDK lib/fib/dir24_8, 8-byte entries).
int or_fib_build(or_topo_t *, uint16_t vrf_id);

// IPv6 RIB (exact-prefix hash per length, link-local prefixes scoped to
// iface_id as addr6_linklocal_scope, modules/ip6/control/ip6.h:23-36).
int or_fib6_create(or_topo_t *, uint16_t vrf_id);
int or_route6_add(or_topo_t *, const struct gr_hip_route6 *, uint32_t n, int replace);
int or_route6_del(or_topo_t *, uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16], uint8_t prefixlen);
// IPv6 LPM (scoped): hash-per-length probe and brute force.
uint32_t or_lpm6(const or_topo_t *, uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16]);
uint32_t or_lpm6_brute(const or_topo_t *, uint16_t vrf_id, uint16_t iface_id, const uint8_t ip[16]);
int or_edge_ip6_input_nh_type(or_topo_t *, uint8_t nh_type, uint8_t edge);
int or_edge_ip6_output_nh_type(or_topo_t *, uint8_t nh_type, uint8_t edge);
int or_edge_ip6_output_iface_type(or_topo_t *, uint8_t iface_type, uint8_t edge);

// LPM: hash-per-length probe (truth) and DIR24_8 restatement. ip host order.
// Return the nexthop slot, 0 = no route.
uint32_t or_lpm_hash(const or_topo_t *, uint16_t vrf_id, uint32_t ip);
uint32_t or_lpm_dir24(const or_topo_t *, uint16_t vrf_id, uint32_t ip);
// Brute force over every installed route (small tables only).
uint32_t or_lpm_brute(const or_topo_t *, uint16_t vrf_id, uint32_t ip);

// Run n packets through the node chain. Same buffer contract as
// struct gr_hip_batch (grout_hip.h). stats: max_ifaces entries, accumulated.
// Graph walks as a batch defines them (GR_HIP_META_WALK): one starts at
// packet 0, at each multiple of 64 and at each marked packet.
// OR_F_MBUF_WALKS (a flags bit): walks as the rte_graph node cuts its mbufs
// instead (gr_hip_node_layout): at each marked packet and `burst` packets
// (OR_F_BURST below) after the previous start, wherever that falls.
#define OR_F_MBUF_WALKS 0x80000000u
// With OR_F_MBUF_WALKS: a walk is at most OR_F_BURST(b) packets (1..256,
// grout's rx_burst_max / vector_max, gr_infra.h:446-453, graph.c:612-650);
// 0 = 64, the default burst (graph.c:88-91).
#define OR_F_BURST_SHIFT 16
#define OR_F_BURST(b) ((uint32_t)((b) & 0x1ff) << OR_F_BURST_SHIFT)
int or_process(
	or_topo_t *,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *verdicts,
	struct gr_hip_iface_stats *stats,
	uint32_t flags
);

// or_process, plus the mbuf state grout leaves at each packet's edge (mo[n],
// frame NULL, data_off relative to an RX data_off of 128; a punted packet's
// mbuf is reported untouched) and the per-node counters of the walks (ns,
// accumulated; punted packets are not counted).
int or_process_ex(
	or_topo_t *,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *verdicts,
	struct gr_hip_iface_stats *stats,
	uint32_t flags,
	struct gr_hip_mbuf *mo,
	struct gr_hip_node_stats *ns
);

// One graph walk of the chain over n <= 256 packets whose frames lie in
// place (frames[i]: the Ethernet header, `readable` bytes), rewritten there
// as grout's nodes rewrite an mbuf's data. mo[i]: the mbuf state at the
// packet's edge (fields as or_process_ex; frame untouched). For the walk
// harness's CPU chain node (tests/standin/walk_harness.c). 0 or -EINVAL.
int or_walk_frames(const or_topo_t *, uint8_t *const *frames, uint32_t readable, const struct gr_hip_pkt_meta *meta,
		   uint16_t n, struct gr_hip_mbuf *mo);

// CPU baseline: `threads` pthreads, one per core, pinned.
// Worker i starts at packet i * n / threads of the sample and walks it in
// bursts of 64, wrapping. Each first makes its own copy of the IPv4 FIBs on
// transparent huge pages (OR_BENCH_FIB_COPY; else all share the topology's,
// as grout's workers share one rte_fib per VRF) and warms up with one
// untimed pass over the whole sample; then all start together and each
// processes pkts_per_thread packets (rounded up to bursts). Returns the
// aggregate Mpps over the timed part (CLOCK_MONOTONIC), -1 on error.
#define OR_BENCH_FIB_COPY 0x1
// or_bench_set_cpus: worker i of later or_bench runs pinned to cpus[i] (a
// placement, e.g. one core per L3 domain) instead of the i-th allowed CPU;
// n = 0 goes back to that. 0, or -1 when a CPU is out of range.
int or_bench_set_cpus(const int *cpus, int n);
double or_bench(
	or_topo_t *,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	int threads,
	uint64_t pkts_per_thread,
	uint32_t flags,
	uint64_t *forwarded
);

#ifdef __cplusplus
}
#endif
