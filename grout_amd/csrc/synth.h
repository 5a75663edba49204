// SPDX-License-Identifier: BSD-3-Clause
//
// synth.h -- deterministic synthetic inputs: the full-view
// route set of grout's smoke/fib_inject.c and 64 B / IMIX IPv4 UDP streams.
// A tool like fib_inject, not part of the forwarding path.
#pragma once

#include "../../include/grout_hip.h"

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint64_t gr_synth_splitmix64(uint64_t *state);

// fib_inject -4 -n count (smoke/fib_inject.c:23-34,53-79,107-134): prefix
// length picked round-robin from the BGP distribution by route index % 1000,
// ip = (per-length seq + 1) << (32 - len), nexthop = (i % n_nh) + 1, here
// mapped to slot nh_base + (i % n_nh).
int gr_synth_fullview_routes(
	uint32_t count,
	uint16_t vrf_id,
	uint32_t nh_base,
	uint32_t n_nh,
	struct gr_hip_route4 *out
);

// fib_inject -6 -n count (smoke/fib_inject.c:38-47,53-79,136-179): the IPv6
// full view of smoke/fib6_fullview_manualtest.sh (200,000 routes), route i
// -> nexthop nh_base + i % n_nh.
int gr_synth_fullview6_routes(
	uint32_t count,
	uint16_t vrf_id,
	uint32_t nh_base,
	uint32_t n_nh,
	struct gr_hip_route6 *out
);

enum {
	GR_SYNTH_DST_RANGE = 0, // dst uniform in [dst_lo, dst_hi] (host order)
	GR_SYNTH_DST_ROUTES = 1, // pick a route uniformly, random host bits
};
enum {
	GR_SYNTH_SIZE_64 = 0, // 60 bytes in buffer (64 on the wire with FCS)
	GR_SYNTH_SIZE_IMIX = 1, // 60 / 566 / 1514 in buffer, 7:4:1
};

struct gr_synth_stream {
	uint64_t seed;
	uint32_t dst_mode;
	uint32_t size_mode;
	uint32_t dst_lo, dst_hi; // DST_RANGE
	const struct gr_hip_route4 *routes; // DST_ROUTES
	uint32_t n_routes;
	uint16_t in_iface;
	uint8_t dst_mac[6]; // the RX port MAC
	uint8_t src_mac[6];
	uint8_t ttl;
	uint8_t _pad;
};

// Fill n frames (frames + i * stride, each slot zeroed first up to
// min(stride, frame length)) and their metadata. stride must be >= 64 and
// >= 1514 for IMIX unless lines_only (then only the first 64 bytes of each
// frame are written). Returns 0 or -EINVAL.
int gr_synth_packets(
	const struct gr_synth_stream *,
	uint32_t n,
	uint32_t stride,
	int lines_only,
	void *frames,
	struct gr_hip_pkt_meta *meta
);

// IPv4 header checksum as a sender computes it (RFC 791): returns the value
// to store in network order at bytes 10-11 of the header.
uint16_t gr_synth_ip4_cksum(const uint8_t *ip, uint32_t hl);

#ifdef __cplusplus
}
#endif
