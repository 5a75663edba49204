// SPDX-License-Identifier: BSD-3-Clause
//
// synth.c -- deterministic synthetic route sets and packet streams.
#include "synth.h"

#include <errno.h>
#include <string.h>

uint64_t gr_synth_splitmix64(uint64_t *s) {
	uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

// ipv4_dist, smoke/fib_inject.c:23-34 (parts per thousand)
static const struct {
	uint8_t len;
	uint16_t weight;
} dist4[] = {
	{16, 14}, {17, 8}, {18, 14}, {19, 25}, {20, 45},
	{21, 51}, {22, 109}, {23, 106}, {24, 620}, {32, 8},
};
#define N_DIST4 (sizeof(dist4) / sizeof(dist4[0]))

int gr_synth_fullview_routes(
	uint32_t count,
	uint16_t vrf_id,
	uint32_t nh_base,
	uint32_t n_nh,
	struct gr_hip_route4 *out
) {
	if (n_nh == 0 || nh_base == 0)
		return -EINVAL;
	uint32_t seq[N_DIST4] = {0};
	for (uint32_t i = 0; i < count; i++) {
		// pick_prefix, fib_inject.c:53-79
		uint32_t slot = i % 1000, cum = 0;
		unsigned b = N_DIST4 - 1;
		for (unsigned k = 0; k < N_DIST4; k++) {
			cum += dist4[k].weight;
			if (slot < cum) {
				b = k;
				break;
			}
		}
		uint8_t len = dist4[b].len;
		uint32_t s = seq[b]++;
		uint32_t ip = (s + 1) << (32 - len); // fib_inject.c:122
		out[i].ip = __builtin_bswap32(ip);
		out[i].prefixlen = len;
		out[i]._pad0 = 0;
		out[i].vrf_id = vrf_id;
		out[i].nh = nh_base + (i % n_nh); // fib_inject.c:125
	}
	return 0;
}

// ipv6_dist, smoke/fib_inject.c:38-47 (parts per thousand, in table order:
// the bucket index also picks the route's /8 base)
static const struct {
	uint8_t len;
	uint16_t weight;
} dist6[] = {
	{32, 130}, {36, 40}, {40, 95}, {44, 105}, {48, 500}, {128, 10}, {46, 50}, {42, 40}, {38, 30},
};
#define N_DIST6 (sizeof(dist6) / sizeof(dist6[0]))

// fib_inject -6 -n count (inject_ipv6, fib_inject.c:136-179): route i takes
// the bucket pick_prefix gives index i (round robin over i % 1000), the /8
// base 0x20 + bucket, and its per-bucket sequence number + 1 placed after
// the /8 as the reference computes it.
int gr_synth_fullview6_routes(
	uint32_t count,
	uint16_t vrf_id,
	uint32_t nh_base,
	uint32_t n_nh,
	struct gr_hip_route6 *out
) {
	if (n_nh == 0 || nh_base == 0)
		return -EINVAL;
	uint32_t seq[N_DIST6] = {0};
	for (uint32_t i = 0; i < count; i++) {
		uint32_t slot = i % 1000, cum = 0; // pick_prefix, fib_inject.c:53-79
		unsigned b = N_DIST6 - 1;
		for (unsigned k = 0; k < N_DIST6; k++) {
			cum += dist6[k].weight;
			if (slot < cum) {
				b = k;
				break;
			}
		}
		const uint8_t len = dist6[b].len;
		const uint32_t v = seq[b]++ + 1; // fib_inject.c:145,159
		struct gr_hip_route6 *r = &out[i];
		memset(r, 0, sizeof(*r));
		r->ip[0] = (uint8_t)(0x20 + b); // :152-153
		const unsigned net_bits = len > 8 ? len - 8u : 1u; // :160
		const unsigned bit_offset = net_bits > 32 ? net_bits - 32 : 0; // :163
		const uint32_t shifted = v << (32 - net_bits + bit_offset); // :164
		const unsigned start = bit_offset / 8; // :165
		r->ip[1 + start] = (uint8_t)(shifted >> 24); // :166-169
		r->ip[2 + start] = (uint8_t)(shifted >> 16);
		r->ip[3 + start] = (uint8_t)(shifted >> 8);
		r->ip[4 + start] = (uint8_t)shifted;
		r->prefixlen = len;
		r->vrf_id = vrf_id;
		r->nh = nh_base + (i % n_nh); // :170
	}
	return 0;
}

uint16_t gr_synth_ip4_cksum(const uint8_t *ip, uint32_t hl) {
	uint32_t sum = 0;
	for (uint32_t i = 0; i < hl; i += 2) {
		if (i == 10)
			continue;
		sum += (uint32_t)((ip[i] << 8) | ip[i + 1]);
	}
	while (sum >> 16)
		sum = (sum & 0xffff) + (sum >> 16);
	return (uint16_t)~sum;
}

static void put16(uint8_t *p, uint16_t v) {
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}

static void put32(uint8_t *p, uint32_t v) {
	p[0] = (uint8_t)(v >> 24);
	p[1] = (uint8_t)(v >> 16);
	p[2] = (uint8_t)(v >> 8);
	p[3] = (uint8_t)v;
}

int gr_synth_packets(
	const struct gr_synth_stream *c,
	uint32_t n,
	uint32_t stride,
	int lines_only,
	void *frames,
	struct gr_hip_pkt_meta *meta
) {
	if (stride < GR_HIP_LINE)
		return -EINVAL;
	if (c->size_mode == GR_SYNTH_SIZE_IMIX && !lines_only && stride < 1514)
		return -EINVAL;
	if (c->dst_mode == GR_SYNTH_DST_ROUTES && (c->routes == NULL || c->n_routes == 0))
		return -EINVAL;
	if (c->dst_mode == GR_SYNTH_DST_RANGE && c->dst_hi < c->dst_lo)
		return -EINVAL;
	uint64_t st = c->seed;
	uint8_t *base = frames;
	for (uint32_t i = 0; i < n; i++) {
		uint64_t x0 = gr_synth_splitmix64(&st);
		uint64_t x1 = gr_synth_splitmix64(&st);
		uint64_t x2 = gr_synth_splitmix64(&st);
		uint64_t x3 = gr_synth_splitmix64(&st);
		uint32_t dst;
		if (c->dst_mode == GR_SYNTH_DST_ROUTES) {
			const struct gr_hip_route4 *r = &c->routes[x0 % c->n_routes];
			uint32_t m = r->prefixlen ? ~0u << (32 - r->prefixlen) : 0;
			dst = (__builtin_bswap32(r->ip) & m) | ((uint32_t)x1 & ~m);
		} else {
			uint64_t span = (uint64_t)c->dst_hi - c->dst_lo + 1;
			dst = c->dst_lo + (uint32_t)(x0 % span);
		}
		uint32_t len = 60;
		if (c->size_mode == GR_SYNTH_SIZE_IMIX) {
			uint32_t r = (uint32_t)((x3 >> 32) % 12);
			len = r < 7 ? 60 : (r < 11 ? 566 : 1514);
		}
		uint8_t *f = base + (size_t)i * stride;
		uint32_t clear = lines_only ? GR_HIP_LINE : (len > stride ? stride : len);
		if (clear < GR_HIP_LINE)
			clear = GR_HIP_LINE;
		memset(f, 0, clear);
		memcpy(f, c->dst_mac, 6);
		memcpy(f + 6, c->src_mac, 6);
		put16(f + 12, 0x0800);
		uint8_t *ip = f + 14;
		ip[0] = 0x45;
		ip[1] = 0;
		put16(ip + 2, (uint16_t)(len - 14));
		put16(ip + 4, (uint16_t)(x2 >> 32)); // packet id
		put16(ip + 6, 0); // DF=0, offset 0
		ip[8] = c->ttl ? c->ttl : 64;
		ip[9] = 17;
		put32(ip + 12, 0xc6120000u | ((uint32_t)x2 & 0x1ffff)); // 198.18.0.0/15
		put32(ip + 16, dst);
		put16(ip + 10, gr_synth_ip4_cksum(ip, 20));
		uint8_t *udp = ip + 20;
		put16(udp, (uint16_t)(x2 >> 48));
		put16(udp + 2, (uint16_t)x3);
		put16(udp + 4, (uint16_t)(len - 34));
		put16(udp + 6, 0);
		meta[i].iface = c->in_iface;
		meta[i].vlan_ck = (GR_HIP_CKSUM_UNKNOWN << 12);
		meta[i].pkt_len = (uint16_t)len;
		meta[i].rss = (uint16_t)(x3 >> 16);
	}
	return 0;
}
