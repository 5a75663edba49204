// SPDX-License-Identifier: BSD-3-Clause
//
// oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). A from-scratch CPU
// restatement of grout's IPv4 forwarding node chain. Reference paths are
// relative to the grout tree (DPDK/grout); "[DPDK]" marks DPDK 25.11 library
// semantics that grout calls but does not vendor.
#define _GNU_SOURCE
#include "oracle.h"

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#define OR_BURST 64 // rx_burst_max / vector_max defaults, graph.c:88-91
#define OR_BURST_MAX 256 // their maximum, RTE_GRAPH_BURST_SIZE (graph.c:619)
#define OR_HEADROOM 128 // RTE_PKTMBUF_HEADROOM
#define OR_DATAROOM 2048 // align32pow2(128+14+4+1800), mempool.c:66-68
#define NEXT GR_HIP_EDGE_CHAIN
#define NEXT6 GR_HIP_EDGE_CHAIN6 // eth_input: continue into ip6_input

// ---------------------------------------------------------------------------
// Topology (control-plane objects the nodes dereference)
// ---------------------------------------------------------------------------

struct or_ht { // open addressing, key = masked host-order ip
	uint32_t *keys;
	uint32_t *vals; // nh slot, 0 = empty
	uint32_t cap; // power of two
	uint32_t count;
};

struct or_fib {
	bool exists;
	uint32_t num_tbl8;
	struct or_ht len[33]; // RIB: one exact-match table per prefix length
	// DIR24_8 restatement [DPDK lib/fib/dir24_8.c], nh_sz = 8B (modules/ip/control/route.c:72-74)
	uint64_t *tbl24; // 1<<24 entries: (nh << 1) | ext
	uint64_t *tbl8; // num_tbl8 * 256
	uint32_t tbl8_used;
	bool built;
};

struct or_ht6 { // open addressing, key = masked 128-bit prefix
	uint8_t (*keys)[16];
	uint32_t *vals; // nh slot, 0 = empty
	uint32_t cap;
	uint32_t count;
};

struct or_fib6 { // RIB6: one exact-match table per prefix length
	bool exists;
	struct or_ht6 len[129];
};

struct or_topo {
	uint32_t max_ifaces;
	uint32_t max_nh;
	struct gr_hip_iface *ifaces;
	struct gr_hip_nh *nh;
	uint32_t *reta;
	uint32_t reta_cap;
	struct or_fib *fibs; // indexed by vrf_id (an iface id)
	struct or_fib6 *fibs6;
	uint8_t eth_edges[65536]; // l2l3_edges indexed by BE ether type, eth_input.c:24
	uint8_t mode_edges[GR_HIP_IFACE_MODE_COUNT]; // iface_input.c:20
	uint8_t in_nh_edges[256]; // ip_input.c:34
	uint8_t out_nh_edges[256]; // ip_output.c:44
	uint8_t out_iface_edges[256]; // ip_output.c:32
	uint8_t iout_type_edges[256]; // iface_output.c:23
	uint8_t in6_nh_edges[256]; // ip6_input.c:32
	uint8_t out6_nh_edges[256]; // ip6_output.c:40
	uint8_t out6_iface_edges[256]; // ip6_output.c:28
};

static uint16_t be16(uint16_t host) {
	return (uint16_t)((host >> 8) | (host << 8));
}

// Default registrations of grout's module set (grep of the *_register calls):
// ip_input.c:200-203, arp_input.c:62, ip6_input.c:161, lacp_input.c:66-68,
// eth_input.c:115, xconnect.c:65, bridge_input.c:124-125, vxlan_output.c:138,
// bond_output.c:250, port_output.c:51, xvrf.c:63, ipip/datapath_out.c:91,
// srv6_output.c:152, dnat44_static.c:102.
static void or_default_edges(or_topo_t *t) {
	memset(t->eth_edges, GR_HIP_E_ETH_INPUT_UNKNOWN_TYPE, sizeof(t->eth_edges));
	t->eth_edges[be16(0x0800)] = NEXT;
	t->eth_edges[be16(0x0806)] = GR_HIP_E_ARP_INPUT;
	t->eth_edges[be16(0x86dd)] = NEXT6; // ip6_input.c:161
	t->eth_edges[be16(0x8809)] = GR_HIP_E_LACP_INPUT;
	for (int i = 0; i < GR_HIP_IFACE_MODE_COUNT; i++)
		t->mode_edges[i] = GR_HIP_E_IFACE_MODE_UNKNOWN;
	t->mode_edges[GR_HIP_IFACE_MODE_VRF] = NEXT;
	t->mode_edges[GR_HIP_IFACE_MODE_BOND] = NEXT;
	t->mode_edges[GR_HIP_IFACE_MODE_XC] = GR_HIP_E_XCONNECT;
	t->mode_edges[GR_HIP_IFACE_MODE_BRIDGE] = GR_HIP_E_BRIDGE_INPUT;
	memset(t->in_nh_edges, NEXT, sizeof(t->in_nh_edges));
	t->in_nh_edges[GR_HIP_NH_T_BLACKHOLE] = GR_HIP_E_IP_BLACKHOLE;
	t->in_nh_edges[GR_HIP_NH_T_REJECT] = GR_HIP_E_IP_ERROR_DEST_UNREACH;
	t->in_nh_edges[GR_HIP_NH_T_DNAT] = GR_HIP_E_DNAT44_STATIC;
	memset(t->out_nh_edges, NEXT, sizeof(t->out_nh_edges));
	t->out_nh_edges[GR_HIP_NH_T_SR6_OUTPUT] = GR_HIP_E_SR6_OUTPUT;
	memset(t->out_iface_edges, NEXT, sizeof(t->out_iface_edges));
	t->out_iface_edges[GR_HIP_IFACE_TYPE_VRF] = GR_HIP_E_XVRF;
	t->out_iface_edges[GR_HIP_IFACE_TYPE_IPIP] = GR_HIP_E_IPIP_OUTPUT;
	memset(t->iout_type_edges, GR_HIP_E_IFACE_OUTPUT_INVAL_TYPE, sizeof(t->iout_type_edges));
	t->iout_type_edges[GR_HIP_IFACE_TYPE_PORT] = GR_HIP_E_PORT_OUTPUT;
	t->iout_type_edges[GR_HIP_IFACE_TYPE_BOND] = GR_HIP_E_BOND_OUTPUT;
	t->iout_type_edges[GR_HIP_IFACE_TYPE_VXLAN] = GR_HIP_E_VXLAN_OUTPUT;
	t->iout_type_edges[GR_HIP_IFACE_TYPE_BRIDGE] = GR_HIP_E_BRIDGE_INPUT;
	memset(t->in6_nh_edges, NEXT, sizeof(t->in6_nh_edges));
	t->in6_nh_edges[GR_HIP_NH_T_BLACKHOLE] = GR_HIP_E_IP6_BLACKHOLE; // ip6_input.c:163
	t->in6_nh_edges[GR_HIP_NH_T_REJECT] = GR_HIP_E_IP6_ERROR_DEST_UNREACH; // :164
	t->in6_nh_edges[GR_HIP_NH_T_SR6_LOCAL] = GR_HIP_E_SR6_LOCAL; // srv6_local.c:481
	memset(t->out6_nh_edges, NEXT, sizeof(t->out6_nh_edges));
	t->out6_nh_edges[GR_HIP_NH_T_SR6_OUTPUT] = GR_HIP_E_SR6_OUTPUT; // srv6_output.c:153
	memset(t->out6_iface_edges, NEXT, sizeof(t->out6_iface_edges));
	t->out6_iface_edges[GR_HIP_IFACE_TYPE_VRF] = GR_HIP_E_XVRF; // xvrf.c:64
}

or_topo_t *or_topo_new(uint32_t max_ifaces, uint32_t max_nexthops) {
	if (max_ifaces == 0 || max_ifaces > 65535 || max_nexthops == 0
	    || max_nexthops > GR_HIP_MAX_NEXTHOPS)
		return NULL;
	or_topo_t *t = calloc(1, sizeof(*t));
	if (t == NULL)
		return NULL;
	t->max_ifaces = max_ifaces;
	t->max_nh = max_nexthops;
	t->ifaces = calloc(max_ifaces, sizeof(*t->ifaces));
	t->nh = calloc((size_t)max_nexthops + 1, sizeof(*t->nh));
	t->fibs = calloc(max_ifaces, sizeof(*t->fibs));
	t->fibs6 = calloc(max_ifaces, sizeof(*t->fibs6));
	if (!t->ifaces || !t->nh || !t->fibs || !t->fibs6) {
		or_topo_free(t);
		return NULL;
	}
	or_default_edges(t);
	return t;
}

static void ht_free(struct or_ht *h) {
	free(h->keys);
	free(h->vals);
	memset(h, 0, sizeof(*h));
}

static void fib_free_tables(struct or_fib *f) {
	if (f->tbl24)
		munmap(f->tbl24, (size_t)8 << 24);
	free(f->tbl8);
	f->tbl24 = NULL;
	f->tbl8 = NULL;
	f->built = false;
}

void or_topo_free(or_topo_t *t) {
	if (t == NULL)
		return;
	if (t->fibs) {
		for (uint32_t v = 0; v < t->max_ifaces; v++) {
			for (int l = 0; l <= 32; l++)
				ht_free(&t->fibs[v].len[l]);
			fib_free_tables(&t->fibs[v]);
		}
	}
	free(t->fibs);
	if (t->fibs6) {
		for (uint32_t v = 0; v < t->max_ifaces; v++) {
			for (int l = 0; l <= 128; l++) {
				free(t->fibs6[v].len[l].keys);
				free(t->fibs6[v].len[l].vals);
			}
		}
	}
	free(t->fibs6);
	free(t->ifaces);
	free(t->nh);
	free(t->reta);
	free(t);
}

#define EDGE_SETTER(fn, table, limit)                                                              \
	int fn(or_topo_t *t, uint8_t key, uint8_t edge) {                                          \
		if ((unsigned)key + 1 > (unsigned)(limit))                                         \
			return -EINVAL;                                                            \
		t->table[key] = edge;                                                              \
		return 0;                                                                          \
	}
EDGE_SETTER(or_edge_iface_mode, mode_edges, GR_HIP_IFACE_MODE_COUNT)
EDGE_SETTER(or_edge_ip_input_nh_type, in_nh_edges, 256)
EDGE_SETTER(or_edge_ip_output_nh_type, out_nh_edges, 256)
EDGE_SETTER(or_edge_ip_output_iface_type, out_iface_edges, 256)
EDGE_SETTER(or_edge_iface_output_type, iout_type_edges, 256)
EDGE_SETTER(or_edge_ip6_input_nh_type, in6_nh_edges, 256)
EDGE_SETTER(or_edge_ip6_output_nh_type, out6_nh_edges, 256)
EDGE_SETTER(or_edge_ip6_output_iface_type, out6_iface_edges, 256)

int or_edge_eth_type(or_topo_t *t, uint16_t be_type, uint8_t edge) {
	t->eth_edges[be_type] = edge;
	return 0;
}

int or_iface_set(or_topo_t *t, const struct gr_hip_iface *ifs, uint32_t n) {
	for (uint32_t i = 0; i < n; i++) {
		if (ifs[i].id == 0 || ifs[i].id >= t->max_ifaces)
			return -EINVAL;
		t->ifaces[ifs[i].id] = ifs[i];
	}
	return 0;
}

int or_nh_set(or_topo_t *t, uint32_t first, const struct gr_hip_nh *nh, uint32_t n) {
	if (first == 0 || (uint64_t)first + n > (uint64_t)t->max_nh + 1)
		return -EINVAL;
	memcpy(&t->nh[first], nh, (size_t)n * sizeof(*nh));
	return 0;
}

int or_reta_set(or_topo_t *t, uint32_t first, const uint32_t *slots, uint32_t n) {
	uint64_t need = (uint64_t)first + n;
	if (need > t->reta_cap) {
		uint32_t cap = t->reta_cap ? t->reta_cap : 1024;
		while (cap < need)
			cap *= 2;
		uint32_t *r = realloc(t->reta, (size_t)cap * sizeof(*r));
		if (r == NULL)
			return -ENOMEM;
		memset(r + t->reta_cap, 0, (size_t)(cap - t->reta_cap) * sizeof(*r));
		t->reta = r;
		t->reta_cap = cap;
	}
	memcpy(&t->reta[first], slots, (size_t)n * sizeof(*slots));
	return 0;
}

// iface_from_id, modules/infra/control/iface.c:459-466
static const struct gr_hip_iface *iface_from_id(const or_topo_t *t, uint16_t id) {
	if (id == GR_HIP_IFACE_ID_UNDEF || id >= t->max_ifaces || t->ifaces[id].id != id)
		return NULL;
	return &t->ifaces[id];
}

// vlan_get_iface, modules/infra/control/vlan.c:27-34 (hash on {parent, vlan})
static const struct gr_hip_iface *vlan_get_iface(const or_topo_t *t, uint16_t parent, uint16_t vid) {
	for (uint32_t i = 1; i < t->max_ifaces; i++) {
		const struct gr_hip_iface *v = &t->ifaces[i];
		if (v->id == i && v->type == GR_HIP_IFACE_TYPE_VLAN && v->parent_id == parent
		    && v->vlan_id == vid)
			return v;
	}
	return NULL;
}

// ---------------------------------------------------------------------------
// RIB and LPMs
// ---------------------------------------------------------------------------

static uint32_t depth_mask(uint8_t len) { // rte_rib_depth_to_mask [DPDK]
	return len == 0 ? 0 : (uint32_t)(~0u << (32 - len));
}

static uint32_t ht_hash(uint32_t k) {
	k ^= k >> 16;
	k *= 0x7feb352du;
	k ^= k >> 15;
	k *= 0x846ca68bu;
	k ^= k >> 16;
	return k;
}

static int ht_grow(struct or_ht *h) {
	uint32_t ncap = h->cap ? h->cap * 2 : 64;
	uint32_t *nk = calloc(ncap, sizeof(*nk));
	uint32_t *nv = calloc(ncap, sizeof(*nv));
	if (!nk || !nv) {
		free(nk);
		free(nv);
		return -ENOMEM;
	}
	for (uint32_t i = 0; i < h->cap; i++) {
		if (h->vals[i] == 0)
			continue;
		uint32_t j = ht_hash(h->keys[i]) & (ncap - 1);
		while (nv[j] != 0)
			j = (j + 1) & (ncap - 1);
		nk[j] = h->keys[i];
		nv[j] = h->vals[i];
	}
	free(h->keys);
	free(h->vals);
	h->keys = nk;
	h->vals = nv;
	h->cap = ncap;
	return 0;
}

static uint32_t *ht_find(const struct or_ht *h, uint32_t key) {
	if (h->cap == 0)
		return NULL;
	uint32_t j = ht_hash(key) & (h->cap - 1);
	while (h->vals[j] != 0) {
		if (h->keys[j] == key)
			return &h->vals[j];
		j = (j + 1) & (h->cap - 1);
	}
	return NULL;
}

int or_fib_create(or_topo_t *t, uint16_t vrf, uint32_t num_tbl8) {
	if (vrf == 0 || vrf >= t->max_ifaces)
		return -EINVAL;
	struct or_fib *f = &t->fibs[vrf];
	f->exists = true;
	f->num_tbl8 = num_tbl8 ? num_tbl8 : 256;
	return 0;
}

// rib4_insert_or_replace, modules/ip/control/route.c:212-275: an existing
// prefix is EEXIST unless replace is set; rte_fib_add masks host bits [DPDK].
int or_route_add(or_topo_t *t, const struct gr_hip_route4 *r, uint32_t n, int replace) {
	for (uint32_t i = 0; i < n; i++) {
		if (r[i].vrf_id == 0 || r[i].vrf_id >= t->max_ifaces || r[i].prefixlen > 32
		    || r[i].nh == 0 || r[i].nh > t->max_nh)
			return -EINVAL;
		struct or_fib *f = &t->fibs[r[i].vrf_id];
		if (!f->exists)
			return -ENONET;
		struct or_ht *h = &f->len[r[i].prefixlen];
		uint32_t key = __builtin_bswap32(r[i].ip) & depth_mask(r[i].prefixlen);
		uint32_t *v = ht_find(h, key);
		if (v != NULL) {
			if (!replace)
				return -EEXIST;
			*v = r[i].nh;
			f->built = false;
			continue;
		}
		if ((h->count + 1) * 2 > h->cap && ht_grow(h) < 0)
			return -ENOMEM;
		uint32_t j = ht_hash(key) & (h->cap - 1);
		while (h->vals[j] != 0)
			j = (j + 1) & (h->cap - 1);
		h->keys[j] = key;
		h->vals[j] = r[i].nh;
		h->count++;
		f->built = false;
	}
	return 0;
}

int or_route_del(or_topo_t *t, uint16_t vrf, uint32_t ip_be, uint8_t len) {
	if (vrf == 0 || vrf >= t->max_ifaces || len > 32 || !t->fibs[vrf].exists)
		return -EINVAL;
	struct or_fib *f = &t->fibs[vrf];
	struct or_ht *h = &f->len[len];
	uint32_t key = __builtin_bswap32(ip_be) & depth_mask(len);
	if (ht_find(h, key) == NULL)
		return -ENOENT;
	// rebuild the table without the key (deletions are rare in the oracle)
	struct or_ht nh = {0};
	for (uint32_t i = 0; i < h->cap; i++) {
		if (h->vals[i] == 0 || h->keys[i] == key)
			continue;
		if ((nh.count + 1) * 2 > nh.cap && ht_grow(&nh) < 0)
			return -ENOMEM;
		uint32_t j = ht_hash(h->keys[i]) & (nh.cap - 1);
		while (nh.vals[j] != 0)
			j = (j + 1) & (nh.cap - 1);
		nh.keys[j] = h->keys[i];
		nh.vals[j] = h->vals[i];
		nh.count++;
	}
	ht_free(h);
	*h = nh;
	f->built = false;
	return 0;
}

// ---- IPv6 RIB: exact-prefix hash per length (rib6_insert_or_replace /
// rib6_delete, modules/ip6/control/route.c:230-345)

// addr6_linklocal_scope, modules/ip6/control/ip6.h:23-36.
static void scope6(uint8_t out[16], const uint8_t ip[16], uint16_t iface_id) {
	memcpy(out, ip, 16);
	if (ip[0] == 0xfe && (ip[1] & 0xc0) == 0x80) { // rte_ipv6_addr_is_linklocal [DPDK]
		out[2] = (uint8_t)(iface_id >> 8);
		out[3] = (uint8_t)iface_id;
	}
}

static void mask6(uint8_t out[16], const uint8_t ip[16], unsigned len) { // rte_ipv6_addr_mask [DPDK]
	for (unsigned i = 0; i < 16; i++) {
		int bits = (int)len - 8 * (int)i;
		out[i] = ip[i] & (bits >= 8 ? 0xff : bits <= 0 ? 0 : (uint8_t)(0xff << (8 - bits)));
	}
}

static uint32_t ht6_hash(const uint8_t k[16]) {
	uint32_t h = 2166136261u; // FNV-1a
	for (int i = 0; i < 16; i++)
		h = (h ^ k[i]) * 16777619u;
	return h;
}

static uint32_t *ht6_find(const struct or_ht6 *h, const uint8_t k[16]) {
	if (h->cap == 0)
		return NULL;
	for (uint32_t j = ht6_hash(k) & (h->cap - 1);; j = (j + 1) & (h->cap - 1)) {
		if (h->vals[j] == 0)
			return NULL;
		if (memcmp(h->keys[j], k, 16) == 0)
			return &h->vals[j];
	}
}

static int ht6_put(struct or_ht6 *h, const uint8_t k[16], uint32_t v) {
	if ((h->count + 1) * 2 > h->cap) {
		struct or_ht6 n = {0};
		n.cap = h->cap ? h->cap * 2 : 16;
		n.keys = calloc(n.cap, 16);
		n.vals = calloc(n.cap, sizeof(uint32_t));
		if (!n.keys || !n.vals) {
			free(n.keys);
			free(n.vals);
			return -ENOMEM;
		}
		for (uint32_t i = 0; i < h->cap; i++)
			if (h->vals[i])
				ht6_put(&n, h->keys[i], h->vals[i]);
		free(h->keys);
		free(h->vals);
		*h = n;
	}
	uint32_t j = ht6_hash(k) & (h->cap - 1);
	while (h->vals[j] != 0)
		j = (j + 1) & (h->cap - 1);
	memcpy(h->keys[j], k, 16);
	h->vals[j] = v;
	h->count++;
	return 0;
}

int or_fib6_create(or_topo_t *t, uint16_t vrf) {
	if (vrf == 0 || vrf >= t->max_ifaces)
		return -EINVAL;
	t->fibs6[vrf].exists = true;
	return 0;
}

int or_route6_add(or_topo_t *t, const struct gr_hip_route6 *r, uint32_t n, int replace) {
	for (uint32_t i = 0; i < n; i++) {
		if (r[i].vrf_id == 0 || r[i].vrf_id >= t->max_ifaces || r[i].prefixlen > 128 || r[i].nh == 0
		    || r[i].nh > t->max_nh)
			return -EINVAL;
		struct or_fib6 *f = &t->fibs6[r[i].vrf_id];
		if (!f->exists)
			return -ENONET;
		uint8_t sc[16], key[16];
		scope6(sc, r[i].ip, r[i].iface_id);
		mask6(key, sc, r[i].prefixlen);
		uint32_t *v = ht6_find(&f->len[r[i].prefixlen], key);
		if (v != NULL) {
			if (!replace)
				return -EEXIST;
			*v = r[i].nh;
			continue;
		}
		if (ht6_put(&f->len[r[i].prefixlen], key, r[i].nh) < 0)
			return -ENOMEM;
	}
	return 0;
}

int or_route6_del(or_topo_t *t, uint16_t vrf, uint16_t iface_id, const uint8_t ip[16], uint8_t len) {
	if (vrf == 0 || vrf >= t->max_ifaces || len > 128 || !t->fibs6[vrf].exists)
		return -EINVAL;
	struct or_ht6 *h = &t->fibs6[vrf].len[len];
	uint8_t sc[16], key[16];
	scope6(sc, ip, iface_id);
	mask6(key, sc, len);
	if (ht6_find(h, key) == NULL)
		return -ENOENT;
	struct or_ht6 n = {0};
	for (uint32_t i = 0; i < h->cap; i++)
		if (h->vals[i] && memcmp(h->keys[i], key, 16) != 0 && ht6_put(&n, h->keys[i], h->vals[i]) < 0)
			return -ENOMEM;
	free(h->keys);
	free(h->vals);
	*h = n;
	return 0;
}

// fib6_lookup's LPM (route.c:151-173, rte_fib6_lookup_bulk): probe each
// prefix length, longest first, on the scoped address.
uint32_t or_lpm6(const or_topo_t *t, uint16_t vrf, uint16_t iface_id, const uint8_t ip[16]) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs6[vrf].exists)
		return 0;
	uint8_t sc[16], key[16];
	scope6(sc, ip, iface_id);
	for (int l = 128; l >= 0; l--) {
		mask6(key, sc, (unsigned)l);
		const uint32_t *v = ht6_find(&t->fibs6[vrf].len[l], key);
		if (v != NULL)
			return *v;
	}
	return 0;
}

// Brute force: every stored prefix, keep the longest covering one.
uint32_t or_lpm6_brute(const or_topo_t *t, uint16_t vrf, uint16_t iface_id, const uint8_t ip[16]) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs6[vrf].exists)
		return 0;
	uint8_t sc[16], key[16];
	scope6(sc, ip, iface_id);
	int best = -1;
	uint32_t nh = 0;
	for (int l = 0; l <= 128; l++) {
		const struct or_ht6 *h = &t->fibs6[vrf].len[l];
		mask6(key, sc, (unsigned)l);
		for (uint32_t i = 0; i < h->cap; i++)
			if (h->vals[i] && memcmp(h->keys[i], key, 16) == 0 && l > best) {
				best = l;
				nh = h->vals[i];
			}
	}
	return nh;
}

// Longest-prefix match by probing each prefix length, longest first.
uint32_t or_lpm_hash(const or_topo_t *t, uint16_t vrf, uint32_t ip) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs[vrf].exists)
		return 0;
	const struct or_fib *f = &t->fibs[vrf];
	for (int l = 32; l >= 0; l--) {
		const uint32_t *v = ht_find(&f->len[l], ip & depth_mask((uint8_t)l));
		if (v != NULL)
			return *v;
	}
	return 0;
}

uint32_t or_lpm_brute(const or_topo_t *t, uint16_t vrf, uint32_t ip) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs[vrf].exists)
		return 0;
	const struct or_fib *f = &t->fibs[vrf];
	int best = -1;
	uint32_t nh = 0;
	for (int l = 0; l <= 32; l++) {
		const struct or_ht *h = &f->len[l];
		for (uint32_t i = 0; i < h->cap; i++) {
			if (h->vals[i] == 0)
				continue;
			if ((ip & depth_mask((uint8_t)l)) == h->keys[i] && l > best) {
				best = l;
				nh = h->vals[i];
			}
		}
	}
	return nh;
}

// DIR24_8 [DPDK lib/fib/dir24_8.c]: tbl24[ip >> 8]; bit 0 set = extended, the
// entry >> 1 is a tbl8 group whose [ip & 0xff] entry holds (nh << 1).
// Built by painting prefixes in increasing length so longer ones win, which
// gives the same table content as DPDK's incremental rte_fib_add sequence.
int or_fib_build(or_topo_t *t, uint16_t vrf) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs[vrf].exists)
		return -EINVAL;
	struct or_fib *f = &t->fibs[vrf];
	fib_free_tables(f);
	f->tbl24 = mmap(NULL, (size_t)8 << 24, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (f->tbl24 == MAP_FAILED) {
		f->tbl24 = NULL;
		return -ENOMEM;
	}
	madvise(f->tbl24, (size_t)8 << 24, MADV_HUGEPAGE); // grout's rte_fib is on hugepages
	f->tbl8 = calloc((size_t)f->num_tbl8 * 256, sizeof(uint64_t));
	if (f->tbl8 == NULL)
		return -ENOMEM;
	f->tbl8_used = 0;
	for (int l = 0; l <= 24; l++) {
		const struct or_ht *h = &f->len[l];
		for (uint32_t i = 0; i < h->cap; i++) {
			if (h->vals[i] == 0)
				continue;
			uint32_t first = h->keys[i] >> 8, count = 1u << (24 - l);
			for (uint32_t k = 0; k < count; k++)
				f->tbl24[first + k] = (uint64_t)h->vals[i] << 1;
		}
	}
	for (int l = 25; l <= 32; l++) {
		const struct or_ht *h = &f->len[l];
		for (uint32_t i = 0; i < h->cap; i++) {
			if (h->vals[i] == 0)
				continue;
			uint32_t ip = h->keys[i];
			uint64_t *e = &f->tbl24[ip >> 8];
			if (!(*e & 1)) {
				if (f->tbl8_used >= f->num_tbl8)
					return -ENOSPC;
				uint64_t *g = &f->tbl8[(size_t)f->tbl8_used * 256];
				for (int k = 0; k < 256; k++)
					g[k] = *e;
				*e = ((uint64_t)f->tbl8_used << 1) | 1;
				f->tbl8_used++;
			}
			uint64_t *g = &f->tbl8[(size_t)(*e >> 1) * 256];
			uint32_t first = ip & 0xff, count = 1u << (32 - l);
			for (uint32_t k = 0; k < count; k++)
				g[first + k] = (uint64_t)h->vals[i] << 1;
		}
	}
	f->built = true;
	return 0;
}

static inline uint32_t dir24_lookup(const struct or_fib *f, uint32_t ip) {
	uint64_t e = f->tbl24[ip >> 8];
	if (e & 1)
		e = f->tbl8[(e >> 1) * 256 + (ip & 0xff)];
	return (uint32_t)(e >> 1);
}

uint32_t or_lpm_dir24(const or_topo_t *t, uint16_t vrf, uint32_t ip) {
	if (vrf == 0 || vrf >= t->max_ifaces || !t->fibs[vrf].exists || !t->fibs[vrf].built)
		return 0;
	return dir24_lookup(&t->fibs[vrf], ip);
}

// fib4_lookup, modules/ip/control/route.c:147-167: get_fib() (:51-61) needs
// the VRF iface (get_vrf_iface, modules/infra/control/vrf.c:51-57) and its
// FIB; value 0 is no route (.default_nh = 0, :65); a GROUP nexthop is
// resolved through nexthop_group_get_nh (modules/infra/control/nexthop.h:89-96).
static uint32_t fib4_lookup(const or_topo_t *t, uint16_t vrf_id, uint32_t dst_be, uint16_t rss) {
	const struct gr_hip_iface *vrf = iface_from_id(t, vrf_id);
	if (vrf == NULL || vrf->type != GR_HIP_IFACE_TYPE_VRF)
		return 0;
	const struct or_fib *f = &t->fibs[vrf_id];
	if (!f->exists)
		return 0;
	uint32_t ip = __builtin_bswap32(dst_be);
	uint32_t nh = f->built ? dir24_lookup(f, ip) : or_lpm_hash(t, vrf_id, ip);
	if (nh == 0 || nh > t->max_nh)
		return 0;
	const struct gr_hip_nh *n = &t->nh[nh];
	if (n->type == GR_HIP_NH_T_GROUP) {
		if (n->n_members == 1)
			return n->single > t->max_nh ? 0 : n->single;
		if (n->n_members == 0)
			return 0;
		uint32_t i = n->reta_off + (rss & (uint32_t)(n->reta_size - 1));
		nh = i < t->reta_cap ? t->reta[i] : 0;
		return nh > t->max_nh ? 0 : nh;
	}
	return nh;
}

// fib6_lookup, modules/ip6/control/route.c:151-173: the VRF's FIB6, the
// scoped destination, 0 = no route, GROUP resolved as for IPv4.
static uint32_t fib6_lookup(const or_topo_t *t, uint16_t vrf_id, uint16_t iface_id, const uint8_t dst[16], uint16_t rss) {
	const struct gr_hip_iface *vrf = iface_from_id(t, vrf_id);
	if (vrf == NULL || vrf->type != GR_HIP_IFACE_TYPE_VRF)
		return 0;
	uint32_t nh = or_lpm6(t, vrf_id, iface_id, dst);
	if (nh == 0 || nh > t->max_nh)
		return 0;
	const struct gr_hip_nh *n = &t->nh[nh];
	if (n->type == GR_HIP_NH_T_GROUP) {
		if (n->n_members == 1)
			return n->single > t->max_nh ? 0 : n->single;
		if (n->n_members == 0)
			return 0;
		uint32_t i = n->reta_off + (rss & (uint32_t)(n->reta_size - 1));
		nh = i < t->reta_cap ? t->reta[i] : 0;
		return nh > t->max_nh ? 0 : nh;
	}
	return nh;
}

// ---------------------------------------------------------------------------
// mbuf stand-in and the nodes
// ---------------------------------------------------------------------------

struct or_mbuf {
	uint8_t *buf; // OR_DATAROOM bytes
	uint16_t data_off;
	uint16_t data_len;
	uint32_t pkt_len;
	uint8_t ck; // GR_HIP_CKSUM_*
	uint16_t rss;
	uint32_t packet_type;
	// private area: modules/infra/datapath/mbuf.h:29-38 (traces, iface) and
	// the per-node views iface_mbuf_data (rxtx.h:45-48), eth_input_mbuf_data
	// and eth_output_mbuf_data (eth.h:23-36), l3_mbuf_data (l3.h:9)
	uint16_t iface;
	uint16_t vlan_id;
	uint8_t domain;
	uint32_t e_nh; // eth_input_mbuf_data.nh
	uint32_t l3_nh; // l3_mbuf_data.nh
	uint8_t eth_dst[6]; // eth_output_mbuf_data
	uint16_t eth_type; // BE
	// result
	uint8_t edge;
	uint16_t visited; // bit per enum gr_hip_node this packet was handed to
	uint8_t rx_counted, tx_counted;
	uint16_t tx_iface, tx_parent;
	uint16_t rx_iface, rx_parent;
	uint32_t orig_len;
};

#define MTOD(m) ((m)->buf + (m)->data_off)

// rte_pktmbuf_adj [DPDK]: no-op returning NULL when len > data_len.
static void mbuf_adj(struct or_mbuf *m, uint16_t len) {
	if (len > m->data_len)
		return;
	m->data_off += len;
	m->data_len -= len;
	m->pkt_len -= len;
}

static void mbuf_prepend(struct or_mbuf *m, uint16_t len) { // headroom is always there
	m->data_off -= len;
	m->data_len += len;
	m->pkt_len += len;
}

struct or_stream {
	struct or_mbuf *objs[OR_BURST_MAX];
	uint16_t n;
};

// The nodes after iface_input, by enum gr_hip_node.
struct or_graph {
	const or_topo_t *t;
	uint32_t flags;
	uint32_t readable; // frame bytes present: 64 (lines only) or in_stride
	struct or_stream st[GR_HIP_NODE_COUNT];
	// rte_graph's pending queue [DPDK lib/graph rte_graph_walk]: a node
	// joins its tail when its stream goes from empty to non-empty, the walk
	// runs the queue head first (so a node may run again later in the walk)
	uint8_t pend[4 * GR_HIP_NODE_COUNT];
	uint32_t pend_head, pend_tail;
};

static inline void enqueue(struct or_graph *g, int node, struct or_mbuf *m) {
	struct or_stream *s = &g->st[node];
	if (s->n == 0)
		g->pend[g->pend_tail++ % (4 * GR_HIP_NODE_COUNT)] = (uint8_t)node;
	s->objs[s->n++] = m;
}

static inline void terminal(struct or_mbuf *m, uint8_t edge) {
	m->edge = edge;
}

// iface_input_process, modules/infra/datapath/iface_input.c:52-112
static void node_iface_input(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const struct gr_hip_iface *iface = iface_from_id(t, m->iface);
		if (iface == NULL) { // port_rx always sets a valid iface: not grout's case
			terminal(m, GR_HIP_E_PUNT);
			continue;
		}
		uint16_t parent = m->iface;
		if (m->vlan_id != 0 && iface->mode == GR_HIP_IFACE_MODE_VRF) { // :74-86
			const struct gr_hip_iface *v = vlan_get_iface(t, iface->id, m->vlan_id);
			if (v == NULL) {
				terminal(m, GR_HIP_E_IFACE_INPUT_UNKNOWN_VLAN);
				continue;
			}
			m->iface = v->id;
			m->vlan_id = 0;
			iface = v;
		}
		if (!(iface->flags & GR_HIP_IFACE_F_UP)) { // :88-91
			terminal(m, GR_HIP_E_IFACE_INPUT_ADMIN_DOWN);
			continue;
		}
		m->rx_counted = 1; // IFACE_STATS_INC :93-95
		m->rx_iface = iface->id;
		m->rx_parent = parent != iface->id ? parent : 0;
		uint8_t e = t->mode_edges[iface->mode < GR_HIP_IFACE_MODE_COUNT ? iface->mode : 0];
		if (iface->mode >= GR_HIP_IFACE_MODE_COUNT)
			e = GR_HIP_E_IFACE_MODE_UNKNOWN;
		if (e == NEXT)
			enqueue(g, GR_HIP_NODE_ETH_INPUT, m);
		else
			terminal(m, e);
	}
}

// eth_input_process, modules/infra/datapath/eth_input.c:35-88. The
// last_iface_id cache (:62-68) only skips repeated iface_get_eth_addr() calls
// of the same iface, so a per-packet lookup of the mirrored MAC is equivalent.
static void node_eth_input(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const uint8_t *eth = MTOD(m);
		uint16_t type_be = (uint16_t)(eth[12] | (eth[13] << 8)); // as stored
		uint16_t type = (uint16_t)((eth[12] << 8) | eth[13]);
		if (type < 1536 || type == 0x8870) { // SNAP_MAX_LEN, JUMBO_LLC snap.h:11-12
			terminal(m, GR_HIP_E_SNAP_INPUT);
			continue;
		}
		const struct gr_hip_iface *iface = iface_from_id(t, m->iface);
		if (iface == NULL || !iface->mac_ok) {
			terminal(m, GR_HIP_E_ETH_INPUT_INVALID_IFACE);
			continue;
		}
		m->e_nh = 0;
		if (eth[0] & 1) { // rte_is_multicast_ether_addr [DPDK]
			bool bcast = eth[0] == 0xff && eth[1] == 0xff && eth[2] == 0xff
				&& eth[3] == 0xff && eth[4] == 0xff && eth[5] == 0xff;
			m->domain = bcast ? GR_HIP_ETH_DOMAIN_BROADCAST : GR_HIP_ETH_DOMAIN_MULTICAST;
		} else if (memcmp(eth, iface->mac, 6) == 0) {
			m->domain = GR_HIP_ETH_DOMAIN_LOCAL;
		} else {
			m->domain = GR_HIP_ETH_DOMAIN_OTHER;
		}
		mbuf_adj(m, 14);
		uint8_t e = t->eth_edges[type_be];
		if (e == NEXT)
			enqueue(g, GR_HIP_NODE_IP_INPUT, m);
		else if (e == NEXT6)
			enqueue(g, GR_HIP_NODE_IP6_INPUT, m);
		else
			terminal(m, e);
	}
}

// rte_raw_cksum [DPDK lib/net/rte_cksum.h]: 16-bit little-endian host words,
// summed in 32 bits and folded twice.
static uint16_t raw_cksum(const uint8_t *p, uint32_t len) {
	uint32_t sum = 0;
	for (uint32_t i = 0; i + 1 < len; i += 2)
		sum += (uint32_t)(p[i] | (p[i + 1] << 8));
	if (len & 1)
		sum += p[len - 1];
	sum = (sum & 0xffff) + (sum >> 16);
	sum = (sum & 0xffff) + (sum >> 16);
	return (uint16_t)sum;
}

// ip_input_process, modules/ip/datapath/ip_input.c:47-197
static void node_ip_input(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const uint8_t *ip = MTOD(m);
		const struct gr_hip_iface *iface = iface_from_id(t, m->iface);
		uint8_t domain = m->domain;
		uint8_t edge;

		if (m->data_len < 20) { // (1) :70-77
			edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
			goto next;
		}
		switch (m->ck) { // (2) :80-92, rte_ipv4_cksum = ~raw_cksum(ihl*4)
		case GR_HIP_CKSUM_UNKNOWN: {
			uint32_t hl = (uint32_t)(ip[0] & 0xf) * 4;
			if (14 + hl > g->readable) {
				edge = GR_HIP_E_PUNT; // header bytes not present: grout's CPU path
				goto next;
			}
			if ((uint16_t)~raw_cksum(ip, hl) != 0) {
				edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
				goto next;
			}
			break;
		}
		case GR_HIP_CKSUM_BAD:
			edge = GR_HIP_E_IP_INPUT_BAD_CHECKSUM;
			goto next;
		default:
			break;
		}
		uint32_t dst; // network order, as stored
		memcpy(&dst, ip + 16, 4);
		if (dst == 0) { // :94-97
			edge = GR_HIP_E_IP_INPUT_BAD_ADDRESS;
			goto next;
		}
		if ((ip[0] >> 4) != 4) { // (3) :102-105
			edge = GR_HIP_E_IP_INPUT_BAD_VERSION;
			goto next;
		}
		if ((ip[0] & 0xf) * 4 < 20) { // (4) :109-112
			edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
			goto next;
		}
		if (((ip[2] << 8) | ip[3]) < 20) { // (5) :117-120
			edge = GR_HIP_E_IP_INPUT_BAD_LENGTH;
			goto next;
		}
		switch (domain) { // :122-137
		case GR_HIP_ETH_DOMAIN_LOOPBACK:
		case GR_HIP_ETH_DOMAIN_LOCAL:
			break;
		case GR_HIP_ETH_DOMAIN_BROADCAST:
		case GR_HIP_ETH_DOMAIN_MULTICAST:
			edge = GR_HIP_E_IP_INPUT_LOCAL;
			goto next;
		default:
			edge = GR_HIP_E_IP_INPUT_OTHER_HOST;
			goto next;
		}
		// IPV4_ADDR_BCAST / ip4_addr_is_mcast (api/gr_net_types.h:97-106)
		if (dst == 0xffffffffu || (ip[16] >= 224 && ip[16] <= 239)) { // :139-142
			edge = GR_HIP_E_IP_INPUT_LOCAL;
			goto next;
		}
		uint32_t nh = m->e_nh ? m->e_nh : fib4_lookup(t, iface->vrf_id, dst, m->rss); // :146-149
		if (nh == 0) { // :150-153
			edge = GR_HIP_E_IP_ERROR_DEST_UNREACH;
			goto next;
		}
		m->l3_nh = nh; // :156
		const struct gr_hip_nh *h = &t->nh[nh];
		edge = t->in_nh_edges[h->type];
		if (edge != NEXT)
			goto next;
		if (domain == GR_HIP_ETH_DOMAIN_LOOPBACK) { // :164-165 (not reachable from ports)
			enqueue(g, GR_HIP_NODE_IP_OUTPUT, m);
			continue;
		} else if (h->type == GR_HIP_NH_T_L3) { // :166-187
			if ((h->flags & GR_HIP_NH_F_LOCAL) && dst == h->ipv4) {
				edge = (iface->flags & GR_HIP_IFACE_F_SNAT_DYNAMIC)
					? GR_HIP_E_IP_INPUT_LOCAL_CT
					: GR_HIP_E_IP_INPUT_LOCAL;
				goto next;
			}
		}
		enqueue(g, GR_HIP_NODE_IP_FORWARD, m);
		continue;
next:
		terminal(m, edge);
	}
}

// ip_forward_process, modules/ip/datapath/ip_forward.c:14-41. The checksum
// field is read as a host (little-endian) u16, RTE_BE16(0x0100) == 0x0001.
static void node_ip_forward(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		uint8_t *ip = MTOD(m);
		if (ip[8] <= 1) {
			terminal(m, GR_HIP_E_IP_ERROR_TTL_EXCEEDED);
			continue;
		}
		ip[8] -= 1;
		uint32_t csum = (uint32_t)(ip[10] | (ip[11] << 8)) + 0x0001;
		csum += csum >= 0xffff;
		ip[10] = (uint8_t)csum;
		ip[11] = (uint8_t)(csum >> 8);
		enqueue(g, GR_HIP_NODE_IP_OUTPUT, m);
	}
}

// ip_output_process, modules/ip/datapath/ip_output.c:62-163
static void node_ip_output(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const uint8_t *ip = MTOD(m);
		uint8_t edge;
		if (m->l3_nh == 0) { // :79-83
			edge = GR_HIP_E_IP_ERROR_DEST_UNREACH;
			goto next;
		}
		m->packet_type = 0x10; // :85, RTE_PTYPE_L3_IPV4 [DPDK rte_mbuf_ptype.h]
		const struct gr_hip_nh *h = &t->nh[m->l3_nh];
		edge = t->out_nh_edges[h->type]; // :87-89
		if (edge != NEXT)
			goto next;
		const struct gr_hip_iface *iface = iface_from_id(t, h->iface_id);
		if (iface == NULL) { // :91-95
			edge = GR_HIP_E_IP_OUTPUT_ERROR;
			goto next;
		}
		m->iface = iface->id; // :97
		if (m->pkt_len > iface->mtu) { // :99-106, DF = BE 0x4000
			edge = (ip[6] & 0x40) ? GR_HIP_E_IP_ERROR_FRAG_NEEDED : GR_HIP_E_IP_FRAGMENT;
			goto next;
		}
		edge = t->out_iface_edges[iface->type]; // :110
		if (iface->flags & (GR_HIP_IFACE_F_SNAT_STATIC | GR_HIP_IFACE_F_SNAT_DYNAMIC)) {
			edge = GR_HIP_E_IP_OUTPUT_SNAT; // snat44_process :112-119 needs the NAT tables
			goto next;
		}
		if (edge != NEXT) // :121-122
			goto next;
		uint32_t dst;
		memcpy(&dst, ip + 16, 4);
		if (h->state != GR_HIP_NH_S_REACHABLE
		    || ((h->flags & GR_HIP_NH_F_LINK) && dst != h->ipv4)) { // :124-138
			edge = GR_HIP_E_IP_HOLD;
			goto next;
		}
		memcpy(m->eth_dst, h->mac, 6); // :140-152 (vtep: not on the forward path)
		m->eth_type = be16(0x0800);
		enqueue(g, GR_HIP_NODE_ETH_OUTPUT, m);
		continue;
next:
		terminal(m, edge);
	}
}

// ip6_input_process, modules/ip6/datapath/ip6_input.c:44-158
static void node_ip6_input(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const uint8_t *ip = MTOD(m); // struct rte_ipv6_hdr
		const uint8_t *src = ip + 8, *dst = ip + 24;
		const struct gr_hip_iface *iface = iface_from_id(t, m->iface);
		uint32_t nh = 0;
		uint8_t edge;
		if (m->data_len < 40) { // :63-70
			edge = GR_HIP_E_IP6_INPUT_BAD_LENGTH;
			goto next;
		}
		if ((ip[0] & 0xf0) != 0x60) { // :72-75, rte_ipv6_check_version [DPDK]
			edge = GR_HIP_E_IP6_INPUT_BAD_VERSION;
			goto next;
		}
		static const uint8_t zero[16];
		if (src[0] == 0xff || memcmp(dst, zero, 16) == 0) { // mcast src, unspec dst :77-81
			edge = GR_HIP_E_IP6_INPUT_BAD_ADDR;
			goto next;
		}
		if (dst[0] == 0xff) { // :83-103
			uint8_t scope = dst[1] & 0x0f; // rte_ipv6_mc_scope [DPDK]
			if (scope == 0 || scope == 1) { // SCOPE_NONE, SCOPE_IFACELOCAL
				edge = GR_HIP_E_IP6_INPUT_BAD_ADDR;
				goto next;
			}
			// mcast6_get_member: multicast group state stays with grout's
			// CPU nodes, the packet is handed back whole
			terminal(m, GR_HIP_E_PUNT);
			continue;
		}
		switch (m->domain) { // :105-120
		case GR_HIP_ETH_DOMAIN_LOOPBACK:
		case GR_HIP_ETH_DOMAIN_LOCAL:
			break;
		case GR_HIP_ETH_DOMAIN_BROADCAST:
		case GR_HIP_ETH_DOMAIN_MULTICAST:
			edge = GR_HIP_E_IP6_INPUT_LOCAL;
			goto next;
		default:
			edge = GR_HIP_E_IP6_INPUT_OTHER_HOST;
			goto next;
		}
		nh = m->e_nh ? m->e_nh : fib6_lookup(t, iface->vrf_id, iface->id, dst, m->rss); // :124-131
		if (nh == 0) {
			edge = GR_HIP_E_IP6_ERROR_DEST_UNREACH;
			goto next;
		}
		const struct gr_hip_nh *h = &t->nh[nh];
		edge = t->in6_nh_edges[h->type]; // :133-135
		if (edge != NEXT)
			goto next;
		if (h->type == GR_HIP_NH_T_L3 && (h->flags & GR_HIP_NH_F_LOCAL)
		    && memcmp(dst, h->ipv6, 16) == 0) { // :137-145
			edge = GR_HIP_E_IP6_INPUT_LOCAL;
			goto next;
		}
		m->l3_nh = nh; // :151-153 (every edge: l3_mbuf_data nh)
		enqueue(g, GR_HIP_NODE_IP6_FORWARD, m);
		continue;
next:
		m->l3_nh = nh;
		terminal(m, edge);
	}
}

// ip6_forward_process, modules/ip6/datapath/ip6_forward.c:13-34
static void node_ip6_forward(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		uint8_t *ip = MTOD(m);
		if (ip[7] <= 1) { // hop_limits
			terminal(m, GR_HIP_E_IP6_ERROR_TTL_EXCEEDED);
			continue;
		}
		ip[7] -= 1;
		enqueue(g, GR_HIP_NODE_IP6_OUTPUT, m);
	}
}

// ip6_output_process, modules/ip6/datapath/ip6_output.c:58-145
static void node_ip6_output(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const uint8_t *ip = MTOD(m);
		uint8_t edge;
		if (m->l3_nh == 0) { // :75-79
			edge = GR_HIP_E_IP6_ERROR_DEST_UNREACH;
			goto next;
		}
		m->packet_type = 0x40; // :81, RTE_PTYPE_L3_IPV6 [DPDK rte_mbuf_ptype.h]
		const struct gr_hip_nh *h = &t->nh[m->l3_nh];
		edge = t->out6_nh_edges[h->type]; // :83-85
		if (edge != NEXT)
			goto next;
		// no multicast destination comes out of ip6_input here (:87-91)
		const struct gr_hip_iface *iface = iface_from_id(t, h->iface_id);
		if (iface == NULL) { // :92-95
			edge = GR_HIP_E_IP6_OUTPUT_ERROR;
			goto next;
		}
		if (m->pkt_len > iface->mtu) { // :97-100
			edge = GR_HIP_E_IP6_OUTPUT_TOO_BIG;
			goto next;
		}
		edge = t->out6_iface_edges[iface->type]; // :104
		m->iface = iface->id; // :105
		if (edge != NEXT)
			goto next;
		if (h->state != GR_HIP_NH_S_REACHABLE
		    || ((h->flags & GR_HIP_NH_F_LINK) && memcmp(ip + 24, h->ipv6, 16) != 0)) { // :111-117
			edge = GR_HIP_E_IP6_HOLD;
			goto next;
		}
		memcpy(m->eth_dst, h->mac, 6); // :119-134
		m->eth_type = be16(0x86dd);
		enqueue(g, GR_HIP_NODE_ETH_OUTPUT, m);
		continue;
next:
		terminal(m, edge);
	}
}

// eth_output_process, modules/infra/datapath/eth_output.c:27-77. The source
// MAC is looked up only when the iface differs from last_iface_id, which a
// failed lookup leaves as it was while zeroing the cached MAC (:51-58): in
// one walk, after an eth_output_no_mac packet, the next packet of the cached
// iface leaves with source MAC 00:00:00:00:00:00. The prepend cannot fail
// here (NO_HEADROOM, :43-49): eth_input's adj(14) left the headroom
// (gr_mbuf_prepend: modules/infra/datapath/mbuf.h:89-106).
static void node_eth_output(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	uint16_t last_iface_id = GR_HIP_IFACE_ID_UNDEF;
	uint8_t src_mac[6] = {0};
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		mbuf_prepend(m, 14);
		uint8_t *eth = MTOD(m);
		memcpy(eth, m->eth_dst, 6); // eth_output.c:50
		if (m->iface != last_iface_id) {
			const struct gr_hip_iface *iface = iface_from_id(t, m->iface);
			if (iface == NULL || !iface->mac_ok) { // iface_get_eth_addr() < 0
				memset(src_mac, 0, 6);
				terminal(m, GR_HIP_E_ETH_OUTPUT_NO_MAC);
				m->vlan_id = 0; // :71
				continue;
			}
			memcpy(src_mac, iface->mac, 6);
			last_iface_id = m->iface;
		}
		memcpy(eth + 6, src_mac, 6); // :59
		memcpy(eth + 12, &m->eth_type, 2); // :60
		m->vlan_id = 0; // :71
		enqueue(g, GR_HIP_NODE_IFACE_OUTPUT, m);
	}
}

// iface_output_process, modules/infra/datapath/iface_output.c:60-117
static void node_iface_output(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	const or_topo_t *t = g->t;
	for (uint16_t i = 0; i < n; i++) {
		struct or_mbuf *m = objs[i];
		const struct gr_hip_iface *d_iface = iface_from_id(t, m->iface);
		const struct gr_hip_iface *iface = d_iface, *parent = NULL;
		if (d_iface->type == GR_HIP_IFACE_TYPE_VLAN) { // :81-86
			m->vlan_id = d_iface->vlan_id;
			iface = iface_from_id(t, d_iface->parent_id);
			parent = iface;
		}
		if (iface == NULL) { // :94-97
			terminal(m, GR_HIP_E_IFACE_OUTPUT_VLAN_NO_PARENT);
			continue;
		}
		if (!(d_iface->flags & GR_HIP_IFACE_F_UP)) { // :98-101
			terminal(m, GR_HIP_E_IFACE_OUTPUT_ADMIN_DOWN);
			continue;
		}
		m->tx_counted = 1; // IFACE_STATS_INC :103-105
		m->tx_iface = d_iface->id;
		m->tx_parent = parent ? parent->id : 0;
		m->iface = iface->id;
		terminal(m, t->iout_type_edges[iface->type]); // :107-108
	}
}

static void mark(struct or_mbuf **objs, uint16_t n, int node) {
	for (uint16_t i = 0; i < n; i++)
		objs[i]->visited |= (uint16_t)(1u << node);
}

// One graph walk over a burst (rte_graph_walk from gr_datapath_loop,
// modules/infra/datapath/main_loop.c:459): iface_input on the RX burst, then
// the pending queue in order.
static void graph_walk(struct or_graph *g, struct or_mbuf **objs, uint16_t n) {
	mark(objs, n, GR_HIP_NODE_IFACE_INPUT);
	node_iface_input(g, objs, n);
	struct or_mbuf *batch[OR_BURST_MAX];
	while (g->pend_head != g->pend_tail) {
		const int node = g->pend[g->pend_head++ % (4 * GR_HIP_NODE_COUNT)];
		struct or_stream *s = &g->st[node];
		const uint16_t k = s->n;
		memcpy(batch, s->objs, k * sizeof(batch[0]));
		s->n = 0;
		mark(batch, k, node);
		switch (node) {
		case GR_HIP_NODE_ETH_INPUT:
			node_eth_input(g, batch, k);
			break;
		case GR_HIP_NODE_IP_INPUT:
			node_ip_input(g, batch, k);
			break;
		case GR_HIP_NODE_IP_FORWARD:
			node_ip_forward(g, batch, k);
			break;
		case GR_HIP_NODE_IP_OUTPUT:
			node_ip_output(g, batch, k);
			break;
		case GR_HIP_NODE_IP6_INPUT:
			node_ip6_input(g, batch, k);
			break;
		case GR_HIP_NODE_IP6_FORWARD:
			node_ip6_forward(g, batch, k);
			break;
		case GR_HIP_NODE_IP6_OUTPUT:
			node_ip6_output(g, batch, k);
			break;
		case GR_HIP_NODE_ETH_OUTPUT:
			node_eth_output(g, batch, k);
			break;
		case GR_HIP_NODE_IFACE_OUTPUT:
			node_iface_output(g, batch, k);
			break;
		}
	}
	g->pend_head = g->pend_tail = 0;
}

// Node counters of one walk as grout collects them (node_stats_callback,
// modules/infra/datapath/main_loop.c:40-66, over DPDK's per-node totals):
// calls = process() invocations, packets = their return values; ip_output
// returns only what it enqueued to eth_output (ip_output.c:153,162).
// Punted packets restart on grout's CPU nodes, which count them there.
static void walk_node_stats(struct or_mbuf *mb, uint16_t k, struct gr_hip_node_stats *ns) {
	uint32_t cnt[GR_HIP_NODE_COUNT] = {0}, sent4 = 0, sent6 = 0;
	for (uint16_t i = 0; i < k; i++) {
		if (mb[i].edge == GR_HIP_E_PUNT)
			continue;
		for (int j = 0; j < GR_HIP_NODE_COUNT; j++)
			cnt[j] += (mb[i].visited >> j) & 1;
		if (mb[i].visited & (1u << GR_HIP_NODE_ETH_OUTPUT)) { // ip(6)_output's return value
			sent4 += (mb[i].visited >> GR_HIP_NODE_IP_OUTPUT) & 1;
			sent6 += (mb[i].visited >> GR_HIP_NODE_IP6_OUTPUT) & 1;
		}
	}
	for (int j = 0; j < GR_HIP_NODE_COUNT; j++) {
		ns->calls[j] += cnt[j] != 0;
		ns->packets[j] += j == GR_HIP_NODE_IP_OUTPUT ? sent4 : j == GR_HIP_NODE_IP6_OUTPUT ? sent6 : cnt[j];
	}
}

static void rx_fill(struct or_mbuf *m, const uint8_t *frame, uint32_t copy, const struct gr_hip_pkt_meta *md) {
	m->data_off = OR_HEADROOM;
	memcpy(m->buf + OR_HEADROOM, frame, copy);
	m->data_len = md->pkt_len;
	m->pkt_len = md->pkt_len;
	m->orig_len = md->pkt_len;
	m->ck = (uint8_t)((md->vlan_ck >> 12) & 3);
	m->rss = md->rss;
	m->packet_type = 0;
	m->iface = md->iface;
	m->vlan_id = md->vlan_ck & 0xfff;
	m->domain = 0;
	m->e_nh = 0;
	m->l3_nh = 0;
	m->edge = 0;
	m->visited = 0;
	m->rx_counted = m->tx_counted = 0;
}

static void count_stats(const struct or_mbuf *m, struct gr_hip_iface_stats *st, uint32_t max) {
	if (st == NULL || m->edge == GR_HIP_E_PUNT)
		return;
	if (m->rx_counted) {
		if (m->rx_iface < max) {
			st[m->rx_iface].rx_packets++;
			st[m->rx_iface].rx_bytes += m->orig_len;
		}
		if (m->rx_parent && m->rx_parent < max) {
			st[m->rx_parent].rx_packets++;
			st[m->rx_parent].rx_bytes += m->orig_len;
		}
	}
	if (m->tx_counted) {
		if (m->tx_iface < max) {
			st[m->tx_iface].tx_packets++;
			st[m->tx_iface].tx_bytes += m->orig_len;
		}
		if (m->tx_parent && m->tx_parent < max) {
			st[m->tx_parent].tx_packets++;
			st[m->tx_parent].tx_bytes += m->orig_len;
		}
	}
}

int or_process(
	or_topo_t *t,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *v,
	struct gr_hip_iface_stats *stats,
	uint32_t flags
) {
	return or_process_ex(t, in_frames, in_stride, meta, n, out_lines, out_stride, v, stats, flags, NULL, NULL);
}

// One graph walk over frames in place (test measurement: the walk harness's
// "chain" node, tests/standin/walk_harness.c, runs grout's CPU chain on its
// own mbufs for the like-for-like comparison with the GPU node). mb[i].buf
// is set so that MTOD is frames[i]: the chain reads and rewrites each frame
// where it lies, as grout's nodes rewrite an mbuf's data. mo[i]: the mbuf
// state at the packet's edge (data_off relative to 128, as or_process_ex).
int or_walk_frames(
	const or_topo_t *t,
	uint8_t *const *frames,
	uint32_t readable,
	const struct gr_hip_pkt_meta *meta,
	uint16_t n,
	struct gr_hip_mbuf *mo
) {
	if (n > OR_BURST_MAX || (n && (frames == NULL || meta == NULL || mo == NULL)))
		return -EINVAL;
	struct or_graph g = {.t = t, .flags = 0, .readable = readable};
	struct or_mbuf mb[OR_BURST_MAX];
	struct or_mbuf *objs[OR_BURST_MAX];
	for (uint16_t i = 0; i < n; i++) {
		const struct gr_hip_pkt_meta *md = &meta[i];
		mb[i].buf = frames[i] - OR_HEADROOM;
		rx_fill(&mb[i], frames[i], 0, md);
		objs[i] = &mb[i];
	}
	graph_walk(&g, objs, n);
	for (uint16_t i = 0; i < n; i++) {
		const struct or_mbuf *m = &mb[i];
		const struct gr_hip_pkt_meta *md = &meta[i];
		const bool punt = m->edge == GR_HIP_E_PUNT;
		struct gr_hip_mbuf *b = &mo[i];
		b->pkt_len = punt ? md->pkt_len : m->pkt_len;
		b->data_len = (uint16_t)(punt ? md->pkt_len : m->data_len);
		b->data_off = (uint16_t)(punt ? OR_HEADROOM : m->data_off);
		b->packet_type = punt ? 0 : m->packet_type;
		b->iface = punt ? md->iface : m->iface;
		b->vlan_id = punt ? (md->vlan_ck & 0xfff) : m->vlan_id;
		b->edge = m->edge;
		b->domain = punt ? 0 : m->domain;
		b->nh = punt ? 0 : m->l3_nh;
	}
	return 0;
}

int or_process_ex(
	or_topo_t *t,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	void *out_lines,
	uint32_t out_stride,
	struct gr_hip_verdict *v,
	struct gr_hip_iface_stats *stats,
	uint32_t flags,
	struct gr_hip_mbuf *mo,
	struct gr_hip_node_stats *ns
) {
	if (in_stride < GR_HIP_LINE || out_stride < GR_HIP_LINE)
		return -EINVAL;
	uint32_t readable = (flags & GR_HIP_BATCH_F_LINES_ONLY) ? GR_HIP_LINE : in_stride;
	if (readable > OR_DATAROOM - OR_HEADROOM)
		readable = OR_DATAROOM - OR_HEADROOM;
	struct or_graph g = {.t = t, .flags = flags, .readable = readable};
	uint32_t burst = (flags >> OR_F_BURST_SHIFT) & 0x1ff; // mbuf walks: the walk length cap
	if (burst == 0 || burst > OR_BURST_MAX)
		burst = OR_BURST;
	struct or_mbuf mb[OR_BURST_MAX];
	struct or_mbuf *objs[OR_BURST_MAX];
	uint8_t *bufs = malloc((size_t)OR_BURST_MAX * OR_DATAROOM);
	if (bufs == NULL)
		return -ENOMEM;
	memset(bufs, 0, (size_t)OR_BURST_MAX * OR_DATAROOM);
	for (int i = 0; i < OR_BURST_MAX; i++)
		mb[i].buf = bufs + (size_t)i * OR_DATAROOM;
	const uint8_t *in = in_frames;
	uint8_t *out = out_lines;
	for (uint32_t base = 0, k; base < n; base += k) {
		// this graph walk: up to the next GR_HIP_META_WALK mark; for node
		// mbufs (OR_F_MBUF_WALKS) at most `burst` packets (graph.c:88-91,
		// 612-650), for a batch never past a multiple of 64 (include/grout_hip.h)
		uint32_t end = base + burst;
		if (!(flags & OR_F_MBUF_WALKS))
			end = (base / OR_BURST + 1) * OR_BURST;
		if (end > n)
			end = n;
		for (k = 1; base + k < end && !(meta[base + k].vlan_ck & GR_HIP_META_WALK); k++)
			;
		for (uint16_t i = 0; i < k; i++) {
			const struct gr_hip_pkt_meta *md = &meta[base + i];
			rx_fill(&mb[i], in + (size_t)(base + i) * in_stride, readable, md);
			objs[i] = &mb[i];
		}
		graph_walk(&g, objs, (uint16_t)k);
		for (uint16_t i = 0; i < k; i++) {
			const struct or_mbuf *m = &mb[i];
			struct gr_hip_verdict *o = &v[base + i];
			o->edge = m->edge;
			o->domain = m->domain;
			o->iface = m->iface;
			o->nh = m->l3_nh;
			if (m->edge == GR_HIP_E_PUNT) {
				o->domain = 0;
				o->iface = meta[base + i].iface;
				o->nh = 0;
			}
			// the frame start is OR_HEADROOM whatever data_off became
			memcpy(out + (size_t)(base + i) * out_stride, m->buf + OR_HEADROOM, GR_HIP_LINE);
			if (m->edge == GR_HIP_E_PUNT) // untouched copy of the input
				memcpy(out + (size_t)(base + i) * out_stride,
				       in + (size_t)(base + i) * in_stride, GR_HIP_LINE);
			count_stats(m, stats, t->max_ifaces);
			if (mo != NULL) { // the mbuf as grout leaves it at the edge (untouched if punted)
				struct gr_hip_mbuf *b = &mo[base + i];
				const struct gr_hip_pkt_meta *md = &meta[base + i];
				const bool punt = m->edge == GR_HIP_E_PUNT;
				memset(b, 0, sizeof(*b));
				b->pkt_len = punt ? md->pkt_len : m->pkt_len;
				b->data_len = (uint16_t)(punt ? md->pkt_len : m->data_len);
				b->data_off = (uint16_t)(punt ? OR_HEADROOM : m->data_off);
				b->packet_type = punt ? 0 : m->packet_type;
				b->rss = md->rss;
				b->iface = punt ? md->iface : m->iface;
				b->vlan_id = punt ? (md->vlan_ck & 0xfff) : m->vlan_id;
				b->ck = (uint8_t)((md->vlan_ck >> 12) & 3);
				b->edge = m->edge;
				b->domain = punt ? 0 : m->domain;
				b->nh = punt ? 0 : m->l3_nh;
			}
		}
		if (ns != NULL)
			walk_node_stats(mb, (uint16_t)k, ns);
	}
	free(bufs);
	return 0;
}

// ---------------------------------------------------------------------------
// CPU baseline
// ---------------------------------------------------------------------------

struct bench_arg {
	or_topo_t *t;
	const uint8_t *frames;
	uint32_t stride;
	const struct gr_hip_pkt_meta *meta;
	uint32_t n;
	uint32_t start; // this worker's first packet of the sample
	uint64_t todo;
	uint64_t forwarded;
	uint32_t flags;
	int cpu;
	int err;
	pthread_barrier_t *ready, *go;
};

// 2 MiB-aligned anonymous memory advised onto transparent huge pages (grout's
// rte_fib lives in EAL hugepages); *map / *len: what to munmap.
static void *thp_alloc(size_t bytes, void **map, size_t *len) {
	const size_t huge = (size_t)2 << 20;
	*len = ((bytes + huge - 1) & ~(huge - 1)) + huge;
	*map = mmap(NULL, *len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (*map == MAP_FAILED)
		return NULL;
	void *a = (void *)(((uintptr_t)*map + huge - 1) & ~(uintptr_t)(huge - 1));
	madvise(a, *len - (size_t)((uint8_t *)a - (uint8_t *)*map), MADV_HUGEPAGE);
	return a;
}

// A worker's own copy of the IPv4 FIBs (tbl24 on THP, tbl8), written by the
// worker itself so that its pages are on its NUMA node; the
// rest of the topology (ifaces, nexthops, reta, the IPv6 RIB) is shared,
// read-only.
struct fib_copies {
	or_topo_t t;
	void *maps[GR_HIP_MAX_IFACES];
	size_t lens[GR_HIP_MAX_IFACES];
};

static struct fib_copies *fib_copy(const or_topo_t *src) {
	struct fib_copies *c = calloc(1, sizeof(*c));
	if (c == NULL)
		return NULL;
	c->t = *src;
	c->t.fibs = calloc(src->max_ifaces, sizeof(struct or_fib));
	if (c->t.fibs == NULL) {
		free(c);
		return NULL;
	}
	memcpy(c->t.fibs, src->fibs, src->max_ifaces * sizeof(struct or_fib));
	for (uint32_t v = 0; v < src->max_ifaces && v < GR_HIP_MAX_IFACES; v++) {
		const struct or_fib *f = &src->fibs[v];
		struct or_fib *d = &c->t.fibs[v];
		d->tbl24 = NULL;
		d->tbl8 = NULL;
		if (f->tbl24 != NULL && (d->tbl24 = thp_alloc((size_t)8 << 24, &c->maps[v], &c->lens[v])) != NULL)
			memcpy(d->tbl24, f->tbl24, (size_t)8 << 24);
		if (f->tbl8 != NULL && f->num_tbl8 && (d->tbl8 = malloc((size_t)f->num_tbl8 * 256 * 8)) != NULL)
			memcpy(d->tbl8, f->tbl8, (size_t)f->num_tbl8 * 256 * 8);
		if ((f->tbl24 != NULL && d->tbl24 == NULL) || (f->tbl8 != NULL && f->num_tbl8 && d->tbl8 == NULL))
			d->exists = false; // no memory: never looked up (the worker reports it)
	}
	return c;
}

static void fib_copies_free(struct fib_copies *c) {
	if (c == NULL)
		return;
	for (uint32_t v = 0; v < c->t.max_ifaces && v < GR_HIP_MAX_IFACES; v++) {
		if (c->maps[v] != NULL && c->maps[v] != MAP_FAILED)
			munmap(c->maps[v], c->lens[v]);
		free(c->t.fibs[v].tbl8);
	}
	free(c->t.fibs);
	free(c);
}

// Bursts of OR_BURST from the sample, from `pos` on, wrapping; returns the
// packets forwarded (port_tx stand-in: net_null).
static uint64_t bench_run(struct or_graph *g, struct or_mbuf *mb, struct or_mbuf **objs, const struct bench_arg *a,
			  uint32_t *pos, uint64_t todo) {
	uint64_t done = 0, fwd = 0;
	while (done < todo) {
		for (uint16_t i = 0; i < OR_BURST; i++) {
			rx_fill(&mb[i], a->frames + (size_t)*pos * a->stride, GR_HIP_LINE, &a->meta[*pos]);
			objs[i] = &mb[i];
			if (++*pos == a->n)
				*pos = 0;
		}
		graph_walk(g, objs, OR_BURST);
		for (uint16_t i = 0; i < OR_BURST; i++)
			fwd += mb[i].edge == GR_HIP_E_PORT_OUTPUT;
		done += OR_BURST;
	}
	return fwd;
}

static void *bench_thread(void *p) {
	struct bench_arg *a = p;
	if (a->cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(a->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	struct fib_copies *own = (a->flags & OR_BENCH_FIB_COPY) ? fib_copy(a->t) : NULL;
	if ((a->flags & OR_BENCH_FIB_COPY) && own == NULL)
		a->err = -ENOMEM;
	// mbuf pool of the worker: OR_BURST mbufs re-filled by the rx stand-in
	// (the NIC DMA of a ring PMD: the 64-byte header line lands in the mbuf)
	struct or_mbuf mb[OR_BURST];
	struct or_mbuf *objs[OR_BURST];
	uint8_t *bufs = aligned_alloc(64, (size_t)OR_BURST * OR_DATAROOM);
	memset(bufs, 0, (size_t)OR_BURST * OR_DATAROOM);
	for (int i = 0; i < OR_BURST; i++)
		mb[i].buf = bufs + (size_t)i * OR_DATAROOM;
	struct or_graph g = {.t = own != NULL ? &own->t : a->t, .flags = 0, .readable = GR_HIP_LINE};
	// warm-up, untimed: one pass over the whole sample from this worker's
	// offset (its FIB pages, the nexthops and the sample in its caches / TLB)
	uint32_t pos = a->start;
	bench_run(&g, mb, objs, a, &pos, a->n);
	pthread_barrier_wait(a->ready);
	pthread_barrier_wait(a->go);
	a->forwarded = bench_run(&g, mb, objs, a, &pos, a->todo);
	free(bufs);
	fib_copies_free(own);
	return NULL;
}

static int bench_cpus[CPU_SETSIZE], bench_ncpus;

int or_bench_set_cpus(const int *cpus, int n) {
	if (n < 0 || n > CPU_SETSIZE)
		return -1;
	for (int i = 0; i < n; i++)
		if (cpus[i] < 0 || cpus[i] >= CPU_SETSIZE)
			return -1;
	if (n > 0)
		memcpy(bench_cpus, cpus, sizeof(int) * (size_t)n);
	bench_ncpus = n;
	return 0;
}

double or_bench(
	or_topo_t *t,
	const void *in_frames,
	uint32_t in_stride,
	const struct gr_hip_pkt_meta *meta,
	uint32_t n,
	int threads,
	uint64_t pkts_per_thread,
	uint32_t flags,
	uint64_t *forwarded
) {
	if (threads < 1 || n == 0)
		return -1.0;
	pthread_t th[threads];
	struct bench_arg args[threads];
	pthread_barrier_t ready, go;
	pthread_barrier_init(&ready, NULL, (unsigned)threads + 1);
	pthread_barrier_init(&go, NULL, (unsigned)threads + 1);
	// the CPUs this process may run on (a container's cpuset), in order, or
	// the placement or_bench_set_cpus gave: worker i is pinned to the i-th of
	// them when there are enough
	cpu_set_t allowed;
	int cpus[CPU_SETSIZE], ncpu = 0;
	if (bench_ncpus > 0) {
		memcpy(cpus, bench_cpus, sizeof(int) * (size_t)bench_ncpus);
		ncpu = bench_ncpus;
	} else if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
		for (int c = 0; c < CPU_SETSIZE; c++)
			if (CPU_ISSET(c, &allowed))
				cpus[ncpu++] = c;
	}
	for (int i = 0; i < threads; i++) {
		args[i] = (struct bench_arg) {
			.t = t,
			.frames = in_frames,
			.stride = in_stride,
			.meta = meta,
			.n = n,
			.start = (uint32_t)((uint64_t)i * n / (uint64_t)threads), // each worker its own part first
			.todo = (pkts_per_thread + OR_BURST - 1) / OR_BURST * OR_BURST,
			.flags = flags,
			.cpu = threads <= ncpu ? cpus[i] : -1,
			.ready = &ready,
			.go = &go,
		};
		pthread_create(&th[i], NULL, bench_thread, &args[i]);
	}
	struct timespec t0, t1;
	pthread_barrier_wait(&ready); // every worker has its FIB copy and is warm
	clock_gettime(CLOCK_MONOTONIC, &t0);
	pthread_barrier_wait(&go);
	uint64_t fwd = 0;
	int err = 0;
	for (int i = 0; i < threads; i++) {
		pthread_join(th[i], NULL);
		fwd += args[i].forwarded;
		err |= args[i].err;
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	pthread_barrier_destroy(&ready);
	pthread_barrier_destroy(&go);
	if (forwarded)
		*forwarded = fwd;
	if (err)
		return -1.0;
	double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
	return (double)args[0].todo * threads / s / 1e6;
}
