// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_pipe.hip -- the software-pipelined forwarding kernel for gfx950.
//
// Same node chain and results as fwd4_kernel.hip, laid out so that no wave
// ever waits on HBM or on its own stores:
//
//  * Each wave is independent (no workgroup barrier in the loop): it owns a
//    64-packet tile at a time and a private 4 KiB LDS image of the tile's
//    64-byte header lines (row r = packet r of the tile, 16-byte chunk j at
//    slot j ^ ((r >> 2) & 3), so both the coalesced 4-lanes-per-line fill and
//    the one-row-per-lane reads are free of bank conflicts).
//  * The next tile's metadata and lines are loaded into registers while the
//    current tile walks its dependent lookups (RX view -> FIB -> adjacency),
//    and the current tile's rewritten lines and verdicts are held in
//    registers and stored only after the NEXT tile's last lookup has been
//    issued. gfx9 retires loads, stores and LDS-DMA in issue order from one
//    vmcnt, so a load issued after a store cannot be consumed before the
//    store retires: issuing stores after the dependent loads keeps them off
//    the critical path.
//  * The RX view of a wave whose packets all come from one iface (one RX
//    queue per port) is read with a scalar load, off the vector counter.
//
// Node citations are the same as process() in fwd4_kernel.hip.
#include "fwd4_chain.h"

#define PIPE_WAVES 4 // waves per workgroup
#define PIPE_TILE 64 // packets per wave tile

template <bool STATS, bool NT>
__global__ void __launch_bounds__(PIPE_WAVES * 64) gr_fwd4_pipe(const fwd4_params A) {
	__shared__ __attribute__((aligned(16))) uint8_t lines[PIPE_WAVES * PIPE_TILE * 64];
	__shared__ stat_slot slots[FWD4_STAT_SLOTS];
	__shared__ fwd4_edges edges;
	const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
	const fwd4_tables *T = A.T;

	for (uint32_t i = tid; i < sizeof(fwd4_edges); i += PIPE_WAVES * 64)
		reinterpret_cast<uint8_t *>(&edges)[i] = reinterpret_cast<const uint8_t *>(&T->edges)[i];
	if (STATS && tid < FWD4_STAT_SLOTS) {
		slots[tid].key = 0;
		slots[tid].pkts = 0;
		slots[tid].bytes = 0;
	}
	kctx P;
	P.rx = T->rx;
	P.adj = T->adj;
	P.reta = T->reta;
	P.vlan_keys = T->vlan_keys;
	P.vlan_vals = T->vlan_vals;
	P.reta_cap = T->reta_cap;
	P.vlan_mask = T->vlan_mask;
	P.max_ifaces = T->max_ifaces;
	P.max_nh = T->max_nh;
	P.readable = A.readable;
	P.edges = &edges;
	P.stats = A.stats;
	__syncthreads();
	P.ip4_edge = ip4_edge_of(edges);

	uint8_t *R = lines + wv * (PIPE_TILE * 64);
	// Piece k of a tile (one 16-byte load per lane) covers rows 16k .. 16k+15,
	// four lanes per row; the chunk slot swizzle of those rows is lane-only.
	const uint32_t prow = lane >> 2, part = lane & 3;
	const uint32_t pslot = ((part ^ ((lane >> 4) & 3)) << 4);
	const uint32_t n_wt = (A.n + PIPE_TILE - 1) / PIPE_TILE;
	const uint32_t step = gridDim.x * PIPE_WAVES;
	uint32_t t = blockIdx.x * PIPE_WAVES + wv;

	u4v pf[4] = {};
	u2v pm = {0, 0};
	auto prefetch = [&](uint32_t tt) {
		const uint32_t base = tt * PIPE_TILE, cnt = min((uint32_t)PIPE_TILE, A.n - base);
		if (lane < cnt) {
			const u2v *mp = reinterpret_cast<const u2v *>(A.meta + base + lane);
			pm = NT ? __builtin_nontemporal_load(mp) : *mp;
		}
#pragma unroll
		for (uint32_t k = 0; k < 4; k++) {
			const uint32_t r = k * 16 + prow;
			if (r < cnt)
				pf[k] = ld16<NT>(A.in + (size_t)(base + r) * A.in_stride + part * 16);
		}
	};
	if (t < n_wt)
		prefetch(t);

	// the previous tile, stored after this tile's lookups are issued
	u4v ov[4] = {};
	u2v pv = {0, 0};
	uint32_t prev_base = 0, prev_cnt = 0;
	auto store_prev = [&]() {
#pragma unroll
		for (uint32_t k = 0; k < 4; k++) {
			const uint32_t r = k * 16 + prow;
			if (r < prev_cnt)
				st16<NT>(A.out + (size_t)(prev_base + r) * A.out_stride + part * 16, ov[k]);
		}
		if (lane < prev_cnt) {
			u2v *vp = reinterpret_cast<u2v *>(A.verdicts + prev_base + lane);
			if (NT)
				__builtin_nontemporal_store(pv, vp);
			else
				*vp = pv;
		}
	};

	for (; t < n_wt; t += step) {
		const uint32_t base = t * PIPE_TILE, cnt = min((uint32_t)PIPE_TILE, A.n - base);
		const bool live = lane < cnt;
		// land the prefetched lines in the wave's LDS image
#pragma unroll
		for (uint32_t k = 0; k < 4; k++)
			if (k * 16 + prow < cnt)
				*reinterpret_cast<u4v *>(R + (k * 16 + prow) * 64 + pslot) = pf[k];
		gr_hip_pkt_meta m = {0, 0, 0, 0};
		if (live) {
			m.iface = pm.x & 0xffff;
			m.vlan_ck = pm.x >> 16;
			m.pkt_len = pm.y & 0xffff;
			m.rss = pm.y >> 16;
		}
		compiler_fence();

		// RX view: scalar when the wave's packets share one iface
		const uint32_t if0 = __builtin_amdgcn_readfirstlane(m.iface);
		rxv rx;
		if (__ballot(live && m.iface != if0) == 0)
			rx = load_rx_scalar(P, if0);
		else
			rx = load_rx(P, m.iface);

		result r = {GR_HIP_E_PUNT, 0, m.iface, 0, 0, 0, 0, 0};
		uint32_t dst = 0, data_len = 0, slot = 0;
		bool go = false;
		if (live) {
			const uint8_t *frame = A.in + (size_t)(base + lane) * A.in_stride;
			go = pipe_head(P, R, lane, m, rx, r, dst, data_len, frame);
		}
		uint4 aa = {0, 0, 0, 0}, ab = {0, 0, 0, 0};
		if (go) {
			slot = pipe_fib(rx, dst);
			if (slot == 0 || slot > P.max_nh) {
				r.edge = GR_HIP_E_IP_ERROR_DEST_UNREACH; // NO_ROUTE :150-153
				go = false;
			} else {
				const uint4 *ap = reinterpret_cast<const uint4 *>(P.adj + slot);
				aa = gld4(ap);
				ab = gld4(ap + 1);
			}
		}

		// the previous tile leaves, the next one is requested
		if (prev_cnt)
			store_prev();
		const uint32_t tn = t + step;
		if (tn < n_wt)
			prefetch(tn);

		if (go)
			pipe_tail(P, R, lane, m, rx.flags, r, dst, data_len, slot, aa, ab);
		compiler_fence();
#pragma unroll
		for (uint32_t k = 0; k < 4; k++)
			ov[k] = *reinterpret_cast<const u4v *>(R + (k * 16 + prow) * 64 + pslot);
		pv = u2v{r.edge | (r.domain << 8) | (r.iface << 16), r.nh};
		prev_base = base;
		prev_cnt = cnt;

		if (STATS) {
			const uint32_t len = m.pkt_len;
			wave_count(slots, P, r.rx_if ? r.rx_if + 1 : 0, len);
			wave_count(slots, P, r.rx_par ? r.rx_par + 1 : 0, len);
			wave_count(slots, P, r.tx_if ? (r.tx_if | 0x10000u) + 1 : 0, len);
			wave_count(slots, P, r.tx_par ? (r.tx_par | 0x10000u) + 1 : 0, len);
		}
		compiler_fence();
	}
	if (prev_cnt)
		store_prev();

	if (STATS) {
		__syncthreads();
		if (tid < FWD4_STAT_SLOTS && slots[tid].key != 0) {
			const uint32_t key = slots[tid].key - 1;
			shard_add(A.stats, P.max_ifaces, key >> 16, key & 0xffff, slots[tid].pkts, slots[tid].bytes);
		}
	}
}

typedef void (*fwd4_pfn)(const fwd4_params);
static const fwd4_pfn pipe_kernels[4] = {
	gr_fwd4_pipe<false, false>,
	gr_fwd4_pipe<true, false>,
	gr_fwd4_pipe<false, true>,
	gr_fwd4_pipe<true, true>,
};

// variant: FWD4_V_STATS | FWD4_V_NT. grid: workgroups of PIPE_WAVES waves,
// each wave striding over 64-packet tiles.
extern "C" hipError_t gr_fwd4_pipe_launch(const fwd4_params *A, uint32_t grid, hipStream_t s, int variant) {
	hipLaunchKernelGGL(pipe_kernels[variant & 3], dim3(grid), dim3(PIPE_WAVES * 64), 0, s, *A);
	return hipGetLastError();
}

extern "C" int gr_fwd4_pipe_occupancy(int variant) {
	int b = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, pipe_kernels[variant & 3], PIPE_WAVES * 64, 0) != hipSuccess) {
		(void)hipGetLastError();
		return 0;
	}
	return b;
}
