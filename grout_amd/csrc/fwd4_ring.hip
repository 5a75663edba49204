// SPDX-License-Identifier: BSD-3-Clause
//
// fwd4_ring.hip -- the warp-specialised forwarding kernel for gfx950.
//
// gfx9 retires a wave's vector loads, stores and LDS-DMA in issue order
// from one counter (vmcnt), so a wave that streams header lines AND walks
// the dependent lookups (RX view -> FIB -> adjacency) pays the HBM latency
// of its streams at its first lookup. Here the two never share a wave:
//
//   loader waves:  LDS-DMA (global_load_lds) of each 64-packet tile's
//                  header lines and metadata into a ring slot, AHEAD tiles
//                  in flight per loader, published behind a counted vmcnt;
//   compute waves: the node chain of a tile out of its slot (only the
//                  dependent lookups on their vmcnt), rewritten rows and
//                  verdicts back into the slot;
//   storer waves:  drain finished slots to HBM (coalesced 16-byte stores)
//                  and hand them back to the loaders.
// The geometry (waves, loaders, storers, slots, AHEAD) is a ring_cfg; tile
// k of a workgroup goes to loader k % LOADERS, compute wave k % COMPUTE,
// storer k % STORERS and slot k % SLOTS.
//
// The hand-offs are LDS words with tile sequence numbers: ready[s] (loader
// -> compute), done[s] (compute -> storer), free[s] (storer -> loader).
// Every wait is bounded (RING_SPIN_MAX polls); a wave that gives up sets
// the workgroup's abort word and every role leaves its loop, so the grid
// always drains; the workgroup then reports it in *A.err (the queue's error
// word: the next sync returns -ETIMEDOUT). Tiles of a workgroup are b,
// b + G, b + 2G ... (G = grid), or one contiguous run per workgroup
// (fwd4_params.chunk).
#include "fwd4_chain.h"

#define RING_GLDS_PER_TILE 6 // 4 x 1 KiB of lines + 2 x 256 B of metadata
#define RING_SPIN_MAX (1u << 24)
#define RING_NHF_LDS_MAX 2304 // fast adjacencies staged in LDS (36 KiB)

template <int WAVES_, int LOADERS_, int STORERS_, int SLOTS_, int AHEAD_>
struct ring_cfg {
	static constexpr uint32_t WAVES = WAVES_, LOADERS = LOADERS_, STORERS = STORERS_;
	static constexpr uint32_t COMPUTE = WAVES_ - LOADERS_ - STORERS_;
	static constexpr uint32_t SLOTS = SLOTS_, AHEAD = AHEAD_;
	// vmcnt that leaves AHEAD - 1 tiles of one loader in flight
	static constexpr int VMCNT_AHEAD = RING_GLDS_PER_TILE * (AHEAD_ - 1);
	static_assert(COMPUTE >= 1 && SLOTS_ >= LOADERS_ * AHEAD_ && VMCNT_AHEAD <= 63, "ring geometry");
};

// The measured geometries (gr_hip_tune "ring"); 0 is the default.
typedef ring_cfg<8, 1, 1, 8, 4> ring_cfg0;
typedef ring_cfg<8, 2, 1, 8, 3> ring_cfg1;
typedef ring_cfg<16, 2, 2, 16, 4> ring_cfg2;
typedef ring_cfg<12, 2, 1, 12, 4> ring_cfg3;
typedef ring_cfg<8, 1, 1, 8, 6> ring_cfg4;
typedef ring_cfg<16, 2, 2, 16, 6> ring_cfg5;
typedef ring_cfg<16, 3, 1, 20, 4> ring_cfg6;
typedef ring_cfg<16, 4, 2, 24, 3> ring_cfg7;
typedef ring_cfg<16, 2, 2, 16, 8> ring_cfg8;
// two workgroups per CU (8 slots each): more compute waves per CU
typedef ring_cfg<14, 1, 1, 8, 8> ring_cfg9;
typedef ring_cfg<14, 2, 2, 8, 4> ring_cfg10;
typedef ring_cfg<12, 1, 1, 8, 8> ring_cfg11;
// geometry 2 with lanes [0, SG) of each FIB gather through the scalar cache
// (fib_tbl24_split): 12, 13, 14 = SG 16, 32, 64
#define RING_NCFG 15

template <class C, bool PTRS>
struct ring_lds {
	uint8_t lines[C::SLOTS][64 * 64]; // the tile's header lines (fwd4_chain.h image)
	u2v meta[C::SLOTS][64]; // gr_hip_pkt_meta in, then the lane's gr_hip_verdict out
	uint64_t ptrs[PTRS ? C::SLOTS : 1][64]; // GR_HIP_BATCH_F_FRAME_PTRS: the tile's frames
	uint32_t ready[C::SLOTS], done[C::SLOTS], free_[C::SLOTS];
	uint32_t abort;
	uint32_t spin_max;
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
	return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// LDS-DMA: 16 (or 4) bytes per active lane from gsrc to lds_base + lane * 16 (or 4).
template <bool NT>
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_base) {
	uint32_t keep;
	if (NT)
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_base)
			     : "memory");
	else
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_base)
			     : "memory");
}

template <bool NT>
__device__ __forceinline__ void glds4(const void *gsrc, uint32_t lds_base) {
	uint32_t keep;
	if (NT)
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_base)
			     : "memory");
	else
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_base)
			     : "memory");
}

__device__ __forceinline__ uint32_t flag_get(const uint32_t *f) {
	return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void flag_set(uint32_t *f, uint32_t v) {
	compiler_fence();
	__hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Wait until *f >= want. False when the wait gave up or another wave did.
template <class L_t>
__device__ __forceinline__ bool flag_wait(L_t &L, const uint32_t *f, uint32_t want) {
	const uint32_t lim = L.spin_max;
	for (uint32_t spin = 0;; spin++) {
		if ((int32_t)(flag_get(f) - want) >= 0)
			return true;
		if (flag_get(&L.abort))
			return false;
		if (spin >= lim) {
			flag_set(&L.abort, 1);
			return false;
		}
		__builtin_amdgcn_s_sleep(1);
	}
}

// This workgroup's index and the workgroup count in the tile order: the
// launch's, or the resident kernel's per-batch ones (fwd4_params.wgs).
__device__ __forceinline__ uint32_t wg_id(const fwd4_params &A) {
	return A.wgs ? A.wg0 : blockIdx.x;
}
__device__ __forceinline__ uint32_t wg_count(const fwd4_params &A) {
	return A.wgs ? A.wgs : gridDim.x;
}

// Tile k of this workgroup (see fwd4_params.chunk).
__device__ __forceinline__ uint32_t tile_of(const fwd4_params &A, uint32_t k) {
	const uint32_t b = wg_id(A), G = wg_count(A);
	if (A.order == 2) { // XCD x = b % 8 interleaves its workgroups over region x
		const uint32_t x = b & 7, l = b >> 3, per = G >> 3;
		return x * A.chunk + l + k * per;
	}
	if (A.order == 3) { // runs of A.chunk tiles: the grid's window moves as in order 0,
		const uint32_t j = k / A.chunk; // each CU's tiles come in contiguous runs
		return (j * G + b) * A.chunk + (k - j * A.chunk);
	}
	return A.chunk ? b * A.chunk + k : b + k * G;
}

// How many tiles this workgroup takes (tile_of's k ranges over [0, that)).
__device__ __forceinline__ uint32_t local_tiles(const fwd4_params &A) {
	if (A.wgs && A.wg0 >= A.wgs)
		return 0; // a resident ring beyond the batch's split: its seq only
	const uint32_t n_tiles = (A.n + 63) >> 6, b = wg_id(A), G = wg_count(A);
	if (A.order == 2) {
		const uint32_t x = b & 7, l = b >> 3, per = G >> 3;
		const uint32_t lo = x * A.chunk + l, hi = min((x + 1) * A.chunk, n_tiles);
		return lo < hi ? (hi - 1 - lo) / per + 1 : 0;
	}
	if (A.order == 3) {
		const uint32_t S = G * A.chunk, r = n_tiles % S, b0 = b * A.chunk;
		return n_tiles / S * A.chunk + (r > b0 ? min(A.chunk, r - b0) : 0);
	}
	if (A.chunk)
		return b * A.chunk < n_tiles ? min(A.chunk, n_tiles - b * A.chunk) : 0;
	return b < n_tiles ? (n_tiles - 1 - b) / G + 1 : 0;
}

// Frame pointers of tile t, one per lane (rows past the batch repeat its last
// packet, so that every tile issues the same number of loads).
__device__ __forceinline__ uint64_t load_ptr(const fwd4_params &A, uint32_t t, uint32_t lane) {
	const uint32_t i = min(t * 64 + lane, A.n - 1);
	return gld(reinterpret_cast<const uint64_t *>(A.in) + i);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
	const uint32_t lo = __shfl((uint32_t)v, (int)src, 64), hi = __shfl((uint32_t)(v >> 32), (int)src, 64);
	return ((uint64_t)hi << 32) | lo;
}

// Every tile issues exactly RING_GLDS_PER_TILE LDS-DMA loads (rows and
// metadata past a ragged last tile repeat its last packet into rows nobody
// reads), so that the counted vmcnt waits below stay exact. In PTRS mode a
// loader also loads the next tile's frame pointers ahead (one more load per
// tile, issued before the tile's DMA, which only makes the waits longer).
template <class C, bool NT, bool PTRS, class LT>
__device__ void ring_loader(const fwd4_params &A, LT &L, uint32_t n_local, uint32_t j, uint32_t lane) {
	const uint32_t prow = lane >> 2;
	const uint32_t pchunk = (lane & 3) ^ ((lane >> 4) & 3); // chunk this lane lands in slot lane & 3
	uint32_t pub = j; // oldest of this loader's tiles not yet published
	bool ok = true;
	uint64_t pnext = 0;
	if (PTRS && j < n_local)
		pnext = load_ptr(A, tile_of(A, j), lane);
	for (uint32_t k = j; k < n_local && ok; k += C::LOADERS) {
		const uint32_t s = k % C::SLOTS;
		if (k >= C::SLOTS && (int32_t)(flag_get(&L.free_[s]) - (k - C::SLOTS + 1)) < 0) {
			// ring full: publish what is in flight, then wait for the storer
			wait_vmcnt<0>();
			for (; pub < k; pub += C::LOADERS)
				flag_set(&L.ready[pub % C::SLOTS], pub + 1);
			ok = flag_wait(L, &L.free_[s], k - C::SLOTS + 1);
			if (!ok)
				break;
		}
		const uint32_t t = tile_of(A, k);
		const uint32_t base = t * 64, last = min(64u, A.n - base) - 1;
		uint64_t pk = 0;
		if (PTRS) {
			pk = pnext;
			if (k + C::LOADERS < n_local)
				pnext = load_ptr(A, tile_of(A, k + C::LOADERS), lane);
			if (k == j)
				wait_vmcnt<0>();
			else
				wait_vmcnt<RING_GLDS_PER_TILE>(); // pk's load is older than the last tile's DMA
			L.ptrs[s][lane] = pk; // for the storer and the compute waves
		}
		const uint32_t lb = lds_addr(L.lines[s]);
#pragma unroll
		for (uint32_t q = 0; q < 4; q++) {
			const uint32_t r = min(q * 16 + prow, last);
			const uint8_t *src = PTRS ? reinterpret_cast<const uint8_t *>(shfl64(pk, r))
						  : A.in + (size_t)(base + r) * A.in_stride;
			glds16<NT>(src + pchunk * 16, lb + q * 1024);
		}
		const uint32_t mb = lds_addr(L.meta[s]);
		const uint8_t *msrc = reinterpret_cast<const uint8_t *>(A.meta + base);
#pragma unroll
		for (uint32_t q = 0; q < 2; q++) {
			// 4 bytes per lane: packet q * 32 + lane / 2, half lane & 1
			const uint32_t pkt = min(q * 32 + (lane >> 1), last);
			glds4<NT>(msrc + pkt * 8 + (lane & 1) * 4, mb + q * 256);
		}
		if (k - pub == (C::AHEAD - 1) * C::LOADERS) {
			wait_vmcnt<C::VMCNT_AHEAD>();
			flag_set(&L.ready[pub % C::SLOTS], pub + 1);
			pub += C::LOADERS;
		}
	}
	wait_vmcnt<0>();
	if (ok)
		for (; pub < n_local; pub += C::LOADERS)
			flag_set(&L.ready[pub % C::SLOTS], pub + 1);
}

template <class C, bool NT, bool PTRS, class LT>
__device__ void ring_storer(const fwd4_params &A, LT &L, uint32_t n_local, uint32_t j, uint32_t lane) {
	const uint32_t prow = lane >> 2, part = lane & 3;
	const uint32_t pslot = (part ^ ((lane >> 4) & 3)) << 4;
	const bool prefix = A.out_stride == GR_HIP_PREFIX; // packed 32-byte prefixes (whole lines are >= 64)
	for (uint32_t k = j; k < n_local; k += C::STORERS) {
		const uint32_t s = k % C::SLOTS;
		if (!flag_wait(L, &L.done[s], k + 1))
			break;
		const uint32_t t = tile_of(A, k);
		const uint32_t base = t * 64, cnt = min(64u, A.n - base);
		u4v o[4];
#pragma unroll
		for (uint32_t q = 0; q < 4; q++)
			o[q] = *reinterpret_cast<const u4v *>(&L.lines[s][(q * 16 + prow) * 64 + pslot]);
		const u2v v = L.meta[s][lane];
		uint8_t *dst[4];
#pragma unroll
		for (uint32_t q = 0; q < 4; q++) {
			const uint32_t r = q * 16 + prow;
			// in place at each frame (PTRS without out lines), else the lines
			dst[q] = PTRS && A.out == nullptr ? reinterpret_cast<uint8_t *>(L.ptrs[s][r])
							  : A.out + (size_t)(base + r) * A.out_stride;
		}
		// the registers hold the tile: hand the slot back before storing
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		flag_set(&L.free_[s], k + 1);
#pragma unroll
		for (uint32_t q = 0; q < 4; q++) {
			const uint32_t r = q * 16 + prow;
			if (r < cnt && (!prefix || part < 2)) // GR_HIP_BATCH_F_PREFIX32: bytes 0-31 only
				st16<NT>(dst[q] + part * 16, o[q]);
		}
		if (lane < cnt) {
			u2v *vp = reinterpret_cast<u2v *>(A.verdicts + base + lane);
			if (NT)
				__builtin_nontemporal_store(v, vp);
			else
				*vp = v;
		}
	}
}

// The tbl24 gather of a wave's IPv4 lanes (chain_fib's first load, 4-byte
// DIR24_8 of one VRF), SG of them through the scalar cache. A vector gather
// of 64 unrelated destinations is 64 L1 tag lookups and translations, and the
// addresser stalls on the L1's translations in flight (DESIGN.md §6.1:
// TCP_UTCL1_STALL_INFLIGHT_MAX); lanes [0, SG) go through the scalar cache
// instead, which has its own translation path: one readlane and one scalar
// load per lane, all issued before the vector gather of the other lanes and
// waited for together. Wave-uniform control flow only. Returns true for the
// lanes whose entry is in `ent` (the others call chain_fib). The scalar cache
// is not invalidated by anything but a launch, so only gr_fwd4_ring uses this
// (the resident kernel sees FIB updates between its batches).
template <int SG>
__device__ __forceinline__ bool fib_tbl24_split(const rxv &rx, uint32_t dst, bool want, uint32_t lane, uint32_t &ent) {
	want = want && rx.tbl24 != nullptr && (rx.flags & (FWD4_RX_FIB16 | FWD4_RX_FIB24W2)) == 0;
	const uint64_t wm = __ballot(want);
	if (wm == 0)
		return false;
	const uint32_t f = (uint32_t)__builtin_ctzll(wm);
	const uint64_t tb = reinterpret_cast<uint64_t>(rx.tbl24);
	const uint32_t blo = __builtin_amdgcn_readlane((uint32_t)tb, f);
	const uint32_t bhi = __builtin_amdgcn_readlane((uint32_t)(tb >> 32), f);
	want = want && (uint32_t)tb == blo && (uint32_t)(tb >> 32) == bhi; // the first lane's VRF
	const uint32_t idx = want ? __builtin_bswap32(dst) >> 8 : 0; // entry 0 for the others: a harmless read
	const __attribute__((address_space(4))) uint32_t *base =
		(const __attribute__((address_space(4))) uint32_t *)(((uint64_t)bhi << 32) | blo);
	uint32_t sv[SG];
#pragma unroll
	for (int i = 0; i < SG; i++)
		sv[i] = base[(uint32_t)__builtin_amdgcn_readlane(idx, i)];
	uint32_t v = 0, w = 0;
	if (want && lane >= (uint32_t)SG)
		v = gld(rx.tbl24 + idx);
	// into their own register, so that waiting for the scalar loads does not
	// wait for the vector gather too
#pragma unroll
	for (int i = 0; i < SG; i++)
		asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"(sv[i]), "i"(i));
	ent = lane < (uint32_t)SG ? w : v;
	return want;
}

template <class C, bool STATS, bool PTRS, int SG = 0, class LT>
__device__ void ring_compute(const fwd4_params &A, const kctx &P, LT &L, stat_slot *slots,
			     const uint4 *nhf_lds, uint32_t n_local, uint32_t c, uint32_t lane) {
	for (uint32_t k = c; k < n_local; k += C::COMPUTE) {
		const uint32_t s = k % C::SLOTS;
		if (!flag_wait(L, &L.ready[s], k + 1))
			break;
		const uint32_t t = tile_of(A, k);
		const uint32_t base = t * 64, cnt = min(64u, A.n - base);
		const bool live = lane < cnt;
		uint8_t *R = L.lines[s];
		gr_hip_pkt_meta m = {0, 0, 0, 0};
		if (live) {
			const u2v pm = L.meta[s][lane];
			m.iface = pm.x & 0xffff;
			m.vlan_ck = pm.x >> 16;
			m.pkt_len = pm.y & 0xffff;
			m.rss = pm.y >> 16;
		}
		const uint32_t if0 = __builtin_amdgcn_readfirstlane(m.iface);
		rxv rx;
		if (__ballot(live && m.iface != if0) == 0)
			rx = load_rx_scalar(P, if0);
		else
			rx = load_rx(P, m.iface);

		result r = {GR_HIP_E_PUNT, 0, m.iface, 0, 0, 0, 0, 0};
		uint32_t fam = 0; // the packet entered ip_input (1) / ip6_input (2)
		// from the FIB's nexthop slot to the verdict
		auto tail4 = [&](uint32_t slot, uint32_t dst, uint32_t data_len) {
			if (slot == 0 || slot > P.max_nh) {
				r.edge = GR_HIP_E_IP_ERROR_DEST_UNREACH; // NO_ROUTE :150-153
			} else {
				// fast adjacency: from LDS for the first slots, else one 16-byte gather
				const uint4 f = slot <= A.nhf_lds ? nhf_lds[slot - 1] : gld4(tload(&P.T->nhf) + slot);
				if (f.w >> 16) {
					fast_tail(R, lane, r, data_len, slot, f);
				} else {
					const uint4 *ap = reinterpret_cast<const uint4 *>(tload(&P.T->adj) + slot);
					chain_tail(P, R, lane, m, rx.flags, r, dst, data_len, slot, gld4(ap), gld4(ap + 1));
				}
			}
		};
		// the IPv6 chain (trie walk included) waits on dependent loads: its
		// wave issues ahead of the streaming waves (s_setprio) until it leaves
		// it; the IPv4 chain and the ring waits keep the default (raising them
		// costs IPv4)
		auto tail6 = [&](uint32_t data_len) {
			__builtin_amdgcn_s_setprio(2);
			chain6(P, R, lane, m, rx, r, data_len);
			__builtin_amdgcn_s_setprio(0);
		};
		if constexpr (SG == 0) {
			if (live) {
				uint32_t dst = 0, data_len = 0;
				const uint8_t *frame = PTRS ? reinterpret_cast<const uint8_t *>(L.ptrs[s][lane])
							    : A.in + (size_t)(base + lane) * A.in_stride;
				const int head = chain_head(P, R, lane, m, rx, r, dst, data_len, frame);
				fam = head == HEAD_IN4 || head == HEAD_IP4 ? 1 : head == HEAD_IP6 ? 2 : 0;
				if (head == HEAD_IP4)
					tail4(chain_fib(rx, dst), dst, data_len);
				else if (head == HEAD_IP6)
					tail6(data_len);
			}
		} else { // the tbl24 gathers wave-wide, between the head and the tails
			uint32_t dst = 0, data_len = 0;
			int head = HEAD_DONE;
			if (live) {
				const uint8_t *frame = PTRS ? reinterpret_cast<const uint8_t *>(L.ptrs[s][lane])
							    : A.in + (size_t)(base + lane) * A.in_stride;
				head = chain_head(P, R, lane, m, rx, r, dst, data_len, frame);
				fam = head == HEAD_IN4 || head == HEAD_IP4 ? 1 : head == HEAD_IP6 ? 2 : 0;
			}
			uint32_t ent = 0;
			const bool got = fib_tbl24_split<SG>(rx, dst, head == HEAD_IP4, lane, ent);
			if (live) {
				if (head == HEAD_IP4) {
					uint32_t slot = ent; // chain_fib's tbl8 step, or all of it
					if (!got)
						slot = chain_fib(rx, dst);
					else if (ent & 0x80000000u)
						slot = gld(rx.tbl8 + (size_t)(ent & 0x7fffffffu) * 256 + (__builtin_bswap32(dst) & 0xff));
					tail4(slot, dst, data_len);
				} else if (head == HEAD_IP6) {
					tail6(data_len);
				}
			}
		}
		if (__ballot(r.edge == GR_HIP_E_ETH_OUTPUT_NO_MAC) != 0
		    && eth_output_walks(P, lane, live, (m.vlan_ck & GR_HIP_META_WALK) != 0, fam, r)) {
			u4v c0 = lds_get(R, lane, 0); // source MAC, bytes 6-11: zero
			c0.y &= 0xffffu;
			c0.z = 0;
			lds_put(R, lane, 0, c0);
		}
		L.meta[s][lane] = u2v{r.edge | (r.domain << 8) | (r.iface << 16), r.nh};
		flag_set(&L.done[s], k + 1);
		if (STATS) {
			const uint32_t len = m.pkt_len;
			wave_count(slots, P, r.rx_if ? r.rx_if + 1 : 0, len);
			wave_count(slots, P, r.rx_par ? r.rx_par + 1 : 0, len);
			wave_count(slots, P, r.tx_if ? (r.tx_if | 0x10000u) + 1 : 0, len);
			wave_count(slots, P, r.tx_par ? (r.tx_par | 0x10000u) + 1 : 0, len);
		}
	}
}

#ifdef RING_TRACE
#define RING_TRACE_MAX 4096
__device__ uint64_t ring_trace[2 * RING_TRACE_MAX];
extern "C" int gr_fwd4_ring_trace(uint64_t *out, uint32_t n) {
	if (n > 2 * RING_TRACE_MAX)
		n = 2 * RING_TRACE_MAX;
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(ring_trace), n * sizeof(uint64_t)) == hipSuccess ? 0 : -5;
}
#endif

template <class C, bool STATS, bool NT, bool PTRS = false, int SG = 0>
__global__ void __launch_bounds__(C::WAVES * 64) gr_fwd4_ring(const fwd4_params A) {
#ifdef RING_TRACE
	if (threadIdx.x == 0 && blockIdx.x < RING_TRACE_MAX)
		ring_trace[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
	__shared__ __attribute__((aligned(16))) ring_lds<C, PTRS> L;
	__shared__ stat_slot slots[FWD4_STAT_SLOTS];
	__shared__ fwd4_edges edges;
	extern __shared__ __attribute__((aligned(16))) uint4 nhf_lds[]; // [A.nhf_lds]: slots 1.., then [A.nhf6_lds]
	const uint32_t tid = threadIdx.x, lane = tid & 63;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	const fwd4_tables *T = A.T;

	{
		const uint4 *src = reinterpret_cast<const uint4 *>(T->nhf) + 1;
		for (uint32_t i = tid; i < A.nhf_lds; i += C::WAVES * 64)
			nhf_lds[i] = gld4(src + i);
		const uint4 *src6 = reinterpret_cast<const uint4 *>(T->nhf6) + 1;
		for (uint32_t i = tid; i < A.nhf6_lds; i += C::WAVES * 64)
			nhf_lds[A.nhf_lds + i] = gld4(src6 + i);
		uint32_t *top6 = reinterpret_cast<uint32_t *>(nhf_lds + A.nhf_lds + A.nhf6_lds);
		for (uint32_t i = tid; i < A.top6_lds; i += C::WAVES * 64)
			top6[i] = gld(A.top6 + FWD4_TOP6_BASE + i);
	}
	for (uint32_t i = tid; i < sizeof(fwd4_edges); i += C::WAVES * 64)
		reinterpret_cast<uint8_t *>(&edges)[i] = reinterpret_cast<const uint8_t *>(&T->edges)[i];
	if (tid < C::SLOTS) {
		L.ready[tid] = 0;
		L.done[tid] = 0;
		L.free_[tid] = 0;
	}
	if (tid == 0) {
		L.abort = 0;
		L.spin_max = A.spin_max ? A.spin_max : RING_SPIN_MAX;
	}
	if (STATS && tid < FWD4_STAT_SLOTS) {
		slots[tid].key = 0;
		slots[tid].pkts = 0;
		slots[tid].bytes = 0;
	}
	__syncthreads();

	const uint32_t n_local = local_tiles(A);
	if (wv < C::LOADERS) {
		ring_loader<C, NT, PTRS>(A, L, n_local, wv, lane);
	} else if (wv < C::LOADERS + C::STORERS) {
		ring_storer<C, NT, PTRS>(A, L, n_local, wv - C::LOADERS, lane);
	} else {
		kctx P = make_kctx(A, &edges);
		P.nhf6_lds = (const __attribute__((address_space(3))) u4v *)(nhf_lds + A.nhf_lds);
		P.nhf6_n = A.nhf6_lds;
		P.top6 = A.top6;
		P.top6_lds = (const __attribute__((address_space(3))) uint32_t *)(nhf_lds + A.nhf_lds + A.nhf6_lds);
		P.top6_n = A.top6_lds;
		ring_compute<C, STATS, PTRS, SG>(A, P, L, slots, nhf_lds, n_local, wv - C::LOADERS - C::STORERS, lane);
	}

	__syncthreads(); // every role has left its loop (each wait is bounded)
	if (tid == 0 && L.abort && A.err != nullptr)
		__hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	if (STATS) {
		if (tid < FWD4_STAT_SLOTS && slots[tid].key != 0) {
			const uint32_t key = slots[tid].key - 1;
			shard_add(A.stats, T->max_ifaces, key >> 16, key & 0xffff, slots[tid].pkts, slots[tid].bytes);
		}
	}
#ifdef RING_TRACE
	// measurement builds: when each workgroup started and finished (s_memrealtime, 100 MHz)
	__syncthreads();
	if (tid == 0 && blockIdx.x < RING_TRACE_MAX) {
		ring_trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
	}
#endif
}

// ---- the resident kernel ----------------------------------------------------
// One long-lived launch per context (gr_hip.cpp, knob "resident"): workgroup
// r serves descriptor ring r (fwd4_res_desc in pinned host memory). It waits
// for the ring's next seq, copies that batch's fwd4_params into LDS, runs the
// three roles over its share of the batch's tiles (tile order 0 over the
// queue's rings: wg0 of wgs), makes those writes visible to the host and
// stores the seq into done[r]. No launch and no hardware queue per batch: what small host batches
// pay otherwise. A workgroup idle past its lifetime sets
// *stop, and every workgroup leaves at *stop (host's or that one's) after the
// batch it is running (its waits are bounded as in a launch), so the grid
// always drains; each then marks its ring's exited word. Counters are the
// hand-back's (no STATS variant), adjacencies are read from the global
// tables (nothing staged).
typedef ring_cfg2 ring_cfg_res;

__device__ __forceinline__ uint64_t sys_load64(const uint64_t *p) {
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(ring_cfg_res::WAVES * 64) gr_fwd4_resident(const fwd4_res_params R) {
	typedef ring_cfg_res C;
	__shared__ __attribute__((aligned(16))) ring_lds<C, true> L;
	__shared__ __attribute__((aligned(16))) fwd4_params A;
	__shared__ fwd4_edges edges;
	__shared__ uint64_t seq_s;
	__shared__ uint32_t go;
	const uint32_t tid = threadIdx.x, lane = tid & 63;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	uint64_t *done = R.done + (size_t)blockIdx.x * R.stride;
	const fwd4_res_desc *ring = R.descs + (size_t)blockIdx.x * R.ndesc;
	uint64_t idle_since = __builtin_amdgcn_s_memrealtime(); // thread 0's: its last batch done
	if (tid == 0) {
		seq_s = sys_load64(done) + 1; // a relaunch resumes after the last batch done
		go = __hip_atomic_load(R.taken + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
	__syncthreads();
	if (go == 0) { // no queue holds this ring: nothing to poll (a queue taking it relaunches)
		if (tid == 0)
			__hip_atomic_store(R.exited + (size_t)blockIdx.x * R.stride, R.launch_id, __ATOMIC_RELEASE,
					   __HIP_MEMORY_SCOPE_SYSTEM);
		return;
	}
	// a queue's first ring polls its descriptor in host memory at full rate;
	// its helper rings (taken 2: batches of more than 8 tiles reach them) poll
	// their wake word in device memory, which the first ring's workgroup
	// writes when it takes a batch split over them, backed off to R.nap_max,
	// and read the stop word over PCIe only every 16th poll
	const bool helper = go == 2;
	const uint32_t nap_max = helper ? R.nap_max : 1;
	const uint32_t stop_every = helper ? 15u : 3u; // mask
	const uint64_t *wake = R.wake + (size_t)blockIdx.x * R.stride;
	__syncthreads(); // every wave has read go
	uint32_t nap = 1; // idle polls back off
	for (;;) {
		if (tid == 0) {
			const uint64_t want = seq_s;
			const fwd4_res_desc *d = ring + want % R.ndesc;
			uint32_t g = 0;
			for (uint32_t poll = 0;; poll++) {
				if ((poll & stop_every) == 0
				    && __hip_atomic_load(R.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
					break; // every workgroup leaves: the host relaunches once all have
				// relaxed polls (they bypass the caches; an acquire would invalidate
				// this XCD's L2 on every poll, which idle rings then do all the
				// time), one acquire fence once the batch is there
				if ((!helper || __hip_atomic_load(wake, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want)
				    && __hip_atomic_load(&d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == want) {
					__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
					g = 1;
					break;
				}
				// idle past the lifetime, and so is every ring (the last batch
				// any workgroup finished, *R.active): the kernel leaves. Helpers
				// leave with the first rings, never of their own accord
				const uint64_t now = __builtin_amdgcn_s_memrealtime();
				if (!helper && now - idle_since > R.lifetime) {
					const uint64_t act = __hip_atomic_load(R.active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if (act > now || now - act <= R.lifetime) {
						idle_since = act > now ? now : act; // another ring is busy: look again later
					} else {
						__hip_atomic_store(R.stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
						break;
					}
				}
				for (uint32_t i = 0; i < nap; i++)
					__builtin_amdgcn_s_sleep(8);
				nap = nap * 2 < nap_max ? nap * 2 : nap_max;
			}
			go = g;
		}
		__syncthreads();
		const uint32_t gv = go;
		__syncthreads(); // every wave has read go before thread 0 writes the next one
		if (!gv)
			break;
		nap = 1;
		{ // the batch's parameters, from host memory
			const uint32_t *src = reinterpret_cast<const uint32_t *>(&ring[seq_s % R.ndesc].A);
			uint32_t *dst = reinterpret_cast<uint32_t *>(&A);
			for (uint32_t i = tid; i < sizeof(fwd4_params) / 4; i += C::WAVES * 64)
				dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
		__syncthreads();
		// wake the helpers it is split over: only as the batch's first ring
		// (wg0 0; a workgroup that took its role under an older grouping of the
		// rings may hold a helper's descriptor, whose helper_seq are zeros), and
		// by a max, so that no wake word ever goes back
		if (!helper && A.wg0 == 0 && tid > 0 && tid < A.wgs && blockIdx.x + tid < gridDim.x) {
			// relaxed both: the helper acquires its own descriptor's seq before
			// it reads it, so nothing here needs ordering (and a release would
			// write back this XCD's L2)
			const uint64_t hs = __hip_atomic_load(&ring[seq_s % R.ndesc].helper_seq[tid - 1], __ATOMIC_RELAXED,
							      __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_fetch_max(R.wake + (size_t)(blockIdx.x + tid) * R.stride, hs, __ATOMIC_RELAXED,
					       __HIP_MEMORY_SCOPE_AGENT);
		}
		// the edge table of the generation this batch names
		for (uint32_t i = tid; i < sizeof(fwd4_edges); i += C::WAVES * 64)
			reinterpret_cast<uint8_t *>(&edges)[i] = reinterpret_cast<const uint8_t *>(&A.T->edges)[i];
		if (tid < C::SLOTS) {
			L.ready[tid] = 0;
			L.done[tid] = 0;
			L.free_[tid] = 0;
		}
		if (tid == 0) {
			L.abort = 0;
			L.spin_max = A.spin_max ? A.spin_max : RING_SPIN_MAX;
		}
		__syncthreads();
		const uint32_t n_local = local_tiles(A);
		const bool ptrs = A.ptrs != 0;
		if (wv < C::LOADERS) {
			if (ptrs)
				ring_loader<C, false, true>(A, L, n_local, wv, lane);
			else
				ring_loader<C, false, false>(A, L, n_local, wv, lane);
		} else if (wv < C::LOADERS + C::STORERS) {
			if (ptrs)
				ring_storer<C, false, true>(A, L, n_local, wv - C::LOADERS, lane);
			else
				ring_storer<C, false, false>(A, L, n_local, wv - C::LOADERS, lane);
		} else {
			const kctx P = make_kctx(A, &edges);
			if (ptrs)
				ring_compute<C, false, true>(A, P, L, nullptr, nullptr, n_local, wv - C::LOADERS - C::STORERS, lane);
			else
				ring_compute<C, false, false>(A, P, L, nullptr, nullptr, n_local, wv - C::LOADERS - C::STORERS, lane);
		}
		wait_vmcnt<0>(); // this wave's stores of the batch are done
		__syncthreads();
		if (tid == 0) {
			if (L.abort && A.err != nullptr)
				__hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			// release at system scope: the batch's lines and verdicts before its seq
			__hip_atomic_store(done, seq_s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
			seq_s++;
			idle_since = __builtin_amdgcn_s_memrealtime();
			__hip_atomic_store(R.active, idle_since, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		__syncthreads();
	}
	if (tid == 0) // this ring's workgroup is gone: the host may relaunch once every ring's is
		__hip_atomic_store(R.exited + (size_t)blockIdx.x * R.stride, R.launch_id, __ATOMIC_RELEASE,
				   __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" hipError_t gr_fwd4_resident_launch(const fwd4_res_params *R, uint32_t rings, hipStream_t s) {
	hipLaunchKernelGGL(gr_fwd4_resident, dim3(rings), dim3(ring_cfg_res::WAVES * 64), 0, s, *R);
	return hipGetLastError();
}

// Resident workgroups per CU (its static LDS decides): how many rings a device
// can serve at once (gr_hip.cpp res_take).
extern "C" int gr_fwd4_resident_occupancy(void) {
	int b = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, gr_fwd4_resident, ring_cfg_res::WAVES * 64, 0) != hipSuccess) {
		(void)hipGetLastError();
		return 0;
	}
	return b;
}

// ---- the per-iface counters, read at the memory side -----------------------
// The kernels add to the counters with agent-scope atomics, which execute at
// the memory side and leave no line in any XCD's L2; a plain read (a copy, a
// memset's zeroes) may meet a line another XCD's L2 still holds from before.
// So the host reads them, and resets them, through this kernel only: one
// agent-scope atomic per 8-byte counter (fetch-add 0, or exchange with 0 to
// read and reset at once: nothing counted in between is lost), each value
// stored at system scope into pinned host memory. d: [rows][pitch] counters
// of 4 u64, of which the first w of each row; out: [rows][w] of 4 u64.
__global__ void __launch_bounds__(256) gr_stats_collect(unsigned long long *d, unsigned long long *out, uint32_t w,
							uint32_t pitch, uint32_t rows, int reset) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x, per = w * 4;
	if (i >= per * rows)
		return;
	const uint32_t r = i / per, k = i % per;
	GR_GLOBAL unsigned long long *p = (GR_GLOBAL unsigned long long *)(d + (size_t)r * pitch * 4 + k);
	const unsigned long long v = reset ? __hip_atomic_exchange(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
					   : __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__hip_atomic_store(out + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" hipError_t gr_stats_collect_launch(void *d, void *out, uint32_t w, uint32_t pitch, uint32_t rows, int reset,
					      hipStream_t s) {
	const uint32_t n = w * 4 * rows;
	if (n == 0)
		return hipSuccess;
	hipLaunchKernelGGL(gr_stats_collect, dim3((n + 255) / 256), dim3(256), 0, s, static_cast<unsigned long long *>(d),
			   static_cast<unsigned long long *>(out), w, pitch, rows, reset);
	return hipGetLastError();
}

typedef void (*fwd4_rfn)(const fwd4_params);
struct ring_entry {
	fwd4_rfn fn[4]; // by FWD4_V_STATS | FWD4_V_NT
	uint32_t threads;
};
#define RING_ENTRY_SG(C, SG) {{gr_fwd4_ring<C, false, false, false, SG>, gr_fwd4_ring<C, true, false, false, SG>, \
			 gr_fwd4_ring<C, false, true, false, SG>, gr_fwd4_ring<C, true, true, false, SG>}, C::WAVES * 64}
#define RING_ENTRY(C) RING_ENTRY_SG(C, 0)
static const ring_entry ring_kernels[RING_NCFG] = {
	RING_ENTRY(ring_cfg0), RING_ENTRY(ring_cfg1), RING_ENTRY(ring_cfg2),
	RING_ENTRY(ring_cfg3), RING_ENTRY(ring_cfg4), RING_ENTRY(ring_cfg5),
	RING_ENTRY(ring_cfg6), RING_ENTRY(ring_cfg7), RING_ENTRY(ring_cfg8),
	RING_ENTRY(ring_cfg9), RING_ENTRY(ring_cfg10), RING_ENTRY(ring_cfg11),
	RING_ENTRY_SG(ring_cfg2, 16), RING_ENTRY_SG(ring_cfg2, 32), RING_ENTRY_SG(ring_cfg2, 64),
};

// Frame-pointer batches (GR_HIP_BATCH_F_FRAME_PTRS) run on geometry 2, the
// default, only.
#define RING_PTRS_CFG 2
typedef ring_cfg2 ring_cfg_ptrs;
static const ring_entry ring_ptrs_kernel = {
	{gr_fwd4_ring<ring_cfg_ptrs, false, false, true>, gr_fwd4_ring<ring_cfg_ptrs, true, false, true>,
	 gr_fwd4_ring<ring_cfg_ptrs, false, true, true>, gr_fwd4_ring<ring_cfg_ptrs, true, true, true>},
	ring_cfg_ptrs::WAVES * 64};

// variant: FWD4_V_STATS | FWD4_V_NT | FWD4_V_PTRS; cfg: ring geometry
// (ignored for FWD4_V_PTRS). A->nhf_lds fast adjacencies are staged in
// dynamic LDS.
extern "C" hipError_t gr_fwd4_ring_launch(const fwd4_params *A, uint32_t grid, hipStream_t s, int variant, int cfg) {
	const ring_entry &e = (variant & FWD4_V_PTRS) ? ring_ptrs_kernel : ring_kernels[(unsigned)cfg % RING_NCFG];
	const size_t lds = (A->nhf_lds + A->nhf6_lds) * sizeof(fwd4_nhf) + A->top6_lds * sizeof(uint32_t);
	hipLaunchKernelGGL(e.fn[variant & 3], dim3(grid), dim3(e.threads), lds, s, *A);
	return hipGetLastError();
}

extern "C" uint32_t gr_fwd4_ring_nhf_max(void) {
	return RING_NHF_LDS_MAX;
}

extern "C" int gr_fwd4_ring_ncfg(void) {
	return RING_NCFG;
}

extern "C" int gr_fwd4_ring_occupancy(int variant, int cfg, uint32_t nhf_lds) {
	const ring_entry &e = (variant & FWD4_V_PTRS) ? ring_ptrs_kernel : ring_kernels[(unsigned)cfg % RING_NCFG];
	int b = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, e.fn[variant & 3], (int)e.threads, nhf_lds * sizeof(fwd4_nhf))
	    != hipSuccess) {
		(void)hipGetLastError();
		return 0;
	}
	return b;
}
