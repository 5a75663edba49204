// SPDX-License-Identifier: BSD-3-Clause
// Measurement tool (not the product): does a plain stream copy of the
// forwarding kernel's shape (read 64 B line + 8 B meta, write 64 B + 8 B per
// packet, 2^24 packets, 4 lanes per packet, nontemporal) show the same
// set-to-set spread over separate hipMalloc allocations as the ring kernel
// (tools/placement_probe.py)? SETS allocations, PASSES round-robin passes,
// best of 5 launches each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy(const u4 *in4, u4 *out4, const u2v *meta, u2v *v, uint32_t n) {
	const uint32_t lane = threadIdx.x & 3;
	for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < 4 * n; q += gridDim.x * 256) {
		const uint32_t i = q >> 2;
		u4 a = __builtin_nontemporal_load(in4 + q);
		__builtin_nontemporal_store(a, out4 + q);
		if (lane == 0)
			__builtin_nontemporal_store(__builtin_nontemporal_load(meta + i), v + i);
	}
}

// Persistent grid (256 workgroups x 16 waves), 64-packet tiles of 4 KiB
// lines + 512 B meta, tile k of wave w at w + k * (waves in grid) -- the
// ring kernel's access order. LDS: 0 = loads into VGPRs; 1 = LDS-DMA
// (global_load_lds_dwordx4 nt) with the ring's swizzled chunk order;
// 2 = LDS-DMA in plain lane order.
template <int LDS>
__global__ void __launch_bounds__(1024) tiles(const uint8_t *in, uint8_t *out, const u2v *meta, u2v *v, uint32_t n) {
	__shared__ __attribute__((aligned(16))) uint8_t buf[16][4096];
	const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t W = gridDim.x * 16, n_tiles = n / 64;
	const uint32_t prow = lane >> 2;
	const uint32_t pchunk = LDS == 1 ? ((lane & 3) ^ ((lane >> 4) & 3)) : (lane & 3);
	for (uint32_t t = blockIdx.x * 16 + w; t < n_tiles; t += W) {
		const uint8_t *src = in + (size_t)t * 4096;
		uint8_t *dst = out + (size_t)t * 4096;
		u4 o[4];
		if (LDS == 0) {
#pragma unroll
			for (uint32_t q = 0; q < 4; q++)
				o[q] = __builtin_nontemporal_load(reinterpret_cast<const u4 *>(src + q * 1024 + prow * 64 + pchunk * 16));
		} else {
			const uint32_t lb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)buf[w];
#pragma unroll
			for (uint32_t q = 0; q < 4; q++) {
				uint32_t keep;
				asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
					     : "=&s"(keep)
					     : "v"(src + q * 1024 + prow * 64 + pchunk * 16), "s"(lb + q * 1024)
					     : "memory");
			}
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
			for (uint32_t q = 0; q < 4; q++)
				o[q] = *reinterpret_cast<const u4 *>(&buf[w][q * 1024 + lane * 16]);
		}
		const u2v m = __builtin_nontemporal_load(meta + (size_t)t * 64 + lane);
#pragma unroll
		for (uint32_t q = 0; q < 4; q++)
			__builtin_nontemporal_store(o[q], reinterpret_cast<u4 *>(dst + q * 1024 + prow * 64 + pchunk * 16));
		__builtin_nontemporal_store(m, v + (size_t)t * 64 + lane);
	}
}

int main() {
	const uint32_t n = 1u << 24, SETS = 8, PASSES = 2;
	u4 *in[SETS], *out[SETS];
	u2v *meta[SETS], *v[SETS];
	for (uint32_t s = 0; s < SETS; s++) {
		CK(hipMalloc(&in[s], (size_t)n * 64));
		CK(hipMalloc(&meta[s], (size_t)n * 8));
		CK(hipMalloc(&out[s], (size_t)n * 64));
		CK(hipMalloc(&v[s], (size_t)n * 8));
		CK(hipMemset(in[s], 1, (size_t)n * 64));
		CK(hipMemset(meta[s], 2, (size_t)n * 8));
	}
	CK(hipDeviceSynchronize());
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const char *names[] = {"copy", "tiles_vgpr", "tiles_lds_swz", "tiles_lds"};
	for (uint32_t p = 0; p < PASSES; p++)
		for (uint32_t s = 0; s < SETS; s++)
			for (int kind = 0; kind < 4; kind++) {
				float best = 1e9;
				for (int r = 0; r < 6; r++) {
					CK(hipEventRecord(e0));
					if (kind == 0)
						hipLaunchKernelGGL(copy, dim3(65536), dim3(256), 0, 0, in[s], out[s], meta[s], v[s], n);
					else if (kind == 1)
						hipLaunchKernelGGL(tiles<0>, dim3(256), dim3(1024), 0, 0, (const uint8_t *)in[s], (uint8_t *)out[s], meta[s], v[s], n);
					else if (kind == 2)
						hipLaunchKernelGGL(tiles<1>, dim3(256), dim3(1024), 0, 0, (const uint8_t *)in[s], (uint8_t *)out[s], meta[s], v[s], n);
					else
						hipLaunchKernelGGL(tiles<2>, dim3(256), dim3(1024), 0, 0, (const uint8_t *)in[s], (uint8_t *)out[s], meta[s], v[s], n);
					CK(hipEventRecord(e1));
					CK(hipEventSynchronize(e1));
					float ms;
					CK(hipEventElapsedTime(&ms, e0, e1));
					if (r && ms < best)
						best = ms;
				}
				printf("{\"pass\": %u, \"set\": %u, \"kind\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", p, s, names[kind], best,
				       n * 144.0 / best / 1e6);
			}
	return 0;
}
