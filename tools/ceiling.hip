// SPDX-License-Identifier: BSD-3-Clause
// Measurement tool (not the product): ceilings of the memory patterns the
// forwarding kernel combines, at the headline size (2^24 packets).
//   stream:  per packet read a 64 B line + 8 B meta, write 64 B + 8 B
//   gather:  per packet one random read in the touched tbl24 window
//            (14 MiB of 4 B entries, or 7 MiB of 2 B entries)
//   both:    stream + a gather whose index depends on the loaded line
// Layout variants: LANE = each lane moves its packet's 64 B (4 x 16 B);
// QUAD = 4 lanes per packet, 16 B each (coalesced 1 KiB per instruction).
// NT = nontemporal loads/stores on the streamed data.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
	x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
	return x;
}

template <bool NT, typename T> __device__ __forceinline__ T ld(const T *p) {
	if (NT) return __builtin_nontemporal_load(p);
	return *p;
}
template <bool NT, typename T> __device__ __forceinline__ void st(T *p, T v) {
	if (NT) __builtin_nontemporal_store(v, p);
	else *p = v;
}

// MODE: 0 stream, 1 gather only, 2 both. QUAD: lane layout. W2: 2-byte table.
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int MODE, bool QUAD, bool NT, bool W2>
__global__ void __launch_bounds__(256) k(const uint32_t *in, uint32_t *out, const u2v *meta, u2v *v,
                                         const void *tbl, uint32_t window, uint32_t n) {
	const u4 *in4 = reinterpret_cast<const u4 *>(in);
	u4 *out4 = reinterpret_cast<u4 *>(out);
	if (MODE == 1) {
		for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
			uint32_t idx = mix(i) % window;
			uint32_t g = W2 ? reinterpret_cast<const uint16_t *>(tbl)[idx] : reinterpret_cast<const uint32_t *>(tbl)[idx];
			v[i] = u2v{g, i};
		}
		return;
	}
	if (!QUAD) {
		for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
			u2v m = ld<NT>(meta + i);
			u4 a = ld<NT>(in4 + 4 * (size_t)i), b = ld<NT>(in4 + 4 * (size_t)i + 1);
			u4 c = ld<NT>(in4 + 4 * (size_t)i + 2), d = ld<NT>(in4 + 4 * (size_t)i + 3);
			uint32_t g = 0;
			if (MODE == 2) {
				uint32_t idx = mix(a.x ^ c.y ^ i) % window;
				g = W2 ? reinterpret_cast<const uint16_t *>(tbl)[idx] : reinterpret_cast<const uint32_t *>(tbl)[idx];
			}
			a.x ^= g;
			st<NT>(out4 + 4 * (size_t)i, a); st<NT>(out4 + 4 * (size_t)i + 1, b);
			st<NT>(out4 + 4 * (size_t)i + 2, c); st<NT>(out4 + 4 * (size_t)i + 3, d);
			st<NT>(v + i, u2v{m.x ^ g, m.y});
		}
	} else {
		// 4 lanes per packet; a packet's 4 lanes are consecutive in the wave
		const uint32_t lane = threadIdx.x & 3;
		for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < 4 * n; q += gridDim.x * 256) {
			uint32_t i = q >> 2;
			u4 a = ld<NT>(in4 + q);
			u2v m = u2v{0, 0};
			if (lane == 0)
				m = ld<NT>(meta + i);
			uint32_t g = 0;
			if (MODE == 2) {
				// the dst word straddles chunks 1 and 2: combine via a shuffle
				uint32_t other = __shfl(a.x, (threadIdx.x & 63) + 1, 64);
				if (lane == 1) {
					uint32_t idx = mix(a.w ^ other ^ i) % window;
					g = W2 ? reinterpret_cast<const uint16_t *>(tbl)[idx] : reinterpret_cast<const uint32_t *>(tbl)[idx];
				}
				g = __shfl(g, (threadIdx.x & 63) | 1, 64);
			}
			if (lane == 0)
				a.x ^= g;
			st<NT>(out4 + q, a);
			if (lane == 0)
				st<NT>(v + i, u2v{m.x ^ g, m.y});
		}
	}
}

template <int MODE, bool QUAD, bool NT, bool W2>
static int run(const char *name, const uint32_t *in, uint32_t *out, const u2v *meta, u2v *v, const void *tbl, uint32_t n) {
	uint32_t window = W2 ? (7u << 19) : (14u << 18); // 7 MiB / 14 MiB
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	int grids[] = {256 * 8, 65536};
	for (int gi = 0; gi < 2; gi++) {
		float best = 1e9;
		for (int r = 0; r < 6; r++) {
			CK(hipEventRecord(e0));
			hipLaunchKernelGGL((k<MODE, QUAD, NT, W2>), dim3(grids[gi]), dim3(256), 0, 0, in, out, meta, v, tbl, window, n);
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (r && ms < best)
				best = ms;
		}
		double bytes = MODE == 1 ? n * 12.0 : (MODE == 0 ? n * 144.0 : n * (W2 ? 146.0 : 148.0));
		printf("{\"pattern\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"mpps\": %.1f, \"GBps\": %.1f}\n", name, grids[gi],
		       best, n / best / 1e3, bytes / best / 1e6);
	}
	return 0;
}

int main() {
	const uint32_t n = 1u << 24;
	uint32_t *in, *out;
	u2v *meta, *v;
	void *tbl;
	CK(hipMalloc(&in, (size_t)n * 64));
	CK(hipMalloc(&out, (size_t)n * 64));
	CK(hipMalloc(&meta, (size_t)n * 8));
	CK(hipMalloc(&v, (size_t)n * 8));
	CK(hipMalloc(&tbl, 64u << 20));
	CK(hipMemset(in, 1, (size_t)n * 64));
	CK(hipMemset(meta, 2, (size_t)n * 8));
	CK(hipMemset(tbl, 3, 64u << 20));
	CK(hipDeviceSynchronize());
	run<0, false, false, false>("stream lane", in, out, meta, v, tbl, n);
	run<0, false, true, false>("stream lane nt", in, out, meta, v, tbl, n);
	run<0, true, false, false>("stream quad", in, out, meta, v, tbl, n);
	run<0, true, true, false>("stream quad nt", in, out, meta, v, tbl, n);
	run<1, false, false, false>("gather 4B", in, out, meta, v, tbl, n);
	run<1, false, false, true>("gather 2B", in, out, meta, v, tbl, n);
	run<2, false, false, false>("both lane", in, out, meta, v, tbl, n);
	run<2, false, true, false>("both lane nt", in, out, meta, v, tbl, n);
	run<2, false, true, true>("both lane nt 2B", in, out, meta, v, tbl, n);
	run<2, true, false, false>("both quad", in, out, meta, v, tbl, n);
	run<2, true, true, false>("both quad nt", in, out, meta, v, tbl, n);
	run<2, true, true, true>("both quad nt 2B", in, out, meta, v, tbl, n);
	return 0;
}
