// Exactness check of the solve's fp64-reciprocal float quotient (gd_math.h: gd_div / quot64)
// against the compiler's IEEE float division, on the device:
//   1. every pair of special values (zeros, infinities, NaN, denormals, extremes);
//   2. all 2^32 dividends for a set of divisors (powers of two, near-one, random, denormal);
//   3. random pairs: full exponent range, and exponents kept close (normal-range quotients);
//   4. constructed exact-midpoint quotients in the denormal range (the only case where a
//      quotient of two floats can be a rounding midpoint: a = m * B * 2^(e-150), b = B * 2^e,
//      m odd), which the fp64 residual correction must round to even.
// Prints one JSON line; every count must be 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/div_exact_check.hip -o build/div_exact_check
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../many_bone_ik_amd/csrc/gd_math.h"

using namespace gd;

__device__ __forceinline__ uint64_t splitmix(uint64_t &s) {
	uint64_t z = (s += 0x9e3779b97f4a7c15ull);
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}
__device__ __forceinline__ bool same(float x, float y) { return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y); }
__device__ __forceinline__ void tally(unsigned long long *bad, unsigned *first, int cls, float a, float b) {
	const float ref = a / b;
	const float got = gd_div(a, b);
	if (!same(ref, got)) {
		if (atomicAdd(&bad[cls], 1ull) == 0ull) {
			first[2 * cls] = __float_as_uint(a);
			first[2 * cls + 1] = __float_as_uint(b);
		}
	}
}

__device__ const unsigned specials[] = {0x00000000u, 0x80000000u, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0xffc00001u,
		0x00000001u, 0x80000003u, 0x007fffffu, 0x807fffffu, 0x00800000u, 0x7f7fffffu, 0xff7fffffu, 0x3f800000u, 0xbf800000u,
		0x3f7fffffu, 0x3f800001u, 0x34000000u, 0x5f000000u, 0x1f800000u, 0x00400000u, 0x7f000000u, 0x40400000u, 0x3dcccccdu};
constexpr int NSPEC = sizeof(specials) / sizeof(specials[0]);
__device__ const unsigned divisors[] = {0x3f800000u, 0x40000000u, 0x3f800001u, 0x3f7fffffu, 0x40400000u, 0x3dcccccdu,
		0x4049a0b1u, 0x00000003u, 0x00400001u, 0x7e800001u, 0xbf9d70a4u, 0x3a83126fu};
constexpr int NDIV = sizeof(divisors) / sizeof(divisors[0]);

__global__ void k_specials(unsigned long long *bad, unsigned *first) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= NSPEC * NSPEC) return;
	tally(bad, first, 0, __uint_as_float(specials[i % NSPEC]), __uint_as_float(specials[i / NSPEC]));
}
__global__ void k_all_dividends(unsigned long long *bad, unsigned *first, unsigned d) {
	const float b = __uint_as_float(divisors[d]);
	for (uint64_t a = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; a < (1ull << 32); a += (uint64_t)gridDim.x * blockDim.x)
		tally(bad, first, 1, __uint_as_float((unsigned)a), b);
}
// N / b for N = 0.5, 1, 2 (gd_pow2_over) over all 2^32 divisors
__global__ void k_pow2_over(unsigned long long *bad, unsigned *first) {
	for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < (1ull << 32); b += (uint64_t)gridDim.x * blockDim.x) {
		const float bf = __uint_as_float((unsigned)b);
		const float n[3] = {0.5f, 1.0f, 2.0f};
#pragma unroll
		for (int k = 0; k < 3; k++) {
			if (!same(n[k] / bf, gd_pow2_over(n[k], bf)) && atomicAdd(&bad[4], 1ull) == 0ull) {
				first[8] = __float_as_uint(n[k]);
				first[9] = (unsigned)b;
			}
		}
	}
}
__global__ void k_random(unsigned long long *bad, unsigned *first, int iters) {
	uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 0x2545f4914f6cdd1dull + 777;
	for (int it = 0; it < iters; it++) {
		const uint64_t z = splitmix(s);
		unsigned ab = (unsigned)z, bb = (unsigned)(z >> 32);
		if (it & 1) {
			ab = (ab & 0x807fffffu) | ((110u + ((z >> 8) & 31)) << 23);
			bb = (bb & 0x807fffffu) | ((110u + ((z >> 40) & 31)) << 23);
		}
		tally(bad, first, 2, __uint_as_float(ab), __uint_as_float(bb));
	}
}
// exact denormal midpoints m * 2^-150 (m odd): b = B * 2^e, a = m * B * 2^(e - 150)
__global__ void k_ties(unsigned long long *bad, unsigned *first, int iters) {
	uint64_t s = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 0x9e3779b97f4a7c15ull + 99;
	for (int it = 0; it < iters; it++) {
		const uint64_t z = splitmix(s);
		const int mbits = 1 + (int)(z % 23);                   // m < 2^mbits, odd
		const uint32_t m = ((uint32_t)(z >> 8) & ((1u << mbits) - 1u)) | 1u;
		const int bbits = 1 + (int)((z >> 40) % (uint64_t)(24 - mbits + 1));
		const uint32_t B = ((uint32_t)(z >> 20) & ((1u << bbits) - 1u)) | 1u | (1u << (bbits - 1));
		const uint64_t mb = (uint64_t)m * B;                   // <= 24 bits: a is exact
		const int e = 100 + (int)((z >> 50) % 60);             // b = B * 2^(e - bbits...) normal
		const double bd = ldexp((double)B, e - bbits);
		const double ad = ldexp((double)mb, e - bbits - 150);
		const float a = (float)ad, b = (float)bd;
		if ((double)a != ad || (double)b != bd) continue;      // not representable: skip
		const float sa = (z >> 62) & 1 ? -a : a, sb = (z >> 63) ? -b : b;
		tally(bad, first, 3, sa, sb);
	}
}

int main(int argc, char **argv) {
	const int iters = argc > 1 ? atoi(argv[1]) : 2048;
	unsigned long long *bad; unsigned *first;
	(void)hipMalloc(&bad, 5 * sizeof(unsigned long long));
	(void)hipMalloc(&first, 10 * sizeof(unsigned));
	(void)hipMemset(bad, 0, 5 * sizeof(unsigned long long));
	(void)hipMemset(first, 0, 10 * sizeof(unsigned));
	k_specials<<<(NSPEC * NSPEC + 63) / 64, 64>>>(bad, first);
	for (int d = 0; d < NDIV; d++) k_all_dividends<<<8192, 256>>>(bad, first, d);
	k_random<<<8192, 256>>>(bad, first, iters);
	k_ties<<<8192, 256>>>(bad, first, iters);
	k_pow2_over<<<8192, 256>>>(bad, first);
	if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"launch failed\"}\n"); return 1; }
	unsigned long long hb[5]; unsigned hf[10];
	(void)hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
	(void)hipMemcpy(hf, first, sizeof(hf), hipMemcpyDeviceToHost);
	const double rnd = 8192.0 * 256 * iters;
	printf("{\"special_pairs\": %d, \"special_mismatch\": %llu, \"all_dividends_divisors\": %d, \"all_dividends_mismatch\": %llu, "
		   "\"random_pairs\": %.4g, \"random_mismatch\": %llu, \"tie_draws\": %.4g, \"tie_mismatch\": %llu, "
		   "\"pow2_over_all_divisors_mismatch\": %llu, "
		   "\"first_mismatch\": [\"0x%08x/0x%08x\", \"0x%08x/0x%08x\", \"0x%08x/0x%08x\", \"0x%08x/0x%08x\"]}\n",
			NSPEC * NSPEC, hb[0], NDIV, hb[1], rnd, hb[2], rnd, hb[3], hb[4], hf[0], hf[1], hf[2], hf[3], hf[4], hf[5], hf[6], hf[7]);
	return (hb[0] | hb[1] | hb[2] | hb[3] | hb[4]) ? 2 : 0;
}
