// Exhaustive check of candidate fast square roots against the correctly rounded sqrtf, over
// all 2^32 float bit patterns (the solve needs bitwise-identical results, and a one-input
// function can be proven identical by enumeration).  Prints, per candidate, the number of
// inputs whose result differs bitwise (non-NaN), differs only in NaN payload, and the first
// few differing inputs.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/sqrt_exhaustive.hip -o build/sqrt_exhaustive
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

#define NC 4
// candidate 0: float rsq + one Newton correction (Markstein form), 2^32 pre-scale below 2^-96
__device__ __forceinline__ float c0(float x) {
	const bool small = x < 0x1p-96f;
	const float xs = x * (small ? 0x1p32f : 1.0f);
	const float y = __builtin_amdgcn_rsqf(xs);
	const float g = xs * y, h = 0.5f * y;
	const float e = fmaf(-g, g, xs);
	float r = fmaf(e, h, g) * (small ? 0x1p-16f : 1.0f);
	return __builtin_amdgcn_class(x, 0x260) ? x : r;
}
// candidate 1: the same in fp64 (no pre-scale needed: float denormals are normal doubles)
__device__ __forceinline__ float c1(float x) {
	const double xd = x;
	const double y = __builtin_amdgcn_rsq(xd);
	const double g = xd * y, h = 0.5 * y;
	const double e = fma(-g, g, xd);
	float r = (float)fma(e, h, g);
	return __builtin_amdgcn_class(x, 0x260) ? x : r;
}
// candidate 2: hardware v_sqrt_f32 + Newton correction using the rsq estimate
__device__ __forceinline__ float c2(float x) {
	const bool small = x < 0x1p-96f;
	const float xs = x * (small ? 0x1p32f : 1.0f);
	const float g = __builtin_amdgcn_sqrtf(xs);
	const float h = 0.5f * __builtin_amdgcn_rsqf(xs);
	const float e = fmaf(-g, g, xs);
	float r = fmaf(e, h, g) * (small ? 0x1p-16f : 1.0f);
	return __builtin_amdgcn_class(x, 0x260) ? x : r;
}
// candidate 3: fp64 hardware sqrt + fp64 Newton correction
__device__ __forceinline__ float c3(float x) {
	const double xd = x;
	const double g = __builtin_amdgcn_sqrt(xd);
	const double h = 0.5 * __builtin_amdgcn_rsq(xd);
	const double e = fma(-g, g, xd);
	float r = (float)fma(e, h, g);
	return __builtin_amdgcn_class(x, 0x260) ? x : r;
}

__global__ void check(unsigned long long *bad, unsigned long long *nanbad, unsigned *first, unsigned *nfirst) {
	const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
	const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	unsigned long long b[NC] = {}, nb[NC] = {};
	for (uint64_t i = tid; i < (1ull << 32); i += nthreads) {
		const float x = __uint_as_float((unsigned)i);
		const float ref = sqrtf(x);
		const unsigned rb = __float_as_uint(ref);
		float c[NC] = {c0(x), c1(x), c2(x), c3(x)};
#pragma unroll
		for (int k = 0; k < NC; k++) {
			const unsigned cb = __float_as_uint(c[k]);
			if (cb != rb) {
				if (ref != ref && c[k] != c[k]) {
					nb[k]++;
				} else {
					b[k]++;
					unsigned slot = atomicAdd(&nfirst[k], 1u);
					if (slot < 8) first[k * 8 + slot] = (unsigned)i;
				}
			}
		}
	}
#pragma unroll
	for (int k = 0; k < NC; k++) {
		if (b[k]) atomicAdd(&bad[k], b[k]);
		if (nb[k]) atomicAdd(&nanbad[k], nb[k]);
	}
}

// Dependent-chain latency of each candidate (one wave per CU, clock64 around 256 x 16 calls).
template <int C>
__device__ __forceinline__ float cand(float x) {
	if constexpr (C == 0) return c0(x);
	else if constexpr (C == 1) return c1(x);
	else if constexpr (C == 2) return c2(x);
	else if constexpr (C == 3) return c3(x);
	else return sqrtf(x);
}
template <int C, bool IND>
__global__ __launch_bounds__(64) void lat(float *out, long long *cyc, float seed) {
	float a = seed + threadIdx.x * 1e-3f, a2 = a + 1, a3 = a + 2, a4 = a + 3;
	const float d = 1.5f;
	long long t0 = clock64();
#pragma unroll 1
	for (int i = 0; i < 256; i++) {
		if constexpr (IND) {
#pragma unroll
			for (int k = 0; k < 4; k++) { a = cand<C>(a) + d; a2 = cand<C>(a2) + d; a3 = cand<C>(a3) + d; a4 = cand<C>(a4) + d; }
		} else {
#pragma unroll
			for (int k = 0; k < 16; k++) a = cand<C>(a) + d;
		}
	}
	long long t1 = clock64();
	out[blockIdx.x * 64 + threadIdx.x] = a + a2 + a3 + a4;
	if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int C, bool IND>
double lat_run(float *o, long long *c) {
	long long h[256];
	for (int rep = 0; rep < 2; rep++) lat<C, IND><<<256, 64>>>(o, c, 1.25f);
	hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
	double s = 0;
	for (int i = 0; i < 256; i++) s += (double)h[i];
	return s / 256 / (256 * 16);
}

int main() {
	{
		float *o; long long *c;
		hipMalloc(&o, 256 * 64 * 4);
		hipMalloc(&c, 256 * 8);
		double l[5] = {lat_run<0, false>(o, c), lat_run<1, false>(o, c), lat_run<2, false>(o, c), lat_run<3, false>(o, c), lat_run<4, false>(o, c)};
		double t[5] = {lat_run<0, true>(o, c), lat_run<1, true>(o, c), lat_run<2, true>(o, c), lat_run<3, true>(o, c), lat_run<4, true>(o, c)};
		for (int k = 0; k < 5; k++)
			printf("{\"candidate\": %d, \"cycles_per_sqrt_plus_add_dep\": %.2f, \"indep4\": %.2f}\n", k == 4 ? -1 : k, l[k], t[k]);
	}
	unsigned long long *bad, *nanbad;
	unsigned *first, *nfirst;
	hipMalloc(&bad, NC * 8);
	hipMalloc(&nanbad, NC * 8);
	hipMalloc(&first, NC * 8 * 4);
	hipMalloc(&nfirst, NC * 4);
	hipMemset(bad, 0, NC * 8);
	hipMemset(nanbad, 0, NC * 8);
	hipMemset(first, 0, NC * 32);
	hipMemset(nfirst, 0, NC * 4);
	hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, bad, nanbad, first, nfirst);
	if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
	unsigned long long hb[NC], hn[NC];
	unsigned hf[NC * 8], hnf[NC];
	hipMemcpy(hb, bad, NC * 8, hipMemcpyDeviceToHost);
	hipMemcpy(hn, nanbad, NC * 8, hipMemcpyDeviceToHost);
	hipMemcpy(hf, first, NC * 32, hipMemcpyDeviceToHost);
	hipMemcpy(hnf, nfirst, NC * 4, hipMemcpyDeviceToHost);
	for (int k = 0; k < NC; k++) {
		printf("{\"candidate\": %d, \"mismatches\": %llu, \"nan_payload_only\": %llu, \"first\": [", k, hb[k], hn[k]);
		for (int j = 0; j < 8 && j < (int)hnf[k]; j++) printf("%s\"0x%08x\"", j ? ", " : "", hf[k * 8 + j]);
		printf("]}\n");
	}
	return 0;
}
