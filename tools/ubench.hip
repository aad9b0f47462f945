// Single-wave instruction cost micro-benchmark (one wave per CU, s_memtime around a loop of
// N repetitions): how many cycles one wave's dependent / independent streams of the solve
// kernel's building blocks cost on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/ubench.hip -o build/ubench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include "../many_bone_ik_amd/csrc/gd_math.h"
using namespace gd;

// quad broadcast of lane r's value (DPP quad_perm), the cooperative-helper primitive
template <int R>
__device__ __forceinline__ float qb(float v) {
	return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), R * 0x55, 0xf, 0xf, true));
}
__device__ __forceinline__ V3 qb3_0(V3 v) { return v3(qb<0>(v.x), qb<0>(v.y), qb<0>(v.z)); }
__device__ __forceinline__ V3 qb3_1(V3 v) { return v3(qb<1>(v.x), qb<1>(v.y), qb<1>(v.z)); }
__device__ __forceinline__ V3 qb3_2(V3 v) { return v3(qb<2>(v.x), qb<2>(v.y), qb<2>(v.z)); }
// per-lane select with a constant lane mask (u == 0 lanes: 0x1111..., u == 1: 0x2222...), kept
// as a v_cndmask so that the compiler cannot turn a select of struct fields into an indexed load
__device__ __forceinline__ float lsel(float if_set, float if_clear, unsigned long long mask) {
	float r;
	asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(mask));
	return r;
}
__device__ __forceinline__ float pick3(float x0, float x1, float x2) {
	return lsel(x0, lsel(x1, x2, 0x2222222222222222ull), 0x1111111111111111ull);
}
// row u of a*b computed by quad lane u (u = 3 repeats row 2), gathered to every lane
__device__ __forceinline__ B3 mul_coop(const B3 &a, const B3 &b, int u) {
	V3 ar = v3(pick3(a.r[0].x, a.r[1].x, a.r[2].x), pick3(a.r[0].y, a.r[1].y, a.r[2].y), pick3(a.r[0].z, a.r[1].z, a.r[2].z));
	V3 row = v3(b.r[0].x * ar.x + b.r[1].x * ar.y + b.r[2].x * ar.z, b.r[0].y * ar.x + b.r[1].y * ar.y + b.r[2].y * ar.z,
			b.r[0].z * ar.x + b.r[1].z * ar.y + b.r[2].z * ar.z);
	B3 r;
	r.r[0] = qb3_0(row);
	r.r[1] = qb3_1(row);
	r.r[2] = qb3_2(row);
	return r;
}
__device__ __forceinline__ V3 normalized_coop(V3 a, int u) {
	float l = length_sq(a);
	if (l == 0) return v3(0, 0, 0);
	float len = gd_sqrt(l);
	float c = pick3(a.x, a.y, a.z);
	float q = c / len;
	return v3(qb<0>(q), qb<1>(q), qb<2>(q));
}

// candidate exact f32 division: (float)((double)a * r), r = 1/(double)b from v_rcp_f64 with
// one Newton step, special operands fixed by v_div_fixup_f32 (NOT exact for denormal quotients)
__device__ __forceinline__ float div_rcp64(float a, float b) {
	const double bd = b;
	double r = __builtin_amdgcn_rcp(bd);
	const double e = __builtin_fma(-bd, r, 1.0);
	r = __builtin_fma(e, r, r);
	const float q = (float)((double)a * r);
	return __builtin_amdgcn_div_fixupf(q, b, a);
}
__device__ __forceinline__ V3 normalized_rcp64(V3 a) {
	float l = length_sq(a);
	if (l == 0) return v3(0, 0, 0);
	float len = gd_sqrt(l);
	const double bd = len;
	double r = __builtin_amdgcn_rcp(bd);
	const double e = __builtin_fma(-bd, r, 1.0);
	r = __builtin_fma(e, r, r);
	return v3((float)((double)a.x * r), (float)((double)a.y * r), (float)((double)a.z * r));
}

// exact f32 quotient: fp64 reciprocal, one Newton step, product, one residual
// correction in fp64 (makes exact-midpoint denormal quotients exact), v_div_fixup for specials
__device__ __forceinline__ double rcp64_refined(double bd) {
	double r = __builtin_amdgcn_rcp(bd);
	const double e = __builtin_fma(-bd, r, 1.0);
	return __builtin_fma(e, r, r);
}
__device__ __forceinline__ float quot64(float a, float b, double bd, double r) {
	const double ad = a;
	const double q0 = ad * r;
	const double rem = __builtin_fma(-bd, q0, ad);
	const double q1 = __builtin_fma(rem, r, q0);
	return __builtin_amdgcn_div_fixupf((float)q1, b, a);
}
__device__ __forceinline__ float div_exact64(float a, float b) {
	const double bd = b;
	return quot64(a, b, bd, rcp64_refined(bd));
}
__device__ __forceinline__ V3 normalized_exact64(V3 a) {
	float l = length_sq(a);
	if (l == 0) return v3(0, 0, 0);
	float len = gd_sqrt(l);
	const double bd = len, r = rcp64_refined(bd);
	return v3(quot64(a.x, len, bd, r), quot64(a.y, len, bd, r), quot64(a.z, len, bd, r));
}
// sin(x) in double for |x| <= pi/2 by an odd Taylor/minimax-free polynomial (degree 17): timing only
__device__ __forceinline__ double sin_poly64(double x) {
	const double x2 = x * x;
	double p = -7.647163731819816e-13;
	p = __builtin_fma(p, x2, 1.6059043836821613e-10);
	p = __builtin_fma(p, x2, -2.505210838544172e-08);
	p = __builtin_fma(p, x2, 2.7557319223985893e-06);
	p = __builtin_fma(p, x2, -0.0001984126984126984);
	p = __builtin_fma(p, x2, 0.008333333333333333);
	p = __builtin_fma(p, x2, -0.16666666666666666);
	return __builtin_fma(x * x2, p, x);
}

typedef float fl2 __attribute__((ext_vector_type(2)));
// Basis product with the x/y columns packed (v_pk_mul_f32 / v_pk_add_f32) and z scalar: the
// same roundings as gd::operator*(B3, B3), two columns per instruction
struct PB3 { fl2 xy[3]; float z[3]; };
__device__ __forceinline__ PB3 pmul(const PB3 &a, const PB3 &b) {
	PB3 r;
#pragma unroll
	for (int i = 0; i < 3; i++) {
		const float ax = a.xy[i].x, ay = a.xy[i].y, az = a.z[i];
		r.xy[i] = (b.xy[0] * ax + b.xy[1] * ay) + b.xy[2] * az;
		r.z[i] = (b.z[0] * ax + b.z[1] * ay) + b.z[2] * az;
	}
	return r;
}

#define REPS 256

template <int OP>
__global__ __launch_bounds__(64) void kern(float *out, double *outd, long long *cyc, float seed) {
	float a = seed + threadIdx.x * 1e-3f, b = 1.0001f, c = 0.999f, d = 1.5f + threadIdx.x * 1e-4f;
	float a2 = a + 1, a3 = a + 2, a4 = a + 3;
	double x = (double)a, y = 1.0000001, z = 0.9999999, x2 = x + 1, x3 = x + 2, x4 = x + 3;
	__shared__ float sh[256];
	sh[threadIdx.x] = (float)threadIdx.x;
	sh[threadIdx.x + 64] = 0.0f;
	__syncthreads();
	int idx = threadIdx.x;
	fl2 p = {a, a2}, q = {a3, a4}, pb = {b, c}, pc = {c, b};
	const int u = threadIdx.x & 3;
	B3 M = bset(a, 0.1f, 0.2f, 0.3f, a2, 0.1f, 0.2f, 0.1f, a3), A = bset(0.9f, 0.1f, 0.05f, -0.1f, 0.95f, 0.02f, 0.03f, -0.04f, 1.01f);
	V3 vv = v3(a, a2, a3);
	X3 X = {M, vv}, XA = {A, v3(0.1f, 0.2f, 0.3f)};
	PB3 PM, PA;
	for (int i = 0; i < 3; i++) {
		PM.xy[i] = fl2{M.r[i].x, M.r[i].y}; PM.z[i] = M.r[i].z;
		PA.xy[i] = fl2{A.r[i].x, A.r[i].y}; PA.z[i] = A.r[i].z;
	}
	long long t0 = clock64();
#pragma unroll 1
	for (int i = 0; i < REPS; i++) {
		if constexpr (OP == 0) { // dependent fp32 fma chain x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = __builtin_fmaf(a, b, c);
		} else if constexpr (OP == 1) { // 4 independent fp32 fma chains x4
#pragma unroll
			for (int k = 0; k < 4; k++) { a = __builtin_fmaf(a, b, c); a2 = __builtin_fmaf(a2, b, c); a3 = __builtin_fmaf(a3, b, c); a4 = __builtin_fmaf(a4, b, c); }
		} else if constexpr (OP == 2) { // dependent fp64 fma chain x16
#pragma unroll
			for (int k = 0; k < 16; k++) x = __builtin_fma(x, y, z);
		} else if constexpr (OP == 3) { // 4 independent fp64 fma chains x4
#pragma unroll
			for (int k = 0; k < 4; k++) { x = __builtin_fma(x, y, z); x2 = __builtin_fma(x2, y, z); x3 = __builtin_fma(x3, y, z); x4 = __builtin_fma(x4, y, z); }
		} else if constexpr (OP == 4) { // dependent IEEE fp32 division x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = d / a;
		} else if constexpr (OP == 5) { // 4 independent IEEE fp32 divisions x4
#pragma unroll
			for (int k = 0; k < 4; k++) { a = d / a; a2 = d / a2; a3 = d / a3; a4 = d / a4; }
		} else if constexpr (OP == 6) { // dependent IEEE fp32 sqrt x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = sqrtf(a) + d;
		} else if constexpr (OP == 7) { // 4 independent IEEE sqrt x4
#pragma unroll
			for (int k = 0; k < 4; k++) { a = sqrtf(a) + d; a2 = sqrtf(a2) + d; a3 = sqrtf(a3) + d; a4 = sqrtf(a4) + d; }
		} else if constexpr (OP == 8) { // dependent fp64 division x16
#pragma unroll
			for (int k = 0; k < 16; k++) x = y / x;
		} else if constexpr (OP == 9) { // dependent double sin x4
#pragma unroll
			for (int k = 0; k < 4; k++) x = sin(x) + 0.5;
		} else if constexpr (OP == 10) { // dependent double acos x4
#pragma unroll
			for (int k = 0; k < 4; k++) x = acos(x * 0.5);
		} else if constexpr (OP == 11) { // dependent ds_read_b32 chain x16 (pointer chase)
#pragma unroll
			for (int k = 0; k < 16; k++) idx = (int)sh[idx & 63];
		} else if constexpr (OP == 12) { // dependent fp64 sqrt x16
#pragma unroll
			for (int k = 0; k < 16; k++) x = sqrt(x) + y;
		} else if constexpr (OP == 13) { // dependent cvt f32->f64->f32 + fp64 add x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = (float)((double)a + y);
		} else if constexpr (OP == 14) { // dependent fp32 mul+add pairs x8 (two ops each)
#pragma unroll
			for (int k = 0; k < 8; k++) a = a * b + c;
		} else if constexpr (OP == 15) { // 2 independent v_pk_mul_f32 chains x8
#pragma unroll
			for (int k = 0; k < 8; k++) { p = p * pb; q = q * pc; }
		} else if constexpr (OP == 16) { // 4 independent v_mul_f32 chains x4 (same work as 15)
#pragma unroll
			for (int k = 0; k < 4; k++) { a = a * b; a2 = a2 * c; a3 = a3 * b; a4 = a4 * c; }
		} else if constexpr (OP == 17) { // 2 independent v_pk_add_f32 chains x8
#pragma unroll
			for (int k = 0; k < 8; k++) { p = p + pb; q = q + pc; }
		} else if constexpr (OP == 18) { // dependent B3 product chain x4 (scalar, compiler's packing)
#pragma unroll
			for (int k = 0; k < 4; k++) M = M * A;
		} else if constexpr (OP == 19) { // dependent B3 product chain x4 (quad-cooperative rows)
#pragma unroll
			for (int k = 0; k < 4; k++) M = mul_coop(M, A, u);
		} else if constexpr (OP == 20) { // dependent orthonormalize chain x4
#pragma unroll
			for (int k = 0; k < 4; k++) { M = orthonormalized(M); M.r[0].x += b; }
		} else if constexpr (OP == 21) { // dependent normalize chain x16
#pragma unroll
			for (int k = 0; k < 16; k++) { vv = normalized(vv); vv.x += b; }
		} else if constexpr (OP == 22) { // dependent normalize chain x16 (quad-cooperative)
#pragma unroll
			for (int k = 0; k < 16; k++) { vv = normalized_coop(vv, u); vv.x += b; }
		} else if constexpr (OP == 23) { // dependent X3 product chain x4
#pragma unroll
			for (int k = 0; k < 4; k++) X = X * XA;
		} else if constexpr (OP == 24) { // dependent f32 quotient via an fp64 reciprocal + Newton, div_fixup x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = div_rcp64(d, a);
		} else if constexpr (OP == 25) { // dependent normalize with a shared fp64 reciprocal x16
#pragma unroll
			for (int k = 0; k < 16; k++) { vv = normalized_rcp64(vv); vv.x += b; }
		} else if constexpr (OP == 26) { // 4 independent fp64 mul chains x4
#pragma unroll
			for (int k = 0; k < 4; k++) { x = x * y; x2 = x2 * z; x3 = x3 * y; x4 = x4 * z; }
		} else if constexpr (OP == 27) { // dependent cvt f32->f64->f32 x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = (float)((double)a);
		} else if constexpr (OP == 28) { // dependent v_mul_f32 chain x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = a * b;
		} else if constexpr (OP == 29) { // 4 independent IEEE fp32 divisions by one divisor x4
#pragma unroll
			for (int k = 0; k < 4; k++) { a = a / d; a2 = a2 / d; a3 = a3 / d; a4 = a4 / d; d += 1e-7f; }
		} else if constexpr (OP == 30) { // dependent fp64 add chain x16
#pragma unroll
			for (int k = 0; k < 16; k++) x = x + y;
		} else if constexpr (OP == 32) { // dependent exact fp64-reciprocal division x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = div_exact64(d, a);
		} else if constexpr (OP == 33) { // dependent exact normalize (shared fp64 reciprocal) x16
#pragma unroll
			for (int k = 0; k < 16; k++) { vv = normalized_exact64(vv); vv.x += b; }
		} else if constexpr (OP == 34) { // dependent degree-17 double sin polynomial x16
#pragma unroll
			for (int k = 0; k < 16; k++) x = sin_poly64(x) + 0.5;
		} else if constexpr (OP == 35) { // dependent gd_sqrt (fp64 rsq + Newton) x16
#pragma unroll
			for (int k = 0; k < 16; k++) a = gd_sqrt(a) + d;
		} else if constexpr (OP == 36) { // dependent packed-column B3 product chain x4
#pragma unroll
			for (int k = 0; k < 4; k++) PM = pmul(PM, PA);
		} else if constexpr (OP == 31) { // 4 independent fp64 add chains x4
#pragma unroll
			for (int k = 0; k < 4; k++) { x = x + y; x2 = x2 + z; x3 = x3 + y; x4 = x4 + z; }
		}
	}
	asm volatile("" :: "v"(a), "v"(PM.xy[0].x), "v"(PM.z[2]), "v"(M.r[0].x), "v"(vv.x), "v"(X.o.x), "v"(x));
	long long t1 = clock64();
	out[blockIdx.x * 64 + threadIdx.x] = a + a2 + a3 + a4 + (float)idx + p.x + p.y + q.x + q.y + M.r[0].x + M.r[1].y + M.r[2].z + M.r[2].x + PM.xy[0].x + PM.xy[1].y + PM.z[2] + PM.xy[2].x + vv.x + vv.y + vv.z + X.o.x + X.b.r[1].z + X.o.z;
	outd[blockIdx.x * 64 + threadIdx.x] = x + x2 + x3 + x4;
	if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
double run(float *o, double *od, long long *c, long long *h, int blocks) {
	hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(64), 0, 0, o, od, c, 1.25f);
	hipDeviceSynchronize();
	hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(64), 0, 0, o, od, c, 1.25f);
	hipMemcpy(h, c, blocks * sizeof(long long), hipMemcpyDeviceToHost);
	double s = 0;
	for (int i = 0; i < blocks; i++) s += (double)h[i];
	return s / blocks;
}

int main() {
	const int blocks = 256;
	float *o; double *od; long long *c;
	hipMalloc(&o, blocks * 64 * sizeof(float));
	hipMalloc(&od, blocks * 64 * sizeof(double));
	hipMalloc(&c, blocks * sizeof(long long));
	long long h[blocks];
	const char *names[] = {"fma_f32 dep", "fma_f32 indep4", "fma_f64 dep", "fma_f64 indep4", "div_f32 dep", "div_f32 indep4",
			"sqrt_f32(+add) dep", "sqrt_f32(+add) indep4", "div_f64 dep", "sin_f64(+add) dep", "acos_f64(*0.5) dep",
			"ds_read_b32 chase", "sqrt_f64(+add) dep", "cvt+add_f64+cvt dep", "mul+add f32 dep", "pk_mul_f32 indep2 (per pk op)", "mul_f32 indep4", "pk_add_f32 indep2 (per pk op)", "B3*B3 dep", "B3*B3 quad-coop dep", "orthonormalize dep", "normalize V3 dep", "normalize V3 quad-coop dep", "X3*X3 dep", "div_rcp64 dep", "normalize rcp64 dep", "mul_f64 indep4",
			"cvt f32-f64-f32 dep", "mul_f32 dep", "div_f32 same-divisor indep4", "add_f64 dep", "add_f64 indep4",
			"div_exact64 dep", "normalize exact64 dep", "sin_poly64(+add) dep", "gd_sqrt(+add) dep", "B3*B3 packed-xy dep"};
	double per[] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 4, 4, 16, 16, 16, 8, 16, 16, 16, 4, 4, 4, 16, 16, 4, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
	double r[36];
	r[0] = run<0>(o, od, c, h, blocks); r[1] = run<1>(o, od, c, h, blocks); r[2] = run<2>(o, od, c, h, blocks);
	r[3] = run<3>(o, od, c, h, blocks); r[4] = run<4>(o, od, c, h, blocks); r[5] = run<5>(o, od, c, h, blocks);
	r[6] = run<6>(o, od, c, h, blocks); r[7] = run<7>(o, od, c, h, blocks); r[8] = run<8>(o, od, c, h, blocks);
	r[9] = run<9>(o, od, c, h, blocks); r[10] = run<10>(o, od, c, h, blocks); r[11] = run<11>(o, od, c, h, blocks);
	r[12] = run<12>(o, od, c, h, blocks); r[13] = run<13>(o, od, c, h, blocks); r[14] = run<14>(o, od, c, h, blocks);
	r[15] = run<15>(o, od, c, h, blocks); r[16] = run<16>(o, od, c, h, blocks); r[17] = run<17>(o, od, c, h, blocks);
	r[18] = run<18>(o, od, c, h, blocks); r[19] = run<19>(o, od, c, h, blocks); r[20] = run<20>(o, od, c, h, blocks);
	r[21] = run<21>(o, od, c, h, blocks); r[22] = run<22>(o, od, c, h, blocks); r[23] = run<23>(o, od, c, h, blocks);
	r[24] = run<24>(o, od, c, h, blocks); r[25] = run<25>(o, od, c, h, blocks); r[26] = run<26>(o, od, c, h, blocks);
	r[27] = run<27>(o, od, c, h, blocks); r[28] = run<28>(o, od, c, h, blocks); r[29] = run<29>(o, od, c, h, blocks);
	r[30] = run<30>(o, od, c, h, blocks); r[31] = run<31>(o, od, c, h, blocks);
	r[32] = run<32>(o, od, c, h, blocks); r[33] = run<33>(o, od, c, h, blocks); r[34] = run<34>(o, od, c, h, blocks);
	r[35] = run<35>(o, od, c, h, blocks); r[36] = run<36>(o, od, c, h, blocks);
	for (int i = 0; i < 37; i++)
		printf("{\"op\": \"%s\", \"cycles_per_op\": %.2f}\n", names[i], r[i] / (REPS * per[i]));
	return 0;
}
