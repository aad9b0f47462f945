// Device self-tests and known-answer tests: the solve's own device functions (square root,
// division, the glibc transcendental restatements, QCP, the cone / twist limit query, the
// Transform3D ops) on the device, against IEEE results, host glibc values and the reference's
// unit-test inputs (tests/golden/reference_kats.json; DESIGN.md §4 Numerics, §7).
#include "host.h"

#include "bone_step.h"

using namespace mbik_host;

namespace {
// ---- Device known-answer tests: the solve kernel's own device functions on the reference's
// unit-test inputs (tests/golden/reference_kats.json: tests/test_qcp.h, test_ik_kusudama_3d.h,
// test_ik_node_3d.h), so the HIP code -- not only the oracle -- is pinned to the reference. ----
// QCP::weighted_superpose + get_translation (qcp.cpp:220-248, 135-137) with the primitives and the
// order of bone_step's one-lane branch: the centroids accumulated from zero in float with a
// double weight sum and divided through divs, the fp64 inner-product sums of qcp_accumulate in
// heading order, then qcp_single (one pair) or qcp_adjugate.  out: quaternion (x, y, z, w) and
// translation, for the plain (SEL false) and the select-form (SEL true) normalizations.
template <bool SEL>
__device__ void kat_qcp(const float *mv, const float *tg, const double *w, int n, int translate, double prec, float *out) {
	auto M = [&](int i) { return v3(mv[3 * i], mv[3 * i + 1], mv[3 * i + 2]); };
	auto T = [&](int i) { return v3(tg[3 * i], tg[3 * i + 1], tg[3 * i + 2]); };
	V3 mc = v3(0, 0, 0), tc = v3(0, 0, 0);
	if (translate) {
		double wsum = 0;
		for (int i = 0; i < n; i++) {
			mc = mc + M(i) * (float)w[i];
			tc = tc + T(i) * (float)w[i];
			wsum += w[i];
		}
		if (wsum > 0) {
			mc = divs(mc, (float)wsum);
			tc = divs(tc, (float)wsum);
		}
	}
	const V3 nmc = mc * -1.0f, ntc = tc * -1.0f;
	QSums S = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
	for (int i = 0; i < n; i++) {
		const V3 c1 = translate ? T(i) + ntc : T(i), c2 = translate ? M(i) + nmc : M(i);
		qcp_accumulate(S, c1 * (float)w[i], c1, c2, w[i]);
	}
	Q q;
	if (n == 1) q = qcp_single<SEL>(translate ? M(0) + nmc : M(0), translate ? T(0) + ntc : T(0));
	else q = qcp_adjugate(S, prec);
	const V3 tr = tc - mc;
	out[0] = q.x; out[1] = q.y; out[2] = q.z; out[3] = q.w;
	out[4] = tr.x; out[5] = tr.y; out[6] = tr.z;
}
__global__ __launch_bounds__(64) void mbik_kat_qcp_kernel(const float *mv, const float *tg, const double *w, int n, int translate,
		double prec, float *out) {
	if (threadIdx.x == 0) kat_qcp<false>(mv, tg, w, n, translate, prec, out);
	if (threadIdx.x == 1) kat_qcp<true>(mv, tg, w, n, translate, prec, out + 7);
}
// IKKusudama3D::get_local_point_in_limits (ik_kusudama_3d.cpp:273-332) through the solve's own
// local_point_in_limits on a plan's setup tables (constraint slot `slot` of skeleton s), both
// normalization forms.  out: point (3) + in_bounds (as float) per form.
__global__ __launch_bounds__(64) void mbik_kat_limits_kernel(DevPlan t, int slot, int s, float px, float py, float pz, float *out,
		double *ib) {
	// the topology tables straight from the plan's blob in device memory (the solve copies it to LDS)
	const uint32_t *topo = reinterpret_cast<const uint32_t *>(t.topo_blob);
#define MBIK_REPOINT(T, name) t.name = reinterpret_cast<const T *>(topo + t.o_##name);
	MBIK_TOPO_TABLES(MBIK_REPOINT)
#undef MBIK_REPOINT
	double in_bounds = 1.0;
	V3 r;
	if (threadIdx.x == 0) r = local_point_in_limits<kTab64, false>(t, slot, (size_t)s, v3(px, py, pz), in_bounds);
	else if (threadIdx.x == 1) r = local_point_in_limits<kTab64, true>(t, slot, (size_t)s, v3(px, py, pz), in_bounds);
	else return;
	out[3 * threadIdx.x] = r.x;
	out[3 * threadIdx.x + 1] = r.y;
	out[3 * threadIdx.x + 2] = r.z;
	ib[threadIdx.x] = in_bounds;
}
// Transform3D ops of the IKNode3D tree (ik_node_3d.cpp:56-113): op 0 a * b, op 1 a.affine_inverse().
__global__ __launch_bounds__(64) void mbik_kat_xform_kernel(int op, const float *a, const float *b, float *out) {
	if (threadIdx.x != 0) return;
	auto X = [](const float *v) { return X3{bset(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]), v3(v[9], v[10], v[11])}; };
	const X3 r = op == 0 ? X(a) * X(b) : affine_inverse(X(a));
	const float v[12] = {r.b.r[0].x, r.b.r[0].y, r.b.r[0].z, r.b.r[1].x, r.b.r[1].y, r.b.r[1].z,
			r.b.r[2].x, r.b.r[2].y, r.b.r[2].z, r.o.x, r.o.y, r.o.z};
	for (int i = 0; i < 12; i++) out[i] = v[i];
}
} // namespace

namespace {
__global__ void mbik_selftest_math_kernel(unsigned long long *out) {
	const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
	unsigned long long bad = 0, nan_bad = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += nthreads) {
		const float x = __uint_as_float((unsigned)i);
		const float ref = sqrtf(x), got = gd_sqrt(x);
		const bool rn = ref != ref, gn = got != got;
		if (rn != gn) nan_bad++;
		else if (!rn && __float_as_uint(ref) != __float_as_uint(got)) bad++;
	}
	if (bad) atomicAdd(&out[0], bad);
	if (nan_bad) atomicAdd(&out[1], nan_bad);
}
// mbik_selftest_div: the kernel's float quotients (gd_math.h gd_quot / gd_pow2_over /
// gd_sqrt_rcp) against the compiler's IEEE division.  out[c] counts mismatches per class c
// (MBIK_DIV_*); out[8 + 2c], out[9 + 2c] keep the bit patterns of one mismatching operand pair.
__device__ __forceinline__ uint64_t st_mix(uint64_t &s) {
	uint64_t z = (s += 0x9e3779b97f4a7c15ull);
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}
__device__ __forceinline__ bool same_f(float x, float y) { return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y); }
__device__ __forceinline__ void div_tally(unsigned long long *out, int cls, float ref, float got, float a, float b) {
	if (same_f(ref, got)) return;
	if (atomicAdd(&out[cls], 1ull) == 0ull) {
		out[8 + 2 * cls] = __float_as_uint(a);
		out[9 + 2 * cls] = __float_as_uint(b);
	}
}
__device__ const unsigned kDivSpecials[] = {0x00000000u, 0x80000000u, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0xffc00001u,
		0x00000001u, 0x80000003u, 0x007fffffu, 0x807fffffu, 0x00800000u, 0x7f7fffffu, 0xff7fffffu, 0x3f800000u, 0xbf800000u,
		0x3f7fffffu, 0x3f800001u, 0x34000000u, 0x5f000000u, 0x1f800000u, 0x00400000u, 0x7f000000u, 0x40400000u, 0x3dcccccdu};
__device__ const unsigned kDivFixed[] = {0x3f800000u, 0x40000000u, 0x3f800001u, 0x3f7fffffu, 0x40400000u, 0x3dcccccdu,
		0x4049a0b1u, 0x00000003u, 0x00400001u, 0x7e800001u, 0xbf9d70a4u, 0x3a83126fu};
// dividends of normalized(): a component against the rounded length of its vector
__device__ const unsigned kDivNormA[] = {0x3f800000u, 0x3f333333u, 0x0da24260u, 0x00200000u, 0xc0200000u, 0x00000001u,
		0x7f7fffffu, 0x80000000u};
__global__ void mbik_selftest_div_kernel(int cls, int sel, uint64_t iters, unsigned long long *out) {
	const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nthreads = (uint64_t)gridDim.x * blockDim.x;
	constexpr int NS = sizeof(kDivSpecials) / sizeof(kDivSpecials[0]);
	if (cls == MBIK_DIV_SPECIALS) {
		if (tid < NS * NS) {
			const float a = __uint_as_float(kDivSpecials[tid % NS]), b = __uint_as_float(kDivSpecials[tid / NS]);
			div_tally(out, cls, a / b, gd_div(a, b), a, b);
		}
	} else if (cls == MBIK_DIV_ALL_DIVIDENDS) { // every float dividend, divisor kDivFixed[sel]
		const float b = __uint_as_float(kDivFixed[sel]);
		for (uint64_t i = tid; i < (1ull << 32); i += nthreads) {
			const float a = __uint_as_float((unsigned)i);
			div_tally(out, cls, a / b, gd_div(a, b), a, b);
		}
	} else if (cls == MBIK_DIV_RANDOM) { // random pairs: free exponents, and close exponents
		uint64_t s = tid * 0x2545f4914f6cdd1dull + 777;
		for (uint64_t it = 0; it < iters; it++) {
			const uint64_t z = st_mix(s);
			unsigned ab = (unsigned)z, bb = (unsigned)(z >> 32);
			if (it & 1) {
				ab = (ab & 0x807fffffu) | ((110u + ((z >> 8) & 31)) << 23);
				bb = (bb & 0x807fffffu) | ((110u + ((z >> 40) & 31)) << 23);
			}
			const float a = __uint_as_float(ab), b = __uint_as_float(bb);
			div_tally(out, cls, a / b, gd_div(a, b), a, b);
		}
	} else if (cls == MBIK_DIV_MIDPOINTS) { // exact denormal midpoints m * 2^-150, m odd
		uint64_t s = tid * 0x9e3779b97f4a7c15ull + 99;
		for (uint64_t it = 0; it < iters; it++) {
			const uint64_t z = st_mix(s);
			const int mbits = 1 + (int)(z % 23);
			const uint32_t m = ((uint32_t)(z >> 8) & ((1u << mbits) - 1u)) | 1u;
			const int bbits = 1 + (int)((z >> 40) % (uint64_t)(24 - mbits + 1));
			const uint32_t B = ((uint32_t)(z >> 20) & ((1u << bbits) - 1u)) | 1u | (1u << (bbits - 1));
			const int e = 100 + (int)((z >> 50) % 60);
			const double bd = ldexp((double)B, e - bbits), ad = ldexp((double)((uint64_t)m * B), e - bbits - 150);
			float a = (float)ad, b = (float)bd;
			if ((double)a != ad || (double)b != bd) continue;
			a = (z >> 62) & 1 ? -a : a;
			b = (z >> 63) ? -b : b;
			div_tally(out, cls, a / b, gd_div(a, b), a, b);
		}
	} else if (cls == MBIK_DIV_POW2_NUMERATOR) { // N / b, N = 0.5, 1, 2, every float b
		for (uint64_t i = tid; i < (1ull << 32); i += nthreads) {
			const float b = __uint_as_float((unsigned)i);
			div_tally(out, cls, 0.5f / b, gd_pow2_over(0.5f, b), 0.5f, b);
			div_tally(out, cls, 1.0f / b, gd_pow2_over(1.0f, b), 1.0f, b);
			div_tally(out, cls, 2.0f / b, gd_pow2_over(2.0f, b), 2.0f, b);
		}
	} else if (cls == MBIK_DIV_NORMALIZE) { // a / sqrtf(l), every float l, a = kDivNormA[sel]
		const float a = __uint_as_float(kDivNormA[sel]);
		for (uint64_t i = tid; i < (1ull << 32); i += nthreads) {
			const float l = __uint_as_float((unsigned)i);
			float len;
			const GdRcp d = gd_sqrt_rcp(l, len);
			div_tally(out, cls, a / sqrtf(l), gd_quot(a, d), a, l);
			div_tally(out, cls, sqrtf(l), len, a, l);
		}
	}
}
// mbik_selftest_libm: the device's transcendental call sites against host-computed values.
// out[0] = observable mismatches, out[1] = lowest such index (atomicMin; ~0 if none),
// out[2] = results whose bits differ at all.
template <class T>
__device__ __forceinline__ bool same_bits(T a, T b) {
	if (a != a && b != b) return true; // NaN payloads aside
	return a == b && (a != 0 || signbit(a) == signbit(b));
}
// Two double results the solve cannot tell apart: the setup's double cosines are only
// compared with float-valued doubles (ik_open_cone_3d.cpp:358-381, :285-321) or rounded to
// float (:36-120), so they are equivalent when no float lies in [lo, hi) ... (lo, hi] and
// both round to the same float (a comparison d > c, d a float, then resolves alike).
__device__ __forceinline__ bool same_for_float_use(double a, double b) {
	if (same_bits(a, b)) return true;
	if (a != a || b != b) return false;
	const double lo = a < b ? a : b, hi = a < b ? b : a;
	if ((float)lo != (float)hi) return false;
	return !((double)__double2float_rd(hi) > lo); // no float f with lo < f <= hi
}
__global__ void mbik_selftest_libm_kernel(int fn, uint64_t first, uint64_t count, const double *__restrict__ inputs,
		const void *__restrict__ expected, unsigned long long *out) {
	const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
	unsigned long long bad = 0, lo = ~0ull, diff = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += nthreads) {
		const float x = __uint_as_float((unsigned)(first + i));
		bool ok, exact;
		const bool f32 = fn <= MBIK_LIBM_SLERP_SCALE0 || fn >= MBIK_LIBM_SINF_SSE2;
		if (f32) {
			const float e = static_cast<const float *>(expected)[i];
			const float g = fn == MBIK_LIBM_SINF ? sin_f(x) : fn == MBIK_LIBM_COSF ? cos_f(x) : fn == MBIK_LIBM_ACOSF ? acos_f(x)
					: fn == MBIK_LIBM_SLERP_SCALE0 ? slerp_scale0(x) : fn == MBIK_LIBM_SINF_SSE2 ? sin_f(x, LIBM_SSE2)
					: fn == MBIK_LIBM_COSF_SSE2 ? cos_f(x, LIBM_SSE2) : fn == MBIK_LIBM_SLERP_SCALE0_SSE2 ? slerp_scale0(x, LIBM_SSE2)
					: (x > -0.5f && x < 1.0f) ? glibc::acosf_unit(x) : acos_f(x); // MBIK_LIBM_ACOSF_UNIT
			ok = exact = same_bits(e, g);
		} else {
			const double e = static_cast<const double *>(expected)[i];
			const double g = fn == MBIK_LIBM_COS_F64_OF_F32 ? ::cos((double)x) : ::cos(inputs[i]);
			exact = same_bits(e, g);
			ok = same_for_float_use(e, g);
		}
		diff += !exact;
		if (!ok) {
			bad++;
			lo = i < lo ? i : lo;
		}
	}
	if (bad) {
		atomicAdd(&out[0], bad);
		atomicMin(&out[1], lo);
	}
	if (diff) atomicAdd(&out[2], diff);
}
} // namespace
extern "C" {

int32_t mbik_selftest_math(int32_t device, uint64_t out[2]) {
	if (!out) return fail(MBIK_EINVAL, "null output");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MBIK_ENODEV, "no HIP device");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device out of range");
	DeviceGuard guard(device);
	unsigned long long *d = nullptr;
	if (hipMalloc(&d, 2 * sizeof(unsigned long long)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc");
	int rc = MBIK_OK;
	if (hipMemset(d, 0, 2 * sizeof(unsigned long long)) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemset");
	if (rc == MBIK_OK) {
		hipLaunchKernelGGL(mbik_selftest_math_kernel, dim3(8192), dim3(256), 0, 0, d);
		if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = fail(MBIK_EHIP, "self-test kernel");
	}
	unsigned long long h[2] = {0, 0};
	if (rc == MBIK_OK && hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemcpy");
	(void)hipFree(d);
	out[0] = h[0];
	out[1] = h[1];
	return rc;
}

// A device buffer of n bytes holding the host data (or zeroed): the KAT entry points' staging.
namespace {
struct DevBuf {
	void *p = nullptr;
	~DevBuf() {
		if (p) (void)hipFree(p);
	}
	int put(const void *h, size_t n) {
		if (hipMalloc(&p, std::max<size_t>(n, 8)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc");
		if (h ? hipMemcpy(p, h, n, hipMemcpyHostToDevice) != hipSuccess : hipMemset(p, 0, std::max<size_t>(n, 8)) != hipSuccess)
			return fail(MBIK_EHIP, "hipMemcpy");
		return MBIK_OK;
	}
};
int kat_device(int32_t device) {
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MBIK_ENODEV, "no HIP device");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device out of range");
	return MBIK_OK;
}
int kat_finish(void *dst, const DevBuf &b, size_t n) {
	if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return fail(MBIK_EHIP, "KAT kernel");
	if (hipMemcpy(dst, b.p, n, hipMemcpyDeviceToHost) != hipSuccess) return fail(MBIK_EHIP, "hipMemcpy");
	return MBIK_OK;
}
} // namespace

int32_t mbik_selftest_qcp(int32_t n, const float *moved, const float *target, const double *weights, int32_t translate,
		double precision, int32_t device, float out[14]) {
	if (n < 1 || !moved || !target || !weights || !out) return fail(MBIK_EINVAL, "n >= 1 and non-null buffers");
	if (int rc = kat_device(device)) return rc;
	DeviceGuard guard(device);
	DevBuf m, t, w, o;
	int rc = m.put(moved, 12 * (size_t)n);
	if (!rc) rc = t.put(target, 12 * (size_t)n);
	if (!rc) rc = w.put(weights, 8 * (size_t)n);
	if (!rc) rc = o.put(nullptr, 14 * sizeof(float));
	if (rc) return rc;
	hipLaunchKernelGGL(mbik_kat_qcp_kernel, dim3(1), dim3(64), 0, 0, (const float *)m.p, (const float *)t.p, (const double *)w.p, n,
			translate, precision, (float *)o.p);
	return kat_finish(out, o, 14 * sizeof(float));
}

int32_t mbik_selftest_point_in_limits(const mbik_plan *p, int32_t slot, int32_t skeleton, const float point[3], float out[6],
		double in_bounds[2]) {
	if (!p || !point || !out || !in_bounds) return fail(MBIK_EINVAL, "null argument");
	if (slot < 0 || slot >= p->host.NC || skeleton < 0 || skeleton >= p->host.N) return fail(MBIK_EINVAL, "slot or skeleton out of range");
	DeviceGuard guard(p->device);
	// the topology blob the kernel reads, uploaded with the plan's launch schedule (finish_plan):
	// the plan is only read here, never rescheduled, so a solve of it may be in flight
	if (!p->dev.topo_blob) return fail(MBIK_EHIP, "plan has no topology blob");
	DevBuf o, ib;
	int rc = o.put(nullptr, 6 * sizeof(float));
	if (!rc) rc = ib.put(nullptr, 2 * sizeof(double));
	if (rc) return rc;
	DevPlan d = p->dev; // the plain [item][field][N] tables (kTab64)
	hipLaunchKernelGGL(mbik_kat_limits_kernel, dim3(1), dim3(64), 0, 0, d, slot, skeleton, point[0], point[1], point[2], (float *)o.p,
			(double *)ib.p);
	if ((rc = kat_finish(out, o, 6 * sizeof(float))) != MBIK_OK) return rc;
	if (hipMemcpy(in_bounds, ib.p, 2 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return fail(MBIK_EHIP, "hipMemcpy");
	return MBIK_OK;
}

int32_t mbik_selftest_xform(int32_t op, const float a[12], const float b[12], int32_t device, float out[12]) {
	if ((op != 0 && op != 1) || !a || (op == 0 && !b) || !out) return fail(MBIK_EINVAL, "op 0 (a * b) or 1 (affine_inverse(a)), non-null buffers");
	if (int rc = kat_device(device)) return rc;
	DeviceGuard guard(device);
	DevBuf da, db, o;
	int rc = da.put(a, 12 * sizeof(float));
	if (!rc) rc = db.put(op == 0 ? b : a, 12 * sizeof(float));
	if (!rc) rc = o.put(nullptr, 12 * sizeof(float));
	if (rc) return rc;
	hipLaunchKernelGGL(mbik_kat_xform_kernel, dim3(1), dim3(64), 0, 0, op, (const float *)da.p, (const float *)db.p, (float *)o.p);
	return kat_finish(out, o, 12 * sizeof(float));
}

int32_t mbik_selftest_div(int32_t device, uint64_t random_iterations, uint64_t out[20]) {
	if (!out) return fail(MBIK_EINVAL, "null output");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MBIK_ENODEV, "no HIP device");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device out of range");
	DeviceGuard guard(device);
	unsigned long long *d = nullptr;
	if (hipMalloc(&d, 20 * sizeof(unsigned long long)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc");
	int rc = MBIK_OK;
	if (hipMemset(d, 0, 20 * sizeof(unsigned long long)) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemset");
	auto run = [&](int cls, int sel) {
		if (rc != MBIK_OK) return;
		hipLaunchKernelGGL(mbik_selftest_div_kernel, dim3(8192), dim3(256), 0, 0, cls, sel, random_iterations, d);
		if (hipGetLastError() != hipSuccess) rc = fail(MBIK_EHIP, "self-test kernel launch");
	};
	run(MBIK_DIV_SPECIALS, 0);
	for (int k = 0; k < 12; k++) run(MBIK_DIV_ALL_DIVIDENDS, k);
	run(MBIK_DIV_RANDOM, 0);
	run(MBIK_DIV_MIDPOINTS, 0);
	run(MBIK_DIV_POW2_NUMERATOR, 0);
	for (int k = 0; k < 8; k++) run(MBIK_DIV_NORMALIZE, k);
	if (rc == MBIK_OK && hipDeviceSynchronize() != hipSuccess) rc = fail(MBIK_EHIP, "self-test kernel");
	unsigned long long h[20] = {};
	if (rc == MBIK_OK && hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemcpy");
	(void)hipFree(d);
	for (int i = 0; i < 20; i++) out[i] = h[i];
	return rc;
}

int32_t mbik_selftest_libm(int32_t fn, uint64_t first, uint64_t count, const double *inputs, const void *expected,
		uint64_t out[3], void *hip_stream) {
	if (!out || !expected) return fail(MBIK_EINVAL, "null argument");
	if (fn < MBIK_LIBM_SINF || fn > MBIK_LIBM_ACOSF_UNIT) return fail(MBIK_EINVAL, "unknown function code");
	if (fn == MBIK_LIBM_COS_F64 ? !inputs : first + count > (1ull << 32)) return fail(MBIK_EINVAL, "input range");
	out[0] = 0;
	out[1] = ~0ull;
	out[2] = 0;
	if (count == 0) return MBIK_OK;
	hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
	unsigned long long *d = nullptr;
	if (hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc");
	unsigned long long h[3] = {0, ~0ull, 0};
	int rc = MBIK_OK;
	if (hipMemcpyAsync(d, h, sizeof(h), hipMemcpyHostToDevice, st) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemcpyAsync");
	if (rc == MBIK_OK) {
		hipLaunchKernelGGL(mbik_selftest_libm_kernel, dim3(4096), dim3(256), 0, st, (int)fn, first, count, inputs, expected, d);
		if (hipGetLastError() != hipSuccess) rc = fail(MBIK_EHIP, "self-test launch");
	}
	if (rc == MBIK_OK && hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess) rc = fail(MBIK_EHIP, "hipMemcpyAsync");
	if (rc == MBIK_OK && hipStreamSynchronize(st) != hipSuccess) rc = fail(MBIK_EHIP, "self-test kernel");
	(void)hipFree(d);
	out[0] = h[0];
	out[1] = h[1];
	out[2] = h[2];
	return rc;
}

} // extern "C"
