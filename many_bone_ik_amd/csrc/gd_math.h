// Godot-4.3 core math semantics (real_t == float) for host and device code.
//
// The reference module (Ughuuu/many_bone_ik) does its arithmetic through Godot's
// Vector3 / Quaternion / Basis / Transform3D.  This header gives
// the product -- the gfx950 solve kernel and the host plan builder -- the same operation
// order, so the GPU reproduces the reference's float rounding instead of an algebraically
// equivalent but differently rounded formula.  Compile with -ffp-contract=off where the
// rounding matters (the kernel does; see build.py).
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GDI __host__ __device__ __forceinline__
#else
#define GDI inline
#endif

namespace gd {
#if !defined(__HIPCC__)
using std::isfinite; // a plain C++ compiler (the sanitizer build, tools/san) puts them in std::
using std::isnan;
#endif

// Timing-only ablation builds: tools/ablate.sh compiles with -DMBIK_ABLATE=<mask of the bits
// below> to time the solve with one phase removed (the results are wrong on purpose).  The
// shipped library is built with mask 0, where every `if constexpr (kAblate & ...)` is dead.
#ifndef MBIK_ABLATE
#define MBIK_ABLATE 0
#endif
enum : unsigned {
	ABL_SQRT = 1, ABL_ORTHO = 2, ABL_MATMUL = 4, ABL_SOA = 8, ABL_SOALDS = 16, ABL_CONVERT = 32, ABL_SLERP = 64,
	ABL_SWING = 128, ABL_TWIST = 256, ABL_XCD = 512,
	// load-site ablations (the same loads, all from one hot address of the skeleton's own state):
	// the effector path walks' locals, the checkpoint globals, the targets, the other local reads
	ABL_WALK = 1024, ABL_GCK = 2048, ABL_TGT = 4096, ABL_LOCAL = 8192
};
constexpr unsigned kAblate = MBIK_ABLATE;

constexpr double CMP_EPSILON = 0.00001;
constexpr double PI = 3.1415926535897932384626433833;

// Square root, correctly rounded (IEEE), as Godot's Math::sqrt(float) on x86.
// On the device: v_rsq_f64 of the widened input and one fp64 Newton correction, rounded
// once to float.  tools/sqrt_exhaustive.hip checks all 2^32 inputs against the compiler's
// correctly rounded sqrtf: identical for every non-NaN result (NaN payloads may differ;
// NaN-ness does not).  Half the latency of the fp32 sequence (55 vs 107 cycles, same tool).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_IEEE_SQRT)
GDI float gd_sqrt(float x) {
	if constexpr (kAblate & ABL_SQRT) return __builtin_amdgcn_sqrtf(x); // timing experiment only (1 ulp)
	const double xd = x;
	const double y = __builtin_amdgcn_rsq(xd);
	const double g = xd * y, h = 0.5 * y;
	const double e = fma(-g, g, xd);
	const float r = (float)fma(e, h, g);
	return __builtin_amdgcn_class(x, 0x260) ? x : r; // +-0 and +inf pass through
}
#else
GDI float gd_sqrt(float x) { return sqrtf(x); }
#endif

// Float quotient a / b, correctly rounded (IEEE), as the reference's x86 divss.
// On the device: r = 1/(double)b from v_rcp_f64 and one Newton step (relative error ~2^-52),
// q0 = (double)a * r, one fp64 residual correction q1 = q0 + (a - b*q0) * r, rounded once to
// float; v_div_fixup_f32 supplies the IEEE result for zero / infinite / NaN operands.  Exact:
// a quotient of two floats that is not a float rounding midpoint lies at least 2^-49 (relative)
// from every midpoint, far beyond q1's error; a midpoint quotient (possible only for denormal
// results) is a double, which the residual correction lands on exactly, so the final rounding
// ties to even as IEEE does.  tools/div_exact_check.hip checks special pairs, all 2^32
// dividends for a set of divisors, random pairs and constructed midpoints on the device.
// A divisor shared by several quotients (normalized(), divs()) computes its reciprocal once.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_IEEE_DIV)
struct GdRcp {
	float b;
	double bd, r;
};
GDI GdRcp gd_rcp(float b) {
	const double bd = b;
	double r = __builtin_amdgcn_rcp(bd);
	const double e = fma(-bd, r, 1.0);
	return GdRcp{b, bd, fma(e, r, r)};
}
GDI float gd_quot(float a, const GdRcp &d) {
	const double ad = a;
	const double q0 = ad * d.r;
	const double rem = fma(-d.bd, q0, ad);
	return __builtin_amdgcn_div_fixupf((float)fma(rem, d.r, q0), d.b, a);
}
#else
struct GdRcp {
	float b;
};
GDI GdRcp gd_rcp(float b) { return GdRcp{b}; }
GDI float gd_quot(float a, const GdRcp &d) { return a / d.b; }
#endif
GDI float gd_div(float a, float b) { return gd_quot(a, gd_rcp(b)); }
// N / b for a power-of-two constant N (0.5f, 1.0f, 2.0f: Basis::set_quaternion's 2/d,
// get_quaternion's 0.5/s, inverse's 1/det, ...).  (double)N * r is r scaled exactly, so the
// quotient is one rounding of r, and no residual correction is needed: such a quotient is
// never a float rounding midpoint (N/b = m * 2^-150 with m odd would need b = N * 2^150 / m,
// not a float), and r is far closer to N/b than any midpoint.  tools/div_exact_check.hip
// checks all 2^32 divisors for N = 0.5, 1, 2.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_IEEE_DIV)
GDI float gd_pow2_over(float n, float b) {
	const GdRcp d = gd_rcp(b);
	return __builtin_amdgcn_div_fixupf((float)((double)n * d.r), b, n);
}
#else
GDI float gd_pow2_over(float n, float b) { return n / b; }
#endif

// x / RN(sqrt(l)) for several x at once (normalized()): the square root as gd_sqrt, and the
// reciprocal of the rounded root refined from the same v_rsq_f64 estimate (one Newton step,
// ~2^-44) instead of a separate v_rcp_f64; the quotients as gd_quot.  Same exactness argument
// (the residual correction squares the reciprocal's error).  Host: sqrtf and IEEE division.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_IEEE_DIV) && !defined(MBIK_IEEE_SQRT)
GDI GdRcp gd_sqrt_rcp(float l, float &len) {
	const double ld = l;
	const double y = __builtin_amdgcn_rsq(ld);
	const double g = ld * y, h = 0.5 * y;
	const double e = fma(-g, g, ld);
	len = __builtin_amdgcn_class(l, 0x260) ? l : (float)fma(e, h, g);
	const double Ld = len;
	const double e2 = fma(-Ld, y, 1.0);
	return GdRcp{len, Ld, fma(e2, y, y)};
}
#else
GDI GdRcp gd_sqrt_rcp(float l, float &len) {
	len = gd_sqrt(l);
	return gd_rcp(len);
}
#endif

// ---------------- Float transcendentals: the platform libm of the reference ----------------
// Godot's Math::sin/cos/acos(float) call ::sinf/::cosf/::acosf (core/math/math_funcs.h).  On
// the reference's Linux x86-64 build that is glibc; the solve amplifies a 1-ulp libm
// difference ~2x per iteration, so the product reproduces glibc's float
// results bit for bit on the device and on the host, instead of OCML's own versions.
// Restated from glibc 2.35 (the image's libm):
//   sinf/cosf  sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c, in the
//              x86-64 FMA build the ifunc selects on every CPU with FMA (each a*b+c that GCC
//              contracts there is an explicit fma() here);
//   acosf      sysdeps/ieee754/flt-32/e_acosf.c (fdlibm, float arithmetic, IEEE sqrt/div).
// mbik_selftest_libm (tests/test_gpu_libm.py) proves the device results equal to the host
// libm's on all 2^32 inputs; tools/libm_exhaustive.c does the same for the oracle's copy.
//
// Third-party notices (THIRD_PARTY_NOTICES.md): the coefficient and 2/pi tables and the
// algorithms of the sinf/cosf below come from the GNU C Library, Copyright (C) 2018-2022
// Free Software Foundation, Inc., licensed under the GNU Lesser General Public License
// v2.1 or later.  acosf follows fdlibm's e_acosf.c: "Copyright (C) 1993 by Sun
// Microsystems, Inc. All rights reserved. Developed at SunPro, a Sun Microsystems, Inc.
// business. Permission to use, copy, modify, and distribute this software is freely
// granted, provided that this notice is preserved." (float conversion by Ian Lance
// Taylor, Cygnus Support).
namespace glibc {
GDI uint32_t top12(float x) { // exponent and top mantissa bits of |x|
	union {
		float f;
		uint32_t u;
	} c{x};
	return (c.u >> 20) & 0x7ffu;
}
// the four reduced-argument polynomials' coefficients (sincosf_data.c, first table; the
// second table is the first with the cosine coefficients negated)
constexpr double kHalfPiInv24 = 0x1.45F306DC9C883p+23; // 2/pi * 2^24
constexpr double kHalfPi = 0x1.921FB54442D18p0;
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5, kC3 = -0x1.6c087e89a359dp-10,
				 kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
// a*b + c as glibc's build computes it: one fused multiply-add in the FMA ifunc variant
// (s_sinf-fma.c, what every CPU with FMA selects), two roundings in the SSE2 variant
// (the plain s_sinf.c build, a host without FMA or with the FMA ifunc disabled)
template <bool FMA>
GDI double gmadd(double a, double b, double c) {
	if constexpr (FMA) return fma(a, b, c);
	else return a * b + c;
}
// sin(x) for the reduced x, x2 = x*x (sinf_poly, even quadrant)
template <bool FMA>
GDI float sin_poly(double x, double x2) {
	const double x3 = x * x2;
	const double s1 = gmadd<FMA>(x2, kS3, kS2);
	const double x7 = x3 * x2;
	const double s = gmadd<FMA>(x3, kS1, x);
	return (float)gmadd<FMA>(x7, s1, s);
}
// cos(x) for the reduced x (sinf_poly, odd quadrant, first table)
template <bool FMA>
GDI float cos_poly(double x2) {
	const double x4 = x2 * x2;
	const double c2 = gmadd<FMA>(x2, kC4, kC3);
	const double c1 = gmadd<FMA>(x2, kC1, kC0);
	const double x6 = x4 * x2;
	const double c = gmadd<FMA>(x4, kC2, c1);
	return (float)gmadd<FMA>(x6, c2, c);
}
// Payne-Hanek reduction for |y| >= 120 (reduce_large): x * 2^63 / (pi/2) from the bits of
// 2/pi, in 64-bit integers.  Returns the reduced argument and the quadrant count.
GDI double reduce_large(uint32_t xi, int &quadrant) {
	// 2/pi = 0x0.a2f9836e4e441529fc2757d1f534ddc0db629599..., read as 32-bit windows
	// starting at byte k - 3 (the __inv_pio4 table): window(k) for k = i, i + 4, i + 8.
	constexpr uint32_t w[24] = {0x000000a2u, 0x0000a2f9u, 0x00a2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
								0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
								0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
								0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
	const int i = (xi >> 26) & 15;
	const int shift = (xi >> 23) & 7;
	const uint32_t m = ((xi & 0xffffffu) | 0x800000u) << shift;
	uint64_t a = (uint64_t)(uint32_t)(m * w[i]); // low 32 bits only, as the C source's 32-bit product
	const uint64_t b = (uint64_t)m * w[i + 4];
	const uint64_t c = (uint64_t)m * w[i + 8];
	a = (c >> 32) | (a << 32);
	a += b;
	const uint64_t n = (a + (1ull << 61)) >> 62;
	a -= n << 62;
	quadrant = (int)n;
	return (double)(int64_t)a * 0x1.921FB54442D18p-62;
}
// sinf (cos_variant 0) / cosf (cos_variant 1); FMA: glibc's FMA ifunc variant, else SSE2
template <bool FMA>
GDI float sincosf(float y, int cos_variant) {
	const uint32_t t = top12(y);
	double x = y;
	if (t < 0x3f4u) { // |y| < 0.75 (abstop12(pi/4))
		if (t < 0x398u) return cos_variant ? 1.0f : y; // |y| < 2^-12
		return cos_variant ? cos_poly<FMA>(x * x) : sin_poly<FMA>(x, x * x);
	}
	int n, ns; // quadrant; quadrant for the sign pattern and table (large inputs add the sign bit)
	if (t < 0x42fu) { // |y| < 120: reduce_fast
		const double r = x * kHalfPiInv24;
		n = ((int32_t)r + 0x800000) >> 24;
		x = FMA ? fma(-(double)n, kHalfPi, x) : x - (double)n * kHalfPi; // x - n * hpi
		ns = n;
	} else if (t < 0x7f8u) {
		union {
			float f;
			uint32_t u;
		} c{y};
		x = reduce_large(c.u, n);
		ns = n + (int)(c.u >> 31);
	} else {
		return y - y; // inf or NaN -> NaN (__math_invalidf)
	}
	// sign of the reduced argument (+, -, -, +) by ns, the sin or cos polynomial by n, the
	// cosine one negated when ns is in quadrant 2 or 3 (the second table)
	const double xs = ((ns + 1) & 2) ? -x : x;
	if (((n ^ cos_variant) & 1) == 0) return sin_poly<FMA>(xs, xs * xs);
	const float c = cos_poly<FMA>(xs * xs);
	return (ns & 2) ? -c : c;
}
// acosf (e_acosf.c)
GDI float acosf(float x) {
	constexpr float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
	constexpr float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
					pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
	constexpr float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
	union {
		float f;
		int32_t i;
	} c{x};
	const int32_t hx = c.i, ix = hx & 0x7fffffff;
	if (ix >= 0x3f800000) { // |x| >= 1
		if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
		return (x - x) / (x - x);
	}
	auto rat = [&](float z) {
		const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		return p / q;
	};
	if (ix < 0x3f000000) { // |x| < 0.5
		if (ix <= 0x32800000) return pio2_hi + pio2_lo;
		const float r = rat(x * x);
		return pio2_hi - (x - (pio2_lo - x * r));
	}
	if (hx < 0) { // x <= -0.5
		const float z = (1.0f + x) * 0.5f;
		const float s = gd_sqrt(z);
		const float r = rat(z);
		const float w = r * s - pio2_lo;
		return pi - 2.0f * (s + w);
	}
	const float z = (1.0f - x) * 0.5f; // x >= 0.5
	const float s = gd_sqrt(z);
	union {
		float f;
		uint32_t u;
	} d{s};
	d.u &= 0xfffff000u;
	const float df = d.f;
	const float cc = (z - df * df) / (s + df);
	const float r = rat(z);
	const float w = r * s + cc;
	return 2.0f * (df + w);
}
// sinf for |y| <= 1.6 (the slerp coefficient's omega), branch-free: the same operations as
// sincosf above on each path -- below |y| = 0.75 the reduction's n is 0, so x - 0 * (pi/2) is
// x exactly and the reduced path computes what the direct one does -- with both polynomials
// evaluated and the result selected, so lanes on different paths do not run them in turn.
template <bool FMA>
GDI float sinf_small(float y) {
	const double x = y;
	const double r = x * kHalfPiInv24;
	const int n = ((int32_t)r + 0x800000) >> 24;
	const double xr = FMA ? fma(-(double)n, kHalfPi, x) : x - (double)n * kHalfPi;
	const double xs = ((n + 1) & 2) ? -xr : xr;
	const float sp = sin_poly<FMA>(xs, xs * xs);
	const float cp = cos_poly<FMA>(xs * xs);
	const float v = (n & 1) == 0 ? sp : ((n & 2) ? -cp : cp);
	return top12(y) < 0x398u ? y : v;
}
// acosf for 0 <= x < 1 (the slerp's cosine of the half angle), branch-free: both of acosf's
// paths for that range share one rational approximation at their own z.
GDI float acosf_unit(float x) {
	constexpr float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
	constexpr float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
					pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
	constexpr float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
	union {
		float f;
		int32_t i;
	} c{x};
	const int32_t ix = c.i & 0x7fffffff;
	const bool lo = ix < 0x3f000000; // |x| < 0.5
	const float z = lo ? x * x : (1.0f - x) * 0.5f;
	const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
	const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
	const float r = p / q;
	const float a = pio2_hi - (x - (pio2_lo - x * r));
	const float s = gd_sqrt(z);
	union {
		float f;
		uint32_t u;
	} d{s};
	d.u &= 0xfffff000u;
	const float df = d.f;
	const float cc = (z - df * df) / (s + df);
	const float w = r * s + cc;
	const float h = 2.0f * (df + w);
	return ix <= 0x32800000 ? pio2_hi + pio2_lo : (lo ? a : h);
}
} // namespace glibc

// Which glibc build the reference host's sinf/cosf are (the plan's libm_variant,
// mbik_plan_options): LIBM_FMA (0) the FMA ifunc variant -- any x86-64 CPU with FMA, the
// default; LIBM_SSE2 (1) the SSE2 build -- a CPU without FMA, or GLIBC_TUNABLES=
// glibc.cpu.hwcaps=-FMA,-AVX2_Usable.  They differ on 12 (sinf) and 22 (cosf) of the 2^32
// inputs; acosf has one build.
constexpr int LIBM_FMA = 0, LIBM_SSE2 = 1;
GDI float sin_f(float x, int lv = LIBM_FMA) { return lv == LIBM_SSE2 ? glibc::sincosf<false>(x, 0) : glibc::sincosf<true>(x, 0); }
GDI float cos_f(float x, int lv = LIBM_FMA) { return lv == LIBM_SSE2 ? glibc::sincosf<false>(x, 1) : glibc::sincosf<true>(x, 1); }
GDI float acos_f(float x) { return glibc::acosf(x); }
// Quaternion::slerp's coefficient of the start quaternion at weight 0 (Godot 4.3
// quaternion.cpp, reached from Basis::slerp at ik_bone_segment_3d.cpp:148-151):
// scale0 = Math::sin((1.0 - p_weight) * omega) / sinom, the numerator a double ::sin, the
// denominator sinom = Math::sin(omega) a float sinf.  (scale1 = sinf(0 * omega) / sinom = +0.)
// The double sin is the device's own (OCML); mbik_selftest_libm proves this quotient equal
// to the host glibc's for every float omega.
//
// Device fast path: sin(omega) by its odd Taylor polynomial through x^21 for |omega| <= 1.6
// (the solve's omega, an acos of a non-negative cosine, lies in [0, pi/2]; truncation
// < 2^-58, evaluation < 2^-50 relative), the quotient through an fp64 reciprocal, and the
// float rounding of the ends of a 2^-46 (relative) interval around that estimate: the exact
// RN(RN(sin(w) / sinom)) lies inside it (the estimate is within ~2^-48), so when both ends
// round to the same float, that float is the result.  Otherwise -- essentially never -- the
// device's own double sin and division run.  mbik_selftest_libm's SLERP_SCALE0 class compares
// the result with the host glibc's for all 2^32 omega.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_EXACT_SLERP_SIN)
GDI double sin_taylor(double x) {
	const double x2 = x * x;
	double p = 0x1.71b8ef6dcf572p-66;        //  1/21!
	p = fma(p, x2, -0x1.2f49b46814157p-57);  // -1/19!
	p = fma(p, x2, 0x1.952c77030ad4ap-49);   //  1/17!
	p = fma(p, x2, -0x1.ae7f3e733b81fp-41);  // -1/15!
	p = fma(p, x2, 0x1.6124613a86d09p-33);   //  1/13!
	p = fma(p, x2, -0x1.ae64567f544e4p-26);  // -1/11!
	p = fma(p, x2, 0x1.71de3a556c734p-19);   //  1/9!
	p = fma(p, x2, -0x1.a01a01a01a01ap-13);  // -1/7!
	p = fma(p, x2, 0x1.1111111111111p-7);    //  1/5!
	p = fma(p, x2, -0x1.5555555555555p-3);   // -1/3!
	return fma(x * x2, p, x);
}
GDI float slerp_scale0(float omega, int lv = LIBM_FMA) {
	if (fabsf(omega) <= 1.6f) {
		const float sinom = lv == LIBM_SSE2 ? glibc::sinf_small<false>(omega) : glibc::sinf_small<true>(omega);
		const double q = sin_taylor((double)omega) * gd_rcp(sinom).r;
		const double w = fabs(q) * 0x1p-46;
		const float lo = (float)(q - w), hi = (float)(q + w);
		if (lo == hi) return lo; // (a NaN estimate, sinom == 0, falls through)
	}
	return (float)(sin((double)omega) / (double)sin_f(omega, lv));
}
#else
GDI float slerp_scale0(float omega, int lv = LIBM_FMA) {
	const float sinom = sin_f(omega, lv);
	return (float)(sin((double)omega) / (double)sinom);
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define GD_PACK 1
typedef float F2 __attribute__((ext_vector_type(2)));
#endif
struct V3 {
	float x, y, z;
	GDI float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
struct Q {
	float x, y, z, w;
};
struct B3 { // rows, like Godot's Basis
	V3 r[3];
};
struct X3 { // Transform3D
	B3 b;
	V3 o;
};

GDI V3 v3(float x, float y, float z) { return V3{x, y, z}; }
// Packed-pair arithmetic (device): the x and y lanes of a vector op go through one
// v_pk_{add,mul}_f32 (two IEEE float operations, each rounded exactly as the scalar one),
// z through a scalar op; sums keep the reference's left-to-right order.  One wave issues a
// packed op in about the time of a scalar one (tools/ubench.hip), so this is up to a third
// fewer VALU cycles for vector and basis arithmetic.
#ifdef GD_PACK
GDI F2 f2(float a, float b) { return F2{a, b}; }
GDI F2 xy(V3 a) { return F2{a.x, a.y}; }
GDI V3 v3(F2 p, float z) { return V3{p.x, p.y, z}; }
#endif
// (subtraction stays scalar: packing it made the compiler keep V3 temporaries on the stack)
GDI V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
#ifdef GD_PACK
GDI V3 operator+(V3 a, V3 b) { return v3(xy(a) + xy(b), a.z + b.z); }
GDI V3 operator*(V3 a, float s) { return v3(xy(a) * s, a.z * s); }
GDI V3 mulv(V3 a, V3 b) { return v3(xy(a) * xy(b), a.z * b.z); }
GDI float dot(V3 a, V3 b) {
	const F2 p = xy(a) * xy(b);
	return (p.x + p.y) + a.z * b.z;
}
GDI float length_sq(V3 a) {
	const F2 p = xy(a) * xy(a);
	return (p.x + p.y) + a.z * a.z;
}
#else
GDI V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
GDI V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
GDI V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
GDI float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GDI float length_sq(V3 a) {
	float x2 = a.x * a.x, y2 = a.y * a.y, z2 = a.z * a.z;
	return x2 + y2 + z2;
}
#endif
GDI V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
GDI V3 divs(V3 a, float s) {
	const GdRcp d = gd_rcp(s);
	return v3(gd_quot(a.x, d), gd_quot(a.y, d), gd_quot(a.z, d));
}
GDI V3 cross(V3 a, V3 b) { return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
GDI float length(V3 a) { return gd_sqrt(length_sq(a)); }
GDI V3 normalized(V3 a) {
	float l = length_sq(a);
	if (l == 0) return v3(0, 0, 0);
	// IEEE quotients by the rounded length (gd_sqrt_rcp / gd_quot: one reciprocal shared by
	// the three components)
	float len;
	const GdRcp d = gd_sqrt_rcp(l, len);
	return v3(gd_quot(a.x, d), gd_quot(a.y, d), gd_quot(a.z, d));
}
// The same with the zero-vector case selected instead of branched on (same operations, bit for
// bit).  The one-wave builds call it where it is faster there: straight-line code for the
// orthonormalizations.  The two-wave builds keep the branch, which costs them fewer registers.
GDI V3 normalized_sel(V3 a) {
	float l = length_sq(a);
	float len;
	const GdRcp d = gd_sqrt_rcp(l, len);
	const V3 n = v3(gd_quot(a.x, d), gd_quot(a.y, d), gd_quot(a.z, d));
	return l == 0 ? v3(0, 0, 0) : n;
}
template <bool SEL>
GDI V3 normalized_t(V3 a) {
	if constexpr (SEL) return normalized_sel(a);
	else return normalized(a);
}
GDI bool is_zero_approx(float s) { return fabsf(s) < (float)CMP_EPSILON; }
GDI bool is_equal_approx(float a, float b) {
	if (a == b) return true;
	float tol = (float)CMP_EPSILON * fabsf(a);
	if (tol < (float)CMP_EPSILON) tol = (float)CMP_EPSILON;
	return fabsf(a - b) < tol;
}
GDI bool is_zero_approx(V3 a) { return is_zero_approx(a.x) && is_zero_approx(a.y) && is_zero_approx(a.z); }
GDI bool is_finite(V3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }
GDI bool is_nan3(V3 a) { return isnan(a.x) || isnan(a.y) || isnan(a.z); }
GDI bool eq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
template <bool SEL = false>
GDI V3 any_perpendicular(V3 a) {
	V3 ax = (fabsf(a.x) <= fabsf(a.y) && fabsf(a.x) <= fabsf(a.z)) ? v3(1, 0, 0) : v3(0, 1, 0);
	return normalized_t<SEL>(cross(a, ax));
}

// ---------------- Quaternion ----------------
GDI Q q4(float x, float y, float z, float w) { return Q{x, y, z, w}; }
GDI Q qid() { return Q{0, 0, 0, 1}; }
#ifdef GD_PACK
GDI float dot(Q a, Q b) {
	const F2 p = f2(a.x, a.y) * f2(b.x, b.y), q = f2(a.z, a.w) * f2(b.z, b.w);
	return ((p.x + p.y) + q.x) + q.y;
}
GDI Q operator*(Q a, float s) {
	const F2 p = f2(a.x, a.y) * s, q = f2(a.z, a.w) * s;
	return q4(p.x, p.y, q.x, q.y);
}
#else
GDI float dot(Q a, Q b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
GDI Q operator*(Q a, float s) { return q4(a.x * s, a.y * s, a.z * s, a.w * s); }
#endif
GDI Q normalized(Q a) { // operator/ multiplies by 1/s
	float len;
	const GdRcp d = gd_sqrt_rcp(dot(a, a), len);
	return a * gd_quot(1.0f, d);
}
GDI Q inverse(Q a) { return q4(-a.x, -a.y, -a.z, a.w); }
GDI Q operator*(Q a, Q b) {
	float xx = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
	float yy = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
	float zz = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
	float ww = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
	return q4(xx, yy, zz, ww);
}
GDI V3 xform(Q q, V3 v) {
	V3 u = v3(q.x, q.y, q.z);
	V3 uv = cross(u, v);
	return v + ((uv * q.w) + cross(u, uv)) * 2.0f;
}
// Quaternion(axis, angle): s = sin(a/2) / |axis|
GDI Q axis_angle(V3 axis, float angle, int lv = LIBM_FMA) {
	float d = length(axis);
	if (d == 0) return q4(0, 0, 0, 0);
	float s = sin_f(angle * 0.5f, lv) / d;
	return q4(axis.x * s, axis.y * s, axis.z * s, cos_f(angle * 0.5f, lv));
}
// IKKusudama3D::get_quaternion_axis_angle (ik_kusudama_3d.cpp:417-427): divides by |axis|^2
GDI Q axis_angle_sq(V3 axis, float angle, int lv = LIBM_FMA) {
	float d = length_sq(axis);
	if (d == 0) return qid();
	float sin_angle = sin_f(angle * 0.5f, lv);
	float cos_angle = cos_f(angle * 0.5f, lv);
	float s = sin_angle / d;
	return q4(axis.x * s, axis.y * s, axis.z * s, cos_angle);
}
// The two constructors above with sin/cos of the half angle precomputed (for per-cone
// constant angles: the plan stores them, the solve never re-evaluates the trig).
GDI Q axis_angle_sc(V3 axis, float sin_half, float cos_half) {
	float d = length(axis);
	if (d == 0) return q4(0, 0, 0, 0);
	float s = sin_half / d;
	return q4(axis.x * s, axis.y * s, axis.z * s, cos_half);
}
GDI Q axis_angle_sq_sc(V3 axis, float sin_half, float cos_half) {
	float d = length_sq(axis);
	if (d == 0) return qid();
	float s = sin_half / d;
	return q4(axis.x * s, axis.y * s, axis.z * s, cos_half);
}
// Quaternion(v0, v1) shortest arc (Godot 4.3: normalising form)
template <bool SEL = false>
GDI Q arc(V3 v0, V3 v1) {
	const float ALMOST_ONE = 1.0f - (float)CMP_EPSILON;
	V3 n0 = normalized_t<SEL>(v0), n1 = normalized_t<SEL>(v1);
	float d = dot(n0, n1);
	if (fabsf(d) > ALMOST_ONE) {
		if (d >= 0) return qid();
		V3 a = any_perpendicular<SEL>(n0);
		return q4(a.x, a.y, a.z, 0);
	}
	V3 c = cross(n0, n1);
	float s = gd_sqrt((1.0f + d) * 2.0f);
	float rs = gd_pow2_over(1.0f, s);
	return q4(c.x * rs, c.y * rs, c.z * rs, s * 0.5f);
}
GDI V3 get_axis(Q q) {
	if (fabsf(q.w) > 1 - CMP_EPSILON) return v3(q.x, q.y, q.z);
	float r = gd_pow2_over(1.0f, gd_sqrt(1 - q.w * q.w));
	return v3(q.x * r, q.y * r, q.z * r);
}
GDI float get_angle(Q q) { return 2 * acos_f(q.w); }

// ---------------- Basis ----------------
GDI B3 bset(float xx, float xy, float xz, float yx, float yy, float yz, float zx, float zy, float zz) {
	B3 b;
	b.r[0] = v3(xx, xy, xz);
	b.r[1] = v3(yx, yy, yz);
	b.r[2] = v3(zx, zy, zz);
	return b;
}
GDI B3 bid() { return bset(1, 0, 0, 0, 1, 0, 0, 0, 1); }
GDI float at(const B3 &b, int i, int j) { return b.r[i][j]; }
GDI V3 col(const B3 &b, int i) { return v3(b.r[0][i], b.r[1][i], b.r[2][i]); }
GDI B3 from_cols(V3 x, V3 y, V3 z) { return bset(x.x, y.x, z.x, x.y, y.y, z.y, x.z, y.z, z.z); }
// Basis::set_quaternion
GDI B3 from_quat(Q q) {
	float d = dot(q, q);
	float s = gd_pow2_over(2.0f, d);
	float xs = q.x * s, ys = q.y * s, zs = q.z * s;
	float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
	float xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
	float yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
	return bset(1.0f - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0f - (xx + zz), yz - wx, xz - wy, yz + wx, 1.0f - (xx + yy));
}
// Basis::get_quaternion (the major-diagonal branch is spelled out per case so that no
// runtime-indexed array exists -- on the GPU that would live in scratch memory).
GDI Q get_quaternion(const B3 &m) {
	float r00 = m.r[0].x, r11 = m.r[1].y, r22 = m.r[2].z;
	float trace = r00 + r11 + r22;
	if (trace > 0.0f) {
		float s = gd_sqrt(trace + 1.0f);
		float w = s * 0.5f;
		s = gd_pow2_over(0.5f, s);
		return q4((m.r[2].y - m.r[1].z) * s, (m.r[0].z - m.r[2].x) * s, (m.r[1].x - m.r[0].y) * s, w);
	}
	int i = r00 < r11 ? (r11 < r22 ? 2 : 1) : (r00 < r22 ? 2 : 0);
	if (i == 0) { // j = 1, k = 2
		float s = gd_sqrt(r00 - r11 - r22 + 1.0f);
		float ti = s * 0.5f;
		s = gd_pow2_over(0.5f, s);
		return q4(ti, (m.r[1].x + m.r[0].y) * s, (m.r[2].x + m.r[0].z) * s, (m.r[2].y - m.r[1].z) * s);
	} else if (i == 1) { // j = 2, k = 0
		float s = gd_sqrt(r11 - r22 - r00 + 1.0f);
		float ti = s * 0.5f;
		s = gd_pow2_over(0.5f, s);
		return q4((m.r[0].y + m.r[1].x) * s, ti, (m.r[2].y + m.r[1].z) * s, (m.r[0].z - m.r[2].x) * s);
	} else { // i = 2: j = 0, k = 1
		float s = gd_sqrt(r22 - r00 - r11 + 1.0f);
		float ti = s * 0.5f;
		s = gd_pow2_over(0.5f, s);
		return q4((m.r[0].z + m.r[2].x) * s, (m.r[1].z + m.r[2].y) * s, ti, (m.r[1].x - m.r[0].y) * s);
	}
}
// Basis::orthonormalize (Gram-Schmidt on columns)
template <bool SEL = false>
GDI B3 orthonormalized(const B3 &b) {
	if constexpr (kAblate & ABL_ORTHO) return b; // timing experiment only
	V3 x = col(b, 0), y = col(b, 1), z = col(b, 2);
	x = normalized_t<SEL>(x);
	y = (y - x * dot(x, y));
	y = normalized_t<SEL>(y);
	z = (z - x * dot(x, z) - y * dot(y, z));
	z = normalized_t<SEL>(z);
	return from_cols(x, y, z);
}
GDI float determinant(const B3 &b) {
	const V3 *r = b.r;
	return r[0].x * (r[1].y * r[2].z - r[2].y * r[1].z) - r[1].x * (r[0].y * r[2].z - r[2].y * r[0].z) +
			r[2].x * (r[0].y * r[1].z - r[1].y * r[0].z);
}
template <bool SEL = false>
GDI Q get_rotation_quaternion(const B3 &b) {
	B3 m = orthonormalized<SEL>(b);
	if (determinant(m) < 0) {
		for (int i = 0; i < 3; i++) m.r[i] = m.r[i] * -1.0f;
	}
	return get_quaternion(m);
}
#define GD_COF(b, r1, c1, r2, c2) (at(b, r1, c1) * at(b, r2, c2) - at(b, r1, c2) * at(b, r2, c1))
GDI B3 inverse(const B3 &b) {
	float co0 = GD_COF(b, 1, 1, 2, 2), co1 = GD_COF(b, 1, 2, 2, 0), co2 = GD_COF(b, 1, 0, 2, 1);
	float det = b.r[0].x * co0 + b.r[0].y * co1 + b.r[0].z * co2;
	float s = gd_pow2_over(1.0f, det);
	return bset(co0 * s, GD_COF(b, 0, 2, 2, 1) * s, GD_COF(b, 0, 1, 1, 2) * s, co1 * s, GD_COF(b, 0, 0, 2, 2) * s,
			GD_COF(b, 0, 2, 1, 0) * s, co2 * s, GD_COF(b, 0, 1, 2, 0) * s, GD_COF(b, 0, 0, 1, 1) * s);
}
#undef GD_COF
// Basis::operator*: (A*B)[i][j] = B[0][j]*A[i][0] + B[1][j]*A[i][1] + B[2][j]*A[i][2]
GDI B3 operator*(const B3 &a, const B3 &b) {
	B3 r;
	if constexpr (kAblate & ABL_MATMUL) {
		for (int i = 0; i < 3; i++) r.r[i] = a.r[i] * b.r[i].x; // timing experiment only
		return r;
	}
#pragma unroll
	for (int i = 0; i < 3; i++) {
		V3 ar = a.r[i];
#ifdef GD_PACK
		r.r[i] = v3((xy(b.r[0]) * ar.x + xy(b.r[1]) * ar.y) + xy(b.r[2]) * ar.z, b.r[0].z * ar.x + b.r[1].z * ar.y + b.r[2].z * ar.z);
#else
		r.r[i] = v3(b.r[0].x * ar.x + b.r[1].x * ar.y + b.r[2].x * ar.z, b.r[0].y * ar.x + b.r[1].y * ar.y + b.r[2].y * ar.z,
				b.r[0].z * ar.x + b.r[1].z * ar.y + b.r[2].z * ar.z);
#endif
	}
	return r;
}
GDI V3 xform(const B3 &b, V3 v) { return v3(dot(b.r[0], v), dot(b.r[1], v), dot(b.r[2], v)); }
GDI bool is_finite(const B3 &b) { return is_finite(b.r[0]) && is_finite(b.r[1]) && is_finite(b.r[2]); }
GDI bool eq(const B3 &a, const B3 &b) { return eq(a.r[0], b.r[0]) && eq(a.r[1], b.r[1]) && eq(a.r[2], b.r[2]); }
GDI bool eq(const X3 &a, const X3 &b) { return eq(a.b, b.b) && eq(a.o, b.o); }
GDI V3 get_scale(const B3 &b) {
	float det = determinant(b);
	float sg = det == 0 ? 0.0f : (det < 0 ? -1.0f : 1.0f);
	return v3(length(col(b, 0)), length(col(b, 1)), length(col(b, 2))) * sg;
}
// Basis(axis, angle)
GDI B3 axis_angle_basis(V3 axis, float angle, int lv = LIBM_FMA) {
	B3 b;
	V3 sq = v3(axis.x * axis.x, axis.y * axis.y, axis.z * axis.z);
	float c = cos_f(angle, lv);
	b.r[0].x = sq.x + c * (1.0f - sq.x);
	b.r[1].y = sq.y + c * (1.0f - sq.y);
	b.r[2].z = sq.z + c * (1.0f - sq.z);
	float s = sin_f(angle, lv);
	float t = 1 - c;
	float xyzt = axis.x * axis.y * t, zyxs = axis.z * s;
	b.r[0].y = xyzt - zyxs;
	b.r[1].x = xyzt + zyxs;
	xyzt = axis.x * axis.z * t;
	zyxs = axis.y * s;
	b.r[0].z = xyzt + zyxs;
	b.r[2].x = xyzt - zyxs;
	xyzt = axis.y * axis.z * t;
	zyxs = axis.x * s;
	b.r[1].z = xyzt - zyxs;
	b.r[2].y = xyzt + zyxs;
	return b;
}

// ---------------- Transform3D ----------------
GDI X3 xid() { return X3{bid(), v3(0, 0, 0)}; }
GDI V3 xform(const X3 &t, V3 v) {
	return v3(dot(t.b.r[0], v) + t.o.x, dot(t.b.r[1], v) + t.o.y, dot(t.b.r[2], v) + t.o.z);
}
GDI X3 operator*(const X3 &a, const X3 &b) {
	X3 r;
	r.o = xform(a, b.o);
	r.b = a.b * b.b;
	return r;
}
GDI X3 affine_inverse(const X3 &t) {
	X3 r;
	r.b = inverse(t.b);
	r.o = xform(r.b, -t.o);
	return r;
}

// Skeleton3D bone pose: Basis(rotation) * diag(scale), origin = position.
GDI X3 pose_to_xform(const float *p) {
	B3 d = bset(p[7], 0, 0, 0, p[8], 0, 0, 0, p[9]);
	return X3{from_quat(q4(p[0], p[1], p[2], p[3])) * d, v3(p[4], p[5], p[6])};
}

} // namespace gd
