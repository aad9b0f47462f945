/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * Plain-C restatement of the platform libm's float sinf / cosf / acosf, the functions
 * Godot's Math::sin/cos/acos(float) call on a Linux x86-64 build (core/math/math_funcs.h
 * forwards to ::sinf, ::cosf, ::acosf).  The reference calls them on its solve path:
 *   Basis::slerp -> Quaternion::slerp (acos, sin)   ik_bone_segment_3d.cpp:148-151
 *   Quaternion(axis, angle) (sin, cos)              ik_open_cone_3d.cpp:297,312
 *   get_quaternion_axis_angle (sin, cos)            ik_kusudama_3d.cpp:417-427
 *   set_axial_limits (cos)                          ik_kusudama_3d.cpp:112
 *
 * Third-party dependency: GNU C Library 2.35 (Ubuntu 2.35-0ubuntu3.x, the image's libm).
 * Its published algorithms, restated here:
 *   sinf/cosf  sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c
 *              (Szabolcs Nagy's double-precision polynomial, glibc >= 2.28).  On x86-64
 *              the multiarch ifunc picks a build of that C file compiled with -mfma -mavx2
 *              when the CPU has FMA (s_sinf-fma.c); GCC then contracts a*b+c into fused
 *              multiply-adds.  GLIBC_SINCOSF_FMA selects that contraction (1, the default:
 *              every x86-64 CPU of this pool has FMA) or the SSE2 build (0).
 *   acosf      sysdeps/ieee754/flt-32/e_acosf.c (fdlibm, single precision; no x86-64
 *              multiarch variant).
 * tools/libm_exhaustive.c checks this file against the platform libm on all 2^32 inputs
 * (profiles/r02_libm_exhaustive.txt).  Build with -ffp-contract=off: every contraction
 * here is written out as fma().
 *
 * Third-party notices (THIRD_PARTY_NOTICES.md): sinf/cosf tables and algorithms from the
 * GNU C Library, Copyright (C) 2018-2022 Free Software Foundation, Inc., LGPL-2.1-or-later.
 * acosf from fdlibm: Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 * Developed at SunPro, a Sun Microsystems, Inc. business. Permission to use, copy, modify,
 * and distribute this software is freely granted, provided that this notice is preserved.
 * (Float conversion by Ian Lance Taylor, Cygnus Support.)
 */
#ifndef MBIK_ORACLE_GLIBC_LIBM_H
#define MBIK_ORACLE_GLIBC_LIBM_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef GLIBC_SINCOSF_FMA
#define GLIBC_SINCOSF_FMA 1
#endif

#if GLIBC_SINCOSF_FMA
#define GL_MADD(a, b, c) fma((a), (b), (c)) /* a*b + c, one rounding */
#else
#define GL_MADD(a, b, c) ((a) * (b) + (c))
#endif

static inline uint32_t gl_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float gl_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* top 12 bits of |x| (sign cleared) */
static inline uint32_t gl_abstop12(float x) { return (gl_asuint(x) >> 20) & 0x7ff; }

/* sincosf.h: the two polynomial sets (sin/cos of the reduced argument, with the sign
 * pattern of quadrants 0/1 and 2/3). */
typedef struct {
	double sign[4];
	double hpi_inv, hpi;
	double c0, c1, c2, c3, c4;
	double s1, s2, s3;
} gl_sincos_t;

static const gl_sincos_t gl_sincosf_table[2] = {
	{{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
	 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
	 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
	{{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
	 -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
	 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
};

/* 2/pi in sliding 32-bit windows (sincosf_data.c __inv_pio4) */
static const uint32_t gl_inv_pio4[24] = {
	0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
	0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
	0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041,
};

/* sincosf.h sinf_poly: n even -> sin polynomial, n odd -> cos polynomial */
static inline float gl_sinf_poly(double x, double x2, const gl_sincos_t *p, int n) {
	if ((n & 1) == 0) {
		double x3 = x * x2;
		double s1 = GL_MADD(x2, p->s3, p->s2);
		double x7 = x3 * x2;
		double s = GL_MADD(x3, p->s1, x);
		return (float)GL_MADD(x7, s1, s);
	} else {
		double x4 = x2 * x2;
		double c2 = GL_MADD(x2, p->c4, p->c3);
		double c1 = GL_MADD(x2, p->c1, p->c0);
		double x6 = x4 * x2;
		double c = GL_MADD(x4, p->c2, c1);
		return (float)GL_MADD(x6, c2, c);
	}
}

/* sincosf.h reduce_fast (TOINT_INTRINSICS == 0 on x86-64): |x| < 120 */
static inline double gl_reduce_fast(double x, const gl_sincos_t *p, int *np) {
	double r = x * p->hpi_inv;
	int n = ((int32_t)r + 0x800000) >> 24;
	*np = n;
#if GLIBC_SINCOSF_FMA
	return fma(-(double)n, p->hpi, x);
#else
	return x - n * p->hpi;
#endif
}

/* sincosf.h reduce_large: Payne-Hanek with 2/pi bits, 64-bit integer arithmetic */
static inline double gl_reduce_large(uint32_t xi, int *np) {
	const uint32_t *arr = &gl_inv_pio4[(xi >> 26) & 15];
	int shift = (xi >> 23) & 7;
	uint64_t n, res0, res1, res2;
	xi = (xi & 0xffffff) | 0x800000;
	xi <<= shift;
	res0 = xi * arr[0]; /* 32-bit product, as the C source */
	res1 = (uint64_t)xi * arr[4];
	res2 = (uint64_t)xi * arr[8];
	res0 = (res2 >> 32) | (res0 << 32);
	res0 += res1;
	n = (res0 + (1ULL << 61)) >> 62;
	res0 -= n << 62;
	double x = (double)(int64_t)res0;
	*np = (int)n;
	return x * 0x1.921FB54442D18p-62;
}

/* s_sinf.c */
static inline float glibc_sinf(float y) {
	double x = y, s;
	int n;
	const gl_sincos_t *p = &gl_sincosf_table[0];
	if (gl_abstop12(y) < gl_abstop12(0x1.921FB6p-1f)) {
		s = x * x;
		if (gl_abstop12(y) < gl_abstop12(0x1p-12f)) return y;
		return gl_sinf_poly(x, s, p, 0);
	} else if (gl_abstop12(y) < gl_abstop12(120.0f)) {
		x = gl_reduce_fast(x, p, &n);
		s = p->sign[n & 3];
		if (n & 2) p = &gl_sincosf_table[1];
		return gl_sinf_poly(x * s, x * x, p, n);
	} else if (gl_abstop12(y) < gl_abstop12(INFINITY)) {
		uint32_t xi = gl_asuint(y);
		int sign = xi >> 31;
		x = gl_reduce_large(xi, &n);
		s = p->sign[(n + sign) & 3];
		if ((n + sign) & 2) p = &gl_sincosf_table[1];
		return gl_sinf_poly(x * s, x * x, p, n);
	}
	return (y - y) / (y - y); /* __math_invalidf: NaN */
}

/* s_cosf.c */
static inline float glibc_cosf(float y) {
	double x = y, s;
	int n;
	const gl_sincos_t *p = &gl_sincosf_table[0];
	if (gl_abstop12(y) < gl_abstop12(0x1.921FB6p-1f)) {
		double x2 = x * x;
		if (gl_abstop12(y) < gl_abstop12(0x1p-12f)) return 1.0f;
		return gl_sinf_poly(x, x2, p, 1);
	} else if (gl_abstop12(y) < gl_abstop12(120.0f)) {
		x = gl_reduce_fast(x, p, &n);
		s = p->sign[n & 3];
		if (n & 2) p = &gl_sincosf_table[1];
		return gl_sinf_poly(x * s, x * x, p, n ^ 1);
	} else if (gl_abstop12(y) < gl_abstop12(INFINITY)) {
		uint32_t xi = gl_asuint(y);
		int sign = xi >> 31;
		x = gl_reduce_large(xi, &n);
		s = p->sign[(n + sign) & 3];
		if ((n + sign) & 2) p = &gl_sincosf_table[1];
		return gl_sinf_poly(x * s, x * x, p, n ^ 1);
	}
	return (y - y) / (y - y);
}

/* e_acosf.c (fdlibm): float arithmetic throughout, IEEE sqrtf */
static inline float glibc_acosf(float x) {
	static const float one = 1.0000000000e+00f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f,
	                   pio2_lo = 7.5497894159e-08f, pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f,
	                   pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f,
	                   pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
	                   qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
	float z, p, q, r, w, s, c, df;
	int32_t hx = (int32_t)gl_asuint(x), ix = hx & 0x7fffffff;
	if (ix == 0x3f800000) {
		if (hx > 0) return 0.0f;
		return pi + 2.0f * pio2_lo;
	} else if (ix > 0x3f800000) {
		return (x - x) / (x - x);
	}
	if (ix < 0x3f000000) { /* |x| < 0.5 */
		if (ix <= 0x32800000) return pio2_hi + pio2_lo;
		z = x * x;
		p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		r = p / q;
		return pio2_hi - (x - (pio2_lo - x * r));
	} else if (hx < 0) { /* x < -0.5 */
		z = (one + x) * 0.5f;
		p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		s = sqrtf(z);
		r = p / q;
		w = r * s - pio2_lo;
		return pi - 2.0f * (s + w);
	} else { /* x > 0.5 */
		z = (one - x) * 0.5f;
		s = sqrtf(z);
		df = gl_asfloat(gl_asuint(s) & 0xfffff000u);
		c = (z - df * df) / (s + df);
		p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
		q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
		r = p / q;
		w = r * s + c;
		return 2.0f * (df + w);
	}
}

#endif
