/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * Plain-C restatement of the Godot 4.3 core math that the reference module
 * (Ughuuu/many_bone_ik @ 2024-08-07) calls on its solve path.  Godot core is an
 * external, un-vendored dependency of the reference, so
 * its published semantics are restated here with real_t == float, in the same
 * operation order, so that the oracle reproduces the reference arithmetic:
 *   Vector3      core/math/vector3.h       (dot, cross, length, normalize, ...)
 *   Quaternion   core/math/quaternion.{h,cpp} (product, xform, arc ctor,
 *                axis-angle ctor, slerp, get_axis, get_angle, normalized)
 *   Basis        core/math/basis.{h,cpp}   (set_quaternion, get_quaternion,
 *                orthonormalize, get_rotation_quaternion, invert, operator*,
 *                xform, get_scale, set_axis_angle)
 *   Transform3D  core/math/transform_3d.{h,cpp} (operator*, xform, affine_inverse)
 * Assumed Godot version: 4.3 (the shortest-arc constructor normalises its inputs
 * and uses get_any_perpendicular for antiparallel vectors).
 *
 * Floating point: every float expression is evaluated in float, every mixed
 * float/double expression is promoted exactly as C++ would promote it.  Build
 * with -ffp-contract=off (see Makefile) so no FMA contraction happens.
 */
#ifndef MBIK_ORACLE_GODOT_MATH_H
#define MBIK_ORACLE_GODOT_MATH_H

#include <math.h>
#include <stdint.h>

#define GD_CMP_EPSILON 0.00001
#define GD_PI 3.1415926535897932384626433833
#define GD_TAU 6.2831853071795864769252867666

/* Float transcendentals.  Godot's Math::sin/cos/acos(float) call the platform libm
 * (::sinf/::cosf/::acosf, core/math/math_funcs.h); Math::sin(double) calls ::sin.  The
 * reference's dynamics amplify a 1-ulp difference ~2x per iteration, so the libm is part
 * of the reference's behaviour.  The oracle calls the platform libm, as a Linux x86-64
 * Godot build does: glibc 2.35 here and on the GPU boxes (same image).  glibc_libm.h
 * restates its sinf/cosf/acosf and tools/libm_exhaustive.c shows the two equal on all
 * 2^32 inputs (FMA ifunc variant; profiles/r02_libm_exhaustive.txt).  Two study builds:
 *   -DORACLE_GLIBC_RESTATED  the restatement instead of the platform libm (a host whose
 *                            libm is not glibc 2.35 still gets the reference's rounding);
 *   -DORACLE_PINNED_TRIG     round-1's convention, (float)f((double)x), for
 *                            tools/libm_sensitivity.py only. */
#if defined(ORACLE_PINNED_TRIG)
static inline float gd_sinf(float x) { return (float)sin((double)x); }
static inline float gd_cosf(float x) { return (float)cos((double)x); }
static inline float gd_acosf(float x) { return (float)acos((double)x); }
#elif defined(ORACLE_GLIBC_RESTATED)
#include "glibc_libm.h"
static inline float gd_sinf(float x) { return glibc_sinf(x); }
static inline float gd_cosf(float x) { return glibc_cosf(x); }
static inline float gd_acosf(float x) { return glibc_acosf(x); }
#else
static inline float gd_sinf(float x) { return sinf(x); }
static inline float gd_cosf(float x) { return cosf(x); }
static inline float gd_acosf(float x) { return acosf(x); }
#endif

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } quat;
typedef struct { v3 rows[3]; } basis;
typedef struct { basis b; v3 o; } xform;

static inline v3 v3_make(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline float v3_get(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline void v3_set(v3 *v, int i, float s) { if (i == 0) v->x = s; else if (i == 1) v->y = s; else v->z = s; }
static inline v3 v3_add(v3 a, v3 b) { return v3_make(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v3_sub(v3 a, v3 b) { return v3_make(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v3_scale(v3 a, float s) { return v3_make(a.x * s, a.y * s, a.z * s); }
static inline v3 v3_div(v3 a, float s) { return v3_make(a.x / s, a.y / s, a.z / s); }
static inline v3 v3_mulv(v3 a, v3 b) { return v3_make(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 v3_neg(v3 a) { return v3_make(-a.x, -a.y, -a.z); }
static inline float v3_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 v3_cross(v3 a, v3 b) {
	return v3_make((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
static inline float v3_length_squared(v3 a) {
	float x2 = a.x * a.x, y2 = a.y * a.y, z2 = a.z * a.z;
	return x2 + y2 + z2;
}
static inline float v3_length(v3 a) {
	float x2 = a.x * a.x, y2 = a.y * a.y, z2 = a.z * a.z;
	return sqrtf(x2 + y2 + z2);
}
/* Vector3::normalize(): zero stays zero, otherwise divide by the length. */
static inline v3 v3_normalized(v3 a) {
	float l = v3_length_squared(a);
	if (l == 0) return v3_make(0, 0, 0);
	float len = sqrtf(l);
	return v3_make(a.x / len, a.y / len, a.z / len);
}
static inline int gd_is_zero_approx(float s) { return fabsf(s) < (float)GD_CMP_EPSILON; }
static inline int gd_is_equal_approx(float a, float b) {
	if (a == b) return 1;
	float tol = (float)GD_CMP_EPSILON * fabsf(a);
	if (tol < (float)GD_CMP_EPSILON) tol = (float)GD_CMP_EPSILON;
	return fabsf(a - b) < tol;
}
static inline int v3_is_zero_approx(v3 a) { return gd_is_zero_approx(a.x) && gd_is_zero_approx(a.y) && gd_is_zero_approx(a.z); }
static inline int v3_is_equal_approx(v3 a, v3 b) { return gd_is_equal_approx(a.x, b.x) && gd_is_equal_approx(a.y, b.y) && gd_is_equal_approx(a.z, b.z); }
static inline int v3_is_finite(v3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }
static inline int v3_eq(v3 a, v3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static inline float v3_distance_to(v3 a, v3 b) { return v3_length(v3_sub(b, a)); }
/* Vector3::get_any_perpendicular (Godot 4.3). */
static inline v3 v3_any_perpendicular(v3 a) {
	v3 ax = (fabsf(a.x) <= fabsf(a.y) && fabsf(a.x) <= fabsf(a.z)) ? v3_make(1, 0, 0) : v3_make(0, 1, 0);
	return v3_normalized(v3_cross(a, ax));
}

/* ---------------- Quaternion ---------------- */
static inline quat q_make(float x, float y, float z, float w) { quat q = {x, y, z, w}; return q; }
static inline quat q_identity(void) { return q_make(0, 0, 0, 1); }
static inline float q_dot(quat a, quat b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
static inline float q_length_squared(quat a) { return q_dot(a, a); }
static inline float q_length(quat a) { return sqrtf(q_length_squared(a)); }
static inline quat q_scale(quat a, float s) { return q_make(a.x * s, a.y * s, a.z * s, a.w * s); }
/* operator/(real_t) multiplies by the reciprocal. */
static inline quat q_div(quat a, float s) { return q_scale(a, 1.0f / s); }
static inline quat q_normalized(quat a) { return q_div(a, q_length(a)); }
static inline quat q_inverse(quat a) { return q_make(-a.x, -a.y, -a.z, a.w); }
static inline quat q_mul(quat a, quat b) {
	float xx = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
	float yy = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
	float zz = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
	float ww = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
	return q_make(xx, yy, zz, ww);
}
static inline v3 q_xform(quat q, v3 v) {
	v3 u = v3_make(q.x, q.y, q.z);
	v3 uv = v3_cross(u, v);
	return v3_add(v, v3_scale(v3_add(v3_scale(uv, q.w), v3_cross(u, uv)), 2.0f));
}
static inline int q_is_finite(quat q) { return isfinite(q.x) && isfinite(q.y) && isfinite(q.z) && isfinite(q.w); }
/* Quaternion(const Vector3 &axis, real_t angle). */
static inline quat q_axis_angle(v3 axis, float angle) {
	float d = v3_length(axis);
	if (d == 0) return q_make(0, 0, 0, 0);
	float sin_angle = gd_sinf(angle * 0.5f);
	float cos_angle = gd_cosf(angle * 0.5f);
	float s = sin_angle / d;
	return q_make(axis.x * s, axis.y * s, axis.z * s, cos_angle);
}
/* Quaternion(const Vector3 &v0, const Vector3 &v1): shortest arc, Godot 4.3. */
static inline quat q_arc(v3 v0, v3 v1) {
	const float ALMOST_ONE = 1.0f - (float)GD_CMP_EPSILON;
	v3 n0 = v3_normalized(v0);
	v3 n1 = v3_normalized(v1);
	float d = v3_dot(n0, n1);
	if (fabsf(d) > ALMOST_ONE) {
		if (d >= 0) return q_identity();
		v3 ax = v3_any_perpendicular(n0);
		return q_make(ax.x, ax.y, ax.z, 0);
	}
	v3 c = v3_cross(n0, n1);
	float s = sqrtf((1.0f + d) * 2.0f);
	float rs = 1.0f / s;
	return q_make(c.x * rs, c.y * rs, c.z * rs, s * 0.5f);
}
static inline v3 q_get_axis(quat q) {
	if (fabsf(q.w) > 1 - GD_CMP_EPSILON) return v3_make(q.x, q.y, q.z);
	float r = ((float)1) / sqrtf(1 - q.w * q.w);
	return v3_make(q.x * r, q.y * r, q.z * r);
}
static inline float q_get_angle(quat q) { return 2 * gd_acosf(q.w); }
/* Quaternion::slerp (Godot 4.3); note the (1.0 - weight) * omega term is double. */
static inline quat q_slerp(quat from, quat to, float weight) {
	quat to1;
	float omega, cosom, sinom, scale0, scale1;
	cosom = q_dot(from, to);
	if (cosom < 0.0f) {
		cosom = -cosom;
		to1 = q_make(-to.x, -to.y, -to.z, -to.w);
	} else {
		to1 = to;
	}
	if ((1.0f - cosom) > (float)GD_CMP_EPSILON) {
		omega = gd_acosf(cosom);
		sinom = gd_sinf(omega);
		scale0 = (float)(sin((1.0 - weight) * omega) / sinom);
		scale1 = gd_sinf(weight * omega) / sinom;
	} else {
		scale0 = 1.0f - weight;
		scale1 = weight;
	}
	return q_make(scale0 * from.x + scale1 * to1.x, scale0 * from.y + scale1 * to1.y,
			scale0 * from.z + scale1 * to1.z, scale0 * from.w + scale1 * to1.w);
}

/* ---------------- Basis (row major, like Godot) ---------------- */
static inline basis b_identity(void) {
	basis b;
	b.rows[0] = v3_make(1, 0, 0);
	b.rows[1] = v3_make(0, 1, 0);
	b.rows[2] = v3_make(0, 0, 1);
	return b;
}
static inline basis b_set(float xx, float xy, float xz, float yx, float yy, float yz, float zx, float zy, float zz) {
	basis b;
	b.rows[0] = v3_make(xx, xy, xz);
	b.rows[1] = v3_make(yx, yy, yz);
	b.rows[2] = v3_make(zx, zy, zz);
	return b;
}
static inline float b_at(const basis *b, int r, int c) { return v3_get(b->rows[r], c); }
static inline v3 b_get_column(basis b, int i) {
	return v3_make(v3_get(b.rows[0], i), v3_get(b.rows[1], i), v3_get(b.rows[2], i));
}
static inline void b_set_column(basis *b, int i, v3 v) {
	v3_set(&b->rows[0], i, v.x);
	v3_set(&b->rows[1], i, v.y);
	v3_set(&b->rows[2], i, v.z);
}
/* Basis::set_quaternion (s = 2/|q|^2, tolerates non-unit input). */
static inline basis b_from_quat(quat q) {
	float d = q_length_squared(q);
	float s = 2.0f / d;
	float xs = q.x * s, ys = q.y * s, zs = q.z * s;
	float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
	float xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
	float yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
	return b_set(1.0f - (yy + zz), xy - wz, xz + wy,
			xy + wz, 1.0f - (xx + zz), yz - wx,
			xz - wy, yz + wx, 1.0f - (xx + yy));
}
/* Basis::get_quaternion (no MATH_CHECKS in release builds). */
static inline quat b_get_quaternion(basis m) {
	float r00 = m.rows[0].x, r11 = m.rows[1].y, r22 = m.rows[2].z;
	float trace = r00 + r11 + r22;
	float temp[4];
	if (trace > 0.0f) {
		float s = sqrtf(trace + 1.0f);
		temp[3] = (s * 0.5f);
		s = 0.5f / s;
		temp[0] = ((m.rows[2].y - m.rows[1].z) * s);
		temp[1] = ((m.rows[0].z - m.rows[2].x) * s);
		temp[2] = ((m.rows[1].x - m.rows[0].y) * s);
	} else {
		int i = r00 < r11 ? (r11 < r22 ? 2 : 1) : (r00 < r22 ? 2 : 0);
		int j = (i + 1) % 3;
		int k = (i + 2) % 3;
		float s = sqrtf(b_at(&m, i, i) - b_at(&m, j, j) - b_at(&m, k, k) + 1.0f);
		temp[i] = s * 0.5f;
		s = 0.5f / s;
		temp[3] = (b_at(&m, k, j) - b_at(&m, j, k)) * s;
		temp[j] = (b_at(&m, j, i) + b_at(&m, i, j)) * s;
		temp[k] = (b_at(&m, k, i) + b_at(&m, i, k)) * s;
	}
	return q_make(temp[0], temp[1], temp[2], temp[3]);
}
/* Basis::orthonormalize (Gram-Schmidt over columns x, y, z). */
static inline basis b_orthonormalized(basis b) {
	v3 x = b_get_column(b, 0);
	v3 y = b_get_column(b, 1);
	v3 z = b_get_column(b, 2);
	x = v3_normalized(x);
	y = v3_sub(y, v3_scale(x, v3_dot(x, y)));
	y = v3_normalized(y);
	z = v3_sub(v3_sub(z, v3_scale(x, v3_dot(x, z))), v3_scale(y, v3_dot(y, z)));
	z = v3_normalized(z);
	b_set_column(&b, 0, x);
	b_set_column(&b, 1, y);
	b_set_column(&b, 2, z);
	return b;
}
static inline float b_determinant(basis b) {
	const v3 *r = b.rows;
	return r[0].x * (r[1].y * r[2].z - r[2].y * r[1].z) -
			r[1].x * (r[0].y * r[2].z - r[2].y * r[0].z) +
			r[2].x * (r[0].y * r[1].z - r[1].y * r[0].z);
}
/* Basis::scale(Vector3): scales rows. */
static inline basis b_scale_rows(basis b, v3 s) {
	b.rows[0] = v3_scale(b.rows[0], s.x);
	b.rows[1] = v3_scale(b.rows[1], s.y);
	b.rows[2] = v3_scale(b.rows[2], s.z);
	return b;
}
static inline quat b_get_rotation_quaternion(basis b) {
	basis m = b_orthonormalized(b);
	float det = b_determinant(m);
	if (det < 0) m = b_scale_rows(m, v3_make(-1, -1, -1));
	return b_get_quaternion(m);
}
#define GD_COFAC(b, r1, c1, r2, c2) (b_at(&(b), r1, c1) * b_at(&(b), r2, c2) - b_at(&(b), r1, c2) * b_at(&(b), r2, c1))
/* Basis::inverse (cofactor form). */
static inline basis b_inverse(basis b) {
	float co0 = GD_COFAC(b, 1, 1, 2, 2), co1 = GD_COFAC(b, 1, 2, 2, 0), co2 = GD_COFAC(b, 1, 0, 2, 1);
	float det = b.rows[0].x * co0 + b.rows[0].y * co1 + b.rows[0].z * co2;
	float s = 1.0f / det;
	return b_set(co0 * s, GD_COFAC(b, 0, 2, 2, 1) * s, GD_COFAC(b, 0, 1, 1, 2) * s,
			co1 * s, GD_COFAC(b, 0, 0, 2, 2) * s, GD_COFAC(b, 0, 2, 1, 0) * s,
			co2 * s, GD_COFAC(b, 0, 1, 2, 0) * s, GD_COFAC(b, 0, 0, 1, 1) * s);
}
/* Basis::operator* : (A*B)[i][j] = B[0][j]*A[i][0] + B[1][j]*A[i][1] + B[2][j]*A[i][2]. */
static inline basis b_mul(basis a, basis b) {
	basis r;
	for (int i = 0; i < 3; i++) {
		v3 ar = a.rows[i];
		r.rows[i].x = b.rows[0].x * ar.x + b.rows[1].x * ar.y + b.rows[2].x * ar.z;
		r.rows[i].y = b.rows[0].y * ar.x + b.rows[1].y * ar.y + b.rows[2].y * ar.z;
		r.rows[i].z = b.rows[0].z * ar.x + b.rows[1].z * ar.y + b.rows[2].z * ar.z;
	}
	return r;
}
static inline v3 b_xform(basis b, v3 v) { return v3_make(v3_dot(b.rows[0], v), v3_dot(b.rows[1], v), v3_dot(b.rows[2], v)); }
static inline int b_is_finite(basis b) { return v3_is_finite(b.rows[0]) && v3_is_finite(b.rows[1]) && v3_is_finite(b.rows[2]); }
static inline int b_eq(basis a, basis b) { return v3_eq(a.rows[0], b.rows[0]) && v3_eq(a.rows[1], b.rows[1]) && v3_eq(a.rows[2], b.rows[2]); }
/* Basis::get_scale: SIGN(det) * column lengths. */
static inline v3 b_get_scale(basis b) {
	float det = b_determinant(b);
	float sg = det > 0 ? 1.0f : (det < 0 ? -1.0f : 0.0f);
	v3 s = v3_make(v3_length(b_get_column(b, 0)), v3_length(b_get_column(b, 1)), v3_length(b_get_column(b, 2)));
	return v3_scale(s, sg);
}
/* Basis(axis, angle) == set_axis_angle. */
static inline basis b_axis_angle(v3 axis, float angle) {
	basis b;
	v3 sq = v3_make(axis.x * axis.x, axis.y * axis.y, axis.z * axis.z);
	float cosine = gd_cosf(angle);
	b.rows[0].x = sq.x + cosine * (1.0f - sq.x);
	b.rows[1].y = sq.y + cosine * (1.0f - sq.y);
	b.rows[2].z = sq.z + cosine * (1.0f - sq.z);
	float sine = gd_sinf(angle);
	float t = 1 - cosine;
	float xyzt = axis.x * axis.y * t;
	float zyxs = axis.z * sine;
	b.rows[0].y = xyzt - zyxs;
	b.rows[1].x = xyzt + zyxs;
	xyzt = axis.x * axis.z * t;
	zyxs = axis.y * sine;
	b.rows[0].z = xyzt + zyxs;
	b.rows[2].x = xyzt - zyxs;
	xyzt = axis.y * axis.z * t;
	zyxs = axis.x * sine;
	b.rows[1].z = xyzt - zyxs;
	b.rows[2].y = xyzt + zyxs;
	return b;
}
/* Basis::slerp (Godot 4.3): quaternion slerp, rows rescaled by lerped row lengths. */
static inline basis b_slerp(basis from_b, basis to_b, float weight) {
	quat from = b_get_quaternion(from_b);
	quat to = b_get_quaternion(to_b);
	basis b = b_from_quat(q_slerp(from, to, weight));
	for (int i = 0; i < 3; i++) {
		float la = v3_length(from_b.rows[i]);
		float lb = v3_length(to_b.rows[i]);
		b.rows[i] = v3_scale(b.rows[i], la + (lb - la) * weight);
	}
	return b;
}

/* ---------------- Transform3D ---------------- */
static inline xform x_identity(void) { xform t; t.b = b_identity(); t.o = v3_make(0, 0, 0); return t; }
static inline xform x_make(basis b, v3 o) { xform t; t.b = b; t.o = o; return t; }
static inline v3 x_xform(xform t, v3 v) {
	return v3_make(v3_dot(t.b.rows[0], v) + t.o.x, v3_dot(t.b.rows[1], v) + t.o.y, v3_dot(t.b.rows[2], v) + t.o.z);
}
/* Transform3D::operator*: origin = xform(p.origin); basis *= p.basis. */
static inline xform x_mul(xform a, xform b) {
	xform r;
	r.o = x_xform(a, b.o);
	r.b = b_mul(a.b, b.b);
	return r;
}
static inline xform x_affine_inverse(xform t) {
	xform r;
	r.b = b_inverse(t.b);
	r.o = b_xform(r.b, v3_neg(t.o));
	return r;
}
static inline int x_eq(xform a, xform b) { return b_eq(a.b, b.b) && v3_eq(a.o, b.o); }

#endif
