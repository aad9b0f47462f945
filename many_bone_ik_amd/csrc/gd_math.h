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

constexpr double CMP_EPSILON = 0.00001;
constexpr double PI = 3.1415926535897932384626433833;

// Float transcendentals, rounded once from a double evaluation.  The reference calls the
// platform libm (Math::sin(float) -> sinf); its dynamics amplify 1-ulp libm differences
// ~2x per iteration, so the product and the oracle pin the same (correctly rounded,
// barring rare double-rounding cases) result instead of OCML's own float versions.
#ifdef MBIK_ABLATE_TRIG
GDI float sin_f(float x) { return sinf(x); }
GDI float cos_f(float x) { return cosf(x); }
GDI float acos_f(float x) { return acosf(x); }
#else
GDI float sin_f(float x) { return (float)sin((double)x); }
GDI float cos_f(float x) { return (float)cos((double)x); }
GDI float acos_f(float x) { return (float)acos((double)x); }
#endif

// Square root, correctly rounded (IEEE), as Godot's Math::sqrt(float) on x86.
// On the device: v_rsq_f64 of the widened input and one fp64 Newton correction, rounded
// once to float.  tools/sqrt_exhaustive.hip checks all 2^32 inputs against the compiler's
// correctly rounded sqrtf: identical for every non-NaN result (NaN payloads may differ;
// NaN-ness does not).  Half the latency of the fp32 sequence (55 vs 107 cycles, same tool).
#if defined(MBIK_ABLATE_SQRT) && defined(__HIP_DEVICE_COMPILE__)
GDI float gd_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); } // timing experiment only (1 ulp)
#elif defined(__HIP_DEVICE_COMPILE__) && !defined(MBIK_IEEE_SQRT)
GDI float gd_sqrt(float x) {
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
GDI V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
GDI V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
GDI V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
GDI V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
GDI V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
GDI V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
GDI float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GDI V3 cross(V3 a, V3 b) { return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
GDI float length_sq(V3 a) {
	float x2 = a.x * a.x, y2 = a.y * a.y, z2 = a.z * a.z;
	return x2 + y2 + z2;
}
GDI float length(V3 a) { return gd_sqrt(length_sq(a)); }
GDI V3 normalized(V3 a) {
	float l = length_sq(a);
	if (l == 0) return v3(0, 0, 0);
	float len = gd_sqrt(l);
#ifdef MBIK_ABLATE_NORMDIV
	float r = 1.0f / len; // timing experiment only
	return v3(a.x * r, a.y * r, a.z * r);
#else
	// IEEE quotients.  A shared fp64 reciprocal ((float)((double)a * r), exact except for
	// denormal quotients -- tools/div_check.hip) measured slower in the kernel once the
	// denormal/range guard branch is paid (C2 1.596 vs 1.525 ms).
	return v3(a.x / len, a.y / len, a.z / len);
#endif
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
GDI V3 any_perpendicular(V3 a) {
	V3 ax = (fabsf(a.x) <= fabsf(a.y) && fabsf(a.x) <= fabsf(a.z)) ? v3(1, 0, 0) : v3(0, 1, 0);
	return normalized(cross(a, ax));
}

// ---------------- Quaternion ----------------
GDI Q q4(float x, float y, float z, float w) { return Q{x, y, z, w}; }
GDI Q qid() { return Q{0, 0, 0, 1}; }
GDI float dot(Q a, Q b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
GDI Q operator*(Q a, float s) { return q4(a.x * s, a.y * s, a.z * s, a.w * s); }
GDI Q normalized(Q a) { return a * (1.0f / gd_sqrt(dot(a, a))); } // operator/ multiplies by 1/s
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
GDI Q axis_angle(V3 axis, float angle) {
	float d = length(axis);
	if (d == 0) return q4(0, 0, 0, 0);
	float s = sin_f(angle * 0.5f) / d;
	return q4(axis.x * s, axis.y * s, axis.z * s, cos_f(angle * 0.5f));
}
// IKKusudama3D::get_quaternion_axis_angle (ik_kusudama_3d.cpp:417-427): divides by |axis|^2
GDI Q axis_angle_sq(V3 axis, float angle) {
	float d = length_sq(axis);
	if (d == 0) return qid();
	float sin_angle = sin_f(angle * 0.5f);
	float cos_angle = cos_f(angle * 0.5f);
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
GDI Q arc(V3 v0, V3 v1) {
	const float ALMOST_ONE = 1.0f - (float)CMP_EPSILON;
	V3 n0 = normalized(v0), n1 = normalized(v1);
	float d = dot(n0, n1);
	if (fabsf(d) > ALMOST_ONE) {
		if (d >= 0) return qid();
		V3 a = any_perpendicular(n0);
		return q4(a.x, a.y, a.z, 0);
	}
	V3 c = cross(n0, n1);
	float s = gd_sqrt((1.0f + d) * 2.0f);
	float rs = 1.0f / s;
	return q4(c.x * rs, c.y * rs, c.z * rs, s * 0.5f);
}
GDI V3 get_axis(Q q) {
	if (fabsf(q.w) > 1 - CMP_EPSILON) return v3(q.x, q.y, q.z);
	float r = 1.0f / gd_sqrt(1 - q.w * q.w);
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
	float s = 2.0f / d;
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
		s = 0.5f / s;
		return q4((m.r[2].y - m.r[1].z) * s, (m.r[0].z - m.r[2].x) * s, (m.r[1].x - m.r[0].y) * s, w);
	}
	int i = r00 < r11 ? (r11 < r22 ? 2 : 1) : (r00 < r22 ? 2 : 0);
	if (i == 0) { // j = 1, k = 2
		float s = gd_sqrt(r00 - r11 - r22 + 1.0f);
		float ti = s * 0.5f;
		s = 0.5f / s;
		return q4(ti, (m.r[1].x + m.r[0].y) * s, (m.r[2].x + m.r[0].z) * s, (m.r[2].y - m.r[1].z) * s);
	} else if (i == 1) { // j = 2, k = 0
		float s = gd_sqrt(r11 - r22 - r00 + 1.0f);
		float ti = s * 0.5f;
		s = 0.5f / s;
		return q4((m.r[0].y + m.r[1].x) * s, ti, (m.r[2].y + m.r[1].z) * s, (m.r[0].z - m.r[2].x) * s);
	} else { // i = 2: j = 0, k = 1
		float s = gd_sqrt(r22 - r00 - r11 + 1.0f);
		float ti = s * 0.5f;
		s = 0.5f / s;
		return q4((m.r[0].z + m.r[2].x) * s, (m.r[1].z + m.r[2].y) * s, ti, (m.r[1].x - m.r[0].y) * s);
	}
}
// Basis::orthonormalize (Gram-Schmidt on columns)
GDI B3 orthonormalized(const B3 &b) {
#ifdef MBIK_ABLATE_ORTHO
	return b; // timing experiment only
#endif
	V3 x = col(b, 0), y = col(b, 1), z = col(b, 2);
	x = normalized(x);
	y = (y - x * dot(x, y));
	y = normalized(y);
	z = (z - x * dot(x, z) - y * dot(y, z));
	z = normalized(z);
	return from_cols(x, y, z);
}
GDI float determinant(const B3 &b) {
	const V3 *r = b.r;
	return r[0].x * (r[1].y * r[2].z - r[2].y * r[1].z) - r[1].x * (r[0].y * r[2].z - r[2].y * r[0].z) +
			r[2].x * (r[0].y * r[1].z - r[1].y * r[0].z);
}
GDI Q get_rotation_quaternion(const B3 &b) {
	B3 m = orthonormalized(b);
	if (determinant(m) < 0) {
		for (int i = 0; i < 3; i++) m.r[i] = m.r[i] * -1.0f;
	}
	return get_quaternion(m);
}
#define GD_COF(b, r1, c1, r2, c2) (at(b, r1, c1) * at(b, r2, c2) - at(b, r1, c2) * at(b, r2, c1))
GDI B3 inverse(const B3 &b) {
	float co0 = GD_COF(b, 1, 1, 2, 2), co1 = GD_COF(b, 1, 2, 2, 0), co2 = GD_COF(b, 1, 0, 2, 1);
	float det = b.r[0].x * co0 + b.r[0].y * co1 + b.r[0].z * co2;
	float s = 1.0f / det;
	return bset(co0 * s, GD_COF(b, 0, 2, 2, 1) * s, GD_COF(b, 0, 1, 1, 2) * s, co1 * s, GD_COF(b, 0, 0, 2, 2) * s,
			GD_COF(b, 0, 2, 1, 0) * s, co2 * s, GD_COF(b, 0, 1, 2, 0) * s, GD_COF(b, 0, 0, 1, 1) * s);
}
#undef GD_COF
// Basis::operator*: (A*B)[i][j] = B[0][j]*A[i][0] + B[1][j]*A[i][1] + B[2][j]*A[i][2]
GDI B3 operator*(const B3 &a, const B3 &b) {
	B3 r;
#ifdef MBIK_ABLATE_MATMUL
	for (int i = 0; i < 3; i++) r.r[i] = a.r[i] * b.r[i].x; // timing experiment only
	return r;
#endif
#pragma unroll
	for (int i = 0; i < 3; i++) {
		V3 ar = a.r[i];
		r.r[i] = v3(b.r[0].x * ar.x + b.r[1].x * ar.y + b.r[2].x * ar.z, b.r[0].y * ar.x + b.r[1].y * ar.y + b.r[2].y * ar.z,
				b.r[0].z * ar.x + b.r[1].z * ar.y + b.r[2].z * ar.z);
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
GDI B3 axis_angle_basis(V3 axis, float angle) {
	B3 b;
	V3 sq = v3(axis.x * axis.x, axis.y * axis.y, axis.z * axis.z);
	float c = cos_f(angle);
	b.r[0].x = sq.x + c * (1.0f - sq.x);
	b.r[1].y = sq.y + c * (1.0f - sq.y);
	b.r[2].z = sq.z + c * (1.0f - sq.z);
	float s = sin_f(angle);
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
