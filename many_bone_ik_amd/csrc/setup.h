// Per-skeleton plan setup, shared by the host builder (plan.cpp) and the GPU builder
// (k_aux.hip: mbik_setup_kernel): the bone-direction frames and the Kusudama frames that
// ManyBoneIK3D::_bone_list_changed derives from a skeleton's setup pose, cones and twist
// (IKBone3D::update_default_bone_direction_transform ik_bone_3d.cpp:57-93,
//  IKLimitCone3D::update_tangent_handles ik_open_cone_3d.cpp:36-120, IKRay3D
//  ik_ray_3d.cpp:64-166, IKKusudama3D::set_axial_limits / _update_constraint
//  ik_kusudama_3d.cpp:37-115).  One code path for both sides, so a GPU rebuild produces the
// host's tables (same operations, -ffp-contract=off; transcendentals evaluated in double).
#pragma once

#include <cstddef>
#include <cstdint>

#include "gd_math.h"
#include "plan.h"

namespace mbik {

using namespace gd;

struct Cone {
	V3 cp;
	double radius, rcos;
	V3 t1, t2;
	double tr, trcos;
};

// Read-only topology the setup needs (host or device pointers).
struct SetupView {
	int B, NC, N, max_cones_in, desc_constraint_count, cfs, cds;
	int n_topo, n_list, n_cons_order;
	const int *topo;           // bones, parents before children
	const int *bone_list;      // ManyBoneIK3D::bone_list order
	const int *bone_flags, *bone_pose_parent, *bone_ik_parent;
	const int *ik_child_off, *ik_children; // IK children of each bone, ascending
	const int *cons_order, *cons_order_slot, *cons_order_ncones, *cons_bone;
	int libm = LIBM_FMA; // the reference host's glibc sinf/cosf build (HostPlan::libm_variant)
};

// Scratch one skeleton's setup needs (callers size it with setup_scratch_bytes).
struct SetupScratch {
	X3 *L, *G;
	B3 *Dm, *T;
	Cone *kc, *cs; // kc: [NC][max_cones_in] final cones per slot, cs: [max_cones_in] working set
	int *kcn;      // cones per slot
	Q *tcr;
	float *thc;
};
GDI size_t setup_scratch_bytes(int B, int NC, int max_cones) {
	return (size_t)B * (2 * sizeof(X3) + sizeof(B3)) + (size_t)NC * (sizeof(B3) + sizeof(int) + sizeof(Q) + sizeof(float)) +
			(size_t)(NC + 1) * max_cones * sizeof(Cone) + 64;
}
GDI SetupScratch setup_scratch_at(void *base, int B, int NC, int max_cones) {
	char *p = static_cast<char *>(base);
	SetupScratch s;
	auto take = [&](size_t bytes) {
		char *r = p;
		p += (bytes + 15) & ~size_t(15);
		return r;
	};
	s.L = reinterpret_cast<X3 *>(take(sizeof(X3) * B));
	s.G = reinterpret_cast<X3 *>(take(sizeof(X3) * B));
	s.Dm = reinterpret_cast<B3 *>(take(sizeof(B3) * B));
	s.T = reinterpret_cast<B3 *>(take(sizeof(B3) * (NC ? NC : 1)));
	s.kc = reinterpret_cast<Cone *>(take(sizeof(Cone) * (size_t)(NC ? NC : 1) * max_cones));
	s.cs = reinterpret_cast<Cone *>(take(sizeof(Cone) * max_cones));
	s.kcn = reinterpret_cast<int *>(take(sizeof(int) * (NC ? NC : 1)));
	s.tcr = reinterpret_cast<Q *>(take(sizeof(Q) * (NC ? NC : 1)));
	s.thc = reinterpret_cast<float *>(take(sizeof(float) * (NC ? NC : 1)));
	return s;
}

// ---- IKRay3D / IKLimitCone3D setup geometry ----
struct Ray {
	V3 p1, p2;
};
GDI void elongate(Ray &r, float amt) {
	V3 mid = (r.p1 + r.p2) * 0.5f;
	V3 h1 = r.p1 - mid, h2 = r.p2 - mid;
	V3 a1 = normalized(h1) * amt, a2 = normalized(h2) * amt;
	r.p1 = h1 + a1 + mid;
	r.p2 = h2 + a2 + mid;
}
GDI V3 intersects_plane(const Ray &r, V3 ta, V3 tb, V3 tc) {
	V3 tta = ta - r.p1, ttb = tb - r.p1, ttc = tc - r.p1;
	V3 u = ttb - tta, v = ttc - tta;
	V3 dir = r.p2 - r.p1;
	V3 n = normalized(cross(u, v));
	V3 w0 = v3(0, 0, 0) - tta;
	float a = -(dot(n, w0));
	float b = dot(n, dir);
	float rr = a / b;
	return dir * rr + r.p1;
}
GDI void intersects_sphere(const Ray &r, float radius, V3 &S1, V3 &S2) {
	V3 rp1 = r.p1 - v3(0, 0, 0), rp2 = r.p2 - v3(0, 0, 0);
	V3 e = normalized(rp2 - rp1);
	V3 h = v3(0, 0, 0) - rp1;
	float lf = dot(e, h);
	float radpow = radius * radius;
	float hdh = length_sq(h);
	float lfpow = lf * lf;
	float s = radpow - hdh + lfpow;
	if (s >= 0.0f) {
		s = sqrtf(s);
		if (lf < s) {
			if (lf + s >= 0) s = -s;
		}
		S1 = e * (lf - s) + rp1;
		S2 = e * (lf + s) + rp1;
	}
	S1 = S1 + v3(0, 0, 0);
	S2 = S2 + v3(0, 0, 0);
}
GDI V3 get_orthogonal(V3 p) {
	float threshold = length(p) * 0.6f;
	if (threshold > 0.f) {
		if (fabsf(p.x) <= threshold) {
			float inv = 1.f / sqrtf(p.y * p.y + p.z * p.z);
			return v3(0.f, inv * p.z, -inv * p.y);
		} else if (fabsf(p.y) <= threshold) {
			float inv = 1.f / sqrtf(p.x * p.x + p.z * p.z);
			return v3(-inv * p.z, 0.f, inv * p.x);
		}
		float inv = 1.f / sqrtf(p.x * p.x + p.y * p.y);
		return v3(inv * p.y, -inv * p.x, 0.f);
	}
	return v3(0, 0, 0);
}
GDI void set_control_point(Cone &c, V3 v) {
	if (is_zero_approx(length_sq(v))) c.cp = v3(0, 1, 0);
	else c.cp = normalized(v);
}
GDI void update_tangent_handles(Cone &c, const Cone *next, int lv) {
	if (!next) return;
	double radA = c.radius, radB = next->radius;
	V3 A = c.cp, Bv = next->cp;
	V3 arc_normal = normalized(cross(A, Bv));
	double tRadius = (gd::PI - (radA + radB)) / 2;
	double bA = radA + tRadius, bB = radB + tRadius;
	V3 scaledAxisA = A * (float)::cos(bA);
	V3 planeDir1A = xform(axis_angle_sq(arc_normal, (float)bA, lv), A);
	V3 planeDir2A = xform(axis_angle_sq(A, (float)(gd::PI / 2), lv), planeDir1A);
	V3 scaledAxisB = Bv * (float)::cos(bB);
	V3 planeDir1B = xform(axis_angle_sq(arc_normal, (float)bB, lv), Bv);
	V3 planeDir2B = xform(axis_angle_sq(Bv, (float)(gd::PI / 2), lv), planeDir1B);
	Ray r1B{planeDir1B, scaledAxisB}, r2B{planeDir1B, planeDir2B};
	elongate(r1B, 99);
	elongate(r2B, 99);
	V3 i1 = intersects_plane(r1B, scaledAxisA, planeDir1A, planeDir2A);
	V3 i2 = intersects_plane(r2B, scaledAxisA, planeDir1A, planeDir2A);
	Ray ir{i1, i2};
	elongate(ir, 99);
	V3 S1 = v3(0, 0, 0), S2 = v3(0, 0, 0);
	intersects_sphere(ir, 1.0f, S1, S2);
	c.t1 = normalized(S1);
	c.t2 = normalized(S2);
	c.tr = tRadius;
	c.trcos = ::cos(tRadius);
	if (is_zero_approx(length_sq(c.t1))) c.t1 = normalized(get_orthogonal(c.cp));
	if (is_zero_approx(length_sq(c.t2))) c.t2 = normalized(get_orthogonal(c.t1 * -1.0f));
}
GDI void update_tangent_radii(Cone *cs, int n, int lv) {
	for (int i = 0; i < n; i++) update_tangent_handles(cs[i], i + 1 < n ? &cs[i + 1] : nullptr, lv);
}

// Setup of one skeleton: reads its setup pose [B][10] and entry s_in of cones
// [.][constraints][max_cones_in][4] and twist [.][constraints][2]; writes column s of
// D [B][9][N], CF [NC][cfs][N], CD [NC][cds][N].
GDI void setup_skeleton(const SetupView &v, int s_in, int s, const float *pose, const float *cones, const float *twist,
		SetupScratch w, float *D, float *CF, double *CD) {
	const int B = v.B, NC = v.NC;
	const size_t N = (size_t)v.N;
	for (int b = 0; b < B; b++) w.L[b] = (v.bone_flags[b] & BF_IN_LIST) ? pose_to_xform(pose + 10 * b) : xid();
	for (int i = 0; i < v.n_topo; i++) {
		const int b = v.topo[i];
		const int pp = v.bone_pose_parent[b];
		if (pp >= 0) w.G[b] = w.G[pp] * w.L[b];
		else if (pp == POSE_PARENT_ORIGIN) w.G[b] = xid() * w.L[b];
		else w.G[b] = w.L[b];
	}
	for (int b = 0; b < B; b++) w.Dm[b] = bid();
	// IKBone3D::update_default_bone_direction_transform (ik_bone_3d.cpp:57-93), bone_list order.
	for (int i = 0; i < v.n_list; i++) {
		const int b = v.bone_list[i];
		V3 cc = v3(0, 0, 0);
		int count = 0;
		for (int k = v.ik_child_off[b]; k < v.ik_child_off[b + 1]; k++) {
			cc = cc + w.G[v.ik_children[k]].o;
			count++;
		}
		cc = divs(cc, (float)count); // count == 0 -> 0/0 (NaN), as the reference
		cc = cc - w.G[b].o;
		if (is_zero_approx(length_sq(cc))) {
			const int par = v.bone_ik_parent[b];
			cc = par >= 0 ? col(w.G[par].b * w.Dm[par], 1) : col(w.G[b].b * w.Dm[b], 1);
		}
		if (!is_zero_approx(length_sq(cc)) && count > 0) {
			cc = normalized(cc);
			V3 bd = normalized(col(w.G[b].b * w.Dm[b], 1));
			B3 P = w.G[b].b;
			w.Dm[b] = ((inverse(P) * from_quat(arc(cc, bd))) * P) * w.Dm[b];
		}
	}
	for (int b = 0; b < B; b++)
		for (int f = 0; f < 9; f++) D[((size_t)b * 9 + f) * N + s] = w.Dm[b].r[f / 3][f % 3];
	if (NC == 0) return;
	// Kusudama setup, in the constraint order of the description (many_bone_ik_3d.cpp:1037-1067).
	const int mc = v.max_cones_in;
	for (int c = 0; c < NC; c++) {
		w.T[c] = bid();
		w.kcn[c] = 0;
		w.tcr[c] = qid();
		w.thc[c] = 0.0f;
	}
	for (int c = 0; c < v.n_cons_order; c++) {
		const int ci = v.cons_order[c]; // index into the description's constraint array
		const int slot = v.cons_order_slot[c];
		const int b = v.cons_bone[slot];
		const int ncones = v.cons_order_ncones[c];
		const float *cn = cones + ((size_t)s_in * v.desc_constraint_count + ci) * mc * 4;
		const float *tw = twist + ((size_t)s_in * v.desc_constraint_count + ci) * 2;
		Cone *cs = w.cs;
		int ncs = 0;
		for (int k = 0; k < ncones; k++) {
			Cone cone;
			cone.t1 = v3(0, 0, 0);
			cone.t2 = v3(0, 0, 0);
			cone.tr = 0;
			cone.trcos = 0;
			double rad = cn[4 * k + 3];
			cone.radius = 1.0e-38 > rad ? 1.0e-38 : rad;
			cone.rcos = ::cos(cone.radius);
			set_control_point(cone, normalized(v3(cn[4 * k], cn[4 * k + 1], cn[4 * k + 2])));
			cs[ncs++] = cone;
			update_tangent_radii(cs, ncs, v.libm);
		}
		// set_axial_limits (ik_kusudama_3d.cpp:103-115)
		float min_angle = tw[0], range = tw[1];
		V3 y_axis = v3(0, 1, 0), z_axis = v3(0, 0, 1);
		Q twist_min_rot = axis_angle_sq(y_axis, min_angle, v.libm);
		V3 twist_min_vec = normalized(xform(twist_min_rot, z_axis));
		V3 twist_center_vec = normalized(xform(twist_min_rot, twist_min_vec));
		w.tcr[slot] = arc(z_axis, twist_center_vec);
		w.thc[slot] = cos_f(range / 4.0f, v.libm);
		// _update_constraint(twist node) (ik_kusudama_3d.cpp:37-89)
		V3 sum = v3(0, 0, 0);
		int nd = 0;
		if (ncs == 1) {
			sum = sum + cs[0].cp;
			nd = 1;
		} else {
			for (int k = 0; k + 1 < ncs; k++) {
				Q ttn = arc(cs[k].cp, cs[k + 1].cp);
				V3 axis = get_axis(ttn);
				double angle = get_angle(ttn) / 2.0;
				V3 half = xform(axis_angle_basis(axis, (float)angle, v.libm), cs[k].cp);
				half = half * get_angle(ttn);
				half = normalized(half);
				sum = sum + half;
				nd++;
			}
		}
		V3 new_y = sum;
		if (nd) new_y = normalized(divs(new_y, (float)nd));
		const int par = v.bone_ik_parent[b];
		if (par >= 0) {
			B3 gb = w.G[par].b * w.T[slot]; // twist node global = parent pose global * local
			Q otn = arc(normalized(col(gb, 1)), normalized(xform(gb, new_y)));
			B3 Pb = w.G[par].b;
			w.T[slot] = ((inverse(Pb) * from_quat(otn)) * Pb) * w.T[slot];
		}
		for (int k = 0; k < ncs; k++) set_control_point(cs[k], normalized(cs[k].cp));
		update_tangent_radii(cs, ncs, v.libm);
		for (int k = 0; k < ncs; k++) w.kc[(size_t)slot * mc + k] = cs[k];
		w.kcn[slot] = ncs;
	}
	for (int slot = 0; slot < NC; slot++) {
		float *cf = CF + (size_t)slot * v.cfs * N + s;
		double *cd = CD + (size_t)slot * v.cds * N + s;
		cf[(CF_TWIST_Q + 0) * N] = w.tcr[slot].x;
		cf[(CF_TWIST_Q + 1) * N] = w.tcr[slot].y;
		cf[(CF_TWIST_Q + 2) * N] = w.tcr[slot].z;
		cf[(CF_TWIST_Q + 3) * N] = w.tcr[slot].w;
		cf[CF_TWIST_COS * N] = w.thc[slot];
		for (int f = 0; f < 9; f++) cf[(CF_TWIST_T + f) * N] = w.T[slot].r[f / 3][f % 3];
		for (int k = 0; k < w.kcn[slot]; k++) {
			const Cone &c = w.kc[(size_t)slot * mc + k];
			const int o = CF_CONE0 + CF_PER_CONE * k;
			const float rf = (float)c.radius, trf = (float)c.tr;
			cf[(o + 0) * N] = c.cp.x; cf[(o + 1) * N] = c.cp.y; cf[(o + 2) * N] = c.cp.z;
			cf[(o + 3) * N] = sin_f(rf * 0.5f, v.libm); cf[(o + 4) * N] = cos_f(rf * 0.5f, v.libm);
			cf[(o + 5) * N] = c.t1.x; cf[(o + 6) * N] = c.t1.y; cf[(o + 7) * N] = c.t1.z;
			cf[(o + 8) * N] = c.t2.x; cf[(o + 9) * N] = c.t2.y; cf[(o + 10) * N] = c.t2.z;
			cf[(o + 11) * N] = sin_f(trf * 0.5f, v.libm); cf[(o + 12) * N] = cos_f(trf * 0.5f, v.libm);
			const V3 ncp = normalized(c.cp);
			cf[(o + CFC_NCP) * N] = ncp.x; cf[(o + CFC_NCP + 1) * N] = ncp.y; cf[(o + CFC_NCP + 2) * N] = ncp.z;
			if (k + 1 < w.kcn[slot]) {
				const V3 nx = w.kc[(size_t)slot * mc + k + 1].cp;
				const V3 pr[5] = {cross(c.cp, nx), normalized(cross(c.cp, c.t1)), normalized(cross(c.t2, c.cp)),
						normalized(cross(c.t1, nx)), normalized(cross(nx, c.t2))};
				for (int q = 0; q < 5; q++) {
					cf[(o + CFC_C1XC2 + 3 * q) * N] = pr[q].x;
					cf[(o + CFC_C1XC2 + 3 * q + 1) * N] = pr[q].y;
					cf[(o + CFC_C1XC2 + 3 * q + 2) * N] = pr[q].z;
				}
			}
			cd[(CD_PER_CONE * k + 0) * N] = c.rcos;
			cd[(CD_PER_CONE * k + 1) * N] = c.trcos;
		}
	}
}

} // namespace mbik
