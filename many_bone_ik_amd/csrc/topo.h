// GPU-side topology build: ManyBoneIK3D::_bone_list_changed's
// segmentation and heading weights for one rig, written allocation-free and recursion-free so
// that one GPU thread builds one rig (k_aux.hip: mbik_topology_kernel, a crowd of distinct rigs
// at once).  It restates, table for table, what plan.cpp's build_topology computes on the host:
//   IKBoneSegment3D::generate_default_segments    ik_bone_segment_3d.cpp:352-427 (preorder
//                                                  segment creation, _create_next_bone :401-407)
//   create_bone_list / the post-order solve order  :210-225, many_bone_ik_3d.cpp:1011-1068
//   update_pinned_list                            ik_bone_segment_3d.cpp:74-88
//   create_headings_arrays / recursive_create_penalty_array  :281-343
//   _qcp_solver's per-bone damping                 :227-240 (the cosines come in from the
//                                                  config: the device's double cos is not glibc's)
//   constraint slots                               many_bone_ik_3d.cpp:1037-1067
// The recursions of the reference become explicit stacks visiting in the same order, so every
// table comes out identical (mbik_selftest_topology compares them with build_topology's).
#pragma once

#include <cstddef>
#include <cstdint>

#include "gd_math.h"
#include "plan.h"

namespace mbik {

// One rig as the builder reads it (device pointers on the GPU).
struct TopoRig {
	int B, P, C, max_cones, stab;
	const int *parents;                  // [B]
	const int *pin_bone;                 // [P]
	const float *pin_weight, *pin_prio;  // [P], [P][3]
	const float *pin_mpf;                // [P] motion_propagation_factor (unclamped)
	const int *cons_bone, *cons_ncones;  // [C]
	const double *bone_chd;              // [B] cos(damp/2) of each bone in a non-root segment
	double root_chd;                     // cos(PI/2) of the root segments' bones
};

// Error codes of topo_build (0 = built); topo_error() gives build_topology's message.
enum TopoErr : int32_t {
	TE_OK = 0, TE_BONES = 1, TE_PARENTS = 2, TE_CYCLE = 3, TE_PIN = 4, TE_NOROOT = 5, TE_HEADINGS = 6,
	TE_CONS_BONE = 7, TE_CONS_CONES = 8, TE_LIMIT = 9
};
inline const char *topo_error(int e) {
	switch (e) {
	case TE_BONES: return "bone_count must be > 0 and parents non-null";
	case TE_PARENTS: return "parents out of range";
	case TE_CYCLE: return "parents contain a cycle";
	case TE_PIN: return "pin bone out of range";
	case TE_NOROOT: return "skeleton has no parentless bone";
	case TE_HEADINGS: return "heading count mismatch between effector list and penalty array";
	case TE_CONS_BONE: return "constraint bone out of range";
	case TE_CONS_CONES: return "constraint cone_count exceeds max_cones";
	case TE_LIMIT: return "more than 32767 bones or pins (the solve's step records hold 16-bit fields)";
	default: return "";
	}
}

// Counters of a built rig (TopoOut::count[...]).
enum TopoCount : int32_t {
	TC_ERR = 0, TC_NS, TC_NLIST, TC_NSEGEFF, TC_NHW, TC_NC, TC_MAXH, TC_CM_MAXD, TC_CM_NPOS, TC_NROOTS, TC_NPATH,
	TC_NCHILDEFF, TC_NCONSORD, TC_N
};

// The built tables (each sized for the worst case of B, P, C).
struct TopoOut {
	int32_t *count;  // [TC_N]
	int32_t *bone_pose_parent, *bone_ik_parent, *bone_depth, *bone_flags, *bone_pin, *bone_cons, *bone_list;
	int32_t *bone_child_eff_off, *bone_child_effs;
	int32_t *seg_root, *seg_tip, *seg_parent, *seg_child_off, *seg_children, *seg_bone_off, *seg_bones;
	int32_t *seg_eff_off, *seg_effs, *seg_eff_hoff, *seg_nh, *seg_flags, *seg_hw_off, *seg_height, *seg_tin, *seg_tout;
	int32_t *roots, *eff_parent_bone, *eff_path_off, *eff_path;
	int32_t *cons_bone, *cons_ncones, *cons_order, *cons_order_slot, *cons_order_ncones, *cm_pre, *cm_sub;
	double *seg_hw, *seg_cos_half_damp;
	float *seg_wsum2;
};
// Working memory of one build.
struct TopoScratch {
	int32_t *kid_off, *kids, *stack, *sg_root, *sg_tip, *sg_parent, *sg_pinned, *new_id, *kept_off, *kept, *order;
	int32_t *effl_off, *effl, *pk_off, *pk, *pk_fill;
	double *fstack;
};

// Element counts of the int32 / double / float parts of TopoOut, and of TopoScratch's ints
// and doubles, for a rig of B bones, P pins, C constraints.
struct TopoSizes {
	size_t out_ints, out_dbls, out_flts, scr_ints, scr_dbls;
};
GDI size_t topo_align4(size_t n) { return (n + 3) & ~size_t(3); }
GDI TopoSizes topo_sizes(int B, int P, int C) {
	const size_t b = (size_t)B, p = (size_t)P, c = (size_t)C;
	TopoSizes s;
	s.out_ints = topo_align4(TC_N) + 7 * topo_align4(b) + topo_align4(b + 1) + topo_align4(p + 1) + 3 * topo_align4(b) +
			topo_align4(b + 1) + topo_align4(b) + topo_align4(b + 1) + topo_align4(b) + topo_align4(b + 1) +
			2 * topo_align4(b * p + 1) + 7 * topo_align4(b) + topo_align4(b) + 2 * topo_align4(p + 1) +
			topo_align4(p * b + 1) + 5 * topo_align4(c + 1) + 2 * topo_align4(b);
	s.out_dbls = topo_align4(b * 7 * p + 1) + topo_align4(b);
	s.out_flts = topo_align4(b);
	s.scr_ints = topo_align4(b + 1) + topo_align4(b) + topo_align4(4 * b + 4) + 4 * topo_align4(b) + topo_align4(b) +
			topo_align4(b + 1) + topo_align4(b) + topo_align4(b) + topo_align4(b + 1) + topo_align4(b * p + 1) +
			topo_align4(b + 1) + topo_align4(b) + topo_align4(b + 1);
	s.scr_dbls = topo_align4(b + 1);
	return s;
}
GDI TopoOut topo_out_at(int32_t *ib, double *db, float *fb, int B, int P, int C) {
	const size_t b = (size_t)B, p = (size_t)P, c = (size_t)C;
	TopoOut o;
	auto ti = [&](size_t n) {
		int32_t *r = ib;
		ib += topo_align4(n);
		return r;
	};
	o.count = ti(TC_N);
	o.bone_pose_parent = ti(b); o.bone_ik_parent = ti(b); o.bone_depth = ti(b); o.bone_flags = ti(b);
	o.bone_pin = ti(b); o.bone_cons = ti(b); o.bone_list = ti(b);
	o.bone_child_eff_off = ti(b + 1); o.bone_child_effs = ti(p + 1);
	o.seg_root = ti(b); o.seg_tip = ti(b); o.seg_parent = ti(b);
	o.seg_child_off = ti(b + 1); o.seg_children = ti(b); o.seg_bone_off = ti(b + 1); o.seg_bones = ti(b);
	o.seg_eff_off = ti(b + 1); o.seg_effs = ti(b * p + 1); o.seg_eff_hoff = ti(b * p + 1);
	o.seg_nh = ti(b); o.seg_flags = ti(b); o.seg_hw_off = ti(b); o.seg_height = ti(b); o.seg_tin = ti(b); o.seg_tout = ti(b);
	o.roots = ti(b);
	o.eff_parent_bone = ti(b); // (p entries; b >= 1 keeps the layout simple)
	o.eff_path_off = ti(p + 1); o.eff_path = ti(p * b + 1);
	o.cons_bone = ti(c + 1); o.cons_ncones = ti(c + 1); o.cons_order = ti(c + 1); o.cons_order_slot = ti(c + 1);
	o.cons_order_ncones = ti(c + 1);
	o.cm_pre = ti(b); o.cm_sub = ti(b);
	o.seg_hw = db;
	o.seg_cos_half_damp = db + topo_align4(b * 7 * p + 1);
	o.seg_wsum2 = fb;
	return o;
}
GDI TopoScratch topo_scratch_at(int32_t *ib, double *db, int B, int P) {
	const size_t b = (size_t)B, p = (size_t)P;
	TopoScratch s;
	auto ti = [&](size_t n) {
		int32_t *r = ib;
		ib += topo_align4(n);
		return r;
	};
	s.kid_off = ti(b + 1); s.kids = ti(b); s.stack = ti(4 * b + 4);
	s.sg_root = ti(b); s.sg_tip = ti(b); s.sg_parent = ti(b); s.sg_pinned = ti(b); s.new_id = ti(b);
	s.kept_off = ti(b + 1); s.kept = ti(b); s.order = ti(b);
	s.effl_off = ti(b + 1); s.effl = ti(b * p + 1);
	s.pk_off = ti(b + 1); s.pk = ti(b); s.pk_fill = ti(b + 1);
	s.fstack = db;
	return s;
}

GDI float topo_mpf(const TopoRig &r, int pin) { // IKEffector3D::set_motion_propagation_factor clamps
	const double v = r.pin_mpf[pin];
	return (float)(v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
}
GDI int topo_nheads(const TopoRig &r, int pin) {
	int n = 1;
	for (int a = 0; a < 3; a++)
		if (r.pin_prio[3 * pin + a] > 0.0f) n += 2;
	return n;
}

// Builds one rig's tables into o; returns 0 or a TopoErr (also in o.count[TC_ERR]).
GDI int topo_build(const TopoRig &r, const TopoOut &o, const TopoScratch &w) {
	const int B = r.B, P = r.P;
	int32_t *cnt = o.count;
	for (int i = 0; i < TC_N; i++) cnt[i] = 0;
	auto fail = [&](int e) {
		cnt[TC_ERR] = e;
		return e;
	};
	if (B <= 0 || !r.parents) return fail(TE_BONES);
	for (int b = 0; b < B; b++)
		if (r.parents[b] < -1 || r.parents[b] >= B || r.parents[b] == b) return fail(TE_PARENTS);
	// Skeleton3D::get_bone_children: ascending bone index (CSR)
	for (int b = 0; b <= B; b++) w.kid_off[b] = 0;
	for (int b = 0; b < B; b++)
		if (r.parents[b] >= 0) w.kid_off[r.parents[b] + 1]++;
	for (int b = 0; b < B; b++) w.kid_off[b + 1] += w.kid_off[b];
	for (int b = 0; b <= B; b++) w.pk_fill[b] = w.kid_off[b];
	for (int b = 0; b < B; b++)
		if (r.parents[b] >= 0) w.kids[w.pk_fill[r.parents[b]]++] = b;
	// depths (and the cycle check) with an explicit stack
	for (int b = 0; b < B; b++) o.bone_depth[b] = -1;
	for (int b = 0; b < B; b++) {
		int n = 0, x = b;
		while (x >= 0 && o.bone_depth[x] < 0) {
			if (n > B) return fail(TE_CYCLE);
			w.stack[n++] = x;
			x = r.parents[x];
		}
		int d = x < 0 ? -1 : o.bone_depth[x];
		while (n > 0) o.bone_depth[w.stack[--n]] = ++d;
	}
	// IKBone3D ctor: the first matching IKEffectorTemplate3D (ik_bone_3d.cpp:209-222)
	for (int b = 0; b < B; b++) o.bone_pin[b] = -1;
	for (int i = P; i-- > 0;) {
		const int b = r.pin_bone[i];
		if (b < 0 || b >= B) return fail(TE_PIN);
		o.bone_pin[b] = i;
	}
	// generate_default_segments: segments created depth first (preorder ids), a segment ends
	// at a leaf, a branch or a pinned bone, and each child of its tip roots a new segment
	for (int b = 0; b < B; b++) o.bone_ik_parent[b] = -1;
	int nseg = 0, sp = 0;
	for (int root = 0; root < B; root++) {
		if (r.parents[root] >= 0) continue;
		w.stack[sp++] = root;
		w.stack[sp++] = -1;
		while (sp > 0) {
			const int ps = w.stack[--sp], rb = w.stack[--sp];
			const int si = nseg++;
			w.sg_root[si] = rb;
			w.sg_parent[si] = ps;
			int cur = rb;
			for (;;) {
				const int c0 = w.kid_off[cur], nch = w.kid_off[cur + 1] - c0;
				if (nch != 1 || o.bone_pin[cur] >= 0) {
					for (int k = nch; k-- > 0;) { // the first child is created (popped) first
						const int c = w.kids[c0 + k];
						o.bone_ik_parent[c] = cur; // root->set_parent(p_parent->get_tip()) :259-262
						w.stack[sp++] = c;
						w.stack[sp++] = si;
					}
					break;
				}
				const int nx = w.kids[c0];
				o.bone_ik_parent[nx] = cur; // _create_next_bone :401-407
				cur = nx;
			}
			w.sg_tip[si] = cur;
		}
	}
	if (nseg == 0) return fail(TE_NOROOT);
	if (B > 32767 || P > 32767) return fail(TE_LIMIT);
	// a segment is kept when a pinned bone is at or below its tip (children have larger ids)
	for (int si = 0; si < nseg; si++) w.sg_pinned[si] = o.bone_pin[w.sg_tip[si]] >= 0;
	for (int si = nseg; si-- > 1;)
		if (w.sg_pinned[si] && w.sg_parent[si] >= 0) w.sg_pinned[w.sg_parent[si]] = 1;
	for (int si = 0; si <= nseg; si++) w.kept_off[si] = 0;
	for (int si = 0; si < nseg; si++)
		if (w.sg_parent[si] >= 0 && w.sg_pinned[si]) w.kept_off[w.sg_parent[si] + 1]++;
	for (int si = 0; si < nseg; si++) w.kept_off[si + 1] += w.kept_off[si];
	for (int si = 0; si <= nseg; si++) w.pk_fill[si] = w.kept_off[si];
	for (int si = 0; si < nseg; si++)
		if (w.sg_parent[si] >= 0 && w.sg_pinned[si]) w.kept[w.pk_fill[w.sg_parent[si]]++] = si;
	// post-order solve numbering of the kept segments, root segments in creation order
	int ns = 0, nroots = 0;
	for (int si = 0; si < nseg; si++) w.new_id[si] = -1;
	for (int rs = 0; rs < nseg; rs++) {
		if (w.sg_parent[rs] >= 0) continue;
		w.stack[0] = rs;
		w.stack[1] = 0;
		sp = 2;
		while (sp > 0) {
			const int si = w.stack[sp - 2], c = w.stack[sp - 1];
			if (c < w.kept_off[si + 1] - w.kept_off[si]) {
				w.stack[sp - 1] = c + 1;
				w.stack[sp++] = w.kept[w.kept_off[si] + c];
				w.stack[sp++] = 0;
			} else {
				sp -= 2;
				w.order[ns] = si;
				w.new_id[si] = ns++;
			}
		}
		o.roots[nroots++] = w.new_id[rs];
	}
	cnt[TC_NS] = ns;
	cnt[TC_NROOTS] = nroots;
	int nlist = 0;
	o.seg_bone_off[0] = 0;
	o.seg_child_off[0] = 0;
	for (int i = 0; i < ns; i++) {
		const int g = w.order[i];
		o.seg_root[i] = w.sg_root[g];
		o.seg_tip[i] = w.sg_tip[g];
		o.seg_parent[i] = w.sg_parent[g] >= 0 ? w.new_id[w.sg_parent[g]] : -1;
		int nc = o.seg_child_off[i];
		for (int k = w.kept_off[g]; k < w.kept_off[g + 1]; k++) o.seg_children[nc++] = w.new_id[w.kept[k]];
		o.seg_child_off[i + 1] = nc;
		o.seg_flags[i] = 0;
		if (w.sg_parent[g] < 0) o.seg_flags[i] |= SF_TRANSLATE;
		if (w.sg_parent[g] < 0 && r.stab > 0) o.seg_flags[i] |= SF_STAB;
		for (int b = o.seg_tip[i]; b >= 0; b = o.bone_ik_parent[b]) { // tip -> root
			o.seg_bones[nlist] = b;
			o.bone_list[nlist++] = b;
			if (b == o.seg_root[i]) break;
		}
		o.seg_bone_off[i + 1] = nlist;
	}
	cnt[TC_NLIST] = nlist;
	// pose-node parents: only the last root keeps the ik_origin (many_bone_ik_3d.cpp:1022-1023)
	for (int b = 0; b < B; b++) o.bone_pose_parent[b] = o.bone_ik_parent[b];
	{
		int k = 0;
		for (int si = 0; si < nseg; si++)
			if (w.sg_parent[si] < 0) {
				k++;
				o.bone_pose_parent[w.sg_root[si]] = k == nroots ? POSE_PARENT_ORIGIN : POSE_PARENT_NONE;
			}
	}
	// update_pinned_list (:74-88): a segment's effectors, children's after its own
	w.effl_off[0] = 0;
	for (int i = 0; i < ns; i++) {
		int n = w.effl_off[i];
		const int tip = o.seg_tip[i];
		const bool pinned = o.bone_pin[tip] >= 0;
		if (pinned) w.effl[n++] = o.bone_pin[tip];
		const double f = pinned ? (double)topo_mpf(r, o.bone_pin[tip]) : 1.0;
		if (f > 0.0)
			for (int k = o.seg_child_off[i]; k < o.seg_child_off[i + 1]; k++) {
				const int c = o.seg_children[k];
				for (int q = w.effl_off[c]; q < w.effl_off[c + 1]; q++) w.effl[n++] = w.effl[q];
			}
		w.effl_off[i + 1] = n;
	}
	// recursive_create_penalty_array (:309-343) per segment, preorder with the falloff
	int nse = 0, nhw = 0, maxh = 0;
	o.seg_eff_off[0] = 0;
	for (int i = 0; i < ns; i++) {
		o.seg_hw_off[i] = nhw;
		sp = 0;
		w.stack[sp] = i;
		w.fstack[sp++] = 1.0;
		while (sp > 0) {
			--sp;
			const int si = w.stack[sp];
			const double falloff = w.fstack[sp];
			if (falloff <= 0.0) continue;
			double current = 1.0;
			const int tip = o.seg_tip[si];
			if (o.bone_pin[tip] >= 0) {
				const int pin = o.bone_pin[tip];
				const double weight = r.pin_weight[pin];
				o.seg_hw[nhw++] = weight * falloff;
				const float *pr = r.pin_prio + 3 * pin;
				const float m01 = pr[0] < pr[1] ? pr[1] : pr[0]; // std::max
				const float mx = m01 < pr[2] ? pr[2] : m01;
				double mpw = mx;
				mpw = mpw == 0.0 ? 1.0 : mpw;
				for (int a = 0; a < 3; a++) {
					const double pri = pr[a];
					if (pri > 0.0) {
						const double sub = weight * (pri / mpw) * falloff;
						o.seg_hw[nhw++] = sub;
						o.seg_hw[nhw++] = sub;
					}
				}
				current = topo_mpf(r, pin);
			}
			for (int k = o.seg_child_off[si + 1]; k-- > o.seg_child_off[si];) { // first child on top
				w.stack[sp] = o.seg_children[k];
				w.fstack[sp++] = falloff * current;
			}
		}
		int h = 0;
		for (int q = w.effl_off[i]; q < w.effl_off[i + 1]; q++) {
			o.seg_effs[nse] = w.effl[q];
			o.seg_eff_hoff[nse++] = h;
			h += topo_nheads(r, w.effl[q]);
		}
		if (h != nhw - o.seg_hw_off[i]) return fail(TE_HEADINGS);
		o.seg_eff_off[i + 1] = nse;
		o.seg_nh[i] = h;
		maxh = h > maxh ? h : maxh;
		float ws = 0.0f; // _get_manual_msd (:114-127): float w_sum += double weight
		for (int q = o.seg_hw_off[i]; q < nhw; q++) ws = (float)((double)ws + o.seg_hw[q]);
		o.seg_wsum2[i] = ws * ws;
	}
	cnt[TC_NSEGEFF] = nse;
	cnt[TC_NHW] = nhw;
	cnt[TC_MAXH] = maxh;
	// damping per (segment, bone): _qcp_solver (:227-240), the root segment uses PI (:217-222)
	for (int i = 0; i < ns; i++)
		for (int k = o.seg_bone_off[i]; k < o.seg_bone_off[i + 1]; k++)
			o.seg_cos_half_damp[k] = (o.seg_flags[i] & SF_TRANSLATE) ? r.root_chd : r.bone_chd[o.seg_bones[k]];
	// effector paths from the skeleton root
	int npath = 0;
	o.eff_path_off[0] = 0;
	for (int e = 0; e < P; e++) {
		const int b = r.pin_bone[e];
		o.eff_parent_bone[e] = o.bone_ik_parent[b];
		const int len = o.bone_depth[b] + 1;
		int x = b;
		for (int q = len; q-- > 0; x = r.parents[x]) o.eff_path[npath + q] = x;
		npath += len;
		o.eff_path_off[e + 1] = npath;
	}
	cnt[TC_NPATH] = npath;
	for (int b = 0; b < B; b++) o.bone_flags[b] = 0;
	for (int k = 0; k < nlist; k++) o.bone_flags[o.bone_list[k]] |= BF_IN_LIST;
	for (int b = 0; b < B; b++)
		if (o.bone_pin[b] >= 0 && (o.bone_flags[b] & BF_IN_LIST)) o.bone_flags[b] |= BF_PINNED;
	int nce = 0;
	o.bone_child_eff_off[0] = 0;
	for (int b = 0; b < B; b++) {
		for (int k = w.kid_off[b]; k < w.kid_off[b + 1]; k++) {
			const int c = w.kids[k];
			if ((o.bone_flags[c] & BF_PINNED) && o.bone_ik_parent[c] == b) o.bone_child_effs[nce++] = o.bone_pin[c];
		}
		o.bone_child_eff_off[b + 1] = nce;
	}
	cnt[TC_NCHILDEFF] = nce;
	// constraint slots: named constraints whose bone is in the bone list (:1037-1067)
	for (int b = 0; b < B; b++) o.bone_cons[b] = -1;
	int nc = 0, nord = 0;
	for (int c = 0; c < r.C; c++) {
		const int b = r.cons_bone[c], ncones = r.cons_ncones[c];
		if (b < 0 || b >= B) return fail(TE_CONS_BONE);
		if (ncones < 0 || ncones > r.max_cones) return fail(TE_CONS_CONES);
		if (!(o.bone_flags[b] & BF_IN_LIST)) continue;
		if (o.bone_cons[b] < 0) {
			o.bone_cons[b] = nc;
			o.cons_bone[nc] = b;
			o.cons_ncones[nc++] = ncones;
		} else {
			o.cons_ncones[o.bone_cons[b]] = ncones; // a later constraint replaces
		}
		o.cons_order[nord] = c;
		o.cons_order_slot[nord] = o.bone_cons[b];
		o.cons_order_ncones[nord++] = ncones;
		if (o.bone_ik_parent[b] >= 0) o.bone_flags[b] |= BF_ORIENT | BF_AXIAL;
	}
	cnt[TC_NC] = nc;
	cnt[TC_NCONSORD] = nord;
	// segment heights and subtree ranges (post-order: the subtree of i is [tin, i])
	for (int i = 0; i < ns; i++) {
		int h = 0, lo = i;
		for (int k = o.seg_child_off[i]; k < o.seg_child_off[i + 1]; k++) {
			const int c = o.seg_children[k];
			h = o.seg_height[c] + 1 > h ? o.seg_height[c] + 1 : h;
			lo = o.seg_tin[c] < lo ? o.seg_tin[c] : lo;
		}
		o.seg_height[i] = h;
		o.seg_tin[i] = lo;
		o.seg_tout[i] = i;
	}
	// constraint_mode node caches: pre-order positions over the pose-node forest of the list
	// bones (children in bone-list order)
	for (int b = 0; b < B; b++) {
		o.cm_pre[b] = -1;
		o.cm_sub[b] = 0;
	}
	for (int b = 0; b <= B; b++) w.pk_off[b] = 0;
	for (int k = 0; k < nlist; k++) {
		const int pp = o.bone_pose_parent[o.bone_list[k]];
		if (pp >= 0) w.pk_off[pp + 1]++;
	}
	for (int b = 0; b < B; b++) w.pk_off[b + 1] += w.pk_off[b];
	for (int b = 0; b <= B; b++) w.pk_fill[b] = w.pk_off[b];
	for (int k = 0; k < nlist; k++) {
		const int b = o.bone_list[k], pp = o.bone_pose_parent[b];
		if (pp >= 0) w.pk[w.pk_fill[pp]++] = b;
	}
	int pos = 0, maxd = 1;
	for (int k = 0; k < nlist; k++) {
		const int rb = o.bone_list[k];
		if (o.bone_pose_parent[rb] >= 0) continue;
		sp = 0;
		w.stack[sp++] = rb;
		w.stack[sp++] = 0;
		while (sp > 0) {
			const int d = w.stack[--sp], b = w.stack[--sp];
			if (b < 0) {
				o.cm_sub[-b - 1] = pos - o.cm_pre[-b - 1];
				continue;
			}
			o.cm_pre[b] = pos++;
			maxd = d + 1 > maxd ? d + 1 : maxd;
			w.stack[sp++] = -b - 1;
			w.stack[sp++] = d;
			for (int q = w.pk_off[b + 1]; q-- > w.pk_off[b];) {
				w.stack[sp++] = w.pk[q];
				w.stack[sp++] = d + 1;
			}
		}
	}
	cnt[TC_CM_MAXD] = maxd;
	cnt[TC_CM_NPOS] = pos;
	return TE_OK;
}

} // namespace mbik
