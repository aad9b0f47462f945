// Host plan builder: a flat restatement of ManyBoneIK3D::_bone_list_changed
// (src/many_bone_ik_3d.cpp:1011-1068) and everything it calls, producing the tables
// the gfx950 solve kernel reads.  No object graph: segment structure, effector lists and
// heading weights are computed once per topology; bone-direction and Kusudama frames once
// per skeleton (they depend on the setup pose).
#include "plan.h"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "gd_math.h"
#include "setup.h"
#include "topo.h"

namespace mbik {

using namespace gd;

// ---------------------------------------------------------------------------------------
// Topology
// ---------------------------------------------------------------------------------------
std::string build_topology(const mbik_skeleton_desc &desc, const mbik_config &cfg, HostPlan &p) {
	const int B = desc.bone_count;
	if (B <= 0 || !desc.parents) return "bone_count must be > 0 and parents non-null";
	if (desc.pin_count < 0 || (desc.pin_count > 0 && !desc.pins)) return "invalid pins";
	if (desc.constraint_count < 0 || (desc.constraint_count > 0 && !desc.constraints)) return "invalid constraints";
	if (cfg.iterations_per_frame < 0) return "iterations_per_frame must be >= 0";
	if (cfg.bone_damp_count < 0) return "negative count";
	p.B = B;
	p.P = desc.pin_count;
	p.max_cones = std::max(1, desc.max_cones);
	p.iterations = cfg.iterations_per_frame;
	p.constraint_mode = cfg.constraint_mode;
	p.stabilization_passes = cfg.stabilization_passes;
	p.parents.assign(desc.parents, desc.parents + B);
	for (int b = 0; b < B; b++)
		if (p.parents[b] < -1 || p.parents[b] >= B || p.parents[b] == b) return "parents out of range";
	// Skeleton3D::get_bone_children: ascending bone index.
	std::vector<std::vector<int>> kids(B);
	for (int b = 0; b < B; b++)
		if (p.parents[b] >= 0) kids[p.parents[b]].push_back(b);
	// cycle check + depth
	p.bone_depth.assign(B, -1);
	std::function<int(int, int)> depth_of = [&](int b, int guard) -> int {
		if (guard > B) return -1000000;
		if (p.bone_depth[b] >= 0) return p.bone_depth[b];
		int d = p.parents[b] < 0 ? 0 : depth_of(p.parents[b], guard + 1) + 1;
		p.bone_depth[b] = d;
		return d;
	};
	for (int b = 0; b < B; b++)
		if (depth_of(b, 0) < 0) return "parents contain a cycle";
	// IKBone3D ctor: first matching IKEffectorTemplate3D (ik_bone_3d.cpp:209-222).
	p.bone_pin.assign(B, -1);
	for (int i = desc.pin_count; i-- > 0;) {
		int b = desc.pins[i].bone;
		if (b < 0 || b >= B) return "pin bone out of range";
		p.bone_pin[b] = i;
	}
	p.eff_bone.resize(p.P);
	p.eff_prio.resize(3 * p.P);
	for (int i = 0; i < p.P; i++) {
		p.eff_bone[i] = desc.pins[i].bone;
		for (int a = 0; a < 3; a++) p.eff_prio[3 * i + a] = desc.pins[i].direction_priorities[a];
	}
	auto mpf = [&](int pin) -> float { // IKEffector3D::set_motion_propagation_factor clamps
		double v = desc.pins[pin].motion_propagation_factor;
		return (float)(v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
	};

	// IKBoneSegment3D::generate_default_segments (ik_bone_segment_3d.cpp:352-427).
	struct Seg {
		int root, tip = -1, parent;
		std::vector<int> kept, bones;
		bool pinned_desc = false;
	};
	std::vector<Seg> segs;
	p.bone_ik_parent.assign(B, -1);
	std::function<void(int)> gen = [&](int si) {
		int cur = segs[si].root;
		for (;;) {
			const auto &ch = kids[cur];
			if (ch.empty() || ch.size() > 1 || p.bone_pin[cur] >= 0) {
				segs[si].tip = cur;
				for (int c : ch) {
					int ci = (int)segs.size();
					segs.push_back(Seg{c, -1, si});
					p.bone_ik_parent[c] = cur; // root->set_parent(p_parent->get_tip()) :259-262
					gen(ci);
					if (segs[ci].pinned_desc) {
						segs[si].pinned_desc = true;
						segs[si].kept.push_back(ci);
					}
				}
				break;
			}
			int nx = ch[0];
			p.bone_ik_parent[nx] = cur; // _create_next_bone :401-407
			cur = nx;
		}
		Seg &g = segs[si];
		g.tip = cur;
		if (p.bone_pin[g.tip] >= 0) g.pinned_desc = true;
		for (int b = g.tip; b >= 0; b = p.bone_ik_parent[b]) {
			g.bones.push_back(b);
			if (b == g.root) break;
		}
	};
	std::vector<int> root_segs;
	for (int r = 0; r < B; r++) {
		if (p.parents[r] >= 0) continue;
		root_segs.push_back((int)segs.size());
		segs.push_back(Seg{r, -1, -1});
		gen(root_segs.back());
	}
	if (root_segs.empty()) return "skeleton has no parentless bone";
	if (B > 32767 || p.P > 32767) return "more than 32767 bones or pins (the solve's step records hold 16-bit fields)";

	// Kept segments in solve (post-order) numbering; bone_list per create_bone_list(true).
	std::vector<int> order; // old ids in post-order
	std::function<void(int)> post = [&](int si) {
		for (int c : segs[si].kept) post(c);
		order.push_back(si);
	};
	std::vector<int> new_id(segs.size(), -1);
	for (int r : root_segs) post(r);
	for (size_t i = 0; i < order.size(); i++) new_id[order[i]] = (int)i;
	p.NS = (int)order.size();
	p.seg_root.resize(p.NS);
	p.seg_tip.resize(p.NS);
	p.seg_parent.resize(p.NS);
	p.seg_children.assign(p.NS, {});
	p.seg_flags.assign(p.NS, 0);
	p.seg_bone_off.assign(1, 0);
	p.bone_list.clear();
	for (int i = 0; i < p.NS; i++) {
		const Seg &g = segs[order[i]];
		p.seg_root[i] = g.root;
		p.seg_tip[i] = g.tip;
		p.seg_parent[i] = g.parent >= 0 ? new_id[g.parent] : -1;
		for (int c : g.kept) p.seg_children[i].push_back(new_id[c]);
		if (g.parent < 0) p.seg_flags[i] |= SF_TRANSLATE;
		if (g.parent < 0 && cfg.stabilization_passes > 0) p.seg_flags[i] |= SF_STAB;
		for (int b : g.bones) {
			p.seg_bones.push_back(b);
			p.bone_list.push_back(b);
		}
		p.seg_bone_off.push_back((int)p.seg_bones.size());
	}
	for (int r : root_segs) p.roots.push_back(new_id[r]);

	// Pose-node parents: ik_origin is re-instantiated per root, so only the last root keeps
	// one (many_bone_ik_3d.cpp:1022-1023; the released origin's cleanup() detaches its child).
	p.bone_pose_parent.assign(B, POSE_PARENT_NONE);
	for (int b = 0; b < B; b++) p.bone_pose_parent[b] = p.bone_ik_parent[b];
	for (size_t i = 0; i < root_segs.size(); i++)
		p.bone_pose_parent[segs[root_segs[i]].root] = (i + 1 == root_segs.size()) ? POSE_PARENT_ORIGIN : POSE_PARENT_NONE;

	// update_pinned_list (:74-88) and recursive_create_penalty_array (:309-343).
	std::vector<std::vector<int>> effl(p.NS);
	for (int i = 0; i < p.NS; i++) { // post-order: children done first
		int tip = p.seg_tip[i];
		bool pinned = p.bone_pin[tip] >= 0;
		if (pinned) effl[i].push_back(p.bone_pin[tip]);
		double f = pinned ? (double)mpf(p.bone_pin[tip]) : 1.0;
		if (f > 0.0)
			for (int c : p.seg_children[i]) effl[i].insert(effl[i].end(), effl[c].begin(), effl[c].end());
	}
	std::function<void(int, std::vector<double> &, double)> penalty = [&](int si, std::vector<double> &out, double falloff) {
		if (falloff <= 0.0) return;
		double current = 1.0;
		int tip = p.seg_tip[si];
		if (p.bone_pin[tip] >= 0) {
			const mbik_pin &pin = desc.pins[p.bone_pin[tip]];
			double weight = pin.weight;
			out.push_back(weight * falloff);
			const float *pr = pin.direction_priorities;
			float mx = std::max(std::max(pr[0], pr[1]), pr[2]);
			double mpw = mx;
			mpw = mpw == 0.0 ? 1.0 : mpw;
			for (int a = 0; a < 3; a++) {
				double pri = pr[a];
				if (pri > 0.0) {
					double sub = weight * (pri / mpw) * falloff;
					out.push_back(sub);
					out.push_back(sub);
				}
			}
			current = mpf(p.bone_pin[tip]);
		}
		for (int c : p.seg_children[si]) penalty(c, out, falloff * current);
	};
	auto nheads = [&](int pin) {
		int n = 1;
		for (int a = 0; a < 3; a++)
			if (desc.pins[pin].direction_priorities[a] > 0.0) n += 2;
		return n;
	};
	p.seg_eff_off.assign(1, 0);
	p.seg_hw_off.assign(p.NS, 0);
	p.seg_nh.assign(p.NS, 0);
	p.max_headings = 0;
	for (int i = 0; i < p.NS; i++) {
		std::vector<double> w;
		penalty(i, w, 1.0);
		int h = 0;
		for (int e : effl[i]) {
			p.seg_effs.push_back(e);
			p.seg_eff_hoff.push_back(h);
			h += nheads(e);
		}
		if ((size_t)h != w.size()) return "heading count mismatch between effector list and penalty array";
		p.seg_eff_off.push_back((int)p.seg_effs.size());
		p.seg_hw_off[i] = (int)p.seg_hw.size();
		p.seg_hw.insert(p.seg_hw.end(), w.begin(), w.end());
		p.seg_nh[i] = h;
		p.max_headings = std::max(p.max_headings, h);
		// _get_manual_msd (ik_bone_segment_3d.cpp:114-127): float w_sum += double weight.
		float ws = 0.0f;
		for (double x : w) ws = (float)((double)ws + x);
		p.seg_wsum2.push_back(ws * ws);
	}
	// Damping per (segment, bone): _qcp_solver (:227-240); the root segment uses PI (:217-222).
	p.seg_cos_half_damp.clear();
	for (int i = 0; i < p.NS; i++) {
		for (int k = p.seg_bone_off[i]; k < p.seg_bone_off[i + 1]; k++) {
			int b = p.seg_bones[k];
			float d;
			if (p.seg_flags[i] & SF_TRANSLATE) {
				d = (float)gd::PI;
			} else {
				float def = cfg.default_damp;
				d = def;
				if (b < cfg.bone_damp_count && cfg.bone_damp) d = cfg.bone_damp[b];
				if (def < d) d = def;
			}
			double dampening = (double)(float)(double)d; // float -> double -> float p_dampening -> double
			p.seg_cos_half_damp.push_back(std::cos(dampening / 2.0));
		}
	}
	// Effector paths from the skeleton root, pinned IK children per bone.
	p.eff_parent_bone.assign(p.P, -1);
	p.eff_path_off.assign(1, 0);
	for (int e = 0; e < p.P; e++) {
		int b = p.eff_bone[e];
		p.eff_parent_bone[e] = p.bone_ik_parent[b];
		std::vector<int> path;
		for (int x = b; x >= 0; x = p.parents[x]) path.push_back(x);
		std::reverse(path.begin(), path.end());
		p.eff_path.insert(p.eff_path.end(), path.begin(), path.end());
		p.eff_path_off.push_back((int)p.eff_path.size());
	}
	p.bone_flags.assign(B, 0);
	for (int b : p.bone_list) p.bone_flags[b] |= BF_IN_LIST;
	for (int b = 0; b < B; b++)
		if (p.bone_pin[b] >= 0 && (p.bone_flags[b] & BF_IN_LIST)) p.bone_flags[b] |= BF_PINNED;
	p.bone_child_eff_off.assign(1, 0);
	for (int b = 0; b < B; b++) {
		for (int c : kids[b])
			if ((p.bone_flags[c] & BF_PINNED) && p.bone_ik_parent[c] == b) p.bone_child_effs.push_back(p.bone_pin[c]);
		p.bone_child_eff_off.push_back((int)p.bone_child_effs.size());
	}
	// Constraint slots: named constraints whose bone is in the bone list (:1037-1067).
	p.bone_cons.assign(B, -1);
	p.cons_bone.clear();
	p.cons_ncones.clear();
	p.cons_order.clear();
	p.cons_order_slot.clear();
	p.cons_order_ncones.clear();
	p.desc_constraint_count = desc.constraint_count;
	for (int c = 0; c < desc.constraint_count; c++) {
		int b = desc.constraints[c].bone;
		if (b < 0 || b >= B) return "constraint bone out of range";
		if (desc.constraints[c].cone_count < 0 || desc.constraints[c].cone_count > desc.max_cones)
			return "constraint cone_count exceeds max_cones";
		if (!(p.bone_flags[b] & BF_IN_LIST)) continue;
		if (p.bone_cons[b] < 0) {
			p.bone_cons[b] = (int)p.cons_bone.size();
			p.cons_bone.push_back(b);
			p.cons_ncones.push_back(desc.constraints[c].cone_count);
		} else {
			p.cons_ncones[p.bone_cons[b]] = desc.constraints[c].cone_count; // later constraint replaces
		}
		p.cons_order.push_back(c);
		p.cons_order_slot.push_back(p.bone_cons[b]);
		p.cons_order_ncones.push_back(desc.constraints[c].cone_count);
		if (p.bone_ik_parent[b] >= 0) p.bone_flags[b] |= BF_ORIENT | BF_AXIAL;
	}
	p.NC = (int)p.cons_bone.size();
	// Segment heights (for sibling-level scheduling) and Euler-tour ranges.
	p.seg_height.assign(p.NS, 0);
	for (int i = 0; i < p.NS; i++)
		for (int c : p.seg_children[i]) p.seg_height[i] = std::max(p.seg_height[i], p.seg_height[c] + 1);
	p.seg_hbase.assign(p.NS, 0); // laid out by build_schedule
	p.seg_tin.assign(p.NS, 0);
	p.seg_tout.assign(p.NS, 0);
	for (int i = 0; i < p.NS; i++) { // post-order: subtree of i = [tin, i]
		int lo = i;
		for (int c : p.seg_children[i]) lo = std::min(lo, p.seg_tin[c]);
		p.seg_tin[i] = lo;
		p.seg_tout[i] = i;
	}
	// constraint_mode node caches (cmode.h): pre-order positions over the pose-node forest of
	// the list bones, so a propagation (IKNode3D::_propagate_transform_changed) marks a range.
	p.cm_pre.assign(B, -1);
	p.cm_sub.assign(B, 0);
	p.cm_maxd = 1;
	{
		std::vector<std::vector<int>> pk(B);
		std::vector<int> roots_in_list;
		for (int b : p.bone_list) {
			const int pp = p.bone_pose_parent[b];
			if (pp >= 0) pk[pp].push_back(b);
			else roots_in_list.push_back(b);
		}
		int pos = 0;
		std::vector<std::pair<int, int>> stack; // (bone, depth); a negative bone closes -(b+1)
		for (int r : roots_in_list) {
			stack.push_back({r, 0});
			while (!stack.empty()) {
				auto [b, d] = stack.back();
				stack.pop_back();
				if (b < 0) {
					p.cm_sub[-b - 1] = pos - p.cm_pre[-b - 1];
					continue;
				}
				p.cm_pre[b] = pos++;
				p.cm_maxd = std::max(p.cm_maxd, d + 1);
				stack.push_back({-b - 1, d});
				for (size_t k = pk[b].size(); k-- > 0;) stack.push_back({pk[b][k], d + 1});
			}
		}
		p.cm_npos = pos;
	}
	return "";
}


// ---------------------------------------------------------------------------------------
// GPU-side topology build (topo.h): the host half
// ---------------------------------------------------------------------------------------
static double damp_cosine(float d) {
	double dampening = (double)(float)(double)d; // float -> double -> float p_dampening -> double
	return std::cos(dampening / 2.0);
}
void topology_damp_cosines(const mbik_skeleton_desc &desc, const mbik_config &cfg, std::vector<double> &bone_chd,
		double &root_chd) {
	bone_chd.assign(std::max(1, desc.bone_count), 0.0);
	for (int b = 0; b < desc.bone_count; b++) { // build_topology's damping rule, per bone
		float def = cfg.default_damp, d = def;
		if (b < cfg.bone_damp_count && cfg.bone_damp) d = cfg.bone_damp[b];
		if (def < d) d = def;
		bone_chd[b] = damp_cosine(d);
	}
	root_chd = damp_cosine((float)gd::PI);
}

std::string assemble_topology(const TopoOut &o, const mbik_skeleton_desc &desc, const mbik_config &cfg, HostPlan &p) {
	const int32_t *cnt = o.count;
	if (cnt[TC_ERR]) return topo_error(cnt[TC_ERR]);
	const int B = desc.bone_count, P = desc.pin_count;
	const int NS = cnt[TC_NS];
	auto v = [](const auto *a, int n) { return std::vector<std::remove_const_t<std::remove_pointer_t<decltype(a)>>>(a, a + n); };
	p.B = B;
	p.P = P;
	p.max_cones = std::max(1, desc.max_cones);
	p.iterations = cfg.iterations_per_frame;
	p.constraint_mode = cfg.constraint_mode;
	p.stabilization_passes = cfg.stabilization_passes;
	p.parents.assign(desc.parents, desc.parents + B);
	p.bone_depth = v(o.bone_depth, B);
	p.bone_pin = v(o.bone_pin, B);
	p.eff_bone.resize(P);
	p.eff_prio.resize(3 * P);
	for (int i = 0; i < P; i++) {
		p.eff_bone[i] = desc.pins[i].bone;
		for (int a = 0; a < 3; a++) p.eff_prio[3 * i + a] = desc.pins[i].direction_priorities[a];
	}
	p.bone_ik_parent = v(o.bone_ik_parent, B);
	p.NS = NS;
	p.seg_root = v(o.seg_root, NS);
	p.seg_tip = v(o.seg_tip, NS);
	p.seg_parent = v(o.seg_parent, NS);
	p.seg_children.assign(NS, {});
	for (int i = 0; i < NS; i++) p.seg_children[i] = v(o.seg_children + o.seg_child_off[i], o.seg_child_off[i + 1] - o.seg_child_off[i]);
	p.seg_flags = v(o.seg_flags, NS);
	p.seg_bone_off = v(o.seg_bone_off, NS + 1);
	p.seg_bones = v(o.seg_bones, cnt[TC_NLIST]);
	p.bone_list = v(o.bone_list, cnt[TC_NLIST]);
	p.roots = v(o.roots, cnt[TC_NROOTS]);
	p.bone_pose_parent = v(o.bone_pose_parent, B);
	p.seg_eff_off = v(o.seg_eff_off, NS + 1);
	p.seg_effs = v(o.seg_effs, cnt[TC_NSEGEFF]);
	p.seg_eff_hoff = v(o.seg_eff_hoff, cnt[TC_NSEGEFF]);
	p.seg_hw_off = v(o.seg_hw_off, NS);
	p.seg_hw = v(o.seg_hw, cnt[TC_NHW]);
	p.seg_nh = v(o.seg_nh, NS);
	p.max_headings = cnt[TC_MAXH];
	p.seg_wsum2 = v(o.seg_wsum2, NS);
	p.seg_cos_half_damp = v(o.seg_cos_half_damp, cnt[TC_NLIST]);
	p.eff_parent_bone = v(o.eff_parent_bone, P);
	p.eff_path_off = v(o.eff_path_off, P + 1);
	p.eff_path = v(o.eff_path, cnt[TC_NPATH]);
	p.bone_flags = v(o.bone_flags, B);
	p.bone_child_eff_off = v(o.bone_child_eff_off, B + 1);
	p.bone_child_effs = v(o.bone_child_effs, cnt[TC_NCHILDEFF]);
	p.bone_cons = v(o.bone_cons, B);
	p.NC = cnt[TC_NC];
	p.cons_bone = v(o.cons_bone, p.NC);
	p.cons_ncones = v(o.cons_ncones, p.NC);
	p.cons_order = v(o.cons_order, cnt[TC_NCONSORD]);
	p.cons_order_slot = v(o.cons_order_slot, cnt[TC_NCONSORD]);
	p.cons_order_ncones = v(o.cons_order_ncones, cnt[TC_NCONSORD]);
	p.desc_constraint_count = desc.constraint_count;
	p.seg_height = v(o.seg_height, NS);
	p.seg_hbase.assign(NS, 0); // laid out by build_schedule
	p.seg_tin = v(o.seg_tin, NS);
	p.seg_tout = v(o.seg_tout, NS);
	p.cm_pre = v(o.cm_pre, B);
	p.cm_sub = v(o.cm_sub, B);
	p.cm_maxd = cnt[TC_CM_MAXD];
	p.cm_npos = cnt[TC_CM_NPOS];
	return "";
}

int compare_topology(const HostPlan &a, const HostPlan &b, std::string *first) {
	int n = 0;
	auto note = [&](bool same, const char *name) {
		if (same) return;
		if (n++ == 0 && first) *first = name;
	};
	auto dbl_eq = [](const std::vector<double> &x, const std::vector<double> &y) {
		return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), x.size() * sizeof(double)) == 0);
	};
	auto flt_eq = [](const std::vector<float> &x, const std::vector<float> &y) {
		return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), x.size() * sizeof(float)) == 0);
	};
#define MBIK_CMP(f) note(a.f == b.f, #f);
	MBIK_CMP(B) MBIK_CMP(P) MBIK_CMP(NS) MBIK_CMP(NC) MBIK_CMP(max_cones) MBIK_CMP(iterations) MBIK_CMP(constraint_mode)
	MBIK_CMP(stabilization_passes) MBIK_CMP(parents) MBIK_CMP(bone_pose_parent) MBIK_CMP(bone_ik_parent) MBIK_CMP(bone_depth)
	MBIK_CMP(bone_flags) MBIK_CMP(bone_pin) MBIK_CMP(bone_cons) MBIK_CMP(bone_list) MBIK_CMP(bone_child_eff_off)
	MBIK_CMP(bone_child_effs) MBIK_CMP(seg_root) MBIK_CMP(seg_tip) MBIK_CMP(seg_parent) MBIK_CMP(seg_children)
	MBIK_CMP(seg_bone_off) MBIK_CMP(seg_bones) MBIK_CMP(seg_eff_off) MBIK_CMP(seg_effs) MBIK_CMP(seg_eff_hoff) MBIK_CMP(seg_nh)
	MBIK_CMP(seg_flags) MBIK_CMP(seg_hw_off) MBIK_CMP(seg_height) MBIK_CMP(seg_tin) MBIK_CMP(seg_tout) MBIK_CMP(roots)
	MBIK_CMP(eff_bone) MBIK_CMP(eff_parent_bone) MBIK_CMP(eff_path_off) MBIK_CMP(eff_path) MBIK_CMP(eff_prio)
	MBIK_CMP(cons_bone) MBIK_CMP(cons_ncones) MBIK_CMP(cons_order) MBIK_CMP(cons_order_slot) MBIK_CMP(cons_order_ncones)
	MBIK_CMP(desc_constraint_count) MBIK_CMP(max_headings) MBIK_CMP(cm_pre) MBIK_CMP(cm_sub) MBIK_CMP(cm_maxd) MBIK_CMP(cm_npos)
#undef MBIK_CMP
	note(dbl_eq(a.seg_hw, b.seg_hw), "seg_hw");
	note(dbl_eq(a.seg_cos_half_damp, b.seg_cos_half_damp), "seg_cos_half_damp");
	note(flt_eq(a.seg_wsum2, b.seg_wsum2), "seg_wsum2");
	return n;
}

// ---------------------------------------------------------------------------------------
// Per-skeleton setup data
// ---------------------------------------------------------------------------------------
void setup_tables(HostPlan &p) {
	const int B = p.B;
	std::vector<std::vector<int>> kids(B);
	for (int b = 0; b < B; b++)
		if (p.parents[b] >= 0) kids[p.parents[b]].push_back(b);
	p.setup_topo.clear();
	std::vector<int> stack;
	for (int b = B; b-- > 0;)
		if (p.parents[b] < 0) stack.push_back(b);
	while (!stack.empty()) {
		int b = stack.back();
		stack.pop_back();
		p.setup_topo.push_back(b);
		for (size_t k = kids[b].size(); k-- > 0;) stack.push_back(kids[b][k]);
	}
	p.ik_child_off.assign(1, 0);
	p.ik_children.clear();
	for (int b = 0; b < B; b++) {
		for (int c = 0; c < B; c++)
			if (p.bone_ik_parent[c] == b) p.ik_children.push_back(c);
		p.ik_child_off.push_back((int)p.ik_children.size());
	}
}

SetupView setup_view(const HostPlan &p, int32_t n, int32_t max_cones_in) {
	SetupView v;
	v.B = p.B;
	v.NC = p.NC;
	v.N = n;
	v.max_cones_in = max_cones_in;
	v.desc_constraint_count = p.desc_constraint_count;
	v.libm = p.libm_variant;
	v.cfs = p.cf_stride();
	v.cds = p.cd_stride();
	v.n_topo = (int)p.setup_topo.size();
	v.n_list = (int)p.bone_list.size();
	v.n_cons_order = (int)p.cons_order.size();
	v.topo = p.setup_topo.data();
	v.bone_list = p.bone_list.data();
	v.bone_flags = p.bone_flags.data();
	v.bone_pose_parent = p.bone_pose_parent.data();
	v.bone_ik_parent = p.bone_ik_parent.data();
	v.ik_child_off = p.ik_child_off.data();
	v.ik_children = p.ik_children.data();
	v.cons_order = p.cons_order.data();
	v.cons_order_slot = p.cons_order_slot.data();
	v.cons_order_ncones = p.cons_order_ncones.data();
	v.cons_bone = p.cons_bone.data();
	return v;
}

std::string build_skeletons(HostPlan &p, int32_t n, const float *setup_pose, const float *cones, const float *twist,
		int32_t max_cones_in) {
	const int B = p.B, NC = p.NC;
	if (n <= 0 || !setup_pose) return "n_skeletons must be > 0 and setup_pose non-null";
	if (NC > 0 && (!cones || !twist)) return "cones/twist required when constraints exist";
	for (int c : p.cons_order_ncones)
		if (c > max_cones_in) return "a constraint has more cones than max_cones";
	p.N = n;
	const size_t N = (size_t)n;
	p.D.assign((size_t)B * 9 * N, 0.0f);
	p.CF.assign((size_t)NC * p.cf_stride() * N, 0.0f);
	p.CD.assign((size_t)NC * p.cd_stride() * N, 0.0);
	setup_tables(p);
	p.setup_max_cones = std::max(1, max_cones_in);
	const SetupView v = setup_view(p, n, max_cones_in);
	// Skeletons split across host threads; each writes only its own SoA column s.
	auto setup_range = [&](int s0, int s1) {
		std::vector<char> buf(setup_scratch_bytes(B, NC, std::max(1, max_cones_in)));
		const SetupScratch w = setup_scratch_at(buf.data(), B, NC, std::max(1, max_cones_in));
		for (int s = s0; s < s1; s++)
			setup_skeleton(v, s, s, setup_pose + (size_t)s * B * 10, cones, twist, w, p.D.data(), p.CF.data(), p.CD.data());
	};
	const int hw = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
	const int nthreads = (int)std::min<int64_t>(hw, std::max<int64_t>(1, (int64_t)n / 64));
	if (nthreads <= 1) {
		setup_range(0, n);
	} else {
		std::vector<std::thread> pool;
		for (int t = 0; t < nthreads; t++) {
			const int s0 = (int)((int64_t)n * t / nthreads), s1 = (int)((int64_t)n * (t + 1) / nthreads);
			pool.emplace_back(setup_range, s0, s1);
		}
		for (auto &th : pool) th.join();
	}
	return "";
}

// ---------------------------------------------------------------------------------------
// Launch shape + sibling-level schedule
// ---------------------------------------------------------------------------------------
int32_t lds_floats_per_skeleton(const HostPlan &p) {
	const int32_t all = state_floats_per_skeleton(p);
	return p.state_hbm == 2 ? 0 : (p.state_hbm == 1 ? all - p.B * 12 : all);
}
// The whole per-skeleton state: L, checkpoint globals, targets, stale caches, staging, stabilization.
int32_t state_floats_per_skeleton(const HostPlan &p) {
	return p.B * 12 + p.n_gck * 12 + p.P * 25 + p.hs_floats + (p.stabilization_passes > 0 ? p.P * 10 : 0);
}

// Upper bound of the LDS bytes taken by the topology blob (host_plan.cpp: upload_topology).
int64_t topology_bytes(const HostPlan &p) {
	int64_t w = 4 * (int64_t)p.sched.size() + 4;
	auto ints = [&](size_t n) { w += (int64_t)std::max<size_t>(n, 1) + 1; };
	// the tables MBIK_TOPO_TABLES lists (kernels.h), in its order
	ints(p.bone_pose_parent.size()); ints(p.bone_flags.size()); ints(p.bone_pin.size());
	ints(p.bone_cons.size()); ints(p.bone_child_effs.size());
	ints(p.seg_bone_off.size()); ints(p.seg_bones.size()); ints(p.seg_eff_off.size()); ints(p.seg_effs.size());
	ints(p.seg_eff_hoff.size()); ints(p.seg_nh.size()); ints(p.seg_flags.size()); ints(p.seg_hw_off.size());
	ints(p.seg_wsum2.size()); ints(p.seg_hbase.size()); ints(p.B);
	ints(p.eff_bone.size()); ints(p.eff_path_off.size()); ints(p.eff_path.size()); ints(p.eff_prio.size());
	ints(p.cons_ncones.size()); ints(2 * p.seg_hw.size()); ints(2 * p.seg_cos_half_damp.size());
	ints(4 * p.seg_bones.size() + 3); // step_rec, 16-byte aligned
	ints(p.seg_effs.size() + 1);      // seg_eff_lcp
	ints(p.seg_effs.size() + 1);      // seg_eff_grp
	return (w + 4) * 4;
}

static int ceil_log2(int v) {
	int l = 0;
	while ((1 << l) < v) l++;
	return l;
}

// constraint_mode, wave roles: the split of a multi-effector segment's effector reads over its
// group of m waves (cmode.h mbik_cmode_kernel_rw).  The reference reads the effectors in order,
// each read cleaning the dirty pose chain above its effector.  All of the segment's effector
// paths from the root share a trunk down to the deepest common bone T (path length L).  Once T is
// clean, a read never walks above T, so two effectors may be read concurrently on separate waves
// if their paths share nothing below T (lcp(a, b) <= L); effectors that share more (transitively)
// form a cluster that one wave reads in the reference's order.  Clusters go to waves longest
// first.  A recomputed node's value does not depend on which read recomputes it (nothing above
// the reads changes during them), so the caches end as after the sequential reads.
// seg_eff_grp[i]: the wave of effector i's cluster (bits 0-3); the segment's first entry also
// holds T + 1 (bits 4 and up).  False (no split) with fewer than two clusters.
static bool cm_split_groups(HostPlan &p, int sg, int m) {
	const int e0 = p.seg_eff_off[sg], e1 = p.seg_eff_off[sg + 1], n = e1 - e0;
	auto plen = [&](int a) { const int e = p.seg_effs[a]; return p.eff_path_off[e + 1] - p.eff_path_off[e]; };
	auto lcp = [&](int a, int b) {
		const int ea = p.seg_effs[a], eb = p.seg_effs[b];
		const int la = plen(a), lb = plen(b);
		int l = 0;
		while (l < la && l < lb && p.eff_path[p.eff_path_off[ea] + l] == p.eff_path[p.eff_path_off[eb] + l]) l++;
		return l;
	};
	if (n < 2 || n > 256 || m > 16) return false; // (the pairwise test is quadratic; such segments run on one wave)
	int L = plen(e0);
	for (int a = 1; a < n; a++) L = std::min(L, lcp(e0, e0 + a));
	if (L < 1) return false;
	std::vector<int> par(n); // clusters: union over the pairs that share a node below T
	for (int i = 0; i < n; i++) par[i] = i;
	auto find = [&](int x) {
		while (par[x] != x) x = par[x] = par[par[x]];
		return x;
	};
	for (int a = 0; a < n; a++)
		for (int b = a + 1; b < n; b++)
			if (lcp(e0 + a, e0 + b) > L) par[find(b)] = find(a);
	std::vector<int> roots;
	std::vector<int64_t> cost(n, 0);
	for (int a = 0; a < n; a++) {
		const int r = find(a);
		if (cost[r] == 0) roots.push_back(r);
		cost[r] += std::max(1, plen(e0 + a) - L); // the nodes below T
	}
	if ((int)roots.size() < 2) return false;
	std::stable_sort(roots.begin(), roots.end(), [&](int x, int y) { return cost[x] > cost[y]; });
	std::vector<int64_t> load(m, 0);
	std::vector<int> wave(n, 0);
	for (int r : roots) {
		int w = 0;
		for (int q = 1; q < m; q++)
			if (load[q] < load[w]) w = q;
		wave[r] = w;
		load[w] += cost[r];
	}
	for (int a = 0; a < n; a++) p.seg_eff_grp[e0 + a] = wave[find(a)];
	const int T = p.eff_path[p.eff_path_off[p.seg_effs[e0]] + L - 1];
	p.seg_eff_grp[e0] |= (T + 1) << 4;
	return true;
}

void build_schedule(HostPlan &p, int32_t lanes, int64_t nlaunch, int32_t spw_override, int32_t interval_override,
		BlocksPerCU blocks_per_cu, void *ctx, int cus) {
	p.seg_eff_lcp.assign(p.seg_effs.size() + 1, 0);
	p.seg_eff_grp.assign(p.seg_effs.size() + 1, 0);
	for (int sg = 0; sg < p.NS; sg++)
		for (int i = p.seg_eff_off[sg] + 1; i < p.seg_eff_off[sg + 1]; i++) {
			const int a = p.seg_effs[i - 1], b = p.seg_effs[i];
			const int la = p.eff_path_off[a + 1] - p.eff_path_off[a], lb = p.eff_path_off[b + 1] - p.eff_path_off[b];
			int l = 0;
			while (l < la && l < lb && p.eff_path[p.eff_path_off[a] + l] == p.eff_path[p.eff_path_off[b] + l]) l++;
			p.seg_eff_lcp[i] = l;
		}
	int maxh = 0;
	for (int i = 0; i < p.NS; i++) maxh = std::max(maxh, p.seg_height[i]);
	std::vector<std::vector<int>> lev(maxh + 1);
	for (int i = 0; i < p.NS; i++) lev[p.seg_height[i]].push_back(i);
	int widest = 1;
	for (auto &l : lev) widest = std::max(widest, (int)l.size());
	int K;
	if (lanes > 0) {
		K = 1 << ceil_log2(lanes);
	} else {
		// One lane per segment of the widest sibling level.  The solve is a serial chain
		// per skeleton (latency-bound), so lanes beyond the sibling parallelism only add
		// redundant work: measured on MI355X (tools/sweep.py) the widest
		// level's width is the fastest lane count for C2-C5, also where it leaves the chip
		// with fewer than one wave per SIMD.
		K = std::min(64, 1 << ceil_log2(widest));
	}
	K = std::max(1, std::min(64, K));
	p.K = K;
	p.log2K = ceil_log2(K);
	p.sched.clear();
	p.nrows = 0;
	p.has_xs = false;
	p.has_chain = false;
	// A level with more segments than lanes runs in several rows of single-lane tasks.  Its
	// segments are independent, so the rows are packed instead: each lane gets a sequence of
	// segments (longest processing time first, by an estimate of each segment's step work:
	// per bone-step its effectors' path walks plus a constant), and the kernel runs a lane's
	// sequence back to back with no barrier between the rows (SCHED_CHAIN).  A lane then waits
	// for the most loaded lane of the level, not for the longest segment of every row.
	std::vector<int> depth(p.B, 0);
	for (size_t e = 0; e + 1 < p.eff_path_off.size(); e++)
		for (int i = p.eff_path_off[e]; i < p.eff_path_off[e + 1]; i++) depth[p.eff_path[i]] = i - p.eff_path_off[e];
	auto seg_cost = [&](int sg) {
		int64_t c = 0;
		for (int k = p.seg_bone_off[sg]; k < p.seg_bone_off[sg + 1]; k++) {
			c += 24;
			for (int i = p.seg_eff_off[sg]; i < p.seg_eff_off[sg + 1]; i++) {
				const int e = p.seg_effs[i];
				c += std::max(0, p.eff_path_off[e + 1] - p.eff_path_off[e] - 1 - depth[p.seg_bones[k]]);
			}
		}
		return c;
	};
	for (auto &l : lev) {
		// (constraint_mode keeps at most four pending chain cleanings per lane: cmode.h)
		if ((int)l.size() > K && (!p.constraint_mode || (int)l.size() <= 4 * K)) {
			std::vector<int> order(l);
			std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return seg_cost(a) > seg_cost(b); });
			std::vector<std::vector<int>> per(K);
			std::vector<int64_t> load(K, 0);
			// (eight wave roles put roles 2i and 2i + 1 on one SIMD, MBIK_RW_PERM: the SIMDs' loads
			// are balanced first, then the two roles' on each)
			const bool pair = MBIK_RW_PERM && p.wave_roles && !p.constraint_mode && K == 8;
			for (int sg : order) {
				int i = -1;
				if (pair) {
					int sm = 0;
					for (int q = 1; q < K / 2; q++)
						if (load[2 * q] + load[2 * q + 1] < load[2 * sm] + load[2 * sm + 1]) sm = q;
					i = load[2 * sm + 1] < load[2 * sm] ? 2 * sm + 1 : 2 * sm;
				} else {
					for (int q = 0; q < K; q++)
						if ((!p.constraint_mode || per[q].size() < 4) && (i < 0 || load[q] < load[i])) i = q;
				}
				per[i].push_back(sg);
				load[i] += seg_cost(sg);
			}
			size_t nr = 0;
			for (auto &v : per) nr = std::max(nr, v.size());
			for (size_t q = 0; q < nr; q++) {
				const int32_t ch = q > 0 ? SCHED_CHAIN : 0;
				std::vector<SchedTask> row(K, SchedTask{-1, 0, 1, ch});
				for (int i = 0; i < K; i++)
					if (q < per[i].size()) row[i] = SchedTask{per[i][q], 0, 1, ch};
				p.sched.insert(p.sched.end(), row.begin(), row.end());
				p.nrows++;
			}
			p.has_chain |= nr > 1;
			continue;
		}
		for (size_t start = 0; start < l.size(); start += K) {
			int cnt = (int)std::min<size_t>(K, l.size() - start);
			int m = K >> ceil_log2(cnt);
			bool cmsplit_row = false;
			if (p.wave_roles) {
				// Wave roles: each segment of the row on a group of m waves.  A segment of two or
				// more effectors is solved cooperatively (SCHED_XS): its waves split the effector path
				// walks and its first wave runs the rest of each bone-step once; a single-effector
				// segment runs on the group's first wave alone.  No wave repeats another's work.
				std::vector<SchedTask> row(K, SchedTask{-1, 0, 1, 0});
				bool coop = false;
				for (int i = 0; i < cnt; i++) {
					const int sg = l[start + i];
					const bool multi = p.seg_eff_off[sg + 1] - p.seg_eff_off[sg] >= 2;
					if (multi && m >= 2) {
						for (int j = 0; j < m; j++) row[i * m + j] = SchedTask{sg, j, m, SCHED_XS};
						coop = true;
					} else {
						row[i * m] = SchedTask{sg, 0, 1, 0};
					}
				}
				if (coop)
					for (auto &tk : row) tk.flags |= SCHED_COOP;
				p.sched.insert(p.sched.end(), row.begin(), row.end());
				p.nrows++;
				continue;
			}
			// without staging, the m lanes of a group each solve the whole segment (j 0 of 1):
			// identical work and identical stores, so no lane waits on another
			std::vector<SchedTask> row(K, SchedTask{-1, 0, 1, 0});
			for (int i = 0; i < cnt; i++) {
				const int sg = l[start + i];
				const bool multi = p.seg_eff_off[sg + 1] - p.seg_eff_off[sg] >= 2;
				const bool tr = (p.seg_flags[sg] & SF_TRANSLATE) != 0;
				const bool staged = p.staging == 1 || (p.staging == 2 && tr) || (p.staging == 3 && multi) || (p.staging == 5 && tr && multi);
				const bool solo = !p.constraint_mode && !staged;
				// staging 4 / 5: multi-effector segments not staged in memory split their effectors
				// over the group's lanes and exchange the headings lane to lane
				// (the two-waves-per-SIMD build is the one that serves them; one wave: solo)
				const bool xs = solo && multi && m >= 2 && (p.staging == 4 || p.staging == 5) && p.waves_per_simd == 2;
				// constraint_mode with wave roles: the group's waves split the step's effector reads when
				// into two or more clusters (cm_split_groups); else the group's first wave runs the segment alone
				const bool cms = p.constraint_mode && p.cm_roles && multi && m >= 2 && cm_split_groups(p, sg, m);
				cmsplit_row |= cms;
				for (int j = 0; j < m; j++)
					row[i * m + j] = xs ? SchedTask{sg, j, m, SCHED_XS}
										: (solo ? SchedTask{sg, 0, 1, 0} : SchedTask{sg, j, m, cms ? SCHED_CMSPLIT : 0});
				p.has_xs |= xs;
			}
			if (cmsplit_row)
				for (auto &tk : row) tk.flags |= SCHED_COOP;
			p.sched.insert(p.sched.end(), row.begin(), row.end());
			p.nrows++;
		}
	}
	// Staged-heading area (bone_step.h, segments solved by several lanes of a row): 12 floats per
	// heading plus 24 for the exchanged sums.  A translating split-exchange segment (staging 4 /
	// 5, state placement 2) keeps there instead the effector globals its lanes built in the centroid pass, 12
	// floats per lane and round, so that the sums pass rebuilds their headings without walking
	// the paths again.  The segments of one row run concurrently, so their areas are disjoint;
	// offsets restart at every row.
	p.seg_hbase.assign(p.NS, 0);
	p.hs_floats = 0;
	p.rw_xslots = 0;
	if (p.wave_roles) {
		// wave roles: a cooperative segment's effector globals go through LDS, one slot per
		// effector; the segments of a row run concurrently, so their slots are disjoint
		for (int r = 0; r < p.nrows; r++) {
			int used = 0;
			for (int l = 0; l < K; l++) {
				const SchedTask &tk = p.sched[(size_t)r * K + l];
				if (tk.seg < 0 || tk.j != 0 || !(tk.flags & SCHED_XS)) continue;
				p.seg_hbase[tk.seg] = used;
				used += p.seg_eff_off[tk.seg + 1] - p.seg_eff_off[tk.seg];
			}
			p.rw_xslots = std::max(p.rw_xslots, used);
		}
	}
	for (int r = 0; r < p.nrows && !p.wave_roles; r++) {
		int used = 0;
		for (int l = 0; l < K; l++) {
			const SchedTask &tk = p.sched[(size_t)r * K + l];
			if (tk.seg < 0 || tk.j != 0 || tk.m < 2 || p.seg_nh[tk.seg] < 2) continue;
			if (tk.flags & SCHED_XS) {
				// (only with the whole state in device memory: in LDS the area would cost residency)
				if (!(p.seg_flags[tk.seg] & SF_TRANSLATE) || p.state_hbm != 2) continue;
				const int ne = p.seg_eff_off[tk.seg + 1] - p.seg_eff_off[tk.seg];
				p.seg_hbase[tk.seg] = used;
				used += 12 * tk.m * ((ne + tk.m - 1) / tk.m);
				continue;
			}
			p.seg_hbase[tk.seg] = used;
			used += 12 * p.seg_nh[tk.seg] + 24;
		}
		p.hs_floats = std::max(p.hs_floats, used);
	}
	// Skeletons per block and the checkpoint interval of the iteration-start globals.  LDS
	// (160 KiB per CU) bounds how many skeletons a CU holds at once; a block's LDS is spw
	// skeletons plus one copy of the topology blob.  A launch that fits the chip at the full
	// 64 / K per wave with every global kept keeps that (a chain of skeletons is
	// latency-bound, so fewer waves of full width cost nothing).  A larger launch takes the
	// (interval, spw) with the most skeletons resident per CU, discounted by what sparser
	// checkpoints cost in recomputed products (per-wave cycles from tools/prof_phases.py on
	// MI355X: interval 2 ~1.5 %, no interior checkpoints 6-8 %; mbik_plan_autotune measures
	// instead of modelling).  Residency comes from the runtime's occupancy query (LDS
	// allocation granularity and the register budget: at most one wave per SIMD).
	const int64_t topo = topology_bytes(p);
	const int64_t kCUs = cus;
	auto set_interval = [&](int c) -> double {
		p.g_interval = c;
		p.bone_gslot.assign(p.B, -1);
		for (int sg = 0; sg < p.NS; sg++) {
			const int k0 = p.seg_bone_off[sg], k1 = p.seg_bone_off[sg + 1];
			for (int k = k0; k < k1; k++)
				if ((k1 - 1 - k) % c == 0) p.bone_gslot[p.seg_bones[k]] = 0;
			const int pp = p.bone_pose_parent[p.seg_bones[k1 - 1]];
			if (pp >= 0) p.bone_gslot[pp] = 0;
		}
		p.n_gck = 0;
		for (int b = 0; b < p.B; b++)
			if (p.bone_gslot[b] >= 0) p.bone_gslot[b] = p.n_gck++;
		p.seg_anchor.assign(p.seg_bones.size(), -1);
		int64_t extra = 0;
		for (int sg = 0; sg < p.NS; sg++) {
			const int k0 = p.seg_bone_off[sg], k1 = p.seg_bone_off[sg + 1];
			for (int k = k0; k < k1 - 1; k++) {
				int kc = k + 1;
				while (p.bone_gslot[p.seg_bones[kc]] < 0) kc++; // ends at the segment root
				p.seg_anchor[k] = kc;
				extra += kc - (k + 1);
			}
		}
		return p.seg_bones.empty() ? 0.0 : (double)extra / (double)p.seg_bones.size();
	};
	auto resident = [&](int spw) -> int64_t {
		const int64_t block = spw * (int64_t)(((lds_floats_per_skeleton(p) + 3) & ~3) * 4) + topo;
		if (block > 160 * 1024) return 0;
		const int64_t blocks = blocks_per_cu ? blocks_per_cu(ctx, block) : 160 * 1024 / block;
		return blocks * spw;
	};
	set_interval(interval_override > 0 ? interval_override : 1);
	int best = 64 / K;
	while (best > 1 && resident(best) == 0) best--;
	int best_c = interval_override > 0 ? interval_override : 1;
	if (p.wave_roles) {
		// wave roles: a lane per skeleton, 64 per block of K waves (fewer when pinned: partly
		// filled waves, more blocks for a small launch); the state is in device memory, so LDS
		// holds the topology, the non-finite flags and the cooperative rows' exchange
		best = spw_override > 0 ? std::min(64, spw_override) : 64;
	} else if (spw_override > 0) {
		best = std::min(spw_override, 64 / K);
		while (best > 1 && resident(best) == 0) best--;
	} else if (resident(best) * kCUs < nlaunch) {
		double best_score = -1.0;
		std::vector<int> cands = interval_override > 0 ? std::vector<int>{interval_override} : std::vector<int>{1, 2, 1 << 20};
		for (int c : cands) {
			set_interval(c);
			const double factor = c == 1 ? 1.0 : (c == 2 ? 0.985 : 0.92);
			for (int spw = 1; spw <= 64 / K; spw++) {
				const int64_t res = resident(spw);
				if (res == 0) continue;
				const int64_t blocks = res / spw;
				// more than ~4 single-wave blocks per CU share SIMDs (issue-bound)
				const double score = (double)res * factor * std::min(1.0, 4.0 / (double)blocks);
				if (score >= best_score) {
					best_score = score;
					best = spw;
					best_c = c;
				}
			}
		}
	}
	set_interval(best_c);
	p.step_rec.assign(4 * p.seg_bones.size(), 0);
	for (size_t k = 0; k < p.seg_bones.size(); k++) {
		const int b = p.seg_bones[k], pp = p.bone_pose_parent[b], kc = p.seg_anchor[k];
		const int pslot = pp >= 0 ? p.bone_gslot[kc < 0 ? pp : p.seg_bones[kc]] : -1;
		const int c0 = p.bone_child_eff_off[b], c1 = p.bone_child_eff_off[b + 1];
		int32_t *r = &p.step_rec[4 * k];
		r[0] = b | ((kc + 1) << 16);
		r[1] = (pslot + 1) | ((p.bone_cons[b] + 1) << 16);
		r[2] = p.bone_flags[b] | (pp != POSE_PARENT_NONE ? SR_HAS_POSE_PARENT : 0) | (pp >= 0 ? SR_PARENT_GLOBAL : 0) |
				((p.bone_depth[b] + 1) << 16);
		r[3] = c0 | ((c1 - c0) << 16);
	}
	p.spw = best;
	p.lds_block_bytes = best * (int64_t)(((lds_floats_per_skeleton(p) + 3) & ~3) * 4) + topo +
			(p.wave_roles ? 64 * 4 + (p.rw_xslots ? ((int64_t)p.P + p.rw_xslots) * 12 * 64 * 4 + rw_record_bytes(p) : 0) : 0);
}

int64_t rw_record_bytes(const HostPlan &p) {
	// K / 2 records, then K / 2 counters and the block's gave-up word (16-byte aligned)
	return p.wave_roles && p.rw_xslots ? (int64_t)(p.K / 2) * kRwRecF4 * 64 * 16 + ((p.K / 2 + 1) * 4 + 15) / 16 * 16 : 0;
}

} // namespace mbik
