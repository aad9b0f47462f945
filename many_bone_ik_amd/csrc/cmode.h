// constraint_mode (ManyBoneIK3D::constraint_mode, ik_bone_segment_3d.cpp:142): every bone-step
// skips the QCP fit and only applies the Kusudama swing and twist snaps.  Device code of
// k_cmode.hip (DevPlan and the device helpers from bone_step.h).
//
// Without the fit's set_global_pose nothing refreshes the IKNode3D tree as a whole, so the
// result depends on which cached globals are stale:
//   * rotate_local_with_global (the swing snap) dirties only the node it rotates
//     (ik_node_3d.cpp:56-67), leaving its subtree's caches clean but stale;
//   * set_transform (the twist snap, the stabilization restore and the frame's pose load)
//     propagates through the subtree only if the local transform changed (:69-75);
//   * get_global_transform recomputes a dirty node from its parent, and the parent only if
//     that is dirty too (:93-113);
//   * these caches outlive the frame.
// So this path keeps the reference's node caches themselves: per skeleton, the pose local
// and the cached globals of the pose, bone-direction, constraint-orientation and twist nodes
// in HBM (SoA [slot][12][N], persistent across mbik_solve calls), and one dirty bit per node
// in LDS for the launch (word-packed by pre-order position, so a propagation marks a range).
// Every node read goes through the same lazy recomputation, in the reference's order.
//
// Lanes: K per skeleton, sibling segments of one schedule row (plan.cpp build_schedule) on
// separate lanes, as in the default kernel.  Sibling segments touch disjoint subtrees, so a
// lane writes only nodes of its own segment root's subtree (its pre-order range).  A dirty
// chain that reaches above the segment root is recomputed privately (no write: every sibling
// would compute the same bits, since nothing above a row changes during it), and the cleaning
// the reference does at the first such read is applied after the row, one lane at a time.
// Dirty words are shared by the skeleton's lanes: updates are LDS atomics.

#pragma once
#include "solve_block.h"

namespace {

using mbik::CmodeState;
using mbik::kCmodeMaxWaves;
using mbik::kNodeTile;
using mbik::node_area_floats;
using mbik::node_at;

#ifndef MBIK_CM_GROUP
#define MBIK_CM_GROUP 2
#endif
constexpr int kChainGroup = MBIK_CM_GROUP; // dirty-chain nodes per load group (CmodeLane::pose_global)
constexpr unsigned kWaitVmAll = 0x0F70;       // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): gfx9 encoding

enum { CK_POSE = 0, CK_BDIR = 1, CK_COR = 2, CK_CTW = 3 };

// NB32: the node area and the setup tables are below 4 GiB (the usual case), so a node read is
// three 16-byte buffer loads off one 32-bit lane offset (the element offsets are immediates)
// and the setup tables are read with the solve kernel's 32-bit addressing (kTab32); else
// 64-bit addresses.
template <bool NB32>
struct CmodeLane {
	const DevPlan &t;
	const CmodeState &c;
	size_t s;             // absolute skeleton index (plan tables)
	float *node;          // this skeleton's node state: element f of slot k at node[k * 192 + (f / 4) * 64 + f % 4]
	int slots;            // node slots per skeleton (3 B + 2 NC)
	uint32_t *dl;         // this skeleton's dirty words: dl[(kind * W + w) * dls]
	int dls;              // their interleave (skeletons per block)
	int *stk;             // this lane's chain stack: stk[i * 64]
	const int *pre, *sub; // LDS copies
	int lo, hi;           // pre-order range this lane may write (its segment root's subtree)
	int *pend;            // pose node whose dirty chain this lane read privately (-1 none)
	__amdgpu_buffer_rsrc_t r; // NB32: the whole node area
	uint32_t nb;          // NB32: byte offset of this skeleton's slot 0, element 0
#ifdef MBIK_PROF
	uint64_t *pf;         // diagnostic counters (tools/prof_cmode.py): see mbik_cmode_kernel
	int prof_m = 1;       // the running step's lane-group size
#endif

	__device__ __forceinline__ X3 ld(int k) const {
		X3 x;
		float v[12];
		if constexpr (NB32) {
			const uint32_t o = nb + (uint32_t)k * (48u * kNodeTile);
#pragma unroll
			for (int f = 0; f < 12; f++)
				v[f] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, o + 16u * kNodeTile * (f >> 2) + 4u * (f & 3), 0, 0));
		} else {
			const float *p = node + (size_t)k * 12 * kNodeTile;
#pragma unroll
			for (int f = 0; f < 12; f++) v[f] = p[(f >> 2) * 4 * kNodeTile + (f & 3)];
		}
#pragma unroll
		for (int i = 0; i < 3; i++) x.b.r[i] = v3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
		x.o = v3(v[9], v[10], v[11]);
		return x;
	}
	__device__ __forceinline__ void st(int k, const X3 &x) const {
		const float v[12] = {x.b.r[0].x, x.b.r[0].y, x.b.r[0].z, x.b.r[1].x, x.b.r[1].y, x.b.r[1].z,
				x.b.r[2].x, x.b.r[2].y, x.b.r[2].z, x.o.x, x.o.y, x.o.z};
		if constexpr (NB32) {
			const uint32_t o = nb + (uint32_t)k * (48u * kNodeTile);
#pragma unroll
			for (int f = 0; f < 12; f++)
				__builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[f]), r, o + 16u * kNodeTile * (f >> 2) + 4u * (f & 3), 0, 0);
		} else {
			float *p = node + (size_t)k * 12 * kNodeTile;
#pragma unroll
			for (int f = 0; f < 12; f++) p[(f >> 2) * 4 * kNodeTile + (f & 3)] = v[f];
		}
	}
	__device__ __forceinline__ int LP(int b) const { return b; }
	__device__ __forceinline__ int GP(int b) const { return t.B + b; }
	__device__ __forceinline__ int GD(int b) const { return 2 * t.B + b; }
	__device__ __forceinline__ int GC(int slot_) const { return 3 * t.B + slot_; }
	__device__ __forceinline__ int GT(int slot_) const { return 3 * t.B + t.NC + slot_; }

	__device__ __forceinline__ uint32_t *word(int kind, int w) const { return dl + (kind * c.W + w) * dls; }
	__device__ __forceinline__ bool dirty(int kind, int b) const {
		const int p = pre[b];
		return (*word(kind, p >> 5) >> (p & 31)) & 1u;
	}
	__device__ __forceinline__ void set_clean(int kind, int b) const {
		const int p = pre[b];
		atomicAnd(word(kind, p >> 5), ~(1u << (p & 31)));
	}
	__device__ __forceinline__ void set_dirty(int kind, int b) const {
		const int p = pre[b];
		atomicOr(word(kind, p >> 5), 1u << (p & 31));
	}
	__device__ __forceinline__ void mark_range(int kind, int a0, int z0) const { // positions [a0, z0)
		for (int w = a0 >> 5; w <= ((z0 - 1) >> 5) && a0 < z0; w++) {
			const int a = max(a0, w * 32) - w * 32, z = min(z0, w * 32 + 32) - w * 32; // bits [a, z)
			const uint32_t m = (z == 32 ? ~0u : ((1u << z) - 1u)) & ~((1u << a) - 1u);
			atomicOr(word(kind, w), m);
		}
	}
	__device__ __forceinline__ bool owned(int b) const { return pre[b] >= lo && pre[b] < hi; }
	// IKNode3D::_propagate_transform_changed on bone b's pose node (ik_node_3d.cpp:33-49): the
	// node, its bone-direction child, and every node of the list bones below it.
	__device__ __forceinline__ void propagate(int b) const {
		const int lo = pre[b], hi = lo + sub[b];
		mark_range(CK_POSE, lo, hi);
		mark_range(CK_BDIR, lo, hi);
		mark_range(CK_COR, lo + 1, hi);
		mark_range(CK_CTW, lo + 1, hi);
	}

	// get_global_transform of bone b's pose node (ik_node_3d.cpp:93-113): the dirty chain
	// above it is recomputed top-down from its first clean ancestor.
	// Nodes outside the lane's range are computed but not written; the lowest such node is
	// recorded in *pend for the after-row cleaning.
	// dq (bdir_global): also loads bone b's bone-direction basis D, with the chain's last group.
	__device__ __forceinline__ X3 pose_global(int b, B3 *dq = nullptr) const {
		if (!dirty(CK_POSE, b)) {
			if (dq) *dq = ld_soa_basis<NB32 ? kTab32 : kTab64>(t, t.D, b, 9, 0, s);
			return ld(GP(b));
		}
		MBIK_PROF_T(q0);
		int n = 0, x = b, pp;
		for (;;) {
			stk[64 * n++] = x;
			pp = t.bone_pose_parent[x];
			if (pp < 0 || !dirty(CK_POSE, pp)) break;
			x = pp;
		}
		// Top-down over stk[n-1] (= x) .. stk[0] (= b), kChainGroup nodes at a time: a group's
		// locals (and, first, the clean parent's global) are loaded together, then its products
		// run and its globals are stored.  gfx9's vmcnt counts stores as well as loads, and with
		// both pending a wait can only be for all of them: a load issued after a store waits for
		// that store's write to complete (~3,000 cycles on a busy chip).  Grouped, a chain pays
		// that round trip once per group instead of once per node.  The products and their order
		// are unchanged.
		X3 G;
		for (int i = n - 1; i >= 0; i -= kChainGroup) {
			X3 Lq[kChainGroup];
#pragma unroll
			for (int u = 0; u < kChainGroup; u++)
				if (i - u >= 0) Lq[u] = ld(LP(stk[64 * (i - u)]));
			X3 Gp;
			if (i == n - 1 && pp >= 0) Gp = ld(GP(pp));
			if (dq && i < kChainGroup) *dq = ld_soa_basis<NB32 ? kTab32 : kTab64>(t, t.D, b, 9, 0, s);
			// every load of the group lands before the group's first store (else the compiler's
			// wait for a later local, now behind a store, would be for that store too)
			__builtin_amdgcn_s_waitcnt(kWaitVmAll);
#pragma unroll
			for (int u = 0; u < kChainGroup; u++) {
				if (i - u < 0) break;
				if (u == 0 && i == n - 1)
					G = pp >= 0 ? Gp * Lq[0] : (pp == mbik::POSE_PARENT_ORIGIN ? xid() * Lq[0] : Lq[0]);
				else
					G = G * Lq[u];
				keep(stk[64 * (i - u)], G);
			}
		}
#ifdef MBIK_PROF
		MBIK_PROF_T(q1);
		pf[4] += q1 - q0;
		pf[5] += n;
		pf[6] += 1;
		if (prof_m > 1) pf[11] += n;
#endif
		return G;
	}
	__device__ __forceinline__ void keep(int x, const X3 &G) const {
		if (owned(x)) {
			st(GP(x), G);
			set_clean(CK_POSE, x);
		} else {
			*pend = x; // visited top-down: ends as the lowest outside node (the segment root's parent)
#ifdef MBIK_PROF
			pf[10] += 1;
#endif
		}
	}
	// IKBone3D::get_bone_direction_global_pose (ik_bone_3d.cpp:157-159): local = (D, 0).
	__device__ __forceinline__ X3 bdir_global(int b) const {
		if (!dirty(CK_BDIR, b)) return ld(GD(b));
#ifdef MBIK_PROF
		pf[9] += 1;
#endif
		B3 D;
		const X3 Gp = pose_global(b, &D);
		const X3 G = Gp * X3{D, v3(0, 0, 0)};
		st(GD(b), G);
		set_clean(CK_BDIR, b);
		return G;
	}
	// A read whose value is not used (the heading builds' reads in a plain constraint_mode
	// step only matter for the caches they refresh): the recomputation of a dirty node, no
	// load of a clean one.
	__device__ __forceinline__ void bdir_touch(int b) const {
		if (dirty(CK_BDIR, b)) (void)bdir_global(b);
	}
	// constraint_orientation_transform: parent = the parent bone's pose node; its local stays
	// the identity (only set_global_pose copies an origin into it, ik_bone_3d.cpp:145-151).
	__device__ __forceinline__ X3 orient_global(int b) const {
		const int k = GC(t.bone_cons[b]);
		if (!dirty(CK_COR, b)) return ld(k);
		const X3 G = pose_global(t.bone_pose_parent[b]) * xid();
		st(k, G);
		set_clean(CK_COR, b);
		return G;
	}
	// constraint_twist_transform: local = (twist frame basis, 0) (ik_kusudama_3d.cpp:37-89).
	__device__ __forceinline__ X3 twist_global(int b) const {
		const int slot_ = t.bone_cons[b];
		const int k = GT(slot_);
		if (!dirty(CK_CTW, b)) return ld(k);
		const X3 G = pose_global(t.bone_pose_parent[b]) *
				X3{ld_soa_basis<NB32 ? kTab32 : kTab64>(t, t.CF, slot_, t.cf_stride, mbik::CF_TWIST_T, s), v3(0, 0, 0)};
		st(k, G);
		set_clean(CK_CTW, b);
		return G;
	}
};

// One constraint_mode bone-step: _qcp_solver's and _set_optimal_rotation's heading builds
// (ik_bone_segment_3d.cpp:230-231,135,141: only their node reads matter, plus the target
// headings' origins for stabilization), the swing snap (ik_kusudama_3d.cpp:347-376), the
// twist snap (:117-132) and, for stabilized root segments, the MSD accept / restore loop
// (ik_bone_segment_3d.cpp:163-180).  OE: the lane's target-heading origins, OE[64 * (3e + i)].
// j / m: this lane's index in the segment's lane group and the group's size.  Every lane of the
// group runs the step (the same reads, products and stores of the same bits); the heading
// builds' node reads are split over the group: lane j reads effectors e0+j, e0+j+m, ...  Those
// reads only fill caches -- a dirty node is recomputed top-down from its first clean ancestor,
// nothing they touch changes a local -- so which lane fills a node, and in which order, leaves
// the same cached bits and dirty words as the reference's sequential loop; lanes that share a
// chain recompute it alike.  Stabilized segments keep every read on every lane: the MSD loop
// needs each effector's target-heading origin on the lane that sums them.
// reads false (wave roles, SCHED_CMSPLIT): the effector reads were made by the segment's waves
// before (cmode_coop_step); the step starts at the solved bone's own read.
template <bool STAB, bool NB32>
__device__ __forceinline__ void cmode_step(const CmodeLane<NB32> &C, int seg, int k, int j, int m, const float *tg, float *OE, double &prev_dev,
		bool reads = true) {
	const int ls = 64;
	const DevPlan &t = C.t;
	const int b = t.seg_bones[k];
	const int e0 = t.seg_eff_off[seg], e1 = t.seg_eff_off[seg + 1];
	const bool stab = STAB && (t.seg_flags[seg] & mbik::SF_STAB) != 0;
	const int flags = t.bone_flags[b];
#ifdef MBIK_PROF
	uint64_t *pf = C.pf;
	const_cast<CmodeLane<NB32> &>(C).prof_m = m;
#endif
	MBIK_PROF_T(c0);
	const int i0 = stab ? e0 : e0 + j, di = stab ? 1 : m;
	for (int i = reads ? i0 : e1; i < e1; i += di) {
		const int e = t.seg_effs[i];
		if (stab) {
			const X3 E = C.bdir_global(t.eff_bone[e]);
			OE[ls * (3 * e)] = E.o.x;
			OE[ls * (3 * e + 1)] = E.o.y;
			OE[ls * (3 * e + 2)] = E.o.z;
		} else {
			C.bdir_touch(t.eff_bone[e]);
		}
	}
	if (e1 > e0) C.bdir_touch(b);
	const X3 prev = C.ld(C.LP(b));
	for (int attempt = 0;; attempt++) {
		if (attempt > 0 && e1 > e0) { // the retry's tip headings (:141)
			for (int i = e0; i < e1; i++) C.bdir_touch(t.eff_bone[t.seg_effs[i]]);
			C.bdir_touch(b);
		}
		MBIK_PROF_T(c1);
		MBIK_PROF_ADD(0, c0, c1);
		if (flags & mbik::BF_ORIENT) {
			const int slot_ = t.bone_cons[b];
			const X3 Gc = C.orient_global(b);
			const X3 Gd = C.bdir_global(b);
			const V3 p1 = Gc.o;
			const V3 p2 = xform(Gd, v3(0.0f, 1.0f, 0.0f));
			const V3 tip = xform(affine_inverse(Gc), p2);
			double in_bounds = 1.0;
			const V3 inl = local_point_in_limits<NB32 ? kTab32 : kTab64>(t, slot_, C.s, tip, in_bounds);
			if (in_bounds < 0) {
				const V3 cp2 = xform(Gc, inl);
				const Q rect = arc(p2 - p1, cp2 - p1);
				// rotate_local_with_global (ik_node_3d.cpp:56-67): no propagation
				const B3 Pb = C.pose_global(t.bone_pose_parent[b]).b;
				X3 Lb = C.ld(C.LP(b));
				Lb.b = ((inverse(Pb) * from_quat(rect)) * Pb) * Lb.b;
				C.st(C.LP(b), Lb);
				C.set_dirty(CK_POSE, b);
			}
		}
		MBIK_PROF_T(c2);
		MBIK_PROF_ADD(1, c1, c2);
		if (flags & mbik::BF_AXIAL) {
			const int slot_ = t.bone_cons[b];
			const int cs = t.cf_stride;
			const X3 Gt = C.twist_global(b);
			const X3 Gs = C.pose_global(b);
			const B3 pgi = inverse(C.pose_global(t.bone_pose_parent[b]).b);
			constexpr int TA = NB32 ? kTab32 : kTab64;
			const Q tcr = q4(soa<TA>(t, t.CF, slot_, cs, mbik::CF_TWIST_Q, C.s), soa<TA>(t, t.CF, slot_, cs, mbik::CF_TWIST_Q + 1, C.s),
					soa<TA>(t, t.CF, slot_, cs, mbik::CF_TWIST_Q + 2, C.s), soa<TA>(t, t.CF, slot_, cs, mbik::CF_TWIST_Q + 3, C.s));
			const float half_cos = soa<TA>(t, t.CF, slot_, cs, mbik::CF_TWIST_COS, C.s);
			const B3 gtc = Gt.b * from_quat(tcr);
			const B3 align = orthonormalized(inverse(gtc) * Gs.b);
			Q sw, tw;
			swing_twist_y(get_rotation_quaternion(align), sw, tw);
			tw = clamp_cos_half(tw, (double)half_cos);
			const B3 recomposition = orthonormalized(gtc * from_quat(sw * tw));
			X3 Lb = C.ld(C.LP(b));
			const X3 next = {pgi * recomposition, Lb.o};
			if (!eq(Lb, next)) { // set_transform (ik_node_3d.cpp:69-75)
				C.st(C.LP(b), next);
				C.propagate(b);
			}
		}
		MBIK_PROF_T(c3);
		MBIK_PROF_ADD(2, c2, c3);
#ifdef MBIK_PROF
		if (m > 1) pf[12] += c3 - c0;
		if (e1 - e0 > 1) pf[13] += c3 - c0;
#endif
		if (!stab) break;
		// _get_manual_msd(tip_headings_uniform, target_headings, weights) (:114-127)
		const double *hw = t.seg_hw + t.seg_hw_off[seg];
		float msd = 0.0f;
		for (int i = e0; i < e1; i++) {
			const int e = t.seg_effs[i];
			const X3 E = C.bdir_global(t.eff_bone[e]);
			const V3 ob = C.bdir_global(b).o;
			const float *T12 = tg + 12 * e;
			const X3 T = {bset(T12[0], T12[1], T12[2], T12[3], T12[4], T12[5], T12[6], T12[7], T12[8]), v3(T12[9], T12[10], T12[11])};
			const V3 oe = v3(OE[ls * (3 * e)], OE[ls * (3 * e + 1)], OE[ls * (3 * e + 2)]);
			Headings H;
			heading_terms(t, e, E, T, oe, ob, hw + t.seg_eff_hoff[i], H);
#pragma unroll
			for (int h = 0; h < 7; h++) {
				if (H.mask & (1 << h)) {
					const V3 d = H.ht[h] - H.hm[h];
					msd += (float)(H.w[h] * (double)(d.x * d.x + d.y * d.y + d.z * d.z));
				}
			}
		}
		msd /= t.seg_wsum2[seg];
		if ((double)msd <= prev_dev * 1.0001) {
			prev_dev = msd;
			break;
		}
		const X3 Lb = C.ld(C.LP(b));
		if (!eq(Lb, prev)) { // set_pose(prev_transform): set_transform
			C.st(C.LP(b), prev);
			C.propagate(b);
		}
		if (attempt + 1 >= t.stab) break;
	}
	if (k == t.seg_bone_off[seg + 1] - 1) prev_dev = INFINITY; // the segment root (:178-180)
}

// _process_modification (many_bone_ik_3d.cpp:645-694) in constraint_mode: K = 2^log2K lanes
// per skeleton, c.spw (<= 64 / K) skeletons per wave, c.wpb waves per block, the default
// kernel's sibling-row schedule (t.sched).  LDS: the topology blob and the pre-order tables
// once per block, then per wave the dirty words (4 W per skeleton, interleaved by skeleton),
// per lane (interleaved by 64) the chain stack (maxd) and, with STAB, the target-heading
// origins (3 P).  The solve is a chain of node-cache reads that miss to HBM (C5: 786 MB of
// node state), so what pays is memory-level parallelism: several waves per SIMD, which the
// shared topology copy makes fit in LDS (cmode_autotune times spw x K).  The node state stays in HBM:
// staging it through LDS was measured slower (one lane per skeleton: C2 5.6 vs 5.1 ms, C5
// 1003 vs 56 ms; LDS caps how many skeletons are resident;
// profiles/r01_cmode_layout_sweep.jsonl).
// CHAIN: the schedule has packed levels (SCHED_CHAIN rows); plans without them keep the plain
// row loop (its registers: the packed loop measured +2 % on C2).
template <bool STAB, bool NB32, bool CHAIN = false>
__global__ __launch_bounds__(64 * kCmodeMaxWaves) void mbik_cmode_kernel(DevPlan t, CmodeState c, int first, int count,
		const float *__restrict__ pose_in, const float *__restrict__ targets, float *__restrict__ pose_out, int iterations,
		int seg_lo, int seg_hi) {
	extern __shared__ float4 lds4[];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	{
		uint4 *dst = reinterpret_cast<uint4 *>(lds4);
		for (int i = threadIdx.x; i < (t.topo_words >> 2); i += blockDim.x) dst[i] = t.topo_blob[i];
	}
	const uint32_t *topo = reinterpret_cast<const uint32_t *>(lds4);
#define MBIK_REPOINT(T, name) t.name = reinterpret_cast<const T *>(topo + t.o_##name);
	MBIK_TOPO_TABLES(MBIK_REPOINT)
#undef MBIK_REPOINT
	const int B = t.B, P = t.P, K = t.K;
	const int spw = c.spw; // skeletons of this wave (<= 64 / K)
	int *pre = reinterpret_cast<int *>(lds4) + t.topo_words;
	int *sub = pre + B;
	for (int i = threadIdx.x; i < B; i += blockDim.x) {
		pre[i] = c.pre[i];
		sub[i] = c.sub[i];
	}
	// this wave's region: dirty words, chain stacks, target-heading origins (cmode_lds_bytes)
	uint32_t *dl0 = reinterpret_cast<uint32_t *>(sub + B) +
			(size_t)wv * (4 * c.W * spw + 64 * (c.maxd + (STAB ? 3 * P : 0)));
	int *stk0 = reinterpret_cast<int *>(dl0 + (size_t)4 * c.W * spw);
	float *OE = reinterpret_cast<float *>(stk0 + (size_t)c.maxd * 64) + lane;
	const int g = lane >> t.log2K, role = lane & (K - 1);
	// XCD-aware block order: neighbouring skeletons' node rows share L2 lines
	const int local = (xcd_block() * c.wpb + wv) * spw + g;
	const bool valid = g < spw && local < count;
	const size_t s = (size_t)first + (valid ? local : 0);
	int pend = -1;
	const int slots = 3 * B + 2 * t.NC;
	const uint32_t node_bytes = NB32 ? (uint32_t)(node_area_floats(slots, (size_t)t.N) * 4) : 0u;
	const size_t n0 = node_at(slots, s, 0, 0);
	CmodeLane<NB32> C{t, c, s, c.node + n0, slots, dl0 + (g < spw ? g : 0), spw, stk0 + lane, pre, sub, 0, 0x7fffffff,
			&pend, buf_rsrc(c.node, node_bytes), (uint32_t)(n0 * 4)};
#ifdef MBIK_PROF
	// 0 effector heading reads, 1 swing, 2 twist, 4 dirty pose chains (cycles), 5 chain nodes,
	// 6 dirty pose reads, 7 total, 8 after-row cleaning, 9 bone-direction recomputes, 10 chain
	// nodes above the segment root (private), 11 chain nodes in lane groups of m > 1, 12 / 13
	// step cycles with m > 1 / in multi-effector segments
	uint64_t pfa[24] = {};
	C.pf = pfa;
	uint64_t *pf = pfa;
#endif
	MBIK_PROF_T(k0);
	if (valid)
		for (int w = role; w < 4 * c.W; w += K) C.dl[spw * w] = c.dirty[(size_t)w * t.N + s];
	__syncthreads();
	// _update_ik_bones_transform (:91-102): set_transform of every list bone's pose
	if (valid)
		for (int b = role; b < B; b += K) {
			if (!(t.bone_flags[b] & mbik::BF_IN_LIST)) continue;
			const X3 L = pose_to_xform(pose_in + ((size_t)local * B + b) * 10);
			if (!eq(C.ld(C.LP(b)), L)) {
				C.st(C.LP(b), L);
				C.propagate(b);
			}
		}
	__syncthreads();
	const float *tg = targets + (size_t)local * P * 12;
	for (int it = 0; it < iterations; it++) {
		if constexpr (!CHAIN) {
		for (int r = 0; r < t.nrows; r++) {
			const int4 task = t.sched[r * K + role];
			if (valid && task.x >= seg_lo && task.x <= seg_hi) {
				const int root = t.seg_bones[t.seg_bone_off[task.x + 1] - 1];
				C.lo = pre[root];
				C.hi = pre[root] + sub[root];
				double prev_dev = INFINITY; // reset after the segment root bone (:178-180)
				for (int k = t.seg_bone_off[task.x]; k < t.seg_bone_off[task.x + 1]; k++)
					cmode_step<STAB, NB32>(C, task.x, k, task.y, task.z, tg, OE, prev_dev);
			}
			__syncthreads();
			// The cleaning the reference's first read above the segment root did: the dirty
			// chain from the recorded node up, one lane at a time (siblings share it).
			MBIK_PROF_T(r0);
			uint64_t todo = __ballot(pend >= 0);
			while (todo) {
				const int l = __ffsll((unsigned long long)todo) - 1;
				todo &= todo - 1;
				if (lane == l) {
					C.lo = 0;
					C.hi = 0x7fffffff;
					(void)C.pose_global(pend);
					pend = -1;
				}
				__threadfence_block();
			}
			MBIK_PROF_T(r1);
			MBIK_PROF_ADD(8, r0, r1);
			__syncthreads();
		}
		} else {
		for (int r = 0; r < t.nrows;) {
			// rows r .. r1-1: one row, or a packed level (SCHED_CHAIN rows, at most four
			// segments per lane): each lane runs its segments back to back.  Nothing above the
			// level changes during it, so a sibling's private reads of the chains above its root
			// give the same bits before or after another sibling's cleaning; every segment's
			// pending chain is kept (p0..p3) and cleaned after the level.
			int r1 = r + 1;
			while (r1 < t.nrows && (t.sched[r1 * K].w & mbik::SCHED_CHAIN)) r1++;
			int rr = r - 1, k = 0, ke = 0, seg = 0, j = 0, m = 1;
			int p1 = -1, p2 = -1, p3 = -1;
			double prev_dev = INFINITY;
			for (;;) {
				while (k >= ke && rr + 1 < r1) {
					const int4 task = t.sched[++rr * K + role];
					if (valid && task.x >= seg_lo && task.x <= seg_hi) {
						if (pend >= 0) {
							p3 = p2;
							p2 = p1;
							p1 = pend;
							pend = -1;
						}
						seg = task.x;
						j = task.y;
						m = task.z;
						const int root = t.seg_bones[t.seg_bone_off[seg + 1] - 1];
						C.lo = pre[root];
						C.hi = pre[root] + sub[root];
						k = t.seg_bone_off[seg];
						ke = t.seg_bone_off[seg + 1];
						prev_dev = INFINITY; // reset after the segment root bone (:178-180)
					}
				}
				if (k >= ke) break;
				cmode_step<STAB, NB32>(C, seg, k, j, m, tg, OE, prev_dev);
				k++;
			}
			__syncthreads();
			// The cleaning the reference's first read above the segment root did: the dirty
			// chain from the recorded node up, one lane at a time (siblings share it).
			MBIK_PROF_T(rc0);
#pragma unroll
			for (int q = 0; q < 4; q++) {
				uint64_t todo = __ballot(pend >= 0);
				while (todo) {
					const int l = __ffsll((unsigned long long)todo) - 1;
					todo &= todo - 1;
					if (lane == l) {
						C.lo = 0;
						C.hi = 0x7fffffff;
						(void)C.pose_global(pend);
					}
					__threadfence_block();
				}
				pend = p1;
				p1 = p2;
				p2 = p3;
				p3 = -1;
				if (!__any(pend >= 0)) break;
			}
			MBIK_PROF_T(rc1);
			MBIK_PROF_ADD(8, rc0, rc1);
			__syncthreads();
			r = r1;
		}
		}
	}
	bool bad = false;
	if (valid) {
		for (int b = role; b < B; b += K) {
			float *dst = pose_out + ((size_t)local * B + b) * 10;
			if (t.bone_flags[b] & mbik::BF_IN_LIST) {
				bad |= write_pose(C.ld(C.LP(b)), dst);
			} else {
				const float *src = pose_in + ((size_t)local * B + b) * 10;
				for (int f = 0; f < 10; f++) dst[f] = src[f];
			}
		}
	}
	write_nonfinite(t, valid, bad, g, role, local);
	__syncthreads();
	if (valid)
		for (int w = role; w < 4 * c.W; w += K) c.dirty[(size_t)w * t.N + s] = C.dl[spw * w];
#ifdef MBIK_PROF
	MBIK_PROF_T(k1);
	pfa[7] += k1 - k0;
	if (valid)
		for (int i = 0; i < 24; i++) atomicAdd(&g_mbik_prof[i], (unsigned long long)pfa[i]);
#endif
}

// constraint_mode with wave roles (HostPlan::cm_roles; mbik_plan_set_wave_roles): a block is KW
// waves x c.spw skeletons, a lane per skeleton and a wave per role of the sibling schedule.  A
// wave then follows one segment for all its skeletons -- its topology is wave-uniform and its
// dirty chains have the same shape on every lane -- and each role waits for its own node-cache
// misses instead of for the union of the wave's roles' paths.  LDS: the topology and pre-order
// tables, the block's dirty words (shared by a skeleton's waves through LDS atomics, as the
// classic kernel shares them between lanes), per wave its lanes' chain stacks, then the row's
// pending cleanings ([KW][4][64]) and the non-finite flags (64).  No stabilization.
//
// Rows with a SCHED_CMSPLIT segment (SCHED_COOP): each bone-step is three phases between two
// block barriers -- the group's first wave cleans the segment's trunk as the reference's first
// effective read would, then every wave of the group reads its clusters of effectors
// (plan.cpp cm_split_groups: effectors whose paths share a node below the trunk stay on one
// wave, in order), then the first wave runs the rest of the step (the bone's own read, the swing
// and the twist).  The other tasks of such a row run their whole step in the last phase.
// Sibling segments touch disjoint subtrees, and a wave's writes reach the others through the
// barriers.
template <bool NB32, bool CHAIN, int KW>
__global__ __launch_bounds__(64 * KW) void mbik_cmode_kernel_rw(DevPlan t, CmodeState c, int first, int count,
		const float *__restrict__ pose_in, const float *__restrict__ targets, float *__restrict__ pose_out, int iterations,
		int seg_lo, int seg_hi) {
	extern __shared__ float4 lds4[];
	const int lane = threadIdx.x & 63;
	const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
	{
		uint4 *dst = reinterpret_cast<uint4 *>(lds4);
		for (int i = threadIdx.x; i < (t.topo_words >> 2); i += 64 * KW) dst[i] = t.topo_blob[i];
	}
	const uint32_t *topo = reinterpret_cast<const uint32_t *>(lds4);
#define MBIK_REPOINT(T, name) t.name = reinterpret_cast<const T *>(topo + t.o_##name);
	MBIK_TOPO_TABLES(MBIK_REPOINT)
#undef MBIK_REPOINT
	const int B = t.B, K = KW;
	const int spw = c.spw; // skeletons of this block (<= 64)
	int *pre = reinterpret_cast<int *>(lds4) + t.topo_words;
	int *sub = pre + B;
	for (int i = threadIdx.x; i < B; i += 64 * KW) {
		pre[i] = c.pre[i];
		sub[i] = c.sub[i];
	}
	uint32_t *dl0 = reinterpret_cast<uint32_t *>(sub + B);                        // [4 W][spw]
	int *stks = reinterpret_cast<int *>(dl0 + (size_t)4 * c.W * spw);           // [KW][maxd][64]
	int *pv = stks + (size_t)KW * c.maxd * 64;                                   // [KW][4][64]
	int *nf = pv + KW * 4 * 64;                                                   // [64]
	const int g = lane, role = wv;
	const int local = xcd_block() * spw + g;
	const bool valid = g < spw && local < count;
	const size_t s = (size_t)first + (valid ? local : 0);
	int pend = -1;
	const int slots = 3 * B + 2 * t.NC;
	const uint32_t node_bytes = NB32 ? (uint32_t)(node_area_floats(slots, (size_t)t.N) * 4) : 0u;
	const size_t n0 = node_at(slots, s, 0, 0);
	CmodeLane<NB32> C{t, c, s, c.node + n0, slots, dl0 + (g < spw ? g : 0), spw, stks + (size_t)wv * c.maxd * 64 + lane, pre, sub, 0,
			0x7fffffff, &pend, buf_rsrc(c.node, node_bytes), (uint32_t)(n0 * 4)};
#ifdef MBIK_PROF
	uint64_t pfa[24] = {};
	C.pf = pfa;
	uint64_t *pf = pfa;
#endif
	MBIK_PROF_T(k0);
	if (wv == 0) nf[lane] = 0;
	if (valid)
		for (int w = role; w < 4 * c.W; w += K) C.dl[spw * w] = c.dirty[(size_t)w * t.N + s];
	__syncthreads();
	// _update_ik_bones_transform (:91-102): set_transform of every list bone's pose
	if (valid)
		for (int b = role; b < B; b += K) {
			if (!(t.bone_flags[b] & mbik::BF_IN_LIST)) continue;
			const X3 L = pose_to_xform(pose_in + ((size_t)local * B + b) * 10);
			if (!eq(C.ld(C.LP(b)), L)) {
				C.st(C.LP(b), L);
				C.propagate(b);
			}
		}
	__syncthreads();
	const float *tg = targets + (size_t)local * t.P * 12;
	double prev_dev = INFINITY; // (stabilization only)
	auto set_range = [&](int seg) {
		const int root = t.seg_bones[t.seg_bone_off[seg + 1] - 1];
		C.lo = pre[root];
		C.hi = pre[root] + sub[root];
	};
	for (int it = 0; it < iterations; it++) {
		for (int r = 0; r < t.nrows;) {
			const int4 task0 = t.sched[r * K + role];
			int r1 = r + 1;
			if constexpr (CHAIN)
				while (r1 < t.nrows && (t.sched[r1 * K].w & mbik::SCHED_CHAIN)) r1++;
			int p1 = -1, p2 = -1, p3 = -1;
			// One loop for both kinds of row, with one site each for the effector reads, the
			// bone-step and the cleaning: every extra inlined copy of the node-cache code costs
			// thousands of instructions.
			//   cooperative row (SCHED_COOP): nq bone-steps of three phases between two block
			//   barriers -- the group's first wave reads the first effector, the group's waves
			//   read their clusters of the others, the first wave runs the rest of the step (the
			//   row's other tasks run their whole step then);
			//   other rows (one row, or a packed level): the wave's segments back to back.
			const bool coop = (task0.w & mbik::SCHED_COOP) != 0;
			const int j = task0.y;
			const bool split = coop && (task0.w & mbik::SCHED_CMSPLIT) != 0;
			const int nq = coop ? row_steps(t, r, seg_lo, seg_hi) : 0;
			// (the segment bookkeeping is wave-uniform; only the work is per lane, for valid lanes)
			int seg = coop ? task0.x : -1, k = 0, ke = 0, rr = r - 1, q = 0;
			if (coop && seg >= 0 && seg >= seg_lo && seg <= seg_hi) {
				set_range(seg);
				k = t.seg_bone_off[seg];
				ke = t.seg_bone_off[seg + 1];
			}
			const int e0 = seg >= 0 ? t.seg_eff_off[seg] : 0, e1 = seg >= 0 ? t.seg_eff_off[seg + 1] : 0;
			for (;;) {
				bool run;
				if (coop) {
					if (q >= nq) break;
					const bool step = k + q < ke;
					// Phase 0, the group's first wave: the trunk bone T (plan.cpp cm_split_groups)
					// made clean the way the reference's reads clean it.  Only the first effector
					// whose bone-direction cache is dirty walks (the earlier reads find their caches
					// clean); if T is dirty and that walk runs through T, its part from T up is
					// T's own chain -- recomputed here, the same nodes and values -- and the rest
					// of the walk is left to phase 1.  A walk that would stop below T (rare: a
					// clean node under a dirty T) leaves every read to this wave, in order.
					if (split && step && j == 0 && valid) {
						const int T = (t.seg_eff_grp[e0] >> 4) - 1;
						int from = e0, seq = 0;
						if (C.dirty(CK_POSE, T)) {
							while (from < e1 && !C.dirty(CK_BDIR, t.eff_bone[t.seg_effs[from]])) from++;
							if (from < e1) {
								int x = t.eff_bone[t.seg_effs[from]];
								while (x != T && C.dirty(CK_POSE, x)) x = t.bone_pose_parent[x];
								if (x == T) (void)C.pose_global(T);
								else seq = 1;
							}
						}
						pv[role * 4 * 64 + lane] = from | seq << 16;
					}
					__syncthreads();
					// Phase 1: each wave reads its clusters from there on, in order (or the first
					// wave all of them, in order).
					if (split && step && valid) {
						const int v = pv[(role - j) * 4 * 64 + lane], seq = v >> 16;
#pragma nounroll
						for (int i = v & 0xffff; i < e1; i++)
							if (seq ? j == 0 : (t.seg_eff_grp[i] & 15) == j) C.bdir_touch(t.eff_bone[t.seg_effs[i]]);
					}
					__syncthreads();
					run = step && j == 0;
				} else {
					while (k >= ke && rr + 1 < r1) {
						const int4 task = t.sched[++rr * K + role];
						if (task.x >= 0 && task.x >= seg_lo && task.x <= seg_hi && task.y == 0) {
							if (pend >= 0) {
								p3 = p2;
								p2 = p1;
								p1 = pend;
								pend = -1;
							}
							seg = task.x;
							set_range(seg);
							k = t.seg_bone_off[seg];
							ke = t.seg_bone_off[seg + 1];
						}
					}
					if (k >= ke) break;
					run = true;
				}
				if (run && valid) cmode_step<false, NB32>(C, seg, coop ? k + q : k, 0, 1, tg, nullptr, prev_dev, !split);
				if (coop) q++;
				else k++;
			}
			// The cleaning the reference's first read above a segment root did, for every pending
			// chain of the row (siblings share them; a chain is computed once and then clean): the
			// first wave cleans them all, lane by lane for its own skeleton.
			pv[(role * 4 + 0) * 64 + lane] = pend;
			pv[(role * 4 + 1) * 64 + lane] = p1;
			pv[(role * 4 + 2) * 64 + lane] = p2;
			pv[(role * 4 + 3) * 64 + lane] = p3;
			pend = -1;
			__syncthreads();
			MBIK_PROF_T(rc0);
			if (wv == 0 && valid) {
				C.lo = 0;
				C.hi = 0x7fffffff;
#pragma nounroll
				for (int w = 0; w < 4 * K; w++) {
					const int x = pv[w * 64 + lane];
					if (x >= 0) (void)C.pose_global(x);
				}
			}
			MBIK_PROF_T(rc1);
			MBIK_PROF_ADD(8, rc0, rc1);
			__syncthreads();
			r = r1;
		}
	}
	bool bad = false;
	if (valid) {
		for (int b = role; b < B; b += K) {
			float *dst = pose_out + ((size_t)local * B + b) * 10;
			if (t.bone_flags[b] & mbik::BF_IN_LIST) {
				bad |= write_pose(C.ld(C.LP(b)), dst);
			} else {
				const float *src = pose_in + ((size_t)local * B + b) * 10;
				for (int f = 0; f < 10; f++) dst[f] = src[f];
			}
		}
	}
	// a skeleton's bones are written by all its waves: their flags meet in LDS
	if (valid && bad) nf[lane] = 1;
	__syncthreads();
	if (t.nonfinite && valid && wv == 0) t.nonfinite[local] = nf[lane] != 0;
	if (valid)
		for (int w = role; w < 4 * c.W; w += K) c.dirty[(size_t)w * t.N + s] = C.dl[spw * w];
#ifdef MBIK_PROF
	MBIK_PROF_T(k1);
	pfa[7] += k1 - k0;
	if (valid)
		for (int i = 0; i < 24; i++) atomicAdd(&g_mbik_prof[i], (unsigned long long)pfa[i]);
#endif
}

// A fresh node tree (_bone_list_changed): pose locals = the setup pose, every cache dirty.
__global__ __launch_bounds__(64) void mbik_cmode_reset_kernel(DevPlan t, CmodeState c, int first, int count,
		const float *__restrict__ setup_pose) {
	const int local = blockIdx.x * 64 + threadIdx.x;
	if (local >= count) return;
	t.bone_flags = reinterpret_cast<const int *>(reinterpret_cast<const uint32_t *>(t.topo_blob) + t.o_bone_flags);
	const size_t s = (size_t)first + local;
	for (int b = 0; b < t.B; b++) {
		if (!(t.bone_flags[b] & mbik::BF_IN_LIST)) continue;
		const X3 L = pose_to_xform(setup_pose + ((size_t)local * t.B + b) * 10);
		float *p = c.node + node_at(3 * t.B + 2 * t.NC, s, b, 0);
		const float v[12] = {L.b.r[0].x, L.b.r[0].y, L.b.r[0].z, L.b.r[1].x, L.b.r[1].y, L.b.r[1].z,
				L.b.r[2].x, L.b.r[2].y, L.b.r[2].z, L.o.x, L.o.y, L.o.z};
		for (int f = 0; f < 12; f++) p[(f >> 2) * 4 * kNodeTile + (f & 3)] = v[f];
	}
	for (int w = 0; w < 4 * c.W; w++) c.dirty[(size_t)w * t.N + s] = ~0u;
}
} // namespace
