// One bone-step of the solve and the work around it (device code; included by the kernel TUs
// after dev_common.h): the helper wave's records, the staged-heading terms, bone_step itself
// (IKBoneSegment3D::_update_optimal_rotation + _set_optimal_rotation, ik_bone_segment_3d.cpp:90-181),
// the iteration-start global passes, the wave-roles cooperative walk and the pose write-back.
#pragma once
#include "dev_common.h"

namespace {

using mbik::kHelpF4;
using mbik::kHelpSlots;
using mbik::kHelpRingBytes;

// ------------------------------------------------------------------------------------
// One bone-step: IKBoneSegment3D::_update_optimal_rotation + _set_optimal_rotation
// (ik_bone_segment_3d.cpp:90-181), including the stabilization retry loop (:163-180) of
// root segments and constraint_mode (:142).  prev_dev is the segment's previous_deviation.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync_lds() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// The parent's iteration-start global of bone-step k (step record sr): its checkpoint, times the
// locals of the bones between that checkpoint and the step's bone (none when no checkpoint is
// skipped), with the global pass's own products in its order.  The first three of those locals
// load together before the products (sparse checkpoints with the locals in device memory: C3's
// interval-4 layout waited for each load in turn; same products, same order).
template <class LV, class GV>
__device__ __forceinline__ X3 parent_global(const DevPlan &t, const int4 sr, int k, const LV &L, const GV &G) {
	X3 P = G.ld((sr.y & 0xffff) - 1);
	const int q0 = (sr.x >> 16) - 2;
	if (q0 > k) {
		const X3 a = L.ld(t.seg_bones[q0]);
		const X3 b = L.ld(t.seg_bones[max(q0 - 1, k + 1)]);
		const X3 c = L.ld(t.seg_bones[max(q0 - 2, k + 1)]);
		P = P * a;
		if (q0 - 1 > k) P = P * b;
		if (q0 - 2 > k) P = P * c;
		for (int q = q0 - 3; q > k; q--) P = P * L.ld(t.seg_bones[q]);
	}
	return P;
}
// ---- Helper wave (HELP, fully resident placement-0 launches) ----
// A bone-step's parent-side work depends only on the iteration-start state: the parent's global
// P (a checkpoint, or rebuilt from one through ancestors not yet solved this iteration), the
// bone's own iteration-start local (only its own step writes it), and per-skeleton constants.
// A second wave of the block -- on another SIMD of the CU, which a fully resident launch
// leaves idle -- runs the global pass and computes that work one step ahead into an LDS ring,
// so the solving wave's chain keeps only what depends on the step's fit:
//   P, Gb = P * Lb, inverse(P.b), xform(inverse(P.b), -P.o), the slerp's p_to side,
//   the bone-direction basis (swing), the twist frame gtc = (P.b * T) * R(centre), its inverse
//   and the twist limit's half cosine (ik_bone_segment_3d.cpp:129-154, ik_kusudama_3d.cpp:117-132).
// Same operations on the same inputs: the record's values are the bits the solving wave would
// have computed.  Ring: kHelpSlots records of kHelpF4 float4 per lane, [slot][field][64 lanes];
// four LDS counters (part A produced, part B produced, records consumed, iterations finished)
// order the two waves; a fifth word is set when either wave gave up waiting (help_wait).
enum HelpCounter { HC_A = 0, HC_B = 1, HC_CONSUMED = 2, HC_ITER = 3, HC_STUCK = 4 };
enum HelpField { HF_P = 0, HF_GB = 12, HF_PINV = 24, HF_PNP = 33, HF_STO = 36, HF_HC = 43, HF_DB = 44, HF_GTC = 53, HF_GTCI = 62 };
__device__ __forceinline__ float hrf(const float4 *r, int i) { return reinterpret_cast<const float *>(r + (i >> 2) * 64)[i & 3]; }
__device__ __forceinline__ V3 hrv(const float4 *r, int i) { return v3(hrf(r, i), hrf(r, i + 1), hrf(r, i + 2)); }
__device__ __forceinline__ B3 hrb(const float4 *r, int i) { return B3{{hrv(r, i), hrv(r, i + 3), hrv(r, i + 6)}}; }
__device__ __forceinline__ X3 hrx(const float4 *r, int i) { return X3{hrb(r, i), hrv(r, i + 9)}; }
__device__ __forceinline__ void hw_v(float *f, int i, V3 v) { f[i] = v.x; f[i + 1] = v.y; f[i + 2] = v.z; }
__device__ __forceinline__ void hw_b(float *f, int i, const B3 &b) { hw_v(f, i, b.r[0]); hw_v(f, i + 3, b.r[1]); hw_v(f, i + 6, b.r[2]); }
// Waits until counter hfl[k] reaches v.  Every wait has an exit: when the counter has not
// moved for `timeout` wall-clock ticks (a couple of seconds; a real wait lasts at most one
// iteration of the partner wave) the wave stops waiting for the rest of the launch and raises
// hfl[HC_STUCK].  The kernel then drains instead of hanging the GPU, and the solving wave writes
// its skeletons as failed (write_help_timeout): flagged non-finite, the plan's timeout flag set.
__device__ __forceinline__ void help_give_up(int *hfl, bool &stuck) {
	stuck = true;
	__hip_atomic_store(hfl + HC_STUCK, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// t0: when the counter was last seen to move; tl: the previous poll.  Polls come every s_sleep
// (microseconds apart), so a gap between two polls of more than timeout / 200 (10 ms of the 2 s
// deadline) means the waves were suspended (preemption, context save/restore), not that the
// partner stalled: the gap is not counted (t0 moves forward by it), the rest of the wait is.  So
// a stalled partner is still detected however often the waves are suspended.
__device__ __forceinline__ bool help_expired(uint64_t &t0, uint64_t &tl, int &seen, int now_val, uint64_t timeout) {
	const uint64_t now = (uint64_t)wall_clock64();
	if (t0 == 0 || now_val != seen) {
		t0 = tl = now;
		seen = now_val;
		return false;
	}
	if (now - tl > timeout / 200) t0 += now - tl;
	tl = now;
	return now - t0 > timeout;
}
__device__ __forceinline__ void help_wait(int *hfl, int k, int v, bool &stuck, uint64_t timeout) {
	if (stuck) return;
	uint64_t t0 = 0, tl = 0;
	int seen = 0;
	for (;;) {
		const int c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(hfl + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
		if (c >= v) return;
		if (help_expired(t0, tl, seen, c, timeout)) return help_give_up(hfl, stuck);
		__builtin_amdgcn_s_sleep(1);
	}
}
// The solving wave's wait for record v - 1: counters [0] part A and [1] part B in one 64-bit
// read; b_ready tells whether part B is already there too (then bone_step skips its wait).
__device__ __forceinline__ void help_wait_ab(int *hfl, int v, bool &stuck, bool &b_ready, uint64_t timeout) {
	b_ready = stuck;
	if (stuck) return;
	unsigned long long *f2 = reinterpret_cast<unsigned long long *>(hfl);
	uint64_t t0 = 0, tl = 0;
	int seen = 0;
	for (;;) {
		const unsigned long long ab = __hip_atomic_load(f2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
		const int a = __builtin_amdgcn_readfirstlane((int)(uint32_t)ab), b = __builtin_amdgcn_readfirstlane((int)(uint32_t)(ab >> 32));
		if (a >= v) {
			b_ready = b >= v;
			return;
		}
		if (help_expired(t0, tl, seen, a, timeout)) {
			b_ready = true;
			return help_give_up(hfl, stuck);
		}
		__builtin_amdgcn_s_sleep(1);
	}
}
__device__ __forceinline__ void help_post(int *f, int v) { __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
// The record of bone-step k (the helper wave), in two parts so that the solving wave can start
// a step as soon as the bone's global is there: part A (P, Gb: the headings need Gb), part B
// (the rest, needed from the rotation on).  The per-skeleton table rows a record reads are
// constants; HelpRows holds them so the helper can issue the loads early.
struct HelpRows {
	B3 Db, Tb;
	Q tcr;
	float hc;
};
template <int TA>
__device__ __forceinline__ HelpRows help_rows(const DevPlan &t, int k, size_t s) {
	HelpRows r;
	const int4 sr = t.step_rec[k];
	const int b = sr.x & 0xffff;
	const int flags = sr.z & 0xffff;
	const int slot = (sr.y >> 16) - 1;
	r.Db = B3{};
	r.Tb = B3{};
	r.tcr = q4(0, 0, 0, 1);
	r.hc = 0.0f;
	if (flags & mbik::BF_ORIENT) r.Db = ld_soa_basis<TA>(t, t.D, b, 9, 0, s);
	if (flags & mbik::BF_AXIAL) {
		const int cs = t.cf_stride;
		r.tcr = q4(soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q, s), soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 1, s),
				soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 2, s), soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 3, s));
		r.hc = soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_COS, s);
		r.Tb = ld_soa_basis<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_T, s);
	}
	return r;
}
__device__ __forceinline__ void hw_store(float4 *rec, const float *f, int f4a, int f4b) {
	for (int i = f4a; i < f4b; i++) rec[i * 64] = make_float4(f[4 * i], f[4 * i + 1], f[4 * i + 2], f[4 * i + 3]);
}
// part A: P and Gb (float4 fields 0-5)
template <class LV, class GV>
__device__ __forceinline__ void help_part_a(const DevPlan &t, int k, const LV &L, const GV &G, float4 *rec, X3 &P, B3 &Gbb) {
	const int4 sr = t.step_rec[k];
	const int b = sr.x & 0xffff;
	const int flags = sr.z & 0xffff;
	const bool hasP = (flags & mbik::SR_HAS_POSE_PARENT) != 0;
	P = xid();
	if (flags & mbik::SR_PARENT_GLOBAL) {
		P = parent_global(t, sr, k, L, G);
	}
	const X3 Lb = L.ld(b);
	const X3 Gb = hasP ? P * Lb : Lb;
	Gbb = Gb.b;
	float f[24];
	hw_b(f, HF_P, P.b);
	hw_v(f, HF_P + 9, P.o);
	hw_b(f, HF_GB, Gb.b);
	hw_v(f, HF_GB + 9, Gb.o);
	hw_store(rec, f, 0, 6);
}
// part B: everything else (float4 fields 6-17)
__device__ __forceinline__ void help_part_b(const DevPlan &t, int k, const X3 &P, const B3 &Gbb, const HelpRows &rw, float4 *rec) {
	const int flags = t.step_rec[k].z & 0xffff;
	const B3 Pinv = inverse(P.b);
	const SlerpTo sto = slerp_to(Gbb);
	float f[4 * kHelpF4];
	hw_b(f, HF_PINV, Pinv);
	hw_v(f, HF_PNP, xform(Pinv, -P.o));
	f[HF_STO] = sto.q.x; f[HF_STO + 1] = sto.q.y; f[HF_STO + 2] = sto.q.z; f[HF_STO + 3] = sto.q.w;
	f[HF_STO + 4] = sto.len[0]; f[HF_STO + 5] = sto.len[1]; f[HF_STO + 6] = sto.len[2];
	f[HF_HC] = rw.hc;
	hw_b(f, HF_DB, rw.Db);
	for (int i = HF_GTC; i < 4 * kHelpF4; i++) f[i] = 0.0f;
	if (flags & mbik::BF_AXIAL) {
		const B3 Gct = P.b * rw.Tb;
		const B3 gtc = Gct * from_quat(rw.tcr);
		hw_b(f, HF_GTC, gtc);
		hw_b(f, HF_GTCI, inverse(gtc));
	}
	hw_store(rec, f, 6, kHelpF4);
}

// ---- Wave roles, cooperative segments: the parent-side record of the group's second wave ----
// While a cooperative group's first wave runs bone-step k's chain, the group's other waves wait
// at the block barrier.  The second wave instead computes step k + 1's parent-side values --
// they depend only on iteration-start state, as the helper wave's records do (a tip -> root pass
// leaves the ancestors unsolved): the parent's global P, the bone's origin Gb.o, inverse(P.b),
// xform(inverse(P.b), -P.o) and the slerp's p_to side -- with bone_step's own operations on the
// same inputs, so the first wave reads the bits it would have computed.  Layout as the helper
// ring's, [float4 field][64 lanes], one record per group (kernels.h kRwRecF4; the writes of step
// k + 1's record come after the barrier that ends step k, when its reader is done).
enum RwRecField { RF_P = 0, RF_GBO = 12, RF_PINV = 15, RF_PNP = 24, RF_STO = 27 };
struct RwRec {
	X3 P;
	V3 gbo;
	B3 Pinv;
	V3 pnp;
	SlerpTo sto;
};
template <class LV, class GV>
__device__ __forceinline__ RwRec rw_record(const DevPlan &t, int k, const LV &L, const GV &G) {
	const int4 sr = t.step_rec[k];
	const int b = sr.x & 0xffff;
	const int flags = sr.z & 0xffff;
	RwRec r;
	r.P = xid();
	if (flags & mbik::SR_PARENT_GLOBAL) {
		r.P = parent_global(t, sr, k, L, G);
	}
	r.Pinv = inverse(r.P.b);
	const X3 Lb = L.ld(b);
	const X3 Gb = (flags & mbik::SR_HAS_POSE_PARENT) ? r.P * Lb : Lb;
	r.gbo = Gb.o;
	r.pnp = xform(r.Pinv, -r.P.o);
	r.sto = slerp_to(Gb.b);
	return r;
}
// The second wave's wait until the group's first wave has read the current record (its counter
// reaches v).  Every wait has an exit, as the helper wave's: when the counter has not moved for
// `timeout` wall-clock ticks (help_expired) the wave raises the block's gave-up word and stops
// waiting for the rest of the launch; the block then writes its skeletons as failures
// (write_help_timeout) and sets the plan's timeout flag, as a helper-wave block does.
__device__ __forceinline__ void rw_wait(const int *cnt, int v, bool &stuck, int *gave_up, uint64_t timeout) {
	if (stuck) return;
	uint64_t t0 = 0, tl = 0;
	int seen = 0;
	for (;;) {
		const int c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
		if (c >= v) return;
		if (help_expired(t0, tl, seen, c, timeout)) {
			stuck = true;
			__hip_atomic_store(gave_up, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
			return;
		}
		__builtin_amdgcn_s_sleep(1);
	}
}
__device__ __forceinline__ void rw_record_store(float4 *rec, const RwRec &r) {
	float f[4 * mbik::kRwRecF4];
	hw_b(f, RF_P, r.P.b);
	hw_v(f, RF_P + 9, r.P.o);
	hw_v(f, RF_GBO, r.gbo);
	hw_b(f, RF_PINV, r.Pinv);
	hw_v(f, RF_PNP, r.pnp);
	f[RF_STO] = r.sto.q.x; f[RF_STO + 1] = r.sto.q.y; f[RF_STO + 2] = r.sto.q.z; f[RF_STO + 3] = r.sto.q.w;
	f[RF_STO + 4] = r.sto.len[0]; f[RF_STO + 5] = r.sto.len[1]; f[RF_STO + 6] = r.sto.len[2];
	for (int i = RF_STO + 7; i < 4 * mbik::kRwRecF4; i++) f[i] = 0.0f;
	hw_store(rec, f, 0, mbik::kRwRecF4);
}

// Staged-heading record (multi-lane segments): the 11 QCP::inner_product terms of one heading
// pair, as floats -- wc1_a * c2_b (a, b = x, y, z), dot(wc1, c1), dot(c2, c2).
constexpr int HS_REC = 12;
template <class FP>
__device__ __forceinline__ void qcp_terms(const V3 wc1, const V3 c1, const V3 c2, const FP r) {
	// the nine float products as four packed pairs and one scalar (each lane of a pair is the
	// scalar IEEE product, so the terms are the same bits)
#ifdef GD_PACK
	const F2 px = xy(c2) * wc1.x, py = xy(c2) * wc1.y, pz = xy(c2) * wc1.z, pc = xy(wc1) * c2.z;
#else
	const V3 px = v3(c2.x * wc1.x, c2.y * wc1.x, 0), py = v3(c2.x * wc1.y, c2.y * wc1.y, 0),
			pz = v3(c2.x * wc1.z, c2.y * wc1.z, 0), pc = v3(wc1.x * c2.z, wc1.y * c2.z, 0);
#endif
	r[0] = px.x; r[1] = px.y; r[2] = pc.x;
	r[3] = py.x; r[4] = py.y; r[5] = pc.y;
	r[6] = pz.x; r[7] = pz.y; r[8] = wc1.z * c2.z;
	r[9] = dot(wc1, c1);
	r[10] = dot(c2, c2);
}
// One heading's terms added to QCP::inner_product's sums (qcp.cpp:162-218): float products
// (packed as in qcp_terms), each widened and added to its fp64 sum in the reference's order.
__device__ __forceinline__ void qcp_accumulate(QSums &S, const V3 wc1, const V3 c1, const V3 c2, double w) {
	S.ss1 += (double)dot(wc1, c1);
	S.ss2 += w * (double)dot(c2, c2);
#ifdef GD_PACK
	const F2 px = xy(c2) * wc1.x, py = xy(c2) * wc1.y, pz = xy(c2) * wc1.z, pc = xy(wc1) * c2.z;
#else
	const V3 px = v3(c2.x * wc1.x, c2.y * wc1.x, 0), py = v3(c2.x * wc1.y, c2.y * wc1.y, 0),
			pz = v3(c2.x * wc1.z, c2.y * wc1.z, 0), pc = v3(wc1.x * c2.z, wc1.y * c2.z, 0);
#endif
	S.xx += (double)px.x;
	S.xy += (double)px.y;
	S.xz += (double)pc.x;
	S.yx += (double)py.x;
	S.yy += (double)py.y;
	S.yz += (double)pc.y;
	S.zx += (double)pz.x;
	S.zy += (double)pz.y;
	S.zz += (double)(wc1.z * c2.z);
}
// STAB: the plan has stabilization passes (a separate instantiation keeps the retry loop and
// its LDS staging out of the default kernel).
// PR: reuse effector path prefixes (PathCk) in multi-effector segments solved from registers.
// HELP: the parent-side values come from the helper wave's record hrec (kHelpF4 float4 at
// stride 64), not from this wave.  XS: the build serves split-exchange tasks (xs, staging 4 /
// 5): only the two-waves-per-SIMD build, so that the one-wave kernels keep their registers.
// SEL: the orthonormalizations' zero-vector tests as selects (normalized_sel; the one-wave builds).
// XW (wave roles): xs marks a cooperative segment whose effector globals the group's waves left in
// the exchange area xw (coop_walk); this wave, the group's first, consumes them, and with hrec
// its parent-side values come from the group's second wave's record (rw_record): it reads the
// whole record first and posts hseq in the group's counter hfl (rw_wait).
template <bool STAB, bool PR, int TA, bool HELP, bool XS, int PM, bool SEL, bool XW, class LV, class GV, class FP, class IP>
__device__ void bone_step(const DevPlan &t, int seg, int k, int j, int m, int xs, size_t s, const LV &L, const GV &G, const FP TG,
		const FP ST, const IP SF, const FP HS, const FP OE, const FP MS, double &prev_dev, const EffPre &pre, bool hoist,
		const float4 *hrec, int *hfl, int hseq, bool *hstuck, const float *xw MBIK_PROF_PARAM) {
	MBIK_PROF_T(pt0);
#ifdef MBIK_PROF
	uint64_t pt1 = pt0, pt3 = pt0;
	const bool seg_translate = (t.seg_flags[seg] & mbik::SF_TRANSLATE) != 0;
#endif
	// the step's topology, resolved on the host (HostPlan::step_rec): no dependent lookups
	const int4 sr = t.step_rec[k];
	const int b = sr.x & 0xffff;
	const int flags = sr.z & 0xffff;           // bone_flags | SR_* bits
	const int d0 = sr.z >> 16;                 // path index of b's first descendant
	const int slot = (sr.y >> 16) - 1;         // constraint slot
	const bool hasP = (flags & mbik::SR_HAS_POSE_PARENT) != 0;
	// The parent's iteration-start global: stored if the parent is a checkpoint, else rebuilt
	// from the nearest checkpoint above it, with the global pass's own products.
	X3 P = xid();
	B3 Pinv;
	// wave roles: a cooperative segment's step with its parent-side record (rw_record)
	const bool rrec = XW && xs && hrec != nullptr;
	V3 rgbo, rpnp;
	SlerpTo rsto;
	if constexpr (HELP) {
		// (P, Pinv: read after the wait for the record's part B, below)
	} else if (rrec) {
		P = hrx(hrec, RF_P);
		Pinv = hrb(hrec, RF_PINV);
		rgbo = hrv(hrec, RF_GBO);
		rpnp = hrv(hrec, RF_PNP);
		rsto.q = q4(hrf(hrec, RF_STO), hrf(hrec, RF_STO + 1), hrf(hrec, RF_STO + 2), hrf(hrec, RF_STO + 3));
		rsto.len[0] = hrf(hrec, RF_STO + 4);
		rsto.len[1] = hrf(hrec, RF_STO + 5);
		rsto.len[2] = hrf(hrec, RF_STO + 6);
		// read: the group's second wave may store the next step's record (test hook: a first wave
		// that stops posting after record help_drop, mbik_plan_debug_helper)
		if (t.help_drop < 0 || hseq <= t.help_drop) help_post(hfl, hseq);
	} else {
		if (flags & mbik::SR_PARENT_GLOBAL) {
			P = parent_global(t, sr, k, L, G);
		}
		Pinv = inverse(P.b);
	}
	const bool stab = STAB && (t.seg_flags[seg] & mbik::SF_STAB) != 0;
	const X3 Lprev = L.ld(b); // prev_transform (:136)
	for (int attempt = 0;; attempt++) {
	const int oe_mode = stab ? (attempt == 0 ? 1 : 2) : 0;
	X3 Lb = L.ld(b);
	X3 Gb;
	SlerpTo sto;
	if constexpr (HELP) {
		Gb = hrx(hrec, HF_GB);
	} else if (rrec) {
		// (a cooperative segment has two or more effectors: its headings read only Gb.o)
		Gb = X3{B3{}, rgbo};
		sto = rsto;
	} else {
		Gb = hasP ? P * Lb : Lb;
		sto = slerp_to(Gb.b);
	}
	const bool translate = (t.seg_flags[seg] & mbik::SF_TRANSLATE) != 0;
	const int e0 = t.seg_eff_off[seg], e1 = t.seg_eff_off[seg + 1];
	const int nh = t.seg_nh[seg];
	MBIK_PROF_T(ph0);
	MBIK_PROF_ADD(8, pt0, ph0);
	const double *hw = t.seg_hw + t.seg_hw_off[seg];

	if (!(STAB && t.constraint_mode)) { // constraint_mode is refused at plan creation
	// ---- QCP::weighted_superpose(tip headings, target headings, weights, translate) ----
	Q qrot;
	V3 translation = v3(0, 0, 0);
	Headings H;
	if (nh == 1) {
		// one heading in the segment: every lane of the group computes it (qcp.cpp:59-78)
		if (hoist) effector_headings<PM>(t, pre, d0, Gb, L, ST, SF, H, OE, oe_mode);
		else effector_headings<TA, PM>(t, t.seg_effs[e0], d0, Gb, L, TG, ST, SF, s, hw, H, OE, oe_mode);
		V3 mvd = H.hm[0], tgt = H.ht[0];
		if (translate) {
			double w = H.w[0];
			// move_to_weighted_center (qcp.cpp:139-160) accumulates from zero: 0 + p*w (a -0
			// component comes out +0)
			V3 mc = v3(0, 0, 0) + H.hm[0] * (float)w, tc = v3(0, 0, 0) + H.ht[0] * (float)w;
			if (w > 0) {
				mc = divs(mc, (float)w);
				tc = divs(tc, (float)w);
			}
			mvd = mvd + mc * -1.0f;
			tgt = tgt + tc * -1.0f;
			translation = tc - mc;
		}
		qrot = qcp_single<SEL>(mvd, tgt);
	} else if (XW && xs) {
		// Wave roles, cooperative segment: every effector's bone-direction global E comes from the
		// block's exchange area, where the group's waves left it after walking its path from this
		// step's Gb (coop_walk, the same products as effector_headings).  The headings are built
		// from E in the reference's effector order and summed as the one-lane branch below does,
		// so every sum rounds the same; a translating segment builds them twice, as
		// weighted_superpose does (qcp.cpp:220-248).
		// (the block's copy of the targets precedes the exchange area: [pin][12][64 lanes])
		const float *xe = xw + (size_t)t.seg_hbase[seg] * (12 * 64) + __lane_id();
		const float *xt = xw - (size_t)t.P * (12 * 64) + __lane_id();
		auto each = [&](auto &&use) __attribute__((always_inline)) {
			for (int i = e0; i < e1; i++) {
				const int e = t.seg_effs[i];
				EffPre p;
				eff_weights<PM>(t, e, hw + t.seg_eff_hoff[i], p);
				p.T = ld_x64(xt + (size_t)e * (12 * 64));
				const X3 E = ld_x64(xe + (size_t)(i - e0) * (12 * 64));
				Headings Hm;
				heading_terms<PM>(p, E, E.o, Gb.o, Hm);
#pragma unroll
				for (int h = 0; h < 7; h++)
					if (Hm.mask & (1 << h)) use(Hm.ht[h], Hm.hm[h], Hm.w[h]);
			}
		};
		V3 mc = v3(0, 0, 0), tc = v3(0, 0, 0);
		if (translate) {
			double wsum = 0;
			each([&](V3 ht, V3 hm, double w) __attribute__((always_inline)) {
				mc = mc + hm * (float)w;
				tc = tc + ht * (float)w;
				wsum += w;
			});
			if (wsum > 0) {
				mc = divs(mc, (float)wsum);
				tc = divs(tc, (float)wsum);
			}
			translation = tc - mc;
		}
		QSums S = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
		const V3 nmc = mc * -1.0f, ntc = tc * -1.0f;
		each([&](V3 ht, V3 hm, double w) __attribute__((always_inline)) {
			const V3 c1 = translate ? ht + ntc : ht, c2 = translate ? hm + nmc : hm;
			qcp_accumulate(S, c1 * (float)w, c1, c2, w);
		});
		qrot = qcp_adjugate(S);
	} else if (XS && xs) {
		// Split-exchange (staging 4 / 5; m >= 2, several effectors): lane j of the group builds
		// the headings of effectors e0+j, e0+j+m, ... with path sharing along its own sequence
		// (the depth it shares with its previous / next effector is the least shared depth of
		// the adjacent effectors in between: a lower bound on the true one, since shared path
		// depths form an ultrametric, so the reused product is a prefix of both paths).  Each
		// round the group's m effectors' headings go lane to lane (ds_bpermute), and every lane
		// consumes all of them in the reference's effector order, exactly as the one-lane
		// branch below does, so every sum rounds the same.  No staging memory.
		const int lb = (int)__lane_id() - j;
		// A translating segment builds every heading twice (centroids, then sums, as
		// weighted_superpose needs both): the first pass keeps each of this lane's effector
		// globals in the segment's staging area (build_schedule), the second rebuilds the
		// headings from them -- the same heading_terms of the same E, without walking the paths
		// again.  (State placement 2 only, where that area is device memory: build_schedule.)
		constexpr bool kXE = std::is_same_v<FP, BPtr<float>>;
		const int rounds = (e1 - e0 + m - 1) / m;
		const auto xe = HS + t.seg_hbase[seg] + 12 * rounds * j;
		auto each = [&](auto &&use, int pass) __attribute__((always_inline)) {
			PathCk pc;
			pc.d = -1;
			for (int i0 = e0, r = 0; i0 < e1; i0 += m, r++) {
				const int i = i0 + j;
				Headings Hm;
				if (i < e1 && pass == 2) {
					EffPre p;
					load_eff<TA, PM>(t, t.seg_effs[i], TG, s, hw + t.seg_eff_hoff[i], p);
					const X3 E = ld_x(xe + 12 * r);
					heading_terms<PM>(p, E, E.o, Gb.o, Hm);
				} else if (i < e1) {
					int lc[2] = {0, 0};
					if (i - m >= e0) {
						lc[0] = t.seg_eff_lcp[i];
						for (int u = i - m + 1; u < i; u++) lc[0] = min(lc[0], t.seg_eff_lcp[u]);
					}
					if (i + m < e1) {
						lc[1] = t.seg_eff_lcp[i + 1];
						for (int u = i + 2; u <= i + m; u++) lc[1] = min(lc[1], t.seg_eff_lcp[u]);
					}
					X3 E;
					effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], Hm, OE, oe_mode,
							PR ? &pc : nullptr, lc, pass == 1 ? &E : nullptr);
					if (pass == 1) st_x(xe + 12 * r, E);
				}
				auto take = [&](int v) __attribute__((always_inline)) {
					Headings H; // (weights and mask only)
					heading_weights<PM>(t, t.seg_effs[i0 + v], hw + t.seg_eff_hoff[i0 + v], H);
					const int src = lb + v;
#pragma unroll
					for (int h = 0; h < 7; h++) {
						if (H.mask & (1 << h)) {
							const V3 ht = v3(__shfl(Hm.ht[h].x, src), __shfl(Hm.ht[h].y, src), __shfl(Hm.ht[h].z, src));
							const V3 hm = v3(__shfl(Hm.hm[h].x, src), __shfl(Hm.hm[h].y, src), __shfl(Hm.hm[h].z, src));
							use(ht, hm, H.w[h]);
						}
					}
				};
				// the round's first two effectors peeled out of the loop, as the swing's cones are
				// (C3 -1.3 %, C4 -0.9 %, bitwise; profiles/r04_xs_take_peel_ab.jsonl)
				const int nv = min(m, e1 - i0);
				if (nv > 0) take(0);
				if (nv > 1) take(1);
				for (int v = 2; v < nv; v++) take(v);
			}
		};
		V3 mc = v3(0, 0, 0), tc = v3(0, 0, 0);
		if (translate) {
			double wsum = 0;
			each([&](V3 ht, V3 hm, double w) __attribute__((always_inline)) {
				mc = mc + hm * (float)w;
				tc = tc + ht * (float)w;
				wsum += w;
			}, kXE ? 1 : 0);
			wave_sync_lds(); // (this lane's own records: program order, made explicit for device memory)
			if (wsum > 0) {
				mc = divs(mc, (float)wsum);
				tc = divs(tc, (float)wsum);
			}
			translation = tc - mc;
		}
		QSums S = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
		const V3 nmc = mc * -1.0f, ntc = tc * -1.0f;
		each([&](V3 ht, V3 hm, double w) __attribute__((always_inline)) {
			V3 c1 = translate ? ht + ntc : ht;
			V3 c2 = translate ? hm + nmc : hm;
			qcp_accumulate(S, c1 * (float)w, c1, c2, w);
		}, kXE && translate ? 2 : 0);
		qrot = qcp_adjugate(S);
	} else if (m == 1 || nh == 0) {
		// Several headings (or none: a pinless root segment, whose sums stay zero), one lane or
		// every lane of the group alike; only nh >= 2 segments own a staged-heading LDS area
		// (build_schedule).  QCP::move_to_weighted_center (qcp.cpp:139-160, float)
		// and QCP::inner_product (:162-218, fp64) straight from registers, heading by heading
		// in the reference's order.  The translate case builds the headings twice, as the
		// reference's weighted_superpose does.
		V3 mc = v3(0, 0, 0), tc = v3(0, 0, 0);
		if (translate) {
			double wsum = 0;
			PathCk pc;
			pc.d = -1;
			for (int i = e0; i < e1; i++) {
				if (hoist) effector_headings<PM>(t, pre, d0, Gb, L, ST, SF, H, OE, oe_mode);
				else effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, oe_mode,
						PR ? &pc : nullptr, t.seg_eff_lcp + i);
#pragma unroll
				for (int h = 0; h < 7; h++) {
					if (H.mask & (1 << h)) {
						mc = mc + H.hm[h] * (float)H.w[h];
						tc = tc + H.ht[h] * (float)H.w[h];
						wsum += H.w[h];
					}
				}
			}
			if (wsum > 0) {
				mc = divs(mc, (float)wsum);
				tc = divs(tc, (float)wsum);
			}
			translation = tc - mc;
		}
		QSums S = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
		const V3 nmc = mc * -1.0f, ntc = tc * -1.0f;
		PathCk pc;
		pc.d = -1;
		auto one = [&](int i, auto tr) __attribute__((always_inline)) {
			MBIK_PROF_T(ph1);
			if (hoist) effector_headings<PM>(t, pre, d0, Gb, L, ST, SF, H, OE, oe_mode);
			else effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, oe_mode,
					PR ? &pc : nullptr, t.seg_eff_lcp + i);
			MBIK_PROF_T(ph2);
			MBIK_PROF_ADD(9, ph1, ph2);
#pragma unroll
			for (int h = 0; h < 7; h++) {
				if (H.mask & (1 << h)) {
					const double w = H.w[h];
					if constexpr (decltype(tr)::value) {
						const V3 c1 = H.ht[h] + ntc, c2 = H.hm[h] + nmc;
						qcp_accumulate(S, c1 * (float)w, c1, c2, w);
					} else {
						qcp_accumulate(S, H.ht[h] * (float)w, H.ht[h], H.hm[h], w);
					}
				}
			}
			MBIK_PROF_T(ph6);
			MBIK_PROF_ADD(14, ph2, ph6);
		};
		// Builds with the state in LDS or the locals in device memory: the translate test taken
		// out of the heading loop and the first effector peeled (C2 -0.7 %, C3 -1.3 %); the
		// all-state-in-device-memory build keeps the plain loop (C4 / C5 +0.7 % otherwise;
		// profiles/r04_one_lane_loop_ab.jsonl).
		if constexpr (!std::is_same_v<FP, BPtr<float>>) {
			if (translate) {
				for (int i = e0; i < e1; i++) one(i, std::true_type{});
			} else {
				if (e0 < e1) one(e0, std::false_type{});
				for (int i = e0 + 1; i < e1; i++) one(i, std::false_type{});
			}
		} else {
			for (int i = e0; i < e1; i++) {
				MBIK_PROF_T(ph1);
				if (hoist) effector_headings<PM>(t, pre, d0, Gb, L, ST, SF, H, OE, oe_mode);
				else effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, oe_mode,
						PR ? &pc : nullptr, t.seg_eff_lcp + i);
				MBIK_PROF_T(ph2);
				MBIK_PROF_ADD(9, ph1, ph2);
#pragma unroll
				for (int h = 0; h < 7; h++) {
					if (H.mask & (1 << h)) {
						const double w = H.w[h];
						V3 c1 = translate ? H.ht[h] + ntc : H.ht[h];
						V3 c2 = translate ? H.hm[h] + nmc : H.hm[h];
						qcp_accumulate(S, c1 * (float)w, c1, c2, w);
					}
				}
				MBIK_PROF_T(ph6);
				MBIK_PROF_ADD(14, ph2, ph6);
			}
		}
		MBIK_PROF_T(ph7);
		qrot = qcp_adjugate(S);
		MBIK_PROF_T(ph8);
		MBIK_PROF_ADD(10, ph7, ph8);
	} else {
		// Several headings, several lanes.  Every sum of QCP::move_to_weighted_center
		// (qcp.cpp:139-160, float) and QCP::inner_product (:162-218, fp64) is one accumulator
		// over the headings in the reference's order (effector-list order; origin, +axis,
		// -axis per prioritised axis), and the accumulators are independent of each other:
		//   1. lanes build their effectors' headings into the segment's LDS area, one
		//      12-float record per heading: the inner-product terms (9 products wc1_a*c2_b,
		//      dot(wc1,c1), dot(c2,c2)), or for translate the raw target/tip headings;
		//   2. translate only: lane j takes the centroid sums q = j, j+m, ... < 7; the results
		//      go through LDS and the lanes turn their records into centred terms;
		//   3. lane j takes the inner-product sums q = j, j+m, ... < 11, exchanged through LDS.
		// Each sum is accumulated in exactly the reference's order and rounding.
		const auto hsg = HS + t.seg_hbase[seg];
		const auto ex = rebind<double>(hsg + HS_REC * nh);
		for (int i = e0 + j; i < e1; i += m) {
			MBIK_PROF_T(ph1);
			effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, oe_mode);
			MBIK_PROF_T(ph2);
			MBIK_PROF_ADD(9, ph1, ph2);
			auto r = hsg + HS_REC * t.seg_eff_hoff[i];
#pragma unroll
			for (int h = 0; h < 7; h++) {
				if (H.mask & (1 << h)) {
					if (translate) {
						r[0] = H.ht[h].x; r[1] = H.ht[h].y; r[2] = H.ht[h].z;
						r[3] = H.hm[h].x; r[4] = H.hm[h].y; r[5] = H.hm[h].z;
					} else {
						qcp_terms(H.ht[h] * (float)H.w[h], H.ht[h], H.hm[h], r);
					}
					r += HS_REC;
				}
			}
		}
		wave_sync_lds();
		MBIK_PROF_T(ph5);
		if (translate) {
			// centroid sums: q 0-2 moved centre (tip headings), 3-5 target centre, 6 weight sum
			float fa0 = 0.0f, fa1 = 0.0f;
			double wacc = 0.0;
			const int q0 = j, q1 = j + m;
			const int o0 = q0 < 3 ? 3 + q0 : q0 - 3, o1 = q1 < 3 ? 3 + q1 : q1 - 3;
			const int p0 = q0 < 6 ? o0 : 0, p1 = q1 < 6 ? o1 : 0;
			int c = 0;
			for (; c + 4 <= nh; c += 4) { // 4 headings per LDS round trip
				const auto r = hsg + HS_REC * c;
				float x0[4], x1[4];
				double w[4];
#pragma unroll
				for (int u = 0; u < 4; u++) {
					x0[u] = r[HS_REC * u + p0];
					x1[u] = r[HS_REC * u + p1];
					w[u] = hw[c + u];
				}
#pragma unroll
				for (int u = 0; u < 4; u++) {
					const float wf = (float)w[u];
					fa0 = fa0 + x0[u] * wf;
					fa1 = fa1 + x1[u] * wf;
					wacc += w[u];
				}
			}
			for (; c < nh; c++) {
				const auto r = hsg + HS_REC * c;
				const double w = hw[c];
				const float wf = (float)w;
				fa0 = fa0 + r[p0] * wf;
				fa1 = fa1 + r[p1] * wf;
				wacc += w;
			}
			if (q0 < 6) ex[q0] = (double)fa0;
			if (q1 < 6) ex[q1] = (double)fa1;
			if (j == 0) ex[6] = wacc;
			if (m == 2) { // q = j + 4 (target centre y, z) as well
				float fa2 = 0.0f;
				for (int c = 0; c < nh; c++) fa2 = fa2 + hsg[HS_REC * c + j + 1] * (float)hw[c];
				ex[j + 4] = (double)fa2;
			}
			wave_sync_lds();
			V3 mc = v3((float)ex[0], (float)ex[1], (float)ex[2]);
			V3 tc = v3((float)ex[3], (float)ex[4], (float)ex[5]);
			const double wsum = ex[6];
			if (wsum > 0) {
				mc = divs(mc, (float)wsum);
				tc = divs(tc, (float)wsum);
			}
			translation = tc - mc;
			const V3 nmc = mc * -1.0f, ntc = tc * -1.0f;
			wave_sync_lds();
			for (int c = j; c < nh; c += m) {
				const auto r = hsg + HS_REC * c;
				const V3 c1 = v3(r[0], r[1], r[2]) + ntc;
				const V3 c2 = v3(r[3], r[4], r[5]) + nmc;
				qcp_terms(c1 * (float)hw[c], c1, c2, r);
			}
			wave_sync_lds();
		}
		// inner-product sums q = j + u*m < 11: q < 10 -> (double)term, q == 10 -> w * (double)term
		{
			double a0 = 0.0, a1 = 0.0, a2 = 0.0;
			const int q0 = j, q1 = j + m, q2 = j + 2 * m;
			const int i0 = q0 < 11 ? q0 : 0, i1 = q1 < 11 ? q1 : 0, i2 = q2 < 11 ? q2 : 0;
			int c = 0;
			for (; c + 4 <= nh; c += 4) { // 4 headings per LDS round trip
				const auto r = hsg + HS_REC * c;
				float x0[4], x1[4], x2[4];
				double w[4];
#pragma unroll
				for (int u = 0; u < 4; u++) {
					x0[u] = r[HS_REC * u + i0];
					x1[u] = r[HS_REC * u + i1];
					x2[u] = r[HS_REC * u + i2];
					w[u] = hw[c + u];
				}
#pragma unroll
				for (int u = 0; u < 4; u++) {
					a0 += q0 == 10 ? w[u] * (double)x0[u] : (double)x0[u];
					a1 += q1 == 10 ? w[u] * (double)x1[u] : (double)x1[u];
					a2 += q2 == 10 ? w[u] * (double)x2[u] : (double)x2[u];
				}
			}
			for (; c < nh; c++) {
				const auto r = hsg + HS_REC * c;
				const double w0 = hw[c];
				const float x0 = r[q0], x1 = r[q1 < 11 ? q1 : 0], x2 = r[q2 < 11 ? q2 : 0];
				a0 += q0 == 10 ? w0 * (double)x0 : (double)x0;
				a1 += q1 == 10 ? w0 * (double)x1 : (double)x1;
				a2 += q2 == 10 ? w0 * (double)x2 : (double)x2;
			}
			if (q0 < 11) ex[q0] = a0;
			if (q1 < 11) ex[q1] = a1;
			if (q2 < 11) ex[q2] = a2;
			if (m == 2) {
				// q = j + 6, j + 8, j + 10 as well
				double b0 = 0.0, b1 = 0.0, b2 = 0.0;
				const int p0 = j + 6, p1 = j + 8, p2 = j + 10;
				for (c = 0; c < nh; c++) {
					const auto r = hsg + HS_REC * c;
					const double w0 = hw[c];
					b0 += (double)r[p0];
					b1 += (double)r[p1];
					if (p2 < 11) b2 += w0 * (double)r[p2];
				}
				ex[p0] = b0;
				ex[p1] = b1;
				if (p2 < 11) ex[p2] = b2;
			}
		}
		wave_sync_lds();
		QSums S;
		S.xx = ex[0]; S.xy = ex[1]; S.xz = ex[2];
		S.yx = ex[3]; S.yy = ex[4]; S.yz = ex[5];
		S.zx = ex[6]; S.zy = ex[7]; S.zz = ex[8];
		S.ss1 = ex[9]; S.ss2 = ex[10];
		wave_sync_lds();
		MBIK_PROF_T(ph3);
		MBIK_PROF_ADD(14, ph5, ph3);
#ifdef MBIK_PROF
		if (translate) {
			MBIK_PROF_ADD(15, ph0, ph5);
			MBIK_PROF_ADD(16, ph5, ph3);
		}
#endif
		qrot = qcp_adjugate(S);
		MBIK_PROF_T(ph4);
		MBIK_PROF_ADD(10, ph3, ph4);
	}

	if constexpr (HELP) {
		MBIK_PROF_T(hb0);
		if (hfl) help_wait(hfl, HC_B, hseq + 1, *hstuck, t.help_timeout);
		MBIK_PROF_T(hb1);
		MBIK_PROF_ADD(19, hb0, hb1);
		P = hrx(hrec, HF_P);
		Pinv = hrb(hrec, HF_PINV);
		sto.q = q4(hrf(hrec, HF_STO), hrf(hrec, HF_STO + 1), hrf(hrec, HF_STO + 2), hrf(hrec, HF_STO + 3));
		sto.len[0] = hrf(hrec, HF_STO + 4);
		sto.len[1] = hrf(hrec, HF_STO + 5);
		sto.len[2] = hrf(hrec, HF_STO + 6);
	}
	MBIK_PROF_SET(pt1);
	MBIK_PROF_ADD(1, pt0, pt1);
	// ---- damp clamp, slerp(…, 0), rotate, translate, set_global_pose (:144-154) ----
	const double chd = t.seg_cos_half_damp[k];
	B3 rot = (kAblate & ABL_CONVERT) ? from_quat(qrot) : from_quat(clamp_cos_half(get_rotation_quaternion<SEL>(from_quat(qrot)), chd));
	MBIK_PROF_T(pc0);
	MBIK_PROF_ADD(11, pt1, pc0);
	if constexpr (!(kAblate & ABL_SLERP)) rot = slerp_weight0(rot, sto, t.libm);
	MBIK_PROF_T(pc1);
	MBIK_PROF_ADD(12, pc0, pc1);
	if (hasP) Lb.b = ((Pinv * rot) * P.b) * Lb.b;
	X3 Gn = hasP ? P * Lb : Lb;
	X3 result = {Gn.b, Gn.o + translation};
	// affine_inverse(P) with P.basis.inverse() already at hand (same arithmetic)
	if constexpr (HELP) Lb = hasP ? X3{Pinv, hrv(hrec, HF_PNP)} * result : result;
	else Lb = hasP ? X3{Pinv, rrec ? rpnp : xform(Pinv, -P.o)} * result : result;
	// set_global_pose propagates through b's subtree: pinned children's stale
	// bone-direction caches are refreshed from here on.
	// Every lane of the group holds identical values, so each writes its own copy (same
	// bytes) and later reads never depend on another lane's store ordering.
	// (Without stabilization nothing reads those flags before the step's end, where the stores
	// go instead: placed here, in device memory they were the stores the swing's and twist's
	// table loads then waited for -- vmcnt counts stores too.)
	if constexpr (STAB)
		for (int c = sr.w & 0xffff, ce = c + (sr.w >> 16); c < ce; c++) SF[t.bone_child_effs[c]] = 0;
	} else if (STAB && oe_mode == 1) {
		// constraint_mode still builds the target headings before the loop (:135)
		Headings H;
		const double *hw = t.seg_hw + t.seg_hw_off[seg];
		for (int i = t.seg_eff_off[seg] + j; i < t.seg_eff_off[seg + 1]; i += m)
			effector_headings<TA, PM>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, 1);
	}

	MBIK_PROF_T(pt2);
	MBIK_PROF_ADD(2, pt1, pt2);
#ifdef MBIK_PROF
	if (seg_translate) MBIK_PROF_ADD(17, pt1, pt2);
#endif
	// ---- Kusudama: orientation (swing) snap (ik_kusudama_3d.cpp:347-376) ----
	bool swung = false;
	X3 Gbd_stale;
	B3 GsB = {};     // P.basis * Lb.basis after the swing check, reused by the twist if not swung
	bool gs_ok = false;
	if (!(kAblate & ABL_SWING) && (flags & mbik::BF_ORIENT)) {
		X3 Gs = P * Lb;
		GsB = Gs.b;
		gs_ok = true;
		if constexpr (HELP) Gbd_stale.b = Gs.b * hrb(hrec, HF_DB);
		else Gbd_stale.b = Gs.b * ld_soa_basis<TA>(t, t.D, b, 9, 0, s);
		Gbd_stale.o = Gs.o;
		X3 Gco = {P.b, xform(P, Lb.o)}; // constraint_orientation: (I, pose local origin) under the parent
		V3 bdx = xform(Gbd_stale, v3(0.0f, 1.0f, 0.0f));
		V3 tip = xform(X3{Pinv, xform(Pinv, -Gco.o)}, bdx); // Gco.basis == P.basis
		double in_bounds = 1.0;
		V3 inl = local_point_in_limits<TA, SEL>(t, slot, s, tip, in_bounds);
		if (in_bounds < 0) {
			V3 p2 = xform(Gco, inl);
			Q rect = arc<SEL>(bdx - Gco.o, p2 - Gco.o);
			Lb.b = ((Pinv * from_quat(rect)) * P.b) * Lb.b;
			swung = true;
		}
	}
	MBIK_PROF_SET(pt3);
	MBIK_PROF_ADD(3, pt2, pt3);
	// ---- Kusudama: twist snap (ik_kusudama_3d.cpp:117-132) ----
	bool twist_changed = false;
	if (!(kAblate & ABL_TWIST) && (flags & mbik::BF_AXIAL)) {
		B3 gtc, gtci;
		float half_cos;
		if constexpr (HELP) {
			gtc = hrb(hrec, HF_GTC);
			gtci = hrb(hrec, HF_GTCI);
			half_cos = hrf(hrec, HF_HC);
		} else {
			const int cs = t.cf_stride;
			Q tcr = q4(soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q, s), soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 1, s),
					soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 2, s), soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_Q + 3, s));
			half_cos = soa<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_COS, s);
			B3 Tb = ld_soa_basis<TA>(t, t.CF, slot, cs, mbik::CF_TWIST_T, s);
			B3 Gct = P.b * Tb;
			gtc = Gct * from_quat(tcr);
		}
		X3 Gs;
		if (gs_ok && !swung) Gs.b = GsB;
		else Gs.b = P.b * Lb.b;
		if constexpr (!HELP) gtci = inverse(gtc);
		B3 align = orthonormalized<SEL>(gtci * Gs.b);
		Q sw, tw;
		swing_twist_y(get_rotation_quaternion<SEL>(align), sw, tw);
		tw = clamp_cos_half(tw, (double)half_cos);
		B3 recomposition = orthonormalized<SEL>(gtc * from_quat(sw * tw));
		B3 rotation = Pinv * recomposition;
		twist_changed = !eq(rotation, Lb.b);
		Lb.b = rotation;
	}
	{
		L.st(b, Lb);
		if constexpr (!STAB)
			for (int c = sr.w & 0xffff, ce = c + (sr.w >> 16); c < ce; c++) SF[t.bone_child_effs[c]] = 0;
		// A swing with no propagating twist leaves b's bone-direction cache stale until the
		// parent's set_global_pose (IKNode3D::rotate_local_with_global, ik_node_3d.cpp:56-67).
		if ((flags & mbik::BF_PINNED) && swung && !twist_changed) {
			const int e = t.bone_pin[b];
			st_x(ST + 12 * e, Gbd_stale);
			SF[e] = 1;
		}
	}
	if (!stab) break;
	{
		// _get_manual_msd(tip_headings_uniform, target_headings, weights) (:114-127): lanes
		// build their effectors' terms, every lane of the group sums them in heading order.
		wave_sync_lds();
		const X3 Gnow = hasP ? P * Lb : Lb;
		const double *hw = t.seg_hw + t.seg_hw_off[seg];
		Headings H;
		for (int i = t.seg_eff_off[seg] + j; i < t.seg_eff_off[seg + 1]; i += m) {
			const int e = t.seg_effs[i];
			effector_headings<TA, PM>(t, e, d0, Gnow, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, OE, 2);
#pragma unroll
			for (int h = 0; h < 7; h++) {
				if (H.mask & (1 << h)) {
					const V3 d = H.ht[h] - H.hm[h];
					MS[7 * e + h] = (float)(H.w[h] * (double)(d.x * d.x + d.y * d.y + d.z * d.z));
				}
			}
		}
		wave_sync_lds();
		float msd = 0.0f;
		for (int i = t.seg_eff_off[seg]; i < t.seg_eff_off[seg + 1]; i++) {
			const int e = t.seg_effs[i];
			msd += MS[7 * e];
#pragma unroll
			for (int a = 0; a < 3; a++) {
				if (t.eff_prio[3 * e + a] > 0.0f) {
					msd += MS[7 * e + 1 + 2 * a];
					msd += MS[7 * e + 2 + 2 * a];
				}
			}
		}
		msd /= t.seg_wsum2[seg];
		if ((double)msd <= prev_dev * 1.0001) {
			prev_dev = msd;
			break;
		}
		// reject: set_pose(prev_transform) -> IKNode3D::set_transform propagates only when the
		// local transform changes (ik_node_3d.cpp:69-75), refreshing b's subtree caches.
		if (!eq(Lb, Lprev)) {
			L.st(b, Lprev);
			if (flags & mbik::BF_PINNED) SF[t.bone_pin[b]] = 0;
			for (int c = sr.w & 0xffff, ce = c + (sr.w >> 16); c < ce; c++) SF[t.bone_child_effs[c]] = 0;
		}
		wave_sync_lds();
		if (attempt + 1 >= t.stab) break;
	}
	} // attempt loop
	MBIK_PROF_T(pt4);
	MBIK_PROF_ADD(4, pt3, pt4);
#ifdef MBIK_PROF
	if (seg_translate) MBIK_PROF_ADD(13, pt0, pt4);
#endif
}

// Iteration-start globals of one segment, root -> tip (IKNode3D::get_global_transform), with
// the next bone's index and local loaded before this bone's product and store (the helper
// wave's global pass is the solving wave's wait at each iteration start).
template <class LV, class GV>
__device__ void global_pass_pipelined(const DevPlan &t, int seg, const LV &L, const GV &G) {
	// two bones per trip, so the two local registers keep their roles (no 12-register rotation
	// per product); each product's successor local loads during it
	const int kb = t.seg_bone_off[seg], kt = t.seg_bone_off[seg + 1] - 1;
	const int b = t.seg_bones[kt];
	const int pp = t.bone_pose_parent[b];
	X3 La = L.ld(b);
	X3 Lb;
	int ga = t.bone_gslot[b], gb = -1;
	if (kt > kb) {
		const int bn = t.seg_bones[kt - 1];
		Lb = L.ld(bn);
		gb = t.bone_gslot[bn];
	}
	X3 Gprev = pp >= 0 ? G.ld(t.bone_gslot[pp]) * La : (pp == mbik::POSE_PARENT_ORIGIN ? xid() * La : La);
	if (ga >= 0) G.st(ga, Gprev);
	int k = kt - 1;
	for (; k > kb; k -= 2) { // bones k (in Lb) and k - 1
		const int bn = t.seg_bones[k - 1];
		La = L.ld(bn);
		ga = t.bone_gslot[bn];
		Gprev = Gprev * Lb;
		if (gb >= 0) G.st(gb, Gprev);
		if (k - 2 >= kb) {
			const int bm = t.seg_bones[k - 2];
			Lb = L.ld(bm);
			gb = t.bone_gslot[bm];
		}
		Gprev = Gprev * La;
		if (ga >= 0) G.st(ga, Gprev);
	}
	if (k == kb) {
		Gprev = Gprev * Lb;
		if (gb >= 0) G.st(gb, Gprev);
	}
}

// The same with the globals in device memory (state placement 2), kGpGroup bones at a time: a
// group's locals (and, first, the parent's checkpoint global) load together, one wait, then its
// products and stores.  gfx9's vmcnt counts stores as well as loads, and with both pending a wait
// can only be for all of them: in the pipelined pass every product waited for the previous
// bone's store (~2,000 cycles on a busy chip) before its local.  Same products, same order.
constexpr int kGpGroup = 4;
constexpr unsigned kWaitVm0 = 0x0F70; // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): gfx9 encoding
template <class LV, class GV>
__device__ void global_pass_grouped(const DevPlan &t, int seg, const LV &L, const GV &G) {
	const int kb = t.seg_bone_off[seg], kt = t.seg_bone_off[seg + 1] - 1;
	const int pp = t.bone_pose_parent[t.seg_bones[kt]];
	X3 Gprev;
	for (int k = kt; k >= kb; k -= kGpGroup) {
		X3 Lq[kGpGroup];
#pragma unroll
		for (int u = 0; u < kGpGroup; u++)
			if (k - u >= kb) Lq[u] = L.ld(t.seg_bones[k - u]);
		X3 Gp;
		if (k == kt && pp >= 0) Gp = G.ld(t.bone_gslot[pp]);
		__builtin_amdgcn_s_waitcnt(kWaitVm0);
#pragma unroll
		for (int u = 0; u < kGpGroup; u++) {
			if (k - u < kb) break;
			if (u == 0 && k == kt)
				Gprev = pp >= 0 ? Gp * Lq[0] : (pp == mbik::POSE_PARENT_ORIGIN ? xid() * Lq[0] : Lq[0]);
			else
				Gprev = Gprev * Lq[u];
			const int gs = t.bone_gslot[t.seg_bones[k - u]];
			if (gs >= 0) G.st(gs, Gprev);
		}
	}
}

// Iteration-start globals of one segment, root -> tip (IKNode3D::get_global_transform): the
// pipelined pass above (its products and stores, in the same order); placement 2 the grouped one.
template <class LV, class GV>
__device__ __forceinline__ void global_pass(const DevPlan &t, int seg, const LV &L, const GV &G) {
	if constexpr (std::is_same_v<GV, GTiled<BPtr<float>>>)
		global_pass_grouped(t, seg, L, G);
	else
		global_pass_pipelined(t, seg, L, G);
}

// Wave roles, cooperative segment (SCHED_XS): wave j of the segment's group of m waves walks the
// paths of the j-th contiguous run of the segment's effectors from bone-step k's Gb -- the
// parent's iteration-start global and the bone's local, exactly as bone_step forms them -- with
// path sharing along the run, and leaves each effector's bone-direction global E in the block's
// exchange area xw: [slot][12 floats][64 lanes], slot = seg_hbase[seg] + i - e0.
template <int TA, int PM, class LV, class GV, class FP, class IP>
__device__ void coop_walk(const DevPlan &t, int seg, int k, int j, int m, size_t s, const LV &L, const GV &G, const FP TG,
		const FP ST, const IP SF, float *xw) {
	const int4 sr = t.step_rec[k];
	const int b = sr.x & 0xffff;
	const int flags = sr.z & 0xffff;
	const int d0 = sr.z >> 16;
	X3 P = xid();
	if (flags & mbik::SR_PARENT_GLOBAL) {
		P = parent_global(t, sr, k, L, G);
	}
	const X3 Lb = L.ld(b);
	const X3 Gb = (flags & mbik::SR_HAS_POSE_PARENT) ? P * Lb : Lb;
	const int e0 = t.seg_eff_off[seg], e1 = t.seg_eff_off[seg + 1];
	const double *hw = t.seg_hw + t.seg_hw_off[seg];
	float *xe = xw + (size_t)t.seg_hbase[seg] * (12 * 64) + __lane_id();
	// a contiguous run of the segment's effectors per wave: neighbouring effectors (the fingers of
	// one arm) share the longest path prefixes, so the run reuses them (PathCk)
	const int ne = e1 - e0;
	const int i0 = e0 + (ne * j) / m, i1 = e0 + (ne * (j + 1)) / m;
	PathCk pc;
	pc.d = -1;
	for (int i = i0; i < i1; i++) {
		const int lc[2] = {i > i0 ? t.seg_eff_lcp[i] : 0, i + 1 < i1 ? t.seg_eff_lcp[i + 1] : 0};
		X3 E;
		Headings H; // (unused: the group's first wave builds the headings from E)
		effector_headings<TA, PM, true>(t, t.seg_effs[i], d0, Gb, L, TG, ST, SF, s, hw + t.seg_eff_hoff[i], H, TG, 0, &pc, lc, &E);
		float *r = xe + (size_t)(i - e0) * (12 * 64);
		r[0] = E.b.r[0].x; r[64] = E.b.r[0].y; r[128] = E.b.r[0].z;
		r[192] = E.b.r[1].x; r[256] = E.b.r[1].y; r[320] = E.b.r[1].z;
		r[384] = E.b.r[2].x; r[448] = E.b.r[2].y; r[512] = E.b.r[2].z;
		r[576] = E.o.x; r[640] = E.o.y; r[704] = E.o.z;
	}
}

// IKBone3D::set_skeleton_bone_pose (ik_bone_3d.cpp:170-179); returns whether the basis was
// non-finite (and replaced by the identity, :174-176).
template <bool SEL = false>
__device__ __forceinline__ bool write_pose(const X3 &t, float *out) {
	B3 b = t.b;
	const bool bad = !is_finite(b);
	if (bad) b = bid();
	Q q = get_rotation_quaternion<SEL>(b);
	V3 sc = get_scale(b);
	out[0] = q.x; out[1] = q.y; out[2] = q.z; out[3] = q.w;
	out[4] = t.o.x; out[5] = t.o.y; out[6] = t.o.z;
	out[7] = sc.x; out[8] = sc.y; out[9] = sc.z;
	return bad;
}
// A skeleton of a block whose helper-wave handshake timed out (help_wait): its solve used
// unfinished records, so every solved bone is written as a failure -- identity rotation, as
// for a non-finite basis (ik_bone_3d.cpp:174-176), NaN position so the result cannot pass for
// a pose, unit scale -- and the skeleton is flagged non-finite (mbik_solve_checked).
__device__ __forceinline__ bool write_help_timeout(float *out) {
	out[0] = 0.0f; out[1] = 0.0f; out[2] = 0.0f; out[3] = 1.0f;
	out[4] = NAN; out[5] = NAN; out[6] = NAN;
	out[7] = 1.0f; out[8] = 1.0f; out[9] = 1.0f;
	return true;
}
// The skeleton's non-finite flag: OR over the K lanes of its group, written by lane role 0.
__device__ __forceinline__ void write_nonfinite(const DevPlan &t, bool valid, bool bad, int g, int role, int local) {
	if (!t.nonfinite) return;
	const unsigned long long bits = __ballot(valid && bad);
	const unsigned long long mask = t.K >= 64 ? ~0ull : ((1ull << t.K) - 1ull);
	if (valid && role == 0) t.nonfinite[local] = ((bits >> (g * t.K)) & mask) != 0ull;
}
} // namespace
