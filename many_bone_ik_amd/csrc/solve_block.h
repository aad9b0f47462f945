// The solve of one workgroup (device code; included by the solve kernel TUs): the topology copy
// into LDS, the pose / target load, the iteration loop over the sibling-segment schedule in its
// three forms (classic lanes, helper wave, wave roles) and the pose write-back.
#pragma once
#include "bone_step.h"

namespace {

// One wave per block, and LDS caps residency at <= 4 blocks per CU (one wave per SIMD), so
// the kernel may use the whole register file (MBIK_WAVES_PER_EU 1: up to 512 VGPRs).
#ifndef MBIK_WAVES_PER_EU
#define MBIK_WAVES_PER_EU 1
#endif
// Wave roles: a cooperative row is block-synchronous (two barriers per bone-step), and while its
// first wave runs a step the rest of the block waits, so its waves are their block's critical
// path; a wave of the other block resident on the SIMD, in a row without barriers, has slack.
// The row's waves run it at raised issue priority (s_setprio; arbitration is priority, then
// age).  C4 -4.3 % against none (only the stepping wave raised: -2.6 %; the walks and the step
// raised to 2: -1.4 %), C5 within noise (same box, interleaved: profiles/r06_rw_priority_ab.txt).
// 0 = off.
#ifndef MBIK_RW_PRIO
#define MBIK_RW_PRIO 1
#endif
// Eight roles (MBIK_RW_PERM): a group of four or eight waves takes its record producer from
// role 2, whose wave runs on another SIMD than the stepping wave's (role 1 shares it).  C5
// -0.2 %, four of four interleaved reps (profiles/r06_rw_priority_ab.txt).
#ifndef MBIK_RW_PROD2
#define MBIK_RW_PROD2 1
#endif
// The solve of one block (blk = the plan-local block index after the XCD remap).
// Wave-uniform bone-step count of schedule row r: the longest segment among its tasks (the
// helper and the solving wave walk the same (row, step) sequence).  For a whole-plan solve it
// comes precomputed in the row's first task (.w >> 8, upload_topology): the K dependent table
// reads of the loop below sat in the helper's iteration-start path.
__device__ __forceinline__ int row_steps(const DevPlan &t, int r, int seg_lo, int seg_hi) {
	if (seg_lo == 0 && seg_hi >= t.NS - 1) return __builtin_amdgcn_readfirstlane(t.sched[r * t.K].w >> 8);
	int n = 0;
	for (int i = 0; i < t.K; i++) {
		const int sg = t.sched[r * t.K + i].x;
		if (sg >= seg_lo && sg <= seg_hi && sg >= 0) n = max(n, t.seg_bone_off[sg + 1] - t.seg_bone_off[sg]);
	}
	return __builtin_amdgcn_readfirstlane(n);
}

// RW (wave roles, HostPlan::wave_roles): the block is RW waves; lane = skeleton (64 per block),
// wave = the schedule's role, so every topology value a wave reads is uniform over it.
template <bool STAB, int PL, bool HOIST = true, bool T32 = true, bool HELP = false, bool XS = false, int PM = 0, int RW = 0>
__device__ __forceinline__ void solve_block(DevPlan &t, int blk, int first, int count, const float *__restrict__ pose_in,
		const float *__restrict__ targets, float *__restrict__ pose_out, int iterations, int seg_lo, int seg_hi) {
	static_assert(!HELP || (!STAB && PL == 0), "the helper wave serves placement-0 launches without stabilization");
	static_assert(!RW || (!STAB && !HELP && !XS && PL == 2), "wave roles: whole state in device memory, no stabilization");
	extern __shared__ float4 lds4[];
	const int lane = (HELP || RW) ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
	const int wave = HELP ? (int)(threadIdx.x >> 6) : RW ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
#ifdef MBIK_PROF
	uint64_t pfa[24] = {};
	uint64_t *pf = pfa;
#endif
	MBIK_PROF_T(pk0);
	{
		uint4 *dst = reinterpret_cast<uint4 *>(lds4);
		for (int i = (int)threadIdx.x; i < (t.topo_words >> 2); i += HELP ? 128 : RW ? 64 * RW : 64) dst[i] = t.topo_blob[i];
	}
	// several waves copied the blob: every wave reads all of it from here on (the pose load below
	// reads bone_flags), so the copy must be complete -- a one-wave block's own LDS writes are
	// ordered before its reads already
	if constexpr (HELP || RW > 1) __syncthreads();
	const uint32_t *topo = reinterpret_cast<const uint32_t *>(lds4);
#ifdef MBIK_TOPO_CONST
	// timing-only diagnostic build (tools/topo_const.py): one plan's table offsets compiled in, so
	// that no SGPR holds them; any other plan reads wrong tables
#include "topo_const.h"
#define MBIK_REPOINT(T, name) t.name = reinterpret_cast<const T *>(topo + MBIK_TC_##name);
#else
#define MBIK_REPOINT(T, name) t.name = reinterpret_cast<const T *>(topo + t.o_##name);
#endif
	MBIK_TOPO_TABLES(MBIK_REPOINT)
#undef MBIK_REPOINT
	float *lds = reinterpret_cast<float *>(lds4) + t.topo_words;
	if constexpr (kAblate & ABL_SOALDS) {
		float *dl = lds + (size_t)t.spw * t.lds_stride;
		float *cl = dl + t.B * 9;
		double *xl = reinterpret_cast<double *>(cl + ((t.NC * t.cf_stride + 1) & ~1));
		for (int i = lane; i < t.B * 9; i += 64) dl[i] = t.D[(size_t)i * t.N + first];
		for (int i = lane; i < t.NC * t.cf_stride; i += 64) cl[i] = t.CF[(size_t)i * t.N + first];
		for (int i = lane; i < t.NC * t.cd_stride; i += 64) xl[i] = t.CD[(size_t)i * t.N + first];
		t.D = dl; t.CF = cl; t.CD = xl; t.N = 1;
	}
	const int g = RW ? lane : lane >> t.log2K;
	// (MBIK_RW_PERM, plan.h: the role of each wave)
	const int role = RW ? ((RW == 8 && MBIK_RW_PERM) ? 2 * (wave & 3) + (wave >> 2) : wave) : lane & (t.K - 1);
	const int local = blk * t.spw + g;
	const bool valid = g < t.spw && local < count;
	const size_t s = (size_t)first + (size_t)(valid ? local : 0);
	const int B = t.B, P = t.P, K = RW ? RW : t.K;
	// PL (HostPlan::state_hbm): 0 the state in LDS; 1 the locals in device memory (L2-resident
	// during the launch), the rest in LDS; 2 all of it in device memory
	// FP / IP: the float / int state pointers: LDS, or for PL 2 BPtr into device memory.  (PL 1
	// keeps 64-bit pointers to its locals: in its two-wave build, C3's pick, the buffer form
	// spilled more, not less.)
	using FP = std::conditional_t<PL == 2, BPtr<float>, float *>;
	using IP = std::conditional_t<PL == 2, BPtr<int>, int *>;
	using LV = std::conditional_t<PL >= 1, LocTiled<FP>, LocContig>;
	using GV = std::conditional_t<PL == 2, GTiled<FP>, GFlat<FP>>;
	LV L;
	GV G;
	FP S0; // the skeleton's state after its locals (placement 2: and after its checkpoint globals)
	const size_t loc0 = (s / kLocTile) * (size_t)(12 * kLocTile) * B + (s % kLocTile) * 4;
	if constexpr (PL == 2) L.p = bptr<float>(t.Lg, t.lg_bytes, (uint32_t)(loc0 * sizeof(float)), 0u, t.lg_bytes);
	else if constexpr (PL == 1) L.p = t.Lg + loc0;
	if constexpr (PL == 2) {
		const uint32_t sb = (uint32_t)(s * (size_t)t.state_stride * sizeof(float));
		S0 = bptr<float>(t.Sg, t.sg_bytes, sb, sb, sb + (uint32_t)(t.state_stride * sizeof(float)));
		const size_t g0 = (s / kLocTile) * (size_t)(12 * kLocTile) * t.n_gck + (s % kLocTile) * 4;
		G.p = bptr<float>(t.Gg, t.gg_bytes, (uint32_t)(g0 * sizeof(float)), 0u, t.gg_bytes);
	} else if constexpr (PL == 1) {
		S0 = lds + (size_t)g * t.lds_stride;
		G.p = S0;
	} else {
		L.p = lds + (size_t)g * t.lds_stride;
		S0 = L.p + 12 * B;
		G.p = S0;
	}
	const FP TG = uplus(S0, PL == 2 ? 0 : 12 * t.n_gck);
	const FP ST = uplus(TG, 12 * P);
	const FP HS = uplus(ST, 12 * P);               // staged headings (t.seg_hbase), 16-B aligned
	const IP SF = rebind<int>(uplus(HS, t.hs_floats));
	constexpr int TA = PL == 2 ? kTabTiled : (T32 ? kTab32 : kTab64); // placement 2 reads the tiled table copy
	const FP OE = rebind<float>(uplus(SF, P));    // stabilization only: 3 per pin
	const FP MS = uplus(OE, 3 * P);              // stabilization only: 7 per pin
	// wave roles: the block's 64 non-finite flags after the topology (write_nonfinite), then the
	// cooperative segments' effector-global exchange area (coop_walk)
	int *nf_rw = RW ? reinterpret_cast<int *>(lds) : nullptr;
	// (a plan with cooperative rows keeps the block's targets in LDS too, [pin][12][64], before
	// the exchange area: the cooperative consumer reads them for every effector at every step)
	float *xt = RW ? lds + 64 : nullptr;
	float *xw = RW ? xt + (t.rw_xslots ? (size_t)t.P * (12 * 64) : 0) : nullptr;
	// (then the cooperative groups' parent-side records, kRwRecF4 float4 x 64 lanes each, K / 2 of
	// them: rw_record; then one counter per group and the block's gave-up word: rw_wait)
	float4 *xr4 = RW ? reinterpret_cast<float4 *>(xw + (size_t)t.rw_xslots * (12 * 64)) : nullptr;
	int *rw_cnt = RW ? reinterpret_cast<int *>(xr4 + (K / 2) * (mbik::kRwRecF4 * 64)) : nullptr;
	bool rw_stuck = false; // this wave gave up waiting for its group's first wave (rw_wait)
	if constexpr (RW) {
		if (threadIdx.x < 64) nf_rw[threadIdx.x] = 0;
		if (t.rw_xslots && threadIdx.x <= K / 2) rw_cnt[threadIdx.x] = 0; // counters, gave-up word
	}
	if (valid && (RW || wave == 0)) {
		for (int b = role; b < B; b += K)
			if (t.bone_flags[b] & mbik::BF_IN_LIST) L.st(b, pose_to_xform(pose_in + ((size_t)local * B + b) * 10));
		for (int e = role; e < P; e += K) {
			const float *src = targets + ((size_t)local * P + e) * 12;
			for (int f = 0; f < 12; f++) TG[12 * e + f] = src[f];
			if constexpr (RW > 0)
				if (t.rw_xslots)
					for (int f = 0; f < 12; f++) xt[((size_t)e * 12 + f) * 64 + lane] = src[f];
			SF[e] = 0;
		}
	}
	float4 *ring = nullptr;
	int *hfl = nullptr; // HelpCounter: records produced (part A, part B), consumed, iterations finished, gave up
	bool help_stuck = false; // this block's waves gave up waiting for each other (help_wait)
	if constexpr (HELP) {
		ring = reinterpret_cast<float4 *>(lds + (size_t)t.spw * t.lds_stride) + lane;
		hfl = reinterpret_cast<int *>(reinterpret_cast<float4 *>(lds + (size_t)t.spw * t.lds_stride) + kHelpSlots * kHelpF4 * 64);
		if (threadIdx.x < 8) hfl[threadIdx.x] = 0;
	}
	__syncthreads();
	MBIK_PROF_T(pk1);
	MBIK_PROF_ADD(0, pk0, pk1);
	if constexpr (HELP) {
		if (wave == 1) {
			// the helper: per iteration the global pass, then every bone-step's record in the
			// solving wave's (row, step) order, at most kHelpSlots ahead of it.  The first
			// record's table rows load before the wait for the iteration's end (they are
			// per-skeleton constants), so that record costs only its arithmetic.
			int seq = 0, slot = 0;
			bool stuck = false;
			const int4 task0 = t.sched[role];
			const bool act0 = valid && task0.x >= seg_lo && task0.x <= seg_hi;
			for (int it = 0; it < iterations; it++) {
				const HelpRows first_rows = help_rows<kTab32>(t, act0 ? t.seg_bone_off[task0.x] : 0, s);
				help_wait(hfl, HC_ITER, it, stuck, t.help_timeout);
				MBIK_PROF_T(hg0);
				for (int r = t.nrows - 1; r >= 0; r--) {
					const int4 task = t.sched[r * K + role];
					if (valid && task.x >= 0 && task.y == 0) global_pass_pipelined(t, task.x, L, G);
					wave_sync_lds();
				}
				MBIK_PROF_T(hg1);
				MBIK_PROF_ADD(21, hg0, hg1);
				for (int r = 0; r < t.nrows; r++) {
					const int4 task = t.sched[r * K + role];
					const bool act = valid && task.x >= seg_lo && task.x <= seg_hi;
					const int k0 = act ? t.seg_bone_off[task.x] : 0, k1 = act ? t.seg_bone_off[task.x + 1] : 0;
					const int nq = row_steps(t, r, seg_lo, seg_hi);
					for (int q = 0; q < nq; q++, seq++) {
						const HelpRows rw = (r == 0 && q == 0) ? first_rows : help_rows<kTab32>(t, k0 + q < k1 ? k0 + q : 0, s);
						if (seq == t.help_drop) return; // test hook (mbik_plan_debug_helper): a helper that dies
						help_wait(hfl, HC_CONSUMED, seq - kHelpSlots + 1, stuck, t.help_timeout);
						float4 *rec = ring + slot * (kHelpF4 * 64);
						X3 P;
						B3 Gbb;
						if (k0 + q < k1) help_part_a(t, k0 + q, L, G, rec, P, Gbb);
						help_post(hfl, seq + 1);
#ifdef MBIK_PROF
						if (r == 0 && q == 0) {
							MBIK_PROF_T(hg2);
							MBIK_PROF_ADD(22, hg1, hg2);
						}
#endif
						if (k0 + q < k1) help_part_b(t, k0 + q, P, Gbb, rw, rec);
#ifdef MBIK_REPLAY
						if (t.replay == 1)
							for (int i = 0; i < kHelpF4; i++)
								t.rec_dump[((size_t)blk * t.rec_per_block + seq) * kHelpF4 * 64 + (size_t)i * 64 + lane] = rec[i * 64];
#endif
						help_post(hfl + 1, seq + 1);
						slot = slot + 1 == kHelpSlots ? 0 : slot + 1;
					}
				}
			}
#ifdef MBIK_PROF
			if (lane == 0)
				for (int i = 20; i < 24; i++) atomicAdd(&g_mbik_prof[i], (unsigned long long)pfa[i]);
#endif
			return;
		}
		int seq = 0, slot = 0;
		bool stuck = false;
#ifdef MBIK_REPLAY
		// replay: no partner to wait for (stuck skips every wait); records come from rec_dump
		const float4 *rp = t.replay == 2 ? t.rec_dump + (size_t)blk * t.rec_per_block * kHelpF4 * 64 + lane : nullptr;
		if (rp) stuck = true;
#endif
		for (int it = 0; it < iterations; it++) {
			for (int r = 0; r < t.nrows; r++) {
				const int4 task = t.sched[r * K + role];
				const bool act = valid && task.x >= seg_lo && task.x <= seg_hi;
				const int seg = act ? task.x : 0;
				const int k0 = act ? t.seg_bone_off[seg] : 0, k1 = act ? t.seg_bone_off[seg + 1] : 0;
				const int nq = row_steps(t, r, seg_lo, seg_hi);
				double prev_dev = INFINITY;
				const int e0 = t.seg_eff_off[seg];
				EffPre pre;
				const bool hoist = act && t.seg_eff_off[seg + 1] - e0 == 1 && (task.z == 1 || t.seg_nh[seg] == 1);
				if (hoist) load_eff<kTab32>(t, t.seg_effs[e0], TG, s, t.seg_hw + t.seg_hw_off[seg] + t.seg_eff_hoff[e0], pre);
				for (int q = 0; q < nq; q++, seq++) {
					MBIK_PROF_T(hw0);
					bool b_ready;
					help_wait_ab(hfl, seq + 1, stuck, b_ready, t.help_timeout);
					MBIK_PROF_T(hw1);
					MBIK_PROF_ADD(18, hw0, hw1);
#ifdef MBIK_PROF
					if (r == 0 && q == 0) MBIK_PROF_ADD(20, hw0, hw1);
#endif
					const float4 *hrec = ring + slot * (kHelpF4 * 64);
#ifdef MBIK_REPLAY
					if (rp) hrec = rp + (size_t)seq * kHelpF4 * 64;
#endif
					if (k0 + q < k1)
						bone_step<false, true, kTab32, true, false, PM, true, false>(t, seg, k0 + q, task.y, task.z, task.w & mbik::SCHED_XS, s, L, G, TG,
								ST, SF, HS, OE, MS, prev_dev, pre, hoist, hrec, b_ready ? nullptr : hfl, seq, &stuck, nullptr MBIK_PROF_ARG);
					help_post(hfl + 2, seq + 1);
					slot = slot + 1 == kHelpSlots ? 0 : slot + 1;
				}
				wave_sync_lds();
			}
			help_post(hfl + 3, it + 1);
		}
		// (the helper raises HC_STUCK before any record it writes without waiting, so a record
		// this wave read from an overwritten slot is covered by the flag read here)
		help_stuck = stuck || __builtin_amdgcn_readfirstlane(__hip_atomic_load(hfl + HC_STUCK, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
#ifdef MBIK_REPLAY
		if (rp) help_stuck = false;
#endif
	} else
	for (int it = 0; it < iterations; it++) {
		MBIK_PROF_T(pg0);
		for (int r = t.nrows - 1; r >= 0; r--) {
			const int4 task = t.sched[r * K + role];
			if (valid && task.x >= 0 && task.y == 0) global_pass(t, task.x, L, G);
			__syncthreads();
		}
		MBIK_PROF_T(pg1);
		MBIK_PROF_ADD(5, pg0, pg1);
		for (int r = 0; r < t.nrows;) {
			if constexpr (RW) {
				if (t.sched[r * K].w & mbik::SCHED_COOP) {
					// A row with cooperative segments: per bone-step, the groups' waves walk their
					// effectors' paths (coop_walk) and meet; each group's first wave -- and each wave
					// of a segment solved alone -- runs the step; the block meets again before the
					// next step walks from the bones just solved.  Every wave runs the row's step
					// count, so the barriers match.  Meanwhile a group's second wave computes the next
					// step's parent-side record (rw_record): the first wave reads its record at the
					// start of its step and posts that in the group's LDS counter, and the second wave
					// stores the next record once the counter shows it (rw_wait; the first step's
					// record is stored before the row's first walk).
					const int4 task = t.sched[r * K + role];
					const bool act = valid && task.x >= seg_lo && task.x <= seg_hi;
					const int seg = task.x >= 0 ? task.x : 0;
					const int k0 = t.seg_bone_off[seg], k1 = task.x >= 0 ? t.seg_bone_off[seg + 1] : k0;
					const bool coop = (task.w & mbik::SCHED_XS) != 0;
					const int nq = row_steps(t, r, seg_lo, seg_hi);
					double prev_dev = INFINITY;
					EffPre pre;
					const int e0 = t.seg_eff_off[seg];
					const bool hoist = HOIST && act && !coop && t.seg_eff_off[seg + 1] - e0 == 1;
					if (hoist) load_eff<TA>(t, t.seg_effs[e0], TG, s, t.seg_hw + t.seg_hw_off[seg] + t.seg_eff_hoff[e0], pre);
					// the group's record and counter: the groups of a row have equal sizes, so the
					// group is its first wave's index / m (the wave's task is uniform: readfirstlane
					// makes the role branches scalar)
					const int ty = __builtin_amdgcn_readfirstlane(task.y);
					const bool rec_on = coop;
					const int grp = rec_on ? (role - ty) / __builtin_amdgcn_readfirstlane(task.z) : 0;
					float4 *rec = rec_on ? xr4 + grp * (mbik::kRwRecF4 * 64) + lane : nullptr;
					int *rcnt = rec_on ? rw_cnt + grp : nullptr;
					const bool leader = ty == 0;
					const bool producer = rec_on && ty == ((MBIK_RW_PROD2 && RW == 8 && MBIK_RW_PERM && task.z >= 4) ? 2 : 1);
					if (leader && rec_on) *rcnt = 0; // (read only after the row's first barrier)
					if (producer && act && k0 < k1) rw_record_store(rec, rw_record(t, k0, L, G));
					// (MBIK_PROF, wave roles: 18 packed / plain rows, 19 coop_walk, 21 waiting at the
					// cooperative rows' barriers, 22 the steps run after them, 23 cooperative rows)
					MBIK_PROF_T(cr0);
					if constexpr (MBIK_RW_PRIO > 0) __builtin_amdgcn_s_setprio(MBIK_RW_PRIO);
					for (int q = 0; q < nq; q++) {
						const bool step = act && k0 + q < k1;
						MBIK_PROF_T(c0);
						if (coop && step) coop_walk<TA, PM>(t, seg, k0 + q, task.y, task.z, s, L, G, TG, ST, SF, xw);
						MBIK_PROF_T(c1);
						MBIK_PROF_ADD(19, c0, c1);
						__syncthreads();
						MBIK_PROF_T(c2);
						MBIK_PROF_ADD(21, c1, c2);
						if (leader) {
							if (step)
								bone_step<false, true, TA, false, false, PM, HOIST, true>(t, seg, k0 + q, 0, 1, coop ? 1 : 0, s, L, G, TG, ST,
										SF, HS, OE, MS, prev_dev, pre, hoist, rec, rcnt, q + 1, nullptr, xw MBIK_PROF_ARG);
						} else if (producer && act && k0 + q + 1 < k1) {
							// the next step's record, stored once the first wave has read this step's
							const RwRec next = rw_record(t, k0 + q + 1, L, G);
							rw_wait(rcnt, q + 1, rw_stuck, rw_cnt + K / 2, t.help_timeout);
							rw_record_store(rec, next);
						}
						MBIK_PROF_T(c3);
						MBIK_PROF_ADD(22, c2, c3);
						__syncthreads();
						MBIK_PROF_T(c4);
						MBIK_PROF_ADD(21, c3, c4);
					}
					if constexpr (MBIK_RW_PRIO > 0) __builtin_amdgcn_s_setprio(0);
					MBIK_PROF_T(cr1);
					MBIK_PROF_ADD(23, cr0, cr1);
					r++;
					continue;
				}
			}
			MBIK_PROF_T(pr0);
			// rows r .. r1-1: one row, or a packed level (SCHED_CHAIN rows, build_schedule) whose
			// lanes each run their sequence of segments back to back, without a barrier
			int r1 = r + 1;
			while (r1 < t.nrows && (t.sched[r1 * K].w & mbik::SCHED_CHAIN)) r1++;
			int rr = r - 1, k = 0, ke = 0, seg = 0;
			int4 task = make_int4(-1, 0, 1, 0);
			double prev_dev = INFINITY;
			EffPre pre;
			bool hoist = false;
			for (;;) {
				while (k >= ke && rr + 1 < r1) {
					task = t.sched[++rr * K + role];
					if (valid && task.x >= seg_lo && task.x <= seg_hi) {
						seg = task.x;
						k = t.seg_bone_off[seg];
						ke = t.seg_bone_off[seg + 1];
						prev_dev = INFINITY; // reset after the segment root bone (:178-180)
						// A single-effector segment solved by one lane (or with a single heading)
						// reads the same effector data at every bone-step: load it once for the segment.
						// (not in the two-waves-per-SIMD build: the hoisted data's ~66 registers are
						// what push that build past 256 and into scratch spills)
						const int e0 = t.seg_eff_off[seg];
						hoist = HOIST && !STAB && t.seg_eff_off[seg + 1] - e0 == 1 && (task.z == 1 || t.seg_nh[seg] == 1);
						if (hoist) load_eff<TA>(t, t.seg_effs[e0], TG, s, t.seg_hw + t.seg_hw_off[seg] + t.seg_eff_hoff[e0], pre);
					}
				}
				if (k >= ke) break;
				bone_step<STAB, HOIST || PL == 2, TA, false, XS, PM, HOIST, false>(t, seg, k, task.y, task.z, task.w & mbik::SCHED_XS, s, L, G, TG,
						ST, SF, HS, OE, MS, prev_dev, pre, hoist, nullptr, nullptr, 0, nullptr, nullptr MBIK_PROF_ARG);
				k++;
			}
			__syncthreads();
			MBIK_PROF_T(pr1);
			MBIK_PROF_ADD(18, pr0, pr1);
			r = r1;
		}
	}
	if constexpr (RW) {
		// a wave that gave up in rw_wait raised the block's word before the row's last barrier
		if (t.rw_xslots)
			help_stuck = __builtin_amdgcn_readfirstlane(__hip_atomic_load(rw_cnt + K / 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
	}
	MBIK_PROF_T(pk2);
	bool bad = false;
	if (valid) {
		for (int b = role; b < B; b += K) {
			float *dst = pose_out + ((size_t)local * B + b) * 10;
			if (t.bone_flags[b] & mbik::BF_IN_LIST) {
				if (help_stuck) bad = write_help_timeout(dst);
				else bad |= write_pose<HOIST>(L.ld(b), dst);
			} else {
				const float *src = pose_in + ((size_t)local * B + b) * 10;
				for (int f = 0; f < 10; f++) dst[f] = src[f];
			}
		}
	}
	if constexpr (RW) {
		// a skeleton's bones are written by all K waves: their flags meet in LDS
		if (valid && bad) nf_rw[lane] = 1;
		__syncthreads();
		if (t.nonfinite && valid && wave == 0) t.nonfinite[local] = nf_rw[lane] != 0;
	} else {
		write_nonfinite(t, valid, bad, g, role, local);
	}
	if (help_stuck && lane == 0 && t.help_flag) __hip_atomic_store(t.help_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	MBIK_PROF_T(pk3);
	MBIK_PROF_ADD(6, pk2, pk3);
	MBIK_PROF_ADD(7, pk0, pk3);
#ifdef MBIK_PROF
	if (lane == 0)
		for (int i = 0; i < 24; i++) atomicAdd(&g_mbik_prof[i], (unsigned long long)pfa[i]);
#endif
}

// XCD-aware block order: the hardware deals consecutive blocks round-robin to the 8 XCDs
// (separate L2s), so hand each XCD a contiguous run of skeletons; SoA plan rows of
// neighbouring skeletons then share cache lines in one L2 instead of eight.
__device__ __forceinline__ int xcd_block() {
	const int nb = gridDim.x, nb8 = nb & ~7, bx = blockIdx.x;
	if constexpr (kAblate & ABL_XCD) return bx;
	return bx < nb8 ? (bx & 7) * (nb8 >> 3) + (bx >> 3) : bx;
}
} // namespace

namespace {
// WPE: waves per SIMD the register budget is sized for.  1 (the default): the whole register
// file, no spills.  2: at most 256 registers, some spilled to scratch, but two one-wave
// blocks share a SIMD -- for launches whose skeletons no longer fit the chip at once and
// whose state is not in LDS (mbik_plan_set_waves_per_simd; autotune decides).
// XS: the build with split-exchange segments (staging 4 / 5; two waves per SIMD only), a separate
// instantiation so the other builds keep their register allocation.
// PM: kPrioDefault for plans whose effectors all have the reference's default priorities
// (DevPlan::prio_mask), a separate instantiation with compile-time heading slots; else 0.
template <bool STAB, int PL, int WPE = MBIK_WAVES_PER_EU, bool T32 = true, bool XS = false, int PM = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mbik_solve_kernel(DevPlan t, int first, int count, const float *__restrict__ pose_in,
		const float *__restrict__ targets, float *__restrict__ pose_out, int iterations, int seg_lo, int seg_hi) {
	solve_block<STAB, PL, WPE == 1, T32, false, XS, PM>(t, xcd_block(), first, count, pose_in, targets, pose_out, iterations, seg_lo, seg_hi);
}
} // namespace
