// mbik_plan_autotune: times the launch layouts a plan can run (lanes, skeletons per block,
// checkpoint interval, heading staging, state placement, waves per SIMD, wave roles, the helper
// wave; constraint_mode's lane counts) on the caller's batch and keeps the fastest.  Every
// layout computes the same bits (tests/test_gpu_layouts.py); only the time differs.
#include <array>
#include <tuple>

#include "host.h"

using namespace mbik_host;

namespace {
// The layout settings a caller may pin, and what an autotune may change.  An autotune that fails,
// or that times nothing (no eligible candidate), leaves them as the caller set them.
struct Overrides {
	int lanes, spw, interval, staging, locals, waves, helper, roles, cm_lanes, cm_spw_div;
};
Overrides save_overrides(const mbik_plan *p) {
	return Overrides{p->lanes_override, p->spw_override, p->interval_override, p->staging_override, p->locals_override,
			p->waves_override, p->helper_override, p->roles_override, p->cm_lanes, p->cm_spw_div};
}
void restore_overrides(mbik_plan *p, const Overrides &o) {
	p->lanes_override = o.lanes;
	p->spw_override = o.spw;
	p->interval_override = o.interval;
	p->staging_override = o.staging;
	p->locals_override = o.locals;
	p->waves_override = o.waves;
	p->helper_override = o.helper;
	p->roles_override = o.roles;
	p->cm_lanes = o.cm_lanes;
	p->cm_spw_div = o.cm_spw_div;
	p->sched_K = -1;
}
constexpr int kNothingTimed = 1; // (internal: no candidate was eligible)
} // namespace
static int autotune_layouts(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out,
		hipStream_t st);

extern "C" {

// constraint_mode: every solve advances the persistent node caches (a frame), so the caches
// are saved first, each candidate lane count is timed from that saved state, and the state is
// put back: the caller's next frame sees the caches as they were.
static int cmode_autotune(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out,
		hipStream_t st) {
	if (p->lanes_override) return MBIK_OK; // pinned by mbik_plan_set_launch / set_layout
	mbik::HostPlan &h = p->host;
	// candidates: 1, 2, 4, ... up to the widest sibling level's power of two (the default K)
	mbik::build_schedule(h, 0, count, 0, 0, blocks_per_cu, p, p->cu_count);
	const int max_lanes = h.K;
	const size_t N = (size_t)h.N;
	const size_t node_bytes = node_area_floats(3 * h.B + 2 * h.NC, N) * sizeof(float);
	const size_t dirty_bytes = 4 * (size_t)p->cm.W * N * sizeof(uint32_t);
	void *save = nullptr;
	if (hipMalloc(&save, node_bytes + dirty_bytes) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc autotune state copy");
	char *sv = static_cast<char *>(save);
	auto copy = [&](bool to_save) {
		hipError_t a = to_save ? hipMemcpyAsync(sv, p->cm.node, node_bytes, hipMemcpyDeviceToDevice, st)
							   : hipMemcpyAsync(p->cm.node, sv, node_bytes, hipMemcpyDeviceToDevice, st);
		hipError_t b = to_save ? hipMemcpyAsync(sv + node_bytes, p->cm.dirty, dirty_bytes, hipMemcpyDeviceToDevice, st)
							   : hipMemcpyAsync(p->cm.dirty, sv + node_bytes, dirty_bytes, hipMemcpyDeviceToDevice, st);
		return a == hipSuccess && b == hipSuccess ? MBIK_OK : fail(MBIK_EHIP, "hipMemcpyAsync autotune state");
	};
	hipEvent_t e0, e1;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
		(void)hipFree(save);
		return fail(MBIK_EHIP, "hipEventCreate");
	}
	int rc = copy(true);
	float best_ms = 0.0f;
	int best = 0, best_div = 0, best_rw = 0;
	// classic: lanes per skeleton x skeletons per wave (full waves, or half: twice the waves per
	// SIMD for the node-cache misses to overlap); wave roles (cmode.h mbik_cmode_kernel_rw, plans
	// without stabilization, unless pinned off): 2, 4 or 8 roles x 64, 32 or 16 skeletons per block
	const int roles0 = p->roles_override;
	std::vector<std::array<int, 3>> cands; // lanes, spw div, wave roles
	if (roles0 != 1)
		for (int lanes = 1; lanes <= max_lanes && lanes <= 64; lanes <<= 1)
			for (int div = 0; div < 2; div++) cands.push_back({lanes, div, 0});
	if (roles0 != 0 && h.stabilization_passes == 0)
		for (int lanes = 2; lanes <= std::min(8, std::max(2, max_lanes)); lanes <<= 1)
			for (int div = 0; div < 3; div++) cands.push_back({lanes, div, 1});
	for (size_t ci = 0; ci < cands.size() && rc == MBIK_OK; ci++) {
		const int lanes = cands[ci][0], div = cands[ci][1];
		p->cm_lanes = lanes;
		p->cm_spw_div = div;
		p->roles_override = cands[ci][2];
		if ((rc = ensure_schedule(p, count)) != MBIK_OK) break;
		if (cands[ci][2] && !h.cm_roles) continue; // (not eligible: 64-bit addressing)
		float ms = 0.0f;
		for (int r = 0; r < 3 && rc == MBIK_OK; r++) { // first run warms up, untimed
			if ((rc = copy(false)) != MBIK_OK) break;
			(void)hipEventRecord(e0, st);
			rc = launch(p, first, count, pose_in, targets, pose_out, st, h.iterations, 0, h.NS - 1);
			(void)hipEventRecord(e1, st);
			if (rc == MBIK_OK && hipEventSynchronize(e1) != hipSuccess) rc = fail(MBIK_EHIP, "hipEventSynchronize");
			float t = 0.0f;
			(void)hipEventElapsedTime(&t, e0, e1);
			if (r > 0) ms += t;
		}
		if (rc == MBIK_OK && (best == 0 || ms < best_ms)) {
			best_ms = ms;
			best = lanes;
			best_div = div;
			best_rw = cands[ci][2];
		}
	}
	if (rc == MBIK_OK) rc = copy(false);
	if (rc == MBIK_OK && hipStreamSynchronize(st) != hipSuccess) rc = fail(MBIK_EHIP, "hipStreamSynchronize");
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	(void)hipFree(save);
	if (rc != MBIK_OK) return rc;
	if (best == 0) return kNothingTimed;
	p->cm_lanes = best;
	p->cm_spw_div = best_div;
	p->roles_override = best_rw;
	return ensure_schedule(p, count);
}

// A fully resident launch (the layout is fixed): with the helper wave left automatic, time the
// launch without and with it and keep the helper only if it is faster beyond the near-tie margin.
// The helper's second wave needs a free SIMD: at most two blocks of it per CU.
static int autotune_helper(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out,
		hipStream_t st) {
	if (p->helper_override != -1) return MBIK_OK;
	p->helper_override = 1;
	const int64_t blocks = (count + p->host.spw - 1) / p->host.spw;
	if (!helper_on(p) || blocks > 2 * (int64_t)p->cu_count) {
		p->helper_override = 0;
		return MBIK_OK;
	}
	hipEvent_t e0, e1;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return fail(MBIK_EHIP, "hipEventCreate");
	float ms[2] = {0.0f, 0.0f};
	int rc = MBIK_OK;
	for (int h = 0; h < 2 && rc == MBIK_OK; h++) {
		p->helper_override = h;
		if ((rc = launch(p, first, count, pose_in, targets, pose_out, st, p->host.iterations, 0, p->host.NS - 1)) != MBIK_OK) break;
		(void)hipEventRecord(e0, st);
		for (int r = 0; r < 3 && rc == MBIK_OK; r++)
			rc = launch(p, first, count, pose_in, targets, pose_out, st, p->host.iterations, 0, p->host.NS - 1);
		(void)hipEventRecord(e1, st);
		if (rc == MBIK_OK && hipEventSynchronize(e1) != hipSuccess) rc = fail(MBIK_EHIP, "hipEventSynchronize");
		(void)hipEventElapsedTime(&ms[h], e0, e1);
	}
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	if (rc == MBIK_OK) rc = take_helper_timeout(p);
	p->helper_override = rc == MBIK_OK && ms[1] * 1.015f < ms[0] ? 1 : 0;
	return rc;
}

int32_t mbik_plan_autotune(mbik_plan *p, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out, void *hip_stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (count <= 0) return MBIK_OK;
	{
		// every candidate is timed on the same input: an in-place call would advance the
		// caller's pose by one frame per timed run
		const size_t bytes = (size_t)count * p->host.B * 10 * sizeof(float);
		const char *a = reinterpret_cast<const char *>(pose_in), *b = reinterpret_cast<const char *>(pose_out);
		if (a && b && a < b + bytes && b < a + bytes) return fail(MBIK_EINVAL, "autotune needs pose_in and pose_out not to overlap");
	}
	DeviceGuard guard(p->device);
	hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
	const Overrides o0 = save_overrides(p);
	int rc = p->host.constraint_mode ? cmode_autotune(p, first, count, pose_in, targets, pose_out, st)
									 : autotune_layouts(p, first, count, pose_in, targets, pose_out, st);
	if (rc == kNothingTimed) {
		// nothing eligible was timed (e.g. wave roles pinned on a plan that cannot have them):
		// the caller's settings stand
		restore_overrides(p, o0);
		return ensure_schedule(p, count);
	}
	if (rc != MBIK_OK) {
		// a candidate failed: the plan goes back to the caller's settings, and the error stands
		const std::string err = g_err;
		restore_overrides(p, o0);
		(void)ensure_schedule(p, count);
		g_err = err;
	}
	return rc;
}

} // extern "C"

// The layout search of mbik_plan_autotune (plans without constraint_mode).
static int autotune_layouts(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out,
		hipStream_t st) {
	const int lanes = p->lanes_override;
	const int staging0 = p->staging_override;
	const int locals0 = p->locals_override;
	const int waves0 = p->waves_override;
	const int roles0 = p->roles_override;
	if (roles0 != 1) {
		// A launch whose skeletons are all resident at the default layout is bound by one
		// skeleton's dependency chain; no layout shortens that, so there is nothing to time.
		p->spw_override = 0;
		p->interval_override = 0;
		p->staging_override = staging0 < 0 ? 1 : staging0;
		p->locals_override = locals0 < 0 ? 0 : locals0;
		p->waves_override = waves0 < 0 ? 1 : waves0;
		p->roles_override = 0;
		int rc0 = ensure_schedule(p, count);
		if (rc0 != MBIK_OK) return rc0;
		if ((int64_t)blocks_per_cu(p, p->host.lds_block_bytes) * p->host.spw * p->cu_count >= count && p->host.g_interval == 1) {
			p->roles_override = roles0 < 0 ? 0 : roles0;
			return autotune_helper(p, first, count, pose_in, targets, pose_out, st);
		}
	}
	// Candidate layouts: for each heading-staging mode and checkpoint interval, the largest
	// skeletons-per-block at each distinct residency (blocks per CU).  Every layout computes
	// the same bits; only the time differs.
	// Lane counts: the pinned one, or the widest sibling level and half of it (two sibling
	// segments per lane: a longer chain, twice the skeletons per wave).
	// staging 2 (only translating root segments staged) differs from 0 only with such a
	// segment of several headings
	// (3: only segments of two or more effectors)
	bool has_staged_root = false, has_multi_eff = false;
	for (int sg = 0; sg < p->host.NS; sg++) {
		has_staged_root |= (p->host.seg_flags[sg] & mbik::SF_TRANSLATE) && p->host.seg_nh[sg] >= 2;
		has_multi_eff |= p->host.seg_eff_off[sg + 1] - p->host.seg_eff_off[sg] >= 2;
	}
	std::vector<int> lane_cands = {lanes};
	if (lanes == 0 && p->host.K >= 2) lane_cands.push_back(p->host.K / 2);
	std::vector<std::tuple<int, int, int, int, int, int, int>> cands; // (spw override, interval, staging, state placement, lanes, waves, wave roles)
	// Wave roles (one wave per role, a lane per skeleton, 64 per block): the widest sibling level
	// and its halves as the number of waves, within what a CU holds at the register budget.
	// (after the classic candidates, so that a near-tie keeps the classic layout)
	std::vector<std::tuple<int, int, int, int, int, int, int>> rw_cands;
	p->host.wave_roles = 0;
	if (roles0 != 0 && p->host.stabilization_passes == 0 && !p->host.constraint_mode) {
		mbik::build_schedule(p->host, 0, count, 0, 0, nullptr, nullptr, p->cu_count);
		const int widest = p->host.K;
		for (int wv : {1, 2}) {
			if (waves0 > 0 && wv != waves0) continue;
			for (int k : lanes > 0 ? std::vector<int>{lanes} : std::vector<int>{widest, widest / 2, widest / 4}) {
				if (k < 2 || k > 4 * wv) continue;
				for (int c : {1, 2}) rw_cands.push_back({0, c, 0, 2, k, wv, 1});
			}
		}
	}
	if (roles0 != 1)
	for (int wv : {1, 2}) {
	if (waves0 > 0 && wv != waves0) continue;
	if (wv == 2 && p->host.stabilization_passes > 0) continue;
	p->host.waves_per_simd = wv;
	for (int ln : lane_cands) {
		for (int lh : {0, 1, 2}) {
			if (locals0 >= 0 && lh != locals0) continue;
			// a second wave per SIMD only pays where LDS no longer bounds the blocks per CU
			if (wv == 2 && lh == 0 && locals0 < 0) continue;
			p->host.state_hbm = lh;
			bool nothing_staged = false;
			for (int stg : {1, 3, 2, 0, 4, 5}) {
				if (staging0 >= 0 && stg != staging0) continue;
				if (stg <= 3 && nothing_staged) continue;   // (the same layouts as the first)
				if (stg == 2 && !has_staged_root) continue; // (the same layouts as 0)
				if (stg == 3 && !has_multi_eff) continue;   // (the same layouts as 0)
				if (stg == 4 && !has_multi_eff) continue;   // (the same layouts as 0)
				if (stg == 5 && !(has_multi_eff && has_staged_root)) continue; // (as 4, or as 0)
				p->host.staging = stg;
				// with the whole state in device memory the interval does not change residency, only
				// the checkpoint writes against the rebuild products (C5: 2 is 0.7 % faster than 1)
				const std::vector<int> intervals = lh == 2 ? std::vector<int>{1, 2} : std::vector<int>{1, 2, 4, 1 << 20};
				for (int c : intervals) {
					int last_blocks = -1;
					bool split = true;
					for (int spw = 64; spw >= 1 && split; spw--) {
						mbik::build_schedule(p->host, ln, count, spw, c, blocks_per_cu, p, p->cu_count);
						// 4 / 5 with no segment split over lanes (one lane per skeleton) are 0 / 2
						if (stg >= 4 && !p->host.has_xs) {
							split = false;
							break;
						}
						if (p->host.spw != spw) continue; // capped by 64 / K or by LDS
						const int blocks = blocks_per_cu(p, p->host.lds_block_bytes);
						if (blocks != last_blocks) {
							cands.push_back({spw, c, stg, lh, ln, wv, 0});
							last_blocks = blocks;
						}
					}
				}
				if (stg <= 3 && p->host.hs_floats == 0) nothing_staged = true; // nothing is staged: 3, 2, 0 are the same
			}
		}
	}
	}
	cands.insert(cands.end(), rw_cands.begin(), rw_cands.end());
	hipEvent_t e0, e1;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return fail(MBIK_EHIP, "hipEventCreate");
	float best_ms = 0.0f;
	int best_spw = 0, best_c = 0, best_stg = 1, best_lh = 0, best_ln = lanes, best_wv = 1, best_rw = 0, rc = MBIK_OK;
	std::vector<std::tuple<int, int, int, int, int, int, int>> seen; // resolved (K, spw, interval, staging, locals, waves, roles)
	struct Timed {
		float ms;
		int spw, interval, stg, lh, ln, wv, rw;
	};
	std::vector<Timed> timed;
	for (auto [spw, c, stg, lh, ln, wv, rw] : cands) {
		p->spw_override = spw;
		p->interval_override = c;
		p->lanes_override = ln;
		p->staging_override = stg;
		p->locals_override = lh;
		p->waves_override = wv;
		p->roles_override = rw;
		if ((rc = ensure_schedule(p, count)) != MBIK_OK) {
			// a placement this batch cannot have (device memory, or the 4 GiB buffer limit) is skipped
			if (rc == MBIK_ENOMEM || rc == MBIK_EUNSUPPORTED) {
				rc = MBIK_OK;
				continue;
			}
			break;
		}
		const auto key = std::make_tuple(p->host.K, p->host.spw, p->host.g_interval, stg, lh, wv, (int)p->host.wave_roles);
		if (std::find(seen.begin(), seen.end(), key) != seen.end()) continue;
		seen.push_back(key);
		if ((rc = launch(p, first, count, pose_in, targets, pose_out, st, p->host.iterations, 0, p->host.NS - 1)) != MBIK_OK) break;
		(void)hipEventRecord(e0, st);
		for (int r = 0; r < 2 && rc == MBIK_OK; r++)
			rc = launch(p, first, count, pose_in, targets, pose_out, st, p->host.iterations, 0, p->host.NS - 1);
		if (rc != MBIK_OK) break;
		(void)hipEventRecord(e1, st);
		if (hipEventSynchronize(e1) != hipSuccess) {
			rc = fail(MBIK_EHIP, "hipEventSynchronize");
			break;
		}
		float ms = 0.0f;
		(void)hipEventElapsedTime(&ms, e0, e1);
		timed.push_back({ms, p->host.spw, p->host.g_interval, stg, lh, ln, wv, rw});
		if (best_c == 0 || ms < best_ms) {
			best_ms = ms;
			best_c = p->host.g_interval;
		}
	}
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	if (rc != MBIK_OK) return rc;
	if (timed.empty()) return kNothingTimed;
	// Near-ties go to the earliest candidate (a fixed order), not to run-to-run timing noise
	// (~1 %), so that boxes agree on the layout and per-layout evidence stays comparable.
	for (const Timed &c : timed)
		if (c.ms <= best_ms * 1.015f) {
			best_spw = c.spw;
			best_c = c.interval;
			best_stg = c.stg;
			best_lh = c.lh;
			best_ln = c.ln;
			best_wv = c.wv;
			best_rw = c.rw;
			break;
		}
	p->roles_override = best_rw;
	p->spw_override = best_spw;
	p->interval_override = best_c;
	p->staging_override = best_stg;
	p->locals_override = best_lh;
	p->lanes_override = best_ln;
	p->waves_override = best_wv;
	return ensure_schedule(p, count);
}
