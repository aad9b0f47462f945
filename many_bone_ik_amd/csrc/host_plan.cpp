// The C ABI's core (include/mbik.h): plan creation and upload, the launch layout
// (ensure_schedule), kernel selection and launch, the solve entry points, groups, target capture
// and the layout setters.  Replaces the reference's ManyBoneIK3D::_bone_list_changed
// (many_bone_ik_3d.cpp:1011-1068) and the per-frame _process_modification (:645-694) with its
// pose capture / write-back (:91-116); DESIGN.md §2.
#include "host.h"

#include "gd_math.h"

using namespace gd;
using namespace mbik_host;

namespace mbik_host {
thread_local std::string g_err;
int fail(int code, const std::string &msg) {
	g_err = msg;
	return code;
}

template <typename T>
int upload(mbik_plan *p, const std::vector<T> &v, const T *&dst) {
	size_t n = std::max<size_t>(1, v.size());
	void *d = nullptr;
	if (hipMalloc(&d, n * sizeof(T)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc failed for plan table");
	p->allocs.push_back(d);
	p->device_bytes += (int64_t)(n * sizeof(T));
	if (!v.empty() && hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpy failed for plan table");
	dst = reinterpret_cast<const T *>(d);
	return MBIK_OK;
}

// Packs the topology tables (and the schedule for the current lane count) into one blob.
int upload_topology(mbik_plan *p) {
	const mbik::HostPlan &h = p->host;
	DevPlan &d = p->dev;
	std::vector<uint32_t> blob;
	auto add = [&](const void *data, size_t bytes, size_t align_words, int &off) {
		while (blob.size() % align_words) blob.push_back(0);
		off = (int)blob.size();
		size_t w = (bytes + 3) / 4;
		blob.resize(blob.size() + std::max<size_t>(w, 1), 0);
		if (bytes) std::memcpy(blob.data() + off, data, bytes);
	};
	std::vector<int4> rows(h.sched.size());
	for (size_t i = 0; i < rows.size(); i++) {
		// .w: the SCHED_* bits, and above bit 8 the row's longest segment in bone-steps (row_steps)
		const size_t r0 = i / (size_t)h.K * (size_t)h.K;
		int nq = 0;
		for (int l = 0; l < h.K; l++) {
			const int sg = h.sched[r0 + l].seg;
			if (sg >= 0) nq = std::max(nq, h.seg_bone_off[sg + 1] - h.seg_bone_off[sg]);
		}
		rows[i] = make_int4(h.sched[i].seg, h.sched[i].j, h.sched[i].m, h.sched[i].flags | (nq << 8));
	}
	add(rows.data(), rows.size() * sizeof(int4), 4, d.o_sched);
#define MBIK_ADD(T, name) \
	if (std::string(#name) != "sched") add(h.name.data(), h.name.size() * sizeof(h.name[0]), sizeof(T) >= 16 ? 4 : (sizeof(T) >= 8 ? 2 : 1), d.o_##name);
	MBIK_TOPO_TABLES(MBIK_ADD)
#undef MBIK_ADD
	while (blob.size() % 4) blob.push_back(0);
	if (p->d_sched) (void)hipFree(p->d_sched);
	p->d_sched = nullptr;
	if (hipMalloc(&p->d_sched, blob.size() * 4) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc topology blob");
	if (hipMemcpy(p->d_sched, blob.data(), blob.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpy topology blob");
	d.topo_blob = reinterpret_cast<const uint4 *>(p->d_sched);
	d.topo_words = (int)blob.size();
	// diagnostics (tools/topo_const.py): the blob's table offsets, for a timing-only build that
	// compiles one plan's offsets in (solve_block.h MBIK_TOPO_CONST)
	if (getenv("MBIK_DEBUG_TOPO_OFFSETS")) {
#define MBIK_PRINT(T, name) fprintf(stderr, "MBIK_TC %s %d\n", #name, d.o_##name);
		MBIK_TOPO_TABLES(MBIK_PRINT)
#undef MBIK_PRINT
		fprintf(stderr, "MBIK_TC_K %d\n", h.K);
	}
	return MBIK_OK;
}

// Every setup table (D, CF, CD, and their skeleton-tiled copies, sized for the padded N) below
// 4 GiB: the solve can address them with 32-bit offsets.  Placement-0 plans beyond that run
// the 64-bit-index instantiation; placements 1 and 2 require it.
bool tables_fit_32(const mbik_plan *p) {
	const mbik::HostPlan &h = p->host;
	if (p->tab64) return false;
	const size_t n = (size_t)(h.N + kRowTile - 1) / kRowTile * kRowTile;
	return (size_t)h.B * 9 * n * sizeof(float) <= kMaxBufBytes && (size_t)h.NC * h.cf_stride() * n * sizeof(float) <= kMaxBufBytes &&
			(size_t)h.NC * h.cd_stride() * n * sizeof(double) <= kMaxBufBytes;
}
// The solve kernel instantiation of a plan's current layout (stabilization x locals placement
// x waves per SIMD, and for placement 0 the table addressing): k_solve_w1.hip, k_solve_w2.hip,
// k_solve_rw.hip.
mbik::SolveKernel solve_kernel_for(const mbik_plan *p) {
	const mbik::HostPlan &h = p->host;
	if (h.wave_roles) return mbik::solve_kernel_rw(h.K, h.waves_per_simd, p->dev.prio_mask);
	const int pl = std::min(2, std::max(0, (int)h.state_hbm));
	const bool two = h.waves_per_simd == 2 && h.stabilization_passes == 0;
	// placement 0 with tables of 4 GiB or more: 64-bit element indices
	const bool t32 = !(pl == 0 && !tables_fit_32(p));
	if (two) return mbik::solve_kernel_w2(pl, t32, h.has_xs, p->dev.prio_mask);
	return mbik::solve_kernel_w1(h.stabilization_passes > 0, pl, t32, p->dev.prio_mask);
}

// Whether a launch of the plan's current layout runs with the helper wave
// (mbik_solve_kernel_help): asked for, and a layout it serves -- state in LDS, no
// stabilization, one wave per SIMD, 32-bit tables -- whose block LDS still fits with the ring.
bool helper_on(const mbik_plan *p) {
	const mbik::HostPlan &h = p->host;
	if (p->helper_override != 1) return false;
	// (packed levels run row by row there: both waves walk the same rows)
	if (h.state_hbm != 0 || h.stabilization_passes != 0 || h.waves_per_simd != 1 || h.constraint_mode || !tables_fit_32(p)) return false;
	const size_t lds = ((size_t)h.spw * p->dev.lds_stride + p->dev.topo_words) * sizeof(float) + kHelpRingBytes;
	return lds <= 160 * 1024;
}

// The helper wave's handshake deadline: a wait gives up when the awaited counter has not moved
// for this long.  A real wait lasts at most one iteration of the partner wave (under a
// millisecond at the BASELINE sizes, tens of milliseconds for a 4,096-bone chain).
constexpr int kHelpTimeoutMs = 2000;
// A helper-wave launch needs the plan's timeout flag and the deadline in wall-clock ticks.
int ensure_help_flag(mbik_plan *p) {
	if (!p->help_flag) {
		void *h = nullptr;
		if (hipHostMalloc(&h, sizeof(unsigned int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
			return fail(MBIK_ENOMEM, "hipHostMalloc helper timeout flag");
		p->help_flag = static_cast<unsigned int *>(h);
		*p->help_flag = 0u;
		void *d = nullptr;
		if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return fail(MBIK_EHIP, "hipHostGetDevicePointer");
		p->dev.help_flag = static_cast<unsigned int *>(d);
	}
	int khz = 0;
	if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device) != hipSuccess || khz <= 0) khz = 100000;
	const uint64_t us = p->help_timeout_us > 0 ? (uint64_t)p->help_timeout_us : (uint64_t)kHelpTimeoutMs * 1000u;
	p->dev.help_timeout = (uint64_t)khz * us / 1000u;
	return MBIK_OK;
}
// Reports (once) a helper-wave timeout of an earlier launch of this plan: its skeletons were
// written as failures (write_help_timeout) and flagged non-finite.  The asynchronous calls report
// it on the plan's next call; the synchronous ones right after their own launch.
int take_helper_timeout(mbik_plan *p) {
	// one exchange: a still-running launch that sets the flag between a load and a clear would
	// otherwise have its timeout cleared unreported
	if (!p->help_flag || __atomic_exchange_n(p->help_flag, 0u, __ATOMIC_ACQ_REL) == 0u) return MBIK_OK;
	return fail(MBIK_EHIP, "helper wave: a launch of this plan timed out in the two-wave handshake; its skeletons "
						   "were written as failures (identity rotation, NaN position) and flagged non-finite");
}

// Resident one-wave blocks per CU for a block's LDS size, from the runtime's occupancy
// query on the kernel instantiation the plan launches (LDS granularity and registers).
int blocks_per_cu(void *ctx, int64_t lds_bytes) {
	const mbik_plan *p = static_cast<const mbik_plan *>(ctx);
	int n = 0;
	const void *k = (const void *)solve_kernel_for(p);
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64, (size_t)lds_bytes) != hipSuccess || n <= 0)
		return (int)(160 * 1024 / std::max<int64_t>(1, lds_bytes));
	return n;
}

// constraint_mode lanes per skeleton without a measurement: at most 4.  Its bone-steps are
// cheap and its state lives in HBM, so the chip's VALU issue (many narrow waves), not one
// skeleton's chain, bounds it beyond that (C2 / C3 / C5: DESIGN.md §1, profiles/r01_cmode_lanes_sweep.jsonl).
constexpr int kCmodeLanes = 4;
// The constraint_mode wave-roles block's LDS for this launch, bounded from the host plan alone
// (the topology blob's upper bound; cmode_lds_bytes needs the uploaded blob and node state).
static int64_t cmode_rw_lds_bound(const mbik_plan *p, int64_t nlaunch) {
	const mbik::HostPlan &h = p->host;
	const int64_t W = std::max(1, (h.cm_npos + 31) / 32);
	const int64_t spw = cmode_shape_of(p, nlaunch).spw;
	return mbik::topology_bytes(h) + (2 * (int64_t)h.B + spw * 4 * W + (int64_t)h.K * 64 * h.cm_maxd + (int64_t)h.K * 4 * 64 + 64) * 4;
}

// roles_ok false: the classic layout even where wave roles are asked for (their block does not
// fit the LDS, below).
static int ensure_schedule_as(mbik_plan *p, int64_t nlaunch, bool roles_ok) {
	mbik::HostPlan &h = p->host;
	int lanes = p->lanes_override;
	if (lanes == 0 && h.constraint_mode && p->cm_lanes > 0) lanes = p->cm_lanes;
	h.staging = p->staging_override < 0 ? 1 : p->staging_override;
	h.state_hbm = h.constraint_mode ? 0 : std::max(0, p->locals_override);
	h.waves_per_simd = (p->waves_override == 2 && !h.constraint_mode && h.stabilization_passes == 0) ? 2 : 1;
	// Wave roles (mbik_plan_set_wave_roles): the whole state in device memory, one wave per role
	// (K = 2, 4 or 8 waves per block; 8 only at two waves per SIMD), no stabilization, 32-bit tables.
	h.wave_roles = roles_ok && p->roles_override == 1 && !h.constraint_mode && h.stabilization_passes == 0 && tables_fit_32(p) ? 1 : 0;
	if (h.wave_roles) {
		const int cap = 4 * h.waves_per_simd;
		int roles = std::min(lanes, cap);
		if (roles == 0) {
			mbik::build_schedule(h, 0, nlaunch, 0, p->interval_override, nullptr, nullptr, p->cu_count);
			roles = std::min(h.K, cap);
		}
		// one role is the classic layout with 64 skeletons per wave: no wave roles then
		if (roles >= 2) {
			lanes = roles;
			h.state_hbm = 2;
			h.staging = 0;
		} else {
			h.wave_roles = 0;
		}
	}
	// constraint_mode with wave roles (cmode.h mbik_cmode_kernel_rw): K = 2, 4 or 8 waves per block
	h.cm_roles = 0;
	if (roles_ok && h.constraint_mode && p->roles_override == 1 && h.stabilization_passes == 0 && tables_fit_32(p) &&
			node_area_floats(3 * h.B + 2 * h.NC, (size_t)h.N) * sizeof(float) < (size_t(1) << 32)) {
		int roles = 1;
		while (roles < (lanes > 0 ? lanes : kCmodeLanes)) roles <<= 1;
		roles = std::min(8, roles);
		if (roles >= 2) {
			lanes = roles;
			h.cm_roles = 1;
		}
	}
	if (h.state_hbm >= 1 && !tables_fit_32(p))
		return fail(MBIK_EUNSUPPORTED, "state placements 1 and 2 need every setup table < 4 GiB (fewer skeletons per plan)");
	if (h.state_hbm >= 1 && !p->d_locals) {
		// LocTiled: whole tiles of kLocTile skeletons
		const size_t bytes = (size_t)((h.N + kLocTile - 1) / kLocTile) * kLocTile * h.B * 12 * sizeof(float);
		if (hipMalloc(&p->d_locals, bytes) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc locals");
		p->allocs.push_back(p->d_locals);
		p->device_bytes += (int64_t)bytes;
		p->dev.Lg = p->d_locals;
		p->dev.lg_bytes = (uint32_t)std::min<size_t>(bytes, 0xFFFFFFFFu); // (placement 2 refuses > kMaxBufBytes)
	}
	// split-exchange (staging 4 / 5) runs in the 32-bit-table two-wave builds; the 64-bit-index
	// two-wave build solves those segments alone (4 -> 0) or staged (5 -> 2)
	if (h.waves_per_simd == 2 && !tables_fit_32(p) && h.staging >= 4) h.staging = h.staging == 4 ? 0 : 2;
	mbik::build_schedule(h, lanes, nlaunch, p->spw_override, p->interval_override, blocks_per_cu, p, p->cu_count);
	if (lanes == 0 && h.constraint_mode && h.K > kCmodeLanes && !h.cm_roles)
		mbik::build_schedule(h, kCmodeLanes, nlaunch, p->spw_override, p->interval_override, blocks_per_cu, p, p->cu_count);
	// A wave-roles block holds the topology, the non-finite flags and, with cooperative rows, the
	// block's targets and the effector-global exchange (the root segment's row alone takes a slot
	// per pin); constraint_mode's holds per-wave chain stacks of the deepest pose chain.  Where that
	// exceeds the LDS the plan falls back to the classic layout, as it does for stabilization or
	// 64-bit tables: a pinned mbik_plan_set_wave_roles(1) still solves, and the autotune times the
	// classic layout for such a candidate instead of failing on it.
	if (roles_ok && ((h.wave_roles && h.lds_block_bytes > 160 * 1024) || (h.cm_roles && cmode_rw_lds_bound(p, nlaunch) > 160 * 1024)))
		return ensure_schedule_as(p, nlaunch, false);
	if (h.state_hbm == 2) {
		// the whole state in device memory: one skeleton's LDS layout per skeleton (the locals
		// and the checkpoint globals live in skeleton-tiled areas, d_locals and d_gtile)
		const int stride = (mbik::state_floats_per_skeleton(h) - 12 * h.B - 12 * h.n_gck + 3) & ~3;
		const size_t need = (size_t)h.N * stride;
		const size_t gneed = (size_t)((h.N + kLocTile - 1) / kLocTile) * kLocTile * (size_t)std::max(1, h.n_gck) * 12;
		if (need * sizeof(float) > kMaxBufBytes || p->dev.lg_bytes > kMaxBufBytes || gneed * sizeof(float) > kMaxBufBytes)
			return fail(MBIK_EUNSUPPORTED, "solve state in device memory needs < 4 GiB per area (fewer skeletons per plan)");
		if (gneed > p->d_gtile_floats) {
			void *a = nullptr;
			if (hipMalloc(&a, gneed * sizeof(float)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc checkpoint globals");
			if (p->d_gtile) {
				(void)hipFree(p->d_gtile);
				p->allocs.erase(std::remove(p->allocs.begin(), p->allocs.end(), (void *)p->d_gtile), p->allocs.end());
				p->device_bytes -= (int64_t)(p->d_gtile_floats * sizeof(float));
			}
			p->d_gtile = static_cast<float *>(a);
			p->d_gtile_floats = gneed;
			p->allocs.push_back(a);
			p->device_bytes += (int64_t)(gneed * sizeof(float));
		}
		p->dev.Gg = p->d_gtile;
		p->dev.gg_bytes = (uint32_t)(p->d_gtile_floats * sizeof(float));
		if (need > p->d_state_floats) {
			void *a = nullptr;
			if (hipMalloc(&a, need * sizeof(float)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc state");
			if (p->d_state) {
				(void)hipFree(p->d_state);
				p->allocs.erase(std::remove(p->allocs.begin(), p->allocs.end(), (void *)p->d_state), p->allocs.end());
				p->device_bytes -= (int64_t)(p->d_state_floats * sizeof(float));
			}
			p->d_state = static_cast<float *>(a);
			p->d_state_floats = need;
			p->allocs.push_back(a);
			p->device_bytes += (int64_t)(need * sizeof(float));
		}
		p->dev.Sg = p->d_state;
		p->dev.sg_bytes = (uint32_t)(p->d_state_floats * sizeof(float));
		p->dev.state_stride = stride;
	}
	if (p->sched_K == h.K && p->sched_c == h.g_interval && p->sched_staging == h.staging &&
			p->sched_locals == h.state_hbm && p->sched_roles == (h.wave_roles | h.cm_roles << 1) && p->d_sched) {
		p->dev.spw = h.spw;
		return MBIK_OK;
	}
	int rc = upload_topology(p);
	if (rc) return rc;
	p->sched_K = h.K;
	p->sched_c = h.g_interval;
	p->sched_staging = h.staging;
	p->sched_locals = h.state_hbm;
	p->sched_roles = h.wave_roles | h.cm_roles << 1;
	p->dev.nrows = h.nrows;
	p->dev.K = h.K;
	p->dev.log2K = h.log2K;
	p->dev.spw = h.spw;
	p->dev.hs_floats = h.hs_floats;
	p->dev.rw_xslots = h.rw_xslots;
	p->dev.n_gck = h.n_gck;
	p->dev.lds_stride = (mbik::lds_floats_per_skeleton(h) + 3) & ~3;
	return MBIK_OK;
}

int ensure_schedule(mbik_plan *p, int64_t nlaunch) { return ensure_schedule_as(p, nlaunch, true); }

// constraint_mode block LDS (cmode.h): topology blob, pre-order tables, the dirty words of
// the block's 64 / K skeletons, then per lane the chain stack and, with stabilization, the
// target-heading origins.
// Per wave: the dirty words of its spw skeletons, and per lane the chain stack and (STAB) the
// target-heading origins; the topology and pre-order tables once per block.
static size_t cmode_wave_words(const mbik_plan *p, int spw) {
	const mbik::HostPlan &h = p->host;
	return (size_t)spw * 4 * p->cm.W + 64 * ((size_t)p->cm.maxd + (h.stabilization_passes > 0 ? 3 * (size_t)h.P : 0));
}
// constraint_mode launch shape: spw skeletons per wave (cm_spw_div halves 64 / K that many
// times), and as many waves per block (<= kCmodeMaxWaves) as share the block's LDS within
// 160 KiB and leave the launch with at least one block per CU.
CmShape cmode_shape_of(const mbik_plan *p, int64_t count) {
	const mbik::HostPlan &h = p->host;
	if (h.cm_roles) // wave roles: a block is K waves x spw skeletons (64, halved cm_spw_div times)
		return CmShape{p->spw_override > 0 ? std::min(64, p->spw_override) : std::max(1, 64 >> std::max(0, p->cm_spw_div)), 1};
	const int full = 64 >> h.log2K;
	const int spw = p->spw_override > 0 ? std::min(full, p->spw_override) : std::max(1, full >> std::max(0, p->cm_spw_div));
	int wpb = kCmodeMaxWaves;
	const size_t fixed = (size_t)p->dev.topo_words + 2 * (size_t)h.B;
	while (wpb > 1 && ((fixed + (size_t)wpb * cmode_wave_words(p, spw)) * sizeof(float) > 160 * 1024 ||
							  (size_t)(count + (int64_t)wpb * spw - 1) / ((size_t)wpb * spw) < (size_t)p->cu_count))
		wpb >>= 1;
	return CmShape{spw, wpb};
}
size_t cmode_lds_bytes(const mbik_plan *p, CmShape sh) {
	const mbik::HostPlan &h = p->host;
	if (h.cm_roles) // topology, pre-order tables, dirty words, per wave the chain stacks, pending cleanings, flags
		return ((size_t)p->dev.topo_words + 2 * (size_t)h.B + (size_t)sh.spw * 4 * p->cm.W + (size_t)h.K * 64 * p->cm.maxd +
					   (size_t)h.K * 4 * 64 + 64) *
				sizeof(float);
	return ((size_t)p->dev.topo_words + 2 * (size_t)h.B + (size_t)sh.wpb * cmode_wave_words(p, sh.spw)) * sizeof(float);
}
void cmode_shape(mbik_plan *p, int count) {
	const CmShape sh = cmode_shape_of(p, count);
	p->cm.spw = sh.spw;
	p->cm.wpb = sh.wpb;
}

// Resets the constraint_mode node caches of skeletons [first, first+count) to a fresh tree
// built on `setup_pose` (device pointer, indexed from `first`).
int cmode_reset(mbik_plan *p, int first, int count, const float *setup_pose, hipStream_t stream) {
	if (count <= 0) return MBIK_OK;
	hipError_t e = mbik::launch_cmode_reset(stream, p->dev, p->cm, first, count, setup_pose);
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("constraint_mode reset launch: ") + hipGetErrorString(e));
	return MBIK_OK;
}

// Plan files keep constraint_mode's node caches in the plain [slot][12][N] order (format 1's);
// the device holds them skeleton-tiled (node_at).
size_t cmode_file_node_bytes(const mbik::HostPlan &h) { return (size_t)(3 * h.B + 2 * h.NC) * 12 * (size_t)h.N * sizeof(float); }
std::vector<float> cmode_nodes_tiled(const mbik::HostPlan &h, const float *plain) {
	const int slots = 3 * h.B + 2 * h.NC;
	const size_t N = (size_t)h.N;
	std::vector<float> t(node_area_floats(slots, N), 0.0f);
	for (int k = 0; k < slots; k++)
		for (int f = 0; f < 12; f++)
			for (size_t s = 0; s < N; s++) t[node_at(slots, s, k, f)] = plain[((size_t)k * 12 + f) * N + s];
	return t;
}
void cmode_nodes_plain(const mbik::HostPlan &h, const float *tiled, float *plain) {
	const int slots = 3 * h.B + 2 * h.NC;
	const size_t N = (size_t)h.N;
	for (int k = 0; k < slots; k++)
		for (int f = 0; f < 12; f++)
			for (size_t s = 0; s < N; s++) plain[((size_t)k * 12 + f) * N + s] = tiled[node_at(slots, s, k, f)];
}

// constraint_mode: allocates the persistent node caches and builds the fresh tree from the
// host setup poses of mbik_plan_create.
int cmode_create(mbik_plan *p, const float *setup_pose, const void *saved) {
	const mbik::HostPlan &h = p->host;
	CmodeState &c = p->cm;
	c.W = std::max(1, (h.cm_npos + 31) / 32);
	c.maxd = h.cm_maxd;
	int rc = upload(p, h.cm_pre, c.pre);
	rc = rc ? rc : upload(p, h.cm_sub, c.sub);
	if (rc) return rc;
	const size_t N = (size_t)h.N;
	const size_t node_bytes = node_area_floats(3 * h.B + 2 * h.NC, N) * sizeof(float);
	const size_t dirty_bytes = 4 * (size_t)c.W * N * sizeof(uint32_t);
	void *a = nullptr, *d = nullptr, *sp = nullptr;
	if (hipMalloc(&a, std::max<size_t>(node_bytes, 4)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc constraint_mode node caches");
	p->allocs.push_back(a);
	if (hipMalloc(&d, std::max<size_t>(dirty_bytes, 4)) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc constraint_mode dirty bits");
	p->allocs.push_back(d);
	p->device_bytes += (int64_t)(node_bytes + dirty_bytes);
	c.node = static_cast<float *>(a);
	c.dirty = static_cast<uint32_t *>(d);
	if (N == 0) return MBIK_OK;
	if (saved) { // mbik_plan_load: the saved frame-to-frame node caches ([slot][12][N] in the file)
		const char *sv = static_cast<const char *>(saved);
		const std::vector<float> tiled = cmode_nodes_tiled(h, reinterpret_cast<const float *>(sv));
		if (hipMemcpy(a, tiled.data(), node_bytes, hipMemcpyHostToDevice) != hipSuccess ||
				hipMemcpy(d, sv + cmode_file_node_bytes(h), dirty_bytes, hipMemcpyHostToDevice) != hipSuccess)
			return fail(MBIK_EHIP, "hipMemcpy constraint_mode state");
		return MBIK_OK;
	}
	if (p->setup_on_device) { // mbik_plan_create_device: the setup pose already lives on the device
		rc = cmode_reset(p, 0, (int)N, setup_pose, nullptr);
		if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = fail(MBIK_EHIP, "constraint_mode reset");
		return rc;
	}
	const size_t pose_bytes = N * h.B * 10 * sizeof(float);
	if (hipMalloc(&sp, pose_bytes) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc setup pose");
	rc = hipMemcpy(sp, setup_pose, pose_bytes, hipMemcpyHostToDevice) == hipSuccess ? MBIK_OK : fail(MBIK_EHIP, "hipMemcpy setup pose");
	if (rc == 0) rc = cmode_reset(p, 0, (int)N, static_cast<const float *>(sp), nullptr);
	if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = fail(MBIK_EHIP, "constraint_mode reset");
	(void)hipFree(sp);
	return rc;
}

// The skeleton-tiled copies of the plan's D / CF / CD (DevPlan::row_at) for launches with the
// whole state in device memory, (re)built on the launch stream when the tables changed.
int ensure_tiled_rows(mbik_plan *p, hipStream_t stream) {
	if (p->tiled_version == p->tables_version && p->d_Dt) return MBIK_OK;
	const mbik::HostPlan &h = p->host;
	const int Npad = (h.N + kRowTile - 1) / kRowTile * kRowTile;
	const size_t nD = (size_t)h.B * 9 * Npad, nCF = (size_t)h.NC * h.cf_stride() * Npad, nCD = (size_t)h.NC * h.cd_stride() * Npad;
	if (!p->d_Dt) {
		void *a = nullptr, *b = nullptr, *c = nullptr;
		if (hipMalloc(&a, std::max<size_t>(nD, 1) * sizeof(float)) != hipSuccess ||
				hipMalloc(&b, std::max<size_t>(nCF, 1) * sizeof(float)) != hipSuccess ||
				hipMalloc(&c, std::max<size_t>(nCD, 1) * sizeof(double)) != hipSuccess) {
			if (a) (void)hipFree(a);
			if (b) (void)hipFree(b);
			if (c) (void)hipFree(c);
			return fail(MBIK_ENOMEM, "hipMalloc tiled setup tables");
		}
		// padding skeletons read zeros
		if (hipMemsetAsync(a, 0, std::max<size_t>(nD, 1) * sizeof(float), stream) != hipSuccess ||
				hipMemsetAsync(b, 0, std::max<size_t>(nCF, 1) * sizeof(float), stream) != hipSuccess ||
				hipMemsetAsync(c, 0, std::max<size_t>(nCD, 1) * sizeof(double), stream) != hipSuccess) {
			(void)hipStreamSynchronize(stream);
			(void)hipFree(a);
			(void)hipFree(b);
			(void)hipFree(c);
			return fail(MBIK_EHIP, "hipMemsetAsync tiled setup tables");
		}
		p->d_Dt = static_cast<float *>(a);
		p->d_CFt = static_cast<float *>(b);
		p->d_CDt = static_cast<double *>(c);
		p->allocs.push_back(a);
		p->allocs.push_back(b);
		p->allocs.push_back(c);
		p->device_bytes += (int64_t)((nD + nCF) * sizeof(float) + nCD * sizeof(double));
	}
	hipError_t e = hipSuccess;
	if (nD && e == hipSuccess) e = mbik::launch_tile_rows(stream, p->dev.D, p->d_Dt, h.B, 9, h.N, Npad);
	if (nCF && e == hipSuccess) e = mbik::launch_tile_rows(stream, p->dev.CF, p->d_CFt, h.NC, h.cf_stride(), h.N, Npad);
	if (nCD && e == hipSuccess) e = mbik::launch_tile_rows(stream, p->dev.CD, p->d_CDt, h.NC, h.cd_stride(), h.N, Npad);
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("tile launch failed: ") + hipGetErrorString(e));
	// A launch on another stream must not read the copy before the tiling has run: record its
	// completion; launch() makes other streams wait on it until it has completed.
	if (!p->tile_ev && hipEventCreateWithFlags(&p->tile_ev, hipEventDisableTiming) != hipSuccess) {
		p->tile_ev = nullptr;
		return fail(MBIK_EHIP, "hipEventCreate");
	}
	if (hipEventRecord(p->tile_ev, stream) != hipSuccess) return fail(MBIK_EHIP, "hipEventRecord");
	p->tile_stream = stream;
	p->tile_pending = true;
	p->tiled_version = p->tables_version;
	return MBIK_OK;
}
// Orders a launch on `stream` after the last tiling of the plan's tables (ensure_tiled_rows).
int wait_tiled_rows(mbik_plan *p, hipStream_t stream) {
	if (!p->tile_pending) return MBIK_OK;
	if (hipEventQuery(p->tile_ev) == hipSuccess) {
		p->tile_pending = false;
		return MBIK_OK;
	}
	if (stream != p->tile_stream && hipStreamWaitEvent(stream, p->tile_ev, 0) != hipSuccess)
		return fail(MBIK_EHIP, "hipStreamWaitEvent");
	return MBIK_OK;
}

int launch(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out,
		hipStream_t stream, int iterations, int seg_lo, int seg_hi) {
	if (first < 0 || count < 0 || (int64_t)first + count > p->host.N) return fail(MBIK_EINVAL, "skeleton range out of plan");
	if (count == 0) return MBIK_OK;
	if (!pose_in || !pose_out || (p->host.P > 0 && !targets)) return fail(MBIK_EINVAL, "null buffer");
	const mbik::HostPlan &h = p->host;
	if (h.P == 0) {
		// get_effector_count() == 0: _process_modification returns before solving
		// (many_bone_ik_3d.cpp:649-651) and the skeleton keeps its pose.
		if (pose_out != pose_in &&
				hipMemcpyAsync(pose_out, pose_in, (size_t)count * h.B * 10 * sizeof(float), hipMemcpyDeviceToDevice, stream) != hipSuccess)
			return fail(MBIK_EHIP, "hipMemcpyAsync");
		return MBIK_OK;
	}
	int rc = ensure_schedule(p, count);
	if (rc) return rc;
	if (h.constraint_mode) {
		cmode_shape(p, count);
		const size_t clds = cmode_lds_bytes(p, CmShape{p->cm.spw, p->cm.wpb});
		if (clds > 160 * 1024) return fail(MBIK_EUNSUPPORTED, "skeleton too large for the constraint_mode LDS layout");
		// node caches below 4 GiB: buffer-resource addressing (cmode.h, NB32)
		const bool nb32 = node_area_floats(3 * h.B + 2 * h.NC, (size_t)h.N) * sizeof(float) < (size_t(1) << 32) && tables_fit_32(p);
		mbik::CmodeKernel ck = mbik::cmode_kernel(h.stabilization_passes > 0, nb32, h.has_chain);
		const int per_block = p->cm.spw * p->cm.wpb;
		unsigned threads = 64 * p->cm.wpb;
		if (h.cm_roles) {
			// wave roles: K waves x spw skeletons per block (ensure_schedule: K in {2, 4, 8}, 32-bit addressing)
			if (h.K != 2 && h.K != 4 && h.K != 8) return fail(MBIK_EINVAL, "constraint_mode wave roles: 2, 4 or 8 roles");
			ck = mbik::cmode_kernel_rw(h.has_chain, h.K);
			threads = 64 * h.K;
		}
		hipLaunchKernelGGL(ck, dim3((unsigned)((count + per_block - 1) / per_block)), dim3(threads), clds, stream, p->dev,
				p->cm, first, count, pose_in, targets, pose_out, iterations, seg_lo, seg_hi);
		hipError_t e = hipGetLastError();
		if (e != hipSuccess) return fail(MBIK_EHIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
		return MBIK_OK;
	}
	size_t lds = ((size_t)h.spw * p->dev.lds_stride + p->dev.topo_words) * sizeof(float);
	if constexpr (kAblate & ABL_SOALDS) lds += ((size_t)p->dev.B * 9 + p->dev.NC * p->dev.cf_stride + 2 * p->dev.NC * p->dev.cd_stride + 2) * sizeof(float);
	if (lds > 160 * 1024) return fail(MBIK_EUNSUPPORTED, "skeleton too large for LDS at this lane count");
	unsigned blocks = (unsigned)((count + h.spw - 1) / h.spw);
	auto kern = solve_kernel_for(p);
	unsigned threads = 64;
	if (h.wave_roles) {
		threads = 64u * (unsigned)h.K; // a wave per role
		// non-finite flags; with cooperative rows the targets, the effector-global exchange and the
		// groups' parent-side records
		lds += 64 * sizeof(int) + (h.rw_xslots ? ((size_t)h.P + h.rw_xslots) * 12 * 64 * sizeof(float) + mbik::rw_record_bytes(h) : 0);
		if (lds > 160 * 1024) return fail(MBIK_EUNSUPPORTED, "wave roles: a row's effector-global exchange exceeds the LDS");
		// the cooperative groups' record handshake has a deadline and reports through the plan's
		// timeout flag, as the helper wave's does (rw_wait)
		if (h.rw_xslots && (rc = ensure_help_flag(p)) != MBIK_OK) return rc;
	} else if (helper_on(p)) {
		if ((rc = ensure_help_flag(p)) != MBIK_OK) return rc;
		lds += kHelpRingBytes;
		threads = 128;
#ifdef MBIK_REPLAY
		const bool replay = p->dev.replay == 2;
		if (replay) threads = 64;
#else
		const bool replay = false;
#endif
		kern = mbik::solve_kernel_help(p->dev.prio_mask, replay);
	}
	DevPlan d = p->dev;
	if (h.state_hbm == 2) {
		if ((rc = ensure_tiled_rows(p, stream)) != MBIK_OK) return rc;
		if ((rc = wait_tiled_rows(p, stream)) != MBIK_OK) return rc;
		d.D = p->d_Dt;
		d.CF = p->d_CFt;
		d.CD = p->d_CDt;
		d.row_n = (h.N + kRowTile - 1) / kRowTile * kRowTile;
	}
	hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, stream, d, first, count, pose_in, targets, pose_out,
			iterations, seg_lo, seg_hi);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
	return MBIK_OK;
}

} // namespace

namespace mbik_host {
// mbik_plan_options: NULL = the defaults; fields past struct_size keep theirs.
int read_options(const mbik_plan_options *opts, int &libm) {
	libm = MBIK_LIBM_VARIANT_FMA;
	if (!opts) return MBIK_OK;
	if (opts->struct_size < (int32_t)sizeof(int32_t)) return fail(MBIK_EINVAL, "mbik_plan_options.struct_size too small");
	if (opts->struct_size >= (int32_t)(offsetof(mbik_plan_options, libm_variant) + sizeof(int32_t))) libm = opts->libm_variant;
	if (libm != MBIK_LIBM_VARIANT_FMA && libm != MBIK_LIBM_VARIANT_SSE2) return fail(MBIK_EINVAL, "unknown libm_variant");
	return MBIK_OK;
}

} // namespace mbik_host

extern "C" {

const char *mbik_last_error(void) { return g_err.c_str(); }

int32_t mbik_describe_topology(const mbik_skeleton_desc *desc, const mbik_config *config, int32_t *bone_list,
		int32_t *bone_list_count, int32_t *seg_root, int32_t *seg_tip, int32_t *seg_parent, int32_t *seg_headings) {
	if (!desc || !config) return fail(MBIK_EINVAL, "null argument");
	mbik::HostPlan h;
	std::string err = mbik::build_topology(*desc, *config, h);
	if (!err.empty()) return fail(MBIK_EINVAL, err);
	if (bone_list) std::copy(h.bone_list.begin(), h.bone_list.end(), bone_list);
	if (bone_list_count) *bone_list_count = (int32_t)h.bone_list.size();
	for (int i = 0; i < h.NS; i++) {
		if (seg_root) seg_root[i] = h.seg_root[i];
		if (seg_tip) seg_tip[i] = h.seg_tip[i];
		if (seg_parent) seg_parent[i] = h.seg_parent[i];
		if (seg_headings) seg_headings[i] = h.seg_nh[i];
	}
	return h.NS;
}

int32_t mbik_plan_create(const mbik_skeleton_desc *desc, const mbik_config *config, int32_t n_skeletons, const float *setup_pose,
		const float *cones, const float *twist, int32_t device, mbik_plan **out_plan) {
	return mbik_plan_create_opts(desc, config, nullptr, n_skeletons, setup_pose, cones, twist, device, out_plan);
}

int32_t mbik_plan_create_opts(const mbik_skeleton_desc *desc, const mbik_config *config, const mbik_plan_options *opts,
		int32_t n_skeletons, const float *setup_pose, const float *cones, const float *twist, int32_t device,
		mbik_plan **out_plan) {
	if (!desc || !config || !out_plan) return fail(MBIK_EINVAL, "null argument");
	int libm = 0;
	if (read_options(opts, libm)) return MBIK_EINVAL;
	*out_plan = nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MBIK_ENODEV, "no HIP device visible");
	if (device < 0 || device >= ndev) return fail(MBIK_EINVAL, "device index out of range");
	std::unique_ptr<mbik_plan> p(new mbik_plan());
	p->device = device;
	if (desc->bone_count < 0 || desc->pin_count < 0 || desc->constraint_count < 0 || config->bone_damp_count < 0)
		return fail(MBIK_EINVAL, "negative count");
	keep_inputs(p.get(), *desc, *config);
	std::string err = mbik::build_topology(*desc, *config, p->host);
	if (!err.empty()) return fail(MBIK_EINVAL, err);
	p->host.libm_variant = libm;
	err = mbik::build_skeletons(p->host, n_skeletons, setup_pose, cones, twist, std::max(1, desc->max_cones));
	if (!err.empty()) return fail(MBIK_EINVAL, err);
	const int rc = finish_plan(p.get(), setup_pose, nullptr);
	if (rc) return rc;
	*out_plan = p.release();
	return MBIK_OK;
}

} // extern "C"
namespace mbik_host {
void keep_inputs(mbik_plan *p, const mbik_skeleton_desc &desc, const mbik_config &cfg) {
	p->src_parents.assign(desc.parents, desc.parents + (desc.parents ? desc.bone_count : 0));
	p->src_pins.assign(desc.pins, desc.pins + (desc.pins ? desc.pin_count : 0));
	p->src_cons.assign(desc.constraints, desc.constraints + (desc.constraints ? desc.constraint_count : 0));
	p->src_bone_damp.assign(cfg.bone_damp, cfg.bone_damp + (cfg.bone_damp ? std::max(0, cfg.bone_damp_count) : 0));
	p->src_max_cones = desc.max_cones;
	p->src_cfg = cfg;
	p->src_cfg.bone_damp = nullptr;
}

// The device side of a plan whose HostPlan holds the topology and the per-skeleton tables
// (D / CF / CD): uploads them, builds the launch schedule, and the constraint_mode node caches
// -- from the setup pose (a new plan), or copied from a saved plan's bytes (cm_state: node
// caches then dirty words, as mbik_plan_save wrote them).
int finish_plan(mbik_plan *p, const float *setup_pose, const void *cm_state) {
	const int device = p->device;
	const int n_skeletons = p->host.N;
	for (int b = 0; b < p->host.B; b++)
		if ((p->host.bone_flags[b] & mbik::BF_PINNED) && p->host.bone_pin[b] >= 0) {
			int e = p->host.bone_pin[b];
			if (p->host.eff_path_off[e + 1] - p->host.eff_path_off[e] > 4096) return fail(MBIK_EUNSUPPORTED, "skeleton too deep");
		}
	DeviceGuard guard(device);
	{
		int cus = 0;
		if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
			p->cu_count = cus;
	}
	mbik::HostPlan &h = p->host;
	DevPlan &d = p->dev;
	d.B = h.B; d.P = h.P; d.NS = h.NS; d.NC = h.NC; d.max_cones = h.max_cones; d.N = h.N;
	d.cf_stride = h.cf_stride(); d.cd_stride = h.cd_stride();
	d.stab = h.stabilization_passes; d.constraint_mode = h.constraint_mode; d.hs_floats = h.hs_floats;
	d.libm = h.libm_variant;
	d.n_gck = h.n_gck;
	// One heading slot mask shared by every effector -- the reference's default priorities, the
	// usual case -- runs bone-steps specialised for it (kPrioDefault).
	{
		int pm = -1;
		for (int e = 0; e < h.P && pm != 0; e++) {
			int m = 1;
			for (int a = 0; a < 3; a++)
				if (h.eff_prio[3 * e + a] > 0.0f) m |= 6 << (2 * a);
			pm = pm < 0 || pm == m ? m : 0;
		}
		d.prio_mask = pm == kPrioDefault ? pm : 0;
	}
	d.lds_stride = (mbik::lds_floats_per_skeleton(h) + 3) & ~3;
	int rc = 0;
	rc = rc ? rc : upload(p, h.D, d.D);
	rc = rc ? rc : upload(p, h.CF, d.CF);
	rc = rc ? rc : upload(p, h.CD, d.CD);
	if (rc) {
		for (void *a : p->allocs) (void)hipFree(a);
		p->allocs.clear();
		return rc;
	}
	rc = ensure_schedule(p, n_skeletons);
	if (rc == 0 && h.constraint_mode) rc = cmode_create(p, setup_pose, cm_state);
	if (rc) {
		for (void *a : p->allocs) (void)hipFree(a);
		p->allocs.clear();
		if (p->d_sched) (void)hipFree(p->d_sched);
		p->d_sched = nullptr;
		return rc;
	}
	// Algorithmic flops: per bone-step 50 H + 14 H [translate] + 72 E_seg
	// + 465, plus 770 + 140 C - 60 for a constrained bone with C cones; x iterations.
	double f = 0;
	for (int sg = 0; sg < h.NS; sg++) {
		const int H = h.seg_nh[sg], E = h.seg_eff_off[sg + 1] - h.seg_eff_off[sg];
		const bool tr = (h.seg_flags[sg] & mbik::SF_TRANSLATE) != 0;
		for (int k = h.seg_bone_off[sg]; k < h.seg_bone_off[sg + 1]; k++) {
			const int b = h.seg_bones[k];
			if (!h.constraint_mode) f += 50.0 * H + (tr ? 14.0 * H : 0.0) + 72.0 * E + 465.0; // no fit in constraint_mode
			if (h.bone_flags[b] & (mbik::BF_ORIENT | mbik::BF_AXIAL)) {
				const int C = (h.bone_flags[b] & mbik::BF_ORIENT) ? h.cons_ncones[h.bone_cons[b]] : 0;
				f += 770.0 + 140.0 * C - 60.0;
			}
		}
	}
	p->alg_flops = f * h.iterations;
	// Algorithmic HBM bytes per skeleton, SURVEY.md §8(d)'s definition (the one bench.py's
	// roofline and BASELINE.md divide by): each input the solve needs read once, each output
	// written once -- per bone the input pose (quaternion, position, scale: 40 B), its
	// bone-direction quaternion (16 B) and damp (4 B), and the output pose (40 B); per
	// effector the target transform (48 B) and its weight and priorities (16 B); per
	// constrained bone the orientation and twist quaternions, the twist centre (16 B each),
	// the twist half-cosine (4 B) and 52 B per cone.  C2 8,292 B, C3 3,456, C4 6,912,
	// C5 52,068.
	double cons = 0;
	for (int c = 0; c < h.NC; c++) cons += 16.0 * 3 + 4.0 + 52.0 * h.cons_ncones[c];
	p->alg_bytes = (double)h.B * (40 + 16 + 4 + 40) + (double)h.P * (48 + 16) + cons;
	if (h.constraint_mode) // the persistent node caches, read and written once per frame
		p->alg_bytes += 2.0 * ((double)(3 * h.B + 2 * h.NC) * 12 * 4 + 4.0 * p->cm.W * 4);
	h.D.clear(); h.D.shrink_to_fit();
	h.CF.clear(); h.CF.shrink_to_fit();
	h.CD.clear(); h.CD.shrink_to_fit();
	return MBIK_OK;
}
} // namespace

extern "C" {

void mbik_plan_destroy(mbik_plan *p) {
	if (!p) return;
	DeviceGuard guard(p->device);
	for (void *a : p->allocs) (void)hipFree(a);
	if (p->d_sched) (void)hipFree(p->d_sched);
	if (p->d_in) (void)hipFree(p->d_in);
	if (p->d_tg) (void)hipFree(p->d_tg);
	if (p->d_out) (void)hipFree(p->d_out);
	if (p->tile_ev) (void)hipEventDestroy(p->tile_ev);
	if (p->help_flag) (void)hipHostFree(p->help_flag);
	delete p;
}

int32_t mbik_plan_get_info(const mbik_plan *p, mbik_plan_info *o) {
	if (!p || !o) return fail(MBIK_EINVAL, "null argument");
	const mbik::HostPlan &h = p->host;
	int maxh = 0;
	for (int i = 0; i < h.NS; i++) maxh = std::max(maxh, h.seg_height[i]);
	o->abi_version = MBIK_ABI_VERSION;
	o->skeleton_count = h.N;
	o->bone_count = h.B;
	o->pin_count = h.P;
	o->segment_count = h.NS;
	o->level_count = maxh + 1;
	o->lanes_per_skeleton = h.K;
	o->skeletons_per_block = h.constraint_mode ? (h.cm_roles ? cmode_shape_of(p, h.N).spw : 64 >> h.log2K) : h.spw;
	o->max_headings = h.max_headings;
	o->device = p->device;
	o->device_bytes = p->device_bytes;
	o->algorithmic_bytes_per_skeleton = p->alg_bytes;
	o->algorithmic_flops_per_skeleton = p->alg_flops;
	// (constraint_mode: the block of a whole-plan launch, independent of earlier launches' counts)
	o->lds_bytes_per_block = h.constraint_mode ? (int64_t)cmode_lds_bytes(p, cmode_shape_of(p, h.N)) : p->host.lds_block_bytes;
	o->checkpoint_interval = h.g_interval;
	o->heading_staging = h.staging;
	o->state_placement = h.state_hbm;
	o->waves_per_simd = h.waves_per_simd;
	o->constraint_slots = h.NC;
	o->cf_stride = h.cf_stride();
	o->cd_stride = h.cd_stride();
	o->libm_variant = h.libm_variant;
	o->helper_wave = helper_on(p) ? 1 : 0;
	o->heading_slots = p->dev.prio_mask;
	o->wave_roles = h.wave_roles | h.cm_roles;
	return MBIK_OK;
}

int32_t mbik_plan_set_launch(mbik_plan *p, int32_t lanes) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (lanes < 0 || lanes > 64 || (lanes & (lanes - 1))) return fail(MBIK_EINVAL, "lanes_per_skeleton must be 0 or a power of two <= 64");
	p->lanes_override = lanes;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_layout(mbik_plan *p, int32_t lanes, int32_t skeletons_per_block, int32_t global_checkpoint_interval) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (lanes < 0 || lanes > 64 || (lanes & (lanes - 1))) return fail(MBIK_EINVAL, "lanes_per_skeleton must be 0 or a power of two <= 64");
	if (skeletons_per_block < 0 || skeletons_per_block > 64) return fail(MBIK_EINVAL, "skeletons_per_block must be in [0, 64]");
	if (global_checkpoint_interval < 0) return fail(MBIK_EINVAL, "global_checkpoint_interval must be >= 0");
	p->lanes_override = lanes;
	p->spw_override = skeletons_per_block;
	p->interval_override = global_checkpoint_interval;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_waves_per_simd(mbik_plan *p, int32_t waves) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (waves != -1 && waves != 1 && waves != 2) return fail(MBIK_EINVAL, "waves_per_simd must be -1 (automatic), 1 or 2");
	p->waves_override = waves;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_helper_wave(mbik_plan *p, int32_t helper) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (helper < -1 || helper > 1) return fail(MBIK_EINVAL, "helper wave must be -1 (automatic), 0 (off) or 1 (on)");
	p->helper_override = helper;
	return MBIK_OK;
}

int32_t mbik_plan_set_wave_roles(mbik_plan *p, int32_t roles) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (roles < -1 || roles > 1) return fail(MBIK_EINVAL, "wave roles must be -1 (automatic), 0 (off) or 1 (on)");
	p->roles_override = roles;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_table_addressing(mbik_plan *p, int32_t wide) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (wide != 0 && wide != 1) return fail(MBIK_EINVAL, "table addressing must be 0 (automatic) or 1 (64-bit indices)");
	p->tab64 = wide;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_locals_placement(mbik_plan *p, int32_t placement) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (placement < -1 || placement > 2)
		return fail(MBIK_EINVAL, "placement must be -1 (automatic), 0 (LDS), 1 (locals in device memory) or 2 (all state)");
	p->locals_override = placement;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_set_heading_staging(mbik_plan *p, int32_t staging) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (staging < -1 || staging > 5) return fail(MBIK_EINVAL, "staging must be -1 (automatic), 0, 1, 2, 3, 4 or 5");
	p->staging_override = staging;
	p->sched_K = -1;
	return MBIK_OK;
}

int32_t mbik_plan_rebuild_setup(mbik_plan *p, int32_t first, int32_t count, const float *setup_pose, const float *cones,
		const float *twist, void *hip_stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	mbik::HostPlan &h = p->host;
	if (first < 0 || count < 0 || (int64_t)first + count > h.N) return fail(MBIK_EINVAL, "skeleton range out of plan");
	if (count == 0) return MBIK_OK;
	if (!setup_pose || (h.NC > 0 && (!cones || !twist))) return fail(MBIK_EINVAL, "null buffer");
	DeviceGuard guard(p->device);
	if (!p->dsetup_ready) {
		mbik::SetupView v = mbik::setup_view(h, h.N, h.setup_max_cones);
		int rc = 0;
		auto up = [&](const std::vector<int32_t> &vec, const int *&dst) {
			if (rc == 0) rc = upload(p, vec, dst);
		};
		up(h.setup_topo, v.topo);
		up(h.bone_list, v.bone_list);
		up(h.bone_flags, v.bone_flags);
		up(h.bone_pose_parent, v.bone_pose_parent);
		up(h.bone_ik_parent, v.bone_ik_parent);
		up(h.ik_child_off, v.ik_child_off);
		up(h.ik_children, v.ik_children);
		up(h.cons_order, v.cons_order);
		up(h.cons_order_slot, v.cons_order_slot);
		up(h.cons_order_ncones, v.cons_order_ncones);
		up(h.cons_bone, v.cons_bone);
		if (rc) return rc;
		p->dsetup = v;
		p->dsetup_ready = true;
	}
	const mbik::SetupView &v = p->dsetup;
	const size_t stride = (mbik::setup_scratch_bytes(v.B, v.NC, v.max_cones_in) + 255) & ~size_t(255);
	const int threads = std::min(count, 8192);
	void *scratch = nullptr;
	if (hipMalloc(&scratch, stride * (size_t)threads) != hipSuccess) return fail(MBIK_ENOMEM, "hipMalloc setup scratch");
	hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
	const DevPlan &d = p->dev;
	hipError_t e = mbik::launch_setup(st, threads, v, first, count, setup_pose, cones, twist, static_cast<char *>(scratch), stride,
			const_cast<float *>(d.D), const_cast<float *>(d.CF), const_cast<double *>(d.CD));
	// the scratch is freed after the kernel; a fault while it runs surfaces at this sync and
	// must not be reported as success (the D/CF/CD tables may be partly written)
	hipError_t es = hipStreamSynchronize(st);
	(void)hipFree(scratch);
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("setup launch: ") + hipGetErrorString(e));
	if (es != hipSuccess) return fail(MBIK_EHIP, std::string("setup kernel: ") + hipGetErrorString(es));
	p->tables_version++;
	// a rebuilt tree starts with fresh node caches (_bone_list_changed)
	if (h.constraint_mode) return cmode_reset(p, first, count, setup_pose, st);
	return MBIK_OK;
}

int32_t mbik_plan_setup_tables(const mbik_plan *p, float *D, float *CF, double *CD) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	const mbik::HostPlan &h = p->host;
	DeviceGuard guard(p->device);
	const size_t N = (size_t)h.N;
	if (D && hipMemcpy(D, p->dev.D, (size_t)h.B * 9 * N * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpy D");
	if (CF && h.NC && hipMemcpy(CF, p->dev.CF, (size_t)h.NC * h.cf_stride() * N * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpy CF");
	if (CD && h.NC && hipMemcpy(CD, p->dev.CD, (size_t)h.NC * h.cd_stride() * N * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpy CD");
	return MBIK_OK;
}

int32_t mbik_plan_resident_blocks(const mbik_plan *p, int64_t lds_bytes_per_block) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	DeviceGuard guard(p->device);
	return blocks_per_cu(const_cast<mbik_plan *>(p), lds_bytes_per_block);
}

int32_t mbik_solve(mbik_plan *p, int32_t first, int32_t count, const float *pose_in, const float *targets, float *pose_out,
		void *stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (int rc = take_helper_timeout(p)) return rc;
	DeviceGuard guard(p->device);
	return launch(p, first, count, pose_in, targets, pose_out, (hipStream_t)stream, p->host.iterations, 0, p->host.NS - 1);
}

int32_t mbik_plan_status(const mbik_plan *p, uint32_t *status) {
	if (!p || !status) return fail(MBIK_EINVAL, "null argument");
	*status = (p->help_flag && __atomic_load_n(p->help_flag, __ATOMIC_ACQUIRE)) ? MBIK_STATUS_HELPER_TIMEOUT : 0u;
	return MBIK_OK;
}

int32_t mbik_plan_debug_helper(mbik_plan *p, int32_t drop_record, int32_t timeout_us) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (drop_record < -1 || timeout_us < 0) return fail(MBIK_EINVAL, "drop_record must be >= -1 and timeout_us >= 0");
	p->dev.help_drop = drop_record;
	p->help_timeout_us = timeout_us;
	return MBIK_OK;
}

int32_t mbik_solve_checked(mbik_plan *p, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out, uint8_t *nonfinite, void *stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (!nonfinite) return fail(MBIK_EINVAL, "null nonfinite buffer");
	if (int rc = take_helper_timeout(p)) return rc;
	DeviceGuard guard(p->device);
	if (p->host.P == 0 && count > 0 && first >= 0 && (int64_t)first + count <= p->host.N &&
			hipMemsetAsync(nonfinite, 0, (size_t)count, (hipStream_t)stream) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemsetAsync");
	p->dev.nonfinite = nonfinite;
	const int rc = launch(p, first, count, pose_in, targets, pose_out, (hipStream_t)stream, p->host.iterations, 0, p->host.NS - 1);
	p->dev.nonfinite = nullptr;
	return rc;
}

int32_t mbik_segment_solve(mbik_plan *p, int32_t seg, int32_t first, int32_t count, float *pose_inout, const float *targets,
		void *stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (seg < 0 || seg >= p->host.NS) return fail(MBIK_EINVAL, "segment out of range");
	if (int rc = take_helper_timeout(p)) return rc;
	DeviceGuard guard(p->device);
	return launch(p, first, count, pose_inout, targets, pose_inout, (hipStream_t)stream, 1, p->host.seg_tin[seg], seg);
}

int32_t mbik_group_create(mbik_plan *const *plans, int32_t n_plans, mbik_group **out_group) {
	if (!plans || n_plans <= 0 || !out_group) return fail(MBIK_EINVAL, "null argument or empty group");
	*out_group = nullptr;
	for (int i = 0; i < n_plans; i++) {
		if (!plans[i]) return fail(MBIK_EINVAL, "null plan in group");
		if (plans[i]->device != plans[0]->device) return fail(MBIK_EINVAL, "group plans must share one device");
	}
	std::unique_ptr<mbik_group> g(new mbik_group());
	g->plans.assign(plans, plans + n_plans);
	g->device = plans[0]->device;
	DeviceGuard guard(g->device);
	if (hipMalloc(&g->d_plans, sizeof(DevPlan) * n_plans) != hipSuccess ||
			hipMalloc(&g->d_entries, sizeof(GroupEntry) * n_plans) != hipSuccess) {
		if (g->d_plans) (void)hipFree(g->d_plans);
		return fail(MBIK_ENOMEM, "hipMalloc group tables");
	}
	*out_group = g.release();
	return MBIK_OK;
}

void mbik_group_destroy(mbik_group *g) {
	if (!g) return;
	DeviceGuard guard(g->device);
	if (g->d_plans) (void)hipFree(g->d_plans);
	if (g->d_entries) (void)hipFree(g->d_entries);
	delete g;
}

int32_t mbik_group_solve(mbik_group *g, const int32_t *first, const int32_t *count, const float *const *pose_in,
		const float *const *targets, float *const *pose_out, void *hip_stream) {
	if (!g) return fail(MBIK_EINVAL, "null group");
	if (!pose_in || !targets || !pose_out) return fail(MBIK_EINVAL, "null buffer array");
	for (mbik_plan *p : g->plans)
		if (int rc = take_helper_timeout(p)) return rc;
	DeviceGuard guard(g->device);
	hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
	const int n = (int)g->plans.size();
	std::vector<DevPlan> dp;
	std::vector<GroupEntry> ent;
	size_t lds = 0;
	int blocks = 0;
	bool stab = false;
	// Longest chain first (iterations x critical-path bone-steps of the plan's schedule).
	std::vector<std::pair<double, int>> order;
	for (int i = 0; i < n; i++) {
		const mbik::HostPlan &h = g->plans[i]->host;
		double steps = 0;
		for (int r = 0; r < h.nrows; r++) {
			int m = 0;
			for (int l = 0; l < h.K; l++) {
				const int sg = h.sched[(size_t)r * h.K + l].seg;
				if (sg >= 0) m = std::max(m, h.seg_bone_off[sg + 1] - h.seg_bone_off[sg]);
			}
			steps += m;
		}
		order.push_back({-(double)h.iterations * steps, i});
	}
	std::stable_sort(order.begin(), order.end());
	for (auto [key, i] : order) {
		(void)key;
		mbik_plan *p = g->plans[i];
		const int f = first ? first[i] : 0;
		const int c = count ? count[i] : p->host.N - f;
		if (f < 0 || c < 0 || (int64_t)f + c > p->host.N) return fail(MBIK_EINVAL, "skeleton range out of plan");
		if (c == 0) continue;
		if (!pose_in[i] || !pose_out[i] || (p->host.P > 0 && !targets[i])) return fail(MBIK_EINVAL, "null buffer");
		int rc = p->host.P > 0 ? ensure_schedule(p, c) : MBIK_OK;
		if (rc) return rc;
		if (p->host.constraint_mode || p->host.P == 0 || p->host.state_hbm != 0 || !tables_fit_32(p) || p->host.has_xs) {
			// constraint_mode plans have their own kernel, so do plans laid out with their
			// locals in HBM, plans whose setup tables need 64-bit indices and plans with
			// split-exchange segments (the two-wave build); pinless plans only copy
			rc = launch(p, f, c, pose_in[i], targets[i], pose_out[i], stream, p->host.iterations, 0, p->host.NS - 1);
			if (rc) return rc;
			continue;
		}
		const mbik::HostPlan &h = p->host;
		const size_t l = ((size_t)h.spw * p->dev.lds_stride + p->dev.topo_words) * sizeof(float);
		if (l > 160 * 1024) return fail(MBIK_EUNSUPPORTED, "skeleton too large for LDS at this lane count");
		lds = std::max(lds, l);
		stab = stab || h.stabilization_passes > 0;
		dp.push_back(p->dev);
		ent.push_back(GroupEntry{blocks, f, c, h.iterations, pose_in[i], targets[i], pose_out[i]});
		blocks += (c + h.spw - 1) / h.spw;
	}
	if (ent.empty()) return MBIK_OK;
	if (hipMemcpyAsync(g->d_plans, dp.data(), sizeof(DevPlan) * dp.size(), hipMemcpyHostToDevice, stream) != hipSuccess ||
			hipMemcpyAsync(g->d_entries, ent.data(), sizeof(GroupEntry) * ent.size(), hipMemcpyHostToDevice, stream) != hipSuccess)
		return fail(MBIK_EHIP, "hipMemcpyAsync group tables");
	const mbik::GroupKernel kern = mbik::group_kernel(stab);
	hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64), lds, stream, (const DevPlan *)g->d_plans,
			(const GroupEntry *)g->d_entries, (int)ent.size());
	hipError_t e = hipGetLastError();
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("group launch failed: ") + hipGetErrorString(e));
	// the staged tables above are pageable: hipMemcpyAsync has consumed them on return
	return MBIK_OK;
}
int32_t mbik_capture_targets(mbik_plan *p, int32_t first, int32_t count, const float *skeleton_global,
		const float *target_global, const uint8_t *visible, float *targets, void *hip_stream) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (first < 0 || count < 0 || (int64_t)first + count > p->host.N) return fail(MBIK_EINVAL, "skeleton range out of plan");
	const int P = p->host.P;
	if (count == 0 || P == 0) return MBIK_OK;
	if (!skeleton_global || !target_global || !targets) return fail(MBIK_EINVAL, "null buffer");
	DeviceGuard guard(p->device);
	hipError_t e = mbik::launch_capture_targets(reinterpret_cast<hipStream_t>(hip_stream), count, P, skeleton_global, target_global,
			visible, targets);
	if (e != hipSuccess) return fail(MBIK_EHIP, std::string("capture launch failed: ") + hipGetErrorString(e));
	return MBIK_OK;
}

int32_t mbik_plan_segment_table(const mbik_plan *p, int32_t *root, int32_t *tip, int32_t *parent, int32_t cap) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	const mbik::HostPlan &h = p->host;
	for (int i = 0; i < h.NS && i < cap; i++) {
		if (root) root[i] = h.seg_root[i];
		if (tip) tip[i] = h.seg_tip[i];
		if (parent) parent[i] = h.seg_parent[i];
	}
	return h.NS;
}

int32_t mbik_solve_host(mbik_plan *p, int32_t first, int32_t count, const float *pose_in, const float *targets, float *pose_out) {
	if (!p) return fail(MBIK_EINVAL, "null plan");
	if (count <= 0) return count == 0 ? MBIK_OK : fail(MBIK_EINVAL, "negative count");
	DeviceGuard guard(p->device);
	const mbik::HostPlan &h = p->host;
	size_t need = (size_t)count;
	if (need > p->scratch_skel) {
		if (p->d_in) (void)hipFree(p->d_in);
		if (p->d_tg) (void)hipFree(p->d_tg);
		if (p->d_out) (void)hipFree(p->d_out);
		p->d_in = p->d_tg = p->d_out = nullptr;
		if (hipMalloc(&p->d_in, need * h.B * 10 * sizeof(float)) != hipSuccess ||
				hipMalloc(&p->d_tg, std::max<size_t>(1, need * h.P * 12) * sizeof(float)) != hipSuccess ||
				hipMalloc(&p->d_out, need * h.B * 10 * sizeof(float)) != hipSuccess)
			return fail(MBIK_ENOMEM, "hipMalloc scratch");
		p->scratch_skel = need;
	}
	if (hipMemcpy(p->d_in, pose_in, need * h.B * 10 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
			(h.P > 0 && hipMemcpy(p->d_tg, targets, need * h.P * 12 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess))
		return fail(MBIK_EHIP, "hipMemcpy H2D");
	if (int rc = take_helper_timeout(p)) return rc;
	int rc = launch(p, first, count, p->d_in, p->d_tg, p->d_out, nullptr, h.iterations, 0, h.NS - 1);
	if (rc) return rc;
	if (hipMemcpy(pose_out, p->d_out, need * h.B * 10 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
		return fail(MBIK_EHIP, std::string("hipMemcpy D2H / kernel: ") + hipGetErrorString(hipGetLastError()));
	return take_helper_timeout(p); // this launch's own (the copy waited for it)
}

} // extern "C"

#ifdef MBIK_REPLAY
// Diagnostic: mode 1 runs a helper-wave solve that saves every helper record, mode 2 the solving
// wave alone replaying them (same inputs, same skeletons), mode 0 frees the buffer.
extern "C" int mbik_debug_replay(mbik_plan *p, int32_t mode, int32_t first, int32_t count, const float *pose_in,
		const float *targets, float *pose_out, void *stream) {
	DeviceGuard guard(p->device);
	if (mode == 0) {
		if (p->dev.rec_dump) (void)hipFree(p->dev.rec_dump);
		p->dev.rec_dump = nullptr;
		p->dev.replay = 0;
		return MBIK_OK;
	}
	int rc = ensure_schedule(p, count);
	if (rc) return rc;
	if (!helper_on(p)) return fail(MBIK_EINVAL, "replay needs a helper-wave layout");
	const mbik::HostPlan &h = p->host;
	int per_iter = 0;
	for (int r = 0; r < h.nrows; r++) {
		int nq = 0;
		for (int l = 0; l < h.K; l++) {
			const int sg = h.sched[(size_t)r * h.K + l].seg;
			if (sg >= 0) nq = std::max(nq, h.seg_bone_off[sg + 1] - h.seg_bone_off[sg]);
		}
		per_iter += nq;
	}
	const size_t blocks = (size_t)(count + h.spw - 1) / h.spw;
	if (mode == 1) {
		if (p->dev.rec_dump) (void)hipFree(p->dev.rec_dump);
		p->dev.rec_per_block = per_iter * h.iterations;
		if (hipMalloc(&p->dev.rec_dump, blocks * p->dev.rec_per_block * kHelpF4 * 64 * sizeof(float4)) != hipSuccess)
			return fail(MBIK_ENOMEM, "replay buffer");
	}
	p->dev.replay = mode;
	rc = launch(p, first, count, pose_in, targets, pose_out, (hipStream_t)stream, h.iterations, 0, h.NS - 1);
	p->dev.replay = 0;
	return rc;
}
#endif

#ifdef MBIK_PROF
// Diagnostic cycle accounting: the sum of every kernel TU's counters, cleared.
extern "C" int mbik_debug_prof(unsigned long long *out) {
	for (int i = 0; i < 24; i++) out[i] = 0;
	return mbik::prof_take_w1(out) | mbik::prof_take_w2(out) | mbik::prof_take_rw(out) | mbik::prof_take_cmode(out);
}
#endif
