// The host side of the C ABI (host_*.cpp): the plan and group objects behind mbik.h's opaque
// handles, and the internal functions the host translation units share (schedule, launch, errors).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"

using mbik::CmodeState;
using mbik::DevPlan;
using mbik::GroupEntry;
using mbik::kCmodeMaxWaves;
using mbik::kHelpF4;
using mbik::kHelpRingBytes;
using mbik::kLocTile;
using mbik::kPrioDefault;
using mbik::kRowTile;
using mbik::node_area_floats;
using mbik::node_at;
using mbik::TopoSlice;

struct mbik_group {
	std::vector<mbik_plan *> plans; // not owned
	int device = 0;
	void *d_plans = nullptr, *d_entries = nullptr;
};

struct mbik_plan {
	mbik::HostPlan host;
	int device = 0;
	int lanes_override = 0, spw_override = 0, interval_override = 0;
	int cu_count = 256;
	std::vector<void *> allocs;
	DevPlan dev{};
	int64_t device_bytes = 0;
	double alg_bytes = 0;
	double alg_flops = 0;
	int sched_K = -1, sched_c = -1, sched_staging = -1; // layout of the uploaded topology blob
	int staging_override = -1;                           // mbik_plan_set_heading_staging; -1 = automatic
	int tab64 = 0;                                       // mbik_plan_set_table_addressing
	int locals_override = -1;                            // mbik_plan_set_locals_placement; -1 = automatic
	int waves_override = -1;                             // mbik_plan_set_waves_per_simd; -1 = automatic
	int helper_override = -1;                            // mbik_plan_set_helper_wave; -1 = automatic
	int roles_override = -1;                             // mbik_plan_set_wave_roles; -1 = automatic (off until autotuned)
	int sched_locals = -1, sched_roles = -1;
	float *d_locals = nullptr;                           // [N][B][12] for state_hbm 1
	float *d_state = nullptr;                            // [N][state stride] for state_hbm 2
	size_t d_state_floats = 0;
	float *d_gtile = nullptr;                            // state_hbm 2: checkpoint globals, skeleton-tiled
	size_t d_gtile_floats = 0;
	void *d_sched = nullptr; // topology blob (includes the lane schedule)
	// scratch for mbik_solve_host
	float *d_in = nullptr, *d_tg = nullptr, *d_out = nullptr;
	size_t scratch_skel = 0;
	// device copies of the setup tables (mbik_plan_rebuild_setup)
	mbik::SetupView dsetup{};
	bool dsetup_ready = false;
	// constraint_mode: the persistent IKNode3D caches (cmode.h), lanes per skeleton (0 = auto)
	CmodeState cm{};
	int cm_lanes = 0;
	int cm_spw_div = 0;                                  // constraint_mode: skeletons per wave = (64 / K) >> cm_spw_div
	// the creation inputs, for mbik_plan_save (the topology is rebuilt from them on load)
	std::vector<int32_t> src_parents;
	std::vector<mbik_pin> src_pins;
	std::vector<mbik_constraint> src_cons;
	std::vector<float> src_bone_damp;
	int32_t src_max_cones = 1;
	mbik_config src_cfg{};
	bool setup_on_device = false; // mbik_plan_create_device: the setup pose given to finish_plan is a device buffer
	// skeleton-tiled copies of D / CF / CD for launches with the whole state in device memory
	// (DevPlan::row_at); rebuilt when the tables changed since (tables_version)
	float *d_Dt = nullptr, *d_CFt = nullptr;
	double *d_CDt = nullptr;
	int tables_version = 1, tiled_version = 0;
	// the tiling's completion, for launches on another stream than the one that tiled
	hipEvent_t tile_ev = nullptr;
	hipStream_t tile_stream = nullptr;
	bool tile_pending = false;
	// helper-wave timeouts (DevPlan::help_flag): the plan's own host-mapped flag word, which a
	// launch's kernel sets and the plan's next call reports (take_helper_timeout); the deadline
	// override of mbik_plan_debug_helper (0: kHelpTimeoutMs)
	unsigned int *help_flag = nullptr;
	int help_timeout_us = 0;
};

namespace mbik_host {

// The calling thread's last error message (mbik_last_error) and the error-return helper.
extern thread_local std::string g_err;
int fail(int code, const std::string &msg);

struct DeviceGuard {
	int prev = -1;
	explicit DeviceGuard(int dev) {
		if (hipGetDevice(&prev) != hipSuccess) prev = -1;
		if (prev != dev) (void)hipSetDevice(dev);
	}
	~DeviceGuard() {
		int cur = -1;
		if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
	}
};

// device-memory areas addressed through buffer resources (32-bit byte offsets): the state of
// placements 1 and 2, and the setup tables of every layout that can (kTab32 / kTabTiled)
constexpr size_t kMaxBufBytes = 0xFFFFFFF0u;
bool tables_fit_32(const mbik_plan *p);
mbik::SolveKernel solve_kernel_for(const mbik_plan *p);
bool helper_on(const mbik_plan *p);
int take_helper_timeout(mbik_plan *p);
int blocks_per_cu(void *ctx, int64_t lds_bytes);
int ensure_schedule(mbik_plan *p, int64_t nlaunch);
int launch(mbik_plan *p, int first, int count, const float *pose_in, const float *targets, float *pose_out, hipStream_t stream,
		int iterations, int seg_lo, int seg_hi);

// constraint_mode launch shape and node-cache layout conversions (host_plan.cpp)
struct CmShape {
	int spw, wpb;
};
CmShape cmode_shape_of(const mbik_plan *p, int64_t count);
size_t cmode_lds_bytes(const mbik_plan *p, CmShape sh);
size_t cmode_file_node_bytes(const mbik::HostPlan &h);
std::vector<float> cmode_nodes_tiled(const mbik::HostPlan &h, const float *plain);
void cmode_nodes_plain(const mbik::HostPlan &h, const float *tiled, float *plain);

// plan creation (host_plan.cpp)
int read_options(const mbik_plan_options *opts, int &libm);
void keep_inputs(mbik_plan *p, const mbik_skeleton_desc &desc, const mbik_config &cfg);
int finish_plan(mbik_plan *p, const float *setup_pose, const void *cm_state);

} // namespace mbik_host
