// What the kernel translation units (k_*.hip) and the host side (host_*.cpp) share: the device
// view of a plan (DevPlan), the launch-shape constants both sides size LDS with, and the kernel
// handles and launchers each kernel TU exports.  Each kernel family is its own TU so that they
// compile in parallel (build.py); none needs relocatable device code: the host only takes kernel
// handles (host stubs) and launches them.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "plan.h"
#include "setup.h"
#include "topo.h"

namespace mbik {

// Topology tables (shared by every skeleton of the plan).  They are packed into one blob
// in HBM and copied into LDS at kernel start, so the many small dependent lookups of a
// bone-step (segment -> effector -> path -> bone) are LDS reads, not L2 round trips.
#define MBIK_TOPO_TABLES(X)                                                                         \
	X(int, bone_pose_parent) X(int, bone_flags) X(int, bone_pin) X(int, bone_cons)                    \
	X(int, bone_child_effs) X(int, seg_bone_off) X(int, seg_bones)                                    \
	X(int, seg_eff_off) X(int, seg_effs) X(int, seg_eff_hoff) X(int, seg_nh) X(int, seg_flags)         \
	X(int, seg_hw_off) X(int, eff_bone) X(int, eff_path_off) X(int, eff_path) X(float, eff_prio)       \
	X(int, cons_ncones) X(float, seg_wsum2) X(int, seg_hbase) X(int, bone_gslot) X(double, seg_hw) X(double, seg_cos_half_damp) X(int4, sched) \
	X(int4, step_rec) X(int, seg_eff_lcp) X(int, seg_eff_grp)

struct DevPlan {
	int B, P, NS, NC, max_cones, nrows, K, log2K, spw, lds_stride;
	int N, cf_stride, cd_stride;
	int stab;            // stabilization_passes (root segments only, SF_STAB)
	int prio_mask = 0;   // kPrioDefault if every effector has that heading slot mask, else 0
	int hs_floats;       // staged-heading LDS floats per skeleton
	int rw_xslots = 0;   // wave roles: effector-global exchange slots (12 floats x 64 lanes of LDS each)
	int n_gck;           // checkpoint globals per skeleton (HostPlan::bone_gslot)
	int constraint_mode; // ManyBoneIK3D::constraint_mode
	int libm;            // the reference host's glibc sinf/cosf build (gd::LIBM_FMA / LIBM_SSE2)
	int topo_words; // blob size in 32-bit words (multiple of 4)
	const uint4 *topo_blob;
#define MBIK_DECL(T, name) const T *name; int o_##name;
	MBIK_TOPO_TABLES(MBIK_DECL)
#undef MBIK_DECL
	const float *D, *CF;
	const double *CD;
	// The per-skeleton tables D / CF / CD are [item][field][N].  Launches with the whole state in
	// device memory read a skeleton-tiled copy instead, [item][row_n/kRowTile][field][kRowTile]
	// (row_n = N rounded up; row_at<kTabTiled>): one lane group's skeletons x all fields of a
	// slot are then whole cache lines.
	int row_n = 0;
	// mbik_solve_checked: per-skeleton flag, 1 when any bone's solved basis was non-finite and
	// was written as the identity rotation (ik_bone_3d.cpp:174-176); null otherwise.
	unsigned char *nonfinite = nullptr;
	// state_hbm 1: the bone locals, [N/kLocTile][B][3][kLocTile][4] (LocTiled); state_hbm 2: the whole
	// other state at Sg + s * state_stride (one skeleton's LDS layout after its locals)
	float *Lg = nullptr, *Sg = nullptr;
	int state_stride = 0;
	uint32_t lg_bytes = 0, sg_bytes = 0; // their sizes (< 4 GiB: buffer-resource addressing)
	// state_hbm 2: the checkpoint globals, skeleton-tiled like the locals, [N/kLocTile][n_gck][3][kLocTile][4]
	float *Gg = nullptr;
	uint32_t gg_bytes = 0;
	// Helper-wave launches: the plan's timeout flag (host-mapped, one word per plan), set to 1 by
	// a block whose waves gave up waiting for each other; the wait's deadline in wall-clock ticks
	// (s_memrealtime, since the awaited counter last moved); and a test hook: the helper stops
	// before producing record help_drop (-1: never; mbik_plan_debug_helper).
	unsigned int *help_flag = nullptr;
	uint64_t help_timeout = 0;
	int help_drop = -1;
#ifdef MBIK_REPLAY
	// Diagnostic build (tools/replay_count.sh): the helper wave's records of one launch saved to
	// rec_dump ([block][record][kHelpF4][64 lanes] float4), and a launch of the solving wave alone
	// that reads them back instead of waiting for a helper -- its instruction counters are then
	// the solving wave's own.  replay: 0 off, 1 save, 2 replay.
	float4 *rec_dump = nullptr;
	int rec_per_block = 0, replay = 0;
#endif
};

// Heading slot masks: bit 0 the origin heading, bits 1+2a / 2+2a the +/- headings of axis a
// (present when direction priority a > 0).  PM != 0: every effector of the plan has that mask
// (DevPlan::prio_mask), so the slot tests are compile-time constants and the heading loops
// compile to straight-line code; PM == 0: tested per effector at run time.  The one
// specialised mask is the reference's default priorities (0.2, 0, 0.2)
// (ik_effector_template_3d.h:45): origin, +/-x, +/-z.
constexpr int kPrioDefault = 1 | (6 << 0) | (6 << 4);
// Skeleton tiles of the locals / checkpoint globals in device memory (LocTiled) and of the
// setup-table copy (row_at<kTabTiled>).
constexpr int kLocTile = 16;
constexpr int kRowTile = 16;
// Helper-wave ring (bone_step.h): kHelpSlots records of kHelpF4 float4 per lane, plus counters.
constexpr int kHelpF4 = 18, kHelpSlots = 4;
constexpr int kHelpRingBytes = kHelpSlots * kHelpF4 * 64 * 16 + 32;

// A heterogeneous batch (mbik_group_solve): plan i owns blocks [block_off[i], block_off[i + 1]).
struct GroupEntry {
	int block_off, first, count, iterations;
	const float *pose_in, *targets;
	float *pose_out;
};

// GPU-side topology build (topo.h): one thread per rig, each with its own output and scratch slices.
struct TopoSlice {
	TopoRig rig;
	int32_t *out_i;
	double *out_d;
	float *out_f;
	int32_t *scr_i;
	double *scr_d;
};

// ---- constraint_mode node caches (cmode.h) ----
// The node state is skeleton-tiled like the default kernel's locals (LocTiled):
// [N/16][slot][3 quads][16 skeletons][4], element f of node slot k of skeleton s at node_at(),
// so one node of 16 consecutive skeletons is 768 contiguous bytes and a lane reads its node as
// three 16-byte quads -- a wave's lane group (consecutive skeletons, one slot) reads 256
// contiguous bytes per load instruction.  With the plain [slot][12][N] rows (round 2) every
// element was its own dword load and a 16-skeleton group used half of each 128-B line.
constexpr int kNodeTile = 16;
__host__ __device__ __forceinline__ size_t node_at(int slots, size_t s, int k, int f) {
	return ((s / kNodeTile) * (size_t)slots + (size_t)k) * (12 * kNodeTile) + (size_t)(f >> 2) * (4 * kNodeTile) +
			(s % kNodeTile) * 4 + (f & 3);
}
__host__ __device__ __forceinline__ size_t node_area_floats(int slots, size_t N) { return (N + kNodeTile - 1) / kNodeTile * kNodeTile * (size_t)slots * 12; }

struct CmodeState {
	float *node;        // node_at(): slots pose local (B), pose global (B), bone-direction global (B),
	                    // constraint-orientation global (NC), twist global (NC)
	uint32_t *dirty;    // [kind * W + word][N], kinds: pose, bone direction, orientation, twist
	const int *pre;     // [B] pre-order position in the pose-node forest (list bones)
	const int *sub;     // [B] subtree size
	int W;              // dirty words per kind
	int maxd;           // deepest pose chain
	int spw = 0;        // skeletons per wave (<= 64 / K; fewer leave lanes idle but put more waves per SIMD)
	int wpb = 1;        // waves per block: they share the block's LDS copy of the topology
};
// waves per classic constraint_mode block (launch bound)
constexpr int kCmodeMaxWaves = 4;

// ---- kernel handles, each exported by the TU that instantiates the kernels ----
using SolveKernel = void (*)(DevPlan, int, int, const float *, const float *, float *, int, int, int);
using GroupKernel = void (*)(const DevPlan *, const GroupEntry *, int);
using CmodeKernel = void (*)(DevPlan, CmodeState, int, int, const float *, const float *, float *, int, int, int);
// k_solve_w1.hip: the one-wave classic kernels (WPE 1), including the 64-bit-index ones, and the
// fused group kernel; k_solve_w2.hip: the two-waves-per-SIMD builds.  Every handle has its
// 160 KiB dynamic-LDS attribute set.
SolveKernel solve_kernel_w1(bool stab, int pl, bool t32, int pm);
SolveKernel solve_kernel_w2(int pl, bool t32, bool xs, int pm);
GroupKernel group_kernel(bool stab);
// k_solve_rw.hip: wave roles (KW 2 / 4 / 8 waves, WPE 1 / 2) and the helper-wave kernels
SolveKernel solve_kernel_rw(int kw, int wpe, int pm);
SolveKernel solve_kernel_help(int pm, bool replay);
// k_cmode.hip
CmodeKernel cmode_kernel(bool stab, bool nb32, bool chain);
CmodeKernel cmode_kernel_rw(bool chain, int kw); // (32-bit node addressing only)
hipError_t launch_cmode_reset(hipStream_t st, const DevPlan &t, const CmodeState &c, int first, int count, const float *setup_pose);
// k_aux.hip: target capture, the GPU setup / topology builds and the tiled-row copy.  (The
// self-test and device-KAT kernels live with their entry points in host_selftest.cpp.)
hipError_t launch_capture_targets(hipStream_t st, int count, int P, const float *skel_global, const float *target_global,
		const uint8_t *visible, float *targets);
hipError_t launch_setup(hipStream_t st, int threads, const SetupView &v, int first, int count, const float *pose, const float *cones,
		const float *twist, char *scratch, size_t scratch_stride, float *D, float *CF, double *CD);
hipError_t launch_topology(const TopoSlice *slices, int n);
hipError_t launch_tile_rows(hipStream_t st, const float *src, float *dst, int items, int fields, int N, int Npad);
hipError_t launch_tile_rows(hipStream_t st, const double *src, double *dst, int items, int fields, int N, int Npad);
#ifdef MBIK_PROF
// Diagnostic cycle accounting (-DMBIK_PROF): each kernel TU has its own counters; adds them to
// out[24] and clears them.
int prof_take_w1(unsigned long long *out);
int prof_take_w2(unsigned long long *out);
int prof_take_rw(unsigned long long *out);
int prof_take_cmode(unsigned long long *out);
#endif

} // namespace mbik
