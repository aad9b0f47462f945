// Flat, SoA plan for the batched solve: the output of ManyBoneIK3D::_bone_list_changed
// (src/many_bone_ik_3d.cpp:1011-1068) for a topology shared by a batch of skeletons,
// plus each skeleton's setup-dependent tables (bone directions, Kusudama frames).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mbik.h"

namespace mbik {

enum BoneFlags : int32_t {
	BF_IN_LIST = 1,    // in ManyBoneIK3D::bone_list (solved and written back)
	BF_ORIENT = 2,     // IK parent valid && orientationally constrained (ik_bone_segment_3d.cpp:156-159)
	BF_AXIAL = 4,      // IK parent valid && axially constrained (:160-162)
	BF_PINNED = 8,     // carries an IKEffector3D
};

// Extra bits of a step record's flags word (HostPlan::step_rec).
enum StepRecBits : int32_t {
	SR_HAS_POSE_PARENT = 1 << 8,   // bone_pose_parent != POSE_PARENT_NONE (parented, maybe by the origin)
	SR_PARENT_GLOBAL = 1 << 9,     // bone_pose_parent >= 0: the parent's global is a G slot
};

enum SegFlags : int32_t {
	SF_TRANSLATE = 1,  // root segment: translate=true, damp=PI (ik_bone_segment_3d.cpp:217-222)
	SF_STAB = 2,       // root segment built with default_stabilizing_pass_count > 0 (many_bone_ik_3d.cpp:1046;
	                   // child segments get 0, ik_bone_segment_3d.cpp:398)
};

// Pose-node parent codes (IKNode3D parent of godot_skeleton_aligned_transform).
constexpr int32_t POSE_PARENT_NONE = -1;      // released ik_origin (earlier roots of a multi-root skeleton)
constexpr int32_t POSE_PARENT_ORIGIN = -2;    // the live ik_origin (identity)

// Per-skeleton float fields of one constraint slot: twist centre rotation (4), twist half-range
// half-cosine (1), twist frame local basis (9), then per cone: control point (3), sin/cos of
// half the radius (2), tangent centre 1 (3), tangent centre 2 (3), sin/cos of half the tangent
// radius (2).  The half-angle sin/cos are what Quaternion(axis, angle) and
// get_quaternion_axis_angle evaluate on the cone's constant angles (ik_open_cone_3d.cpp:297,312,371).
constexpr int CF_TWIST_Q = 0;
constexpr int CF_TWIST_COS = 4;
constexpr int CF_TWIST_T = 5;
constexpr int CF_CONE0 = 14;
constexpr int CF_PER_CONE = 31;
constexpr int CFC_CP = 0, CFC_SR = 3, CFC_CR = 4, CFC_T1 = 5, CFC_T2 = 8, CFC_ST = 11, CFC_CT = 12;
// Per-cone constants the cone queries would otherwise re-derive every bone-step, computed at
// setup with the same operations (so bitwise what the queries compute): the normalized
// control point (closest_to_cone, ik_open_cone_3d.cpp:358-381) and, for the pair (cone,
// next cone), cross(cp, next cp) and the four normalized edge normals of the tangent
// triangles (get_on_great_tangent_triangle, :285-321).
constexpr int CFC_NCP = 13, CFC_C1XC2 = 16, CFC_A1 = 19, CFC_A2 = 22, CFC_B1 = 25, CFC_B2 = 28;
// Per-skeleton double fields of one constraint slot, per cone: radius cosine, tangent radius cosine.
constexpr int CD_PER_CONE = 2;

// Wave roles with eight roles: a block's waves w and w + 4 share a SIMD, and waves 0-3 sit on
// four different SIMDs (measured: tools/hwid_probe.hip, profiles/r06_wave_placement_probe_*).  Roles 2i and
// 2i + 1 -- a two-wave cooperative group's stepping wave and its partner -- go to waves i and
// i + 4 (solve_block.h), so that the groups' stepping waves run on four different SIMDs instead
// of two (C5 -1.9 %), and a packed level balances the SIMDs' estimated work before the two
// roles' within each SIMD (build_schedule; C5 -2.5 %).  Same box, interleaved:
// profiles/r06_rw_priority_ab.txt.  0 = roles in wave order, per-role packing.
#ifndef MBIK_RW_PERM
#define MBIK_RW_PERM 1
#endif

struct SchedTask {
	int32_t seg;  // -1 idle
	int32_t j;    // index of this lane inside the segment's lane group
	int32_t m;    // lanes in the group (power of two, aligned)
	int32_t flags; // bit 0 (SCHED_XS): split-exchange (staging 4/5): the group's lanes build alternate effectors'
	               // headings and share them through cross-lane reads; every lane sums them all in order (no
	               // staging memory).  bit 1 (SCHED_CHAIN): this row continues the previous one's packed level
};
// SCHED_COOP (wave roles only): every task of this row carries it when some segment of the row is
// solved by a group of waves (SCHED_XS, m > 1): the group's waves walk alternate effectors' paths
// and leave the effector globals in LDS, the group's first wave consumes them all in order and runs
// the step's rotation chain; the whole block meets at two barriers per bone-step of the row.
// SCHED_CMSPLIT (constraint_mode with wave roles): a multi-effector segment whose group of m waves
// splits the step's effector reads -- the first effector's read alone, then the others, whose
// dirty chains are disjoint once it has cleaned its own, over the group's waves (cmode.h); its
// row's tasks carry SCHED_COOP too (two block barriers per bone-step).
constexpr int32_t SCHED_XS = 1, SCHED_CHAIN = 2, SCHED_COOP = 4, SCHED_CMSPLIT = 8;

struct HostPlan {
	// ---- topology (shared by the batch) ----
	int32_t B = 0, P = 0, NS = 0, NC = 0, max_cones = 1;
	int32_t iterations = 15;
	int32_t constraint_mode = 0, stabilization_passes = 0;
	std::vector<int32_t> parents;
	std::vector<int32_t> bone_pose_parent, bone_ik_parent, bone_depth, bone_flags, bone_pin, bone_cons;
	std::vector<int32_t> bone_list;                 // ManyBoneIK3D::bone_list order
	std::vector<int32_t> bone_child_eff_off, bone_child_effs; // pinned IK children of each bone
	// segments, numbered in creation order (parents before children)
	std::vector<int32_t> seg_root, seg_tip, seg_parent;
	std::vector<std::vector<int32_t>> seg_children;
	std::vector<int32_t> seg_bone_off, seg_bones;   // tip -> root
	std::vector<int32_t> seg_eff_off, seg_effs, seg_eff_hoff;
	std::vector<int32_t> seg_nh, seg_flags, seg_hw_off, seg_height, seg_tin, seg_tout;
	std::vector<double> seg_hw;                     // heading weights (recursive_create_penalty_array)
	std::vector<double> seg_cos_half_damp;          // per (segment, bone position): cos(damp / 2.0)
	std::vector<float> seg_wsum2;                   // _get_manual_msd's (float) w_sum squared, per segment
	std::vector<int32_t> seg_hbase;                 // staged-heading LDS offset (floats) of multi-heading segments
	int32_t hs_floats = 0;                          // staged-heading LDS floats per skeleton
	std::vector<int32_t> roots;                     // root segments (segmented_skeletons)
	std::vector<int32_t> eff_bone, eff_parent_bone, eff_path_off, eff_path;
	std::vector<float> eff_prio;
	std::vector<int32_t> cons_bone, cons_ncones;    // constraint slots (bones in the list only)
	std::vector<int32_t> cons_order, cons_order_slot, cons_order_ncones; // applied constraints, desc order
	int32_t desc_constraint_count = 0;
	std::vector<int32_t> setup_topo;                // bones, parents before children
	std::vector<int32_t> ik_child_off, ik_children; // IK children of each bone, ascending (setup.h)
	int32_t setup_max_cones = 1;                    // cones stride of the setup inputs
	int32_t libm_variant = 0;                       // reference host's glibc sinf/cosf build (gd::LIBM_FMA / LIBM_SSE2)
	int32_t max_headings = 0;
	// constraint_mode node caches: pre-order position and subtree size of each list bone in
	// the pose-node forest (-1 / 0 elsewhere), deepest pose chain, positions used.
	std::vector<int32_t> cm_pre, cm_sub;
	int32_t cm_maxd = 1, cm_npos = 0;
	// ---- launch shape ----
	int32_t K = 4, log2K = 2, spw = 16;
	int64_t lds_block_bytes = 0;
	// Heading staging of multi-effector segments: split the heading work over the segment's
	// lanes and exchange terms through LDS (1), or let every lane of the group solve the
	// segment alone from registers (0: no staging LDS, more skeletons resident per CU,
	// longer steps for those segments), or stage only the translating root segments -- the
	// ones with the most effectors (2), or only segments with two or more effectors, whose
	// path walks are what the lanes split (3).  4: no segment is staged in memory; the lanes of
	// a multi-effector segment's group build alternate effectors' headings and read each
	// other's through cross-lane operations, every lane summing all of them in order (the split
	// of 1 and 3 without the memory round trips); 5: translating root segments staged as in 2,
	// the other multi-effector segments as in 4.  Not for constraint_mode (its lanes own tree
	// ranges).
	int staging = 1;
	bool has_xs = false;     // the schedule has split-exchange tasks (staging 4 / 5, two-wave build only)
	bool has_chain = false;  // the schedule has packed levels (rows chained without a barrier)
	// Where the per-skeleton solve state lives during a launch: 0 all of it in LDS; 1 the
	// bone local transforms L in a per-skeleton device-memory area (L2-resident), the rest in
	// LDS; 2 all of it in device memory (LDS holds only the block's topology copy).  Less LDS
	// per skeleton means more skeletons resident per CU, for L2 instead of LDS latency.
	int32_t state_hbm = 0;
	// Waves per SIMD the solve kernel's registers are sized for (1, or 2 with spills).
	int32_t waves_per_simd = 1;
	// Wave roles (the north star's "one wavefront per segment"): each lane of a wave is one
	// skeleton (64 per block) and the K roles of the sibling schedule are the block's K waves, so a
	// segment runs on one wave with its topology wave-uniform and no lane of a skeleton repeats
	// another's work.  Whole state in device memory (state_hbm 2).  0: roles are lanes of a wave.
	int32_t wave_roles = 0;
	// wave roles: effector-global exchange slots of the cooperative rows (SCHED_COOP), the most any
	// row needs; a slot is 12 floats x 64 lanes of LDS.  seg_hbase[seg] is the segment's first slot.
	int32_t rw_xslots = 0;
	// constraint_mode with wave roles (cmode.h): the K roles are the block's waves, a lane per
	// skeleton; build_schedule marks the splittable multi-effector tasks (SCHED_CMSPLIT).
	int32_t cm_roles = 0;
	// Iteration-start globals kept in LDS only for checkpoint bones: every g_interval-th bone
	// of a segment counted from its root (the root included) and every parent of a segment
	// root; a bone-step rebuilds its parent's global from the nearest checkpoint above it.
	int32_t g_interval = 1, n_gck = 0;
	std::vector<int32_t> bone_gslot;                // LDS slot of a checkpoint bone, else -1
	std::vector<int32_t> seg_anchor;                // per seg_bones index: the checkpoint's index, -1 = parent outside
	// Per seg_bones index k, what a bone-step looks up, resolved into one 16-byte record (no
	// dependent lookups), 16-bit fields: x = bone | (checkpoint index + 1) << 16; y = (G slot of
	// the parent's global or of its checkpoint, + 1) | (constraint slot + 1) << 16; z = bone
	// flags | SR_* bits | path start (depth + 1) << 16; w = child-effector offset | count << 16.
	std::vector<int32_t> step_rec;
	// Per seg_effs index i: how many leading bones effector seg_effs[i]'s path (from the root)
	// shares with the previous effector's of the same segment (0 for a segment's first), plus
	// a trailing 0.  The solve reuses the previous effector's walk down to that depth.
	std::vector<int32_t> seg_eff_lcp;
	// constraint_mode with wave roles, per seg_effs index i of a SCHED_CMSPLIT segment: the wave of
	// the segment's group that reads effector i after the first effector's read (cm_split_groups);
	// 0 elsewhere, plus a trailing 0.
	std::vector<int32_t> seg_eff_grp;
	std::vector<SchedTask> sched;                   // [nrows][K]
	int32_t nrows = 0;
	// ---- per skeleton, SoA [item][field][N] ----
	int32_t N = 0;
	std::vector<float> D;    // [B][9][N] bone-direction local basis
	std::vector<float> CF;   // [NC][CF_CONE0 + CF_PER_CONE*max_cones][N]
	std::vector<double> CD;  // [NC][CD_PER_CONE*max_cones][N]

	int cf_stride() const { return CF_CONE0 + CF_PER_CONE * max_cones; }
	int cd_stride() const { return CD_PER_CONE * max_cones; }
};

// Builds the topology tables; returns an empty string on success, else the error.
std::string build_topology(const mbik_skeleton_desc &desc, const mbik_config &cfg, HostPlan &plan);

// The GPU-side topology build (topo.h), host half.
struct TopoRig;
struct TopoOut;
// cos(damp/2) per bone of a non-root segment and of the root segments, as build_topology
// evaluates them (the host libm's cos: the reference's), for TopoRig::bone_chd / root_chd.
void topology_damp_cosines(const mbik_skeleton_desc &desc, const mbik_config &cfg, std::vector<double> &bone_chd,
		double &root_chd);
// A plan's topology from a topo_build result (o: host copies of the built tables), filled as
// build_topology fills it.  Returns an empty string or the build's error.
std::string assemble_topology(const TopoOut &o, const mbik_skeleton_desc &desc, const mbik_config &cfg, HostPlan &plan);
// Number of topology tables that differ between two plans (0: identical), and the first
// differing table's name.
int compare_topology(const HostPlan &a, const HostPlan &b, std::string *first = nullptr);
// Fills D / CF / CD for skeletons [0, n) from their setup poses, cones and twist.
std::string build_skeletons(HostPlan &plan, int32_t n, const float *setup_pose, const float *cones, const float *twist,
		int32_t max_cones_in);
// Host-side tables the per-skeleton setup reads (setup.h); filled by build_skeletons.
void setup_tables(HostPlan &plan);
struct SetupView;
SetupView setup_view(const HostPlan &plan, int32_t n, int32_t max_cones_in);
// Chooses lanes-per-skeleton / skeletons-per-block and the sibling-level schedule.
// spw_override / interval_override: 0 = automatic (mbik_plan_set_layout).
// blocks_per_cu(lds_bytes): how many one-wave blocks of that LDS size a CU holds at once
// (the device's occupancy query); nullptr = LDS-only estimate.  cus: compute units.
using BlocksPerCU = int (*)(void *ctx, int64_t lds_bytes);
void build_schedule(HostPlan &plan, int32_t lanes_per_skeleton, int64_t skeletons_in_launch, int32_t spw_override = 0,
		int32_t interval_override = 0, BlocksPerCU blocks_per_cu = nullptr, void *ctx = nullptr, int cus = 256);
// LDS floats per skeleton used by the kernel: L (12 per bone), G (12 per checkpoint), targets + stale cache
// (12 + 12 per pin), stale flags (1 per pin), the staged-heading area (hs_floats), and with
// stabilization the pre-loop target
// origins (3 per pin) and the manual-MSD terms (7 per pin).
int32_t lds_floats_per_skeleton(const HostPlan &plan);
int32_t state_floats_per_skeleton(const HostPlan &plan);
int64_t topology_bytes(const HostPlan &plan);
// Wave roles: the parent-side record of a cooperative group (bone_step.h rw_record), kRwRecF4
// float4 per lane, one per group of a row (at most K / 2 groups of two or more waves), and the
// groups' counters (rw_wait), after the effector-global exchange; 0 without cooperative rows.
constexpr int kRwRecF4 = 9;
int64_t rw_record_bytes(const HostPlan &plan);

} // namespace mbik
