/*
 * mbik.h -- C ABI of the MI355X-native batched many-bone IK solver.
 *
 * Drop-in boundary for the per-frame solve path of Ughuuu/many_bone_ik
 * (snapshot 2024-08-07).  Each entry point names the reference interface it replaces:
 *
 *   mbik_plan_create   <- ManyBoneIK3D::_bone_list_changed()      src/many_bone_ik_3d.cpp:1011-1068
 *                         (segmentation, heading weights, bone directions, Kusudama setup;
 *                          IKBoneSegment3D::generate_default_segments ik_bone_segment_3d.cpp:352-427,
 *                          IKBone3D::update_default_bone_direction_transform ik_bone_3d.cpp:57-93,
 *                          IKLimitCone3D::update_tangent_handles ik_open_cone_3d.cpp:36-120,
 *                          IKKusudama3D::set_axial_limits/_update_constraint ik_kusudama_3d.cpp:37-115)
 *   mbik_solve         <- ManyBoneIK3D::_process_modification()   src/many_bone_ik_3d.cpp:645-694
 *                         (the virtual SkeletonModifier3D hook, many_bone_ik_3d.h:90; preceded by
 *                          _update_ik_bones_transform :91-102 and followed by
 *                          _update_skeleton_bones_transform :104-116), for a batch of skeletons
 *   mbik_solve_host    <- same, synchronous, host buffers
 *   mbik_segment_solve <- IKBoneSegment3D::segment_solver()       src/ik_bone_segment_3d.cpp:210-225
 *                         (one call = one segment_solver() of one segment subtree)
 *   mbik_plan_destroy  <- ~ManyBoneIK3D / set_dirty() rebuild
 *   mbik_last_error    <- ERR_FAIL_* messages (the reference prints and returns)
 *
 * Plain pointers and sizes only.  All float arrays are float32, row-major, one skeleton
 * after another:
 *   pose    [skel][bone][10]  quaternion x,y,z,w | position x,y,z | scale x,y,z
 *                             (Skeleton3D bone pose; ik_bone_3d.cpp:161-179)
 *   target  [skel][pin][12]   basis rows r0,r1,r2 | origin, in skeleton space
 *                             (IKEffector3D::target_relative_to_skeleton_origin, ik_effector_3d.cpp:77-84)
 *   cones   [skel][constraint][max_cones][4]  centre x,y,z | radius (kusudama_open_cones)
 *   twist   [skel][constraint][2]             from, range (joint_twist)
 *
 * Threading: a plan is not thread-safe; distinct plans may be used concurrently on
 * distinct streams.  mbik_solve is asynchronous on the given HIP stream.
 * Errors: 0 on success, a negative MBIK_E* code otherwise; mbik_last_error() explains.
 * Non-finite output bases become identity rotations, as ik_bone_3d.cpp:174-176 does.
 */
#ifndef MBIK_H
#define MBIK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MBIK_OK 0
#define MBIK_EINVAL (-1)
#define MBIK_ENOMEM (-2)
#define MBIK_EHIP (-3)
#define MBIK_EUNSUPPORTED (-4)
#define MBIK_ENODEV (-5)

#define MBIK_ABI_VERSION 8

typedef struct mbik_plan mbik_plan;
typedef struct mbik_group mbik_group;
typedef struct mbik_multi mbik_multi;

/* == IKEffectorTemplate3D (src/ik_effector_template_3d.h:40-47). */
typedef struct mbik_pin {
	int32_t bone;                      /* skeleton bone index (template name) */
	float weight;                      /* reference default 0.0 */
	float direction_priorities[3];     /* reference default (0.2, 0, 0.2) */
	float motion_propagation_factor;   /* reference default 1.0, clamped to [0,1] */
} mbik_pin;

/* == one ManyBoneIK3D "constraints/<i>" entry (many_bone_ik_3d.cpp:1037-1067). */
typedef struct mbik_constraint {
	int32_t bone;                      /* constraint_names[i] resolved to a bone index */
	int32_t cone_count;                /* kusudama_open_cone_count[i] */
} mbik_constraint;

typedef struct mbik_skeleton_desc {
	int32_t bone_count;
	const int32_t *parents;            /* [bone_count]; -1 = parentless */
	int32_t pin_count;
	const mbik_pin *pins;
	int32_t constraint_count;
	const mbik_constraint *constraints;
	int32_t max_cones;                 /* stride of the cones array */
} mbik_skeleton_desc;

/* ManyBoneIK3D solver properties (many_bone_ik_3d.h:49-68). */
typedef struct mbik_config {
	int32_t iterations_per_frame;      /* reference default 15 */
	float default_damp;                /* radians; reference default deg_to_rad(5) */
	int32_t constraint_mode;           /* reference default false */
	int32_t stabilization_passes;      /* reference default 0 */
	int32_t bone_damp_count;           /* ManyBoneIK3D::bone_damp, usually empty */
	const float *bone_damp;
} mbik_config;

typedef struct mbik_plan_info {
	int32_t abi_version;
	int32_t skeleton_count;
	int32_t bone_count;
	int32_t pin_count;
	int32_t segment_count;
	int32_t level_count;               /* sibling-segment levels solved concurrently */
	int32_t lanes_per_skeleton;
	int32_t skeletons_per_block;
	int32_t max_headings;
	int32_t device;
	int64_t device_bytes;              /* per-skeleton plan tables resident in HBM */
	double algorithmic_bytes_per_skeleton; /* per bone pose in/out 80 B + bone-direction quaternion 16 B + damp 4 B; per effector 64 B; per constrained bone 52 B + 52 B per cone (C2 8,292 B) */
	double algorithmic_flops_per_skeleton; /* SURVEY.md §8(d) per-bone-step formula x bone-steps x iterations */
	int64_t lds_bytes_per_block;       /* LDS of one launch block (spw skeletons + topology tables) */
	int32_t checkpoint_interval;       /* iteration-start globals kept every n-th bone (1 << 20: segment roots only) */
	int32_t heading_staging;           /* mbik_plan_set_heading_staging in effect (0 .. 5) */
	int32_t state_placement;           /* mbik_plan_set_locals_placement in effect (0 / 1 / 2) */
	int32_t waves_per_simd;            /* mbik_plan_set_waves_per_simd in effect (1 / 2) */
	int32_t constraint_slots;          /* slots of mbik_plan_setup_tables' CF / CD (ABI 3) */
	int32_t cf_stride;                 /* floats per slot of CF = 14 + 31*max_cones (ABI 3) */
	int32_t cd_stride;                 /* doubles per slot of CD = 2*max_cones (ABI 3) */
	int32_t libm_variant;              /* mbik_plan_options.libm_variant the plan was created with (ABI 4) */
	int32_t helper_wave;               /* 1 when the current layout launches with the helper wave (ABI 5) */
	int32_t heading_slots;             /* 0x67 when every effector has the reference's default direction
	                                      priorities (x, z > 0, y = 0: ik_effector_template_3d.h:45), so the
	                                      plan launches the kernels built for that heading set; 0 when the
	                                      priorities differ, and each effector's slots are tested at run
	                                      time (ABI 7).  Bits: 0 the origin heading, 1+2a and 2+2a the
	                                      +/- headings of axis a. */
	int32_t wave_roles;                /* 1 when the current layout runs with wave roles
	                                      (mbik_plan_set_wave_roles): lanes_per_skeleton is then the
	                                      number of waves per block (ABI 8) */
} mbik_plan_info;

/* Which reference host the plan reproduces bit for bit (ABI 4).  Godot's Math::sin/cos(float)
 * call the platform ::sinf/::cosf -- glibc on the reference's Linux x86-64 build -- and glibc
 * 2.35 ships two builds of them, picked per CPU by an ifunc; they differ on 12 (sinf) and 22
 * (cosf) of the 2^32 float inputs, and the solve amplifies a 1-ulp difference ~2x per
 * iteration, so the choice is part of the reference's behaviour:
 *   MBIK_LIBM_VARIANT_FMA   (0, default) the FMA build: a reference running on any x86-64
 *                           CPU with FMA (every Intel since Haswell, AMD since Piledriver;
 *                           the GPU boxes' EPYC 9575F);
 *   MBIK_LIBM_VARIANT_SSE2  (1) the SSE2 build: a reference on a CPU without FMA, or with the
 *                           ifunc disabled (GLIBC_TUNABLES=glibc.cpu.hwcaps=-FMA,-AVX2_Usable).
 * acosf has a single build.  The variant applies to the setup tables (cone and twist
 * half-angle sines/cosines, tangent frames) and to the solve's slerp coefficient. */
#define MBIK_LIBM_VARIANT_FMA 0
#define MBIK_LIBM_VARIANT_SSE2 1
typedef struct mbik_plan_options {
	int32_t struct_size;               /* sizeof(mbik_plan_options): later fields are optional */
	int32_t libm_variant;              /* MBIK_LIBM_VARIANT_* */
} mbik_plan_options;

/* Builds the per-topology tables and the per-skeleton setup data for skeletons
 * [0, n_skeletons) from their setup poses, uploads them to `device`.  cones/twist may be
 * NULL when constraint_count == 0. */
int32_t mbik_plan_create(const mbik_skeleton_desc *desc, const mbik_config *config, int32_t n_skeletons,
		const float *setup_pose, const float *cones, const float *twist, int32_t device, mbik_plan **out_plan);
/* mbik_plan_create with creation options (ABI 4; opts NULL = the defaults). */
int32_t mbik_plan_create_opts(const mbik_skeleton_desc *desc, const mbik_config *config, const mbik_plan_options *opts,
		int32_t n_skeletons, const float *setup_pose, const float *cones, const float *twist, int32_t device,
		mbik_plan **out_plan);
void mbik_plan_destroy(mbik_plan *plan);
/* Plan serialisation to a flat binary (checkpoint / resume, or a plan built once and shipped):
 * the creation inputs (topology, pins, constraints, config), the per-skeleton setup tables as
 * they are on the device (including any mbik_plan_rebuild_setup), the layout overrides and
 * autotune choice, and for constraint_mode the persistent node caches.  mbik_plan_save with
 * buf == NULL stores the needed size in *size; otherwise capacity must be at least that
 * (MBIK_EINVAL).  It reads the device tables back, so the streams using the plan must be
 * idle.  mbik_plan_load rebuilds the plan on `device` from such a buffer; the loaded plan
 * solves bitwise like the saved one.  Format version 5 (1-4 still load), little-endian,
 * host-independent. */
int32_t mbik_plan_save(const mbik_plan *plan, void *buf, uint64_t capacity, uint64_t *size);
int32_t mbik_plan_load(const void *buf, uint64_t size, int32_t device, mbik_plan **out_plan);
int32_t mbik_plan_get_info(const mbik_plan *plan, mbik_plan_info *out);
/* Launch-shape override (0 = automatic).  lanes_per_skeleton must be a power of two <= 64. */
int32_t mbik_plan_set_launch(mbik_plan *plan, int32_t lanes_per_skeleton);
/* Full layout override, each 0 = automatic: lanes per skeleton (power of two <= 64),
 * skeletons per block (<= 64 / lanes), and the checkpoint interval of the iteration-start
 * globals kept in LDS (1 = every bone; n = every n-th bone of a segment from its root, plus
 * the parents of segment roots).  Results do not depend on the layout. */
int32_t mbik_plan_set_layout(mbik_plan *plan, int32_t lanes_per_skeleton, int32_t skeletons_per_block,
		int32_t global_checkpoint_interval);
/* Heading staging of segments with several effectors (default 1): the lanes of the
 * segment's group split its effectors' heading builds and stage the QCP terms in LDS.  0:
 * every lane of the group solves the segment alone from registers -- no staging LDS, so
 * more skeletons fit per CU, at a longer step for those segments.  2: only the translating
 * root segments (the ones with the most effectors) are staged; 3: only segments with two or
 * more effectors (whose path walks the lanes split).
 * 4: split-exchange -- no segment is staged in memory; the lanes of a multi-effector segment's
 * group build alternate effectors' headings and read each other's through cross-lane
 * operations (ds_bpermute), every lane summing all of them in the reference's order; 5: the
 * translating root segments staged as in 2, the other multi-effector segments split-exchanged
 * as in 4.  Modes 4 and 5 are served by the two-waves-per-SIMD build only
 * (mbik_plan_set_waves_per_simd 2): with one wave per SIMD their split-exchange segments are
 * solved as in 0 (each lane alone); when the setup tables need 64-bit indices
 * (mbik_plan_set_table_addressing) 4 becomes 0 and 5 becomes 2, which
 * mbik_plan_info.heading_staging then reports.  -1: automatic (mbik_plan_autotune times them; it picks 4 for the
 * residency-bound BASELINE configs C3-C5).  Not used by constraint_mode (its lanes own tree
 * ranges).  Results do not depend on it. */
int32_t mbik_plan_set_heading_staging(mbik_plan *plan, int32_t staging);
/* Where the solve keeps its per-skeleton state during a launch: 0 (default) all in LDS;
 * 1 the bone local transforms in a per-skeleton device-memory area (L2-resident; about half
 * the LDS of a long-chain skeleton), the rest in LDS; 2 all of it in device memory (LDS holds
 * only the block's topology copy).  Less LDS per skeleton, more skeletons resident per CU.
 * -1: automatic (mbik_plan_autotune times each).  Results do not depend on it. */
int32_t mbik_plan_set_locals_placement(mbik_plan *plan, int32_t placement);
/* Waves per SIMD the solve kernel is built for: 1 (default) the whole register file; 2 at
 * most 256 registers (some spilled), so two blocks share a SIMD -- for launches too large to
 * be resident at once.  -1: automatic (mbik_plan_autotune times both).  Plans with
 * stabilization passes always use 1.  Results do not depend on it. */
int32_t mbik_plan_set_waves_per_simd(mbik_plan *plan, int32_t waves);
/* Helper wave: 1 launches two waves per block, on two SIMDs of a CU; the second runs the
 * global pass and computes each bone-step's parent-side work (the parent's global and its
 * inverse, the bone's global, the slerp's target side, the bone-direction and twist frames)
 * one step ahead of the solving wave, which then runs only what depends on the step's fit.
 * It pays where SIMDs would otherwise idle: launches resident at once with their state in LDS
 * (a frame of BASELINE configs[1]).  Serves state placement 0 without stabilization; other
 * layouts ignore it.  0 off, -1 (default) automatic: off until mbik_plan_autotune has timed
 * it on a fully resident launch.  Results do not depend on it.
 * Every wait between the two waves has an exit: a wait whose counter has not moved for two
 * seconds (a real wait lasts at most one iteration of the partner) gives up for the rest of
 * the launch.  The block's skeletons are then written as failures -- identity rotation, NaN
 * position, unit scale for every solved bone -- with their mbik_solve_checked flag set, and
 * the plan's own timeout flag is raised (mbik_plan_status).  The synchronous calls
 * (mbik_solve_host, mbik_plan_autotune) return MBIK_EHIP for their own launch; the
 * asynchronous ones (mbik_solve, mbik_solve_checked, mbik_segment_solve, mbik_group_solve)
 * return MBIK_EHIP, without launching, on the plan's next call, which clears the flag.
 * Plans never see each other's timeouts. */
int32_t mbik_plan_set_helper_wave(mbik_plan *plan, int32_t helper);
/* Wave roles (ABI 8): one wavefront per segment, a lane per skeleton.  A block is 64 skeletons
 * and K waves; the K roles of the sibling-segment schedule (lanes_per_skeleton, a power of two
 * 2..8; 8 only with two waves per SIMD) are the block's waves instead of K lanes of one wave, so
 * sibling segments run on separate waves that meet at a barrier per tree level, each wave reads
 * its segment's topology as wave-uniform values, and no lane repeats another lane's work (a
 * segment with fewer lanes than effectors is solved by one wave, effector by effector, in the
 * reference's order: ik_bone_segment_3d.cpp:210-240).  The whole solve state lives in device
 * memory (state placement 2).  1 on, 0 off, -1 (default) automatic: off until mbik_plan_autotune
 * has timed it.  constraint_mode plans have their own wave-roles kernel (2, 4 or 8 roles; a
 * multi-effector segment's effector reads split over its waves where their dirty chains are
 * disjoint).  Plans with stabilization passes and plans whose setup tables (or constraint_mode
 * node caches) need 64-bit indices run without it.  Results do not depend on it. */
int32_t mbik_plan_set_wave_roles(mbik_plan *plan, int32_t roles);
/* Status of a plan's earlier launches, for callers that poll instead of waiting for the next
 * call's return code (ABI 6): *status = MBIK_STATUS_HELPER_TIMEOUT when a helper-wave launch of
 * this plan that has completed timed out (see mbik_plan_set_helper_wave), else 0.  Reading
 * does not clear it. */
#define MBIK_STATUS_HELPER_TIMEOUT 1u
int32_t mbik_plan_status(const mbik_plan *plan, uint32_t *status);
/* Test hook (ABI 6): the helper wave stops before producing record drop_record of each block
 * (-1: never), and the handshake deadline is timeout_us microseconds (0: the default two
 * seconds) -- to exercise the timeout path above.  Not for production use. */
int32_t mbik_plan_debug_helper(mbik_plan *plan, int32_t drop_record, int32_t timeout_us);
/* How the solve addresses the per-skeleton setup tables (D, CF, CD).  0 (default): with
 * 32-bit offsets from a buffer resource when every table is below 4 GiB, else with 64-bit
 * element indices.  1: always 64-bit indices (state placement 0 only: placements 1 and 2 need
 * the 32-bit form and return MBIK_EUNSUPPORTED, which mbik_plan_autotune skips).  Plans whose
 * tables reach 4 GiB therefore solve in placement 0, and mbik_group_solve launches them on
 * their own.  Results do not depend on it. */
int32_t mbik_plan_set_table_addressing(mbik_plan *plan, int32_t wide);
/* Re-derives the per-skeleton setup data (bone-direction frames, Kusudama cones, tangent
 * circles and twist frames -- what mbik_plan_create computes on the host from the setup
 * pose, ManyBoneIK3D::_bone_list_changed many_bone_ik_3d.cpp:1011-1068) on the GPU for
 * skeletons [first, first+count), from device buffers indexed from skeleton `first`:
 * setup_pose [count][bones][10], cones [count][constraints][max_cones][4], twist
 * [count][constraints][2].  Same topology, pins and constraint bones as the plan; the
 * result equals the host builder's.  Synchronizes hip_stream. */
int32_t mbik_plan_rebuild_setup(mbik_plan *plan, int32_t first, int32_t count, const float *setup_pose,
		const float *cones, const float *twist, void *hip_stream);
/* GPU-side plan build for a crowd of distinct rigs: the segmentation, effector
 * lists, heading weights (generate_default_segments ik_bone_segment_3d.cpp:352-427,
 * update_pinned_list :74-88, create_headings_arrays / recursive_create_penalty_array
 * :281-343), damping, effector paths and constraint slots of every rig are built on `device`,
 * one GPU thread per rig (topo.h), and each rig's per-skeleton frames by mbik_setup_kernel
 * from device buffers: setup_pose[i] [n_skeletons[i]][bones][10], cones[i] / twist[i] as for
 * mbik_plan_rebuild_setup (NULL for rigs without constraints).  The host only reads the built
 * tables back to size the launch layout; the damping cosines cos(damp/2) come from the host's
 * libm (the reference's: the device's double cos differs in the last bit on ~1.6 % of inputs).
 * out_plans[i] receives rig i's plan (equal to what mbik_plan_create builds from the same
 * inputs); on error no plan is returned.  Combine them with mbik_group_create. */
int32_t mbik_plan_create_device(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs,
		const int32_t *n_skeletons, const float *const *setup_pose, const float *const *cones, const float *const *twist,
		int32_t device, mbik_plan **out_plans);
/* mbik_plan_create_device with creation options, the same for every rig (ABI 4). */
int32_t mbik_plan_create_device_opts(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs,
		const mbik_plan_options *opts, const int32_t *n_skeletons, const float *const *setup_pose, const float *const *cones,
		const float *const *twist, int32_t device, mbik_plan **out_plans);
/* Self-test of the GPU topology build: builds the n rigs with topo.h on `device` (or on the
 * host when device < 0: the same code) and compares every topology table with the host
 * builder's (mbik_plan_create's).  mismatches[i] = number of differing tables of rig i (0 when
 * equal, also when both refuse the rig with the same error); mbik_last_error() names the
 * first difference. */
int32_t mbik_selftest_topology(int32_t n_rigs, const mbik_skeleton_desc *descs, const mbik_config *configs, int32_t device,
		int32_t *mismatches);
/* Copies the plan's per-skeleton setup tables to host buffers (any may be NULL):
 * D [bones][9][n], CF [slots][14 + 31*max_cones][n] floats, CD [slots][2*max_cones][n]
 * doubles, n = skeleton_count; slots = constraints on bones in the IK bone list
 * (mbik_plan_info.constraint_slots; the strides are mbik_plan_info.cf_stride / cd_stride). */
int32_t mbik_plan_setup_tables(const mbik_plan *plan, float *D, float *CF, double *CD);
/* Diagnostic: how many one-wave blocks using lds_bytes_per_block of LDS one CU of the plan's
 * device holds at once (the runtime occupancy query for the plan's kernel). */
int32_t mbik_plan_resident_blocks(const mbik_plan *plan, int64_t lds_bytes_per_block);
/* Times candidate layouts on a real batch and keeps the fastest as the plan's layout: lanes
 * per skeleton (the widest sibling level or half of it), skeletons per block, checkpoint
 * interval, heading staging, state placement and waves per SIMD; dimensions pinned by the
 * setters above (a value other than 0 / -1) are kept.  A launch that is fully resident at the
 * default layout is left as it is (one skeleton's chain bounds it).  Runs the solve several
 * times from pose_in into pose_out (identical results); candidates within 1.5 % of the fastest
 * count as tied and the earliest in the candidate order wins, so that timing noise does not
 * change the pick from box to box; the two buffers must not overlap
 * (MBIK_EINVAL otherwise).  Synchronizes hip_stream.  The chosen layout is
 * fixed afterwards; mbik_plan_set_layout(plan, 0, 0, 0) and the staging / placement / waves
 * setters with -1 return to the defaults. */
int32_t mbik_plan_autotune(mbik_plan *plan, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out, void *hip_stream);

/* One frame for skeletons [first, first+count): device pointers (hipMalloc'd, on the
 * plan's device), asynchronous on hip_stream (NULL = default stream).  pose_in, targets
 * and pose_out are indexed from skeleton `first`; pose_out may equal pose_in (in place).
 *
 * Size limits (MBIK_EUNSUPPORTED, from mbik_plan_create or the first solve):
 *   - an effector's path from the root may hold at most MBIK_MAX_PATH_BONES bones;
 *   - the LDS of one launch block, mbik_plan_info.lds_bytes_per_block = the topology tables
 *     plus the solve state of its skeletons (state placement 0 keeps ~12 floats per bone and
 *     ~25 per pin per skeleton there, placement 2 none), must fit MBIK_MAX_LDS_BYTES; the
 *     automatic layout shrinks skeletons per block and moves state to device memory first,
 *     so only the topology tables of a very large rig (several thousand bones) hit this;
 *   - constraint_mode stages its per-lane stacks in LDS with the same limit. */
#define MBIK_MAX_PATH_BONES 4096
#define MBIK_MAX_LDS_BYTES (160 * 1024)
int32_t mbik_solve(mbik_plan *plan, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out, void *hip_stream);
/* mbik_solve plus a per-skeleton status byte (device buffer of `count` bytes, indexed from
 * skeleton `first`): nonfinite[i] = 1 when any bone of skeleton first+i ended the frame with
 * a non-finite basis, which is written out as the identity rotation exactly as
 * IKBone3D::set_skeleton_bone_pose does (ik_bone_3d.cpp:174-176); 0 otherwise.  The
 * reference reports nothing; the flag lets a caller find the skeletons it silently reset. */
int32_t mbik_solve_checked(mbik_plan *plan, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out, uint8_t *nonfinite, void *hip_stream);
/* Same with host buffers; synchronous (copies in, solves, copies out). */
int32_t mbik_solve_host(mbik_plan *plan, int32_t first, int32_t count, const float *pose_in, const float *targets,
		float *pose_out);
/* == IKEffector3D::update_target_global_transform for every pin of skeletons [first,
 * first+count) (ik_effector_3d.cpp:77-84, called by _update_ik_bones_transform,
 * many_bone_ik_3d.cpp:91-102): targets[s][e] = skeleton_global[s].affine_inverse() *
 * target_global[s][e] where visible[s][e] != 0 (visible NULL = every target node visible in
 * the tree); elsewhere targets[s][e] keeps its previous value, as the reference keeps
 * target_relative_to_skeleton_origin.  Transforms are 12 floats (basis rows, origin):
 * skeleton_global [count][12], target_global and targets [count][pins][12], visible
 * [count][pins] bytes; device pointers indexed from `first`, asynchronous on hip_stream. */
int32_t mbik_capture_targets(mbik_plan *plan, int32_t first, int32_t count, const float *skeleton_global,
		const float *target_global, const uint8_t *visible, float *targets, void *hip_stream);

/* Heterogeneous batches: several plans (distinct rigs, e.g. a crowd of different characters)
 * solved by ONE launch, each plan with its own layout.  The reference runs one
 * ManyBoneIK3D::_process_modification per rig (many_bone_ik_3d.cpp:645-694); a group is
 * that loop over rigs, fused.  Plans stay owned by the caller and must outlive the group;
 * all on one device.  constraint_mode and pinless plans run their own launches in order. */
int32_t mbik_group_create(mbik_plan *const *plans, int32_t n_plans, mbik_group **out_group);
/* One frame of every plan in the group: per plan i, skeletons [first[i], first[i]+count[i])
 * (first NULL = 0, count NULL = the plan's skeleton count), device buffers pose_in[i],
 * targets[i], pose_out[i] as for mbik_solve.  Asynchronous on hip_stream; calls on one group
 * are stream-ordered (use one stream per group). */
int32_t mbik_group_solve(mbik_group *group, const int32_t *first, const int32_t *count, const float *const *pose_in,
		const float *const *targets, float *const *pose_out, void *hip_stream);
void mbik_group_destroy(mbik_group *group);

/* Multi-GPU in one process (ABI 8): one batch of skeletons sharded over several
 * plans, typically one per GPU, for an engine that is a single process (Godot is): contiguous
 * shards in plan order -- plan i owns skeletons [off_i, off_i + N_i) of the batch, off_i the sum
 * of the earlier plans' skeleton counts -- solved concurrently, each on its plan's device, with
 * the poses gathered to the root device by peer copies over xGMI (no collective library: the
 * solve has no exchange step).  The plans must agree on bone and pin counts (any topology,
 * layout or setup data otherwise) and stay owned by the caller; they must outlive the handle and
 * must not be solved elsewhere while a mbik_multi_solve on them is in flight.
 *   flags MBIK_MULTI_STAGE_ALL: stage every shard through the handle's own device buffers, even a
 *   shard whose plan lives on the root device (the copy path a one-GPU machine can test). */
#define MBIK_MULTI_STAGE_ALL 1u
int32_t mbik_multi_create(mbik_plan *const *plans, int32_t n_plans, int32_t root_device, uint32_t flags, mbik_multi **out);
/* One frame of the whole batch.  pose_in / targets / pose_out are device buffers on the root
 * device holding every skeleton ([total][bones][10], [total][pins][12]; pose_out may equal
 * pose_in).  Asynchronous on root_stream (a stream of the root device, NULL = its default
 * stream): each plan's work -- the copy of its shard to its device, its mbik_solve, the copy of
 * its poses back into pose_out -- runs on a stream the handle owns on the plan's device, after
 * everything already queued on root_stream, and root_stream waits for all of them, so work
 * queued after the call sees the gathered poses.  Shards whose plan lives on the root device
 * solve in place in the caller's buffers (unless MBIK_MULTI_STAGE_ALL).  Calls on one handle are
 * ordered by root_stream; use one root stream per handle.  Returns the first error; a helper-wave
 * timeout of any plan is reported as by mbik_solve.  Shards run in plan order and the first
 * failing shard ends the call: pose_out is then defined only for the shards before it, and
 * root_stream still waits for everything the call queued (so the buffers are free to reuse once
 * root_stream reaches that point). */
int32_t mbik_multi_solve(mbik_multi *multi, const float *pose_in, const float *targets, float *pose_out, void *root_stream);
/* The batch size (the plans' skeleton counts summed) and shard offsets (off[n_plans + 1],
 * may be NULL). */
int64_t mbik_multi_skeletons(const mbik_multi *multi, int64_t *off);
void mbik_multi_destroy(mbik_multi *multi);

/* Runs IKBoneSegment3D::segment_solver() once on `segment` (index in post-order segment
 * numbering of mbik_plan_segment_table) for every skeleton in [first, first+count), updating
 * pose_inout in place (device pointers).  No pose write-back conversion is skipped: the
 * output is the Skeleton3D pose of every IK bone after that call.
 * segment_solver's other arguments are not parameters here:
 *   p_damp / p_default_damp / p_constraint_mode  come from the plan (mbik_config's bone_damp,
 *                         default_damp, constraint_mode), as the reference passes its own
 *                         members (many_bone_ik_3d.cpp:685-693);
 *   p_current_iteration / p_total_iteration  are accepted by segment_solver but never reach
 *                         _set_optimal_rotation (ik_bone_segment_3d.cpp:94 calls it without them,
 *                         so its slerp weight is always 0 and every iteration is alike); the
 *                         solve has no use for them, and a caller that tracks them loses nothing. */
int32_t mbik_segment_solve(mbik_plan *plan, int32_t segment, int32_t first, int32_t count, float *pose_inout,
		const float *targets, void *hip_stream);
/* Segment table: for each segment, its root bone, tip bone and parent segment (-1). */
int32_t mbik_plan_segment_table(const mbik_plan *plan, int32_t *root_bone, int32_t *tip_bone, int32_t *parent_segment,
		int32_t capacity);

/* Host-only (no device needed): runs the _bone_list_changed segmentation for `desc` and
 * reports the solve order.  bone_list receives ManyBoneIK3D::bone_list (capacity
 * bone_count), segment_* receive the post-order segment table (capacity bone_count), and
 * segment_headings the heading count of each segment.  Returns the segment count. */
int32_t mbik_describe_topology(const mbik_skeleton_desc *desc, const mbik_config *config, int32_t *bone_list,
		int32_t *bone_list_count, int32_t *segment_root, int32_t *segment_tip, int32_t *segment_parent,
		int32_t *segment_headings);

/* Device self-test of the kernel's own float primitives against the compiler's IEEE ones,
 * over every float bit pattern (2^32 inputs, ~1 s): out[0] = inputs where the solve's square
 * root differs from the correctly rounded sqrtf (non-NaN results), out[1] = inputs where
 * exactly one of them is NaN.  Both must be 0 (gd_math.h: gd_sqrt). */
int32_t mbik_selftest_math(int32_t device, uint64_t out[2]);

/* Device known-answer tests (ABI 8): the solve kernel's own device functions on the inputs of
 * the reference's unit tests (tests/test_qcp.h:40-113, tests/test_ik_kusudama_3d.h:38-156,
 * tests/test_ik_node_3d.h:39-106), so the HIP code itself -- not only the CPU oracle -- is
 * checked against their expectations.
 * mbik_selftest_qcp: QCP::weighted_superpose + get_translation (qcp.cpp:220-248, 135-137) of n
 *   pairs (moved, target: [n][3]; weights [n]), with eigenvector precision `precision` (the solve
 *   uses 1e-6, ik_bone_segment_3d.h:85), through the primitives of the solve's one-lane heading
 *   branch: out[0..3] the rotation (x, y, z, w), out[4..6] the translation; out[7..13] the same
 *   from the select-form normalizations of the one-wave builds.
 * mbik_selftest_point_in_limits: IKKusudama3D::get_local_point_in_limits (ik_kusudama_3d.cpp:
 *   273-332) through the solve's own local_point_in_limits on the plan's setup tables (constraint
 *   slot `slot`, i.e. the slot-th constraint on a bone of the IK bone list, of skeleton
 *   `skeleton`): out[0..2] / in_bounds[0] the plain form, out[3..5] / in_bounds[1] the select form.
 * mbik_selftest_xform: Transform3D as the IKNode3D tree uses it (ik_node_3d.cpp:56-113), 12 floats
 *   (basis rows, origin): op 0 out = a * b, op 1 out = a.affine_inverse() (b unused). */
int32_t mbik_selftest_qcp(int32_t n, const float *moved, const float *target, const double *weights, int32_t translate,
		double precision, int32_t device, float out[14]);
int32_t mbik_selftest_point_in_limits(const mbik_plan *plan, int32_t slot, int32_t skeleton, const float point[3], float out[6],
		double in_bounds[2]);
int32_t mbik_selftest_xform(int32_t op, const float a[12], const float b[12], int32_t device, float out[12]);

/* Device self-test of the kernel's float quotients (gd_math.h: an fp64 reciprocal with a
 * residual correction, or one rounding for power-of-two numerators) against IEEE division:
 * out[c] = mismatching results of class c below (two NaNs compare equal), out[8 + 2c] and
 * out[9 + 2c] the operand bit patterns of one mismatch.  All counts must be 0.
 *   SPECIALS          every pair of 24 special values (zeros, infinities, NaNs, denormals, extremes)
 *   ALL_DIVIDENDS     all 2^32 dividends for 12 divisors
 *   RANDOM            random_iterations x 2^21 random pairs (free and close exponents)
 *   MIDPOINTS         random_iterations x 2^21 constructed denormal midpoint quotients
 *   POW2_NUMERATOR    0.5 / b, 1 / b, 2 / b for all 2^32 divisors
 *   NORMALIZE         a / sqrtf(l) (normalized()) and the root itself for all 2^32 l, 8 values of a */
#define MBIK_DIV_SPECIALS 0
#define MBIK_DIV_ALL_DIVIDENDS 1
#define MBIK_DIV_RANDOM 2
#define MBIK_DIV_MIDPOINTS 3
#define MBIK_DIV_POW2_NUMERATOR 4
#define MBIK_DIV_NORMALIZE 5
int32_t mbik_selftest_div(int32_t device, uint64_t random_iterations, uint64_t out[20]);

/* Device self-test of the solve's transcendental call sites against values the caller
 * computed with the host's libm (the reference's: Godot's Math::sin/cos/acos call ::sinf,
 * ::cosf, ::acosf and ::sin/::cos; glibc on Linux x86-64).  For fn = SINF, COSF, ACOSF,
 * SLERP_SCALE0 and COS_F64_OF_F32 the inputs are the float bit patterns first ..
 * first+count-1 (first + count <= 2^32); for COS_F64 they are `inputs` (device, count
 * doubles).  expected (device): count floats (SINF..SLERP_SCALE0) or doubles (the two COS
 * variants).  out[0] = results whose bits differ (two NaNs compare equal), out[1] = the
 * lowest differing index (~0 when none).  Synchronizes hip_stream.
 *   SINF, COSF, ACOSF    sin_f / cos_f / acos_f of gd_math.h (glibc 2.35 restated)
 *   SLERP_SCALE0         (float)(sin((double)w) / (double)sinf(w)): Quaternion::slerp's
 *                        weight-0 coefficient (ik_bone_segment_3d.cpp:148-151)
 *   COS_F64_OF_F32       cos((double)x): a cone radius cosine (ik_open_cone_3d.h:47-56)
 *   COS_F64              cos(x): tangent-radius cosines (ik_open_cone_3d.cpp:36-120)
 *   SINF_SSE2, COSF_SSE2, SLERP_SCALE0_SSE2   the same for a plan created with
 *                        libm_variant = MBIK_LIBM_VARIANT_SSE2 (compare with a host libm
 *                        whose FMA ifunc is disabled: GLIBC_TUNABLES=glibc.cpu.hwcaps=-FMA,-AVX2_Usable)
 *   ACOSF_UNIT           the slerp's acosf call site: the branch-free form for -0.5 < x < 1,
 *                        acosf elsewhere; compare with the host acosf */
#define MBIK_LIBM_SINF 0
#define MBIK_LIBM_COSF 1
#define MBIK_LIBM_ACOSF 2
#define MBIK_LIBM_SLERP_SCALE0 3
#define MBIK_LIBM_COS_F64_OF_F32 4
#define MBIK_LIBM_COS_F64 5
#define MBIK_LIBM_SINF_SSE2 6
#define MBIK_LIBM_COSF_SSE2 7
#define MBIK_LIBM_SLERP_SCALE0_SSE2 8
#define MBIK_LIBM_ACOSF_UNIT 9
int32_t mbik_selftest_libm(int32_t fn, uint64_t first, uint64_t count, const double *inputs, const void *expected,
		uint64_t out[3], void *hip_stream);

const char *mbik_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MBIK_H */
