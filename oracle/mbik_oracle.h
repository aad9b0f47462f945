/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle; the product library never does.
 *
 * C API of the CPU restatement of Ughuuu/many_bone_ik's solve path
 * (see ik_oracle.c for the file:line of every function it follows).
 *
 * Parity status: the oracle is pinned against every known-answer test the
 * reference ships (tests/test_qcp.h, tests/test_ik_kusudama_3d.h,
 * tests/test_ik_node_3d.h -> tests/golden/reference_kats.json).  The reference
 * cannot be compiled here (it needs the Godot engine tree), so
 * full-solve behaviour beyond those unit KATs is "parity unpinned" against the
 * reference itself and rests on this restatement.
 *
 * Array layouts (all float32, row-major, one skeleton after another):
 *   pose    [bone][10]  = quaternion x,y,z,w | position x,y,z | scale x,y,z
 *   target  [pin][12]   = basis rows r0 r1 r2 (9) | origin (3)   (skeleton space)
 *   cones   [constraint][max_cones][4] = centre x,y,z | radius (radians)
 *   twist   [constraint][2] = min_angle, range (radians)
 */
#ifndef MBIK_ORACLE_H
#define MBIK_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_desc {
	int32_t bone_count;
	const int32_t *parents;          /* [bone_count], -1 = parentless */
	int32_t pin_count;
	const int32_t *pin_bone;         /* [pin_count] */
	const float *pin_weight;         /* [pin_count] */
	const float *pin_priority;       /* [pin_count][3] */
	const float *pin_propagation;    /* [pin_count] */
	int32_t constraint_count;
	const int32_t *constraint_bone;  /* [constraint_count] */
	const int32_t *constraint_cone_count; /* [constraint_count] */
	int32_t max_cones;
	int32_t iterations;
	float default_damp;
	int32_t constraint_mode;
	int32_t stabilization_passes;
	int32_t bone_damp_count;         /* ManyBoneIK3D::bone_damp (usually empty) */
	const float *bone_damp;
} oracle_desc;

/* Builds one reference object graph per skeleton (== _bone_list_changed). */
void *oracle_create(const oracle_desc *desc, int32_t n_skel, const float *setup_pose,
		const float *cones, const float *twist);
/* One frame per skeleton in [first, first+count): _update_ik_bones_transform +
 * _process_modification + _update_skeleton_bones_transform.  pose_in/targets/pose_out
 * are indexed from skeleton `first`.  trace (optional) receives the pose after every
 * iteration: [count][iterations][bone][10]. */
int32_t oracle_solve(void *h, int32_t first, int32_t count, const float *pose_in,
		const float *targets, float *pose_out, float *trace, int32_t n_threads);
void oracle_destroy(void *h);
/* Introspection for tests: segment/effector structure of skeleton 0. */
int32_t oracle_segment_count(void *h);
int32_t oracle_bone_list(void *h, int32_t *out_bone_ids, int32_t cap);
/* Post-order (children first) segment table of skeleton 0: root bone, tip bone, headings. */
int32_t oracle_segment_table(void *h, int32_t *root, int32_t *tip, int32_t *nh, int32_t cap);
/* One segment_solver() call on segment `post_index` (post-order numbering), in place. */
int32_t oracle_segment_solve(void *h, int32_t post_index, int32_t first, int32_t count, float *pose_inout,
		const float *targets);

/* Unit entry points mirroring the reference's own KATs. */
/* QCP::weighted_superpose (qcp.cpp:220) + get_translation (qcp.cpp:135). */
void oracle_qcp(const float *moved, const float *target, const double *weight, int32_t n,
		int32_t translate, double precision, float *quat_out, float *translation_out);
/* Kusudama built from cones [n][4]; optional tangent centres [n][6] (t1, t2) are set
 * on each cone before add_open_cone (as tests/test_ik_kusudama_3d.h does; cones with
 * a successor get them recomputed).  Pass NULL to skip.  Returns in_bounds[0]. */
double oracle_local_point_in_limits(const float *cones, int32_t n, const float *tangents, const float *point, float *out);
/* use_next: 0 = null successor, 1 = the cone itself, 2 = the following cone */
void oracle_closest_path_point(const float *cones, int32_t n, const float *tangents, int32_t cone_index,
		int32_t use_next, const float *point, float *out);
void oracle_cone_tangents(const float *cones, int32_t n, float *out /* [n][8]: t1, t2, tr, trcos */);
void oracle_xform_mul(const float *a, const float *b, float *out);
void oracle_xform_affine_inverse(const float *a, float *out);
void oracle_basis_to_quat(const float *basis9, float *quat_out);
void oracle_quat_to_basis(const float *q, float *basis9);

#ifdef __cplusplus
}
#endif
#endif
