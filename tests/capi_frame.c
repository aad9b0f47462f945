/*
 * capi_frame.c -- a plain C99 consumer of include/mbik.h and libmbik.so: the frame loop of
 * INTEGRATION.md §3, as a Godot-side binding would run it for a batch of skeletons
 * (ManyBoneIK3D::_process_modification, src/many_bone_ik_3d.cpp:645-694):
 *
 *   mbik_plan_create                    <- _bone_list_changed (many_bone_ik_3d.cpp:1011-1068)
 *   per frame:
 *     mbik_capture_targets              <- IKEffector3D::update_target_global_transform
 *                                          (ik_effector_3d.cpp:77-84, via _update_ik_bones_transform :91-102)
 *     mbik_solve_checked                <- the iterations x segment_solver loop (:685-693)
 *     read back                         <- _update_skeleton_bones_transform (:104-116)
 *   the frame's output pose is the next frame's input (the Skeleton3D pose the reference
 *   captures again, the warm start)
 * and, when header[7] = S > 0, frame 0 once more through the single-process multi-GPU entry
 * points: the batch split into S plans (contiguous shards), mbik_multi_create (root device 0,
 * MBIK_MULTI_STAGE_ALL so the scatter / gather copies run even with one GPU) and
 * mbik_multi_solve on the whole batch.
 *
 * Built by __graft_entry__.build() (many_bone_ik_amd/build.py: build_capi_frame) with gcc -std=c99
 * -Wall -Wextra -Werror; run by tests/test_capi_frame.py, which compares every frame bitwise
 * with the oracle.
 *
 *   capi_frame <input.bin> <output.bin>
 *
 * input.bin (little-endian): int32 header[8] = {bones B, pins P, constraints C, max_cones MC,
 * iterations, skeletons n, frames F, multi shards S}; int32 parents[B]; int32 pin_bone[P]; float
 * pin_weight[P]; float pin_priority[P][3]; float pin_propagation[P]; int32 cons_bone[C]; int32
 * cons_cones[C]; float default_damp; float setup_pose[n][B][10]; float cones[n][C][MC][4];
 * float twist[n][C][2]; float skeleton_global[n][12]; float target_global[F][n][P][12].
 * output.bin: per frame: float targets[n][P][12] (captured), float pose[n][B][10], uint8
 * nonfinite[n]; then, when S > 0, float pose[n][B][10] (frame 0 through mbik_multi_solve).
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mbik.h"

static unsigned char *g_in;
static size_t g_in_size, g_at;

static void *take(size_t bytes) {
	if (g_at + bytes > g_in_size) {
		fprintf(stderr, "capi_frame: input truncated at byte %zu (+%zu of %zu)\n", g_at, bytes, g_in_size);
		exit(2);
	}
	void *p = g_in + g_at;
	g_at += bytes;
	return p;
}

static int check_mbik(int rc, const char *what) {
	if (rc != MBIK_OK) {
		fprintf(stderr, "capi_frame: %s failed (%d): %s\n", what, rc, mbik_last_error());
		exit(3);
	}
	return rc;
}

static void check_hip(hipError_t e, const char *what) {
	if (e != hipSuccess) {
		fprintf(stderr, "capi_frame: %s failed: %s\n", what, hipGetErrorString(e));
		exit(4);
	}
}

static void *dev_alloc(size_t bytes) {
	void *p = NULL;
	check_hip(hipMalloc(&p, bytes ? bytes : 4), "hipMalloc");
	return p;
}

int main(int argc, char **argv) {
	if (argc != 3) {
		fprintf(stderr, "usage: capi_frame <input.bin> <output.bin>\n");
		return 1;
	}
	FILE *f = fopen(argv[1], "rb");
	if (!f) {
		perror(argv[1]);
		return 1;
	}
	fseek(f, 0, SEEK_END);
	g_in_size = (size_t)ftell(f);
	rewind(f);
	g_in = malloc(g_in_size);
	if (!g_in || fread(g_in, 1, g_in_size, f) != g_in_size) {
		fprintf(stderr, "capi_frame: cannot read %s\n", argv[1]);
		return 1;
	}
	fclose(f);

	const int32_t *hdr = take(8 * sizeof(int32_t));
	const int32_t B = hdr[0], P = hdr[1], C = hdr[2], MC = hdr[3], iterations = hdr[4], n = hdr[5], F = hdr[6], S = hdr[7];
	const int32_t *parents = take((size_t)B * 4);
	const int32_t *pin_bone = take((size_t)P * 4);
	const float *pin_weight = take((size_t)P * 4);
	const float *pin_priority = take((size_t)P * 12);
	const float *pin_propagation = take((size_t)P * 4);
	const int32_t *cons_bone = take((size_t)C * 4);
	const int32_t *cons_cones = take((size_t)C * 4);
	const float *default_damp = take(4);
	const float *setup_pose = take((size_t)n * B * 10 * 4);
	const float *cones = take((size_t)n * C * MC * 4 * 4);
	const float *twist = take((size_t)n * C * 2 * 4);
	const float *skeleton_global = take((size_t)n * 12 * 4);
	const float *target_global = take((size_t)F * n * P * 12 * 4);

	/* _bone_list_changed: pins (IKEffectorTemplate3D), constraints, solver properties */
	mbik_pin *pins = calloc((size_t)(P > 0 ? P : 1), sizeof(mbik_pin));
	mbik_constraint *cons = calloc((size_t)(C > 0 ? C : 1), sizeof(mbik_constraint));
	for (int e = 0; e < P; e++) {
		pins[e].bone = pin_bone[e];
		pins[e].weight = pin_weight[e];
		for (int a = 0; a < 3; a++) pins[e].direction_priorities[a] = pin_priority[3 * e + a];
		pins[e].motion_propagation_factor = pin_propagation[e];
	}
	for (int c = 0; c < C; c++) {
		cons[c].bone = cons_bone[c];
		cons[c].cone_count = cons_cones[c];
	}
	mbik_skeleton_desc desc;
	memset(&desc, 0, sizeof(desc));
	desc.bone_count = B;
	desc.parents = parents;
	desc.pin_count = P;
	desc.pins = pins;
	desc.constraint_count = C;
	desc.constraints = cons;
	desc.max_cones = MC;
	mbik_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	cfg.iterations_per_frame = iterations;
	cfg.default_damp = *default_damp;
	cfg.constraint_mode = 0;
	cfg.stabilization_passes = 0;
	cfg.bone_damp_count = 0;
	cfg.bone_damp = NULL;

	check_hip(hipSetDevice(0), "hipSetDevice");
	mbik_plan *plan = NULL;
	check_mbik(mbik_plan_create(&desc, &cfg, n, setup_pose, C ? cones : NULL, C ? twist : NULL, 0, &plan), "mbik_plan_create");
	mbik_plan_info info;
	check_mbik(mbik_plan_get_info(plan, &info), "mbik_plan_get_info");
	if (info.abi_version != MBIK_ABI_VERSION || info.bone_count != B || info.pin_count != P || info.skeleton_count != n) {
		fprintf(stderr, "capi_frame: plan info does not match the header (abi %d)\n", info.abi_version);
		return 5;
	}

	hipStream_t stream;
	check_hip(hipStreamCreate(&stream), "hipStreamCreate");
	const size_t pose_bytes = (size_t)n * B * 10 * sizeof(float), tg_bytes = (size_t)n * P * 12 * sizeof(float);
	float *d_pose[2] = {dev_alloc(pose_bytes), dev_alloc(pose_bytes)};
	float *d_targets = dev_alloc(tg_bytes), *d_target_global = dev_alloc(tg_bytes);
	float *d_skeleton_global = dev_alloc((size_t)n * 12 * sizeof(float));
	uint8_t *d_nonfinite = dev_alloc((size_t)n);
	check_hip(hipMemcpy(d_pose[0], setup_pose, pose_bytes, hipMemcpyHostToDevice), "hipMemcpy pose");
	check_hip(hipMemcpy(d_skeleton_global, skeleton_global, (size_t)n * 12 * sizeof(float), hipMemcpyHostToDevice),
			"hipMemcpy skeleton_global");
	check_hip(hipMemset(d_targets, 0, tg_bytes), "hipMemset targets");

	FILE *out = fopen(argv[2], "wb");
	if (!out) {
		perror(argv[2]);
		return 1;
	}
	float *h_targets = malloc(tg_bytes ? tg_bytes : 4), *h_pose = malloc(pose_bytes);
	uint8_t *h_nonfinite = malloc((size_t)n);
	for (int frame = 0; frame < F; frame++) {
		const float *tgl = target_global + (size_t)frame * n * P * 12;
		check_hip(hipMemcpyAsync(d_target_global, tgl, tg_bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync targets");
		/* every target node visible (visible == NULL) */
		check_mbik(mbik_capture_targets(plan, 0, n, d_skeleton_global, d_target_global, NULL, d_targets, stream),
				"mbik_capture_targets");
		float *in = d_pose[frame & 1], *res = d_pose[(frame + 1) & 1];
		check_mbik(mbik_solve_checked(plan, 0, n, in, d_targets, res, d_nonfinite, stream), "mbik_solve_checked");
		check_hip(hipMemcpyAsync(h_targets, d_targets, tg_bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
		check_hip(hipMemcpyAsync(h_pose, res, pose_bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
		check_hip(hipMemcpyAsync(h_nonfinite, d_nonfinite, (size_t)n, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
		check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");
		uint32_t status = 0;
		check_mbik(mbik_plan_status(plan, &status), "mbik_plan_status");
		if (status != 0) {
			fprintf(stderr, "capi_frame: plan status %u after frame %d\n", status, frame);
			return 6;
		}
		if (fwrite(h_targets, 1, tg_bytes, out) != tg_bytes || fwrite(h_pose, 1, pose_bytes, out) != pose_bytes ||
				fwrite(h_nonfinite, 1, (size_t)n, out) != (size_t)n) {
			fprintf(stderr, "capi_frame: short write\n");
			return 1;
		}
	}
	if (S > 0) {
		/* frame 0 again, sharded: S plans over contiguous skeleton ranges, one mbik_multi */
		mbik_plan **shard = calloc((size_t)S, sizeof(mbik_plan *));
		for (int k = 0; k < S; k++) {
			const int32_t lo = (int32_t)((int64_t)n * k / S), hi = (int32_t)((int64_t)n * (k + 1) / S);
			check_mbik(mbik_plan_create(&desc, &cfg, hi - lo, setup_pose + (size_t)lo * B * 10, C ? cones + (size_t)lo * C * MC * 4 : NULL,
							   C ? twist + (size_t)lo * C * 2 : NULL, 0, &shard[k]),
					"mbik_plan_create (shard)");
		}
		mbik_multi *multi = NULL;
		check_mbik(mbik_multi_create(shard, S, 0, MBIK_MULTI_STAGE_ALL, &multi), "mbik_multi_create");
		if (mbik_multi_skeletons(multi, NULL) != n) {
			fprintf(stderr, "capi_frame: mbik_multi_skeletons != n\n");
			return 7;
		}
		check_hip(hipMemcpyAsync(d_pose[0], setup_pose, pose_bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync pose");
		check_hip(hipMemcpyAsync(d_target_global, target_global, tg_bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync targets");
		check_mbik(mbik_capture_targets(plan, 0, n, d_skeleton_global, d_target_global, NULL, d_targets, stream), "mbik_capture_targets");
		check_mbik(mbik_multi_solve(multi, d_pose[0], d_targets, d_pose[1], stream), "mbik_multi_solve");
		check_hip(hipMemcpyAsync(h_pose, d_pose[1], pose_bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
		check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");
		if (fwrite(h_pose, 1, pose_bytes, out) != pose_bytes) {
			fprintf(stderr, "capi_frame: short write\n");
			return 1;
		}
		mbik_multi_destroy(multi);
		for (int k = 0; k < S; k++) mbik_plan_destroy(shard[k]);
		free(shard);
	}
	fclose(out);
	check_hip(hipFree(d_pose[0]), "hipFree");
	check_hip(hipFree(d_pose[1]), "hipFree");
	check_hip(hipFree(d_targets), "hipFree");
	check_hip(hipFree(d_target_global), "hipFree");
	check_hip(hipFree(d_skeleton_global), "hipFree");
	check_hip(hipFree(d_nonfinite), "hipFree");
	check_hip(hipStreamDestroy(stream), "hipStreamDestroy");
	mbik_plan_destroy(plan);
	free(pins);
	free(cons);
	free(h_targets);
	free(h_pose);
	free(h_nonfinite);
	free(g_in);
	printf("capi_frame: %d frames x %d skeletons OK\n", F, n);
	return 0;
}
