// Sanitizer drivers' input: one skeleton batch as written by tests/test_sanitizers.py
// (little-endian int32 / float32 stream; see write_case there).
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct san_case {
	int32_t B, P, C, max_cones, iterations, N, constraint_mode, stab, bone_damp_count;
	float default_damp;
	int32_t *parents, *pin_bone, *cons_bone, *cons_ncones;
	float *pin_weight, *pin_prio, *pin_prop, *bone_damp, *pose, *targets, *cones, *twist;
} san_case;

static void *san_read(FILE *f, size_t n) {
	void *p = malloc(n ? n : 1);
	if (!p || (n && fread(p, 1, n, f) != n)) {
		fprintf(stderr, "short case file\n");
		exit(3);
	}
	return p;
}

static san_case san_load(const char *path) {
	san_case c;
	memset(&c, 0, sizeof(c));
	FILE *f = fopen(path, "rb");
	if (!f) {
		fprintf(stderr, "cannot open %s\n", path);
		exit(3);
	}
	char magic[4];
	if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "MBKC", 4) != 0) {
		fprintf(stderr, "not a case file\n");
		exit(3);
	}
	int32_t *hdr = (int32_t *)san_read(f, 9 * sizeof(int32_t));
	c.B = hdr[0]; c.P = hdr[1]; c.C = hdr[2]; c.max_cones = hdr[3]; c.iterations = hdr[4]; c.N = hdr[5];
	c.constraint_mode = hdr[6]; c.stab = hdr[7]; c.bone_damp_count = hdr[8];
	free(hdr);
	float *dd = (float *)san_read(f, sizeof(float));
	c.default_damp = *dd;
	free(dd);
	const size_t B = (size_t)c.B, P = (size_t)c.P, C = (size_t)c.C, N = (size_t)c.N, MC = (size_t)c.max_cones;
	c.parents = (int32_t *)san_read(f, B * 4);
	c.pin_bone = (int32_t *)san_read(f, P * 4);
	c.pin_weight = (float *)san_read(f, P * 4);
	c.pin_prio = (float *)san_read(f, P * 12);
	c.pin_prop = (float *)san_read(f, P * 4);
	c.cons_bone = (int32_t *)san_read(f, C * 4);
	c.cons_ncones = (int32_t *)san_read(f, C * 4);
	c.bone_damp = (float *)san_read(f, (size_t)c.bone_damp_count * 4);
	c.pose = (float *)san_read(f, N * B * 10 * 4);
	c.targets = (float *)san_read(f, N * P * 12 * 4);
	c.cones = (float *)san_read(f, N * C * MC * 4 * 4);
	c.twist = (float *)san_read(f, N * C * 2 * 4);
	fclose(f);
	return c;
}

static void san_free(san_case *c) {
	free(c->parents); free(c->pin_bone); free(c->cons_bone); free(c->cons_ncones); free(c->pin_weight);
	free(c->pin_prio); free(c->pin_prop); free(c->bone_damp); free(c->pose); free(c->targets); free(c->cones);
	free(c->twist);
}
