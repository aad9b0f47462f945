/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * Host reference values for the device's transcendental call sites (mbik_selftest_libm,
 * tests/test_gpu_libm.py), computed with the platform libm -- what the reference calls
 * (Godot's Math::sin/cos/acos forward to ::sinf/::cosf/::acosf and ::sin/::cos,
 * core/math/math_funcs.h) -- and a check of glibc_libm.h against that libm.
 * Built with -fno-builtin so every call reaches libm.so at run time.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#define GLIBC_SINCOSF_FMA 1
#include "glibc_libm.h"

/* function codes, as MBIK_LIBM_* in include/mbik.h */
enum { L_SINF, L_COSF, L_ACOSF, L_SLERP_SCALE0, L_COS_F64_OF_F32, L_COS_F64 };

static float bits_f(uint64_t u) { return gl_asfloat((uint32_t)u); }

/* Quaternion::slerp at weight 0 (Godot 4.3 quaternion.cpp; ik_bone_segment_3d.cpp:148-151):
 * sinom = Math::sin(omega) (float), scale0 = Math::sin((1.0 - 0) * omega) / sinom. */
static float slerp_scale0(float omega) {
	float sinom = sinf(omega);
	return (float)(sin((1.0 - 0.0f) * omega) / sinom);
}

typedef struct {
	int fn;
	uint64_t first, lo, hi;
	const double *in;
	void *out;
} fill_job;

static void *fill_run(void *arg) {
	fill_job *j = arg;
	float *of = j->out;
	double *od = j->out;
	for (uint64_t i = j->lo; i < j->hi; i++) {
		float x = bits_f(j->first + i);
		switch (j->fn) {
		case L_SINF: of[i] = sinf(x); break;
		case L_COSF: of[i] = cosf(x); break;
		case L_ACOSF: of[i] = acosf(x); break;
		case L_SLERP_SCALE0: of[i] = slerp_scale0(x); break;
		case L_COS_F64_OF_F32: od[i] = cos((double)x); break;
		default: od[i] = cos(j->in[i]); break;
		}
	}
	return NULL;
}

/* out[i] = f(input i) for i in [0, count): inputs are the float bit patterns first + i, or
 * in[i] for L_COS_F64.  out holds floats (codes 0-3) or doubles (4, 5). */
int32_t oracle_libm_fill(int32_t fn, uint64_t first, uint64_t count, const double *in, void *out, int32_t n_threads) {
	if (fn < L_SINF || fn > L_COS_F64 || (fn == L_COS_F64 && !in) || !out) return -1;
	if (n_threads < 1) n_threads = 1;
	if (n_threads > 256) n_threads = 256;
	pthread_t th[256];
	fill_job jobs[256];
	for (int t = 0; t < n_threads; t++) {
		fill_job j = {fn, first, count * t / n_threads, count * (t + 1) / n_threads, in, out};
		jobs[t] = j;
		pthread_create(&th[t], NULL, fill_run, &jobs[t]);
	}
	for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
	return 0;
}

/* glibc_libm.h against the platform libm (codes 0-2) on inputs first, first + stride, ...
 * (count of them).  Returns the number of differing results; *first_bad = the first
 * differing bit pattern (unchanged if none). */
uint64_t oracle_libm_restated_mismatches(int32_t fn, uint64_t first, uint64_t count, uint64_t stride, uint64_t *first_bad) {
	uint64_t bad = 0;
	for (uint64_t k = 0; k < count; k++) {
		uint64_t u = first + k * stride;
		float x = bits_f(u), a, b;
		if (fn == L_SINF) { a = sinf(x); b = glibc_sinf(x); }
		else if (fn == L_COSF) { a = cosf(x); b = glibc_cosf(x); }
		else { a = acosf(x); b = glibc_acosf(x); }
		if (!((isnan(a) && isnan(b)) || gl_asuint(a) == gl_asuint(b))) {
			if (!bad && first_bad) *first_bad = u;
			bad++;
		}
	}
	return bad;
}
