/* Checks oracle/glibc_libm.h (the restated glibc sinf/cosf/acosf) against the platform libm
 * on all 2^32 float inputs, both FMA and SSE2 contraction variants.  CPU only.
 *
 *   gcc -O2 -ffp-contract=off -fno-builtin -pthread -I oracle tools/libm_exhaustive.c -lm \
 *       -o /tmp/libm_exhaustive && /tmp/libm_exhaustive
 *
 * Output: per function and variant, the number of inputs whose result bits differ (two NaNs
 * count as equal) and the first few differing inputs.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#define GLIBC_SINCOSF_FMA 1
#include "glibc_libm.h"
#undef GL_MADD
static inline float sse_sinf(float), sse_cosf(float);
/* second copy of the sin/cos part with the SSE2 (uncontracted) arithmetic */
#define NOFMA_MADD(a, b, c) ((a) * (b) + (c))
static inline float nofma_poly(double x, double x2, const gl_sincos_t *p, int n) {
	if ((n & 1) == 0) {
		double x3 = x * x2, s1 = NOFMA_MADD(x2, p->s3, p->s2), x7 = x3 * x2, s = NOFMA_MADD(x3, p->s1, x);
		return (float)NOFMA_MADD(x7, s1, s);
	}
	double x4 = x2 * x2, c2 = NOFMA_MADD(x2, p->c4, p->c3), c1 = NOFMA_MADD(x2, p->c1, p->c0), x6 = x4 * x2;
	double c = NOFMA_MADD(x4, p->c2, c1);
	return (float)NOFMA_MADD(x6, c2, c);
}
static inline float sse_sc(float y, int cos) {
	double x = y, s;
	int n;
	const gl_sincos_t *p = &gl_sincosf_table[0];
	if (gl_abstop12(y) < gl_abstop12(0x1.921FB6p-1f)) {
		s = x * x;
		if (gl_abstop12(y) < gl_abstop12(0x1p-12f)) return cos ? 1.0f : y;
		return nofma_poly(x, s, p, cos);
	} else if (gl_abstop12(y) < gl_abstop12(120.0f)) {
		double r = x * p->hpi_inv;
		n = ((int32_t)r + 0x800000) >> 24;
		x = x - n * p->hpi;
		s = p->sign[n & 3];
		if (n & 2) p = &gl_sincosf_table[1];
		return nofma_poly(x * s, x * x, p, n ^ cos);
	} else if (gl_abstop12(y) < gl_abstop12(INFINITY)) {
		uint32_t xi = gl_asuint(y);
		int sign = xi >> 31;
		x = gl_reduce_large(xi, &n);
		s = p->sign[(n + sign) & 3];
		if ((n + sign) & 2) p = &gl_sincosf_table[1];
		return nofma_poly(x * s, x * x, p, n ^ cos);
	}
	return (y - y) / (y - y);
}
static inline float sse_sinf(float y) { return sse_sc(y, 0); }
static inline float sse_cosf(float y) { return sse_sc(y, 1); }

typedef float (*ffn)(float);
static float (*volatile libm_sin)(float) = sinf;
static float (*volatile libm_cos)(float) = cosf;
static float (*volatile libm_acos)(float) = acosf;

enum { NF = 5, NT = 8, MAXREC = 4 };
static const char *names[NF] = {"sinf[fma]", "cosf[fma]", "sinf[sse2]", "cosf[sse2]", "acosf"};
typedef struct {
	uint64_t lo, hi;
	uint64_t bad[NF];
	uint32_t rec[NF][MAXREC];
} job_t;

static int same(float a, float b) { return (isnan(a) && isnan(b)) || gl_asuint(a) == gl_asuint(b); }

static void *run(void *arg) {
	job_t *j = arg;
	for (uint64_t u = j->lo; u < j->hi; u++) {
		float x = gl_asfloat((uint32_t)u);
		float ref[NF] = {libm_sin(x), libm_cos(x), 0, 0, libm_acos(x)};
		ref[2] = ref[0];
		ref[3] = ref[1];
		float got[NF] = {glibc_sinf(x), glibc_cosf(x), sse_sinf(x), sse_cosf(x), glibc_acosf(x)};
		for (int f = 0; f < NF; f++)
			if (!same(ref[f], got[f])) {
				if (j->bad[f] < MAXREC) j->rec[f][j->bad[f]] = (uint32_t)u;
				j->bad[f]++;
			}
	}
	return NULL;
}

int main(int argc, char **argv) {
	uint64_t total = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 32);
	pthread_t th[NT];
	job_t jobs[NT] = {0};
	for (int t = 0; t < NT; t++) {
		jobs[t].lo = total * t / NT;
		jobs[t].hi = total * (t + 1) / NT;
		pthread_create(&th[t], 0, run, &jobs[t]);
	}
	for (int t = 0; t < NT; t++) pthread_join(th[t], 0);
	printf("inputs checked: %llu (float bit patterns 0 .. %llu)\n", (unsigned long long)total,
			(unsigned long long)(total - 1));
	for (int f = 0; f < NF; f++) {
		uint64_t bad = 0;
		for (int t = 0; t < NT; t++) bad += jobs[t].bad[f];
		printf("%-11s mismatches vs platform libm: %llu", names[f], (unsigned long long)bad);
		int shown = 0;
		for (int t = 0; t < NT && shown < MAXREC; t++)
			for (uint64_t k = 0; k < jobs[t].bad[f] && k < MAXREC && shown < MAXREC; k++, shown++) {
				float x = gl_asfloat(jobs[t].rec[f][k]);
				printf("  [x=%a]", x);
			}
		printf("\n");
	}
	return 0;
}
