// Host build of the product's gd_math.h transcendentals (the same source the gfx950 kernel
// compiles) against the platform libm on all 2^32 float inputs -- a CPU pre-check before the
// device proof (mbik_selftest_libm, tests/test_gpu_libm.py).
//
//   g++ -O2 -std=c++17 -ffp-contract=off -fno-builtin -pthread -I many_bone_ik_amd/csrc \
//       tools/gdmath_host_check.cpp -o /tmp/gdmath_host_check && /tmp/gdmath_host_check [VARIANT [STRIDE | list X...]]
// VARIANT: 0 the FMA build of glibc's sinf/cosf (default), 1 the SSE2 build -- run that one with
// GLIBC_TUNABLES=glibc.cpu.hwcaps=-FMA,-AVX2_Usable so the platform libm is the SSE2 build too.
// STRIDE: check every STRIDE-th bit pattern (default 1: all 2^32); `list X...`: only the hex
// floats X (e.g. 0x1.ab6152p+5).
#include <math.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gd_math.h"

static float (*volatile libm_sin)(float) = sinf;
static float (*volatile libm_cos)(float) = cosf;
static float (*volatile libm_acos)(float) = acosf;

static bool same(float a, float b) {
	uint32_t x, y;
	std::memcpy(&x, &a, 4);
	std::memcpy(&y, &b, 4);
	return (a != a && b != b) || x == y;
}

static uint32_t bits_of(float x) {
	uint32_t u;
	std::memcpy(&u, &x, 4);
	return u;
}

int main(int argc, char **argv) {
	const int lv = argc > 1 ? std::atoi(argv[1]) : 0;
	const bool list = argc > 2 && std::strcmp(argv[2], "list") == 0;
	const uint64_t stride = !list && argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 1;
	std::vector<uint32_t> inputs;
	if (list)
		for (int i = 3; i < argc; i++) inputs.push_back(bits_of(std::strtof(argv[i], nullptr)));
	const uint64_t n = list ? inputs.size() : ((1ull << 32) + stride - 1) / stride;
	const int NT = 8;
	std::vector<uint64_t> bad(NT * 4, 0), first(NT * 4, ~0ull);
	std::vector<std::thread> th;
	for (int t = 0; t < NT; t++)
		th.emplace_back([&, t] {
			for (uint64_t k = n * t / NT; k < n * (t + 1) / NT; k++) {
				const uint32_t v = list ? inputs[k] : (uint32_t)(k * stride);
				float x;
				std::memcpy(&x, &v, 4);
				const bool ok[4] = {same(libm_sin(x), gd::sin_f(x, lv)), same(libm_cos(x), gd::cos_f(x, lv)),
						same(libm_acos(x), gd::acos_f(x)),
						same((float)(std::sin(1.0 * x) / libm_sin(x)), gd::slerp_scale0(x, lv))};
				for (int f = 0; f < 4; f++)
					if (!ok[f]) {
						if (!bad[t * 4 + f]) first[t * 4 + f] = v;
						bad[t * 4 + f]++;
					}
			}
		});
	for (auto &x : th) x.join();
	const char *names[4] = {"sin_f", "cos_f", "acos_f", "slerp_scale0"};
	for (int f = 0; f < 4; f++) {
		uint64_t b = 0, fb = ~0ull;
		for (int t = 0; t < NT; t++) {
			b += bad[t * 4 + f];
			if (first[t * 4 + f] < fb) fb = first[t * 4 + f];
		}
		std::printf("%-13s variant %s mismatches vs platform libm over %llu inputs: %llu", names[f], lv ? "sse2" : "fma",
				(unsigned long long)n, (unsigned long long)b);
		if (b) std::printf("  (first bit pattern %#llx)", (unsigned long long)fb);
		std::printf("\n");
	}
	return 0;
}
