// Host build of the product's gd_math.h transcendentals (the same source the gfx950 kernel
// compiles) against the platform libm on all 2^32 float inputs -- a CPU pre-check before the
// device proof (mbik_selftest_libm, tests/test_gpu_libm.py).
//
//   g++ -O2 -std=c++17 -ffp-contract=off -fno-builtin -pthread -I many_bone_ik_amd/csrc \
//       tools/gdmath_host_check.cpp -o /tmp/gdmath_host_check && /tmp/gdmath_host_check
#include <math.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
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

int main() {
	const int NT = 8;
	std::vector<uint64_t> bad(NT * 4, 0), first(NT * 4, ~0ull);
	std::vector<std::thread> th;
	for (int t = 0; t < NT; t++)
		th.emplace_back([&, t] {
			for (uint64_t u = (1ull << 32) * t / NT; u < (1ull << 32) * (t + 1) / NT; u++) {
				float x;
				uint32_t v = (uint32_t)u;
				std::memcpy(&x, &v, 4);
				const bool ok[4] = {same(libm_sin(x), gd::sin_f(x)), same(libm_cos(x), gd::cos_f(x)),
						same(libm_acos(x), gd::acos_f(x)),
						same((float)(std::sin(1.0 * x) / libm_sin(x)), gd::slerp_scale0(x))};
				for (int f = 0; f < 4; f++)
					if (!ok[f]) {
						if (!bad[t * 4 + f]) first[t * 4 + f] = u;
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
		std::printf("%-13s mismatches vs platform libm over 2^32 inputs: %llu", names[f], (unsigned long long)b);
		if (b) std::printf("  (first bit pattern %#llx)", (unsigned long long)fb);
		std::printf("\n");
	}
	return 0;
}
