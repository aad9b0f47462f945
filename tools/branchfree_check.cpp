// Host check of gd_math.h's branch-free slerp forms against the branchy glibc restatements they
// replace on the solve's hot path (the same source the gfx950 kernel compiles):
//   glibc::sinf_small<FMA>(y)  vs glibc::sincosf<FMA>(y, 0)  for |y| <= 1.6, both builds
//   glibc::acosf_unit(x)       vs glibc::acosf(x)            for -0.5 < x < 1
// Every STRIDE-th float bit pattern of each range (default 1: all of them).  The device proof is
// mbik_selftest_libm (SLERP_SCALE0, ACOSF_UNIT; tests/test_gpu_libm.py).
//
//   g++ -O2 -std=c++17 -ffp-contract=off -fno-builtin -pthread -I many_bone_ik_amd/csrc \
//       tools/branchfree_check.cpp -o /tmp/branchfree_check && /tmp/branchfree_check [STRIDE]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gd_math.h"

static float f_of(uint32_t u) {
	float f;
	std::memcpy(&f, &u, 4);
	return f;
}
static uint32_t u_of(float f) {
	uint32_t u;
	std::memcpy(&u, &f, 4);
	return u;
}

int main(int argc, char **argv) {
	const uint64_t stride = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
	const int T = 8;
	std::vector<long> bs(T), bc(T), ba(T), n(T);
	std::vector<std::thread> th;
	const uint32_t lim = u_of(1.6f), one = u_of(1.0f), half = u_of(0.5f);
	for (int k = 0; k < T; k++)
		th.emplace_back([&, k] {
			for (uint64_t u = k * stride; u <= lim; u += T * stride)
				for (uint32_t sg : {0u, 0x80000000u}) {
					const float y = f_of((uint32_t)u | sg);
					bs[k] += u_of(gd::glibc::sinf_small<true>(y)) != u_of(gd::glibc::sincosf<true>(y, 0));
					bc[k] += u_of(gd::glibc::sinf_small<false>(y)) != u_of(gd::glibc::sincosf<false>(y, 0));
					n[k]++;
				}
			for (uint64_t u = k * stride; u < one; u += T * stride) {
				const float x = f_of((uint32_t)u);
				ba[k] += u_of(gd::glibc::acosf_unit(x)) != u_of(gd::glibc::acosf(x));
				if (u < half) ba[k] += u_of(gd::glibc::acosf_unit(-x)) != u_of(gd::glibc::acosf(-x));
				n[k]++;
			}
		});
	for (auto &t : th) t.join();
	long s = 0, c = 0, a = 0, tot = 0;
	for (int k = 0; k < T; k++) s += bs[k], c += bc[k], a += ba[k], tot += n[k];
	std::printf("checked %ld inputs: sinf_small FMA mismatches %ld, SSE2 mismatches %ld; acosf_unit mismatches %ld\n", tot, s, c, a);
	return (s || c || a) ? 1 : 0;
}
