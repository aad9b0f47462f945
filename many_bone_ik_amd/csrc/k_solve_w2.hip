// The classic solve kernels built for two waves per SIMD (at most 256 registers, so that two
// one-wave blocks share a SIMD: launches whose skeletons do not fit the chip at once), with and
// without split-exchange segments (XS), and the 64-bit-index build.
#include <mutex>

#include "solve_block.h"

namespace mbik {

SolveKernel solve_kernel_w2(int pl, bool t32, bool xs, int pm) {
	static const SolveKernel k2[3] = {mbik_solve_kernel<false, 0, 2>, mbik_solve_kernel<false, 1, 2>, mbik_solve_kernel<false, 2, 2>};
	static const SolveKernel k2x[3] = {mbik_solve_kernel<false, 0, 2, true, true>, mbik_solve_kernel<false, 1, 2, true, true>,
			mbik_solve_kernel<false, 2, 2, true, true>};
	static const SolveKernel k64 = mbik_solve_kernel<false, 0, 2, false>;
	constexpr int D = kPrioDefault;
	static const SolveKernel k2d[3] = {mbik_solve_kernel<false, 0, 2, true, false, D>, mbik_solve_kernel<false, 1, 2, true, false, D>,
			mbik_solve_kernel<false, 2, 2, true, false, D>};
	static const SolveKernel k2xd[3] = {mbik_solve_kernel<false, 0, 2, true, true, D>, mbik_solve_kernel<false, 1, 2, true, true, D>,
			mbik_solve_kernel<false, 2, 2, true, true, D>};
	static std::once_flag once;
	std::call_once(once, [] {
		for (const SolveKernel *a : {k2, k2x, k2d, k2xd})
			for (int i = 0; i < 3; i++) (void)hipFuncSetAttribute((const void *)a[i], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		(void)hipFuncSetAttribute((const void *)k64, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	if (!t32) return k64;
	const bool dflt = pm == kPrioDefault;
	return xs ? (dflt ? k2xd[pl] : k2x[pl]) : (dflt ? k2d[pl] : k2[pl]);
}

} // namespace mbik

#ifdef MBIK_PROF
int mbik::prof_take_w2(unsigned long long *out) {
	unsigned long long v[24] = {}, z[24] = {};
	if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_mbik_prof), sizeof(v)) != hipSuccess) return -1;
	for (int i = 0; i < 24; i++) out[i] += v[i];
	return hipMemcpyToSymbol(HIP_SYMBOL(g_mbik_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
