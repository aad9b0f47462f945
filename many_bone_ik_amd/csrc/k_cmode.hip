// constraint_mode kernels (cmode.h): the classic lane layout and wave roles, and the fresh-tree
// reset of the persistent node caches.
#include <mutex>

#include "cmode.h"

namespace mbik {

CmodeKernel cmode_kernel(bool stab, bool nb32, bool chain) {
	static std::once_flag once;
	static const CmodeKernel ks[2][2][2] = {
			{{mbik_cmode_kernel<false, false>, mbik_cmode_kernel<false, false, true>}, {mbik_cmode_kernel<false, true>, mbik_cmode_kernel<false, true, true>}},
			{{mbik_cmode_kernel<true, false>, mbik_cmode_kernel<true, false, true>}, {mbik_cmode_kernel<true, true>, mbik_cmode_kernel<true, true, true>}}};
	std::call_once(once, [] {
		for (auto &a : ks)
			for (auto &b : a)
				for (CmodeKernel k : b) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	return ks[stab ? 1 : 0][nb32 ? 1 : 0][chain ? 1 : 0];
}

// wave roles: K = 2, 4 or 8 waves per block, 32-bit addressing
CmodeKernel cmode_kernel_rw(bool chain, int kw) {
	static const CmodeKernel krw[2][3] = {{mbik_cmode_kernel_rw<true, false, 2>, mbik_cmode_kernel_rw<true, false, 4>, mbik_cmode_kernel_rw<true, false, 8>},
			{mbik_cmode_kernel_rw<true, true, 2>, mbik_cmode_kernel_rw<true, true, 4>, mbik_cmode_kernel_rw<true, true, 8>}};
	static std::once_flag once;
	std::call_once(once, [] {
		for (auto &row : krw)
			for (CmodeKernel k : row) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	return krw[chain ? 1 : 0][kw == 2 ? 0 : kw == 4 ? 1 : 2];
}

hipError_t launch_cmode_reset(hipStream_t st, const DevPlan &t, const CmodeState &c, int first, int count, const float *setup_pose) {
	hipLaunchKernelGGL(mbik_cmode_reset_kernel, dim3((unsigned)((count + 63) / 64)), dim3(64), 0, st, t, c, first, count, setup_pose);
	return hipGetLastError();
}

} // namespace mbik

#ifdef MBIK_PROF
int mbik::prof_take_cmode(unsigned long long *out) {
	unsigned long long v[24] = {}, z[24] = {};
	if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_mbik_prof), sizeof(v)) != hipSuccess) return -1;
	for (int i = 0; i < 24; i++) out[i] += v[i];
	return hipMemcpyToSymbol(HIP_SYMBOL(g_mbik_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
