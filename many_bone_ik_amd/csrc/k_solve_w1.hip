// The classic solve kernels built for one wave per SIMD (the whole register file): the LDS and
// device-memory state placements, stabilization, the 64-bit-index builds for tables of 4 GiB or
// more, the default-priority instantiations, and the fused group kernel (mbik_group_solve).
#include <mutex>

#include "solve_block.h"

namespace {
using mbik::GroupEntry;
// A heterogeneous batch (mbik_group_solve): several plans -- distinct rigs -- in one launch.
// Plan i owns blocks [block_off[i], block_off[i + 1]) of the grid; each block loads its
// plan's tables and buffers and runs the plan's own layout.
template <bool STAB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MBIK_WAVES_PER_EU, MBIK_WAVES_PER_EU))) void mbik_group_kernel(const DevPlan *__restrict__ plans,
		const GroupEntry *__restrict__ entries, int n_plans) {
	// No XCD remap here: the host orders the plans longest chain first, and blocks are
	// dispatched in grid order, so the long chains start first (LPT) and short rigs fill in.
	const int gb = blockIdx.x;
	int lo = 0, hi = n_plans - 1; // the last plan whose first block is <= gb
	while (lo < hi) {
		const int mid = (lo + hi + 1) >> 1;
		if (entries[mid].block_off <= gb) lo = mid;
		else hi = mid - 1;
	}
	DevPlan t = plans[lo];
	const GroupEntry e = entries[lo];
	solve_block<STAB, 0>(t, gb - e.block_off, e.first, e.count, e.pose_in, e.targets, e.pose_out, e.iterations, 0, t.NS - 1);
}
} // namespace

namespace mbik {

SolveKernel solve_kernel_w1(bool stab, int pl, bool t32, int pm) {
	static const SolveKernel ks[2][3] = {{mbik_solve_kernel<false, 0>, mbik_solve_kernel<false, 1>, mbik_solve_kernel<false, 2>},
			{mbik_solve_kernel<true, 0>, mbik_solve_kernel<true, 1>, mbik_solve_kernel<true, 2>}};
	// placement 0 with tables of 4 GiB or more: 64-bit element indices
	static const SolveKernel k64[2] = {mbik_solve_kernel<false, 0, 1, false>, mbik_solve_kernel<true, 0, 1, false>};
	// the default-priority instantiations (PM = kPrioDefault) of the non-stabilized 32-bit builds
	constexpr int D = kPrioDefault;
	static const SolveKernel kd[3] = {mbik_solve_kernel<false, 0, 1, true, false, D>, mbik_solve_kernel<false, 1, 1, true, false, D>,
			mbik_solve_kernel<false, 2, 1, true, false, D>};
	static std::once_flag once;
	std::call_once(once, [] {
		for (auto &row : ks)
			for (SolveKernel k : row) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		for (SolveKernel k : k64) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		for (SolveKernel k : kd) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	if (!t32) return k64[stab ? 1 : 0];
	if (stab) return ks[1][pl];
	return pm == kPrioDefault ? kd[pl] : ks[0][pl];
}

GroupKernel group_kernel(bool stab) {
	static std::once_flag once;
	std::call_once(once, [] {
		(void)hipFuncSetAttribute((const void *)mbik_group_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		(void)hipFuncSetAttribute((const void *)mbik_group_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	return stab ? mbik_group_kernel<true> : mbik_group_kernel<false>;
}

} // namespace mbik

#ifdef MBIK_PROF
int mbik::prof_take_w1(unsigned long long *out) {
	unsigned long long v[24] = {}, z[24] = {};
	if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_mbik_prof), sizeof(v)) != hipSuccess) return -1;
	for (int i = 0; i < 24; i++) out[i] += v[i];
	return hipMemcpyToSymbol(HIP_SYMBOL(g_mbik_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
