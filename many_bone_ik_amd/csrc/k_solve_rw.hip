// Wave roles (one wavefront per sibling-segment role, a lane per skeleton) and the
// helper-wave kernels (a second wave per block precomputing each bone-step's parent-side record;
// DESIGN.md §4b).
#include <mutex>

#include "solve_block.h"

namespace {
// Wave roles (HostPlan::wave_roles): KW waves per block, one per role of the sibling schedule,
// a lane per skeleton; the whole state in device memory.  WPE: waves per SIMD the register budget
// is sized for; KW waves of a block need KW / 4 waves per SIMD.  (The two-wave build does not
// hoist a single-effector segment's effector rows: 121 VGPRs spilled, round 5.)
template <int KW, int WPE, int PM>
__global__ __launch_bounds__(64 * KW) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mbik_solve_kernel_rw(DevPlan t, int first,
		int count, const float *__restrict__ pose_in, const float *__restrict__ targets, float *__restrict__ pose_out, int iterations,
		int seg_lo, int seg_hi) {
	static_assert(KW <= 4 * WPE, "a block's waves must fit the CU at this register budget");
	solve_block<false, 2, WPE == 1, true, false, false, PM, KW>(t, xcd_block(), first, count, pose_in, targets, pose_out,
			iterations, seg_lo, seg_hi);
}

// The helper-wave build (two waves per block, on two SIMDs of a CU): placement 0, no
// stabilization, 32-bit table addressing (mbik_plan_set_helper_wave; autotune decides).
template <int PM>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(1, 1))) void mbik_solve_kernel_help(DevPlan t, int first, int count,
		const float *__restrict__ pose_in, const float *__restrict__ targets, float *__restrict__ pose_out, int iterations, int seg_lo,
		int seg_hi) {
	solve_block<false, 0, true, true, true, false, PM>(t, xcd_block(), first, count, pose_in, targets, pose_out, iterations, seg_lo, seg_hi);
}

#ifdef MBIK_REPLAY
// The solving wave alone, replaying saved helper records (diagnostic build only).
template <int PM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void mbik_solve_kernel_replay(DevPlan t, int first, int count,
		const float *__restrict__ pose_in, const float *__restrict__ targets, float *__restrict__ pose_out, int iterations, int seg_lo,
		int seg_hi) {
	solve_block<false, 0, true, true, true, false, PM>(t, xcd_block(), first, count, pose_in, targets, pose_out, iterations, seg_lo, seg_hi);
}
#endif
} // namespace

namespace mbik {

SolveKernel solve_kernel_rw(int kw, int wpe, int pm) {
	constexpr int D = kPrioDefault;
	// [PM default?][K 2 / 4 / 8, waves per SIMD 1 / 2] (K 8 needs two waves per SIMD)
	static const SolveKernel krw[2][5] = {
			{mbik_solve_kernel_rw<2, 1, 0>, mbik_solve_kernel_rw<2, 2, 0>, mbik_solve_kernel_rw<4, 1, 0>, mbik_solve_kernel_rw<4, 2, 0>,
					mbik_solve_kernel_rw<8, 2, 0>},
			{mbik_solve_kernel_rw<2, 1, D>, mbik_solve_kernel_rw<2, 2, D>, mbik_solve_kernel_rw<4, 1, D>, mbik_solve_kernel_rw<4, 2, D>,
					mbik_solve_kernel_rw<8, 2, D>}};
	static std::once_flag once;
	std::call_once(once, [] {
		for (auto &row : krw)
			for (SolveKernel k : row) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
	});
	const int i = kw == 2 ? (wpe == 2 ? 1 : 0) : kw == 4 ? (wpe == 2 ? 3 : 2) : 4;
	return krw[pm == kPrioDefault ? 1 : 0][i];
}

SolveKernel solve_kernel_help(int pm, bool replay) {
	static std::once_flag once;
	std::call_once(once, [] {
		(void)hipFuncSetAttribute((const void *)mbik_solve_kernel_help<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		(void)hipFuncSetAttribute((const void *)mbik_solve_kernel_help<kPrioDefault>, hipFuncAttributeMaxDynamicSharedMemorySize,
				160 * 1024);
#ifdef MBIK_REPLAY
		(void)hipFuncSetAttribute((const void *)mbik_solve_kernel_replay<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
		(void)hipFuncSetAttribute((const void *)mbik_solve_kernel_replay<kPrioDefault>, hipFuncAttributeMaxDynamicSharedMemorySize,
				160 * 1024);
#endif
	});
#ifdef MBIK_REPLAY
	if (replay) return pm == kPrioDefault ? mbik_solve_kernel_replay<kPrioDefault> : mbik_solve_kernel_replay<0>;
#else
	(void)replay;
#endif
	return pm == kPrioDefault ? mbik_solve_kernel_help<kPrioDefault> : mbik_solve_kernel_help<0>;
}

} // namespace mbik

#ifdef MBIK_PROF
int mbik::prof_take_rw(unsigned long long *out) {
	unsigned long long v[24] = {}, z[24] = {};
	if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_mbik_prof), sizeof(v)) != hipSuccess) return -1;
	for (int i = 0; i < 24; i++) out[i] += v[i];
	return hipMemcpyToSymbol(HIP_SYMBOL(g_mbik_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
