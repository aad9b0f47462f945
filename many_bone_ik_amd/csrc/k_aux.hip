// Small kernels around the solve: batched target capture, the GPU plan setup (setup.h) and
// topology build (topo.h), and the skeleton-tiled copy of the setup tables.
#include "dev_common.h"
#include "setup.h"
#include "topo.h"

namespace {
using mbik::kRowTile;
using mbik::TopoSlice;
// IKEffector3D::update_target_global_transform (ik_effector_3d.cpp:77-84) for a batch: one
// thread per (skeleton, pin).  Transforms are 12 floats: basis rows, then origin.
__global__ __launch_bounds__(256) void mbik_capture_targets_kernel(int count, int P, const float *__restrict__ skel_global,
		const float *__restrict__ target_global, const uint8_t *__restrict__ visible, float *__restrict__ targets) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= (int64_t)count * P) return;
	if (visible && !visible[i]) return; // not visible in tree: the previous target stays
	const int64_t sk = i / P;
	const float *a = skel_global + sk * 12, *b = target_global + i * 12;
	auto xf = [](const float *v) {
		return X3{bset(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]), v3(v[9], v[10], v[11])};
	};
	const X3 r = affine_inverse(xf(a)) * xf(b);
	float *o = targets + i * 12;
	const float w[12] = {r.b.r[0].x, r.b.r[0].y, r.b.r[0].z, r.b.r[1].x, r.b.r[1].y, r.b.r[1].z,
			r.b.r[2].x, r.b.r[2].y, r.b.r[2].z, r.o.x, r.o.y, r.o.z};
	for (int f = 0; f < 12; f++) o[f] = w[f];
}

// GPU plan setup: the per-skeleton bone-direction and Kusudama frames of
// mbik_plan_create, derived on the device with the host builder's own code (setup.h), one
// thread per skeleton over a grid-stride loop, each with a private scratch slice.
__global__ __launch_bounds__(64) void mbik_setup_kernel(mbik::SetupView v, int first, int count, const float *__restrict__ pose,
		const float *__restrict__ cones, const float *__restrict__ twist, char *scratch, size_t scratch_stride, float *D,
		float *CF, double *CD) {
	const int tid = blockIdx.x * blockDim.x + threadIdx.x;
	const int nthreads = gridDim.x * blockDim.x;
	const mbik::SetupScratch w = mbik::setup_scratch_at(scratch + (size_t)tid * scratch_stride, v.B, v.NC, v.max_cones_in);
	for (int i = tid; i < count; i += nthreads)
		mbik::setup_skeleton(v, i, first + i, pose + (size_t)i * v.B * 10, cones, twist, w, D, CF, CD);
}

// [items*fields][N] -> [items][Npad/kRowTile][fields][kRowTile] (DevPlan::row_at), one element a thread
template <class T>
__global__ __launch_bounds__(256) void mbik_tile_rows_kernel(const T *__restrict__ src, T *__restrict__ dst, int items,
		int fields, int N, int Npad) {
	const size_t n = (size_t)items * fields * N;
	for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		const size_t row = i / N, sk = i % N;
		const size_t item = row / fields, f = row % fields;
		dst[item * fields * Npad + (sk / kRowTile) * fields * kRowTile + f * kRowTile + sk % kRowTile] = src[i];
	}
}

__global__ __launch_bounds__(64) void mbik_topology_kernel(const TopoSlice *__restrict__ slices, int n) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const TopoSlice sl = slices[i];
	const mbik::TopoRig &r = sl.rig;
	mbik::topo_build(r, mbik::topo_out_at(sl.out_i, sl.out_d, sl.out_f, r.B, r.P, r.C), mbik::topo_scratch_at(sl.scr_i, sl.scr_d, r.B, r.P));
}
} // namespace

namespace mbik {

hipError_t launch_capture_targets(hipStream_t st, int count, int P, const float *skel_global, const float *target_global,
		const uint8_t *visible, float *targets) {
	const int64_t n = (int64_t)count * P;
	hipLaunchKernelGGL(mbik_capture_targets_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, count, P, skel_global,
			target_global, visible, targets);
	return hipGetLastError();
}

hipError_t launch_setup(hipStream_t st, int threads, const SetupView &v, int first, int count, const float *pose, const float *cones,
		const float *twist, char *scratch, size_t scratch_stride, float *D, float *CF, double *CD) {
	hipLaunchKernelGGL(mbik_setup_kernel, dim3((threads + 63) / 64), dim3(64), 0, st, v, first, count, pose, cones, twist, scratch,
			scratch_stride, D, CF, CD);
	return hipGetLastError();
}

hipError_t launch_topology(const TopoSlice *slices, int n) {
	hipLaunchKernelGGL(mbik_topology_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, slices, n);
	return hipGetLastError();
}

static dim3 tile_grid(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 65536)); }
hipError_t launch_tile_rows(hipStream_t st, const float *src, float *dst, int items, int fields, int N, int Npad) {
	hipLaunchKernelGGL(mbik_tile_rows_kernel<float>, tile_grid((size_t)items * fields * N), dim3(256), 0, st, src, dst, items, fields, N, Npad);
	return hipGetLastError();
}
hipError_t launch_tile_rows(hipStream_t st, const double *src, double *dst, int items, int fields, int N, int Npad) {
	hipLaunchKernelGGL(mbik_tile_rows_kernel<double>, tile_grid((size_t)items * fields * N), dim3(256), 0, st, src, dst, items, fields, N, Npad);
	return hipGetLastError();
}

} // namespace mbik
