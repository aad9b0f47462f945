// Probe: does a VALU write to a VGPR that holds the data of the immediately preceding
// buffer_store_dwordx4 change what the store writes, and does that depend on whether the
// instruction's SGPR-offset field is a register or the constant 0?
// (LLVM's GCNHazardRecognizer::createsVALUHazard models this "store of more than 8 bytes"
// hazard only when soffset is NOT a register, so it inserts no wait state after a wide store
// with an SGPR soffset.  DESIGN.md §10: the SGPR-offset state addressing.)
//   hipcc --offload-arch=gfx950 -O2 tools/store_hazard.hip -o build/store_hazard && build/store_hazard
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

// MODE 0: soffset = SGPR holding 0; MODE 1: soffset = constant 0; MODE 2: SGPR, one s_nop
// between the store and the overwrite.  Each lane stores {1000+4l .. 1003+4l} at l*16 and then
// overwrites the second data register with 0xdead.
template <int MODE>
__global__ void probe(uint32_t *base, uint32_t bytes, uint32_t so) {
	const uint32_t l = threadIdx.x;
	const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
	const uint32_t vo = l * 16;
	const uint32_t a = 1000 + 4 * l, b = a + 1, c = a + 2, d = a + 3;
	if constexpr (MODE == 0)
		asm volatile("v_mov_b32 v40, %3\n\tv_mov_b32 v41, %4\n\tv_mov_b32 v42, %5\n\tv_mov_b32 v43, %6\n\ts_nop 4\n\t"
					 "buffer_store_dwordx4 v[40:43], %0, %1, %2 offen\n\t"
					 "v_mov_b32 v41, 0xdead\n\ts_waitcnt vmcnt(0)" ::"v"(vo),
				"s"(r), "s"(so), "v"(a), "v"(b), "v"(c), "v"(d)
				: "v40", "v41", "v42", "v43", "memory");
	if constexpr (MODE == 1)
		asm volatile("v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %5\n\ts_nop 4\n\t"
					 "buffer_store_dwordx4 v[40:43], %0, %1, 0 offen\n\t"
					 "v_mov_b32 v41, 0xdead\n\ts_waitcnt vmcnt(0)" ::"v"(vo),
				"s"(r), "v"(a), "v"(b), "v"(c), "v"(d)
				: "v40", "v41", "v42", "v43", "memory");
	if constexpr (MODE == 3) // soffset = SGPR holding 16 (so passed in): the record lands 16 B further
		asm volatile("v_mov_b32 v40, %3\n\tv_mov_b32 v41, %4\n\tv_mov_b32 v42, %5\n\tv_mov_b32 v43, %6\n\ts_nop 4\n\t"
					 "buffer_store_dwordx4 v[40:43], %0, %1, %2 offen\n\t"
					 "v_mov_b32 v41, 0xdead\n\ts_waitcnt vmcnt(0)" ::"v"(vo),
				"s"(r), "s"(so), "v"(a), "v"(b), "v"(c), "v"(d)
				: "v40", "v41", "v42", "v43", "memory");
	if constexpr (MODE == 4) // dwordx3, soffset = SGPR
		asm volatile("v_mov_b32 v40, %3\n\tv_mov_b32 v41, %4\n\tv_mov_b32 v42, %5\n\tv_mov_b32 v43, %6\n\ts_nop 4\n\t"
					 "buffer_store_dwordx3 v[40:42], %0, %1, %2 offen\n\t"
					 "v_mov_b32 v41, 0xdead\n\ts_waitcnt vmcnt(0)" ::"v"(vo),
				"s"(r), "s"(so), "v"(a), "v"(b), "v"(c), "v"(d)
				: "v40", "v41", "v42", "v43", "memory");
	if constexpr (MODE == 2)
		asm volatile("v_mov_b32 v40, %3\n\tv_mov_b32 v41, %4\n\tv_mov_b32 v42, %5\n\tv_mov_b32 v43, %6\n\ts_nop 4\n\t"
					 "buffer_store_dwordx4 v[40:43], %0, %1, %2 offen\n\t"
					 "s_nop 0\n\tv_mov_b32 v41, 0xdead\n\ts_waitcnt vmcnt(0)" ::"v"(vo),
				"s"(r), "s"(so), "v"(a), "v"(b), "v"(c), "v"(d)
				: "v40", "v41", "v42", "v43", "memory");
}

int main() {
	uint32_t *d;
	const uint32_t bytes = 64 * 16 + 16;
	if (hipMalloc(&d, bytes)) return 1;
	const char *names[5] = {"soffset = SGPR (0), VALU overwrite next", "soffset = constant 0, VALU overwrite next",
			"soffset = SGPR (0), s_nop 0 then overwrite", "soffset = SGPR (16), VALU overwrite next",
			"dwordx3, soffset = SGPR (0), overwrite next"};
	int total = 0;
	for (int mode = 0; mode < 5; mode++) {
		int wrong = 0;
		for (int rep = 0; rep < 100; rep++) {
			if (hipMemset(d, 0, bytes)) return 1;
			if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, d, bytes, 0u);
			if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, bytes, 0u);
			if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, bytes, 0u);
			if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, d, bytes, 16u);
			if (mode == 4) hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, d, bytes, 0u);
			uint32_t h[260];
			const int sh = mode == 3 ? 4 : 0, nk = mode == 4 ? 3 : 4;
			if (hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost)) return 1;
			for (int l = 0; l < 64; l++)
				for (int k = 0; k < nk; k++) wrong += h[sh + 4 * l + k] != 1000u + 4 * l + k;
		}
		printf("%-45s: %6d of %d stored words wrong\n", names[mode], wrong, 100 * 64 * (mode == 4 ? 3 : 4));
		total += wrong;
	}
	return 0;
}
