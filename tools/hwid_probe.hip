// Where the hardware places the waves of co-resident workgroups (diagnostic, not product code):
// launches NB workgroups of W waves with LDS bytes per block chosen so that two blocks fit a CU
// (as C4's wave-roles launch: 4 waves, 73.6 KB), and each wave records its HW_ID
// (CU / SIMD / wave slot / workgroup slot TG_ID) and XCC_ID.  Prints, per CU, the blocks it
// held and each block's (wave -> SIMD) map and TG_ID, and a summary: whether wave w always sits
// on SIMD w % 4, and how often two blocks on one CU differ in TG_ID parity.
//   hipcc --offload-arch=gfx950 -O2 tools/hwid_probe.hip -o build/hwid_probe && build/hwid_probe [NB] [W] [LDS]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

__global__ void probe(unsigned *out, int spin) {
	extern __shared__ float lds[];
	const int wave = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0) lds[wave] = 0.0f;
	// keep the block resident for a while so that the next blocks fill the other CU slots
	const long long t0 = clock64();
	while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(4);
	const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, 32 bits
	const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // HW_REG_XCC_ID
	if ((threadIdx.x & 63) == 0) {
		out[(blockIdx.x * (blockDim.x >> 6) + wave) * 2] = hw;
		out[(blockIdx.x * (blockDim.x >> 6) + wave) * 2 + 1] = xcc;
	}
}

int main(int argc, char **argv) {
	const int nb = argc > 1 ? atoi(argv[1]) : 512, w = argc > 2 ? atoi(argv[2]) : 4;
	const int ldsb = argc > 3 ? atoi(argv[3]) : 73664;
	unsigned *d = nullptr;
	const size_t n = (size_t)nb * w * 2;
	if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
	hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb);
	hipLaunchKernelGGL(probe, dim3(nb), dim3(64 * w), ldsb, 0, d, 2000000);
	if (hipDeviceSynchronize() != hipSuccess) return 2;
	std::vector<unsigned> h(n);
	hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
	// key: (xcc, se, sh, cu) -> blocks
	std::map<std::tuple<int, int, int, int>, std::vector<int>> cu;
	int simd_mod = 0, total = 0;
	for (int b = 0; b < nb; b++) {
		const unsigned hw0 = h[(size_t)b * w * 2], xcc = h[(size_t)b * w * 2 + 1];
		const int cuid = (hw0 >> 8) & 15, sh = (hw0 >> 12) & 1, se = (hw0 >> 13) & 7;
		cu[{(int)(xcc & 15), se, sh, cuid}].push_back(b);
		for (int v = 0; v < w; v++) {
			const unsigned hv = h[((size_t)b * w + v) * 2];
			total++;
			simd_mod += (int)((hv >> 4) & 3) == v % 4;
		}
	}
	int pairs = 0, diff_parity = 0, printed = 0;
	for (auto &kv : cu) {
		auto &bl = kv.second;
		if (bl.size() >= 2) {
			pairs++;
			const int tg0 = (h[(size_t)bl[0] * w * 2] >> 16) & 15, tg1 = (h[(size_t)bl[1] * w * 2] >> 16) & 15;
			diff_parity += (tg0 & 1) != (tg1 & 1);
		}
		if (printed++ < 12) {
			printf("xcc %d se %d sh %d cu %2d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), std::get<3>(kv.first));
			for (int b : bl) {
				printf("  blk %3d tg %2u simd[", b, (h[(size_t)b * w * 2] >> 16) & 15);
				for (int v = 0; v < w; v++) printf("%u", (h[((size_t)b * w + v) * 2] >> 4) & 3);
				printf("]");
			}
			printf("\n");
		}
	}
	printf("CUs %zu, waves on SIMD (wave %% 4): %d of %d, CUs with >= 2 blocks %d, of them TG_ID parity differs: %d\n", cu.size(), simd_mod,
			total, pairs, diff_parity);
	hipFree(d);
	return 0;
}
