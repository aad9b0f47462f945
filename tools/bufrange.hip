// Probe of the raw-buffer range check on gfx950: which (VGPR offset, SGPR offset) pairs of a
// buffer_load_dword read memory and which read 0, for a resource of R records (bytes) over a
// larger allocation.  Answers whether the SGPR offset takes part in the check (DESIGN.md §10,
// the SGPR-offset state addressing).
//   hipcc --offload-arch=gfx950 -O2 tools/bufrange.hip -o build/bufrange && build/bufrange
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void probe(const uint32_t *base, uint32_t records, const uint32_t *vo, uint32_t so, uint32_t *out, int n) {
	const int i = threadIdx.x;
	const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(base), 0, (int)records, 0x00020000);
	if (i < n) out[i] = __builtin_amdgcn_raw_buffer_load_b32(r, vo[i], so, 0);
}

int wide_probe();
int main() {
	const int W = 1024; // allocation: 4 KiB of words w[k] = 1000 + k
	uint32_t h[W];
	for (int k = 0; k < W; k++) h[k] = 1000 + k;
	uint32_t *d, *dvo, *dout;
	if (hipMalloc(&d, sizeof h) || hipMalloc(&dvo, 64 * 4) || hipMalloc(&dout, 64 * 4)) return 1;
	if (hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice)) return 1;
	const uint32_t R = 256; // records: bytes [0, 256) = words 0..63
	const uint32_t vos[] = {0, 248, 252, 256, 260, 512, 764};
	const uint32_t sos[] = {0, 4, 8, 256, 512};
	int nv = (int)(sizeof vos / sizeof vos[0]);
	if (hipMemcpy(dvo, vos, sizeof vos, hipMemcpyHostToDevice)) return 1;
	printf("records %u bytes; value 1000+k = word k read, 0 = dropped\n", R);
	printf("%10s", "voff\\soff");
	for (uint32_t so : sos) printf(" %8u", so);
	printf("\n");
	uint32_t res[5][64];
	for (int j = 0; j < 5; j++) {
		hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, R, dvo, sos[j], dout, nv);
		if (hipMemcpy(res[j], dout, 64 * 4, hipMemcpyDeviceToHost)) return 1;
	}
	for (int i = 0; i < nv; i++) {
		printf("%10u", vos[i]);
		for (int j = 0; j < 5; j++) printf(" %8u", res[j][i]);
		printf("\n");
	}
	return wide_probe();
}

// Part 2: multi-dword accesses with a non-zero SGPR offset.  Each lane stores 4 / 3 / 2 words
// at voffset = lane * 16 with soffset so through one b128 / b96 / b64 buffer store, then the
// whole area is read back with dword loads (another lane's words after a wave barrier) and
// with the same-width load.  Any mismatch against plain addressing is printed.
typedef unsigned int U4 __attribute__((ext_vector_type(4)));
typedef unsigned int U3 __attribute__((ext_vector_type(3)));
typedef unsigned int U2 __attribute__((ext_vector_type(2)));
template <int W>
__global__ void wide(uint32_t *base, uint32_t bytes, uint32_t so, uint32_t *back, uint32_t *same) {
	const uint32_t l = threadIdx.x;
	const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
	const uint32_t vo = l * 16;
	if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b128(U4{7000 + 4 * l, 7001 + 4 * l, 7002 + 4 * l, 7003 + 4 * l}, r, vo, so, 0);
	if constexpr (W == 3) __builtin_amdgcn_raw_buffer_store_b96(U3{7000 + 4 * l, 7001 + 4 * l, 7002 + 4 * l}, r, vo, so, 0);
	if constexpr (W == 2) __builtin_amdgcn_raw_buffer_store_b64(U2{7000 + 4 * l, 7001 + 4 * l}, r, vo, so, 0);
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	const uint32_t o = ((l + 1) & 63) * 16; // the next lane's record
	for (int k = 0; k < 4; k++) back[l * 4 + k] = __builtin_amdgcn_raw_buffer_load_b32(r, o + 4 * k, so, 0);
	U4 v = {0, 0, 0, 0};
	if constexpr (W == 4) v = __builtin_amdgcn_raw_buffer_load_b128(r, o, so, 0);
	if constexpr (W == 3) {
		U3 t = __builtin_amdgcn_raw_buffer_load_b96(r, o, so, 0);
		v = U4{t.x, t.y, t.z, 0};
	}
	if constexpr (W == 2) {
		U2 t = __builtin_amdgcn_raw_buffer_load_b64(r, o, so, 0);
		v = U4{t.x, t.y, 0, 0};
	}
	for (int k = 0; k < 4; k++) same[l * 4 + k] = v[k];
}

int wide_probe() {
	const size_t words = 4096;
	uint32_t *d, *back, *same;
	if (hipMalloc(&d, words * 4) || hipMalloc(&back, 256 * 4) || hipMalloc(&same, 256 * 4)) return 1;
	int bad = 0;
	for (int W = 2; W <= 4; W++)
		for (uint32_t so : {0u, 16u, 48u, 1024u, 1040u}) {
			if (hipMemset(d, 0, words * 4)) return 1;
			if (W == 4) hipLaunchKernelGGL(wide<4>, dim3(1), dim3(64), 0, 0, d, (uint32_t)(words * 4), so, back, same);
			if (W == 3) hipLaunchKernelGGL(wide<3>, dim3(1), dim3(64), 0, 0, d, (uint32_t)(words * 4), so, back, same);
			if (W == 2) hipLaunchKernelGGL(wide<2>, dim3(1), dim3(64), 0, 0, d, (uint32_t)(words * 4), so, back, same);
			uint32_t hb[256], hs[256], hm[4096];
			if (hipMemcpy(hb, back, sizeof hb, hipMemcpyDeviceToHost) || hipMemcpy(hs, same, sizeof hs, hipMemcpyDeviceToHost) ||
					hipMemcpy(hm, d, sizeof hm, hipMemcpyDeviceToHost))
				return 1;
			int nb = 0, ns = 0, nm = 0;
			for (uint32_t l = 0; l < 64; l++) {
				const uint32_t n = (l + 1) & 63;
				for (int k = 0; k < 4; k++) {
					const uint32_t want = k < W ? 7000 + 4 * n + k : 0;
					nb += hb[l * 4 + k] != want;
					ns += hs[l * 4 + k] != want;
					nm += hm[so / 4 + 4 * l + k] != (k < W ? 7000 + 4 * l + k : 0u); // memory image at base + so
				}
			}
			printf("b%-3d soff %5u: cross-lane dword reads wrong %3d, same-width reads wrong %3d, memory image wrong %3d\n", 32 * W, so,
					nb, ns, nm);
			bad += nb + ns + nm;
		}
	return bad ? 2 : 0;
}
