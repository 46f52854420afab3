// Microbenchmark: does an in-flight global_load_lds (LDS-DMA) delay a later
// ds_read + s_waitcnt lgkmcnt(0) on gfx950?  Prints cycles for
//   A: ds_read + lgkmcnt(0) alone
//   B: DMA issued (cold HBM line), then ds_read + lgkmcnt(0)
//   C: DMA issued, then s_waitcnt vmcnt(0)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void lds_void_t;
__global__ void k(const uint8_t* g, uint64_t* out, int mode, size_t base) {
	__shared__ __attribute__((aligned(16))) uint32_t lds[2048];
	const uint32_t lane = threadIdx.x;
	lds[lane] = lane;
	__syncthreads();
	uint64_t t0 = __builtin_amdgcn_s_memtime();
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	t0 = __builtin_amdgcn_s_memtime();
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	if (mode >= 1)
		__builtin_amdgcn_global_load_lds((const void*)(g + base + (size_t)blockIdx.x * 65536 + 16 * lane),
		                                 (lds_void_t*)(lds + 1024), 16, 0, 0);
	uint32_t v = 0;
	if (mode == 2) {
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	} else {
		asm volatile("" ::: "memory");
		v = lds[(lane * 7) & 511];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	}
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	out[blockIdx.x * 64 + lane] = (t1 - t0) + ((uint64_t)v << 40);
}
int main() {
	uint8_t* g; uint64_t* o;
	const int nb = 256;
	uint8_t* f;
	const size_t gsz = (size_t)16 * nb * 65536, fsz = (size_t)1 << 29;
	hipMalloc(&g, gsz);
	hipMemset(g, 1, gsz);
	hipMalloc(&f, fsz);
	hipMalloc(&o, nb * 64 * 8);
	static uint64_t h[nb * 64];
	for (int mode = 0; mode < 3; ++mode) {
		for (int rep = 0; rep < 3; ++rep) {
			// evict: touch a big buffer between reps
			hipMemset(f, rep, fsz);   // push g's lines out of L2 / Infinity Cache
			hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, g, o, mode, (size_t)(mode * 3 + rep) * nb * 65536);
			hipDeviceSynchronize();
		}
		hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
		uint64_t s = 0, mx = 0;
		for (int i = 0; i < nb; ++i) { uint64_t c = h[i * 64] & ((1ull << 40) - 1); s += c; if (c > mx) mx = c; }
		printf("mode %d (%s): mean %.0f max %llu cycles\n", mode,
		       mode == 0 ? "ds_read+lgkmcnt(0)" : mode == 1 ? "DMA then ds_read+lgkmcnt(0)" : "DMA then vmcnt(0)",
		       (double)s / nb, (unsigned long long)mx);
	}
	return 0;
}
