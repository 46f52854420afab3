// PMC calibration (MI355X_MICROARCH.md, HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel moves a known number of bytes in one access class the product
// uses; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over this binary gives the
// counter per class, and scripts/pmc_calib.py turns them into factors.
//   stream16   coalesced 16 B/lane global loads          (CRC, staging)
//   dma16      16 B/lane global_load_lds (LDS-DMA)       (onepass windows, member staging)
//   stream8    coalesced 8 B/lane global loads           (CRC rows beside the onepass kernel)
//   dma4       4 B/lane global_load_lds, coalesced       (the serialisers' record rings)
//   rand16     one 16 B load per lane at a random 128 B line (onepass table tier)
//   rand4      one 4 B load per lane at a random line    (correcting index probes)
//   store16    coalesced 16 B/lane stores                 (serialisers, decode)
//   store16r   one 16 B store per lane at a random line  (table-tier first writers)
// Every buffer is 2 GiB (> the 256 MiB Infinity Cache), every random line is
// touched once per launch (a permutation), so no byte is served on-die.
// Build: hipcc --offload-arch=gfx950 -O3 -x hip scripts/micro/pmc_calib.cpp -o scripts/micro/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr size_t kBytes = 2ull << 30;        // 2 GiB per buffer
constexpr size_t kLines = kBytes / 128;      // 16 Mi lines

__device__ __forceinline__ uint32_t perm_line(uint32_t i) {
	// a bijection on [0, 2^24): odd multiplier, xorshift (mod 2^24)
	uint32_t x = i * 0x9E3779Bu;
	x ^= x >> 11;
	x *= 0x2C1B3C6Du;
	x ^= x >> 13;
	return x & (uint32_t)(kLines - 1);
}

__global__ __launch_bounds__(256) void stream16(const uint4* p, size_t n, uint32_t* sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		const uint4 v = p[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x9u) sink[0] = acc;
}

__global__ __launch_bounds__(64) void dma16(const uint8_t* p, size_t n, uint32_t* sink) {
	__shared__ __attribute__((aligned(16))) uint8_t lds[4096];
	const uint32_t lane = threadIdx.x;
	for (size_t o = (size_t)blockIdx.x * 4096; o < n; o += (size_t)gridDim.x * 4096) {
#pragma unroll
		for (int k = 0; k < 4; ++k)
			__builtin_amdgcn_global_load_lds((const void*)(p + o + 1024 * k + 16 * lane), (lds_void_t*)(lds + 1024 * k), 16, 0, 0);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	}
	__syncthreads();
	if (lds[lane] == 0xFF && lds[lane + 64] == 0xFE && lane == 77) sink[0] = 1;
}

__global__ __launch_bounds__(256) void stream8(const uint2* p, size_t n, uint32_t* sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		const uint2 v = p[i];
		acc ^= v.x ^ v.y;
	}
	if (acc == 0x9u) sink[0] = acc;
}

__global__ __launch_bounds__(64) void dma4(const uint8_t* p, size_t n, uint32_t* sink) {
	__shared__ __attribute__((aligned(16))) uint8_t lds[4096];
	const uint32_t lane = threadIdx.x;
	for (size_t o = (size_t)blockIdx.x * 4096; o < n; o += (size_t)gridDim.x * 4096) {
#pragma unroll
		for (int k = 0; k < 16; ++k)
			__builtin_amdgcn_global_load_lds((const void*)(p + o + 256 * k + 4 * lane), (lds_void_t*)(lds + 256 * k), 4, 0, 0);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	}
	__syncthreads();
	if (lds[lane] == 0xFF && lds[lane + 64] == 0xFE && lane == 77) sink[0] = 1;
}

// one load per lane: line perm(i), at a 16 B slot inside it chosen by i
__global__ __launch_bounds__(256) void rand16(const uint8_t* p, uint32_t n, uint32_t* sink) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	const uint4 v = *(const uint4*)(p + 128ull * perm_line(i) + 16 * (i & 7));
	if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9u) sink[0] = 1;
}

__global__ __launch_bounds__(256) void rand4(const uint8_t* p, uint32_t n, uint32_t* sink) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	const uint32_t v = *(const uint32_t*)(p + 128ull * perm_line(i) + 4 * (i & 31));
	if (v == 0x9u) sink[0] = 1;
}

__global__ __launch_bounds__(256) void store16(uint4* p, size_t n) {
	for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
		p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ __launch_bounds__(256) void store16r(uint8_t* p, uint32_t n) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n) return;
	*(uint4*)(p + 128ull * perm_line(i) + 16 * (i & 7)) = make_uint4(i, 1u, 2u, 3u);
}

int main(int argc, char** argv) {
	const char* which = argc > 1 ? argv[1] : "all";
	uint8_t *a = nullptr, *b = nullptr;
	uint32_t* sink = nullptr;
	if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&b, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
		fprintf(stderr, "alloc failed\n");
		return 1;
	}
	hipMemset(a, 1, kBytes);
	hipMemset(b, 0, kBytes);
	hipDeviceSynchronize();
	const uint32_t nr = (uint32_t)kLines;   // one access per line of the 2 GiB buffer
	auto on = [&](const char* k) { return !strcmp(which, "all") || !strcmp(which, k); };
	// known bytes per launch (printed for pmc_calib.py)
	if (on("stream16")) { hipLaunchKernelGGL(stream16, dim3(2048), dim3(256), 0, 0, (const uint4*)a, kBytes / 16, sink); printf("stream16 %zu\n", kBytes); }
	if (on("dma16")) { hipLaunchKernelGGL(dma16, dim3(8192), dim3(64), 0, 0, a, kBytes, sink); printf("dma16 %zu\n", kBytes); }
	if (on("stream8")) { hipLaunchKernelGGL(stream8, dim3(2048), dim3(256), 0, 0, (const uint2*)a, kBytes / 8, sink); printf("stream8 %zu\n", kBytes); }
	if (on("dma4")) { hipLaunchKernelGGL(dma4, dim3(8192), dim3(64), 0, 0, a, kBytes, sink); printf("dma4 %zu\n", kBytes); }
	if (on("rand16")) { hipLaunchKernelGGL(rand16, dim3(nr / 256), dim3(256), 0, 0, a, nr, sink); printf("rand16 %zu\n", (size_t)nr * 16); }
	if (on("rand4")) { hipLaunchKernelGGL(rand4, dim3(nr / 256), dim3(256), 0, 0, a, nr, sink); printf("rand4 %zu\n", (size_t)nr * 4); }
	if (on("store16")) { hipLaunchKernelGGL(store16, dim3(2048), dim3(256), 0, 0, (uint4*)b, kBytes / 16); printf("store16 %zu\n", kBytes); }
	if (on("store16r")) { hipLaunchKernelGGL(store16r, dim3(nr / 256), dim3(256), 0, 0, b, nr); printf("store16r %zu\n", (size_t)nr * 16); }
	const hipError_t e = hipDeviceSynchronize();
	if (e != hipSuccess) {
		fprintf(stderr, "%s\n", hipGetErrorString(e));
		return 1;
	}
	hipFree(a);
	hipFree(b);
	hipFree(sink);
	return 0;
}
