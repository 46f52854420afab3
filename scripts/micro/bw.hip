// HBM read-bandwidth calibration on MI355X: (a) grid-stride coalesced 16 B
// loads, (b) one wave per 64 KiB / 256 KiB region in 4 KiB passes (the member
// scan's access pattern, two streams), (c) same with 16 KiB per pass.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void gs_read(const uint4* p, size_t n, uint32_t* out) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		uint4 v = p[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) out[0] = acc;
}

template <int ROWS>
__global__ __launch_bounds__(64) void wave_region(const uint8_t* a, const uint8_t* b, uint32_t region, uint32_t* out) {
	const uint8_t* A = a + (size_t)blockIdx.x * region;
	const uint8_t* B = b + (size_t)blockIdx.x * region;
	uint32_t acc = 0;
	const uint32_t lane = threadIdx.x;
	for (uint32_t o = 0; o < region; o += 1024 * ROWS) {
		uint4 va[ROWS], vb[ROWS];
#pragma unroll
		for (int k = 0; k < ROWS; ++k) {
			va[k] = *(const uint4*)(A + o + 1024 * k + 16 * lane);
			vb[k] = *(const uint4*)(B + o + 1024 * k + 16 * lane);
		}
#pragma unroll
		for (int k = 0; k < ROWS; ++k) acc ^= va[k].x ^ vb[k].y ^ va[k].z ^ vb[k].w;
	}
	if (acc == 0x12345678u) out[0] = acc;
}

int main() {
	const size_t bytes = 1ull << 30;   // per stream
	uint8_t *a, *b;
	uint32_t* out;
	hipMalloc(&a, bytes);
	hipMalloc(&b, bytes);
	hipMalloc(&out, 4);
	hipMemset(a, 1, bytes);
	hipMemset(b, 2, bytes);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	float ms;
	for (int blocks : {1024, 2048, 4096, 8192}) {
		for (int r = 0; r < 2; ++r) {
			hipEventRecord(e0);
			hipLaunchKernelGGL(gs_read, dim3(blocks), dim3(256), 0, 0, (const uint4*)a, bytes / 16, out);
			hipEventRecord(e1);
			hipEventSynchronize(e1);
			hipEventElapsedTime(&ms, e0, e1);
		}
		printf("grid-stride %5d x 256: %.1f GB/s\n", blocks, bytes / (ms * 1e6));
	}
	for (uint32_t region : {65536u, 262144u}) {
		const uint32_t waves = bytes / region;
		for (int rows : {4, 16}) {
			for (int r = 0; r < 2; ++r) {
				hipEventRecord(e0);
				if (rows == 4) hipLaunchKernelGGL(wave_region<4>, dim3(waves), dim3(64), 0, 0, a, b, region, out);
				else hipLaunchKernelGGL(wave_region<16>, dim3(waves), dim3(64), 0, 0, a, b, region, out);
				hipEventRecord(e1);
				hipEventSynchronize(e1);
				hipEventElapsedTime(&ms, e0, e1);
			}
			printf("wave per %6u B region, %2d KiB/pass, 2 streams: %.1f GB/s (%u waves)\n", region, rows, 2.0 * bytes / (ms * 1e6), waves);
		}
	}
	return 0;
}
