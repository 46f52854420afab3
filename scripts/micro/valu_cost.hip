// Issue cost of the vector instructions the member and onepass kernels lean
// on (gfx950): 8 independent chains of one operation, 64 rounds, timed with
// s_memtime inside the kernel; one wave alone on its SIMD (latency + issue)
// and 8 waves per SIMD (issue throughput: cycles per wave-instruction, SIMD
// busy).  Weights for the member-kernel census (profiles/r05_member_census.md).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip scripts/micro/valu_cost.hip -o scripts/micro/valu_cost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

enum Op {
	ADD, XOR3, DOT4, MUL_LO, MUL_HI, MUL24, MAD64, LSHL64, FMA64, CVT_F64_U32, FLOOR64, CVT_U32_F64, PERM, CNDMASK,
	BPERM, READLANE, NOPS
};
static const char* kNames[NOPS] = {"v_add_u32",     "v_bitop3_b32 (xor3)", "v_dot4_u32_u8",  "v_mul_lo_u32",
                                   "v_mul_hi_u32",  "v_mul_u32_u24",       "v_mad_u64_u32",  "v_lshlrev_b64",
                                   "v_fma_f64",     "v_cvt_f64_u32",       "v_floor_f64",    "cvt_u32_f64+cvt_f64_u32",
                                   "v_perm_b32",    "and+cmp+cndmask",       "ds_bpermute_b32", "v_readlane_b32"};

constexpr int kRounds = 64;

template <int OP>
__global__ __launch_bounds__(64) void op_kernel(uint32_t seed, uint64_t* cyc, uint32_t* sink) {
	const uint32_t lane = threadIdx.x;
	uint32_t x[8];
	uint64_t y[8];
	double d[8];
#pragma unroll
	for (int k = 0; k < 8; ++k) {
		x[k] = seed * (lane + 1) + k;
		y[k] = ((uint64_t)x[k] << 17) ^ k;
		d[k] = (double)x[k] * 0.5;
	}
	const uint32_t c = seed | 1u, c2 = seed ^ 0x9E3779B9u;
	__syncthreads();
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int r = 0; r < kRounds; ++r) {
#pragma unroll
		for (int k = 0; k < 8; ++k) {
			if constexpr (OP == ADD) x[k] = x[k] + c;
			else if constexpr (OP == XOR3) x[k] = __builtin_amdgcn_bitop3_b32(x[k], c, c2, 0x96);
			else if constexpr (OP == DOT4) x[k] = __builtin_amdgcn_udot4(c, c2, x[k], false);
			else if constexpr (OP == MUL_LO) x[k] = x[k] * c;
			else if constexpr (OP == MUL_HI) x[k] = __umulhi(x[k], c);
			else if constexpr (OP == MUL24) x[k] = __umul24(x[k], c) + 0u;
			else if constexpr (OP == MAD64) y[k] = (uint64_t)(uint32_t)y[k] * c + y[k];
			else if constexpr (OP == LSHL64) y[k] = y[k] << (c & 31);
			else if constexpr (OP == FMA64) d[k] = __fma_rn(d[k], 0.999, 1.0);
			else if constexpr (OP == CVT_F64_U32) d[k] = (double)(uint32_t)__double2hiint(d[k]);
			else if constexpr (OP == FLOOR64) d[k] = floor(d[k] + 0.25);
			else if constexpr (OP == CVT_U32_F64) d[k] = (double)(uint32_t)d[k];   // + a v_cvt_f64_u32
			else if constexpr (OP == PERM) x[k] = __builtin_amdgcn_perm(x[k], c, 0x07060501u);
			else if constexpr (OP == CNDMASK) x[k] = (x[k] & 1u) ? x[k] : c;
			else if constexpr (OP == BPERM) x[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + 1) & 63) << 2), (int)x[k]);
			else if constexpr (OP == READLANE) x[k] = x[k] + (uint32_t)__builtin_amdgcn_readlane((int)x[k], k);
			// opaque to the optimiser: no folding of the chain across rounds
			asm volatile("" : "+v"(x[k]), "+v"(y[k]), "+v"(d[k]));
		}
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	uint32_t acc = 0;
#pragma unroll
	for (int k = 0; k < 8; ++k) acc ^= x[k] ^ (uint32_t)y[k] ^ (uint32_t)__double2loint(d[k]);
	sink[blockIdx.x * 64 + lane] = acc;
	if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*kfn)(uint32_t, uint64_t*, uint32_t*);
static const kfn kFns[NOPS] = {op_kernel<ADD>,      op_kernel<XOR3>,      op_kernel<DOT4>,   op_kernel<MUL_LO>,
                               op_kernel<MUL_HI>,   op_kernel<MUL24>,     op_kernel<MAD64>,  op_kernel<LSHL64>,
                               op_kernel<FMA64>,    op_kernel<CVT_F64_U32>, op_kernel<FLOOR64>, op_kernel<CVT_U32_F64>,
                               op_kernel<PERM>,     op_kernel<CNDMASK>,   op_kernel<BPERM>,  op_kernel<READLANE>};

int main() {
	int ncu = 0;
	(void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
	const int max_blocks = ncu * 32;
	uint64_t* cyc;
	uint32_t* sink;
	if (hipMalloc(&cyc, 8ull * max_blocks) != hipSuccess || hipMalloc(&sink, 256ull * max_blocks) != hipSuccess) return 2;
	printf("%-22s %14s %14s\n", "instruction", "1 wave/SIMD", "8 waves/SIMD");
	for (int op = 0; op < NOPS; ++op) {
		double per[2];
		const int grids[2] = {ncu * 4, ncu * 32};
		for (int g = 0; g < 2; ++g) {
			for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kFns[op], dim3(grids[g]), dim3(64), 0, 0, 12345u, cyc, sink);
			(void)hipDeviceSynchronize();
			uint64_t h[8192];
			const int n = grids[g] < 8192 ? grids[g] : 8192;
			(void)hipMemcpy(h, cyc, 8ull * n, hipMemcpyDeviceToHost);
			double s = 0;
			for (int i = 0; i < n; ++i) s += (double)h[i];
			per[g] = s / n / (kRounds * 8.0);   // cycles per wave-instruction of this wave
		}
		// at 8 waves per SIMD each wave sees ~8x its share: the SIMD's issue cost is per[1] / 8
		printf("%-22s %10.2f cyc %10.2f cyc (SIMD issue %.2f)\n", kNames[op], per[0], per[1], per[1] / 8.0);
	}
	return 0;
}
