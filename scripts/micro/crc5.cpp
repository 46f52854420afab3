// CRC-64/XZ segment kernels, LDS table shapes compared (row-interleaved
// segments as crc_seg_rows in dg_kernels.hip: lane l folds piece l of every
// 64 x PB-byte row; U = "advance past the rest of the row" folded into tables):
//   byte  8 tables x 256 entries (2 KiB each): one lookup per byte; a 32-lane
//         group of ds_read_b64 spreads over 256 entries on 32 bank pairs, so
//         random bytes collide (~3.5 LDS cycles per group)
//   five  13 tables x 32 entries (256 B each = one LDS row of 64 banks): one
//         lookup per 5 bits, and a group can never conflict (distinct entries
//         sit on distinct bank pairs, equal ones broadcast)
// Prints GB/s of each over a 1 GiB buffer (one wave per 64 KiB segment) and
// checks both against a host CRC of a few segments.
// Build: hipcc --offload-arch=gfx950 -O3 -x hip scripts/micro/crc5.cpp -o scripts/micro/crc5
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

constexpr uint64_t kPoly = 0xC96C5795D7870F42ull;   // reflected CRC-64/XZ
constexpr uint32_t kSeg = 65536, kPB = 8, kRB = 64 * kPB, kNR = kSeg / kRB;

static uint64_t T0[256];
static uint64_t zstep(uint64_t x) { return T0[x & 0xff] ^ (x >> 8); }
static uint64_t zpow(uint64_t x, int n) {
	for (int i = 0; i < n; ++i) x = zstep(x);
	return x;
}
// multiply in GF(2)[x]/P, reflected (bit 63 = x^0)
static uint64_t gmul(uint64_t a, uint64_t b) {
	uint64_t r = 0;
	for (int i = 0; i < 64; ++i) {
		if (b & (1ull << 63)) r ^= a;
		b <<= 1;
		a = (a & 1) ? (a >> 1) ^ kPoly : a >> 1;
	}
	return r;
}
static uint64_t gdivx(uint64_t z) { return (z & (1ull << 63)) ? ((z ^ kPoly) << 1) | 1 : z << 1; }

__device__ __forceinline__ uint64_t ldsq(uint32_t a) {
	return *(const __attribute__((address_space(3))) uint64_t*)(size_t)a;
}
__device__ __forceinline__ uint64_t gmul_dev(uint64_t a, uint64_t b) {
	uint64_t r = 0;
	for (int i = 0; i < 64; ++i) {
		if (b & (1ull << 63)) r ^= a;
		b <<= 1;
		a = (a & 1) ? (a >> 1) ^ kPoly : a >> 1;
	}
	return r;
}

template <int MODE>
__global__ __launch_bounds__(256) void seg_kernel(const uint8_t* buf, uint32_t nseg, const uint64_t* tabs,
                                                  const uint64_t* klane, uint64_t* out) {
	__shared__ __attribute__((aligned(256))) uint64_t T[MODE == 0 ? 8 * 256 : 13 * 32];
	constexpr uint32_t NT = MODE == 0 ? 8 * 256 : 13 * 32;
	for (uint32_t i = threadIdx.x; i < NT; i += 256) T[i] = tabs[i];
	__syncthreads();
	const uint32_t tb = (uint32_t)(size_t)(const __attribute__((address_space(3))) uint64_t*)T;
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t kl = klane[lane];
	for (uint32_t seg = blockIdx.x * 4 + (threadIdx.x >> 6); seg < nseg; seg += gridDim.x * 4) {
		const uint8_t* p0 = buf + (size_t)seg * kSeg + kPB * lane;
		uint64_t A = 0;
		for (uint32_t r0 = 0; r0 < kNR; r0 += 8) {
			uint64_t xs[8];
#pragma unroll
			for (int u = 0; u < 8; ++u) xs[u] = *(const uint64_t*)(p0 + (size_t)(r0 + u) * kRB);
#pragma unroll
			for (int u = 0; u < 8; ++u) {
				const uint64_t y = A ^ xs[u];
				const uint32_t lo = (uint32_t)y, hi = (uint32_t)(y >> 32);
				if constexpr (MODE == 0) {
					A = ldsq(tb + 0 * 2048 + (lo & 0xff) * 8) ^ ldsq(tb + 1 * 2048 + ((lo >> 8) & 0xff) * 8) ^
					    ldsq(tb + 2 * 2048 + ((lo >> 16) & 0xff) * 8) ^ ldsq(tb + 3 * 2048 + (lo >> 24) * 8) ^
					    ldsq(tb + 4 * 2048 + (hi & 0xff) * 8) ^ ldsq(tb + 5 * 2048 + ((hi >> 8) & 0xff) * 8) ^
					    ldsq(tb + 6 * 2048 + ((hi >> 16) & 0xff) * 8) ^ ldsq(tb + 7 * 2048 + (hi >> 24) * 8);
				} else {
					const uint32_t mid = __builtin_amdgcn_alignbit(hi, lo, 30);
					A = ldsq(tb + 0 * 256 + ((lo << 3) & 0xF8)) ^ ldsq(tb + 1 * 256 + ((lo >> 2) & 0xF8)) ^
					    ldsq(tb + 2 * 256 + ((lo >> 7) & 0xF8)) ^ ldsq(tb + 3 * 256 + ((lo >> 12) & 0xF8)) ^
					    ldsq(tb + 4 * 256 + ((lo >> 17) & 0xF8)) ^ ldsq(tb + 5 * 256 + ((lo >> 22) & 0xF8)) ^
					    ldsq(tb + 6 * 256 + ((mid << 3) & 0xF8)) ^ ldsq(tb + 7 * 256 + ((hi >> 0) & 0xF8)) ^
					    ldsq(tb + 8 * 256 + ((hi >> 5) & 0xF8)) ^ ldsq(tb + 9 * 256 + ((hi >> 10) & 0xF8)) ^
					    ldsq(tb + 10 * 256 + ((hi >> 15) & 0xF8)) ^ ldsq(tb + 11 * 256 + ((hi >> 20) & 0xF8)) ^
					    ldsq(tb + 12 * 256 + ((hi >> 25) & 0x78));
				}
			}
		}
		uint64_t c = A ? gmul_dev(A, kl) : 0ull;
#pragma unroll
		for (int d = 32; d >= 1; d >>= 1) {
			const uint32_t l2 = (uint32_t)__shfl_xor((int)(uint32_t)c, d, 64);
			const uint32_t h2 = (uint32_t)__shfl_xor((int)(uint32_t)(c >> 32), d, 64);
			c ^= ((uint64_t)h2 << 32) | l2;
		}
		if (lane == 0) out[seg] = c;
	}
}

int main() {
	for (int i = 0; i < 256; ++i) {
		uint64_t c = (uint64_t)i;
		for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
		T0[i] = c;
	}
	// byte tables: U_j[b] = Z^(RB - j)(b) (byte j of the piece, then the rest of the row)
	std::vector<uint64_t> tb(8 * 256), t5(13 * 32), kl(64);
	for (int j = 0; j < 8; ++j)
		for (int b = 0; b < 256; ++b) tb[j * 256 + b] = zpow((uint64_t)b, kRB - j);
	// five-bit tables: F_k[v] = Z^RB(v << 5k), from the images of the 64 basis bits
	uint64_t col[64];
	for (int i = 0; i < 64; ++i) col[i] = zpow(1ull << i, kRB);
	for (int k = 0; k < 13; ++k)
		for (int v = 0; v < 32; ++v) {
			uint64_t r = 0;
			for (int bit = 0; bit < 5; ++bit)
				if ((v >> bit) & 1 && 5 * k + bit < 64) r ^= col[5 * k + bit];
			t5[k * 32 + v] = r;
		}
	uint64_t z = 1ull << 63;   // x^(-8 PB l)
	for (int l = 0; l < 64; ++l) {
		kl[l] = z;
		for (int b = 0; b < 8 * (int)kPB; ++b) z = gdivx(z);
	}
	const size_t bytes = 1ull << 30;
	const uint32_t nseg = (uint32_t)(bytes / kSeg);
	std::vector<uint8_t> h(bytes);
	uint64_t s = 0x1234567;
	for (size_t i = 0; i < bytes; i += 8) {
		s = s * 6364136223846793005ull + 1442695040888963407ull;
		*(uint64_t*)&h[i] = s ^ (s >> 29);
	}
	uint8_t* d;
	uint64_t *dtb, *dt5, *dkl, *out;
	hipMalloc(&d, bytes);
	hipMalloc(&dtb, 8 * 256 * 8);
	hipMalloc(&dt5, 13 * 32 * 8);
	hipMalloc(&dkl, 64 * 8);
	hipMalloc(&out, 8ull * nseg * 2);
	hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
	hipMemcpy(dtb, tb.data(), tb.size() * 8, hipMemcpyHostToDevice);
	hipMemcpy(dt5, t5.data(), t5.size() * 8, hipMemcpyHostToDevice);
	hipMemcpy(dkl, kl.data(), 64 * 8, hipMemcpyHostToDevice);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	for (int grid : {256 * 2, 256 * 4, 256 * 8}) {
		for (int mode = 0; mode < 2; ++mode) {
			float best = 1e9f;
			for (int rep = 0; rep < 6; ++rep) {
				hipEventRecord(e0, 0);
				if (mode == 0)
					hipLaunchKernelGGL(seg_kernel<0>, dim3(grid), dim3(256), 0, 0, d, nseg, dtb, dkl, out);
				else
					hipLaunchKernelGGL(seg_kernel<1>, dim3(grid), dim3(256), 0, 0, d, nseg, dt5, dkl, out + nseg);
				hipEventRecord(e1, 0);
				hipEventSynchronize(e1);
				float ms;
				hipEventElapsedTime(&ms, e0, e1);
				if (rep && ms < best) best = ms;
			}
			printf("grid %d %s: %.3f ms  %.0f GB/s\n", grid, mode ? "five-bit" : "byte", best, bytes / best / 1e6);
		}
	}
	std::vector<uint64_t> r(2ull * nseg);
	hipMemcpy(r.data(), out, r.size() * 8, hipMemcpyDeviceToHost);
	int bad = 0;
	for (uint32_t sg = 0; sg < nseg; sg += nseg / 7) {
		uint64_t c = 0;   // raw CRC (init 0) of the segment
		for (uint32_t i = 0; i < kSeg; ++i) c = T0[(c ^ h[(size_t)sg * kSeg + i]) & 0xff] ^ (c >> 8);
		if (r[sg] != c || r[nseg + sg] != c) {
			++bad;
			printf("seg %u: host %016llx byte %016llx five %016llx\n", sg, (unsigned long long)c,
			       (unsigned long long)r[sg], (unsigned long long)r[nseg + sg]);
		}
	}
	printf("%s\n", bad ? "MISMATCH" : "both match the host CRC");
	return bad ? 1 : 0;
}
