// CRC-64/XZ segment-pass lab: the product's row fold (delta-compression_amd/
// csrc/dg_crc.h crc_seg_rows) alone on the GPU, per piece size, table shape,
// load depth and grid, over a 4 GiB span (past the 256 MiB Infinity Cache),
// each checked against a host CRC of sampled segments; beside it the same
// access pattern with no CRC work (the streaming ceiling).
// Round-5 history (profiles/r05_crc_lab.txt): the first version of this lab
// compared XOR chains with 3-input XOR trees (v_bitop3_b32) on byte tables
// (4.7-5.2 vs 5.0-5.4 TB/s) and byte / nibble / five-bit tables.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip scripts/micro/crc_lab.hip -o scripts/micro/crc_lab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../delta-compression_amd/csrc/dg_crc.h"

using namespace dg;

constexpr uint32_t kSeg = kCrcSegBytes;   // 64 KiB

static uint64_t T0[256];
static uint64_t zstep(uint64_t x) { return T0[x & 0xff] ^ (x >> 8); }
static uint64_t gmul(uint64_t a, uint64_t b) {   // reflected GF(2)[x] mod P
	uint64_t p = 0;
	for (int i = 0; i < 64; ++i) {
		if ((a >> (63 - i)) & 1) p ^= b;
		b = (b & 1) ? (b >> 1) ^ kCrcPoly : (b >> 1);
	}
	return p;
}
static uint64_t gdivx(uint64_t z) { return (z & (1ull << 63)) ? ((z ^ kCrcPoly) << 1) | 1 : z << 1; }

// tables as the product lays them out (dg_host.cpp): U_j for PB = 16 at 0
// (16 x 256), for PB = 8 at 4096 (8 x 256); five-bit for PB = 8 at 6144 (13 x
// 32); the lane constants x^(-8 PB l) for PB = 16, then for PB = 8
constexpr uint32_t kR16 = 0, kR8 = 16 * 256, kF8 = 24 * 256, kL16 = kF8 + 13 * 32, kL8 = kL16 + 64;
constexpr uint32_t kWords = kL8 + 64;

template <uint32_t PB, uint32_t NC, int PF, int TAB, uint32_t BLOCK, int MINB = 8>
__global__ __launch_bounds__(BLOCK, BLOCK == 256 ? MINB : 1) void seg_kernel(const uint8_t* buf, uint64_t len, uint32_t nseg,
                                                    const uint64_t* tabs, uint64_t* out) {
	constexpr uint32_t nt = TAB == kCrcFive ? 13 * 32 : (PB == 16 ? 16 : 8) * 256 * NC;
	__shared__ __attribute__((aligned(256))) uint64_t T[nt];
	const uint32_t src = TAB == kCrcFive ? kF8 : (PB == 16 ? kR16 : kR8);
	for (uint32_t i = threadIdx.x; i < nt; i += BLOCK) T[i] = tabs[src + i / NC];
	__syncthreads();
	const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
	const uint32_t tb = lds_addr(T) + 8u * (lane % NC);
	const uint32_t tbh = tb + 8u * 2048u * NC;
	const uint64_t kl = tabs[(PB == 16 ? kL16 : kL8) + lane];
	constexpr uint32_t W = BLOCK / 64;
	for (uint32_t seg = uni(blockIdx.x * W + wave); seg < nseg; seg += gridDim.x * W) {
		const uint64_t c = crc_seg_rows<PB, NC, PF, kCrcSegBytes, false, TAB>((uintptr_t)buf, len, nseg, seg, tb,
		                                                                       tbh, kl);
		if (lane == 0) out[seg] = c;
	}
}

// the first lab's kernel (no span edges, unconditional loads, bit-serial lane
// fix, no VGPR cap): the reference point the product fold is compared with
template <int PF>
__global__ __launch_bounds__(256) void v1_kernel(const uint8_t* buf, uint64_t, uint32_t nseg, const uint64_t* tabs,
                                                 uint64_t* out) {
	constexpr uint32_t RB = 512, NR = kSeg / RB;
	typedef uint32_t v2u __attribute__((ext_vector_type(2)));
	typedef __attribute__((address_space(1))) const v2u gv2;
	__shared__ __attribute__((aligned(256))) uint64_t T[8 * 256];
	for (uint32_t i = threadIdx.x; i < 8 * 256; i += 256) T[i] = tabs[kR8 + i];
	__syncthreads();
	const uint32_t tb = lds_addr(T);
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t kl = tabs[kL8 + lane];
	for (uint32_t seg = blockIdx.x * 4 + (threadIdx.x >> 6); seg < nseg; seg += gridDim.x * 4) {
		const uintptr_t p0 = (uintptr_t)buf + (size_t)seg * kSeg + 8 * lane;
		uint32_t ylo = 0, yhi = 0;
		bool first = true;
		v2u xa[PF], xb[PF];
		auto load = [&](v2u* xs, uint32_t r0) {
#pragma unroll
			for (int u = 0; u < PF; ++u) xs[u] = *reinterpret_cast<gv2*>(p0 + (uintptr_t)(r0 + u) * RB);
		};
		auto step = [&](const v2u* xs) {
			if (first) {
				ylo = xs[0].x;
				yhi = xs[0].y;
				first = false;
			} else {
				crc_fold<kCrcByte, 8, 1>(ylo, yhi, 0, 0, xs[0].x, xs[0].y, tb, tb);
			}
#pragma unroll
			for (int u = 1; u < PF; ++u) crc_fold<kCrcByte, 8, 1>(ylo, yhi, 0, 0, xs[u].x, xs[u].y, tb, tb);
		};
		load(xa, 0);
		for (uint32_t r0 = 0; r0 < NR; r0 += 2 * PF) {
			load(xb, r0 + PF);
			step(xa);
			if (r0 + 2 * PF < NR) load(xa, r0 + 2 * PF);
			step(xb);
		}
		crc_fold<kCrcByte, 8, 1>(ylo, yhi, 0, 0, 0u, 0u, tb, tb);
		const uint64_t A = ((uint64_t)yhi << 32) | ylo;
		uint64_t c = A ? gf2_mulmod(A, kl) : 0ull;
		c = wave_xor64(c);
		if (lane == 0) out[seg] = c;
	}
}

// the same rows of 8-byte pieces, loads only (one XOR per piece)
__global__ __launch_bounds__(256) void read_kernel(const uint8_t* buf, uint32_t nseg, uint64_t* out) {
	constexpr uint32_t RB = 512, NR = kSeg / RB;
	typedef uint32_t v2u __attribute__((ext_vector_type(2)));
	const uint32_t lane = lane_id();
	for (uint32_t seg = uni(blockIdx.x * 4 + (threadIdx.x >> 6)); seg < nseg; seg += gridDim.x * 4) {
		const uintptr_t p0 = (uintptr_t)buf + (size_t)seg * kSeg + 8 * lane;
		uint32_t acc = 0;
		for (uint32_t r0 = 0; r0 < NR; r0 += 8) {
			v2u xs[8];
#pragma unroll
			for (int u = 0; u < 8; ++u) xs[u] = *reinterpret_cast<const v2u*>(p0 + (uintptr_t)(r0 + u) * RB);
#pragma unroll
			for (int u = 0; u < 8; ++u) acc ^= xs[u].x ^ xs[u].y;
		}
		if (acc == 0x9e3779b9u) out[seg] = acc;
	}
}

typedef void (*seg_fn)(const uint8_t*, uint64_t, uint32_t, const uint64_t*, uint64_t*);
struct Variant {
	const char* name;
	seg_fn fn;
	uint32_t block;
	int grids[3];
};

int main() {
	for (int i = 0; i < 256; ++i) {
		uint64_t c = (uint64_t)i;
		for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
		T0[i] = c;
	}
	std::vector<uint64_t> tab(kWords);
	auto img = [&](int rb, uint64_t v, int shift) {   // Z^rb(v << shift), bit by bit
		uint64_t r = 0;
		for (int b = 0; b < 64; ++b)
			if (((v >> b) & 1) && shift + b < 64) {
				uint64_t x = 1ull << (shift + b);
				for (int k = 0; k < rb; ++k) x = zstep(x);
				r ^= x;
			}
		return r;
	};
	{   // byte tables from the advance of single bytes (img is too slow for all)
		std::vector<uint64_t> adv(256);
		for (int i = 0; i < 256; ++i) adv[i] = T0[i];
		for (int n = 1; n <= 1023; ++n) {
			for (int i = 0; i < 256; ++i) adv[i] = (adv[i] >> 8) ^ T0[adv[i] & 0xff];
			if (n >= 1008)
				for (int i = 0; i < 256; ++i) tab[kR16 + (1023 - n) * 256 + i] = adv[i];
			if (n >= 504 && n <= 511)
				for (int i = 0; i < 256; ++i) tab[kR8 + (511 - n) * 256 + i] = adv[i];
		}
	}
	for (int k = 0; k < 13; ++k)
		for (int v = 0; v < 32; ++v) tab[kF8 + 32 * k + v] = img(512, (uint64_t)v, 5 * k);
	uint64_t z16 = 1ull << 63, z8 = 1ull << 63;
	for (int l = 0; l < 64; ++l) {
		tab[kL16 + l] = z16;
		tab[kL8 + l] = z8;
		for (int b = 0; b < 128; ++b) z16 = gdivx(z16);
		for (int b = 0; b < 64; ++b) z8 = gdivx(z8);
	}

	const size_t bytes = 4ull << 30;
	const uint32_t nseg = (uint32_t)(bytes / kSeg);
	uint8_t* d;
	uint64_t *dt, *out;
	if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&dt, 8ull * kWords) != hipSuccess ||
	    hipMalloc(&out, 8ull * nseg) != hipSuccess)
		return 2;
	(void)hipMemcpy(dt, tab.data(), 8ull * kWords, hipMemcpyHostToDevice);
	{
		const size_t chunk = 64ull << 20;
		std::vector<uint64_t> h(chunk / 8);
		uint64_t s = 0x1234567;
		for (size_t off = 0; off < bytes; off += chunk) {
			for (auto& w : h) {
				s = s * 6364136223846793005ull + 1442695040888963407ull;
				w = s ^ (s >> 29);
			}
			(void)hipMemcpy(d + off, h.data(), chunk, hipMemcpyHostToDevice);
		}
	}
	// host raw CRCs of sampled segments (segment 0: the span's first 8 bytes inverted)
	const int ncheck = 9;
	std::vector<uint32_t> cseg(ncheck);
	std::vector<uint64_t> cref(ncheck);
	{
		std::vector<uint8_t> hs(kSeg);
		for (int i = 0; i < ncheck; ++i) {
			cseg[i] = (uint32_t)((uint64_t)i * (nseg - 1) / (ncheck - 1));
			(void)hipMemcpy(hs.data(), d + (size_t)cseg[i] * kSeg, kSeg, hipMemcpyDeviceToHost);
			if (cseg[i] == 0)
				for (int k = 0; k < 8; ++k) hs[k] ^= 0xFF;
			uint64_t c = 0;
			for (uint32_t k = 0; k < kSeg; ++k) c = T0[(c ^ hs[k]) & 0xff] ^ (c >> 8);
			cref[i] = c;
		}
	}
	const Variant vs[] = {
	    {"v1 pf8 pipe (no init)", v1_kernel<8>, 256, {512, 1024, 2048}},
	    {"rows8 byte pf2", seg_kernel<8, 1, 2, kCrcByte, 256>, 256, {512, 1024, 2048}},
	    {"rows8 byte pf4", seg_kernel<8, 1, 4, kCrcByte, 256>, 256, {512, 1024, 2048}},
	    {"rows8 byte pf4 5w", seg_kernel<8, 1, 4, kCrcByte, 256, 5>, 256, {512, 1024, 2048}},
	    {"rows8 byte pf8 uncapped", seg_kernel<8, 1, 8, kCrcByte, 256, 1>, 256, {512, 1024, 2048}},
	    {"rows8 five pf2", seg_kernel<8, 1, 2, kCrcFive, 256>, 256, {512, 1024, 2048}},
	    {"rows16 byte nc4 pf4 wide", seg_kernel<16, 4, 4, kCrcByte, 1024>, 1024, {256, 0, 0}},
	    {"rows16 byte nc1 pf4 wide", seg_kernel<16, 1, 4, kCrcByte, 1024>, 1024, {256, 0, 0}},
	    {"rows16 byte nc4 pf2 wide", seg_kernel<16, 4, 2, kCrcByte, 1024>, 1024, {256, 0, 0}},
	};
	hipEvent_t e0, e1;
	(void)hipEventCreate(&e0);
	(void)hipEventCreate(&e1);
	auto timeit = [&](auto launch) {
		float best = 1e9f;
		for (int rep = 0; rep < 5; ++rep) {
			(void)hipEventRecord(e0, 0);
			launch();
			(void)hipEventRecord(e1, 0);
			(void)hipEventSynchronize(e1);
			float ms;
			(void)hipEventElapsedTime(&ms, e0, e1);
			if (rep && ms < best) best = ms;
		}
		return best;
	};
	for (int grid : {512, 1024, 2048}) {
		float ms = timeit([&] { hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, d, nseg, out); });
		printf("grid %4d  %-26s %.3f ms  %6.0f GB/s\n", grid, "read only", ms, bytes / ms / 1e6);
	}
	int bad = 0;
	for (const Variant& v : vs) {
		for (int grid : v.grids) {
			if (!grid) continue;
			(void)hipMemset(out, 0, 8ull * nseg);
			float ms = timeit([&] { hipLaunchKernelGGL(v.fn, dim3(grid), dim3(v.block), 0, 0, d, (uint64_t)bytes, nseg, dt, out); });
			std::vector<uint64_t> r(nseg);
			(void)hipMemcpy(r.data(), out, 8ull * nseg, hipMemcpyDeviceToHost);
			int vbad = 0;
			for (int i = 0; i < ncheck; ++i) vbad += r[cseg[i]] != cref[i];
			const bool timing_only = strstr(v.name, "no init") != nullptr;
			if (!timing_only) bad += vbad;
			printf("grid %4d  %-32s %.3f ms  %6.0f GB/s %s\n", grid, v.name, ms, bytes / ms / 1e6,
			       timing_only ? "(timing only)" : (vbad ? "MISMATCH" : "ok"));
			fflush(stdout);
		}
	}
	printf("%s\n", bad ? "MISMATCH" : "all variants match the host CRC");
	return bad ? 1 : 0;
}
