// dg_devutil.h — device helpers shared by the gfx950 kernels (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dg_device.h"

namespace dg {


__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
	return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint64_t mask_le(uint32_t j) {   // lanes 0..j
	return j >= 63 ? ~0ULL : ((2ULL << j) - 1ULL);
}

__device__ __forceinline__ uint32_t ffs64(uint64_t m) {     // m != 0
	return (uint32_t)__builtin_ctzll(m);
}

// x mod (2^61-1) for x < 2^63, canonical (src/c/hash.c:15-24).
__device__ __forceinline__ uint64_t mod_m61(uint64_t x) {
	uint64_t r = (x & kMersenne) + (x >> 61);
	return r >= kMersenne ? r - kMersenne : r;
}

// x mod q by Barrett with magic = floor((2^64-1)/q).
__device__ __forceinline__ uint64_t mod_q(uint64_t x, uint64_t q, uint64_t magic) {
	uint64_t qh = __umul64hi(x, magic);
	uint64_t r = x - qh * q;
	if (r >= q) r -= q;
	if (r >= q) r -= q;
	return r;
}

// x mod q for q < 2^25 in FP64 (full-rate FMA on CDNA; the 64-bit Barrett
// above needs four quarter-rate 32x32 multiplies).  x = xh 2^32 + xl:
//   r1 = xh - floor(xh / q) q        (== xh mod q up to one q either way)
//   y  = r1 (2^32 mod q) + xl        (|y| < 2^52: exact)
//   r  = y - floor(y / q) q          (in [-q, 2q), exact)
// and two unsigned minimums bring r into [0, q).  The quotients are off by at
// most one because |quotient| * 2^-52 < 1.
struct ModQ {
	double qd, inv, k1;   // q, 1/q, 2^32 mod q
	bool ok;              // q < 2^25: this path applies
};

__device__ __forceinline__ ModQ make_modq(uint64_t q, uint64_t magic) {
	ModQ m;
	m.ok = q < (1ull << 25);
	m.qd = (double)q;
	m.inv = 1.0 / m.qd;
	m.k1 = (double)mod_q(1ull << 32, q, magic);
	return m;
}

__device__ __forceinline__ uint32_t mod_q_small(uint64_t x, const ModQ& m) {
	const double xh = (double)(uint32_t)(x >> 32), xl = (double)(uint32_t)x;
	const double r1 = __fma_rn(-floor(xh * m.inv), m.qd, xh);
	const double y = __fma_rn(r1, m.k1, xl);
	const uint32_t u = (uint32_t)(int32_t)__fma_rn(-floor(y * m.inv), m.qd, y);
	const uint32_t q = (uint32_t)m.qd;
	const uint32_t v = min(u, u + q);
	return min(v, v - q);
}

// slot = x mod q by whichever path applies (m.ok is wave-uniform)
__device__ __forceinline__ uint32_t slot_of(uint64_t x, const ModQ& m, uint64_t q, uint64_t magic) {
	return m.ok ? mod_q_small(x, m) : (uint32_t)mod_q(x, q, magic);
}

// Karp-Rabin fingerprint of d[0..p) (src/c/hash.c:28-38) as a dot product
// with the constants powc[k] = 263^(p-1-k) mod M: each term is an 8-bit x
// 61-bit product, split into 32-bit halves so that both partial sums fit in
// 64 bits; one fold at the end.
template <int PF>
__device__ __forceinline__ uint64_t window_fp(const uint8_t* d, uint32_t p,
                                              const uint64_t* __restrict__ powc) {
	uint64_t lo = 0, hi = 0;
	if constexpr (PF > 0) {
#pragma unroll
		for (int k = 0; k < PF; ++k) {
			const uint64_t c = powc[k];
			const uint64_t b = d[k];
			lo += b * (uint32_t)c;
			hi += b * (uint32_t)(c >> 32);
		}
	} else {
		for (uint32_t k = 0; k < p; ++k) {
			const uint64_t c = powc[k];
			const uint64_t b = d[k];
			lo += b * (uint32_t)c;
			hi += b * (uint32_t)(c >> 32);
		}
	}
	// hi * 2^32 == (hi >> 29) * 2^61 + (hi & (2^29-1)) * 2^32 == (hi >> 29) + ...
	const uint64_t t = lo + ((hi & ((1ULL << 29) - 1)) << 32) + (hi >> 29);
	return mod_m61(t);
}

// Wave-parallel forward match extension (src/c/onepass.c:229-234): number of
// equal leading bytes of a[] and b[], at most `limit`.  Uniform call.
__device__ __forceinline__ uint64_t extend_fwd(const uint8_t* a, const uint8_t* b,
                                            uint64_t limit) {
	const uint32_t lane = lane_id();
	uint64_t ml = 0;
	while (ml < limit) {
		const uint64_t base = ml + 4ull * lane;
		uint32_t bad = 4;
#pragma unroll
		for (int k = 3; k >= 0; --k) {
			const uint64_t pos = base + k;
			bool ok = false;
			if (pos < limit) ok = a[pos] == b[pos];
			if (!ok) bad = k;
		}
		const uint64_t m = __ballot(bad < 4);
		if (m) {
			const uint32_t f = ffs64(m);
			return ml + 4ull * f + rdlane(bad, f);
		}
		ml += 256;
	}
	return limit;
}

__device__ __forceinline__ void vm_drain() {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// make a value provably wave-uniform (lane 0's copy)
__device__ __forceinline__ uint32_t uni(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
	return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

}  // namespace dg
