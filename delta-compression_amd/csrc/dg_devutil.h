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

// x mod q for q < 2^23 in FP64 (full-rate FMA on CDNA; the 64-bit Barrett
// above needs four quarter-rate 32x32 multiplies).  x = xh 2^32 + xl with
// xh < 2^29:
//   y = xh (2^32 mod q) + xl         (< 2^52 + 2^32: exact in one FMA)
//   r = y - floor(y inv) q           (exact)
// with inv = 1/q rounded DOWN: y inv never exceeds y / q, and the product's
// rounding (half an ulp of a quotient < 2^52 / q) stays below the 1/q gap
// to the next integer, so floor(y inv) is the quotient or one less and r is
// in [0, 2q): one unsigned minimum brings it into [0, q).
struct ModQ {
	double qd, inv, k1;   // q, 1/q, 2^32 mod q
	bool ok;              // q < 2^23: this path applies
};

__device__ __forceinline__ ModQ make_modq(uint64_t q, uint64_t magic) {
	ModQ m;
	m.ok = q < (1ull << 23);
	m.qd = (double)q;
	m.inv = 1.0 / m.qd;
	if (__fma_rn(m.inv, m.qd, -1.0) > 0.0) m.inv = __longlong_as_double(__double_as_longlong(m.inv) - 1);
	m.k1 = (double)mod_q(1ull << 32, q, magic);
	return m;
}

// (xh converted as a signed dword, xh < 2^29: the unsigned form of
// (x >> 32) is lowered as a 64-bit conversion, an extra ldexp + add per call)
__device__ __forceinline__ uint32_t mod_q_small(uint64_t x, const ModQ& m) {
	const double y = __fma_rn((double)(int32_t)(uint32_t)(x >> 32), m.k1, (double)(uint32_t)x);
	const uint32_t u = (uint32_t)__fma_rn(-floor(y * m.inv), m.qd, y);
	return min(u, u - (uint32_t)m.qd);
}

// slot = x mod q by whichever path applies (m.ok is wave-uniform)
__device__ __forceinline__ uint32_t slot_of(uint64_t x, const ModQ& m, uint64_t q, uint64_t magic) {
	return m.ok ? mod_q_small(x, m) : (uint32_t)mod_q(x, q, magic);
}

// p = 16 fingerprints by byte dot products.  fp = sum_k b_k * c_k mod M with
// c_k = 263^(15-k); splitting every c_k into its 8 bytes gives
//   fp = sum_j 2^(8j) * D_j,  D_j = sum_k b_k * byte_j(c_k) < 2^20,
// and each D_j is four v_dot4_u32_u8 over the window's four dwords (zero
// constant bytes drop out at compile time).  kFpLimb[j][g] packs byte j of
// c_{4g..4g+3}.
constexpr uint32_t kFpLimb[8][4] = {
    {0x90948E99u, 0xCA791EB5u, 0x61A791F7u, 0x01073157u},
    {0x1E666240u, 0xAE927B7Cu, 0x6526B587u, 0x00010E94u},
    {0x58871A1Bu, 0xBBD04668u, 0x2B953A50u, 0x00000115u},
    {0xC9D97A71u, 0x30104632u, 0x1DF75AB2u, 0x00000001u},
    {0x5F67B04Du, 0x15C57474u, 0x0124FA32u, 0x00000000u},
    {0xCCF624B1u, 0xA7A654C3u, 0x00012C35u, 0x00000000u},
    {0x03E64716u, 0xA94AB12Du, 0x00000135u, 0x00000000u},
    {0x140F1603u, 0x1D191B13u, 0x00000001u, 0x00000000u},
};

__device__ __forceinline__ uint64_t fp16_dot(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
	const uint32_t w[4] = {w0, w1, w2, w3};
	uint32_t D[8];
#pragma unroll
	for (int j = 0; j < 8; ++j) {
		uint32_t acc = 0;
#pragma unroll
		for (int g = 0; g < 4; ++g)
			if (kFpLimb[j][g]) acc = __builtin_amdgcn_udot4(w[g], kFpLimb[j][g], acc, false);
		D[j] = acc;
	}
	// Combine in 32-bit pieces: P_i = D_2i + D_2i+1 2^8 < 2^29 and
	//   fp = P0 + P1 2^16 + P2 2^32 + P3 2^48  (mod M),
	// with P3 2^48 = (P3 & 0x1FFF) 2^48 + (P3 >> 13) 2^61 == ... + (P3 >> 13).
	const uint32_t P0 = D[0] + (D[1] << 8), P1 = D[2] + (D[3] << 8);
	const uint32_t P2 = D[4] + (D[5] << 8), P3 = D[6] + (D[7] << 8);
	const uint32_t t = P0 + (P3 >> 13);                 // < 2^30
	const uint32_t lo = t + (P1 << 16);
	const uint32_t c = lo < t ? 1u : 0u;
	const uint32_t hi = P2 + ((P3 & 0x1FFFu) << 16) + (P1 >> 16) + c;   // < 2^31
	// x = hi 2^32 + lo < 2^63: one Mersenne fold and a final subtract
	const uint32_t lo2 = lo + (hi >> 29);
	const uint32_t hi2 = (hi & 0x1FFFFFFFu) + (lo2 < lo ? 1u : 0u);
	uint64_t r = ((uint64_t)hi2 << 32) | lo2;            // <= 2^61 + 2
	return r >= kMersenne ? r - kMersenne : r;
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

// The correcting checkpoint test (correcting.c:164-198): f = fp mod |F|
// passes iff f mod m == k, and its slot is f / m (< cap).  FP64 path for
// |F| < 2^23: mod_q_small, then one floor-quotient by m fixed up by one.
struct Ckpt {
	ModQ mf;            // |F|
	double md, inv_m;   // m, 1/m
	uint32_t k, cap;    // class, slots
	int32_t mshift;     // log2 m when m is a power of two, else -1
};

__device__ __forceinline__ Ckpt make_ckpt(uint64_t f_size, uint64_t f_magic, uint64_t m, uint64_t k,
                                          uint64_t cap) {
	Ckpt c;
	c.mf = make_modq(f_size, f_magic);
	c.md = (double)m;
	c.inv_m = 1.0 / c.md;
	c.k = (uint32_t)k;
	c.cap = cap < 0xFFFFFFFFull ? (uint32_t)cap : 0xFFFFFFFFu;
	c.mshift = (m & (m - 1)) == 0 && m < (1ull << 31) ? (int32_t)__builtin_ctzll(m) : -1;
	return c;
}

// c.mf.ok must hold
__device__ __forceinline__ bool ckpt_test(uint64_t fp, const Ckpt& c, uint32_t* slot) {
	if (c.mshift >= 0) {   // m = 2^s (the default --table-size gives m = 1)
		const uint32_t f = mod_q_small(fp, c.mf);
		const uint32_t i = f >> c.mshift;
		*slot = i;
		return (f & ((1u << c.mshift) - 1u)) == c.k && i < c.cap;
	}
	const double fd = (double)mod_q_small(fp, c.mf);
	double id = floor(fd * c.inv_m);
	double r = __fma_rn(-id, c.md, fd);
	if (r < 0.0) { r += c.md; id -= 1.0; }
	if (r >= c.md) { r -= c.md; id += 1.0; }
	const uint32_t i = (uint32_t)id;
	*slot = i;
	return (uint32_t)r == c.k && i < c.cap;
}

// 16 bytes at any address: the dwords that hold them (the fifth only when
// the address is unaligned, so nothing past the last byte's dword is read)
__device__ __forceinline__ void ld16u(const uint8_t* p, uint32_t (&w)[4]) {
	const uintptr_t a = (uintptr_t)p;
	const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
	const uint32_t s = (uint32_t)(a & 3);
	const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
	const uint32_t d4 = s ? q[4] : 0u;
	w[0] = __builtin_amdgcn_alignbyte(d1, d0, s);
	w[1] = __builtin_amdgcn_alignbyte(d2, d1, s);
	w[2] = __builtin_amdgcn_alignbyte(d3, d2, s);
	w[3] = __builtin_amdgcn_alignbyte(d4, d3, s);
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

// ── wave-level DPP helpers (no LDS round trips) ──

__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }

// x + (lane ^ 1) and x + (lane ^ 2) within quads, via DPP (no LDS traffic)
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
}
// lane l receives x of lane l-1 (lane 0: 0) — DPP wave_shr:1, no LDS
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);
}
// same shift, lane 0 receives 0 (bound_ctrl: one instruction, no old value)
__device__ __forceinline__ uint32_t wave_shr1z(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x138, 0xF, 0xF, true);
}
// inclusive prefix sum over the wave: row_shr 1/2/4/8 inside rows of 16, then
// row_bcast:15 / row_bcast:31 across rows (all DPP, no LDS round trips)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
	return x;
}

// inclusive prefix max over the wave (same DPP network as wave_incl_scan)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
	x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
	return x;
}

// Two-probe Bloom filter of slots over W 32-bit LDS words: the slot's low
// bits and a multiplicative hash.  With 64-256 slots in 2048-4096 bits a
// probe of an absent slot passes ~0.3-1.5 % of the time instead of 3-6 % with
// one probe, so far fewer steps need the exact (ballot) resolution.
template <uint32_t W>
__device__ __forceinline__ uint32_t bloom_h2(uint32_t s) {
	constexpr uint32_t lg = W == 64 ? 11u : (W == 128 ? 12u : (W == 256 ? 13u : 0u));
	static_assert(lg != 0, "64, 128 or 256 words");
	return (s * 0x9E3779B1u) >> (32u - lg);
}
template <uint32_t W>
__device__ __forceinline__ void bloom_add(uint32_t* b, uint32_t s) {
	const uint32_t h1 = s & (32u * W - 1u), h2 = bloom_h2<W>(s);
	atomicOr(&b[h1 >> 5], 1u << (h1 & 31u));
	atomicOr(&b[h2 >> 5], 1u << (h2 & 31u));
}
template <uint32_t W>
__device__ __forceinline__ bool bloom_has(const uint32_t* b, uint32_t s) {
	const uint32_t h1 = s & (32u * W - 1u), h2 = bloom_h2<W>(s);
	return ((b[h1 >> 5] >> (h1 & 31u)) & (b[h2 >> 5] >> (h2 & 31u)) & 1u) != 0u;
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

// ── 3-input XOR (gfx950 v_bitop3_b32, truth table 0x96) ──
// The compiler fuses AND/OR/XOR mixes into v_bitop3 but not XOR chains, so
// table folds (CRC, GF(2) products) build their XORs as explicit trees: N
// terms cost ceil((N - 1) / 2) instructions instead of N - 1.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
template <int N>
__device__ __forceinline__ uint32_t xor_tree(const uint32_t* v) {
	if constexpr (N == 1) {
		return v[0];
	} else if constexpr (N == 2) {
		return v[0] ^ v[1];
	} else {
		constexpr int M = (N + 2) / 3;
		uint32_t w[M];
#pragma unroll
		for (int i = 0; i < M; ++i) {
			if (3 * i + 2 < N) w[i] = xor3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
			else if (3 * i + 1 < N) w[i] = v[3 * i] ^ v[3 * i + 1];
			else w[i] = v[3 * i];
		}
		return xor_tree<M>(w);
	}
}
template <int N>
__device__ __forceinline__ uint64_t xor_tree64(const uint64_t* v) {
	uint32_t l[N], h[N];
#pragma unroll
	for (int k = 0; k < N; ++k) {
		l[k] = (uint32_t)v[k];
		h[k] = (uint32_t)(v[k] >> 32);
	}
	return ((uint64_t)xor_tree<N>(h) << 32) | xor_tree<N>(l);
}

// ── CRC-64/XZ helpers (reflected representation: bit 63 = x^0) ──

// c * K mod P by the constant's nibble tables (tab[16 j + n] = (n x^(4 j)) K)
__device__ __forceinline__ uint64_t mul_nib(uint64_t c, const uint64_t* __restrict__ tab) {
	uint64_t v[16];
#pragma unroll
	for (int j = 0; j < 16; ++j) v[j] = tab[16 * j + ((c >> (4 * j)) & 15)];
	return xor_tree64<16>(v);
}

// slicing-by-4 step: the register's low 32 bits absorb one little-endian word
__device__ __forceinline__ uint64_t slice4(uint64_t crc, uint32_t w, const uint64_t* __restrict__ T) {
	const uint64_t x = crc ^ w;
	const uint64_t v[5] = {T[3 * 256 + (x & 0xff)], T[2 * 256 + ((x >> 8) & 0xff)], T[256 + ((x >> 16) & 0xff)],
	                       T[(x >> 24) & 0xff], x >> 32};
	return xor_tree64<5>(v);
}

// a * b mod P, bit-serial (64 steps; for products by a per-lane constant)
__device__ __forceinline__ uint64_t gf2_mulmod(uint64_t a, uint64_t b) {
	uint64_t p = 0;
#pragma unroll 8
	for (int i = 0; i < 64; ++i) {
		p ^= ((a >> (63 - i)) & 1) ? b : 0ull;
		b = (b >> 1) ^ ((b & 1) ? kCrcPoly : 0ull);
	}
	return p;
}

}  // namespace dg
