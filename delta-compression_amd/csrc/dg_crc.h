// dg_crc.h — CRC-64/XZ segment folds for gfx950 (src/c/delta.h:294-322).
//
// A span is cut into segments of SEG bytes tiled from its 16-byte aligned-up
// end backwards (the leading bytes before the span read as zeros, which a
// raw CRC ignores; the trailing pad is undone by the finaliser).  One wave
// folds one segment as rows of 64 pieces of PB bytes, lane l taking piece l
// of every row (one load instruction reads 64 PB contiguous bytes).  Lane l
// keeps y = A ^ (low 8 bytes of its current piece) and folds
//     y <- L(y) ^ Lh(high 8 bytes of the piece, PB = 16) ^ (next piece's low 8 bytes)
// where L advances a register past the rest of the row (64 PB bytes from the
// piece's first byte), applied as one table lookup per byte:
//     L(y) = XOR_j U_j[byte j of y],   U_j = T advanced by 64 PB - 1 - j bytes.
// The XOR of the 8 (PB = 16: 16) looked-up words and the next piece is a tree
// of 3-input XORs (v_bitop3_b32): with two-input XORs the fold cost ~27 VALU
// per 8 bytes and the pass was VALU-bound below 4.4 TB/s; with the tree it is
// 16 (8 address extracts, 8 XORs) and the pass alone reads 5.0-5.4 TB/s of the
// 6.4 TB/s the same access pattern streams without any CRC work
// (scripts/micro/crc_lab.hip, profiles/r05_crc_lab.txt).
//
// After the last row lane l's register is advanced PB l bytes too far (the
// row tail after its piece is 63 PB - PB l bytes, not 63 PB): one bit-serial
// product with the per-lane constant x^(-8 PB l) fixes it, and the segment's
// raw CRC is the XOR over the lanes.  (Measured: the product by the lane's
// own nibble tables in HBM, 16 gathered loads, ran the pass at 3.9-4.1 TB/s
// instead of 4.9: each gather touches 64 cache lines.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dg_device.h"
#include "dg_devutil.h"

namespace dg {

typedef const __attribute__((address_space(3))) uint64_t lds_cu64;
__device__ __forceinline__ uint64_t ldsq(uint32_t a) { return *(lds_cu64*)(size_t)a; }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
	return (uint32_t)(size_t)(lds_cu64*)(const uint64_t*)p;
}

// keep-mask of bytes [lo, hi) within an 8-byte word (0 <= lo, hi <= 8)
__device__ __forceinline__ uint64_t byte_mask(int lo, int hi) {
	lo = lo < 0 ? 0 : lo;   // clamp first: a negative shift count is undefined
	hi = hi > 8 ? 8 : hi;   // (gfx950 would use its low 6 bits)
	if (hi <= lo) return 0;
	const uint64_t up = hi == 8 ? ~0ULL : ((1ULL << (8 * hi)) - 1);
	const uint64_t dn = lo == 0 ? 0ULL : ((1ULL << (8 * lo)) - 1);
	return up & ~dn;
}

// segments of seg bytes of a span of len >= 8 bytes at start
__device__ __forceinline__ uint32_t crc_nseg(uintptr_t start, uint64_t len, uint64_t seg) {
	const uintptr_t a0 = start & ~(uintptr_t)15, a1 = (start + len + 15) & ~(uintptr_t)15;
	return (uint32_t)((a1 - a0 + seg - 1) / seg);
}

// XOR over the wave (uniform result)
__device__ __forceinline__ uint64_t wave_xor64(uint64_t c) {
#pragma unroll
	for (int d = 32; d >= 1; d >>= 1) {
		const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)c, d, 64);
		const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(c >> 32), d, 64);
		c ^= ((uint64_t)hi << 32) | lo;
	}
	return uni64(c);
}

// Table shapes of the row fold:
//   kCrcByte  one lookup per byte, U_j[256] (2 KiB each; 8 tables for PB = 8,
//             16 for PB = 16).  NC copies interleaved per entry, entry (j, b)
//             of copy c at tb + 2048 NC j + 8 NC b + 8 c, lane l reading copy
//             l % NC (NC = 4: 8 lanes of a 32-lane ds_read_b64 group per copy,
//             over 8 bank pairs, instead of 32 lanes over 32); tables j >= 8
//             from tbh (ds_read offsets are 16-bit)
//   kCrcFive  the 64-bit y split into 13 five-bit fields looked up in tables of
//             32 entries (256 B = one LDS row: a group never conflicts), 3.25
//             KiB for PB = 8; for PB = 16 thirteen more on the high half at
//             tb + 13 * 256.  More VALU per byte, a quarter of the LDS.
enum : int { kCrcByte = 0, kCrcFive = 1 };

template <int TAB, uint32_t PB, uint32_t NC>
__device__ __forceinline__ void crc_fold(uint32_t& ylo, uint32_t& yhi, uint32_t h0, uint32_t h1, uint32_t xlo,
                                         uint32_t xhi, uint32_t tb, uint32_t tbh) {
	constexpr int NL = TAB == kCrcByte ? 8 : 13;
	constexpr int N = PB == 16 ? 2 * NL : NL;
	uint64_t v[N];
	if constexpr (TAB == kCrcByte) {
		constexpr uint32_t TS = 2048 * NC, BS = 8 * NC;
		auto L = [&](uint32_t t, uint32_t b) -> uint64_t {
			return t < 8 ? ldsq(tb + t * TS + b * BS) : ldsq(tbh + (t - 8) * TS + b * BS);
		};
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			v[k] = L(k, (ylo >> (8 * k)) & 0xff);
			v[4 + k] = L(4 + k, (yhi >> (8 * k)) & 0xff);
			if constexpr (PB == 16) {
				v[8 + k] = L(8 + k, (h0 >> (8 * k)) & 0xff);
				v[12 + k] = L(12 + k, (h1 >> (8 * k)) & 0xff);
			}
		}
	} else {
		auto five = [&](uint64_t* o, uint32_t lo, uint32_t hi, uint32_t t) {
			const uint32_t mid = __builtin_amdgcn_alignbit(hi, lo, 30);   // bits 30..34
			o[0] = ldsq(t + 0 * 256 + ((lo << 3) & 0xF8));
			o[1] = ldsq(t + 1 * 256 + ((lo >> 2) & 0xF8));
			o[2] = ldsq(t + 2 * 256 + ((lo >> 7) & 0xF8));
			o[3] = ldsq(t + 3 * 256 + ((lo >> 12) & 0xF8));
			o[4] = ldsq(t + 4 * 256 + ((lo >> 17) & 0xF8));
			o[5] = ldsq(t + 5 * 256 + ((lo >> 22) & 0xF8));
			o[6] = ldsq(t + 6 * 256 + ((mid << 3) & 0xF8));
			o[7] = ldsq(t + 7 * 256 + (hi & 0xF8));
			o[8] = ldsq(t + 8 * 256 + ((hi >> 5) & 0xF8));
			o[9] = ldsq(t + 9 * 256 + ((hi >> 10) & 0xF8));
			o[10] = ldsq(t + 10 * 256 + ((hi >> 15) & 0xF8));
			o[11] = ldsq(t + 11 * 256 + ((hi >> 20) & 0xF8));
			o[12] = ldsq(t + 12 * 256 + ((hi >> 25) & 0x78));
		};
		five(v, ylo, yhi, tb);
		if constexpr (PB == 16) five(v + 13, h0, h1, tb + 13 * 256);
	}
	uint32_t l[N + 1], h[N + 1];
#pragma unroll
	for (int k = 0; k < N; ++k) {
		l[k] = (uint32_t)v[k];
		h[k] = (uint32_t)(v[k] >> 32);
	}
	l[N] = xlo;
	h[N] = xhi;
	ylo = xor_tree<N + 1>(l);
	yhi = xor_tree<N + 1>(h);
}

// The raw CRC (init 0) of segment j of nseg (SEG bytes each) of the span
// [start, start + len), len >= 8, the span's first 8 bytes inverted (init =
// ~0).  Uniform result.  kPf pieces per lane per batch; the next batch is
// loaded before the current one is folded (two register buffers).  kCopy (PB
// = 8): every piece wholly inside [start, copy_hi) is also stored at its
// address + copy_delta (the decode kernel's in-place image of R, made from
// the same loads as R's CRC).  klane: this lane's x^(-8 PB l).
template <uint32_t PB, uint32_t NC, int kPf, uint32_t SEG = kCrcSegBytes, bool kCopy = false, int TAB = kCrcByte>
__device__ __forceinline__ uint64_t crc_seg_rows(uintptr_t start, uint64_t len, uint32_t nseg, uint32_t j,
                                                 uint32_t tb, uint32_t tbh, uint64_t klane,
                                                 intptr_t copy_delta = 0, uintptr_t copy_hi = 0) {
	static_assert(PB == 8 || PB == 16, "piece bytes");
	static_assert(!kCopy || PB == 8, "copy: 8-byte pieces");
	static_assert(TAB == kCrcByte || NC == 1, "five-bit tables: one copy");
	constexpr uint32_t RB = 64 * PB, NR = SEG / RB;
	static_assert(NR % (2 * kPf) == 0, "two batches of rows per loop");
	const uint32_t lane = lane_id();
	const uintptr_t end = start + len;
	const uintptr_t a0 = start & ~(uintptr_t)15;
	const uintptr_t a1 = (end + 15) & ~(uintptr_t)15;
	const uintptr_t dom = a1 - (uintptr_t)nseg * SEG;   // may wrap below a0
	const uintptr_t p0 = dom + (uintptr_t)j * SEG + (uintptr_t)lane * PB;
	// span edges relative to the lane's row-0 piece, clamped so the per-row
	// tests stay in 32-bit arithmetic
	auto clamp32 = [](intptr_t v) -> int32_t {
		return (int32_t)(v < -(intptr_t)RB ? -(intptr_t)RB : (v > (intptr_t)(SEG + RB) ? (intptr_t)(SEG + RB) : v));
	};
	const int32_t f0 = clamp32((intptr_t)start - (intptr_t)p0);
	const int32_t l0 = clamp32((intptr_t)end - (intptr_t)p0);
	const int32_t z0 = clamp32((intptr_t)a0 - (intptr_t)p0);
	typedef uint32_t v4u __attribute__((ext_vector_type(4)));
	typedef uint32_t v2u __attribute__((ext_vector_type(2)));
	typedef typename std::conditional<PB == 16, v4u, v2u>::type piece_t;
	typedef __attribute__((address_space(1))) const piece_t gpiece;
	uint32_t ylo = 0, yhi = 0, h0 = 0, h1 = 0;   // y = A ^ the current piece's low 8 bytes
	// fold one piece into y (from y = 0, h = 0 the first fold is the piece
	// itself: every table maps 0 to 0)
	auto fold_piece = [&](const piece_t& p, uint32_t inv) {
		if constexpr (PB == 16) {
			crc_fold<TAB, PB, NC>(ylo, yhi, h0, h1, p.x ^ inv, p.y ^ inv, tb, tbh);
			h0 = p.z;
			h1 = p.w;
		} else {
			crc_fold<TAB, PB, NC>(ylo, yhi, h0, h1, p.x ^ inv, p.y ^ inv, tb, tbh);
		}
	};
	auto copy = [&](const piece_t* xs, uint32_t r0) {
		if constexpr (kCopy) {
#pragma unroll
			for (int u = 0; u < kPf; ++u) {
				const uintptr_t pa = p0 + (uintptr_t)(r0 + u) * RB;
				if (pa >= start && pa + PB <= copy_hi)
					*reinterpret_cast<__attribute__((address_space(1))) v2u*>(pa + copy_delta) = xs[u];
			}
		}
	};
	// A segment wholly inside a 16-aligned span (every segment but a span's
	// first and last one, and those too when the span is 16-aligned at both
	// ends: C2, C3, the decode's R) has no edge: every load is unconditional,
	// no piece is masked, and init = ~0 is lane 0's first piece inverted.
	const bool edge = (j == 0 && dom != start) || (j + 1 == nseg && end != a1);
	if (!edge) {
		const uint32_t inv = j == 0 && lane == 0 ? ~0u : 0u;
		piece_t xa[kPf], xb[kPf];
		auto load = [&](piece_t* xs, uint32_t r0) {
#pragma unroll
			for (int u = 0; u < kPf; ++u) xs[u] = *reinterpret_cast<gpiece*>(p0 + (uintptr_t)(r0 + u) * RB);
		};
		auto consume = [&](const piece_t* xs, uint32_t r0) {
			copy(xs, r0);
			fold_piece(xs[0], r0 == 0 ? inv : 0u);
#pragma unroll
			for (int u = 1; u < kPf; ++u) fold_piece(xs[u], 0u);
		};
		load(xa, 0);
		for (uint32_t r0 = 0; r0 < NR; r0 += 2 * kPf) {
			load(xb, r0 + kPf);
			consume(xa, r0);
			if (r0 + 2 * kPf < NR) load(xa, r0 + 2 * kPf);
			consume(xb, r0 + kPf);
		}
	} else {
		// a span's first / last segment: pieces wholly before the span are zeros
		// and not loaded (they may lie before the arena), edge pieces masked
		for (uint32_t r0 = 0; r0 < NR; r0 += kPf) {
			piece_t xs[kPf];
#pragma unroll
			for (int u = 0; u < kPf; ++u) {
				const int32_t o = (int32_t)((r0 + u) * RB);
				xs[u] = piece_t{};
				if (o + (int32_t)PB > z0) xs[u] = *reinterpret_cast<gpiece*>(p0 + (uintptr_t)(r0 + u) * RB);
			}
			copy(xs, r0);
#pragma unroll
			for (int u = 0; u < kPf; ++u) {
				const int32_t o = (int32_t)((r0 + u) * RB);
				v4u x;
				if constexpr (PB == 16) x = xs[u];
				else x = v4u{xs[u].x, xs[u].y, 0u, 0u};
				const int32_t f = f0 - o, l = l0 - o;
				if (f > -8 || l < (int32_t)PB) {   // a span edge in this piece
					const int fc = max(min(f, 24), -8);
					const int lc = max(min(l, 24), -8);
					uint64_t lo = ((uint64_t)x.y << 32) | x.x, hi = ((uint64_t)x.w << 32) | x.z;
					lo &= byte_mask(fc, lc);
					hi &= byte_mask(fc - 8, lc - 8);
					lo ^= byte_mask(fc, fc + 8);   // init = ~0
					hi ^= byte_mask(fc - 8, fc);
					x = v4u{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
				}
				piece_t px;
				if constexpr (PB == 16) px = x;
				else px = piece_t{x.x, x.y};
				fold_piece(px, 0u);
			}
		}
	}
	crc_fold<TAB, PB, NC>(ylo, yhi, h0, h1, 0u, 0u, tb, tbh);   // the last row's pieces
	const uint64_t A = ((uint64_t)yhi << 32) | ylo;
	return wave_xor64(A ? gf2_mulmod(A, klane) : 0ull);
}

}  // namespace dg
