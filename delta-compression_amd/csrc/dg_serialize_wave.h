// dg_serialize_wave.h — one wave serialises its own pair's delta as soon as
// its differencing finishes (placement + DLT\x03 encoding, src/c/apply.c:136-164
// and src/c/encoding.c:39-90), instead of a separate scan + serialise launch.
//
// The pair's place in the packed output is the sum of the sizes of the pairs
// before it, found by a decoupled look-back over per-pair words published in
// HBM (flag in the top bits, value below): AGGREGATE = this pair's size,
// PREFIX = the sizes of all pairs up to and including it.  Waves are
// dispatched in pair order, so every pair a wave waits on is resident or done.
//
// The CRC bytes of the header (9..24) are left to crc_patch_kernel, which runs
// after the CRC kernels (on their own stream) have joined.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dg_devutil.h"

namespace dg {

constexpr unsigned long long kLbAggregate = 1ull << 62;
constexpr unsigned long long kLbPrefix = 2ull << 62;
constexpr unsigned long long kLbValue = (1ull << 62) - 1;

// exclusive prefix of the pair sizes (uniform); publishes this pair's words.
// The look-back reads 64 predecessors per step, one per lane, and stops at
// the nearest PREFIX word once every word after it is published.
__device__ inline uint64_t lookback_offset(unsigned long long* lb, uint32_t pair, uint64_t size) {
	const uint32_t lane = lane_id();
	if (lane == 0)
		__hip_atomic_store(&lb[pair], (pair == 0 ? kLbPrefix : kLbAggregate) | size, __ATOMIC_RELAXED,
		                   __HIP_MEMORY_SCOPE_AGENT);
	if (pair == 0) return 0;
	uint64_t excl = 0;
	uint32_t end = pair;   // predecessors [0, end) not yet summed
	while (true) {
		const uint32_t j = end - 1 - lane;   // lane 0 = nearest predecessor
		unsigned long long w = kLbPrefix;    // below pair 0: an empty prefix
		if (lane < end) w = __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const bool pre = (w & ~kLbValue) == kLbPrefix;
		const uint64_t pm = __ballot(pre);
		const uint32_t stop = pm ? ffs64(pm) : 64u;   // nearest prefix among these lanes
		const uint64_t unready = __ballot((w & ~kLbValue) == 0) & mask_le(stop < 64 ? stop : 63u);
		if (unready) {   // wait for the nearest unpublished word, then look again
			__builtin_amdgcn_s_sleep(1);
			continue;
		}
		// sum lanes 0..stop (inclusive of the prefix word)
		uint64_t v = lane <= stop ? (w & kLbValue) : 0;
		for (int d = 32; d >= 1; d >>= 1) {
			const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d, 64);
			const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d, 64);
			v += ((uint64_t)hi << 32) | lo;
		}
		excl += uni64(v);
		if (stop < 64) break;
		end -= 64;
	}
	if (lane == 0)
		__hip_atomic_store(&lb[pair], kLbPrefix | (excl + size), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return excl;
}

typedef __attribute__((address_space(3))) uint8_t sw_lds8;

template <typename P>
__device__ __forceinline__ void be32_store(P o, uint32_t x) {
	o[0] = (uint8_t)(x >> 24);
	o[1] = (uint8_t)(x >> 16);
	o[2] = (uint8_t)(x >> 8);
	o[3] = (uint8_t)x;
}

// one command per lane (ADD header + short payload + COPY) at base + my;
// long payloads are copied by the whole wave
template <typename P>
__device__ __forceinline__ void put_tile(P base, bool valid, uint32_t my, uint32_t gap, uint32_t prev,
                                         uint32_t cr, uint32_t cv, uint32_t cl, const uint8_t* V) {
	const uint32_t lane = lane_id();
	bool big = false;
	if (valid) {
		P o = base + my;
		if (gap) {
			o[0] = 2;
			be32_store(o + 1, prev);
			be32_store(o + 5, gap);
			if (gap <= 32) {
				for (uint32_t i = 0; i < gap; ++i) o[9 + i] = V[prev + i];
			} else {
				big = true;
			}
			o += 9 + gap;
		}
		o[0] = 1;
		be32_store(o + 1, cr);
		be32_store(o + 5, cv);
		be32_store(o + 9, cl);
	}
	for (uint64_t bm = __ballot(big); bm; bm &= bm - 1) {
		const uint32_t k = ffs64(bm);
		const uint32_t src = rdlane(prev, k), len = rdlane(gap, k), dst = rdlane(my, k) + 9;
		for (uint32_t i = lane; i < len; i += 64) base[dst + i] = V[src + i];
	}
}

// Wave-wide serialisation of one pair.  `out` = the pair's first output
// byte, `size` = its delta size (as accumulated by the differencing), `rec`
// its COPY records (v, r, len) in V order, `stage` >= kStageBytes of LDS.
// Returns 0, or 5 when the bytes written disagree with `size`.
template <uint32_t kStageBytes>
__device__ inline int32_t serialize_wave(uint8_t* out, uint64_t size, const uint8_t* V, uint32_t vl,
                                         const uint32_t* rec, uint32_t n, sw_lds8* stage) {
	const uint32_t lane = lane_id();
	if (lane == 0) {
		out[0] = 'D'; out[1] = 'L'; out[2] = 'T'; out[3] = 3;
		out[4] = 0;   // standard delta
		be32_store(out + 5, vl);
	}
	uint64_t pos = 25;
	uint32_t prev_end = 0;   // end of the previous tile's last COPY
	for (uint32_t t0 = 0; t0 < n; t0 += 64) {
		const uint32_t j = t0 + lane;
		const bool valid = j < n;
		uint32_t cv = 0, cr = 0, cl = 0;
		if (valid) {
			cv = rec[3u * j];
			cr = rec[3u * j + 1];
			cl = rec[3u * j + 2];
		}
		uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)prev_end, (int)(cv + cl), 0x138, 0xF, 0xF, false);
		if (lane == 0) prev = prev_end;
		const uint32_t gap = valid ? cv - prev : 0u;
		const uint32_t sz = valid ? 13u + (gap ? 9u + gap : 0u) : 0u;
		// inclusive prefix of the sizes (DPP network; tile bytes < 4 GiB)
		uint32_t incl = sz;
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xF, 0xF, false);
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xF, 0xF, false);
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xF, 0xF, false);
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xF, 0xF, false);
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x142, 0xA, 0xF, false);
		incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x143, 0xC, 0xF, false);
		const uint32_t my = incl - sz;
		const uint32_t S = rdlane(incl, 63);
		if (S <= kStageBytes) {
			put_tile(stage, valid, my, gap, prev, cr, cv, cl, V);
			__builtin_amdgcn_s_waitcnt(0xc07f);   // staged bytes are in LDS
			__builtin_amdgcn_wave_barrier();
			// flush: head bytes to a dword boundary, dwords, tail bytes
			uint8_t* dst = out + pos;
			const uint32_t head = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);
			if (lane < head && lane < S) dst[lane] = stage[lane];
			if (S > head) {
				const uint32_t nd = (S - head) / 4;
				uint32_t* dw = reinterpret_cast<uint32_t*>(dst + head);
				for (uint32_t k = lane; k < nd; k += 64) {
					const uint32_t o = head + 4 * k;
					typedef __attribute__((address_space(3))) const uint32_t sw_lds32c;
					const sw_lds32c* w = (const sw_lds32c*)(stage + (o & ~3u));
					dw[k] = __builtin_amdgcn_alignbyte(w[1], w[0], o & 3u);
				}
				const uint32_t tail0 = head + 4 * nd;
				if (lane < S - tail0) dst[tail0 + lane] = stage[tail0 + lane];
			}
			__builtin_amdgcn_s_waitcnt(0xc07f);   // LDS reads done before the next tile
			__builtin_amdgcn_wave_barrier();
		} else {
			put_tile(out + pos, valid, my, gap, prev, cr, cv, cl, V);
		}
		pos += S;
		prev_end = rdlane(cv + cl, n - 1 - t0 < 63u ? n - 1 - t0 : 63u);
	}
	if (prev_end < vl) {   // trailing ADD (src/c/onepass.c:268-275)
		const uint32_t len = vl - prev_end;
		if (lane == 0) {
			out[pos] = 2;
			be32_store(out + pos + 1, prev_end);
			be32_store(out + pos + 5, len);
		}
		for (uint32_t i = lane; i < len; i += 64) out[pos + 9 + i] = V[prev_end + i];
		pos += 9 + len;
	}
	if (lane == 0) out[pos] = 0;   // END
	return pos + 1 == size ? 0 : 5;
}

}  // namespace dg
