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

// kCmd consecutive commands per lane: command i of lane L is record
// t0 + kCmd*L + i.  `prev0` = end of the command before the lane's first.
// Writes the lane's commands back to back from base + my; long payloads
// (> 32 bytes) are copied by the whole wave afterwards.
template <int kCmd, typename P>
__device__ __forceinline__ void put_cmds(P base, const bool (&valid)[kCmd], uint32_t my, uint32_t prev0,
                                         const uint32_t (&cv)[kCmd], const uint32_t (&cr)[kCmd],
                                         const uint32_t (&cl)[kCmd], const uint32_t (&cw)[kCmd], bool inl,
                                         const uint8_t* V, uint32_t vl) {
	const uint32_t lane = lane_id();
	uint32_t prev = prev0, o = my;
	bool big[kCmd];
	uint32_t bsrc[kCmd], blen[kCmd], bdst[kCmd];
#pragma unroll
	for (int i = 0; i < kCmd; ++i) {
		big[i] = false;
		bsrc[i] = blen[i] = bdst[i] = 0;
		if (valid[i]) {
			const uint32_t gap = cv[i] - prev;
			P q = base + o;
			if (gap) {
				q[0] = 2;
				be32_store(q + 1, prev);
				be32_store(q + 5, gap);
				if (inl && gap <= 4) {   // payload carried in the record
					for (uint32_t k = 0; k < gap; ++k) q[9 + k] = (uint8_t)(cw[i] >> (8 * k));
				} else if (gap <= 32) {
					// 8 unaligned dword loads, all issued unconditionally (a
					// per-word condition made the compiler branch around each
					// load and wait for it, and for every store before it: up to
					// 8 dependent round trips per tile), at addresses clamped
					// inside V (gap > 4 and prev + gap <= |V|, so |V| >= 5); a
					// word that crosses |V| is loaded from |V| - 4 and shifted
					// down, a word past |V| is never used
					uint32_t wd[8];
					const uint32_t vl4 = vl - 4u;
#pragma unroll
					for (int k = 0; k < 8; ++k) {
						const uint32_t o4 = prev + 4u * k;
						const uint32_t a4 = umin32(o4, vl4);
						uint32_t w;
						__builtin_memcpy(&w, V + a4, 4);
						wd[k] = w >> (8u * umin32(o4 - a4, 3u));
					}
#pragma unroll
					for (int k = 0; k < 32; ++k)
						if ((uint32_t)k < gap) q[9 + k] = (uint8_t)(wd[k >> 2] >> (8 * (k & 3)));
				} else {
					big[i] = true;
					bsrc[i] = prev;
					blen[i] = gap;
					bdst[i] = o + 9;
				}
				q += 9 + gap;
				o += 9 + gap;
			}
			q[0] = 1;
			be32_store(q + 1, cr[i]);
			be32_store(q + 5, cv[i]);
			be32_store(q + 9, cl[i]);
			o += 13;
			prev = cv[i] + cl[i];
		}
	}
	// long payloads: the whole wave, 4 bytes per lane per pass (unaligned
	// dword loads, never past the end of V)
#pragma unroll
	for (int i = 0; i < kCmd; ++i)
		for (uint64_t bm = __ballot(big[i]); bm; bm &= bm - 1) {
			const uint32_t k = ffs64(bm);
			const uint32_t src = rdlane(bsrc[i], k), len = rdlane(blen[i], k), dst = rdlane(bdst[i], k);
			for (uint32_t x = 4 * lane; x < len; x += 256) {
				uint32_t w = 0;
				if (src + x + 4 <= vl) {
					__builtin_memcpy(&w, V + src + x, 4);
				} else {
					for (uint32_t b = 0; b < 4 && src + x + b < vl; ++b) w |= (uint32_t)V[src + x + b] << (8 * b);
				}
#pragma unroll
				for (uint32_t b = 0; b < 4; ++b)
					if (x + b < len) base[dst + x + b] = (uint8_t)(w >> (8 * b));
			}
		}
}

// Record sources for serialize_run: COPY record j as (v, r, len, ADD head).
struct RecWords {   // the record arrays: W words per record, ADD head in the 4th when W >= 4
	const uint32_t* rec;
	uint32_t W;
	static constexpr bool kAlwaysHead = false;
	__device__ bool inl() const { return W >= 4; }
	__device__ void load(uint32_t j, uint32_t& v, uint32_t& r, uint32_t& l, uint32_t& w) const {
		v = rec[W * j];
		r = rec[W * j + 1];
		l = rec[W * j + 2];
		w = W >= 4 ? rec[W * j + 3] : 0u;
	}
};

// Serialises n consecutive COPY records (each preceded by the ADD of its gap)
// from `out`; prev_end = the V position the first gap starts at.  kCmd
// records per lane per tile (64 * kCmd commands per tile: fewer dependent
// load rounds).  Returns the bytes written.
// The next tile's record words are loaded behind the compiler's back and
// waited for by hand with vmcnt(kTileStores): loads and stores share the one
// vmcnt counter, which drains in issue order, so the compiler's own wait at
// the records' use (placed after this tile's stores, uncountable across the
// loop) waited for every store to land; serialize_wave_kernel 40.1 -> 35.7 us
// at C2 (profiles/r05_experiments.md).  The wait holds the registers ("+v"),
// so nothing reads them before it.  The four loads are one asm block ending in
// `s_nop 5`, the wait is `s_nop 4` + `s_waitcnt vmcnt(N)`: markers by which
// tests/test_isa_serialize.py finds both in the built code object and checks,
// over every control-flow path between them, that N is covered by the VMEM
// operations issued after the loads and that nothing touches their registers
// before the wait.
__device__ __forceinline__ void rec_load4(const uint32_t* p, const uint32_t* p3, uint32_t& a, uint32_t& b,
                                          uint32_t& c, uint32_t& d) {
	asm volatile(
	    "global_load_dword %0, %4, off\n\t"
	    "global_load_dword %1, %4, off offset:4\n\t"
	    "global_load_dword %2, %4, off offset:8\n\t"
	    "global_load_dword %3, %5, off\n\t"
	    "s_nop 5"
	    : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
	    : "v"(p), "v"(p3)
	    : "memory");
}

template <uint32_t kStageBytes, int kCmd, class Src>
__device__ inline uint64_t serialize_run(uint8_t* out, const uint8_t* V, uint32_t vl, const Src& src, uint32_t n,
                                         uint32_t prev_end, sw_lds8* stage) {
	const bool inl = src.inl();
	const uint32_t lane = lane_id();
	uint64_t pos = 0;
	// the next tile's records are loaded while this tile is assembled: their
	// latency hides under this tile's payload loads
	uint32_t ncv[kCmd], ncr[kCmd], ncl[kCmd], ncw[kCmd];
	static_assert(kCmd == 1, "one record per lane per tile (the hand-counted wait below)");
	constexpr uint32_t kTileStores = kStageBytes / 256 + 2;   // head bytes, dwords, tail bytes
	static_assert(kTileStores <= 63, "vmcnt holds 6 bits");
	constexpr bool kAsm = !Src::kAlwaysHead;
	// Records t + lane, clamped to the last record (n >= 1): every lane loads,
	// unconditionally, so the destination registers have no merge point the
	// compiler could copy them across before the hand-counted wait.  The 4th
	// word comes from word 2 when W < 4 (never read then: inl() is false).
	auto load_tile = [&](uint32_t t) {
		const uint32_t j = umin32(t + lane, n - 1);
		const uint32_t* r = src.rec + (uint64_t)src.W * j;
		rec_load4(r, r + (src.W >= 4 ? 3 : 2), ncv[0], ncr[0], ncl[0], ncw[0]);
	};
	if constexpr (kAsm) {
		if (n == 0) return 0;
		load_tile(0);
		asm volatile("s_nop 4\n\ts_waitcnt vmcnt(0)" : "+v"(ncv[0]), "+v"(ncr[0]), "+v"(ncl[0]), "+v"(ncw[0])::"memory");
	} else
#pragma unroll
	for (int i = 0; i < kCmd; ++i) {
		const uint32_t j = kCmd * lane + i;
		ncv[i] = ncr[i] = ncl[i] = ncw[i] = 0;
		if (j < n) src.load(j, ncv[i], ncr[i], ncl[i], ncw[i]);
	}
	for (uint32_t t0 = 0; t0 < n; t0 += 64 * kCmd) {
		bool valid[kCmd];
		uint32_t cv[kCmd], cr[kCmd], cl[kCmd], cw[kCmd];
#pragma unroll
		for (int i = 0; i < kCmd; ++i) {
			const uint32_t j = t0 + kCmd * lane + i;
			valid[i] = j < n;
			cv[i] = ncv[i];
			cr[i] = ncr[i];
			cl[i] = ncl[i];
			cw[i] = ncw[i];
			const uint32_t jn = j + 64 * kCmd;
			if constexpr (kAsm) continue;
			ncv[i] = ncr[i] = ncl[i] = ncw[i] = 0;
			if (jn < n) src.load(jn, ncv[i], ncr[i], ncl[i], ncw[i]);
		}
		if constexpr (kAsm) load_tile(t0 + 64);   // past the end: record n - 1 again (not used)
		// the lane's last valid command end, and the lane's byte count
		uint32_t last = 0, sz = 0;
#pragma unroll
		for (int i = 0; i < kCmd; ++i)
			if (valid[i]) last = cv[i] + cl[i];
		uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)prev_end, (int)last, 0x138, 0xF, 0xF, false);
		if (lane == 0) prev = prev_end;
		{
			uint32_t pv = prev;
#pragma unroll
			for (int i = 0; i < kCmd; ++i)
				if (valid[i]) {
					const uint32_t gap = cv[i] - pv;
					sz += 13u + (gap ? 9u + gap : 0u);
					pv = cv[i] + cl[i];
				}
		}
		const uint32_t incl = wave_incl_scan(sz);   // tile bytes < 4 GiB
		const uint32_t my = incl - sz;
		const uint32_t S = rdlane(incl, 63);
		if (S <= kStageBytes) {
			put_cmds<kCmd>(stage, valid, my, prev, cv, cr, cl, cw, inl, V, vl);
			__builtin_amdgcn_s_waitcnt(0xc07f);   // staged bytes are in LDS
			__builtin_amdgcn_wave_barrier();
			// flush: head bytes to a dword boundary, dwords, tail bytes, as
			// buffer stores of a fixed count per tile (kTileStores): lanes past
			// the end are dropped by the descriptor's size, so no store sits in
			// a branch and the next tile's record wait can count them
			uint8_t* dst = out + pos;
			const uint32_t head = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);
			{
				typedef __attribute__((address_space(3))) const uint32_t sw_lds32c;
				const uint32_t hb = umin32(head, S);
				const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)hb, 0x00020000);
				__builtin_amdgcn_raw_buffer_store_b8(stage[lane & 3u], rh, (int)lane, 0, 0);
				const uint32_t nd = S > head ? (S - head) / 4 : 0u;
				const __amdgpu_buffer_rsrc_t rd =
				    __builtin_amdgcn_make_buffer_rsrc(dst + head, (short)0, (int)(4 * nd), 0x00020000);
#pragma unroll
				for (uint32_t i = 0; i < kStageBytes / 256; ++i) {
					const uint32_t k = lane + 64 * i;
					const uint32_t o = head + 4 * k;
					const uint32_t oc = o < kStageBytes ? o : 0u;
					const sw_lds32c* w = (const sw_lds32c*)(stage + (oc & ~3u));
					__builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_alignbyte(w[1], w[0], oc & 3u), rd, (int)(4 * k), 0, 0);
				}
				const uint32_t tail0 = umin32(head + 4 * nd, S);
				const __amdgpu_buffer_rsrc_t rt =
				    __builtin_amdgcn_make_buffer_rsrc(dst + tail0, (short)0, (int)(S - tail0), 0x00020000);
				__builtin_amdgcn_raw_buffer_store_b8(stage[umin32(tail0 + (lane & 3u), kStageBytes)], rt, (int)lane, 0, 0);
			}
			__builtin_amdgcn_s_waitcnt(0xc07f);   // LDS reads done before the next tile
			__builtin_amdgcn_wave_barrier();
		} else {
			put_cmds<kCmd>(out + pos, valid, my, prev, cv, cr, cl, cw, inl, V, vl);
			// (rare: a tile over the stage) its stores drained here, so at
			// most kTileStores stores are pending at the next tile's wait
			__builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
		}
		pos += S;
		// the next tile's records: issued before this tile's kTileStores
		// buffer stores (a tile past the stage drained its stores with
		// vmcnt(0)), so vmcnt(kTileStores) covers them and no store
		if constexpr (kAsm)
			asm volatile("s_nop 4\n\ts_waitcnt vmcnt(%4)"
			             : "+v"(ncv[0]), "+v"(ncr[0]), "+v"(ncl[0]), "+v"(ncw[0])
			             : "n"(kTileStores)
			             : "memory");
		{   // lanes past the end hold last = 0: take the highest lane with a command
			const uint64_t has = __ballot(valid[0]);
			if (has) prev_end = rdlane(last, 63u - (uint32_t)__builtin_clzll(has));
		}
	}
	return pos;
}

// The delta header without its CRCs (bytes 9..24, crc_patch_kernel), lane 0
__device__ __forceinline__ void put_header(uint8_t* out, uint32_t vl) {
	if (lane_id() == 0) {
		out[0] = 'D'; out[1] = 'L'; out[2] = 'T'; out[3] = 3;
		out[4] = 0;   // standard delta
		be32_store(out + 5, vl);
	}
}

// The trailing ADD of V[from, vl) (src/c/onepass.c:268-275) and END; returns
// the bytes written.
__device__ __forceinline__ uint64_t put_tail(uint8_t* out, const uint8_t* V, uint32_t vl, uint32_t from) {
	const uint32_t lane = lane_id();
	uint64_t pos = 0;
	if (from < vl) {
		const uint32_t len = vl - from;
		if (lane == 0) {
			out[0] = 2;
			be32_store(out + 1, from);
			be32_store(out + 5, len);
		}
		for (uint32_t i = lane; i < len; i += 64) out[9 + i] = V[from + i];
		pos = 9 + len;
	}
	if (lane == 0) out[pos] = 0;   // END
	return pos + 1;
}

// Wave-wide serialisation of one pair.  `out` = the pair's first output
// byte, `size` = its delta size (as accumulated by the differencing), `rec`
// its COPY records (v, r, len) in V order, `stage` >= kStageBytes of LDS.
// Returns 0, or 12 (DG_ERR_INTERNAL) when the bytes written disagree with `size`.
template <uint32_t kStageBytes, int kCmd = 1>
__device__ inline int32_t serialize_wave(uint8_t* out, uint64_t size, const uint8_t* V, uint32_t vl,
                                         const uint32_t* rec, uint32_t W, uint32_t n, sw_lds8* stage) {
	put_header(out, vl);
	uint64_t pos = 25;
	const RecWords src{rec, W};
	pos += serialize_run<kStageBytes, kCmd>(out + pos, V, vl, src, n, 0u, stage);
	// the end of the last COPY
	uint32_t prev_end = 0;
	if (n) {
		const uint32_t* r = rec + (uint64_t)W * (n - 1);
		prev_end = r[0] + r[2];
	}
	pos += put_tail(out + pos, V, vl, prev_end);
	return pos == size ? 0 : 12;   // DG_ERR_INTERNAL
}

}  // namespace dg
