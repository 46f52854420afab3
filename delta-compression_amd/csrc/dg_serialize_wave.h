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

// One command per lane: the ADD of the gap before record (v, r, len) and the
// COPY, written back to back from base + my; prev = where the gap starts.
// The gap's payload comes from the record's head word (gaps up to 4 bytes,
// onepass records) or, up to 32 bytes, from pay(prev, w): the 8 words
// V[prev .. prev + 32) (loaded there, or a tile ahead by the pipeline);
// longer gaps are copied by the whole wave afterwards, straight from V.
template <typename P, typename Pay>
__device__ __forceinline__ void put_cmds(P base, bool valid, uint32_t my, uint32_t prev, uint32_t cv, uint32_t cr,
                                         uint32_t cl, uint32_t cw, bool inl, const Pay& pay, const uint8_t* V,
                                         uint32_t vl) {
	const uint32_t lane = lane_id();
	bool big = false;
	uint32_t bsrc = 0, blen = 0, bdst = 0;
	if (valid) {
		const uint32_t gap = cv - prev;
		P q = base + my;
		if (gap) {
			q[0] = 2;
			be32_store(q + 1, prev);
			be32_store(q + 5, gap);
			if (inl && gap <= 4) {   // payload carried in the record
				for (uint32_t k = 0; k < gap; ++k) q[9 + k] = (uint8_t)(cw >> (8 * k));
			} else if (gap <= 32) {
				uint32_t wd[8];
				pay(prev, wd);
#pragma unroll
				for (int k = 0; k < 32; ++k)
					if ((uint32_t)k < gap) q[9 + k] = (uint8_t)(wd[k >> 2] >> (8 * (k & 3)));
			} else {
				big = true;
				bsrc = prev;
				blen = gap;
				bdst = my + 9;
			}
			q += 9 + gap;
		}
		q[0] = 1;
		be32_store(q + 1, cr);
		be32_store(q + 5, cv);
		be32_store(q + 9, cl);
	}
	// long payloads: the whole wave, 4 bytes per lane per pass (unaligned
	// dword loads, never past the end of V)
	for (uint64_t bm = __ballot(big); bm; bm &= bm - 1) {
		const uint32_t k = ffs64(bm);
		const uint32_t src = rdlane(bsrc, k), len = rdlane(blen, k), dst = rdlane(bdst, k);
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

// The 8 words V[from .. from + 32) of a lane's ADD gap (5..32 bytes, so
// |V| >= 5), as unaligned dword loads issued unconditionally (a per-word
// condition made the compiler branch around each load and wait for it, and
// for every store before it: up to 8 dependent round trips per tile), at
// addresses clamped inside V: a word that crosses |V| is loaded from |V| - 4
// and shifted down, a word past |V| is never used.
__device__ __forceinline__ void pay_words(const uint8_t* V, uint32_t vl, uint32_t from, uint32_t (&w)[8]) {
	const uint32_t vl4 = vl - 4u;
#pragma unroll
	for (int k = 0; k < 8; ++k) {
		const uint32_t o4 = from + 4u * k;
		const uint32_t a4 = umin32(o4, vl4);
		uint32_t x;
		__builtin_memcpy(&x, V + a4, 4);
		w[k] = x >> (8u * umin32(o4 - a4, 3u));
	}
}

// Record sources for serialize_run: W words per record (v, r, len[, ADD head]).
struct RecWords {   // the record arrays: W words per record, ADD head in the 4th when W >= 4
	const uint32_t* rec;
	uint32_t W;
	__device__ bool inl() const { return W >= 4; }
};

// Serialises n consecutive COPY records (each preceded by the ADD of its gap)
// from `out`; prev_end = the V position the first gap starts at.  One record
// per lane per tile of 64.  Returns the bytes written.
// The next tile's record words are loaded behind the compiler's back and
// waited for by hand with vmcnt(kTileStores): loads and stores share the one
// vmcnt counter, which drains in issue order, so the compiler's own wait at
// the records' use (placed after this tile's stores, uncountable across the
// loop) waited for every store to land; serialize_wave_kernel 40.1 -> 35.7 us
// at C2 (profiles/r05_experiments.md).  The wait holds the registers ("+v"),
// so nothing reads them before it.  The four loads are one asm block ending in
// `s_nop 7; s_nop 4`, the wait is `s_nop 7; s_nop 5` + `s_waitcnt vmcnt(N)`:
// markers by which tests/test_isa_serialize.py finds both in the built code
// object and checks, over every control-flow path between them, that N is
// covered by the VMEM operations issued after the loads and that nothing
// touches their registers before the wait.  (Round 6 tried the compiler's own
// waits, with the payload words loaded a tile ahead: C2's serialiser 37.7 ->
// 63.7 us; and an LDS-DMA pipeline, serialize_pipe below: 74.9 us.)
__device__ __forceinline__ void rec_load4(const uint32_t* p, const uint32_t* p3, uint32_t& a, uint32_t& b,
                                          uint32_t& c, uint32_t& d) {
	asm volatile(
	    "global_load_dword %0, %4, off\n\t"
	    "global_load_dword %1, %4, off offset:4\n\t"
	    "global_load_dword %2, %4, off offset:8\n\t"
	    "global_load_dword %3, %5, off\n\t"
	    "s_nop 7\n\t"
	    "s_nop 4"
	    : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
	    : "v"(p), "v"(p3)
	    : "memory");
}

template <uint32_t kStageBytes, class Src>
__device__ inline uint64_t serialize_run(uint8_t* out, const uint8_t* V, uint32_t vl, const Src& src, uint32_t n,
                                         uint32_t prev_end, sw_lds8* stage) {
	if (n == 0) return 0;
	const bool inl = src.inl();
	const uint32_t lane = lane_id();
	uint64_t pos = 0;
	constexpr uint32_t kTileStores = kStageBytes / 256 + 2;   // head bytes, dwords, tail bytes
	static_assert(kTileStores <= 63, "vmcnt holds 6 bits");
	auto pay = [&](uint32_t from, uint32_t (&w)[8]) { pay_words(V, vl, from, w); };
	// the next tile's records are loaded while this tile is assembled: their
	// latency hides under this tile's payload loads.  Records t + lane,
	// clamped to the last record (n >= 1): every lane loads, unconditionally,
	// so the destination registers have no merge point the compiler could copy
	// them across before the hand-counted wait.  The 4th word comes from word
	// 2 when W < 4 (never read then: inl() is false).
	uint32_t ncv, ncr, ncl, ncw;
	auto load_tile = [&](uint32_t t) {
		const uint32_t j = umin32(t + lane, n - 1);
		const uint32_t* r = src.rec + (uint64_t)src.W * j;
		rec_load4(r, r + (src.W >= 4 ? 3 : 2), ncv, ncr, ncl, ncw);
	};
	load_tile(0);
	asm volatile("s_nop 7\n\ts_nop 5\n\ts_waitcnt vmcnt(0)" : "+v"(ncv), "+v"(ncr), "+v"(ncl), "+v"(ncw)::"memory");
	for (uint32_t t0 = 0; t0 < n; t0 += 64) {
		const bool valid = t0 + lane < n;
		const uint32_t cv = ncv, cr = ncr, cl = ncl, cw = ncw;
		load_tile(t0 + 64);   // past the end: record n - 1 again (not used)
		// the lane's command end, and the lane's byte count
		const uint32_t last = valid ? cv + cl : 0u;
		uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)prev_end, (int)last, 0x138, 0xF, 0xF, false);
		if (lane == 0) prev = prev_end;
		const uint32_t gap = cv - prev;
		const uint32_t sz = valid ? 13u + (gap ? 9u + gap : 0u) : 0u;
		const uint32_t incl = wave_incl_scan(sz);   // tile bytes < 4 GiB
		const uint32_t my = incl - sz;
		const uint32_t S = rdlane(incl, 63);
		if (S <= kStageBytes) {
			put_cmds(stage, valid, my, prev, cv, cr, cl, cw, inl, pay, V, vl);
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
			put_cmds(out + pos, valid, my, prev, cv, cr, cl, cw, inl, pay, V, vl);
			// (rare: a tile over the stage) its stores drained here, so at
			// most kTileStores stores are pending at the next tile's wait
			__builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
		}
		pos += S;
		// the next tile's records: issued before this tile's kTileStores
		// buffer stores (a tile past the stage drained its stores with
		// vmcnt(0)), so vmcnt(kTileStores) covers them and no store
		asm volatile("s_nop 7\n\ts_nop 5\n\ts_waitcnt vmcnt(%4)"
		             : "+v"(ncv), "+v"(ncr), "+v"(ncl), "+v"(ncw)
		             : "n"(kTileStores)
		             : "memory");
		{   // lanes past the end hold last = 0: take the highest lane with a command
			const uint64_t has = __ballot(valid);
			if (has) prev_end = rdlane(last, 63u - (uint32_t)__builtin_clzll(has));
		}
	}
	return pos;
}

// ── the wave-per-pair serialiser's pipeline (A/B: DG_SER_PIPE=1) ──
//
// Measured slower than serialize_run at C2 (serialize_wave_kernel 37.7 ->
// 74.9 us, profiles/r06_experiments.md; why is not established: its stage is
// 2 KiB, the rings taking the rest of the LDS).  Kept as a compile-time switch.
//
// serialize_run above waits, in every tile, for the tile's ADD payload words
// and (one tile ahead) its records; loads and stores share the one vmcnt
// counter, which drains in issue order, so a load issued after a tile's
// stores cannot be waited for without waiting for those stores too.  Here
// every load a tile needs is issued before the previous tile's stores, by
// LDS-DMA into rings (so no register holds a load in flight across the loop):
//   records  3 slots of 64 x 16 B (word-major; 12 B correcting records), tile t + 2
//            loaded while tile t is assembled;
//   payload  2 slots of 8 x 64 dwords: the words V[from .. from + 32) of
//            each lane's gap in tile t + 1 (clamped inside V), loaded while
//            tile t is assembled;
// and each tile's flush is a fixed kTileStores buffer stores, so one
// hand-counted s_waitcnt vmcnt(kTileStores) at the top of the next tile
// covers both (tests/test_isa_serialize.py checks the count on every path).
constexpr uint32_t kPipeRecSlot = 1024, kPipePaySlot = 2048;
template <uint32_t kStageBytes>
constexpr uint32_t pipe_lds_bytes() { return kStageBytes + 32 + 3 * kPipeRecSlot + 2 * kPipePaySlot; }

template <uint32_t kStageBytes>
__device__ inline uint64_t serialize_pipe(uint8_t* out, const uint8_t* V, uint32_t vl, const uint32_t* rec,
                                          uint32_t W, uint32_t n, uint32_t prev_end, sw_lds8* lds) {
	typedef __attribute__((address_space(3))) void sp_lds_void;
	typedef __attribute__((address_space(3))) const uint32_t sp_lds32c;
	if (n == 0) return 0;
	constexpr uint32_t kTileStores = kStageBytes / 256 + 2;   // head bytes, dwords, tail bytes
	static_assert(kTileStores <= 63, "vmcnt holds 6 bits");
	const uint32_t lane = lane_id();
	const bool inl = W >= 4;
	sw_lds8* stage = lds;
	sw_lds8* rring = lds + kStageBytes + 32;
	sw_lds8* pring = rring + 3 * kPipeRecSlot;
	const uint32_t nt = (n + 63) / 64;
	// tile t's records (clamped) into slot t % 3, word k of every lane's
	// record by the k-th DMA (word-major: [k][lane]); W = 3 or 4 DMAs
	auto rec_dma = [&](uint32_t t) {
		const uint32_t* p = rec + (uint64_t)W * umin32(64u * t + lane, n - 1);
		sw_lds8* d = rring + kPipeRecSlot * (t % 3u);
		__builtin_amdgcn_global_load_lds((const void*)p, (sp_lds_void*)d, 4, 0, 0);
		__builtin_amdgcn_global_load_lds((const void*)(p + 1), (sp_lds_void*)(d + 256), 4, 0, 0);
		__builtin_amdgcn_global_load_lds((const void*)(p + 2), (sp_lds_void*)(d + 512), 4, 0, 0);
		if (W >= 4) __builtin_amdgcn_global_load_lds((const void*)(p + 3), (sp_lds_void*)(d + 768), 4, 0, 0);
	};
	auto rec_read = [&](uint32_t t, uint32_t (&r)[4]) {
		const sp_lds32c* p = (const sp_lds32c*)(rring + kPipeRecSlot * (t % 3u) + 4u * lane);
		r[0] = p[0];
		r[1] = p[64];
		r[2] = p[128];
		r[3] = inl ? p[192] : 0u;
	};
	// eight DMAs: the lane's gap words into slot t % 2 (word k at 256 k + 4 lane);
	// |V| < 4 reads a dummy source (the record) and takes the bytes at use
	auto pay_dma = [&](uint32_t t, uint32_t from) {
		sw_lds8* d = pring + kPipePaySlot * (t & 1u);
		const bool ok = vl >= 4;
		const uint8_t* src = ok ? V : (const uint8_t*)rec;
		const uint32_t vl4 = ok ? vl - 4u : 0u;
#pragma unroll
		for (uint32_t k = 0; k < 8; ++k)
			__builtin_amdgcn_global_load_lds((const void*)(src + (ok ? umin32(from + 4u * k, vl4) : 0u)),
			                                 (sp_lds_void*)(d + 256u * k), 4, 0, 0);
	};
	auto pay_read = [&](uint32_t t, uint32_t from, uint32_t (&w)[8]) {
		if (vl >= 4) {
			const sp_lds32c* p = (const sp_lds32c*)(pring + kPipePaySlot * (t & 1u) + 4u * lane);
			const uint32_t vl4 = vl - 4u;
#pragma unroll
			for (uint32_t k = 0; k < 8; ++k) {
				const uint32_t o4 = from + 4u * k;
				w[k] = p[64u * k] >> (8u * umin32(o4 - umin32(o4, vl4), 3u));
			}
		} else {
#pragma unroll
			for (uint32_t k = 0; k < 8; ++k) {
				w[k] = 0;
				for (uint32_t b = 0; b < 4; ++b)
					if (from + 4u * k + b < vl) w[k] |= (uint32_t)V[from + 4u * k + b] << (8 * b);
			}
		}
	};
	auto gap_from = [&](const uint32_t (&r)[4], uint32_t before) {
		uint32_t pv = (uint32_t)__builtin_amdgcn_update_dpp((int)before, (int)(r[0] + r[2]), 0x138, 0xF, 0xF, false);
		if (lane == 0) pv = before;
		return pv;
	};
	// prologue: tiles 0 and 1's records, tile 0's payload words
	rec_dma(0);
	if (nt > 1) rec_dma(1);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	uint32_t rc[4];
	rec_read(0, rc);
	uint32_t from_c = gap_from(rc, prev_end);
	pay_dma(0, from_c);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (no stores follow them yet)
	uint64_t pos = 0;
	for (uint32_t t = 0; t < nt; ++t) {
		// tile t + 1's records and tile t's payload words have landed: only
		// tile t - 1's kTileStores stores were issued after them
		asm volatile("s_nop 7\n\ts_nop 5\n\ts_waitcnt vmcnt(%0)" ::"n"(kTileStores) : "memory");
		if (t) rec_read(t, rc);
		const bool valid = 64u * t + lane < n;
		uint32_t from_n = 0;
		if (t + 1 < nt) {   // (tile t is full)
			uint32_t rn[4];
			rec_read(t + 1, rn);
			from_n = gap_from(rn, rdlane(rc[0] + rc[2], 63));
			pay_dma(t + 1, from_n);
			if (t + 2 < nt) rec_dma(t + 2);
			asm volatile("s_nop 7\n\ts_nop 6" ::: "memory");   // (the ISA check's marker: DMAs above)
		}
		uint32_t pc[8];
		pay_read(t, from_c, pc);
		auto pay = [&](uint32_t, uint32_t (&w)[8]) {
#pragma unroll
			for (int k = 0; k < 8; ++k) w[k] = pc[k];
		};
		const uint32_t gap = rc[0] - from_c;
		const uint32_t sz = valid ? 13u + (gap ? 9u + gap : 0u) : 0u;
		const uint32_t incl = wave_incl_scan(sz);   // tile bytes < 4 GiB
		const uint32_t my = incl - sz;
		const uint32_t S = rdlane(incl, 63);
		if (S <= kStageBytes) {
			put_cmds(stage, valid, my, from_c, rc[0], rc[1], rc[2], rc[3], inl, pay, V, vl);
			__builtin_amdgcn_s_waitcnt(0xc07f);   // staged bytes are in LDS
			__builtin_amdgcn_wave_barrier();
			uint8_t* dst = out + pos;
			const uint32_t head = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);
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
				const sp_lds32c* w = (const sp_lds32c*)(stage + (oc & ~3u));
				__builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_alignbyte(w[1], w[0], oc & 3u), rd, (int)(4 * k), 0, 0);
			}
			const uint32_t tail0 = umin32(head + 4 * nd, S);
			const __amdgpu_buffer_rsrc_t rt =
			    __builtin_amdgcn_make_buffer_rsrc(dst + tail0, (short)0, (int)(S - tail0), 0x00020000);
			__builtin_amdgcn_raw_buffer_store_b8(stage[umin32(tail0 + (lane & 3u), kStageBytes)], rt, (int)lane, 0, 0);
			__builtin_amdgcn_s_waitcnt(0xc07f);   // LDS reads done before the next tile
			__builtin_amdgcn_wave_barrier();
		} else {
			// (rare: a tile over the stage) written in place; its stores are
			// drained here, so the next tile's counted wait still covers its loads
			put_cmds(out + pos, valid, my, from_c, rc[0], rc[1], rc[2], rc[3], inl, pay, V, vl);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
		pos += S;
		from_c = from_n;
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the loop
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
template <uint32_t kStageBytes, bool kPipe = false>
__device__ inline int32_t serialize_wave(uint8_t* out, uint64_t size, const uint8_t* V, uint32_t vl,
                                         const uint32_t* rec, uint32_t W, uint32_t n, sw_lds8* stage) {
	put_header(out, vl);
	uint64_t pos = 25;
	if constexpr (kPipe) {
		pos += serialize_pipe<kStageBytes>(out + pos, V, vl, rec, W, n, 0u, stage);
	} else {
		const RecWords src{rec, W};
		pos += serialize_run<kStageBytes>(out + pos, V, vl, src, n, 0u, stage);
	}
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
