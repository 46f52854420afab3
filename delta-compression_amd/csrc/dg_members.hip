// dg_members.hip — onepass as verified diagonal members (gfx950).
//
// The reference's onepass (src/c/onepass.c:32-297) is a serial chain of
// epochs: every match bumps the table version (:263), so an epoch is fully
// described by its start (v0, r0).  On data whose matches lie on diagonal 0
// (V[x] vs R[x]: substitution edits, the C2/C3 workloads) the chain is a
// function of the mismatch positions alone — group the mismatches (with a
// virtual one at -1 and the end E = min(|R|, |V|) as a sentinel) into runs
// separated by gaps > p; member k starts its epoch at s_k (0, then the first
// mismatch of run k), first sees equal windows at x_k = last mismatch of run
// k + 1, matches there (lookup 1 or 2 finds step x_k - s_k itself) and extends
// to s_{k+1} — provided its lookups behave as on random data.  That proviso
// is checked per member, independently, so the chain is verified in parallel
// instead of walked.
//
// member_chunk_kernel: one wave per 2 KiB chunk of a pair.  Both streams'
// bytes [chunk - 16, chunk + 2 KiB + 1 KiB) go to LDS by LDS-DMA (one HBM
// round trip, coalesced 16 B per lane); the wave
//   * builds the chunk's mismatch bitmap, the run starts (no mismatch in the
//     16 bytes before) and, for each run starting in the chunk (a member),
//     its end x = last mismatch before the next run start + 1 and that next
//     start — members whose next start lies past the look-ahead are left
//     unverified;
//   * packs the members' steps over the 64 lanes (lane = step), fingerprints
//     both windows of every step from LDS, and passes a member when
//       (A) no V window of a step equals (low 32 fingerprint bits) an R
//           window of another step of the member — no lookup before T can
//           verify (:169-219), and
//       (B) at T = x - s, slot_V(T) is not among slot_V(0..T-1) or slot_R(T)
//           is not among slot_R(0..T-1) — step T is the first writer its
//           lookup 1 or lookup 2 finds (:141-166);
//   * writes each member's start and its COPY record (x, x, next - x, first
//     4 bytes of its ADD) with the verdict into the chunk's slots.
//
// The per-pair chain (onepass16_kernel in member mode, dg_onepass.hip) then
// takes verified members as they are and runs the exact epoch machinery only
// from an unverified member until the chain lands on a later member start,
// and for the final epoch (the run holding the sentinel is never closed).
// oracle/spec_model.c is the CPU model of exactly these decisions
// (tests/test_spec_model.py checks it against the oracle).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dg_device.h"
#include "dg_devutil.h"
#include "dg_serialize_wave.h"

namespace dg {

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr uint32_t kStage = kMemChunk + kMemAhead + 16;   // staged bytes per stream (lookbehind 16)
constexpr uint32_t kMaskWords = (kStage + 31) / 32;        // mismatch bitmap words
constexpr uint32_t kRunList = kStage / 17 + 4;             // run starts in the staged region (>= 17 apart)
constexpr uint32_t kLongChunks = 8;
#ifndef DG_MEM_WAVES
#define DG_MEM_WAVES 7   // minimum waves per SIMD the register budget must allow
#endif                    // persistent waves (LDS allows 17)                        // members of up to 512 steps are verified
static_assert(kStage % 16 == 0, "16-byte blocks");

// Profiling build (DG_LIB_VARIANT=prof, scripts/member_phases.py): per-phase
// shader-clock cycles and counts of member_chunk_kernel, summed over waves
#ifdef DG_ONEPASS_PROF
enum : int { MP_STAGE, MP_MASK, MP_RUNS, MP_SNLAST, MP_SETUP, MP_SHORT, MP_LONG, MP_PREFIX, MP_TOTAL, MP_CHUNKS,
             MP_MEMBERS, MP_SHORT_N, MP_LONG_N, MP_ROUNDS, MP_UNVER, MP_FLAGGED, MP_D1, kMemProfN };
constexpr uint32_t kMemProfSlots = 256;   // spread: one set of counters per blockIdx % 256
__device__ unsigned long long g_member_prof[kMemProfSlots * kMemProfN];
struct MemProf {
	uint64_t v[kMemProfN] = {};
};
#define MPROF_T(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define MPROF_ADD(k, t) mp.v[k] += __builtin_amdgcn_s_memtime() - (t)
#define MPROF_INC(k, n) mp.v[k] += (n)
#else
struct MemProf {};
#define MPROF_T(t)
#define MPROF_ADD(k, t)
#define MPROF_INC(k, n)
#endif

// 16 mismatch bits of 16 bytes (bit i: byte i of the chunk differs)
__device__ __forceinline__ uint32_t mismatch16(const uint4& v, const uint4& r) {
	const uint32_t x[4] = {v.x ^ r.x, v.y ^ r.y, v.z ^ r.z, v.w ^ r.w};
	uint32_t m = 0;
#pragma unroll
	for (int d = 0; d < 4; ++d) {
		const uint32_t t = (((x[d] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x[d]) & 0x80808080u;
		const uint32_t b = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
		m |= b << (4 * d);
	}
	return m;
}

__device__ __forceinline__ uint64_t lanes_mask(uint32_t first, uint32_t n) {   // lanes [first, first + n), n >= 1
	return (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << first;
}

__device__ __forceinline__ void lds_fence() {
	__builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
	__builtin_amdgcn_wave_barrier();
}

// Bloom filter of the V window hashes of a member set's steps other than
// their T steps.  Check (A) splits by whether a pair of steps involves T:
// V(T) == R(T) by construction (no mismatch in [x, x + 16)), so V(c) == R(T)
// is V(c) == V(T) and V(T) == R(l) is R(T) == R(l), both plain ballots at T;
// the other pairs (c, l != T) can exist only for an R hash in the filter, and
// those rare flagged steps are resolved exactly with ballots.
// Probes: the hash's low bits, and a 24x24 multiplicative mix of its bits
// 8..31 (v_mul_u32_u24, full rate, instead of the quarter-rate v_mul_lo_u32):
// between them every hash bit reaches a probe, so the V and R windows of one
// step, whose hashes differ in the few bits a mismatched byte flips, do not
// share both probes.
template <uint32_t W>
struct VFilter {
	static constexpr uint32_t kLg = W == 64 ? 11u : (W == 128 ? 12u : 13u);
	uint32_t* f;   // W words
	__device__ void clear() {
		for (uint32_t i = lane_id(); i < W; i += 64) f[i] = 0u;
	}
	__device__ static uint32_t h2(uint32_t h) {
		// (HIP's __umul24 returns int: shift the product as unsigned)
		return (uint32_t)__umul24(__builtin_amdgcn_alignbit(h, h, 8), 0x9E3779u) >> (32u - kLg);
	}
	__device__ void add(uint32_t h) {
		const uint32_t a = h & (32u * W - 1u), b = h2(h);
		atomicOr(&f[a >> 5], 1u << (a & 31u));
		atomicOr(&f[b >> 5], 1u << (b & 31u));
	}
	__device__ bool has(uint32_t h) const {
		const uint32_t a = h & (32u * W - 1u), b = h2(h);
		return ((f[a >> 5] >> (a & 31u)) & (f[b >> 5] >> (b & 31u)) & 1u) != 0u;
	}
};

// Intra-wave LDS hand-offs (lane A stores, lane B loads) need only program
// order: a wave's LDS instructions execute in issue order, so a compiler
// barrier replaces s_waitcnt + wave_barrier.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

struct ChunkLds {
	uint8_t v[kStage + 16];   // + slack: the fifth dword of a window read
	uint8_t r[kStage + 16];
	uint32_t mask[kMaskWords];
	uint16_t last[kMaskWords];   // max mismatch offset + 1 over words <= j (0: none)
	uint16_t run[kRunList];      // run starts (offsets), ascending
	uint8_t mark[64];
	uint32_t filt[64];           // V-hash filter of a round or a long member
};

// the 16 bytes at offset o of a staged stream (s 16-byte aligned): five
// aligned dwords and four funnel shifts.  gfx950 accepts an unaligned
// ds_read_b128, but it stalls the LDS pipe: on C3 SQ_LDS_UNALIGNED_STALL was
// 61 % of the member kernel's LDS-active cycles (profiles/r05_member_census.md).
__device__ __forceinline__ uint4 lds16(const uint8_t* s, uint32_t o) {
#ifdef DG_LDS16_UNALIGNED   // A/B variant: the unaligned ds_read_b128
	uint4 w;
	__builtin_memcpy(&w, s + o, 16);
	return w;
#endif
	const uint32_t* d = reinterpret_cast<const uint32_t*>(s + (o & ~3u));
	const uint32_t sh = (o & 3u) * 8u;
	const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
	return make_uint4(__builtin_amdgcn_alignbit(d1, d0, sh), __builtin_amdgcn_alignbit(d2, d1, sh),
	                  __builtin_amdgcn_alignbit(d3, d2, sh), __builtin_amdgcn_alignbit(d4, d3, sh));
}

// An equality-preserving 32-bit hash of a window for check (A): only byte-
// equal windows can make a lookup verify (memcmp, onepass.c:186,212), so
// equal windows must hash equal; unequal ones that collide only make the
// check conservative.  Six VALU ops instead of a second fingerprint.
__device__ __forceinline__ uint32_t win_hash(const uint4& w) {
	return w.x ^ __builtin_amdgcn_alignbit(w.y, w.y, 27) ^ __builtin_amdgcn_alignbit(w.z, w.z, 21) ^
	       __builtin_amdgcn_alignbit(w.w, w.w, 15);
}

__device__ __forceinline__ uint32_t slot_lds(const uint8_t* s, uint32_t o, const ModQ& mq, uint64_t q, uint64_t qmag) {
	const uint4 w = lds16(s, o);
	return slot_of(fp16_dot(w.x, w.y, w.z, w.w), mq, q, qmag);
}

// lanes [a, b) (a <= b <= 64)
__device__ __forceinline__ uint64_t lanes_range(uint32_t a, uint32_t b) {
	const uint64_t hi = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
	return hi & ~((1ull << a) - 1ull);
}

// One long member (64 <= T < 64 kLongChunks) at staged offset s0: 64 steps
// per lane row, history in VGPRs, W-word filters.  Returns its verdict.
template <uint32_t W>
__device__ __forceinline__ bool long_member_ok(const uint8_t* SV, const uint8_t* SR, uint32_t s0, uint32_t tl,
                                               uint32_t* filt, const ModQ& mq, uint64_t q, uint64_t qmag,
                                               uint32_t& pw) {
	const uint32_t lane = lane_id();
	const uint32_t C = tl / 64 + 1, CT = tl / 64, LT = tl % 64;
	VFilter<W> fl{filt};
	uint32_t hsV[kLongChunks], hfV[kLongChunks], hfR[kLongChunks];   // V slots, V / R window hashes
	lds_order();
	fl.clear();
	lds_order();
	pw = 0;
#pragma unroll
	for (uint32_t cc = 0; cc < kLongChunks; ++cc) {
		hsV[cc] = kSentinel;
		hfV[cc] = 0u;
		hfR[cc] = 1u;
		const uint32_t t = 64 * cc + lane;
		if (cc < C && t <= tl) {
			const uint4 wv = lds16(SV, s0 + t), wr = lds16(SR, s0 + t);
			hsV[cc] = slot_of(fp16_dot(wv.x, wv.y, wv.z, wv.w), mq, q, qmag);
			hfV[cc] = win_hash(wv);
			hfR[cc] = win_hash(wr);
			if (cc == 0) pw = wv.x;
			if (t != tl) fl.add(hfV[cc]);
		}
	}
	pw = rdlane(pw, 0);
	lds_order();
	bool bad = false;
	// (A) through T: V(c) == V(T) or R(l) == R(T) for a step before T
	uint32_t hT = 0, vT = 0;
#pragma unroll
	for (uint32_t cc = 0; cc < kLongChunks; ++cc)
		if (cc == CT) {
			hT = rdlane(hfV[cc], LT);
			vT = rdlane(hsV[cc], LT);
		}
#pragma unroll
	for (uint32_t c2 = 0; c2 < kLongChunks; ++c2)
		if (c2 <= CT)
			bad = bad || (__ballot(hfV[c2] == hT || hfR[c2] == hT) & (c2 < CT ? ~0ull : lanes_range(0, LT))) != 0;
	// (A) off T: flagged steps' R hashes against every other step's V hash
#pragma unroll
	for (uint32_t cc = 0; cc < kLongChunks; ++cc) {
		if (cc < C) {
			const uint32_t t = 64 * cc + lane;
			for (uint64_t w = __ballot(t < tl && fl.has(hfR[cc])); w && !bad; w &= w - 1) {
				const uint32_t Lx = ffs64(w);
				const uint32_t fR = rdlane(hfR[cc], Lx);
#pragma unroll
				for (uint32_t c2 = 0; c2 < kLongChunks; ++c2) {
					if (c2 < C) {
						const bool other = 64 * c2 + lane <= tl && !(c2 == cc && lane == Lx);
						if (__ballot(other && hfV[c2] == fR)) bad = true;
					}
				}
			}
		}
	}
	if (bad) return false;
	// (B): the T step's V slot against the earlier V slots; R slots only when
	// it repeats
	bool d1 = false;
#pragma unroll
	for (uint32_t c2 = 0; c2 < kLongChunks; ++c2)
		if (c2 <= CT) d1 = d1 || (__ballot(hsV[c2] == vT) & (c2 < CT ? ~0ull : lanes_range(0, LT))) != 0;
	if (!d1) return true;
	const uint32_t rT = slot_lds(SR, s0 + tl, mq, q, qmag);
	bool d2 = false;
	for (uint32_t c2 = 0; c2 <= CT; ++c2) {
		const uint32_t t2 = 64 * c2 + lane;
		const uint32_t sr2 = t2 < tl ? slot_lds(SR, s0 + t2, mq, q, qmag) : kSentinel;
		d2 = d2 || __ballot(t2 < tl && sr2 == rT) != 0;
	}
	return !d2;
}

// long_member_ok for a member of exactly K rows (64 (K - 1) <= T < 64 K):
// the row count is a compile-time constant, so none of the per-row uniform
// predicates remain (88 % of C3's long members have K = 2, 11 % K = 3).
template <uint32_t W, uint32_t K>
__device__ __forceinline__ bool long_member_rows(const uint8_t* SV, const uint8_t* SR, uint32_t s0, uint32_t tl,
                                                 uint32_t* filt, const ModQ& mq, uint64_t q, uint64_t qmag,
                                                 uint32_t& pw) {
	const uint32_t lane = lane_id();
	constexpr uint32_t CT = K - 1;
	const uint32_t LT = tl % 64;
	VFilter<W> fl{filt};
	uint32_t hsV[K], hfV[K], hfR[K];   // V slots, V / R window hashes
	lds_order();
	fl.clear();
	lds_order();
#pragma unroll
	for (uint32_t cc = 0; cc < K; ++cc) {
		hsV[cc] = kSentinel;
		hfV[cc] = 0u;
		hfR[cc] = 1u;
		const uint32_t t = 64 * cc + lane;
		if (cc < CT || t <= tl) {
			const uint4 wv = lds16(SV, s0 + t), wr = lds16(SR, s0 + t);
			hsV[cc] = slot_of(fp16_dot(wv.x, wv.y, wv.z, wv.w), mq, q, qmag);
			hfV[cc] = win_hash(wv);
			hfR[cc] = win_hash(wr);
			if (cc == 0) pw = wv.x;
			if (t != tl) fl.add(hfV[cc]);
		}
	}
	pw = rdlane(pw, 0);
	lds_order();
	// (A) through T: V(c) == V(T) or R(l) == R(T) for a step before T
	const uint32_t hT = rdlane(hfV[CT], LT), vT = rdlane(hsV[CT], LT);
	bool bad = false;
#pragma unroll
	for (uint32_t c2 = 0; c2 < K; ++c2)
		bad = bad || (__ballot(hfV[c2] == hT || hfR[c2] == hT) & (c2 < CT ? ~0ull : lanes_range(0, LT))) != 0;
	// (A) off T: flagged steps' R hashes against every other step's V hash
#pragma unroll
	for (uint32_t cc = 0; cc < K; ++cc) {
		const uint32_t t = 64 * cc + lane;
		for (uint64_t w = __ballot(t < tl && fl.has(hfR[cc])); w && !bad; w &= w - 1) {
			const uint32_t Lx = ffs64(w);
			const uint32_t fR = rdlane(hfR[cc], Lx);
#pragma unroll
			for (uint32_t c2 = 0; c2 < K; ++c2) {
				const bool other = 64 * c2 + lane <= tl && !(c2 == cc && lane == Lx);
				if (__ballot(other && hfV[c2] == fR)) bad = true;
			}
		}
	}
	if (bad) return false;
	// (B): the T step's V slot against the earlier V slots; R slots only when
	// it repeats
	bool d1 = false;
#pragma unroll
	for (uint32_t c2 = 0; c2 < K; ++c2)
		d1 = d1 || (__ballot(hsV[c2] == vT) & (c2 < CT ? ~0ull : lanes_range(0, LT))) != 0;
	if (!d1) return true;
	const uint32_t rT = slot_lds(SR, s0 + tl, mq, q, qmag);
	bool d2 = false;
	for (uint32_t c2 = 0; c2 <= CT; ++c2) {
		const uint32_t t2 = 64 * c2 + lane;
		const uint32_t sr2 = t2 < tl ? slot_lds(SR, s0 + t2, mq, q, qmag) : kSentinel;
		d2 = d2 || __ballot(t2 < tl && sr2 == rT) != 0;
	}
	return !d2;
}

// the staged region of one chunk in VGPRs (16 bytes per lane per row), loaded
// while the previous chunk is verified
constexpr uint32_t kStageRows = (kStage + 1023) / 1024;   // rows of 64 x 16 B (the last one partial)
struct StageRegs {
	uint4 v[kStageRows], r[kStageRows];
};

// A wave's walk over its contiguous run of (pair, chunk) jobs: the jobs are
// laid out pair after pair, chunk after chunk, so the next job follows from
// this one and only a new pair's descriptors are loaded (wave-uniform).
struct JobCursor {
	uint32_t pair, c, n_chunks, chunk_base;
	uint32_t vl, rl;
	uint64_t v_off, r_off, mem_base, q, q_magic, rec_base;
	template <class Args>
	__device__ void load_pair(const Args& a) {
		// (wave-uniform: into SGPRs, so the member kernel's 72-VGPR budget
		// holds no 64-bit descriptor copies)
		const PairDev& pd = a.pairs[pair];
		const PairPlanDev& pp = a.pplan[pair];
		v_off = uni64(pd.v_off);
		r_off = uni64(pd.r_off);
		vl = uni((uint32_t)pd.v_len);
		rl = uni((uint32_t)pd.r_len);
		mem_base = uni64(pp.mem_base);
		q = uni64(pp.q);
		q_magic = uni64(pp.q_magic);
		chunk_base = uni(pp.chunk_base);
		n_chunks = uni(pp.n_chunks);
		rec_base = uni64(pp.rec_base);
	}
	template <class Args>
	__device__ void start(const Args& a, uint32_t job) {
		const uint2 jb = a.chunks[job];
		pair = uni(jb.x);
		c = uni(jb.y);
		load_pair(a);
	}
	template <class Args>
	__device__ void next(const Args& a) {
		if (c + 1 < n_chunks) {
			++c;
		} else {
			++pair;
			c = 0;
			load_pair(a);
		}
	}
};

__device__ const uint4 g_zero16 = {0u, 0u, 0u, 0u};

// 16 bytes of a stream at p (16-aligned), issued without a wait: a piece
// wholly inside the stream loads directly, any other reads a zero block; the
// one piece per stream that straddles its end is rebuilt from bytes at use
// (stage_piece), so no load sits in a branch the compiler must drain.
__device__ __forceinline__ uint4 load16_async(const uint8_t* S, int64_t p, uint32_t len) {
	const bool full = p >= 0 && p + 16 <= (int64_t)len;
	return *(const uint4*)(full ? S + p : (const uint8_t*)&g_zero16);
}

__device__ __forceinline__ uint4 stage_piece(const uint4& v, const uint8_t* S, int64_t p, uint32_t len) {
	if (!(p >= 0 && p < (int64_t)len && p + 16 > (int64_t)len)) return v;
	uint32_t w[4] = {0u, 0u, 0u, 0u};
	for (uint32_t b = 0; p + b < (int64_t)len; ++b) w[b >> 2] |= (uint32_t)S[p + b] << (8 * (b & 3u));
	return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void stage_load(const SpecArgs& a, const JobCursor& J, StageRegs& S) {
	const int64_t g0 = (int64_t)J.c * kMemChunk - 16;
	const uint8_t* V = a.ver + J.v_off;
	const uint8_t* R = a.ref + J.r_off;
	const uint32_t lane = lane_id();
#pragma unroll
	for (uint32_t k = 0; k < kStageRows; ++k) {
		const int64_t p = g0 + 1024 * k + 16 * lane;
		S.v[k] = load16_async(V, p, J.vl);
		S.r[k] = load16_async(R, p, J.rl);
	}
}

// the staged bytes into LDS (straddling pieces rebuilt here)
__device__ __forceinline__ void stage_store(const SpecArgs& a, const JobCursor& J, const StageRegs& S, ChunkLds& L) {
	const int64_t g0 = (int64_t)J.c * kMemChunk - 16;
	const uint32_t lane = lane_id();
	const uint32_t vl = J.vl, rl = J.rl;
	const bool tail = g0 + (int64_t)kStage > (int64_t)umin32(vl, rl);   // (uniform) the streams end in this region
#pragma unroll
	for (uint32_t k = 0; k < kStageRows; ++k) {
		const int64_t p = g0 + 1024 * k + 16 * lane;
		uint4 v = S.v[k], r = S.r[k];
		if (tail) {
			v = stage_piece(v, a.ver + J.v_off, p, vl);
			r = stage_piece(r, a.ref + J.r_off, p, rl);
		}
		*(uint4*)(L.v + 1024 * k + 16 * lane) = v;
		*(uint4*)(L.r + 1024 * k + 16 * lane) = r;
	}
}

__device__ __forceinline__ void member_chunk(const SpecArgs& a, ChunkLds& L, const JobCursor& J,
                                             [[maybe_unused]] MemProf& mp) {
	const uint32_t lane = lane_id();
	const uint32_t c = J.c;
	const uint32_t vl = J.vl, rl = J.rl;
	const uint32_t E = umin32(vl, rl);
	const uint32_t cw = c * kMemChunk;                  // chunk start (position)
	const int64_t g0 = (int64_t)cw - 16;                // position of staged offset 0
	const uint64_t slot0 = J.mem_base + (uint64_t)c * kMemChunkSlots;

	// ── 2. mismatch bitmap: bit o = position g0 + o differs (or is E, the
	//    sentinel); chunk 0's lookbehind holds only the virtual mismatch at -1 ──
	const int64_t lim = (int64_t)E - g0;   // offset of the sentinel
	MPROF_T(tm0);
	for (uint32_t j = lane; j < kMaskWords; j += 64) {
		const uint32_t o = 32 * j;
		uint32_t m = 0;
		if ((int64_t)o < lim) {
			const uint4* pv = (const uint4*)(L.v + o);
			const uint4* pr = (const uint4*)(L.r + o);
			m = mismatch16(pv[0], pr[0]) | (mismatch16(pv[1], pr[1]) << 16);
			if ((int64_t)o + 32 > lim) m &= (1u << (uint32_t)(lim - o)) - 1u;
		}
		if (lim >= (int64_t)o && lim < (int64_t)o + 32) m |= 1u << (uint32_t)(lim - o);
		if (o + 32 > kStage) m &= (1u << (kStage - o)) - 1u;
		if (g0 < 0 && j == 0) m = (m & ~0xFFFFu) | 0x8000u;   // offsets 0..15 = positions -16..-1
		L.mask[j] = m;
	}
	lds_fence();
	MPROF_ADD(MP_MASK, tm0);
	MPROF_T(tr0);
	// ── 3. run starts (offsets >= 16: positions of this chunk and the
	//    look-ahead) and the running last-mismatch maximum ──
	uint32_t nrun = g0 < 0 ? 1u : 0u, carry = 0;   // chunk 0: slot 0 is member 0 (position 0)
	for (uint32_t j0 = 0; j0 < kMaskWords; j0 += 64) {
		const uint32_t j = j0 + lane;
		const bool in = j < kMaskWords;
		const uint32_t m = in ? L.mask[j] : 0u;
		const uint32_t mp = (in && j > 0) ? L.mask[j - 1] : 0u;
		uint64_t cov = ((uint64_t)m << 32) | mp;
		cov |= cov << 1;
		cov |= cov << 2;
		cov |= cov << 4;
		cov |= cov << 8;
		uint32_t rs = m & ~(uint32_t)((cov << 1) >> 32);
		if (j == 0) rs &= ~0xFFFFu;   // the lookbehind starts no run
		const uint32_t last1 = m ? 32 * j + 32u - (uint32_t)__builtin_clz(m) : 0u;
		const uint32_t lm = umax32(wave_incl_max(last1), carry);
		if (in) L.last[j] = (uint16_t)lm;
		carry = rdlane(lm, 63);
		const uint32_t cnt = (uint32_t)__builtin_popcount(rs);
		const uint32_t incl = wave_incl_scan(cnt);
		uint32_t idx = nrun + incl - cnt;
		for (uint32_t b = rs; b; b &= b - 1) {
			if (idx < kRunList) L.run[idx] = (uint16_t)(32 * j + (uint32_t)__builtin_ctz(b));
			++idx;
		}
		nrun += rdlane(incl, 63);
	}
	if (g0 < 0 && lane == 0) L.run[0] = 16;   // member 0 starts its epoch at position 0 (offset 16)
	nrun = umin32(nrun, kRunList);
	lds_fence();
	// members: runs starting in [16, 16 + kMemChunk) (a prefix of the list)
	uint32_t nm = 0;
	for (uint32_t i0 = 0; i0 < nrun; i0 += 64) {
		const uint32_t i = i0 + lane;
		nm += (uint32_t)__builtin_popcountll(__ballot(i < nrun && L.run[i] < 16 + kMemChunk));
	}
	if (lane == 0) a.n_mem[J.chunk_base + c] = nm;
	MPROF_ADD(MP_RUNS, tr0);
	MPROF_INC(MP_MEMBERS, nm);
	MPROF_T(ts0);

	// The last member when no later run starts in the staged region (sparse
	// edits: 1 MiB pairs at 1 %): its run has ended once 16 clean bytes follow
	// its last mismatch inside the region, so x is known; its COPY runs to the
	// first mismatch past the region (or the end E, the sentinel), found here
	// from HBM, and that position is the next run start (>= 16 clean bytes
	// before it) in a later chunk.  Without it the member stays unverified and
	// the chain runs the exact epoch machinery from it.  The search is capped
	// at kSnScanRows KiB past the region (one dependent round trip per KiB):
	// past the cap the member stays unverified, as before.
	constexpr uint32_t kSnScanRows = 16;
	uint32_t sn_last = 0;   // its next run start (offset from g0), 0: unknown
	if (nm > 0 && nm == nrun && (int64_t)E > g0 + (int64_t)kStage) {
		const uint32_t xl = L.last[kMaskWords - 1];   // last mismatch + 1 (the sentinel is past the region)
		if (xl + 16 <= kStage) {
			const uint8_t* V = a.ver + J.v_off;
			const uint8_t* R = a.ref + J.r_off;
			uint32_t y = ~0u;
			const uint64_t b_end = (uint64_t)(g0 + (int64_t)kStage) + 1024ull * kSnScanRows;
			for (uint64_t b = (uint64_t)(g0 + (int64_t)kStage); y == ~0u && b < b_end; b += 1024) {
				if (b >= E) { y = E; break; }
				const uint64_t p0 = b + 16ull * lane;
				uint32_t m = 0;   // bit k: byte p0 + k differs (or is at/after E)
				if (p0 < E) {
					if (p0 + 16 <= E) {
						uint4 v, r;
						__builtin_memcpy(&v, V + p0, 16);
						__builtin_memcpy(&r, R + p0, 16);
						m = mismatch16(v, r);
					} else {
						for (uint32_t k = 0; k < 16; ++k)
							if (p0 + k >= E || V[p0 + k] != R[p0 + k]) m |= 1u << k;
					}
				} else {
					m = 0xFFFFu;
				}
				const uint64_t w = __ballot(m != 0u);
				if (w) {
					const uint32_t L0 = ffs64(w);
					const uint32_t mb = rdlane(m, L0);
					const uint64_t yy = b + 16ull * L0 + (uint32_t)__builtin_ctz(mb);
					y = yy < E ? (uint32_t)yy : E;
				}
			}
			if (y != ~0u) sn_last = (uint32_t)((int64_t)y - g0);
		}
	}

	MPROF_ADD(MP_SNLAST, ts0);
	const uint64_t q = J.q, qmag = J.q_magic;
	const ModQ mq = make_modq(q, qmag);
	VFilter<64> fs{L.filt};
	const uint8_t* SV = L.v;
	const uint8_t* SR = L.r;

	uint32_t vp = 0, vbytes = 0;   // verified prefix of the chunk's members, its delta bytes
	bool open = true;
	for (uint32_t k0 = 0; k0 < nm; k0 += 64) {
		MPROF_T(tb0);
		// lane m: member k0 + m (offsets; x = last mismatch before the next
		// run start + 1; a member whose next start is unknown stays unverified)
		const uint32_t k1 = umin32(k0 + 64, nm);
		const uint32_t i = k0 + lane;
		const bool mine = i < k1;
		const uint32_t s = mine ? L.run[i] : 0u;
		const bool in_region = mine && i + 1 < nrun;   // the next run start is staged
		const bool known = in_region || (mine && i + 1 == nrun && sn_last != 0u);
		const uint32_t sn = in_region ? L.run[i + 1] : (known ? sn_last : 0u);
		uint32_t x = 0;
		if (in_region) {   // highest mismatch offset below sn, + 1
			const uint32_t j = sn >> 5, b = sn & 31u;
			const uint32_t below = L.mask[j] & ((1u << b) - 1u);
			x = below ? 32 * j + 32u - (uint32_t)__builtin_clz(below) : (j ? L.last[j - 1] : 0u);
		} else if (known) {   // every staged mismatch is below sn
			x = L.last[kMaskWords - 1];
		}
		const uint32_t T = x - s;
		const bool shrt = known && T < 64;
		const uint32_t P = wave_incl_scan(shrt ? T + 1 : 0u);   // packed end of each short member
		uint32_t* mem_s = a.mem_s + slot0 + k0;
		uint32_t* srec = a.srec + 4ull * (slot0 + k0);
		bool myok = false;   // this lane's member verified
		if (mine) {
			mem_s[lane] = (uint32_t)(g0 + (int64_t)s);
			if (!known || T >= 64u * kLongChunks) {   // unverified: the chain runs its epoch exactly
				uint32_t z;   // a zero made here: a hoisted constant uint4 was spilled to scratch
				asm volatile("v_mov_b32 %0, 0" : "=v"(z));
				*(uint4*)(srec + 4 * lane) = make_uint4(z, z, z, z);
			}
		}

		MPROF_INC(MP_SHORT_N, __builtin_popcountll(__ballot(shrt)));
		MPROF_INC(MP_UNVER, __builtin_popcountll(__ballot(mine && (!known || T >= 64u * kLongChunks))));
		MPROF_ADD(MP_SETUP, tb0);
		MPROF_T(tq0);
		// ── short members, packed 64 steps per round (lane = step) ──
		uint32_t done = 0;
		for (;;) {
			const bool in = shrt && P > done && P <= done + 64;
			const uint64_t RM = __ballot(in);
			if (!RM) break;
#ifdef DG_MEM_SKIP_SHORT   // timing variants only
			break;
#endif
			MPROF_INC(MP_ROUNDS, 1);
			const uint32_t hi = 63u - (uint32_t)__builtin_clzll(RM);
			const uint32_t B = rdlane(P, hi) - done;   // live steps of the round
			// lane -> member: a mark at each member's first step, prefix max
			lds_order();
			L.mark[lane] = 0u;
			fs.clear();
			lds_order();
			const uint32_t st = P - (T + 1) - done;   // first step lane (members in the round)
			if (in) L.mark[st] = (uint8_t)(lane + 1u);
			lds_order();
			const bool live = lane < B;
			const uint32_t mk = wave_incl_max(L.mark[lane]);   // lane 0 always holds a mark
			const uint32_t mj = live ? mk - 1u : 0u;            // member lane
			// (start, T, first step lane) of this lane's member, one bpermute
			const uint32_t inf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)(s | (T << 12) | (st << 18)));
			const uint32_t ms_j = inf & 0xFFFu, mt_j = (inf >> 12) & 63u, fb = inf >> 18;
			const uint32_t t = lane - fb;
			const bool isT = live && t == mt_j;
			uint32_t sV = kSentinel, fVl = 0, fRl = 1;   // (fVl, fRl: window hashes)
			if (live) {
				const uint4 wv = lds16(SV, ms_j + t), wr = lds16(SR, ms_j + t);
#ifdef DG_MEM_SKIP_FP   // timing variants only: no fingerprints
				sV = wv.x % 16411u;
#else
				sV = slot_of(fp16_dot(wv.x, wv.y, wv.z, wv.w), mq, q, qmag);
#endif
				fVl = win_hash(wv);
				fRl = win_hash(wr);
			}
#ifndef DG_MEM_SKIP_A
			if (live && !isT) fs.add(fVl);
#endif
			lds_order();
			const uint64_t mem = live ? lanes_mask(fb, mt_j + 1) : 0ull;   // this lane's member
			bool bad = false;
			// (A) off T: steps whose R hash may equal another step's V hash
#ifdef DG_MEM_SKIP_A
			for (uint64_t w = 0; w; w &= w - 1) {
#else
			for (uint64_t w = __ballot(live && !isT && fs.has(fRl)); w; w &= w - 1) {
#endif
				MPROF_INC(MP_FLAGGED, 1);
				const uint32_t Lx = ffs64(w);
				const uint64_t others = ((uint64_t)rdlane((uint32_t)(mem >> 32), Lx) << 32 | rdlane((uint32_t)mem, Lx)) &
				                        ~(1ull << Lx);
				const bool hit = (__ballot(fVl == rdlane(fRl, Lx)) & others) != 0;
				bad = bad || (hit && lane == Lx);
			}
			// T steps, all members at once: (A) through T (a V or R repeat of
			// the T window among the member's earlier steps), then (B) — the T
			// step's V slot against the earlier V slots, R slots only when one
			// repeats.  Every step lane fetches its T step's values, the
			// ballots flag the steps, and each T lane reads its member's bits.
			{
				const int tsel = (int)(((fb + mt_j) & 63u) << 2);   // this lane's T lane
				const uint32_t hT = (uint32_t)__builtin_amdgcn_ds_bpermute(tsel, (int)fVl);
				const uint32_t vT = (uint32_t)__builtin_amdgcn_ds_bpermute(tsel, (int)sV);
				const bool step = live && !isT;
				const uint64_t A1 = __ballot(step && (fVl == hT || fRl == hT));
				const uint64_t B1 = __ballot(step && sV == vT);
				bool badT = isT && (A1 & mem) != 0;
				const bool d1 = isT && !badT && (B1 & mem) != 0;
				if (__ballot(d1)) {   // rare: the R slots
					MPROF_INC(MP_D1, 1);
					const uint32_t sR = live ? slot_lds(SR, ms_j + t, mq, q, qmag) : kSentinel - 1u;
					const uint32_t rT = (uint32_t)__builtin_amdgcn_ds_bpermute(tsel, (int)sR);
					const uint64_t C1 = __ballot(step && sR == rT);
					badT = badT || (d1 && (C1 & mem) != 0);
				}
				bad = bad || badT;
			}
			// verdict at each member's T step; the record carries the ADD head
			// (the first step's V window) and the COPY length
			// verdicts and records on the member lanes themselves (no gathers):
			// member m's steps are lanes [P - T - 1 - done, P - done) of the
			// round; its ADD head is the first word of its first V window
			const uint64_t BA = __ballot(bad);
			if (in) {
				const bool ok = (BA & lanes_mask(P - T - 1u - done, T + 1u)) == 0;
				const uint32_t* d = reinterpret_cast<const uint32_t*>(SV + (s & ~3u));
				const uint32_t head = __builtin_amdgcn_alignbit(d[1], d[0], (s & 3u) * 8u);
				*(uint4*)(srec + 4 * lane) = make_uint4((uint32_t)(g0 + (int64_t)(s + T)), sn - (s + T), head, ok ? 1u : 0u);
				myok = ok;
			}
			done += B;
		}

		MPROF_ADD(MP_SHORT, tq0);
		MPROF_T(tl0);
		// ── long members (64 <= T < 512): 64-step rows, history in VGPRs ──
#ifdef DG_MEM_SKIP_LONG   // timing variants only
		for (uint64_t LM = 0; LM; LM &= LM - 1) {
#else
		for (uint64_t LM = __ballot(known && !shrt && T < 64u * kLongChunks); LM; LM &= LM - 1) {
#endif
			MPROF_INC(MP_LONG_N, 1);
			const uint32_t M = ffs64(LM);
			const uint32_t s0 = rdlane(s, M), tl = rdlane(T, M), sn0 = rdlane(sn, M);
			uint32_t pw;
			const bool ok = tl < 128 ? long_member_rows<64, 2>(SV, SR, s0, tl, L.filt, mq, q, qmag, pw)
			                : tl < 192 ? long_member_rows<64, 3>(SV, SR, s0, tl, L.filt, mq, q, qmag, pw)
			                           : long_member_ok<64>(SV, SR, s0, tl, L.filt, mq, q, qmag, pw);
			if (lane == 0) {
				*(uint4*)(srec + 4 * M) = make_uint4((uint32_t)(g0 + (int64_t)(s0 + tl)), sn0 - (s0 + tl), pw,
				                                     ok ? 1u : 0u);
			}
			if (lane == M) myok = ok;
		}
		MPROF_ADD(MP_LONG, tl0);
		MPROF_T(tp0);
		// the chunk's verified prefix through this batch
		if (open) {
			const uint32_t lim2 = k1 - k0;
			const uint64_t live = lim2 == 64 ? ~0ull : ((1ull << lim2) - 1ull);
			const uint64_t gaps = ~__ballot(mine && myok) & live;
			const uint32_t take = gaps ? ffs64(gaps) : lim2;
			const uint32_t b = lane < take ? 13u + (T ? 9u + T : 0u) : 0u;
			vbytes += rdlane(wave_incl_scan(b), 63);
			vp += take;
			open = take == lim2;
		}
		MPROF_ADD(MP_PREFIX, tp0);
	}
	// ── 5. chunk summary for the chain: the verified prefix and its delta
	//    bytes (accumulated per batch above) ──
	if (lane == 0) {
		a.csum[2ull * (J.chunk_base + c)] = vp;
		a.csum[2ull * (J.chunk_base + c) + 1] = vbytes;
		*(uint2*)(a.cmap + 2ull * (J.chunk_base + c)) = make_uint2(0u, 0u);   // no bulk piece yet
	}
}

// One wave per (pair, chunk) job.  The chunk's bytes are staged by LDS-DMA
// (no VGPRs held for them), which keeps the wave within 96 VGPRs and 8 KiB
// of LDS: 5 waves per SIMD to hide the LDS and DMA latencies of the rounds.

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DG_MEM_WAVES, 8))) void member_chunk_kernel(SpecArgs a, uint32_t n_chunks) {
	// The member waves issue ahead of the CRC pass's waves sharing their SIMDs
	// (the five-bit CRC rows take the VALU slots they leave): C3 444 -> 458,
	// c6 1177 -> 1287 GiB/s; with the lane-contiguous CRC pass the CRC starved
	// (profiles/r05_experiments.md)
	__builtin_amdgcn_s_setprio(1);
	__shared__ __attribute__((aligned(16))) ChunkLds L;
	const uint32_t lane = lane_id();
	JobCursor J;
	J.start(a, a.job0 + blockIdx.x);
	MemProf mp;
	MPROF_T(tk0);
	{
		const int64_t g0 = (int64_t)J.c * kMemChunk - 16;
		const uint8_t* V = a.ver + J.v_off;
		const uint8_t* R = a.ref + J.r_off;
#pragma unroll
		for (uint32_t k = 0; k < kStageRows; ++k) {
			const int64_t p = g0 + 1024 * k + 16 * lane;
			if (1024 * k + 16 * lane >= kStage) continue;
			// whole pieces by DMA; the piece straddling a stream's end (and
			// the lookbehind before position 0) through registers
			if (p >= 0 && p + 16 <= (int64_t)J.vl)
				__builtin_amdgcn_global_load_lds((const void*)(V + p), (lds_void_t*)(L.v + 1024 * k), 16, 0, 0);
			else
				*(uint4*)(L.v + 1024 * k + 16 * lane) = stage_piece(make_uint4(0u, 0u, 0u, 0u), V, p, J.vl);
			if (p >= 0 && p + 16 <= (int64_t)J.rl)
				__builtin_amdgcn_global_load_lds((const void*)(R + p), (lds_void_t*)(L.r + 1024 * k), 16, 0, 0);
			else
				*(uint4*)(L.r + 1024 * k + 16 * lane) = stage_piece(make_uint4(0u, 0u, 0u, 0u), R, p, J.rl);
		}
		vm_drain();
		__syncthreads();
	}
	MPROF_ADD(MP_STAGE, tk0);
	member_chunk(a, L, J, mp);
#ifdef DG_ONEPASS_PROF
	MPROF_ADD(MP_TOTAL, tk0);
	MPROF_INC(MP_CHUNKS, 1);
	if (lane == 0)
		for (int k = 0; k < kMemProfN; ++k)
			atomicAdd(&g_member_prof[(blockIdx.x % kMemProfSlots) * kMemProfN + k], (unsigned long long)mp.v[k]);
#endif
}

#ifdef DG_ONEPASS_PROF
extern "C" int dg_member_prof_read(unsigned long long* out, int n) {
	if (n > kMemProfN) n = kMemProfN;
	static unsigned long long h[kMemProfSlots * kMemProfN];
	if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_member_prof), sizeof h) != hipSuccess) return -1;
	for (int k = 0; k < n; ++k) {
		out[k] = 0;
		for (uint32_t s = 0; s < kMemProfSlots; ++s) out[k] += h[s * kMemProfN + k];
	}
	return n;
}
extern "C" int dg_member_prof_reset(void) {
	static unsigned long long z[kMemProfSlots * kMemProfN] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_member_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

// ── member-mode serialisation ──────────────────────────────────────────

// big-endian u32 / u8 at any byte address (unaligned LDS or global stores)
template <typename P>
__device__ __forceinline__ void put_be32(P p, uint32_t x) {
	const uint32_t b = __builtin_bswap32(x);
	__builtin_memcpy(p, &b, 4);
}

// Commands of up to 64 bulk members (lane = member) into dst at byte `my`
// (LDS stage or, for an oversized tile, the output itself): ADD header and
// payload, then the COPY.  Payloads come from the chunk's V bytes staged in
// LDS (vb = position g0); a payload of > 64 bytes is copied by the whole wave.
template <typename P>
__device__ __forceinline__ void put_bulk(P dst, bool valid, uint32_t my, uint32_t prev, uint32_t x, uint32_t len,
                                         uint32_t pw, const uint8_t* vb, int64_t g0) {
	const uint32_t lane = lane_id();
	const uint32_t gap = x - prev;
	const bool add = valid && gap != 0;
	if (add) {
		P q = dst + my;
		q[0] = 2;
		put_be32(q + 1, prev);
		put_be32(q + 5, gap);
		if (gap <= 4) {
			__builtin_memcpy(q + 9, &pw, 4);   // spill past the payload lands in the COPY, written below
		} else if (gap < 16) {
			const uint8_t* src = vb + (prev - g0);
			for (uint32_t k = 0; k < gap; k += 4) {   // spill <= 3 bytes: as above
				uint32_t w;
				__builtin_memcpy(&w, src + k, 4);
				__builtin_memcpy(q + 9 + k, &w, 4);
			}
		} else if (gap <= 64) {
			// 16-byte pieces, the last one ending at the payload's end (no spill)
			const uint8_t* src = vb + (prev - g0);
			for (uint32_t k = 0; k < gap; k += 16) {
				const uint32_t kk = umin32(k, gap - 16);
				uint4 w;
				__builtin_memcpy(&w, src + kk, 16);
				__builtin_memcpy(q + 9 + kk, &w, 16);
			}
		}
	}
	for (uint64_t bm = __ballot(add && gap > 64); bm; bm &= bm - 1) {
		const uint32_t k = ffs64(bm);
		const uint32_t src = rdlane(prev, k) - (uint32_t)g0, n = rdlane(gap, k), o = rdlane(my, k) + 9;
		for (uint32_t i = 16 * lane; i < n; i += 1024) {
			const uint32_t ii = umin32(i, n - 16);   // the last piece ends at the payload's end
			uint4 w;
			__builtin_memcpy(&w, vb + src + ii, 16);
			__builtin_memcpy(dst + o + ii, &w, 16);
		}
	}
	__builtin_amdgcn_wave_barrier();
	if (valid) {
		P q = dst + my + (gap ? 9u + gap : 0u);
		q[0] = 1;
		put_be32(q + 1, x);
		put_be32(q + 5, x);
		put_be32(q + 9, len);
	}
}

constexpr uint32_t kMemSerStage = 4096;
#ifndef DG_MSER_WAVES
#define DG_MSER_WAVES 16
#endif
constexpr uint32_t kSerWavesPerCu = DG_MSER_WAVES;   // persistent serialiser waves per CU (LDS allows 24)
#ifndef DG_MSER_WAVES_SPARSE
#define DG_MSER_WAVES_SPARSE 24
#endif
constexpr uint32_t kSerWavesSparse = DG_MSER_WAVES_SPARSE;   // ... for a sparse batch (delta < |V| / 2)

// one job's inputs, loaded a job ahead (descriptors wave-uniform)
struct SerFetch {
	JobCursor J;
	uint32_t cnt, boff, first;
	int32_t st;
	uint64_t base, end, slot0;
	uint4 v[kStageRows];   // the chunk's staged V bytes (as the member kernel's)
	uint4 r;               // member record of this lane (first 64)
};

// every load unconditional (no branch for the compiler to drain before the
// loads of the job after it are issued)
__device__ __forceinline__ void ser_fetch(const MemSerArgs& a, SerFetch& F) {
	const uint32_t lane = lane_id();
	const JobCursor& J = F.J;
	F.st = a.status[J.pair];
	F.base = a.offsets[J.pair];
	F.end = a.offsets[J.pair + 1];
	const uint2 cm = *(const uint2*)(a.cmap + 2ull * (J.chunk_base + J.c));
	F.cnt = cm.x;
	F.boff = cm.y;
	F.slot0 = J.mem_base + (uint64_t)J.c * kMemChunkSlots;
	const int64_t g0 = (int64_t)J.c * kMemChunk - 16;
	const uint8_t* V = a.ver + J.v_off;
#pragma unroll
	for (uint32_t k = 0; k < kStageRows; ++k) F.v[k] = load16_async(V, g0 + 1024 * k + 16 * lane, J.vl);
	F.r = make_uint4(0u, 0u, 0u, 0u);   // (slots 0..63 of the chunk's 129, only the bulk members')
	if (lane < F.cnt) F.r = *(const uint4*)(a.srec + 4ull * (F.slot0 + lane));
	F.first = a.mem_s[F.slot0];
}

// Member-mode serialisation: each chunk's job writes its bulk piece (the
// members the chain took as they are, from the member records, payloads from
// the chunk's V bytes in LDS) at the piece's byte offset, plus the pair's
// segments 2c, 2c + 1 (record runs of the chain's own epochs, the tail), so
// all the chunks of a pair serialise at once.  Persistent waves over
// contiguous jobs, each job's inputs loaded while the previous one is written.
// (ADD payloads read straight from V instead of the staged chunk measured
// slower even on the sparsest bench batch, c6: profiles/r04_experiments.md.)
__device__ __forceinline__ void member_serialize(const MemSerArgs& a, uint32_t j0, uint32_t j1, uint8_t* vbuf,
                                                 uint8_t* stage) {
	const uint32_t lane = lane_id();
	SerFetch F, N;
	F.J.start(a, j0);
	ser_fetch(a, F);
	for (uint32_t j = j0; j < j1; ++j) {
		if (j + 1 < j1) {
			N.J = F.J;
			N.J.next(a);
			ser_fetch(a, N);
		}
		const uint32_t vl = F.J.vl;
		const uint8_t* V = a.ver + F.J.v_off;
		if (F.st == 0) {
			if (F.end > a.out_cap) {
				if (F.J.c == 0 && lane == 0) a.status[F.J.pair] = 7;
			} else {
				uint8_t* out = a.out + F.base;
				if (F.J.c == 0) put_header(out, vl);
				if (F.cnt) {
					// ADD payloads from the chunk's V bytes staged in LDS
					const int64_t g0 = (int64_t)F.J.c * kMemChunk - 16;
					const uint8_t* vb = vbuf;
					lds_order();
#pragma unroll
					for (uint32_t k = 0; k < kStageRows; ++k)
						if (1024 * k + 16 * lane < kStage)
							*(uint4*)(vbuf + 1024 * k + 16 * lane) = stage_piece(F.v[k], V, g0 + 1024 * k + 16 * lane, vl);
					lds_order();
					uint64_t pos = F.boff;
					uint32_t prev_end = F.first;
					for (uint32_t t0 = 0; t0 < F.cnt; t0 += 64) {
						uint4 r = F.r;
						if (t0 && t0 + lane < F.cnt) r = *(const uint4*)(a.srec + 4ull * (F.slot0 + t0 + lane));
						const bool valid = t0 + lane < F.cnt;
						const uint32_t x = r.x, len = r.y;
						const uint32_t last = valid ? x + len : 0u;
						uint32_t prev = wave_shr1(last);
						if (lane == 0) prev = prev_end;
						const uint32_t gap = x - prev;
						const uint32_t sz = valid ? 13u + (gap ? 9u + gap : 0u) : 0u;
						const uint32_t incl = wave_incl_scan(sz);
						const uint32_t my = incl - sz;
						const uint32_t S = rdlane(incl, 63);
						if (S <= kMemSerStage) {
							lds_order();
							put_bulk(stage, valid, my, prev, x, len, r.z, vb, g0);
							lds_order();
							// flush: head bytes to a 16-byte boundary, 16-byte stores, tail bytes
							uint8_t* dst = out + pos;
							const uint32_t head = umin32((uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u), S);
							if (lane < head) dst[lane] = stage[lane];
							const uint32_t nq = (S - head) / 16;
							uint4* dq = reinterpret_cast<uint4*>(dst + head);
							for (uint32_t k = lane; k < nq; k += 64) {
								uint4 w;
								__builtin_memcpy(&w, stage + head + 16 * k, 16);
								dq[k] = w;
							}
							const uint32_t tail0 = head + 16 * nq;
							if (lane < S - tail0) dst[tail0 + lane] = stage[tail0 + lane];
						} else {
							put_bulk(out + pos, valid, my, prev, x, len, r.z, vb, g0);
						}
						pos += S;
						const uint64_t has = __ballot(valid);
						prev_end = rdlane(last, 63u - (uint32_t)__builtin_clzll(has));
					}
				}
				// the chain's own record runs and the tail (segments 2c, 2c + 1;
				// the pair's last chunk takes the rest)
				const uint32_t ns = a.nseg[F.J.pair];
				const uint32_t* seg = a.seg + 4ull * ((uint64_t)F.J.chunk_base + 2ull * F.J.pair);
				const uint32_t k1 = F.J.c + 1 == F.J.n_chunks ? ns : umin32(2 * F.J.c + 2, ns);
				for (uint32_t k = 2 * F.J.c; k < k1; ++k) {
					const uint4 e = *(const uint4*)(seg + 4ull * k);
					uint8_t* o = out + e.z;
					if (e.x == kSegTail) {
						const uint64_t n = put_tail(o, V, vl, e.w);
						if (e.z + n != F.end - F.base && lane == 0) a.status[F.J.pair] = 12;   // DG_ERR_INTERNAL: sizes disagree
					} else {
						const RecWords src{a.rec + (uint64_t)kRecWordsOnepass * (F.J.rec_base + e.x), kRecWordsOnepass};
						serialize_run<kMemSerStage>(o, V, vl, src, e.y, e.w, (sw_lds8*)stage);
					}
				}
			}
		}
		F = N;
	}
}

// ── member-mode serialisation, software-pipelined (DG_MSER_PIPE, default) ──
//
// member_serialize waits, for every job, for the next job's loads issued
// after this job's stores (loads and stores share the vmcnt counter, which
// drains in issue order: the copy of the prefetched registers waits for the
// stores too).  Here the next job's V bytes and member records go by LDS-DMA
// into rings of two slots, its descriptors by scalar loads (lgkmcnt, not
// vmcnt), and a job's flush is a fixed count of buffer stores, so one
// hand-counted s_waitcnt vmcnt(kMserTileStores) at the top of the next job
// covers its DMAs without waiting for a single store; a job that writes more
// (a second tile, the chain's own record runs, the tail, an oversized tile)
// drains with vmcnt(0) instead.
constexpr uint32_t kMserPipeStage = 2048;
constexpr uint32_t kMserTileStores = kMserPipeStage / 1024 + 2;   // head bytes, 16-byte pieces, tail bytes
constexpr uint32_t kMserVSlot = kStage + 16;
typedef __attribute__((address_space(4))) const uint32_t c4_u32;
typedef __attribute__((address_space(4))) const uint64_t c4_u64;

struct SerJob {   // one job's descriptors, wave-uniform (scalar loads)
	uint32_t pair, c, n_chunks, chunk_base, vl, cnt, boff, first;
	int32_t st;
	uint64_t v_off, mem_base, rec_base, base, end, slot0;
};

__device__ __forceinline__ void ser_job_pair(const MemSerArgs& a, SerJob& J) {
	static_assert(sizeof(PairDev) == 32, "pair: r_off, r_len, v_off, v_len");
	const c4_u64* pd = (const c4_u64*)(a.pairs + J.pair);
	const PairPlanDev* pp = a.pplan + J.pair;
	J.v_off = pd[2];
	J.vl = (uint32_t)pd[3];
	J.mem_base = ((const c4_u64*)&pp->mem_base)[0];
	J.rec_base = ((const c4_u64*)&pp->rec_base)[0];
	J.chunk_base = ((const c4_u32*)&pp->chunk_base)[0];
	J.n_chunks = ((const c4_u32*)&pp->n_chunks)[0];
}

__device__ __forceinline__ void ser_job_chunk(const MemSerArgs& a, SerJob& J) {
	J.st = (int32_t)((c4_u32*)(a.status + J.pair))[0];
	J.base = ((c4_u64*)(a.offsets + J.pair))[0];
	J.end = ((c4_u64*)(a.offsets + J.pair))[1];
	const c4_u32* cm = (c4_u32*)(a.cmap + 2ull * (J.chunk_base + J.c));
	J.cnt = cm[0];
	J.boff = cm[1];
	J.slot0 = J.mem_base + (uint64_t)J.c * kMemChunkSlots;
	J.first = ((c4_u32*)(a.mem_s + J.slot0))[0];
}

__device__ __forceinline__ void ser_job_start(const MemSerArgs& a, SerJob& J, uint32_t job) {
	const c4_u32* jb = (c4_u32*)(a.chunks + job);
	J.pair = jb[0];
	J.c = jb[1];
	ser_job_pair(a, J);
	ser_job_chunk(a, J);
}

__device__ __forceinline__ void ser_job_next(const MemSerArgs& a, SerJob& J) {
	if (J.c + 1 < J.n_chunks) {
		++J.c;
	} else {
		++J.pair;
		J.c = 0;
		ser_job_pair(a, J);
	}
	ser_job_chunk(a, J);
}

// the job's V region [c * 2048 - 16, + kStage) and member records 0..63 into
// ring slot s; pieces not wholly inside V are left out (never read, except the
// one that straddles |V|, rebuilt after landing)
__device__ __forceinline__ void ser_job_dma(const MemSerArgs& a, const SerJob& J, uint8_t* vslot, uint8_t* rslot) {
	const uint32_t lane = lane_id();
	const int64_t g0 = (int64_t)J.c * kMemChunk - 16;
	const uint8_t* V = a.ver + J.v_off;
#pragma unroll
	for (uint32_t k = 0; k < kStageRows; ++k) {
		const int64_t p = g0 + 1024 * k + 16 * lane;
		if (1024 * k + 16 * lane < kStage && p >= 0 && p + 16 <= (int64_t)J.vl)
			__builtin_amdgcn_global_load_lds((const void*)(V + p), (lds_void_t*)(vslot + 1024 * k), 16, 0, 0);
	}
	if (lane < J.cnt && lane < 64)
		__builtin_amdgcn_global_load_lds((const void*)(a.srec + 4ull * (J.slot0 + lane)), (lds_void_t*)rslot, 16, 0, 0);
}

__device__ __forceinline__ void member_serialize_pipe(const MemSerArgs& a, uint32_t j0, uint32_t j1, uint8_t* vring,
                                                      uint8_t* rring, uint8_t* stage) {
	typedef __attribute__((address_space(3))) const uint32_t lds32c;
	const uint32_t lane = lane_id();
	SerJob F, N;
	ser_job_start(a, F, j0);
	ser_job_dma(a, F, vring, rring);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	for (uint32_t j = j0, slot = 0; j < j1; ++j, slot ^= 1u) {
		// this job's DMAs have landed: only the previous job's kMserTileStores
		// stores were issued after them (or everything was drained)
		asm volatile("s_nop 7\n\ts_nop 5\n\ts_waitcnt vmcnt(%0)" ::"n"(kMserTileStores) : "memory");
		uint8_t* vb = vring + kMserVSlot * slot;
		const uint8_t* rb = rring + 1024 * slot;
		if (j + 1 < j1) {
			N = F;
			ser_job_next(a, N);
			ser_job_dma(a, N, vring + kMserVSlot * (slot ^ 1u), rring + 1024 * (slot ^ 1u));
			asm volatile("s_nop 7\n\ts_nop 6" ::: "memory");   // (the ISA check's marker: DMAs above)
		}
		// The next job's wait counts exactly one staged tile's stores after its
		// DMAs; every other path through this job drains right where it
		// departs from that (drain()), so the count holds on every path
		// (tests/test_isa_serialize.py walks them).
		auto drain = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
		const uint32_t vl = F.vl;
		const uint8_t* V = a.ver + F.v_off;
		const int64_t g0 = (int64_t)F.c * kMemChunk - 16;
		if (F.st != 0) {
			drain();
		} else if (F.end > a.out_cap) {
			if (F.c == 0 && lane == 0) a.status[F.pair] = 7;
			drain();
		} else {
			uint8_t* out = a.out + F.base;
			if (F.c == 0) {
				put_header(out, vl);
				drain();
			}
			if (!F.cnt) {
				drain();
			} else {
				// the piece that straddles |V| (the pair's last chunk): from bytes
				if (g0 + (int64_t)kStage > (int64_t)vl) {
#pragma unroll
					for (uint32_t k = 0; k < kStageRows; ++k) {
						const int64_t p = g0 + 1024 * k + 16 * lane;
						if (1024 * k + 16 * lane < kStage && p >= 0 && p < (int64_t)vl && p + 16 > (int64_t)vl) {
							const uint4 z = make_uint4(0u, 0u, 0u, 0u);
							*(uint4*)(vb + 1024 * k + 16 * lane) = stage_piece(z, V, p, vl);
						}
					}
					drain();
				}
				lds_order();
				uint64_t pos = F.boff;
				uint32_t prev_end = F.first;
				// one tile of up to 64 members; tile 0 (records from the ring) is
				// straight-line code, so every path through a job with members
				// passes its fixed stores (or a drain)
				auto tile = [&](uint32_t t0, const uint4& r) {
					const bool valid = t0 + lane < F.cnt;
					const uint32_t x = r.x, len = r.y;
					const uint32_t last = valid ? x + len : 0u;
					uint32_t prev = wave_shr1(last);
					if (lane == 0) prev = prev_end;
					const uint32_t gap = x - prev;
					const uint32_t sz = valid ? 13u + (gap ? 9u + gap : 0u) : 0u;
					const uint32_t incl = wave_incl_scan(sz);
					const uint32_t my = incl - sz;
					const uint32_t S = rdlane(incl, 63);
					if (S <= kMserPipeStage) {
						lds_order();
						put_bulk(stage, valid, my, prev, x, len, r.z, vb, g0);
						lds_order();
						__builtin_amdgcn_s_waitcnt(0xc07f);
						// flush as a fixed count of buffer stores: head bytes to a
						// 16-byte boundary, 16-byte pieces, tail bytes (lanes past
						// the end dropped by each descriptor's size)
						uint8_t* dst = out + pos;
						const uint32_t head = umin32((uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u), S);
						const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)head, 0x00020000);
						__builtin_amdgcn_raw_buffer_store_b8(stage[lane & 15u], rh, (int)lane, 0, 0);
						const uint32_t nq = (S - head) / 16;
						const __amdgpu_buffer_rsrc_t rq =
						    __builtin_amdgcn_make_buffer_rsrc(dst + head, (short)0, (int)(16 * nq), 0x00020000);
#pragma unroll
						for (uint32_t i = 0; i < kMserPipeStage / 1024; ++i) {
							const uint32_t k = lane + 64 * i;
							const uint32_t o = umin32(head + 16 * k, kMserPipeStage);
							uint32_t w[4];
							__builtin_memcpy(w, stage + o, 16);
							typedef uint32_t v4u __attribute__((ext_vector_type(4)));
							__builtin_amdgcn_raw_buffer_store_b128(v4u{w[0], w[1], w[2], w[3]}, rq, (int)(16 * k), 0, 0);
						}
						const uint32_t tail0 = head + 16 * nq;
						const __amdgpu_buffer_rsrc_t rt =
						    __builtin_amdgcn_make_buffer_rsrc(dst + tail0, (short)0, (int)(S - tail0), 0x00020000);
						__builtin_amdgcn_raw_buffer_store_b8(stage[umin32(tail0 + (lane & 15u), kMserPipeStage + 15)], rt, (int)lane, 0, 0);
						__builtin_amdgcn_s_waitcnt(0xc07f);   // the stage's reads before its next writes
					} else {
						put_bulk(out + pos, valid, my, prev, x, len, r.z, vb, g0);
						drain();
					}
					pos += S;
					const uint64_t has = __ballot(valid);
					prev_end = rdlane(last, 63u - (uint32_t)__builtin_clzll(has));
				};
				{
					const lds32c* q = (const lds32c*)(rb + 16 * lane);
					tile(0u, make_uint4(q[0], q[1], q[2], q[3]));
				}
				for (uint32_t t0 = 64; t0 < F.cnt; t0 += 64) {
					drain();   // (the tile before flushed its stores)
					uint4 r = make_uint4(0u, 0u, 0u, 0u);
					if (t0 + lane < F.cnt) r = *(const uint4*)(a.srec + 4ull * (F.slot0 + t0 + lane));
					tile(t0, r);
					drain();
				}
			}
			// the chain's own record runs and the tail (segments 2c, 2c + 1;
			// the pair's last chunk takes the rest)
			const uint32_t ns = ((c4_u32*)(a.nseg + F.pair))[0];
			const uint32_t* seg = a.seg + 4ull * ((uint64_t)F.chunk_base + 2ull * F.pair);
			const uint32_t k1 = F.c + 1 == F.n_chunks ? ns : umin32(2 * F.c + 2, ns);
			for (uint32_t k = 2 * F.c; k < k1; ++k) {
				const uint4 e = *(const uint4*)(seg + 4ull * k);
				uint8_t* o = out + e.z;
				if (e.x == kSegTail) {
					const uint64_t n = put_tail(o, V, vl, e.w);
					if (e.z + n != F.end - F.base && lane == 0) a.status[F.pair] = 12;   // DG_ERR_INTERNAL: sizes disagree
				} else {
					const RecWords src{a.rec + (uint64_t)kRecWordsOnepass * (F.rec_base + e.x), kRecWordsOnepass};
					serialize_run<kMserPipeStage>(o, V, vl, src, e.y, e.w, (sw_lds8*)stage);
				}
				drain();
			}
		}
		F = N;
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the wave
}

// staged_grid: the waves a dense batch uses; a sparse one (delta under half
// of sum |V|) uses the whole grid (the launch gives it kSerWavesSparse per
// CU): its jobs are bound by their dependent descriptor loads, and more,
// shorter job ranges finish sooner (c6 1090 -> 1192 GiB/s), while a dense
// batch's staging traffic is fastest at 16 waves per CU (C3 447 vs 435 at 24)
#ifndef DG_MSER_PIPE   // A/B: 0 = round 5's member_serialize
#define DG_MSER_PIPE 1
#endif
__global__ __launch_bounds__(64) void member_serialize_kernel(MemSerArgs a, uint32_t n_jobs, uint32_t staged_grid) {
#if DG_MSER_PIPE
	__shared__ __attribute__((aligned(16))) uint8_t vring[2 * kMserVSlot];
	__shared__ __attribute__((aligned(16))) uint8_t rring[2 * 1024];
	__shared__ __attribute__((aligned(16))) uint8_t stage[kMserPipeStage + 96];
#else
	__shared__ __attribute__((aligned(16))) uint8_t vbuf[kStage + 16];
	__shared__ __attribute__((aligned(16))) uint8_t stage[kMemSerStage + 96];
#endif
	// (uniform for the launch: the scan's total is final before this kernel)
	const uint64_t dtot = a.v_total ? uni64(a.offsets[a.n_pairs]) : ~0ull;
	const uint32_t grid = dtot * 2 < a.v_total ? gridDim.x : umin32(gridDim.x, staged_grid);
	if (blockIdx.x >= grid) return;
	const uint32_t j0 = a.job0 + (uint32_t)((uint64_t)n_jobs * blockIdx.x / grid);
	const uint32_t j1 = a.job0 + (uint32_t)((uint64_t)n_jobs * (blockIdx.x + 1) / grid);
	if (j0 >= j1) return;
#if DG_MSER_PIPE
	member_serialize_pipe(a, j0, j1, vring, rring, stage);
#else
	member_serialize(a, j0, j1, vbuf, stage);
#endif
}

hipError_t launch_members(const SpecArgs& a, uint32_t n_chunks, uint32_t n_cu, hipStream_t st) {
	if (n_chunks == 0) return hipSuccess;
	(void)n_cu;
	hipLaunchKernelGGL(member_chunk_kernel, dim3(n_chunks), dim3(64), 0, st, a, n_chunks);
	return hipGetLastError();
}

hipError_t launch_member_serialize(const MemSerArgs& a, uint32_t n_chunks, uint32_t n_cu, hipStream_t st) {
	if (n_chunks == 0) return hipSuccess;
	const uint32_t waves = std::min<uint32_t>(n_chunks, kSerWavesPerCu * std::max(n_cu, 1u));
	const uint32_t grid = a.v_total ? std::min<uint32_t>(n_chunks, kSerWavesSparse * std::max(n_cu, 1u)) : waves;
	hipLaunchKernelGGL(member_serialize_kernel, dim3(grid), dim3(64), 0, st, a, n_chunks, waves);
	return hipGetLastError();
}

}  // namespace dg
