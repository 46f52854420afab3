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

#include "dg_device.h"
#include "dg_devutil.h"

namespace dg {

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr uint32_t kStage = kMemChunk + kMemAhead + 16;   // staged bytes per stream (lookbehind 16)
constexpr uint32_t kMaskWords = (kStage + 31) / 32;        // mismatch bitmap words
constexpr uint32_t kRunList = kStage / 17 + 4;             // run starts in the staged region (>= 17 apart)
constexpr uint32_t kLongChunks = 8;                        // members of up to 512 steps are verified
static_assert(kStage % 16 == 0, "16-byte blocks");

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

// Filters of a member set's steps other than their T steps (where V(T) ==
// R(T) by construction): V window hashes, R window hashes, V slots.  A step
// can fail (A) only if its R hash is in the first (or, at T, its V hash in
// the second), and (B) only if the T step's V slot is in the third; the rare
// flagged steps are resolved exactly with ballots.
template <uint32_t W>
struct MemberFilters {
	uint32_t* f;   // 3 x W words
	__device__ void clear() {
		for (uint32_t i = lane_id(); i < 3 * W; i += 64) f[i] = 0u;
	}
	__device__ void add(uint32_t fVl, uint32_t fRl, uint32_t sV) {
		bloom_add<W>(f, fVl);
		bloom_add<W>(f + W, fRl);
		bloom_add<W>(f + 2 * W, sV);
	}
	__device__ bool flagA(uint32_t fVl, uint32_t fRl, bool isT) const {
		return bloom_has<W>(f, fRl) || (isT && bloom_has<W>(f + W, fVl));
	}
	__device__ bool flagB(uint32_t sV) const { return bloom_has<W>(f + 2 * W, sV); }
};

struct ChunkLds {
	uint8_t v[kStage + 16];   // + slack: the fifth dword of a window read
	uint8_t r[kStage + 16];
	uint32_t mask[kMaskWords];
	uint32_t last[kMaskWords];   // max mismatch offset + 1 over words <= j (0: none)
	uint16_t run[kRunList];      // run starts (offsets), ascending
	uint32_t mark[64];
	uint32_t filt[3 * 256];      // member filters: short rounds 3 x 64 words, long members 3 x 256
	uint8_t ok[kMemChunkSlots];  // per member of the chunk: verified
	uint16_t sz[kMemChunkSlots]; // per member: its ADD + COPY bytes in the delta
};

// the 16 bytes at offset o of a staged stream, as little-endian words
__device__ __forceinline__ void win16(const uint8_t* s, uint32_t o, uint32_t (&w)[4]) {
	const uint32_t* d = (const uint32_t*)(s + (o & ~3u));
	const uint32_t sh = o & 3u;
	const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
	w[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
	w[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
	w[2] = __builtin_amdgcn_alignbyte(d3, d2, sh);
	w[3] = __builtin_amdgcn_alignbyte(d4, d3, sh);
}

// An equality-preserving 32-bit hash of a window for check (A): only byte-
// equal windows can make a lookup verify (memcmp, onepass.c:186,212), so
// equal windows must hash equal; unequal ones that collide only make the
// check conservative.  Six VALU ops instead of a second fingerprint.
__device__ __forceinline__ uint32_t win_hash(const uint32_t (&w)[4]) {
	return w[0] ^ __builtin_amdgcn_alignbit(w[1], w[1], 27) ^ __builtin_amdgcn_alignbit(w[2], w[2], 21) ^
	       __builtin_amdgcn_alignbit(w[3], w[3], 15);
}

__device__ __forceinline__ uint64_t fp_lds(const uint8_t* s, uint32_t o, uint32_t& w0) {
	uint32_t w[4];
	win16(s, o, w);
	w0 = w[0];
	return fp16_dot(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(64) void member_chunk_kernel(SpecArgs a) {
	__shared__ __attribute__((aligned(16))) ChunkLds L;
	const uint32_t lane = lane_id();
	const uint2 job = a.chunks[blockIdx.x];   // (pair, chunk)
	const uint32_t pair = job.x, c = job.y;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	const uint32_t vl = uni((uint32_t)pd.v_len), rl = uni((uint32_t)pd.r_len);
	const uint32_t E = umin32(vl, rl);
	const uint32_t cw = c * kMemChunk;                  // chunk start (position)
	const int64_t g0 = (int64_t)cw - 16;                // position of staged offset 0
	const uint64_t slot0 = pp.mem_base + (uint64_t)c * kMemChunkSlots;

	// ── 1. stage [g0, g0 + kStage) of both streams (positions >= 0, < E) ──
	{
		const uint8_t* V = a.ver + pd.v_off;
		const uint8_t* R = a.ref + pd.r_off;
#pragma unroll
		for (uint32_t k = 0; k < (kStage + 1023) / 1024; ++k) {
			const uint32_t o = 1024 * k + 16 * lane;
			const int64_t p = g0 + (int64_t)o;
			if (o < kStage && p >= 0 && p < (int64_t)E) {
				__builtin_amdgcn_global_load_lds((const void*)(V + p), (lds_void_t*)(L.v + 1024 * k), 16, 0, 0);
				__builtin_amdgcn_global_load_lds((const void*)(R + p), (lds_void_t*)(L.r + 1024 * k), 16, 0, 0);
			}
		}
		vm_drain();
		__syncthreads();
	}
	// ── 2. mismatch bitmap: bit o = position g0 + o differs (or is E, the
	//    sentinel); chunk 0's lookbehind holds only the virtual mismatch at -1 ──
	const int64_t lim = (int64_t)E - g0;   // offset of the sentinel
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
		if (in) L.last[j] = lm;
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
	if (lane == 0) a.n_mem[pp.chunk_base + c] = nm;

	const uint64_t q = uni64(pp.q), qmag = uni64(pp.q_magic);
	const ModQ mq = make_modq(q, qmag);
	MemberFilters<64> fs{L.filt};
	MemberFilters<256> fl{L.filt};
	const uint8_t* SV = L.v;
	const uint8_t* SR = L.r;

	for (uint32_t k0 = 0; k0 < nm; k0 += 64) {
		// lane m: member k0 + m (offsets; x = last mismatch before the next
		// run start + 1; a member whose next start is unknown stays unverified)
		const uint32_t k1 = umin32(k0 + 64, nm);
		const uint32_t i = k0 + lane;
		const bool mine = i < k1;
		const uint32_t s = mine ? L.run[i] : 0u;
		const bool known = mine && i + 1 < nrun;
		const uint32_t sn = known ? L.run[i + 1] : 0u;
		uint32_t x = 0;
		if (known) {   // highest mismatch offset below sn, + 1
			const uint32_t j = sn >> 5, b = sn & 31u;
			const uint32_t below = L.mask[j] & ((1u << b) - 1u);
			x = below ? 32 * j + 32u - (uint32_t)__builtin_clz(below) : (j ? L.last[j - 1] : 0u);
		}
		const uint32_t T = x - s;
		const bool shrt = known && T < 64;
		const uint32_t P = wave_incl_scan(shrt ? T + 1 : 0u);   // packed end of each short member
		uint32_t* mem_s = a.mem_s + slot0 + k0;
		uint32_t* srec = a.srec + 4ull * (slot0 + k0);
		if (mine) {
			mem_s[lane] = (uint32_t)(g0 + (int64_t)s);
			L.ok[i] = 0;
			L.sz[i] = (uint16_t)(13u + (T ? 9u + T : 0u));
			if (!known || T >= 64u * kLongChunks)   // unverified: the chain runs its epoch exactly
				*(uint4*)(srec + 4 * lane) = make_uint4(0u, 0u, 0u, 0u);
		}

		// ── short members, packed 64 steps per round (lane = step) ──
		uint32_t done = 0;
		for (;;) {
			const bool in = shrt && P > done && P <= done + 64;
			const uint64_t RM = __ballot(in);
			if (!RM) break;
			const uint32_t hi = 63u - (uint32_t)__builtin_clzll(RM);
			const uint32_t B = rdlane(P, hi) - done;   // live steps of the round
			// lane -> member: a mark at each member's first step, prefix max
			__builtin_amdgcn_wave_barrier();
			L.mark[lane] = 0u;
			fs.clear();
			lds_fence();
			const uint32_t st = P - (T + 1) - done;   // first step lane (members in the round)
			if (in) L.mark[st] = lane + 1u;
			lds_fence();
			const bool live = lane < B;
			const uint32_t mk = wave_incl_max(L.mark[lane]);   // lane 0 always holds a mark
			const uint32_t mj = live ? mk - 1u : 0u;            // member lane
			const uint32_t ms_j = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)s);
			const uint32_t mt_j = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)T);
			const uint32_t fb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)st);
			const uint32_t snj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)sn);
			const uint32_t t = lane - fb;
			const bool isT = live && t == mt_j;
			uint32_t sV = kSentinel, fVl = 0, fRl = 1, w0 = 0;   // (fVl, fRl: window hashes)
			if (live) {
				uint32_t wv[4], wr[4];
				win16(SV, ms_j + t, wv);
				win16(SR, ms_j + t, wr);
				sV = slot_of(fp16_dot(wv[0], wv[1], wv[2], wv[3]), mq, q, qmag);
				fVl = win_hash(wv);
				fRl = win_hash(wr);
				w0 = wv[0];
			}
			if (live && !isT) fs.add(fVl, fRl, sV);
			lds_fence();
			const uint64_t mem = live ? lanes_mask(fb, mt_j + 1) : 0ull;   // this lane's member
			bool bad = false;
			// (A): steps with an off-diagonal equal-window candidate
			for (uint64_t w = __ballot(live && fs.flagA(fVl, fRl, isT)); w; w &= w - 1) {
				const uint32_t Lx = ffs64(w);
				const uint64_t others = ((uint64_t)rdlane((uint32_t)(mem >> 32), Lx) << 32 | rdlane((uint32_t)mem, Lx)) &
				                        ~(1ull << Lx);
				bool hit = (__ballot(fVl == rdlane(fRl, Lx)) & others) != 0;
				if (rdlane(isT ? 1u : 0u, Lx)) hit = hit || (__ballot(fRl == rdlane(fVl, Lx)) & others) != 0;
				bad = bad || (hit && lane == Lx);
			}
			// (B): T steps whose V slot may repeat an earlier V slot of the
			// member; R slots (needed only then) are computed on demand
			uint32_t sR = kSentinel - 1u;
			bool have_sR = false;
			for (uint64_t w = __ballot(isT && fs.flagB(sV)); w; w &= w - 1) {
				const uint32_t Lx = ffs64(w);
				const uint64_t before = ((uint64_t)rdlane((uint32_t)(mem >> 32), Lx) << 32 | rdlane((uint32_t)mem, Lx)) &
				                        ((1ull << Lx) - 1ull);
				const bool d1 = (__ballot(sV == rdlane(sV, Lx)) & before) != 0;
				if (d1 && !have_sR) {
					uint32_t dummy;
					if (live) sR = slot_of(fp_lds(SR, ms_j + t, dummy), mq, q, qmag);
					have_sR = true;
				}
				const bool d2 = d1 && (__ballot(sR == rdlane(sR, Lx)) & before) != 0;
				bad = bad || (d2 && lane == Lx);
			}
			// verdict at each member's T step; the record carries the ADD head
			// (the first step's V window) and the COPY length
			const uint64_t BA = __ballot(bad);
			const uint32_t pw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fb << 2), (int)w0);
			if (isT) {
				const uint32_t xx = (uint32_t)(g0 + (int64_t)(ms_j + mt_j));
				const uint32_t v = (BA & mem) == 0 ? 1u : 0u;
				*(uint4*)(srec + 4 * mj) = make_uint4(xx, snj - (ms_j + mt_j), pw, v);
				L.ok[k0 + mj] = (uint8_t)v;
			}
			done += B;
		}

		// ── long members (64 <= T < 512): 64-step chunks, history in VGPRs ──
		for (uint64_t LM = __ballot(known && !shrt && T < 64u * kLongChunks); LM; LM &= LM - 1) {
			const uint32_t M = ffs64(LM);
			const uint32_t s0 = rdlane(s, M), tl = rdlane(T, M), sn0 = rdlane(sn, M);
			const uint32_t C = tl / 64 + 1;   // chunks
			uint32_t hsV[kLongChunks], hfV[kLongChunks], hfR[kLongChunks];   // V slots, V / R window hashes
			uint32_t pw = 0;
			__builtin_amdgcn_wave_barrier();
			fl.clear();
			lds_fence();
#pragma unroll
			for (uint32_t cc = 0; cc < kLongChunks; ++cc) {
				hsV[cc] = kSentinel;
				hfV[cc] = 0u;
				hfR[cc] = 1u;
				const uint32_t t = 64 * cc + lane;
				if (cc < C && t <= tl) {
					uint32_t wv[4], wr[4];
					win16(SV, s0 + t, wv);
					win16(SR, s0 + t, wr);
					hsV[cc] = slot_of(fp16_dot(wv[0], wv[1], wv[2], wv[3]), mq, q, qmag);
					hfV[cc] = win_hash(wv);
					hfR[cc] = win_hash(wr);
					if (cc == 0) pw = wv[0];
					if (t != tl) fl.add(hfV[cc], hfR[cc], hsV[cc]);
				}
			}
			pw = rdlane(pw, 0);
			lds_fence();
			bool bad = false;
#pragma unroll
			for (uint32_t cc = 0; cc < kLongChunks; ++cc) {
				if (cc < C) {
					const uint32_t t = 64 * cc + lane;
					const bool stp = t <= tl, isT = t == tl;
					// (A)
					for (uint64_t w = __ballot(stp && fl.flagA(hfV[cc], hfR[cc], isT)); w && !bad; w &= w - 1) {
						const uint32_t Lx = ffs64(w);
						const uint32_t fR = rdlane(hfR[cc], Lx), fV = rdlane(hfV[cc], Lx);
						const bool atT = 64 * cc + Lx == tl;
#pragma unroll
						for (uint32_t c2 = 0; c2 < kLongChunks; ++c2) {
							if (c2 < C) {
								const bool other = 64 * c2 + lane <= tl && !(c2 == cc && lane == Lx);
								if (__ballot(other && (hfV[c2] == fR || (atT && hfR[c2] == fV)))) bad = true;
							}
						}
					}
					// (B), R slots recomputed only when the V slot repeats
					if (__ballot(isT && fl.flagB(hsV[cc])) && !bad) {
						const uint32_t LT = tl % 64;
						const uint32_t vT = rdlane(hsV[cc], LT);
						bool d1 = false;
#pragma unroll
						for (uint32_t c2 = 0; c2 < kLongChunks; ++c2) {
							if (c2 <= cc) {
								const uint64_t below = c2 < cc ? ~0ull : ((1ull << LT) - 1ull);
								d1 = d1 || (__ballot(hsV[c2] == vT) & below) != 0;
							}
						}
						if (d1) {
							uint32_t dummy;
							const uint32_t rT = slot_of(fp_lds(SR, s0 + tl, dummy), mq, q, qmag);
							bool d2 = false;
							for (uint32_t c2 = 0; c2 <= cc; ++c2) {
								const uint32_t t2 = 64 * c2 + lane;
								const uint32_t sr2 = t2 < tl ? slot_of(fp_lds(SR, s0 + t2, dummy), mq, q, qmag) : kSentinel;
								d2 = d2 || __ballot(t2 < tl && sr2 == rT) != 0;
							}
							bad = d2;
						}
					}
				}
			}
			if (lane == 0) {
				*(uint4*)(srec + 4 * M) = make_uint4((uint32_t)(g0 + (int64_t)(s0 + tl)), sn0 - (s0 + tl), pw,
				                                     bad ? 0u : 1u);
				L.ok[k0 + M] = bad ? 0u : 1u;
			}
		}
	}
	// ── 5. chunk summary for the chain: the verified prefix and its delta
	//    bytes; the gather map starts empty ──
	lds_fence();
	uint32_t vp = 0, vbytes = 0;
	bool open = true;
	for (uint32_t k0 = 0; k0 < nm && open; k0 += 64) {
		const uint32_t i = k0 + lane;
		const bool v = i < nm && L.ok[i];
		const uint32_t lim2 = umin32(nm - k0, 64u);
		const uint64_t live = lim2 == 64 ? ~0ull : ((1ull << lim2) - 1ull);
		const uint64_t gaps = ~__ballot(v) & live;
		const uint32_t take = gaps ? ffs64(gaps) : lim2;
		const uint32_t b = lane < take ? (uint32_t)L.sz[i] : 0u;
		vbytes += rdlane(wave_incl_scan(b), 63);
		vp += take;
		open = take == lim2;
	}
	if (lane == 0) {
		a.csum[2ull * (pp.chunk_base + c)] = vp;
		a.csum[2ull * (pp.chunk_base + c) + 1] = vbytes;
		*(uint4*)(a.cmap + 4ull * (pp.chunk_base + c)) = make_uint4(0u, 0u, 0u, 0u);
	}
}

// Copies every chunk's taken member records (the chain kernel's map: record
// index, first and end member) into the pair's record array as (x, x, len,
// ADD head) onepass records.
__global__ __launch_bounds__(64) void member_gather_kernel(SpecArgs a, uint32_t* rec) {
	const uint32_t lane = lane_id();
	const uint2 job = a.chunks[blockIdx.x];
	const uint32_t pair = job.x, c = job.y;
	const PairPlanDev pp = a.pplan[pair];
	const uint4 m = *(const uint4*)(a.cmap + 4ull * (pp.chunk_base + c));   // (dst, from, to, -)
	const uint64_t slot0 = pp.mem_base + (uint64_t)c * kMemChunkSlots;
	uint32_t* out = rec + (uint64_t)kRecWordsOnepass * (pp.rec_base + m.x);
	for (uint32_t i = m.y + lane; i < m.z; i += 64) {
		const uint4 r = *(const uint4*)(a.srec + 4ull * (slot0 + i));
		*(uint4*)(out + (uint64_t)kRecWordsOnepass * (i - m.y)) = make_uint4(r.x, r.x, r.y, r.z);
	}
}

hipError_t launch_members(const SpecArgs& a, uint32_t n_chunks, hipStream_t st) {
	if (n_chunks == 0) return hipSuccess;
	hipLaunchKernelGGL(member_chunk_kernel, dim3(n_chunks), dim3(64), 0, st, a);
	return hipGetLastError();
}

hipError_t launch_member_gather(const SpecArgs& a, uint32_t n_chunks, uint32_t* rec, hipStream_t st) {
	if (n_chunks == 0) return hipSuccess;
	hipLaunchKernelGGL(member_gather_kernel, dim3(n_chunks), dim3(64), 0, st, a, rec);
	return hipGetLastError();
}

}  // namespace dg
