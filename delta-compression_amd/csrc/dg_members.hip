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
// is checked per member, independently, so the whole chain is verified in
// parallel instead of walked:
//
//   member_scan_kernel    one wave per pair: coalesced 1 KiB rows of both
//                         streams (16 bytes per lane), mismatch masks, run
//                         starts by a "no mismatch in the 16 bytes before"
//                         test, members (s_k, x_k);
//   member_verify_kernel  kVerifyWaves waves per pair, each taking every
//                         kVerifyWaves-th group of 64 members (no queue, no
//                         atomics); members are packed over the 64 lanes
//                         (lane = step), both windows of every step are
//                         fingerprinted, and each member passes when
//                           (A) no V window of a step equals (low 32
//                               fingerprint bits) an R window of another step
//                               of the member — no lookup before T can verify
//                               (:169-219), and
//                           (B) at T = x - s, slot_V(T) is not among
//                               slot_V(0..T-1) or slot_R(T) is not among
//                               slot_R(0..T-1) — step T is the first writer
//                               its lookup 1 or lookup 2 finds (:141-166),
//                         and writes the member's COPY record (x, x, s_{k+1}
//                         - x, first 4 bytes of its ADD) plus the verdict.
//
// The per-pair chain (onepass16_kernel in member mode, dg_onepass.hip) then
// takes verified members as they are and runs the exact epoch machinery only
// from an unverified member until the chain lands on a later member start,
// and for the final epoch.  oracle/spec_model.c is the CPU model of exactly
// these decisions (tests/test_spec_model.py checks it against the oracle).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dg_device.h"
#include "dg_devutil.h"

namespace dg {

// ───────────────────────────── scan ────────────────────────────────────────

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

// One pass of the scan: 4 rows of 1 KiB of each stream, 16 bytes per lane.
struct ScanPass {
	uint4 v0, v1, v2, v3, r0, r1, r2, r3;
	__device__ __forceinline__ void load(const uint8_t* V, const uint8_t* R, uint32_t pos, uint32_t lastblk) {
		v0 = *(const uint4*)(V + umin32(pos, lastblk));
		r0 = *(const uint4*)(R + umin32(pos, lastblk));
		v1 = *(const uint4*)(V + umin32(pos + 1024, lastblk));
		r1 = *(const uint4*)(R + umin32(pos + 1024, lastblk));
		v2 = *(const uint4*)(V + umin32(pos + 2048, lastblk));
		r2 = *(const uint4*)(R + umin32(pos + 2048, lastblk));
		v3 = *(const uint4*)(V + umin32(pos + 3072, lastblk));
		r3 = *(const uint4*)(R + umin32(pos + 3072, lastblk));
	}
};

// One 1 KiB row: bytes [c0, c0 + 16) of this lane.  Bit i starts a run iff
// no mismatch lies in the 16 bytes before it: inside the chunk by an OR of
// the preceding bits; for the chunk's lowest mismatch by the last mismatch
// of the earlier lanes / rows / passes (prev1, +1).  Run idx's start goes to
// ms[idx] and its predecessor's x (last mismatch + 1) to mx[idx - 1].
__device__ __forceinline__ void scan_row(const uint4& v, const uint4& r, uint32_t c0, uint32_t E, uint32_t lane,
                                         uint32_t& runs, uint32_t& prev1, uint32_t* __restrict__ ms,
                                         uint32_t* __restrict__ mx) {
	uint32_t m = mismatch16(v, r);
	if (c0 + 16 > E) {   // bytes past E do not exist; E itself is the sentinel
		m = E > c0 ? (m & ((1u << (E - c0)) - 1u)) : 0u;
		if (E >= c0) m |= 1u << (E - c0);   // E - c0 < 16
	}
	uint32_t W = m;
	W |= W << 1;
	W |= W << 2;
	W |= W << 4;
	W |= W << 8;
	const uint32_t low = m & (0u - m);
	const uint32_t last1 = m ? c0 + 32u - (uint32_t)__builtin_clz(m) : 0u;
	const uint32_t inc = wave_incl_max(last1);
	const uint32_t before1 = umax32(wave_shr1z(inc), prev1);
	uint32_t rs = m & ~(W << 1) & ~low;
	if (m && c0 + (uint32_t)__builtin_ctz(m) + 1u - before1 > 16u) rs |= low;
	const uint32_t cnt = (uint32_t)__builtin_popcount(rs);
	const uint32_t incl = wave_incl_scan(cnt);
	uint32_t idx = runs + incl - cnt;
	for (uint32_t b = rs; b; b &= b - 1) {
		const uint32_t i = (uint32_t)__builtin_ctz(b);
		const uint32_t below = m & ((1u << i) - 1u);
		++idx;
		ms[idx] = c0 + i;
		mx[idx - 1] = below ? c0 + 32u - (uint32_t)__builtin_clz(below) : before1;
	}
	runs += rdlane(incl, 63);
	prev1 = umax32(prev1, rdlane(inc, 63));
	(void)lane;
}

__global__ __launch_bounds__(64) void member_scan_kernel(SpecArgs a) {
	const uint32_t pair = blockIdx.x;
	if (pair >= a.n_pairs) return;
	const uint32_t lane = lane_id();
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	const uint32_t vl = uni((uint32_t)pd.v_len), rl = uni((uint32_t)pd.r_len);
	const uint32_t E = umin32(vl, rl);
	uint32_t* __restrict__ ms = a.mem_s + pp.rec_base;
	uint32_t* __restrict__ mx = a.mem_x + pp.rec_base;
	const uint8_t* V = a.ver + pd.v_off;
	const uint8_t* R = a.ref + pd.r_off;
	if (lane == 0) ms[0] = 0;   // member 0's epoch starts at 0
	uint32_t runs = 0;          // real runs so far (run 0 holds the virtual mismatch at -1)
	uint32_t prev1 = 0;         // (last mismatch so far) + 1; 0: the virtual one at -1
	if (vl != 0 && E != 0) {   // E = 0: only the sentinel, no run closes
		// passes of 4 coalesced 1 KiB rows (lane l: bytes 16 l .. 16 l + 15
		// of each row); the next pass's loads are in flight while this one
		// is processed.  Rows past E load an in-bounds block (their bits are
		// masked), so the loads carry no branches.
		const uint32_t lastblk = E ? (E - 1) & ~15u : 0u;
		ScanPass cur, nxt;
		cur.load(V, R, 16 * lane, lastblk);
		for (uint32_t o = 0; o <= E; o += 4096) {
			if (o + 4096 <= E) nxt.load(V, R, o + 4096 + 16 * lane, lastblk);
			scan_row(cur.v0, cur.r0, o + 16 * lane, E, lane, runs, prev1, ms, mx);
			if (o + 1024 <= E) scan_row(cur.v1, cur.r1, o + 1024 + 16 * lane, E, lane, runs, prev1, ms, mx);
			if (o + 2048 <= E) scan_row(cur.v2, cur.r2, o + 2048 + 16 * lane, E, lane, runs, prev1, ms, mx);
			if (o + 3072 <= E) scan_row(cur.v3, cur.r3, o + 3072 + 16 * lane, E, lane, runs, prev1, ms, mx);
			cur = nxt;
		}
	}
	// runs closed by a later run are the members; the last run (with the
	// sentinel) starts the final epoch at ms[runs]
	if (lane == 0) a.n_mem[pair] = runs;
}

// ───────────────────────────── verify ──────────────────────────────────────

// 16 bytes at any address as four little-endian words (dg_devutil.h ld16u)
__device__ __forceinline__ uint64_t fp_at(const uint8_t* p, uint32_t& w0) {
	uint32_t w[4];
	ld16u(p, w);
	w0 = w[0];
	return fp16_dot(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint64_t lanes_mask(uint32_t first, uint32_t n) {   // lanes [first, first + n), n >= 1
	return (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << first;
}

constexpr uint32_t kLongChunks = 4;   // members of up to 256 steps are verified here

// Filters of a member set's steps other than their T steps (where V(T) ==
// R(T) by construction): V fingerprints, R fingerprints, V slots.  A step
// can fail (A) only if its R fingerprint is in the first (or, at T, its V
// fingerprint in the second), and (B) only if the T step's V slot is in the
// third; the rare flagged steps are resolved exactly with ballots.
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

__device__ __forceinline__ void lds_fence() {
	__builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
	__builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64) void member_verify_kernel(SpecArgs a) {
	__shared__ uint32_t mark[64];
	__shared__ uint32_t filt[3 * 256];   // short rounds: 3 x 2048 bits; long members: 3 x 8192 bits
	const uint32_t lane = lane_id();
	const uint32_t pair = blockIdx.x / kVerifyWaves, g = blockIdx.x % kVerifyWaves;
	if (pair >= a.n_pairs) return;
	const uint32_t K = uni(a.n_mem[pair]);
	const uint32_t nit = (K + 63) / 64;
	if (g >= nit) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	const uint64_t q = uni64(pp.q), qmag = uni64(pp.q_magic);
	const ModQ mq = make_modq(q, qmag);
	const uint8_t* V = a.ver + pd.v_off;
	const uint8_t* R = a.ref + pd.r_off;
	const uint32_t* ms = a.mem_s + pp.rec_base;
	const uint32_t* mx = a.mem_x + pp.rec_base;
	MemberFilters<64> fs{filt};
	MemberFilters<256> fl{filt};

	for (uint32_t it = g; it < nit; it += kVerifyWaves) {
		const uint32_t k0 = 64 * it, k1 = umin32(k0 + 64, K);
		uint32_t* srec = a.srec + 4ull * (pp.rec_base + k0);
		// lane m: member k0 + m
		const uint32_t nm = k1 - k0;
		const bool mine = lane < nm;
		const uint32_t s = mine ? ms[k0 + lane] : 0u;
		const uint32_t x = mine ? mx[k0 + lane] : 0u;
		const uint32_t snext = mine ? ms[k0 + lane + 1] : 0u;
		const uint32_t T = x - s;
		const bool shrt = mine && T < 64;
		const uint32_t P = wave_incl_scan(shrt ? T + 1 : 0u);   // packed end of each short member

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
			mark[lane] = 0u;
			fs.clear();
			lds_fence();
			const uint32_t st = P - (T + 1) - done;   // first step lane (members in the round)
			if (in) mark[st] = lane + 1u;
			lds_fence();
			const bool live = lane < B;
			const uint32_t mk = wave_incl_max(mark[lane]);   // lane 0 always holds a mark
			const uint32_t mj = live ? mk - 1u : 0u;          // member lane
			const uint32_t ms_j = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)s);
			const uint32_t mt_j = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)T);
			const uint32_t fb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)st);
			const uint32_t sn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(mj << 2), (int)snext);
			const uint32_t t = lane - fb;
			const bool isT = live && t == mt_j;
			uint32_t sV = kSentinel, sR = kSentinel - 1u, fVl = 0, fRl = 1, w0 = 0;
			if (live) {
				uint32_t dummy;
				const uint64_t fV = fp_at(V + ms_j + t, w0);
				const uint64_t fR = fp_at(R + ms_j + t, dummy);
				sV = slot_of(fV, mq, q, qmag);
				sR = slot_of(fR, mq, q, qmag);
				fVl = (uint32_t)fV;
				fRl = (uint32_t)fR;
			}
			if (live && !isT) fs.add(fVl, fRl, sV);
			lds_fence();
			const uint64_t mem = live ? lanes_mask(fb, mt_j + 1) : 0ull;   // this lane's member
			bool bad = false;
			// (A): steps with an off-diagonal fingerprint candidate
			for (uint64_t w = __ballot(live && fs.flagA(fVl, fRl, isT)); w; w &= w - 1) {
				const uint32_t L = ffs64(w);
				const uint64_t others = ((uint64_t)rdlane((uint32_t)(mem >> 32), L) << 32 | rdlane((uint32_t)mem, L)) &
				                        ~(1ull << L);
				bool hit = (__ballot(fVl == rdlane(fRl, L)) & others) != 0;
				if (rdlane(isT ? 1u : 0u, L)) hit = hit || (__ballot(fRl == rdlane(fVl, L)) & others) != 0;
				bad = bad || (hit && lane == L);
			}
			// (B): T steps whose V slot may repeat an earlier V slot of the member
			for (uint64_t w = __ballot(isT && fs.flagB(sV)); w; w &= w - 1) {
				const uint32_t L = ffs64(w);
				const uint64_t before = ((uint64_t)rdlane((uint32_t)(mem >> 32), L) << 32 | rdlane((uint32_t)mem, L)) &
				                        ((1ull << L) - 1ull);
				const bool d1 = (__ballot(sV == rdlane(sV, L)) & before) != 0;
				const bool d2 = d1 && (__ballot(sR == rdlane(sR, L)) & before) != 0;
				bad = bad || (d2 && lane == L);
			}
			// verdict at each member's T step; the record carries the ADD head
			// (the first step's V window) and the COPY length
			const uint64_t BA = __ballot(bad);
			const uint32_t pw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fb << 2), (int)w0);
			if (isT) {
				const uint32_t xx = ms_j + mt_j;
				*(uint4*)(srec + 4 * mj) = make_uint4(xx, sn - xx, pw, (BA & mem) == 0 ? 1u : 0u);
			}
			done += B;
		}

		// ── long members (64 <= T < 256): 64-step chunks, history in VGPRs ──
		for (uint64_t LM = __ballot(mine && !shrt); LM; LM &= LM - 1) {
			const uint32_t M = ffs64(LM);
			const uint32_t s0 = rdlane(s, M), tl = rdlane(T, M), sn = rdlane(snext, M);
			uint32_t ok = 0, pw = 0;
			if (tl < 64u * kLongChunks) {
				const uint32_t C = tl / 64 + 1;   // chunks
				uint32_t hsV[kLongChunks], hsR[kLongChunks], hfV[kLongChunks], hfR[kLongChunks];
				__builtin_amdgcn_wave_barrier();
				fl.clear();
				lds_fence();
#pragma unroll
				for (uint32_t c = 0; c < kLongChunks; ++c) {
					hsV[c] = kSentinel;
					hsR[c] = kSentinel - 1u;
					hfV[c] = 0u;
					hfR[c] = 1u;
					const uint32_t t = 64 * c + lane;
					if (c < C && t <= tl) {
						uint32_t w0, dummy;
						const uint64_t fV = fp_at(V + s0 + t, w0);
						const uint64_t fR = fp_at(R + s0 + t, dummy);
						hsV[c] = slot_of(fV, mq, q, qmag);
						hsR[c] = slot_of(fR, mq, q, qmag);
						hfV[c] = (uint32_t)fV;
						hfR[c] = (uint32_t)fR;
						if (c == 0) pw = w0;
						if (t != tl) fl.add(hfV[c], hfR[c], hsV[c]);
					}
				}
				pw = rdlane(pw, 0);
				lds_fence();
				bool bad = false;
#pragma unroll
				for (uint32_t c = 0; c < kLongChunks; ++c) {
					if (c < C) {
						const uint32_t t = 64 * c + lane;
						const bool stp = t <= tl, isT = t == tl;
						// (A)
						for (uint64_t w = __ballot(stp && fl.flagA(hfV[c], hfR[c], isT)); w && !bad; w &= w - 1) {
							const uint32_t L = ffs64(w);
							const uint32_t fR = rdlane(hfR[c], L), fV = rdlane(hfV[c], L);
							const bool atT = 64 * c + L == tl;
#pragma unroll
							for (uint32_t c2 = 0; c2 < kLongChunks; ++c2) {
								if (c2 < C) {
									const bool other = 64 * c2 + lane <= tl && !(c2 == c && lane == L);
									if (__ballot(other && (hfV[c2] == fR || (atT && hfR[c2] == fV)))) bad = true;
								}
							}
						}
						// (B)
						if (__ballot(isT && fl.flagB(hsV[c])) && !bad) {
							const uint32_t LT = tl % 64;
							const uint32_t vT = rdlane(hsV[c], LT), rT = rdlane(hsR[c], LT);
							bool d1 = false, d2 = false;
#pragma unroll
							for (uint32_t c2 = 0; c2 < kLongChunks; ++c2) {
								if (c2 <= c) {
									const uint64_t below = c2 < c ? ~0ull : ((1ull << LT) - 1ull);
									d1 = d1 || (__ballot(hsV[c2] == vT) & below) != 0;
									d2 = d2 || (__ballot(hsR[c2] == rT) & below) != 0;
								}
							}
							bad = d1 && d2;
						}
					}
				}
				ok = bad ? 0u : 1u;
			}
			if (lane == 0) *(uint4*)(srec + 4 * M) = make_uint4(s0 + tl, sn - (s0 + tl), pw, ok);
		}
	}
}

hipError_t launch_members(const SpecArgs& a, hipStream_t st) {
	if (a.n_pairs == 0) return hipSuccess;
	hipLaunchKernelGGL(member_scan_kernel, dim3(a.n_pairs), dim3(64), 0, st, a);
	hipLaunchKernelGGL(member_verify_kernel, dim3(a.n_pairs * kVerifyWaves), dim3(64), 0, st, a);
	return hipGetLastError();
}

}  // namespace dg
