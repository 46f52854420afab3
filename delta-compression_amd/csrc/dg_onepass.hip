// dg_onepass.hip — onepass differencing on gfx950 (src/c/onepass.c:32-297).
//
// One wave64 per (R, V) pair.  The reference's scan is a chain of *epochs*:
// every match bumps the table version (onepass.c:263), so both hash tables
// are logically empty when an epoch starts and the state between epochs is
// just the cursor pair (v0, r0).  Step t of an epoch looks at the windows
// V[v0+t..+p) and R[r0+t..+p); the reference stores each window's offset into
// HV/HR keeping the first writer of the version (:141-166), then looks R's
// fingerprint up in HV, then V's in HR (:169-219).  Hence:
//
//   lookup 1 at step t: candidate = EARLIEST s <= t with slotV(s) == slotR(t);
//                       match iff V[v0+s..+p) == R[r0+t..+p)   (memcmp, :186)
//   lookup 2 at step t: candidate = EARLIEST s <= t with slotR(s) == slotV(t);
//                       match iff R[r0+s..+p) == V[v0+t..+p)
//   the epoch ends at the first step with a match; the match is extended
//   forward (:229-234) and the next epoch starts at its end.
//
// Equal bytes imply equal fingerprints, so the stored fingerprint test of the
// reference is only a filter here.  Slots are fp mod q exactly as in the
// reference, so collisions — and therefore the output — depend on q the same
// way.
//
// Evaluation per epoch:
//   phase A (p = 16): steps 0..7 at once, 4 lanes per window (most epochs
//                     after a substitution end at step 1);
//   phase B:          64 steps per chunk (lane = step), fingerprints in
//                     parallel, then an in-order walk over the steps with
//                     ballots against the slot history kept in VGPRs
//                     (kHistChunks chunks);
//   phase C:          epochs longer than the register history insert their
//                     (slot -> earliest step) entries into a per-pair table in
//                     HBM tagged with a per-epoch tag (no clearing).
// Bytes come from per-wave LDS windows over V and R (p = 16): both cursors
// only move forward within a pair, so a 4 KiB window per stream is refilled
// with coalesced 16-byte loads every few dozen epochs instead of paying two
// dependent HBM round trips per epoch.  Other seed lengths read HBM/L2
// directly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dg_device.h"
#include "dg_devutil.h"

namespace dg {

// ───────────────────────────── table tier ─────────────────────────────────

__device__ __forceinline__ unsigned long long tab_key(uint32_t tag, uint32_t rel) {
	return ((unsigned long long)tag << 32) | (0xFFFFFFFFu - rel);
}

__device__ __forceinline__ void tab_insert(unsigned long long* t, uint32_t slot, uint32_t tag,
                                           uint32_t rel) {
	if (slot != kSentinel)
		__hip_atomic_fetch_max(t + slot, tab_key(tag, rel), __ATOMIC_RELAXED,
		                       __HIP_MEMORY_SCOPE_AGENT);
}

// earliest step stored in `slot` under `tag` (<= max_rel), else kSentinel.
// Read at the memory side (an atomic no-op max): coherent with the inserts
// whatever XCD last cached the line.
__device__ __forceinline__ uint32_t tab_lookup(unsigned long long* t, uint32_t slot, uint32_t tag,
                                               uint32_t max_rel) {
	if (slot == kSentinel) return kSentinel;
	const unsigned long long e =
	    __hip_atomic_fetch_max(t + slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if ((uint32_t)(e >> 32) != tag) return kSentinel;
	const uint32_t rel = 0xFFFFFFFFu - (uint32_t)e;
	return rel <= max_rel ? rel : kSentinel;
}

// ───────────────────────────── byte sources ───────────────────────────────

// Generic seed length: windows and extensions read HBM/L2 directly.
template <int PF>
struct GlobalSrc {
	static constexpr bool kPhaseA = false;
	const uint8_t* V;
	const uint8_t* R;
	uint32_t p;
	const uint64_t* powc;
	__device__ void chunk(uint64_t, uint64_t, bool) {}
	__device__ uint64_t fpV(uint64_t pos) { return window_fp<PF>(V + pos, p, powc); }
	__device__ uint64_t fpR(uint64_t pos) { return window_fp<PF>(R + pos, p, powc); }
	__device__ uint64_t extend(uint64_t vpos, uint64_t rpos, uint64_t lim) {
		return uni64(extend_fwd(V + vpos, R + rpos, lim));
	}
};

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int kWin = 4096;                 // bytes per stream window
constexpr int kWinStride = kWin + 16;      // + slack for the 2nd dword of rd4

// p = 16: sliding LDS windows over both streams.
struct WinSrc {
	static constexpr bool kPhaseA = true;
	const uint8_t* S[2];     // V, R
	uint64_t len[2];
	int64_t base[2];         // stream offset held at win[s][0] (wave-uniform)
	uint8_t* win;            // LDS, 2 x kWinStride
	const uint64_t* powc;

	// (re)load whichever windows do not cover [lo, lo+need); both streams'
	// loads are issued before either is waited for
	__device__ void ensure2(int64_t vlo, int64_t rlo, int need, bool wantV, bool wantR) {
		const bool fv = wantV && (vlo < base[0] || vlo + need > base[0] + kWin);
		const bool fr = wantR && (rlo < base[1] || rlo + need > base[1] + kWin);
		if (!fv && !fr) return;
		const uint32_t lane = lane_id();
		__syncthreads();   // the wave's reads of the old windows are complete
		// LDS-DMA: lane l's 16 source bytes land at lds + 16*l (lane-linear),
		// no VGPR staging.  The new base keeps every source block 16-byte
		// aligned in memory, so a block holding any stream byte cannot cross
		// a page; blocks wholly outside the stream are skipped (their window
		// bytes are never consumed: every use is bounded by |V| or |R|).
		if (fv) {
			const int64_t nb = vlo - (int64_t)(((uintptr_t)(S[0] + vlo)) & 15);
#pragma unroll
			for (int k = 0; k < kWin / 1024; ++k) {
				const int64_t off = nb + 1024 * k + 16 * lane;
				if (off < (int64_t)len[0] && off + 16 > 0)
					__builtin_amdgcn_global_load_lds((const void*)(S[0] + off),
					                                 (lds_void_t*)(win + 1024 * k), 16, 0, 0);
			}
			base[0] = nb;
		}
		if (fr) {
			const int64_t nb = rlo - (int64_t)(((uintptr_t)(S[1] + rlo)) & 15);
#pragma unroll
			for (int k = 0; k < kWin / 1024; ++k) {
				const int64_t off = nb + 1024 * k + 16 * lane;
				if (off < (int64_t)len[1] && off + 16 > 0)
					__builtin_amdgcn_global_load_lds((const void*)(S[1] + off),
					                                 (lds_void_t*)(win + kWinStride + 1024 * k), 16, 0, 0);
			}
			base[1] = nb;
		}
		vm_drain();        // DMA landed (ordered by vmcnt) ...
		__syncthreads();   // ... and is visible to every lane
	}

	// 4 bytes of stream s at offset x (little-endian), x inside the window
	__device__ __forceinline__ uint32_t rd4(uint32_t s, int64_t x) const {
		const uint32_t i = (uint32_t)(x - (s ? base[1] : base[0]));
		const uint8_t* w = win + (s ? kWinStride : 0) + (i & ~3u);
		const uint32_t w0 = *reinterpret_cast<const uint32_t*>(w);
		const uint32_t w1 = *reinterpret_cast<const uint32_t*>(w + 4);
		return __builtin_amdgcn_alignbyte(w1, w0, i & 3u);
	}

	__device__ __forceinline__ uint64_t fp16(uint32_t s, int64_t x) const {
		uint64_t lo = 0, hi = 0;
#pragma unroll
		for (int g = 0; g < 4; ++g) {
			const uint32_t w = rd4(s, x + 4 * g);
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				const uint64_t c = powc[4 * g + j];
				const uint64_t b = (w >> (8 * j)) & 0xff;
				lo += b * (uint32_t)c;
				hi += b * (uint32_t)(c >> 32);
			}
		}
		return mod_m61(lo + ((hi & ((1ULL << 29) - 1)) << 32) + (hi >> 29));
	}

	// windows for a 64-step chunk starting at (vpos, rpos)
	__device__ void chunk(uint64_t vpos, uint64_t rpos, bool any) {
		if (any) ensure2((int64_t)vpos, (int64_t)rpos, 64 + 16 + 8, vpos < len[0], rpos < len[1]);
	}
	__device__ uint64_t fpV(uint64_t pos) const { return fp16(0, (int64_t)pos); }
	__device__ uint64_t fpR(uint64_t pos) const { return fp16(1, (int64_t)pos); }

	// wave-parallel forward extension (onepass.c:229-234), 256 B per pass
	__device__ uint64_t extend(uint64_t vpos, uint64_t rpos, uint64_t lim) {
		const uint32_t lane = lane_id();
		uint64_t ml = 0;
		while (ml < lim) {
			ensure2((int64_t)(vpos + ml), (int64_t)(rpos + ml), 256 + 8, true, true);
			const uint32_t x = rd4(0, (int64_t)(vpos + ml + 4 * lane)) ^
			                   rd4(1, (int64_t)(rpos + ml + 4 * lane));
			uint32_t fb = x ? ((uint32_t)__builtin_ctz(x) >> 3) : 4u;
			const int64_t rem = (int64_t)lim - (int64_t)(ml + 4 * lane);
			if (rem < (int64_t)fb) fb = rem < 0 ? 0u : (uint32_t)rem;
			const uint64_t m = __ballot(fb < 4);
			if (m) {
				const uint32_t f = ffs64(m);
				return ml + 4ull * f + rdlane(fb, f);
			}
			ml += 256;
		}
		return lim;
	}
};

// ───────────────────────────── kernel ─────────────────────────────────────

template <class Src>
__device__ __forceinline__ void onepass_pair(Src& src, const EncodeArgs& a, uint32_t pair,
                                             const PairDev& pd, const PairPlanDev& pp, uint32_t p,
                                             const uint64_t (&cA)[4]) {
	const uint32_t lane = lane_id();
	const uint64_t rl = pd.r_len, vl = pd.v_len;
	const uint64_t q = pp.q, qmag = pp.q_magic;
	uint32_t* __restrict__ rec = a.rec + 3ull * pp.rec_base;

	uint32_t nrec = 0;
	uint64_t dsz = 26;   // header (25) + END
	int32_t st = 0;

	int32_t tslot = -1;  // table tier state
	uint32_t tag = 0;
	unsigned long long* HV = nullptr;
	unsigned long long* HR = nullptr;

	uint64_t v0 = 0, r0 = 0;
	bool scanning = vl > 0;
	while (scanning) {
		// no match is possible once either stream cannot supply a window at
		// the epoch start (onepass.c:102-104 keeps scanning the other one)
		if (v0 + p > vl || r0 + p > rl) break;

		bool matched = false;
		uint64_t vm = 0, rm = 0, ml = 0;

		// ── phase A: steps 0..7, four lanes per window ──
		if constexpr (Src::kPhaseA) {
			src.ensure2((int64_t)v0, (int64_t)r0, 8 + 16 + 8, true, true);
			const uint32_t side = lane >> 5, w = (lane >> 2) & 7u, part = lane & 3u;
			const uint64_t spos = (side ? r0 : v0) + w;
			const bool valid = spos + 16 <= (side ? rl : vl);
			const uint32_t bytes = src.rd4(side, (int64_t)(spos + 4 * part));
			uint64_t lo = 0, hi = 0;
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				const uint64_t b = (bytes >> (8 * j)) & 0xff;
				lo += b * (uint32_t)cA[j];
				hi += b * (uint32_t)(cA[j] >> 32);
			}
			lo += __shfl_xor(lo, 1, 64);
			hi += __shfl_xor(hi, 1, 64);
			lo += __shfl_xor(lo, 2, 64);
			hi += __shfl_xor(hi, 2, 64);
			const uint64_t fp = mod_m61(lo + ((hi & ((1ULL << 29) - 1)) << 32) + (hi >> 29));
			const uint32_t slot = valid ? (uint32_t)mod_q(fp, q, qmag) : kSentinel;
			const uint32_t fpl = (uint32_t)fp;
			const bool head = part == 0;
			for (uint32_t t = 0; t < 8 && !matched; ++t) {
				const bool ucr = r0 + t + 16 <= rl, ucv = v0 + t + 16 <= vl;
				if (!ucr && !ucv) { scanning = false; break; }
				if (ucr) {
					const uint32_t x = rdlane(slot, 32 + 4 * t), xf = rdlane(fpl, 32 + 4 * t);
					const uint64_t m = __ballot(side == 0 && head && w <= t && slot == x);
					if (m) {
						const uint32_t l = ffs64(m), s = l >> 2;
						if (rdlane(fpl, l) == xf) {
							const uint64_t e = src.extend(v0 + s, r0 + t, min(vl - (v0 + s), rl - (r0 + t)));
							if (e >= 16) { matched = true; vm = v0 + s; rm = r0 + t; ml = e; }
						}
					}
				}
				if (!matched && ucv) {
					const uint32_t x = rdlane(slot, 4 * t), xf = rdlane(fpl, 4 * t);
					const uint64_t m = __ballot(side == 1 && head && w <= t && slot == x);
					if (m) {
						const uint32_t l = ffs64(m), s = (l - 32) >> 2;
						if (rdlane(fpl, l) == xf) {
							const uint64_t e = src.extend(v0 + t, r0 + s, min(vl - (v0 + t), rl - (r0 + s)));
							if (e >= 16) { matched = true; vm = v0 + t; rm = r0 + s; ml = e; }
						}
					}
				}
			}
			if (!scanning) break;
		}

		// ── phases B and C: 64 steps per chunk ──
		uint32_t hsV[kHistChunks], hsR[kHistChunks], hfV[kHistChunks], hfR[kHistChunks];
		bool in_table = false;
		for (uint32_t c = 0; !matched; ++c) {
			const uint64_t step = 64ull * c + lane;
			const uint64_t vp = v0 + step, rp = r0 + step;
			const bool cv = vp + p <= vl;
			const bool cr = rp + p <= rl;
			const uint64_t live = __ballot(cv || cr);
			if (live == 0) { scanning = false; break; }   // both streams exhausted
			const uint32_t nlive = (uint32_t)__popcll(live);
			src.chunk(v0 + 64ull * c, r0 + 64ull * c, true);

			uint64_t fV = 0, fR = 0;
			uint32_t sV = kSentinel, sR = kSentinel;
			if (cv) { fV = src.fpV(vp); sV = (uint32_t)mod_q(fV, q, qmag); }
			if (cr) { fR = src.fpR(rp); sR = (uint32_t)mod_q(fR, q, qmag); }
			const uint32_t fVl = (uint32_t)fV, fRl = (uint32_t)fR;

			if (c < (uint32_t)kHistChunks) {
#pragma unroll
				for (int k = 0; k < kHistChunks; ++k)
					if ((uint32_t)k == c) { hsV[k] = sV; hsR[k] = sR; hfV[k] = fVl; hfR[k] = fRl; }
				// steps a phase-A pass already ruled out are skipped
				const uint32_t j0 = (Src::kPhaseA && c == 0) ? 8u : 0u;
				for (uint32_t j = j0; j < nlive && !matched; ++j) {
					const uint64_t t = 64ull * c + j;
					const bool ucr = r0 + t + p <= rl;
					const bool ucv = v0 + t + p <= vl;
					if (ucr) {
						const uint32_t x = rdlane(sR, j), xf = rdlane(fRl, j);
						uint32_t s = kSentinel, sf = 0;
#pragma unroll
						for (int k = 0; k < kHistChunks; ++k) {
							if (s == kSentinel && (uint32_t)k <= c) {
								uint64_t m = __ballot(hsV[k] == x);
								if ((uint32_t)k == c) m &= mask_le(j);
								if (m) { const uint32_t l = ffs64(m); s = 64u * k + l; sf = rdlane(hfV[k], l); }
							}
						}
						if (s != kSentinel && sf == xf) {
							const uint64_t e = src.extend(v0 + s, r0 + t, min(vl - (v0 + s), rl - (r0 + t)));
							if (e >= p) { matched = true; vm = v0 + s; rm = r0 + t; ml = e; }
						}
					}
					if (!matched && ucv) {
						const uint32_t x = rdlane(sV, j), xf = rdlane(fVl, j);
						uint32_t s = kSentinel, sf = 0;
#pragma unroll
						for (int k = 0; k < kHistChunks; ++k) {
							if (s == kSentinel && (uint32_t)k <= c) {
								uint64_t m = __ballot(hsR[k] == x);
								if ((uint32_t)k == c) m &= mask_le(j);
								if (m) { const uint32_t l = ffs64(m); s = 64u * k + l; sf = rdlane(hfR[k], l); }
							}
						}
						if (s != kSentinel && sf == xf) {
							const uint64_t e = src.extend(v0 + t, r0 + s, min(vl - (v0 + t), rl - (r0 + s)));
							if (e >= p) { matched = true; vm = v0 + t; rm = r0 + s; ml = e; }
						}
					}
				}
			} else {
				// ── phase C: per-pair (tag, earliest step) table in HBM ──
				if (!in_table) {
					in_table = true;
					if (tslot < 0) {
						uint32_t got = 0xFFFFFFFFu;
						if (lane == 0) {   // bounded spin over the pool
							const uint32_t n = a.n_tables;
							for (uint32_t it = 0; it < (1u << 26) && got == 0xFFFFFFFFu; ++it) {
								const uint32_t sl = (pair + it) % n;
								if (atomicCAS(&a.table_locks[sl], 0u, 1u) == 0u) got = sl;
								else if ((it % n) == n - 1) __builtin_amdgcn_s_sleep(8);
							}
						}
						got = rdlane(got, 0);
						if (got == 0xFFFFFFFFu) { st = 5; scanning = false; break; }
						tslot = (int32_t)got;
						HV = a.tables + (uint64_t)got * 2ull * a.qmax;
						HR = HV + a.qmax;
						uint32_t t0 = 0;
						if (lane == 0)
							t0 = __hip_atomic_load(&a.table_tags[got], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						tag = rdlane(t0, 0);
					}
					if (tag == 0xFFFFFFFFu) {   // tag space exhausted: clear the table
						for (uint64_t i = lane; i < 2ull * a.qmax; i += 64)
							__hip_atomic_store(HV + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						vm_drain();
						tag = 0;
					}
					++tag;
#pragma unroll
					for (int k = 0; k < kHistChunks; ++k) {
						tab_insert(HV, hsV[k], tag, 64u * k + lane);
						tab_insert(HR, hsR[k], tag, 64u * k + lane);
					}
				}
				tab_insert(HV, sV, tag, (uint32_t)step);
				tab_insert(HR, sR, tag, (uint32_t)step);
				vm_drain();
				const uint32_t c1 = cr ? tab_lookup(HV, sR, tag, (uint32_t)step) : kSentinel;
				const uint32_t c2 = cv ? tab_lookup(HR, sV, tag, (uint32_t)step) : kSentinel;
				const uint64_t any = __ballot(c1 != kSentinel || c2 != kSentinel);
				for (uint32_t j = 0; j < nlive && !matched && any; ++j) {
					if (!((any >> j) & 1)) continue;
					const uint64_t t = 64ull * c + j;
					const uint32_t s1 = rdlane(c1, j);
					if (s1 != kSentinel) {
						const uint64_t e = src.extend(v0 + s1, r0 + t, min(vl - (v0 + s1), rl - (r0 + t)));
						if (e >= p) { matched = true; vm = v0 + s1; rm = r0 + t; ml = e; }
					}
					const uint32_t s2 = rdlane(c2, j);
					if (!matched && s2 != kSentinel) {
						const uint64_t e = src.extend(v0 + t, r0 + s2, min(vl - (v0 + t), rl - (r0 + s2)));
						if (e >= p) { matched = true; vm = v0 + t; rm = r0 + s2; ml = e; }
					}
				}
			}
		}
		if (!matched) break;

		// emit ADD (implicit gap) + COPY, flush the tables (:243-263)
		if (nrec >= pp.rec_cap) { st = 7; break; }
		if (lane == 0) {
			rec[3u * nrec + 0] = (uint32_t)vm;
			rec[3u * nrec + 1] = (uint32_t)rm;
			rec[3u * nrec + 2] = (uint32_t)ml;
		}
		++nrec;
		dsz += 13 + (vm > v0 ? 9 + (vm - v0) : 0);
		v0 = vm + ml;
		r0 = rm + ml;
	}
	if (v0 < vl) dsz += 9 + (vl - v0);   // trailing ADD (:268-275)

	if (tslot >= 0 && lane == 0) {
		__hip_atomic_store(&a.table_tags[tslot], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		vm_drain();
		__hip_atomic_store(&a.table_locks[tslot], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
	}
	if (lane == 0) {
		a.n_rec[pair] = nrec;
		a.dsize[pair] = dsz;
		a.status[pair] = st;
	}
}

// p = 16, LDS windows (the hot configuration)
__global__ __launch_bounds__(64, 4) void onepass16_kernel(EncodeArgs a) {
	__shared__ __attribute__((aligned(16))) uint8_t win[2 * kWinStride];
	const uint32_t pair = blockIdx.x;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	WinSrc src;
	src.S[0] = a.ver + pd.v_off;
	src.S[1] = a.ref + pd.r_off;
	src.len[0] = pd.v_len;
	src.len[1] = pd.r_len;
	src.base[0] = src.base[1] = INT64_MIN / 2;   // nothing loaded yet
	src.win = win;
	src.powc = a.powc;
	uint64_t cA[4];
	const uint32_t part = lane_id() & 3u;
#pragma unroll
	for (int j = 0; j < 4; ++j) cA[j] = a.powc[4 * part + j];
	onepass_pair(src, a, pair, pd, pp, 16u, cA);
}

// any seed length, bytes from HBM/L2
template <int PF>
__global__ __launch_bounds__(64, 4) void onepass_kernel(EncodeArgs a) {
	const uint32_t pair = blockIdx.x;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	GlobalSrc<PF> src{a.ver + pd.v_off, a.ref + pd.r_off, PF > 0 ? (uint32_t)PF : a.p, a.powc};
	const uint64_t cA[4] = {0, 0, 0, 0};
	onepass_pair(src, a, pair, pd, pp, src.p, cA);
}

// DG_ONEPASS_GLOBAL=1 selects the HBM-direct p=16 kernel (A/B measurements)
static bool getenv_flag_global_src() {
	const char* e = getenv("DG_ONEPASS_GLOBAL");
	return e && e[0] == '1';
}

hipError_t launch_onepass(const EncodeArgs& a, uint32_t p, hipStream_t st) {
	if (a.n_pairs == 0) return hipSuccess;
	if (p == 16 && !getenv_flag_global_src())
		hipLaunchKernelGGL(onepass16_kernel, dim3(a.n_pairs), dim3(64), 0, st, a);
	else if (p == 16)
		hipLaunchKernelGGL(onepass_kernel<16>, dim3(a.n_pairs), dim3(64), 0, st, a);
	else
		hipLaunchKernelGGL(onepass_kernel<0>, dim3(a.n_pairs), dim3(64), 0, st, a);
	return hipGetLastError();
}

}  // namespace dg
