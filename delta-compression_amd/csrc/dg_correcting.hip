// dg_correcting.hip — correcting differencing on gfx950
// (src/c/correcting.c:81-495, hash-table path; restated in oracle/delta_oracle.c
// or_diff_correcting).
//
// Two kernels per batch:
//
//   correcting_build_kernel   the checkpointed R index (correcting.c:164-198).
//       Every R seed a whose fingerprint passes the checkpoint test
//       (fp mod |F|) mod m == k stores itself at slot i = (fp mod |F|) / m
//       when i < cap, FIRST FOUND WINS — i.e. the smallest offset per slot, so
//       the build is an order-free atomicMin over all seeds in parallel.  The
//       grid is (pair, 4 KiB of R); each lane rolls the hash over 16
//       consecutive seeds.  The table stores offsets only: the reference's
//       stored-fingerprint test (`h[i].fp == fp`, :268) is implied by the
//       memcmp that follows it, since equal bytes have equal fingerprints.
//
//   correcting_scan_kernel    the V scan with forward/backward extension and
//       the lookback buffer's tail correction (correcting.c:229-468), one
//       wave64 per pair.  The scan advances one position at a time until a
//       verified match, so a chunk of 64 consecutive positions is tested at
//       once (lane = position) and the first verified lane is the reference's
//       next match.  Extensions are wave-parallel, 16 bytes per lane per
//       step.  The lookback buffer (a ring of buf_cap entries) lives in LDS
//       and is driven by wave-uniform scalar code; entries that leave it are
//       final and become COPY records (ADDs are the gaps between COPYs, as
//       for onepass, so the serialiser is shared).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dg_device.h"
#include "dg_devutil.h"

namespace dg {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kBuildSeedsPerLane = 32;
constexpr uint32_t kBuildBlock = 256;
constexpr uint32_t kBuildSeedsPerBlock = kBuildSeedsPerLane * kBuildBlock;   // 8192


__device__ __forceinline__ uint32_t umin_(uint32_t a, uint32_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint64_t fold61c(uint64_t lo, uint64_t hi) {
	// lo + hi * 2^32 mod (2^61 - 1), lo < 2^48, hi < 2^45
	return mod_m61(lo + ((hi & ((1ULL << 29) - 1)) << 32) + (hi >> 29));
}

// One rolling step (hash.c:62-98) fp' = (fp - out 263^(p-1)) 263 + in
// = fp 263 + nb + in (mod M), with nb = -out 263^p mod M from a table
// (roll_table): with fp = h 2^32 + l (h < 2^29),
//   fp 263 + nb + in = (l 263 + nb_lo + in) + (h 263 + nb_hi) 2^32
// and (h 263 + nb_hi) 2^32 == (.. >> 29) + (.. & (2^29-1)) 2^32, so the sum
// is < 2^62 and one fold plus one subtract make it canonical.  Two 32x32
// multiply-adds instead of the subtract-fold-multiply-fold of the textbook
// form.  fp must be canonical (< M); so is the result.
__device__ __forceinline__ uint64_t roll61(uint64_t fp, uint64_t nb, uint32_t in) {
	const uint64_t plo = (uint64_t)(uint32_t)fp * (uint32_t)kBase + (uint32_t)nb + in;   // < 2^42
	const uint64_t phi = (uint64_t)(uint32_t)(fp >> 32) * (uint32_t)kBase + (nb >> 32);  // < 2^39
	const uint64_t t = plo + ((phi & ((1ULL << 29) - 1)) << 32) + (phi >> 29);           // < 2^61 + 2^43
	const uint64_t r = (t & kMersenne) + (t >> 61);
	return r >= kMersenne ? r - kMersenne : r;
}

// The same step on a weakly reduced fingerprint (any value <= M + 2 with
// the high dword <= 2^29, i.e. the residue plus 0..2 M), for the build's
// unrolled seed loop.  With fp = h 2^32 + l:
//   P = l 263 + nb (one 32x32+64 multiply-add, nb straight from the table),
//   Q = h 263 < 2^39, and Q 2^32 == (Q & (2^29-1)) 2^32 + (Q >> 29),
//   t = P + (Q >> 29) + in + (Q & (2^29-1)) 2^32 < 2^62 + 2^42,
// folded once: (t & M) + (t >> 61) <= M + 2.  The canonical value (the
// checkpoint test needs it, not the next roll) is fp61_canon's.
__device__ __forceinline__ uint64_t roll61w(uint64_t fp, uint64_t nb, uint32_t in) {
	const uint64_t P = (uint64_t)(uint32_t)fp * (uint32_t)kBase + nb;
	const uint64_t Q = (uint64_t)(uint32_t)(fp >> 32) * (uint32_t)kBase;
	const uint32_t s = (uint32_t)(Q >> 29) + in;
	// dword arithmetic with explicit carries (no 64-bit adds of zero-extended
	// halves, which cost a register move each)
	const uint32_t tl = (uint32_t)P + s;
	const uint32_t th = (uint32_t)(P >> 32) + ((uint32_t)Q & 0x1FFFFFFFu) + (tl < s ? 1u : 0u);
	const uint32_t f = th >> 29;
	const uint32_t rl = tl + f;
	const uint32_t rh = (th & 0x1FFFFFFFu) + (rl < f ? 1u : 0u);
	return ((uint64_t)rh << 32) | rl;
}

// roll61w with the leaving byte's term computed instead of looked up: x *
// cneg == -x 263^p (mod M) for cneg = M - 263^p mod M, split into its dwords
// (x cneg_lo < 2^40, x cneg_hi < 2^37), so P < 2^41 and Q < 2^39 and the same
// fold applies.  Two more multiply-adds per step, and no LDS read (with its
// wait, which also waited for the slot atomics issued before it) on the
// rolling chain.
__device__ __forceinline__ uint64_t roll61x(uint64_t fp, uint32_t x, uint32_t cneg_lo, uint32_t cneg_hi, uint32_t in) {
	const uint64_t P = (uint64_t)(uint32_t)fp * (uint32_t)kBase + (uint64_t)x * cneg_lo;
	const uint64_t Q = (uint64_t)(uint32_t)(fp >> 32) * (uint32_t)kBase + (uint64_t)x * cneg_hi;
	const uint32_t s = (uint32_t)(Q >> 29) + in;
	const uint32_t tl = (uint32_t)P + s;
	const uint32_t th = (uint32_t)(P >> 32) + ((uint32_t)Q & 0x1FFFFFFFu) + (tl < s ? 1u : 0u);
	const uint32_t f = th >> 29;
	const uint32_t rl = tl + f;
	const uint32_t rh = (th & 0x1FFFFFFFu) + (rl < f ? 1u : 0u);
	return ((uint64_t)rh << 32) | rl;
}

// r <= M + 2 to [0, M): r - M = r + 1 - 2^61 leaves only the low dword + 1
__device__ __forceinline__ uint64_t fp61_canon(uint64_t r) {
	const bool ge = r >= kMersenne;
	const uint32_t lo = (uint32_t)r + (ge ? 1u : 0u);
	const uint32_t hi = ge ? 0u : (uint32_t)(r >> 32);
	return ((uint64_t)hi << 32) | lo;
}

// x * c mod M for x < 2^61 and c < 2^32
__device__ __forceinline__ uint64_t mulsmall61(uint64_t x, uint32_t c) {
	return fold61c((x & 0xFFFFFFFFull) * c, (x >> 32) * c);
}

// the roll61 table entry of byte x: -x 263^p mod M (c = 263^(p-1) mod M)
__device__ __forceinline__ uint64_t roll_table(uint32_t x, uint64_t c) {
	const uint64_t v = mulsmall61(mulsmall61(c, (uint32_t)kBase), x);   // x 263^p
	return v ? kMersenne - v : 0;
}

// checkpoint class k: fingerprint of V[|V|/2 .. +p) (correcting.c:131-136),
// bytes past |V| read as zero (the reference's out-of-bounds read, see
// oracle/delta_oracle.c), reduced mod |F| then mod m.
__device__ uint64_t checkpoint_class(const uint8_t* V, uint64_t vl, uint32_t p,
                                     const PairPlanDev& pp) {
	if (vl < p) return 0;
	uint64_t h = 0;
	for (uint32_t j = 0; j < p; ++j) {
		const uint64_t at = vl / 2 + j;
		h = mod_m61(mulsmall61(h, (uint32_t)kBase) + (at < vl ? V[at] : 0));
	}
	return mod_q(h, pp.f_size, pp.f_magic) % pp.m;
}

// f = fp mod |F|; passes iff f mod m == k; slot = f / m
__device__ __forceinline__ bool checkpoint_slot(uint64_t fp, const PairPlanDev& pp, uint64_t k,
                                                uint32_t* slot) {
	const uint64_t f = mod_q(fp, pp.f_size, pp.f_magic);
	uint64_t i, r;
	if (pp.m == 1) {
		i = f;
		r = 0;
	} else {
		i = __umul64hi(f, pp.m_magic);
		r = f - i * pp.m;
		if (r >= pp.m) { r -= pp.m; ++i; }
		if (r >= pp.m) { r -= pp.m; ++i; }
	}
	*slot = (uint32_t)i;
	return r == k && i < pp.q;
}

// the checkpoint test alone (f mod m == k), whether or not f / m is a slot
// (--verbose counts it as the reference does, correcting.c:173, 242)
__device__ __forceinline__ bool checkpoint_only(uint64_t fp, const PairPlanDev& pp, uint64_t k, uint64_t* slot) {
	const uint64_t f = mod_q(fp, pp.f_size, pp.f_magic);
	*slot = f / pp.m;
	return f % pp.m == k;
}

// Extensions compare 4 KiB per wave step: 4 chunks of 16 bytes per lane,
// all loads issued before any compare (the byte streams come from HBM/L2,
// so a step is one load latency rather than four).
constexpr int kExtChunks = 4;

// first mismatching byte (0..15) of two 16-byte words, 16 if equal; `back`:
// in back-offset order (the highest address first)
__device__ __forceinline__ uint32_t first_diff16(const uint32_t (&x)[4], bool back) {
	uint32_t bad = 16;
#pragma unroll
	for (int g = 3; g >= 0; --g) {   // later groups first, so the nearest wins
		const uint32_t v = back ? x[3 - g] : x[g];
		if (v) bad = 4u * g + (back ? ((uint32_t)__builtin_clz(v) >> 3) : ((uint32_t)__builtin_ctz(v) >> 3));
	}
	return bad;
}

// Extensions (correcting.c:293-303) in steps of 4 KiB per wave: lane l holds
// bytes [ml + 1024 u + 16 l, +16) of step u (BACK: back-offsets, i.e. the
// bytes a[-(base+16)] .. a[-(base+1)]).  A step's loads are issued apart from
// its compare, so the forward and the backward extension of one match share
// their first round trip.
template <int N>
struct ExtStep {
	uint32_t wa[N][4], wb[N][4];
};

template <bool BACK, int N>
__device__ __forceinline__ void ext_load(const uint8_t* a, const uint8_t* b, uint32_t ml, uint32_t lim, ExtStep<N>& s) {
	const uint32_t lane = lane_id();
#pragma unroll
	for (int u = 0; u < N; ++u) {
		const uint32_t base = ml + 1024u * u + 16 * lane;
		if (base + 16 <= lim) {
			__builtin_memcpy(s.wa[u], BACK ? a - base - 16 : a + base, 16);   // one unaligned 16-byte load
			__builtin_memcpy(s.wb[u], BACK ? b - base - 16 : b + base, 16);
		}
	}
}

// the step's compare: true with *len the extension's length when it ends in
// this step (a mismatch, or lim)
template <bool BACK, int N>
__device__ __forceinline__ bool ext_eval(const uint8_t* a, const uint8_t* b, uint32_t ml, uint32_t lim,
                                         const ExtStep<N>& s, uint32_t* len) {
	const uint32_t lane = lane_id();
	uint32_t bad[N];
#pragma unroll
	for (int u = 0; u < N; ++u) {
		const uint32_t base = ml + 1024u * u + 16 * lane;
		bad[u] = 16;
		if (base + 16 <= lim) {
			const uint32_t x[4] = {s.wa[u][0] ^ s.wb[u][0], s.wa[u][1] ^ s.wb[u][1], s.wa[u][2] ^ s.wb[u][2],
			                       s.wa[u][3] ^ s.wb[u][3]};
			bad[u] = first_diff16(x, BACK);
		} else if (base < lim) {   // the last bytes before lim: no read beyond them
			const uint32_t n = lim - base;
			uint32_t e = n;
			for (uint32_t t = 0; t < n; ++t) {
				const bool ne = BACK ? *(a - (base + t + 1)) != *(b - (base + t + 1)) : a[base + t] != b[base + t];
				if (e == n && ne) e = t;
			}
			bad[u] = e;   // == n when all equal: a mismatch at lim
		}
	}
#pragma unroll
	for (int u = 0; u < N; ++u) {
		const uint64_t m = __ballot(bad[u] < 16);
		if (m) {
			const uint32_t f = ffs64(m);
			*len = umin_(lim, ml + 1024u * u + 16 * f + rdlane(bad[u], f));
			return true;
		}
	}
	if (ml + 1024u * N >= lim) {
		*len = lim;
		return true;
	}
	return false;
}

// the rest of an extension from ml on
template <bool BACK>
__device__ uint32_t ext_from(const uint8_t* a, const uint8_t* b, uint32_t ml, uint32_t lim) {
	uint32_t len = lim;
	while (ml < lim) {
		ExtStep<kExtChunks> s;
		ext_load<BACK>(a, b, ml, lim, s);
		if (ext_eval<BACK>(a, b, ml, lim, s, &len)) return len;
		ml += 1024u * kExtChunks;
	}
	return lim;
}

// both extensions of a seed match: forward a[0..) vs b[0..) up to flim,
// backward a[-1], a[-2], ... vs b[-1], ... up to blim; their first steps
// (kFwdFirst / kBwdFirst KiB) together, loaded with the seed verify of the
// candidates (correcting_scan_kernel), the rest in 4 KiB steps
#ifndef DG_EXT_FWD_FIRST
#define DG_EXT_FWD_FIRST 1
#endif
#ifndef DG_EXT_BWD_FIRST
#define DG_EXT_BWD_FIRST 1
#endif
constexpr int kFwdFirst = DG_EXT_FWD_FIRST, kBwdFirst = DG_EXT_BWD_FIRST;
struct ExtPair {
	ExtStep<kFwdFirst> f;
	ExtStep<kBwdFirst> b;
};

__device__ __forceinline__ void ext_pair_load(const uint8_t* fa, const uint8_t* fb, uint32_t flim, const uint8_t* ba,
                                             const uint8_t* bb, uint32_t blim, ExtPair& e) {
	ext_load<false>(fa, fb, 0, flim, e.f);
	ext_load<true>(ba, bb, 0, blim, e.b);
}

__device__ __forceinline__ void ext_pair_eval(const uint8_t* fa, const uint8_t* fb, uint32_t flim, const uint8_t* ba,
                                             const uint8_t* bb, uint32_t blim, const ExtPair& e, uint32_t* fwd,
                                             uint32_t* bwd) {
	if (blim == 0) *bwd = 0;
	else if (!ext_eval<true>(ba, bb, 0, blim, e.b, bwd)) *bwd = ext_from<true>(ba, bb, 1024u * kBwdFirst, blim);
	if (flim == 0) *fwd = 0;
	else if (!ext_eval<false>(fa, fb, 0, flim, e.f, fwd)) *fwd = ext_from<false>(fa, fb, 1024u * kFwdFirst, flim);
}

__device__ __forceinline__ void ext_both(const uint8_t* fa, const uint8_t* fb, uint32_t flim, const uint8_t* ba,
                                        const uint8_t* bb, uint32_t blim, uint32_t* fwd, uint32_t* bwd) {
	ExtPair e;
	ext_pair_load(fa, fb, flim, ba, bb, blim, e);
	ext_pair_eval(fa, fb, flim, ba, bb, blim, e, fwd, bwd);
}

}  // namespace

// ───────────────────────────── build ──────────────────────────────────────

// checkpoint class of every pair, one thread per pair (the p-byte Horner
// chain is serial; computing it once here keeps it off the build blocks)
__global__ __launch_bounds__(64) void correcting_class_kernel(EncodeArgs a) {
	const uint32_t pair = blockIdx.x * 64 + threadIdx.x;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	a.kcls[pair] = checkpoint_class(a.ver + pd.v_off, pd.v_len, a.p, a.pplan[pair]);
	if (a.stats) a.stats[8ull * pair + 6] = a.kcls[pair];
}

// --verbose only (a.stats): the build's counts, recomputed apart from the
// build kernels so they carry no counters — seeds passing the checkpoint
// test (correcting.c:174) and the slots they filled (first-found policy:
// stored = occupied slots, collisions = passed - stored, :176-196)
__global__ __launch_bounds__(256) void correcting_stats_kernel(EncodeArgs a) {
	const uint32_t pair = blockIdx.x;
	const PairPlanDev pp = a.pplan[pair];
	const PairDev pd = a.pairs[pair];
	const uint32_t p = a.p;
	const uint64_t seeds = pd.r_len >= p ? pd.r_len - p + 1 : 0;
	unsigned long long passed = 0, in_cap = 0, stored = 0;
	if (pd.v_len > 0) {
		const uint64_t k = a.kcls[pair];
		const uint8_t* R = a.ref + pd.r_off;
		for (uint64_t s = threadIdx.x; s < seeds; s += 256) {
			const uint64_t fp = window_fp<0>(R + s, p, a.powc);
			uint64_t slot;
			if (checkpoint_only(fp, pp, k, &slot)) {
				++passed;
				in_cap += slot < pp.q ? 1u : 0u;
			}
		}
		const uint32_t* H = a.ctab + pp.tab_base;
		for (uint64_t i = threadIdx.x; i < pp.q; i += 256) stored += H[i] != kNone ? 1u : 0u;
	}
	if (passed) atomicAdd((unsigned long long*)&a.stats[8ull * pair + 0], passed);
	if (stored) atomicAdd((unsigned long long*)&a.stats[8ull * pair + 1], stored);
	if (in_cap) atomicAdd((unsigned long long*)&a.stats[8ull * pair + 7], in_cap);
}

__global__ __launch_bounds__(kBuildBlock) void correcting_build_kernel(EncodeArgs a, uint32_t nchunk,
                                                                       uint32_t lds_cap) {
	__shared__ uint64_t nb[256];   // roll61 table: -x 263^p mod M for the byte leaving the window
	const uint32_t xcd = blockIdx.x & 7u, i = blockIdx.x >> 3;
	const uint32_t gi = (i / nchunk) * 8u + xcd, chunk = i % nchunk;
	if (gi >= a.n_gpairs) return;   // (only the pairs whose index is too big for LDS)
	const uint32_t pair = a.gpairs[gi];
	const PairPlanDev pp = a.pplan[pair];
	const PairDev pd = a.pairs[pair];
	const uint32_t p = a.p;
	const uint64_t seeds = pd.r_len >= p ? pd.r_len - p + 1 : 0;
	const uint64_t blk0 = (uint64_t)chunk * kBuildSeedsPerBlock;
	if (blk0 >= seeds || pd.v_len == 0) return;
	const uint8_t* R = a.ref + pd.r_off;
	const uint64_t top = a.powc[0];
	nb[threadIdx.x] = roll_table(threadIdx.x, top);
	__syncthreads();
	const uint64_t k = a.kcls[pair];
	uint32_t* H = a.ctab + pp.tab_base;
	const Ckpt ck = make_ckpt(pp.f_size, pp.f_magic, pp.m, k, pp.q);
	auto passes = [&](uint64_t fp, uint32_t* slot) -> bool {
		return ck.mf.ok ? ckpt_test(fp, ck, slot) : checkpoint_slot(fp, pp, k, slot);
	};

	const uint64_t s0 = blk0 + (uint64_t)threadIdx.x * kBuildSeedsPerLane;
	if (s0 >= seeds) return;
	const uint32_t cnt = (uint32_t)(seeds - s0 < kBuildSeedsPerLane ? seeds - s0 : kBuildSeedsPerLane);
	if (p == 16 && cnt == kBuildSeedsPerLane) {
		// the lane's 47 bytes R[s0 .. s0+47) in three (unaligned) 16-byte
		// loads; s0 + 47 <= |R| here, and the 48th byte is read only if it
		// exists
		uint32_t w[12];
		__builtin_memcpy(w, R + s0, 32);
		if (s0 + 48 <= pd.r_len) {
			__builtin_memcpy(w + 8, R + s0 + 32, 16);
		} else {
			__builtin_memcpy(w + 8, R + s0 + 32, 12);
			w[11] = (uint32_t)R[s0 + 44] | ((uint32_t)R[s0 + 45] << 8) | ((uint32_t)R[s0 + 46] << 16);
		}
		auto byte_at = [&](uint32_t i) -> uint32_t { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
		// the first window by byte dot products, the rest by rolling
		uint64_t fp = fp16_dot(w[0], w[1], w[2], w[3]);
#pragma unroll
		for (uint32_t j = 0; j < kBuildSeedsPerLane; ++j) {
			if (j) {   // roll (hash.c:62-98)
				fp = roll61(fp, nb[byte_at(j - 1)], byte_at(j + 15));
			}
			uint32_t slot;
			if (passes(fp, &slot)) atomicMin(&H[slot], (uint32_t)(s0 + j));
		}
		return;
	}
	uint64_t fp = window_fp<0>(R + s0, p, a.powc);
	for (uint32_t j = 0; j < cnt; ++j) {
		if (j) {   // roll: (fp - R[a-1] * 263^(p-1)) * 263 + R[a-1+p]   (hash.c:62-98)
			const uint64_t s = s0 + j;
			fp = roll61(fp, nb[R[s - 1]], R[s - 1 + p]);
		}
		uint32_t slot;
		if (passes(fp, &slot)) atomicMin(&H[slot], (uint32_t)(s0 + j));
	}
}

// The same index built in LDS: one 1024-thread block per pair holds the
// pair's whole table (cap x u32 <= kBuildLdsMaxBytes), so the first-found
// minimum is a ds_min_u32 instead of a memory-side atomic (device-scope
// atomics are not performed in an XCD's L2), and the finished table — empty
// slots included — is written out once with coalesced stores (no memset).
//
// CRC (a.crc_out != nullptr): the block also computes the CRC-64/XZ of R
// (delta.h:294-322) from the bytes its lanes already hold, so correcting
// plans need no separate CRC pass over R.  Iteration k of lane t owns
// R[32 t + 32 Ki k, +32) (bytes past |R| read as zero); the lane folds its
// pieces Horner-wise by x^(8 * 32 Ki) (the context's level-5 nibble table),
// multiplies the result by x^(8 * 32 * (1023 - t)) (the context's per-lane
// constants, bit-serially, once) and the block XOR-reduces.  That is the
// raw CRC of R followed by pad = 32 Ki * iterations - |R| zero bytes; the
// plan's per-pair x^(-8 pad) removes them.  init = ~0 is the first 8 bytes
// XOR-ed with 0xFF (lane 0, iteration 0), xorout the final inversion.
#ifndef DG_CORR_CHAINS   // rolling chains per lane in the LDS build (2 or 4)
#define DG_CORR_CHAINS 2
#endif
constexpr uint32_t kCorrChains = DG_CORR_CHAINS;
static_assert(kCorrChains == 2 || kCorrChains == 4, "chains per lane");
#ifndef DG_CORR_NB_LDS   // 0 (A/B): the leaving byte's term computed (roll61x), measured 1-2 % slower
#define DG_CORR_NB_LDS 1
#endif
constexpr uint32_t kBuildLdsBlock = 1024;
constexpr uint32_t kCrcPiece = kBuildSeedsPerLane;                    // bytes per lane per iteration
constexpr uint32_t kCrcStride = kBuildLdsBlock * kBuildSeedsPerLane;  // 32 KiB per iteration

template <bool CRC>
__global__ __launch_bounds__(kBuildLdsBlock) void correcting_build_lds_kernel(EncodeArgs a, uint32_t lds_cap) {
	extern __shared__ uint32_t T[];
	__shared__ uint64_t nb[256];   // roll61 table
	__shared__ uint64_t CT[CRC ? 5 * 256 : 1];   // slicing-by-4 tables, then x^(8 * 32 Ki) nibbles
	__shared__ uint64_t red[CRC ? kBuildLdsBlock / 64 : 1];
	const uint32_t pair = blockIdx.x;
	const uint32_t tid = threadIdx.x;
	const PairPlanDev pp = a.pplan[pair];
	if (pp.q > lds_cap) return;   // built by correcting_build_kernel
	const PairDev pd = a.pairs[pair];
	const uint32_t cap = (uint32_t)pp.q;
	uint32_t* H = a.ctab + pp.tab_base;
	for (uint32_t i = tid; i < cap; i += kBuildLdsBlock) T[i] = kNone;
	if (tid < 256) nb[tid] = roll_table(tid, a.powc[0]);
	// -263^p mod M as dwords (roll61x); uniform
	[[maybe_unused]] const uint64_t cneg = [&] {
		const uint64_t v = mulsmall61(a.powc[0], (uint32_t)kBase);
		return v ? kMersenne - v : 0ull;
	}();
	[[maybe_unused]] const uint32_t cneg_lo = (uint32_t)cneg, cneg_hi = (uint32_t)(cneg >> 32);
	if constexpr (CRC) {
		for (uint32_t i = tid; i < 4 * 256; i += kBuildLdsBlock) CT[i] = a.crc_tab[i];
		if (tid < 256) CT[4 * 256 + tid] = a.crc_tab[8 * 256 + 5 * kCrcNibTabWords + tid];   // level 5: x^(8*32 Ki)
	}
	__syncthreads();
	const uint32_t p = a.p;
	const uint64_t rl = pd.r_len;
	const uint64_t seeds = rl >= p ? rl - p + 1 : 0;
	const uint8_t* R = a.ref + pd.r_off;
	const bool build = seeds > 0 && pd.v_len > 0;
	uint64_t acc = 0;   // CRC: this lane's Horner fold over its pieces
	const bool crc_wide = CRC && rl >= 64;   // (shorter spans: one thread, byte by byte)
	if (build || crc_wide) {
		const uint64_t k = a.kcls[pair];
		const Ckpt ck = make_ckpt(pp.f_size, pp.f_magic, pp.m, k, pp.q);
		// the checkpoint path is chosen once per pair (uniform), so the
		// unrolled seed loop below has no per-seed branches
		auto run = [&](auto mode) {
			constexpr int kMode = decltype(mode)::value;   // 0: m = 2^s, 1: FP64, 2: Barrett
			auto insert = [&](uint64_t fp, uint32_t off) {
				uint32_t slot;
				bool pass;
				if constexpr (kMode == 0) {
					const uint32_t f = mod_q_small(fp, ck.mf);
					slot = f >> ck.mshift;
					// (slot < cap always: m = ceil(|F| / cap), dg_host.cpp:629)
					pass = (f & ((1u << ck.mshift) - 1u)) == ck.k;
				} else if constexpr (kMode == 1) {
					pass = ckpt_test(fp, ck, &slot);
				} else {
					pass = checkpoint_slot(fp, pp, k, &slot);
				}
				if (pass) __hip_atomic_fetch_min(&T[slot], off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
			};
			// CRC: every lane runs the same number of iterations (the Horner
			// fold), covering every byte of R; the build only the seeds
			const uint64_t lim = crc_wide ? rl : (build ? seeds : 0);
			const uint64_t iters = (lim + kCrcStride - 1) / kCrcStride;
			// a lane's full 32-seed piece (p = 16) is held in registers as
			// R[s0 .. s0+47), the 48th byte only if it exists; the next
			// iteration's piece is loaded before this one is hashed, so with
			// one 1024-thread block per CU the load latency is not exposed
			auto full_piece = [&](uint64_t s0) {
				return p == 16 && build && s0 < seeds && seeds - s0 >= kBuildSeedsPerLane;
			};
			auto fetch = [&](uint64_t s0, uint32_t (&w)[12]) {   // branch-free, so nothing waits on it
				__builtin_memcpy(w, R + s0, 32);
				// bytes 32..47; at the end of R (s0 + 47 == |R|) bytes 31..46,
				// shifted down by the iteration that uses the piece
				__builtin_memcpy(w + 8, R + s0 + (s0 + 48 <= rl ? 32 : 31), 16);
			};
			// one iteration over buffer `w` (already fetched when held), the
			// next iteration's piece prefetched into `nx`; the loop alternates
			// the two buffers, so no register copy waits on the loads
			auto step = [&](uint64_t it, uint32_t (&w)[12], uint32_t (&nx)[12]) -> bool {
				const uint64_t s0 = (uint64_t)tid * kBuildSeedsPerLane + it * kCrcStride;
				if (!CRC && s0 >= seeds) return false;
				const uint32_t cnt = build && s0 < seeds
				                         ? (uint32_t)(seeds - s0 < kBuildSeedsPerLane ? seeds - s0 : kBuildSeedsPerLane)
				                         : 0u;
				const bool held = full_piece(s0);
				if (it + 1 < iters && full_piece(s0 + kCrcStride)) fetch(s0 + kCrcStride, nx);
				if (held) {
					if (s0 + 48 > rl) {
						w[8] = __builtin_amdgcn_alignbit(w[9], w[8], 8);
						w[9] = __builtin_amdgcn_alignbit(w[10], w[9], 8);
						w[10] = __builtin_amdgcn_alignbit(w[11], w[10], 8);
						w[11] >>= 8;
					}
					auto byte_at = [&](uint32_t i) -> uint32_t { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
					if constexpr (kCorrChains == 4) {
						// four independent rolling chains (seeds 0..7, 8..15,
						// 16..23, 24..31): two more direct fingerprints per piece,
						// half the dependent rolls per chain
						uint64_t f[4];
#pragma unroll
						for (uint32_t c = 0; c < 4; ++c) f[c] = fp16_dot(w[2 * c], w[2 * c + 1], w[2 * c + 2], w[2 * c + 3]);
#pragma unroll
						for (uint32_t j = 0; j < kBuildSeedsPerLane / 4; ++j) {
							if (j) {
#pragma unroll
								for (uint32_t c = 0; c < 4; ++c)
									f[c] = roll61w(f[c], nb[byte_at(8 * c + j - 1)], byte_at(8 * c + j + 15));
							}
							if (__ballot(f[0] >= kMersenne || f[1] >= kMersenne || f[2] >= kMersenne || f[3] >= kMersenne)) {
#pragma unroll
								for (uint32_t c = 0; c < 4; ++c) f[c] = fp61_canon(f[c]);
							}
#pragma unroll
							for (uint32_t c = 0; c < 4; ++c) insert(f[c], (uint32_t)(s0 + 8 * c + j));
						}
					} else {
					// two independent rolling chains (seeds 0..15 and 16..31)
					uint64_t fa = fp16_dot(w[0], w[1], w[2], w[3]);
					uint64_t fb = fp16_dot(w[4], w[5], w[6], w[7]);
#pragma unroll
					for (uint32_t j = 0; j < kBuildSeedsPerLane / 2; ++j) {
						if (j) {   // roll (hash.c:62-98), weakly reduced
#if DG_CORR_NB_LDS
							fa = roll61w(fa, nb[byte_at(j - 1)], byte_at(j + 15));
							fb = roll61w(fb, nb[byte_at(j + 15)], byte_at(j + 31));
#else
							fa = roll61x(fa, byte_at(j - 1), cneg_lo, cneg_hi, byte_at(j + 15));
							fb = roll61x(fb, byte_at(j + 15), cneg_lo, cneg_hi, byte_at(j + 31));
#endif
						}
						// a weakly reduced value >= M is ~2^-60 likely: one
						// compare per seed, the subtract only in a wave that has one
						if (__ballot(fa >= kMersenne || fb >= kMersenne)) {
							fa = fp61_canon(fa);
							fb = fp61_canon(fb);
						}
						insert(fa, (uint32_t)(s0 + j));
						insert(fb, (uint32_t)(s0 + 16 + j));
					}
					}
				} else if (cnt) {
					uint64_t fp = window_fp<0>(R + s0, p, a.powc);
					for (uint32_t j = 0; j < cnt; ++j) {
						if (j) {
							const uint64_t s = s0 + j;
							fp = roll61(fp, nb[R[s - 1]], R[s - 1 + p]);
						}
						insert(fp, (uint32_t)(s0 + j));
					}
				}
				if constexpr (CRC) {
					if (!held) {   // the lane's piece near or past the end of R: byte loads, zeros past |R|
						for (uint32_t j = 0; j < 8; ++j) w[j] = 0;
						for (uint32_t j = 0; j < kCrcPiece && s0 + j < rl; ++j) w[j >> 2] |= (uint32_t)R[s0 + j] << (8 * (j & 3));
					}
					if (s0 == 0) {   // init = ~0
						w[0] = ~w[0];
						w[1] = ~w[1];
					}
					uint64_t c = 0;
#pragma unroll
					for (uint32_t j = 0; j < 8; ++j) c = slice4(c, w[j], CT);
					acc = (it ? mul_nib(acc, CT + 4 * 256) : 0ull) ^ c;
				}
				return true;
			};
			uint32_t ba[12], bb[12];
			if (iters && full_piece((uint64_t)tid * kBuildSeedsPerLane)) fetch((uint64_t)tid * kBuildSeedsPerLane, ba);
			for (uint64_t it = 0; it < iters; it += 2) {
				if (!step(it, ba, bb)) break;
				if (it + 1 < iters && !step(it + 1, bb, ba)) break;
			}
		};
		if (ck.mf.ok && ck.mshift >= 0) run(std::integral_constant<int, 0>{});
		else if (ck.mf.ok) run(std::integral_constant<int, 1>{});
		else run(std::integral_constant<int, 2>{});
	}
	if constexpr (CRC) {
		// lane t's fold * x^(8 * 32 * (1023 - t)), XOR over the block
		uint64_t x = crc_wide ? gf2_mulmod(acc, a.crc_k32[kBuildLdsBlock - 1 - tid]) : 0ull;
#pragma unroll
		for (int d = 32; d >= 1; d >>= 1) {
			const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, d, 64);
			const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), d, 64);
			x ^= ((uint64_t)hi << 32) | lo;
		}
		if ((tid & 63) == 0) red[tid >> 6] = x;
	}
	__syncthreads();
	for (uint32_t i = tid; i < cap; i += kBuildLdsBlock) H[i] = T[i];
	if constexpr (CRC) {
		if (tid == 0) {
			uint64_t crc;
			if (crc_wide) {
				uint64_t raw = 0;
				for (uint32_t w2 = 0; w2 < kBuildLdsBlock / 64; ++w2) raw ^= red[w2];
				crc = ~gf2_mulmod(raw, pp.crc_unpad);   // drop the zero padding
			} else {
				uint64_t c = ~0ull;
				for (uint64_t i = 0; i < rl; ++i) c = CT[(uint8_t)(c ^ R[i])] ^ (c >> 8);
				crc = ~c;
			}
			a.crc_out[2ull * pair] = crc;
		}
	}
}

// ───────────────────────────── scan ───────────────────────────────────────

struct RingEnt {
	uint32_t vs, ve, r_off, kind;   // kind: 1 COPY, 2 ADD
};

// waves per SIMD the scan is compiled for: 4 holds one wave per pair of a
// 4096-pair batch resident (DG_SCAN_WAVES=6 leaves room for the CRC, A/B)
#ifndef DG_SCAN_WAVES
#define DG_SCAN_WAVES 4
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DG_SCAN_WAVES, 8))) void correcting_scan_kernel(
    EncodeArgs a) {
	extern __shared__ RingEnt ring[];   // buf_cap + 1 entries
	const uint32_t pair = blockIdx.x;
	const uint32_t lane = lane_id();
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	const uint32_t p = a.p;
	const uint32_t vl = uni((uint32_t)pd.v_len), rl = uni((uint32_t)pd.r_len);
	const uint8_t* V = a.ver + pd.v_off;
	const uint8_t* R = a.ref + pd.r_off;
	const uint32_t* H = a.ctab + pp.tab_base;
	const uint32_t bc = uni(a.buf_cap ? a.buf_cap : 1u);
	const uint32_t rcap = bc + 1;
	const uint32_t rec_cap = uni(pp.rec_cap);
	uint32_t* __restrict__ rec = a.rec + (uint64_t)kRecWordsCorrecting * pp.rec_base;

	uint32_t nrec = 0, head = 0, n = 0;
	uint64_t dsz = 26;   // header + END
	int32_t st = 0;

	// the oldest buffer entry leaves for the output when the buffer is full
	// (correcting.c:319-330, 343-350, 421-428)
	auto emit_oldest_if_full = [&]() {
		if (n >= bc) {
			const RingEnt o = ring[head];
			if (o.kind == 1) {
				if (nrec >= rec_cap) st = 7;
				else if (lane < 3) rec[3u * nrec + lane] = lane == 0 ? o.vs : (lane == 1 ? o.r_off : o.ve - o.vs);
				++nrec;
				dsz += 13;
			} else {
				dsz += 9ull + (o.ve - o.vs);
			}
			head = head + 1 == rcap ? 0 : head + 1;
			--n;
		}
	};
	auto push = [&](uint32_t kind, uint32_t vs_, uint32_t ve_, uint32_t r_off) {
		uint32_t at = head + n;
		if (at >= rcap) at -= rcap;
		__builtin_amdgcn_wave_barrier();
		if (lane == 0) ring[at] = RingEnt{vs_, ve_, r_off, kind};
		__builtin_amdgcn_s_waitcnt(0xc07f);
		__builtin_amdgcn_wave_barrier();
		++n;
	};

	if (vl > 0) {
		const uint64_t k = uni64(a.kcls[pair]);
		const Ckpt ck = make_ckpt(pp.f_size, pp.f_magic, pp.m, k, pp.q);
		uint32_t vc = 0, vs = 0;
		uint64_t n_ck = 0, n_fpm = 0, n_bm = 0, n_match = 0;   // --verbose counters (a.stats)
		while (st == 0 && vc + p <= vl) {
			// ── positions vc .. vc+63: fingerprint, checkpoint, lookup, memcmp ──
			const uint32_t pos = vc + lane;
			const bool in_v = pos + p <= vl;
			bool hit = false, passed = false, fpm = false, bm = false;
			uint32_t off = kNone;
			uint32_t wv[4] = {0, 0, 0, 0};
			uint64_t fp = 0;
			if (in_v) {
				if (p == 16) {   // dot-product fingerprint of the 16 bytes (dg_devutil.h)
					ld16u(V + pos, wv);
					fp = fp16_dot(wv[0], wv[1], wv[2], wv[3]);
				} else {
					fp = window_fp<0>(V + pos, p, a.powc);
				}
				uint32_t slot;
				if (ck.mf.ok ? ckpt_test(fp, ck, &slot) : checkpoint_slot(fp, pp, k, &slot)) {
					passed = true;
					off = H[slot];
				} else if (a.stats) {   // a checkpoint whose f / m is past the table (:242, :268)
					uint64_t sl;
					passed = checkpoint_only(fp, pp, k, &sl);
				}
			}
			const uint64_t C = __ballot(off != kNone);   // candidates, in position order
			// The first candidate is usually the match: its extensions' first
			// steps are loaded together with every candidate's seed bytes, so a
			// verified first candidate costs no round trip of its own.
			ExtPair ex;
			uint32_t vc0 = 0, ro0 = 0;
			if (C) {
				const uint32_t j0 = ffs64(C);
				vc0 = uni(vc + j0);
				ro0 = uni(rdlane(off, j0));
				ext_pair_load(V + vc0 + p, R + ro0 + p, umin_(vl - vc0 - p, rl - ro0 - p), V + vc0, R + ro0,
				              umin_(vc0, ro0), ex);
			}
			if (off != kNone) {   // correcting.c:268-285: verify the seed bytes
				if (p == 16) {
					uint32_t wr[4];
					ld16u(R + off, wr);
					hit = ((wr[0] ^ wv[0]) | (wr[1] ^ wv[1]) | (wr[2] ^ wv[2]) | (wr[3] ^ wv[3])) == 0u;
				} else {
					hit = true;
					for (uint32_t j = 0; j < p && hit; ++j) hit = R[off + j] == V[pos + j];
				}
				if (a.stats && !hit) {   // the reference's stored-fingerprint test (:254-283)
					const bool fpeq = window_fp<0>(R + off, p, a.powc) == fp;
					fpm = !fpeq;
					bm = fpeq;
				}
			}
			const uint64_t M = __ballot(hit);
			if (a.stats) {   // positions the reference visits: up to the first match
				const uint64_t seen = M ? mask_le(ffs64(M)) : ~0ull;
				n_ck += __builtin_popcountll(__ballot(passed) & seen);
				n_fpm += __builtin_popcountll(__ballot(fpm) & seen);
				n_bm += __builtin_popcountll(__ballot(bm) & seen);
				n_match += M ? 1u : 0u;
			}
			if (!M) { vc += 64; continue; }
			const uint32_t jf = ffs64(M);
			vc = uni(vc + jf);
			const uint32_t ro = uni(rdlane(off, jf));
			// ── extensions (correcting.c:293-303) ──
			uint32_t fx, bx;
			const uint32_t flim = umin_(vl - vc - p, rl - ro - p), blim = umin_(vc, ro);
			if (vc == vc0 && ro == ro0) ext_pair_eval(V + vc + p, R + ro + p, flim, V + vc, R + ro, blim, ex, &fx, &bx);
			else ext_both(V + vc + p, R + ro + p, flim, V + vc, R + ro, blim, &fx, &bx);
			const uint32_t fwd = p + uni(fx);
			const uint32_t bwd = uni(bx);
			const uint32_t vm = vc - bwd, rm = ro - bwd, mend = vm + bwd + fwd;
			if (vs <= vm) {
				// 6a: the match lies in the unencoded suffix (correcting.c:316-363)
				if (vs < vm) { emit_oldest_if_full(); push(2, vs, vm, 0); }
				emit_oldest_if_full();
				push(1, vm, mend, rm);
			} else {
				// 6b: tail correction (correcting.c:364-445)
				uint32_t eff = vs;
				while (n > 0) {
					uint32_t at = head + n - 1;
					if (at >= rcap) at -= rcap;
					const RingEnt t = ring[at];
					if (t.vs >= vm && t.ve <= mend) {   // wholly absorbed
						eff = umin_(eff, t.vs);
						--n;
						continue;
					}
					if (t.ve > vm && t.vs < vm && t.kind == 2) {   // trim the ADD
						__builtin_amdgcn_wave_barrier();
						if (lane == 0) ring[at].ve = vm;
						__builtin_amdgcn_s_waitcnt(0xc07f);
						__builtin_amdgcn_wave_barrier();
						eff = umin_(eff, vm);
					}
					break;
				}
				if (mend > eff) {
					emit_oldest_if_full();
					push(1, eff, mend, rm + (eff - vm));
				}
			}
			vs = mend;
			vc = mend;   // correcting.c:448
		}
		// flush the buffer (correcting.c:452-460) and the trailing ADD (:461-468)
		while (n > 0) {
			const RingEnt o = ring[head];
			if (o.kind == 1) {
				if (nrec >= rec_cap) st = 7;
				else if (lane < 3) rec[3u * nrec + lane] = lane == 0 ? o.vs : (lane == 1 ? o.r_off : o.ve - o.vs);
				++nrec;
				dsz += 13;
			} else {
				dsz += 9ull + (o.ve - o.vs);
			}
			head = head + 1 == rcap ? 0 : head + 1;
			--n;
		}
		if (vs < vl) dsz += 9ull + (vl - vs);
		if (a.stats && lane == 0) {
			a.stats[8ull * pair + 2] = n_ck;
			a.stats[8ull * pair + 3] = n_fpm;
			a.stats[8ull * pair + 4] = n_bm;
			a.stats[8ull * pair + 5] = n_match;
		}
	}
	if (lane == 0) {
		a.n_rec[pair] = nrec;
		a.dsize[pair] = dsz;
		a.status[pair] = st;
	}
}

// lds_cap: the largest R index (slots) built in one block's LDS, 0 = none;
// pairs with larger indexes take the memory-atomic build (their tables must
// have been cleared to ~0 by the caller).  qmin/qmax: index sizes in the batch.
// empty slots (~0) in the memory-built pairs' R indexes only (the LDS build
// writes its indexes whole): blockIdx.y = listed pair
__global__ __launch_bounds__(256) void correcting_clear_kernel(EncodeArgs a) {
	const uint32_t pair = a.gpairs[blockIdx.y];
	const PairPlanDev& pp = a.pplan[pair];
	uint32_t* H = a.ctab + pp.tab_base;
	for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < pp.q; i += (uint64_t)gridDim.x * 256) H[i] = kNone;
}

hipError_t launch_correcting_clear(const EncodeArgs& a, hipStream_t st) {
	if (a.n_gpairs == 0) return hipSuccess;
	hipLaunchKernelGGL(correcting_clear_kernel, dim3(16, a.n_gpairs), dim3(256), 0, st, a);
	return hipGetLastError();
}

hipError_t launch_correcting(const EncodeArgs& a, uint32_t p, hipStream_t st, uint32_t lds_cap,
                             uint64_t qmin, hipEvent_t ev_built, hipEvent_t ev_fork) {
	(void)p;
	if (a.n_pairs == 0) return hipSuccess;
	hipLaunchKernelGGL(correcting_class_kernel, dim3((a.n_pairs + 63) / 64), dim3(64), 0, st, a);
	if (lds_cap && qmin <= lds_cap) {
		const size_t tb = 4ull * (a.qmax < lds_cap ? a.qmax : lds_cap);
		if (a.crc_out)
			hipLaunchKernelGGL(correcting_build_lds_kernel<true>, dim3(a.n_pairs), dim3(kBuildLdsBlock), tb, st, a, lds_cap);
		else
			hipLaunchKernelGGL(correcting_build_lds_kernel<false>, dim3(a.n_pairs), dim3(kBuildLdsBlock), tb, st, a, lds_cap);
	}
	if (a.max_seeds && a.n_gpairs) {
		// 1-D grid over the memory-built pairs, XCD-aware: block b runs on
		// XCD b mod 8, which takes the listed pairs == b (mod 8) one after
		// another, all of a pair's chunks in a row, so each XCD's L2 holds the
		// few R indexes its atomics hit
		const uint32_t nchunk = (uint32_t)((a.max_seeds + kBuildSeedsPerBlock - 1) / kBuildSeedsPerBlock);
		const uint64_t blocks = 8ull * ((a.n_gpairs + 7) / 8) * nchunk;
		if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
		hipLaunchKernelGGL(correcting_build_kernel, dim3((uint32_t)blocks), dim3(kBuildBlock), 0, st, a, nchunk, lds_cap);
	}
	if (a.stats) hipLaunchKernelGGL(correcting_stats_kernel, dim3(a.n_pairs), dim3(256), 0, st, a);
	for (hipEvent_t ev : {ev_built, ev_fork}) {
		if (!ev) continue;
		const hipError_t e = hipEventRecord(ev, st);
		if (e != hipSuccess) return e;
	}
	const size_t lds = sizeof(RingEnt) * ((size_t)(a.buf_cap ? a.buf_cap : 1) + 1);
	hipLaunchKernelGGL(correcting_scan_kernel, dim3(a.n_pairs), dim3(64), lds, st, a);
	return hipGetLastError();
}

}  // namespace dg
