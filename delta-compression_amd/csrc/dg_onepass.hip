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
// way.  Steps where V (R) has no full window insert nothing
// into HV (HR) and skip lookup 2 (1); the scan ends when neither stream has a
// window left (:102-104).
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
//                     HBM under a per-epoch tag (never cleared).
// Bytes come from per-wave LDS windows over V and R (p = 16, 16-byte aligned
// pairs): both cursors only move forward within a pair, so a 3 KiB window per
// stream (kWin) is refilled by LDS-DMA every few dozen epochs instead of paying two
// dependent HBM round trips per epoch.  Other seed lengths / unaligned pairs
// read HBM/L2 directly.
//
// All cursors are 32-bit (the format caps buffers below 4 GiB) and every
// per-epoch decision is made on wave-uniform values, so the scalar unit — not
// exec-mask juggling — runs the control flow.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dg_crc.h"
#include "dg_device.h"
#include "dg_devutil.h"
#include "dg_serialize_wave.h"

namespace dg {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// ───────────────────────────── profiling build ────────────────────────────
// make -C delta-compression_amd prof  →  lib/libdeltagpu_prof.so with per-wave
// phase counters / cycle totals (scripts/onepass_phases.py).  Compiled out of
// the product library.
#ifdef DG_ONEPASS_PROF
enum { P_EPOCHS, P_DIAG_CALLS, P_DIAG_EPOCHS, P_DIAG_ZERO, P_A_ENTRIES, P_A_MATCH, P_B_ENTRIES,
       P_B_CHUNKS, P_C_CHUNKS, P_EXTENDS, P_REFILLS, P_T_DIAG, P_T_A, P_T_BC, P_T_EXT, P_T_REFILL,
       P_T_TOTAL, P_B_WALKED, P_T_D1, P_T_D2, P_T_D3, P_T_D4, P_D_MEMBERS, P_D_STEPS, P_T_D3A, P_T_D3B,
       P_T_TAKE, P_T_RESYNC, P_TAKES, P_RESYNCS, P_T_FINAL, P_T_C, P_T_B1, P_T_B2, P_T_B3, kProfN };
__device__ unsigned long long g_onepass_prof[kProfN];
constexpr uint32_t kPairProfMax = 16384;   // per pair: start, end (realtime), t_bc, exact epochs
__device__ unsigned long long g_pair_prof[kPairProfMax * 4];
#define PROF_DECL uint64_t prof[kProfN];
#define PROF_INIT(o) for (int _i = 0; _i < kProfN; ++_i) (o).prof[_i] = 0;
#ifdef DG_ONEPASS_PROF_LITE   // only the refill wait, the epoch counts and the total are timed
#define PROF_NOW() 0ull
#define PROF_NOW_R() ((uint64_t)__builtin_amdgcn_s_memtime())
#else
#define PROF_NOW() ((uint64_t)clock64())
#define PROF_NOW_R() ((uint64_t)clock64())
#endif
#define PROF_ADD(o, i, v) ((o).prof[(i)] += (uint64_t)(v))
#else
#define PROF_DECL
#define PROF_INIT(o)
#define PROF_NOW() 0ull
#define PROF_NOW_R() 0ull
#define PROF_ADD(o, i, v) ((void)0)
#endif

#ifdef DG_PAIR_TIME   // variant build: per pair start/end (s_memrealtime, 100 MHz) and placement
constexpr uint32_t kPairTimeMax = 16384;
__device__ unsigned long long g_pair_time[kPairTimeMax * 3];
extern "C" int dg_pair_time_read(unsigned long long* out, int n) {
	if (n > (int)kPairTimeMax) n = (int)kPairTimeMax;
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pair_time), 24ull * n) == hipSuccess ? n : -1;
}
#endif
#ifdef DG_REFILL_PROF   // variant build: refill-wait cycles, refills, pair cycles
__device__ unsigned long long g_refill_prof[3];
extern "C" int dg_refill_prof_read(unsigned long long* out) {
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_refill_prof), 24) == hipSuccess ? 0 : -1;
}
extern "C" int dg_refill_prof_reset(void) {
	unsigned long long z[3] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_refill_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

// ───────────────────────────── small helpers ──────────────────────────────

__device__ __forceinline__ uint64_t quad_sum64(uint64_t x) {
	uint64_t y = ((uint64_t)dpp_xor1((uint32_t)(x >> 32)) << 32) | dpp_xor1((uint32_t)x);
	x += y;
	y = ((uint64_t)dpp_xor2((uint32_t)(x >> 32)) << 32) | dpp_xor2((uint32_t)x);
	return x + y;
}

__device__ __forceinline__ uint64_t fold61(uint64_t lo, uint64_t hi) {
	// lo + hi * 2^32 mod (2^61 - 1), lo < 2^48, hi < 2^45
	return mod_m61(lo + ((hi & ((1ULL << 29) - 1)) << 32) + (hi >> 29));
}

// Bit 8j + g -> bit 4g + j (j < 4, g < 8): the 5-bit index (j1 j0 g2 g1 g0)
// becomes (g2 g1 g0 j1 j0), a rotation done as index-bit swaps (delta swaps).
__device__ __forceinline__ uint32_t delta_swap(uint32_t x, uint32_t mask, uint32_t sh) {
	const uint32_t t = ((x >> sh) ^ x) & mask;
	return x ^ t ^ (t << sh);
}
__device__ __forceinline__ uint32_t mask_transpose_8x4(uint32_t x) {
	// the index-bit 5-cycle 0->2->4->1->3->0 as the swaps (0 2)(0 4)(0 1)(0 3)
	x = delta_swap(x, 0x0A0A0A0Au, 3);
	x = delta_swap(x, 0x0000AAAAu, 15);
	x = delta_swap(x, 0x22222222u, 1);
	x = delta_swap(x, 0x00AA00AAu, 7);
	return x;
}

// ───────────────────────────── table tier ─────────────────────────────────

// A wave waits at most this long (s_memrealtime runs at 100 MHz) for a pool
// table before its pair fails with DG_ERR_TABLE_POOL.
constexpr uint64_t kTableWaitTicks = 20ull * 100000000ull;   // 20 s
constexpr int32_t kStatusTablePool = 11;                     // DG_ERR_TABLE_POOL
constexpr int32_t kStatusInternal = 12;                      // DG_ERR_INTERNAL

// Table = 2 x qmax entries, HV[s] at 2s and HR[s] at 2s + 1: one 16-byte
// load at slot s gives both the lookup of a window whose slot is s and the
// test whether s already has a writer in the window's own table.
// Entry = tag (16 bits) | step (32 bits) | fingerprint bits 0..15 (the
// reference's stored-fingerprint test, onepass.c:180-186, without reading the
// candidate's bytes).  Tags run 1..kTagMax per table; a table whose tags ran
// out is cleared.  No atomics: global atomics execute at the memory side
// (~10x a plain access here); the first writer of a slot is the only writer,
// found from the slot's entry (an earlier chunk) and a duplicate scan of the
// chunk's lanes.
constexpr uint32_t kTagMax = 0xFFFFu;

__device__ __forceinline__ unsigned long long tab_key(uint32_t tag, uint32_t step, uint32_t fp) {
	return ((unsigned long long)tag << 48) | ((unsigned long long)step << 16) | (fp & 0xFFFFu);
}
__device__ __forceinline__ bool tab_cur(unsigned long long e, uint32_t tag) { return (uint32_t)(e >> 48) == tag; }
__device__ __forceinline__ uint32_t tab_step(unsigned long long e) { return (uint32_t)(e >> 16); }
__device__ __forceinline__ bool tab_fpok(unsigned long long e, uint32_t fp) {
	return ((uint32_t)e & 0xFFFFu) == (fp & 0xFFFFu);
}

// The pair (HV[s], HR[s]), read past the L1 (an sc1 load, served by the L2
// that took the stores).  A table is held by one wave at a time, so one XCD's
// L2 sees all of a holding's stores and loads; a holding ends with an
// agent-scope release (L2 write-back) before the lock is freed, so the only
// stale lines another XCD can hold carry older tags, which no lookup accepts.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64x2 tab_load(const unsigned long long* t, uint32_t slot) {
	return __builtin_nontemporal_load((const u64x2*)(t + 2ull * slot));
}

// ───────────────────────────── byte sources ───────────────────────────────

// Any seed length / alignment: windows and extensions read HBM/L2 directly.
template <int PF>
struct GlobalSrc {
	static constexpr bool kPhaseA = false;
	static constexpr uint32_t kBmWords = 64;   // phase-B bitmap: 2048 bits per table
	const uint8_t* V;
	const uint8_t* R;
	uint32_t p;
	const uint64_t* powc;
	__device__ void chunk(uint32_t, uint32_t, bool, bool) {}
	__device__ uint64_t fpV(uint32_t pos) { return window_fp<PF>(V + pos, p, powc); }
	__device__ uint64_t fpR(uint32_t pos) { return window_fp<PF>(R + pos, p, powc); }
	__device__ uint32_t extend(uint32_t vpos, uint32_t rpos, uint32_t lim) {
		return uni((uint32_t)extend_fwd(V + vpos, R + rpos, lim));
	}
};

#ifndef DG_WIN_BYTES      // tuning knobs (make variant); window: a multiple of 16, >= 64 * kLook + 48
#define DG_WIN_BYTES 3072
#endif
#ifndef DG_LOOK_BYTES
#define DG_LOOK_BYTES 32
#endif
#ifndef DG_WAVES_PER_EU
#define DG_WAVES_PER_EU 5
#endif
constexpr uint32_t kWin = DG_WIN_BYTES;     // bytes per stream window (3 KiB: 7.2 KiB LDS per wave, 5 waves/SIMD)
constexpr uint32_t kLook = DG_LOOK_BYTES;   // diagonal batch: lookahead bytes per lane
#ifndef DG_SHORT_T
#define DG_SHORT_T 32
#endif
constexpr uint32_t kShortT = DG_SHORT_T;    // look-back by DPP shifts up to this epoch length
constexpr uint32_t kWinStride = kWin + 16;  // + slack for the 2nd dword of rd4
constexpr uint32_t kListCap = 128;          // mismatch-list entries of a diagonal batch (u16, LDS)
#ifndef DG_BLOOM_BASE
#define DG_BLOOM_BASE 48
#endif
// look-back choice per round: DPP shifts cost ~6 VALU per step of the
// longest member, the Bloom filter a fixed ~kBloomBase plus ~10 per member
constexpr uint32_t kBloomBase = DG_BLOOM_BASE;
#ifndef DG_BACKOFF_MAX
#define DG_BACKOFF_MAX 4
#endif
constexpr uint32_t kBackoffMax = DG_BACKOFF_MAX;   // tier backoff: at most 2^k - 1 epochs skipped
#ifndef DG_DIAG_WINLIM
#define DG_DIAG_WINLIM 0
#endif
#ifndef DG_DIAG_MINSCAN
#define DG_DIAG_MINSCAN 512
#endif
#ifndef DG_REFILL_TOUCH
#define DG_REFILL_TOUCH 0
#endif
#ifndef DG_PRIO_PROGRESS   // issue priority by progress through V (set at each V refill); 0: A/B
#define DG_PRIO_PROGRESS 1
#endif
constexpr bool kPrioProgress = DG_PRIO_PROGRESS != 0;
constexpr uint32_t kTouchAhead = DG_REFILL_TOUCH;   // bytes past a refilled window warmed in the caches
static_assert(kTouchAhead % 128 == 0 && kTouchAhead <= 8192, "one lane per 128-byte line");
constexpr bool kDiagWinLim = DG_DIAG_WINLIM != 0;    // diagonal batch scans what the windows hold first
constexpr uint32_t kDiagMinScan = DG_DIAG_MINSCAN;  // ... when that is at least this many bytes

// p = 16 and 16-byte aligned stream bases: sliding LDS windows.  kCrc: the
// wave also computes both streams' CRC-64/XZ (onepass16_crc_kernel), folding
// the rows its windows hold (crc_fold_window, between epochs).
template <bool kCrc = false>
struct WinSrcT {
	static constexpr bool kPhaseA = true;
	static constexpr uint32_t kBmWords = 128;  // phase-B bitmap: 4096 bits per table (bm[256])
	const uint8_t* S[2];     // V, R (16-byte aligned)
	uint32_t len[2];
	uint32_t base[2];        // stream offset held at win[s][0], multiple of 16
	lds_u8* win;             // LDS (address space 3), 2 x kWinStride
	lds_u8* touch;           // DG_REFILL_TOUCH: 256 bytes of LDS the cache-warming DMA lands in
	const uint64_t* powc;
	// Mismatch list of the diagonal batch (LDS, u16 offsets from lc_base,
	// ascending; the stream end counts as one), made afresh by every call.
	// (Keeping it across calls measured +2.5 % at C3, -6 % at C2: removed.)
	uint16_t* lc;            // kListCap entries
	uint32_t lc_base = 0, lc_n = 0;
	// kCrc: per stream (0 = V, 1 = R) the CRC row fold of dg_crc.h over one
	// segment of crow_n rows of 64 x 8 bytes tiled back from the stream's
	// 16-byte aligned end (row 0 starts cdom <= 0 bytes from the stream's
	// first byte; bytes outside the stream read as zeros), lane l folding
	// piece l of every row into (cy_lo, cy_hi); crow = the next row to fold
	uint32_t crc_tb = 0;     // LDS byte address of the five-bit row tables
	uint32_t cy_lo[2] = {0u, 0u}, cy_hi[2] = {0u, 0u};
	uint32_t crow[2] = {0u, 0u}, crow_n[2] = {0u, 0u};
	int32_t cdom[2] = {0, 0};
	PROF_DECL
#ifdef DG_REFILL_PROF
	uint64_t refill_cycles = 0;
	uint32_t refill_count = 0;
#endif

	// (re)load whichever window does not cover [lo, lo+need); both streams'
	// LDS-DMA requests are in flight before the single wait
	__device__ void ensure2(uint32_t vlo, uint32_t rlo, uint32_t need, bool wantV, bool wantR) {
		const bool fv = wantV && (vlo < base[0] || vlo + need > base[0] + kWin);
		const bool fr = wantR && (rlo < base[1] || rlo + need > base[1] + kWin);
		if (!fv && !fr) return;
		[[maybe_unused]] const uint64_t t0 = PROF_NOW_R();
		const uint32_t lane = lane_id();
		if constexpr (kCrc) {   // (two pairs per block: wave-local ordering only)
			__builtin_amdgcn_s_waitcnt(0xc07f);   // the wave's reads of the old window are complete
			__builtin_amdgcn_wave_barrier();
		} else {
			__syncthreads();   // the wave's reads of the old window are complete
		}
		// lane l's 16 bytes land at lds + 16*l (lane-linear).  Blocks past the
		// stream end are skipped: their window bytes are never consumed, every
		// use being bounded by |V| or |R|; a block holding any stream byte is
		// 16-byte aligned and cannot cross a page.
		if (fv) {
			const uint32_t nb = vlo & ~15u;
#pragma unroll
			for (uint32_t k = 0; k < (kWin + 1023) / 1024; ++k) {
				const uint32_t off = nb + 1024 * k + 16 * lane;
				if (off < len[0] && 1024 * k + 16 * lane < kWin)
					__builtin_amdgcn_global_load_lds((const void*)(S[0] + off),
					                                 (lds_void_t*)(win + 1024 * k), 16, 0, 0);
			}
			base[0] = nb;
		}
		if (fr) {
			const uint32_t nb = rlo & ~15u;
#pragma unroll
			for (uint32_t k = 0; k < (kWin + 1023) / 1024; ++k) {
				const uint32_t off = nb + 1024 * k + 16 * lane;
				if (off < len[1] && 1024 * k + 16 * lane < kWin)
					__builtin_amdgcn_global_load_lds((const void*)(S[1] + off),
					                                 (lds_void_t*)(win + kWinStride + 1024 * k), 16, 0, 0);
			}
			base[1] = nb;
		}
#ifdef DG_REFILL_PROF
		const uint64_t tr0 = __builtin_amdgcn_s_memtime();
#endif
		vm_drain();        // the DMA landed (ordered by vmcnt) ...
		if constexpr (kCrc) {
			__builtin_amdgcn_wave_barrier();   // ... and is visible to every lane of the wave
		} else {
			__syncthreads();   // ... and is visible to every lane
		}
#ifdef DG_REFILL_PROF
		refill_cycles += __builtin_amdgcn_s_memtime() - tr0;
		++refill_count;
#endif
		if constexpr (kTouchAhead > 0) {
			// warm the caches for the next refill: one dword per 128-byte line
			// of the kTouchAhead bytes past each refilled window, by LDS-DMA into
			// a dummy area (nothing waits for it: the next refill's own loads are
			// issued after it, and vmcnt drains in order)
			const uint32_t lanes = kTouchAhead / 128;
			if (lane < lanes) {
				if (fv) {
					const uint32_t off = base[0] + kWin + 128 * lane;
					if (off < len[0]) __builtin_amdgcn_global_load_lds((const void*)(S[0] + off), (lds_void_t*)touch, 4, 0, 0);
				}
				if (fr) {
					const uint32_t off = base[1] + kWin + 128 * lane;
					if (off < len[1]) __builtin_amdgcn_global_load_lds((const void*)(S[1] + off), (lds_void_t*)touch, 4, 0, 0);
				}
			}
		}
		if constexpr (kPrioProgress) {
			// issue priority by progress through V: a wave behind the others
			// on its SIMD outranks them, so the SIMD's waves finish together
			// instead of oldest first (C2 per-pair durations p10..max 166..244
			// -> 185..232 us, c3s_chain +4 %: profiles/r06_experiments.md)
			if (fv) {
				const uint64_t b4 = 4ull * base[0], l = len[0];
				if (b4 < l) __builtin_amdgcn_s_setprio(3);
				else if (b4 < 2 * l) __builtin_amdgcn_s_setprio(2);
				else if (b4 < 3 * l) __builtin_amdgcn_s_setprio(1);
				else __builtin_amdgcn_s_setprio(0);
			}
		}
		PROF_ADD(*this, P_REFILLS, 1);
		PROF_ADD(*this, P_T_REFILL, PROF_NOW_R() - t0);
	}

	// ── kCrc: the streams' CRC-64/XZ (delta.h:294-322) by the row fold of
	//    dg_crc.h, with the five-bit tables at crc_tb ──
	__device__ void crc_init(uint32_t tb) {
		crc_tb = tb;
#pragma unroll
		for (uint32_t s = 0; s < 2; ++s) {
			const uint32_t a1 = (len[s] + 15u) & ~15u;   // (|stream| < 4 GiB - 16)
			crow_n[s] = (a1 + 511u) / 512u;
			cdom[s] = (int32_t)(a1 - 512u * crow_n[s]);   // in (-512, 0]
		}
	}
	// fold one row's pieces (lane l: the 8 bytes at stream offset o, zeros
	// outside the stream, init = ~0 XOR-ed into the first 8 bytes)
	__device__ __forceinline__ void crc_fold_piece(uint32_t s, int32_t o, uint64_t x) {
		const uint32_t L = len[s];
		if (o < 0 || (uint32_t)o >= L) x = 0ull;
		else if ((uint32_t)o + 8u > L) x &= byte_mask(0, (int)(L - (uint32_t)o));   // past the end
		if (o == 0) x = ~x;                                                          // init (|stream| >= 8)
		crc_fold<kCrcFive, 8, 1>(cy_lo[s], cy_hi[s], 0u, 0u, (uint32_t)x, (uint32_t)(x >> 32), crc_tb, crc_tb);
	}
	// fold stream s's next rows while the window holds them (LDS reads);
	// a row that started before the window (the window jumped past it) from
	// memory; stops at the first row that reaches past the window, or past
	// lim rows.  The window's bytes are the stream's (read-only) bytes, so
	// any row inside it may be folded, ahead of the chain or behind it.
	__device__ void crc_fold_window(uint32_t s, uint32_t lim) {
		if (base[s] == 0xFFFF0000u) return;   // nothing loaded yet
		const uint32_t lane = lane_id();
		const uint32_t L = len[s];
		const uint32_t wend = umin32(base[s] + kWin, L);   // window bytes that are stream bytes
		const uint32_t stop = umin32(crow_n[s], lim);
		while (crow[s] < stop) {
			const int32_t rs = cdom[s] + (int32_t)(512u * crow[s]);
			const int32_t o = rs + (int32_t)(8u * lane);
			const uint32_t re = umin32((uint32_t)(rs + 512), L);   // (rs + 512 > 0)
			if (re > wend) break;   // reaches past the window: a later call
			uint64_t x = 0ull;
			if (rs >= (int32_t)base[s] || (rs < 0 && base[s] == 0u)) {
				if (o >= (int32_t)base[s] && (uint32_t)o < L) {
					const lds_u32* w = (const lds_u32*)(win + (s ? kWinStride : 0) + ((uint32_t)o - base[s]));
					x = ((uint64_t)w[1] << 32) | w[0];
				}
			} else if (o >= 0 && (uint32_t)o < L) {   // (the window moved past the row's start)
				const uint2 g = *reinterpret_cast<const uint2*>(S[s] + o);
				x = ((uint64_t)g.y << 32) | g.x;
			}
			crc_fold_piece(s, o, x);
			++crow[s];
		}
	}
	// between epochs (the chain's registers are few there): the rows the
	// windows hold
	__device__ __forceinline__ void crc_step() {
		if constexpr (kCrc) {
			crc_fold_window(0, 0xFFFFFFFFu);
			crc_fold_window(1, 0xFFFFFFFFu);
		}
	}
	// the rows no window held whole (the streams' ends, long jumps), from memory
	__device__ void crc_fold_rest(uint32_t s) {
		const uint32_t lane = lane_id();
		const uint32_t L = len[s];
		for (; crow[s] < crow_n[s]; ++crow[s]) {
			const int32_t o = cdom[s] + (int32_t)(512u * crow[s] + 8u * lane);
			uint64_t x = 0ull;
			if (o >= 0 && (uint32_t)o < L) {
				const uint2 g = *reinterpret_cast<const uint2*>(S[s] + o);
				x = ((uint64_t)g.y << 32) | g.x;
			}
			crc_fold_piece(s, o, x);
		}
	}
	// stream s's CRC-64/XZ (uniform): the remaining rows, the last row's
	// advance, the per-lane x^(-64 l), the wave XOR, the end pad undone
	__device__ uint64_t crc_final(uint32_t s, const uint64_t* tabs) {
		const uint32_t L = len[s];
		if (L < 8) {   // byte by byte (crc_finalize_kernel's short path)
			uint64_t c = ~0ull;
			for (uint32_t k = 0; k < L; ++k) c = tabs[(uint8_t)(c ^ S[s][k])] ^ (c >> 8);
			return ~c;
		}
		crc_fold_window(s, 0xFFFFFFFFu);
		crc_fold_rest(s);
		crc_fold<kCrcFive, 8, 1>(cy_lo[s], cy_hi[s], 0u, 0u, 0u, 0u, crc_tb, crc_tb);
		const uint64_t A = ((uint64_t)cy_hi[s] << 32) | cy_lo[s];
		uint64_t acc = wave_xor64(A ? gf2_mulmod(A, tabs[kCrcRowK8 + lane_id()]) : 0ull);
		const uint32_t t = ((L + 15u) & ~15u) - L;
		if (t) acc = mul_nib(acc, tabs + 8 * 256 + kCrcLevels * kCrcNibTabWords + (1 + t) * kCrcNibTabWords);   // x^(-8t)
		return ~acc;
	}

	// 4 bytes of stream s at offset x (little-endian), x inside the window
	__device__ __forceinline__ uint32_t rd4(uint32_t s, uint32_t x) const {
		const uint32_t i = x - (s ? base[1] : base[0]);
		const lds_u32* w = (const lds_u32*)(win + (s ? kWinStride : 0) + (i & ~3u));
		const uint32_t w0 = w[0];
		const uint32_t w1 = w[1];
		return __builtin_amdgcn_alignbyte(w1, w0, i & 3u);
	}

	// the 8 words at stream offset x .. x+31 (x - window base: the same value
	// mod 16 in every lane)
	template <uint32_t Q>
	__device__ __forceinline__ static void pick8(const uint32_t (&d)[12], uint32_t r, uint32_t (&w)[8]) {
#pragma unroll
		for (uint32_t k = 0; k < 8; ++k) w[k] = __builtin_amdgcn_alignbyte(d[Q + k + 1], d[Q + k], r);
	}
	__device__ __forceinline__ void lane_words32(uint32_t s, uint32_t x, uint32_t (&w)[8]) const {
		const uint32_t i = x - (s ? base[1] : base[0]);
		typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
		typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
		const lds_u32x4* p = (const lds_u32x4*)(win + (s ? kWinStride : 0) + (i & ~15u));
		const u32x4 a = p[0], b = p[1], c = p[2];
		const uint32_t d[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
		const uint32_t o = uni(i & 15u), r = o & 3u;
		switch (o >> 2) {
		case 0: pick8<0>(d, r, w); break;
		case 1: pick8<1>(d, r, w); break;
		case 2: pick8<2>(d, r, w); break;
		default: pick8<3>(d, r, w); break;
		}
	}

	__device__ __forceinline__ uint64_t fp16(uint32_t s, uint32_t x) const {
		// the window's 16 bytes as one unaligned ds_read_b128 (gfx950 runs with
		// unaligned LDS access) instead of eight dword reads and four
		// alignbytes: C2 1721 -> 1732 GiB/s over 4 x 100 steps on one box
		typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
		typedef __attribute__((address_space(3))) const u32x4u lds_u32x4u;
		const uint32_t i = x - (s ? base[1] : base[0]);
		const u32x4u w = *(lds_u32x4u*)(win + (s ? kWinStride : 0) + i);
		return fp16_dot(w.x, w.y, w.z, w.w);
	}

	// windows for a 64-step chunk starting at (vpos, rpos)
	__device__ void chunk(uint32_t vpos, uint32_t rpos, bool wantV, bool wantR) {
		ensure2(vpos, rpos, 64 + 16 + 8, wantV, wantR);
	}
	__device__ uint64_t fpV(uint32_t pos) const { return fp16(0, pos); }
	__device__ uint64_t fpR(uint32_t pos) const { return fp16(1, pos); }

	// ── diagonal batch ──────────────────────────────────────────────────
	// State (v0, r0) sits on a mismatch (V[v0] != R[r0]) left by the previous
	// extension.  Let a_0 = 0 < a_1 < ... be the mismatch offsets along the
	// diagonal within the next 64 * kLook bytes (the end of the shorter stream counts as
	// one).  An epoch starting at a_k first sees equal windows at step
	//   T_k = a_m + 1 - a_k,  m = the first index >= k with a_{m+1} - a_m > p,
	// and, if it resolves there on the diagonal, emits ADD(T_k bytes) +
	// COPY(a_k + T_k .. a_{m+1}) and hands over to the epoch at a_{m+1}.  The
	// chain of such epochs is laid out over the lanes (one lane per step of
	// each epoch, at most 64 steps in all) and each epoch is checked exactly
	// against the reference's lookups (onepass.c:169-219):
	//   step t < T_k:  neither lookup may verify.  The diagonal candidate
	//                  (s = t) differs in its bytes by construction; an earlier
	//                  candidate (s < t) must differ in its fingerprint —
	//                  equal fingerprints (a possible genuine match elsewhere)
	//                  end the batch and the exact path takes the epoch;
	//   step T_k:      lookup 1 must find s = T_k, or fail on the fingerprint
	//                  with lookup 2 then finding s = T_k.
	// "Earliest s" is the reference's first-writer slot (HV/HR hold the first
	// step of the epoch that hashed to the slot).  The epochs before the first
	// one that fails the check are committed.  Returns (all wave-uniform, by
	// value so nothing goes through scratch): the number committed, adv =
	// offset of the new state, more = the batch ended only because the chain
	// left the known region (another batch can follow directly), dadd = their
	// delta bytes, long_first = 1: nothing was committed because the first
	// epoch's diagonal step is past 63 (phase A cannot resolve it on the
	// diagonal: the caller starts phase B at step 0); 2: a scan truncated to
	// the windows found no member (the caller runs the batch again in full).
	struct DiagOut {
		uint32_t committed, adv, more, dadd, long_first;
	};
	__device__ DiagOut diag_batch(uint32_t v0, uint32_t r0, uint32_t vl, uint32_t rl, uint64_t q,
	                              uint64_t qmag, const ModQ& mq, uint32_t p, uint32_t* rec, uint32_t nrec,
	                              uint32_t rec_cap, uint32_t* mlist, bool full_scan) {
		const uint32_t lane = lane_id();
		const uint32_t lim = umin32(vl - v0, rl - r0);
		if (lim < p + 1) return DiagOut{0, 0, 0, 0, 0};
		[[maybe_unused]] uint64_t tq = PROF_NOW();
		// 1. the list of mismatch offsets from v0, over `scan` bytes.  With
		// DG_DIAG_WINLIM the batch first scans only what both windows already
		// hold from (v0, r0) when that is at least kDiagMinScan bytes, so a
		// window is refilled when the chain nears its end instead of whenever
		// less than the full look-ahead is left (fewer refills, less overlap
		// re-read); a truncated scan that yields no member returns long_first
		// = 2 and the caller runs the batch again in full (full_scan).
		uint32_t scan = 64 * kLook;
		bool trunc = false;
		if (kDiagWinLim && !full_scan) {
			const uint32_t hv = v0 - base[0] < kWin ? base[0] + kWin - v0 : 0u;
			const uint32_t hr = r0 - base[1] < kWin ? base[1] + kWin - r0 : 0u;
			const uint32_t have = umin32(hv, hr);
			if (have < 64 * kLook + 48 && have >= kDiagMinScan + 48) {
				scan = (have - 48) & ~(kLook - 1u);
				trunc = true;
			}
		}
		if (!trunc) ensure2(v0, r0, 64 * kLook + 48, true, true);
		{
			// mismatch bits of offsets [kLook*lane, kLook*lane + kLook)
			const uint32_t base = kLook * lane;
			const bool inscan = base < scan;   // (scan is a multiple of kLook)
			// The lane's 32 bytes of each stream come in as three ds_read_b128 from
			// the 16-byte-aligned address below them (2-way bank conflicts; word
			// reads at a 32-byte lane stride are 8-way).  The offset inside the
			// 16 bytes is wave-uniform (windows and lane chunks are 16-aligned),
			// so picking the 8 words is a uniform switch plus alignbytes.
			static_assert(kLook == 32, "one 32-bit mask per lane, 16-byte-aligned lane chunks");
			uint32_t wv[8], wr[8];
			lane_words32(0, v0 + (inscan ? base : 0u), wv);
			lane_words32(1, r0 + (inscan ? base : 0u), wr);
			// byte j of word g first lands at bit 8j + g (one shift-and-or per
			// word), then a 5-bit index rotation (four delta swaps) moves it to
			// bit 4g + j, i.e. offset order
			uint32_t bits = 0;
#pragma unroll
			for (uint32_t g = 0; g < 8; ++g) {
				const uint32_t x = wv[g] ^ wr[g];
				const uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;   // bit 8j+7: byte j != 0
				bits |= (t >> (7 - g)) & (0x01010101u << g);
			}
			bits = mask_transpose_8x4(bits);
			if (!inscan) {
				bits = 0u;   // not scanned: unknown, not a terminator
			} else if (base + kLook > lim) {   // past the shorter stream: only its end terminates a match
				bits = lim > base ? (bits & ((1u << (lim - base)) - 1u)) : 0u;
				if (lim >= base && lim < base + kLook) bits |= 1u << (lim - base);
			}
			// ordered list (exclusive prefix of counts), at most kListCap entries
			const uint32_t cnt = (uint32_t)__builtin_popcount(bits);
			const uint32_t incl = wave_incl_scan(cnt);
			uint32_t pos = incl - cnt;
			const uint32_t total = rdlane(incl, 63);
			for (uint32_t b = bits; b && pos < kListCap; b &= b - 1, ++pos) lc[pos] = (uint16_t)(base + __builtin_ctz(b));
			lc_n = umin32(total, kListCap);
			lc_base = v0;
			__builtin_amdgcn_s_waitcnt(0xc07f);
			__builtin_amdgcn_wave_barrier();
		}
		const uint32_t K = umin32(lc_n, 64u);
		if (K < 2) return DiagOut{0, 0, 0, 0, trunc ? 2u : 0u};
		{
			// the window must hold every byte the batch's steps read
			const uint32_t last = (uint32_t)lc[K - 1];
			ensure2(v0, r0, last + 16 + 8, true, true);
		}
		PROF_ADD(*this, P_T_D1, PROF_NOW() - tq);
		tq = PROF_NOW();
		const uint32_t ak = lane < K ? (uint32_t)lc[lane] : 0xFFFFFFFFu;
		const uint32_t an = lane + 1 < K ? (uint32_t)lc[lane + 1] : 0xFFFFFFFFu;
		const bool gap = lane + 1 < K && an - ak > p;   // a long gap follows a_lane
		const uint64_t G = __ballot(gap);
		// 3. the chain of epochs.  From a_0 the chain visits exactly the
		//    mismatches that follow a long gap: member r starts right after
		//    the (r-1)-th long gap and ends (first equal step) at the r-th,
		//    whose lane k computes it.  Members are laid out over the lanes in
		//    order, T + 1 steps each, while they fit in 64 lanes and T < 64.
		const uint64_t gbelow = G & ((1ull << lane) - 1ull);
		const uint32_t sidx = gbelow ? 64u - (uint32_t)__builtin_clzll(gbelow) : 0u;
		const uint32_t astart = (uint32_t)lc[sidx];   // sidx <= lane < K
		const uint32_t T = gap ? ak + 1 - astart : 0u;
		const uint64_t tooLong = __ballot(gap && T > 63);
		const uint32_t kb = tooLong ? ffs64(tooLong) : 64u;
		const bool cand = gap && lane < kb;        // members, in chain order
		const uint32_t Bend = wave_incl_scan(cand ? T + 1 : 0u);   // steps through this member
		uint64_t left = __ballot(cand);
		if (!left) return DiagOut{0, 0, 0, 0, tooLong != 0 ? 1u : (trunc ? 2u : 0u)};
		PROF_ADD(*this, P_T_D2, PROF_NOW() - tq);
		// Members are taken in rounds of at most 64 steps (a member never
		// straddles two rounds); the first member that fails its check ends
		// the batch.
		uint32_t committed = 0, dadd = 0, rbase = 0, advance = 0;
		bool all = true;
		while (left) {
			tq = PROF_NOW();
			const bool valid = ((left >> lane) & 1u) && Bend - rbase <= 64;
			const uint64_t VM = __ballot(valid);
			const uint32_t nm = (uint32_t)__builtin_popcountll(VM);
			const uint32_t klast = 63u - (uint32_t)__builtin_clzll(VM);
			const uint32_t B = rdlane(Bend, klast) - rbase;
			const uint32_t maxT = rdlane(wave_incl_max(valid ? T : 0u), 63);
			// member table (LDS, by rank in the round): start | end << 11 |
			// T << 23, and the step lanes where members begin
			__builtin_amdgcn_wave_barrier();
			if (valid) {
				const uint32_t r = (uint32_t)__builtin_popcountll(VM & ((1ull << lane) - 1ull));
				mlist[64 + r] = astart | (an << 11) | (T << 23);
			}
			mlist[lane] = 0u;
			__builtin_amdgcn_s_waitcnt(0xc07f);
			__builtin_amdgcn_wave_barrier();
			if (valid) mlist[Bend - rbase - T - 1] = 1u;
			__builtin_amdgcn_s_waitcnt(0xc07f);
			__builtin_amdgcn_wave_barrier();
			const uint64_t starts = __ballot(mlist[lane] != 0u);
			PROF_ADD(*this, P_D_MEMBERS, nm);
			PROF_ADD(*this, P_D_STEPS, B);
			// 4. windows of every step: lane f is step t of member j
			const bool live = lane < B;
			const uint64_t below = starts & mask_le(lane);
			const uint32_t j = live ? (uint32_t)__builtin_popcountll(below) - 1u : 0u;
			const uint32_t fb = live ? 63u - (uint32_t)__builtin_clzll(below) : 0u;   // member's first lane
			const uint32_t t = lane - fb;
			const uint32_t jw = mlist[64 + (j & 63u)];
			const uint32_t js = jw & 2047u;
			const uint32_t jT = jw >> 23;
			uint32_t sV = kSentinel, sR = kSentinel - 1u, fVl = 0, fRl = 0;
			PROF_ADD(*this, P_T_D3A, PROF_NOW() - tq);
			if (live) {
				const uint64_t fV = fp16(0, v0 + js + t), fR = fp16(1, r0 + js + t);
				sV = slot_of(fV, mq, q, qmag);
				sR = slot_of(fR, mq, q, qmag);
				fVl = (uint32_t)fV;
				fRl = (uint32_t)fR;
			}
			PROF_ADD(*this, P_T_D3B, PROF_NOW() - tq);
			// 5. first writers: s1 = first lane c in [fb, lane] with sV(c) ==
			//    sR(lane), s2 = first with sR(c) == sV(lane).  Lane l looks back
			//    d = 0 .. t lanes (its own member's earlier steps) through DPP
			//    wave shifts; the largest matching d is the earliest writer,
			//    whose fingerprint rides along.
			uint32_t s1 = 64, s2 = 64, f1 = 0, f2 = 0;
			const bool use_dpp = maxT <= kShortT && 6u * maxT <= kBloomBase + 10u * nm;
			if (use_dpp && q < (1ull << 25)) {   // member keys need slot + 1 < 2^25
				// Keys tag each slot with its member (slot + 1 | j << 25), so
				// a shifted key can only equal a lane's own key when it comes
				// from the same member: no per-shift range test, and the
				// fingerprints are fetched once for the final candidates.
				const uint32_t kv = live ? ((sV + 1u) | (j << 25)) : 0xFFFFFFFFu;
				const uint32_t kr = live ? ((sR + 1u) | (j << 25)) : 0xFFFFFFFEu;
				uint32_t d1 = kv == kr ? 0u : 0xFFu;   // largest shift with a match
				uint32_t d2 = d1;
				uint32_t xv = kv, xr = kr;
#pragma unroll
				for (uint32_t d = 1; d <= kShortT; ++d) {
					if (d > maxT) break;
					xv = wave_shr1z(xv);
					xr = wave_shr1z(xr);
					d1 = xv == kr ? d : d1;
					d2 = xr == kv ? d : d2;
				}
				s1 = d1 != 0xFFu ? lane - d1 : 64u;
				s2 = d2 != 0xFFu ? lane - d2 : 64u;
				f1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s1 << 2), (int)fVl);
				f2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s2 << 2), (int)fRl);
			} else if (use_dpp) {
				uint32_t xv = sV, xr = sR, xfv = fVl, xfr = fRl;
				for (uint32_t d = 0; d <= maxT; ++d) {
					if (d) {
						xv = wave_shr1(xv);
						xr = wave_shr1(xr);
						xfv = wave_shr1(xfv);
						xfr = wave_shr1(xfr);
					}
					const bool in = d <= t;
					const bool m1 = in && xv == sR, m2 = in && xr == sV;
					s1 = m1 ? lane - d : s1;
					f1 = m1 ? xfv : f1;
					s2 = m2 ? lane - d : s2;
					f2 = m2 ? xfr : f2;
				}
			} else {
				// Long epochs: a 2048-bit hash of the round's V slots and of
				// its R slots (LDS) flags the steps that can have a candidate
				// at all (every epoch's last step is among them); only those
				// are resolved exactly, one ballot per lookup.
				uint32_t* bmv = mlist + 128;
				uint32_t* bmr = mlist + 192;
				__builtin_amdgcn_wave_barrier();
				bmv[lane] = 0u;
				bmr[lane] = 0u;
				__builtin_amdgcn_s_waitcnt(0xc07f);
				__builtin_amdgcn_wave_barrier();
				if (live) {
					bloom_add<64>(bmv, sV);
					bloom_add<64>(bmr, sR);
				}
				__builtin_amdgcn_s_waitcnt(0xc07f);
				__builtin_amdgcn_wave_barrier();
				const bool q1 = live && bloom_has<64>(bmv, sR);
				const uint64_t Q1 = __ballot(q1);
				for (uint64_t w = Q1; w; w &= w - 1) {
					const uint32_t L = ffs64(w);
					const uint64_t range = mask_le(L) & ~((1ull << rdlane(fb, L)) - 1ull);   // [fb_L, L]
					const uint64_t m = __ballot(sV == rdlane(sR, L)) & range;
					if (m) {
						const uint32_t c = ffs64(m);
						const uint32_t fc = rdlane(fVl, c);
						s1 = lane == L ? c : s1;
						f1 = lane == L ? fc : f1;
					}
				}
				// lookup 2 matters only where lookup 1 neither hit the diagonal
				// nor found a fingerprint-equal candidate (step 6 below)
				const bool hit1 = s1 == lane && t == jT, bad1 = s1 != 64 && s1 != lane && f1 == fRl;
				const bool need2 = live && !hit1 && !bad1 && bloom_has<64>(bmr, sV);
				for (uint64_t w = __ballot(need2); w; w &= w - 1) {
					const uint32_t L = ffs64(w);
					const uint64_t range = mask_le(L) & ~((1ull << rdlane(fb, L)) - 1ull);   // [fb_L, L]
					const uint64_t m = __ballot(sR == rdlane(sV, L)) & range;
					if (m) {
						const uint32_t c = ffs64(m);
						const uint32_t fc = rdlane(fRl, c);
						s2 = lane == L ? c : s2;
						f2 = lane == L ? fc : f2;
					}
				}
			}
			PROF_ADD(*this, P_T_D3, PROF_NOW() - tq);
			tq = PROF_NOW();
			// 6. the reference's resolution of step t
			bool bad = false, hit = false;
			if (s1 != 64) {
				if (s1 == lane) hit = t == jT;          // the diagonal: equal bytes iff t == T
				else if (f1 == fRl) bad = true;         // a possible match off the diagonal
			}
			if (!hit && !bad && s2 != 64) {
				if (s2 == lane) hit = t == jT;
				else if (f2 == fVl) bad = true;
			}
			if (t == jT && !hit) bad = true;            // the epoch would go on past T
			const uint64_t BM = __ballot(live && bad);
			uint32_t fm = nm, fbad = B;   // committed members, their steps
			if (BM) {
				const uint32_t l = ffs64(BM);
				fbad = 63u - (uint32_t)__builtin_clzll(starts & mask_le(l));   // first lane of its member
				fm = (uint32_t)__builtin_popcountll(starts & mask_le(l)) - 1u;
			}
			if (nrec + committed + fm > rec_cap) { fm = 0; fbad = 0; }
			// 7. commit members 0 .. fm-1: ADD(T bytes) + COPY(a + T .. end)
			if (lane < fm) {
				const uint32_t w = mlist[64 + lane];
				const uint32_t ms = w & 2047u, me = (w >> 11) & 4095u, mt = w >> 23;
				uint32_t* o = rec + kRecWordsOnepass * (nrec + committed + lane);
				o[0] = v0 + ms + mt;
				o[1] = r0 + ms + mt;
				o[2] = me - ms - mt;
				o[3] = rd4(0, v0 + ms);   // the ADD's first bytes (gap start = member start)
			}
			// sum over committed members of (T + 1) is the first lane of member fm
			dadd += 21u * fm + fbad;
			committed += fm;
			PROF_ADD(*this, P_T_D4, PROF_NOW() - tq);
			if (fm < nm) {   // stop at the failing member's start
				advance = rdlane(js, fbad);
				all = false;
				break;
			}
			advance = rdlane(an, klast);
			rbase = rdlane(Bend, klast);
			left &= ~VM;
		}
		return DiagOut{committed, advance, all ? 1u : 0u, dadd, 0};
	}

	// wave-parallel forward extension (onepass.c:229-234), 256 B per pass
	__device__ uint32_t extend(uint32_t vpos, uint32_t rpos, uint32_t lim) {
		[[maybe_unused]] const uint64_t t0 = PROF_NOW();
		PROF_ADD(*this, P_EXTENDS, 1);
		const uint32_t lane = lane_id();
		uint32_t ml = 0;
		while (ml < lim) {
			ensure2(vpos + ml, rpos + ml, 256 + 8, true, true);
			const uint32_t x = rd4(0, vpos + ml + 4 * lane) ^ rd4(1, rpos + ml + 4 * lane);
			uint32_t fb = x ? ((uint32_t)__builtin_ctz(x) >> 3) : 4u;
			const int32_t rem = (int32_t)umin32(lim - ml, 512u) - (int32_t)(4 * lane);
			if (rem < (int32_t)fb) fb = rem < 0 ? 0u : (uint32_t)rem;
			const uint64_t m = __ballot(fb < 4);
			if (m) {
				const uint32_t f = ffs64(m);
				PROF_ADD(*this, P_T_EXT, PROF_NOW() - t0);
				return ml + 4 * f + rdlane(fb, f);
			}
			ml += 256;
		}
		PROF_ADD(*this, P_T_EXT, PROF_NOW() - t0);
		return lim;
	}
};
using WinSrc = WinSrcT<false>;

// ───────────────────────────── the epoch chain ────────────────────────────

struct PairResult {
	uint32_t nrec;
	uint64_t dsz;
	int32_t st;
};

template <bool kMembers, class Src, bool kRouted = false>
__device__ __forceinline__ PairResult onepass_pair(Src& src, const EncodeArgs& a, uint32_t pair,
                                             const PairDev& pd, const PairPlanDev& pp, uint32_t p,
                                             uint32_t* bm, uint32_t* cscr) {
	const uint32_t lane = lane_id();
	const uint32_t vl = uni((uint32_t)pd.v_len), rl = uni((uint32_t)pd.r_len);
	const uint64_t q = uni64(pp.q), qmag = uni64(pp.q_magic);
	const ModQ mq = make_modq(q, qmag);
	const uint32_t rec_cap = uni(pp.rec_cap);
	uint32_t* __restrict__ rec = a.rec + (uint64_t)kRecWordsOnepass * pp.rec_base;

	uint32_t nrec = 0;
	uint64_t dsz = 26;   // header (25) + END
	int32_t st = 0;

	int32_t tslot = -1;  // table tier state
	uint32_t tag = 0;
	unsigned long long* HV = nullptr;
	// the epoch's last tag goes back with the table, so its next holder
	// starts above every entry this one wrote
	auto release_table = [&]() {
		if (lane == 0) {
			__hip_atomic_store(&a.table_tags[tslot], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			vm_drain();
			__hip_atomic_store(&a.table_locks[tslot], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
		}
		tslot = -1;
	};

	uint32_t v0 = 0, r0 = 0;
	bool scanning = vl > 0;
	bool at_mismatch = false;   // (v0, r0) is where the last extension stopped
	bool skipA = false;         // the epoch is known to be long: phase B from step 0
	// Backoff of the diagonal batch and of phase A: either only pays when most
	// epochs resolve there (substitutions); after k failures in a row the next
	// 2^k - 1 epochs go straight to the next tier (the result is the same, the
	// tiers only differ in cost)
	uint32_t diag_miss = 0, diag_skip = 0, a_miss = 0, a_skip = 0;
	bool diag_full = false;   // the next diagonal batch scans its full look-ahead

	// ── member mode (dg_members.hip): verified diagonal members are taken as
	//    they are, 64 records per pass, chunk after chunk; the epochs below
	//    run only from an unverified member until the chain lands on a later
	//    member start, and for the final epoch (whose member is never
	//    verified: its run holds the end of the shorter stream) ──
	constexpr bool members = kMembers && Src::kPhaseA;   // (the plain chain compiles none of it)
	uint32_t kc = 0, ki = 0, nch = 0, cnt = 0, s_cur = 0;   // chunk, index in chunk, chunks, members in kc
	const uint32_t* msp = nullptr;   // member starts of chunk 0 (chunk c: + c * kMemChunkSlots)
	const uint32_t* srp = nullptr;
	const uint32_t* ncp = nullptr;   // members per chunk
	bool mem_live = false;           // members remain ahead of the chain
	const uint32_t* csp = nullptr;   // per chunk: verified prefix, its delta bytes
	uint32_t* cmp = nullptr;         // per chunk: bulk piece (member count, byte offset)
	// the delta's other pieces (member_serialize_kernel): the runs of records
	// this chain wrote itself (between bulk pieces, so at most n_chunks + 1)
	// and the tail
	uint32_t* sgp = nullptr;
	uint32_t nseg = 0, seg_cap = 0;
	bool nb_open = false;            // a run of records written here is open
	uint32_t nb_first = 0, nb_boff = 0, nb_prev = 0;
	auto nb_note = [&]() {           // before records are appended to rec
		if (!nb_open) {
			nb_open = true;
			nb_first = nrec;
			nb_boff = (uint32_t)(dsz - 1);   // dsz counts the END byte
			nb_prev = v0;
		}
	};
	auto nb_close = [&]() {
		if (nb_open && nrec > nb_first) {
			if (nseg < seg_cap) {
				if (lane == 0) *(uint4*)(sgp + 4ull * nseg) = make_uint4(nb_first, nrec - nb_first, nb_boff, nb_prev);
			} else {
				st = kStatusInternal;
			}
			++nseg;
		}
		nb_open = false;
	};
	auto take_members = [&]() {
		[[maybe_unused]] const uint64_t tt0 = PROF_NOW();
		if constexpr (Src::kPhaseA) PROF_ADD(src, P_TAKES, 1);
		for (;;) {
			if (kc >= nch) break;
			if (ki == 0) {
				// whole verified chunks from kc, 64 summaries at a time, go to
				// the gather map; the first partial chunk contributes its
				// verified prefix and stops the run
				const uint32_t cj = kc + lane;
				const bool inr = cj < nch;
				const uint32_t cn = inr ? ncp[cj] : 0u;
				const uint32_t vp = inr ? csp[2ull * cj] : 0u;
				const uint32_t vb = inr ? csp[2ull * cj + 1] : 0u;
				const uint64_t full = __ballot(inr && vp == cn);
				const uint32_t nfull = full == ~0ull ? 64u : ffs64(~full);
				const bool use = inr && lane <= nfull;
				const uint32_t ct = use ? vp : 0u;   // == cn for the full chunks
				const uint32_t incl = wave_incl_scan(ct);
				const uint32_t tot = rdlane(incl, 63);
				if (nrec + tot > rec_cap) { st = 7; scanning = false; return; }
				nb_close();
				// the chunks' bulk pieces: member count and byte offset
				const uint32_t bvb = use ? vb : 0u;
				const uint32_t bi = wave_incl_scan(bvb);
				if (use && ct > 0) *(uint2*)(cmp + 2ull * cj) = make_uint2(ct, (uint32_t)(dsz - 1) + bi - bvb);
				dsz += rdlane(bi, 63);
				nrec += tot;
				if (nfull == 64) { kc += 64; continue; }
				kc += nfull;
				if (kc >= nch) break;
				cnt = uni(ncp[kc]);
				ki = rdlane(vp, nfull);   // the first unverified member of chunk kc
				break;
			}
			// mid-chunk, after a re-sync: records of the verified run copied here
			const uint32_t n_in = umin32(cnt - ki, 64u);
			const uint64_t slot = (uint64_t)kc * kMemChunkSlots + ki + lane;
			uint4 r4 = make_uint4(0u, 0u, 0u, 0u);
			uint32_t sj = 0;
			if (lane < n_in) {
				r4 = *(const uint4*)(srp + 4ull * slot);
				sj = msp[slot];
			}
			const uint64_t full = n_in == 64 ? ~0ull : ((1ull << n_in) - 1ull);
			const uint64_t bad = ~__ballot(lane < n_in && r4.w != 0u) & full;
			const uint32_t take = bad ? ffs64(bad) : n_in;   // the verified prefix
			if (nrec + take > rec_cap) { st = 7; scanning = false; return; }
			if (take) nb_note();
			if (lane < take) *(uint4*)(rec + (uint64_t)kRecWordsOnepass * (nrec + lane)) = make_uint4(r4.x, r4.x, r4.y, r4.z);
			const uint32_t gap = r4.x - sj;   // ADD [s_j, x_j) before the COPY
			const uint32_t sz = lane < take ? 13u + (gap ? 9u + gap : 0u) : 0u;
			dsz += rdlane(wave_incl_scan(sz), 63);
			nrec += take;
			ki += take;
			if (take < n_in) break;   // member (kc, ki) is left to the epochs below
			if (ki >= cnt) { ++kc; ki = 0; }
		}
		// the chain always ends on an unverified member (the final epoch's
		// run holds the end of the shorter stream)
		mem_live = kc < nch;
		if (!mem_live) { st = kStatusInternal; scanning = false; return; }
		s_cur = uni(msp[(uint64_t)kc * kMemChunkSlots + ki]);
		v0 = r0 = s_cur;
		at_mismatch = kc != 0 || ki != 0;   // member starts past the first are mismatches
		if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_TAKE, PROF_NOW() - tt0);
	};
	if (members) {
		sgp = a.seg + 4ull * ((uint64_t)pp.chunk_base + 2ull * pair);
		seg_cap = uni(pp.n_chunks) + 2;
	}
	if (members && scanning) {
		msp = a.mem_s + pp.mem_base;
		srp = a.srec + 4ull * pp.mem_base;
		ncp = a.n_mem + pp.chunk_base;
		csp = a.csum + 2ull * pp.chunk_base;
		cmp = a.cmap + 2ull * pp.chunk_base;
		nch = uni(pp.n_chunks);
		cnt = uni(ncp[0]);
		take_members();
	}

	while (scanning) {
		skipA = false;
#ifndef DG_NO_CRC_STEP
		if constexpr (Src::kPhaseA) src.crc_step();   // (kCrc sources only)
#endif
		if (members && mem_live && v0 == r0 && v0 > s_cur) {
			[[maybe_unused]] const uint64_t tr0 = PROF_NOW();
			if constexpr (Src::kPhaseA) PROF_ADD(src, P_RESYNCS, 1);
			// did the exact chain land on a later member start? (ascending
			// over the chunks)
			uint32_t c2 = kc, i2 = ki + 1, n2 = cnt;
			bool found = false, past = false;
			while (!found && !past && c2 < nch) {
				if (c2 != kc) n2 = uni(ncp[c2]);
				for (; i2 < n2; i2 += 64) {
					const uint32_t j = i2 + lane;
					const uint32_t sj = j < n2 ? msp[(uint64_t)c2 * kMemChunkSlots + j] : 0xFFFFFFFFu;
					const uint64_t eq = __ballot(sj == v0);
					if (eq) { i2 += ffs64(eq); found = true; break; }
					if (__ballot(j < n2 && sj > v0)) { past = true; break; }   // (not the padding lanes)
				}
				if (!found && !past) { ++c2; i2 = 0; }
			}
			if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_RESYNC, PROF_NOW() - tr0);
			if (found) {
				kc = c2;
				ki = i2;
				cnt = n2;
				take_members();
				continue;
			}
		}
		// no match is possible once either stream cannot supply a window at
		// the epoch start (the reference keeps scanning the other, :102-104)
		if (v0 + p > vl || r0 + p > rl) break;
		if constexpr (Src::kPhaseA) {
			const bool try_diag = at_mismatch && diag_skip == 0;
			if (at_mismatch && !try_diag) --diag_skip;
			if (try_diag) {
				[[maybe_unused]] const uint64_t td = PROF_NOW();
				if (members) nb_note();
				const auto dg = src.diag_batch(v0, r0, vl, rl, q, qmag, mq, p, rec, nrec, rec_cap, bm, diag_full);
				diag_full = false;
				if (uni(dg.long_first) == 2u) { diag_full = true; continue; }   // the same state, scanned in full
				const uint32_t f = uni(dg.committed);
				skipA = f == 0 && uni(dg.long_first) != 0u;
				// matches that leave the diagonal (insertions, deletions, moved
				// blocks) make the batch commit nothing: back off exponentially
				diag_miss = f == 0 ? umin32(diag_miss + 1u, kBackoffMax) : 0u;
				diag_skip = (1u << diag_miss) - 1u;
				PROF_ADD(src, P_T_DIAG, PROF_NOW() - td);
				PROF_ADD(src, P_DIAG_CALLS, 1);
				PROF_ADD(src, P_DIAG_EPOCHS, f);
				PROF_ADD(src, P_DIAG_ZERO, f == 0);
				if (f) {
					const uint32_t adv = uni(dg.adv);
					nrec += f;
					dsz += uni(dg.dadd);
					v0 += adv;
					r0 += adv;
					if (uni(dg.more)) continue;   // the chain left the region: next batch
					if (v0 + p > vl || r0 + p > rl) break;
				}
			}
		}
		const uint32_t nv = vl - p - v0 + 1;   // steps with a V window
		const uint32_t nr = rl - p - r0 + 1;   // steps with an R window
		const uint32_t nlive = umax32(nv, nr);

		bool matched = false;
		uint32_t vm = 0, rm = 0, ml = 0;
		uint32_t pw = 0;   // 4th record word

		// ── phase A: steps 0..7, four lanes per window ──
		if constexpr (Src::kPhaseA) if (skipA) {
			src.ensure2(v0, r0, 8 + 16 + 8, true, true);
			pw = uni(src.rd4(0, v0));   // V bytes from the epoch start (the ADD payload's head)
		}
		if constexpr (Src::kPhaseA) if (!skipA && a_skip) {
			--a_skip;
			skipA = true;
			src.ensure2(v0, r0, 8 + 16 + 8, true, true);
			pw = uni(src.rd4(0, v0));   // V bytes from the epoch start (the ADD payload's head)
		}
		if constexpr (Src::kPhaseA) if (!skipA) {
			[[maybe_unused]] const uint64_t ta = PROF_NOW();
			PROF_ADD(src, P_A_ENTRIES, 1);
			src.ensure2(v0, r0, 8 + 16 + 8, true, true);
			pw = uni(src.rd4(0, v0));   // V bytes from the epoch start (the ADD payload's head)
			const uint32_t side = lane >> 5, w = (lane >> 2) & 7u, part = lane & 3u;
			const uint32_t bytes = src.rd4(side, (side ? r0 : v0) + w + 4 * part);
			uint64_t lo = 0, hi = 0;
#pragma unroll
			for (int j = 0; j < 4; ++j) {   // constants 263^(15-k) for this lane's 4 bytes (L1-resident)
				const uint64_t c = src.powc[4 * part + j];
				const uint64_t b = (bytes >> (8 * j)) & 0xff;
				lo += b * (uint32_t)c;
				hi += b * (uint32_t)(c >> 32);
			}
			const uint64_t fp = fold61(quad_sum64(lo), quad_sum64(hi));
			const bool valid = w < (side ? nr : nv);
			const uint32_t slot = valid ? slot_of(fp, mq, q, qmag) : kSentinel;
			const uint32_t fpl = (uint32_t)fp;
			const uint32_t tA = umin32(8u, nlive);
			for (uint32_t t = 0; t < tA; ++t) {
				if (t < nr) {   // lookup 1: R(t) in the V heads of steps 0..t
					const uint32_t x = rdlane(slot, 32 + 4 * t);
					const uint64_t m = __ballot(slot == x) & 0x11111111ull & ((2ull << (4 * t)) - 1);
					if (m) {
						const uint32_t l = ffs64(m);
						if (rdlane(fpl, l) == rdlane(fpl, 32 + 4 * t)) {
							const uint32_t s = l >> 2;
							const uint32_t e = src.extend(v0 + s, r0 + t, umin32(vl - (v0 + s), rl - (r0 + t)));
							if (e >= 16) { matched = true; vm = v0 + s; rm = r0 + t; ml = e; break; }
						}
					}
				}
				if (t < nv) {   // lookup 2: V(t) in the R heads of steps 0..t
					const uint32_t x = rdlane(slot, 4 * t);
					const uint64_t m = __ballot(slot == x) & 0x1111111100000000ull & ((2ull << (32 + 4 * t)) - 1);
					if (m) {
						const uint32_t l = ffs64(m);
						if (rdlane(fpl, l) == rdlane(fpl, 4 * t)) {
							const uint32_t s = (l - 32) >> 2;
							const uint32_t e = src.extend(v0 + t, r0 + s, umin32(vl - (v0 + t), rl - (r0 + s)));
							if (e >= 16) { matched = true; vm = v0 + t; rm = r0 + s; ml = e; break; }
						}
					}
				}
			}
			PROF_ADD(src, P_T_A, PROF_NOW() - ta);
			PROF_ADD(src, P_A_MATCH, matched);
			// epochs longer than 8 steps in a row: phase B from step 0 for a while
			a_miss = matched ? 0u : umin32(a_miss + 1u, kBackoffMax);
			a_skip = (1u << a_miss) - 1u;
			if (!matched && nlive <= 8) break;   // both streams exhausted: scan over
		}

		// ── phases B and C: 64 steps per chunk ──
		uint32_t hsV[kHistChunks], hsR[kHistChunks], hfV[kHistChunks], hfR[kHistChunks];
		bool in_table = false;
		[[maybe_unused]] const uint64_t tb = PROF_NOW();
		if constexpr (Src::kPhaseA) { if (!matched) PROF_ADD(src, P_B_ENTRIES, 1); }
		for (uint32_t c = 0; !matched; ++c) {
			const uint32_t b0 = 64 * c;
			if (b0 >= nlive) { scanning = false; break; }   // both streams exhausted
			const uint32_t step = b0 + lane;
			const bool cv = step < nv, cr = step < nr;
			[[maybe_unused]] const uint64_t tb1 = PROF_NOW();
			src.chunk(v0 + b0, r0 + b0, b0 < nv, b0 < nr);

			uint64_t fV = 0, fR = 0;
			uint32_t sV = kSentinel, sR = kSentinel;
			if (cv) { fV = src.fpV(v0 + step); sV = slot_of(fV, mq, q, qmag); }
			if (cr) { fR = src.fpR(r0 + step); sR = slot_of(fR, mq, q, qmag); }
			const uint32_t fVl = (uint32_t)fV, fRl = (uint32_t)fR;
#ifdef DG_ONEPASS_PROF
			if constexpr (Src::kPhaseA) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); PROF_ADD(src, P_T_B1, PROF_NOW() - tb1); }
#endif
			if constexpr (Src::kPhaseA) PROF_ADD(src, c < (uint32_t)kHistChunks ? P_B_CHUNKS : P_C_CHUNKS, 1);
			if (c < (uint32_t)kHistChunks) {
#pragma unroll
				for (int k = 0; k < kHistChunks; ++k)
					if ((uint32_t)k == c) { hsV[k] = sV; hsR[k] = sR; hfV[k] = fVl; hfR[k] = fRl; }
				// Filter: a 2048-bit hash of every slot inserted in this epoch
				// so far, per table.  A step whose slot misses the other
				// table's bitmap has no candidate at all; only the remaining
				// steps are walked exactly (in step order).
				constexpr uint32_t BW = Src::kBmWords;   // bitmap words per table
				if (c == 0) {
#pragma unroll
					for (uint32_t k = 0; k < 2 * BW; k += 64) bm[k + lane] = 0u;
				}
				__builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
				__builtin_amdgcn_wave_barrier();
				if (cv) bloom_add<BW>(bm, sV);
				if (cr) bloom_add<BW>(bm + BW, sR);
				__builtin_amdgcn_s_waitcnt(0xc07f);
				__builtin_amdgcn_wave_barrier();
				const bool p1 = cr && bloom_has<BW>(bm, sR);
				const bool p2 = cv && bloom_has<BW>(bm + BW, sV);
				const uint64_t m1 = __ballot(p1), m2 = __ballot(p2);
				// steps phase A already ruled out are skipped
				const uint32_t j0 = (Src::kPhaseA && c == 0 && !skipA) ? 8u : 0u;
				uint64_t walk = (m1 | m2) & ~((1ull << j0) - 1ull);
				if constexpr (Src::kPhaseA) PROF_ADD(src, P_B_WALKED, __builtin_popcountll(walk));
				[[maybe_unused]] const uint64_t tb3 = PROF_NOW();
				if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_B2, tb3 - tb1);
				while (walk) {
					const uint32_t j = ffs64(walk);
					walk &= walk - 1;
					const uint32_t t = b0 + j;
					if ((m1 >> j) & 1u) {
						const uint32_t x = rdlane(sR, j);
						uint32_t s = kSentinel, sf = 0;
#pragma unroll
						for (int k = 0; k < kHistChunks; ++k) {
							if (s == kSentinel && (uint32_t)k <= c) {
								uint64_t m = __ballot(hsV[k] == x);
								if ((uint32_t)k == c) m &= mask_le(j);
								if (m) { const uint32_t l = ffs64(m); s = 64u * k + l; sf = rdlane(hfV[k], l); }
							}
						}
						if (s != kSentinel && sf == rdlane(fRl, j)) {
							const uint32_t e = src.extend(v0 + s, r0 + t, umin32(vl - (v0 + s), rl - (r0 + t)));
							if (e >= p) { matched = true; vm = v0 + s; rm = r0 + t; ml = e; break; }
						}
					}
					if ((m2 >> j) & 1u) {
						const uint32_t x = rdlane(sV, j);
						uint32_t s = kSentinel, sf = 0;
#pragma unroll
						for (int k = 0; k < kHistChunks; ++k) {
							if (s == kSentinel && (uint32_t)k <= c) {
								uint64_t m = __ballot(hsR[k] == x);
								if ((uint32_t)k == c) m &= mask_le(j);
								if (m) { const uint32_t l = ffs64(m); s = 64u * k + l; sf = rdlane(hfR[k], l); }
							}
						}
						if (s != kSentinel && sf == rdlane(fVl, j)) {
							const uint32_t e = src.extend(v0 + t, r0 + s, umin32(vl - (v0 + t), rl - (r0 + s)));
							if (e >= p) { matched = true; vm = v0 + t; rm = r0 + s; ml = e; break; }
						}
					}
				}
				if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_B3, PROF_NOW() - tb3);
			} else {
				// ── phase C: per-pair (tag, earliest step, fingerprint) table in HBM ──
				// Steps 0 .. 64*kHistChunks-1 stay in registers (their slots in
				// the phase-B bitmaps); later chunks go to the table.  Per chunk:
				// one 16-byte load per window slot gives the lookup and the
				// first-writer test, the chunk's own steps are resolved from
				// registers (a per-chunk bitmap flags candidates and duplicate
				// slots), and the chunk's first writers are stored after it.
				[[maybe_unused]] const uint64_t tc0 = PROF_NOW();
				if (!in_table) {
					in_table = true;
					if (tslot < 0) {
						// Holders never wait (a table is released when its pair
						// ends), so the wait always drains; the wall-clock bound
						// only guarantees every wave an exit.  Running into it is
						// a pool-capacity condition, reported as such.
						// Tables are partitioned by XCD (the plan makes n_tables a
						// multiple of 8): a table's lines are only ever cached in
						// one L2, so no stale copy survives a tag wrap.
						uint32_t got = 0xFFFFFFFFu;
						if (lane == 0) {
							const uint32_t parts = a.n_tables >= 8u ? 8u : 1u;
							const uint32_t n = a.n_tables / parts;
							const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;   // HW_REG_XCC_ID
							const uint32_t tbase = (xcc % parts) * n;
							const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
							for (uint32_t it = 0; got == 0xFFFFFFFFu; ++it) {
								const uint32_t slx = tbase + (pair + it) % n;
								if (atomicCAS(&a.table_locks[slx], 0u, 1u) == 0u) {
									got = slx;
								} else if ((it % n) == n - 1) {
									__builtin_amdgcn_s_sleep(32);
									if (__builtin_amdgcn_s_memrealtime() - t_start > kTableWaitTicks) break;
								}
							}
						}
						got = rdlane(got, 0);
						if (got == 0xFFFFFFFFu) { st = kStatusTablePool; scanning = false; break; }
						tslot = (int32_t)got;
						HV = a.tables + (uint64_t)got * 2ull * a.qmax;
						uint32_t t0 = 0;
						if (lane == 0)
							t0 = __hip_atomic_load(&a.table_tags[got], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
						tag = rdlane(t0, 0);
					}
					if (tag >= kTagMax) {   // tag space exhausted: clear the table
						for (uint64_t i = lane; i < 2ull * a.qmax; i += 64) HV[i] = 0ull;
						vm_drain();
						tag = 0;
					}
					++tag;
				}
				vm_drain();   // the previous chunk's stores are in the L2
				const u64x2 pV = cv ? tab_load(HV, sV) : u64x2{0ull, 0ull};   // HV[sV], HR[sV]
				const u64x2 pR = cr ? tab_load(HV, sR) : u64x2{0ull, 0ull};   // HV[sR], HR[sR]
				// per-chunk bitmaps (1024 bits per table): candidates of the
				// chunk's own steps, and lanes whose slot bit was already set
				// (a possible duplicate slot among the chunk's lanes)
				constexpr uint32_t CW = 32;
				cscr[lane] = 0u;
				__builtin_amdgcn_s_waitcnt(0xc07f);
				__builtin_amdgcn_wave_barrier();
				const uint32_t hv = sV & (32u * CW - 1u), hr = sR & (32u * CW - 1u);
				const uint32_t oV = cv ? atomicOr(&cscr[hv >> 5], 1u << (hv & 31u)) : 0u;
				const uint32_t oR = cr ? atomicOr(&cscr[CW + (hr >> 5)], 1u << (hr & 31u)) : 0u;
				__builtin_amdgcn_s_waitcnt(0xc07f);
				__builtin_amdgcn_wave_barrier();
				const bool i1 = cr && ((cscr[hr >> 5] >> (hr & 31u)) & 1u);        // an sV of the chunk may equal sR
				const bool i2 = cv && ((cscr[CW + (hv >> 5)] >> (hv & 31u)) & 1u);  // an sR of the chunk may equal sV
				// history: the phase-B bitmaps hold the slots of steps 0 .. 64*kHistChunks-1
				constexpr uint32_t BW = Src::kBmWords;
				const bool g1 = cr && bloom_has<BW>(bm, sR);
				const bool g2 = cv && bloom_has<BW>(bm + BW, sV);
				// duplicates: every lane whose slot bit was set by another lane
				// is checked exactly; the others are their slot's only lane
				bool dupV = false, dupR = false;
				for (uint64_t w = __ballot(cv && ((oV >> (hv & 31u)) & 1u)); w; w &= w - 1) {
					const uint32_t L = ffs64(w);
					const uint64_t m = __ballot(cv && sV == rdlane(sV, L));
					dupV |= ((m & ~(1ull << ffs64(m))) >> lane) & 1u;
				}
				for (uint64_t w = __ballot(cr && ((oR >> (hr & 31u)) & 1u)); w; w &= w - 1) {
					const uint32_t L = ffs64(w);
					const uint64_t m = __ballot(cr && sR == rdlane(sR, L));
					dupR |= ((m & ~(1ull << ffs64(m))) >> lane) & 1u;
				}
				vm_drain();
				// earlier chunks of the table tier (the history, if it has the
				// slot, is earlier still and takes precedence)
				const bool x1 = cr && tab_cur(pR.x, tag), x2 = cv && tab_cur(pV.y, tag);
				const bool f1 = x1 && tab_fpok(pR.x, fRl), f2 = x2 && tab_fpok(pV.y, fVl);
				const uint32_t r1 = tab_step(pR.x), r2 = tab_step(pV.y);
				// this chunk's first writers go in (after the lookups' loads)
				if (cv && !dupV && !tab_cur(pV.x, tag)) HV[2ull * sV] = tab_key(tag, step, fVl);
				if (cr && !dupR && !tab_cur(pR.y, tag)) HV[2ull * sR + 1] = tab_key(tag, step, fRl);
				uint64_t walk = __ballot(g1 || f1 || (i1 && !x1) || g2 || f2 || (i2 && !x2));
				const uint64_t G1 = __ballot(g1), G2 = __ballot(g2), X1 = __ballot(x1), X2 = __ballot(x2);
				while (walk) {
					const uint32_t j = ffs64(walk);
					walk &= walk - 1;
					const uint32_t t = b0 + j;
					// lookup 1: the earliest writer of slotR(t) in HV
					if (t < nr) {
						const uint32_t x = rdlane(sR, j);
						uint32_t s1 = kSentinel;
						bool ok = false;
						if ((G1 >> j) & 1u) {
#pragma unroll
							for (int k = 0; k < kHistChunks; ++k) {
								if (s1 == kSentinel) {
									const uint64_t m = __ballot(hsV[k] == x);
									if (m) { const uint32_t l = ffs64(m); s1 = 64u * k + l; ok = rdlane(hfV[k], l) == rdlane(fRl, j); }
								}
							}
						}
						if (s1 == kSentinel && ((X1 >> j) & 1u)) {
							s1 = rdlane(r1, j);
							ok = rdlane((uint32_t)f1, j) != 0u;
						} else if (s1 == kSentinel) {
							const uint64_t m = __ballot(cv && sV == x) & mask_le(j);
							if (m) { const uint32_t l = ffs64(m); s1 = b0 + l; ok = rdlane(fVl, l) == rdlane(fRl, j); }
						}
						if (ok) {
							const uint32_t e = src.extend(v0 + s1, r0 + t, umin32(vl - (v0 + s1), rl - (r0 + t)));
							if (e >= p) { matched = true; vm = v0 + s1; rm = r0 + t; ml = e; break; }
						}
					}
					// lookup 2: the earliest writer of slotV(t) in HR
					if (t < nv) {
						const uint32_t x = rdlane(sV, j);
						uint32_t s2 = kSentinel;
						bool ok = false;
						if ((G2 >> j) & 1u) {
#pragma unroll
							for (int k = 0; k < kHistChunks; ++k) {
								if (s2 == kSentinel) {
									const uint64_t m = __ballot(hsR[k] == x);
									if (m) { const uint32_t l = ffs64(m); s2 = 64u * k + l; ok = rdlane(hfR[k], l) == rdlane(fVl, j); }
								}
							}
						}
						if (s2 == kSentinel && ((X2 >> j) & 1u)) {
							s2 = rdlane(r2, j);
							ok = rdlane((uint32_t)f2, j) != 0u;
						} else if (s2 == kSentinel) {
							const uint64_t m = __ballot(cr && sR == x) & mask_le(j);
							if (m) { const uint32_t l = ffs64(m); s2 = b0 + l; ok = rdlane(fRl, l) == rdlane(fVl, j); }
						}
						if (ok) {
							const uint32_t e = src.extend(v0 + t, r0 + s2, umin32(vl - (v0 + t), rl - (r0 + s2)));
							if (e >= p) { matched = true; vm = v0 + t; rm = r0 + s2; ml = e; break; }
						}
					}
				}
				if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_C, PROF_NOW() - tc0);
			}
		}
		if constexpr (Src::kPhaseA) PROF_ADD(src, P_T_BC, PROF_NOW() - tb);
		if (members && in_table) release_table();   // member mode: held for this epoch only
		if (!matched) break;

		// emit ADD (implicit gap) + COPY, flush the tables (:243-263)
		if (nrec >= rec_cap) { st = 7; break; }
		if constexpr (!Src::kPhaseA) {   // HBM-direct source: the payload word from V
			if (vm > v0) {
				uint32_t w = 0;
				for (uint32_t k = 0; k < 4 && v0 + k < vl; ++k) w |= (uint32_t)src.V[v0 + k] << (8 * k);
				pw = w;
			}
		}
		if (members) nb_note();
		if (lane < 4) rec[kRecWordsOnepass * nrec + lane] = lane == 0 ? vm : (lane == 1 ? rm : (lane == 2 ? ml : pw));
		++nrec;
		dsz += 13 + (vm > v0 ? 9 + (uint64_t)(vm - v0) : 0);
		v0 = vm + ml;
		r0 = rm + ml;
		at_mismatch = true;
	}
	if (members && st == 0) {
		nb_close();
		if (nseg < seg_cap) {
			if (lane == 0) *(uint4*)(sgp + 4ull * nseg) = make_uint4(kSegTail, 0u, (uint32_t)(dsz - 1), v0);
		} else {
			st = kStatusInternal;
		}
		++nseg;
		if (lane == 0) a.nseg[pair] = nseg;
	}
	constexpr bool routed = kRouted && !members;   // the plain chain for a pair of a member plan
	if (routed && st == 0 && lane == 0) {
		// the member serialiser's pieces: every record in one run, then the tail
		uint4* sg = (uint4*)(a.seg + 4ull * ((uint64_t)pp.chunk_base + 2ull * pair));
		uint32_t ns = 0;
		if (nrec) sg[ns++] = make_uint4(0u, nrec, 25u, 0u);
		sg[ns++] = make_uint4(kSegTail, 0u, (uint32_t)(dsz - 1), v0);
		a.nseg[pair] = ns;
	}
	if (v0 < vl) dsz += 9 + (uint64_t)(vl - v0);   // trailing ADD (:268-275)
	if ((members || routed) && (dsz >> 32)) st = 7;   // segment offsets are 32-bit

	if (tslot >= 0) release_table();
	if (lane == 0) {
		a.n_rec[pair] = nrec;
		a.dsize[pair] = dsz;
		a.status[pair] = st;
	}
#ifdef DG_ONEPASS_PROF
	if constexpr (Src::kPhaseA) {
		PROF_ADD(src, P_EPOCHS, nrec);
		if (lane == 0 && pair < kPairProfMax) {
			g_pair_prof[4ull * pair + 2] = src.prof[P_T_BC];
			g_pair_prof[4ull * pair + 3] = src.prof[P_DIAG_CALLS] + src.prof[P_A_ENTRIES] + 1000ull * src.prof[P_RESYNCS];
		}
		if (lane == 0)
			for (int i = 0; i < kProfN; ++i) atomicAdd(&g_onepass_prof[i], (unsigned long long)src.prof[i]);
	}
#endif
	return PairResult{nrec, dsz, st};
}

// p = 16, 16-byte aligned pairs: LDS windows (the hot configuration); the
// member-mode chain is its own instance so the plain chain carries none of
// its registers
template <bool kMembers, bool kRouted = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DG_WAVES_PER_EU, 8))) void onepass16_kernel(EncodeArgs a) {
	__shared__ __attribute__((aligned(16))) uint8_t win[2 * kWinStride];
	__shared__ uint32_t bm[256];   // phase-B bitmaps / batch scratch, member table, round bitmaps
	__shared__ __attribute__((aligned(4))) uint16_t lcache[kListCap];   // the diagonal batch's mismatch list; phase-C chunk bitmaps
	__shared__ __attribute__((aligned(16))) uint8_t touch[kTouchAhead > 0 ? 256 : 4];
	const uint32_t pair = a.pair0 + blockIdx.x;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	if (kMembers || kRouted) {
		if (a.route_min) {
			// member plan, automatic mode: a pair whose chunks verified fewer
			// than route_min members each on average gains nothing from the
			// members (its matches leave diagonal 0) and runs the plain chain
			// (the kRouted instance, launched after the member chain's)
			const uint32_t nch = uni(pp.n_chunks);
			uint32_t v = 0;
			for (uint32_t c = lane_id(); c < nch; c += 64) v += a.csum[2ull * (pp.chunk_base + c)];
			const bool member_pair = rdlane(wave_incl_scan(v), 63) >= a.route_min * nch;
			if (member_pair != kMembers) return;
			if (kRouted && a.route_cnt && lane_id() == 0) atomicAdd(a.route_cnt, 1u);
		}
	}
	WinSrc src;
	src.S[0] = a.ver + pd.v_off;
	src.S[1] = a.ref + pd.r_off;
	src.len[0] = (uint32_t)pd.v_len;
	src.len[1] = (uint32_t)pd.r_len;
	src.base[0] = src.base[1] = 0xFFFF0000u;   // nothing loaded yet (forces a fill)
	src.win = (lds_u8*)win;
	src.touch = (lds_u8*)touch;
	src.lc = lcache;
	src.powc = a.powc;
	PROF_INIT(src)
	[[maybe_unused]] const uint64_t t_start = PROF_NOW_R();
#ifdef DG_ONEPASS_PROF
	if (lane_id() == 0 && pair < kPairProfMax) g_pair_prof[4ull * pair] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef DG_REFILL_PROF
	const uint64_t t_all0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef DG_PAIR_TIME
	const uint64_t t_pt0 = __builtin_amdgcn_s_memrealtime();
#endif
	const PairResult res = onepass_pair<kMembers, WinSrc, kRouted>(src, a, pair, pd, pp, 16u, bm, (uint32_t*)lcache);
#ifdef DG_REFILL_PROF
	if (lane_id() == 0) {
		atomicAdd(&g_refill_prof[0], (unsigned long long)src.refill_cycles);
		atomicAdd(&g_refill_prof[1], (unsigned long long)src.refill_count);
		atomicAdd(&g_refill_prof[2], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_all0));
	}
#endif
	vm_drain();   // no LDS-DMA may outlive the wave's LDS allocation
#ifdef DG_PAIR_TIME
	if (lane_id() == 0 && pair < kPairTimeMax) {
		const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID: wave, simd, cu, se ...
		const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;   // HW_REG_XCC_ID
		g_pair_time[3ull * pair] = t_pt0;
		g_pair_time[3ull * pair + 1] = __builtin_amdgcn_s_memrealtime();
		g_pair_time[3ull * pair + 2] = ((unsigned long long)xcc << 32) | hw;
	}
#endif
	if (!kMembers && !kRouted && a.lookback) {
		// fused placement + serialisation (dg_serialize_wave.h)
		const uint64_t off = lookback_offset(a.lookback, pair, res.dsz);
		const uint32_t lane = lane_id();
		if (lane == 0) {
			a.offsets[pair] = off;
			if (pair + 1 == a.n_pairs) a.offsets[a.n_pairs] = off + res.dsz;
		}
		int32_t st = uni((uint32_t)res.st);
		if (st == 0 && off + res.dsz > a.out_cap) st = 7;
		if (st == 0) {
			vm_drain();   // this wave's record stores have landed
			__builtin_amdgcn_s_waitcnt(0xc07f);
			st = serialize_wave<2 * kWinStride - 32>(a.out + off, res.dsz, a.ver + pd.v_off, (uint32_t)pd.v_len,
			                                         a.rec + (uint64_t)kRecWordsOnepass * pp.rec_base, kRecWordsOnepass,
			                                         res.nrec, (sw_lds8*)win);
		}
		if (lane == 0 && st != res.st) a.status[pair] = st;
	}
#ifdef DG_ONEPASS_PROF
	if (lane_id() == 0) atomicAdd(&g_onepass_prof[P_T_TOTAL], (unsigned long long)(PROF_NOW_R() - t_start));
	if (lane_id() == 0 && pair < kPairProfMax) g_pair_prof[4ull * pair + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// onepass16_kernel for plain plans with both streams' CRC-64/XZ computed by
// the pair's own wave (R and V read once, not again by a
// CRC rows pass beside the kernel).  The wave folds, at every window refill,
// the rows of 64 x 8 bytes its windows have moved past (from L2, where the
// window loads left them) and the rest at the end; two pairs per block share
// one copy of the five-bit row tables (3.25 KiB of LDS; a copy per wave does
// not fit 16 waves per CU beside the windows).  The plan launches no CRC
// pass for such a batch (dg_host.cpp, op_crc).
constexpr uint32_t kOpCrcWaves = 2;
__global__ __launch_bounds__(64 * kOpCrcWaves) __attribute__((amdgpu_waves_per_eu(4, 8))) void onepass16_crc_kernel(EncodeArgs a) {
	__shared__ __attribute__((aligned(16))) uint8_t win[kOpCrcWaves][2 * kWinStride];
	__shared__ uint32_t bm[kOpCrcWaves][256];
	__shared__ __attribute__((aligned(4))) uint16_t lcache[kOpCrcWaves][kListCap];
	__shared__ __attribute__((aligned(16))) uint8_t touch[kOpCrcWaves][kTouchAhead > 0 ? 256 : 4];
	__shared__ __attribute__((aligned(256))) uint64_t T5[32 * kCrc5Tabs8];
	for (uint32_t i = threadIdx.x; i < 32 * kCrc5Tabs8; i += 64 * kOpCrcWaves) T5[i] = a.crc_tab[kCrc5R8 + i];
	__syncthreads();   // (the block's only barrier: each wave runs its own pair after it)
	const uint32_t w = threadIdx.x >> 6;
	const uint32_t pair = a.pair0 + blockIdx.x * kOpCrcWaves + w;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	WinSrcT<true> src;
	src.S[0] = a.ver + pd.v_off;
	src.S[1] = a.ref + pd.r_off;
	src.len[0] = (uint32_t)pd.v_len;
	src.len[1] = (uint32_t)pd.r_len;
	src.base[0] = src.base[1] = 0xFFFF0000u;   // nothing loaded yet (forces a fill)
	src.win = (lds_u8*)win[w];
	src.touch = (lds_u8*)touch[w];
	src.lc = lcache[w];
	src.powc = a.powc;
	src.crc_init(lds_addr(T5));
	PROF_INIT(src)
	(void)onepass_pair<false, WinSrcT<true>, false>(src, a, pair, pd, pp, 16u, bm[w], (uint32_t*)lcache[w]);
	vm_drain();   // no LDS-DMA may outlive the wave's use of its windows
	const uint64_t cv = src.crc_final(0, a.crc_tab);
	const uint64_t cr = src.crc_final(1, a.crc_tab);
	if (lane_id() == 0) {   // (d_crc: per pair the CRC of R, then of V)
		a.crc_out[2ull * pair] = cr;
		a.crc_out[2ull * pair + 1] = cv;
	}
}

// any seed length or alignment, bytes from HBM/L2
template <int PF>
__global__ __launch_bounds__(64, 4) void onepass_kernel(EncodeArgs a) {
	__shared__ uint32_t bm[128];
	__shared__ uint32_t cscr[64];   // phase-C chunk bitmaps
	const uint32_t pair = blockIdx.x;
	if (pair >= a.n_pairs) return;
	const PairDev pd = a.pairs[pair];
	const PairPlanDev pp = a.pplan[pair];
	GlobalSrc<PF> src{a.ver + pd.v_off, a.ref + pd.r_off, PF > 0 ? (uint32_t)PF : a.p, a.powc};
	onepass_pair<false>(src, a, pair, pd, pp, src.p, bm, cscr);
}

// DG_ONEPASS_GLOBAL=1 forces the HBM-direct kernel (A/B builds only)
static bool force_global_src() {
	const char* e = ab_env("DG_ONEPASS_GLOBAL");
	return e && e[0] == '1';
}

bool onepass16_selected() { return !force_global_src(); }

// DG_OP_LDS_PAD=bytes: dynamic LDS added to the onepass16 launches, which caps
// the resident chains per CU (A/B builds only: occupancy experiments)
static uint32_t op_lds_pad() {
	const char* e = ab_env("DG_OP_LDS_PAD");
	return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
}

hipError_t launch_onepass(const EncodeArgs& a, uint32_t p, bool aligned16, hipStream_t st, hipEvent_t routed_after) {
	if (a.n_pairs == 0) return hipSuccess;
	if (p == 16 && aligned16 && !force_global_src()) {
		if (a.srec) {   // member plan: the member chain, and the plain chain for routed pairs
			// (pairs [pair0, n_pairs): one group of a pipelined run)
			const uint32_t g = a.n_pairs - a.pair0;
			if (g == 0) return hipSuccess;
			hipLaunchKernelGGL(onepass16_kernel<true>, dim3(g), dim3(64), op_lds_pad(), st, a);
			if (a.route_min) {
				if (routed_after) {
					const hipError_t e = hipStreamWaitEvent(st, routed_after, 0);
					if (e != hipSuccess) return e;
				}
				hipLaunchKernelGGL((onepass16_kernel<false, true>), dim3(g), dim3(64), op_lds_pad(), st, a);
			}
		} else if (a.crc_out) {   // plain plan, CRCs in the kernel
			const uint32_t g = a.n_pairs - a.pair0;
			if (g) hipLaunchKernelGGL(onepass16_crc_kernel, dim3((g + kOpCrcWaves - 1) / kOpCrcWaves),
			                          dim3(64 * kOpCrcWaves), 0, st, a);
		} else {
			hipLaunchKernelGGL(onepass16_kernel<false>, dim3(a.n_pairs), dim3(64), op_lds_pad(), st, a);
		}
	}
	else if (a.lookback)
		return hipErrorInvalidValue;   // fused serialisation needs onepass16_kernel
	else if (p == 16)
		hipLaunchKernelGGL(onepass_kernel<16>, dim3(a.n_pairs), dim3(64), 0, st, a);
	else
		hipLaunchKernelGGL(onepass_kernel<0>, dim3(a.n_pairs), dim3(64), 0, st, a);
	return hipGetLastError();
}

#ifdef DG_ONEPASS_PROF
extern "C" int dg_onepass_prof_read(unsigned long long* out, int n) {
	if (n > kProfN) n = kProfN;
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_onepass_prof), sizeof(unsigned long long) * n) != hipSuccess) return -1;
	return n;
}
extern "C" int dg_onepass_pair_prof_read(unsigned long long* out, int n_pairs) {
	if (n_pairs > (int)kPairProfMax) n_pairs = (int)kPairProfMax;
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pair_prof), 32ull * n_pairs) != hipSuccess) return -1;
	return n_pairs;
}
extern "C" int dg_onepass_prof_reset(void) {
	unsigned long long z[kProfN] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_onepass_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace dg
