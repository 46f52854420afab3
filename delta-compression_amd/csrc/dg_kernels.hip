// dg_kernels.hip — CDNA4 (gfx950) kernels of the delta codec.
//
//   crc_rows_kernel / crc_rows_wide_kernel / crc_finalize_kernel  CRC-64/XZ
//       of every R and V (segment folds in dg_crc.h)
//       (src/c/delta.h:294-322; main.c:259-260)
//   onepass_kernel   one wave64 per pair, onepass differencing
//       (src/c/onepass.c:32-297) in its epoch form
//   scan_sizes_kernel  exclusive scan of per-pair delta sizes
//   serialize_wave_kernel   placement + DLT\x03 serialisation
//       (src/c/apply.c:136-164, src/c/encoding.c:39-90)
//   synth_*            synthetic batch generators (bench/test inputs)
//
// Written for wave64 / gfx950 only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dg_device.h"
#include "dg_devutil.h"
#include "dg_crc.h"
#include "dg_serialize_wave.h"

namespace dg {

// ───────────────────────────── scan of sizes ──────────────────────────────

// One block: each thread sums a contiguous run of ceil(n / 1024) sizes, the
// block scans the 1024 run sums (wave shuffles + 16 wave totals in LDS), and
// each thread writes its run's exclusive offsets.  One barrier pair.
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x) {
	const uint32_t lane = lane_id();
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d, 64);
		const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d, 64);
		if (lane >= (uint32_t)d) x += ((uint64_t)hi << 32) | lo;
	}
	return x;
}

__global__ __launch_bounds__(1024) void scan_sizes_kernel(const uint64_t* __restrict__ sz,
                                                          uint64_t* __restrict__ off, uint32_t n,
                                                          uint32_t* route_cnt, uint32_t* route_fb) {
	__shared__ uint64_t wsum[16];
	const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
	if (route_cnt && tid == 0) {
		// member plans: the pairs the run routed to the plain chain, for the
		// host's next run (dg_host.cpp, chain_join); zeroed for that run
		__hip_atomic_store(route_fb, *route_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		*route_cnt = 0u;
	}
	const uint32_t per = (n + 1023) / 1024;
	const uint32_t b = tid * per, e = min(b + per, n);
	uint64_t s = 0;
	for (uint32_t k = b; k < e; ++k) s += sz[k];
	const uint64_t incl = wave_incl_scan64(s);
	if (lane == 63) wsum[wave] = incl;
	__syncthreads();
	if (wave == 0) {
		const uint64_t w = lane < 16 ? wsum[lane] : 0;
		const uint64_t wi = wave_incl_scan64(w);
		if (lane < 16) wsum[lane] = wi - w;   // exclusive wave offsets
	}
	__syncthreads();
	uint64_t run = wsum[wave] + incl - s;
	for (uint32_t k = b; k < e; ++k) {
		off[k] = run;
		run += sz[k];
	}
	if (tid == 1023) off[n] = wsum[15] + incl;   // the grand total (thread 1023 holds the last run)
}

// ───────────────────────────── CRC-64/XZ ──────────────────────────────────
//
// Tables (built on the host, uploaded once per context; dg_device.h):
//   slice[8][256]    slicing-by-8 tables of the reflected polynomial
//   lvl[6][256]      nibble tables of "multiply by x^(8*1024*2^l) mod P"
//   the row tables and per-lane constants of dg_crc.h
// The raw CRC (init 0, no xorout) is linear, leading zero bytes are no-ops
// and init = ~0 equals XOR-ing 0xFF into the first 8 data bytes, so each
// segment is hashed from a zero register over a zero-front-padded span and
// the segments are combined as c_left * x^(8*len_right) ^ c_right.

// ── row-interleaved segments (dg_crc.h) ──

// Wide: 16-byte pieces (8 of the 16 lookups per piece do not wait for the
// register), the 16 tables in 32 KiB, one 1024-thread block per CU: for a CRC
// pass that has the GPU to itself.  (Four bank-spread table copies, 128 KiB,
// measured slower: 4.8 vs 5.1 TB/s alone, profiles/r05_crc_lab_product.txt.)
constexpr uint32_t kCrcWideBlock = 1024;
template <uint32_t kBlock = kCrcWideBlock>
__global__ __launch_bounds__(kBlock) void crc_rows_wide_kernel(CrcArgs a) {
	__shared__ __attribute__((aligned(256))) uint64_t TW[16 * 256];
	for (uint32_t i = threadIdx.x; i < 16 * 256; i += kBlock) TW[i] = a.tables[kCrcRows16 + i];
	__syncthreads();
	const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
	const uint32_t tb = lds_addr(TW), tbh = tb + 8u * 2048u;
	const uint64_t kl = a.tables[kCrcRowK16 + lane];
	constexpr uint32_t kWaves = kBlock / 64;
	for (uint32_t seg = uni(blockIdx.x * kWaves + wave); seg < a.n_segs; seg += gridDim.x * kWaves) {
		const CrcSegDev sd = a.segs[seg];
		const CrcSpanDev sp = a.spans[sd.span];
		const uint64_t c = crc_seg_rows<16, 1, 4>((uintptr_t)(a.arena[sp.which] + sp.off), sp.len, sp.nseg, sd.j, tb,
		                                          tbh, kl);
		if (lane == 0) a.seg_crc[seg] = c;
	}
}

// Beside another kernel: 8-byte pieces, one table copy (byte tables: 16 KiB;
// five-bit tables: 3.25 KiB), DG_CRC_PF (byte tables) / DG_CRC_PF5 (five-bit)
// pieces per lane per batch (two batches in flight), at most 72 VGPRs (a
// register budget for 7 blocks per CU).  Four pieces per batch: byte tables
// (58 VGPRs) C2 1762 -> 1801-1819 GiB/s beside the onepass kernel; five-bit
// tables (67 VGPRs; at a 64-VGPR budget they spilled) c6 1340 -> 1358
// (profiles/r06_experiments.md).
#ifndef DG_CRC_PF
#define DG_CRC_PF 4
#endif
#ifndef DG_CRC_PF5
#define DG_CRC_PF5 4
#endif
#ifndef DG_CRC_BESIDE_WIDE
#define DG_CRC_BESIDE_WIDE 0
#endif
#ifndef DG_CRC_PRIO   // A/B: issue priority of the rows pass beside another kernel (0..3)
#define DG_CRC_PRIO 0
#endif
#ifndef DG_CRC_MINBLOCKS   // blocks per CU the register budget is sized for (7: 72 VGPRs, 8: 64)
#define DG_CRC_MINBLOCKS 7
#endif
template <int TAB>
__global__ __launch_bounds__(256, DG_CRC_MINBLOCKS) void crc_rows_kernel(CrcArgs a) {
	if constexpr (DG_CRC_PRIO > 0) __builtin_amdgcn_s_setprio(DG_CRC_PRIO);
	constexpr uint32_t nt = TAB == kCrcByte ? 8 * 256 : 32 * kCrc5Tabs8;
	__shared__ __attribute__((aligned(256))) uint64_t T8[nt];
	for (uint32_t i = threadIdx.x; i < nt; i += 256) T8[i] = a.tables[(TAB == kCrcByte ? kCrcRows8 : kCrc5R8) + i];
	__syncthreads();
	const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
	const uint32_t tb = lds_addr(T8);
	const uint64_t kl = a.tables[kCrcRowK8 + lane];
	bool raised = false;
	for (uint32_t seg = uni(blockIdx.x * kCrcWavesPerBlock + wave); seg < a.n_segs;
	     seg += gridDim.x * kCrcWavesPerBlock) {
		if (a.prio_flag && !raised) {
			// member plans: once the member kernel is done, the rows pass
			// outranks the chains beside it (the routed plain chain's waves
			// otherwise leave it the last issue slots)
			if (uni(__hip_atomic_load(a.prio_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
				__builtin_amdgcn_s_setprio(1);
				raised = true;
			}
		}
		const CrcSegDev sd = a.segs[seg];
		const CrcSpanDev sp = a.spans[sd.span];
		const uint64_t c = crc_seg_rows<8, 1, TAB == kCrcByte ? DG_CRC_PF : DG_CRC_PF5, kCrcSegBytes, false, TAB>(
		    (uintptr_t)(a.arena[sp.which] + sp.off), sp.len, sp.nseg, sd.j, tb, tb, kl);
		if (lane == 0) a.seg_crc[seg] = c;
	}
}

__global__ __launch_bounds__(64) void crc_finalize_kernel(CrcArgs a) {
	const uint32_t i = blockIdx.x * 64 + threadIdx.x;
	if (i >= a.n_spans) return;
	const CrcSpanDev sp = a.spans[i];
	uint64_t crc;
	if (sp.len < 8) {
		const uint8_t* d = a.arena[sp.which] + sp.off;
		uint64_t c = ~0ULL;
		for (uint64_t k = 0; k < sp.len; ++k) c = a.tables[(uint8_t)(c ^ d[k])] ^ (c >> 8);
		crc = ~c;
	} else {
		// constant multiplications by nibble tables (16 cached loads instead
		// of a 64-step bit-serial product), skipped where they are trivial
		const uint64_t* KS = a.tables + 8 * 256 + kCrcLevels * kCrcNibTabWords;   // x^(8 kCrcSegBytes)
		uint64_t acc = 0;
		for (uint32_t j = 0; j < sp.nseg; ++j)
			acc = (j ? mul_nib(acc, KS) : 0ull) ^ a.seg_crc[sp.seg_base + j];
		const uintptr_t end = (uintptr_t)(a.arena[sp.which] + sp.off) + sp.len;
		const uint32_t t = (uint32_t)(((end + 15) & ~(uintptr_t)15) - end);
		if (t) acc = mul_nib(acc, KS + (1 + t) * kCrcNibTabWords);   // undo the trailing pad bytes (x^-8t)
		crc = ~acc;
	}
	a.out[sp.out] = crc;
}

// ───────────────────────────── synthetic inputs ───────────────────────────

__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t k) {
	uint64_t z = seed + k * 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

// R_i = splitmix64 bytes (seed_base + i); V_i = R_i (edits applied after)
__global__ __launch_bounds__(256) void synth_random_kernel(uint8_t* ref, uint8_t* ver,
                                                           uint64_t pair_len, uint64_t seed_base,
                                                           uint64_t words_total) {
	const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (w >= words_total) return;
	const uint64_t words_per_pair = (pair_len + 7) / 8;
	const uint64_t pair = w / words_per_pair, k = w % words_per_pair;
	const uint64_t val = splitmix_at(seed_base + pair, k + 1);
	const uint64_t off = pair * pair_len + 8 * k;
	if (8 * k + 8 <= pair_len) {
		uint8_t* r = ref + off;
		uint8_t* v = ver + off;
		for (int b = 0; b < 8; ++b) { r[b] = (uint8_t)(val >> (8 * b)); v[b] = (uint8_t)(val >> (8 * b)); }
	} else {
		for (uint64_t b = 0; 8 * k + b < pair_len; ++b) {
			ref[off + b] = (uint8_t)(val >> (8 * b));
			ver[off + b] = (uint8_t)(val >> (8 * b));
		}
	}
}

__global__ __launch_bounds__(64) void synth_edits_kernel(uint8_t* ver, uint32_t n_pairs,
                                                         uint64_t pair_len, uint64_t seed_base,
                                                         uint64_t n_edits) {
	const uint32_t pair = blockIdx.x * 64 + threadIdx.x;
	if (pair >= n_pairs || pair_len == 0) return;
	const uint64_t s = (seed_base + pair) ^ 0xD1B54A32D192ED03ULL;
	uint8_t* v = ver + (uint64_t)pair * pair_len;
	for (uint64_t e = 0; e < n_edits; ++e) {
		const uint64_t pos = splitmix_at(s, 2 * e + 1) % pair_len;
		v[pos] = (uint8_t)splitmix_at(s, 2 * e + 2);
	}
}

// Transposition pairs (tests/gen_transpositions.py recipe, planned on the
// host): R bytes are the splitmix64 stream of the pair's seed; V is R's
// blocks in permuted order, one copy command per block.
__global__ __launch_bounds__(256) void synth_stream_kernel(uint8_t* ref, const SynthSpan* spans,
                                                           uint32_t n) {
	const uint32_t i = blockIdx.y;
	if (i >= n) return;
	const SynthSpan sp = spans[i];
	const uint64_t words = (sp.len + 7) / 8;
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < words; k += (uint64_t)gridDim.x * 256) {
		const uint64_t val = splitmix_at(sp.seed, k + 1);
		uint8_t* r = ref + sp.off + 8 * k;
		for (uint64_t b = 0; b < 8 && 8 * k + b < sp.len; ++b) r[b] = (uint8_t)(val >> (8 * b));
	}
}

__global__ __launch_bounds__(256) void synth_copy_kernel(uint8_t* ver, const uint8_t* ref,
                                                         const SynthCopy* cmds, uint32_t n) {
	const SynthCopy c = cmds[blockIdx.x];
	for (uint64_t b = threadIdx.x; b < c.len; b += 256) ver[c.dst + b] = ref[c.src + b];
}

// Shift pairs (oracle/delta_oracle.c or_synth_shift): V = R with one edit per
// stratum of R — a substitution, or an insertion / deletion of 1..8 bytes.
// One block per pair; thread t takes a contiguous range of strata, the
// block's exclusive scan of their length changes places them in V.
struct ShiftEdit {
	uint64_t pos, k, bytes;
	uint32_t kind;   // 0 substitution, 1 insertion, 2 deletion
};
__device__ __forceinline__ ShiftEdit shift_edit(uint64_t s, uint64_t e, uint64_t a, uint64_t b, uint32_t pct) {
	const uint64_t h1 = splitmix_at(s, 3 * e + 1), h2 = splitmix_at(s, 3 * e + 2), h3 = splitmix_at(s, 3 * e + 3);
	ShiftEdit x;
	x.pos = a + h1 % (b - a);
	const uint64_t u = h2 % 100;
	x.k = 1 + (h2 >> 32) % 8;
	x.bytes = h3;
	x.kind = 2 * u < pct ? 1u : (u < pct ? 2u : 0u);
	if (x.kind == 2 && x.k > b - x.pos) x.k = b - x.pos;
	return x;
}
__global__ __launch_bounds__(256) void synth_shift_kernel(uint8_t* ver, const uint8_t* ref, const SynthSpan* spans,
                                                          const uint64_t* v_off, uint32_t n_pairs, uint64_t n_edits,
                                                          uint32_t pct) {
	__shared__ int64_t part[256];
	const uint32_t i = blockIdx.x, tid = threadIdx.x;
	if (i >= n_pairs) return;
	const SynthSpan sp = spans[i];
	const uint64_t len = sp.len;
	const uint8_t* R = ref + sp.off;
	uint8_t* V = ver + v_off[i];
	const uint64_t n = n_edits < len ? n_edits : len;
	if (n == 0) {
		for (uint64_t b = tid; b < len; b += 256) V[b] = R[b];
		return;
	}
	const uint64_t s = sp.seed ^ 0x2545F4914F6CDD1DULL, S = len / n;
	const uint64_t e0 = n * tid / 256, e1 = n * (tid + 1) / 256;
	auto bounds = [&](uint64_t e, uint64_t& a, uint64_t& b) {
		a = e * S;
		b = e + 1 == n ? len : (e + 1) * S;
	};
	int64_t d = 0;
	for (uint64_t e = e0; e < e1; ++e) {
		uint64_t a, b;
		bounds(e, a, b);
		const ShiftEdit x = shift_edit(s, e, a, b, pct);
		d += x.kind == 1 ? (int64_t)x.k : (x.kind == 2 ? -(int64_t)x.k : 0);
	}
	part[tid] = d;
	__syncthreads();
	int64_t before = 0;
	for (uint32_t t = 0; t < tid; ++t) before += part[t];
	uint64_t o = (uint64_t)((int64_t)(e0 * S) + before);
	for (uint64_t e = e0; e < e1; ++e) {
		uint64_t a, b;
		bounds(e, a, b);
		const ShiftEdit x = shift_edit(s, e, a, b, pct);
		for (uint64_t p = a; p < x.pos; ++p) V[o++] = R[p];
		if (x.kind == 1) {
			for (uint64_t j = 0; j < x.k; ++j) V[o++] = (uint8_t)(x.bytes >> (8 * j));
			for (uint64_t p = x.pos; p < b; ++p) V[o++] = R[p];
		} else if (x.kind == 2) {
			for (uint64_t p = x.pos + x.k; p < b; ++p) V[o++] = R[p];
		} else {
			V[o++] = (uint8_t)x.bytes;
			for (uint64_t p = x.pos + 1; p < b; ++p) V[o++] = R[p];
		}
	}
}

}  // namespace dg

// ───────────────────────────── launchers (C++ linkage, internal) ──────────

namespace dg {

hipError_t launch_synth_shift(uint8_t* ref, uint8_t* ver, const SynthSpan* spans, const uint64_t* v_off,
                              uint32_t n, uint64_t n_edits, uint32_t pct, hipStream_t st) {
	if (!n) return hipSuccess;
	hipLaunchKernelGGL(synth_stream_kernel, dim3(64, n), dim3(256), 0, st, ref, spans, n);
	hipLaunchKernelGGL(synth_shift_kernel, dim3(n), dim3(256), 0, st, ver, ref, spans, v_off, n, n_edits, pct);
	return hipGetLastError();
}

hipError_t launch_synth_transpose(uint8_t* ref, uint8_t* ver, const SynthSpan* spans, uint32_t n_spans,
                                  const SynthCopy* cmds, uint32_t n_cmds, hipStream_t st) {
	if (n_spans) hipLaunchKernelGGL(synth_stream_kernel, dim3(64, n_spans), dim3(256), 0, st, ref, spans, n_spans);
	if (n_cmds) hipLaunchKernelGGL(synth_copy_kernel, dim3(n_cmds), dim3(256), 0, st, ver, ref, cmds, n_cmds);
	return hipGetLastError();
}

// One wave per pair (dg_serialize_wave.h): DPP scans instead of block
// barriers, 64 commands per tile staged in a 4 KiB LDS slice, so 32 pairs
// per CU are in flight and their record / payload loads overlap.  The header
// CRC bytes are left to crc_patch_kernel, so this kernel does not wait for
// the CRC stream.
// (one record per lane per tile: 4 measured slower, C2 +18 %, C3 3.6x)
#ifndef DG_SER_PIPE   // A/B: 1 = the LDS-DMA pipeline (serialize_pipe, 2 KiB stage), C2 37.7 -> 74.9 us
#define DG_SER_PIPE 0
#endif
constexpr bool kSerPipe = DG_SER_PIPE != 0;
constexpr uint32_t kSerWaveStage = kSerPipe ? 2048 : 4096;   // (pipeline rings beside a 2 KiB stage: 16 waves per CU)
constexpr uint32_t kSerWaveLds = kSerPipe ? pipe_lds_bytes<kSerWaveStage>() : kSerWaveStage + 32;

__global__ __launch_bounds__(64) void serialize_wave_kernel(SerArgs s) {
	__shared__ __attribute__((aligned(16))) uint8_t stage[kSerWaveLds];
	const uint32_t pair = blockIdx.x;
	const uint64_t base = s.offsets[pair];
	const uint64_t end = s.offsets[pair + 1];
	if (end > s.out_cap) {
		if (lane_id() == 0) s.status[pair] = 7;
		return;
	}
	if (s.status[pair] != 0) return;
	const PairDev pd = s.pairs[pair];
	const PairPlanDev pp = s.pplan[pair];
	const int32_t st = serialize_wave<kSerWaveStage, kSerPipe>(s.out + base, end - base, s.ver + pd.v_off,
	                                                 (uint32_t)pd.v_len, s.rec + (uint64_t)s.rec_words * pp.rec_base,
	                                                 s.rec_words, s.n_rec[pair], (sw_lds8*)stage);
	if (st != 0 && lane_id() == 0) s.status[pair] = st;
	if (st == 0 && s.crc_in) {   // header bytes 9..24: CRC of R, CRC of V, big-endian (encoding.c:52-54)
		const uint32_t lane = lane_id();
		if (lane < 16) {
			const uint64_t c = s.crc[2ull * pair + (lane >> 3)];
			s.out[base + 9 + lane] = (uint8_t)(c >> (56 - 8 * (lane & 7)));
		}
	}
}

// header bytes 9..24 (src/dst CRC, big-endian, encoding.c:52-54) of deltas
// serialised before their CRCs were known
__global__ __launch_bounds__(256) void crc_patch_kernel(uint8_t* out, const uint64_t* offsets,
                                                        const uint64_t* crc, const int32_t* status,
                                                        uint32_t n) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i >= n || status[i] != 0) return;
	uint8_t* h = out + offsets[i];
	const uint64_t cs = crc[2ull * i], cd = crc[2ull * i + 1];
	for (int k = 0; k < 8; ++k) {
		h[9 + k] = (uint8_t)(cs >> (56 - 8 * k));
		h[17 + k] = (uint8_t)(cd >> (56 - 8 * k));
	}
}

hipError_t launch_crc_patch(uint8_t* out, const uint64_t* offsets, const uint64_t* crc,
                            const int32_t* status, uint32_t n, hipStream_t st) {
	if (n) hipLaunchKernelGGL(crc_patch_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out, offsets, crc, status, n);
	return hipGetLastError();
}

hipError_t launch_scan(const uint64_t* sz, uint64_t* off, uint32_t n, hipStream_t st, uint32_t* route_cnt,
                       uint32_t* route_fb) {
	hipLaunchKernelGGL(scan_sizes_kernel, dim3(1), dim3(1024), 0, st, sz, off, n, route_cnt, route_fb);
	return hipGetLastError();
}

hipError_t launch_serialize_wave(const SerArgs& s, hipStream_t st) {
	if (s.n_pairs == 0) return hipSuccess;
	hipLaunchKernelGGL(serialize_wave_kernel, dim3(s.n_pairs), dim3(64), 0, st, s);
	return hipGetLastError();
}

// overlap_cap: grid cap when the CRC runs beside another kernel (0 = none).
// A grid-stride CRC of 2 blocks per CU leaves the co-running kernel its
// issue slots instead of queueing 32 CRC waves per CU behind it (C2: step
// 0.400 -> 0.372 ms).  DG_CRC_BLOCKS overrides (A/B builds only).
hipError_t launch_crc_wide(const CrcArgs& a, uint32_t n_cu, hipStream_t st) {
	if (a.n_segs) {
		const uint32_t blocks = std::min<uint32_t>(n_cu, (a.n_segs + 15) / 16);
		hipLaunchKernelGGL(crc_rows_wide_kernel<kCrcWideBlock>, dim3(blocks), dim3(kCrcWideBlock), 0, st, a);
	}
	if (a.n_spans)
		hipLaunchKernelGGL(crc_finalize_kernel, dim3((a.n_spans + 63) / 64), dim3(64), 0, st, a);
	return hipGetLastError();
}

hipError_t launch_crc_finalize(const CrcArgs& a, hipStream_t st) {
	if (a.n_spans) hipLaunchKernelGGL(crc_finalize_kernel, dim3((a.n_spans + 63) / 64), dim3(64), 0, st, a);
	return hipGetLastError();
}

hipError_t launch_crc(const CrcArgs& a, hipStream_t st, uint32_t overlap_cap, int pass, bool finalize) {
	if (a.n_segs) {
		uint32_t blocks = (a.n_segs + kCrcWavesPerBlock - 1) / kCrcWavesPerBlock;
		static const uint32_t env_cap = [] {
			const char* e = ab_env("DG_CRC_BLOCKS");
			return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
		}();
		const uint32_t cap = env_cap ? env_cap : overlap_cap;
		if (cap && blocks > cap) blocks = cap;
		if (pass == kCrcPassRows5)
			hipLaunchKernelGGL(crc_rows_kernel<kCrcFive>, dim3(blocks), dim3(64 * kCrcWavesPerBlock), 0, st, a);
#if DG_CRC_BESIDE_WIDE   // A/B: 16-byte pieces (32 KiB of tables) in one 4-wave block per CU beside the differencing
		else if (cap)
			hipLaunchKernelGGL(crc_rows_wide_kernel<256>, dim3(std::min<uint32_t>(blocks, cap / 2)), dim3(256), 0, st, a);
#endif
		else
			hipLaunchKernelGGL(crc_rows_kernel<kCrcByte>, dim3(blocks), dim3(64 * kCrcWavesPerBlock), 0, st, a);
	}
	if (finalize) return launch_crc_finalize(a, st);
	return hipGetLastError();
}

hipError_t launch_synth(uint8_t* ref, uint8_t* ver, uint32_t n_pairs, uint64_t pair_len,
                        uint64_t seed_base, uint64_t n_edits, hipStream_t st) {
	const uint64_t words = (uint64_t)n_pairs * ((pair_len + 7) / 8);
	if (words)
		hipLaunchKernelGGL(synth_random_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, st,
		                   ref, ver, pair_len, seed_base, words);
	if (n_edits && n_pairs)
		hipLaunchKernelGGL(synth_edits_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, st, ver,
		                   n_pairs, pair_len, seed_base, n_edits);
	return hipGetLastError();
}

}  // namespace dg

// ───────────────────────────── decode + apply ─────────────────────────────
//
// One wave per delta stream (src/c/encoding.c:111-178 parse,
// src/c/apply.c:229-284 apply).  Lane 0 parses command headers out of an LDS
// window of the stream; commands are applied in batches of up to 64, one per
// lane, when no command of the batch touches bytes another one (earlier in
// stream order) reads or writes; otherwise the batch is replayed strictly in
// order with a wave-wide memmove per command.  Either way the result equals
// the reference's sequential memcpy/memmove replay.  All offsets are bounds
// checked (the reference does not check, apply.c:236-243).

namespace dg {



__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// wave-wide memmove of len bytes (src and dst may overlap)
__device__ void wave_memmove(uint8_t* dst, const uint8_t* src, uint64_t len) {
	const uint32_t lane = lane_id();
	if (len == 0 || dst == src) return;
	const bool backward = dst > src && dst < src + len;
	const uint64_t chunk = 64 * 4;
	const uint64_t nch = (len + chunk - 1) / chunk;
	for (uint64_t c = 0; c < nch; ++c) {
		const uint64_t cc = backward ? nch - 1 - c : c;
		const uint64_t base = cc * chunk + 4ull * lane;
		uint8_t b[4];
#pragma unroll
		for (int k = 0; k < 4; ++k) b[k] = base + k < len ? src[base + k] : 0;
		// every lane's loads of this chunk complete before any store
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int k = 0; k < 4; ++k)
			if (base + k < len) dst[base + k] = b[k];
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__builtin_amdgcn_wave_barrier();
	}
}

__device__ __forceinline__ bool overlap(uint64_t a, uint64_t al, uint64_t b, uint64_t bl) {
	return al && bl && a < b + bl && b < a + al;
}

// Command stream parsing (encoding.c:111-178) is a chain x -> x + |cmd(x)|
// through the stream.  Per 4 KiB window of the stream (staged in LDS):
//   1. every lane computes, for each window offset x it owns, the offset of the
//      next command IF a command started at x (N1), or a code: END, malformed,
//      header cut by the window, next command past the window;
//   2. N2 = N1.N1, N4, N8, N16 by pointer doubling (codes propagate; N16
//      takes N4's place once N8 is built);
//   3. one uniform walk takes 16 commands per step through N16, then at most
//      one N8 step and single steps near the window end; the nodes in between
//      are expanded in parallel.
// So a window of ~300 commands costs ~25 dependent LDS reads instead of ~300
// serial header decodes.  The commands are then applied 64 at a time.
#ifdef DG_ONEPASS_PROF   // profiling build only (make prof): per-phase decode cycles
enum { DP_FILL, DP_LOAD, DP_N1, DP_DBL, DP_WALK, DP_EXP, DP_HDR, DP_COPY, DP_WAIT, DP_WINDOWS, DP_BATCHES, DP_TOTAL,
       DP_ORDERED, DP_C_CMD, DP_C_FLAT, DP_C_BAR, DP_CRC_SYNC, DP_CRC_SEG, DP_CRC_TAIL, kDecProfN };
__device__ unsigned long long g_decode_prof[kDecProfN];
#define DPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define DPROF_ADD(i, t0) (dprof[(i)] += __builtin_amdgcn_s_memtime() - (t0))
#define DPROF_INC(i) (dprof[(i)] += 1)
extern "C" int dg_decode_prof_read(unsigned long long* out, int n) {
	if (n > kDecProfN) n = kDecProfN;
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decode_prof), 8 * n) == hipSuccess ? n : -1;
}
extern "C" int dg_decode_prof_reset(void) {
	unsigned long long z[kDecProfN] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(g_decode_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#else
#define DPROF_T(v) ((void)0)
#define DPROF_ADD(i, t0) ((void)0)
#define DPROF_INC(i) ((void)0)
#endif

constexpr uint32_t kDecWin = 4096;       // bytes of the command stream per window
constexpr uint32_t kDecMaxCmds = 512;    // >= kDecWin / 9 (the shortest command)
constexpr uint16_t kNxEnd = 0xFFFE;      // END at x
constexpr uint16_t kNxBad = 0xFFFD;      // malformed at x
constexpr uint16_t kNxCut = 0xFFFF;      // header not complete in the window: restart at x
constexpr uint16_t kNxFar = 0xFFFC;      // complete command at x, next one at/after the window end
constexpr uint16_t kNxSpecial = 0xFFFC;  // codes are >= this

// inclusive prefix sum over the wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t dec_incl_scan(uint32_t x) {
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
	return x;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
	for (int d = 32; d >= 1; d >>= 1) {
		const uint32_t y = (uint32_t)__shfl_xor((int)x, d, 64);
		x = x > y ? x : y;
	}
	return x;
}

// ── decode: one 256-thread block (4 waves) per delta stream ──
//
// Per window: all four waves build N1..N8; wave 0 walks; all expand.  The
// window's commands are then applied 64 per wave at a time, all four waves
// at once, when the window is provably order-free: destinations increasing
// and disjoint in stream order and no in-place COPY that moves (src == dst
// in-place copies are no-ops).  Any other window is applied by wave 0 alone,
// batch by batch, with the conflict check and the strict memmove replay.
// The block barrier between windows also orders every store of one window
// before the next window's reads and writes.
constexpr uint32_t kDecBlock = 256;
constexpr uint32_t kDecCrcSeg = 16384;                // in-kernel CRC: 16 KiB segments
static_assert(4 * kDecCrcSeg == kCrcSegBytes, "the Horner step (4 segments) is x^(8 kCrcSegBytes)");

// A block barrier that also orders global memory between the block's waves:
// every wave's stores are acknowledged (vmcnt counts stores on gfx9) before
// any wave passes, and the CU's L1 is invalidated after, so loads of bytes
// another wave of the block just wrote see them.  A plain __syncthreads
// orders LDS only (its workgroup-scope fence waits for no global store), and
// agent-scope fences would write back the XCD's L2 (~6x slower decode).
__device__ __forceinline__ void block_sync_global() {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	asm volatile("buffer_inv sc0" ::: "memory");
}
constexpr uint32_t kDecWaves = kDecBlock / 64;

struct DecCmd {
	bool mine;
	uint32_t kind;
	uint64_t src, dst, len;
};

// big-endian u32 at byte 1 + 4i of a 16-byte header image h[4] (i = 0, 1, 2)
__device__ __forceinline__ uint32_t hdr_be32(const uint32_t (&h)[4], int i) {
	return __builtin_bswap32(__builtin_amdgcn_alignbyte(h[i + 1], h[i], 1));
}

// 16 window bytes at any offset as five aligned dwords and four funnel
// shifts (an unaligned ds_read_b128 stalls the LDS pipe on gfx950,
// profiles/r05_member_census.md; here decode_kernel 0.1115 -> 0.1088 ms at
// C5); the window has 32 bytes of slack.
__device__ __forceinline__ void win16(const uint8_t* p, uint32_t (&h)[4]) {
	const uint32_t mis = (uint32_t)(uintptr_t)p & 3u;
	const uint32_t* d = reinterpret_cast<const uint32_t*>(p - mis);
	const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4], sh = 8u * mis;
	h[0] = __builtin_amdgcn_alignbit(d1, d0, sh);
	h[1] = __builtin_amdgcn_alignbit(d2, d1, sh);
	h[2] = __builtin_amdgcn_alignbit(d3, d2, sh);
	h[3] = __builtin_amdgcn_alignbit(d4, d3, sh);
}

// The window holds >= 16 bytes past any command offset (win has 32 bytes of
// slack), so a header is one 16-byte read.
template <typename WP>
__device__ __forceinline__ DecCmd dec_cmd(WP w, const uint16_t* cmds, uint32_t b, uint32_t cnt, uint64_t pos) {
	DecCmd c{false, 0, 0, 0, 0};
	const uint32_t lane = lane_id();
	c.mine = b + lane < cnt;
	if (c.mine) {
		const uint32_t cx = cmds[b + lane];
		uint32_t h[4];
		win16(w + cx, h);
		c.kind = h[0] & 0xFFu;
		if (c.kind == 1) {
			c.src = hdr_be32(h, 0);
			c.dst = hdr_be32(h, 1);
			c.len = hdr_be32(h, 2);
		} else {
			c.src = pos + cx + 9;   // payload offset in the stream
			c.dst = hdr_be32(h, 0);
			c.len = hdr_be32(h, 1);
		}
	}
	return c;
}

// unaligned dword / 16-byte accesses (gfx950 global memory allows them)
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

// A command's last, partial 16-byte chunk (1 <= rem < 16 bytes).  Every load
// is issued before any store, so the chunk costs one memory round trip: the
// dwords at offsets 0, 4, 8, 12 clamped to rem - 4 (the last one overlaps the
// one before it and stores the same bytes again), or, under 4 bytes, the
// bytes at offsets clamped to rem - 1; never a byte outside [0, rem).
// (Round 5 copied dword by dword and byte by byte, each store before the next
// load: up to 6 dependent round trips per partial chunk.)
#ifndef DG_DEC_TAIL1   // A/B: 0 = round 5's dword-then-byte loop
#define DG_DEC_TAIL1 1
#endif
__device__ __forceinline__ void copy_tail(uint8_t* d, const uint8_t* s, uint32_t rem) {
#if DG_DEC_TAIL1
	if (rem >= 4) {
		uint32_t w[4], o[4];
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			o[k] = umin32(4 * k, rem - 4);
			w[k] = *reinterpret_cast<const u32_u*>(s + o[k]);
		}
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k)
			if (4 * k < rem) *reinterpret_cast<u32_u*>(d + o[k]) = w[k];
	} else {
		uint8_t b[3];
#pragma unroll
		for (uint32_t k = 0; k < 3; ++k) b[k] = s[umin32(k, rem - 1)];
#pragma unroll
		for (uint32_t k = 0; k < 3; ++k)
			if (k < rem) d[k] = b[k];
	}
#else
	const uint32_t nd = rem >> 2;
	for (uint32_t k = 0; k < nd; ++k) *reinterpret_cast<u32_u*>(d + 4 * k) = *reinterpret_cast<const u32_u*>(s + 4 * k);
	for (uint32_t k = 4 * nd; k < rem; ++k) d[k] = s[k];
#endif
}

// Per-wave LDS scratch of the flat copy.
struct DecScratch {
	uint32_t* cum;        // [64] chunk prefix per non-empty command
	uint32_t* row;        // [128] row start masks (lo dwords, then hi dwords)
	const uint8_t** sp;   // [64]
	uint8_t** dp;         // [64]
	uint32_t* len;        // [64] bytes per non-empty command
};

// Copy an independent batch (no command overlaps another one's writes, or
// in-place, reads) in 16-byte chunks: chunk j of the batch's concatenation
// (every command cut into 16-byte chunks, its last one partial) goes to lane
// j % 64 in row j / 64; the owning command comes from per-row start masks
// (owner = starts before the row + popcount(mask bits <= lane) - 1).  Full
// chunks are one unaligned 16-byte load and store; a command's partial last
// chunk is copied by dwords and bytes, never touching the next command's
// bytes.  In-place COPYs whose source and destination overlap are memmoved
// after.
__device__ void dec_flat_batch(const DecCmd& c, bool inplace, uint8_t* O, const uint8_t* R, const uint8_t* D,
                               const DecScratch& x) {
	const uint32_t lane = lane_id();
	const uint8_t* sp = c.kind == 1 ? (inplace ? O + c.src : R + c.src) : D + c.src;
	const bool selfov = c.mine && c.kind == 1 && inplace && c.src != c.dst && overlap(c.src, c.len, c.dst, c.len);
	const bool noop = c.mine && c.kind == 1 && inplace && c.src == c.dst;
	const uint32_t flen = (c.mine && !selfov && !noop) ? (uint32_t)c.len : 0u;
	const uint32_t fch = (flen + 15u) >> 4;
	const uint32_t incl = dec_incl_scan(fch);
	const uint32_t cum = incl - fch;
	const uint32_t total = rdlane(incl, 63);   // chunks
	const bool nz = fch != 0;
	const uint32_t ord = dec_incl_scan(nz ? 1u : 0u) - 1u;
	if (nz) {
		x.cum[ord] = cum;
		x.sp[ord] = sp;
		x.dp[ord] = O + c.dst;
		x.len[ord] = flen;
	}
	for (uint32_t r0 = 0; 64 * r0 < total; r0 += 64) {   // 64 rows of 64 chunks = 64 KiB per round
		x.row[lane] = 0;
		x.row[64 + lane] = 0;
		__builtin_amdgcn_s_waitcnt(0xc07f);
		__builtin_amdgcn_wave_barrier();
		if (nz && cum >= 64 * r0 && cum < 64 * (r0 + 64)) {
			const uint32_t row = cum / 64 - r0, bit = cum % 64;
			atomicOr(&x.row[(bit >> 5) * 64 + row], 1u << (bit & 31));
		}
		const uint32_t carry = (uint32_t)__builtin_popcountll(__ballot(nz && cum < 64 * r0));
		__builtin_amdgcn_s_waitcnt(0xc07f);
		__builtin_amdgcn_wave_barrier();
		const uint64_t mrow = ((uint64_t)x.row[64 + lane] << 32) | x.row[lane];   // row r0 + lane
		const uint32_t pc = (uint32_t)__builtin_popcountll(mrow);
		const uint32_t rbase = carry + dec_incl_scan(pc) - pc;   // starts before row r0 + lane
		const uint32_t nrows = min(64u, (total + 63) / 64 - r0);
		constexpr int kQ = 4;   // rows per pass (VGPR budget: 4 waves per SIMD)
		for (uint32_t q0 = 0; q0 < nrows; q0 += kQ) {
			uint8_t* da[kQ];
			const uint8_t* sa[kQ];
			u32x4_u v[kQ];
			uint32_t rem[kQ];
#pragma unroll
			for (int uu = 0; uu < kQ; ++uu) {
				const uint32_t u = q0 + uu;
				const uint32_t j = 64 * (r0 + u) + lane;
				const bool ok = u < nrows && j < total;
				const uint64_t m = ((uint64_t)rdlane((uint32_t)(mrow >> 32), u) << 32) | rdlane((uint32_t)mrow, u);
				const uint32_t oo = rdlane(rbase, u) + (uint32_t)__builtin_popcountll(m & mask_le(lane));
				const uint32_t o = ok && oo ? oo - 1u : 0u;
				const uint32_t boff = 16u * (j - x.cum[o]);
				rem[uu] = ok ? x.len[o] - boff : 0u;   // >= 1 for a valid chunk
				sa[uu] = x.sp[o] + boff;
				da[uu] = x.dp[o] + boff;
				v[uu] = rem[uu] >= 16 ? *reinterpret_cast<const u32x4_u*>(sa[uu]) : u32x4_u{0, 0, 0, 0};
			}
#pragma unroll
			for (int uu = 0; uu < kQ; ++uu) {
				if (rem[uu] >= 16) {
					*reinterpret_cast<u32x4_u*>(da[uu]) = v[uu];
				} else if (rem[uu]) {   // the command's last, partial chunk
					copy_tail(da[uu], sa[uu], rem[uu]);
				}
			}
		}
	}
	for (uint64_t m = __ballot(selfov); m; m &= m - 1) {
		const uint32_t kk = ffs64(m);
		const uint64_t ks = ((uint64_t)rdlane((uint32_t)(c.src >> 32), kk) << 32) | rdlane((uint32_t)c.src, kk);
		const uint64_t kd = ((uint64_t)rdlane((uint32_t)(c.dst >> 32), kk) << 32) | rdlane((uint32_t)c.dst, kk);
		const uint64_t kl = ((uint64_t)rdlane((uint32_t)(c.len >> 32), kk) << 32) | rdlane((uint32_t)c.len, kk);
		wave_memmove(O + kd, O + ks, kl);
	}
}

// One batch in stream order (wave 0 of a window that is not order-free):
// conflict check among the batch's commands, then the flat copy or the
// strict memmove replay (apply.c:257-266), then a full wait.
__device__ void dec_ordered_batch(const DecCmd& c, uint32_t n, bool inplace, uint8_t* O, const uint8_t* R,
                                  const uint8_t* D, const DecScratch& x) {
	const uint32_t lane = lane_id();
	bool conflict = false;
	const bool reads_buf = inplace && c.kind == 1;
	for (uint32_t k = 0; k + 1 < n; ++k) {
		const uint64_t ks = ((uint64_t)rdlane((uint32_t)(c.src >> 32), k) << 32) | rdlane((uint32_t)c.src, k);
		const uint64_t kd = ((uint64_t)rdlane((uint32_t)(c.dst >> 32), k) << 32) | rdlane((uint32_t)c.dst, k);
		const uint64_t kl = ((uint64_t)rdlane((uint32_t)(c.len >> 32), k) << 32) | rdlane((uint32_t)c.len, k);
		const bool kreads = inplace && rdlane(c.kind, k) == 1;
		if (c.mine && lane > k) {
			if (overlap(kd, kl, c.dst, c.len)) conflict = true;
			if (reads_buf && overlap(kd, kl, c.src, c.len)) conflict = true;
			if (kreads && overlap(ks, kl, c.dst, c.len)) conflict = true;
		}
	}
	if (__ballot(conflict) == 0) {
		dec_flat_batch(c, inplace, O, R, D, x);
	} else {
		for (uint32_t k = 0; k < n; ++k) {
			const uint32_t kk = rdlane(c.kind, k);
			const uint64_t ks = ((uint64_t)rdlane((uint32_t)(c.src >> 32), k) << 32) | rdlane((uint32_t)c.src, k);
			const uint64_t kd = ((uint64_t)rdlane((uint32_t)(c.dst >> 32), k) << 32) | rdlane((uint32_t)c.dst, k);
			const uint64_t kl = ((uint64_t)rdlane((uint32_t)(c.len >> 32), k) << 32) | rdlane((uint32_t)c.len, k);
			wave_memmove(O + kd, kk == 1 ? (inplace ? O + ks : R + ks) : D + ks, kl);
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__builtin_amdgcn_wave_barrier();
}

// ── windows that are not order-free (in-place deltas whose COPYs move):
// conflict-free groups, applied by the whole block ──
//
// The reference replays such a stream strictly in order, one memmove per
// command (apply.c:253-267).  Two commands commute unless one writes bytes
// the other reads or writes, so the window is cut into groups: a group is
// the longest run of consecutive commands none of which conflicts with an
// earlier command of the run.  A group's bytes are independent and are
// copied by all four waves at once in 16-byte chunks; a COPY whose own source
// and destination overlap (a real memmove) is a group of its own, moved by
// the block in 4 KiB passes in the direction that never reads a byte it has
// already written.  Block barriers that order global memory separate groups.
struct DecGroupLds {
	uint32_t* src;    // [kDecMaxCmds] COPY source (O or R offset); ADD: payload offset in the window
	uint32_t* dst;    // [kDecMaxCmds]
	uint32_t* len;    // [kDecMaxCmds]
	uint32_t* pre;    // [kDecMaxCmds + 1] exclusive prefix of the 16-byte chunks each command copies
	int16_t* last;    // [kDecMaxCmds] latest earlier command it conflicts with, -1: none
	uint8_t* flag;    // [kDecMaxCmds] kGf* bits
	uint16_t* gs;     // [kDecMaxCmds + 1] group starts, then cnt
	uint32_t* red;    // [8] block scratch
};
constexpr uint8_t kGfCopy = 1, kGfReadsOut = 2, kGfWrites = 4, kGfSelf = 8;

__device__ __forceinline__ bool ov32(uint32_t a, uint32_t al, uint32_t b, uint32_t bl) {
	return al && bl && a < b + bl && b < a + al;
}

template <typename WP>
__device__ void dec_grouped_window(WP w, const uint16_t* cmds, uint32_t cnt, uint64_t pos, bool inplace, uint8_t* O,
                                   const uint8_t* R, const uint8_t* D, const DecGroupLds& g) {
	const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
	static_assert(kDecMaxCmds == 2 * kDecBlock, "two commands per thread in the prefix");
	// 1. headers -> LDS, flags, chunk counts (two consecutive commands per thread)
	uint32_t f2[2];
#pragma unroll
	for (int u = 0; u < 2; ++u) {
		const uint32_t c = 2 * tid + u;
		f2[u] = 0;
		if (c < cnt) {
			const uint32_t cx = cmds[c];
			uint32_t h[4];
			win16(w + cx, h);
			const bool copy = (h[0] & 0xFFu) == 1u;
			const uint32_t src = copy ? hdr_be32(h, 0) : cx + 9u;
			const uint32_t dst = copy ? hdr_be32(h, 1) : hdr_be32(h, 0);
			const uint32_t len = copy ? hdr_be32(h, 2) : hdr_be32(h, 1);
			const bool noop = inplace && copy && src == dst;   // memmove onto itself
			const bool writes = len != 0 && !noop;
			const bool reads_out = inplace && copy && writes;
			const bool self = reads_out && ov32(src, len, dst, len);
			g.src[c] = src;
			g.dst[c] = dst;
			g.len[c] = len;
			g.flag[c] = (copy ? kGfCopy : 0) | (reads_out ? kGfReadsOut : 0) | (writes ? kGfWrites : 0) |
			            (self ? kGfSelf : 0);
			f2[u] = writes && !self ? (len + 15u) >> 4 : 0u;
		}
	}
	{
		const uint32_t v = f2[0] + f2[1];
		const uint32_t incl = dec_incl_scan(v);
		if (lane == 63) g.red[wave] = incl;
		__syncthreads();
		uint32_t off = 0;
		for (uint32_t k = 0; k < wave; ++k) off += g.red[k];
		g.pre[2 * tid] = off + incl - v;
		g.pre[2 * tid + 1] = off + incl - v + f2[0];
		if (tid == kDecBlock - 1) g.pre[kDecMaxCmds] = off + incl;
	}
	__syncthreads();
	// 2. the latest earlier command each one conflicts with (write/write,
	//    write/read, read/write; only in-place COPYs read the output)
	for (uint32_t c = tid; c < cnt; c += kDecBlock) {
		const uint8_t fc = g.flag[c];
		int32_t L = -1;
		if (fc & kGfWrites) {
			const uint32_t sc = g.src[c], dc = g.dst[c], lc = g.len[c];
			const bool rc = fc & kGfReadsOut;
			for (int32_t e = (int32_t)c - 1; e >= 0; --e) {
				const uint8_t fe = g.flag[e];
				if (!(fe & kGfWrites)) continue;
				const uint32_t se = g.src[e], de = g.dst[e], le = g.len[e];
				if (ov32(de, le, dc, lc) || (rc && ov32(de, le, sc, lc)) || ((fe & kGfReadsOut) && ov32(se, le, dc, lc))) {
					L = e;
					break;
				}
			}
		}
		g.last[c] = (int16_t)L;
	}
	__syncthreads();
	// 3. group starts (wave 0): a group ends before the first command that
	//    conflicts with one of the group's, and around every self-overlapping move
	if (wave == 0) {
		uint32_t s = 0, ng = 1;
		if (lane == 0) g.gs[0] = 0;
		for (uint32_t c0 = 1; c0 < cnt; c0 += 64) {
			const uint32_t c = c0 + lane;
			const bool live = c < cnt;
			const int32_t lc = live ? (int32_t)g.last[c] : -1;
			const bool sf = live && ((g.flag[c] & kGfSelf) || (g.flag[c - 1] & kGfSelf));
			for (;;) {
				const uint64_t m = __ballot(live && c > s && (lc >= (int32_t)s || sf));
				if (!m) break;
				const uint32_t b = c0 + ffs64(m);
				if (lane == 0) g.gs[ng] = (uint16_t)b;
				++ng;
				s = b;
			}
		}
		if (lane == 0) {
			g.gs[ng] = (uint16_t)cnt;
			g.red[4] = ng;
		}
	}
	__syncthreads();
	const uint32_t ng = g.red[4];
	// 4. the groups, in stream order
	for (uint32_t k = 0; k < ng; ++k) {
		const uint32_t s = g.gs[k], e = g.gs[k + 1];
		if (e == s + 1 && (g.flag[s] & kGfSelf)) {
			// one in-place COPY onto an overlapping range: memmove by the block
			const uint32_t len = g.len[s];
			const uint8_t* sp = O + g.src[s];
			uint8_t* dp = O + g.dst[s];
			const bool backward = dp > sp;
			const uint32_t npass = (len + 16u * kDecBlock - 1) / (16u * kDecBlock);
			for (uint32_t q = 0; q < npass; ++q) {
				const uint32_t pass = backward ? npass - 1 - q : q;
				const uint32_t b = pass * 16u * kDecBlock + 16u * tid;
				const uint32_t n = b < len ? umin32(len - b, 16u) : 0u;
				u32x4_u v{0, 0, 0, 0};
				uint8_t t[16];
				if (n == 16) {
					v = *reinterpret_cast<const u32x4_u*>(sp + b);
				} else {
					for (uint32_t i = 0; i < n; ++i) t[i] = sp[b + i];
				}
				// every thread's loads of this pass land before any store of
				// it; later passes read only bytes no earlier pass wrote
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				__syncthreads();
				if (n == 16) {
					*reinterpret_cast<u32x4_u*>(dp + b) = v;
				} else {
					for (uint32_t i = 0; i < n; ++i) dp[b + i] = t[i];
				}
			}
		} else {
			// independent commands: chunk j of the group -> thread j % 256
			const uint32_t j0 = g.pre[s], j1 = g.pre[e];
			constexpr int kQ = 4;   // chunks in flight per thread
			for (uint32_t jb = j0; jb < j1; jb += kQ * kDecBlock) {
				uint8_t* da[kQ];
				const uint8_t* sa[kQ];
				u32x4_u v[kQ];
				uint32_t rem[kQ];
#pragma unroll
				for (int u = 0; u < kQ; ++u) {
					const uint32_t j = jb + u * kDecBlock + tid;
					rem[u] = 0;
					da[u] = O;
					sa[u] = O;
					if (j < j1) {
						uint32_t lo = s, hi = e;   // the command holding chunk j: pre[lo] <= j < pre[lo + 1]
						while (hi - lo > 1) {
							const uint32_t mid = (lo + hi) >> 1;
							if (g.pre[mid] <= j) lo = mid;
							else hi = mid;
						}
						const uint32_t boff = 16u * (j - g.pre[lo]);
						rem[u] = g.len[lo] - boff;
						const uint8_t fl = g.flag[lo];
						sa[u] = ((fl & kGfCopy) ? ((fl & kGfReadsOut) ? O : R) + g.src[lo] : D + pos + g.src[lo]) + boff;
						da[u] = O + g.dst[lo] + boff;
					}
					v[u] = rem[u] >= 16 ? *reinterpret_cast<const u32x4_u*>(sa[u]) : u32x4_u{0, 0, 0, 0};
				}
#pragma unroll
				for (int u = 0; u < kQ; ++u) {
					if (rem[u] >= 16) {
						*reinterpret_cast<u32x4_u*>(da[u]) = v[u];
					} else if (rem[u]) {   // the command's last, partial chunk
						copy_tail(da[u], sa[u], rem[u]);
					}
				}
			}
		}
		block_sync_global();   // the group's stores land before the next group reads or writes
	}
}

// The decode kernel's CRC segments: 16 KiB segments as rows of 64 x 8 bytes
// (dg_crc.h).  The byte tables go to LDS at tb (256-byte aligned, inside the
// dead doubling arrays), then the nibble table of x^(8 * 64 KiB) (the Horner
// step of a wave's segments) at TK.
#ifndef DG_DEC_CRC5   // A/B: the decode's CRC folds by five-bit tables (13 conflict-free lookups per piece)
#define DG_DEC_CRC5 0
#endif
constexpr int kDecTab = DG_DEC_CRC5 ? kCrcFive : kCrcByte;
constexpr uint32_t kDecTabWords = kDecTab == kCrcFive ? 32 * kCrc5Tabs8 : 8 * 256;
struct DecCrc {
	uint32_t tb;
	const uint64_t* TK;
	uint64_t klane;
};
__device__ __forceinline__ DecCrc dec_crc_tables(uint16_t* NX, const DecodeArgs& a) {
	const uint32_t tid = threadIdx.x;
	const uint32_t base = lds_addr(NX), tb = (base + 255u) & ~255u;
	uint64_t* T = reinterpret_cast<uint64_t*>(NX) + (tb - base) / 8;
	const uint64_t* src = a.tables + (kDecTab == kCrcFive ? kCrc5R8 : kCrcRows8);
	for (uint32_t k = tid; k < kDecTabWords; k += kDecBlock) T[k] = src[k];
	uint64_t* TK = T + kDecTabWords;
	const uint64_t* KF = a.tables + 8 * 256 + kCrcLevels * kCrcNibTabWords;
	for (uint32_t k = tid; k < kCrcNibTabWords; k += kDecBlock) TK[k] = KF[k];   // x^(8 * 64 KiB)
	static_assert(8 * (8 * 256 + kCrcNibTabWords) + 256 <= 3 * kDecWin * 2, "CRC tables fit NX");
	return DecCrc{tb, TK, a.tables[kCrcRowK8 + lane_id()]};
}
template <bool kCopy = false>
__device__ __forceinline__ uint64_t dec_seg_crc(const DecCrc& t, uintptr_t start, uint64_t len, uint32_t nseg,
                                                uint32_t j, intptr_t copy_delta = 0, uintptr_t copy_hi = 0) {
	return crc_seg_rows<8, 1, 8, kDecCrcSeg, kCopy, kDecTab>(start, len, nseg, j, t.tb, t.tb, t.klane, copy_delta, copy_hi);
}

__global__ __launch_bounds__(kDecBlock) __attribute__((amdgpu_waves_per_eu(4, 8))) void decode_kernel(DecodeArgs a) {
	const uint32_t i = blockIdx.x;
	if (i >= a.n) return;
	const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
	__shared__ __attribute__((aligned(16))) uint8_t win[kDecWin + 32];
	__shared__ __attribute__((aligned(16))) uint16_t N1[kDecWin];
	// N2, N4, N8 during the parse; the waves' flat-copy scratch afterwards
	__shared__ __attribute__((aligned(16))) uint16_t NX[3 * kDecWin];
	__shared__ uint16_t cmds[kDecMaxCmds];
	__shared__ uint16_t jumps[kDecMaxCmds / 16 + 2];   // 16-command jumps, then the one 8-command jump
	__shared__ uint32_t sh[8];   // walk results and window flags
	__shared__ uint32_t bsum[2 * (kDecMaxCmds / 64 + 1)];   // per batch: first written dst, max end
	__shared__ uint64_t cpart[2][kDecWaves];   // crc_check: per span, each wave's Horner partial
	__shared__ uint32_t clast[2][kDecWaves];   // and its last segment
	uint16_t* N2 = NX;
	uint16_t* N4 = NX + kDecWin;
	uint16_t* N8 = NX + 2 * kDecWin;
	uint16_t* N16 = N4;   // (N4 is dead once N8 is built)
	constexpr uint32_t kScratch = 64 * 4 + 128 * 4 + 64 * 8 + 64 * 8 + 64 * 4;
	static_assert(kDecWaves * kScratch <= 3 * kDecWin * 2, "scratch fits NX");
	DecScratch xs;
	{
		uint8_t* base = reinterpret_cast<uint8_t*>(NX) + wave * kScratch;
		xs.sp = reinterpret_cast<const uint8_t**>(base);
		xs.dp = reinterpret_cast<uint8_t**>(base + 64 * 8);
		xs.cum = reinterpret_cast<uint32_t*>(base + 128 * 8);
		xs.row = reinterpret_cast<uint32_t*>(base + 128 * 8 + 64 * 4);
		xs.len = reinterpret_cast<uint32_t*>(base + 128 * 8 + 64 * 4 + 128 * 4);
	}
	// the grouped apply's arrays, after the four waves' flat-copy scratch
	DecGroupLds grp;
	{
		uint8_t* base = reinterpret_cast<uint8_t*>(NX) + kDecWaves * kScratch;
		grp.src = reinterpret_cast<uint32_t*>(base);
		grp.dst = grp.src + kDecMaxCmds;
		grp.len = grp.dst + kDecMaxCmds;
		grp.pre = grp.len + kDecMaxCmds;                     // kDecMaxCmds + 1 (+3 pad)
		grp.red = grp.pre + kDecMaxCmds + 4;                 // 8
		grp.last = reinterpret_cast<int16_t*>(grp.red + 8);  // kDecMaxCmds
		grp.gs = reinterpret_cast<uint16_t*>(grp.last + kDecMaxCmds);   // kDecMaxCmds + 1 (+1 pad)
		grp.flag = reinterpret_cast<uint8_t*>(grp.gs + kDecMaxCmds + 2);
		static_assert(kDecWaves * kScratch + 4 * (4 * kDecMaxCmds + 4 + 8) + 2 * (2 * kDecMaxCmds + 2) + kDecMaxCmds <=
		                  3 * kDecWin * 2,
		              "grouped-apply arrays fit NX");
	}

#ifdef DG_ONEPASS_PROF
	uint64_t dprof[kDecProfN] = {};
	const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
	const dg_decode_desc_dev dd = a.descs[i];
	const uint8_t* D = a.delta + dd.delta_off;
	const uint64_t dl = dd.delta_len;
	const uint8_t* R = a.ref + dd.ref_off;
	const uint64_t rl = dd.ref_len;
	uint8_t* O = a.out + dd.out_off;

	int32_t st = 0;
	uint64_t vsize = 0;
	if (dl < 25 || D[0] != 'D' || D[1] != 'L' || D[2] != 'T' || D[3] != 3) st = 8;
	bool inplace = false;
	if (!st) {
		inplace = D[4] & 1;
		vsize = be32(D + 5);
	}
	const uint64_t bsz = inplace ? max(rl, vsize) : vsize;
	if (!st && bsz > dd.out_cap) st = 7;
	if (st) {
		if (tid == 0) {
			a.status[i] = st;
			a.out_len[i] = 0;
			}
		return;
	}
	// initial image: R then zeros (in-place, apply.c:276-278) or zeros (apply.c:233)
	const uint64_t init = inplace ? (rl < bsz ? rl : bsz) : 0;
	// R's CRC-64/XZ from the loads that make the in-place image (R is read
	// once): 16 KiB segments as rows of 64 x 8 bytes, segment j on wave j % 4,
	// each wave folding its segments Horner-wise; the image's whole 16-byte
	// words are stored from the same pieces
	const bool aligned_or = (((uintptr_t)O | (uintptr_t)R) & 15) == 0;
	const bool rcrc_early = a.crc_check && aligned_or && rl >= 8;
	uint64_t racc = 0;
	uint32_t rlast = ~0u;
	DPROF_T(tf0);
	if (rcrc_early) {
		const DecCrc ct = dec_crc_tables(NX, a);
		__syncthreads();
		const uint32_t nseg = crc_nseg((uintptr_t)R, rl, kDecCrcSeg);
		const uintptr_t copy_hi = (uintptr_t)R + init / 16 * 16;
		for (uint32_t j = wave; j < nseg; j += kDecWaves) {
			const uint64_t c = dec_seg_crc<true>(ct, (uintptr_t)R, rl, nseg, j, (intptr_t)O - (intptr_t)R, copy_hi);
			racc = (rlast != ~0u ? mul_nib(racc, ct.TK) : 0ull) ^ c;
			rlast = j;
		}
		__syncthreads();   // the tables' LDS is the parse's next
	}
	{
		uint64_t k0 = 0;
		if (aligned_or) {   // 16 B per thread, 4 in flight
			const uint64_t n16 = init / 16;
			const uint64_t ncopy = rcrc_early ? 0 : n16;   // (else made with R's CRC above)
			for (uint64_t b = 0; b < ncopy; b += 4 * kDecBlock) {
				typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
				u32x4 x[4];
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					const uint64_t q = b + kDecBlock * u + tid;
					x[u] = q < n16 ? reinterpret_cast<const u32x4*>(R)[q] : u32x4{0, 0, 0, 0};
				}
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					const uint64_t q = b + kDecBlock * u + tid;
					if (q < n16) reinterpret_cast<u32x4*>(O)[q] = x[u];
				}
			}
			const uint64_t z0 = (init + 15) / 16, z1 = bsz / 16;   // whole zero words [z0, z1)
			for (uint64_t q = z0 + tid; q < z1; q += kDecBlock) reinterpret_cast<uint4*>(O)[q] = make_uint4(0, 0, 0, 0);
			for (uint64_t k = n16 * 16 + tid; k < z0 * 16 && k < bsz; k += kDecBlock) O[k] = k < init ? R[k] : 0;
			k0 = (z1 > z0 ? z1 : z0) * 16;
		}
		for (uint64_t k = k0 + tid; k < bsz; k += kDecBlock) O[k] = k < init ? R[k] : 0;
	}
	block_sync_global();   // every wave's image stores complete before any command load or store
	DPROF_ADD(DP_FILL, tf0);

	uint64_t pos = 25;   // stream offset of the current window: a command boundary
	bool done = false;
	while (!done && !st) {
		if (pos >= dl) break;   // missing END: end of input (as the reference's loop)
		const uint32_t avail = (uint32_t)min((uint64_t)kDecWin, dl - pos);
		// ── 1. window -> LDS: aligned 16-byte blocks that hold stream bytes
		//    (a block never crosses a page), win[sh + x] = D[pos + x]
		const uintptr_t wa = (uintptr_t)(D + pos) & ~(uintptr_t)15;
		const uint32_t shf = (uint32_t)((uintptr_t)(D + pos) - wa);
		const uintptr_t dend = (uintptr_t)(D + dl);
		DPROF_INC(DP_WINDOWS);
		DPROF_T(tl0);
		for (uint32_t q = tid; q < (kDecWin + 32) / 16; q += kDecBlock) {
			const uintptr_t ad = wa + 16 * q;
			uint4 x = make_uint4(0, 0, 0, 0);
			if (ad < dend) x = *reinterpret_cast<const uint4*>(ad);
			reinterpret_cast<uint4*>(win)[q] = x;
		}
		__syncthreads();
		const uint8_t* w = win + shf;
		DPROF_ADD(DP_LOAD, tl0);
		DPROF_T(tn0);
		// ── 2. N1: next command offset for a command starting at x.  Thread
		//    tid owns offsets [16 tid, 16 tid + 16): all default to malformed
		//    (two 16-byte stores), and only offsets whose byte is a command
		//    type (0, 1, 2: ~1.3 of 16 in a command stream) are decoded ──
		static_assert(kDecWin == 16 * kDecBlock, "16 window offsets per thread");
		{
			const uint32_t x0 = 16 * tid;
			constexpr uint32_t bb = (uint32_t)kNxBad | ((uint32_t)kNxBad << 16);
			uint4* dst = reinterpret_cast<uint4*>(N1 + x0);
			dst[0] = make_uint4(bb, bb, bb, bb);
			dst[1] = make_uint4(bb, bb, bb, bb);
			uint32_t d[4];
			win16(w + x0, d);
			uint32_t cand = 0;
#pragma unroll
			for (uint32_t k = 0; k < 16; ++k) cand |= (((d[k >> 2] >> (8 * (k & 3))) & 0xFFu) <= 2u ? 1u : 0u) << k;
			const uint32_t lim = avail > x0 ? umin32(avail - x0, 16u) : 0u;
			cand &= (1u << lim) - 1u;
			for (; cand; cand &= cand - 1) {
				const uint32_t x = x0 + (uint32_t)__builtin_ctz(cand);
				const uint32_t t = w[x];
				uint32_t nx = kNxEnd;
				if (t != 0) {
					const uint32_t hdr = t == 1 ? 13u : 9u;
					if (x + hdr > avail) {
						nx = pos + x + hdr > dl ? kNxBad : kNxCut;
					} else {
						uint32_t lw = 0;
						__builtin_memcpy(&lw, w + x + 5, 4);
						const uint64_t len = t == 1 ? 0 : __builtin_bswap32(lw);
						const uint64_t end = (uint64_t)x + hdr + len;
						if (pos + end > dl) nx = kNxBad;
						else nx = end >= avail ? kNxFar : (uint32_t)end;
					}
				}
				N1[x] = (uint16_t)nx;
			}
		}
		__syncthreads();
		DPROF_ADD(DP_N1, tn0);
		DPROF_T(td0);
		// ── 3. pointer doubling ──
		// (16 offsets per thread: two 16-byte reads, 16 independent gathers,
		// two 16-byte stores)
		auto dbl = [&](const uint16_t* src, uint16_t* dstN) {
			const uint32_t x0 = 16 * tid;
			const uint4* sp = reinterpret_cast<const uint4*>(src + x0);
			const uint4 a = sp[0], b = sp[1];
			const uint32_t in[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
			uint32_t o[8];
#pragma unroll
			for (uint32_t k = 0; k < 8; ++k) {
				const uint32_t y0 = in[k] & 0xFFFFu, y1 = in[k] >> 16;
				const uint32_t z0 = y0 >= kNxSpecial ? y0 : src[y0];
				const uint32_t z1 = y1 >= kNxSpecial ? y1 : src[y1];
				o[k] = z0 | (z1 << 16);
			}
			uint4* dp = reinterpret_cast<uint4*>(dstN + x0);
			dp[0] = make_uint4(o[0], o[1], o[2], o[3]);
			dp[1] = make_uint4(o[4], o[5], o[6], o[7]);
		};
		dbl(N1, N2);
		__syncthreads();
		dbl(N2, N4);
		__syncthreads();
		dbl(N4, N8);
		__syncthreads();
		dbl(N8, N16);
		__syncthreads();
		DPROF_ADD(DP_DBL, td0);
		DPROF_T(tw0);
		// ── 4. the walk (wave 0, uniform): 16 commands per N16 step, at most
		//    one N8 step, then single steps ──
		if (wave == 0) {
			uint32_t x = 0, nj = 0, n8 = 0;
			uint32_t term = 0;
			while (true) {
				const uint32_t y = uni(N16[x]);
				if (y >= kNxSpecial || 16 * (nj + 1) > kDecMaxCmds) break;
				if (lane == 0) jumps[nj] = (uint16_t)x;
				++nj;
				x = y;
			}
			uint32_t cnt = 16 * nj;
			{
				const uint32_t y = uni(N8[x]);
				if (y < kNxSpecial && cnt + 8 <= kDecMaxCmds) {
					if (lane == 0) jumps[nj] = (uint16_t)x;
					n8 = 1;
					cnt += 8;
					x = y;
				}
			}
			while (true) {   // single steps from x (at most 7 commands + the terminal)
				const uint32_t y = uni(N1[x]);
				if (y == kNxEnd || y == kNxBad || y == kNxCut) { term = y; break; }
				if (cnt >= kDecMaxCmds) { term = kNxCut; break; }   // restart the window at x
				if (lane == 0) cmds[cnt] = (uint16_t)x;
				++cnt;
				if (y == kNxFar) { term = kNxFar; break; }
				x = y;
			}
			if (lane == 0) {
				sh[0] = cnt;
				sh[1] = nj;
				sh[2] = x;
				sh[3] = term;
				sh[4] = 0;   // a batch out of bounds
				sh[5] = 0;   // the window is not order-free
				sh[6] = n8;
			}
		}
		__syncthreads();
		const uint32_t cnt = sh[0], nj = sh[1], x = sh[2], term = sh[3], n8 = sh[6];
		DPROF_ADD(DP_WALK, tw0);
		DPROF_T(te0);
		// expand the jumps: 8 nodes from each base (e, N1 e, N2 e, ..., N1 N2 N2 N2 e);
		// a 16-command jump has bases e and N8 e
		for (uint32_t k = tid; k < 2 * nj + n8; k += kDecBlock) {
			const uint32_t j = k >> 1;
			const uint32_t e0 = j < nj ? ((k & 1) ? N8[jumps[j]] : jumps[j]) : jumps[nj];
			const uint32_t e2 = N2[e0];
			const uint32_t e4 = N2[e2];
			const uint32_t e6 = N2[e4];
			uint16_t* c = cmds + (j < nj ? 16 * j + 8 * (k & 1) : 16 * nj);
			c[0] = (uint16_t)e0;
			c[1] = N1[e0];
			c[2] = (uint16_t)e2;
			c[3] = N1[e2];
			c[4] = (uint16_t)e4;
			c[5] = N1[e4];
			c[6] = (uint16_t)e6;
			c[7] = N1[e6];
		}
		__syncthreads();   // cmds complete; N2..N8 dead: NX becomes the copy scratch
		DPROF_ADD(DP_EXP, te0);		// the walk's terminal: x is where it stopped
		uint64_t next_pos = pos + x;   // kNxCut: restart at x
		if (term == kNxEnd) done = true;
		else if (term == kNxBad) st = 8;
		else if (term == kNxFar) {
			const uint32_t t = w[x];
			next_pos = pos + x + (t == 1 ? 13u : 9u + be32(w + x + 5));
		}

		// ── 5. bounds and order checks of every batch (waves in parallel) ──
		DPROF_T(th0);
		const uint32_t nb = (cnt + 63) / 64;
		for (uint32_t b = wave; b < nb; b += kDecWaves) {
			const DecCmd c = dec_cmd(w, cmds, 64 * b, cnt, pos);
			bool bad = false;
			if (c.mine) {
				if (c.dst + c.len > bsz) bad = true;
				if (c.kind == 1 && c.src + c.len > (inplace ? bsz : rl)) bad = true;
			}
			// order-free: the commands that write (an in-place COPY with src ==
			// dst writes nothing: apply.c:257-266 memmoves a range onto itself,
			// and the in-place format puts the ADDs after the COPYs,
			// inplace.c:711-725) have increasing, disjoint destinations (< 2^32:
			// bsz checked), and no in-place COPY moves.  Within the batch by a
			// prefix max of the write ends; across batches by the summaries.
			const bool writes = c.mine && c.len != 0 && !(inplace && c.kind == 1 && c.src == c.dst);
			const uint32_t end32 = writes ? (uint32_t)(c.dst + c.len) : 0u, dst32 = (uint32_t)c.dst;
			const uint32_t incl_end = wave_incl_max(end32);
			const bool unordered = writes && dst32 < wave_shr1z(incl_end);
			const bool moves = c.mine && inplace && c.kind == 1 && c.src != c.dst;
			const uint64_t wm = __ballot(writes);
			const uint32_t first_dst = wm ? rdlane(dst32, ffs64(wm)) : ~0u;
			if (lane == 0) {
				bsum[2 * b] = first_dst;
				bsum[2 * b + 1] = rdlane(incl_end, 63);
			}
			if (__ballot(bad) && lane == 0) atomicOr(&sh[4], 1u);
			if (__ballot(unordered || moves) && lane == 0) atomicOr(&sh[5], 1u);
		}
		__syncthreads();
		if (sh[4]) st = 8;
		bool cross = false;   // a batch writes below the end of an earlier batch's writes
		for (uint32_t b = 0, run = 0; b < nb; ++b) {
			const uint32_t f = bsum[2 * b], e = bsum[2 * b + 1];
			if (f != ~0u) {
				cross = cross || f < run;
				run = umax32(run, e);
			}
		}
		const bool free_win = !sh[5] && !cross;
		if (!free_win) DPROF_INC(DP_ORDERED);
		DPROF_ADD(DP_HDR, th0);
		DPROF_T(tc0);
		// ── 6. apply ──
#ifdef DG_AB_SWITCHES
		if (!st && !(a.dbg & 0x100)) {   // 0x100: skip the apply (A/B builds only, never the product)
#else
		if (!st) {
#endif
			if (free_win) {
				for (uint32_t b = wave; b < nb; b += kDecWaves) {
					DPROF_INC(DP_BATCHES);
					DPROF_T(tq0);
					const DecCmd c = dec_cmd(w, cmds, 64 * b, cnt, pos);
#ifdef DG_ONEPASS_PROF
					asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
					DPROF_ADD(DP_C_CMD, tq0);
					DPROF_T(tq1);
					dec_flat_batch(c, inplace, O, R, D, xs);
					DPROF_ADD(DP_C_FLAT, tq1);
				}
			} else {
#ifdef DG_AB_SWITCHES
				if (a.dbg & 0x200) {   // A/B (DG_DEBUG_BITS=0x200): the round-2 one-wave replay
					if (wave == 0)
						for (uint32_t b = 0; b < nb; ++b) {
							const DecCmd c = dec_cmd(w, cmds, 64 * b, cnt, pos);
							dec_ordered_batch(c, cnt - 64 * b < 64 ? cnt - 64 * b : 64, inplace, O, R, D, xs);
						}
				} else
#endif
				dec_grouped_window(w, cmds, cnt, pos, inplace, O, R, D, grp);
			}
		}
		DPROF_T(tq2);
		block_sync_global();   // the window's stores complete before the next window
		DPROF_ADD(DP_C_BAR, tq2);
		DPROF_ADD(DP_COPY, tc0);
		pos = next_pos;
	}
	// ── 7. CRC-64/XZ of R and of the output, checked against the header
	//    (main.c:341-356 before the apply, :376-385 after; a source mismatch
	//    takes precedence, the output is then unspecified).  Segments of
	//    16 KiB (256-byte lanes: a quarter of the encode CRC's serial chain
	//    per lane, every wave busy on a 64 KiB stream); segment j of a span
	//    goes to wave j % 4, which folds its segments Horner-wise by
	//    x^(8 * 64 KiB); thread 0 shifts the partials into place. ──
	int32_t cst = 0;
	if (a.crc_check && !st) {
		DPROF_T(tk0);
		block_sync_global();   // every wave's output stores before any CRC read
		DPROF_ADD(DP_CRC_SYNC, tk0);
		DPROF_T(tk1);
		const uint64_t* Lv = a.tables + 8 * 256;
		const uint64_t* KF = Lv + kCrcLevels * kCrcNibTabWords;   // x^(8 seg), x^(-8t), x^(8 seg k) k = 2..4
		// LDS (the dead doubling arrays): the row tables and x^(8 * 64 KiB);
		// 16 KiB segments read as rows of 64 x 8 bytes (coalesced)
		const DecCrc ct = dec_crc_tables(NX, a);
		const uint64_t* TK = ct.TK;
		__syncthreads();
		const uintptr_t sa[2] = {(uintptr_t)R, (uintptr_t)O};
		const uint64_t sl[2] = {rl, vsize};
#pragma unroll
		for (int sp = 0; sp < 2; ++sp) {
			uint64_t acc = 0;
			uint32_t last = ~0u;
			if (sp == 0 && rcrc_early) {   // R's, from the fill
				acc = racc;
				last = rlast;
			} else if (sl[sp] >= 8) {
				const uint32_t nseg = crc_nseg(sa[sp], sl[sp], kDecCrcSeg);
				for (uint32_t j = wave; j < nseg; j += kDecWaves) {
					const uint64_t c = dec_seg_crc(ct, sa[sp], sl[sp], nseg, j);
					acc = (last != ~0u ? mul_nib(acc, TK) : 0ull) ^ c;   // TK: x^(8 * 64 KiB) = 4 segments
					last = j;
				}
			}
			if (lane == 0) {
				cpart[sp][wave] = acc;
				clast[sp][wave] = last;
			}
		}
		__syncthreads();
		DPROF_ADD(DP_CRC_SEG, tk1);
		DPROF_T(tk2);
		// Wave 0 combines, one lane per (span, wave) partial: the shifts
		// x^(8 * 16 KiB * k) run side by side (one gather round, not eight in
		// a row on thread 0), then the two spans' pad fixes side by side.
		if (wave == 0) {
			const uint32_t sp = lane / kDecWaves, w2 = lane % kDecWaves;
			uint64_t v = 0;
			if (lane < 2 * kDecWaves && sl[sp] >= 8 && clast[sp][w2] != ~0u) {
				const uint32_t k = crc_nseg(sa[sp], sl[sp], kDecCrcSeg) - 1 - clast[sp][w2];   // 0..3 segments after its last
				v = cpart[sp][w2];
				if (k)
					v = mul_nib(v, k == 1 ? Lv + 4 * kCrcNibTabWords      // x^(8 * 16 KiB)
					               : k == 2 ? Lv + 5 * kCrcNibTabWords    // x^(8 * 32 KiB)
					                        : KF + kCrcFinX48K * kCrcNibTabWords);
			}
			const uint64_t raw0 = wave_xor64(lane < kDecWaves ? v : 0ull);
			const uint64_t raw1 = wave_xor64(lane >= kDecWaves && lane < 2 * kDecWaves ? v : 0ull);
			bool bad = false;
			if (lane < 2) {   // lane s: span s (0 = R, 1 = output)
				const uintptr_t s0 = lane ? sa[1] : sa[0];
				const uint64_t len = lane ? sl[1] : sl[0];
				uint64_t c;
				if (len < 8) {
					const uint8_t* d = reinterpret_cast<const uint8_t*>(s0);
					c = ~0ULL;
					for (uint64_t k = 0; k < len; ++k) c = a.tables[(uint8_t)(c ^ d[k])] ^ (c >> 8);
				} else {
					c = lane ? raw1 : raw0;
					const uintptr_t end = s0 + len;
					const uint32_t t = (uint32_t)(((end + 15) & ~(uintptr_t)15) - end);
					if (t) c = mul_nib(c, KF + (1 + t) * kCrcNibTabWords);   // undo the trailing pad
				}
				uint64_t h = 0;
				for (int k = 0; k < 8; ++k) h = (h << 8) | D[9 + 8 * lane + k];
				bad = h != ~c;
			}
			const uint64_t bm = __ballot(bad);
			cst = bm & 1 ? 9 : (bm & 2 ? 10 : 0);
		}
		DPROF_ADD(DP_CRC_TAIL, tk2);
	}
	if (tid == 0) {
		a.status[i] = st ? st : cst;
		a.out_len[i] = st ? 0 : vsize;
	}
#ifdef DG_ONEPASS_PROF
	{
		DPROF_T(tw9);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		DPROF_ADD(DP_WAIT, tw9);
		dprof[DP_TOTAL] = __builtin_amdgcn_s_memtime() - t_start;
		if (tid == 0)
			for (int k = 0; k < kDecProfN; ++k) atomicAdd(&g_decode_prof[k], (unsigned long long)dprof[k]);
	}
#endif
}

hipError_t launch_decode(const DecodeArgs& a, hipStream_t st) {
	if (a.n) hipLaunchKernelGGL(decode_kernel, dim3(a.n), dim3(kDecBlock), 0, st, a);
	return hipGetLastError();
}




}  // namespace dg
