// dg_device.h — device-side data layout shared by the kernels and the host
// plan code.  All structs are plain data (no pointers into host memory).
#pragma once
#include <stdint.h>

typedef struct dg_context dg_context_t;
typedef struct dg_encode_plan dg_encode_plan_t;

namespace dg {

constexpr uint64_t kMersenne = (1ULL << 61) - 1;   // src/c/delta.h:25
constexpr uint64_t kBase = 263;                    // src/c/delta.h:24
constexpr uint64_t kCrcPoly = 0xC96C5795D7870F42ULL;  // reflected, delta.h:303
constexpr uint32_t kSentinel = 0xFFFFFFFFu;        // "no slot" (q < 2^32 - 1)

// CRC segmentation: one wave64 per 64 KiB segment (dg_crc.h).  Segments tile
// a span from its (16-byte aligned-up) end backwards.
constexpr uint32_t kCrcSegBytes = 65536;
constexpr uint32_t kCrcWavesPerBlock = 4;

// Onepass register history: chunks of 64 steps kept in VGPRs before the
// epoch spills into the global table tier.  Round 3 A/B (same box, plain
// chain 90/94/96 VGPRs, no scratch, 5 waves/SIMD for 5/6/7): c3s 54 / 76 /
// 105 / 105 GiB/s at 4/5/6/7 chunks, C2 and C3 unchanged; 8 spills.
#ifndef DG_HIST_CHUNKS   // tuning knob (make variant)
#define DG_HIST_CHUNKS 6
#endif
constexpr int kHistChunks = DG_HIST_CHUNKS;

struct PairDev {          // == dg_pair_t
	uint64_t r_off, r_len, v_off, v_len;
};

struct PairPlanDev {
	uint64_t q;            // table size for this pair (onepass.c:61-62)
	uint64_t q_magic;      // floor((2^64-1)/q), Barrett
	uint64_t rec_base;     // first record slot
	uint32_t rec_cap;      // record capacity (>= #copies possible)
	uint32_t pad;
	// correcting only (correcting.c:116-136)
	uint64_t f_size, f_magic;  // |F| and floor((2^64-1)/|F|)
	uint64_t m, m_magic;       // checkpoint modulus and Barrett
	uint64_t tab_base;         // first entry of this pair's R index (correcting)
	// onepass member mode (dg_members.hip)
	uint64_t mem_base;         // first member slot (n_chunks x kMemChunkSlots slots)
	uint32_t chunk_base;       // first chunk (index into the per-chunk member counts)
	uint32_t n_chunks;         // chunks of kMemChunk positions covering [0, min(|R|,|V|)]
	// correcting, CRC of R in the build: x^(-8 pad), pad = |R| rounded up to
	// 32 KiB minus |R| (the build's zero padding)
	uint64_t crc_unpad;
};

struct CrcSegDev {        // one wave's CRC segment
	uint32_t span;         // span index
	uint32_t j;            // segment index within the span (0 = first)
};

struct CrcSpanDev {
	uint64_t off, len;     // byte range in the arena
	uint32_t seg_base;     // first segment index
	uint32_t nseg;         // number of segments (0 for len < 8)
	uint32_t which;        // arena selector: 0 = reference arena, 1 = version arena
	uint32_t out;          // index of its CRC in CrcArgs::out
};

// Precomputed GF(2) constants for the CRC combine steps, as nibble tables:
// tab[c][16*j + n] = (n << 4j) * K_c mod P  (reflected), see dg_host.cpp.
// Level l = x^(8 * 1024 * 2^l): 16 and 32 KiB are the decode kernel's segment
// combines, 32 KiB the correcting build's piece stride.
constexpr int kCrcLevels = 6;
constexpr int kCrcNibTabWords = 256;   // 16 nibbles x 16 values
// after the level tables (F): x^(8 kCrcSegBytes), x^(-8t) for t = 0..15,
// x^(8 kCrcSegBytes k) for k = 2..4, then for the decode kernel's 256-byte
// lanes x^(8 * 256), x^(8 * 512) (its first two tree levels) and x^(8 * 48 KiB)
constexpr int kCrcFinTabs = 1 + 16 + 3 + 3;
constexpr int kCrcFinX256 = 20, kCrcFinX512 = 21, kCrcFinX48K = 22;   // indices in F
// after F: the row-interleaved segment tables (dg_crc.h crc_seg_rows): for
// 16- and 8-byte pieces, U_j = T advanced by (64 PB - 1 - j) bytes (16 and 8
// tables of 256), then the per-lane constants x^(-8 PB l), l = 0..63, for PB
// = 16, 8; then the five-bit row tables F_k[v] = Z^n(v << 5k), k = 0..12, 32
// entries (256 B: one LDS row, so a 32-lane ds_read_b64 group never
// conflicts) -- for 8-byte pieces n = 512; for 16-byte pieces n = 1024 on
// (A ^ low 8 bytes), then 13 more with n = 1016 on the high 8 bytes
constexpr uint32_t kCrcRowsOff = 8 * 256 + (kCrcLevels + kCrcFinTabs) * kCrcNibTabWords;
constexpr uint32_t kCrcRows16 = kCrcRowsOff, kCrcRows8 = kCrcRowsOff + 16 * 256;
constexpr uint32_t kCrcRowK16 = kCrcRowsOff + 24 * 256, kCrcRowK8 = kCrcRowK16 + 64;
constexpr uint32_t kCrc5Tabs8 = 13, kCrc5Tabs16 = 26;
constexpr uint32_t kCrc5R8 = kCrcRowK8 + 64, kCrc5R16 = kCrc5R8 + 32 * kCrc5Tabs8;
constexpr uint32_t kCrcTabWords = kCrc5R16 + 32 * kCrc5Tabs16;

struct EncodeArgs {
	const uint8_t* ref;
	const uint8_t* ver;
	const PairDev* pairs;
	const PairPlanDev* pplan;
	uint32_t n_pairs;          // pairs [pair0, n_pairs) of the batch in this launch
	uint32_t pair0;
	uint32_t p;
	const uint64_t* powc;      // p constants: 263^(p-1-k) mod (2^61-1)
	uint32_t* rec;             // 3 x u32 per COPY record (v, r, len)
	uint32_t* n_rec;           // per pair
	uint64_t* dsize;           // per pair serialized delta size
	int32_t* status;           // per pair
	// Tier-C table pool (long epochs)
	unsigned long long* tables;   // n_tables x 2 x qmax entries
	uint64_t qmax;
	uint32_t n_tables;
	uint32_t* table_locks;
	uint32_t* table_tags;
	// fused serialisation (onepass16_kernel): packed output, offsets and the
	// per-pair look-back words; lookback == nullptr selects scan + serialise
	uint8_t* out;
	uint64_t out_cap;
	uint64_t* offsets;
	unsigned long long* lookback;
	// correcting
	uint32_t buf_cap;          // lookback buffer entries (correcting.c:14-62)
	uint32_t* ctab;            // R index: per pair q x u32 offsets (~0 = empty)
	uint32_t max_seeds;        // max over pairs of |R| - p + 1
	uint64_t* kcls;            // per pair: checkpoint class k (correcting.c:131-136), computed once
	const uint32_t* gpairs;    // the pairs whose R index is built in memory (q > the LDS capacity)
	uint32_t n_gpairs;
	uint32_t dbg;              // A/B switches (DG_DEBUG_BITS, A/B builds only), 0 in the product
	// member mode (onepass16_kernel after the member kernels, dg_members.hip):
	// verified diagonal members are taken as they are; nullptr = plain chain
	const uint32_t* mem_s;     // per member slot (PairPlanDev::mem_base + chunk slots): epoch start
	const uint32_t* n_mem;     // per chunk (PairPlanDev::chunk_base + c): members starting in it
	const uint32_t* srec;      // per member slot: (x, COPY length, ADD head, verified)
	const uint32_t* csum;      // per chunk: verified prefix length, its delta bytes
	// the delta's pieces for member_serialize_kernel: per chunk (chunk_base +
	// c) the members taken in bulk (count, byte offset in the delta; zeroed by
	// the member kernel), and per pair (n_chunks + 2 entries from chunk_base +
	// 2 pair) the runs of records the chain wrote itself, then the trailing
	// ADD + END: uint4 (first record or kSegTail, count, byte offset, ADD start)
	uint32_t* cmap;
	uint32_t* seg;
	uint32_t* nseg;            // per pair: segments written
	// automatic member mode: pairs averaging fewer verified members per chunk
	// than this run the plain chain (its records as one segment); 0 = never
	uint32_t route_min;
	// ... and the pairs so routed, counted by the routed chain (scan_sizes_kernel
	// hands the count to the host and zeroes it; nullptr = not counted)
	uint32_t* route_cnt;
	// --verbose diagnostics (correcting; nullptr = off): per pair 8 u64 —
	// build seeds passing the checkpoint, slots stored, scan checkpoints, fp
	// mismatches, byte mismatches, matches, k, passing seeds whose slot is in
	// the table (correcting.c:95-98, 137-214, 470-485)
	uint64_t* stats;
	// correcting with every R index in LDS: R's CRC-64/XZ computed by the
	// build (nullptr = a separate CRC pass): out[2 pair] = CRC of R
	uint64_t* crc_out;
	const uint64_t* crc_tab;   // the context's CRC tables (CrcArgs::tables)
	const uint64_t* crc_k32;   // x^(8 * 32 * t), t = 0..1023
};

constexpr uint32_t kSegTail = 0xFFFFFFFFu;

// Speculative diagonal members of the onepass chain (dg_members.hip): one
// wave per chunk of kMemChunk positions, with kMemAhead bytes of look-ahead
// staged for the members that end past the chunk.  Members start >= p = 16
// bytes apart, so a chunk holds at most kMemChunk / 16 of them.
constexpr uint32_t kMemChunk = 2048;
constexpr uint32_t kMemAhead = 240;    // staged: [chunk - 16, chunk + 2048 + 240) = 2304 B
constexpr uint32_t kMemChunkSlots = kMemChunk / 16 + 1;
struct SpecArgs {
	const uint8_t* ref;
	const uint8_t* ver;
	const PairDev* pairs;
	const PairPlanDev* pplan;
	const uint2* chunks;       // per wave: (pair, chunk)
	uint32_t job0;             // wave w of the launch takes job job0 + w
	uint32_t* mem_s;           // per member slot: epoch start s_k
	uint32_t* n_mem;           // per chunk: members starting in it
	uint32_t* srec;            // per member slot: (x, COPY length, ADD head, verified)
	uint32_t* csum;            // per chunk: verified prefix length, its delta bytes
	uint32_t* cmap;            // per chunk: bulk (count, byte offset), zeroed here
};

// member-mode serialisation (dg_members.hip): one wave per (pair, chunk) job
// writes the pair's segments 2c, 2c + 1 (the last chunk's wave the rest)
struct MemSerArgs {
	const uint8_t* ver;
	const PairDev* pairs;
	const PairPlanDev* pplan;
	const uint2* chunks;
	uint32_t job0;             // the launch's jobs: [job0, job0 + n_jobs)
	const uint32_t* cmap;
	const uint32_t* seg;
	const uint32_t* nseg;
	const uint32_t* mem_s;
	const uint32_t* srec;
	const uint32_t* rec;       // kRecWordsOnepass words per record
	const uint64_t* offsets;   // n + 1
	uint8_t* out;
	uint64_t out_cap;
	int32_t* status;
	// sum |V| of the batch: a sparse batch (the scan's total delta bytes,
	// offsets[n_pairs], under half of it) runs the serialiser's whole grid
	uint64_t v_total;
	uint32_t n_pairs;
};

// COPY records: (v, r, len) u32 words, and for onepass a 4th word holding the
// first 4 bytes of V from the gap start (the end of the previous COPY), so a
// gap of <= 4 bytes serialises without reading V (at C2 nearly every ADD).
constexpr uint32_t kRecWordsOnepass = 4;
constexpr uint32_t kRecWordsCorrecting = 3;

struct SerArgs {
	const uint8_t* ver;
	const PairDev* pairs;
	const PairPlanDev* pplan;
	const uint32_t* rec;
	uint32_t rec_words;        // 3 or 4 (kRecWords*)
	const uint32_t* n_rec;
	const uint64_t* crc;       // 2 per pair: R, V
	const uint64_t* offsets;   // n+1
	uint8_t* out;
	uint64_t out_cap;
	int32_t* status;
	uint32_t n_pairs;
	uint32_t crc_in;           // the CRCs are final: write header bytes 9..24 here (no crc_patch_kernel)
};

struct CrcArgs {
	const uint8_t* arena[2];   // selected by CrcSpanDev::which
	const CrcSpanDev* spans;
	const CrcSegDev* segs;
	uint32_t n_segs;
	uint32_t n_spans;
	const uint64_t* tables;    // slice (8x256) + nibble tables: 6 levels, kseg, 16 pad inverses
	uint64_t* seg_crc;
	uint64_t* out;             // per span: CRC-64/XZ value
	const uint64_t* xinv;      // 16 constants x^(-8t) mod P
	uint64_t kseg;             // x^(8*kCrcSegBytes) mod P
	const uint32_t* prio_flag; // member plans: set once the member kernel is done (rows pass to priority 1)
};

struct dg_decode_desc_dev {   // == dg_decode_desc_t
	uint64_t ref_off, ref_len;
	uint64_t delta_off, delta_len;
	uint64_t out_off, out_cap;
};

struct DecodeArgs {
	const uint8_t* ref;
	const uint8_t* delta;
	const dg_decode_desc_dev* descs;
	uint32_t n;
	uint8_t* out;
	uint64_t* out_len;
	int32_t* status;
	uint32_t dbg;              // A/B switches (DG_DEBUG_BITS, A/B builds only), 0 in the product
	const uint64_t* tables;    // CRC tables (CrcArgs::tables); with crc_check
	uint32_t crc_check;        // 1: src/dst CRC-64/XZ computed and checked in-kernel (main.c:341-385)
};

struct SynthSpan {   // synthetic R stream: splitmix64(seed) words at off
	uint64_t off, len, seed;
};
struct SynthCopy {   // V[dst..+len) = R[src..+len)
	uint64_t dst, src, len;
};

// Measurement switches of the A/B builds (make ab / make variant, compiled
// with -DDG_AB_SWITCHES): getenv(name) there, always NULL in the product
// library, which therefore reads no environment variable that changes the
// work it does (dg_host.cpp).
const char* ab_env(const char* name);
// the context's slot for the pipelined host path's state, and its destructor
void** ctx_io(dg_context_t* ctx, void (*release)(void*));
uint64_t ctx_limits_gen(const dg_context_t* ctx);   // changes with every dg_context_set_limit
int ctx_device(const dg_context_t* ctx);            // the context's HIP device
// --verbose: the reference's diagnostic lines for pair i of a plan to stderr,
// from the plan's parameters, its 8 device counters (copied to the host; may
// be NULL for onepass) and the pair's delta (dg_host.cpp)
void print_verbose(const dg_encode_plan_t* P, uint32_t i, const uint64_t* stats, const uint8_t* delta,
                   size_t delta_len);

// launchers (dg_kernels.hip)
// (member plans: routed_after, when set, is waited for between the member
// chain's launch and the routed plain chain's)
hipError_t launch_onepass(const EncodeArgs& a, uint32_t p, bool aligned16, hipStream_t st,
                          hipEvent_t routed_after = nullptr);
bool onepass16_selected();   // false when DG_ONEPASS_GLOBAL=1 forces the HBM-direct kernel
hipError_t launch_members(const SpecArgs& a, uint32_t n_chunks, uint32_t n_cu, hipStream_t st);
hipError_t launch_member_serialize(const MemSerArgs& a, uint32_t n_chunks, uint32_t n_cu, hipStream_t st);
// ev_built, ev_fork (nullable): recorded after the R-index build, before the
// V scan (stage timing; the fork of V's CRC when the build computes R's)
hipError_t launch_correcting_clear(const EncodeArgs& a, hipStream_t st);
hipError_t launch_correcting(const EncodeArgs& a, uint32_t p, hipStream_t st, uint32_t lds_cap, uint64_t qmin,
                             hipEvent_t ev_built, hipEvent_t ev_fork);
// (route_cnt / route_fb: the routed-pair count moved to a host-mapped word)
hipError_t launch_scan(const uint64_t* sz, uint64_t* off, uint32_t n, hipStream_t st,
                       uint32_t* route_cnt = nullptr, uint32_t* route_fb = nullptr);
hipError_t launch_serialize_wave(const SerArgs& s, hipStream_t st);   // wave per pair, CRCs patched after
hipError_t launch_crc_patch(uint8_t* out, const uint64_t* offsets, const uint64_t* crc,
                            const int32_t* status, uint32_t n, hipStream_t st);
// pass: the row-interleaved pass on byte tables (16 KiB LDS per block) or on
// five-bit tables (3.25 KiB: beside the member kernel, which leaves little LDS)
enum : int { kCrcPassRows = 0, kCrcPassRows5 = 1 };
hipError_t launch_crc(const CrcArgs& a, hipStream_t st, uint32_t overlap_cap = 0, int pass = kCrcPassRows,
                      bool finalize = true);
hipError_t launch_crc_finalize(const CrcArgs& a, hipStream_t st);   // the per-span combine alone
// the CRC on 16-byte pieces (32 KiB of tables): for a pass that has the GPU to itself
hipError_t launch_crc_wide(const CrcArgs& a, uint32_t n_cu, hipStream_t st);
hipError_t launch_decode(const DecodeArgs& a, hipStream_t st);
hipError_t launch_synth(uint8_t* ref, uint8_t* ver, uint32_t n_pairs, uint64_t pair_len,
                        uint64_t seed_base, uint64_t n_edits, hipStream_t st);
hipError_t launch_synth_shift(uint8_t* ref, uint8_t* ver, const SynthSpan* spans, const uint64_t* v_off,
                              uint32_t n, uint64_t n_edits, uint32_t pct, hipStream_t st);
hipError_t launch_synth_transpose(uint8_t* ref, uint8_t* ver, const SynthSpan* spans, uint32_t n_spans,
                                  const SynthCopy* cmds, uint32_t n_cmds, hipStream_t st);

}  // namespace dg
