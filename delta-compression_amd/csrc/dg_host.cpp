// dg_host.cpp — host side of libdeltagpu.so: the C ABI of include/delta_gpu.h.
//
// Thin by design: it sizes tables (onepass.c:61-62, correcting.c:116-129),
// lays out device work buffers for a batch, launches the kernels of
// dg_kernels.hip on one HIP stream, and moves host buffers through pinned
// staging for the host-memory entry points.  There is no CPU compute
// fallback: without a GPU every entry point fails with DG_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/delta_gpu.h"
#include "dg_device.h"

using namespace dg;

// ───────────────────────────── small host math ────────────────────────────

namespace {

typedef unsigned __int128 u128;

uint64_t mulmod64(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((u128)a * b % m); }

uint64_t powmod64(uint64_t b, uint64_t e, uint64_t m) {
	uint64_t r = 1 % m;
	b %= m;
	for (; e; e >>= 1) {
		if (e & 1) r = mulmod64(r, b, m);
		b = mulmod64(b, b, m);
	}
	return r;
}

// Deterministic Miller-Rabin; the first 12 prime bases decide every n < 2^64.
// (The reference uses 100 time-seeded random bases, src/c/hash.c:163-178.)
bool is_prime_u64(uint64_t n) {
	static const uint64_t B[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
	if (n < 2) return false;
	for (uint64_t b : B) {
		if (n == b) return true;
		if (n % b == 0) return false;
	}
	uint64_t d = n - 1;
	int s = 0;
	while (!(d & 1)) { d >>= 1; ++s; }
	for (uint64_t b : B) {
		uint64_t x = powmod64(b, d, n);
		if (x == 1 || x == n - 1) continue;
		bool composite = true;
		for (int i = 1; i < s && composite; ++i) {
			x = mulmod64(x, x, n);
			if (x == n - 1) composite = false;
		}
		if (composite) return false;
	}
	return true;
}

// src/c/hash.c:180-190
uint64_t next_prime(uint64_t n) {
	if (n <= 2) return 2;
	uint64_t c = (n % 2 == 0) ? n + 1 : n;
	while (!is_prime_u64(c)) c += 2;
	return c;
}

// ── GF(2)[x] mod P, reflected representation (bit 63 = x^0) ──
uint64_t gf2_mul(uint64_t a, uint64_t b) {
	uint64_t p = 0;
	for (int i = 0; i < 64; ++i) {
		if ((a >> (63 - i)) & 1) p ^= b;
		b = (b & 1) ? (b >> 1) ^ kCrcPoly : (b >> 1);
	}
	return p;
}

uint64_t gf2_xpow(uint64_t n) {   // x^n mod P
	uint64_t r = 1ULL << 63, base = 1ULL << 62;
	for (; n; n >>= 1) {
		if (n & 1) r = gf2_mul(r, base);
		base = gf2_mul(base, base);
	}
	return r;
}

uint64_t gf2_div_x(uint64_t z) {   // z * x^-1 mod P
	const uint64_t l = z >> 63;   // bit 63 of z*... equals the lsb shifted out
	return ((z ^ (l ? kCrcPoly : 0)) << 1) | l;
}

}  // namespace

// ───────────────────────────── context ────────────────────────────────────

struct dg_context {
	int device = -1;
	hipStream_t stream = nullptr;
	uint64_t* d_crc_tables = nullptr;   // slice(8x256) + levels(6x256)
	uint64_t* d_xinv = nullptr;         // 16
	uint64_t* d_k32 = nullptr;          // x^(8 * 32 * t), t = 0..1023 (the correcting build's CRC)
	uint64_t kseg = 0;
	uint32_t n_cu = 256;                // compute units (grid caps)
	uint64_t table_pool_bytes = 0;      // DG_LIMIT_TABLE_POOL_BYTES (0 = automatic)
	uint64_t onepass_members = 0;       // DG_LIMIT_ONEPASS_MEMBERS (0 auto, 1 on, 2 off)
	uint64_t limits_gen = 0;            // bumped by every dg_context_set_limit (cached plans key on it)
	std::string err;
	// scratch reused by the host-buffer entry points
	void* pin = nullptr;
	size_t pin_cap = 0;
	void* io = nullptr;                 // dg_encode_pipelined's slots (dg_host_io.cpp)
	void (*io_free)(void*) = nullptr;
};

uint64_t dg::ctx_limits_gen(const dg_context_t* ctx) { return ctx->limits_gen; }
int dg::ctx_device(const dg_context_t* ctx) { return ctx->device; }

void** dg::ctx_io(dg_context_t* ctx, void (*release)(void*)) {
	ctx->io_free = release;
	return &ctx->io;
}

static int set_err(dg_context_t* ctx, int code, const char* fmt, ...) {
	if (ctx) {
		char buf[512];
		va_list ap;
		va_start(ap, fmt);
		vsnprintf(buf, sizeof buf, fmt, ap);
		va_end(ap);
		ctx->err = buf;
	}
	return code;
}

#define HIPCHK(ctx, expr)                                                                   \
	do {                                                                                    \
		hipError_t e_ = (expr);                                                             \
		if (e_ != hipSuccess)                                                               \
			return set_err((ctx), DG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
	} while (0)

extern "C" {

int dg_abi_version(void) { return DG_ABI_VERSION; }

void dg_diff_options_default(dg_diff_options_t* o) {
	o->p = DG_SEED_LEN;
	o->q = DG_TABLE_SIZE;
	o->buf_cap = DG_BUF_CAP;
	o->max_table = DG_MAX_TABLE_SIZE;
	o->flags = 0;
}


const char* dg_status_string(int s) {
	switch (s) {
	case DG_OK: return "ok";
	case DG_ERR_INVALID_ARG: return "invalid argument";
	case DG_ERR_UNSUPPORTED: return "unsupported option";
	case DG_ERR_TOO_LARGE: return "input too large for the u32 delta format";
	case DG_ERR_NO_DEVICE: return "no HIP device";
	case DG_ERR_HIP: return "HIP runtime error";
	case DG_ERR_NOMEM: return "out of memory";
	case DG_ERR_CAPACITY: return "output buffer too small";
	case DG_ERR_MALFORMED: return "malformed delta";
	case DG_ERR_SRC_CRC: return "source file does not match delta";
	case DG_ERR_DST_CRC: return "output integrity check failed";
	case DG_ERR_TABLE_POOL: return "onepass work-table pool exhausted";
	case DG_ERR_INTERNAL: return "internal invariant failed on the device (library bug)";
	default: return "unknown status";
	}
}

const char* dg_last_error(const dg_context_t* ctx) { return ctx ? ctx->err.c_str() : ""; }

int dg_context_create(int device, dg_context_t** out) {
	*out = nullptr;
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DG_ERR_NO_DEVICE;
	dg_context_t* ctx = new (std::nothrow) dg_context_t();
	if (!ctx) return DG_ERR_NOMEM;
	if (device < 0) {
		if (hipGetDevice(&device) != hipSuccess) device = 0;
	}
	if (device >= n) { delete ctx; return DG_ERR_NO_DEVICE; }
	ctx->device = device;
	if (hipSetDevice(device) != hipSuccess) { delete ctx; return DG_ERR_HIP; }
	if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) { delete ctx; return DG_ERR_HIP; }
	{
		int cus = 0;
		if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
			ctx->n_cu = (uint32_t)cus;
	}

	// CRC tables: slicing-by-8 and nibble tables of the combine constants
	// + the finaliser's constants: x^(8 kCrcSegBytes) and the 16 pad inverses
	std::vector<uint64_t> tab(kCrcTabWords);
	for (int i = 0; i < 256; ++i) {
		uint64_t c = (uint64_t)i;
		for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
		tab[i] = c;
	}
	for (int k = 1; k < 8; ++k)
		for (int i = 0; i < 256; ++i) {
			const uint64_t prev = tab[(k - 1) * 256 + i];
			tab[k * 256 + i] = (prev >> 8) ^ tab[prev & 0xff];
		}
	for (int lv = 0; lv < kCrcLevels; ++lv) {
		const uint64_t K = gf2_xpow(8ull * 1024 << lv);
		for (int j = 0; j < 16; ++j)
			for (int nb = 0; nb < 16; ++nb)
				tab[8 * 256 + lv * kCrcNibTabWords + 16 * j + nb] = gf2_mul(K, (uint64_t)nb << (4 * j));
	}
	uint64_t xinv[16];
	xinv[0] = 1ULL << 63;
	for (int t = 1; t < 16; ++t) {
		uint64_t z = xinv[t - 1];
		for (int b = 0; b < 8; ++b) z = gf2_div_x(z);
		xinv[t] = z;
	}
	ctx->kseg = gf2_xpow(8ull * kCrcSegBytes);
	for (int c = 0; c < kCrcFinTabs; ++c) {   // nibble tables: kseg, xinv[0..15], kseg^2..4, x^(8*256|512|48Ki)
		const uint64_t K = c == 0 ? ctx->kseg
		                 : c <= 16 ? xinv[c - 1]
		                 : c <= 19 ? gf2_xpow(8ull * kCrcSegBytes * (uint64_t)(c - 15))
		                 : c == kCrcFinX256 ? gf2_xpow(8ull * 256)
		                 : c == kCrcFinX512 ? gf2_xpow(8ull * 512) : gf2_xpow(8ull * 48 * 1024);
		for (int j = 0; j < 16; ++j)
			for (int nb = 0; nb < 16; ++nb)
				tab[8 * 256 + (kCrcLevels + c) * kCrcNibTabWords + 16 * j + nb] = gf2_mul(K, (uint64_t)nb << (4 * j));
	}
	{
		// row-interleaved segment tables: byte j of a PB-byte piece followed by
		// the 64 PB - PB bytes of the other lanes' pieces of its row
		std::vector<uint64_t> adv(256);
		for (int i = 0; i < 256; ++i) adv[i] = tab[i];   // T advanced by 0 bytes
		for (int n = 1; n <= 1023; ++n) {
			for (int i = 0; i < 256; ++i) adv[i] = (adv[i] >> 8) ^ tab[adv[i] & 0xff];
			if (n >= 1008)   // n = 1023 - j
				for (int i = 0; i < 256; ++i) tab[kCrcRows16 + (1023 - n) * 256 + i] = adv[i];
			if (n >= 504 && n <= 511)   // n = 511 - j
				for (int i = 0; i < 256; ++i) tab[kCrcRows8 + (511 - n) * 256 + i] = adv[i];
		}
		uint64_t z = 1ULL << 63;   // x^0
		for (int l = 0; l < 64; ++l) {   // x^(-8*16*l), x^(-8*8*l)
			tab[kCrcRowK16 + l] = z;
			for (int b = 0; b < 128; ++b) z = gf2_div_x(z);
		}
		z = 1ULL << 63;
		for (int l = 0; l < 64; ++l) {
			tab[kCrcRowK8 + l] = z;
			for (int b = 0; b < 64; ++b) z = gf2_div_x(z);
		}
		// five-bit row tables: the images Z^n(2^i) of the 64 register bits
		// (Z = one zero byte through the register), combined per 5-bit field
		auto five = [&](uint32_t base, int n) {
			uint64_t col[64];
			for (int i = 0; i < 64; ++i) {
				uint64_t x = 1ULL << i;
				for (int k = 0; k < n; ++k) x = (x >> 8) ^ tab[x & 0xff];
				col[i] = x;
			}
			for (int k = 0; k < 13; ++k)
				for (int v = 0; v < 32; ++v) {
					uint64_t r = 0;
					for (int b = 0; b < 5; ++b)
						if (((v >> b) & 1) && 5 * k + b < 64) r ^= col[5 * k + b];
					tab[base + 32 * k + v] = r;
				}
		};
		five(kCrc5R8, 512);
		five(kCrc5R16, 1024);
		five(kCrc5R16 + 32 * 13, 1016);
	}
	std::vector<uint64_t> k32(1024);
	{
		const uint64_t step = gf2_xpow(8ull * 32);
		k32[0] = 1ULL << 63;
		for (int t = 1; t < 1024; ++t) k32[t] = gf2_mul(k32[t - 1], step);
	}
	if (hipMalloc(&ctx->d_crc_tables, tab.size() * 8) != hipSuccess ||
	    hipMalloc(&ctx->d_xinv, sizeof xinv) != hipSuccess ||
	    hipMalloc(&ctx->d_k32, 8 * k32.size()) != hipSuccess ||
	    hipMemcpy(ctx->d_crc_tables, tab.data(), tab.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
	    hipMemcpy(ctx->d_xinv, xinv, sizeof xinv, hipMemcpyHostToDevice) != hipSuccess ||
	    hipMemcpy(ctx->d_k32, k32.data(), 8 * k32.size(), hipMemcpyHostToDevice) != hipSuccess) {
		dg_context_destroy(ctx);
		return DG_ERR_HIP;
	}
	*out = ctx;
	return DG_OK;
}

void dg_context_destroy(dg_context_t* ctx) {
	if (!ctx) return;
	hipSetDevice(ctx->device);
	if (ctx->stream) hipStreamSynchronize(ctx->stream);
	hipFree(ctx->d_crc_tables);
	hipFree(ctx->d_xinv);
	hipFree(ctx->d_k32);
	if (ctx->pin) hipHostFree(ctx->pin);
	if (ctx->io && ctx->io_free) ctx->io_free(ctx->io);
	if (ctx->stream) hipStreamDestroy(ctx->stream);
	delete ctx;
}

void* dg_context_stream(dg_context_t* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int dg_context_set_limit(dg_context_t* ctx, int limit, uint64_t value) {
	if (!ctx) return DG_ERR_INVALID_ARG;
	switch (limit) {
	case DG_LIMIT_TABLE_POOL_BYTES:
		ctx->table_pool_bytes = value;
		++ctx->limits_gen;
		return DG_OK;
	case DG_LIMIT_ONEPASS_MEMBERS:
		if (value > 2) return set_err(ctx, DG_ERR_INVALID_ARG, "onepass members mode %llu", (unsigned long long)value);
		ctx->onepass_members = value;
		++ctx->limits_gen;
		return DG_OK;
	default: return set_err(ctx, DG_ERR_INVALID_ARG, "unknown limit %d", limit);
	}
}

}  // extern "C"

const char* dg::ab_env(const char* name) {
#ifdef DG_AB_SWITCHES
	return getenv(name);
#else
	(void)name;
	return nullptr;
#endif
}

// ───────────────────────────── CRC planning ───────────────────────────────

namespace {

// Segment layout for spans whose device address is 16-byte aligned at
// offset 0 of the arena (checked at run time): the padded domain is
// [align_down(off,16), align_up(off+len,16)).
// outs: where span i's CRC goes in CrcArgs::out (nullptr: at i)
void plan_crc_spans(const std::vector<dg_span_t>& spans, const std::vector<uint32_t>& which,
                    std::vector<CrcSpanDev>& sd, std::vector<CrcSegDev>& seg,
                    const std::vector<uint32_t>* outs = nullptr) {
	sd.resize(spans.size());
	seg.clear();
	for (size_t i = 0; i < spans.size(); ++i) {
		CrcSpanDev& s = sd[i];
		s.off = spans[i].off;
		s.len = spans[i].len;
		s.seg_base = (uint32_t)seg.size();
		s.nseg = 0;
		s.which = which[i];
		s.out = outs ? (*outs)[i] : (uint32_t)i;
		if (s.len >= 8) {
			const uint64_t a0 = s.off & ~15ull, a1 = (s.off + s.len + 15) & ~15ull;
			s.nseg = (uint32_t)((a1 - a0 + kCrcSegBytes - 1) / kCrcSegBytes);
			for (uint32_t j = 0; j < s.nseg; ++j) seg.push_back(CrcSegDev{(uint32_t)i, j});
		}
	}
}

struct DevBuf {
	void* p = nullptr;
	size_t n = 0;
	~DevBuf() { if (p) hipFree(p); }
	void release() {
		if (p) hipFree(p);
		p = nullptr;
		n = 0;
	}
	int alloc(size_t bytes) {
		if (p) { hipFree(p); p = nullptr; }
		n = bytes;
		if (bytes == 0) return 0;
		return hipMalloc(&p, bytes) == hipSuccess ? 0 : -1;
	}
	template <class T> T* as() const { return static_cast<T*>(p); }
};

// one u32 of mapped, coherent host memory the device writes (h: host address,
// d: its device address)
struct HostWord {
	uint32_t* h = nullptr;
	uint32_t* d = nullptr;
	~HostWord() { release(); }
	void release() {
		if (h) hipHostFree(h);
		h = d = nullptr;
	}
	int alloc() {
		release();
		if (hipHostMalloc((void**)&h, 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
			h = nullptr;
			return -1;
		}
		*h = 0;
		if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) {
			release();
			return -1;
		}
		return 0;
	}
	uint32_t read() const { return __atomic_load_n(h, __ATOMIC_RELAXED); }
};

}  // namespace

// ───────────────────────────── encode plan ────────────────────────────────

struct dg_encode_plan {
	dg_context_t* ctx = nullptr;
	dg_algorithm_t algo = DG_ALGO_ONEPASS;
	dg_diff_options_t opts{};
	uint32_t n = 0;
	std::vector<dg_pair_t> pairs;
	std::vector<PairPlanDev> pp;
	uint64_t out_bound = 0;
	uint64_t total_rec = 0;
	uint64_t qmax = 0;
	uint64_t ctab_entries = 0;   // correcting: sum of per-pair index sizes
	uint64_t max_seeds = 0;
	uint32_t n_tables = 0;
	bool aligned16 = true;   // every pair offset a multiple of 16 (LDS-window kernel)
	// device buffers
	DevBuf d_pairs, d_pplan, d_powc, d_rec, d_nrec, d_dsize, d_crc_spans_r, d_crc_segs,
	    d_seg_crc, d_crc, d_tables, d_locks, d_tags, d_ctab, d_lookback, d_kcls, d_gpairs, d_prio_flag;
	uint32_t n_gpairs = 0;       // correcting: pairs whose R index is built in memory
	// onepass member mode (dg_members.hip): member arrays share the record
	// slots' indexing; the verification work queue
	bool members = false;
	DevBuf d_mem_s, d_srec, d_nmem, d_chunks, d_csum, d_cmap, d_seg, d_nseg;
	uint32_t n_chunks = 0;
	uint32_t n_crc_spans = 0, n_crc_segs = 0;
	// fork/join of the CRC kernels onto a side stream
	hipStream_t side = nullptr;
	hipEvent_t ev_fork = nullptr, ev_join = nullptr;
	bool serial_crc = false;   // DG_SERIAL_CRC=1: CRC on the run stream (A/B)
	bool crc_first = false;    // DG_CRC_FIRST=1: enqueue the CRC before the differencing (A/B)
	bool chain_join = false;   // DG_CHAIN_JOIN=1: member plans' routed chain always waits for the CRC pass (A/B)
	bool crc_late_fin = true;  // member plans: the CRC's combine after the chains (DG_CRC_JOIN=0: not, A/B)
	bool crc_patch = false;    // DG_CRC_PATCH=1: header CRCs by crc_patch_kernel after the serialiser (A/B)
	bool skip_crc = false;     // DG_SKIP_CRC=1: no CRC kernels, wrong header CRCs (A/B bound only)
	uint32_t corr_lds_cap = 0; // correcting: R indexes up to this many slots built in LDS (DG_CORR_BUILD=global: none)
	bool crc_fused = false;    // correcting: R's CRC computed by the LDS build, V's forked after it
	bool op_crc = false;       // onepass plain plans: both CRCs computed by the onepass waves (no CRC pass)
	bool crc_wide = false;     // correcting: R's and V's CRC in one wide-table pass before the build
	bool crc_wide_beside = false;   // ... or forked after the build, beside the V scan
	uint32_t route_min = 0;    // member mode chosen automatically: route poorly verified pairs to the plain chain
	// automatic member mode: the routed-pair count of the last completed run
	// (written by scan_sizes_kernel into mapped host memory) decides whether the
	// routed chain waits for the CRC pass (see the run)
	DevBuf d_route_cnt;
	HostWord route_fb;
	uint32_t plain_streak = 0;   // runs since the last member-mode probe (dg_encode_plan_run)
	uint64_t member_runs = 0, plain_runs = 0;   // dg_encode_plan_run_modes
	uint64_t* stats = nullptr; // dg_encode_plan_set_stats: --verbose counters (device, 8 per pair)
	uint64_t qmin = ~0ull;
	uint64_t v_total = 0;      // sum |V| of the batch
	uint32_t dbg = 0;          // DG_DEBUG_BITS: kernel A/B switches (A/B builds only)
	bool fused = false;        // DG_FUSED=1: onepass16 serialises in-kernel (default: scan + serialise)
	// timing
	bool timing = false;
	int timing_mode = DG_TIMING_ALL;
	// timing: `slots` sets of kTimingEvents events, one set per run (ring);
	// ev holds ev_sets >= slots sets (never shrunk, only the ring is)
	std::vector<hipEvent_t> ev;
	uint32_t slots = 0, runs = 0, ev_sets = 0;
	uint32_t every = 1, calls = 0;   // events on every `every`-th run (dg_*_plan_set_timing_every)
	hipEvent_t* cur = nullptr;   // event set of the run being enqueued
};

static const char* kStageNames[] = {"crc64", "diff", "scan", "serialize+join", "total", "members", "corr_build", "corr_scan"};

// ── --verbose: the reference's diagnostics from device counters and the delta ──

static uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

namespace {
struct Cmd { bool copy; uint64_t src, dst, len; };
// the standard delta's commands (encoding.c:39-90 layout), in stream order
bool parse_cmds(const uint8_t* d, size_t n, std::vector<Cmd>& out) {
	if (n < 26 || memcmp(d, "DLT\x03", 4) != 0) return false;
	size_t i = 25;
	while (i < n) {
		const uint8_t t = d[i];
		if (t == 0) return true;
		if (t == 1 && i + 13 <= n) {
			out.push_back(Cmd{true, be32(d + i + 1), be32(d + i + 5), be32(d + i + 9)});
			i += 13;
		} else if (t == 2 && i + 9 <= n) {
			const uint64_t len = be32(d + i + 5);
			out.push_back(Cmd{false, 0, be32(d + i + 1), len});
			i += 9 + len;
		} else {
			return false;
		}
	}
	return false;
}

// delta_print_command_stats (correcting.c:523-576)
void print_command_stats(const std::vector<Cmd>& cmds) {
	uint64_t tc = 0, ta = 0, nc = 0, na = 0;
	std::vector<uint64_t> lens;
	for (const Cmd& c : cmds) {
		if (c.copy) { tc += c.len; ++nc; lens.push_back(c.len); }
		else { ta += c.len; ++na; }
	}
	const uint64_t tot = tc + ta;
	fprintf(stderr,
	        "  result: %llu copies (%llu bytes), %llu adds (%llu bytes)\n"
	        "  result: copy coverage %.1f%%, output %llu bytes\n",
	        (unsigned long long)nc, (unsigned long long)tc, (unsigned long long)na, (unsigned long long)ta,
	        tot > 0 ? (double)tc / tot * 100.0 : 0.0, (unsigned long long)tot);
	if (!lens.empty()) {
		std::sort(lens.begin(), lens.end());
		fprintf(stderr, "  copies: %llu regions, min=%llu max=%llu mean=%.1f median=%llu bytes\n",
		        (unsigned long long)lens.size(), (unsigned long long)lens.front(), (unsigned long long)lens.back(),
		        (double)tc / lens.size(), (unsigned long long)lens[lens.size() / 2]);
	}
}
}  // namespace

void dg::print_verbose(const dg_encode_plan_t* P, uint32_t i, const uint64_t* st, const uint8_t* delta,
                       size_t delta_len) {
	const dg_pair_t& d = P->pairs[i];
	const PairPlanDev& x = P->pp[i];
	const uint64_t p = P->opts.p;
	if (d.v_len == 0) return;   // the reference returns before printing (onepass.c:58, correcting.c:112)
	std::vector<Cmd> cmds;
	parse_cmds(delta, delta_len, cmds);
	if (P->algo == DG_ALGO_ONEPASS) {
		// onepass.c:64-69 and :277-285.  positions: every epoch's steps up to
		// its match (t + 1, t = max(v_m - v0, r_m - r0)) plus the final
		// epoch's steps while either stream has a window; lookups: one per
		// match (a probe counts only on a full-fingerprint hit, onepass.c:169-
		// 219, and fingerprints of distinct 16-byte windows coincide with
		// probability ~2^-61)
		fprintf(stderr, "onepass: %s, q=%llu, |R|=%llu, |V|=%llu, seed_len=%llu\n", "hash table",
		        (unsigned long long)x.q, (unsigned long long)d.r_len, (unsigned long long)d.v_len,
		        (unsigned long long)p);
		uint64_t pos = 0, matches = 0, v0 = 0, r0 = 0;
		for (const Cmd& c : cmds) {
			if (!c.copy) continue;
			pos += std::max(c.dst - v0, c.src - r0) + 1;
			++matches;
			v0 = c.dst + c.len;
			r0 = c.src + c.len;
		}
		const uint64_t nv = d.v_len + 1 >= v0 + p ? d.v_len + 1 - p - v0 : 0;
		const uint64_t nr = d.r_len + 1 >= r0 + p ? d.r_len + 1 - p - r0 : 0;
		pos += std::max(nv, nr);
		fprintf(stderr,
		        "  scan: %llu positions, %llu lookups, %llu matches (flushes)\n"
		        "  scan: hit rate %.1f%% (of lookups)\n",
		        (unsigned long long)pos, (unsigned long long)matches, (unsigned long long)matches,
		        matches > 0 ? 100.0 : 0.0);
		print_command_stats(cmds);
		return;
	}
	// correcting.c:137-152, 200-214, 470-485
	const uint64_t seeds = d.r_len >= p ? d.r_len - p + 1 : 0;
	const uint64_t cap = x.q, m = x.m, k = st ? st[6] : 0;
	const uint64_t expected = m > 0 ? seeds / m : 0;
	fprintf(stderr,
	        "correcting: %s, |C|=%llu |F|=%llu m=%llu k=%llu\n"
	        "  checkpoint gap=%llu bytes, expected fill ~%llu (~%llu%% table occupancy)\n"
	        "  table memory ~%llu MB\n",
	        "hash table", (unsigned long long)cap, (unsigned long long)x.f_size, (unsigned long long)m,
	        (unsigned long long)k, (unsigned long long)m, (unsigned long long)expected,
	        (unsigned long long)(cap > 0 ? expected * 100 / cap : 0), (unsigned long long)(cap * 24 / 1048576));
	const uint64_t passed = st ? st[0] : 0, stored = st ? st[1] : 0, in_cap = st ? st[7] : 0;
	fprintf(stderr,
	        "  build: %llu seeds, %llu passed checkpoint (%.2f%%), %llu stored, %llu collisions\n"
	        "  build: table occupancy %llu/%llu (%.1f%%)\n",
	        (unsigned long long)seeds, (unsigned long long)passed, seeds > 0 ? (double)passed / seeds * 100.0 : 0.0,
	        (unsigned long long)stored, (unsigned long long)(in_cap - stored), (unsigned long long)stored,
	        (unsigned long long)cap, cap > 0 ? (double)stored / cap * 100.0 : 0.0);
	const uint64_t vseeds = d.v_len >= p ? d.v_len - p + 1 : 0;
	const uint64_t ck = st ? st[2] : 0, fpm = st ? st[3] : 0, bm = st ? st[4] : 0, mt = st ? st[5] : 0;
	fprintf(stderr,
	        "  scan: %llu V positions, %llu checkpoints (%.3f%%), %llu matches\n"
	        "  scan: hit rate %.1f%% (of checkpoints), fp collisions %llu, byte mismatches %llu\n",
	        (unsigned long long)vseeds, (unsigned long long)ck, vseeds > 0 ? (double)ck / vseeds * 100.0 : 0.0,
	        (unsigned long long)mt, ck > 0 ? (double)mt / ck * 100.0 : 0.0, (unsigned long long)fpm,
	        (unsigned long long)bm);
	print_command_stats(cmds);
}

extern "C" {

// member mode wanted for this batch (automatic choice by mean pair size:
// measured C3 (256 KiB pairs) +56 %, C2 (64 KiB pairs) -22 %,
// profiles/r02_experiments.md); the context's mode and the A/B switches
// DG_NO_MEMBERS / DG_MEMBERS override it
static bool members_wanted(const dg_context_t* ctx, const dg_pair_t* pairs, uint32_t n) {
	uint64_t vsum = 0;
	for (uint32_t i = 0; i < n; ++i) vsum += pairs[i].v_len;
	bool want = n && vsum / n >= (128u << 10);
	if (ctx->onepass_members == 1) want = true;
	if (ctx->onepass_members == 2) want = false;
	const char* nm = ab_env("DG_NO_MEMBERS");
	if (nm && nm[0] == '1') want = false;
	const char* fm = ab_env("DG_MEMBERS");
	if (fm && fm[0] == '1') want = true;
	return want;
}
#ifndef DG_CRC_PRIO_FLAG   // A/B: member plans raise the rows pass to priority 1 after the member kernel
#define DG_CRC_PRIO_FLAG 0
#endif
constexpr bool kCrcPrioFlag = DG_CRC_PRIO_FLAG != 0;
#ifndef DG_OP_CRC_DEFAULT   // 1 (A/B): onepass plain plans compute their CRCs in the onepass waves
#define DG_OP_CRC_DEFAULT 0   // (measured slower: C2 1786 -> 1172 GiB/s, profiles/r06_experiments.md)
#endif
constexpr bool kOpCrcDefault = DG_OP_CRC_DEFAULT != 0;

int dg_encode_plan_create(dg_context_t* ctx, dg_algorithm_t algo, const dg_pair_t* pairs,
                          uint32_t n, const dg_diff_options_t* opts, dg_encode_plan_t** out) {
	*out = nullptr;
	if (!ctx) return DG_ERR_INVALID_ARG;
	dg_diff_options_t o;
	if (opts) o = *opts; else dg_diff_options_default(&o);
	if (algo == DG_ALGO_GREEDY)
		return set_err(ctx, DG_ERR_UNSUPPORTED, "greedy is not implemented on the GPU path");
	if (algo != DG_ALGO_ONEPASS && algo != DG_ALGO_CORRECTING)
		return set_err(ctx, DG_ERR_INVALID_ARG, "unknown algorithm %d", (int)algo);
	if ((o.flags >> DG_OPT_SPLAY) & 1)
		return set_err(ctx, DG_ERR_UNSUPPORTED, "--splay is not supported (hash-table path only)");
	if ((o.flags >> DG_OPT_INPLACE) & 1)
		return set_err(ctx, DG_ERR_UNSUPPORTED,
		               "in-place conversion is a host step: encode standard deltas, then dg_make_inplace");
	if (o.p == 0) return set_err(ctx, DG_ERR_INVALID_ARG, "--seed-len must be >= 1");
	if (o.p > 65536) return set_err(ctx, DG_ERR_INVALID_ARG, "--seed-len above 65536 is not supported");
	if (algo == DG_ALGO_CORRECTING && o.buf_cap > 4095)
		return set_err(ctx, DG_ERR_UNSUPPORTED, "--buffer-size above 4095 is not supported (LDS lookback ring)");
	if (n > 0 && !pairs) return DG_ERR_INVALID_ARG;

	dg_encode_plan_t* P = new (std::nothrow) dg_encode_plan_t();
	if (!P) return DG_ERR_NOMEM;
	P->ctx = ctx;
	P->algo = algo;
	P->opts = o;
	P->n = n;
	P->pairs.assign(pairs, pairs + n);
	P->pp.resize(n);
	hipSetDevice(ctx->device);

	std::map<uint64_t, uint64_t> qcache;
	uint64_t rec = 0, bound = 0, ctab = 0;
	const uint64_t p = o.p;
	for (uint32_t i = 0; i < n; ++i) {
		const dg_pair_t& d = pairs[i];
		// the format's u32 fields cap every buffer below 4 GiB (encoding.c:63,72-78);
		// the kernels keep 32-bit cursors with 1 MiB of headroom
		if (d.r_len >= (1ull << 32) - (1ull << 20) || d.v_len >= (1ull << 32) - (1ull << 20)) {
			delete P;
			return set_err(ctx, DG_ERR_TOO_LARGE, "pair %u: buffers of 4 GiB or more do not fit the u32 format", i);
		}
		if ((d.r_off | d.v_off) & 15) P->aligned16 = false;
		PairPlanDev& x = P->pp[i];
		memset(&x, 0, sizeof x);
		const uint64_t seeds = d.r_len >= p ? d.r_len - p + 1 : 0;
		if (algo == DG_ALGO_ONEPASS) {
			const uint64_t want = std::max<uint64_t>(o.q, seeds / p);   // onepass.c:61-62
			auto it = qcache.find(want);
			x.q = it != qcache.end() ? it->second : (qcache[want] = next_prime(want));
		} else {
			// correcting.c:116-129
			const uint64_t mt = o.max_table > 0 ? o.max_table : DG_MAX_TABLE_SIZE;
			uint64_t raw = seeds > 0 ? std::max<uint64_t>(o.q, 2 * seeds / p) : o.q;
			raw = std::min<uint64_t>(raw, mt);
			auto it = qcache.find(raw);
			x.q = it != qcache.end() ? it->second : (qcache[raw] = next_prime(raw));
			x.f_size = seeds > 0 ? next_prime(2 * seeds) : 1;
			x.m = x.f_size <= x.q ? 1 : (x.f_size + x.q - 1) / x.q;
			x.f_magic = UINT64_MAX / x.f_size;
			x.m_magic = UINT64_MAX / x.m;
			x.tab_base = ctab;
			ctab += x.q;
			P->max_seeds = std::max<uint64_t>(P->max_seeds, seeds);
		}
		if (x.q >= 0xFFFFFFFFull) {
			delete P;
			return set_err(ctx, DG_ERR_TOO_LARGE, "table size %llu too large", (unsigned long long)x.q);
		}
		x.q_magic = UINT64_MAX / x.q;
		x.rec_base = rec;
		x.rec_cap = (uint32_t)(d.v_len / p + 1);
		rec += x.rec_cap;
		// onepass: every COPY covers >= p bytes, so
		//   delta <= 35 + |V| + (|V|/p) * max(0, 22 - p);
		// correcting: a tail-corrected COPY may be shorter than p, but there
		// are at most |V|/p + 1 of them, each with at most one ADD header
		if (algo == DG_ALGO_ONEPASS)
			bound += 35 + d.v_len + (d.v_len / p) * (p < 22 ? 22 - p : 0);
		else
			bound += 57 + d.v_len + 22 * (d.v_len / p);
		P->qmax = std::max<uint64_t>(P->qmax, x.q);
		P->qmin = std::min<uint64_t>(P->qmin, x.q);
	}
	P->out_bound = bound;
	P->total_rec = rec;
	P->ctab_entries = ctab;
	if (ctab * 4 > (64ull << 30)) {
		delete P;
		return set_err(ctx, DG_ERR_NOMEM, "correcting R indexes need %llu GiB (limit 64)",
		               (unsigned long long)(ctab >> 28));
	}

	// constants 263^(p-1-k) mod (2^61-1)
	std::vector<uint64_t> powc(p);
	{
		uint64_t c = 1;
		for (uint64_t k = 0; k < p; ++k) {
			powc[p - 1 - k] = c;
			c = (uint64_t)((u128)c * kBase % kMersenne);
		}
	}
	{
		const char* cb = ab_env("DG_CORR_BUILD");
		int shm = 0;
		if (hipDeviceGetAttribute(&shm, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device) != hipSuccess)
			shm = 0;
		// Correcting plans compute the CRCs in one of four ways (A/B:
		// DG_CORR_CRC = fused | wide | widebeside | beside):
		//   fused  (default) the LDS build computes R's CRC from the bytes it
		//          holds and V's runs beside the V scan (C4: 2.77 ms per step);
		//   wide   one pass over R and V before the build, with the GPU to
		//          itself: bank-spread slicing tables in 128 KiB of LDS per CU
		//          (crc_segments_wide_kernel), ~2 LDS cycles a lookup (2.84 ms);
		//   widebeside  the wide pass forked after the build, beside the V
		//          scan (2.80 ms: it outlasts the scan);
		//   beside the onepass arrangement: both CRCs on the side stream
		//          beside the build (whose 130 KiB-LDS blocks leave it ~1/8 of
		//          each CU).
		const char* cm = ab_env("DG_CORR_CRC");
		int mode = 1;
		if (cm) mode = !strcmp(cm, "wide") ? 2 : (!strcmp(cm, "beside") ? 0 : (!strcmp(cm, "widebeside") ? 3 : 1));
		if (algo != DG_ALGO_CORRECTING || !n) mode = 0;
		if ((mode == 2 || mode == 3) && shm < 8 * 4 * 256 * 16 + 1024) mode = 0;
		// one block's LDS less the 2 KiB roll table, the fused R CRC's tables
		// (10 KiB) and reduction words, and some slack
		const int fixed = 2048 + (mode == 1 ? 10240 + 128 : 0) + 256;
		if (algo == DG_ALGO_CORRECTING && !(cb && strcmp(cb, "global") == 0) && shm > fixed + 4096)
			P->corr_lds_cap = (uint32_t)((shm - fixed) / 4);
		// fused: only R indexes built in LDS compute R's CRC; the others' R
		// CRCs run in V's pass
		P->crc_fused = mode == 1 && P->corr_lds_cap && P->qmin <= P->corr_lds_cap;
		P->crc_wide = mode == 2 || mode == 3;
		P->crc_wide_beside = mode == 3;
	}
	if (P->crc_fused) {   // x^(-8 pad) of each R's zero padding to a multiple of 32 KiB
		uint64_t xm8 = 1ULL << 63;
		for (int b = 0; b < 8; ++b) xm8 = gf2_div_x(xm8);
		std::map<uint64_t, uint64_t> cache;
		for (uint32_t i = 0; i < n; ++i) {
			const uint64_t pad = (32768 - pairs[i].r_len % 32768) % 32768;
			auto it = cache.find(pad);
			if (it == cache.end()) {
				uint64_t r = 1ULL << 63, base = xm8;
				for (uint64_t e = pad; e; e >>= 1) {
					if (e & 1) r = gf2_mul(r, base);
					base = gf2_mul(base, base);
				}
				it = cache.emplace(pad, r).first;
			}
			P->pp[i].crc_unpad = it->second;
		}
	}
	// onepass plain plans (the LDS-window chain, no member mode, no in-kernel
	// serialisation) with DG_OP_CRC_DEFAULT=1: the onepass waves compute both
	// CRCs from the bytes their windows stage (onepass16_crc_kernel), so no
	// CRC pass reads R and V a second time.  Off in the product: the folds
	// lengthen every wave's latency-bound chain (C2 kernel 0.221 -> 0.375 ms)
	// by far more than the rows pass beside it costs the step (~0.02 ms).
	// DG_OP_CRC=0 (A/B builds) turns it off in such a build.
	{
		const char* oc = ab_env("DG_OP_CRC");
		const char* fz = ab_env("DG_FUSED");
		P->op_crc = kOpCrcDefault && algo == DG_ALGO_ONEPASS && o.p == 16 && P->aligned16 && onepass16_selected() &&
		            !(fz && fz[0] == '1') && !members_wanted(ctx, pairs, n) && !(oc && oc[0] == '0');
	}
	// CRC spans: 2 per pair (R then V; V only when the build computes R's;
	// none when the onepass waves compute both); arena offsets are rebased at
	// run time
	std::vector<dg_span_t> spans;
	std::vector<uint32_t> which, outs;
	for (uint32_t i = 0; i < n && !P->op_crc; ++i) {
		if (!P->crc_fused || P->pp[i].q > P->corr_lds_cap) {
			spans.push_back(dg_span_t{pairs[i].r_off, pairs[i].r_len});
			which.push_back(0);
			outs.push_back(2 * i);
		}
		spans.push_back(dg_span_t{pairs[i].v_off, pairs[i].v_len});
		which.push_back(1);
		outs.push_back(2 * i + 1);
	}
	std::vector<CrcSpanDev> sd;
	std::vector<CrcSegDev> seg;
	plan_crc_spans(spans, which, sd, seg, &outs);
	P->n_crc_spans = (uint32_t)sd.size();
	P->n_crc_segs = (uint32_t)seg.size();

	// table-tier pool: 2 x qmax u64 per table.  Automatic size: one table per
	// resident onepass wave (CUs x 4 SIMDs x 5 waves) where that fits in
	// 4 GiB, at least 1 GiB; never more tables than pairs.
	const uint64_t per = 16ull * std::max<uint64_t>(P->qmax, 1);
	uint64_t pool = ctx->table_pool_bytes;
	if (pool == 0) {
		const uint64_t resident = 20ull * ctx->n_cu;
		pool = std::max<uint64_t>(1ull << 30, std::min<uint64_t>(resident * per, 4ull << 30));
	}
	P->n_tables = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint32_t>(n, 1), pool / per));
	// the device partitions the pool by XCD (8 per GPU): a multiple of 8
	// tables, at least 8 where the pool holds them
	if (pool / per >= 8) P->n_tables = std::max<uint32_t>(8, P->n_tables & ~7u);

	int bad = 0;
	bad |= P->d_pairs.alloc(sizeof(PairDev) * std::max<uint32_t>(n, 1));
	bad |= P->d_pplan.alloc(sizeof(PairPlanDev) * std::max<uint32_t>(n, 1));
	bad |= P->d_powc.alloc(8 * p);
	bad |= P->d_rec.alloc(4ull * (algo == DG_ALGO_ONEPASS ? kRecWordsOnepass : kRecWordsCorrecting) *
	                      std::max<uint64_t>(rec, 1));
	bad |= P->d_nrec.alloc(4ull * std::max<uint32_t>(n, 1));
	bad |= P->d_dsize.alloc(8ull * std::max<uint32_t>(n, 1));
	bad |= P->d_crc_spans_r.alloc(sizeof(CrcSpanDev) * std::max<size_t>(sd.size(), 1));
	bad |= P->d_crc_segs.alloc(sizeof(CrcSegDev) * std::max<size_t>(seg.size(), 1));
	bad |= P->d_seg_crc.alloc(8 * std::max<size_t>(seg.size(), 1));
	bad |= P->d_crc.alloc(16ull * std::max<uint32_t>(n, 1));   // per pair: CRC of R, of V
	bad |= P->d_tables.alloc(per * P->n_tables);
	bad |= P->d_locks.alloc(4ull * P->n_tables);
	bad |= P->d_tags.alloc(4ull * P->n_tables);
	if (algo == DG_ALGO_CORRECTING) {
		std::vector<uint32_t> gp;
		for (uint32_t i = 0; i < n; ++i)
			if (P->pp[i].q > P->corr_lds_cap) gp.push_back(i);
		P->n_gpairs = (uint32_t)gp.size();
		bad |= P->d_gpairs.alloc(4ull * std::max<size_t>(gp.size(), 1));
		if (!bad && !gp.empty() &&
		    hipMemcpy(P->d_gpairs.p, gp.data(), 4 * gp.size(), hipMemcpyHostToDevice) != hipSuccess)
			bad = 1;
		bad |= P->d_ctab.alloc(4ull * std::max<uint64_t>(ctab, 1));
		bad |= P->d_kcls.alloc(8ull * std::max<uint32_t>(n, 1));
	}
	{
		// DG_FUSED=1: onepass16 serialises in-kernel behind a decoupled look-back.
		// Off by default: the look-back couples every wave to the slowest pair
		// before it, which cost 20-25% at C2/C3 on MI355X (profiles/r01_ab_fused_vs_unfused.txt).
		const char* fz = ab_env("DG_FUSED");
		P->fused = algo == DG_ALGO_ONEPASS && o.p == 16 && P->aligned16 && onepass16_selected() &&
		           fz && fz[0] == '1';
	}
	if (P->fused) bad |= P->d_lookback.alloc(8ull * std::max<uint32_t>(n, 1));
	{
		// member mode: p = 16 onepass over 16-byte aligned pairs (the LDS-window
		// chain), i.e. the batched hot configuration; DG_NO_MEMBERS=1 (A/B
		// builds) runs the plain chain
		// automatic choice by mean pair size for now: measured
		// (profiles/r02_experiments.md) C3 (256 KiB pairs) +56 %, C2 (64 KiB
		// pairs, where the plain chain's latency-bound waves overlap the CRC)
		// -22 %
		const bool want = members_wanted(ctx, pairs, n);
		P->members = algo == DG_ALGO_ONEPASS && o.p == 16 && P->aligned16 && onepass16_selected() &&
		             !P->fused && want;
		// automatic mode: a pair averaging fewer than 2 verified members per
		// 2 KiB chunk runs the plain chain (C3: ~39; shift and transposition
		// pairs, whose matches leave diagonal 0: ~0); forced member mode
		// keeps every pair on the member chain
		const char* rm = ab_env("DG_ROUTE_MIN");
		P->route_min = ctx->onepass_members == 0 ? (rm ? (uint32_t)strtoul(rm, nullptr, 0) : 2u) : 0u;
	}
	for (uint32_t i = 0; i < n; ++i) P->v_total += pairs[i].v_len;
	if (P->members) {
		// chunks of kMemChunk positions covering [0, min(|R|, |V|)]; member
		// slots per chunk; the (pair, chunk) table the member kernel's waves index
		std::vector<uint32_t> jobs;
		uint64_t slots = 0;
		for (uint32_t i = 0; i < n; ++i) {
			const uint64_t E = std::min<uint64_t>(pairs[i].r_len, pairs[i].v_len);
			const uint32_t nch = (uint32_t)(E / kMemChunk + 1);
			P->pp[i].mem_base = slots;
			P->pp[i].chunk_base = P->n_chunks;
			P->pp[i].n_chunks = nch;
			for (uint32_t c = 0; c < nch; ++c) {
				jobs.push_back(i);
				jobs.push_back(c);
			}
			slots += (uint64_t)nch * kMemChunkSlots;
			P->n_chunks += nch;
		}
		int mbad = 0;
		mbad |= P->d_mem_s.alloc(4ull * std::max<uint64_t>(slots, 1));
		mbad |= P->d_srec.alloc(16ull * std::max<uint64_t>(slots, 1));
		mbad |= P->d_nmem.alloc(4ull * std::max<uint32_t>(P->n_chunks, 1));
		mbad |= P->d_chunks.alloc(8ull * std::max<uint32_t>(P->n_chunks, 1));
		mbad |= P->d_csum.alloc(8ull * std::max<uint32_t>(P->n_chunks, 1));
		mbad |= P->d_cmap.alloc(8ull * std::max<uint32_t>(P->n_chunks, 1));
		mbad |= P->d_seg.alloc(16ull * ((uint64_t)P->n_chunks + 2ull * n));
		mbad |= P->d_nseg.alloc(4ull * std::max<uint32_t>(n, 1));
		mbad |= P->d_prio_flag.alloc(4);
		if (P->route_min) {
			mbad |= P->d_route_cnt.alloc(4);
			mbad |= P->route_fb.alloc();
			if (!mbad && hipMemset(P->d_route_cnt.p, 0, 4) != hipSuccess) mbad = 1;
		}
		if (!mbad && !jobs.empty() &&
		    hipMemcpy(P->d_chunks.p, jobs.data(), 4 * jobs.size(), hipMemcpyHostToDevice) != hipSuccess)
			mbad = 1;
		if (mbad && ctx->onepass_members != 1) {
			// automatic mode: member mode is an optimisation, so a batch that
			// fits with the plain chain still gets a plan
			(void)hipGetLastError();
			for (DevBuf* b : {&P->d_mem_s, &P->d_srec, &P->d_nmem, &P->d_chunks, &P->d_csum, &P->d_cmap,
			                  &P->d_seg, &P->d_nseg, &P->d_prio_flag, &P->d_route_cnt})
				b->release();
			P->route_fb.release();
			P->members = false;
			P->n_chunks = 0;
			mbad = 0;
		}
		bad |= mbad;
	}
	if (bad) {
		delete P;
		return set_err(ctx, DG_ERR_NOMEM, "device allocation failed");
	}
	hipStream_t st = ctx->stream;
	hipError_t e = hipSuccess;
	if (n) {
		e = hipMemcpyAsync(P->d_pairs.p, pairs, sizeof(PairDev) * n, hipMemcpyHostToDevice, st);
		if (e == hipSuccess) e = hipMemcpyAsync(P->d_pplan.p, P->pp.data(), sizeof(PairPlanDev) * n, hipMemcpyHostToDevice, st);
		if (e == hipSuccess) e = hipMemcpyAsync(P->d_crc_spans_r.p, sd.data(), sizeof(CrcSpanDev) * sd.size(), hipMemcpyHostToDevice, st);
		if (e == hipSuccess && !seg.empty()) e = hipMemcpyAsync(P->d_crc_segs.p, seg.data(), sizeof(CrcSegDev) * seg.size(), hipMemcpyHostToDevice, st);
	}
	if (e == hipSuccess) e = hipMemcpyAsync(P->d_powc.p, powc.data(), 8 * p, hipMemcpyHostToDevice, st);
	if (e == hipSuccess) e = hipMemsetAsync(P->d_tables.p, 0, P->d_tables.n, st);
	if (e == hipSuccess) e = hipMemsetAsync(P->d_locks.p, 0, P->d_locks.n, st);
	if (e == hipSuccess) e = hipMemsetAsync(P->d_tags.p, 0, P->d_tags.n, st);
	if (e == hipSuccess) e = hipStreamSynchronize(st);
	if (e != hipSuccess) {
		delete P;
		return set_err(ctx, DG_ERR_HIP, "plan upload failed: %s", hipGetErrorString(e));
	}
	const char* sc = ab_env("DG_SERIAL_CRC");
	P->serial_crc = sc && sc[0] == '1';
	const char* db = ab_env("DG_DEBUG_BITS");
	P->dbg = db ? (uint32_t)strtoul(db, nullptr, 0) : 0;
	const char* cf = ab_env("DG_CRC_FIRST");
	P->crc_first = cf && cf[0] == '1';
	const char* chj = ab_env("DG_CHAIN_JOIN");
	P->chain_join = chj && chj[0] == '1';
	const char* cj = ab_env("DG_CRC_JOIN");
	if (cj) P->crc_late_fin = cj[0] != '0';
	const char* cp = ab_env("DG_CRC_PATCH");
	P->crc_patch = cp && cp[0] == '1';
	const char* sk = ab_env("DG_SKIP_CRC");
	P->skip_crc = sk && sk[0] == '1';

	if (!P->serial_crc) {
		e = hipStreamCreateWithFlags(&P->side, hipStreamNonBlocking);
		// stream-to-stream ordering on one device: a device-scope release (the
		// default system-scope one writes back and invalidates the caches)
		if (e == hipSuccess) e = hipEventCreateWithFlags(&P->ev_fork, hipEventDisableTiming | hipEventReleaseToDevice);
		if (e == hipSuccess) e = hipEventCreateWithFlags(&P->ev_join, hipEventDisableTiming | hipEventReleaseToDevice);
		if (e != hipSuccess) {
			dg_encode_plan_destroy(P);
			return set_err(ctx, DG_ERR_HIP, "side stream creation failed: %s", hipGetErrorString(e));
		}
	}
	*out = P;
	return DG_OK;
}

uint64_t dg_encode_plan_output_bound(const dg_encode_plan_t* P) { return P ? P->out_bound : 0; }
uint32_t dg_encode_plan_num_pairs(const dg_encode_plan_t* P) { return P ? P->n : 0; }
uint32_t dg_encode_plan_flags(const dg_encode_plan_t* P) { return P && P->members ? DG_PLAN_MEMBERS : 0u; }
int dg_encode_plan_run_modes(const dg_encode_plan_t* P, uint64_t* member_runs, uint64_t* plain_runs) {
	if (!P || !member_runs || !plain_runs) return DG_ERR_INVALID_ARG;
	*member_runs = P->member_runs;
	*plain_runs = P->plain_runs;
	return DG_OK;
}

int dg_encode_plan_set_stats(dg_encode_plan_t* P, uint64_t* d_stats) {
	if (!P) return DG_ERR_INVALID_ARG;
	P->stats = d_stats;
	return DG_OK;
}
#ifdef DG_AB_SWITCHES
// A/B and profiling builds only: the member kernel's outputs of the last run
// (device pointers; scripts/member_debug.py)
int dg_encode_plan_member_debug(const dg_encode_plan_t* P, void** mem_s, void** srec, void** n_mem,
                                void** csum, uint32_t* n_chunks) {
	if (!P || !P->members) return -1;
	*mem_s = P->d_mem_s.p;
	*srec = P->d_srec.p;
	*n_mem = P->d_nmem.p;
	*csum = P->d_csum.p;
	*n_chunks = P->n_chunks;
	return 0;
}
#endif
uint64_t dg_encode_plan_table_size(const dg_encode_plan_t* P, uint32_t i) {
	return (P && i < P->n) ? P->pp[i].q : 0;
}
const uint32_t* dg_encode_plan_copy_counts_device(const dg_encode_plan_t* P) {
	return P ? P->d_nrec.as<uint32_t>() : nullptr;
}

constexpr int kTimingEvents = 8;
constexpr uint32_t kTimingAll = (1u << kTimingEvents) - 1u;
// the events a run records: all, or around the dominant kernel(s) only —
// the member kernel (2, 6), the correcting build and scan (2, 7, 3), the
// plain onepass kernel (2, 3); member plans also 3 (the chains after the
// member kernel: the routed plain chain dominates on data off diagonal 0)
static uint32_t timing_mask(const dg_encode_plan_t* P) {
	if (P->timing_mode != DG_TIMING_DOMINANT) return kTimingAll;
	if (P->members) return (1u << 2) | (1u << 6) | (1u << 3);   // the member kernel, then the chains
	if (P->algo == DG_ALGO_CORRECTING) return (1u << 2) | (1u << 7) | (1u << 3);
	return (1u << 2) | (1u << 3);
}

int dg_encode_plan_set_timing(dg_encode_plan_t* P, int slots) {
	if (!P || slots < 0) return DG_ERR_INVALID_ARG;
	hipSetDevice(P->ctx->device);
	if ((uint32_t)slots > P->ev_sets) {
		for (auto& e : P->ev) hipEventDestroy(e);
		P->ev.assign((size_t)kTimingEvents * slots, nullptr);
		P->ev_sets = P->slots = 0;
		for (auto& e : P->ev)
			// timing only: no system-scope fence when the event is recorded
			// (a cache writeback + invalidate per event slowed the timed
			// steps by 15 %: C2 0.335 -> 0.391 ms with two events per step)
			if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
				e = nullptr;
				P->timing = false;
				return set_err(P->ctx, DG_ERR_HIP, "hipEventCreate failed");
			}
		P->ev_sets = (uint32_t)slots;
	}
	// the ring is exactly `slots` runs long, so stage_times averages the
	// last `slots` runs even after a longer ring was set before
	P->slots = (uint32_t)slots;
	P->timing = slots > 0;
	P->runs = P->calls = 0;
	return DG_OK;
}

// Per-run events: 0/1 around the CRC kernels (side stream), 2/3 around the
// differencing kernel(s), 4 after the scan, 5 after serialisation + the CRC
// join + the header patch (DG_FUSED=1: the join falls before 4), 6 after
// the member kernel (member mode; else with 2), 7 after the correcting R-index build (before the V scan; onepass: with 3).  Stages
// corr_build (2..7) and corr_scan (7..3) are reported for correcting plans only.
// Returns the mean over the runs recorded since set_timing (at most `slots`).
int dg_encode_plan_stage_times(dg_encode_plan_t* P, float* ms, const char** names, int n) {
	if (!P || !P->slots || !P->runs) return 0;
	const uint32_t used = std::min(P->runs, P->slots);
	const int pairs[8][2] = {{0, 1}, {2, 3}, {3, 4}, {4, 5}, {2, 5}, {2, 6}, {2, 7}, {7, 3}};
	const uint32_t mask = timing_mask(P);
	int sel[8], ns = 0;   // the stages whose two events were recorded
	for (int k = 0; k < 8; ++k) {
		if (k >= 6 && P->algo != DG_ALGO_CORRECTING) continue;
		if (k == 5 && P->members == false && mask != kTimingAll) continue;
		if ((mask >> pairs[k][0] & 1) && (mask >> pairs[k][1] & 1)) sel[ns++] = k;
	}
	const int last = (mask >> 5) & 1 ? 5 : (P->members && !(mask >> 3 & 1) ? 6 : 3);
	double acc[8] = {};
	for (uint32_t s = 0; s < used; ++s) {
		hipEvent_t* e = &P->ev[(size_t)kTimingEvents * s];
		if (hipEventSynchronize(e[last]) != hipSuccess) return 0;
		for (int i = 0; i < ns; ++i) {
			float t = 0;
			hipEventElapsedTime(&t, e[pairs[sel[i]][0]], e[pairs[sel[i]][1]]);
			acc[i] += t;
		}
	}
	int i = 0;
	for (; i < ns && i < n; ++i) {
		if (ms) ms[i] = (float)(acc[i] / used);
		if (names) names[i] = kStageNames[sel[i]];
	}
	return i;
}

int dg_encode_plan_set_timing_mode(dg_encode_plan_t* P, int mode) {
	if (!P || (mode != DG_TIMING_ALL && mode != DG_TIMING_DOMINANT)) return DG_ERR_INVALID_ARG;
	P->timing_mode = mode;
	return DG_OK;
}

int dg_encode_plan_set_timing_every(dg_encode_plan_t* P, int every) {
	if (!P || every < 1) return DG_ERR_INVALID_ARG;
	P->every = (uint32_t)every;
	P->calls = 0;
	return DG_OK;
}

static MemSerArgs mem_ser_args(const dg_encode_plan_t* P, const uint8_t* d_ver, uint8_t* d_out, uint64_t out_cap,
                               const uint64_t* d_offsets, int32_t* d_status) {
	MemSerArgs m{};
	m.ver = d_ver;
	m.pairs = P->d_pairs.as<PairDev>();
	m.pplan = P->d_pplan.as<PairPlanDev>();
	m.chunks = P->d_chunks.as<uint2>();
	m.cmap = P->d_cmap.as<uint32_t>();
	m.seg = P->d_seg.as<uint32_t>();
	m.nseg = P->d_nseg.as<uint32_t>();
	m.mem_s = P->d_mem_s.as<uint32_t>();
	m.srec = P->d_srec.as<uint32_t>();
	m.rec = P->d_rec.as<uint32_t>();
	m.offsets = d_offsets;
	m.out = d_out;
	m.out_cap = out_cap;
	m.status = d_status;
	m.v_total = P->v_total;
	m.n_pairs = P->n;
	return m;
}

// automatic member mode over a batch the member kernel gains nothing on: one
// run in this many runs in member mode (the others as a plain plan)
constexpr uint32_t kProbeEvery = 16;

int dg_encode_plan_run(dg_encode_plan_t* P, const uint8_t* d_ref, const uint8_t* d_ver,
                       uint8_t* d_out, uint64_t out_cap, uint64_t* d_offsets, int32_t* d_status,
                       void* stream) {
	if (!P) return DG_ERR_INVALID_ARG;
	dg_context_t* ctx = P->ctx;
	if (P->n == 0) return DG_OK;
	if (!d_ref || !d_ver || !d_out || !d_offsets || !d_status)
		return set_err(ctx, DG_ERR_INVALID_ARG, "null device buffer");
	if (((uintptr_t)d_ref & 15) || ((uintptr_t)d_ver & 15))
		return set_err(ctx, DG_ERR_INVALID_ARG, "arena base pointers must be 16-byte aligned");
	hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;

	// The CRC-64/XZ of every R (even spans) and V (odd spans) shares nothing
	// with the differencing kernel until the serialiser, so it runs on a
	// forked side stream.  The differencing kernel is enqueued first so its
	// (long, latency-bound) waves are resident before the CRC waves fill the
	// issue slots they leave idle.
	const bool serial = P->serial_crc || (P->crc_wide && !P->crc_wide_beside);   // the CRC pass on the run stream, first
	hipStream_t cs = serial ? st : P->side;
	const bool timed = P->timing && P->calls++ % P->every == 0;   // this run records its events
	if (timed) P->cur = &P->ev[(size_t)kTimingEvents * (P->runs++ % P->slots)];
	// event k on stream s: every stage event, or (DG_TIMING_DOMINANT) only
	// the ones around the dominant kernel(s) (each extra timing event costs
	// the run stream a few microseconds)
	auto rec = [&](int k, hipStream_t s) -> hipError_t {
		if (!timed || !(timing_mask(P) & (1u << k))) return hipSuccess;
		return hipEventRecord(P->cur[k], s);
	};
	// member plans: the per-span combine (crc_finalize) waits on the run
	// stream for the chains.  Enqueued right after the row pass, its waves
	// queue behind the chains' full grid and slowed the routed chain of c3s
	// by 13 % (40.9 vs 36.2 ms, profiles/r05_experiments.md).
	// Automatic member mode: a batch whose every pair the last completed
	// member-mode run of this plan routed to the plain chain (shift and
	// transposition pairs, c3s / c4o) runs as a plain plan, the member kernel
	// and its serialiser skipped, except every kProbeEvery-th run, which
	// refreshes the count.  (A hint only: the output bytes do not depend on
	// it.)
	bool mem = P->members;
	if (mem && P->route_min && P->route_fb.read() >= P->n) {
		if (++P->plain_streak < kProbeEvery) mem = false;
		else P->plain_streak = 0;
	}
	++(mem ? P->member_runs : P->plain_runs);
	const bool late_fin = mem && P->crc_late_fin && !serial && !P->crc_wide && !P->fused;
	// automatic member mode: when the last completed run of this plan routed
	// more pairs to the plain chain than one round of chains fills (16 per
	// CU), the routed chain's grid waits for the CRC pass to end.  Dispatched
	// beside the pass's resident blocks, the chains land unevenly over the
	// SIMDs and the second round's last pairs trail: c3s 39.1 -> 35.7 ms
	// (profiles/r06_experiments.md).  Batches that route fewer pairs keep the
	// pass beside the member chain, whose shadow it is at c6.  (A hint only:
	// the run's bytes do not depend on it.)
	const bool chain_join = mem && !serial && !P->skip_crc &&
	                        (P->chain_join || (P->route_min && P->route_fb.read() > 16u * ctx->n_cu));
	auto crc_args = [&]() {
		CrcArgs a{};
		a.arena[0] = d_ref;
		a.arena[1] = d_ver;
		a.spans = P->d_crc_spans_r.as<CrcSpanDev>();
		a.segs = P->d_crc_segs.as<CrcSegDev>();
		a.n_segs = P->n_crc_segs;
		a.n_spans = P->n_crc_spans;
		a.tables = ctx->d_crc_tables;
		a.seg_crc = P->d_seg_crc.as<uint64_t>();
		a.out = P->d_crc.as<uint64_t>();
		a.xinv = ctx->d_xinv;
		a.kseg = ctx->kseg;
		a.prio_flag = kCrcPrioFlag && mem ? P->d_prio_flag.as<uint32_t>() : nullptr;
		return a;
	};
#ifndef DG_CRC5_ALL   // A/B: the five-bit row pass beside the onepass kernel too
#define DG_CRC5_ALL 0
#endif
	constexpr bool kCrc5All = DG_CRC5_ALL != 0;
	auto run_crc = [&]() -> int {
		HIPCHK(ctx, rec(0, cs));
		const CrcArgs a = crc_args();
		// beside the differencing: 2 blocks per CU per round of differencing
		// waves (16 per CU), so the CRC neither crowds one round out nor
		// trails a multi-round batch (C2: 4096 pairs -> 512 blocks)
		const uint32_t rounds = (P->n + 16u * ctx->n_cu - 1) / (16u * ctx->n_cu);
		if (!P->skip_crc) {
			if (P->crc_wide) HIPCHK(ctx, launch_crc_wide(a, ctx->n_cu, cs));
			// (member plans: the five-bit row pass, 3.25 KiB of LDS: the byte-table
			// pass's 16 KiB blocks find no room beside the member kernel and trail
			// it; the member waves run at a higher issue priority, so the pass
			// takes the VALU slots they leave: C3 +3 %, c6 +10 % over round 4's
			// lane-contiguous pass, profiles/r05_experiments.md)
			// (correcting plans: V's CRC runs beside the latency-bound V scan
			// with its whole grid; capped at 2 blocks per CU it took 0.97 ms
			// there instead of 0.71: C4 731 -> 813 GiB/s)
			else HIPCHK(ctx, launch_crc(a, cs, P->serial_crc || P->crc_fused ? 0u : 2u * ctx->n_cu * std::max(rounds, 1u),
			                            mem || kCrc5All ? kCrcPassRows5 : kCrcPassRows, !late_fin));
		}
		HIPCHK(ctx, rec(1, cs));
		return DG_OK;
	};
	// differencing -> COPY records + per-pair delta sizes
	auto run_diff = [&]() -> int {
		HIPCHK(ctx, rec(2, st));
		if (!mem) HIPCHK(ctx, rec(6, st));
		EncodeArgs a{};
		a.ref = d_ref;
		a.ver = d_ver;
		a.pairs = P->d_pairs.as<PairDev>();
		a.pplan = P->d_pplan.as<PairPlanDev>();
		a.n_pairs = P->n;
		a.p = (uint32_t)P->opts.p;
		a.powc = P->d_powc.as<uint64_t>();
		a.rec = P->d_rec.as<uint32_t>();
		a.n_rec = P->d_nrec.as<uint32_t>();
		a.dsize = P->d_dsize.as<uint64_t>();
		a.status = d_status;
		a.tables = P->d_tables.as<unsigned long long>();
		a.qmax = P->qmax;
		a.n_tables = P->n_tables;
		a.table_locks = P->d_locks.as<uint32_t>();
		a.table_tags = P->d_tags.as<uint32_t>();
		a.buf_cap = (uint32_t)P->opts.buf_cap;
		a.dbg = P->dbg;
		a.stats = P->algo == DG_ALGO_CORRECTING ? P->stats : nullptr;
		if (P->algo == DG_ALGO_ONEPASS) {
			if (P->fused) {
				a.out = d_out;
				a.out_cap = out_cap;
				a.offsets = d_offsets;
				a.lookback = P->d_lookback.as<unsigned long long>();
				HIPCHK(ctx, hipMemsetAsync(P->d_lookback.p, 0, 8ull * P->n, st));
			}
			if (mem) {
				SpecArgs m{};
				m.ref = d_ref;
				m.ver = d_ver;
				m.pairs = a.pairs;
				m.pplan = a.pplan;
				m.chunks = P->d_chunks.as<uint2>();
				m.mem_s = P->d_mem_s.as<uint32_t>();
				m.n_mem = P->d_nmem.as<uint32_t>();
				m.srec = P->d_srec.as<uint32_t>();
				m.csum = P->d_csum.as<uint32_t>();
				m.cmap = P->d_cmap.as<uint32_t>();
				a.csum = m.csum;
				a.cmap = m.cmap;
				a.seg = P->d_seg.as<uint32_t>();
				a.nseg = P->d_nseg.as<uint32_t>();
				a.route_min = P->route_min;
				a.mem_s = m.mem_s;
				a.n_mem = m.n_mem;
				a.srec = m.srec;
				HIPCHK(ctx, launch_members(m, P->n_chunks, ctx->n_cu, st));
				if (kCrcPrioFlag) HIPCHK(ctx, hipMemsetD32Async(P->d_prio_flag.p, 1, 1, st));   // the rows pass to priority 1
				HIPCHK(ctx, rec(6, st));
				if (P->route_min) a.route_cnt = P->d_route_cnt.as<uint32_t>();
				HIPCHK(ctx, launch_onepass(a, a.p, P->aligned16, st, chain_join ? P->ev_join : nullptr));
			} else {
				if (P->op_crc) {
					a.crc_out = P->d_crc.as<uint64_t>();
					a.crc_tab = ctx->d_crc_tables;
				}
				HIPCHK(ctx, launch_onepass(a, a.p, P->aligned16, st));
			}
		} else {
			// fresh R indexes (~0 = empty slot), then build + scan
			a.ctab = P->d_ctab.as<uint32_t>();
			a.kcls = P->d_kcls.as<uint64_t>();
			a.max_seeds = (uint32_t)P->max_seeds;
			// the LDS build writes every slot of every index; the global
			// build only fills, so its tables start empty (~0)
			a.gpairs = P->d_gpairs.as<uint32_t>();
			a.n_gpairs = P->n_gpairs;
			HIPCHK(ctx, launch_correcting_clear(a, st));
			if (P->crc_fused) {
				a.crc_out = P->d_crc.as<uint64_t>();
				a.crc_tab = ctx->d_crc_tables;
				a.crc_k32 = ctx->d_k32;
			}
			HIPCHK(ctx, launch_correcting(a, a.p, st, P->corr_lds_cap, P->qmin,
			                              timed && (timing_mask(P) & (1u << 7)) ? P->cur[7] : nullptr,
			                              (P->crc_fused || P->crc_wide_beside) && !serial ? P->ev_fork : nullptr));
		}
		if (P->algo != DG_ALGO_CORRECTING) HIPCHK(ctx, rec(7, st));
		HIPCHK(ctx, rec(3, st));
		return DG_OK;
	};
	int rc;
	if (serial) {
		if ((rc = run_crc()) != DG_OK) return rc;
		if ((rc = run_diff()) != DG_OK) return rc;
	} else if (P->crc_fused || P->crc_wide_beside) {
		// the build writes R's CRC; V's CRC forks after the build (ev_fork,
		// recorded by launch_correcting) and runs beside the V scan
		if ((rc = run_diff()) != DG_OK) return rc;
		HIPCHK(ctx, hipStreamWaitEvent(cs, P->ev_fork, 0));
		if ((rc = run_crc()) != DG_OK) return rc;
		HIPCHK(ctx, hipEventRecord(P->ev_join, cs));
	} else {
		if (kCrcPrioFlag && mem) HIPCHK(ctx, hipMemsetD32Async(P->d_prio_flag.p, 0, 1, st));
		HIPCHK(ctx, hipEventRecord(P->ev_fork, st));
		HIPCHK(ctx, hipStreamWaitEvent(cs, P->ev_fork, 0));
		if (P->crc_first || chain_join) {   // CRC waves dispatched first (A/B), or the routed chain after them
			if ((rc = run_crc()) != DG_OK) return rc;
			if (chain_join) HIPCHK(ctx, hipEventRecord(P->ev_join, cs));
			if ((rc = run_diff()) != DG_OK) return rc;
		} else {
			if ((rc = run_diff()) != DG_OK) return rc;
			if ((rc = run_crc()) != DG_OK) return rc;
		}
		HIPCHK(ctx, hipEventRecord(P->ev_join, cs));
	}
	if (P->fused) {
		// the differencing kernel placed and serialised every delta; only the
		// header CRCs remain, once the CRC stream has joined
		if (!serial) HIPCHK(ctx, hipStreamWaitEvent(st, P->ev_join, 0));
		HIPCHK(ctx, rec(4, st));
		HIPCHK(ctx, launch_crc_patch(d_out, d_offsets, P->d_crc.as<uint64_t>(), d_status, P->n, st));
		HIPCHK(ctx, rec(5, st));
		return DG_OK;
	}
	// 3. exclusive scan of sizes -> packed offsets
	HIPCHK(ctx, launch_scan(P->d_dsize.as<uint64_t>(), d_offsets, P->n, st,
	                        mem && P->route_min ? P->d_route_cnt.as<uint32_t>() : nullptr, P->route_fb.d));
	SerArgs s{};
	s.ver = d_ver;
	s.pairs = P->d_pairs.as<PairDev>();
	s.pplan = P->d_pplan.as<PairPlanDev>();
	s.rec = P->d_rec.as<uint32_t>();
	s.rec_words = P->algo == DG_ALGO_ONEPASS ? kRecWordsOnepass : kRecWordsCorrecting;
	s.n_rec = P->d_nrec.as<uint32_t>();
	s.crc = P->d_crc.as<uint64_t>();
	s.offsets = d_offsets;
	s.out = d_out;
	s.out_cap = out_cap;
	s.status = d_status;
	s.n_pairs = P->n;
	// 4. serialise.  Member plans serialise everything but the header CRCs
	//    (the CRC stream may still be running beside the chains), then join
	//    and patch them in; the others join first (below)
	HIPCHK(ctx, rec(4, st));
	if (mem) {   // the chains' segment lists, one wave per chunk
		const MemSerArgs m = mem_ser_args(P, d_ver, d_out, out_cap, d_offsets, d_status);
		HIPCHK(ctx, launch_member_serialize(m, P->n_chunks, ctx->n_cu, st));
		if (!serial) HIPCHK(ctx, hipStreamWaitEvent(st, P->ev_join, 0));   // join the CRCs
		if (late_fin && !P->skip_crc) HIPCHK(ctx, launch_crc_finalize(crc_args(), st));
		HIPCHK(ctx, launch_crc_patch(d_out, d_offsets, P->d_crc.as<uint64_t>(), d_status, P->n, st));
	} else if (P->crc_patch) {
		HIPCHK(ctx, launch_serialize_wave(s, st));
		if (!serial) HIPCHK(ctx, hipStreamWaitEvent(st, P->ev_join, 0));
		HIPCHK(ctx, launch_crc_patch(d_out, d_offsets, P->d_crc.as<uint64_t>(), d_status, P->n, st));
	} else {
		// the CRC pass (beside the differencing) has normally finished by
		// now: join it first and let the serialiser write the header CRCs,
		// one dependent launch (crc_patch_kernel, ~12 us at C2) fewer
		if (!serial) HIPCHK(ctx, hipStreamWaitEvent(st, P->ev_join, 0));
		s.crc_in = 1;
		HIPCHK(ctx, launch_serialize_wave(s, st));
	}
	HIPCHK(ctx, rec(5, st));
	return DG_OK;
}

void dg_encode_plan_destroy(dg_encode_plan_t* P) {
	if (!P) return;
	hipSetDevice(P->ctx->device);
	hipStreamSynchronize(P->ctx->stream);
	if (P->side) hipStreamSynchronize(P->side);
	for (auto& e : P->ev)
		if (e) hipEventDestroy(e);
	if (P->ev_fork) hipEventDestroy(P->ev_fork);
	if (P->ev_join) hipEventDestroy(P->ev_join);
	if (P->side) hipStreamDestroy(P->side);
	delete P;
}

}  // extern "C"

// ───────────────────────────── CRC batch (utility) ────────────────────────

extern "C" int dg_crc64_xz_batch_device(dg_context_t* ctx, const uint8_t* d_arena,
                                        const dg_span_t* spans, uint32_t n, uint64_t* d_crc,
                                        void* stream) {
	if (!ctx || (n && (!d_arena || !spans || !d_crc))) return DG_ERR_INVALID_ARG;
	if ((uintptr_t)d_arena & 15)
		return set_err(ctx, DG_ERR_INVALID_ARG, "arena base pointer must be 16-byte aligned");
	if (n == 0) return DG_OK;
	hipSetDevice(ctx->device);
	hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
	std::vector<dg_span_t> sp(spans, spans + n);
	std::vector<uint32_t> which(n, 0);
	std::vector<CrcSpanDev> sd;
	std::vector<CrcSegDev> seg;
	plan_crc_spans(sp, which, sd, seg);
	DevBuf d_sd, d_seg, d_segc;
	if (d_sd.alloc(sizeof(CrcSpanDev) * sd.size()) || d_seg.alloc(sizeof(CrcSegDev) * std::max<size_t>(seg.size(), 1)) ||
	    d_segc.alloc(8 * std::max<size_t>(seg.size(), 1)))
		return set_err(ctx, DG_ERR_NOMEM, "device allocation failed");
	HIPCHK(ctx, hipMemcpyAsync(d_sd.p, sd.data(), sizeof(CrcSpanDev) * sd.size(), hipMemcpyHostToDevice, st));
	if (!seg.empty())
		HIPCHK(ctx, hipMemcpyAsync(d_seg.p, seg.data(), sizeof(CrcSegDev) * seg.size(), hipMemcpyHostToDevice, st));
	CrcArgs a{};
	a.arena[0] = a.arena[1] = d_arena;
	a.spans = d_sd.as<CrcSpanDev>();
	a.segs = d_seg.as<CrcSegDev>();
	a.n_segs = (uint32_t)seg.size();
	a.n_spans = n;
	a.tables = ctx->d_crc_tables;
	a.seg_crc = d_segc.as<uint64_t>();
	a.out = d_crc;
	a.xinv = ctx->d_xinv;
	a.kseg = ctx->kseg;
	HIPCHK(ctx, launch_crc_wide(a, ctx->n_cu, st));   // alone on the device: the wide pass
	HIPCHK(ctx, hipStreamSynchronize(st));   // the temporaries die here
	return DG_OK;
}

// ───────────────────────────── decode plan ────────────────────────────────

struct dg_decode_plan {
	dg_context_t* ctx = nullptr;
	uint32_t n = 0;
	int ignore_hash = 0;
	DevBuf d_desc;   // the decode kernel computes and checks both CRCs itself
	// byte extents the streams touch in each arena (run rejects overlaps),
	// and the intervals themselves, sorted and merged per arena (the exact
	// check when the extents of the arenas overlap)
	uint64_t ref_end = 0, delta_end = 0, out_end = 0;
	std::vector<std::pair<uint64_t, uint64_t>> iv_ref, iv_delta, iv_out;
	bool timing = false;
	std::vector<hipEvent_t> ev;
	uint32_t slots = 0, runs = 0, ev_sets = 0;   // ring length; event sets allocated
	uint32_t every = 1, calls = 0;   // events on every `every`-th run (dg_*_plan_set_timing_every)
};

namespace {
constexpr int kDecEvents = 2;   // decode_kernel's start and end
}  // namespace

extern "C" {

int dg_decode_plan_create(dg_context_t* ctx, const dg_decode_desc_t* descs, uint32_t n,
                          int ignore_hash, dg_decode_plan_t** out) {
	if (!ctx || !out || (n && !descs)) return DG_ERR_INVALID_ARG;
	*out = nullptr;
	hipSetDevice(ctx->device);
	auto* P = new (std::nothrow) dg_decode_plan_t();
	if (!P) return DG_ERR_NOMEM;
	P->ctx = ctx;
	P->n = n;
	P->ignore_hash = ignore_hash;
	for (uint32_t i = 0; i < n; ++i)
		if (descs[i].ref_len >= (1ull << 32) || descs[i].out_cap >= (1ull << 32) + (1ull << 31)) {
			delete P;
			return set_err(ctx, DG_ERR_TOO_LARGE, "stream %u exceeds the u32 format", i);
		}
	for (uint32_t i = 0; i < n; ++i) {
		P->ref_end = std::max(P->ref_end, descs[i].ref_off + descs[i].ref_len);
		P->delta_end = std::max(P->delta_end, descs[i].delta_off + descs[i].delta_len);
		P->out_end = std::max(P->out_end, descs[i].out_off + descs[i].out_cap);
		if (descs[i].ref_len) P->iv_ref.push_back({descs[i].ref_off, descs[i].ref_off + descs[i].ref_len});
		if (descs[i].delta_len) P->iv_delta.push_back({descs[i].delta_off, descs[i].delta_off + descs[i].delta_len});
		if (descs[i].out_cap) P->iv_out.push_back({descs[i].out_off, descs[i].out_off + descs[i].out_cap});
	}
	for (auto* iv : {&P->iv_ref, &P->iv_delta, &P->iv_out}) {
		std::sort(iv->begin(), iv->end());
		size_t k = 0;
		for (const auto& x : *iv) {
			if (k && x.first <= (*iv)[k - 1].second) (*iv)[k - 1].second = std::max((*iv)[k - 1].second, x.second);
			else (*iv)[k++] = x;
		}
		iv->resize(k);
	}
	const size_t nn = std::max<size_t>(n, 1);
	if (P->d_desc.alloc(sizeof(dg_decode_desc_t) * nn)) {
		delete P;
		return set_err(ctx, DG_ERR_NOMEM, "device allocation failed");
	}
	hipStream_t st = ctx->stream;
	hipError_t e = hipSuccess;
	if (n) e = hipMemcpyAsync(P->d_desc.p, descs, sizeof(dg_decode_desc_t) * n, hipMemcpyHostToDevice, st);
	if (e == hipSuccess) e = hipStreamSynchronize(st);
	if (e != hipSuccess) {
		dg_decode_plan_destroy(P);
		return set_err(ctx, DG_ERR_HIP, "decode plan setup failed: %s", hipGetErrorString(e));
	}
	*out = P;
	return DG_OK;
}

int dg_decode_plan_set_timing(dg_decode_plan_t* P, int slots) {
	if (!P || slots < 0) return DG_ERR_INVALID_ARG;
	hipSetDevice(P->ctx->device);
	if ((uint32_t)slots > P->ev_sets) {
		for (auto& e : P->ev) hipEventDestroy(e);
		P->ev.assign((size_t)kDecEvents * slots, nullptr);
		P->ev_sets = P->slots = 0;
		for (auto& e : P->ev)
			// timing only: no system-scope fence when the event is recorded
			// (a cache writeback + invalidate per event slowed the timed
			// steps by 15 %: C2 0.335 -> 0.391 ms with two events per step)
			if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
				e = nullptr;
				P->timing = false;
				return set_err(P->ctx, DG_ERR_HIP, "hipEventCreate failed");
			}
		P->ev_sets = (uint32_t)slots;
	}
	P->slots = (uint32_t)slots;   // the ring: exactly the last `slots` runs
	P->timing = slots > 0;
	P->runs = P->calls = 0;
	return DG_OK;
}

// one stage, "decode": the kernel parses, applies and checks both CRCs
int dg_decode_plan_stage_times(dg_decode_plan_t* P, float* ms, const char** names, int n) {
	if (!P || !P->slots || !P->runs || n < 1) return 0;
	const uint32_t used = std::min(P->runs, P->slots);
	double acc = 0;
	for (uint32_t s = 0; s < used; ++s) {
		hipEvent_t* e = &P->ev[(size_t)kDecEvents * s];
		if (hipEventSynchronize(e[1]) != hipSuccess) return 0;
		float t = 0;
		hipEventElapsedTime(&t, e[0], e[1]);
		acc += t;
	}
	if (ms) ms[0] = (float)(acc / used);
	if (names) names[0] = "decode";
	return 1;
}

int dg_decode_plan_set_timing_every(dg_decode_plan_t* P, int every) {
	if (!P || every < 1) return DG_ERR_INVALID_ARG;
	P->every = (uint32_t)every;
	P->calls = 0;
	return DG_OK;
}

int dg_decode_plan_run(dg_decode_plan_t* P, const uint8_t* d_ref, const uint8_t* d_delta,
                       uint8_t* d_out, uint64_t* d_out_len, int32_t* d_status, void* stream) {
	if (!P) return DG_ERR_INVALID_ARG;
	dg_context_t* ctx = P->ctx;
	if (P->n == 0) return DG_OK;
	if (!d_ref || !d_delta || !d_out || !d_out_len || !d_status)
		return set_err(ctx, DG_ERR_INVALID_ARG, "null device buffer");
	if (((uintptr_t)d_ref & 15) || ((uintptr_t)d_out & 15))
		return set_err(ctx, DG_ERR_INVALID_ARG, "arena base pointers must be 16-byte aligned");
	{
		// the kernel writes the output image before it reads R for the source
		// CRC, and reads the delta while it writes: an output arena that
		// overlaps the reference or delta bytes of the batch is rejected
		auto overlap = [](const void* a, uint64_t na, const void* b, uint64_t nb) {
			const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
			return na && nb && x < y + nb && y < x + na;
		};
		// the exact test (only when the extents overlap): the merged output
		// intervals against the merged reference / delta intervals, one sweep
		auto named_overlap = [&](const void* b, const std::vector<std::pair<uint64_t, uint64_t>>& ivb) {
			const uintptr_t xo = (uintptr_t)d_out, xb = (uintptr_t)b;
			size_t i = 0, j = 0;
			while (i < P->iv_out.size() && j < ivb.size()) {
				const uintptr_t a0 = xo + P->iv_out[i].first, a1 = xo + P->iv_out[i].second;
				const uintptr_t b0 = xb + ivb[j].first, b1 = xb + ivb[j].second;
				if (a0 < b1 && b0 < a1) return true;
				if (a1 <= b1) ++i;
				else ++j;
			}
			return false;
		};
		if ((overlap(d_out, P->out_end, d_ref, P->ref_end) && named_overlap(d_ref, P->iv_ref)) ||
		    (overlap(d_out, P->out_end, d_delta, P->delta_end) && named_overlap(d_delta, P->iv_delta)))
			return set_err(ctx, DG_ERR_INVALID_ARG, "the output bytes overlap the reference or delta bytes");
	}
	hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
	hipEvent_t* ev = nullptr;
	if (P->timing && P->calls++ % P->every == 0) ev = &P->ev[(size_t)kDecEvents * (P->runs++ % P->slots)];
	const bool check = !P->ignore_hash;
	// parse + apply (encoding.c:111-178, apply.c:229-284), then the CRC-64/XZ
	// of R and of the output, checked against the header in the same kernel
	// (main.c:341-356, :376-385); --ignore-hash skips the CRCs.  Two events
	// around the one launch (each event costs the stream ~3.5 us: the three
	// empty stages the round-4 layout also recorded cost C5 ~8 %)
	if (ev) HIPCHK(ctx, hipEventRecord(ev[0], st));
	DecodeArgs a{};
	{
		static const uint32_t dbg = [] {
			const char* e = ab_env("DG_DEBUG_BITS");
			return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
		}();
		a.dbg = dbg;
	}
	a.ref = d_ref;
	a.delta = d_delta;
	a.descs = P->d_desc.as<dg_decode_desc_dev>();
	a.n = P->n;
	a.out = d_out;
	a.out_len = d_out_len;
	a.status = d_status;
	a.tables = ctx->d_crc_tables;
	a.crc_check = check ? 1u : 0u;
	HIPCHK(ctx, launch_decode(a, st));
	if (ev) HIPCHK(ctx, hipEventRecord(ev[1], st));
	return DG_OK;
}

void dg_decode_plan_destroy(dg_decode_plan_t* P) {
	if (!P) return;
	hipSetDevice(P->ctx->device);
	hipStreamSynchronize(P->ctx->stream);
	for (auto& e : P->ev)
		if (e) hipEventDestroy(e);
	delete P;
}

}  // extern "C"
