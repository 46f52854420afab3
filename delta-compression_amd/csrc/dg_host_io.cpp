// dg_host_io.cpp — host-memory entry points of libdeltagpu.so.
//
// These wrap the device-resident batch path (dg_encode_plan_*, the decode
// kernels) with pinned staging and H2D/D2H copies, i.e. the end-to-end form
// of the reference's CLI chain (src/c/main.c:249-292 encode, :335-385 decode).
// The arithmetic always runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/delta_gpu.h"
#include "dg_device.h"

namespace {

struct Dev {
	void* p = nullptr;
	~Dev() { reset(); }
	void reset() { if (p) hipFree(p); p = nullptr; }
	bool alloc(size_t n) { return hipMalloc(&p, n ? n : 16) == hipSuccess; }
	template <class T> T* as() { return static_cast<T*>(p); }
};

struct Pinned {
	void* p = nullptr;
	~Pinned() { reset(); }
	void reset() { if (p) hipHostFree(p); p = nullptr; }
	bool alloc(size_t n) { return hipHostMalloc(&p, n ? n : 16, hipHostMallocDefault) == hipSuccess; }
	template <class T> T* as() { return static_cast<T*>(p); }
};

uint64_t up16(uint64_t x) { return (x + 15) & ~15ull; }

uint32_t rd_u32be(const uint8_t* p) {
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

}  // namespace

extern "C" {

int dg_encode_batch(dg_context_t* ctx, dg_algorithm_t algo, const uint8_t* const* r,
                    const size_t* r_len, const uint8_t* const* v, const size_t* v_len,
                    uint32_t n, const dg_diff_options_t* opts, dg_buffer_t* outs,
                    int32_t* status) {
	if (!ctx || (n && (!r || !r_len || !v || !v_len || !outs))) return DG_ERR_INVALID_ARG;
	for (uint32_t i = 0; i < n; ++i) outs[i].data = nullptr, outs[i].len = 0;
	if (n == 0) return DG_OK;
	if (opts && ((opts->flags >> DG_OPT_INPLACE) & 1)) {
		// main.c:279-292 with --inplace: the standard encode on the device,
		// then delta_make_inplace on the host
		dg_diff_options_t o = *opts;
		o.flags &= ~(1ull << DG_OPT_INPLACE);
		const int policy = ((opts->flags >> DG_OPT_POLICY_CONSTANT) & 1) ? DG_POLICY_CONSTANT : DG_POLICY_LOCALMIN;
		std::vector<int32_t> st(n, 0);
		int rc = dg_encode_batch(ctx, algo, r, r_len, v, v_len, n, &o, outs, st.data());
		if (rc) return rc;
		int first_bad = DG_OK;
		for (uint32_t i = 0; i < n; ++i) {
			if (st[i] == DG_OK && outs[i].data) {
				dg_buffer_t ip{nullptr, 0};
				st[i] = dg_make_inplace(r[i], r_len[i], outs[i].data, outs[i].len, policy, &ip, nullptr);
				free(outs[i].data);
				outs[i] = ip;
			}
			if (status) status[i] = st[i];
			if (st[i] && !first_bad) first_bad = st[i];
		}
		return status ? DG_OK : first_bad;
	}
	hipStream_t st = (hipStream_t)dg_context_stream(ctx);

	std::vector<dg_pair_t> pairs(n);
	uint64_t rt = 0, vt = 0;
	for (uint32_t i = 0; i < n; ++i) {
		pairs[i] = dg_pair_t{rt, r_len[i], vt, v_len[i]};
		rt += up16(r_len[i]);
		vt += up16(v_len[i]);
	}
	dg_encode_plan_t* plan = nullptr;
	int rc = dg_encode_plan_create(ctx, algo, pairs.data(), n, opts, &plan);
	if (rc) return rc;
	const uint64_t bound = dg_encode_plan_output_bound(plan);

	const bool verbose = opts && ((opts->flags >> DG_OPT_VERBOSE) & 1);
	Pinned h_in, h_off, h_st;
	Dev d_ref, d_ver, d_out, d_off, d_st, d_stats;
	std::vector<uint64_t> stats;
	if (verbose) {   // the reference's diagnostics (dg_encode_plan_set_stats)
		if (!d_stats.alloc(64ull * n) || hipMemsetAsync(d_stats.p, 0, 64ull * n, st) != hipSuccess) {
			dg_encode_plan_destroy(plan);
			return DG_ERR_NOMEM;
		}
		dg_encode_plan_set_stats(plan, d_stats.as<uint64_t>());
		stats.assign(8ull * n, 0);
	}
	rc = DG_ERR_NOMEM;
	if (!h_in.alloc(rt + vt) || !h_off.alloc(8ull * (n + 1)) || !h_st.alloc(4ull * n) ||
	    !d_ref.alloc(rt) || !d_ver.alloc(vt) || !d_out.alloc(bound) ||
	    !d_off.alloc(8ull * (n + 1)) || !d_st.alloc(4ull * n)) {
		dg_encode_plan_destroy(plan);
		return rc;
	}
	uint8_t* hr = h_in.as<uint8_t>();
	uint8_t* hv = hr + rt;
	for (uint32_t i = 0; i < n; ++i) {
		if (r_len[i]) memcpy(hr + pairs[i].r_off, r[i], r_len[i]);
		if (v_len[i]) memcpy(hv + pairs[i].v_off, v[i], v_len[i]);
	}
	rc = DG_ERR_HIP;
	if (hipMemcpyAsync(d_ref.p, hr, rt, hipMemcpyHostToDevice, st) != hipSuccess ||
	    hipMemcpyAsync(d_ver.p, hv, vt, hipMemcpyHostToDevice, st) != hipSuccess) {
		dg_encode_plan_destroy(plan);
		return rc;
	}
	rc = dg_encode_plan_run(plan, d_ref.as<uint8_t>(), d_ver.as<uint8_t>(), d_out.as<uint8_t>(),
	                        bound, d_off.as<uint64_t>(), d_st.as<int32_t>(), st);
	if (rc) { dg_encode_plan_destroy(plan); return rc; }
	if (hipMemcpyAsync(h_off.p, d_off.p, 8ull * (n + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
	    hipMemcpyAsync(h_st.p, d_st.p, 4ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
	    hipStreamSynchronize(st) != hipSuccess) {
		dg_encode_plan_destroy(plan);
		return DG_ERR_HIP;
	}
	const uint64_t* off = h_off.as<uint64_t>();
	const uint64_t total = off[n];
	Pinned h_out;
	if (!h_out.alloc(total) ||
	    hipMemcpyAsync(h_out.p, d_out.p, total, hipMemcpyDeviceToHost, st) != hipSuccess ||
	    (verbose && hipMemcpyAsync(stats.data(), d_stats.p, 64ull * n, hipMemcpyDeviceToHost, st) != hipSuccess) ||
	    hipStreamSynchronize(st) != hipSuccess) {
		dg_encode_plan_destroy(plan);
		return DG_ERR_HIP;
	}
	if (verbose)
		for (uint32_t i = 0; i < n; ++i)
			if (h_st.as<int32_t>()[i] == DG_OK)
				dg::print_verbose(plan, i, stats.data() + 8ull * i, h_out.as<uint8_t>() + off[i], off[i + 1] - off[i]);
	dg_encode_plan_destroy(plan);
	int first_bad = DG_OK;
	for (uint32_t i = 0; i < n; ++i) {
		const int32_t s = h_st.as<int32_t>()[i];
		if (status) status[i] = s;
		if (s != DG_OK) {
			if (!first_bad) first_bad = s;
			continue;
		}
		const uint64_t len = off[i + 1] - off[i];
		outs[i].data = (uint8_t*)malloc(len ? len : 1);
		if (!outs[i].data) return DG_ERR_NOMEM;
		memcpy(outs[i].data, h_out.as<uint8_t>() + off[i], len);
		outs[i].len = len;
	}
	return status ? DG_OK : first_bad;
}

// ── pipelined host-to-host encode ──────────────────────────────────────
//
// Two slots, each with its own stream, device buffers, plan and pinned
// staging, kept in the context between calls.  Per chunk (consecutive pairs,
// about chunk_bytes of input): [stage the inputs into pinned memory when the
// caller's arenas are pageable] -> H2D -> dg_encode_plan_run -> D2H of the
// offsets and status -> (when the slot is next needed) D2H of exactly the
// chunk's delta bytes.  Chunk i+1's copies run while chunk i encodes.
}  // extern "C"

namespace {

bool host_pinned(const void* p) {
	if (!p) return false;
	hipPointerAttribute_t at{};
	if (hipPointerGetAttributes(&at, p) != hipSuccess) {
		(void)hipGetLastError();   // pageable memory reports an error: clear it
		return false;
	}
	return at.type == hipMemoryTypeHost;
}

struct IoSlot {
	hipStream_t s = nullptr;
	hipEvent_t ev = nullptr;
	dg_encode_plan_t* plan = nullptr;
	std::vector<dg_pair_t> key;   // the plan's layout (chunk-relative)
	dg_algorithm_t key_algo = DG_ALGO_ONEPASS;
	dg_diff_options_t key_opts{};
	uint64_t key_limits = ~0ull;  // dg::ctx_limits_gen when the plan was made
	Dev d_ref, d_ver, d_out, d_off, d_st;
	uint64_t cap_ref = 0, cap_ver = 0, cap_out = 0, cap_doff = 0, cap_dst = 0;
	Pinned h_in, h_out, h_off, h_st;
	uint64_t cap_hin = 0, cap_hout = 0, cap_hoff = 0, cap_hst = 0;
	// the chunk in flight
	bool pending = false;
	uint32_t p0 = 0, p1 = 0;      // its pairs
	uint64_t bound = 0;
	~IoSlot() {
		if (plan) dg_encode_plan_destroy(plan);
		if (ev) hipEventDestroy(ev);
		if (s) hipStreamDestroy(s);
	}
};

struct IoState {
	IoSlot slot[2];
};

void io_release(void* p) { delete static_cast<IoState*>(p); }

// memcpy for pageable <-> pinned staging, split over a few host threads (one
// thread copies ~10 GB/s, PCIe moves ~50): pieces of >= 8 MiB
void par_memcpy(void* dst, const void* src, uint64_t n) {
	const uint64_t kPiece = 8ull << 20;
	unsigned t = std::thread::hardware_concurrency();
	t = std::max(1u, std::min(8u, t));
	const uint64_t parts = std::min<uint64_t>(t, (n + kPiece - 1) / kPiece);
	if (parts <= 1) {
		memcpy(dst, src, n);
		return;
	}
	std::vector<std::thread> th;
	const uint64_t per = (n + parts - 1) / parts;
	for (uint64_t k = 1; k < parts; ++k) {
		const uint64_t a = k * per, b = std::min(n, a + per);
		if (a < b) th.emplace_back([=] { memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, b - a); });
	}
	memcpy(dst, src, std::min(n, per));
	for (auto& x : th) x.join();
}

// pageable -> pinned staging of a chunk's pairs at their packed (16-byte
// aligned) offsets `rel`, the pairs split over a few host threads
void stage_pairs(uint8_t* dr, uint8_t* dv, const uint8_t* h_ref, const uint8_t* h_ver, const dg_pair_t* src,
                 const dg_pair_t* rel, uint32_t m) {
	auto run = [&](uint32_t a, uint32_t b) {
		for (uint32_t i = a; i < b; ++i) {
			memcpy(dr + rel[i].r_off, h_ref + src[i].r_off, src[i].r_len);
			memcpy(dv + rel[i].v_off, h_ver + src[i].v_off, src[i].v_len);
		}
	};
	uint64_t bytes = 0;
	for (uint32_t i = 0; i < m; ++i) bytes += src[i].r_len + src[i].v_len;
	unsigned t = std::thread::hardware_concurrency();
	t = std::max(1u, std::min(8u, t));
	const uint64_t parts = std::min<uint64_t>({t, m, std::max<uint64_t>(1, bytes >> 23)});
	if (parts <= 1) {
		run(0, m);
		return;
	}
	std::vector<std::thread> th;
	const uint32_t per = (uint32_t)((m + parts - 1) / parts);
	for (uint64_t k = 1; k < parts; ++k) {
		const uint32_t a = (uint32_t)(k * per), b = std::min<uint32_t>(m, a + per);
		if (a < b) th.emplace_back([=] { run(a, b); });
	}
	run(0, std::min<uint32_t>(m, per));
	for (auto& x : th) x.join();
}

template <class B>
bool grow(B& b, uint64_t& cap, uint64_t need) {
	if (need <= cap && b.p) return true;
	b.reset();
	cap = 0;
	if (!b.alloc(need)) return false;
	cap = need;
	return true;
}

}  // namespace

extern "C" {

int dg_host_alloc(dg_context_t* ctx, uint64_t bytes, void** out) {
	if (!ctx || !out) return DG_ERR_INVALID_ARG;
	*out = nullptr;
	return hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault) == hipSuccess ? DG_OK : DG_ERR_NOMEM;
}

void dg_host_free(void* p) {
	if (p) hipHostFree(p);
}

int dg_encode_pipelined_multi(dg_context_t* const* ctxs, uint32_t n_ctx, dg_algorithm_t algo, const uint8_t* h_ref,
                              const uint8_t* h_ver, const dg_pair_t* pairs, uint32_t n, const dg_diff_options_t* opts,
                              uint64_t chunk_bytes, uint8_t* h_out, uint64_t out_cap, uint64_t* out_offsets,
                              int32_t* status) {
	if (!ctxs || n_ctx == 0 || !out_offsets || (n && (!pairs || !h_ref || !h_ver || !h_out))) return DG_ERR_INVALID_ARG;
	for (uint32_t d = 0; d < n_ctx; ++d)
		if (!ctxs[d]) return DG_ERR_INVALID_ARG;
	if (n_ctx == 1 || n < 2)
		return dg_encode_pipelined(ctxs[0], algo, h_ref, h_ver, pairs, n, opts, chunk_bytes, h_out, out_cap,
		                           out_offsets, status);
	dg_diff_options_t o;
	if (opts) o = *opts; else dg_diff_options_default(&o);
	const uint64_t p = o.p ? o.p : DG_SEED_LEN;
	// contiguous ranges, balanced by input bytes (shard.py balanced_ranges)
	uint64_t total = 0;
	for (uint32_t i = 0; i < n; ++i) total += pairs[i].r_len + pairs[i].v_len;
	const uint32_t D = std::min<uint32_t>(n_ctx, n);
	std::vector<uint32_t> cut{0};
	{
		uint64_t acc = 0;
		uint32_t i = 0;
		for (uint32_t d = 1; d < D; ++d) {
			const double target = (double)total * d / D;
			while (i < n && (double)(acc + pairs[i].r_len + pairs[i].v_len) <= target) acc += pairs[i].r_len + pairs[i].v_len, ++i;
			cut.push_back(i);
		}
		cut.push_back(n);
	}
	// each range into its own buffer (its output bound, as dg_encode_plan's)
	struct Range {
		uint32_t lo = 0, hi = 0;
		std::vector<uint8_t> out;
		std::vector<uint64_t> off;
		std::vector<int32_t> st;
		int rc = DG_OK;
	};
	std::vector<Range> R(D);
	for (uint32_t d = 0; d < D; ++d) {
		Range& r = R[d];
		r.lo = cut[d];
		r.hi = cut[d + 1];
		uint64_t bound = 0;
		for (uint32_t i = r.lo; i < r.hi; ++i) {
			const uint64_t vl = pairs[i].v_len;
			bound += algo == DG_ALGO_CORRECTING ? 57 + vl + 22 * (vl / p) : 35 + vl + (vl / p) * (p < 22 ? 22 - p : 0);
		}
		try {
			r.out.resize(std::max<uint64_t>(bound, 1));
			r.off.resize((size_t)(r.hi - r.lo) + 1);
			r.st.resize(std::max<uint32_t>(r.hi - r.lo, 1));
		} catch (...) {
			return DG_ERR_NOMEM;
		}
	}
	{
		// one host thread per context (dg_encode_pipelined makes the thread's
		// current device the context's); a thread that cannot be started runs
		// its range on the calling thread after the others are joined
		auto work = [&](uint32_t d) {
			Range& r = R[d];
			if (r.hi == r.lo) {
				r.off[0] = 0;
				return;
			}
			r.rc = dg_encode_pipelined(ctxs[d], algo, h_ref, h_ver, pairs + r.lo, r.hi - r.lo, opts, chunk_bytes,
			                           r.out.data(), r.out.size(), r.off.data(), r.st.data());
		};
		std::vector<std::thread> th;
		uint32_t started = 0;
		try {
			th.reserve(D);
			for (; started < D; ++started) th.emplace_back(work, started);
		} catch (...) {   // std::system_error / bad_alloc: no exception crosses the C ABI
		}
		for (auto& t : th) t.join();
		for (uint32_t d = started; d < D; ++d) work(d);
	}
	// pack in pair order, as dg_encode_pipelined does: once a pair's delta
	// does not fit, it and every later pair report DG_ERR_CAPACITY (a pair
	// the device failed keeps its own status) at the bytes written so far
	uint64_t pos = 0;
	int rc_all = DG_OK;
	int rc_hard = DG_OK;   // the first range that failed as a whole (HIP, NOMEM, ...)
	bool full = false;
	out_offsets[0] = 0;
	for (uint32_t d = 0; d < D; ++d) {
		Range& r = R[d];
		const uint32_t m = r.hi - r.lo;
		if (r.rc != DG_OK && r.rc != DG_ERR_CAPACITY) {   // the range failed as a whole
			for (uint32_t k = 0; k < m; ++k) {
				out_offsets[r.lo + k + 1] = pos;
				if (status) status[r.lo + k] = r.rc;
			}
			if (rc_hard == DG_OK) rc_hard = r.rc;
			continue;
		}
		uint32_t fit = 0;   // this range's leading pairs that fit
		if (!full) {
			while (fit < m && pos + r.off[fit + 1] <= out_cap) ++fit;
			if (fit < m) full = true;
		}
		par_memcpy(h_out + pos, r.out.data(), r.off[fit]);
		for (uint32_t k = 0; k < m; ++k) {
			if (k < fit) {
				out_offsets[r.lo + k + 1] = pos + r.off[k + 1];
				if (status) status[r.lo + k] = r.st[k];
				if (!status && r.st[k] != DG_OK && rc_all == DG_OK) rc_all = r.st[k];
			} else {
				out_offsets[r.lo + k + 1] = pos + r.off[fit];
				if (status) status[r.lo + k] = r.st[k] != DG_OK ? r.st[k] : DG_ERR_CAPACITY;
			}
		}
		pos += r.off[fit];
	}
	// as the one-device path: a hard failure wins over capacity and over the
	// per-pair status array
	if (rc_hard != DG_OK) return rc_hard;
	if (full) return DG_ERR_CAPACITY;
	return status ? DG_OK : rc_all;
}

namespace {
// restores the calling thread's current device on every return
struct DeviceGuard {
	int dev = -1;
	DeviceGuard() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
	~DeviceGuard() { if (dev >= 0) (void)hipSetDevice(dev); }
};
}  // namespace

int dg_encode_pipelined(dg_context_t* ctx, dg_algorithm_t algo, const uint8_t* h_ref, const uint8_t* h_ver,
                        const dg_pair_t* pairs, uint32_t n, const dg_diff_options_t* opts,
                        uint64_t chunk_bytes, uint8_t* h_out, uint64_t out_cap, uint64_t* out_offsets,
                        int32_t* status) {
	if (!ctx || !out_offsets || (n && (!pairs || !h_ref || !h_ver || !h_out))) return DG_ERR_INVALID_ARG;
	out_offsets[0] = 0;
	if (n == 0) return DG_OK;
	if (opts && ((opts->flags >> DG_OPT_INPLACE) & 1)) return DG_ERR_UNSUPPORTED;   // host step: dg_encode_batch
	// the calling thread's current device becomes the context's before any
	// stream or event of it is made (a new host thread starts on device 0),
	// and is the caller's again on return
	DeviceGuard keep_device;
	if (hipSetDevice(dg::ctx_device(ctx)) != hipSuccess) return DG_ERR_HIP;
	dg_diff_options_t o;
	if (opts) o = *opts; else dg_diff_options_default(&o);
	if (chunk_bytes == 0) chunk_bytes = 256ull << 20;
	void** io = dg::ctx_io(ctx, io_release);
	if (!*io) *io = new (std::nothrow) IoState();
	if (!*io) return DG_ERR_NOMEM;
	IoState& S = *static_cast<IoState*>(*io);
	for (IoSlot& sl : S.slot) {
		if (!sl.s && hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess) return DG_ERR_HIP;
		if (!sl.ev && hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) != hipSuccess) return DG_ERR_HIP;
		sl.pending = false;
	}
	const bool in_pinned = host_pinned(h_ref) && host_pinned(h_ver);
	const bool out_pinned = host_pinned(h_out);

	// chunks of consecutive pairs
	std::vector<uint32_t> cuts{0};
	{
		uint64_t acc = 0;
		for (uint32_t i = 0; i < n; ++i) {
			const uint64_t b = pairs[i].r_len + pairs[i].v_len;
			if (acc && acc + b > chunk_bytes) {
				cuts.push_back(i);
				acc = 0;
			}
			acc += b;
		}
		cuts.push_back(n);
	}
	uint64_t out_pos = 0;
	int rc_all = DG_OK;
	bool full = false;
	std::vector<dg_pair_t> rel;

	// the slot's finished chunk: its delta bytes to h_out, offsets and status
	auto drain = [&](IoSlot& sl) -> int {
		if (!sl.pending) return DG_OK;
		sl.pending = false;
		if (hipEventSynchronize(sl.ev) != hipSuccess) return DG_ERR_HIP;
		const uint32_t m = sl.p1 - sl.p0;
		const uint64_t* off = sl.h_off.as<uint64_t>();
		const int32_t* st = sl.h_st.as<int32_t>();
		const uint64_t total = off[m];
		if (full || out_pos + total > out_cap) {
			// this chunk and every later one do not fit: their offsets stay
			// at the bytes written so far, their status says why
			full = true;
			for (uint32_t k = 0; k < m; ++k) {
				out_offsets[sl.p0 + k + 1] = out_pos;
				// a pair the device already failed keeps its own status
				if (status) status[sl.p0 + k] = st[k] != DG_OK ? st[k] : DG_ERR_CAPACITY;
			}
			return DG_OK;
		}
		if (total) {
			if (out_pinned) {
				if (hipMemcpyAsync(h_out + out_pos, sl.d_out.p, total, hipMemcpyDeviceToHost, sl.s) != hipSuccess)
					return DG_ERR_HIP;
			} else {
				if (!grow(sl.h_out, sl.cap_hout, total)) return DG_ERR_NOMEM;
				if (hipMemcpyAsync(sl.h_out.p, sl.d_out.p, total, hipMemcpyDeviceToHost, sl.s) != hipSuccess ||
				    hipStreamSynchronize(sl.s) != hipSuccess)
					return DG_ERR_HIP;
				par_memcpy(h_out + out_pos, sl.h_out.p, total);
			}
		}
		for (uint32_t k = 0; k < m; ++k) {
			out_offsets[sl.p0 + k + 1] = out_pos + off[k + 1];
			if (status) status[sl.p0 + k] = st[k];
			if (st[k] && !rc_all) rc_all = st[k];
		}
		out_pos += total;
		return DG_OK;
	};

	int rc = DG_OK;
	const uint32_t n_chunks = (uint32_t)cuts.size() - 1;
	for (uint32_t c = 0; c < n_chunks && rc == DG_OK; ++c) {
		IoSlot& sl = S.slot[c & 1];
		if ((rc = drain(sl)) != DG_OK) break;
		// the slot's previous D2H (issued on its stream) orders before this
		// chunk's H2D; its pinned staging is reused only after that drain
		if (hipStreamSynchronize(sl.s) != hipSuccess) { rc = DG_ERR_HIP; break; }
		const uint32_t p0 = cuts[c], p1 = cuts[c + 1], m = p1 - p0;
		uint64_t r_lo = ~0ull, r_hi = 0, v_lo = ~0ull, v_hi = 0;
		for (uint32_t i = p0; i < p1; ++i) {
			r_lo = std::min<uint64_t>(r_lo, pairs[i].r_off);
			r_hi = std::max<uint64_t>(r_hi, pairs[i].r_off + pairs[i].r_len);
			v_lo = std::min<uint64_t>(v_lo, pairs[i].v_off);
			v_hi = std::max<uint64_t>(v_hi, pairs[i].v_off + pairs[i].v_len);
		}
		// pinned arenas go up in one copy per stream and keep the arena's
		// 16-byte phase (aligned layouts stay aligned); pageable arenas are
		// staged pair by pair anyway, so the staging copy packs every stream
		// at a 16-byte offset, which selects the LDS-window kernels
		r_lo &= ~15ull;
		v_lo &= ~15ull;
		uint64_t rn = r_hi - r_lo, vn = v_hi - v_lo;
		rel.resize(m);
		if (in_pinned) {
			for (uint32_t i = p0; i < p1; ++i)
				rel[i - p0] = dg_pair_t{pairs[i].r_off - r_lo, pairs[i].r_len, pairs[i].v_off - v_lo, pairs[i].v_len};
		} else {
			uint64_t ro = 0, vo = 0;
			for (uint32_t i = p0; i < p1; ++i) {
				rel[i - p0] = dg_pair_t{ro, pairs[i].r_len, vo, pairs[i].v_len};
				ro += (pairs[i].r_len + 15) & ~15ull;
				vo += (pairs[i].v_len + 15) & ~15ull;
			}
			rn = ro;
			vn = vo;
		}
		const uint64_t lim = dg::ctx_limits_gen(ctx);
		const bool same = sl.plan && sl.key_algo == algo && !memcmp(&sl.key_opts, &o, sizeof o) &&
		                  sl.key_limits == lim && sl.key.size() == rel.size() &&
		                  !memcmp(sl.key.data(), rel.data(), m * sizeof(dg_pair_t));
		if (!same) {
			if (sl.plan) dg_encode_plan_destroy(sl.plan);
			sl.plan = nullptr;
			if ((rc = dg_encode_plan_create(ctx, algo, rel.data(), m, &o, &sl.plan)) != DG_OK) break;
			sl.key = rel;
			sl.key_algo = algo;
			sl.key_opts = o;
			sl.key_limits = lim;
			sl.bound = dg_encode_plan_output_bound(sl.plan);
		}
		if (!grow(sl.d_ref, sl.cap_ref, rn) || !grow(sl.d_ver, sl.cap_ver, vn) ||
		    !grow(sl.d_out, sl.cap_out, sl.bound) || !grow(sl.d_off, sl.cap_doff, 8ull * (m + 1)) ||
		    !grow(sl.d_st, sl.cap_dst, 4ull * m) || !grow(sl.h_off, sl.cap_hoff, 8ull * (m + 1)) ||
		    !grow(sl.h_st, sl.cap_hst, 4ull * m)) {
			rc = DG_ERR_NOMEM;
			break;
		}
		const uint8_t* src_r = h_ref + r_lo;
		const uint8_t* src_v = h_ver + v_lo;
		if (!in_pinned) {   // stage: every pair's streams at 16-byte offsets
			if (!grow(sl.h_in, sl.cap_hin, rn + vn)) { rc = DG_ERR_NOMEM; break; }
			stage_pairs(sl.h_in.as<uint8_t>(), sl.h_in.as<uint8_t>() + rn, h_ref, h_ver, pairs + p0, rel.data(), m);
			src_r = sl.h_in.as<uint8_t>();
			src_v = src_r + rn;
		}
		if (hipMemcpyAsync(sl.d_ref.p, src_r, rn, hipMemcpyHostToDevice, sl.s) != hipSuccess ||
		    hipMemcpyAsync(sl.d_ver.p, src_v, vn, hipMemcpyHostToDevice, sl.s) != hipSuccess) {
			rc = DG_ERR_HIP;
			break;
		}
		if ((rc = dg_encode_plan_run(sl.plan, sl.d_ref.as<uint8_t>(), sl.d_ver.as<uint8_t>(), sl.d_out.as<uint8_t>(),
		                             sl.bound, sl.d_off.as<uint64_t>(), sl.d_st.as<int32_t>(), sl.s)) != DG_OK)
			break;
		if (hipMemcpyAsync(sl.h_off.p, sl.d_off.p, 8ull * (m + 1), hipMemcpyDeviceToHost, sl.s) != hipSuccess ||
		    hipMemcpyAsync(sl.h_st.p, sl.d_st.p, 4ull * m, hipMemcpyDeviceToHost, sl.s) != hipSuccess ||
		    hipEventRecord(sl.ev, sl.s) != hipSuccess) {
			rc = DG_ERR_HIP;
			break;
		}
		sl.pending = true;
		sl.p0 = p0;
		sl.p1 = p1;
		// the other slot's chunk (one behind) goes out while this one encodes
		if ((rc = drain(S.slot[(c + 1) & 1])) != DG_OK) break;
	}
	// in chunk order: the slot holding the older chunk first
	if (rc == DG_OK && n_chunks >= 2) rc = drain(S.slot[n_chunks & 1]);
	if (rc == DG_OK) rc = drain(S.slot[(n_chunks - 1) & 1]);
	for (IoSlot& sl : S.slot) {
		hipStreamSynchronize(sl.s);
		sl.pending = false;
	}
	if (rc != DG_OK) return rc;
	if (full) return DG_ERR_CAPACITY;
	return status ? DG_OK : rc_all;
}

int dg_encode(dg_context_t* ctx, dg_algorithm_t algo, const uint8_t* r, size_t r_len,
              const uint8_t* v, size_t v_len, const dg_diff_options_t* opts, dg_buffer_t* out) {
	if (!out) return DG_ERR_INVALID_ARG;
	int32_t st = 0;
	int rc = dg_encode_batch(ctx, algo, &r, &r_len, &v, &v_len, 1, opts, out, &st);
	return rc ? rc : st;
}

int dg_diff(dg_context_t* ctx, dg_algorithm_t algo, const uint8_t* r, size_t r_len, const uint8_t* v,
            size_t v_len, const dg_diff_options_t* opts, dg_commands_t* out) {
	// delta_diff + delta_place_commands (delta.h:280-284, apply.c:136-164):
	// the device encodes, the host lists the commands of the standard delta,
	// which holds them 1:1 in algorithm order (encoding.c:69-83)
	if (!out || !opts) return DG_ERR_INVALID_ARG;
	out->data = nullptr;
	out->len = 0;
	out->storage = nullptr;
	dg_diff_options_t o = *opts;
	o.flags &= ~(1ull << DG_OPT_INPLACE);
	dg_buffer_t d{nullptr, 0};
	int rc = dg_encode(ctx, algo, r, r_len, v, v_len, &o, &d);
	if (rc == DG_OK) rc = dg_delta_decode(d.data, d.len, out, nullptr);
	dg_buffer_free(&d);
	return rc;
}

int dg_crc64_xz_batch_device(dg_context_t* ctx, const uint8_t* d_arena, const dg_span_t* spans,
                             uint32_t n, uint64_t* d_crc, void* stream);

int dg_crc64_xz(dg_context_t* ctx, const uint8_t* data, size_t len, uint8_t out[DG_CRC_SIZE]) {
	if (!ctx || (len && !data) || !out) return DG_ERR_INVALID_ARG;
	hipStream_t st = (hipStream_t)dg_context_stream(ctx);
	Dev d, c;
	Pinned h;
	if (!d.alloc(len) || !c.alloc(8) || !h.alloc(8)) return DG_ERR_NOMEM;
	if (len && hipMemcpyAsync(d.p, data, len, hipMemcpyHostToDevice, st) != hipSuccess) return DG_ERR_HIP;
	dg_span_t sp{0, len};
	int rc = dg_crc64_xz_batch_device(ctx, d.as<uint8_t>(), &sp, 1, c.as<uint64_t>(), st);
	if (rc) return rc;
	if (hipMemcpyAsync(h.p, c.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
	    hipStreamSynchronize(st) != hipSuccess)
		return DG_ERR_HIP;
	const uint64_t v = *h.as<uint64_t>();
	for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(v >> (56 - 8 * i));
	return DG_OK;
}

int dg_synth_edit_pairs_device(dg_context_t* ctx, uint8_t* d_ref, uint8_t* d_ver, uint32_t n,
                               uint64_t pair_len, uint64_t seed_base, uint64_t n_edits,
                               void* stream) {
	if (!ctx || (n && (!d_ref || !d_ver))) return DG_ERR_INVALID_ARG;
	hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)dg_context_stream(ctx);
	return dg::launch_synth(d_ref, d_ver, n, pair_len, seed_base, n_edits, st) == hipSuccess
	           ? DG_OK
	           : DG_ERR_HIP;
}

namespace {

uint64_t splitmix_at_host(uint64_t seed, uint64_t k) {
	uint64_t z = seed + k * 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

// One pair's block layout: sizes U[mean/2, 3 mean/2] (gen_transpositions.py
// _gen_sizes), then a permutation moving round(nb * pct / 100) blocks
// (_gen_perm: choose k distinct slots, shuffle their contents).
void transpose_layout(uint64_t seed, uint32_t nb, uint32_t mean, uint32_t pct,
                      std::vector<uint32_t>& sz, std::vector<uint32_t>& perm) {
	const uint64_t s = seed ^ 0x5851F42D4C957F2DULL;
	uint64_t k = 1;
	const uint32_t lo = mean / 2 ? mean / 2 : 1, hi = mean * 3 / 2;
	sz.resize(nb);
	for (uint32_t i = 0; i < nb; ++i) sz[i] = lo + (uint32_t)(splitmix_at_host(s, k++) % (hi - lo + 1));
	perm.resize(nb);
	std::vector<uint32_t> idx(nb), val(nb);
	for (uint32_t i = 0; i < nb; ++i) perm[i] = idx[i] = i;
	// Python's round() is round-half-to-even (gen_transpositions.py:143)
	const uint64_t kq = (uint64_t)nb * pct / 100, kr = (uint64_t)nb * pct % 100;
	const uint32_t kk = (uint32_t)(kq + (kr > 50 || (kr == 50 && (kq & 1))));
	if (kk < 2) return;
	for (uint32_t j = 0; j < kk; ++j) {
		const uint32_t t = j + (uint32_t)(splitmix_at_host(s, k++) % (nb - j));
		std::swap(idx[j], idx[t]);
	}
	for (uint32_t j = 0; j < kk; ++j) val[j] = idx[j];
	for (uint32_t j = kk - 1; j > 0; --j) {
		const uint32_t t = (uint32_t)(splitmix_at_host(s, k++) % (j + 1));
		std::swap(val[j], val[t]);
	}
	for (uint32_t j = 0; j < kk; ++j) perm[idx[j]] = val[j];
}

}  // namespace

int dg_synth_transpose_pairs_device(dg_context_t* ctx, uint64_t seed_base, uint32_t n,
                                    uint64_t target_len, uint32_t pct, dg_pair_t* pairs,
                                    uint64_t* ref_bytes, uint64_t* ver_bytes, uint8_t* d_ref,
                                    uint8_t* d_ver, void* stream) {
	if (!ctx || (n && !pairs) || pct > 100 || target_len < 8) return DG_ERR_INVALID_ARG;
	std::vector<dg::SynthSpan> spans(n);
	std::vector<dg::SynthCopy> cmds;
	std::vector<uint32_t> sz, perm, off;
	uint64_t rt = 0, vt = 0;
	for (uint32_t i = 0; i < n; ++i) {
		const uint32_t nb = 8 + (i % 57);
		transpose_layout(seed_base + i, nb, (uint32_t)(target_len / nb), pct, sz, perm);
		off.assign(nb + 1, 0);
		for (uint32_t b = 0; b < nb; ++b) off[b + 1] = off[b] + sz[b];
		const uint64_t total = off[nb];
		pairs[i] = dg_pair_t{rt, total, vt, total};
		spans[i] = dg::SynthSpan{rt, total, seed_base + i};
		uint64_t o = 0;
		for (uint32_t b = 0; b < nb; ++b) {
			cmds.push_back(dg::SynthCopy{vt + o, rt + off[perm[b]], sz[perm[b]]});
			o += sz[perm[b]];
		}
		rt += up16(total);
		vt += up16(total);
	}
	if (ref_bytes) *ref_bytes = rt;
	if (ver_bytes) *ver_bytes = vt;
	if (!d_ref) return DG_OK;
	if (!d_ver) return DG_ERR_INVALID_ARG;
	hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)dg_context_stream(ctx);
	Dev d_spans, d_cmds;
	if (!d_spans.alloc(sizeof(dg::SynthSpan) * n) || !d_cmds.alloc(sizeof(dg::SynthCopy) * cmds.size()))
		return DG_ERR_NOMEM;
	if (hipMemcpyAsync(d_spans.p, spans.data(), sizeof(dg::SynthSpan) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
	    hipMemcpyAsync(d_cmds.p, cmds.data(), sizeof(dg::SynthCopy) * cmds.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
	    dg::launch_synth_transpose(d_ref, d_ver, d_spans.as<dg::SynthSpan>(), n, d_cmds.as<dg::SynthCopy>(),
	                               (uint32_t)cmds.size(), st) != hipSuccess ||
	    hipStreamSynchronize(st) != hipSuccess)
		return DG_ERR_HIP;
	return DG_OK;
}

int dg_synth_shift_pairs_device(dg_context_t* ctx, uint64_t seed_base, uint32_t n, uint64_t pair_len,
                                uint64_t n_edits, uint32_t indel_pct, dg_pair_t* pairs, uint64_t* ref_bytes,
                                uint64_t* ver_bytes, uint8_t* d_ref, uint8_t* d_ver, void* stream) {
	if (!ctx || (n && !pairs) || indel_pct > 100 || pair_len >= (1ull << 31)) return DG_ERR_INVALID_ARG;
	// |V| of every pair (the edit kinds and sizes, as the device kernel and
	// or_synth_shift draw them), over a few host threads
	std::vector<uint64_t> vlen(n);
	{
		auto run = [&](uint32_t a, uint32_t b) {
			for (uint32_t i = a; i < b; ++i) {
				const uint64_t m = std::min<uint64_t>(n_edits, pair_len);
				int64_t d = 0;
				if (m) {
					const uint64_t s = (seed_base + i) ^ 0x2545F4914F6CDD1DULL, S = pair_len / m;
					for (uint64_t e = 0; e < m; ++e) {
						const uint64_t lo = e * S, hi = e + 1 == m ? pair_len : (e + 1) * S;
						const uint64_t h1 = splitmix_at_host(s, 3 * e + 1), h2 = splitmix_at_host(s, 3 * e + 2);
						const uint64_t pos = lo + h1 % (hi - lo), u = h2 % 100, k = 1 + (h2 >> 32) % 8;
						if (2 * u < indel_pct) d += (int64_t)k;
						else if (u < indel_pct) d -= (int64_t)std::min<uint64_t>(k, hi - pos);
					}
				}
				vlen[i] = (uint64_t)((int64_t)pair_len + d);
			}
		};
		unsigned t = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
		t = std::min<unsigned>(t, std::max(1u, n));
		std::vector<std::thread> th;
		for (unsigned k = 1; k < t; ++k) th.emplace_back(run, (uint32_t)((uint64_t)n * k / t), (uint32_t)((uint64_t)n * (k + 1) / t));
		run(0, (uint32_t)(n / t));
		for (auto& x : th) x.join();
	}
	std::vector<dg::SynthSpan> spans(n);
	std::vector<uint64_t> voff(n);
	uint64_t rt = 0, vt = 0;
	for (uint32_t i = 0; i < n; ++i) {
		pairs[i] = dg_pair_t{rt, pair_len, vt, vlen[i]};
		spans[i] = dg::SynthSpan{rt, pair_len, seed_base + i};
		voff[i] = vt;
		rt += up16(pair_len);
		vt += up16(vlen[i]);
	}
	if (ref_bytes) *ref_bytes = rt;
	if (ver_bytes) *ver_bytes = vt;
	if (!d_ref) return DG_OK;
	if (!d_ver) return DG_ERR_INVALID_ARG;
	hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)dg_context_stream(ctx);
	Dev d_spans, d_voff;
	if (!d_spans.alloc(sizeof(dg::SynthSpan) * std::max<uint32_t>(n, 1)) || !d_voff.alloc(8ull * std::max<uint32_t>(n, 1)))
		return DG_ERR_NOMEM;
	if (n && (hipMemcpyAsync(d_spans.p, spans.data(), sizeof(dg::SynthSpan) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
	          hipMemcpyAsync(d_voff.p, voff.data(), 8ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
	          dg::launch_synth_shift(d_ref, d_ver, d_spans.as<dg::SynthSpan>(), d_voff.as<uint64_t>(), n, n_edits,
	                                 indel_pct, st) != hipSuccess))
		return DG_ERR_HIP;
	return hipStreamSynchronize(st) == hipSuccess ? DG_OK : DG_ERR_HIP;
}

}  // extern "C"

// ───────────────────────────── decode ─────────────────────────────────────

extern "C" int dg_decode_batch_device(dg_context_t* ctx, const uint8_t* d_ref,
                                      const uint8_t* d_delta, const dg_decode_desc_t* descs,
                                      uint32_t n, int ignore_hash, uint8_t* d_out,
                                      uint64_t* d_out_len, int32_t* d_status, void* stream) {
	// one-shot plan: create, run, wait, release
	if (!ctx || (n && (!d_ref || !d_delta || !descs || !d_out || !d_out_len || !d_status)))
		return DG_ERR_INVALID_ARG;
	if (n == 0) return DG_OK;
	dg_decode_plan_t* plan = nullptr;
	int rc = dg_decode_plan_create(ctx, descs, n, ignore_hash, &plan);
	if (rc) return rc;
	hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)dg_context_stream(ctx);
	rc = dg_decode_plan_run(plan, d_ref, d_delta, d_out, d_out_len, d_status, st);
	if (rc == DG_OK && hipStreamSynchronize(st) != hipSuccess) rc = DG_ERR_HIP;
	dg_decode_plan_destroy(plan);
	return rc;
}

extern "C" int dg_decode(dg_context_t* ctx, const uint8_t* r, size_t r_len, const uint8_t* delta,
                         size_t delta_len, int ignore_hash, dg_buffer_t* out) {
	if (!ctx || !out || (r_len && !r) || (delta_len && !delta)) return DG_ERR_INVALID_ARG;
	out->data = nullptr;
	out->len = 0;
	if (delta_len < DG_HEADER_SIZE || memcmp(delta, "DLT\x03", 4) != 0) return DG_ERR_MALFORMED;
	const uint64_t vsize = rd_u32be(delta + 5);
	const uint64_t cap = std::max<uint64_t>(vsize, r_len);
	hipStream_t st = (hipStream_t)dg_context_stream(ctx);
	Dev d_r, d_d, d_o, d_len, d_st;
	Pinned h_o;
	if (!d_r.alloc(r_len) || !d_d.alloc(delta_len) || !d_o.alloc(cap) || !d_len.alloc(8) ||
	    !d_st.alloc(4) || !h_o.alloc(vsize))
		return DG_ERR_NOMEM;
	if ((r_len && hipMemcpyAsync(d_r.p, r, r_len, hipMemcpyHostToDevice, st) != hipSuccess) ||
	    hipMemcpyAsync(d_d.p, delta, delta_len, hipMemcpyHostToDevice, st) != hipSuccess)
		return DG_ERR_HIP;
	dg_decode_desc_t desc{0, r_len, 0, delta_len, 0, cap};
	int rc = dg_decode_batch_device(ctx, d_r.as<uint8_t>(), d_d.as<uint8_t>(), &desc, 1, ignore_hash,
	                                d_o.as<uint8_t>(), d_len.as<uint64_t>(), d_st.as<int32_t>(), st);
	if (rc) return rc;
	int32_t s = 0;
	if (hipMemcpy(&s, d_st.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return DG_ERR_HIP;
	// a failed output CRC still hands back the output: the reference writes
	// the file before its post-check fails (main.c:374-383)
	if (s && s != DG_ERR_DST_CRC) return s;
	if (vsize && (hipMemcpyAsync(h_o.p, d_o.p, vsize, hipMemcpyDeviceToHost, st) != hipSuccess ||
	              hipStreamSynchronize(st) != hipSuccess))
		return DG_ERR_HIP;
	out->data = (uint8_t*)malloc(vsize ? vsize : 1);
	if (!out->data) return DG_ERR_NOMEM;
	if (vsize) memcpy(out->data, h_o.p, vsize);
	out->len = vsize;
	return s;
}
