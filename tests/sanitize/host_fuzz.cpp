// host_fuzz.cpp — drives the library's host-only code (dg_format.cpp,
// dg_inplace.cpp) under AddressSanitizer + UBSan (tests/test_host_sanitize.py).
//
// Input: a corpus file of records [u32 r_len][R][u32 d_len][delta] (little
// endian), written by the test from reference-minted golden deltas and
// oracle-encoded pairs.  For every delta, and for truncations and seeded byte
// mutations of it, the driver runs dg_delta_info, dg_delta_decode (checked
// against dg_delta_info's counts), dg_encode_commands on the decoded list
// (decoding the result must give the same list back) and dg_make_inplace
// under both cycle policies (its output must decode, and apply to the bytes
// the standard delta reconstructs).  Any memory error, UB or failed check
// aborts with a non-zero status.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/delta_gpu.h"

namespace {

int fails = 0;
#define CHECK(c)                                                      \
	do {                                                              \
		if (!(c)) {                                                   \
			fprintf(stderr, "check failed at line %d: %s\n", __LINE__, #c); \
			++fails;                                                  \
		}                                                             \
	} while (0)

uint64_t rng = 0x9E3779B97F4A7C15ull;
uint64_t next() {
	rng ^= rng << 13;
	rng ^= rng >> 7;
	rng ^= rng << 17;
	return rng;
}

bool same(const dg_commands_t& a, const dg_commands_t& b) {
	if (a.len != b.len) return false;
	for (size_t i = 0; i < a.len; ++i) {
		const dg_placed_command_t &x = a.data[i], &y = b.data[i];
		if (x.tag != y.tag || x.src != y.src || x.dst != y.dst || x.length != y.length) return false;
		if (x.tag == DG_CMD_ADD && x.length && memcmp(x.data, y.data, x.length) != 0) return false;
	}
	return true;
}

// Apply placed commands into `out` (version_size bytes) from `r`, as
// delta_apply_placed (apply.c:229-250) or, in place, apply.c:253-284.
bool apply(const uint8_t* r, size_t r_len, const dg_commands_t& c, uint64_t vsize, bool inplace,
           std::vector<uint8_t>& out) {
	const uint64_t cap = inplace ? (vsize > r_len ? vsize : r_len) : vsize;
	out.assign(cap, 0);
	if (inplace && r_len) memcpy(out.data(), r, r_len);
	for (size_t i = 0; i < c.len; ++i) {
		const dg_placed_command_t& x = c.data[i];
		if (x.dst > cap || x.length > cap - x.dst) return false;
		if (x.tag == DG_CMD_COPY) {
			if (inplace) {
				if (x.src > cap || x.length > cap - x.src) return false;
				memmove(out.data() + x.dst, out.data() + x.src, x.length);
			} else {
				if (x.src > r_len || x.length > r_len - x.src) return false;
				if (x.length) memcpy(out.data() + x.dst, r + x.src, x.length);
			}
		} else if (x.length) {
			memcpy(out.data() + x.dst, x.data, x.length);
		}
	}
	out.resize(vsize);
	return true;
}

// Sequential destinations covering [0, vsize): the only layout for which the
// in-place conversion (which re-places by destination order, inplace.c:
// 296-330) must reproduce the standard application byte for byte.
bool canonical(const dg_commands_t& c, uint64_t vsize) {
	std::vector<std::pair<uint64_t, uint64_t>> iv;
	for (size_t i = 0; i < c.len; ++i) iv.push_back({c.data[i].dst, c.data[i].length});
	std::stable_sort(iv.begin(), iv.end(),
	                 [](const std::pair<uint64_t, uint64_t>& a, const std::pair<uint64_t, uint64_t>& b) {
		                 return a.first < b.first;
	                 });
	uint64_t at = 0;
	for (auto& x : iv) {
		if (x.first != at) return false;
		at += x.second;
	}
	return at == vsize;
}

void one(const uint8_t* r, size_t r_len, const uint8_t* d, size_t d_len, bool deep) {
	dg_delta_info_t info;
	const int rc_info = dg_delta_info(d, d_len, &info);
	dg_commands_t c{};
	dg_delta_info_t hdr;
	const int rc = dg_delta_decode(d, d_len, &c, &hdr);
	CHECK(rc == rc_info);
	if (rc != DG_OK) {
		CHECK(c.data == nullptr && c.len == 0);
		return;
	}
	CHECK(c.len == info.num_commands && hdr.inplace == info.inplace && hdr.version_size == info.version_size &&
	      !memcmp(hdr.src_crc, info.src_crc, DG_CRC_SIZE) && !memcmp(hdr.dst_crc, info.dst_crc, DG_CRC_SIZE) &&
	      hdr.num_copies == info.num_copies && hdr.add_bytes == info.add_bytes);
	uint64_t copies = 0, cb = 0, ab = 0;
	for (size_t i = 0; i < c.len; ++i) {
		if (c.data[i].tag == DG_CMD_COPY) {
			++copies;
			cb += c.data[i].length;
		} else {
			ab += c.data[i].length;
		}
	}
	CHECK(copies == info.num_copies && cb == info.copy_bytes && ab == info.add_bytes);

	dg_buffer_t e{};
	int rc2 = dg_encode_commands(c.data, c.len, hdr.inplace, hdr.version_size, hdr.src_crc, hdr.dst_crc, &e);
	CHECK(rc2 == DG_OK);
	if (rc2 == DG_OK) {
		dg_commands_t c2{};
		CHECK(dg_delta_decode(e.data, e.len, &c2, nullptr) == DG_OK && same(c, c2));
		dg_commands_free(&c2);
		dg_buffer_free(&e);
	}

	if (deep && !hdr.inplace) {   // the standard delta reconstructs V; so must both in-place forms
		std::vector<uint8_t> v, w;
		const bool ok = canonical(c, hdr.version_size) && apply(r, r_len, c, hdr.version_size, false, v);
		for (int pol = 0; pol < 2; ++pol) {
			dg_buffer_t ip{};
			dg_inplace_stats_t st;
			const int rc3 = dg_make_inplace(r, r_len, d, d_len, pol, &ip, &st);
			if (rc3 != DG_OK) {
				CHECK(rc3 == DG_ERR_MALFORMED);
				continue;
			}
			dg_commands_t ci{};
			CHECK(dg_delta_decode(ip.data, ip.len, &ci, nullptr) == DG_OK);
			if (ok) CHECK(apply(r, r_len, ci, hdr.version_size, true, w) && w == v);
			dg_commands_free(&ci);
			dg_buffer_free(&ip);
		}
	} else if (hdr.inplace) {
		dg_buffer_t ip{};
		CHECK(dg_make_inplace(r, r_len, d, d_len, 0, &ip, nullptr) == DG_OK && ip.len == d_len &&
		      memcmp(ip.data, d, d_len) == 0);
		dg_buffer_free(&ip);
	}
	dg_commands_free(&c);
}

}  // namespace

int main(int argc, char** argv) {
	if (argc != 2) {
		fprintf(stderr, "usage: %s corpus\n", argv[0]);
		return 2;
	}
	FILE* f = fopen(argv[1], "rb");
	if (!f) return 2;
	std::vector<uint8_t> all;
	uint8_t buf[1 << 16];
	size_t k;
	while ((k = fread(buf, 1, sizeof buf, f)) > 0) all.insert(all.end(), buf, buf + k);
	fclose(f);

	size_t pos = 0, n = 0, variants = 0;
	while (pos + 4 <= all.size()) {
		uint32_t rl, dl;
		memcpy(&rl, &all[pos], 4);
		pos += 4;
		if (all.size() - pos < rl + 4ull) return 2;
		std::vector<uint8_t> r(all.begin() + pos, all.begin() + pos + rl);   // own allocations: ASan sees their bounds
		pos += rl;
		memcpy(&dl, &all[pos], 4);
		pos += 4;
		if (all.size() - pos < dl) return 2;
		std::vector<uint8_t> d(all.begin() + pos, all.begin() + pos + dl);
		pos += dl;
		++n;

		one(r.data(), r.size(), d.data(), d.size(), true);
		// every truncation of a short delta, a sample of a long one
		const size_t step = d.size() <= 2048 ? 1 : d.size() / 512;
		for (size_t t = 0; t < d.size(); t += step, ++variants) {
			std::vector<uint8_t> tr(d.begin(), d.begin() + t);
			one(r.data(), r.size(), tr.data(), tr.size(), t % 7 == 0);
		}
		// seeded mutations: a byte, a length field, a command tag
		for (int m = 0; m < 256 && d.size() > DG_HEADER_SIZE; ++m, ++variants) {
			std::vector<uint8_t> mu(d);
			const size_t at = DG_HEADER_SIZE + next() % (mu.size() - DG_HEADER_SIZE);
			mu[at] = (uint8_t)next();
			if (m & 1) mu[at] = (uint8_t)(mu[at] & 3);
			one(r.data(), r.size(), mu.data(), mu.size(), true);
		}
	}
	if (pos != all.size()) return 2;
	printf("deltas %zu variants %zu failures %d\n", n, variants, fails);
	return fails ? 1 : 0;
}
