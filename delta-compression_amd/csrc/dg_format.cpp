// dg_format.cpp — the DLT\x03 container on the host: header summary, command
// lists in and out (src/c/encoding.c:39-178, apply.c:98-115).
//
// Pure host code with no HIP dependency, so it is also compiled alone under
// AddressSanitizer/UBSan with dg_inplace.cpp by tests/test_host_sanitize.py.
// The device path never comes here: the GPU serializer writes the same bytes
// from its own records (dg_serialize_wave.h) and the decode kernel parses
// them itself; these entry points are for callers that work at the
// command-list level (HOWTO.md:426-464: delta_diff -> delta_place_commands ->
// delta_encode, delta_decode -> delta_apply_placed).
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../../include/delta_gpu.h"

namespace {

uint32_t be32(const uint8_t* p) {
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint8_t* put32(uint8_t* p, uint64_t x) {
	p[0] = (uint8_t)(x >> 24);
	p[1] = (uint8_t)(x >> 16);
	p[2] = (uint8_t)(x >> 8);
	p[3] = (uint8_t)x;
	return p + 4;
}

// One walk of the command stream (encoding.c:134-175).  `each` sees every
// command; returns DG_ERR_MALFORMED on a truncated or unknown command.  A
// stream without the END byte ends at the buffer end, as in the reference.
template <class F>
int walk(const uint8_t* d, size_t len, F&& each) {
	size_t pos = DG_HEADER_SIZE;
	while (pos < len) {
		const uint8_t t = d[pos++];
		if (t == 0) return DG_OK;
		if (t == 1) {
			if (len - pos < 12) return DG_ERR_MALFORMED;
			each(DG_CMD_COPY, (uint64_t)be32(d + pos), (uint64_t)be32(d + pos + 4),
			     (uint64_t)be32(d + pos + 8), (size_t)0);
			pos += 12;
		} else if (t == 2) {
			if (len - pos < 8) return DG_ERR_MALFORMED;
			const uint64_t dst = be32(d + pos), l = be32(d + pos + 4);
			pos += 8;
			if (len - pos < l) return DG_ERR_MALFORMED;
			each(DG_CMD_ADD, (uint64_t)0, dst, l, pos);
			pos += l;
		} else {
			return DG_ERR_MALFORMED;
		}
	}
	return DG_OK;
}

int header(const uint8_t* d, size_t len, dg_delta_info_t* info) {
	memset(info, 0, sizeof *info);
	if (len < DG_HEADER_SIZE || memcmp(d, "DLT\x03", 4) != 0) return DG_ERR_MALFORMED;
	info->inplace = d[4] & 1;
	info->version_size = be32(d + 5);
	memcpy(info->src_crc, d + 9, DG_CRC_SIZE);
	memcpy(info->dst_crc, d + 17, DG_CRC_SIZE);
	return DG_OK;
}

}  // namespace

extern "C" {

void dg_buffer_free(dg_buffer_t* b) {
	if (!b) return;
	free(b->data);
	b->data = nullptr;
	b->len = 0;
}

int dg_delta_info(const uint8_t* d, size_t len, dg_delta_info_t* info) {
	// the walk of encoding.c:111-178, summarised as delta_placed_summary
	// (apply.c:98-115) for main.c:402-425
	if (!info || (len && !d)) return DG_ERR_INVALID_ARG;
	int rc = header(d, len, info);
	if (rc) return rc;
	return walk(d, len, [&](uint32_t tag, uint64_t, uint64_t, uint64_t l, size_t) {
		info->num_commands++;
		if (tag == DG_CMD_COPY) {
			info->num_copies++;
			info->copy_bytes += l;
		} else {
			info->num_adds++;
			info->add_bytes += l;
		}
	});
}

int dg_delta_decode(const uint8_t* d, size_t len, dg_commands_t* out, dg_delta_info_t* hdr) {
	// delta_decode (encoding.c:111-178): the placed commands in stream order.
	// One allocation holds the command array followed by a copy of the delta;
	// ADD data point into that copy.
	if (!out || (len && !d)) return DG_ERR_INVALID_ARG;
	out->data = nullptr;
	out->len = 0;
	out->storage = nullptr;
	dg_delta_info_t info;
	int rc = dg_delta_info(d, len, &info);
	if (rc) return rc;
	const size_t n = (size_t)info.num_commands;
	const size_t head = n * sizeof(dg_placed_command_t);
	uint8_t* blk = (uint8_t*)malloc(head + len + 1);
	if (!blk) return DG_ERR_NOMEM;
	dg_placed_command_t* cmds = (dg_placed_command_t*)blk;
	uint8_t* copy = blk + head;
	memcpy(copy, d, len);
	size_t i = 0;
	walk(copy, len, [&](uint32_t tag, uint64_t src, uint64_t dst, uint64_t l, size_t at) {
		cmds[i++] = dg_placed_command_t{tag, src, dst, l, tag == DG_CMD_ADD ? copy + at : nullptr};
	});
	out->data = cmds;
	out->len = n;
	out->storage = blk;
	if (hdr) *hdr = info;
	return DG_OK;
}

void dg_commands_free(dg_commands_t* c) {
	if (!c) return;
	free(c->storage);
	c->data = nullptr;
	c->len = 0;
	c->storage = nullptr;
}

int dg_encode_commands(const dg_placed_command_t* cmds, size_t n, int inplace,
                       uint64_t version_size, const uint8_t src_crc[DG_CRC_SIZE],
                       const uint8_t dst_crc[DG_CRC_SIZE], dg_buffer_t* out) {
	// delta_encode (encoding.c:39-90).  The format's u32 fields cannot hold
	// offsets or lengths of 4 GiB or more: such commands are rejected rather
	// than truncated.
	if (!out || (n && !cmds) || !src_crc || !dst_crc) return DG_ERR_INVALID_ARG;
	out->data = nullptr;
	out->len = 0;
	if (version_size > UINT32_MAX) return DG_ERR_INVALID_ARG;
	uint64_t total = DG_HEADER_SIZE + 1;
	for (size_t i = 0; i < n; ++i) {
		const dg_placed_command_t& c = cmds[i];
		if (c.dst > UINT32_MAX || c.length > UINT32_MAX) return DG_ERR_INVALID_ARG;
		if (c.tag == DG_CMD_COPY) {
			if (c.src > UINT32_MAX) return DG_ERR_INVALID_ARG;
			total += 13;
		} else if (c.tag == DG_CMD_ADD) {
			if (c.length && !c.data) return DG_ERR_INVALID_ARG;
			total += 9 + c.length;
		} else {
			return DG_ERR_INVALID_ARG;
		}
	}
	uint8_t* buf = (uint8_t*)malloc(total);
	if (!buf) return DG_ERR_NOMEM;
	uint8_t* p = buf;
	memcpy(p, "DLT\x03", 4);
	p[4] = inplace ? 1 : 0;
	p = put32(p + 5, version_size);
	memcpy(p, src_crc, DG_CRC_SIZE);
	memcpy(p + DG_CRC_SIZE, dst_crc, DG_CRC_SIZE);
	p += 2 * DG_CRC_SIZE;
	for (size_t i = 0; i < n; ++i) {
		const dg_placed_command_t& c = cmds[i];
		if (c.tag == DG_CMD_COPY) {
			*p++ = 1;
			p = put32(put32(put32(p, c.src), c.dst), c.length);
		} else {
			*p++ = 2;
			p = put32(put32(p, c.dst), c.length);
			if (c.length) memcpy(p, c.data, c.length);
			p += c.length;
		}
	}
	*p++ = 0;
	out->data = buf;
	out->len = (size_t)(p - buf);
	return DG_OK;
}

}  // extern "C"
