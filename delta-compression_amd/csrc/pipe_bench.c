/* pipe_bench.c — host-to-host throughput of dg_encode_pipelined, in C over
 * the C ABI only (no torch, no HIP headers): n C2-shaped pairs (64 KiB,
 * 1 % substitutions, the bench's splitmix64 generator) in host arenas, the
 * deltas back in a host buffer.  VERDICT r1 item 6.
 *
 * usage: pipe_bench [pairs=16384] [pair_bytes=65536] [chunk_pairs=2048] [reps=5] [pinned=1]
 * prints one JSON line: GiB/s = sum(|R|+|V|) / wall time of one call (median
 * of reps), plus the delta bytes and a spot check of deltas against dg_encode.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "delta_gpu.h"

static uint64_t mix_at(uint64_t seed, uint64_t k) {   /* oracle or_splitmix64_at */
	uint64_t z = seed + k * 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

static void synth_pair(uint64_t seed, uint8_t *r, uint8_t *v, uint64_t len, uint64_t n_edits) {
	for (uint64_t i = 0; i < len; i += 8) {
		const uint64_t w = mix_at(seed, i / 8 + 1);
		for (uint64_t j = 0; j < 8 && i + j < len; ++j) r[i + j] = (uint8_t)(w >> (8 * j));
	}
	memcpy(v, r, len);
	const uint64_t s = seed ^ 0xD1B54A32D192ED03ULL;
	for (uint64_t e = 0; e < n_edits; ++e) v[mix_at(s, 2 * e + 1) % len] = (uint8_t)mix_at(s, 2 * e + 2);
}

static double now(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9 * t.tv_nsec;
}

static int cmp_d(const void *a, const void *b) {
	const double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
	const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 16384;
	const uint64_t L = argc > 2 ? strtoull(argv[2], 0, 0) : 65536;
	const uint32_t chunk_pairs = argc > 3 ? (uint32_t)strtoul(argv[3], 0, 0) : 2048;
	const int reps = argc > 4 ? atoi(argv[4]) : 5;
	const int pinned = argc > 5 ? atoi(argv[5]) : 1;
	dg_context_t *ctx;
	int rc = dg_context_create(-1, &ctx);
	if (rc) { fprintf(stderr, "context: %s\n", dg_status_string(rc)); return 1; }
	const uint64_t arena = (uint64_t)n * L, out_cap = arena + (uint64_t)n * 4096;
	uint8_t *R = 0, *V = 0, *out = 0;
	if (pinned) {
		if (dg_host_alloc(ctx, arena, (void **)&R) || dg_host_alloc(ctx, arena, (void **)&V) ||
		    dg_host_alloc(ctx, out_cap, (void **)&out)) { fprintf(stderr, "pinned alloc failed\n"); return 1; }
	} else {
		R = malloc(arena); V = malloc(arena); out = malloc(out_cap);
		if (!R || !V || !out) { fprintf(stderr, "alloc failed\n"); return 1; }
	}
	dg_pair_t *pairs = malloc(sizeof *pairs * n);
	uint64_t *offs = malloc(8ull * (n + 1));
	int32_t *st = malloc(4ull * n);
	for (uint32_t i = 0; i < n; ++i) {
		synth_pair(0xC2000000ULL + i, R + (uint64_t)i * L, V + (uint64_t)i * L, L, (uint64_t)(0.01 * L + 0.5));
		pairs[i] = (dg_pair_t){(uint64_t)i * L, L, (uint64_t)i * L, L};
	}
	dg_diff_options_t o;
	dg_diff_options_default(&o);
	o.q = 1;   /* C2: --table-size 1 */
	const uint64_t chunk_bytes = 2ull * L * chunk_pairs;
	double t[64];
	const int nr = reps < 1 ? 1 : (reps > 64 ? 64 : reps);
	for (int k = -1; k < nr; ++k) {   /* one warm-up call (plans, buffers) */
		const double t0 = now();
		rc = dg_encode_pipelined(ctx, DG_ALGO_ONEPASS, R, V, pairs, n, &o, chunk_bytes, out, out_cap, offs, st);
		const double dt = now() - t0;
		if (rc) { fprintf(stderr, "encode: %s\n", dg_status_string(rc)); return 1; }
		if (k >= 0) t[k] = dt;
	}
	uint32_t bad = 0;
	for (uint32_t i = 0; i < n; ++i) bad += st[i] != 0;
	/* spot check: the same bytes as the single-pair entry point */
	uint32_t mism = 0, checked = 0;
	for (uint32_t i = 0; i < n; i += n / 7 + 1) {
		dg_buffer_t d = {0, 0};
		if (dg_encode(ctx, DG_ALGO_ONEPASS, R + pairs[i].r_off, L, V + pairs[i].v_off, L, &o, &d)) { ++mism; continue; }
		if (d.len != offs[i + 1] - offs[i] || memcmp(d.data, out + offs[i], d.len)) ++mism;
		dg_buffer_free(&d);
		++checked;
	}
	qsort(t, nr, sizeof t[0], cmp_d);
	const double med = t[nr / 2];
	printf("{\"metric\": \"host-to-host delta-encode GiB/s (dg_encode_pipelined, C only)\", \"value\": %.3f, "
	       "\"unit\": \"GiB/s\", \"pairs\": %u, \"pair_bytes\": %llu, \"chunk_pairs\": %u, \"pinned\": %d, "
	       "\"median_s\": %.6f, \"min_s\": %.6f, \"delta_bytes\": %llu, \"bad_status\": %u, "
	       "\"spot_checked\": %u, \"spot_mismatch\": %u}\n",
	       2.0 * arena / med / (1ull << 30), n, (unsigned long long)L, chunk_pairs, pinned, med, t[0],
	       (unsigned long long)offs[n], bad, checked, mism);
	if (pinned) { dg_host_free(R); dg_host_free(V); dg_host_free(out); } else { free(R); free(V); free(out); }
	free(pairs); free(offs); free(st);
	dg_context_destroy(ctx);
	return bad || mism ? 1 : 0;
}
