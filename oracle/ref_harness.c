/*
 * ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Thin driver linked against the reference's own src/c library (built from
 * /root/reference/src/c by oracle/Makefile into oracle/_ref/).  Two uses:
 *
 *   1. ref_encode_pair(): the reference's CLI chain main.c:257-292
 *      (delta_crc64_xz x2 -> delta_diff -> delta_place_commands ->
 *      delta_encode) for one in-memory pair.  tests/ call it through ctypes to
 *      pin the oracle restatement against the real reference.
 *   2. ref_bench main(): the CPU baseline timed by bench.py's cpu_baseline
 *      leg — a pthread pool, one pair per task, same synthetic inputs and
 *      table size as the GPU run, CRC table warmed first (delta.h:297-312 is
 *      not thread-safe on first use); the rate is taken from the median of
 *      the timed repetitions (times sorted in the output).
 *
 * Nothing here is part of the product.
 */
#define _POSIX_C_SOURCE 200809L
#include "delta.h"   /* the reference header, via -I$(REF) (oracle/Makefile) */

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "delta_oracle.h"

size_t ref_encode_pair(int algo, const uint8_t *r, size_t r_len,
                       const uint8_t *v, size_t v_len, size_t p,
                       size_t q, size_t buf_cap, size_t max_table,
                       uint8_t **out)
{
	uint8_t sc[DELTA_CRC_SIZE], dc[DELTA_CRC_SIZE];
	delta_diff_options_t o = DELTA_DIFF_OPTIONS_DEFAULT;
	o.p = p;
	o.q = q;
	o.buf_cap = buf_cap;
	o.max_table = max_table;
	delta_crc64_xz(r, r_len, sc);
	delta_crc64_xz(v, v_len, dc);
	delta_commands_t cmds = delta_diff((delta_algorithm_t)algo, r, r_len, v, v_len, &o);
	delta_placed_commands_t placed = delta_place_commands(&cmds);
	delta_buffer_t b = delta_encode(&placed, false, v_len, sc, dc);
	delta_placed_commands_free(&placed);
	delta_commands_free(&cmds);
	*out = b.data;
	return b.len;
}

/* main.c:257-292 with --inplace: delta_make_inplace (policy 0 = localmin,
 * 1 = constant) replaces delta_place_commands; the header flag is set.  Used
 * to produce the in-place command streams the decode tests and the C5
 * decode bench replay. */
size_t ref_encode_pair_inplace(int algo, const uint8_t *r, size_t r_len,
                               const uint8_t *v, size_t v_len, size_t p,
                               size_t q, int policy, uint8_t **out)
{
	uint8_t sc[DELTA_CRC_SIZE], dc[DELTA_CRC_SIZE];
	delta_diff_options_t o = DELTA_DIFF_OPTIONS_DEFAULT;
	o.p = p;
	o.q = q;
	delta_crc64_xz(r, r_len, sc);
	delta_crc64_xz(v, v_len, dc);
	delta_commands_t cmds = delta_diff((delta_algorithm_t)algo, r, r_len, v, v_len, &o);
	delta_placed_commands_t placed =
	    delta_make_inplace(r, r_len, &cmds, (delta_cycle_policy_t)policy);
	delta_buffer_t b = delta_encode(&placed, true, v_len, sc, dc);
	delta_placed_commands_free(&placed);
	delta_commands_free(&cmds);
	*out = b.data;
	return b.len;
}

/* main.c:339-385 in memory: delta_decode, the source CRC pre-check, apply
 * (standard or in-place), the output CRC post-check.  Returns 0, or 9 / 10
 * for a source / output CRC mismatch; *out receives the output. */
int ref_decode_pair(const uint8_t *r, size_t r_len, const uint8_t *delta,
                    size_t dl, uint8_t **out, size_t *out_len)
{
	delta_decode_result_t dr = delta_decode(delta, dl);
	uint8_t c[DELTA_CRC_SIZE];
	delta_crc64_xz(r, r_len, c);
	if (memcmp(c, dr.src_crc, DELTA_CRC_SIZE) != 0) {
		delta_decode_result_free(&dr);
		return 9;
	}
	delta_buffer_t b = dr.inplace
	    ? delta_apply_delta_inplace(r, r_len, &dr.commands, dr.version_size)
	    : delta_apply_placed(r, &dr.commands, dr.version_size);
	delta_crc64_xz(b.data, dr.version_size, c);
	int rc = memcmp(c, dr.dst_crc, DELTA_CRC_SIZE) != 0 ? 10 : 0;
	delta_decode_result_free(&dr);
	*out = b.data;
	*out_len = dr.version_size;
	return rc;
}

void ref_free(void *p) { free(p); }

#ifdef REF_BENCH_MAIN
/* ── CPU baseline ───────────────────────────────────────────────────────── */

typedef struct {
	int algo;               /* 1 onepass, 2 correcting; 11 / 12: decode standard / in-place onepass
	                           deltas; 13: decode in-place correcting deltas */
	size_t n_pairs, len, p, q;
	uint8_t **r, **v;
	size_t *lens;           /* per pair |R| (= |V| unless vlens) */
	size_t *vlens;          /* shift pairs: per pair |V| */
	uint8_t **d;            /* decode modes: the deltas */
	size_t *dlens;
	size_t next;
	pthread_mutex_t mu;
	unsigned long long out_bytes;
} job_t;

static void *worker(void *arg)
{
	job_t *j = arg;
	unsigned long long ob = 0;
	for (;;) {
		pthread_mutex_lock(&j->mu);
		size_t i = j->next++;
		pthread_mutex_unlock(&j->mu);
		if (i >= j->n_pairs) break;
		uint8_t *d = NULL;
		if (j->algo >= 10) {
			size_t ol = 0;
			if (ref_decode_pair(j->r[i], j->lens[i], j->d[i], j->dlens[i], &d, &ol) != 0)
				abort();
			ob += ol;
		} else {
			ob += ref_encode_pair(j->algo, j->r[i], j->lens[i], j->v[i], j->vlens ? j->vlens[i] : j->lens[i],
			                      j->p, j->q, DELTA_BUF_CAP,
			                      DELTA_MAX_TABLE_SIZE, &d);
		}
		free(d);
	}
	pthread_mutex_lock(&j->mu);
	j->out_bytes += ob;
	pthread_mutex_unlock(&j->mu);
	return NULL;
}

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec / 1e9;
}

/* usage: ref_bench algo n_pairs pair_len edit_rate seed_base threads q reps [indel_pct]
 * algo 1 / 2: encode onepass / correcting; 11 / 12: decode (+ both CRC checks)
 * of standard / in-place (localmin) onepass deltas, 13: of in-place
 * (localmin) correcting deltas, rate = sum |V| / time;
 * edit_rate >= 0: C2/C3 substitution pairs; edit_rate < 0: C4 transposition
 * pairs (num_blocks = 8 + i mod 57, -edit_rate percent of blocks moved);
 * indel_pct given: shift pairs (or_synth_shift, encode modes only). */
int main(int argc, char **argv)
{
	if (argc < 9) {
		fprintf(stderr, "usage: ref_bench algo n_pairs pair_len edit_rate seed_base threads q reps\n");
		return 2;
	}
	job_t j;
	memset(&j, 0, sizeof(j));
	j.algo = atoi(argv[1]);
	j.n_pairs = strtoull(argv[2], NULL, 0);
	j.len = strtoull(argv[3], NULL, 0);
	double rate = atof(argv[4]);
	unsigned long long seed = strtoull(argv[5], NULL, 0);
	int threads = atoi(argv[6]);
	j.q = strtoull(argv[7], NULL, 0);
	int reps = atoi(argv[8]);
	int indel_pct = argc > 9 ? atoi(argv[9]) : -1;   /* >= 0: shift pairs (or_synth_shift) */
	j.p = DELTA_SEED_LEN;
	j.r = malloc(j.n_pairs * sizeof(uint8_t *));
	j.v = malloc(j.n_pairs * sizeof(uint8_t *));
	j.lens = malloc(j.n_pairs * sizeof(size_t));
	unsigned long long n_edits = rate > 0 ? (unsigned long long)(rate * (double)j.len + 0.5) : 0;
	double total_in = 0;
	for (size_t i = 0; i < j.n_pairs; i++) {
		if (indel_pct >= 0) {
			j.r[i] = malloc(j.len);
			j.v[i] = malloc(j.len + 8 * n_edits + 1);
			size_t vl = or_synth_shift(seed + i, j.len, n_edits, (uint32_t)indel_pct, j.r[i], j.v[i]);
			j.lens[i] = j.len;
			if (!j.vlens) j.vlens = calloc(j.n_pairs, sizeof(size_t));
			j.vlens[i] = vl;
		} else if (rate < 0) {
			uint32_t nb = 8 + (uint32_t)(i % 57), mean = (uint32_t)(j.len / nb);
			size_t cap = (size_t)nb * (mean * 3 / 2 + 1);
			j.r[i] = malloc(cap);
			j.v[i] = malloc(cap);
			j.lens[i] = or_synth_transpose(seed + i, nb, mean, (uint32_t)(-rate), j.r[i], j.v[i], cap);
		} else {
			j.r[i] = malloc(j.len);
			j.v[i] = malloc(j.len);
			j.lens[i] = j.len;
			or_synth_random(seed + i, j.r[i], j.len);
			memcpy(j.v[i], j.r[i], j.len);
			or_synth_edits(seed + i, j.v[i], j.len, n_edits);
		}
		total_in += (double)j.lens[i] + (double)(j.vlens ? j.vlens[i] : j.lens[i]);
	}
	{   /* warm the reference's lazy CRC table before threads start */
		uint8_t c[8];
		delta_crc64_xz(j.r[0], 1, c);
	}
	if (j.algo >= 10) {   /* decode modes: encode every pair first (untimed) */
		j.d = malloc(j.n_pairs * sizeof(uint8_t *));
		j.dlens = malloc(j.n_pairs * sizeof(size_t));
		total_in = 0;
		for (size_t i = 0; i < j.n_pairs; i++) {
			j.dlens[i] = j.algo >= 12
			    ? ref_encode_pair_inplace(j.algo == 13 ? 2 : 1, j.r[i], j.lens[i], j.v[i], j.lens[i], j.p, j.q, 0,
			                              &j.d[i])
			    : ref_encode_pair(1, j.r[i], j.lens[i], j.v[i], j.lens[i], j.p, j.q,
			                      DELTA_BUF_CAP, DELTA_MAX_TABLE_SIZE, &j.d[i]);
			total_in += (double)j.lens[i];   /* decode rate counts |V| reconstructed */
		}
	}
	double best = 1e30, sum = 0;
	double *times = malloc((reps > 0 ? reps : 1) * sizeof(double));
	unsigned long long out_bytes = 0;
	for (int rep = 0; rep < reps; rep++) {
		j.next = 0;
		j.out_bytes = 0;
		pthread_mutex_init(&j.mu, NULL);
		pthread_t *th = malloc(threads * sizeof(pthread_t));
		double t0 = now();
		for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &j);
		for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
		double dt = now() - t0;
		free(th);
		times[rep] = dt;
		if (dt < best) best = dt;
		sum += dt;
		out_bytes = j.out_bytes;
	}
	/* median of the repetitions */
	for (int a = 1; a < reps; a++)
		for (int b = a; b > 0 && times[b - 1] > times[b]; b--) {
			double t = times[b]; times[b] = times[b - 1]; times[b - 1] = t;
		}
	double med = reps % 2 ? times[reps / 2] : 0.5 * (times[reps / 2 - 1] + times[reps / 2]);
	double in_bytes = total_in;
	printf("{\"pairs\": %zu, \"pair_len\": %zu, \"threads\": %d, \"reps\": %d, "
	       "\"best_s\": %.6f, \"mean_s\": %.6f, \"median_s\": %.6f, \"times_s\": [",
	       j.n_pairs, j.len, threads, reps, best, sum / reps, med);
	for (int r = 0; r < reps; r++) printf("%s%.4f", r ? ", " : "", times[r]);
	printf("], \"in_bytes\": %.0f, \"out_bytes\": %llu, \"gib_per_s\": %.6f}\n",
	       in_bytes, out_bytes, in_bytes / med / (1024.0 * 1024.0 * 1024.0));
	free(times);
	return 0;
}
#endif
