/*
 * delta_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference algorithms on the hot path of
 * darrelllong/Delta-Compression (src/c).  It exists to check the MI355X HIP
 * path bit for bit; it is never linked into, loaded by, or called from the
 * product library (delta-compression_amd/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it.
 *
 * Pinning: every function here is checked against the reference itself
 * (oracle/_ref, compiled from /root/reference/src/c by oracle/Makefile) and
 * against the committed golden vectors in tests/golden/ (see
 * tests/test_oracle.py).
 *
 * Commands are represented without payload copies: an ADD always carries
 * V[v_off, v_off+len) in both onepass and correcting (onepass.c:243-250,
 * correcting.c:614-622), so storing the V offset is enough.
 */
#ifndef DELTA_ORACLE_H
#define DELTA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_COPY = 1, OR_ADD = 2 };

typedef struct {
	uint32_t kind;   /* OR_COPY / OR_ADD */
	uint32_t pad;
	uint64_t r_off;  /* COPY: reference offset; ADD: unused */
	uint64_t v_off;  /* position in V (== placed dst, apply.c:136-164) */
	uint64_t len;
} or_cmd_t;

/* hash.c:15-24 */
uint64_t or_mod_mersenne(uint64_t hi, uint64_t lo);
/* hash.c:28-38 */
uint64_t or_fingerprint(const uint8_t *data, size_t off, size_t p);
/* hash.c:163-190, deterministic Miller-Rabin (bases 2..37 are exact for
 * all 64-bit n); the reference draws 100 random bases (hash.c:172). */
int      or_is_prime(uint64_t n);
uint64_t or_next_prime(uint64_t n);
/* onepass.c:61-62 */
uint64_t or_onepass_q(uint64_t r_len, uint64_t p, uint64_t q_floor);
/* correcting.c:116-129 -> cap, |F|, m */
void     or_correcting_params(uint64_t r_len, uint64_t p, uint64_t q_floor,
                              uint64_t max_table, uint64_t *cap,
                              uint64_t *f_size, uint64_t *m);

/* delta.h:294-322 (big-endian output) */
void     or_crc64_xz(const uint8_t *data, size_t len, uint8_t out[8]);
uint64_t or_crc64_xz_u64(const uint8_t *data, size_t len);

/* onepass.c:32-297 (hash-table path).  Returns number of commands; *out is
 * malloc'd (free with or_free). */
size_t or_diff_onepass(const uint8_t *r, size_t r_len,
                       const uint8_t *v, size_t v_len,
                       size_t p, size_t q_floor, or_cmd_t **out);

/* correcting.c:81-495 (hash-table path). */
size_t or_diff_correcting(const uint8_t *r, size_t r_len,
                          const uint8_t *v, size_t v_len,
                          size_t p, size_t q_floor, size_t buf_cap,
                          size_t max_table, or_cmd_t **out);

/* apply.c:136-164 + encoding.c:39-90 (standard delta, flags 0).  Returns the
 * serialized length; *out is malloc'd. */
size_t or_encode(const or_cmd_t *cmds, size_t n, const uint8_t *v,
                 size_t v_len, const uint8_t src_crc[8],
                 const uint8_t dst_crc[8], uint8_t **out);

/* main.c:257-292 chain for one pair: crc x2, diff, place, encode.
 * algo: 1 = onepass, 2 = correcting (delta.h:85 numbering). */
size_t or_encode_pair(int algo, const uint8_t *r, size_t r_len,
                      const uint8_t *v, size_t v_len, size_t p,
                      size_t q_floor, size_t buf_cap, size_t max_table,
                      uint8_t **out);

/* encoding.c:111-178 + apply.c:229-284 + main.c:341-385.
 * Returns 0 ok, 8 malformed, 9 src crc mismatch, 10 dst crc mismatch
 * (numbering of dg_status_t in include/delta_gpu.h).  *out is malloc'd. */
int or_decode_apply(const uint8_t *r, size_t r_len, const uint8_t *delta,
                    size_t delta_len, int ignore_hash, uint8_t **out,
                    size_t *out_len);

/* Synthetic workloads (see DESIGN.md "Synthetic inputs"). */
uint64_t or_splitmix64_at(uint64_t seed, uint64_t k);
void     or_synth_random(uint64_t seed, uint8_t *buf, size_t len);
void     or_synth_edits(uint64_t seed, uint8_t *buf, size_t len,
                        uint64_t n_edits);
/* gen_transpositions.py recipe with a per-pair splitmix seed; writes
 * |R| == |V| == returned length bytes (buffers must hold cap bytes). */
size_t   or_synth_transpose(uint64_t seed, uint32_t num_blocks,
                            uint32_t mean_size, uint32_t perm_pct,
                            uint8_t *r, uint8_t *v, size_t cap);
/* Shift pairs: R = or_synth_random(seed, len); V = R with n_edits edits,
 * one per equal stratum of R, indel_pct percent of them insertions or
 * deletions of 1..8 bytes (half each), the rest byte substitutions (see
 * DESIGN.md "Synthetic inputs").  Returns |V| (v must hold len + 8 n_edits). */
size_t   or_synth_shift(uint64_t seed, size_t len, uint64_t n_edits,
                        uint32_t indel_pct, uint8_t *r, uint8_t *v);

void or_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
