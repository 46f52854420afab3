/*
 * spec_model.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU model of the speculative diagonal-member onepass that the MI355X path
 * runs (DESIGN.md "Onepass as verified diagonal members"), written to be
 * checked command-for-command against the oracle's restatement of
 * src/c/onepass.c:32-297 (or_diff_onepass) on adversarial inputs before and
 * alongside the HIP kernels (tests/test_spec_model.py).  It mirrors the
 * kernels' decisions exactly, including their conservative ones (32-bit
 * fingerprint comparisons, the member-length limit), so a divergence here is
 * a divergence of the design, not of one implementation.
 *
 * The model:
 *   1. Mismatch positions along diagonal 0 (V[x] != R[x], x < E = min(|R|,|V|)),
 *      with a virtual mismatch at -1 and a sentinel at E, are grouped into
 *      runs separated by gaps > p.  Member k starts its epoch at s_k (0 for
 *      k = 0, else the first mismatch of run k) and, if every lookup of the
 *      epoch behaves as on random data, first sees equal windows at
 *      x_k = (last mismatch of run k) + 1, matches there on the diagonal and
 *      extends to s_{k+1}.  The run holding the sentinel starts the final
 *      epoch s_K.
 *   2. A member is verified when (A) no V window of steps 0..T equals, in a
 *      32-bit equality-preserving hash (sm_hash, the kernels' win_hash), an R
 *      window of another step of the member (only byte-equal windows can
 *      verify a lookup, onepass.c:169-219), and (B) at
 *      T = x_k - s_k lookup 1 or lookup 2 finds step T itself as the slot's
 *      first writer of the epoch (onepass.c:141-166): slot_V(T) is not among
 *      slot_V(0..T-1), or slot_R(T) is not among slot_R(0..T-1); and
 *      T < SM_MAX_T, and the next member starts within SM_AHEAD bytes past
 *      the end of the SM_CHUNK-byte chunk holding s_k (the kernel's staged
 *      region).
 *   3. The chain takes verified members as they are; from an unverified one
 *      it runs the reference's epochs exactly until an epoch ends on diagonal
 *      0 at a later member start (re-sync), and the final epoch exactly.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "delta_oracle.h"

#define SM_MAX_T 512   /* members of T + 1 > 512 steps are left to the exact engine */
#define SM_CHUNK 2048  /* member_chunk_kernel: members belong to the chunk of their start ... */
#define SM_AHEAD 240   /* ... and need the next member's start within this look-ahead */

typedef struct {
	uint64_t members, verified, exact_epochs, resyncs;
} sm_stats_t;

typedef struct { or_cmd_t *a; size_t n, cap; } sm_vec_t;

static void sm_push(sm_vec_t *c, uint32_t kind, uint64_t r_off, uint64_t v_off, uint64_t len)
{
	if (c->n == c->cap) {
		c->cap = c->cap ? 2 * c->cap : 64;
		c->a = realloc(c->a, c->cap * sizeof(*c->a));
		if (!c->a) abort();
	}
	or_cmd_t *x = &c->a[c->n++];
	x->kind = kind;
	x->pad = 0;
	x->r_off = r_off;
	x->v_off = v_off;
	x->len = len;
}

typedef struct { uint64_t fp, off, ver; int used; } sm_ent_t;

/* One epoch of onepass.c:94-265 from (*vc, *rc) with tables of a fresh
 * version; emits ADD + COPY on a match and moves the cursors.  Returns 0 when
 * the scan is over (no match before both streams ran out). */
static int sm_epoch(const uint8_t *r, size_t r_len, const uint8_t *v, size_t v_len, size_t p,
                    uint64_t q, sm_ent_t *hv, sm_ent_t *hr, uint64_t ver, size_t *vc, size_t *rc,
                    size_t *vs, sm_vec_t *out)
{
	for (;;) {
		int can_v = *vc + p <= v_len, can_r = *rc + p <= r_len;
		if (!can_v && !can_r) return 0;
		uint64_t fv = can_v ? or_fingerprint(v, *vc, p) : 0;
		uint64_t fr = can_r ? or_fingerprint(r, *rc, p) : 0;
		if (can_v) {
			sm_ent_t *e = &hv[fv % q];
			if (!(e->used && e->ver == ver)) { e->fp = fv; e->off = *vc; e->ver = ver; e->used = 1; }
		}
		if (can_r) {
			sm_ent_t *e = &hr[fr % q];
			if (!(e->used && e->ver == ver)) { e->fp = fr; e->off = *rc; e->ver = ver; e->used = 1; }
		}
		int hit = 0;
		size_t vm = 0, rm = 0;
		if (can_r) {
			sm_ent_t *e = &hv[fr % q];
			if (e->used && e->ver == ver && e->fp == fr && memcmp(r + *rc, v + e->off, p) == 0) {
				hit = 1; rm = *rc; vm = e->off;
			}
		}
		if (!hit && can_v) {
			sm_ent_t *e = &hr[fv % q];
			if (e->used && e->ver == ver && e->fp == fv && memcmp(v + *vc, r + e->off, p) == 0) {
				hit = 1; vm = *vc; rm = e->off;
			}
		}
		if (!hit) { ++*vc; ++*rc; continue; }
		size_t ml = 0;
		while (vm + ml < v_len && rm + ml < r_len && v[vm + ml] == r[rm + ml]) ml++;
		if (*vs < vm) sm_push(out, OR_ADD, 0, *vs, vm - *vs);
		sm_push(out, OR_COPY, rm, vm, ml);
		*vs = vm + ml;
		*vc = vm + ml;
		*rc = rm + ml;
		return 1;
	}
}

static uint32_t sm_rotr(uint32_t x, unsigned s) { return (x >> s) | (x << (32 - s)); }

/* member_chunk_kernel's win_hash of the 16 bytes at d (little-endian words) */
static uint32_t sm_hash(const uint8_t *d)
{
	uint32_t w[4];
	memcpy(w, d, 16);
	return w[0] ^ sm_rotr(w[1], 27) ^ sm_rotr(w[2], 21) ^ sm_rotr(w[3], 15);
}

/* (A) and (B) of the header for the member [s, x]. */
static int sm_verify(const uint8_t *r, const uint8_t *v, size_t s, size_t x, size_t p, uint64_t q)
{
	const size_t T = x - s;
	if (T + 1 > SM_MAX_T) return 0;
	uint64_t fv[SM_MAX_T], fr[SM_MAX_T];
	uint32_t hv[SM_MAX_T], hr[SM_MAX_T];
	for (size_t t = 0; t <= T; ++t) {
		fv[t] = or_fingerprint(v, s + t, p);
		fr[t] = or_fingerprint(r, s + t, p);
		hv[t] = sm_hash(v + s + t);
		hr[t] = sm_hash(r + s + t);
	}
	for (size_t c = 0; c <= T; ++c)
		for (size_t l = 0; l <= T; ++l)
			if (c != l && hv[c] == hr[l]) return 0;
	int dup_v = 0, dup_r = 0;
	for (size_t c = 0; c < T; ++c) {
		if (fv[c] % q == fv[T] % q) dup_v = 1;
		if (fr[c] % q == fr[T] % q) dup_r = 1;
	}
	return !(dup_v && dup_r);
}

size_t sm_diff_onepass_spec(const uint8_t *r, size_t r_len, const uint8_t *v, size_t v_len,
                            size_t p, size_t q_floor, or_cmd_t **out, sm_stats_t *st)
{
	sm_vec_t c = {0};
	sm_stats_t z = {0};
	if (!st) st = &z;
	memset(st, 0, sizeof *st);
	*out = NULL;
	if (v_len == 0) return 0;
	const uint64_t q = or_onepass_q(r_len, p, q_floor);
	const size_t E = r_len < v_len ? r_len : v_len;

	/* 1. members */
	size_t cap = E / p + 2;
	size_t *ms = malloc(cap * sizeof *ms), *mx = malloc(cap * sizeof *mx);
	if (!ms || !mx) abort();
	size_t K = 0;
	long long prev = -1;
	ms[0] = 0;
	for (size_t x = 0; x <= E; ++x) {
		if (x < E && r[x] == v[x]) continue;
		if ((long long)x - prev > (long long)p) {
			mx[K] = (size_t)(prev + 1);
			ms[++K] = x;
		}
		prev = (long long)x;
	}
	/* 2. verification */
	unsigned char *ok = calloc(K + 1, 1);
	if (!ok) abort();
	for (size_t k = 0; k < K; ++k)
		ok[k] = (unsigned char)(ms[k + 1] < (ms[k] / SM_CHUNK + 1) * SM_CHUNK + SM_AHEAD &&
		                        sm_verify(r, v, ms[k], mx[k], p, q));
	st->members = K;
	for (size_t k = 0; k < K; ++k) st->verified += ok[k];

	/* 3. chain */
	sm_ent_t *hv = calloc(q, sizeof *hv), *hr = calloc(q, sizeof *hr);
	if (!hv || !hr) abort();
	uint64_t ver = 0;
	size_t k = 0, vs = 0;
	for (;;) {
		while (k < K && ok[k]) {
			if (mx[k] > ms[k]) sm_push(&c, OR_ADD, 0, ms[k], mx[k] - ms[k]);
			sm_push(&c, OR_COPY, mx[k], mx[k], ms[k + 1] - mx[k]);
			vs = ms[k + 1];
			++k;
		}
		/* exact epochs from member k's start (the final epoch when k == K) */
		size_t vc = ms[k], rc = ms[k];
		int resynced = 0;
		while (sm_epoch(r, r_len, v, v_len, p, q, hv, hr, ++ver, &vc, &rc, &vs, &c)) {
			st->exact_epochs++;
			if (k < K && vc == rc && vc > ms[k]) {
				size_t m = k + 1;
				while (m <= K && ms[m] < vc) ++m;
				if (m <= K && ms[m] == vc) {   /* re-sync */
					k = m;
					st->resyncs++;
					resynced = 1;
					break;
				}
			}
		}
		if (!resynced) break;
	}
	if (vs < v_len) sm_push(&c, OR_ADD, 0, vs, v_len - vs);
	free(hv);
	free(hr);
	free(ok);
	free(ms);
	free(mx);
	*out = c.a;
	return c.n;
}
