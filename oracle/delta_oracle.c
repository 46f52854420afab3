/*
 * delta_oracle.c — TEST INFRASTRUCTURE ONLY (see delta_oracle.h).
 *
 * CPU restatement of the reference's onepass / correcting / CRC-64/XZ /
 * DLT\x03 encode / decode+apply.  Each function cites the reference lines it
 * restates.  Written from the reference's behaviour; validated against the
 * reference build in oracle/_ref and the golden vectors in tests/golden/.
 */
#include "delta_oracle.h"

#include <stdlib.h>
#include <string.h>

#define OR_MOD   ((1ULL << 61) - 1)   /* delta.h:25 */
#define OR_BASE  263ULL               /* delta.h:24 */

typedef unsigned __int128 u128;

void or_free(void *p) { free(p); }

/* ── growable command vector ─────────────────────────────────────────── */

typedef struct { or_cmd_t *a; size_t n, cap; } cvec_t;

static void cvec_push(cvec_t *c, uint32_t kind, uint64_t r_off,
                      uint64_t v_off, uint64_t len)
{
	if (c->n == c->cap) {
		c->cap = c->cap ? 2 * c->cap : 64;
		c->a = realloc(c->a, c->cap * sizeof(*c->a));
		if (!c->a) abort();
	}
	c->a[c->n].kind = kind;
	c->a[c->n].pad = 0;
	c->a[c->n].r_off = r_off;
	c->a[c->n].v_off = v_off;
	c->a[c->n].len = len;
	c->n++;
}

/* ── Mersenne arithmetic, fingerprints (hash.c:15-98) ─────────────────── */

static uint64_t mod_m(u128 x)
{
	/* two folds of 2^61 == 1 (mod 2^61-1), then canonicalise (hash.c:15-24) */
	u128 t = (x & OR_MOD) + (x >> 61);
	t = (t & OR_MOD) + (t >> 61);
	uint64_t r = (uint64_t)t;
	if (r >= OR_MOD) r -= OR_MOD;
	return r;
}

uint64_t or_mod_mersenne(uint64_t hi, uint64_t lo)
{
	return mod_m(((u128)hi << 64) | lo);
}

uint64_t or_fingerprint(const uint8_t *data, size_t off, size_t p)
{
	uint64_t h = 0;
	for (size_t i = 0; i < p; i++)
		h = mod_m((u128)h * OR_BASE + data[off + i]);
	return h;
}

/* rolling window state (hash.c:62-98): roll on +1, recompute otherwise */
typedef struct { uint64_t val, bp; size_t pos; int valid; } roll_t;

static uint64_t roll_at(roll_t *h, const uint8_t *d, size_t at, size_t p)
{
	if (h->valid && at == h->pos)
		return h->val;
	if (h->valid && at == h->pos + 1) {
		uint64_t sub = mod_m((u128)d[at - 1] * h->bp);
		uint64_t x = h->val >= sub ? h->val - sub : OR_MOD - (sub - h->val);
		h->val = mod_m((u128)x * OR_BASE + d[at + p - 1]);
	} else {
		uint64_t bp = 1;                  /* OR_BASE^(p-1), hash.c:42-58 */
		for (size_t i = 1; i < p; i++) bp = mod_m((u128)bp * OR_BASE);
		h->bp = bp;
		h->val = or_fingerprint(d, at, p);
		h->valid = 1;
	}
	h->pos = at;
	return h->val;
}

/* ── primes (hash.c:102-190) ───────────────────────────────────────────── */

static uint64_t mulmod64(uint64_t a, uint64_t b, uint64_t m)
{
	return (uint64_t)((u128)a * b % m);
}

static uint64_t powmod64(uint64_t b, uint64_t e, uint64_t m)
{
	uint64_t r = 1 % m;
	b %= m;
	while (e) {
		if (e & 1) r = mulmod64(r, b, m);
		b = mulmod64(b, b, m);
		e >>= 1;
	}
	return r;
}

int or_is_prime(uint64_t n)
{
	static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
	if (n < 2) return 0;
	for (size_t i = 0; i < sizeof(bases) / sizeof(bases[0]); i++) {
		if (n == bases[i]) return 1;
		if (n % bases[i] == 0) return 0;
	}
	uint64_t d = n - 1;
	int s = 0;
	while ((d & 1) == 0) { d >>= 1; s++; }
	for (size_t i = 0; i < sizeof(bases) / sizeof(bases[0]); i++) {
		uint64_t x = powmod64(bases[i], d, n);
		if (x == 1 || x == n - 1) continue;
		int comp = 1;
		for (int k = 1; k < s; k++) {
			x = mulmod64(x, x, n);
			if (x == n - 1) { comp = 0; break; }
		}
		if (comp) return 0;
	}
	return 1;
}

uint64_t or_next_prime(uint64_t n)
{
	/* hash.c:180-190: 2 for n <= 2, else the first odd prime >= n */
	if (n <= 2) return 2;
	uint64_t c = (n & 1) ? n : n + 1;
	while (!or_is_prime(c)) c += 2;
	return c;
}

uint64_t or_onepass_q(uint64_t r_len, uint64_t p, uint64_t q_floor)
{
	uint64_t seeds = r_len >= p ? r_len - p + 1 : 0;   /* onepass.c:61 */
	uint64_t want = seeds / p;
	return or_next_prime(q_floor > want ? q_floor : want); /* onepass.c:62 */
}

void or_correcting_params(uint64_t r_len, uint64_t p, uint64_t q_floor,
                          uint64_t max_table, uint64_t *cap,
                          uint64_t *f_size, uint64_t *m)
{
	/* correcting.c:116-129 */
	uint64_t seeds = r_len >= p ? r_len - p + 1 : 0;
	uint64_t mt = max_table > 0 ? max_table : 1073741827ULL;
	uint64_t raw = q_floor;
	if (seeds > 0 && 2 * seeds / p > raw) raw = 2 * seeds / p;
	if (raw > mt) raw = mt;
	*cap = or_next_prime(raw);
	*f_size = seeds > 0 ? or_next_prime(2 * seeds) : 1;
	*m = (*f_size <= *cap) ? 1 : (*f_size + *cap - 1) / *cap;
}

/* ── CRC-64/XZ (delta.h:294-322) ──────────────────────────────────────── */

static uint64_t crc_tab[256];
static int crc_ready;

static void crc_init(void)
{
	if (crc_ready) return;
	for (unsigned i = 0; i < 256; i++) {
		uint64_t c = i;
		for (int k = 0; k < 8; k++)
			c = (c >> 1) ^ ((c & 1) ? 0xC96C5795D7870F42ULL : 0);
		crc_tab[i] = c;
	}
	crc_ready = 1;
}

uint64_t or_crc64_xz_u64(const uint8_t *data, size_t len)
{
	crc_init();
	uint64_t c = ~0ULL;
	for (size_t i = 0; i < len; i++)
		c = crc_tab[(uint8_t)(c ^ data[i])] ^ (c >> 8);
	return ~c;
}

void or_crc64_xz(const uint8_t *data, size_t len, uint8_t out[8])
{
	uint64_t c = or_crc64_xz_u64(data, len);
	for (int i = 0; i < 8; i++)
		out[i] = (uint8_t)(c >> (56 - 8 * i));   /* big-endian, delta.h:320 */
}

/* ── onepass (onepass.c:32-297, hash-table path) ──────────────────────── */

typedef struct { uint64_t fp; uint64_t off; uint64_t ver; int used; } op_ent_t;

size_t or_diff_onepass(const uint8_t *r, size_t r_len,
                       const uint8_t *v, size_t v_len,
                       size_t p, size_t q_floor, or_cmd_t **out)
{
	cvec_t c = {0};
	*out = NULL;
	if (v_len == 0) return 0;                               /* :58 */
	uint64_t q = or_onepass_q(r_len, p, q_floor);           /* :61-62 */
	op_ent_t *hv = calloc(q, sizeof(*hv));                  /* :76-77 */
	op_ent_t *hr = calloc(q, sizeof(*hr));
	if (!hv || !hr) abort();

	size_t rc = 0, vc = 0, vs = 0;                          /* :81-83 */
	uint64_t ver = 0;
	roll_t rv = {0}, rr = {0};

	for (;;) {
		int can_v = vc + p <= v_len, can_r = rc + p <= r_len; /* :102-104 */
		if (!can_v && !can_r) break;
		uint64_t fv = 0, fr = 0;
		if (can_v) fv = roll_at(&rv, v, vc, p);             /* :108-117 */
		if (can_r) fr = roll_at(&rr, r, rc, p);

		/* store, keeping an entry already written in this version :141-166 */
		if (can_v) {
			op_ent_t *e = &hv[fv % q];
			if (!(e->used && e->ver == ver)) {
				e->fp = fv; e->off = vc; e->ver = ver; e->used = 1;
			}
		}
		if (can_r) {
			op_ent_t *e = &hr[fr % q];
			if (!(e->used && e->ver == ver)) {
				e->fp = fr; e->off = rc; e->ver = ver; e->used = 1;
			}
		}

		/* R fingerprint into the V table first, then V into R :169-219 */
		int hit = 0;
		size_t vm = 0, rm = 0;
		if (can_r) {
			op_ent_t *e = &hv[fr % q];
			if (e->used && e->ver == ver && e->fp == fr &&
			    memcmp(r + rc, v + e->off, p) == 0) {
				hit = 1; rm = rc; vm = e->off;
			}
		}
		if (!hit && can_v) {
			op_ent_t *e = &hr[fv % q];
			if (e->used && e->ver == ver && e->fp == fv &&
			    memcmp(v + vc, r + e->off, p) == 0) {
				hit = 1; vm = vc; rm = e->off;
			}
		}
		if (!hit) { vc++; rc++; continue; }                 /* :221-225 */

		size_t ml = 0;                                      /* :229-234 */
		while (vm + ml < v_len && rm + ml < r_len && v[vm + ml] == r[rm + ml])
			ml++;
		if (ml < p) { vc++; rc++; continue; }               /* :236-240 */
		if (vs < vm) cvec_push(&c, OR_ADD, 0, vs, vm - vs); /* :243-250 */
		cvec_push(&c, OR_COPY, rm, vm, ml);                 /* :251-257 */
		vs = vm + ml;
		vc = vm + ml;                                       /* :261-263 */
		rc = rm + ml;
		ver++;
	}
	if (vs < v_len) cvec_push(&c, OR_ADD, 0, vs, v_len - vs); /* :268-275 */
	free(hv);
	free(hr);
	*out = c.a;
	return c.n;
}

/* ── correcting (correcting.c:81-495, hash-table path) ─────────────────── */

typedef struct { uint64_t fp; uint64_t off; int used; } co_ent_t;
typedef struct {
	uint64_t vs, ve;        /* V interval covered */
	uint32_t kind;
	uint64_t r_off, len;
} lb_ent_t;                 /* lookback buffer entry, correcting.c:14-22 */

typedef struct { lb_ent_t *a; size_t cap, head, n; } ring_t;

static lb_ent_t *ring_at(ring_t *b, size_t i) { return &b->a[(b->head + i) % b->cap]; }

static void ring_emit_oldest_if_full(ring_t *b, size_t buf_cap, cvec_t *out)
{
	/* correcting.c:603-613: the oldest entry leaves the buffer for output */
	if (b->n >= buf_cap) {
		lb_ent_t *o = ring_at(b, 0);
		if (o->kind == OR_COPY)
			cvec_push(out, OR_COPY, o->r_off, o->vs, o->len);
		else
			cvec_push(out, OR_ADD, 0, o->vs, o->len);
		b->head = (b->head + 1) % b->cap;
		b->n--;
	}
}

static void ring_push(ring_t *b, uint32_t kind, uint64_t vs, uint64_t ve,
                      uint64_t r_off)
{
	lb_ent_t *e = ring_at(b, b->n);
	e->kind = kind; e->vs = vs; e->ve = ve; e->r_off = r_off; e->len = ve - vs;
	b->n++;
}

size_t or_diff_correcting(const uint8_t *r, size_t r_len,
                          const uint8_t *v, size_t v_len,
                          size_t p, size_t q_floor, size_t buf_cap,
                          size_t max_table, or_cmd_t **out)
{
	cvec_t c = {0};
	*out = NULL;
	if (v_len == 0) return 0;                                   /* :97 */
	uint64_t cap, fsz, m, k = 0;
	or_correcting_params(r_len, p, q_floor, max_table, &cap, &fsz, &m);
	uint64_t seeds = r_len >= p ? r_len - p + 1 : 0;
	if (v_len >= p) {                                            /* :131-136 */
		/* The reference reads past |V| when p <= |V| < 2p (undefined in C,
		 * IndexError in Python).  Defined here as zero bytes past the end;
		 * the GPU path does the same.  It only matters when m > 1. */
		uint64_t hk = 0;
		for (size_t j = 0; j < p; j++) {
			size_t at = v_len / 2 + j;
			hk = mod_m((u128)hk * OR_BASE + (at < v_len ? v[at] : 0));
		}
		k = hk % fsz % m;
	}

	co_ent_t *h = calloc(cap, sizeof(*h));
	if (!h) abort();
	/* build: every R seed passing the checkpoint, first found wins :164-198 */
	if (seeds > 0) {
		roll_t rb = {0};
		for (uint64_t a = 0; a < seeds; a++) {
			uint64_t fp = roll_at(&rb, r, a, p);
			uint64_t f = fp % fsz;
			if (f % m != k) continue;
			uint64_t i = f / m;
			if (i >= cap) continue;
			if (!h[i].used) { h[i].fp = fp; h[i].off = a; h[i].used = 1; }
		}
	}

	size_t bc = buf_cap ? buf_cap : 1;
	ring_t buf = { calloc(bc + 1, sizeof(lb_ent_t)), bc + 1, 0, 0 };
	if (!buf.a) abort();
	size_t vc = 0, vs = 0;
	roll_t rv = {0};

	for (;;) {
		if (vc + p > v_len) break;                                 /* :229 */
		uint64_t fp = roll_at(&rv, v, vc, p);
		uint64_t f = fp % fsz;
		if (f % m != k) { vc++; continue; }                        /* :239-246 */
		uint64_t i = f / m;
		if (!(i < cap && h[i].used && h[i].fp == fp)) { vc++; continue; }
		size_t ro = h[i].off;
		if (memcmp(r + ro, v + vc, p) != 0) { vc++; continue; }    /* :268-285 */

		size_t fwd = p;                                            /* :293-297 */
		while (vc + fwd < v_len && ro + fwd < r_len && v[vc + fwd] == r[ro + fwd])
			fwd++;
		size_t bwd = 0;                                            /* :299-303 */
		while (vc >= bwd + 1 && ro >= bwd + 1 && v[vc - bwd - 1] == r[ro - bwd - 1])
			bwd++;
		size_t vm = vc - bwd, rm = ro - bwd, ml = bwd + fwd, mend = vm + ml;
		if (ml < p) { vc++; continue; }

		if (vs <= vm) {
			/* 6a: match lies in the unencoded suffix :316-363 */
			if (vs < vm) {
				ring_emit_oldest_if_full(&buf, bc, &c);
				ring_push(&buf, OR_ADD, vs, vm, 0);
			}
			ring_emit_oldest_if_full(&buf, bc, &c);
			ring_push(&buf, OR_COPY, vm, mend, rm);
			vs = mend;
		} else {
			/* 6b: tail correction :364-445 */
			size_t eff = vs;
			while (buf.n > 0) {
				lb_ent_t *t = ring_at(&buf, buf.n - 1);
				if (t->vs >= vm && t->ve <= mend) {   /* fully absorbed */
					if (t->vs < eff) eff = t->vs;
					buf.n--;
					continue;
				}
				if (t->ve > vm && t->vs < vm && t->kind == OR_ADD) {
					size_t keep = vm - t->vs;   /* > 0 here */
					t->ve = vm;
					t->len = keep;
					if (vm < eff) eff = vm;
				}
				break;
			}
			size_t nl = mend - eff;
			if (nl > 0) {
				ring_emit_oldest_if_full(&buf, bc, &c);
				ring_push(&buf, OR_COPY, eff, mend, rm + (eff - vm));
			}
			vs = mend;
		}
		vc = mend;                                                 /* :448 */
	}
	for (size_t j = 0; j < buf.n; j++) {                               /* :452-460 */
		lb_ent_t *e = ring_at(&buf, j);
		if (e->kind == OR_COPY)
			cvec_push(&c, OR_COPY, e->r_off, e->vs, e->len);
		else
			cvec_push(&c, OR_ADD, 0, e->vs, e->len);
	}
	if (vs < v_len) cvec_push(&c, OR_ADD, 0, vs, v_len - vs);         /* :461-468 */
	free(buf.a);
	free(h);
	*out = c.a;
	return c.n;
}

/* ── placement + DLT\x03 serialization (apply.c:136-164, encoding.c:39-90) */

static uint8_t *put_u32(uint8_t *p, uint64_t x)
{
	p[0] = (uint8_t)(x >> 24); p[1] = (uint8_t)(x >> 16);
	p[2] = (uint8_t)(x >> 8);  p[3] = (uint8_t)x;
	return p + 4;
}

size_t or_encode(const or_cmd_t *cmds, size_t n, const uint8_t *v,
                 size_t v_len, const uint8_t src_crc[8],
                 const uint8_t dst_crc[8], uint8_t **out)
{
	size_t total = 26;
	for (size_t i = 0; i < n; i++)
		total += cmds[i].kind == OR_COPY ? 13 : 9 + cmds[i].len;
	uint8_t *b = malloc(total), *p = b;
	if (!b) abort();
	memcpy(p, "DLT\x03", 4); p += 4;
	*p++ = 0;                                   /* flags: standard */
	p = put_u32(p, v_len);
	memcpy(p, src_crc, 8); p += 8;
	memcpy(p, dst_crc, 8); p += 8;
	uint64_t dst = 0;                           /* sequential placement */
	for (size_t i = 0; i < n; i++) {
		if (cmds[i].kind == OR_COPY) {
			*p++ = 1;
			p = put_u32(p, cmds[i].r_off);
			p = put_u32(p, dst);
			p = put_u32(p, cmds[i].len);
		} else {
			*p++ = 2;
			p = put_u32(p, dst);
			p = put_u32(p, cmds[i].len);
			memcpy(p, v + cmds[i].v_off, cmds[i].len);
			p += cmds[i].len;
		}
		dst += cmds[i].len;
	}
	*p++ = 0;
	(void)v_len;
	*out = b;
	return (size_t)(p - b);
}

size_t or_encode_pair(int algo, const uint8_t *r, size_t r_len,
                      const uint8_t *v, size_t v_len, size_t p,
                      size_t q_floor, size_t buf_cap, size_t max_table,
                      uint8_t **out)
{
	uint8_t sc[8], dc[8];
	or_cmd_t *cmds = NULL;
	size_t n;
	or_crc64_xz(r, r_len, sc);
	or_crc64_xz(v, v_len, dc);
	if (algo == 2)
		n = or_diff_correcting(r, r_len, v, v_len, p, q_floor, buf_cap,
		                       max_table, &cmds);
	else
		n = or_diff_onepass(r, r_len, v, v_len, p, q_floor, &cmds);
	size_t len = or_encode(cmds, n, v, v_len, sc, dc, out);
	free(cmds);
	return len;
}

/* ── decode + apply + CRC checks (encoding.c:111-178, apply.c:229-284,
 *    main.c:341-385) ─────────────────────────────────────────────────── */

static uint32_t get_u32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) |
	       ((uint32_t)p[2] << 8) | p[3];
}

int or_decode_apply(const uint8_t *r, size_t r_len, const uint8_t *d,
                    size_t dl, int ignore_hash, uint8_t **out,
                    size_t *out_len)
{
	*out = NULL;
	*out_len = 0;
	if (dl < 25 || memcmp(d, "DLT\x03", 4) != 0) return 8;
	int inplace = d[4] & 1;
	size_t vsz = get_u32(d + 5);
	if (!ignore_hash && or_crc64_xz_u64(r, r_len) != ((uint64_t)get_u32(d + 9) << 32 | get_u32(d + 13)))
		return 9;
	size_t bsz = inplace ? (r_len > vsz ? r_len : vsz) : vsz;
	uint8_t *buf = calloc(bsz ? bsz : 1, 1);
	if (!buf) abort();
	if (inplace && r_len) memcpy(buf, r, r_len);
	size_t pos = 25;
	while (pos < dl) {
		uint8_t t = d[pos++];
		if (t == 0) break;
		if (t == 1) {
			if (pos + 12 > dl) { free(buf); return 8; }
			size_t s = get_u32(d + pos), o = get_u32(d + pos + 4), l = get_u32(d + pos + 8);
			pos += 12;
			if (inplace) {
				if (s + l > bsz || o + l > bsz) { free(buf); return 8; }
				memmove(buf + o, buf + s, l);
			} else {
				if (s + l > r_len || o + l > vsz) { free(buf); return 8; }
				memcpy(buf + o, r + s, l);
			}
		} else if (t == 2) {
			if (pos + 8 > dl) { free(buf); return 8; }
			size_t o = get_u32(d + pos), l = get_u32(d + pos + 4);
			pos += 8;
			if (pos + l > dl || o + l > bsz) { free(buf); return 8; }
			memcpy(buf + o, d + pos, l);
			pos += l;
		} else {
			free(buf);
			return 8;
		}
	}
	if (!ignore_hash && or_crc64_xz_u64(buf, vsz) != ((uint64_t)get_u32(d + 17) << 32 | get_u32(d + 21))) {
		free(buf);
		return 10;
	}
	*out = buf;
	*out_len = vsz;
	return 0;
}

/* ── synthetic workloads ───────────────────────────────────────────────── */

#define GOLDEN_GAMMA 0x9E3779B97F4A7C15ULL

uint64_t or_splitmix64_at(uint64_t seed, uint64_t k)
{
	/* k-th output (k >= 1) of splitmix64 seeded with `seed` */
	uint64_t z = seed + k * GOLDEN_GAMMA;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

void or_synth_random(uint64_t seed, uint8_t *buf, size_t len)
{
	for (size_t i = 0; i < len; i += 8) {
		uint64_t w = or_splitmix64_at(seed, i / 8 + 1);
		for (size_t j = 0; j < 8 && i + j < len; j++)
			buf[i + j] = (uint8_t)(w >> (8 * j));
	}
}

#define EDIT_SALT 0xD1B54A32D192ED03ULL

void or_synth_edits(uint64_t seed, uint8_t *buf, size_t len, uint64_t n_edits)
{
	if (len == 0) return;
	uint64_t s = seed ^ EDIT_SALT;
	for (uint64_t e = 0; e < n_edits; e++) {
		uint64_t pos = or_splitmix64_at(s, 2 * e + 1) % len;
		buf[pos] = (uint8_t)or_splitmix64_at(s, 2 * e + 2);
	}
}

#define SHIFT_SALT 0x2545F4914F6CDD1DULL

size_t or_synth_shift(uint64_t seed, size_t len, uint64_t n_edits, uint32_t indel_pct, uint8_t *r,
                      uint8_t *v)
{
	/* Edit e owns stratum [e S, (e + 1) S) of R (the last one runs to the
	 * end), S = len / n: a position inside it, and a kind (h2 % 100: below
	 * indel_pct / 2 an insertion, below indel_pct a deletion, else a
	 * substitution) with k = 1 + (h2 >> 32) % 8 bytes.  Sorted positions by
	 * construction, so V is the strata in order. */
	or_synth_random(seed, r, len);
	uint64_t n = n_edits < len ? n_edits : len;
	if (n == 0) {
		memcpy(v, r, len);
		return len;
	}
	uint64_t s = seed ^ SHIFT_SALT, S = len / n;
	size_t o = 0;
	for (uint64_t e = 0; e < n; e++) {
		uint64_t a = e * S, b = e + 1 == n ? len : (e + 1) * S;
		uint64_t h1 = or_splitmix64_at(s, 3 * e + 1), h2 = or_splitmix64_at(s, 3 * e + 2),
		         h3 = or_splitmix64_at(s, 3 * e + 3);
		uint64_t pos = a + h1 % (b - a), u = h2 % 100, k = 1 + (h2 >> 32) % 8;
		memcpy(v + o, r + a, pos - a);
		o += pos - a;
		if (2 * u < indel_pct) {             /* insertion before pos */
			for (uint64_t i = 0; i < k; i++) v[o++] = (uint8_t)(h3 >> (8 * i));
			memcpy(v + o, r + pos, b - pos);
			o += b - pos;
		} else if (u < indel_pct) {          /* deletion of k bytes at pos */
			if (k > b - pos) k = b - pos;
			memcpy(v + o, r + pos + k, b - pos - k);
			o += b - pos - k;
		} else {                             /* substitution */
			v[o++] = (uint8_t)h3;
			memcpy(v + o, r + pos + 1, b - pos - 1);
			o += b - pos - 1;
		}
	}
	return o;
}

#define TRANS_SALT 0x5851F42D4C957F2DULL

size_t or_synth_transpose(uint64_t seed, uint32_t nb, uint32_t mean,
                          uint32_t pct, uint8_t *r, uint8_t *v, size_t cap)
{
	/* tests/gen_transpositions.py:_gen_sizes/_gen_perm/main with a
	 * splitmix stream in place of random.Random(42) */
	uint64_t s = seed ^ TRANS_SALT, k = 1;
	uint32_t lo = mean / 2 ? mean / 2 : 1, hi = mean * 3 / 2;
	uint32_t *sz = malloc(nb * sizeof(uint32_t));
	uint32_t *perm = malloc(nb * sizeof(uint32_t));
	uint32_t *idx = malloc(nb * sizeof(uint32_t));
	uint32_t *val = malloc(nb * sizeof(uint32_t));
	uint64_t *off = malloc((nb + 1) * sizeof(uint64_t));
	if (!sz || !perm || !idx || !val || !off) abort();
	for (uint32_t i = 0; i < nb; i++)
		sz[i] = lo + (uint32_t)(or_splitmix64_at(s, k++) % (hi - lo + 1));
	off[0] = 0;
	for (uint32_t i = 0; i < nb; i++) off[i + 1] = off[i] + sz[i];
	size_t total = off[nb];
	if (total > cap) total = 0;
	/* k = round(n * perm_pct / 100) with Python's round-half-to-even
	 * (gen_transpositions.py:143) */
	uint64_t kq = (uint64_t)nb * pct / 100, kr = (uint64_t)nb * pct % 100;
	uint32_t kk = (uint32_t)(kq + (kr > 50 || (kr == 50 && (kq & 1))));
	for (uint32_t i = 0; i < nb; i++) { perm[i] = i; idx[i] = i; }
	if (kk >= 2) {
		for (uint32_t j = 0; j < kk; j++) {   /* choose kk distinct slots */
			uint32_t t = j + (uint32_t)(or_splitmix64_at(s, k++) % (nb - j));
			uint32_t x = idx[j]; idx[j] = idx[t]; idx[t] = x;
		}
		for (uint32_t j = 0; j < kk; j++) val[j] = idx[j];
		for (uint32_t j = kk - 1; j > 0; j--) {   /* shuffle their values */
			uint32_t t = (uint32_t)(or_splitmix64_at(s, k++) % (j + 1));
			uint32_t x = val[j]; val[j] = val[t]; val[t] = x;
		}
		for (uint32_t j = 0; j < kk; j++) perm[idx[j]] = val[j];
	}
	if (total) {
		or_synth_random(seed, r, total);
		size_t o = 0;
		for (uint32_t i = 0; i < nb; i++) {
			memcpy(v + o, r + off[perm[i]], sz[perm[i]]);
			o += sz[perm[i]];
		}
	}
	free(sz); free(perm); free(idx); free(val); free(off);
	return total;
}
