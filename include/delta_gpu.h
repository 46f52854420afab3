/*
 * delta_gpu.h — C ABI of the MI355X-native delta codec (libdeltagpu.so).
 *
 * Drop-in boundary for the hot path of darrelllong/Delta-Compression:
 *
 *   reference chain (src/c/main.c:257-292)          this library
 *   ---------------------------------------------   ---------------------------
 *   delta_crc64_xz(R), delta_crc64_xz(V)            \
 *     (src/c/delta.h:294-322)                        \
 *   delta_diff(ALGO_ONEPASS|ALGO_CORRECTING, ...)     > dg_encode / dg_encode_batch /
 *     (src/c/correcting.c:499-519 -> onepass.c:32,   /  dg_encode_plan_run
 *      correcting.c:81)                             /
 *   delta_place_commands (src/c/apply.c:136-164)   /
 *   delta_encode(placed, false, |V|, src, dst)    /
 *     (src/c/encoding.c:39-90)
 *   delta_decode + delta_apply_placed(_inplace)     dg_decode / dg_decode_batch
 *     + CRC checks (encoding.c:111-178,
 *       apply.c:229-284, main.c:341-385)
 *   delta_crc64_xz (delta.h:294)                    dg_crc64_xz / dg_crc64_xz_batch_device
 *
 * Output bytes are identical to the reference's `delta encode` at the same
 * --seed-len / --table-size / --max-table (the DLT\x03 format of
 * src/c/encoding.c:39-90, README.md:125-149).
 *
 * Differences from the reference contract (src/c/delta.h), by design:
 *   - every call returns a dg_status_t instead of abort()/exit(1)
 *     (delta.h:44-79, encoding.c:119-172);
 *   - no per-command allocations: results are arenas with explicit frees;
 *   - thread-safe: constant tables are built at context creation;
 *   - DELTA_OPT_SPLAY (delta.h:222) and ALGO_GREEDY are rejected with
 *     DG_ERR_UNSUPPORTED (splay changes correcting output; greedy is outside
 *     the GPU hot path);
 *   - inputs of 4 GiB or more are rejected (DG_ERR_TOO_LARGE): the format's
 *     u32 fields would silently truncate them (encoding.c:63,72-78).
 *
 * All device pointers are plain HIP device pointers; `stream` is a
 * hipStream_t passed as void* (NULL = the context's own stream).  No C++ or
 * torch types cross this boundary.
 */
#ifndef DELTA_GPU_H
#define DELTA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DG_ABI_VERSION 3

/* Defaults mirror src/c/delta.h:21-35. */
#define DG_SEED_LEN        16
#define DG_TABLE_SIZE      1048573UL
#define DG_MAX_TABLE_SIZE  1073741827UL
#define DG_BUF_CAP         256
#define DG_HEADER_SIZE     25
#define DG_CRC_SIZE        8

typedef enum {
	DG_OK              = 0,
	DG_ERR_INVALID_ARG = 1,
	DG_ERR_UNSUPPORTED = 2,   /* greedy, --splay, --inplace encode */
	DG_ERR_TOO_LARGE   = 3,   /* a buffer >= 4 GiB */
	DG_ERR_NO_DEVICE   = 4,
	DG_ERR_HIP         = 5,
	DG_ERR_NOMEM       = 6,
	DG_ERR_CAPACITY    = 7,   /* output arena too small */
	DG_ERR_MALFORMED   = 8,   /* not a delta / truncated / bad command */
	DG_ERR_SRC_CRC     = 9,   /* reference does not match src_crc */
	DG_ERR_DST_CRC     = 10,  /* reconstructed output does not match dst_crc */
	DG_ERR_TABLE_POOL  = 11,  /* onepass: no work table came free within the
	                             wait bound (more long-epoch pairs in flight than
	                             tables; raise DG_LIMIT_TABLE_POOL_BYTES) */
	DG_ERR_INTERNAL    = 12   /* a device-side invariant failed (a library bug:
	                             segment list overflow, a member chain that ran
	                             out of members, serialiser size disagreement) */
} dg_status_t;

/* Numbering matches delta_algorithm_t (src/c/delta.h:85). */
typedef enum {
	DG_ALGO_GREEDY     = 0,
	DG_ALGO_ONEPASS    = 1,
	DG_ALGO_CORRECTING = 2
} dg_algorithm_t;

/* Option bits of delta_flags_t (src/c/delta.h:220-224). */
#define DG_OPT_VERBOSE 0
#define DG_OPT_SPLAY   1
#define DG_OPT_INPLACE 2
/* bit index of the in-place cycle policy for DG_OPT_INPLACE encodes
 * (main.c --policy): clear = localmin, set = constant (delta.h:86) */
#define DG_OPT_POLICY_CONSTANT 3

/* Layout- and meaning-identical to delta_diff_options_t (src/c/delta.h:248-257):
 * p = seed length, q = hash table size floor (--table-size), buf_cap =
 * correcting lookback capacity, max_table = correcting table ceiling. */
typedef struct {
	size_t   p;
	size_t   q;
	size_t   buf_cap;
	size_t   max_table;
	uint64_t flags;
} dg_diff_options_t;

/* DELTA_DIFF_OPTIONS_DEFAULT (src/c/delta.h:256-257). */
void dg_diff_options_default(dg_diff_options_t *opts);

/* A delta / output buffer; layout-identical to delta_buffer_t
 * (src/c/delta.h:331-334).  Free with dg_buffer_free. */
typedef struct {
	uint8_t *data;
	size_t   len;
} dg_buffer_t;

void dg_buffer_free(dg_buffer_t *buf);

/* ── context ───────────────────────────────────────────────────────────── */

typedef struct dg_context dg_context_t;

/* Binds a HIP device (device < 0: the current device) and creates one HIP
 * stream plus the constant tables.  Fails with DG_ERR_NO_DEVICE when no GPU
 * is visible: there is no CPU fallback. */
int  dg_context_create(int device, dg_context_t **out);
void dg_context_destroy(dg_context_t *ctx);
/* Current hipStream_t of the context, as void*. */
void *dg_context_stream(dg_context_t *ctx);
const char *dg_status_string(int status);
/* Last error text recorded on this context (never NULL). */
const char *dg_last_error(const dg_context_t *ctx);
int dg_abi_version(void);

/* Resource limits of a context; they apply to plans created afterwards.
 *   DG_LIMIT_TABLE_POOL_BYTES: device bytes for the onepass work tables that
 *     epochs longer than 256 steps spill into (one table = 16 B x q, held by
 *     a pair from its first long epoch to its end).  0 = automatic: enough
 *     tables for every resident wave, capped at 4 GiB (at least 1 GiB).
 *     Pairs beyond the table count wait for one; a wait longer than the
 *     bound ends the pair with DG_ERR_TABLE_POOL. */
#define DG_LIMIT_TABLE_POOL_BYTES 0
/*   DG_LIMIT_ONEPASS_MEMBERS: how onepass plans (seed length 16, 16-byte
 *     aligned pairs) run the epoch chain.  0 = automatic, 1 = verified
 *     diagonal members first (the chain walks only unverified members), 2 =
 *     the plain per-pair chain.  Output bytes are identical in every mode.
 *     Member mode needs about 1.3 B of extra device memory per position of
 *     min(|R|, |V|) (20 B for each of 129 member slots per 2 KiB chunk); when
 *     that allocation fails in automatic mode the plan falls back to the
 *     plain chain, and only a forced mode 1 returns DG_ERR_NOMEM. */
#define DG_LIMIT_ONEPASS_MEMBERS 1
int dg_context_set_limit(dg_context_t *ctx, int limit, uint64_t value);

/* ── batched, device-resident encode: the hot path ───────────────────────
 *
 * A batch is N independent (reference, version) pairs laid out in two device
 * arenas.  A plan fixes the pair geometry and options once (table sizes,
 * worst-case command capacity, work buffers, CRC segmentation) so that
 * dg_encode_plan_run is pure device work on one stream (graph-capturable:
 * no allocation, no host synchronisation).
 *
 * Output: one packed arena.  Pair i's delta occupies
 * d_out[d_offsets[i] .. d_offsets[i+1]) and is byte-identical to the
 * reference's `delta encode <algo> R_i V_i` output.  d_status[i] is a
 * dg_status_t.  d_offsets has N+1 entries (d_offsets[N] = total bytes).
 */
typedef struct {
	uint64_t r_off;   /* byte offset of R_i in the reference arena */
	uint64_t r_len;
	uint64_t v_off;   /* byte offset of V_i in the version arena */
	uint64_t v_len;
} dg_pair_t;

typedef struct dg_encode_plan dg_encode_plan_t;

int dg_encode_plan_create(dg_context_t *ctx, dg_algorithm_t algo,
                          const dg_pair_t *pairs /* host */, uint32_t n_pairs,
                          const dg_diff_options_t *opts,
                          dg_encode_plan_t **out);
/* Upper bound of the packed output (bytes): size d_out at least this. */
uint64_t dg_encode_plan_output_bound(const dg_encode_plan_t *plan);
uint32_t dg_encode_plan_num_pairs(const dg_encode_plan_t *plan);
/* Table size q actually used for pair i (onepass.c:61-62 /
 * correcting.c:116-123 sizing). */
uint64_t dg_encode_plan_table_size(const dg_encode_plan_t *plan, uint32_t i);
int dg_encode_plan_run(dg_encode_plan_t *plan,
                       const uint8_t *d_ref_arena, const uint8_t *d_ver_arena,
                       uint8_t *d_out, uint64_t out_cap,
                       uint64_t *d_offsets, int32_t *d_status,
                       void *stream);
/* Optional per-stage timing with HIP events on the streams the kernels run on
 * (the CRC kernels run on a plan-owned side stream forked from / joined to
 * the run stream).  dg_encode_plan_set_timing(plan, slots) with slots > 0
 * makes every run record its events into one of `slots` event sets (a ring;
 * 0 disables) and resets the run count; dg_encode_plan_stage_times fills up to
 * `n` stage durations (ms), averaged over the last min(runs, slots) runs, and
 * their names ("crc64", "diff", "scan", "serialize+join", "total", "members";
 * "members" is the member kernel alone, inside "diff", 0 in plain chain mode).  Returns
 * the number of stages.  No host synchronisation happens until stage_times.
 * Correcting plans add "corr_build" and "corr_scan" (the R-index build and
 * the V scan).  dg_encode_plan_set_timing_mode(plan, DG_TIMING_DOMINANT)
 * records only the events around the dominant kernel(s) — the member kernel
 * ("members"), the correcting build and scan ("corr_build", "corr_scan",
 * "diff") or the onepass kernel ("diff") — and stage_times reports those
 * only: each timing event costs the run stream a few microseconds, so a
 * throughput measurement records as few as it needs.
 * dg_encode_plan_set_timing_every(plan, k), k >= 1: only every k-th run
 * (the first after set_timing, then every k-th) records its events; the
 * ring then holds the last `slots` recorded runs.  Resets the run count. */
#define DG_TIMING_ALL      0
#define DG_TIMING_DOMINANT 1
int dg_encode_plan_set_timing(dg_encode_plan_t *plan, int slots);
int dg_encode_plan_set_timing_mode(dg_encode_plan_t *plan, int mode);
int dg_encode_plan_set_timing_every(dg_encode_plan_t *plan, int every);
int dg_encode_plan_stage_times(dg_encode_plan_t *plan, float *ms,
                               const char **names, int n);
/* --verbose counters (correcting plans): d_stats = 8 u64 per pair in device
 * memory, zeroed by the caller (NULL = off, the default): seeds passing the
 * build's checkpoint test, slots stored, scan checkpoints, fingerprint
 * mismatches, byte mismatches, matches, the checkpoint class k, passing
 * seeds whose slot is inside the table (the dbg_* counters of
 * correcting.c:95-98).  dg_encode / dg_encode_batch with DG_OPT_VERBOSE set
 * print the reference's diagnostic lines to stderr from these and the delta
 * (onepass.c:64-69, 277-285; correcting.c:137-152, 200-214, 470-485). */
int dg_encode_plan_set_stats(dg_encode_plan_t *plan, uint64_t *d_stats);
/* How the plan runs (bit flags): DG_PLAN_MEMBERS = onepass through verified
 * diagonal members (DG_LIMIT_ONEPASS_MEMBERS). */
#define DG_PLAN_MEMBERS 1u
uint32_t dg_encode_plan_flags(const dg_encode_plan_t *plan);
/* The plan's runs so far by how they ran: in member mode, and as a plain plan
 * (every run of a plan without member mode; in automatic member mode, the
 * runs of a batch whose every pair the last completed member-mode run routed
 * to the plain chain, between member-mode probes every 16th run).  The output
 * bytes are the same either way.  Returns DG_OK or DG_ERR_INVALID_ARG. */
int dg_encode_plan_run_modes(const dg_encode_plan_t *plan, uint64_t *member_runs, uint64_t *plain_runs);
/* Per-pair command statistics of the last run (device pointers owned by the
 * plan, valid until the next run): number of COPY commands and delta size. */
const uint32_t *dg_encode_plan_copy_counts_device(const dg_encode_plan_t *plan);
void dg_encode_plan_destroy(dg_encode_plan_t *plan);

/* ── host-buffer convenience (end-to-end; includes PCIe transfers) ──────── */

/* One pair: the chain of src/c/main.c:257-292, R and V in host memory.
 * out->data is malloc'd; free with dg_buffer_free. */
int dg_encode(dg_context_t *ctx, dg_algorithm_t algo,
              const uint8_t *r, size_t r_len,
              const uint8_t *v, size_t v_len,
              const dg_diff_options_t *opts, dg_buffer_t *out);

/* N pairs in host memory: pinned staging -> device -> host. outs[i] is
 * malloc'd per pair; status[i] per pair (may be NULL). */
int dg_encode_batch(dg_context_t *ctx, dg_algorithm_t algo,
                    const uint8_t *const *r, const size_t *r_len,
                    const uint8_t *const *v, const size_t *v_len,
                    uint32_t n_pairs, const dg_diff_options_t *opts,
                    dg_buffer_t *outs, int32_t *status);

/* ── Pipelined host-to-host batch encode ──────────
 * The reference's encode reads R and V from host files and writes the delta
 * back (main.c:33-121, 249-292).  For n pairs in host arenas h_ref / h_ver,
 * laid out by pairs[] as for dg_encode_plan_create, this cuts the batch into
 * chunks of consecutive pairs of about chunk_bytes of input each (0: 256 MiB)
 * and keeps two chunks in flight on two streams: the H2D copy of chunk i+1
 * and the D2H copy of chunk i-1's exact delta bytes overlap the encode of
 * chunk i.  The deltas land in h_out (out_cap bytes) packed in pair order,
 * delta i at out_offsets[i] .. out_offsets[i+1] (host, n+1 entries); status[i]
 * per pair (host, may be NULL).  Arenas and h_out from dg_host_alloc (pinned)
 * are copied directly (keeping the arena's 16-byte phase); other host memory
 * goes through pinned staging that the context keeps between calls, which
 * places every pair's streams at 16-byte offsets on the device (so unaligned
 * pageable layouts still take the LDS-window kernels).  Device buffers and
 * plans are kept too: a chunk with the same layout, options and context
 * limits as the slot's last one reuses its plan.
 * Returns DG_OK (per-pair failures in status), DG_ERR_CAPACITY when h_out is
 * too small (the pairs that did not fit get status DG_ERR_CAPACITY and
 * out_offsets equal to the bytes written so far), or the first failure when
 * status is NULL. */
int dg_encode_pipelined(dg_context_t *ctx, dg_algorithm_t algo,
                        const uint8_t *h_ref, const uint8_t *h_ver,
                        const dg_pair_t *pairs, uint32_t n_pairs,
                        const dg_diff_options_t *opts, uint64_t chunk_bytes,
                        uint8_t *h_out, uint64_t out_cap,
                        uint64_t *out_offsets, int32_t *status);

/* The same host-to-host encode sharded over several devices (one context
 * per device, e.g. the 8 MI355X of a node): contiguous pair
 * ranges balanced by sum(|R|+|V|), one host thread per context running
 * dg_encode_pipelined on its range into a private buffer (sized by the
 * range's output bound), then the ranges' deltas are packed into h_out in
 * pair order: when everything fits, h_out, out_offsets and status read
 * exactly as the one-device call leaves them.  Under a tight out_cap the
 * pairs are packed up to the first one that does not fit, and it and every
 * later pair get DG_ERR_CAPACITY (a pair the device failed keeps its own
 * status) with out_offsets at the bytes written (the one-device call stops
 * at a chunk boundary instead).  No bytes move between devices.  n_ctx == 1
 * is dg_encode_pipelined.  Returns as dg_encode_pipelined (the first failing
 * range's code when status is NULL; a range that failed as a whole returns
 * its code even when status is given).  UNVERIFIED on two or more physical
 * devices: the multi-device path has only run with several contexts on one
 * device (tests/test_gpu_pipelined.py); the caller's current device is
 * restored on return. */
int dg_encode_pipelined_multi(dg_context_t *const *ctxs, uint32_t n_ctx, dg_algorithm_t algo,
                              const uint8_t *h_ref, const uint8_t *h_ver,
                              const dg_pair_t *pairs, uint32_t n_pairs,
                              const dg_diff_options_t *opts, uint64_t chunk_bytes,
                              uint8_t *h_out, uint64_t out_cap,
                              uint64_t *out_offsets, int32_t *status);

/* Pinned (page-locked) host memory for the arenas and outputs above. */
int  dg_host_alloc(dg_context_t *ctx, uint64_t bytes, void **out);
void dg_host_free(void *p);

/* ── CRC-64/XZ (delta.h:294-322), computed on the device ──────────────── */

typedef struct {
	uint64_t off;   /* byte offset into the arena */
	uint64_t len;
} dg_span_t;

/* CRC of a host buffer (copied to the device).  out = 8 bytes big-endian. */
int dg_crc64_xz(dg_context_t *ctx, const uint8_t *data, size_t len,
                uint8_t out[DG_CRC_SIZE]);
/* CRC of N spans of one device arena; d_crc receives N u64 values (the CRC
 * register value, not byte-swapped). spans are host descriptors. */
int dg_crc64_xz_batch_device(dg_context_t *ctx, const uint8_t *d_arena,
                             const dg_span_t *spans, uint32_t n,
                             uint64_t *d_crc, void *stream);

/* ── decode + apply + CRC verify (encoding.c:111-178, apply.c:229-284,
 *    main.c:341-385) ────────────────────────────────────────────────────── */

/* Decode one delta against R (host buffers).  Returns DG_OK,
 * DG_ERR_MALFORMED, DG_ERR_SRC_CRC or DG_ERR_DST_CRC (the reference's exit
 * paths); ignore_hash skips both CRC checks (main.c:330-333).  On DG_OK and
 * on DG_ERR_DST_CRC, *out holds the decoded bytes (the reference writes the
 * output before its post-check fails, main.c:374-383): free it with
 * dg_buffer_free in both cases. */
int dg_decode(dg_context_t *ctx, const uint8_t *r, size_t r_len,
              const uint8_t *delta, size_t delta_len, int ignore_hash,
              dg_buffer_t *out);

/* Batched device decode: stream i is d_delta[delta_off[i] .. +delta_len[i])
 * applied to d_ref[ref spans i]; output written to d_out at out_off[i]
 * (capacity out_cap[i] >= version_size, and >= |R| for in-place deltas).
 * d_status[i] receives a dg_status_t. Descriptors are host arrays.  The
 * output bytes the descriptors name must not overlap the reference or delta
 * bytes they name (the in-place replay runs in the output buffer after R is
 * copied into it, and the source CRC is computed from d_ref after the
 * apply): an overlapping call returns DG_ERR_INVALID_ARG and writes nothing.
 * The output is written even when a stream's source CRC check fails. */
typedef struct {
	uint64_t ref_off, ref_len;
	uint64_t delta_off, delta_len;
	uint64_t out_off, out_cap;
} dg_decode_desc_t;

int dg_decode_batch_device(dg_context_t *ctx, const uint8_t *d_ref,
                           const uint8_t *d_delta,
                           const dg_decode_desc_t *descs, uint32_t n,
                           int ignore_hash, uint8_t *d_out,
                           uint64_t *d_out_len, int32_t *d_status,
                           void *stream);

/* Plan form of the batched decode (C5): descriptors uploaded once;
 * dg_decode_plan_run is one kernel launch (no host synchronisation,
 * graph-capturable) that parses and applies every stream and then computes
 * the CRC-64/XZ of its reference and of its output (length from the delta
 * header) and checks both against the header.  Status precedence per
 * stream: DG_ERR_MALFORMED / DG_ERR_CAPACITY, then DG_ERR_SRC_CRC, then
 * DG_ERR_DST_CRC (main.c:335-385).  Arena base pointers d_ref and d_out must
 * be 16-byte aligned.  Timing as for the encode plan, with one stage,
 * "decode" (the kernel, CRC checks included). */
typedef struct dg_decode_plan dg_decode_plan_t;
int dg_decode_plan_create(dg_context_t *ctx, const dg_decode_desc_t *descs,
                          uint32_t n, int ignore_hash,
                          dg_decode_plan_t **out);
int dg_decode_plan_run(dg_decode_plan_t *plan, const uint8_t *d_ref,
                       const uint8_t *d_delta, uint8_t *d_out,
                       uint64_t *d_out_len, int32_t *d_status, void *stream);
int dg_decode_plan_set_timing(dg_decode_plan_t *plan, int slots);
int dg_decode_plan_set_timing_every(dg_decode_plan_t *plan, int every);
int dg_decode_plan_stage_times(dg_decode_plan_t *plan, float *ms,
                               const char **names, int n);
void dg_decode_plan_destroy(dg_decode_plan_t *plan);

/* ── delta inspection (host parse, src/c/main.c:402-425) ─────────────── */

typedef struct {
	int      inplace;
	uint64_t version_size;
	uint8_t  src_crc[DG_CRC_SIZE];
	uint8_t  dst_crc[DG_CRC_SIZE];
	uint64_t num_commands, num_copies, num_adds;
	uint64_t copy_bytes, add_bytes;
} dg_delta_info_t;

int dg_delta_info(const uint8_t *delta, size_t len, dg_delta_info_t *info);

/* ── command lists (delta.h:94-137, 280-284, 326-368) ───────────────────
 *
 * For callers that work between the algorithm and the container, as in
 * HOWTO.md:426-464 (delta_diff -> delta_place_commands -> delta_encode;
 * delta_decode -> delta_apply_placed).  One record type serves both the
 * algorithm's commands (delta_command_t: COPY offset = src, ADD data) and the
 * placed ones (delta_placed_command_t: + dst).  Lengths and offsets are in
 * bytes; ADD data point into storage owned by the list. */
#define DG_CMD_COPY 0   /* == CMD_COPY, PCMD_COPY */
#define DG_CMD_ADD  1   /* == CMD_ADD, PCMD_ADD */
typedef struct {
	uint32_t       tag;      /* DG_CMD_COPY or DG_CMD_ADD */
	uint64_t       src;      /* COPY: offset in R (0 for ADD) */
	uint64_t       dst;      /* offset in V */
	uint64_t       length;
	const uint8_t *data;     /* ADD: `length` literal bytes (NULL for COPY) */
} dg_placed_command_t;
typedef struct {
	dg_placed_command_t *data;
	size_t               len;
	void                *storage;   /* owns data and the ADD bytes */
} dg_commands_t;
void dg_commands_free(dg_commands_t *cmds);

/* delta_diff(algo, R, V, opts) followed by delta_place_commands (apply.c:
 * 136-164): the commands of the delta dg_encode produces, in algorithm order
 * with sequential dst (so dropping dst gives delta_diff's list).  Runs on the
 * GPU; DG_OPT_INPLACE in opts->flags is ignored (in-place conversion is
 * dg_make_inplace on an encoded delta). */
int dg_diff(dg_context_t *ctx, dg_algorithm_t algo,
            const uint8_t *r, size_t r_len, const uint8_t *v, size_t v_len,
            const dg_diff_options_t *opts, dg_commands_t *out);
/* delta_decode (encoding.c:111-178): the placed commands of a delta in stream
 * order, and its header (hdr may be NULL; it receives dg_delta_info's
 * summary).  DG_ERR_MALFORMED where the reference exits with "not a delta
 * file" / "truncated ..." / "unknown command type".  Host only. */
int dg_delta_decode(const uint8_t *delta, size_t len, dg_commands_t *out,
                    dg_delta_info_t *hdr);
/* delta_encode (encoding.c:39-90): placed commands -> DLT\x03 bytes,
 * out->data malloc'd.  Offsets, lengths and version_size of 4 GiB or more
 * (which the format's u32 fields cannot hold) give DG_ERR_INVALID_ARG.  Host
 * only. */
int dg_encode_commands(const dg_placed_command_t *cmds, size_t n, int inplace,
                       uint64_t version_size, const uint8_t src_crc[DG_CRC_SIZE],
                       const uint8_t dst_crc[DG_CRC_SIZE], dg_buffer_t *out);

/* ── in-place conversion (host; src/c/inplace.c:272-736) ───────────────────
 *
 * Converts a standard delta against R into an in-place delta: the chain of
 * main.c `inplace` (main.c:427-480) = delta_decode -> delta_unplace_commands
 * -> delta_make_inplace(policy) -> delta_encode(inplace = true), byte for
 * byte.  A delta that is already in-place is returned unchanged
 * (stats->already_inplace = 1).  Pure host code: no context, no GPU.  The
 * encoders produce in-place deltas by running this on their output
 * (dg_encode / dg_encode_batch with DG_OPT_INPLACE, policy from
 * dg_diff_options_t.flags bit DG_OPT_POLICY_CONSTANT). */
#define DG_POLICY_LOCALMIN 0
#define DG_POLICY_CONSTANT 1
typedef struct {
	int      already_inplace;
	uint64_t num_copies, num_adds;
	uint64_t copy_bytes, add_bytes;
} dg_inplace_stats_t;

int dg_make_inplace(const uint8_t *r, size_t r_len, const uint8_t *delta,
                    size_t delta_len, int policy, dg_buffer_t *out,
                    dg_inplace_stats_t *stats);

/* ── synthetic batch generators (bench / test inputs, on the device) ─────
 * Workload definitions in DESIGN.md ("Synthetic inputs"); the oracle's
 * or_synth_* functions produce the same bytes on the CPU. */
int dg_synth_edit_pairs_device(dg_context_t *ctx, uint8_t *d_ref,
                               uint8_t *d_ver, uint32_t n_pairs,
                               uint64_t pair_len, uint64_t seed_base,
                               uint64_t n_edits, void *stream);
/* C4 transposition pairs (tests/gen_transpositions.py _gen_sizes/_gen_perm
 * with a per-pair splitmix64 seed seed_base + i): pair i has
 * num_blocks = 8 + (i mod 57) blocks of mean size target_len / num_blocks,
 * pct % of them permuted.  Pairs are packed at 16-byte aligned offsets,
 * written to pairs[n].  With d_ref == NULL only the layout is computed and
 * *ref_bytes / *ver_bytes receive the arena sizes to allocate. */
int dg_synth_transpose_pairs_device(dg_context_t *ctx, uint64_t seed_base,
                                    uint32_t n_pairs, uint64_t target_len,
                                    uint32_t pct, dg_pair_t *pairs,
                                    uint64_t *ref_bytes, uint64_t *ver_bytes,
                                    uint8_t *d_ref, uint8_t *d_ver,
                                    void *stream);
/* Shift pairs (a stated extra workload beside C3: edits that move the
 * diagonal): R_i = the splitmix64 stream of seed seed_base + i, pair_len
 * bytes; V_i = R_i with n_edits edits, one per equal stratum of R_i,
 * indel_pct % of them insertions or deletions of 1..8 bytes (half each), the
 * rest byte substitutions (oracle or_synth_shift).  Layout and the
 * d_ref == NULL protocol as for dg_synth_transpose_pairs_device. */
int dg_synth_shift_pairs_device(dg_context_t *ctx, uint64_t seed_base,
                                uint32_t n_pairs, uint64_t pair_len,
                                uint64_t n_edits, uint32_t indel_pct,
                                dg_pair_t *pairs, uint64_t *ref_bytes,
                                uint64_t *ver_bytes, uint8_t *d_ref,
                                uint8_t *d_ver, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* DELTA_GPU_H */
