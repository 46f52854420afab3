/*
 * cli_main.c — `delta` command line over libdeltagpu.so.
 *
 * Same argv surface and stdout report lines as the reference CLI
 * (src/c/main.c:158-180 usage, :189-321 encode, :323-400 decode,
 * :402-425 info), so scripts that parse it (tests/transposition-benchmark.sh
 * :50-62) keep working.  All compute runs on the GPU through the C ABI.
 *
 *   delta encode <onepass|correcting> <ref> <ver> <delta> [options]
 *   delta decode <ref> <delta> <output> [--ignore-hash]
 *   delta info <delta>
 *   delta inplace <ref> <delta_in> <delta_out> [--policy localmin|constant]
 *
 * --inplace / inplace run the CRWI conversion on the host (dg_make_inplace,
 * main.c:279-283 and :427-480).  Not provided by this build (exit 1 with a
 * message): the greedy algorithm and --splay.
 */
#include <errno.h>
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "delta_gpu.h"

static uint8_t *read_file(const char *path, size_t *len)
{
	FILE *f = fopen(path, "rb");
	if (!f) {
		fprintf(stderr, "Error opening %s: %s\n", path, strerror(errno));
		exit(1);
	}
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	fseek(f, 0, SEEK_SET);
	uint8_t *b = malloc(n > 0 ? (size_t)n : 1);
	if (!b || (n > 0 && fread(b, 1, (size_t)n, f) != (size_t)n)) {
		fprintf(stderr, "Error reading %s\n", path);
		exit(1);
	}
	fclose(f);
	*len = (size_t)n;
	return b;
}

static void write_file(const char *path, const uint8_t *d, size_t n)
{
	FILE *f = fopen(path, "wb");
	if (!f) {
		fprintf(stderr, "Error writing %s: %s\n", path, strerror(errno));
		exit(1);
	}
	if (n && fwrite(d, 1, n, f) != n) {
		fprintf(stderr, "Error writing %s\n", path);
		exit(1);
	}
	fclose(f);
}

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec / 1e9;
}

static void hex(FILE *f, const uint8_t *b, size_t n)
{
	for (size_t i = 0; i < n; i++) fprintf(f, "%02x", b[i]);
}

static size_t parse_size_suffix(const char *s)   /* main.c:145-154 */
{
	char *end;
	unsigned long long n = strtoull(s, &end, 10);
	if (*end == 'k' || *end == 'K') n *= 1000ULL;
	else if (*end == 'M' || *end == 'm') n *= 1000000ULL;
	else if (*end == 'B' || *end == 'b') n *= 1000000000ULL;
	return (size_t)n;
}

static void usage(void)
{
	fprintf(stderr,
	    "Usage:\n"
	    "  delta encode <algorithm> <ref> <ver> <delta> [options]\n"
	    "  delta decode <ref> <delta> <output> [--ignore-hash]\n"
	    "  delta info <delta>\n"
	    "  delta inplace <ref> <delta_in> <delta_out> [--policy P]\n"
	    "\n"
	    "Algorithms: onepass, correcting (MI355X)\n"
	    "\n"
	    "Options:\n"
	    "  --seed-len N     Seed length (default %d)\n"
	    "  --table-size N   Hash table size floor (default %lu)\n"
	    "  --max-table N    Max hash table size, k/M/B suffix ok (default %lu)\n"
	    "  --inplace        Produce in-place delta\n"
	    "  --policy P       Cycle policy: localmin (default), constant\n"
	    "  --verbose        Print diagnostics\n",
	    DG_SEED_LEN, (unsigned long)DG_TABLE_SIZE, (unsigned long)DG_MAX_TABLE_SIZE);
	exit(1);
}

static dg_context_t *ctx_or_die(void)
{
	dg_context_t *ctx = NULL;
	int rc = dg_context_create(-1, &ctx);
	if (rc) {
		fprintf(stderr, "delta: no usable GPU (%s)\n", dg_status_string(rc));
		exit(1);
	}
	return ctx;
}

static int cmd_encode(int argc, char **argv)
{
	if (argc < 6) usage();
	const char *algo_str = argv[2], *ref_path = argv[3], *ver_path = argv[4], *delta_path = argv[5];
	dg_algorithm_t algo;
	if (strcmp(algo_str, "onepass") == 0) algo = DG_ALGO_ONEPASS;
	else if (strcmp(algo_str, "correcting") == 0) algo = DG_ALGO_CORRECTING;
	else if (strcmp(algo_str, "greedy") == 0) {
		fprintf(stderr, "greedy is not provided by the MI355X build\n");
		return 1;
	} else {
		fprintf(stderr, "Unknown algorithm: %s\n", algo_str);
		return 1;
	}
	dg_diff_options_t o;
	dg_diff_options_default(&o);
	const char *policy_str = "localmin";
	static struct option lo[] = {
		{"seed-len", required_argument, NULL, 's'},
		{"table-size", required_argument, NULL, 't'},
		{"max-table", required_argument, NULL, 'x'},
		{"inplace", no_argument, NULL, 'i'},
		{"policy", required_argument, NULL, 'p'},
		{"verbose", no_argument, NULL, 'v'},
		{"splay", no_argument, NULL, 'y'},
		{NULL, 0, NULL, 0}};
	optind = 6;
	int opt;
	while ((opt = getopt_long(argc, argv, "", lo, NULL)) != -1) {
		switch (opt) {
		case 's': o.p = (size_t)atol(optarg); break;
		case 't': o.q = (size_t)atol(optarg); break;
		case 'x': o.max_table = parse_size_suffix(optarg); break;
		case 'v': o.flags |= 1ull << DG_OPT_VERBOSE; break;
		case 'i': o.flags |= 1ull << DG_OPT_INPLACE; break;
		case 'y':
			fprintf(stderr, "--splay is not provided by the MI355X build\n");
			return 1;
		case 'p':
			policy_str = optarg;
			if (strcmp(optarg, "constant") == 0) o.flags |= 1ull << DG_OPT_POLICY_CONSTANT;
			break;
		default: usage();
		}
	}
	if (o.p == 0) {
		fprintf(stderr, "error: --seed-len must be >= 1\n");
		return 1;
	}
	size_t rl, vl;
	uint8_t *r = read_file(ref_path, &rl), *v = read_file(ver_path, &vl);
	dg_context_t *ctx = ctx_or_die();
	dg_buffer_t d = {0};
	double t0 = now();
	int rc = dg_encode(ctx, algo, r, rl, v, vl, &o, &d);
	double t1 = now();
	if (rc) {
		fprintf(stderr, "delta: encode failed: %s (%s)\n", dg_status_string(rc), dg_last_error(ctx));
		return 1;
	}
	write_file(delta_path, d.data, d.len);
	dg_delta_info_t inf;
	dg_delta_info(d.data, d.len, &inf);
	if ((o.flags >> DG_OPT_INPLACE) & 1)
		printf("Algorithm:    %s + in-place (%s)\n", algo_str, policy_str);
	else
		printf("Algorithm:    %s\n", algo_str);
	printf("Reference:    %s (%zu bytes)\n", ref_path, rl);
	printf("Version:      %s (%zu bytes)\n", ver_path, vl);
	printf("Delta:        %s (%zu bytes)\n", delta_path, d.len);
	printf("Compression:  %.4f (delta/version)\n", vl == 0 ? 0.0 : (double)d.len / vl);
	printf("Commands:     %llu copies, %llu adds\n", (unsigned long long)inf.num_copies,
	       (unsigned long long)inf.num_adds);
	printf("Copy bytes:   %llu\n", (unsigned long long)inf.copy_bytes);
	printf("Add bytes:    %llu\n", (unsigned long long)inf.add_bytes);
	printf("Src CRC:      "); hex(stdout, inf.src_crc, 8); printf("\n");
	printf("Dst CRC:      "); hex(stdout, inf.dst_crc, 8); printf("\n");
	/* The reference times diff+place only (main.c:262-287); here the whole
	 * device chain incl. CRC and transfers is inside the window. */
	printf("Time:         %.3fs\n", t1 - t0);
	dg_buffer_free(&d);
	dg_context_destroy(ctx);
	free(r);
	free(v);
	return 0;
}

static int cmd_decode(int argc, char **argv)
{
	if (argc < 5) usage();
	const char *ref_path = argv[2], *delta_path = argv[3], *out_path = argv[4];
	int ignore = 0;
	for (int a = 5; a < argc; a++)
		if (strcmp(argv[a], "--ignore-hash") == 0) ignore = 1;
	size_t rl, dl;
	uint8_t *r = read_file(ref_path, &rl), *d = read_file(delta_path, &dl);
	dg_delta_info_t inf;
	if (dg_delta_info(d, dl, &inf) == DG_ERR_MALFORMED && (dl < DG_HEADER_SIZE || memcmp(d, "DLT\x03", 4))) {
		fprintf(stderr, "delta_decode: not a delta file\n");
		return 1;
	}
	dg_context_t *ctx = ctx_or_die();
	dg_buffer_t out = {0};
	uint8_t c[8];
	/* --ignore-hash: the checks still run, a mismatch only warns
	 * (main.c:342-356, :376-385) */
	if (ignore && dg_delta_info(d, dl, &inf) == DG_OK && dg_crc64_xz(ctx, r, rl, c) == DG_OK &&
	    memcmp(c, inf.src_crc, 8) != 0)
		fprintf(stderr, "warning: skipping source CRC check (--ignore-hash)\n");
	double t0 = now();
	int rc = dg_decode(ctx, r, rl, d, dl, ignore, &out);
	double t1 = now();
	if (rc == DG_ERR_SRC_CRC) {
		dg_crc64_xz(ctx, r, rl, c);
		fprintf(stderr, "source file does not match delta: expected ");
		hex(stderr, inf.src_crc, 8);
		fprintf(stderr, ", got ");
		hex(stderr, c, 8);
		fprintf(stderr, "\n");
		return 1;
	}
	if (rc == DG_ERR_DST_CRC) {
		/* the reference writes the output, then fails its post-check */
		write_file(out_path, out.data, out.len);
		fprintf(stderr, "output integrity check failed\n");
		return 1;
	}
	if (rc) {
		fprintf(stderr, "delta_decode: %s\n", dg_status_string(rc));
		return 1;
	}
	write_file(out_path, out.data, out.len);
	if (ignore && dg_crc64_xz(ctx, out.data, out.len, c) == DG_OK && memcmp(c, inf.dst_crc, 8) != 0)
		fprintf(stderr, "warning: skipping output CRC check (--ignore-hash)\n");
	printf("Format:       %s\n", inf.inplace ? "in-place" : "standard");
	printf("Reference:    %s (%zu bytes)\n", ref_path, rl);
	printf("Delta:        %s (%zu bytes)\n", delta_path, dl);
	printf("Output:       %s (%llu bytes)\n", out_path, (unsigned long long)inf.version_size);
	if (!ignore) {
		printf("Src CRC:      "); hex(stdout, inf.src_crc, 8); printf("  OK\n");
		printf("Dst CRC:      "); hex(stdout, inf.dst_crc, 8); printf("  OK\n");
	}
	printf("Time:         %.3fs\n", t1 - t0);
	dg_buffer_free(&out);
	dg_context_destroy(ctx);
	free(r);
	free(d);
	return 0;
}

static int cmd_info(int argc, char **argv)
{
	if (argc < 3) usage();
	size_t dl;
	uint8_t *d = read_file(argv[2], &dl);
	dg_delta_info_t inf;
	int rc = dg_delta_info(d, dl, &inf);
	if (rc) {
		fprintf(stderr, "delta_decode: %s\n",
		        (dl < DG_HEADER_SIZE || memcmp(d, "DLT\x03", 4)) ? "not a delta file" : dg_status_string(rc));
		return 1;
	}
	printf("Delta file:   %s (%zu bytes)\n", argv[2], dl);
	printf("Format:       %s\n", inf.inplace ? "in-place" : "standard");
	printf("Version size: %llu bytes\n", (unsigned long long)inf.version_size);
	printf("Src CRC:      "); hex(stdout, inf.src_crc, 8); printf("\n");
	printf("Dst CRC:      "); hex(stdout, inf.dst_crc, 8); printf("\n");
	printf("Commands:     %llu\n", (unsigned long long)inf.num_commands);
	printf("  Copies:     %llu (%llu bytes)\n", (unsigned long long)inf.num_copies,
	       (unsigned long long)inf.copy_bytes);
	printf("  Adds:       %llu (%llu bytes)\n", (unsigned long long)inf.num_adds,
	       (unsigned long long)inf.add_bytes);
	printf("Output size:  %llu bytes\n", (unsigned long long)(inf.copy_bytes + inf.add_bytes));
	free(d);
	return 0;
}

static int cmd_inplace(int argc, char **argv)   /* main.c:427-480 */
{
	if (argc < 5) usage();
	const char *ref_path = argv[2], *in_path = argv[3], *out_path = argv[4];
	int policy = DG_POLICY_LOCALMIN;
	const char *policy_str = "localmin";
	for (int a = 5; a < argc; a++)
		if (strcmp(argv[a], "--policy") == 0 && a + 1 < argc) {
			policy_str = argv[++a];
			if (strcmp(policy_str, "constant") == 0) policy = DG_POLICY_CONSTANT;
		}
	size_t rl, dl;
	uint8_t *r = read_file(ref_path, &rl), *d = read_file(in_path, &dl);
	dg_buffer_t o = {0};
	dg_inplace_stats_t st;
	double t0 = now();
	int rc = dg_make_inplace(r, rl, d, dl, policy, &o, &st);
	double t1 = now();
	if (rc) {
		fprintf(stderr, "delta_decode: %s\n",
		        (dl < DG_HEADER_SIZE || memcmp(d, "DLT\x03", 4)) ? "not a delta file" : dg_status_string(rc));
		return 1;
	}
	write_file(out_path, o.data, o.len);
	if (st.already_inplace) {
		printf("Delta is already in-place format; copied unchanged.\n");
	} else {
		printf("Reference:    %s (%zu bytes)\n", ref_path, rl);
		printf("Input delta:  %s (%zu bytes)\n", in_path, dl);
		printf("Output delta: %s (%zu bytes)\n", out_path, o.len);
		printf("Format:       in-place (%s)\n", policy_str);
		printf("Commands:     %llu copies, %llu adds\n", (unsigned long long)st.num_copies,
		       (unsigned long long)st.num_adds);
		printf("Copy bytes:   %llu\n", (unsigned long long)st.copy_bytes);
		printf("Add bytes:    %llu\n", (unsigned long long)st.add_bytes);
		printf("Time:         %.3fs\n", t1 - t0);
	}
	dg_buffer_free(&o);
	free(r);
	free(d);
	return 0;
}

int main(int argc, char **argv)
{
	if (argc < 2) usage();
	if (strcmp(argv[1], "encode") == 0) return cmd_encode(argc, argv);
	if (strcmp(argv[1], "decode") == 0) return cmd_decode(argc, argv);
	if (strcmp(argv[1], "info") == 0) return cmd_info(argc, argv);
	if (strcmp(argv[1], "inplace") == 0) return cmd_inplace(argc, argv);
	usage();
	return 1;
}
