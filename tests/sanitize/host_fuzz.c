/*
 * host_fuzz.c -- TEST ONLY.  Drives the host C code of libairscmp.so (the
 * cmp.h API, the cmp_gpu.h batch planner) and the CLI --params parser with
 * deterministic pseudo-random inputs, valid and invalid, under
 * -fsanitize=address,undefined (tests/sanitize/Makefile; device layer =
 * dev_stub.c).  Any sanitizer report aborts the run with a non-zero status;
 * tests/test_sanitize_cpu.py runs it.  usage: host_fuzz [iterations] [seed]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmp.h"
#include "cmp_errors.h"
#include "cmp_gpu.h"
#include "params_parse.h"

static uint64_t g_rng;
/* outcome counters: the run must reach the interesting paths */
extern unsigned long stub_walk_calls; /* dev_stub.c */
static uint32_t n_init_ok, n_frames_ok, n_frames_err, n_batch_ok, n_batch_frames_ok, n_batch_fallback_cap,
	n_stream_ok;

static uint32_t rnd(void)
{
	g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
	return (uint32_t)(g_rng >> 33);
}

static uint32_t pick(uint32_t n)
{
	return n ? rnd() % n : 0u;
}

static void timestamp(uint32_t *coarse, uint16_t *fine)
{
	static uint64_t t = 1000;
	t++;
	*coarse = (uint32_t)(t >> 16);
	*fine = (uint16_t)t;
}

static void random_params(struct cmp_params *p)
{
	static const uint32_t gs[] = { 0, 1, 2, 3, 7, 16, 32, 1055, 65535, 65536, 1u << 31 };
	const int valid = pick(4) != 0; /* mostly in range, so the compress paths run */
	memset(p, 0, sizeof(*p));
	p->primary_preprocessing = (enum cmp_preprocessing)(valid ? pick(3) : pick(6));
	p->primary_encoder_type = (enum cmp_encoder_type)(valid ? pick(3) : pick(4));
	p->primary_encoder_param = valid ? 1u + pick(pick(2) ? 64 : 65535) : gs[pick(11)];
	p->primary_encoder_outlier = pick(3) ? 1u + pick(70000) : gs[pick(11)];
	p->secondary_iterations = pick(3) ? pick(4) : pick(300);
	p->secondary_preprocessing = (enum cmp_preprocessing)(valid ? (pick(2) ? 3 : pick(3)) : pick(6));
	p->secondary_encoder_type = (enum cmp_encoder_type)(valid ? pick(3) : pick(4));
	p->secondary_encoder_param = valid ? 1u + pick(pick(2) ? 64 : 65535) : gs[pick(11)];
	p->secondary_encoder_outlier = 1u + pick(70000);
	p->model_rate = valid ? pick(17) : pick(20);
	p->checksum_enabled = (uint8_t)pick(2);
	p->uncompressed_fallback_enabled = (uint8_t)pick(2);
}

/* host API: initialise / compress / reset sequences on one context */
static void fuzz_host_api(void)
{
	struct cmp_params p;
	struct cmp_context ctx;
	uint32_t n = 1u + pick(pick(2) ? 64 : 5000), wbs, r, i, calls;
	uint8_t *work = NULL, *dst;
	int32_t *src = malloc((size_t)n * 4u);

	random_params(&p);
	for (i = 0; i < n; i++)
		src[i] = (int32_t)rnd();
	wbs = cmp_cal_work_buf_size(&p, 2u * n);
	if (!cmp_is_error(wbs) && wbs)
		work = malloc(wbs + 2u);
	r = cmp_initialise(pick(16) ? &ctx : NULL, &p, pick(16) ? work : NULL,
			   cmp_is_error(wbs) ? pick(100) : (pick(8) ? wbs : wbs + pick(3) - (wbs > 0)));
	n_init_ok += !cmp_is_error(r);
	{
		const uint32_t bound = cmp_compress_bound(2u * n);
		const uint32_t cap = cmp_is_error(bound) ? 64u : (pick(3) ? bound : pick(bound + 1u));
		dst = malloc(cap + 8u);
		calls = 1u + pick(6);
		for (i = 0; i < calls && !cmp_is_error(r); i++) {
			const uint32_t sz = pick(10) ? 2u * n : pick(4u * n + 1u);
			uint32_t out;
			switch (pick(3)) {
			case 0:
				out = cmp_compress_u16(&ctx, dst, cap, (const uint16_t *)src, sz);
				break;
			case 1:
				out = cmp_compress_i16(&ctx, dst, cap, (const int16_t *)src, sz);
				break;
			default:
				out = cmp_compress_i16_in_i32(&ctx, dst, cap, src, 2u * sz > 4u * n ? 4u * n : 2u * sz);
				break;
			}
			if (cmp_is_error(out))
				n_frames_err++;
			else
				n_frames_ok++;
			if (!pick(5))
				(void)cmp_reset(&ctx);
		}
		free(dst);
	}
	(void)cmp_get_error_message(r);
	if (!cmp_is_error(r))
		cmp_deinitialise(&ctx);
	free(work);
	free(src);
}

/* batch API: the planner, exact (step-by-step) and asynchronous modes */
static void fuzz_batch(struct cmp_gpu_engine *eng)
{
	struct cmp_params p;
	const uint32_t nctx = 1u + pick(4), fpc = 1u + pick(5), nf = nctx * fpc;
	const uint32_t type = pick(3), sb = type == 2 ? 4u : 2u;
	/* a quarter of the batches have whole 4096-sample segments: the MODEL
	 * walk path (airs_dev_walk) becomes applicable */
	const uint32_t n = pick(4) ? 1u + pick(pick(2) ? 40 : 3000) : 4096u * (1u + pick(2));
	struct cmp_context *ctx = calloc(nctx, sizeof(*ctx));
	uint8_t **work = calloc(nctx, sizeof(*work));
	uint32_t *sizes = calloc(nf, 4u), c, wbs, ok = 1;
	const uint64_t stride = ((uint64_t)n * sb + 15u) & ~15ull;
	uint8_t *src = malloc(stride * nf);
	uint32_t bound, cap;
	uint64_t dstride;
	uint8_t *dst;
	struct cmp_gpu_batch b;
	uint8_t *draws;

	random_params(&p);
	for (uint64_t i = 0; i < stride * nf; i++)
		src[i] = (uint8_t)rnd();
	bound = cmp_compress_bound(2u * n);
	cap = cmp_is_error(bound) ? 6u * n + 64u : bound;
	if (pick(2))
		cap = 16u + pick(cap);
	dstride = ((uint64_t)(cmp_is_error(bound) ? cap : bound) + 64u + 7u) & ~7ull;
	dst = malloc(dstride * nf);
	wbs = cmp_cal_work_buf_size(&p, 2u * n);
	for (c = 0; c < nctx; c++) {
		if (!cmp_is_error(wbs) && wbs)
			work[c] = calloc(wbs + 16u, 1);
		if (cmp_is_error(cmp_initialise(&ctx[c], &p, work[c], cmp_is_error(wbs) ? 0 : wbs)))
			ok = 0;
	}
	memset(&b, 0, sizeof(b));
	b.type = (enum cmp_gpu_sample_type)type;
	b.src = src;
	b.src_stride = stride;
	b.src_size = n * sb;
	b.dst = dst;
	b.dst_stride = dstride;
	b.dst_capacity = cap;
	b.sizes = sizes;
	b.flags = (pick(2) ? CMP_GPU_AUTO_RICE : 0u) | (pick(4) ? 0u : CMP_GPU_HOST_STEPPED) |
		  (pick(4) ? 0u : CMP_GPU_STEPWISE);
	draws = pick(2) ? calloc(nf, 1) : NULL;
	b.draws = draws;
	if (draws)
		b.flags |= CMP_GPU_REPORT_DRAWS;
	if (ok) {
		if (!cmp_is_error(cmp_gpu_compress(eng, ctx, nctx, fpc, &b))) {
			n_batch_ok++;
			for (c = 0; c < nf; c++)
				n_batch_frames_ok += !cmp_is_error(sizes[c]);
			n_batch_fallback_cap += p.uncompressed_fallback_enabled;
		}
		/* a second call continues the contexts' pass sequence */
		if (pick(2))
			(void)cmp_gpu_compress(eng, ctx, nctx, fpc, &b);
		(void)cmp_gpu_synchronize(eng);
	}
	/* payload-only stream over the batch's samples */
	{
		uint32_t ssz = 0;
		const uint32_t st = pick(5) ? type : pick(9), ssb = st == 2 ? 4u : 2u;
		/* at most the samples the batch buffer holds */
		const uint32_t sn = (uint32_t)(stride * nf / ssb);
		const uint32_t r = cmp_gpu_encode_stream(eng, (enum cmp_gpu_sample_type)st,
							 pick(20) ? src : NULL, pick(20) ? 1u + pick(sn) : 0,
							 (enum cmp_preprocessing)pick(5), (enum cmp_encoder_type)pick(4),
							 pick(8) ? 1u + pick(70) : pick(70000), pick(300), pick(20) ? dst : NULL,
							 pick(2) ? cap : (uint32_t)(dstride * nf), &ssz);
		n_stream_ok += !cmp_is_error(r) && !cmp_is_error(ssz);
	}
	/* argument errors */
	b.dst_stride = pick(2) ? 1 : dstride;
	b.src_size = pick(2) ? 3 : n * sb;
	(void)cmp_gpu_compress(eng, ctx, nctx, fpc, &b);
	(void)cmp_gpu_compress(eng, NULL, nctx, fpc, &b);
	(void)cmp_gpu_compress(eng, ctx, nctx, fpc, NULL);
	for (c = 0; c < nctx; c++)
		free(work[c]);
	free(work);
	free(ctx);
	free(sizes);
	free(src);
	free(dst);
	free(draws);
}

/* CLI --params grammar: valid strings, mutated and truncated */
static void fuzz_params_parse(void)
{
	static const char *base[] = {
		"primary_preprocessing=DIFF,primary_encoder_type=GOLOMB_ZERO,primary_encoder_param=32",
		"secondary_iterations=5, secondary_preprocessing = MODEL ,model_rate=11,checksum_enabled=true",
		"primary_encoder_outlier=107;secondary_encoder_type=GOLOMB_MULTI;secondary_encoder_param=0x10",
		"uncompressed_fallback_enabled=1 primary_preprocessing=IWT",
		"",
	};
	char buf[512], out[512];
	struct cmp_params p;
	const char *s = base[pick(5)];
	size_t len = strlen(s), i;

	memcpy(buf, s, len + 1);
	for (i = pick(4); i > 0 && len; i--)
		buf[pick((uint32_t)len)] = (char)(pick(3) ? 32 + pick(95) : pick(256));
	if (pick(3) == 0)
		buf[pick((uint32_t)len + 1u)] = '\0';
	memset(&p, 0, sizeof(p));
	(void)cmp_params_parse(buf, &p);
	(void)cmp_params_parse(NULL, &p);
	(void)cmp_params_to_string(out, pick(2) ? sizeof(out) : pick(40), &p);
}

/* cmp_gpu_gather_plan (cmp_gather.c): random node tables, every layout,
 * error values, frames without draws; outputs checked for shape */
static uint32_t n_plan_ok, n_plan_refused;
static void fuzz_gather_plan(void)
{
	const uint32_t world = 1u + rnd() % 8u, F = 1u + rnd() % 12u, layout = rnd() % 4u;
	const uint32_t fpc = 1u + rnd() % 4u, total = world * F;
	uint64_t *entries = malloc(total * 8u), *rank_bytes = malloc(world * 8u), *offsets = malloc(total * 8u);
	uint64_t *ids = malloc(total * 8u), sum = 0;
	uint32_t *sizes = malloc(total * 4u), i, r;

	for (i = 0; i < total; i++) {
		uint64_t sz = rnd() % 5000u, dr = rnd() % 4u;

		if (rnd() % 64u == 0u)
			sz = (uint64_t)(0u - 5u); /* an error value in a size slot */
		entries[i] = sz | dr << 32;
	}
	r = cmp_gpu_gather_plan(entries, world, F, layout, fpc, rnd(), rank_bytes, offsets, sizes,
				rnd() % 2u ? ids : NULL);
	if (cmp_is_error(r)) {
		n_plan_refused++;
	} else {
		n_plan_ok++;
		for (i = 0; i < world; i++)
			sum += rank_bytes[i];
		for (i = 0; i < total; i++)
			if ((offsets[i] & 7u) || offsets[i] + sizes[i] > sum)
				abort();
	}
	free(entries);
	free(rank_bytes);
	free(offsets);
	free(ids);
	free(sizes);
}

int main(int argc, char **argv)
{
	const uint32_t iters = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 0) : 3000u;
	struct cmp_gpu_engine *eng = NULL;
	uint32_t i;

	g_rng = argc > 2 ? strtoull(argv[2], NULL, 0) : 12345u;
	cmp_set_timestamp_func(timestamp);
	if (cmp_is_error(cmp_gpu_engine_create(&eng, NULL))) {
		fprintf(stderr, "engine create failed\n");
		return 2;
	}
	for (i = 0; i < iters; i++) {
		fuzz_host_api();
		fuzz_batch(eng);
		fuzz_params_parse();
		fuzz_gather_plan();
	}
	cmp_gpu_engine_destroy(eng);
	printf("gather plans: %u ok, %u refused\n", n_plan_ok, n_plan_refused);
	printf("host_fuzz: %u iterations clean: %u contexts initialised, host frames %u ok / %u errors, "
	       "%u batches (%u frames ok, %u with fallback enabled), %u streams, %lu walks\n",
	       iters, n_init_ok, n_frames_ok, n_frames_err, n_batch_ok, n_batch_frames_ok, n_batch_fallback_cap,
	       n_stream_ok, stub_walk_calls);
	return 0;
}
