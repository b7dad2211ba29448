/*
 * oracle/batch_driver.c -- multi-threaded frame loop over the cmp.h API.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY.  Compiled twice by oracle/Makefile:
 *   - into oracle/liborc.so against the clean-room restatement (kind "port");
 *   - into oracle/_ref/libref.so against the reference's own lib/ sources
 *     compiled from /root/reference (kind "reference").
 * bench.py times it as the CPU baseline; tests use it to produce expected
 * frames for large batches.  It only calls the public cmp.h API.
 *
 * Frame (c, a) -- context c, acquisition a -- lives at index c*fpc + a; the
 * acquisitions of one context run in order (MODEL state is carried), the
 * contexts run in parallel, one OpenMP thread per context at a time.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cmp.h"

static volatile uint64_t drv_counter;

/* thread-safe identifier source for the parallel runs */
static void drv_timestamp(uint32_t *coarse, uint16_t *fine)
{
	uint64_t v = __atomic_fetch_add(&drv_counter, 1, __ATOMIC_RELAXED);

	*coarse = (uint32_t)(v >> 16);
	*fine = (uint16_t)v;
}

/* kind: 0 = u16, 1 = i16, 2 = i16-in-i32 */
static uint32_t drv_one(struct cmp_context *ctx, int kind, void *dst, uint32_t cap, const void *src,
			uint32_t size)
{
	switch (kind) {
	case 1:
		return cmp_compress_i16(ctx, dst, cap, src, size);
	case 2:
		return cmp_compress_i16_in_i32(ctx, dst, cap, src, size);
	default:
		return cmp_compress_u16(ctx, dst, cap, src, size);
	}
}

/* Returns the sum of the compressed sizes, or UINT64_MAX if any frame
 * failed (its error code is left in sizes[]). */
uint64_t drv_run(const struct cmp_params *params, int kind, const void *src, uint32_t src_size,
		 uint64_t src_stride, uint32_t nctx, uint32_t fpc, void *dst, uint64_t dst_stride,
		 uint32_t dst_cap, uint32_t *sizes, int nthreads, int reset_counter)
{
	uint64_t total = 0;
	int failed = 0;
	long c;

	if (reset_counter) {
		drv_counter = 0;
		cmp_set_timestamp_func(drv_timestamp);
	}
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : total) \
	reduction(| : failed)
	for (c = 0; c < (long)nctx; c++) {
		struct cmp_context ctx;
		uint32_t work = cmp_cal_work_buf_size(params, src_size), a;
		void *wb = NULL;

		if (cmp_is_error(work)) {
			failed = 1;
			continue;
		}
		if (work)
			wb = malloc(work);
		if (cmp_is_error(cmp_initialise(&ctx, params, wb, work))) {
			free(wb);
			failed = 1;
			continue;
		}
		for (a = 0; a < fpc; a++) {
			uint64_t idx = (uint64_t)c * fpc + a;
			uint32_t r = drv_one(&ctx, kind, (uint8_t *)dst + idx * dst_stride, dst_cap,
					     (const uint8_t *)src + idx * src_stride, src_size);

			sizes[idx] = r;
			if (cmp_is_error(r))
				failed = 1;
			else
				total += r;
		}
		free(wb);
	}
	if (reset_counter)
		cmp_set_timestamp_func(NULL);
	return failed ? UINT64_MAX : total;
}

/*
 * The per-frame Rice-k rule of the build's CMP_GPU_AUTO_RICE extension
 * (SURVEY.md 8(d) cfg 3; the reference has no k selection): the g = 2^k,
 * k in [0,15], with the fewest payload bits, ties to the smaller k.  Stated
 * here again so that the CPU baseline of that config can run on top of the
 * reference's own encoder (libref.so); oracle/cmp_oracle.c's
 * orc_select_rice_k is the checker's copy.  Samples are u16/i16 (kind 0, 1)
 * or i16 in the low half of i32 (kind 2); pre 1 = DIFF, else NONE.
 */
static uint32_t drv_select_rice_k(const void *src, uint32_t n, int kind, uint32_t pre)
{
	uint64_t bits[16];
	uint32_t i, k, best = 0;
	int16_t prev = 0;

	for (k = 0; k < 16; k++)
		bits[k] = (uint64_t)n * (k + 1u);
	for (i = 0; i < n; i++) {
		int16_t x = kind == 2 ? (int16_t)(((const uint32_t *)src)[i] & 0xFFFFu) : ((const int16_t *)src)[i];
		int16_t r = (pre == 1 && i) ? (int16_t)(x - prev) : x;
		uint16_t u = (uint16_t)r;
		uint32_t v = (uint32_t)(uint16_t)((u << 1) ^ (uint16_t)(0u - (u >> 15))) + 1u;

		prev = x;
		for (k = 0; k < 16; k++) {
			uint32_t q = v >> k;

			bits[k] += q < 16u ? q : 16u;
		}
	}
	for (k = 1; k < 16; k++)
		if (bits[k] < bits[best])
			best = k;
	return best;
}

/* drv_run with the primary encoder parameter chosen per frame by the rule
 * above (one context per frame, frames in parallel); g_out[f] = 2^k */
uint64_t drv_run_autorice(const struct cmp_params *params, int kind, const void *src, uint32_t src_size,
			  uint64_t src_stride, uint32_t nframes, void *dst, uint64_t dst_stride, uint32_t dst_cap,
			  uint32_t *sizes, uint32_t *g_out, int nthreads, int reset_counter)
{
	uint64_t total = 0;
	int failed = 0;
	long f;

	if (reset_counter) {
		drv_counter = 0;
		cmp_set_timestamp_func(drv_timestamp);
	}
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads) reduction(+ : total) \
	reduction(| : failed)
	for (f = 0; f < (long)nframes; f++) {
		struct cmp_context ctx;
		struct cmp_params p = *params;
		const uint8_t *s = (const uint8_t *)src + (uint64_t)f * src_stride;
		uint32_t n = src_size / (kind == 2 ? 4u : 2u), r;

		p.primary_encoder_param = 1u << drv_select_rice_k(s, n, kind, p.primary_preprocessing);
		if (g_out)
			g_out[f] = p.primary_encoder_param;
		if (cmp_is_error(cmp_initialise(&ctx, &p, NULL, 0))) {
			failed = 1;
			continue;
		}
		r = drv_one(&ctx, kind, (uint8_t *)dst + (uint64_t)f * dst_stride, dst_cap, s, src_size);
		sizes[f] = r;
		if (cmp_is_error(r))
			failed = 1;
		else
			total += r;
	}
	if (reset_counter)
		cmp_set_timestamp_func(NULL);
	return failed ? UINT64_MAX : total;
}
