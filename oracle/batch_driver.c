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
