/* tests/dropin/host_probe.c -- TEST ONLY: the cmp.h host API on a plain C
 * process (no torch, /opt/rocm's HIP runtime), two calls on one context with
 * a host work buffer: DIFF + GOLOMB_ZERO g=1055, then MODEL + GOLOMB_MULTI
 * g=8 o=107 (the parameters of the reference's examples/simple_compression.c).
 * Prints each call's result and, on an error, the library's last HIP error. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmp.h>

const char *airs_dev_last_error(void);

static void ts(uint32_t *coarse, uint16_t *fine)
{
	*coarse = 0x12345678u;
	*fine = 0x9ABCu;
}

int main(void)
{
	struct cmp_params p;
	struct cmp_context ctx;
	uint16_t a[3] = { 0, 1, 2 }, b[3] = { 2, 1, 1 };
	uint32_t wbs, cap, r, i;
	void *wb, *dst;
	int bad = 0;

	memset(&p, 0, sizeof(p));
	memset(&ctx, 0, sizeof(ctx));
	cmp_set_timestamp_func(ts);
	p.primary_preprocessing = CMP_PREPROCESS_DIFF;
	p.primary_encoder_type = CMP_ENCODER_GOLOMB_ZERO;
	p.primary_encoder_param = 1055;
	p.secondary_iterations = 15;
	p.secondary_preprocessing = CMP_PREPROCESS_MODEL;
	p.secondary_encoder_type = CMP_ENCODER_GOLOMB_MULTI;
	p.secondary_encoder_param = 8;
	p.secondary_encoder_outlier = 107;
	p.model_rate = 11;
	p.uncompressed_fallback_enabled = 1;
	p.checksum_enabled = 1;
	wbs = cmp_cal_work_buf_size(&p, sizeof(a));
	cap = cmp_compress_bound(sizeof(a));
	printf("work_buf_size %u compress_bound %u\n", wbs, cap);
	wb = malloc(wbs ? wbs : 1);
	dst = malloc(cap);
	r = cmp_initialise(&ctx, &p, wb, wbs);
	printf("initialise %u\n", r);
	for (i = 0; i < 2; i++) {
		r = cmp_compress_u16(&ctx, dst, cap, i ? b : a, sizeof(a));
		printf("compress %u -> %u%s%s\n", i, r, cmp_is_error(r) ? " error; last HIP error: " : "",
		       cmp_is_error(r) ? airs_dev_last_error() : "");
		bad |= cmp_is_error(r) ? 1 : 0;
	}
	fflush(stdout);
	free(dst);
	free(wb);
	return bad;
}
