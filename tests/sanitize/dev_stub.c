/*
 * dev_stub.c -- TEST ONLY.  A host-memory stand-in for the HIP device layer
 * (airs_dev.h), so that the C host library (cmp_host.c: parameter checks,
 * the context state machine, the batch planner and its step-by-step
 * fallback path) and the CLI parser can run under AddressSanitizer and
 * UndefinedBehaviorSanitizer on a machine without a GPU (SURVEY.md section 5,
 * sanitizer row).  It does not encode anything: an "encode" writes a
 * deterministic pseudo-random outcome per frame (a size that fits, or
 * CMP_ERR_DST_TOO_SMALL) plus a header-shaped first 16 bytes, which is
 * enough to drive every branch of the planner.  Device memory is malloc'd
 * host memory, copies are memcpy.  Never linked into the product.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "airs_dev.h"

#define ERRV(code) ((uint32_t)0u - (uint32_t)(code))

struct airs_dev_engine {
	void *scratch[AIRS_NSLOT];
	size_t cap[AIRS_NSLOT];
	void *pinned;
	size_t pinned_cap;
	uint64_t salt;
	uint64_t coll[2 + 2 * AIRS_COLL_MAX_RANKS];
};

/* failure injection for the multi-rank gather harness (gather_sim.c): the
 * scratch slot whose allocation fails on this thread (-1: none) */
__thread int stub_scratch_fail_slot = -1;

uint64_t *airs_dev_coll(struct airs_dev_engine *e)
{
	return e ? e->coll : NULL;
}

static uint64_t mix(uint64_t z)
{
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

int airs_dev_available(void)
{
	return 1;
}

const char *airs_dev_last_error(void)
{
	return "stub";
}

struct airs_dev_engine *airs_dev_engine_create(void *stream)
{
	(void)stream;
	return calloc(1, sizeof(struct airs_dev_engine));
}

uint32_t airs_dev_set_option(struct airs_dev_engine *e, uint32_t option, uint32_t value)
{
	if (!e)
		return (uint32_t)0 - 1u;
	if (option < AIRS_OPT_EXCLUSIVE || option > AIRS_OPT_NO_CONTEXT_WALK)
		return (uint32_t)0 - 10u;
	(void)value;
	return 0;
}

void airs_dev_engine_destroy(struct airs_dev_engine *e)
{
	if (!e)
		return;
	for (int i = 0; i < AIRS_NSLOT; i++)
		free(e->scratch[i]);
	free(e->pinned);
	free(e);
}

void *airs_dev_engine_stream(struct airs_dev_engine *e)
{
	(void)e;
	return NULL;
}

void *airs_dev_scratch(struct airs_dev_engine *e, int slot, size_t bytes)
{
	if (!e || slot < 0 || slot >= AIRS_NSLOT || slot == stub_scratch_fail_slot)
		return NULL;
	if (bytes > e->cap[slot]) {
		free(e->scratch[slot]);
		e->scratch[slot] = malloc(bytes);
		e->cap[slot] = e->scratch[slot] ? bytes : 0;
	}
	return e->scratch[slot];
}

void *airs_dev_host_scratch(struct airs_dev_engine *e, size_t bytes)
{
	if (!e)
		return NULL;
	if (bytes > e->pinned_cap) {
		free(e->pinned);
		e->pinned = malloc(bytes);
		e->pinned_cap = e->pinned ? bytes : 0;
	}
	return e->pinned;
}

uint32_t airs_dev_encode(struct airs_dev_engine *e, const struct airs_launch *L)
{
	if (!e || !L || !L->n || !L->num_frames || !L->status)
		return ERRV(1u);
	for (uint32_t j = 0; j < L->num_frames; j++) {
		const uint32_t f = L->frame_list ? L->frame_list[j] : L->frame_add + j * L->frame_mul;
		if (f == 0xFFFFFFFFu) /* AIRS_NO_FRAME: a hole in a device-planned list */
			continue;
		const uint64_t h = mix(e->salt++ ^ ((uint64_t)f << 32) ^ L->n);
		/* every input byte the kernel would read is read here too */
		const uint8_t *src = (const uint8_t *)L->src + (uint64_t)f * L->src_stride;
		volatile uint8_t sink = src[0] ^ src[(uint64_t)L->n * L->sample_bytes - 1u];
		(void)sink;
		uint32_t size = 16u + (uint32_t)(h % (3ull * L->n + 8u));
		uint8_t *dst = (uint8_t *)L->dst + (uint64_t)f * L->dst_stride;
		if (L->model_mode != AIRS_MODEL_NONE) {
			uint8_t *m = L->model_ptrs ? (uint8_t *)(uintptr_t)L->model_ptrs[j]
						   : (uint8_t *)L->model + (uint64_t)(f / (L->model_div ? L->model_div : 1u)) *
									     L->model_stride;
			m[0] ^= 1u; /* touch both ends of the model */
			m[2u * L->n - 1u] ^= 1u;
		}
		if (L->checksum_enabled && L->checksums)
			(void)L->checksums[f];
		if (L->frame_g)
			(void)L->frame_g[f];
		if (size > L->cap) {
			L->status[f] = ERRV(30u); /* DST_TOO_SMALL */
		} else {
			memset(dst, 0, 16);
			dst[0] = (uint8_t)(size >> 16);
			dst[1] = (uint8_t)(size >> 8);
			dst[2] = (uint8_t)size;
			dst[size - 1u] = 0x5A;
			L->status[f] = size;
		}
		if (L->needed)
			L->needed[f] = size;
	}
	return 0;
}

/* the walk needs n % 4096 == 0 and 16-byte aligned inputs; the stub checks
 * the same so that the host's applicability test is exercised as written */
int airs_dev_walk_supported(const struct airs_walk *w)
{
	if (!w || !w->n || w->n % 4096u || !w->num_ctx || !w->fpc || (w->sample_bytes != 2 && w->sample_bytes != 4))
		return 0;
	if (((uintptr_t)w->src & 15u) || (w->src_stride & 15u))
		return 0;
	if (w->fb && (!w->draws || !w->seq_out || w->cap != w->raw_size))
		return 0;
	return w->model_ptrs || !(((uintptr_t)w->model & 15u) || (w->model_stride & 15u));
}

unsigned long stub_walk_calls;

uint32_t airs_dev_walk(struct airs_dev_engine *e, struct airs_walk *w)
{
	if (!e || !airs_dev_walk_supported(w) || !w->status)
		return ERRV(10u);
	stub_walk_calls++;
	for (uint32_t c = 0; c < w->num_ctx; c++) {
		uint8_t *m = w->model_ptrs ? (uint8_t *)(uintptr_t)w->model_ptrs[c]
					   : (uint8_t *)w->model + (uint64_t)c * w->model_stride;
		m[0] ^= 1u; /* touch both ends of the model */
		m[2u * w->n - 1u] ^= 1u;
		if (w->seq0s)
			(void)w->seq0s[c];
		for (uint32_t a = 0; a < w->fpc; a++) {
			const uint32_t f = c * w->fpc + a;
			const uint64_t h = mix(e->salt++ ^ ((uint64_t)f << 32) ^ w->n);
			const uint8_t *src = (const uint8_t *)w->src + (uint64_t)f * w->src_stride;
			volatile uint8_t sink = src[0] ^ src[(uint64_t)w->n * w->sample_bytes - 1u];
			(void)sink;
			uint32_t size = 16u + (uint32_t)(h % (3ull * w->n + 8u));
			uint8_t *dst = (uint8_t *)w->dst + (uint64_t)f * w->dst_stride;
			if (w->ids)
				(void)w->ids[f];
			if (w->checksum_enabled && w->checksums)
				(void)w->checksums[f];
			if (size > w->cap)
				size = w->cap;
			memset(dst, 0, 16);
			dst[size - 1u] = 0x5A;
			w->status[f] = size;
			if (w->fb) /* the walk's fallback: identifier draws of the frame */
				w->draws[f] = (uint8_t)(h >> 40) & 3u;
		}
		if (w->fb)
			w->seq_out[c] = (uint8_t)(1u + c % 3u);
	}
	return 0;
}

uint32_t airs_dev_encode_stream(struct airs_dev_engine *e, const void *src, uint32_t sample_bytes, uint32_t n,
				uint32_t preprocessing, uint32_t encoder_type, uint32_t encoder_param,
				uint32_t outlier_param, void *dst, uint32_t cap, uint32_t *status)
{
	(void)preprocessing, (void)encoder_type, (void)encoder_param, (void)outlier_param;
	if (!e || !n)
		return ERRV(1u);
	volatile uint8_t sink = ((const uint8_t *)src)[(uint64_t)n * sample_bytes - 1u];
	(void)sink;
	const uint32_t size = 1u + (uint32_t)(mix(e->salt++) % (3ull * n));
	if (size > cap) {
		*status = ERRV(30u);
	} else {
		((uint8_t *)dst)[size - 1u] = 0x5A;
		*status = size;
	}
	return 0;
}

uint32_t airs_dev_pack_frames(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
			      uint32_t max_frame_bytes, const uint32_t *sizes, uint32_t num_frames,
			      uint32_t err_floor, void *out, uint64_t *offsets)
{
	uint64_t o = 0;
	(void)e, (void)max_frame_bytes;
	for (uint32_t f = 0; f < num_frames; f++) {
		const uint32_t sz = sizes[f] > err_floor ? 0u : sizes[f];
		offsets[f] = o;
		memcpy((uint8_t *)out + o, (const uint8_t *)src + (uint64_t)f * src_stride, sz);
		o += ((uint64_t)sz + 7u) & ~7ull;
	}
	offsets[num_frames] = o;
	return 0;
}

/* the per-context state machine of fb_step_kernel (encode.hip), on the host */
uint32_t airs_dev_fb_step(struct airs_dev_engine *e, const struct airs_fb_step *a)
{
	if (!e || !a || !a->num_ctx)
		return ERRV(1u);
	for (uint32_t c = 0; c < a->num_ctx; c++) {
		uint32_t seq = a->state[2u * c], msize = a->state[2u * c + 1u];
		if (a->prev >= 0) {
			const uint32_t f = c * a->fpc + (uint32_t)a->prev;
			uint8_t fb = 0;
			if (a->kind[f]) {
				const uint32_t v = a->status[f];
				if (v <= a->err_floor) {
					seq++;
				} else if (a->fb_eligible && v == a->err_small) {
					fb = 1;
					a->draws[f] = (uint8_t)(a->draws[f] + 2u);
					msize = a->packed;
					a->status[f] = a->raw_size > 0xFFFFFFu ? a->err_too_large : a->raw_size;
					seq = a->raw_size > 0xFFFFFFu ? 0u : 1u;
				}
			}
			a->fb[f] = fb;
		}
		if (a->cur >= 0) {
			const uint32_t f = c * a->fpc + (uint32_t)a->cur;
			uint32_t lp = 0xFFFFFFFFu, ls = 0xFFFFFFFFu;
			uint8_t kind = 0, draws = 0;
			if (seq == 0 || seq > a->iters) {
				seq = 0;
				msize = a->packed;
				draws = 1;
				kind = 1;
				lp = f;
			} else if (a->model_needed && msize != a->packed) {
				a->status[f] = a->err_mismatch;
			} else {
				kind = 2;
				ls = f;
			}
			a->flist_p[c] = lp;
			a->flist_s[c] = ls;
			a->seqs[f] = (uint8_t)seq;
			a->kind[f] = kind;
			a->draws[f] = draws;
		}
		a->state[2u * c] = seq;
		a->state[2u * c + 1u] = msize;
	}
	return 0;
}

/* fb_copy_kernel: raw frames of the previous step's fallbacks */
uint32_t airs_dev_fb_copy(struct airs_dev_engine *e, const struct airs_fb_step *a)
{
	if (!e || !a || !a->num_ctx || a->prev < 0 || !a->n)
		return ERRV(1u);
	for (uint32_t c = 0; c < a->num_ctx; c++) {
		const uint32_t f = c * a->fpc + (uint32_t)a->prev;
		if (!a->fb[f])
			continue;
		const uint8_t *fs = (const uint8_t *)a->src + (uint64_t)f * a->src_stride;
		uint8_t *fd = (uint8_t *)a->dst + (uint64_t)f * a->dst_stride;
		uint16_t *fm = NULL;
		if (a->model_needed)
			fm = (uint16_t *)(a->model_ptrs ? (uint8_t *)(uintptr_t)a->model_ptrs[c]
							: (uint8_t *)a->model + (uint64_t)c * a->model_stride);
		memset(fd, 0, 16);
		for (uint32_t i = 0; i < a->n; i++) {
			const uint16_t x = a->sample_bytes == 2 ? ((const uint16_t *)fs)[i]
							       : (uint16_t)((const uint32_t *)fs)[i];
			fd[16u + 2u * i] = (uint8_t)(x >> 8);
			fd[17u + 2u * i] = (uint8_t)x;
			if (fm)
				fm[i] = x;
		}
		if (a->checksum)
			memcpy(fd + 16u + 2u * a->n, &a->checksums[f], 4);
	}
	return 0;
}

uint32_t airs_dev_checksum(struct airs_dev_engine *e, const void *src, uint64_t src_stride, uint32_t sample_bytes,
			   uint32_t n, uint32_t num_frames, const uint32_t *frame_list, uint32_t *out)
{
	if (!e || !n || !num_frames)
		return ERRV(1u);
	for (uint32_t j = 0; j < num_frames; j++) {
		const uint32_t f = frame_list ? frame_list[j] : j;
		const uint8_t *s = (const uint8_t *)src + (uint64_t)f * src_stride;
		out[frame_list ? f : j] = s[0] + s[(uint64_t)n * sample_bytes - 1u];
	}
	return 0;
}

uint32_t airs_dev_select_rice(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
			      uint32_t sample_bytes, uint32_t n, uint32_t num_frames, const uint32_t *frame_list,
			      uint32_t frame_add, uint32_t frame_mul, uint32_t preprocessing, uint32_t *out_g)
{
	(void)e, (void)src, (void)src_stride, (void)sample_bytes, (void)n, (void)preprocessing;
	for (uint32_t j = 0; j < num_frames; j++) {
		const uint32_t f = frame_list ? frame_list[j] : frame_add + j * frame_mul;
		if (f != 0xFFFFFFFFu)
			out_g[f] = 32u;
	}
	return 0;
}

uint32_t airs_dev_synth(struct airs_dev_engine *e, void *dst, uint32_t sample_bytes, uint64_t seed, uint32_t frame0,
			uint32_t n, uint32_t num_frames, uint64_t stride, uint32_t W)
{
	(void)e, (void)W;
	for (uint32_t f = 0; f < num_frames; f++)
		for (uint32_t i = 0; i < n * sample_bytes; i++)
			((uint8_t *)dst)[(uint64_t)f * stride + i] = (uint8_t)mix(seed + frame0 + f + i);
	return 0;
}

uint32_t airs_dev_patch_ids(struct airs_dev_engine *e, void *dst, uint64_t dst_stride, uint32_t num_frames,
			    uint32_t frame_add, uint32_t frame_mul, const uint64_t *ids, const uint32_t *status)
{
	(void)e;
	for (uint32_t j = 0; j < num_frames; j++) {
		const uint32_t f = frame_add + j * frame_mul;
		if (status && status[f] > ERRV(128u))
			continue;
		for (int b = 0; b < 6; b++)
			((uint8_t *)dst)[(uint64_t)f * dst_stride + 8u + (uint32_t)b] = (uint8_t)(ids[j] >> (40 - 8 * b));
	}
	return 0;
}

uint32_t airs_dev_decode(struct airs_dev_engine *e, const void *src, uint64_t src_stride, uint32_t src_cap,
			 uint32_t num_frames, uint16_t *dst, uint64_t dst_stride, uint32_t dst_samples,
			 uint32_t *status, const uint16_t *model, uint64_t model_stride)
{
	(void)e, (void)dst, (void)dst_stride, (void)dst_samples, (void)model, (void)model_stride;
	for (uint32_t f = 0; f < num_frames; f++) {
		const uint8_t *s = (const uint8_t *)src + (uint64_t)f * src_stride;
		status[f] = src_cap ? s[0] + 0u * s[src_cap - 1u] : 0u;
	}
	return 0;
}

void *airs_dev_malloc(size_t bytes)
{
	return malloc(bytes ? bytes : 1);
}

void airs_dev_free(void *p)
{
	free(p);
}

uint32_t airs_dev_h2d(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes)
{
	(void)e;
	memcpy(dst, src, bytes);
	return 0;
}

uint32_t airs_dev_d2h(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes)
{
	(void)e;
	memcpy(dst, src, bytes);
	return 0;
}

uint32_t airs_dev_sync(struct airs_dev_engine *e)
{
	(void)e;
	return 0;
}

static uint8_t g_commit_flags[8192];

uint32_t airs_dev_memset(struct airs_dev_engine *e, void *dst, int v, size_t bytes)
{
	(void)e;
	memset(dst, v, bytes);
	return 0;
}

uint32_t airs_dev_d2d_rows(struct airs_dev_engine *e, void *dst, size_t dpitch, const void *src, size_t spitch,
			   size_t width, size_t rows)
{
	(void)e;
	for (size_t r = 0; r < rows; r++)
		memmove((uint8_t *)dst + r * dpitch, (const uint8_t *)src + r * spitch, width);
	return 0;
}

uint32_t airs_dev_commit_begin(struct airs_dev_engine *e, const uint32_t *status, uint32_t num_ctx, uint32_t fpc,
			       void *dst, uint64_t dst_stride, uint32_t *seq)
{
	(void)e;
	(void)dst;
	(void)dst_stride;
	for (uint32_t c = 0; c < num_ctx && c < sizeof(g_commit_flags); c++) {
		uint32_t any = 0;
		for (uint32_t a = 0; a < fpc; a++)
			any |= status[(size_t)c * fpc + a] > 0xFFFFFFFFu - 128u;
		g_commit_flags[c] = (uint8_t)any;
	}
	*seq = 1;
	return 0;
}

uint32_t airs_dev_commit_wait(struct airs_dev_engine *e, uint32_t seq, uint32_t num_ctx, uint8_t *flags)
{
	(void)e;
	(void)seq;
	memcpy(flags, g_commit_flags, num_ctx < sizeof(g_commit_flags) ? num_ctx : sizeof(g_commit_flags));
	return 0;
}

int airs_dev_commit_release(struct airs_dev_engine *e, uint32_t seq, const uint64_t *ids, uint32_t total)
{
	(void)e;
	(void)seq;
	(void)ids;
	(void)total;
	return 0; /* the caller patches */
}

/* the gather's identifier patch: six big-endian bytes at data + offsets[i] + 8 */
uint32_t airs_dev_patch_ids_at(struct airs_dev_engine *e, void *data, const uint64_t *offsets, const uint64_t *ids,
			       uint64_t n)
{
	uint64_t i;
	int b;

	(void)e;
	for (i = 0; i < n; i++)
		for (b = 0; b < 6; b++)
			((uint8_t *)data)[offsets[i] + 8u + (uint64_t)b] = (uint8_t)(ids[i] >> (8 * (5 - b)));
	return 0;
}
