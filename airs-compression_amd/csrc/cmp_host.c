/*
 * cmp_host.c -- host side of libairscmp.so: the cmp.h API (drop-in for the
 * reference's lib/compress/cmp.c + lib/common/cmp_errors.c) and the cmp_gpu.h
 * device batch API.  Parameter validation, the context state machine
 * (primary/secondary passes, identifiers, fallback) and all error codes
 * follow the reference exactly; the per-sample work is done by the HIP
 * kernels in encode.hip through airs_dev.h.  There is no CPU encode path:
 * without a usable GPU the compress calls fail with CMP_ERR_GENERIC and a
 * message on stderr.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmp.h"
#include "cmp_errors.h"
#include "cmp_gpu.h"
#include "airs_dev.h"
#include "cmp_engine.h"

#define ERRV(name) ((uint32_t)0u - (uint32_t)CMP_ERR_##name)
#define CTX_MAGIC 34021395u      /* reference lib/compress/cmp.c:23 */
#define EXT_HDR_SIZE 6u          /* reference lib/common/header_private.h:35-39 */
#define HDR_MAX_SIZE (CMP_HDR_SIZE + EXT_HDR_SIZE)
#define MAX_MODEL_RATE 16u

static unsigned is_err(uint32_t v)
{
	return v > ERRV(MAX_CODE);
}

/* ---------------- identifiers (reference cmp.c:27-50, 438-449) ---------------- */
static uint64_t g_counter;

static void counter_timestamp(uint32_t *coarse, uint16_t *fine)
{
	*coarse = (uint32_t)(g_counter >> 16);
	*fine = (uint16_t)g_counter;
	g_counter++;
}

static void (*g_timestamp)(uint32_t *, uint16_t *) = counter_timestamp;

void cmp_set_timestamp_func(void (*f)(uint32_t *coarse, uint16_t *fine))
{
	g_timestamp = f ? f : counter_timestamp;
}

static uint64_t next_identifier(void)
{
	uint32_t coarse = 0;
	uint16_t fine = 0;

	g_timestamp(&coarse, &fine);
	return ((uint64_t)coarse << 16) | (uint64_t)fine;
}

/* ---------------- errors (reference lib/common/cmp_errors.c) ---------------- */
unsigned int cmp_is_error(uint32_t code)
{
	return is_err(code);
}

enum cmp_error cmp_get_error_code(uint32_t code)
{
	if (!is_err(code))
		return CMP_ERR_NO_ERROR;
	return (enum cmp_error)(0u - code);
}

const char *cmp_get_error_string(enum cmp_error code)
{
	static const struct {
		enum cmp_error code;
		const char *text;
	} table[] = {
		{ CMP_ERR_NO_ERROR, "No error detected" },
		{ CMP_ERR_GENERIC, "Error (generic)" },
		{ CMP_ERR_PARAMS_INVALID, "Invalid compression parameters" },
		{ CMP_ERR_DST_TOO_SMALL, "Destination buffer is too small to hold the content" },
		{ CMP_ERR_DST_NULL, "Destination buffer pointer is NULL" },
		{ CMP_ERR_DST_UNALIGNED, "Destination buffer pointer is unaligned" },
		{ CMP_ERR_SRC_SIZE_WRONG, "Source buffer size is invalid" },
		{ CMP_ERR_SRC_NULL, "Source buffer pointer is NULL" },
		{ CMP_ERR_SRC_SIZE_MISMATCH,
		  "Source data size changed using model preprocessing; not allowed until reset" },
		{ CMP_ERR_WORK_BUF_TOO_SMALL, "Work buffer is too small" },
		{ CMP_ERR_WORK_BUF_NULL, "Work buffer is NULL but required" },
		{ CMP_ERR_WORK_BUF_UNALIGNED, "Work buffer is unaligned" },
		{ CMP_ERR_HDR_CMP_SIZE_TOO_LARGE, "Compressed size exceeds header field limit" },
		{ CMP_ERR_HDR_ORIGINAL_TOO_LARGE, "Original size exceeds header field limit" },
		{ CMP_ERR_CONTEXT_INVALID, "Compression context uninitialised or corrupted" },
		{ CMP_ERR_INT_HDR, "Internal header processing error" },
		{ CMP_ERR_INT_ENCODER, "Internal data encoder error" },
		{ CMP_ERR_INT_BITSTREAM, "Internal bitstream writer error" },
	};
	size_t i;

	for (i = 0; i < sizeof(table) / sizeof(table[0]); i++)
		if (table[i].code == code)
			return table[i].text;
	return "Unspecified error code";
}

const char *cmp_get_error_message(uint32_t code)
{
	return cmp_get_error_string(cmp_get_error_code(code));
}

/* ---------------- encoder parameters (reference encoder.c:63-233) ---------------- */
static uint32_t floor_log2(uint32_t x)
{
	return 31u - (uint32_t)__builtin_clz(x);
}

/* validate (type, g, outlier) and resolve the outlier written to the header */
static uint32_t coder_resolve(uint32_t type, uint32_t g, uint32_t outlier, uint32_t *resolved)
{
	uint32_t k, cutoff, limit;
	uint64_t want;

	if (resolved)
		*resolved = 0;
	if (type == CMP_ENCODER_UNCOMPRESSED)
		return 0;
	if (type != CMP_ENCODER_GOLOMB_ZERO && type != CMP_ENCODER_GOLOMB_MULTI)
		return ERRV(PARAMS_INVALID);
	if (g < 1u || g > 0xFFFFu)
		return ERRV(PARAMS_INVALID);
	k = floor_log2(g);
	cutoff = (2u << k) - g;
	limit = cutoff + (31u - k) * g; /* first value needing a > 32-bit codeword */
	if (type == CMP_ENCODER_GOLOMB_MULTI)
		limit = limit > 8u ? limit - 8u : 0u; /* 8 escape symbols for 16-bit samples */
	want = type == CMP_ENCODER_GOLOMB_ZERO ? (uint64_t)cutoff + 16ull * g - 1ull : (uint64_t)outlier;
	if (want > limit)
		want = limit;
	if (want == 0)
		return ERRV(PARAMS_INVALID);
	if (resolved)
		*resolved = (uint32_t)want;
	return 0;
}

/* 48 bits per sample worst case (reference encoder.c:381-386) */
static uint64_t payload_bound(uint32_t size)
{
	uint64_t n = ((uint64_t)size * 8u + 15u) / 16u;

	return (n * 48u + 7u) / 8u;
}

uint32_t cmp_compress_bound(uint32_t packed_size)
{
	uint64_t b;

	if (packed_size > CMP_HDR_MAX_ORIGINAL_SIZE)
		return ERRV(HDR_ORIGINAL_TOO_LARGE);
	b = HDR_MAX_SIZE + CMP_CHECKSUM_SIZE + payload_bound(packed_size);
	if (b > CMP_HDR_MAX_COMPRESSED_SIZE)
		return ERRV(HDR_CMP_SIZE_TOO_LARGE);
	return (uint32_t)b;
}

static uint32_t pre_work_size(uint32_t pre, uint32_t size, int *known)
{
	*known = 1;
	if (pre == CMP_PREPROCESS_NONE || pre == CMP_PREPROCESS_DIFF)
		return 0;
	if (pre == CMP_PREPROCESS_IWT || pre == CMP_PREPROCESS_MODEL)
		return (size + 1u) & ~1u;
	*known = 0;
	return 0;
}

uint32_t cmp_cal_work_buf_size(const struct cmp_params *params, uint32_t src_size)
{
	uint32_t a, b = 0;
	int known;

	if (!params)
		return ERRV(GENERIC);
	if (params->primary_preprocessing == CMP_PREPROCESS_MODEL)
		return ERRV(PARAMS_INVALID);
	a = pre_work_size(params->primary_preprocessing, src_size, &known);
	if (!known)
		return ERRV(PARAMS_INVALID);
	if (params->secondary_iterations) {
		b = pre_work_size(params->secondary_preprocessing, src_size, &known);
		if (!known)
			return ERRV(PARAMS_INVALID);
	}
	return a > b ? a : b;
}

static int model_needed(const struct cmp_params *p)
{
	return p->secondary_preprocessing == CMP_PREPROCESS_MODEL && p->secondary_iterations != 0;
}

/* some pass of the context keeps state in its work buffer: the model, or the
 * IWT coefficients (preprocess.c:321-353 computes them into work_buf), so
 * frames of one context cannot share a launch */
static int work_buf_state(const struct cmp_params *p)
{
	return model_needed(p) || p->primary_preprocessing == CMP_PREPROCESS_IWT ||
	       (p->secondary_iterations && p->secondary_preprocessing == CMP_PREPROCESS_IWT);
}

/* cmp_reset; with `draws` set the identifier draw is only counted (the batch
 * API draws the identifiers afterwards, in the reference's call order) */
/* cmp_gpu_batch.draws is written only when the caller asks for it (ADVICE r3:
 * a caller that fills the struct field by field may leave it uninitialised) */
#define REPORT_DRAWS(b) (((b)->flags & CMP_GPU_REPORT_DRAWS) && (b)->draws)

static uint32_t ctx_reset(struct cmp_context *ctx, uint32_t *draws)
{
	if (!ctx)
		return ERRV(GENERIC);
	if (ctx->magic != CTX_MAGIC)
		return ERRV(CONTEXT_INVALID);
	ctx->sequence_number = 0;
	if (draws) {
		(*draws)++;
		ctx->identifier = 0;
	} else {
		ctx->identifier = next_identifier();
	}
	ctx->model_size = 0;
	return ERRV(NO_ERROR);
}

uint32_t cmp_reset(struct cmp_context *ctx)
{
	return ctx_reset(ctx, NULL);
}

void cmp_deinitialise(struct cmp_context *ctx)
{
	if (ctx)
		memset(ctx, 0, sizeof(*ctx));
}

uint32_t cmp_initialise(struct cmp_context *ctx, const struct cmp_params *params, void *work_buf,
			uint32_t work_buf_size)
{
	uint32_t e, need;

	if (!ctx)
		return ERRV(GENERIC);
	cmp_deinitialise(ctx);
	if (!params || is_err(work_buf_size))
		return ERRV(GENERIC);
	if (params->secondary_iterations >= (1u << CMP_HDR_BITS_SEQUENCE_NUMBER))
		return ERRV(PARAMS_INVALID);
	e = coder_resolve(params->primary_encoder_type, params->primary_encoder_param,
			  params->primary_encoder_outlier, NULL);
	if (is_err(e))
		return e;
	if (params->secondary_iterations) {
		e = coder_resolve(params->secondary_encoder_type, params->secondary_encoder_param,
				  params->secondary_encoder_outlier, NULL);
		if (is_err(e))
			return e;
	}
	if (model_needed(params) && params->model_rate > MAX_MODEL_RATE)
		return ERRV(PARAMS_INVALID);
	need = cmp_cal_work_buf_size(params, 2);
	if (is_err(need))
		return need;
	if (need) {
		if (!work_buf)
			return ERRV(WORK_BUF_NULL);
		if (!work_buf_size)
			return ERRV(WORK_BUF_TOO_SMALL);
		if ((uintptr_t)work_buf & 1u)
			return ERRV(WORK_BUF_UNALIGNED);
	}
	ctx->params = *params;
	ctx->work_buf = work_buf;
	ctx->work_buf_size = work_buf_size;
	ctx->magic = CTX_MAGIC;
	return cmp_reset(ctx);
}

/* ================================================================== */
/* one frame through the GPU (reference compress_engine, cmp.c:213-338) */
/* ================================================================== */
enum sample_kind { KIND_I16 = 0, KIND_I16_IN_I32 = 1, KIND_U16 = 2 };

struct frame_io {
	const void *src;   /* host or device, see `device` */
	uint32_t n;        /* samples */
	uint32_t bytes;    /* 2 or 4 per sample */
	enum sample_kind kind;
	int device;        /* src/dst/work_buf are device pointers (cmp_gpu.h path) */
	struct airs_dev_engine *dev;
	/* device-mode extras */
	uint32_t *d_status;
};

/* the pass a frame will use, resolved from the context (cmp.c:228-248) */
struct pass {
	uint32_t pre, enc, par, outlier_param, outlier;
	uint32_t model_mode;
	uint32_t seq;
	uint32_t hdr_bytes;
};

enum { SLOT_SRC = 0, SLOT_DST, SLOT_MODEL, SLOT_STATUS, SLOT_CK, SLOT_IDS, SLOT_G, SLOT_AUX, SLOT_FL, SLOT_SIZES, SLOT_MSAVE };

/* The host-pointer API stages every frame through one process-wide engine
 * (device scratch slots, look-back state).  Calls on different contexts may
 * come from different threads (the reference allows one context per thread),
 * so host_compress() holds g_host_lock for the whole call: calls are
 * serialised, and the engine is created once, under the lock. */
static pthread_mutex_t g_host_lock = PTHREAD_MUTEX_INITIALIZER;
static struct airs_dev_engine *g_host_dev;

static struct airs_dev_engine *host_dev(void)
{
	if (!g_host_dev) {
		g_host_dev = airs_dev_engine_create(NULL);
		if (!g_host_dev)
			fprintf(stderr, "airscmp: no usable GPU (%s); libairscmp has no CPU encode path\n",
				airs_dev_last_error());
	}
	return g_host_dev;
}

/* checks and state updates of compress_engine up to the encode loop;
 * returns 0 (pass filled in) or the error the reference would return */
static uint32_t engine_prologue(struct cmp_context *ctx, void *dst, uint32_t cap, uint32_t n, struct pass *p,
			       uint32_t *draws)
{
	const uint32_t packed = 2u * n;
	uint32_t e;

	memset(p, 0, sizeof(*p));
	if (ctx->sequence_number == 0 || ctx->sequence_number > ctx->params.secondary_iterations) {
		e = ctx_reset(ctx, draws);
		if (is_err(e))
			return e;
		p->pre = ctx->params.primary_preprocessing;
		p->enc = ctx->params.primary_encoder_type;
		p->par = ctx->params.primary_encoder_param;
		p->outlier_param = ctx->params.primary_encoder_outlier;
		ctx->model_size = packed;
	} else {
		p->pre = ctx->params.secondary_preprocessing;
		p->enc = ctx->params.secondary_encoder_type;
		p->par = ctx->params.secondary_encoder_param;
		p->outlier_param = ctx->params.secondary_encoder_outlier;
		if (model_needed(&ctx->params) && packed != ctx->model_size)
			return ERRV(SRC_SIZE_MISMATCH);
	}
	if (model_needed(&ctx->params) && ctx->work_buf_size < packed)
		return ERRV(WORK_BUF_TOO_SMALL);
	if (!dst)
		return ERRV(DST_NULL);
	if ((uintptr_t)dst & 7u)
		return ERRV(DST_UNALIGNED);
	e = coder_resolve(p->enc, p->par, p->outlier_param, &p->outlier);
	if (is_err(e))
		return e;
	p->hdr_bytes = (p->pre == CMP_PREPROCESS_NONE && p->enc == CMP_ENCODER_UNCOMPRESSED) ? CMP_HDR_SIZE
											   : HDR_MAX_SIZE;
	/* header serialisation (header.c:24-67): original size, then the flush */
	if (packed > CMP_HDR_MAX_ORIGINAL_SIZE)
		return ERRV(HDR_ORIGINAL_TOO_LARGE);
	if (cap < p->hdr_bytes)
		return ERRV(DST_TOO_SMALL);
	/* preprocessing init (preprocess.c:321-393) */
	if (p->pre == CMP_PREPROCESS_IWT || p->pre == CMP_PREPROCESS_MODEL) {
		if (!ctx->work_buf)
			return ERRV(WORK_BUF_NULL);
		if (ctx->work_buf_size < ((packed + 1u) & ~1u))
			return ERRV(WORK_BUF_TOO_SMALL);
		if ((uintptr_t)ctx->work_buf & 1u)
			return ERRV(WORK_BUF_UNALIGNED);
	} else if (p->pre != CMP_PREPROCESS_NONE && p->pre != CMP_PREPROCESS_DIFF) {
		return ERRV(PARAMS_INVALID);
	}
	p->model_mode = model_needed(&ctx->params) ?
				(ctx->sequence_number == 0 ? AIRS_MODEL_STORE : AIRS_MODEL_UPDATE) :
				AIRS_MODEL_NONE;
	p->seq = ctx->sequence_number;
	return 0;
}

/* bit position whose flush fails for capacity cap: samples reaching it keep
 * their old model (cmp.c:300-302 breaks the loop before the model update) */
static uint64_t model_fail_bit(uint32_t cap, uint32_t n)
{
	uint32_t bound = cmp_compress_bound(2u * n);

	if (!is_err(bound) && cap >= bound)
		return UINT64_MAX;
	return 64ull * (cap / 8u) + 63ull;
}

/* largest possible frame for n samples: header + 48 bits/sample + checksum */
static uint64_t frame_worst(uint32_t n)
{
	return HDR_MAX_SIZE + CMP_CHECKSUM_SIZE + payload_bound(2u * n) + 8u;
}

/* an internal failure of the host path (GENERIC), named on stderr */
static uint32_t host_fail(const char *what)
{
	fprintf(stderr, "airscmp: host path: %s failed (%s)\n", what, airs_dev_last_error());
	return ERRV(GENERIC);
}

/* Host-pointer frame: stage through device scratch, run, copy back. */
static uint32_t host_engine(struct cmp_context *ctx, void *dst, uint32_t cap, const struct frame_io *io)
{
	struct pass p;
	struct airs_launch L;
	struct airs_dev_engine *dev;
	uint32_t e, st[2] = { 0, 0 };
	uint64_t worst = frame_worst(io->n);
	uint32_t kcap = (uint64_t)cap < worst ? cap : (uint32_t)worst;
	const uint32_t packed = 2u * io->n;
	void *d_src, *d_dst, *d_model = NULL, *d_status, *d_ck = NULL;

	e = engine_prologue(ctx, dst, cap, io->n, &p, NULL);
	if (is_err(e))
		return e;
	dev = host_dev();
	if (!dev)
		return ERRV(GENERIC);

	d_src = airs_dev_scratch(dev, SLOT_SRC, (size_t)io->n * io->bytes);
	d_dst = airs_dev_scratch(dev, SLOT_DST, (size_t)worst);
	d_status = airs_dev_scratch(dev, SLOT_STATUS, 64);
	if (!d_src || !d_dst || !d_status)
		return host_fail("device scratch");
	if (is_err(airs_dev_h2d(dev, d_src, io->src, (size_t)io->n * io->bytes)))
		return host_fail("sample upload");
	if (p.model_mode != AIRS_MODEL_NONE || p.pre == CMP_PREPROCESS_IWT) {
		/* the work buffer on the device: the model, or the IWT coefficients
		 * (computed there by the launch, so not uploaded) */
		d_model = airs_dev_scratch(dev, SLOT_MODEL, (size_t)packed + 16u);
		if (!d_model)
			return host_fail("model scratch");
		if (p.pre != CMP_PREPROCESS_IWT && is_err(airs_dev_h2d(dev, d_model, ctx->work_buf, packed)))
			return host_fail("model upload");
	}
	if (ctx->params.checksum_enabled) {
		d_ck = airs_dev_scratch(dev, SLOT_CK, 64);
		if (!d_ck || is_err(airs_dev_checksum(dev, d_src, 0, io->bytes, io->n, 1, NULL, d_ck)))
			return host_fail("checksum");
	}

	memset(&L, 0, sizeof(L));
	L.src = d_src;
	L.sample_bytes = io->bytes;
	L.is_unsigned = io->kind == KIND_U16;
	L.n = io->n;
	L.num_frames = 1;
	L.frame_mul = 1;
	L.dst = d_dst;
	L.cap = kcap;
	L.preprocessing = p.pre;
	L.encoder_type = p.enc;
	L.encoder_param = p.par;
	L.outlier_param = p.outlier_param;
	L.model = d_model;
	L.model_div = 1;
	L.model_mode = p.model_mode;
	L.model_rate = ctx->params.model_rate;
	L.fail_bit = model_fail_bit(cap, io->n);
	L.id_base = ctx->identifier;
	L.seq = p.seq;
	L.checksum_enabled = ctx->params.checksum_enabled ? 1u : 0u;
	L.checksums = d_ck;
	L.status = d_status;
	L.needed = (uint32_t *)d_status + 1;
	e = airs_dev_encode(dev, &L);
	if (cmp_get_error_code(e) == CMP_ERR_GENERIC)
		return host_fail("encode launch");
	if (is_err(e))
		return e;
	if (is_err(airs_dev_d2h(dev, st, d_status, sizeof(st))))
		return host_fail("status read-back");
	/* work_buf afterwards holds what the reference leaves there: the model,
	 * or the IWT coefficients (overwritten by the model where it is stored) */
	if (d_model && is_err(airs_dev_d2h(dev, ctx->work_buf, d_model, packed)))
		return host_fail("model read-back");
	if (is_err(airs_dev_sync(dev)))
		return host_fail("synchronisation");
	if (is_err(st[0]))
		return st[0];
	if (is_err(airs_dev_d2h(dev, dst, d_dst, st[0])) || is_err(airs_dev_sync(dev)))
		return host_fail("frame read-back");
	ctx->sequence_number++;
	return st[0];
}

/* uncompressed fallback (reference cmp_compress_generic, cmp.c:342-393) */
static uint32_t host_generic(struct cmp_context *ctx, void *dst, uint32_t cap, const struct frame_io *io)
{
	uint32_t raw = CMP_HDR_SIZE + 2u * io->n, r;
	enum cmp_preprocessing save_pre;
	enum cmp_encoder_type save_enc;

	if (!ctx)
		return ERRV(GENERIC);
	if (ctx->magic != CTX_MAGIC)
		return ERRV(CONTEXT_INVALID);
	if (is_err(cap))
		return ERRV(GENERIC);
	if (ctx->params.checksum_enabled)
		raw += CMP_CHECKSUM_SIZE;
	if (!ctx->params.uncompressed_fallback_enabled || cap < raw)
		return host_engine(ctx, dst, cap, io);
	r = host_engine(ctx, dst, raw, io);
	if (cmp_get_error_code(r) != CMP_ERR_DST_TOO_SMALL)
		return r;
	r = cmp_reset(ctx);
	if (is_err(r))
		return r;
	save_pre = ctx->params.primary_preprocessing;
	save_enc = ctx->params.primary_encoder_type;
	ctx->params.primary_preprocessing = CMP_PREPROCESS_NONE;
	ctx->params.primary_encoder_type = CMP_ENCODER_UNCOMPRESSED;
	r = host_engine(ctx, dst, raw, io);
	ctx->params.primary_preprocessing = save_pre;
	ctx->params.primary_encoder_type = save_enc;
	return r;
}

static uint32_t host_compress(struct cmp_context *ctx, void *dst, uint32_t cap, const void *src,
			      uint32_t size, enum sample_kind kind)
{
	struct frame_io io;
	uint32_t stride = kind == KIND_I16_IN_I32 ? 4u : 2u, r;

	/* reference sample_reader.h:19-51 */
	if (!src)
		return ERRV(SRC_NULL);
	if (size == 0 || size % stride)
		return ERRV(SRC_SIZE_WRONG);
	memset(&io, 0, sizeof(io));
	io.src = src;
	io.n = size / stride;
	io.bytes = stride;
	io.kind = kind;
	pthread_mutex_lock(&g_host_lock);
	r = host_generic(ctx, dst, cap, &io);
	pthread_mutex_unlock(&g_host_lock);
	return r;
}

uint32_t cmp_compress_u16(struct cmp_context *ctx, void *dst, uint32_t dst_capacity, const uint16_t *src,
			  uint32_t src_size)
{
	return host_compress(ctx, dst, dst_capacity, src, src_size, KIND_U16);
}

uint32_t cmp_compress_i16(struct cmp_context *ctx, void *dst, uint32_t dst_capacity, const int16_t *src,
			  uint32_t src_size)
{
	return host_compress(ctx, dst, dst_capacity, src, src_size, KIND_I16);
}

uint32_t cmp_compress_i16_in_i32(struct cmp_context *ctx, void *dst, uint32_t dst_capacity,
				 const int32_t *src, uint32_t src_size)
{
	return host_compress(ctx, dst, dst_capacity, src, src_size, KIND_I16_IN_I32);
}

/* ================================================================== */
/* device batch API (cmp_gpu.h)                                       */
/* ================================================================== */

uint32_t cmp_gpu_decompress(struct cmp_gpu_engine *engine, const struct cmp_gpu_decode_batch *b)
{
	if (!engine || !b || !b->src || !b->dst || !b->status || !b->num_frames || b->num_frames > 65535u)
		return ERRV(GENERIC);
	if (((uintptr_t)b->src & 7u) || (b->src_stride & 7u) || b->src_capacity < HDR_MAX_SIZE ||
	    (b->src_capacity & 3u) || (b->num_frames > 1 && b->src_stride < b->src_capacity))
		return ERRV(GENERIC);
	if (b->model && (((uintptr_t)b->model & 1u) || (b->model_stride & 1u)))
		return ERRV(GENERIC);
	return airs_dev_decode(engine->dev, b->src, b->src_stride, b->src_capacity, b->num_frames, b->dst,
			       b->dst_stride, b->dst_samples, b->status, b->model, b->model_stride);
}

int cmp_gpu_available(void)
{
	return airs_dev_available();
}

uint32_t cmp_gpu_engine_create(struct cmp_gpu_engine **engine, void *hip_stream)
{
	struct cmp_gpu_engine *g;

	if (!engine)
		return ERRV(GENERIC);
	*engine = NULL;
	g = calloc(1, sizeof(*g));
	if (!g)
		return ERRV(GENERIC);
	g->dev = airs_dev_engine_create(hip_stream);
	if (!g->dev) {
		fprintf(stderr, "airscmp: cannot create GPU engine (%s)\n", airs_dev_last_error());
		free(g);
		return ERRV(GENERIC);
	}
	*engine = g;
	return 0;
}

uint32_t cmp_gpu_engine_set_option(struct cmp_gpu_engine *engine, uint32_t option, uint32_t value)
{
	if (!engine)
		return ERRV(GENERIC);
	return airs_dev_set_option(engine->dev, option, value);
}

void cmp_gpu_engine_destroy(struct cmp_gpu_engine *engine)
{
	if (!engine)
		return;
	airs_dev_engine_destroy(engine->dev);
	free(engine);
}

uint32_t cmp_gpu_synchronize(struct cmp_gpu_engine *engine)
{
	if (!engine)
		return ERRV(GENERIC);
	return airs_dev_sync(engine->dev);
}

uint32_t cmp_gpu_encode_stream(struct cmp_gpu_engine *engine, enum cmp_gpu_sample_type type, const void *src,
			       uint32_t num_samples, enum cmp_preprocessing preprocessing,
			       enum cmp_encoder_type encoder_type, uint32_t encoder_param, uint32_t encoder_outlier,
			       void *dst, uint32_t dst_capacity, uint32_t *size)
{
	const uint32_t bytes = type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	uint32_t e, outlier = 0;

	if (!engine || !size)
		return ERRV(GENERIC);
	if ((unsigned)type > CMP_GPU_I16_IN_I32)
		return ERRV(PARAMS_INVALID);
	if (!src)
		return ERRV(SRC_NULL);
	if (num_samples == 0 || num_samples > AIRS_STREAM_MAX)
		return ERRV(SRC_SIZE_WRONG);
	if ((uintptr_t)src % bytes) {
		fprintf(stderr, "airscmp: cmp_gpu_encode_stream: src must be %u-byte aligned\n", bytes);
		return ERRV(GENERIC);
	}
	if (!dst)
		return ERRV(DST_NULL);
	if ((uintptr_t)dst & 7u)
		return ERRV(DST_UNALIGNED);
	if (is_err(dst_capacity))
		return ERRV(GENERIC);
	if (preprocessing != CMP_PREPROCESS_NONE && preprocessing != CMP_PREPROCESS_DIFF)
		return ERRV(PARAMS_INVALID);
	/* the encoder's own checks (encoder.c:185-224) */
	e = coder_resolve(encoder_type, encoder_param, encoder_outlier, &outlier);
	if (is_err(e))
		return e;
	return airs_dev_encode_stream(engine->dev, src, bytes, num_samples, preprocessing, encoder_type,
				      encoder_type == CMP_ENCODER_UNCOMPRESSED ? 1u : encoder_param, encoder_outlier,
				      dst, dst_capacity, size);
}

uint32_t cmp_gpu_pack_frames(struct cmp_gpu_engine *engine, const void *frames, uint64_t frame_stride,
			     uint32_t frame_capacity, const uint32_t *sizes, uint32_t num_frames, void *out,
			     uint64_t *offsets)
{
	if (!engine || !frames || !sizes || !out || !offsets || !num_frames)
		return ERRV(GENERIC);
	if ((frame_stride & 7u) || ((uintptr_t)frames & 7u) || ((uintptr_t)out & 7u) ||
	    (num_frames > 1 && frame_stride < frame_capacity))
		return ERRV(DST_UNALIGNED);
	return airs_dev_pack_frames(engine->dev, frames, frame_stride, frame_capacity, sizes, num_frames,
				    ERRV(MAX_CODE), out, offsets);
}

uint32_t cmp_gpu_synthesize(struct cmp_gpu_engine *engine, void *dst, uint32_t sample_bytes, uint64_t seed,
			    uint32_t frame0, uint32_t samples_per_frame, uint32_t num_frames, uint64_t stride,
			    uint32_t noise_w)
{
	if (!engine || !dst || (sample_bytes != 2 && sample_bytes != 4))
		return ERRV(GENERIC);
	return airs_dev_synth(engine->dev, dst, sample_bytes, seed, frame0, samples_per_frame, num_frames,
			      stride, noise_w);
}

/* per-frame plan of a batch, computed by replaying the context state machine */
struct frame_plan {
	struct pass p;
	uint64_t id;
	uint32_t err; /* host-detected error for this frame, or 0 */
};

static int same_pass(const struct pass *a, const struct pass *b)
{
	return a->pre == b->pre && a->enc == b->enc && a->par == b->par &&
	       a->outlier_param == b->outlier_param && a->model_mode == b->model_mode && a->seq == b->seq;
}

/* is v[j] = v[0] + j*step for all j?  (step returned) */
static int affine_u64(const uint64_t *v, uint32_t cnt, uint64_t *step)
{
	uint32_t j;

	*step = cnt > 1 ? v[1] - v[0] : 0;
	for (j = 2; j < cnt; j++)
		if (v[j] - v[j - 1] != *step)
			return 0;
	return 1;
}

/* size of the raw (fallback) frame of a context, as cmp_compress_generic (cmp.c:342-393) */
static uint32_t raw_frame_size(const struct cmp_context *ctx, uint32_t n)
{
	return CMP_HDR_SIZE + 2u * n + (ctx->params.checksum_enabled ? CMP_CHECKSUM_SIZE : 0u);
}

/* Launch cnt frames that share one pass: launch frame j is batch frame
 * fl[j] (host list) or add + j*mul; output capacity cap.  coef (optional):
 * the work buffer of launch frame j, in place of its context's (IWT frames
 * of one context in one launch, batch_iwt). */
static uint32_t batch_launch(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t fpc,
			     const struct cmp_gpu_batch *b, const struct frame_plan *plan, const uint32_t *fl,
			     uint32_t add, uint32_t mul, uint32_t cnt, uint32_t cap, uint64_t *ids_scratch,
			     uint64_t *ptr_scratch, const uint64_t *coef)
{
	struct airs_dev_engine *dev = eng->dev;
	const uint32_t f0 = fl ? fl[0] : add;
	const struct pass *P = &plan[f0].p;
	const struct cmp_params *prm = &ctx[f0 / fpc].params;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes;
	uint32_t nframes_total = 0;
	struct airs_launch L;
	uint64_t step, worst = frame_worst(n);
	uint32_t j, e, *d_g = NULL, *d_ck = NULL, *d_fl = NULL;

#define FRAME_AT(jj) (fl ? fl[jj] : add + (jj) * mul)
	memset(&L, 0, sizeof(L));
	if (fl) {
		/* an affine list launches without a device copy */
		uint32_t aff = 1, m = cnt > 1 ? fl[1] - fl[0] : 1;

		for (j = 1; j < cnt && aff; j++)
			aff = fl[j] == fl[0] + j * m;
		if (aff) {
			add = fl[0];
			mul = m;
			fl = NULL;
		}
	}
	for (j = 0; j < cnt; j++) {
		const uint32_t f = FRAME_AT(j);

		ids_scratch[j] = plan[f].id;
		if (f + 1u > nframes_total)
			nframes_total = f + 1u;
	}
	if (fl) {
		d_fl = airs_dev_scratch(dev, SLOT_FL, (size_t)cnt * 4u);
		if (!d_fl || is_err(airs_dev_h2d(dev, d_fl, fl, (size_t)cnt * 4u)) || is_err(airs_dev_sync(dev)))
			return ERRV(GENERIC);
	}
	if (affine_u64(ids_scratch, cnt, &step)) {
		L.id_base = ids_scratch[0];
		L.id_step = step;
	} else {
		uint64_t *d_ids = airs_dev_scratch(dev, SLOT_IDS, (size_t)cnt * 8u);

		if (!d_ids || is_err(airs_dev_h2d(dev, d_ids, ids_scratch, (size_t)cnt * 8u)) ||
		    is_err(airs_dev_sync(dev)))
			return ERRV(GENERIC);
		L.ids = d_ids;
	}
	if (P->model_mode != AIRS_MODEL_NONE || P->pre == CMP_PREPROCESS_IWT) {
		for (j = 0; j < cnt; j++)
			ptr_scratch[j] = coef ? coef[j] : (uint64_t)(uintptr_t)ctx[FRAME_AT(j) / fpc].work_buf;
		/* model of frame f = base + (f / fpc) * stride when the work buffers are strided */
		if (coef) {
			uint64_t *d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)cnt * 8u);

			if (!d_ptr || is_err(airs_dev_h2d(dev, d_ptr, ptr_scratch, (size_t)cnt * 8u)) ||
			    is_err(airs_dev_sync(dev)))
				return ERRV(GENERIC);
			L.model_ptrs = d_ptr;
			L.model_ptrs_al16 = 1;
			for (j = 0; j < cnt; j++)
				if (ptr_scratch[j] & 15u)
					L.model_ptrs_al16 = 0;
		} else {
			uint64_t base = (uint64_t)(uintptr_t)ctx[0].work_buf, mstep = 0;
			uint32_t c, ok = 1, nctx = (nframes_total + fpc - 1) / fpc;

			if (nctx > 1)
				mstep = (uint64_t)(uintptr_t)ctx[1].work_buf - base;
			for (c = 0; c < nctx && ok; c++)
				ok = (uint64_t)(uintptr_t)ctx[c].work_buf == base + c * mstep;
			if (ok) {
				L.model = (void *)(uintptr_t)base;
				L.model_stride = mstep;
				L.model_div = fpc;
			} else {
				uint64_t *d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)cnt * 8u);

				if (!d_ptr || is_err(airs_dev_h2d(dev, d_ptr, ptr_scratch, (size_t)cnt * 8u)) ||
				    is_err(airs_dev_sync(dev)))
					return ERRV(GENERIC);
				L.model_ptrs = d_ptr;
				L.model_ptrs_al16 = 1;
				for (j = 0; j < cnt; j++)
					if (ptr_scratch[j] & 15u)
						L.model_ptrs_al16 = 0;
			}
		}
	}
#undef FRAME_AT
	if (prm->checksum_enabled) {
		d_ck = airs_dev_scratch(dev, SLOT_CK, (size_t)nframes_total * 4u);
		if (!d_ck)
			return ERRV(GENERIC);
		if (fl)
			e = airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, cnt, d_fl, d_ck);
		else if (mul == 1)
			e = airs_dev_checksum(dev, (const uint8_t *)b->src + (uint64_t)add * b->src_stride,
					      b->src_stride, bytes, n, cnt, NULL, d_ck + add);
		else
			e = airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, nframes_total, NULL, d_ck);
		if (is_err(e))
			return e;
	}
	if ((b->flags & CMP_GPU_AUTO_RICE) && P->enc == CMP_ENCODER_GOLOMB_ZERO &&
	    (P->pre == CMP_PREPROCESS_NONE || P->pre == CMP_PREPROCESS_DIFF || P->pre == CMP_PREPROCESS_IWT)) {
		d_g = airs_dev_scratch(dev, SLOT_G, (size_t)nframes_total * 4u);
		if (!d_g)
			return ERRV(GENERIC);
		L.auto_rice = 1;
		L.frame_g_scratch = d_g;
	}
	L.src = b->src;
	L.src_stride = b->src_stride;
	L.sample_bytes = bytes;
	L.is_unsigned = b->type == CMP_GPU_U16;
	L.n = n;
	L.num_frames = cnt;
	L.frame_list = d_fl;
	L.frame_add = add;
	L.frame_mul = mul;
	L.dst = b->dst;
	L.dst_stride = b->dst_stride;
	L.cap = (uint64_t)cap < worst ? cap : (uint32_t)worst;
	L.preprocessing = P->pre;
	L.encoder_type = P->enc;
	L.encoder_param = P->par;
	L.outlier_param = P->outlier_param;
	L.model_mode = P->model_mode;
	L.model_rate = prm->model_rate;
	/* a frame that runs out of room in a fallback-sized first attempt falls
	 * back, and the fallback stores the whole model: no fail bit needed */
	L.fail_bit = (prm->uncompressed_fallback_enabled && cap == raw_frame_size(&ctx[f0 / fpc], n))
			     ? UINT64_MAX
			     : model_fail_bit(cap, n);
	L.seq = P->seq;
	L.checksum_enabled = prm->checksum_enabled ? 1u : 0u;
	L.checksums = d_ck;
	L.status = b->sizes;
	return airs_dev_encode(dev, &L);
}

/* launch every frame of `list` (batch frames of one acquisition step): one
 * launch per run of frames with the same pass and capacity */
static uint32_t launch_groups(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t fpc,
			      const struct cmp_gpu_batch *b, const struct frame_plan *plan, const uint32_t *list,
			      const uint32_t *caps, uint32_t cnt, uint32_t *grp, uint8_t *done, uint64_t *ids,
			      uint64_t *ptrs)
{
	uint32_t i, k, e = 0;

	memset(done, 0, cnt);
	for (i = 0; i < cnt && !is_err(e); i++) {
		uint32_t g = 0;

		if (done[i])
			continue;
		for (k = i; k < cnt; k++) {
			if (!done[k] && caps[k] == caps[i] && same_pass(&plan[list[k]].p, &plan[list[i]].p) &&
			    ctx[list[k] / fpc].params.model_rate == ctx[list[i] / fpc].params.model_rate &&
			    ctx[list[k] / fpc].params.checksum_enabled == ctx[list[i] / fpc].params.checksum_enabled &&
			    /* batch_launch decides the model fail bit from the
			     * launch's first context: one fallback setting per launch */
			    !ctx[list[k] / fpc].params.uncompressed_fallback_enabled ==
				    !ctx[list[i] / fpc].params.uncompressed_fallback_enabled) {
				grp[g++] = list[k];
				done[k] = 1;
			}
		}
		e = batch_launch(eng, ctx, fpc, b, plan, grp, 0, 1, g, caps[i], ids, ptrs, NULL);
	}
	return e;
}

/*
 * Exact mode: one acquisition step at a time, as the host API would run it.
 * Used when a frame can fail or fall back to raw storage, because the
 * outcome of frame (c, a) decides the pass (and identifier draws) of frame
 * (c, a+1).  Per step: plan every context, launch, read the sizes back, run
 * the fallback frames (cmp_compress_generic: reset, NONE + UNCOMPRESSED at
 * the raw size), and advance the contexts that succeeded.  Identifier draws
 * are counted per frame and made at the end in the reference's call order
 * (context-major), then written into the headers.
 */
static uint32_t batch_exact(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx, uint32_t fpc,
			    const struct cmp_gpu_batch *b, struct frame_plan *plan, uint64_t *ids, uint64_t *ptrs)
{
	struct airs_dev_engine *dev = eng->dev;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	uint32_t *draws = calloc(total, sizeof(uint32_t));
	uint32_t *list = calloc(num_ctx, sizeof(uint32_t)), *caps = calloc(num_ctx, sizeof(uint32_t));
	uint32_t *grp = calloc(num_ctx, sizeof(uint32_t)), *sz = calloc(num_ctx, sizeof(uint32_t));
	uint32_t *fbl = calloc(num_ctx, sizeof(uint32_t)), *fbc = calloc(num_ctx, sizeof(uint32_t));
	uint32_t *perr = calloc(num_ctx, sizeof(uint32_t));
	uint64_t *id0 = calloc(num_ctx, sizeof(uint64_t));
	uint8_t *done = calloc(num_ctx, 1);
	uint32_t a, c, e = 0;

	if (!draws || !list || !caps || !grp || !sz || !fbl || !fbc || !perr || !id0 || !done) {
		e = ERRV(GENERIC);
		goto out;
	}
	for (c = 0; c < num_ctx; c++)
		id0[c] = ctx[c].identifier;
	for (a = 0; a < fpc && !is_err(e); a++) {
		uint32_t nfb = 0, nl = 0;

		for (c = 0; c < num_ctx && !is_err(e); c++) {
			const uint32_t f = c * fpc + a, raw = raw_frame_size(&ctx[c], n);
			void *dst = (uint8_t *)b->dst + (uint64_t)f * b->dst_stride;

			const uint32_t cap = ctx[c].params.uncompressed_fallback_enabled && b->dst_capacity >= raw
						     ? raw
						     : b->dst_capacity;
			/* a frame the host API rejects before encoding keeps its error */
			perr[c] = engine_prologue(&ctx[c], dst, cap, n, &plan[f].p, &draws[f]);
			plan[f].id = 0; /* written at the end */
			if (is_err(perr[c])) {
				e = airs_dev_h2d(dev, b->sizes + f, &perr[c], 4u);
			} else {
				list[nl] = f;
				caps[nl++] = cap;
			}
		}
		if (is_err(e))
			break;
		if (nl)
			e = launch_groups(eng, ctx, fpc, b, plan, list, caps, nl, grp, done, ids, ptrs);
		if (is_err(e))
			break;
		/* sizes of this step (frames c*fpc + a: strided in the sizes array) */
		for (c = 0; c < num_ctx && !is_err(e); c++) {
			sz[c] = perr[c];
			if (!is_err(perr[c]))
				e = airs_dev_d2h(dev, &sz[c], b->sizes + (uint64_t)c * fpc + a, 4u);
		}
		if (is_err(e) || is_err(e = airs_dev_sync(dev)))
			break;
		for (c = 0; c < num_ctx && !is_err(e); c++) {
			const uint32_t f = c * fpc + a, raw = raw_frame_size(&ctx[c], n);
			enum cmp_preprocessing save_pre;
			enum cmp_encoder_type save_enc;
			void *dst = (uint8_t *)b->dst + (uint64_t)f * b->dst_stride;

			/* sz[c] holds the prologue's error when the frame was rejected
			 * before encoding (e.g. raw size below the compressed header) */
			if (!(ctx[c].params.uncompressed_fallback_enabled && b->dst_capacity >= raw &&
			      cmp_get_error_code(sz[c]) == CMP_ERR_DST_TOO_SMALL))
				continue;
			/* cmp.c:342-393: reset, then the frame again as NONE + UNCOMPRESSED */
			e = ctx_reset(&ctx[c], &draws[f]);
			if (is_err(e))
				break;
			save_pre = ctx[c].params.primary_preprocessing;
			save_enc = ctx[c].params.primary_encoder_type;
			ctx[c].params.primary_preprocessing = CMP_PREPROCESS_NONE;
			ctx[c].params.primary_encoder_type = CMP_ENCODER_UNCOMPRESSED;
			perr[c] = engine_prologue(&ctx[c], dst, raw, n, &plan[f].p, &draws[f]);
			ctx[c].params.primary_preprocessing = save_pre;
			ctx[c].params.primary_encoder_type = save_enc;
			plan[f].id = 0;
			if (is_err(perr[c])) {
				sz[c] = perr[c];
				e = airs_dev_h2d(dev, b->sizes + f, &perr[c], 4u);
				continue;
			}
			fbl[nfb] = f;
			fbc[nfb++] = raw;
		}
		if (is_err(e))
			break;
		if (nfb) {
			e = launch_groups(eng, ctx, fpc, b, plan, fbl, fbc, nfb, grp, done, ids, ptrs);
			for (c = 0; c < nfb && !is_err(e); c++)
				e = airs_dev_d2h(dev, &sz[fbl[c] / fpc], b->sizes + fbl[c], 4u);
			if (is_err(e) || is_err(e = airs_dev_sync(dev)))
				break;
		}
		for (c = 0; c < num_ctx; c++)
			if (!is_err(sz[c]))
				ctx[c].sequence_number++;
	}
	if (is_err(e))
		goto out;
	/* identifiers in call order; frames without a draw carry the context's */
	{
		uint64_t *d_ids;

		for (c = 0; c < num_ctx; c++) {
			uint64_t id = id0[c];

			for (a = 0; a < fpc; a++) {
				const uint32_t f = c * fpc + a;
				uint32_t k;

				for (k = 0; k < draws[f]; k++)
					id = next_identifier();
				ids[f] = id;
				if (REPORT_DRAWS(b))
					b->draws[f] = (uint8_t)draws[f];
			}
			ctx[c].identifier = id;
		}
		d_ids = airs_dev_scratch(dev, SLOT_IDS, (size_t)total * 8u);
		if (!d_ids || is_err(airs_dev_h2d(dev, d_ids, ids, (size_t)total * 8u)))
			e = ERRV(GENERIC);
		else
			e = airs_dev_patch_ids(dev, b->dst, b->dst_stride, total, 0, 1, d_ids, b->sizes);
		if (!is_err(e))
			e = airs_dev_sync(dev);
	}
out:
	free(draws);
	free(list);
	free(caps);
	free(grp);
	free(sz);
	free(fbl);
	free(fbc);
	free(perr);
	free(id0);
	free(done);
	return e;
}

/*
 * Exact mode on the device.  When every context has the same parameters and
 * the prologue's static checks pass for both passes, the state machine
 * that batch_exact() steps on the host runs on the GPU instead
 * (airs_dev_fb_step / airs_dev_fb_copy, airs_dev.h): per acquisition step a
 * planning kernel, the primary-pass launch, the secondary-pass launch (holes
 * in their frame lists skip the contexts on the other pass) and the raw
 * frames of the previous step's fallbacks.  The only host round trip is one
 * read-back of the identifier draw counts and context states at the end;
 * identifiers are then drawn in call order and patched into the headers.
 */
static int same_params(const struct cmp_params *x, const struct cmp_params *y)
{
	return x->primary_preprocessing == y->primary_preprocessing &&
	       x->primary_encoder_type == y->primary_encoder_type &&
	       x->primary_encoder_param == y->primary_encoder_param &&
	       x->primary_encoder_outlier == y->primary_encoder_outlier &&
	       x->secondary_iterations == y->secondary_iterations &&
	       x->secondary_preprocessing == y->secondary_preprocessing &&
	       x->secondary_encoder_type == y->secondary_encoder_type &&
	       x->secondary_encoder_param == y->secondary_encoder_param &&
	       x->secondary_encoder_outlier == y->secondary_encoder_outlier && x->model_rate == y->model_rate &&
	       x->checksum_enabled == y->checksum_enabled &&
	       x->uncompressed_fallback_enabled == y->uncompressed_fallback_enabled;
}

/* first-attempt capacity of a frame (cmp_compress_generic, cmp.c:358-366) */
static uint32_t first_cap(const struct cmp_context *ctx, const struct cmp_gpu_batch *b, uint32_t n)
{
	const uint32_t raw = raw_frame_size(ctx, n);

	return ctx->params.uncompressed_fallback_enabled && b->dst_capacity >= raw ? raw : b->dst_capacity;
}

/* can batch_device_exact() run this batch?  pp / ps receive the two passes */
static int device_exact_ok(const struct cmp_context *ctx, uint32_t num_ctx, const struct cmp_gpu_batch *b,
			   uint32_t n, struct pass *pp, struct pass *ps)
{
	const struct cmp_params *P = &ctx[0].params;
	uint32_t c, draws = 0;

	for (c = 0; c < num_ctx; c++) {
		struct cmp_context t;
		struct pass p;

		if (!same_params(&ctx[c].params, P))
			return 0;
		t = ctx[c];
		t.sequence_number = 0;
		if (is_err(engine_prologue(&t, b->dst, first_cap(&ctx[c], b, n), n, &p, &draws)))
			return 0;
		if (c == 0)
			*pp = p;
		if (P->secondary_iterations) {
			t = ctx[c];
			t.sequence_number = 1;
			t.model_size = 2u * n;
			if (is_err(engine_prologue(&t, b->dst, first_cap(&ctx[c], b, n), n, &p, &draws)))
				return 0;
			if (c == 0)
				*ps = p;
		}
	}
	return 1;
}

static uint32_t batch_device_exact(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx,
				   uint32_t fpc, const struct cmp_gpu_batch *b, const struct pass *pp,
				   const struct pass *ps, uint64_t *ids)
{
	struct airs_dev_engine *dev = eng->dev;
	const struct cmp_params *P = &ctx[0].params;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	const uint32_t cap1 = first_cap(&ctx[0], b, n), mneed = model_needed(P) ? 1u : 0u;
	const uint32_t wneed = work_buf_state(P) ? 1u : 0u; /* the model, or IWT coefficients */
	const size_t words = 4u * (size_t)num_ctx, tb = ((size_t)total + 15u) & ~(size_t)15u;
	uint32_t *host_state = calloc(2u * (size_t)num_ctx, sizeof(uint32_t));
	uint8_t *host_draws = calloc(total, 1);
	uint8_t *scr = airs_dev_scratch(dev, SLOT_FL, words * 4u + 4u * tb);
	uint32_t *d_ck = NULL, *d_g = NULL, c, a, e = 0;
	uint64_t *d_ptr = NULL, mstride = 0;
	void *mbase = NULL;
	uint32_t mal16 = 0;
	struct airs_fb_step S;

	if (!host_state || !host_draws || !scr) {
		e = ERRV(GENERIC);
		goto out;
	}
	memset(&S, 0, sizeof(S));
	S.state = (uint32_t *)scr;
	S.flist_p = S.state + 2u * num_ctx;
	S.flist_s = S.flist_p + num_ctx;
	S.seqs = scr + words * 4u;
	S.draws = S.seqs + tb;
	S.kind = S.draws + tb;
	S.fb = S.kind + tb;
	S.num_ctx = num_ctx;
	S.fpc = fpc;
	S.packed = 2u * n;
	S.iters = P->secondary_iterations;
	S.model_needed = mneed;
	S.raw_size = raw_frame_size(&ctx[0], n);
	S.fb_eligible = cap1 == S.raw_size && P->uncompressed_fallback_enabled;
	S.err_floor = ERRV(MAX_CODE);
	S.err_small = ERRV(DST_TOO_SMALL);
	S.err_mismatch = ERRV(SRC_SIZE_MISMATCH);
	S.err_too_large = ERRV(HDR_CMP_SIZE_TOO_LARGE);
	S.status = b->sizes;
	S.src = b->src;
	S.src_stride = b->src_stride;
	S.sample_bytes = bytes;
	S.n = n;
	S.dst = b->dst;
	S.dst_stride = b->dst_stride;
	S.checksum = P->checksum_enabled ? 1u : 0u;
	for (c = 0; c < num_ctx; c++) {
		host_state[2u * c] = ctx[c].sequence_number;
		host_state[2u * c + 1u] = ctx[c].model_size;
	}
	e = airs_dev_h2d(dev, S.state, host_state, 8u * (size_t)num_ctx);
	if (!is_err(e))
		e = airs_dev_memset(dev, S.fb, 0, tb);
	/* work buffers: strided, or a pointer per context */
	if (!is_err(e) && wneed) {
		uint64_t base = (uint64_t)(uintptr_t)ctx[0].work_buf;
		int ok = 1, al = 1;

		mstride = num_ctx > 1 ? (uint64_t)(uintptr_t)ctx[1].work_buf - base : 0;
		for (c = 0; c < num_ctx; c++) {
			ok = ok && (uint64_t)(uintptr_t)ctx[c].work_buf == base + c * mstride;
			al = al && ((uintptr_t)ctx[c].work_buf & 15u) == 0;
		}
		if (ok) {
			mbase = ctx[0].work_buf;
			S.model = mbase;
			S.model_stride = mstride;
		} else {
			uint64_t *hp = calloc(num_ctx, sizeof(uint64_t));

			d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)num_ctx * 8u);
			if (!hp || !d_ptr) {
				free(hp);
				e = ERRV(GENERIC);
			} else {
				for (c = 0; c < num_ctx; c++)
					hp[c] = (uint64_t)(uintptr_t)ctx[c].work_buf;
				e = airs_dev_h2d(dev, d_ptr, hp, (size_t)num_ctx * 8u);
				if (!is_err(e))
					e = airs_dev_sync(dev);
				free(hp);
				S.model_ptrs = d_ptr;
			}
		}
		mal16 = al;
	}
	if (!is_err(e) && P->checksum_enabled) {
		d_ck = airs_dev_scratch(dev, SLOT_CK, (size_t)total * 4u);
		e = d_ck ? airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, total, NULL, d_ck) : ERRV(GENERIC);
		S.checksums = d_ck;
	}
	if (!is_err(e) && (b->flags & CMP_GPU_AUTO_RICE)) {
		d_g = airs_dev_scratch(dev, SLOT_G, (size_t)total * 4u);
		if (!d_g)
			e = ERRV(GENERIC);
	}
	for (a = 0; a <= fpc && !is_err(e); a++) {
		S.prev = (int32_t)a - 1;
		S.cur = a < fpc ? (int32_t)a : -1;
		e = airs_dev_fb_step(dev, &S);
		if (!is_err(e) && a > 0 && S.fb_eligible)
			e = airs_dev_fb_copy(dev, &S);
		if (a == fpc)
			break;
		for (uint32_t which = 0; which < (S.iters ? 2u : 1u) && !is_err(e); which++) {
			const struct pass *Q = which ? ps : pp;
			struct airs_launch L;

			memset(&L, 0, sizeof(L));
			L.src = b->src;
			L.src_stride = b->src_stride;
			L.sample_bytes = bytes;
			L.is_unsigned = b->type == CMP_GPU_U16;
			L.n = n;
			L.num_frames = num_ctx;
			L.frame_list = which ? S.flist_s : S.flist_p;
			L.dst = b->dst;
			L.dst_stride = b->dst_stride;
			L.cap = (uint64_t)cap1 < frame_worst(n) ? cap1 : (uint32_t)frame_worst(n);
			L.preprocessing = Q->pre;
			L.encoder_type = Q->enc;
			L.encoder_param = Q->par;
			L.outlier_param = Q->outlier_param;
			if (d_g && Q->enc == CMP_ENCODER_GOLOMB_ZERO &&
			    (Q->pre == CMP_PREPROCESS_NONE || Q->pre == CMP_PREPROCESS_DIFF || Q->pre == CMP_PREPROCESS_IWT)) {
				L.auto_rice = 1;
				L.frame_g_scratch = d_g;
			}
			L.model_mode = mneed ? (which ? AIRS_MODEL_UPDATE : AIRS_MODEL_STORE) : AIRS_MODEL_NONE;
			L.model_rate = P->model_rate;
			L.model = mbase;
			L.model_stride = mstride;
			L.model_div = fpc;
			L.model_ptrs = d_ptr;
			L.model_ptrs_al16 = mal16;
			/* a first attempt that runs out of room falls back, and the
			 * fallback stores the whole model: no fail bit needed then */
			L.fail_bit = S.fb_eligible ? UINT64_MAX : model_fail_bit(cap1, n);
			L.seqs = S.seqs;
			L.checksum_enabled = S.checksum;
			L.checksums = d_ck;
			L.status = b->sizes;
			e = airs_dev_encode(dev, &L);
		}
	}
	/* the one read-back: identifier draws and the final context states */
	if (!is_err(e))
		e = airs_dev_d2h(dev, host_draws, S.draws, total);
	if (!is_err(e))
		e = airs_dev_d2h(dev, host_state, S.state, 8u * (size_t)num_ctx);
	if (!is_err(e))
		e = airs_dev_sync(dev);
	if (is_err(e))
		goto out;
	for (c = 0; c < num_ctx; c++) {
		uint64_t id = ctx[c].identifier;

		for (a = 0; a < fpc; a++) {
			const uint32_t f = c * fpc + a;

			for (uint32_t k = 0; k < host_draws[f]; k++)
				id = next_identifier();
			ids[f] = id;
			if (REPORT_DRAWS(b))
				b->draws[f] = host_draws[f];
		}
		ctx[c].identifier = id;
		ctx[c].sequence_number = (uint8_t)host_state[2u * c];
		ctx[c].model_size = host_state[2u * c + 1u];
	}
	{
		uint64_t *d_ids = airs_dev_scratch(dev, SLOT_IDS, (size_t)total * 8u);

		if (!d_ids || is_err(airs_dev_h2d(dev, d_ids, ids, (size_t)total * 8u)))
			e = ERRV(GENERIC);
		else
			e = airs_dev_patch_ids(dev, b->dst, b->dst_stride, total, 0, 1, d_ids, b->sizes);
		if (!is_err(e))
			e = airs_dev_sync(dev);
	}
out:
	free(host_state);
	free(host_draws);
	return e;
}

/*
 * MODEL contexts in one launch (airs_dev_walk, enc_walk.hip): every frame of
 * the batch, acquisition after acquisition, with each context's model kept on
 * the chip.  Used in the asynchronous mode (no frame can fail or fall back)
 * when every context has the same parameters with a MODEL secondary pass and
 * the plan the host replayed is the one the walk's pass rule gives.
 * Returns 0, an error value, or WALK_NO (not applicable; nothing launched).
 */
#define WALK_NO 1u
static uint32_t batch_walk(struct cmp_gpu_engine *eng, const struct cmp_context *ctx, uint32_t num_ctx, uint32_t fpc,
			   const struct cmp_gpu_batch *b, const struct frame_plan *plan)
{
	struct airs_dev_engine *dev = eng->dev;
	const struct cmp_params *P = &ctx[0].params;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	const uint64_t worst = frame_worst(n);
	struct airs_walk w;
	uint32_t c, a, e, seq_same = 1, id_aff = 1, m_strided = 1;
	uint64_t mbase, mstep;

	if (!model_needed(P) || (P->primary_preprocessing != CMP_PREPROCESS_NONE &&
				 P->primary_preprocessing != CMP_PREPROCESS_DIFF))
		return WALK_NO;
	/* the walk codes with the configured parameters (AUTO_RICE: per-step launches) */
	if ((b->flags & CMP_GPU_AUTO_RICE) && P->primary_encoder_type == CMP_ENCODER_GOLOMB_ZERO)
		return WALK_NO;
	for (c = 0; c < num_ctx; c++)
		if (!same_params(&ctx[c].params, P))
			return WALK_NO;
	memset(&w, 0, sizeof(w));
	w.src = b->src;
	w.src_stride = b->src_stride;
	w.sample_bytes = bytes;
	w.is_unsigned = b->type == CMP_GPU_U16;
	w.n = n;
	w.num_ctx = num_ctx;
	w.fpc = fpc;
	w.dst = b->dst;
	w.dst_stride = b->dst_stride;
	w.cap = (uint64_t)b->dst_capacity < worst ? b->dst_capacity : (uint32_t)worst;
	w.pre_p = P->primary_preprocessing;
	w.enc_p = P->primary_encoder_type;
	w.g_p = P->primary_encoder_param;
	w.outl_p = P->primary_encoder_outlier;
	w.enc_s = P->secondary_encoder_type;
	w.g_s = P->secondary_encoder_param;
	w.outl_s = P->secondary_encoder_outlier;
	w.model_rate = P->model_rate;
	w.iters = P->secondary_iterations;
	w.checksum_enabled = P->checksum_enabled ? 1u : 0u;
	w.status = b->sizes;
	/* the walk's pass rule (cmp.c:228-248), started from each context's
	 * first frame, must give the replayed plan frame by frame */
	for (c = 0; c < num_ctx; c++) {
		uint32_t sq = plan[c * fpc].p.seq;

		if (sq != plan[0].p.seq)
			seq_same = 0;
		for (a = 0; a < fpc; a++) {
			const struct pass *p = &plan[c * fpc + a].p;
			const int prim = sq == 0 || sq > w.iters;

			if (p->seq != (prim ? 0u : sq) ||
			    p->pre != (prim ? w.pre_p : (uint32_t)CMP_PREPROCESS_MODEL) ||
			    p->enc != (prim ? w.enc_p : w.enc_s) || p->par != (prim ? w.g_p : w.g_s) ||
			    p->model_mode != (prim ? (uint32_t)AIRS_MODEL_STORE : (uint32_t)AIRS_MODEL_UPDATE))
				return WALK_NO;
			sq = prim ? 1u : sq + 1u;
		}
	}
	w.seq0 = plan[0].p.seq;
	/* model of context c: strided work buffers, or a pointer list */
	mbase = (uint64_t)(uintptr_t)ctx[0].work_buf;
	mstep = num_ctx > 1 ? (uint64_t)(uintptr_t)ctx[1].work_buf - mbase : 0;
	for (c = 0; c < num_ctx && m_strided; c++)
		m_strided = (uint64_t)(uintptr_t)ctx[c].work_buf == mbase + c * mstep;
	if (!m_strided)
		for (c = 0; c < num_ctx; c++)
			if ((uintptr_t)ctx[c].work_buf & 15u)
				return WALK_NO;
	w.model = (void *)(uintptr_t)mbase;
	w.model_stride = m_strided ? mstep : 0;
	/* identifiers: base + c cstep + a astep, or a list */
	w.id_base = plan[0].id;
	w.id_cstep = num_ctx > 1 ? plan[fpc].id - plan[0].id : 0;
	w.id_astep = fpc > 1 ? plan[1].id - plan[0].id : 0;
	for (c = 0; c < num_ctx && id_aff; c++)
		for (a = 0; a < fpc && id_aff; a++)
			id_aff = plan[c * fpc + a].id == w.id_base + c * w.id_cstep + a * w.id_astep;
	{
		struct airs_walk chk = w;

		if (!m_strided) /* the pointer list is checked for alignment above */
			chk.model = NULL, chk.model_stride = 0;
		if (!airs_dev_walk_supported(&chk))
			return WALK_NO;
	}
	/* device copies of what is not affine; the stream is synchronised before
	 * the host arrays are freed */
	if (!m_strided || !id_aff || !seq_same) {
		uint64_t *d_ptr = NULL, *d_ids = NULL, *h_ptr = NULL, *h_ids = NULL;
		uint8_t *d_seq = NULL, *h_seq = NULL;

		e = 0;
		if (!m_strided) {
			h_ptr = malloc((size_t)num_ctx * 8u);
			d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)num_ctx * 8u);
			if (!h_ptr || !d_ptr)
				e = ERRV(GENERIC);
			for (c = 0; c < num_ctx && !is_err(e); c++)
				h_ptr[c] = (uint64_t)(uintptr_t)ctx[c].work_buf;
			if (!is_err(e))
				e = airs_dev_h2d(dev, d_ptr, h_ptr, (size_t)num_ctx * 8u);
			w.model_ptrs = d_ptr;
		}
		if (!id_aff && !is_err(e)) {
			h_ids = malloc((size_t)total * 8u);
			d_ids = airs_dev_scratch(dev, SLOT_IDS, (size_t)total * 8u);
			if (!h_ids || !d_ids)
				e = ERRV(GENERIC);
			for (c = 0; c < total && !is_err(e); c++)
				h_ids[c] = plan[c].id;
			if (!is_err(e))
				e = airs_dev_h2d(dev, d_ids, h_ids, (size_t)total * 8u);
			w.ids = d_ids;
		}
		if (!seq_same && !is_err(e)) {
			h_seq = malloc(num_ctx);
			d_seq = airs_dev_scratch(dev, SLOT_FL, num_ctx);
			if (!h_seq || !d_seq)
				e = ERRV(GENERIC);
			for (c = 0; c < num_ctx && !is_err(e); c++)
				h_seq[c] = (uint8_t)plan[c * fpc].p.seq;
			if (!is_err(e))
				e = airs_dev_h2d(dev, d_seq, h_seq, num_ctx);
			w.seq0s = d_seq;
		}
		if (!is_err(e))
			e = airs_dev_sync(dev);
		free(h_ptr);
		free(h_ids);
		free(h_seq);
		if (is_err(e))
			return e;
	}
	if (P->checksum_enabled) {
		uint32_t *d_ck = airs_dev_scratch(dev, SLOT_CK, (size_t)total * 4u);

		if (!d_ck)
			return ERRV(GENERIC);
		e = airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, total, NULL, d_ck);
		if (is_err(e))
			return e;
		w.checksums = d_ck;
	}
	return airs_dev_walk(dev, &w);
}

/*
 * MODEL contexts with the uncompressed fallback in one launch (the context
 * walk, enc_walk.hip): the walk resolves each frame's fallback on the chip
 * (cmp.c:342-393) and reports every frame's identifier draws and each
 * context's final sequence number; one read-back, then the identifiers are
 * drawn in call order and patched into the headers, as batch_device_exact
 * does.  Applies when the fallback is the only way a frame's outcome can
 * change the next frame's pass: every context with the same parameters, the
 * fallback enabled and dst_capacity >= the raw frame size (the first
 * attempt's capacity is then the raw size, so a frame either fits or falls
 * back), and no secondary first frame whose model size differs (no
 * SRC_SIZE_MISMATCH).  Returns 0, an error value, or WALK_NO.
 */
static uint32_t batch_walk_fb(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx, uint32_t fpc,
			      const struct cmp_gpu_batch *b, uint64_t *ids)
{
	struct airs_dev_engine *dev = eng->dev;
	const struct cmp_params *P = &ctx[0].params;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	const uint32_t raw = raw_frame_size(&ctx[0], n);
	const size_t tb = ((size_t)total + 15u) & ~(size_t)15u;
	struct airs_walk w;
	uint32_t c, a, e = 0, seq_same = 1, m_strided = 1;
	uint64_t mbase, mstep;
	uint8_t *h_draws = NULL, *h_seq = NULL, *scr, *h_seq0 = NULL;
	uint64_t *h_ids = NULL;

	if (!model_needed(P) || !P->uncompressed_fallback_enabled || b->dst_capacity < raw || raw > 0xFFFFFFu ||
	    (P->primary_preprocessing != CMP_PREPROCESS_NONE && P->primary_preprocessing != CMP_PREPROCESS_DIFF))
		return WALK_NO;
	if ((b->flags & CMP_GPU_AUTO_RICE) && P->primary_encoder_type == CMP_ENCODER_GOLOMB_ZERO)
		return WALK_NO;
	for (c = 0; c < num_ctx; c++) {
		const uint32_t sq = ctx[c].sequence_number;

		if (!same_params(&ctx[c].params, P))
			return WALK_NO;
		if (sq != 0u && sq <= P->secondary_iterations && ctx[c].model_size != 2u * n)
			return WALK_NO; /* the reference returns SRC_SIZE_MISMATCH for that frame */
		if (sq != ctx[0].sequence_number)
			seq_same = 0;
	}
	memset(&w, 0, sizeof(w));
	w.src = b->src;
	w.src_stride = b->src_stride;
	w.sample_bytes = bytes;
	w.is_unsigned = b->type == CMP_GPU_U16;
	w.n = n;
	w.num_ctx = num_ctx;
	w.fpc = fpc;
	w.dst = b->dst;
	w.dst_stride = b->dst_stride;
	w.cap = raw; /* the first attempt's capacity (cmp.c:358-366) */
	w.pre_p = P->primary_preprocessing;
	w.enc_p = P->primary_encoder_type;
	w.g_p = P->primary_encoder_param;
	w.outl_p = P->primary_encoder_outlier;
	w.enc_s = P->secondary_encoder_type;
	w.g_s = P->secondary_encoder_param;
	w.outl_s = P->secondary_encoder_outlier;
	w.model_rate = P->model_rate;
	w.iters = P->secondary_iterations;
	w.checksum_enabled = P->checksum_enabled ? 1u : 0u;
	w.status = b->sizes;
	w.seq0 = ctx[0].sequence_number;
	w.fb = 1;
	w.raw_size = raw;
	mbase = (uint64_t)(uintptr_t)ctx[0].work_buf;
	mstep = num_ctx > 1 ? (uint64_t)(uintptr_t)ctx[1].work_buf - mbase : 0;
	for (c = 0; c < num_ctx && m_strided; c++)
		m_strided = (uint64_t)(uintptr_t)ctx[c].work_buf == mbase + c * mstep;
	if (!m_strided)
		for (c = 0; c < num_ctx; c++)
			if ((uintptr_t)ctx[c].work_buf & 15u)
				return WALK_NO;
	w.model = (void *)(uintptr_t)mbase;
	w.model_stride = m_strided ? mstep : 0;
	/* scratch: draws [tb], final sequence numbers [num_ctx], first sequence numbers [num_ctx] */
	scr = airs_dev_scratch(dev, SLOT_FL, tb + 2u * (size_t)num_ctx + 16u);
	if (!scr)
		return ERRV(GENERIC);
	w.draws = scr;
	w.seq_out = scr + tb;
	{
		struct airs_walk chk = w;

		if (!m_strided)
			chk.model = NULL, chk.model_stride = 0;
		if (!airs_dev_walk_supported(&chk))
			return WALK_NO;
	}
	/* page-locked host scratch: draws [tb], final sequence numbers [num_ctx]
	 * (one read-back of the device scratch's first tb + num_ctx bytes), then
	 * the identifiers [total] at the next 8-byte boundary */
	{
		const size_t ioff = (tb + num_ctx + 7u) & ~(size_t)7u;
		uint8_t *hp = airs_dev_host_scratch(dev, ioff + (size_t)total * 8u);

		if (!hp)
			return ERRV(GENERIC);
		h_draws = hp;
		h_seq = hp + tb;
		h_ids = (uint64_t *)(void *)(hp + ioff);
	}
	if (!m_strided) {
		uint64_t *hp = malloc((size_t)num_ctx * 8u), *d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)num_ctx * 8u);

		if (!hp || !d_ptr)
			e = ERRV(GENERIC);
		for (c = 0; c < num_ctx && !is_err(e); c++)
			hp[c] = (uint64_t)(uintptr_t)ctx[c].work_buf;
		if (!is_err(e))
			e = airs_dev_h2d(dev, d_ptr, hp, (size_t)num_ctx * 8u);
		if (!is_err(e))
			e = airs_dev_sync(dev);
		free(hp);
		w.model_ptrs = d_ptr;
	}
	if (!seq_same && !is_err(e)) {
		uint8_t *d_seq = scr + tb + num_ctx;

		h_seq0 = malloc(num_ctx);
		if (!h_seq0) {
			e = ERRV(GENERIC);
			goto out;
		}
		for (c = 0; c < num_ctx; c++)
			h_seq0[c] = ctx[c].sequence_number;
		e = airs_dev_h2d(dev, d_seq, h_seq0, num_ctx);
		if (!is_err(e))
			e = airs_dev_sync(dev);
		w.seq0s = d_seq;
	}
	if (!is_err(e) && P->checksum_enabled) {
		uint32_t *d_ck = airs_dev_scratch(dev, SLOT_CK, (size_t)total * 4u);

		e = d_ck ? airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, total, NULL, d_ck) : ERRV(GENERIC);
		w.checksums = d_ck;
	}
	if (!is_err(e))
		e = airs_dev_walk(dev, &w);
	/* the one read-back: identifier draws and the final sequence numbers
	 * (adjacent in the device scratch, one copy into page-locked memory) */
	if (!is_err(e))
		e = airs_dev_d2h(dev, h_draws, w.draws, tb + num_ctx);
	if (!is_err(e))
		e = airs_dev_sync(dev);
	if (is_err(e))
		goto out;
	/* the identifiers first; the contexts advance only once the headers are
	 * patched (a failed upload or patch leaves them as they were) */
	for (c = 0; c < num_ctx; c++) {
		uint64_t id = ctx[c].identifier;

		for (a = 0; a < fpc; a++) {
			const uint32_t f = c * fpc + a;

			for (uint32_t k = 0; k < h_draws[f]; k++)
				id = next_identifier();
			ids[f] = id;
		}
	}
	{
		/* upload from page-locked memory and patch, both asynchronous
		 * (cmp_gpu_synchronize waits; the next call rewrites the host
		 * scratch only after its own read-back, which follows them) */
		uint64_t *d_ids = airs_dev_scratch(dev, SLOT_IDS, (size_t)total * 8u);

		memcpy(h_ids, ids, (size_t)total * 8u);
		if (!d_ids || is_err(airs_dev_h2d(dev, d_ids, h_ids, (size_t)total * 8u)))
			e = ERRV(GENERIC);
		else
			e = airs_dev_patch_ids(dev, b->dst, b->dst_stride, total, 0, 1, d_ids, b->sizes);
	}
	if (is_err(e))
		goto out;
	for (c = 0; c < num_ctx; c++) {
		for (a = 0; a < fpc; a++)
			if (REPORT_DRAWS(b))
				b->draws[c * fpc + a] = h_draws[c * fpc + a];
		ctx[c].identifier = ids[c * fpc + fpc - 1u];
		ctx[c].sequence_number = h_seq[c];
		ctx[c].model_size = 2u * n; /* every context's model holds a frame of this size */
	}
out:
	free(h_seq0);
	return e;
}

/*
 * MODEL contexts with the uncompressed fallback where the context walk does
 * not apply (frames of another size, or too few contexts to fill the CUs):
 * the segment walk codes every frame as if none fell back, with the raw frame
 * size as the capacity, so a frame that would fall back reports DST_TOO_SMALL
 * (the reference's first attempt, cmp.c:358-366) and nothing else changes for
 * the frames that fit.  One read-back of the statuses; a context with such a
 * frame (data that does not compress: rare) gets its model back from a copy
 * taken before the launch and runs again on the per-acquisition device state
 * machine (batch_device_exact), in call order, so the identifiers are drawn as
 * the call loop draws them.  The other contexts' identifiers follow the pass
 * rule (one draw per primary pass) and are patched into their headers.
 * Returns 0, an error value, or WALK_NO.
 */
static uint32_t batch_walk_spec(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx, uint32_t fpc,
				const struct cmp_gpu_batch *b, const struct pass *pp, const struct pass *ps, uint64_t *ids)
{
	struct airs_dev_engine *dev = eng->dev;
	const struct cmp_params *P = &ctx[0].params;
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	const uint32_t raw = raw_frame_size(&ctx[0], n);
	const size_t mb = 2u * (size_t)n; /* model bytes of a context */
	struct airs_walk w;
	uint32_t c, a, e = 0, seq_same = 1, m_strided = 1, msec = 0, cseq = 0, any_redo = 0;
	uint64_t mbase, mstep;
	uint8_t *msave, *redo = NULL, *hp;
	uint32_t *new_seq = NULL;
	uint64_t *new_id = NULL, *h_ids = NULL;

	if (!model_needed(P) || !P->uncompressed_fallback_enabled || b->dst_capacity < raw || raw > 0xFFFFFFu ||
	    (P->primary_preprocessing != CMP_PREPROCESS_NONE && P->primary_preprocessing != CMP_PREPROCESS_DIFF))
		return WALK_NO;
	if ((b->flags & CMP_GPU_AUTO_RICE) && P->primary_encoder_type == CMP_ENCODER_GOLOMB_ZERO)
		return WALK_NO;
	if (num_ctx > AIRS_COMMIT_MAX_CTX)
		return WALK_NO;
	for (c = 0; c < num_ctx; c++) {
		const uint32_t sq = ctx[c].sequence_number;

		if (!same_params(&ctx[c].params, P))
			return WALK_NO;
		if (sq != 0u && sq <= P->secondary_iterations && ctx[c].model_size != 2u * n)
			return WALK_NO; /* the reference returns SRC_SIZE_MISMATCH for that frame */
		if (sq != ctx[0].sequence_number)
			seq_same = 0;
	}
	memset(&w, 0, sizeof(w));
	w.src = b->src;
	w.src_stride = b->src_stride;
	w.sample_bytes = bytes;
	w.is_unsigned = b->type == CMP_GPU_U16;
	w.n = n;
	w.num_ctx = num_ctx;
	w.fpc = fpc;
	w.dst = b->dst;
	w.dst_stride = b->dst_stride;
	w.cap = raw; /* the first attempt's capacity */
	w.pre_p = P->primary_preprocessing;
	w.enc_p = P->primary_encoder_type;
	w.g_p = P->primary_encoder_param;
	w.outl_p = P->primary_encoder_outlier;
	w.enc_s = P->secondary_encoder_type;
	w.g_s = P->secondary_encoder_param;
	w.outl_s = P->secondary_encoder_outlier;
	w.model_rate = P->model_rate;
	w.iters = P->secondary_iterations;
	w.checksum_enabled = P->checksum_enabled ? 1u : 0u;
	w.status = b->sizes;
	w.seq0 = ctx[0].sequence_number;
	mbase = (uint64_t)(uintptr_t)ctx[0].work_buf;
	mstep = num_ctx > 1 ? (uint64_t)(uintptr_t)ctx[1].work_buf - mbase : 0;
	for (c = 0; c < num_ctx && m_strided; c++)
		m_strided = (uint64_t)(uintptr_t)ctx[c].work_buf == mbase + c * mstep;
	if (!m_strided)
		for (c = 0; c < num_ctx; c++)
			if ((uintptr_t)ctx[c].work_buf & 15u)
				return WALK_NO;
	w.model = (void *)(uintptr_t)mbase;
	w.model_stride = m_strided ? mstep : 0;
	/* identifiers 0: patched once they are drawn */
	{
		struct airs_walk chk = w;

		if (!m_strided)
			chk.model = NULL, chk.model_stride = 0;
		if (!airs_dev_walk_supported(&chk))
			return WALK_NO;
	}
	/* page-locked host scratch: the identifiers for patch_ids_kernel (when
	 * the commit kernel does not take them) */
	msave = airs_dev_scratch(dev, SLOT_MSAVE, mb * num_ctx);
	hp = airs_dev_host_scratch(dev, (size_t)total * 8u);
	new_seq = calloc(num_ctx, sizeof(*new_seq));
	new_id = calloc(num_ctx, sizeof(*new_id));
	redo = calloc(num_ctx, 1);
	if (!msave || !hp || !new_seq || !new_id || !redo) {
		e = ERRV(GENERIC);
		goto out;
	}
	if (!m_strided) {
		uint64_t *hp = malloc((size_t)num_ctx * 8u), *d_ptr = airs_dev_scratch(dev, SLOT_AUX, (size_t)num_ctx * 8u);

		if (!hp || !d_ptr)
			e = ERRV(GENERIC);
		for (c = 0; c < num_ctx && !is_err(e); c++)
			hp[c] = (uint64_t)(uintptr_t)ctx[c].work_buf;
		if (!is_err(e))
			e = airs_dev_h2d(dev, d_ptr, hp, (size_t)num_ctx * 8u);
		if (!is_err(e))
			e = airs_dev_sync(dev);
		free(hp);
		w.model_ptrs = d_ptr;
	}
	if (!seq_same && !is_err(e)) {
		uint8_t *hs = malloc(num_ctx), *d_seq = airs_dev_scratch(dev, SLOT_FL, num_ctx);

		if (!hs || !d_seq)
			e = ERRV(GENERIC);
		for (c = 0; c < num_ctx && !is_err(e); c++)
			hs[c] = ctx[c].sequence_number;
		if (!is_err(e))
			e = airs_dev_h2d(dev, d_seq, hs, num_ctx);
		if (!is_err(e))
			e = airs_dev_sync(dev);
		free(hs);
		w.seq0s = d_seq;
	}
	/* the models as they are before the launch, for contexts run again whose
	 * first frame reads its model (a secondary pass; a primary pass stores
	 * the model without reading it) */
	for (c = 0; c < num_ctx; c++)
		if (ctx[c].sequence_number != 0u && ctx[c].sequence_number <= w.iters)
			msec = 1;
	if (!is_err(e) && msec) {
		if (m_strided)
			e = airs_dev_d2d_rows(dev, msave, mb, ctx[0].work_buf, num_ctx > 1 ? mstep : mb, mb, num_ctx);
		else
			for (c = 0; c < num_ctx && !is_err(e); c++)
				e = airs_dev_d2d_rows(dev, msave + c * mb, mb, ctx[c].work_buf, mb, mb, 1);
	}
	if (!is_err(e) && P->checksum_enabled) {
		uint32_t *d_ck = airs_dev_scratch(dev, SLOT_CK, (size_t)total * 4u);

		e = d_ck ? airs_dev_checksum(dev, b->src, b->src_stride, bytes, n, total, NULL, d_ck) : ERRV(GENERIC);
		w.checksums = d_ck;
	}
	/* the one round trip: which contexts have a frame that did not fit.  The
	 * commit kernel signals them, then waits on the stream for the release
	 * below (it patches the identifiers when no context runs again) */
	h_ids = (uint64_t *)(void *)hp;
	if (!is_err(e))
		e = airs_dev_walk(dev, &w);
	if (!is_err(e)) {
		e = airs_dev_commit_begin(dev, b->sizes, num_ctx, fpc, b->dst, b->dst_stride, &cseq);
		if (!is_err(e)) {
			e = airs_dev_commit_wait(dev, cseq, num_ctx, redo);
			for (c = 0; c < num_ctx && !is_err(e) && !any_redo; c++)
				any_redo = redo[c];
			if (is_err(e) || any_redo) {
				(void)airs_dev_commit_release(dev, cseq, NULL, 0);
				if (is_err(e)) {
					(void)airs_dev_sync(dev); /* reports and clears the fault count */
					goto out;
				}
			}
		}
	}
	if (is_err(e))
		goto out;
	/* in call order: the pass rule's draws, or the context run again */
	for (c = 0; c < num_ctx && !is_err(e); c++) {
		if (!redo[c]) {
			uint32_t sq = ctx[c].sequence_number;
			uint64_t id = ctx[c].identifier;

			for (a = 0; a < fpc; a++) {
				const int prim = sq == 0u || sq > w.iters;

				if (prim)
					id = next_identifier();
				ids[c * fpc + a] = id;
				if (REPORT_DRAWS(b))
					b->draws[c * fpc + a] = prim ? 1u : 0u;
				sq = prim ? 1u : sq + 1u;
			}
			new_seq[c] = sq;
			new_id[c] = id;
		} else {
			struct cmp_gpu_batch sb = *b;

			if (msec)
				e = airs_dev_d2d_rows(dev, ctx[c].work_buf, mb, msave + c * mb, mb, mb, 1);
			sb.src = (const uint8_t *)b->src + (uint64_t)c * fpc * b->src_stride;
			sb.dst = (uint8_t *)b->dst + (uint64_t)c * fpc * b->dst_stride;
			sb.sizes = b->sizes + (size_t)c * fpc;
			sb.draws = b->draws ? b->draws + (size_t)c * fpc : NULL;
			if (!is_err(e))
				e = batch_device_exact(eng, &ctx[c], 1, fpc, &sb, pp, ps, ids + (size_t)c * fpc);
		}
	}
	if (is_err(e))
		goto out;
	/* the identifiers: released to the waiting commit kernel, or (a context
	 * ran again, or more frames than its block holds) patched by
	 * patch_ids_kernel from page-locked memory (batch_device_exact does not
	 * use the host scratch) */
	if (any_redo || !airs_dev_commit_release(dev, cseq, ids, total)) {
		memcpy(h_ids, ids, (size_t)total * 8u);
		e = airs_dev_patch_ids(dev, b->dst, b->dst_stride, total, 0, 1, h_ids, b->sizes);
		if (is_err(e))
			goto out;
	}
	for (c = 0; c < num_ctx; c++) {
		if (redo[c])
			continue; /* committed by batch_device_exact */
		ctx[c].identifier = new_id[c];
		ctx[c].sequence_number = (uint8_t)new_seq[c];
		ctx[c].model_size = 2u * n;
	}
out:
	free(new_seq);
	free(new_id);
	free(redo);
	return e;
}

/*
 * IWT contexts without a MODEL pass, every frame of the batch on the same
 * pass (asynchronous mode): all frames in ONE launch instead of one per
 * acquisition.  The reference computes a frame's coefficients into its
 * context's work buffer (preprocess.c:321-353), so after the batch that
 * buffer holds the coefficients of the context's last frame; the other
 * frames' coefficients go to device scratch (at most IWT_SCRATCH_MAX bytes,
 * else WALK_NO: the per-acquisition launches).
 */
#define IWT_SCRATCH_MAX (1ull << 30)
static uint32_t batch_iwt(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx, uint32_t fpc,
			  const struct cmp_gpu_batch *b, const struct frame_plan *plan, uint64_t *ids, uint64_t *ptrs)
{
	const uint32_t bytes = b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	const uint32_t n = b->src_size / bytes, total = num_ctx * fpc;
	const uint64_t cstride = (2ull * n + 15u) & ~15ull;
	const uint64_t need = (uint64_t)(total - num_ctx) * cstride;
	uint64_t *coef, k = 0;
	uint8_t *scr;
	uint32_t c, a, e;

	if (fpc < 2 || need > IWT_SCRATCH_MAX)
		return WALK_NO;
	scr = airs_dev_scratch(eng->dev, SLOT_MODEL, (size_t)need);
	coef = malloc((size_t)total * sizeof(*coef));
	if (!scr || !coef) {
		free(coef);
		return WALK_NO;
	}
	for (c = 0; c < num_ctx; c++)
		for (a = 0; a < fpc; a++)
			coef[c * fpc + a] = a + 1u == fpc ? (uint64_t)(uintptr_t)ctx[c].work_buf
							  : (uint64_t)(uintptr_t)(scr + (k++) * cstride);
	e = batch_launch(eng, ctx, fpc, b, plan, NULL, 0, 1, total, b->dst_capacity, ids, ptrs, coef);
	free(coef);
	return e == WALK_NO ? ERRV(GENERIC) : e;
}

uint32_t cmp_gpu_compress(struct cmp_gpu_engine *eng, struct cmp_context *ctx, uint32_t num_ctx,
			  uint32_t fpc, const struct cmp_gpu_batch *b)
{
	const uint32_t bytes = b && b->type == CMP_GPU_I16_IN_I32 ? 4u : 2u;
	uint32_t n, c, a, total, e = 0, any_model = 0, any_mneed = 0, exact = 0;
	struct frame_plan *plan;
	uint64_t *ids, *ptrs;

	if (!eng || !ctx || !b || !num_ctx || !fpc)
		return ERRV(GENERIC);
	if (b->type > CMP_GPU_I16_IN_I32)
		return ERRV(PARAMS_INVALID);
	if (!b->src)
		return ERRV(SRC_NULL);
	if (b->src_size == 0 || b->src_size % bytes)
		return ERRV(SRC_SIZE_WRONG);
	if (((uintptr_t)b->src % bytes) || (b->src_stride % bytes)) {
		fprintf(stderr, "airscmp: cmp_gpu_compress: src must be %u-byte aligned\n", bytes);
		return ERRV(GENERIC);
	}
	if (!b->sizes) {
		fprintf(stderr, "airscmp: cmp_gpu_compress: sizes array is NULL\n");
		return ERRV(GENERIC);
	}
	if ((b->flags & CMP_GPU_REPORT_DRAWS) && !b->draws) {
		fprintf(stderr, "airscmp: cmp_gpu_compress: CMP_GPU_REPORT_DRAWS without a draws array\n");
		return ERRV(GENERIC);
	}
	if (b->draws && !(b->flags & CMP_GPU_REPORT_DRAWS)) {
		/* callers of the earlier interface set draws alone: it is left
		 * untouched now, say so once */
		static int warned;
		if (!warned) {
			warned = 1;
			fprintf(stderr, "airscmp: cmp_gpu_compress: draws array given without CMP_GPU_REPORT_DRAWS: "
					"not written\n");
		}
	}
	if (!b->dst)
		return ERRV(DST_NULL);
	if (((uintptr_t)b->dst & 7u) || (b->dst_stride & 7u))
		return ERRV(DST_UNALIGNED);
	if (is_err(b->dst_capacity))
		return ERRV(GENERIC);
	if ((uint64_t)num_ctx * fpc > 0xFFFFFFFull)
		return ERRV(PARAMS_INVALID);
	n = b->src_size / bytes;
	total = num_ctx * fpc;
	/* frames of a batch must not overlap: every workgroup of a frame writes
	 * up to min(capacity, worst-case frame) bytes from its frame base */
	if (total > 1) {
		const uint64_t worst = frame_worst(n), span = b->dst_capacity < worst ? b->dst_capacity : worst;

		if (b->src_stride < b->src_size || b->dst_stride < span) {
			fprintf(stderr, "airscmp: cmp_gpu_compress: frames overlap (src_stride %llu < src_size %u "
					"or dst_stride %llu < %llu)\n",
				(unsigned long long)b->src_stride, b->src_size, (unsigned long long)b->dst_stride,
				(unsigned long long)span);
			return ERRV(GENERIC);
		}
	}
	for (c = 0; c < num_ctx; c++) {
		if (ctx[c].magic != CTX_MAGIC)
			return ERRV(CONTEXT_INVALID);
		if (ctx[c].params.uncompressed_fallback_enabled &&
		    b->dst_capacity >= raw_frame_size(&ctx[c], n))
			exact = 1;
		if (model_needed(&ctx[c].params))
			any_mneed = 1;
		if (work_buf_state(&ctx[c].params)) {
			any_model = 1;
			if ((uintptr_t)ctx[c].work_buf & 1u)
				return ERRV(WORK_BUF_UNALIGNED);
		}
	}

	plan = calloc(total, sizeof(*plan));
	ids = calloc(total, sizeof(*ids));
	ptrs = calloc(total, sizeof(*ptrs));
	if (!plan || !ids || !ptrs) {
		free(plan);
		free(ids);
		free(ptrs);
		return ERRV(GENERIC);
	}
	/* a frame that can fail changes its context's next pass (the reference
	 * does not advance sequence_number on an error), so such batches run step
	 * by step: capacity below the worst case, or a worst case past the 24-bit
	 * size field (n > ~2.8 Mi samples: HDR_CMP_SIZE_TOO_LARGE is possible)
	 * when a context has secondary passes.  Without secondary passes every
	 * frame is a primary pass with one identifier draw whatever the outcome
	 * of the frame before, so the plan does not depend on it. */
	if ((uint64_t)b->dst_capacity < HDR_MAX_SIZE + CMP_CHECKSUM_SIZE + payload_bound(2u * n))
		exact = 1;
	if (is_err(cmp_compress_bound(2u * n)) && fpc > 1)
		for (c = 0; c < num_ctx; c++)
			if (ctx[c].params.secondary_iterations)
				exact = 1;
	if (!exact) {
		/* replay the context state machine in call order (c-major), counting
		 * identifier draws; a frame the host API would reject sends the
		 * batch to the step-by-step path with the contexts untouched */
		struct cmp_context *snap = malloc((size_t)num_ctx * sizeof(*snap));
		uint32_t *draws = calloc(total, sizeof(uint32_t));

		if (!snap || !draws) {
			free(snap);
			free(draws);
			e = ERRV(GENERIC);
			goto out;
		}
		memcpy(snap, ctx, (size_t)num_ctx * sizeof(*snap));
		for (c = 0; c < num_ctx && !exact; c++) {
			for (a = 0; a < fpc; a++) {
				const uint32_t f = c * fpc + a;
				void *dst = (uint8_t *)b->dst + (uint64_t)f * b->dst_stride;

				if (is_err(engine_prologue(&ctx[c], dst, b->dst_capacity, n, &plan[f].p, &draws[f]))) {
					exact = 1;
					break;
				}
				ctx[c].sequence_number++;
			}
		}
		if (exact) {
			memcpy(ctx, snap, (size_t)num_ctx * sizeof(*snap));
		} else {
			/* the identifiers, drawn in call order */
			for (c = 0; c < num_ctx; c++) {
				uint64_t id = snap[c].identifier;

				for (a = 0; a < fpc; a++) {
					const uint32_t f = c * fpc + a;

					for (uint32_t k = 0; k < draws[f]; k++)
						id = next_identifier();
					plan[f].id = id;
					if (REPORT_DRAWS(b))
						b->draws[f] = (uint8_t)draws[f];
				}
				ctx[c].identifier = id;
			}
		}
		free(snap);
		free(draws);
	}
	if (exact) {
		struct pass pp, ps;

		memset(&ps, 0, sizeof(ps));
		if (!(b->flags & (CMP_GPU_HOST_STEPPED | CMP_GPU_STEPWISE)) && device_exact_ok(ctx, num_ctx, b, n, &pp, &ps) &&
		    ((e = batch_walk_fb(eng, ctx, num_ctx, fpc, b, ids)) != WALK_NO ||
		     (e = batch_walk_spec(eng, ctx, num_ctx, fpc, b, &pp, &ps, ids)) != WALK_NO))
			; /* MODEL contexts with the fallback: every acquisition in one launch (or an error) */
		else if (!(b->flags & CMP_GPU_HOST_STEPPED) && device_exact_ok(ctx, num_ctx, b, n, &pp, &ps))
			e = batch_device_exact(eng, ctx, num_ctx, fpc, b, &pp, &ps, ids);
		else
			e = batch_exact(eng, ctx, num_ctx, fpc, b, plan, ids, ptrs);
		goto out;
	}

	/* launch: frames with equal passes share one launch; MODEL contexts
	 * step through acquisitions in order (the model carries state) */
	if (!any_model && (num_ctx == 1 || fpc == 1)) {
		/* contiguous runs of frames with the same pass, one launch each */
		uint32_t f = 0;

		while (f < total && !is_err(e)) {
			uint32_t g = f + 1;

			while (g < total && same_pass(&plan[g].p, &plan[f].p))
				g++;
			e = batch_launch(eng, ctx, fpc, b, plan, NULL, f, 1, g - f, b->dst_capacity, ids, ptrs, NULL);
			f = g;
		}
	} else {
		uint32_t f, uniform = 1;

		for (f = 1; f < total && uniform; f++)
			uniform = same_pass(&plan[f].p, &plan[0].p);
		if (uniform && !any_model) {
			e = batch_launch(eng, ctx, fpc, b, plan, NULL, 0, 1, total, b->dst_capacity, ids, ptrs, NULL);
		} else if (uniform && !any_mneed && plan[0].p.pre == CMP_PREPROCESS_IWT && !(b->flags & CMP_GPU_STEPWISE) &&
			   (e = batch_iwt(eng, ctx, num_ctx, fpc, b, plan, ids, ptrs)) != WALK_NO) {
			/* IWT contexts: every frame in one launch (or an error) */
		} else if (any_model && !(b->flags & CMP_GPU_STEPWISE) &&
			   (e = batch_walk(eng, ctx, num_ctx, fpc, b, plan)) != WALK_NO) {
			/* every acquisition in one launch (or an error) */
		} else {
			e = 0;
			/* one launch per acquisition step across the contexts (one per
			 * pass when contexts are in different states); MODEL contexts
			 * carry state from one step to the next */
			uint32_t *list = calloc(num_ctx, sizeof(uint32_t)), *caps = calloc(num_ctx, sizeof(uint32_t));
			uint32_t *grp = calloc(num_ctx, sizeof(uint32_t));
			uint8_t *done = calloc(num_ctx, 1);

			if (!list || !caps || !grp || !done)
				e = ERRV(GENERIC);
			for (a = 0; a < fpc && !is_err(e); a++) {
				for (c = 0; c < num_ctx; c++) {
					list[c] = c * fpc + a;
					caps[c] = b->dst_capacity;
				}
				e = launch_groups(eng, ctx, fpc, b, plan, list, caps, num_ctx, grp, done, ids, ptrs);
			}
			free(list);
			free(caps);
			free(grp);
			free(done);
		}
	}
out:
	free(plan);
	free(ids);
	free(ptrs);
	return is_err(e) ? e : 0;
}
