/*
 * airs_dev.h -- internal C-ABI between the C host library (cmp_host.c) and
 * the HIP device layer (encode.hip).  Plain C types only.
 *
 * One launch encodes `num_frames` equally sized frames that share one set of
 * pass parameters (the reference's compress_engine, lib/compress/cmp.c:213-338,
 * run for many frames at once).  Per-frame variation (identifier, Golomb
 * parameter, model buffer) comes through optional device arrays.
 */
#ifndef AIRS_DEV_H
#define AIRS_DEV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum airs_model_mode {
	AIRS_MODEL_NONE = 0,   /* no model configured */
	AIRS_MODEL_STORE = 1,  /* primary pass: model[i] = sample[i]   (cmp.c:305-306) */
	AIRS_MODEL_UPDATE = 2  /* secondary pass: model[i] = blend(...) (cmp.c:307-310) */
};

struct airs_launch {
	/* input: frame f's samples at src + f*src_stride; 2 or 4 bytes per sample */
	const void *src;
	uint64_t src_stride;
	uint32_t sample_bytes;   /* 2 (u16/i16) or 4 (i16 in i32) */
	uint32_t is_unsigned;    /* u16: zero-extend in the model update (cmp.c:132-142) */
	uint32_t n;              /* samples per frame, >= 1 */
	uint32_t num_frames;
	/* launch frame j is batch frame frame_list[j] (device, optional) or
	 * frame_add + j*frame_mul; per-frame arrays below are indexed by the
	 * batch frame, identifiers and model pointers by the launch index j */
	const uint32_t *frame_list;
	uint32_t frame_add, frame_mul;

	/* output: frame f at dst + f*dst_stride (8-byte aligned), capacity cap */
	void *dst;
	uint64_t dst_stride;
	uint32_t cap;

	/* pass parameters (already validated by the host) */
	uint32_t preprocessing;  /* enum cmp_preprocessing: NONE, DIFF or MODEL */
	uint32_t encoder_type;   /* enum cmp_encoder_type */
	uint32_t encoder_param;  /* Golomb g (ignored for UNCOMPRESSED) */
	uint32_t outlier_param;  /* user outlier (GOLOMB_MULTI) */
	const uint32_t *frame_g; /* device, optional per-frame g (all powers of two) */
	/* CMP_GPU_AUTO_RICE (GOLOMB_ZERO after NONE or DIFF): g = 2^k per frame by
	 * the build-defined rule.  Frames of a few segments
	 * choose k inside the encode kernel (one read of the samples); otherwise
	 * the sliced Rice selection writes g for the launch's frames into frame_g_scratch
	 * (device, one word per batch frame) first */
	uint32_t auto_rice;
	uint32_t *frame_g_scratch;

	/* model (work buffer): batch frame f's model at model + (f / model_div)*model_stride,
	 * or model_ptrs[j] (device) */
	void *model;
	uint64_t model_stride;
	uint32_t model_div;
	const uint64_t *model_ptrs;
	uint32_t model_ptrs_al16; /* every model_ptrs[j] is 16-byte aligned (host-checked) */
	uint32_t model_mode;     /* enum airs_model_mode */
	uint32_t model_rate;
	uint64_t fail_bit;       /* samples reaching this frame bit keep their old model */

	/* header fields */
	const uint8_t *seqs;     /* device, optional: sequence number per batch frame (else seq) */
	uint64_t id_base;        /* identifier of launch frame j = id_base + j*id_step, or ids[j] */
	uint64_t id_step;
	const uint64_t *ids;     /* device, optional */
	uint32_t seq;            /* sequence number written in the header */
	uint32_t checksum_enabled;
	const uint32_t *checksums; /* device, per frame (airs_dev_checksum output) */

	/* results (device): status[f] = frame size or error value; needed[f] = size in
	 * bytes the frame needs (payload+header+checksum), even when it did not fit */
	uint32_t *status;
	uint32_t *needed;
};

struct airs_dev_engine;

/* create an engine on the current HIP device; stream = hipStream_t or NULL (default) */
struct airs_dev_engine *airs_dev_engine_create(void *stream);
/* engine options (cmp_gpu_engine_set_option): 0 or an error value */
#define AIRS_OPT_EXCLUSIVE 1u
#define AIRS_OPT_WALK_SEGMENT 2u
#define AIRS_OPT_NO_CONTEXT_WALK 3u
uint32_t airs_dev_set_option(struct airs_dev_engine *e, uint32_t option, uint32_t value);
void airs_dev_engine_destroy(struct airs_dev_engine *e);
void *airs_dev_engine_stream(struct airs_dev_engine *e);

/* enqueue one encode launch; returns 0 or a cmp error value (uint32_t)-code */
uint32_t airs_dev_encode(struct airs_dev_engine *e, const struct airs_launch *L);

/* MODEL streams in one launch (enc_walk.hip): context c's frames c*fpc + a
 * (a = 0 .. fpc-1) in acquisition order, the model of each context kept on
 * the chip between acquisitions and written to its work buffer once at the
 * end.  Only for batches whose passes cannot fail or fall back (the host's
 * asynchronous mode): frame (c, a) is a primary pass when the context's
 * sequence number before it is 0 or above `iters` (cmp.c:228-248).
 * Requirements (airs_dev_walk returns CMP_ERR_PARAMS_INVALID otherwise,
 * nothing launched): n a multiple of 4096; src, src_stride and every model
 * 16-byte aligned; primary NONE or DIFF; both encoders GOLOMB_ZERO or
 * GOLOMB_MULTI with g a power of two. */
struct airs_walk {
	const void *src;
	uint64_t src_stride;
	uint32_t sample_bytes, is_unsigned, n;
	uint32_t num_ctx, fpc;
	void *dst;
	uint64_t dst_stride;
	uint32_t cap;
	void *model;              /* context c's model at model + c*model_stride, or model_ptrs[c] */
	uint64_t model_stride;
	const uint64_t *model_ptrs;
	uint32_t pre_p, enc_p, g_p, outl_p; /* primary pass (outl: the user's outlier parameter) */
	uint32_t enc_s, g_s, outl_s;        /* secondary pass, MODEL preprocessing */
	uint32_t model_rate, iters;
	uint32_t seq0;            /* sequence number of every context before the call, or */
	const uint8_t *seq0s;     /* device [num_ctx] */
	uint64_t id_base, id_cstep, id_astep; /* identifier of frame (c, a) = base + c cstep + a astep, or */
	const uint64_t *ids;      /* device [num_ctx * fpc] */
	uint32_t checksum_enabled;
	const uint32_t *checksums; /* device [num_ctx * fpc] */
	uint32_t *status;         /* device [num_ctx * fpc] */
	/* uncompressed fallback on the chip (cmp.c:342-393; the context walk
	 * only): cap is the raw frame size; a frame whose coded size exceeds it is
	 * written raw (NONE + UNCOMPRESSED, sequence number 0), the model takes its
	 * samples and the context continues at sequence number 1.  The identifier
	 * draws of every frame (1 per reset: 0/1, 3 or 2 with a fallback) and the
	 * final sequence numbers are written for the host, which draws the
	 * identifiers in call order and patches the headers. */
	uint32_t fb, raw_size;
	uint8_t *draws;           /* device [num_ctx * fpc], with fb */
	uint8_t *seq_out;         /* device [num_ctx], with fb */
};
int airs_dev_walk_supported(const struct airs_walk *w);
uint32_t airs_dev_walk(struct airs_dev_engine *e, struct airs_walk *w);

/* payload-only stream (cmp_gpu_encode_stream): the n samples at src (device)
 * as ONE bit stream from bit 0 of dst, no header or checksum; *status
 * (device) = bytes or error value.  NONE/DIFF preprocessing. */
#define AIRS_STREAM_MAX 89478485u /* 48 bits per sample stay below 2^32 bits */
uint32_t airs_dev_encode_stream(struct airs_dev_engine *e, const void *src, uint32_t sample_bytes, uint32_t n,
				uint32_t preprocessing, uint32_t encoder_type, uint32_t encoder_param,
				uint32_t outlier_param, void *dst, uint32_t cap, uint32_t *status);

/* Batch fallback path on the device (cmp_gpu_compress): per-context state
 * machine of compress_engine / cmp_compress_generic (cmp.c:228-246, 342-393).
 * airs_dev_fb_step resolves step `prev` (>= 0) and plans step `cur` (>= 0);
 * airs_dev_fb_copy writes the raw frames of step `prev`'s fallbacks. */
struct airs_fb_step {
	uint32_t *state;          /* device [2 num_ctx]: sequence number, model size */
	uint32_t num_ctx, fpc;
	int32_t prev, cur;
	uint32_t packed;          /* 2 n */
	uint32_t iters;           /* secondary_iterations */
	uint32_t model_needed;    /* model_is_needed(params) */
	uint32_t fb_eligible;     /* fallback enabled and dst_capacity >= raw_size */
	uint32_t raw_size;        /* header + 2 n (+ checksum) */
	uint32_t err_floor;       /* values above are errors */
	uint32_t err_small, err_mismatch, err_too_large;
	uint32_t *flist_p, *flist_s; /* device [num_ctx]: launch lists of step cur (AIRS_NO_FRAME holes) */
	uint8_t *seqs, *draws, *kind, *fb; /* device [num frames] */
	uint32_t *status;         /* device [num frames]: the batch sizes */
	/* raw frame writer (fb_copy) */
	const void *src;
	uint64_t src_stride;
	uint32_t sample_bytes, n;
	void *dst;
	uint64_t dst_stride;
	const uint32_t *checksums;
	uint32_t checksum;
	void *model;              /* strided work buffers (context c at model + c model_stride), or */
	uint64_t model_stride;
	const uint64_t *model_ptrs; /* device [num_ctx] */
};
uint32_t airs_dev_fb_step(struct airs_dev_engine *e, const struct airs_fb_step *s);
uint32_t airs_dev_fb_copy(struct airs_dev_engine *e, const struct airs_fb_step *s);

/* frames f < num_frames of a strided buffer packed back to back at 8-byte
 * aligned offsets (offsets[f], offsets[num_frames] = total; frames whose size
 * is an error value take no bytes); reads only the compressed bytes */
uint32_t airs_dev_pack_frames(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
			      uint32_t max_frame_bytes, const uint32_t *sizes, uint32_t num_frames,
			      uint32_t err_floor, void *out, uint64_t *offsets);

/* XXH32 (seed 419764627) over each frame's samples as big-endian 16-bit words */
uint32_t airs_dev_checksum(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
			   uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
			   const uint32_t *frame_list, uint32_t *out);

/* per-frame Rice parameter (build-defined rule): out_g[f] = 2^k
 * for the batch frames f = frame_list[j] (AIRS_NO_FRAME: none) or
 * frame_add + j*frame_mul, j < num_frames */
uint32_t airs_dev_select_rice(struct airs_dev_engine *e, const void *src, uint64_t src_stride,
			      uint32_t sample_bytes, uint32_t n, uint32_t num_frames,
			      const uint32_t *frame_list, uint32_t frame_add, uint32_t frame_mul,
			      uint32_t preprocessing, uint32_t *out_g);

/* counter-hash synthetic frames (bench/test inputs) */
uint32_t airs_dev_synth(struct airs_dev_engine *e, void *dst, uint32_t sample_bytes, uint64_t seed,
			uint32_t frame0, uint32_t n, uint32_t num_frames, uint64_t stride,
			uint32_t W);

/* engine-owned scratch, grown on demand (stream ordered) */
#define AIRS_NSLOT 19 /* scratch slots per engine; the last five are the device layer's (checksum
		       * placement, checksum products, decoder parse arrays, decoder frame info, IWT heads) */
#define AIRS_SLOT_GATHER 11 /* slots 11..13: cmp_gpu_gather (cmp_gather.c); 0..10 cmp_host.c */
void *airs_dev_scratch(struct airs_dev_engine *e, int slot, size_t bytes);
/* engine-owned device words for the gather's status exchanges (cmp_gather.c),
 * allocated with the engine so that taking part in an exchange never needs an
 * allocation that could fail on one rank only: 2 words in, then
 * 2 * AIRS_COLL_MAX_RANKS words out */
#define AIRS_COLL_MAX_RANKS 256
uint64_t *airs_dev_coll(struct airs_dev_engine *e);
/* engine-owned page-locked host scratch, grown on demand: asynchronous
 * read-backs and uploads; the host may rewrite it once the stream has passed
 * the copies that use it */
void *airs_dev_host_scratch(struct airs_dev_engine *e, size_t bytes);

/* rewrite header bytes 8..13 (identifier) of launch frames whose status is
 * not an error: frame j = frame_add + j*frame_mul, identifier ids[j] (device
 * memory, or engine host scratch read over the bus) */
uint32_t airs_dev_patch_ids(struct airs_dev_engine *e, void *dst, uint64_t dst_stride, uint32_t num_frames,
			    uint32_t frame_add, uint32_t frame_mul, const uint64_t *ids,
			    const uint32_t *status);

/* The commit of a speculative batch, without a stream wait: begin launches
 * one kernel that writes flags for the host (context c has a frame whose
 * status is an error) and the fault count, signals, then waits for the host's
 * release and patches identifiers if the release carries them (up to
 * AIRS_HCO_MAX_IDS frames, ids[f] for frame f).  wait polls for the signal
 * and copies the flags out (a fault count is returned as an error).
 * release MUST follow every successful begin (with ids, or NULL: no patch),
 * before any other wait on the stream; it returns 1 when the kernel patches
 * the identifiers, 0 when the caller must: NULL, more than the block holds, or
 * a second release of the same seq (wait released it on its time-out).  The
 * kernel acknowledges whether it patched; the engine checks that at the next
 * stream wait (airs_dev_sync) or commit, and patches the headers itself when
 * the kernel gave up waiting for the release. */
#define AIRS_COMMIT_MAX_CTX 8192u /* contexts a commit kernel flags (AIRS_HCO_MAX_CTX) */
uint32_t airs_dev_commit_begin(struct airs_dev_engine *e, const uint32_t *status, uint32_t num_ctx, uint32_t fpc,
			       void *dst, uint64_t dst_stride, uint32_t *seq);
uint32_t airs_dev_commit_wait(struct airs_dev_engine *e, uint32_t seq, uint32_t num_ctx, uint8_t *flags);
int airs_dev_commit_release(struct airs_dev_engine *e, uint32_t seq, const uint64_t *ids, uint32_t total);

/* header bytes 8..13 of n frames at data + offsets[i] <- ids[i] (offsets and
 * ids device arrays): the multi-GPU gather's identifier patch */
uint32_t airs_dev_patch_ids_at(struct airs_dev_engine *e, void *data, const uint64_t *offsets, const uint64_t *ids,
			       uint64_t n);

/* decoder (decode.hip): frames at src + f*src_stride -> 16-bit samples at
 * dst + f*dst_stride bytes; status[f] = samples or error (see cmp_gpu.h) */
uint32_t airs_dev_decode(struct airs_dev_engine *e, const void *src, uint64_t src_stride, uint32_t src_cap,
			 uint32_t num_frames, uint16_t *dst, uint64_t dst_stride, uint32_t dst_samples,
			 uint32_t *status, const uint16_t *model, uint64_t model_stride);

/* plain memory helpers on the engine stream */
void *airs_dev_malloc(size_t bytes);
void airs_dev_free(void *p);
uint32_t airs_dev_h2d(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes);
uint32_t airs_dev_d2h(struct airs_dev_engine *e, void *dst, const void *src, size_t bytes);
uint32_t airs_dev_sync(struct airs_dev_engine *e);
uint32_t airs_dev_memset(struct airs_dev_engine *e, void *dst, int v, size_t bytes);
/* rows of `width` bytes, device to device: dst + r*dpitch <- src + r*spitch */
uint32_t airs_dev_d2d_rows(struct airs_dev_engine *e, void *dst, size_t dpitch, const void *src, size_t spitch,
			   size_t width, size_t rows);

/* non-zero when a HIP device is usable */
int airs_dev_available(void);
const char *airs_dev_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* AIRS_DEV_H */
