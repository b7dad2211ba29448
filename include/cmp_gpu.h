/*
 * cmp_gpu.h -- device-pointer batch API of the MI355X build (libairscmp.so).
 *
 * No reference counterpart: the reference (lib/cmp.h) compresses one frame
 * from host memory per call.  This API runs the same frame format and the
 * same cmp_context state machine (lib/compress/cmp.c:213-393) over many
 * frames whose samples already live in GPU memory, with one launch per group
 * of frames that share pass parameters.  Frames produced here are
 * byte-identical to what cmp_compress_u16/i16/i16_in_i32 produce for the
 * same inputs, contexts and identifiers.
 *
 * Contexts come from cmp_initialise() exactly as for the host API; when a
 * context needs a work buffer (MODEL preprocessing) its work_buf must be a
 * DEVICE pointer (2-byte aligned; 16 is fastest) holding that context's model.
 *
 * Ordering / identifiers: a call is equivalent to
 *
 *     for c in [0, num_ctx): for a in [0, frames_per_ctx):
 *         sizes[c*fpc + a] = cmp_compress_<type>(&ctx[c], dst(c*fpc+a), dst_capacity,
 *                                                src(c*fpc+a), src_size)
 *
 * including the timestamp-callback sequence that feeds header identifiers.
 */
#ifndef CMP_GPU_H
#define CMP_GPU_H

#include <stdint.h>

#include "cmp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* sample layout of the frames in a batch (the three cmp_compress_* entry points) */
enum cmp_gpu_sample_type {
	CMP_GPU_U16 = 0,       /* cmp_compress_u16 */
	CMP_GPU_I16 = 1,       /* cmp_compress_i16 */
	CMP_GPU_I16_IN_I32 = 2 /* cmp_compress_i16_in_i32 */
};

/* flags */
#define CMP_GPU_AUTO_RICE 0x1u /* GOLOMB_ZERO passes after NONE, DIFF or IWT preprocessing:
				* choose g = 2^k per frame (k in [0,15], fewest payload bits
				* for the pass's residuals -- the IWT coefficients for IWT --,
				* ties to smaller k) instead of the configured encoder
				* parameter; MODEL passes keep theirs; build-defined extension */
#define CMP_GPU_HOST_STEPPED 0x2u /* batches that can fall back or fail: step the context state
				   * machine on the host (one synchronisation per acquisition step)
				   * instead of on the device; same output, for comparisons */
#define CMP_GPU_STEPWISE 0x4u     /* MODEL contexts: one launch per acquisition step instead of
				   * every acquisition in one launch with the models kept on
				   * the chip; same output, for comparisons */
#define CMP_GPU_REPORT_DRAWS 0x8u /* write each frame's identifier-draw count to batch->draws
				   * (which must then be non-NULL); without it draws is never
				   * touched */

struct cmp_gpu_batch {
	enum cmp_gpu_sample_type type;
	const void *src;        /* device; frame i at src + i*src_stride (16-byte aligned frames load fastest) */
	uint64_t src_stride;    /* bytes, multiple of the sample size */
	uint32_t src_size;      /* bytes per frame, as cmp_compress_*'s src_size */
	void *dst;              /* device; frame i at dst + i*dst_stride, 8-byte aligned */
	uint64_t dst_stride;    /* bytes, multiple of 8 */
	uint32_t dst_capacity;  /* bytes available per frame */
	uint32_t *sizes;        /* device [num frames]: frame size or error value */
	uint32_t flags;
	uint8_t *draws;         /* with CMP_GPU_REPORT_DRAWS, HOST [num frames]: timestamp-callback draws each frame made
				 * (0: it carries its context's identifier; 1: a reset; 3 or 2: a
				 * primary or secondary pass that fell back, cmp.c:342-393), for
				 * assigning identifiers across processes (shard.py); valid when the
				 * call returns.  Zero-initialise the struct: fields added later
				 * default to off */
};

struct cmp_gpu_engine;

/* Create an engine bound to the current HIP device and the given hipStream_t
 * (NULL = default stream).  Returns an error value or CMP_ERR_NO_ERROR. */
uint32_t cmp_gpu_engine_create(struct cmp_gpu_engine **engine, void *hip_stream);
void cmp_gpu_engine_destroy(struct cmp_gpu_engine *engine);

/* Engine options, all 0 after cmp_gpu_engine_create.  Returns 0 or an error
 * value (CMP_ERROR(PARAMS_INVALID) for an unknown option or value).
 *   CMP_GPU_OPT_EXCLUSIVE       1: the caller promises that nothing else runs
 *                               on the device while this engine's kernels do
 *                               (one process, one stream).  The MODEL segment
 *                               walk may then order its workgroups by block
 *                               index when its whole grid fits the CUs; without
 *                               it every workgroup numbers itself with a
 *                               ticket as it starts, which stays correct beside
 *                               other kernels and processes.  CMP_GPU_AUTO_RICE
 *                               picks k inside the encode kernel for frames of
 *                               up to 32 segments (16-bit: 512 Ki samples) with
 *                               the option, up to 8 without it (a frame's
 *                               segments meet at a barrier); larger frames take
 *                               the selection kernel first.
 *   CMP_GPU_OPT_WALK_SEGMENT    MODEL segment walk: 0 automatic, or 2048 /
 *                               4096 samples per segment.
 *   CMP_GPU_OPT_NO_CONTEXT_WALK 1: MODEL batches take the segment walk where
 *                               they would take the context walk (not those
 *                               with the uncompressed fallback, which need it). */
#define CMP_GPU_OPT_EXCLUSIVE 1u
#define CMP_GPU_OPT_WALK_SEGMENT 2u
#define CMP_GPU_OPT_NO_CONTEXT_WALK 3u
uint32_t cmp_gpu_engine_set_option(struct cmp_gpu_engine *engine, uint32_t option, uint32_t value);

/* Compress num_ctx * frames_per_ctx frames (see the ordering note above).
 * Returns CMP_ERR_NO_ERROR or a call-level error (batch validation: NULL or
 * misaligned pointers, bad sizes, invalid contexts).  Per-frame results,
 * including frames cmp_compress_* would reject, land in batch->sizes.
 *
 * The call is asynchronous on the engine's stream when the outcome of a
 * frame cannot change the pass of the frames after it: dst_capacity is at
 * least the worst-case frame (26 bytes + 6 per sample), no context can fall
 * back to raw storage, and -- where that worst case exceeds the 24-bit
 * compressed-size field (more than ~2.8 Mi samples, so a frame can fail with
 * CMP_ERR_HDR_CMP_SIZE_TOO_LARGE) -- no context has secondary passes with
 * frames_per_ctx > 1.  Otherwise the outcome of frame (c, a) decides the pass
 * of frame (c, a+1), so the call runs one acquisition step at a time and
 * synchronises after each step (and after the step's fallbacks,
 * cmp.c:342-393).  Identifier draws are counted per frame and made at the
 * end, in the loop's order.
 *
 * Frames must not overlap: with more than one frame, src_stride >= src_size
 * and dst_stride >= min(dst_capacity, worst-case frame), else the call
 * returns CMP_ERR_GENERIC. */
uint32_t cmp_gpu_compress(struct cmp_gpu_engine *engine, struct cmp_context *ctx, uint32_t num_ctx,
			  uint32_t frames_per_ctx, const struct cmp_gpu_batch *batch);

/* Decoder (no reference counterpart: the reference has none, see
 * programs/airspacecli.c:421-423).  Decodes num_frames frames as written by
 * cmp_compress_* / cmp_gpu_compress back into their 16-bit samples (the low
 * halves, for i16-in-i32 sources).  Frames of every preprocessing mode and
 * encoder; MODEL frames need the model each was encoded against (MODEL frames
 * without one get CMP_ERR_PARAMS_INVALID).  The checksum is not verified. */
struct cmp_gpu_decode_batch {
	const void *src;        /* device; frame i at src + i*src_stride, 8-byte aligned */
	uint64_t src_stride;    /* bytes, multiple of 8, >= src_capacity */
	uint32_t src_capacity;  /* bytes readable per frame, multiple of 4, >= 22 */
	uint32_t num_frames;    /* <= 65535 */
	uint16_t *dst;          /* device; frame i's samples at dst + i*dst_stride bytes */
	uint64_t dst_stride;    /* bytes, even */
	uint32_t dst_samples;   /* samples available per frame */
	uint32_t *status;       /* device [num_frames]: samples decoded, or an error value */
	const uint16_t *model;  /* device or NULL; frame i's model at model + i*model_stride bytes */
	uint64_t model_stride;  /* bytes, even */
};

/* Returns CMP_ERR_NO_ERROR or a call-level error; per-frame results land in
 * batch->status.  Synchronises with the host (the parse is sized from the
 * headers and repeated until it settles). */
uint32_t cmp_gpu_decompress(struct cmp_gpu_engine *engine, const struct cmp_gpu_decode_batch *batch);

/*
 * Payload-only stream: the num_samples samples at src (device) encoded as ONE
 * bit stream from bit 0 of dst (device, 8-byte aligned), exactly as the
 * reference's encoder loop writes a frame's payload -- NONE or DIFF
 * preprocessing (lib/compress/preprocess.c:268-300), cmp_encoder_encode_s16
 * (lib/compress/encoder.c:327-378), the big-endian bit writer with its
 * zero-padded flush (lib/common/bitstream_writer.h:124-158, 205-227) -- but
 * without header, checksum or the 24-bit frame size limit of a frame, and
 * without a context.  encoder_outlier is used by GOLOMB_MULTI as by
 * cmp_initialise.  Asynchronous: *size (device) receives the stream's byte
 * count, or CMP_ERR_DST_TOO_SMALL when it exceeds dst_capacity (the bytes that
 * fit are written).  num_samples <= 89478485 (bit offsets stay below 2^32 at
 * the worst case of 48 bits per sample).  Build-defined extension: no
 * reference counterpart at the public API.
 */
uint32_t cmp_gpu_encode_stream(struct cmp_gpu_engine *engine, enum cmp_gpu_sample_type type, const void *src,
			       uint32_t num_samples, enum cmp_preprocessing preprocessing,
			       enum cmp_encoder_type encoder_type, uint32_t encoder_param, uint32_t encoder_outlier,
			       void *dst, uint32_t dst_capacity, uint32_t *size);

/*
 * Pack the frames of a strided batch output (frame f at frames + f*frame_stride,
 * sizes[f] bytes, as cmp_gpu_compress leaves them) back to back into out: frame
 * f at out + offsets[f], offsets 8-byte aligned, offsets[num_frames] = the
 * total.  Frames whose size is an error value take no bytes.  Reads only the
 * compressed bytes (rounded up to 8).  All pointers are device pointers;
 * out must hold the sum of the sizes rounded up to 8 each (at most
 * num_frames * frame_capacity rounded up to 8).  Asynchronous.  This is the
 * compaction step of the multi-GPU gather (shard.py); build-defined extension.
 */
uint32_t cmp_gpu_pack_frames(struct cmp_gpu_engine *engine, const void *frames, uint64_t frame_stride,
			     uint32_t frame_capacity, const uint32_t *sizes, uint32_t num_frames, void *out,
			     uint64_t *offsets);

/*
 * Multi-GPU gather of compressed frames, one call per rank
 * of an RCCL communicator the caller owns (ncclComm_t, passed as void *; one
 * process per GPU): every rank's frames (frame j of this rank at frames +
 * j*frame_stride, sizes[j] bytes, as cmp_gpu_compress leaves them; sizes and
 * frames device pointers) end up on `root`, packed at 8-byte aligned offsets
 * in `out` (device, out_capacity bytes), with out_offsets / out_sizes (host,
 * world * frames_per_rank entries) the frame table in GLOBAL frame order:
 *   CMP_GPU_LAYOUT_ROUNDROBIN  rank r's frame j is global frame r + world*j
 *   CMP_GPU_LAYOUT_BLOCK       rank r's frame j is global frame r*F + j
 *   CMP_GPU_LAYOUT_STREAMS     streams of fpc frames, stream s on rank s mod world
 * draws (host, per local frame; NULL: one each): cmp_gpu_batch.draws with
 * CMP_GPU_REPORT_DRAWS.  With CMP_GPU_GATHER_PATCH_IDS the root rewrites each
 * frame's header identifier (bytes 8..13) to what ONE process would have drawn
 * for the node's frames in global order with the reference's default counter
 * (cmp.c:27-50): id_base + the inclusive scan of the draws; a frame before its
 * context's first draw keeps its identifier.  The frame layouts refuse the
 * patch (CMP_ERR_PARAMS_INVALID on every rank) when a frame made no draw (a
 * secondary pass depends on its rank's previous frame: use STREAMS).  Every
 * rank decides from the same all-gathered table, so all ranks return the same
 * refusal; a frame with an error value is refused the same way
 * (CMP_ERR_GENERIC), and so is a root out_capacity below the packed bytes
 * (CMP_ERR_DST_TOO_SMALL).  Local failures on any rank (NULL frames / sizes,
 * the root's NULL or misaligned out, an allocation, the packing) are shared
 * through two status exchanges before the next collective, so every rank
 * returns the same value and no rank is left waiting in RCCL.  A NULL engine
 * or communicator, or a world above 256 ranks, cannot take part and returns
 * CMP_ERR_GENERIC at once (a caller error on every rank alike).  RCCL is the
 * copy the process already holds, else loaded on first use.  When the call
 * returns, the transfers and the identifier patch are complete.  Build-defined
 * extension (the C form of airs-compression_amd/shard.py).
 */
enum cmp_gpu_layout { CMP_GPU_LAYOUT_ROUNDROBIN = 0, CMP_GPU_LAYOUT_BLOCK = 1, CMP_GPU_LAYOUT_STREAMS = 2 };
#define CMP_GPU_GATHER_PATCH_IDS 0x1u
uint32_t cmp_gpu_gather(struct cmp_gpu_engine *engine, void *nccl_comm, uint32_t root, uint32_t layout, uint32_t fpc,
			const void *frames, uint64_t frame_stride, uint32_t frame_capacity, const uint32_t *sizes,
			const uint8_t *draws, uint32_t frames_per_rank, void *out, uint64_t out_capacity,
			uint64_t *out_offsets, uint32_t *out_sizes, uint64_t id_base, uint32_t flags);

/*
 * The gather's plan on the host (no device, no RCCL): from the all-gathered
 * table (entries[r * frames_per_rank + j] = size of rank r's frame j | its
 * draws << 32), the packed bytes of each rank, and in global frame order each
 * frame's offset in the root's buffer and size; ids (optional, world * F):
 * the identifier to write, or UINT64_MAX for a frame that keeps its own.
 * Returns 0, CMP_ERR_GENERIC (a frame carries an error value) or
 * CMP_ERR_PARAMS_INVALID (layout / fpc, or a frame layout with a frame that
 * made no draw while ids are requested).
 */
uint32_t cmp_gpu_gather_plan(const uint64_t *entries, uint32_t world, uint32_t frames_per_rank, uint32_t layout,
			     uint32_t fpc, uint64_t id_base, uint64_t *rank_bytes, uint64_t *offsets, uint32_t *sizes,
			     uint64_t *ids);

/* wait for all work queued on the engine */
uint32_t cmp_gpu_synchronize(struct cmp_gpu_engine *engine);

/* Fill num_frames device frames with the counter-hash synthetic signal used by
 * the benchmark (sample_bytes 2: u16; 4: i16-in-i32 with junk upper halves). */
uint32_t cmp_gpu_synthesize(struct cmp_gpu_engine *engine, void *dst, uint32_t sample_bytes,
			    uint64_t seed, uint32_t frame0, uint32_t samples_per_frame,
			    uint32_t num_frames, uint64_t stride, uint32_t noise_w);

/* non-zero when a GPU is present and the HIP runtime initialised */
int cmp_gpu_available(void);

#ifdef __cplusplus
}
#endif

#endif /* CMP_GPU_H */
