/*
 * cmp.h -- AIRSPACE compression API, MI355X build (libairscmp.so).
 *
 * Drop-in replacement for the reference's lib/cmp.h.  Types, struct layouts
 * (cmp_params = 44 B, cmp_context = 80 B on x86-64), macros and function
 * signatures match the reference so that programs/airspacecli.c,
 * examples/simple_compression.c and the reference's test/ suite compile and
 * link against this library unchanged.  The encode work behind
 * cmp_compress_*() runs as HIP kernels on the GPU (see cmp_gpu.h for the
 * device-pointer batch API that avoids the PCIe copies).
 *
 * Entry point                 replaces reference
 * ---------------------------------------------------------------------
 * cmp_set_timestamp_func()    lib/cmp.h:154   (lib/compress/cmp.c:44-50)
 * cmp_is_error()              lib/cmp.h:166   (cmp.c:53-56)
 * cmp_compress_bound()        lib/cmp.h:184   (cmp.c:59-74)
 * CMP_UNCOMPRESSED_BOUND()    lib/cmp.h:212-215
 * cmp_cal_work_buf_size()     lib/cmp.h:234   (cmp.c:77-103)
 * cmp_initialise()            lib/cmp.h:260   (cmp.c:152-209)
 * cmp_compress_i16()          lib/cmp.h:282   (cmp.c:410-421)
 * cmp_compress_i16_in_i32()   lib/cmp.h:298   (cmp.c:424-435)
 * cmp_compress_u16()          lib/cmp.h:308   (cmp.c:396-407)
 * cmp_reset()                 lib/cmp.h:329   (cmp.c:452-465)
 * cmp_deinitialise()          lib/cmp.h:344   (cmp.c:468-472)
 */
#ifndef CMP_H
#define CMP_H

#include <stdint.h>

#include "cmp_header.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CMP_QUOTE(str) #str
#define CMP_EXPAND_AND_QUOTE(str) CMP_QUOTE(str)

/* library version 0.6.0: the header's version_id field carries 600 */
#define CMP_VERSION_MAJOR 0
#define CMP_VERSION_MINOR 6
#define CMP_VERSION_RELEASE 0
#define CMP_VERSION_NUMBER \
	(CMP_VERSION_MAJOR * 100 * 100 + CMP_VERSION_MINOR * 100 + CMP_VERSION_RELEASE)
#define CMP_VERSION_STRING \
	CMP_EXPAND_AND_QUOTE(CMP_VERSION_MAJOR.CMP_VERSION_MINOR.CMP_VERSION_RELEASE)

/* predictor applied before entropy coding (header field "preprocessing") */
enum cmp_preprocessing {
	CMP_PREPROCESS_NONE,  /* residual = sample */
	CMP_PREPROCESS_DIFF,  /* residual = sample[i] - sample[i-1] */
	CMP_PREPROCESS_IWT,   /* multi-level integer wavelet transform */
	CMP_PREPROCESS_MODEL  /* residual = sample - model; secondary passes only */
};

/* entropy coder (header field "encoder_type") */
enum cmp_encoder_type {
	CMP_ENCODER_UNCOMPRESSED, /* raw 16-bit big-endian */
	CMP_ENCODER_GOLOMB_ZERO,  /* Golomb, 0 = escape symbol for raw outliers */
	CMP_ENCODER_GOLOMB_MULTI  /* Golomb, multi-level escape symbols */
};

/* compression parameters: a primary pass and optional secondary passes */
struct cmp_params {
	enum cmp_preprocessing primary_preprocessing;
	enum cmp_encoder_type primary_encoder_type;
	uint32_t primary_encoder_param;   /* Golomb parameter g in [1, 65535] */
	uint32_t primary_encoder_outlier; /* escape threshold, GOLOMB_MULTI only */

	uint32_t secondary_iterations;    /* secondary passes before a reset, < 256; 0 = off */
	enum cmp_preprocessing secondary_preprocessing;
	enum cmp_encoder_type secondary_encoder_type;
	uint32_t secondary_encoder_param;
	uint32_t secondary_encoder_outlier;
	uint32_t model_rate;              /* MODEL adaptation rate in [0, 16] */

	uint8_t checksum_enabled;              /* append XXH32 of the samples */
	uint8_t uncompressed_fallback_enabled; /* store raw when coding does not pay */
};

/* compression state; treat as opaque, use the functions below */
struct cmp_context {
	uint32_t magic;
	struct cmp_params params;
	void *work_buf;
	uint32_t work_buf_size;
	uint32_t model_size;
	uint64_t identifier;
	uint8_t sequence_number;
};

/* Set the 48-bit identifier source (coarse:32 << 16 | fine:16).  NULL
 * restores the built-in process-global counter. */
void cmp_set_timestamp_func(void (*get_current_timestamp_func)(uint32_t *coarse, uint16_t *fine));

/* non-zero iff code is an error value */
unsigned int cmp_is_error(uint32_t code);

/* worst-case frame size for packed_size bytes of 16-bit samples, or an error */
uint32_t cmp_compress_bound(uint32_t packed_size);

/* dst size for raw storage (NONE + UNCOMPRESSED, or the fallback path) */
#define CMP_UNCOMPRESSED_BOUND(packed_size)                                                  \
	((packed_size) <= (CMP_HDR_MAX_COMPRESSED_SIZE - CMP_HDR_SIZE - CMP_CHECKSUM_SIZE) ? \
		 (CMP_HDR_SIZE + (packed_size) + CMP_CHECKSUM_SIZE) :                        \
		 SIZE_MAX)

/* bytes of work buffer needed for params and src_size (0 if none) or an error */
uint32_t cmp_cal_work_buf_size(const struct cmp_params *params, uint32_t src_size);

/* validate params / work buffer and reset ctx; returns an error code */
uint32_t cmp_initialise(struct cmp_context *ctx, const struct cmp_params *params, void *work_buf,
			uint32_t work_buf_size);

/* Compress one frame.  dst must be 8-byte aligned; returns the frame size in
 * bytes or an error.  src_size is in bytes and must stay constant between
 * resets when MODEL preprocessing is configured.
 *
 * Threading: as with the reference, one context per thread is allowed (the
 * timestamp callback must then be thread-safe).  This build stages host
 * frames through one process-wide GPU engine, so concurrent calls are
 * serialised by a lock inside the library; for throughput use the batch API
 * in cmp_gpu.h, one engine per thread or stream. */
uint32_t cmp_compress_i16(struct cmp_context *ctx, void *dst, uint32_t dst_capacity,
			  const int16_t *src, uint32_t src_size);
/* as cmp_compress_i16() but only the low 16 bits of each 32-bit word are used */
uint32_t cmp_compress_i16_in_i32(struct cmp_context *ctx, void *dst, uint32_t dst_capacity,
				 const int32_t *src, uint32_t src_size);
uint32_t cmp_compress_u16(struct cmp_context *ctx, void *dst, uint32_t dst_capacity,
			  const uint16_t *src, uint32_t src_size);

/* force the next frame to use the primary parameters (new identifier) */
uint32_t cmp_reset(struct cmp_context *ctx);

/* zero the context; does not free caller memory */
void cmp_deinitialise(struct cmp_context *ctx);

#ifdef __cplusplus
}
#endif

#endif /* CMP_H */
