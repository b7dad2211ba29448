/*
 * oracle/ref_payload.c -- TEST INFRASTRUCTURE ONLY, compiled by
 * oracle/Makefile into _ref/libref.so next to the reference's own lib/
 * sources (never into liborc.so or the product).
 *
 * ref_payload_stream(): the payload-only stream of cmp_gpu_encode_stream as
 * the reference itself writes it, through the reference's INTERNAL encoder
 * API -- sample_read_src_init (lib/common/sample_reader.h:19-58),
 * preprocessing_get_method NONE/DIFF (lib/compress/preprocess.c:250-300,
 * 415-425), cmp_encoder_init / cmp_encoder_encode_s16
 * (lib/compress/encoder.c:185-224, 327-378) and the bit writer with its
 * zero-padded flush (lib/common/bitstream_writer.h:58-227) -- the loop of
 * compress_engine (lib/compress/cmp.c:296-303) without the header.
 * kind: 0 = 16-bit samples, 1 = i16 in i32.  Returns bytes or an error.
 */
#include <stdint.h>

#include "common/bitstream_writer.h"
#include "common/sample_reader.h"
#include "compress/encoder.h"
#include "compress/preprocess.h"

uint32_t ref_payload_stream(const void *src, uint32_t n, uint32_t kind, uint32_t pre, uint32_t enc_type, uint32_t g,
			    uint32_t outlier, void *dst, uint32_t cap)
{
	struct sample_desc desc;
	struct cmp_encoder enc;
	struct bitstream_writer bs;
	const struct preprocessing_method *pm;
	uint32_t e, nv, i;

	if (pre != CMP_PREPROCESS_NONE && pre != CMP_PREPROCESS_DIFF)
		return CMP_ERROR(PARAMS_INVALID);
	e = sample_read_src_init(&desc, src, n * (kind ? 4u : 2u), kind ? CMP_I16_IN_I32 : CMP_U16);
	if (cmp_is_error_int(e))
		return e;
	pm = preprocessing_get_method((enum cmp_preprocessing)pre);
	if (!pm)
		return CMP_ERROR(PARAMS_INVALID);
	nv = pm->init(&desc, NULL, 0);
	if (cmp_is_error_int(nv))
		return nv;
	e = cmp_encoder_init(&enc, (enum cmp_encoder_type)enc_type, g, outlier);
	if (cmp_is_error_int(e))
		return e;
	e = bitstream_writer_init(&bs, dst, cap);
	if (cmp_is_error_int(e))
		return e;
	for (i = 0; i < nv; i++)
		cmp_encoder_encode_s16(&enc, pm->process(i, &desc, NULL), &bs);
	return bitstream_flush(&bs);
}
