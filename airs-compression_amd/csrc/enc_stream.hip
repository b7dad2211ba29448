// enc_stream.hip -- payload-only streams (cmp_gpu_encode_stream): the
// encode kernel in STREAM mode, compiled in its own translation unit.
//
// A stream is one frame without header, checksum or 24-bit size limit: the
// reference's encoder loop as compress_engine runs it for the payload
// (preprocess.c NONE/DIFF -> cmp_encoder_encode_s16 encoder.c:327-378 ->
// bitstream_writer.h:124-158, bitstream_flush :205-227), over up to
// AIRS_STREAM_MAX samples.  Its segments form ONE look-back chain (16 Ki
// segments for 256 Mi samples); its look-back reads one window of 64
// granules per round, like a frame's (AIRS_STREAM_LB_WIN, enc_kernel.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "enc_kernel.h"

namespace airs {

template <int W, int PRE, int ENC, bool RICE>
static void stream_go(const KArgs &k, bool full, uint32_t grid, hipStream_t s)
{
	const size_t lds = (size_t)seg_images(W, 0) * (k.img_words + 4u) * 4u;
	if (full)
		launch_segments(encode_kernel<W, PRE, ENC, RICE, 0, true, false, true>, k, grid, lds, s);
	else
		launch_segments(encode_kernel<W, PRE, ENC, RICE, 0, false, false, true>, k, grid, lds, s);
}

template <int W, int PRE>
static void stream_enc(const KArgs &k, uint32_t enc, bool rice, bool full, uint32_t grid, hipStream_t s)
{
	switch (enc) {
	case ENC_RAW:
		stream_go<W, PRE, ENC_RAW, true>(k, full, grid, s);
		break;
	case ENC_ZERO:
		if (rice)
			stream_go<W, PRE, ENC_ZERO, true>(k, full, grid, s);
		else
			stream_go<W, PRE, ENC_ZERO, false>(k, full, grid, s);
		break;
	default:
		if (rice)
			stream_go<W, PRE, ENC_MULTI, true>(k, full, grid, s);
		else
			stream_go<W, PRE, ENC_MULTI, false>(k, full, grid, s);
		break;
	}
}

uint32_t stream_segn(uint32_t sample_bytes)
{
	return seg_chunks(sample_bytes == 4 ? 4 : 2, 0) * AIRS_SEG;
}

void stream_encode(const KArgs &k, uint32_t sample_bytes, uint32_t pre, uint32_t enc, bool rice, bool full,
		   uint32_t grid, hipStream_t s)
{
	if (sample_bytes == 2) {
		if (pre == PRE_DIFF)
			stream_enc<2, PRE_DIFF>(k, enc, rice, full, grid, s);
		else
			stream_enc<2, PRE_NONE>(k, enc, rice, full, grid, s);
	} else {
		if (pre == PRE_DIFF)
			stream_enc<4, PRE_DIFF>(k, enc, rice, full, grid, s);
		else
			stream_enc<4, PRE_NONE>(k, enc, rice, full, grid, s);
	}
}

} // namespace airs
