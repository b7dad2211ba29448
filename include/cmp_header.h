/*
 * cmp_header.h -- on-disk frame header layout (MI355X build).
 *
 * Drop-in replacement for the reference's lib/cmp_header.h:16-62.  The
 * constants below are the frame format, so they are identical in value.
 *
 * A frame is a big-endian bit-packed record:
 *
 *   byte  0-1   version_flag:1 (=1) | version_id:15 (=CMP_VERSION_NUMBER)
 *   byte  2-4   compressed_size:24   whole frame in bytes incl. header+checksum
 *   byte  5-7   original_size:24     2 * number of samples
 *   byte  8-13  identifier:48        model / acquisition-series identifier
 *   byte 14     sequence_number:8    passes since the last reset
 *   byte 15     preprocessing:4 | checksum_enabled:1 | encoder_type:3
 *   -- extension, present unless (preprocessing NONE and encoder UNCOMPRESSED):
 *   byte 16     model_rate:8
 *   byte 17-18  encoder_param:16
 *   byte 19-21  outlier:24
 *   -- payload (MSB-first bit stream), zero padded to a byte,
 *   -- optional XXH32 checksum, 4 bytes big-endian.
 */
#ifndef CMP_HEADER_H
#define CMP_HEADER_H

/* field widths in bits (reference lib/cmp_header.h:24-40) */
#define CMP_HDR_BITS_VERSION_FLAG 1
#define CMP_HDR_BITS_VERSION_ID 15
#define CMP_HDR_BITS_VERSION (CMP_HDR_BITS_VERSION_FLAG + CMP_HDR_BITS_VERSION_ID)
#define CMP_HDR_BITS_COMPRESSED_SIZE 24
#define CMP_HDR_BITS_ORIGINAL_SIZE 24
#define CMP_HDR_BITS_IDENTIFIER 48
#define CMP_HDR_BITS_SEQUENCE_NUMBER 8
#define CMP_HDR_BITS_METHOD_PREPROCESSING 4
#define CMP_HDR_BITS_METHOD_CHECKSUM_ENABLED 1
#define CMP_HDR_BITS_METHOD_ENCODER_TYPE 3
#define CMP_HDR_BITS_METHOD                                                       \
	(CMP_HDR_BITS_METHOD_PREPROCESSING + CMP_HDR_BITS_METHOD_CHECKSUM_ENABLED + \
	 CMP_HDR_BITS_METHOD_ENCODER_TYPE)

/* largest values the two 24-bit size fields can hold (reference :19-20) */
#define CMP_HDR_MAX_COMPRESSED_SIZE ((1ULL << CMP_HDR_BITS_COMPRESSED_SIZE) - 1)
#define CMP_HDR_MAX_ORIGINAL_SIZE ((1ULL << CMP_HDR_BITS_ORIGINAL_SIZE) - 1)

/* byte offsets of the base header fields (reference :46-51) */
#define CMP_HDR_OFFSET_VERSION 0
#define CMP_HDR_OFFSET_COMPRESSED_SIZE 2
#define CMP_HDR_OFFSET_ORIGINAL_SIZE 5
#define CMP_HDR_OFFSET_IDENTIFIER 8
#define CMP_HDR_OFFSET_SEQUENCE_NUMBER 14
#define CMP_HDR_OFFSET_METHOD 15

/* base header size in bytes: (16+24+24+48+8+8)/8 = 16 (reference :55-58) */
#define CMP_HDR_SIZE                                                                        \
	((CMP_HDR_BITS_VERSION + CMP_HDR_BITS_COMPRESSED_SIZE + CMP_HDR_BITS_ORIGINAL_SIZE + \
	  CMP_HDR_BITS_IDENTIFIER + CMP_HDR_BITS_SEQUENCE_NUMBER + CMP_HDR_BITS_METHOD) /   \
	 8)

/* size of the optional trailing checksum (reference :62) */
#define CMP_CHECKSUM_SIZE sizeof(uint32_t)

#endif /* CMP_HEADER_H */
