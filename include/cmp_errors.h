/*
 * cmp_errors.h -- error codes of the AIRSPACE compression API (MI355X build).
 *
 * Drop-in replacement for the reference's lib/cmp_errors.h:28-105.  The enum
 * values, the "(uint32_t)-code" return convention and the three helper
 * functions are ABI: callers written against the reference link against this
 * library unchanged.
 *
 *   enum cmp_error            <- reference lib/cmp_errors.h:28-60
 *   cmp_get_error_code()      <- reference lib/cmp_errors.h:74  (impl lib/common/cmp_errors.c:17-23)
 *   cmp_get_error_message()   <- reference lib/cmp_errors.h:89
 *   cmp_get_error_string()    <- reference lib/cmp_errors.h:104
 *
 * Every API function returns a uint32_t that is either a size / success value
 * or an error; a value is an error iff it is larger than (uint32_t)-128
 * (CMP_ERR_MAX_CODE).  Test with cmp_is_error() from cmp.h.
 */
#ifndef CMP_ERRORS_H
#define CMP_ERRORS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum cmp_error {
	CMP_ERR_NO_ERROR = 0,

	CMP_ERR_GENERIC = 1,
	CMP_ERR_PARAMS_INVALID = 10,

	CMP_ERR_DST_TOO_SMALL = 30,
	CMP_ERR_DST_NULL = 31,
	CMP_ERR_DST_UNALIGNED = 32,

	CMP_ERR_SRC_SIZE_WRONG = 40,
	CMP_ERR_SRC_NULL = 41,
	CMP_ERR_SRC_SIZE_MISMATCH = 42,

	CMP_ERR_WORK_BUF_TOO_SMALL = 50,
	CMP_ERR_WORK_BUF_NULL = 51,
	CMP_ERR_WORK_BUF_UNALIGNED = 52,

	CMP_ERR_HDR_CMP_SIZE_TOO_LARGE = 60,
	CMP_ERR_HDR_ORIGINAL_TOO_LARGE = 61,

	CMP_ERR_CONTEXT_INVALID = 70,

	CMP_ERR_INT_HDR = 100,
	CMP_ERR_INT_ENCODER = 101,
	CMP_ERR_INT_BITSTREAM = 102,

	/* upper limit of the error code space, never returned */
	CMP_ERR_MAX_CODE = 128
};

/* return value -> error code (CMP_ERR_NO_ERROR for a non-error value) */
enum cmp_error cmp_get_error_code(uint32_t code);

/* return value -> static human-readable description */
const char *cmp_get_error_message(uint32_t code);

/* error code -> static human-readable description */
const char *cmp_get_error_string(enum cmp_error code);

#ifdef __cplusplus
}
#endif

#endif /* CMP_ERRORS_H */
