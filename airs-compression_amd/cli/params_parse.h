/*
 * params_parse.h -- the CLI's "--params key=value,..." grammar.
 *
 * Same contract as the reference's programs/params_parse.h:17-58:
 * cmp_params_parse() fills a struct cmp_params from "key=value" pairs
 * separated by ',' (keys case-insensitive, whitespace around tokens
 * tolerated, empty pairs skipped, the last of a repeated key wins) and stops
 * at the first error; cmp_params_to_string() prints every field, one
 * "name = VALUE" per line.  Exported from lib/libairscli.so so the tests can
 * drive it without the CLI.
 */
#ifndef AIRS_PARAMS_PARSE_H
#define AIRS_PARAMS_PARSE_H

#include <stddef.h>

#include "cmp.h"

#ifdef __cplusplus
extern "C" {
#endif

enum cmp_parse_status {
	CMP_PARSE_OK = 0,
	CMP_PARSE_EMPTY_STR,     /* no key=value pair at all (NULL, blanks, commas) */
	CMP_PARSE_MISSING_EQUAL, /* a pair without '=' */
	CMP_PARSE_INVALID_KEY,   /* unknown key */
	CMP_PARSE_INVALID_VALUE  /* malformed number or unknown enum/bool name */
};

enum cmp_parse_status cmp_params_parse(const char *str, struct cmp_params *params);

/* Writes the text into buf (NUL-terminated, truncated to cap) and returns the
 * length the whole text needs (excluding the NUL), like snprintf. */
size_t cmp_params_to_string(char *buf, size_t cap, const struct cmp_params *params);

#ifdef __cplusplus
}
#endif

#endif /* AIRS_PARAMS_PARSE_H */
