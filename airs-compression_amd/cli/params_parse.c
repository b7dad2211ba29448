/*
 * params_parse.c -- "--params" grammar of the airspace CLI.
 *
 * Behaviour follows the reference's programs/params_parse.c:
 *   - keys and their fields: param_keys :95-113 (order kept for printing);
 *   - enum names with optional prefixes (CMP_PREPROCESS_ / CMP_ / PREPROCESS_,
 *     CMP_ENCODER_ / CMP_ / ENCODER_, CMP_ for booleans), case-insensitive,
 *     at most one prefix stripped: :33-82, :190-199;
 *   - numbers: decimal digits only, no sign, no leading zero, <= UINT32_MAX
 *     (str_slice.h s8_to_u32 :275-299);
 *   - whitespace " \t\n\r\v\f" trimmed around keys, values and pairs
 *     (str_slice.h :218-239); empty pairs skipped; first error stops the
 *     parse (pairs before it stay applied): :259-317;
 *   - printing: "name = VALUE" lines joined by ",\n", a final "\n";
 *     booleans normalised, unknown enum values print as INVALID: :366-396.
 */
#include "params_parse.h"

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "log.h"

/* a (pointer, length) view into the caller's string */
struct span {
	const char *p;
	size_t n;
};

static int is_ws(char c)
{
	return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

static struct span trim(struct span s)
{
	while (s.n && is_ws(s.p[0])) {
		s.p++;
		s.n--;
	}
	while (s.n && is_ws(s.p[s.n - 1]))
		s.n--;
	return s;
}

static char lower(char c)
{
	return (c >= 'A' && c <= 'Z') ? (char)(c - 'A' + 'a') : c;
}

/* case-insensitive: does s start with the NUL-terminated word w (whole match if exact) */
static int word_prefix(struct span s, const char *w, int exact)
{
	size_t n = strlen(w), i;

	if (s.n < n || (exact && s.n != n))
		return 0;
	for (i = 0; i < n; i++)
		if (lower(s.p[i]) != lower(w[i]))
			return 0;
	return 1;
}

enum field_kind { F_U32, F_PRE, F_ENC, F_BOOL };

struct name_value {
	const char *name;
	uint32_t value;
};

static const struct name_value pre_names[] = { { "NONE", CMP_PREPROCESS_NONE },
					       { "DIFF", CMP_PREPROCESS_DIFF },
					       { "IWT", CMP_PREPROCESS_IWT },
					       { "MODEL", CMP_PREPROCESS_MODEL },
					       { NULL, 0 } };
static const struct name_value enc_names[] = { { "UNCOMPRESSED", CMP_ENCODER_UNCOMPRESSED },
					       { "GOLOMB_ZERO", CMP_ENCODER_GOLOMB_ZERO },
					       { "GOLOMB_MULTI", CMP_ENCODER_GOLOMB_MULTI },
					       { NULL, 0 } };
static const struct name_value bool_names[] = { { "FALSE", 0 }, { "TRUE", 1 }, { "0", 0 }, { "1", 1 }, { NULL, 0 } };

static const char *const pre_prefixes[] = { "CMP_PREPROCESS_", "CMP_", "PREPROCESS_", NULL };
static const char *const enc_prefixes[] = { "CMP_ENCODER_", "CMP_", "ENCODER_", NULL };
static const char *const bool_prefixes[] = { "CMP_", NULL };

struct kind_desc {
	const struct name_value *names;
	const char *const *prefixes;
};

static const struct kind_desc kinds[] = {
	[F_U32] = { NULL, NULL },
	[F_PRE] = { pre_names, pre_prefixes },
	[F_ENC] = { enc_names, enc_prefixes },
	[F_BOOL] = { bool_names, bool_prefixes },
};

#define FIELD(f) offsetof(struct cmp_params, f), sizeof(((struct cmp_params *)0)->f)
static const struct key_desc {
	const char *name;
	size_t off, size;
	enum field_kind kind;
} keys[] = {
	{ "primary_preprocessing", FIELD(primary_preprocessing), F_PRE },
	{ "primary_encoder_type", FIELD(primary_encoder_type), F_ENC },
	{ "primary_encoder_param", FIELD(primary_encoder_param), F_U32 },
	{ "primary_encoder_outlier", FIELD(primary_encoder_outlier), F_U32 },
	{ "secondary_iterations", FIELD(secondary_iterations), F_U32 },
	{ "secondary_preprocessing", FIELD(secondary_preprocessing), F_PRE },
	{ "secondary_encoder_type", FIELD(secondary_encoder_type), F_ENC },
	{ "secondary_encoder_param", FIELD(secondary_encoder_param), F_U32 },
	{ "secondary_encoder_outlier", FIELD(secondary_encoder_outlier), F_U32 },
	{ "model_rate", FIELD(model_rate), F_U32 },
	{ "checksum_enabled", FIELD(checksum_enabled), F_BOOL },
	{ "uncompressed_fallback_enabled", FIELD(uncompressed_fallback_enabled), F_BOOL },
};
#undef FIELD
#define NKEYS (sizeof(keys) / sizeof(keys[0]))

static void store(struct cmp_params *par, const struct key_desc *k, uint32_t v)
{
	unsigned char *dst = (unsigned char *)par + k->off;

	if (k->size == 1) {
		uint8_t b = (uint8_t)v;
		memcpy(dst, &b, 1);
	} else if (k->size == 2) {
		uint16_t h = (uint16_t)v;
		memcpy(dst, &h, 2);
	} else {
		memcpy(dst, &v, 4);
	}
}

static uint32_t fetch(const struct cmp_params *par, const struct key_desc *k)
{
	const unsigned char *src = (const unsigned char *)par + k->off;

	if (k->size == 1)
		return src[0];
	if (k->size == 2) {
		uint16_t h;
		memcpy(&h, src, 2);
		return h;
	}
	{
		uint32_t w;
		memcpy(&w, src, 4);
		return w;
	}
}

static int parse_u32(struct span s, uint32_t *out)
{
	uint64_t v = 0;
	size_t i;

	if (!s.n || (s.n > 1 && s.p[0] == '0'))
		return 0;
	for (i = 0; i < s.n; i++) {
		if (s.p[i] < '0' || s.p[i] > '9')
			return 0;
		v = v * 10u + (uint64_t)(s.p[i] - '0');
		if (v > UINT32_MAX)
			return 0;
	}
	*out = (uint32_t)v;
	return 1;
}

static int parse_name(const struct kind_desc *d, struct span s, uint32_t *out)
{
	const char *const *pf;
	const struct name_value *nv;

	for (pf = d->prefixes; *pf; pf++) {
		if (word_prefix(s, *pf, 0)) {
			s.p += strlen(*pf);
			s.n -= strlen(*pf);
			break;
		}
	}
	for (nv = d->names; nv->name; nv++) {
		if (word_prefix(s, nv->name, 1)) {
			*out = nv->value;
			return 1;
		}
	}
	return 0;
}

static void hint(const struct key_desc *k)
{
	const struct name_value *nv;

	if (k->kind == F_U32) {
		log_msg(LOG_INFO, "Hint: Value for '%s' must be a whole number.", k->name);
		return;
	}
	log_msg(LOG_INFO, "Hint: Valid options for '%s' are:", k->name);
	for (nv = kinds[k->kind].names; nv->name; nv++)
		log_msg(LOG_INFO, "  - '%s'", nv->name);
}

static enum cmp_parse_status parse_pair(struct span key, struct span val, struct cmp_params *par)
{
	const struct key_desc *k = NULL;
	uint32_t v;
	size_t i;
	int ok;

	key = trim(key);
	val = trim(val);
	for (i = 0; i < NKEYS && !k; i++)
		if (word_prefix(key, keys[i].name, 1))
			k = &keys[i];
	if (!k) {
		log_msg(LOG_ERROR, "Unknown compression parameter: '%.*s'", (int)key.n, key.p);
		return CMP_PARSE_INVALID_KEY;
	}
	ok = k->kind == F_U32 ? parse_u32(val, &v) : parse_name(&kinds[k->kind], val, &v);
	if (!ok) {
		log_msg(LOG_ERROR, "Invalid value '%.*s' for parameter '%.*s'.", (int)val.n, val.p, (int)key.n,
			key.p);
		hint(k);
		return CMP_PARSE_INVALID_VALUE;
	}
	store(par, k, v);
	return CMP_PARSE_OK;
}

enum cmp_parse_status cmp_params_parse(const char *str, struct cmp_params *params)
{
	struct span rest = { str ? str : "", str ? strlen(str) : 0 };
	int seen = 0;

	rest = trim(rest);
	while (rest.n) {
		const char *comma = memchr(rest.p, ',', rest.n);
		struct span pair = { rest.p, comma ? (size_t)(comma - rest.p) : rest.n };
		const char *eq;
		enum cmp_parse_status r;

		if (comma) {
			rest.n -= pair.n + 1u;
			rest.p = comma + 1;
		} else {
			rest.n = 0;
		}
		pair = trim(pair);
		if (!pair.n)
			continue;
		eq = memchr(pair.p, '=', pair.n);
		if (!eq) {
			log_msg(LOG_ERROR, "Parameters string is missing '=': '%.*s'.", (int)pair.n, pair.p);
			return CMP_PARSE_MISSING_EQUAL;
		}
		{
			struct span key = { pair.p, (size_t)(eq - pair.p) };
			struct span val = { eq + 1, pair.n - key.n - 1u };

			r = parse_pair(key, val, params);
		}
		if (r != CMP_PARSE_OK)
			return r;
		seen = 1;
	}
	if (!seen) {
		log_msg(LOG_ERROR, "Empty parameter string.");
		return CMP_PARSE_EMPTY_STR;
	}
	return CMP_PARSE_OK;
}

/* append to buf (bounded), counting the full length */
static void put(char *buf, size_t cap, size_t *len, const char *s)
{
	size_t n = strlen(s);

	if (cap && *len < cap - 1u) {
		size_t room = cap - 1u - *len;

		memcpy(buf + *len, s, n < room ? n : room);
	}
	*len += n;
}

size_t cmp_params_to_string(char *buf, size_t cap, const struct cmp_params *params)
{
	size_t len = 0, i;

	for (i = 0; i < NKEYS; i++) {
		const struct key_desc *k = &keys[i];
		uint32_t v = fetch(params, k);
		char num[16];
		const char *text = "INVALID";

		if (k->kind == F_U32) {
			snprintf(num, sizeof(num), "%u", v);
			text = num;
		} else {
			const struct name_value *nv;

			if (k->kind == F_BOOL)
				v = v != 0;
			for (nv = kinds[k->kind].names; nv->name; nv++) {
				if (nv->value == v) {
					text = nv->name;
					break;
				}
			}
		}
		put(buf, cap, &len, k->name);
		put(buf, cap, &len, " = ");
		put(buf, cap, &len, text);
		put(buf, cap, &len, i + 1u < NKEYS ? ",\n" : "\n");
	}
	if (cap)
		buf[len < cap ? len : cap - 1u] = '\0';
	return len;
}
