/*
 * airspace.c -- command-line (de)compressor over libairscmp.so (SURVEY.md
 * 8(f) row 3, the caller of the hot path).
 *
 * Same command line, file format and messages as the reference's
 * programs/airspacecli.c:290-433 and programs/file.c:
 *   airspace -c [--params K=V,...] [FILE... | -] [-o OUTPUT | --stdout]
 * Every input file is one frame of big-endian 16-bit samples
 * (file.c:337-358); the output is FILE.air (airspacecli.c:62-88) or OUTPUT,
 * and an existing output file or directory is never overwritten
 * (file.c:381-405).  Without a FILE, or for "-", the samples come from stdin
 * (read once, airspacecli.c:212-245) and go to stdout.
 *
 * MI355X-first: the reference compresses one file per call.  Here runs of
 * consecutive files of the same size (up to BATCH_BYTES) go to the GPU as
 * one cmp_gpu_compress() batch, which produces the same frames, in the same
 * order and with the same context state, as one cmp_compress_u16() per file
 * (cmp_gpu.h).  Parameter sets that need a work buffer (MODEL or IWT) batch
 * the same way since round 5, with the work buffer on the device: the model
 * carries from one file to the next, inside a batch and across batches, as
 * in the reference's per-file loop (file.c:435-488).
 *
 * Decompression (the reference's default mode prints "Decompression not
 * implemented yet", airspacecli.c:421-423) is an extension here: the frames
 * of each .air input are decoded on the GPU with cmp_gpu_decompress() and
 * written back as big-endian 16-bit samples: runs of frames other than MODEL
 * as one batch, each MODEL frame alone, against the model rebuilt from the
 * frames before it.
 */
#include <errno.h>
#include <getopt.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "cmp.h"
#include "cmp_errors.h"
#include "cmp_gpu.h"
#include "log.h"
#include "params_parse.h"

#define PROGRAM_NAME "AIRSPACE CLI"
#define AIR_EXT ".air"
#define STDIN_NAME "//*-stdin-*//"
#define STDOUT_NAME "//*-stdout-*//"
#define NULL_NAME "/dev/null"
/* host bytes of input samples staged per GPU batch */
#define BATCH_BYTES (256u << 20)
#define HDR_MIN 16u

static int g_stdin_console, g_stdout_console;

static int is_console(FILE *f)
{
	if (f == stdin && g_stdin_console)
		return 1;
	if (f == stdout && g_stdout_console)
		return 1;
	return isatty(fileno(f));
}

static void *xmalloc(size_t n)
{
	void *p = malloc(n ? n : 1);

	if (!p) {
		log_errno("Memory allocation failed for size %lu", (unsigned long)n);
		exit(EXIT_FAILURE);
	}
	return p;
}

/* ---- sizes in human-readable form (reference util.c:57-113) ------------- */
struct hsize {
	double v;
	int prec;
	const char *unit;
};

static struct hsize human(uint64_t n, int exact)
{
	static const char *const units[] = { " B", " KiB", " MiB", " GiB", " TiB", " PiB", " EiB" };
	struct hsize h;
	int u = 0;

	if (exact) {
		h.v = n >= (1ull << 53) ? (double)n / (1ull << 20) : (double)n;
		h.unit = n >= (1ull << 53) ? " MiB" : " B";
		h.prec = n >= (1ull << 53) ? 2 : 0;
		return h;
	}
	while (u < 6 && n >= (1ull << (10 * (u + 1))))
		u++;
	h.v = (double)n / (double)(1ull << (10 * u));
	h.unit = units[u];
	if (h.v >= 100 || (uint64_t)h.v == n)
		h.prec = 0;
	else if (h.v >= 10)
		h.prec = 1;
	else if (h.v > 1)
		h.prec = 2;
	else
		h.prec = 3;
	return h;
}

static void log_ratio(int level, const char *in_name, uint64_t in, const char *out_name, uint64_t out)
{
	const int exact = log_level() > LOG_DEBUG;
	const struct hsize a = human(in, exact), b = human(out, exact);

	log_plain(level, "%s: %.2f%% (%.*f%s => %.*f%s, %s)\n", in_name, (double)out / (double)in * 100.0, a.prec,
		  a.v, a.unit, b.prec, b.v, b.unit, out_name);
}

static void log_summary(const char *verb, const char *const *in_names, int n, uint64_t in, const char *out_name,
			uint64_t out)
{
	if (n == 1) {
		if (log_level() < LOG_DEBUG)
			log_ratio(LOG_INFO, in_names[0], in, out_name, out);
	} else {
		const int exact = log_level() > LOG_DEBUG;
		const struct hsize a = human(in, exact), b = human(out, exact);

		log_plain(LOG_INFO, "%d files %s: %.2f%% (%.*f%s => %.*f%s)\n", n, verb,
			  (double)out / (double)in * 100.0, a.prec, a.v, a.unit, b.prec, b.v, b.unit);
	}
}

/* ---- file I/O (reference file.c) ----------------------------------------- */
static const char *display(const char *name)
{
	return strcmp(name, STDIN_NAME) == 0 ? "stdin" : strcmp(name, STDOUT_NAME) == 0 ? "stdout" : name;
}

/* stdin is read once and replayed for every "-" (file.c:121-206) */
static int read_stdin(uint8_t **data, size_t *size)
{
	static uint8_t *buf;
	static size_t len;
	static int done;

	if (!done) {
		size_t cap = 4096;

		buf = xmalloc(cap);
		for (;;) {
			size_t got = fread(buf + len, 1, cap - len, stdin);

			len += got;
			if (len < cap)
				break;
			cap *= 2;
			buf = realloc(buf, cap);
			if (!buf) {
				log_errno("Failed to reallocate memory for stdin");
				return -1;
			}
		}
		if (ferror(stdin)) {
			log_msg(LOG_ERROR, "Error reading from stdin");
			return -1;
		}
		done = 1;
	}
	*data = buf;
	*size = len;
	return 0;
}

/* whole file (or stdin) into memory; *owned tells whether to free it */
static int load_file(const char *name, uint8_t **data, size_t *size, int *owned)
{
	FILE *f;
	struct stat st;

	*owned = 0;
	if (strcmp(name, STDIN_NAME) == 0) {
		if (read_stdin(data, size))
			return -1;
	} else {
		f = fopen(name, "rb");
		if (!f) {
			log_errno("Can't open '%s'", name);
			return -1;
		}
		if (fstat(fileno(f), &st)) {
			log_errno("Can't get size of '%s'", name);
			fclose(f);
			return -1;
		}
		*size = (size_t)st.st_size;
		*data = xmalloc(*size);
		*owned = 1;
		if (fread(*data, 1, *size, f) != *size) {
			log_errno("Can't read '%s'", name);
			fclose(f);
			free(*data);
			*owned = 0;
			return -1;
		}
		fclose(f);
	}
	if (*size == 0) {
		log_msg(LOG_ERROR, "'%s' is empty.", display(name));
		if (*owned)
			free(*data);
		*owned = 0;
		return -1;
	}
	if (*size > UINT32_MAX) {
		log_msg(LOG_ERROR, "File '%s' is too large to read in (size: %llu bytes)", display(name),
			(unsigned long long)*size);
		if (*owned)
			free(*data);
		*owned = 0;
		return -1;
	}
	return 0;
}

/* size of a file (or of stdin's content) with load_file's checks */
static int probe_size(const char *name, size_t *size)
{
	struct stat st;
	uint8_t *data;
	int owned;

	if (strcmp(name, STDIN_NAME) == 0)
		return load_file(name, &data, size, &owned);
	if (stat(name, &st)) {
		log_errno("Can't open '%s'", name);
		return -1;
	}
	*size = (size_t)st.st_size;
	if (*size == 0) {
		log_msg(LOG_ERROR, "'%s' is empty.", name);
		return -1;
	}
	if (*size > UINT32_MAX) {
		log_msg(LOG_ERROR, "File '%s' is too large to read in (size: %llu bytes)", name,
			(unsigned long long)*size);
		return -1;
	}
	return 0;
}

/* never overwrites: refuses directories and existing files (file.c:381-405) */
static int save_file(const char *name, const void *data, size_t size)
{
	FILE *f;
	int err = 0;

	if (strcmp(name, STDOUT_NAME) == 0) {
		f = stdout;
	} else {
		if (strcmp(name, NULL_NAME) != 0) {
			struct stat st;

			if (stat(name, &st) == 0 && S_ISDIR(st.st_mode)) {
				log_msg(LOG_ERROR, "'%s' is a directory", name);
				return -1;
			}
			f = fopen(name, "rb");
			if (f) {
				fclose(f);
				log_msg(LOG_ERROR, "'%s' already exists", name);
				return -1;
			}
		}
		f = fopen(name, "wb");
		if (!f) {
			log_errno("Can't open '%s'", name);
			return -1;
		}
	}
	if (fwrite(data, 1, size, f) != size) {
		log_errno("Error writing '%s'", display(name));
		err = -1;
	}
	if (f == stdout) {
		fflush(stdout);
	} else if (fclose(f) && !err) {
		log_msg(LOG_WARNING, "File '%s' saved successfully but close failed", name);
	}
	return err;
}

static char *with_suffix(const char *name)
{
	size_t n = strlen(name);
	char *s = xmalloc(n + sizeof(AIR_EXT));

	memcpy(s, name, n);
	memcpy(s + n, AIR_EXT, sizeof(AIR_EXT));
	return s;
}

/* ---- device staging -------------------------------------------------------- */
struct dev {
	struct cmp_gpu_engine *eng;
	void *src, *dst, *sizes;
	size_t src_cap, dst_cap, sizes_cap;
};

static int dev_reserve(void **p, size_t *cap, size_t need)
{
	if (need <= *cap)
		return 0;
	if (*p)
		hipFree(*p);
	*p = NULL;
	*cap = 0;
	if (hipMalloc(p, need) != hipSuccess) {
		log_msg(LOG_ERROR, "GPU allocation of %lu bytes failed", (unsigned long)need);
		return -1;
	}
	*cap = need;
	return 0;
}

static int dev_open(struct dev *d)
{
	uint32_t e;

	if (d->eng)
		return 0;
	e = cmp_gpu_engine_create(&d->eng, NULL);
	if (cmp_is_error(e)) {
		log_cmp(e, "No usable GPU");
		d->eng = NULL;
		return -1;
	}
	return 0;
}

static void dev_close(struct dev *d)
{
	if (d->src)
		hipFree(d->src);
	if (d->dst)
		hipFree(d->dst);
	if (d->sizes)
		hipFree(d->sizes);
	if (d->eng)
		cmp_gpu_engine_destroy(d->eng);
	memset(d, 0, sizeof(*d));
}

/* ---- compression ------------------------------------------------------------ */
struct job {
	const char *out_name; /* NULL: FILE.air per input */
	const char *const *in;
	int n_in;
	uint64_t sum_in, sum_out;
	char *last_out; /* display name of the last output written */
};

/* output name of input i (caller frees when *owned) */
static const char *out_name_of(const struct job *j, int i, int *owned)
{
	*owned = !j->out_name;
	return j->out_name ? j->out_name : with_suffix(j->in[i]);
}

static int emit(struct job *j, int i, const void *frame, uint32_t size, uint32_t in_size)
{
	int owned, r;
	const char *out = out_name_of(j, i, &owned);

	r = save_file(out, frame, size);
	if (!r) {
		log_ratio(LOG_DEBUG, display(j->in[i]), in_size, display(out), size);
		j->sum_in += in_size;
		j->sum_out += size;
		free(j->last_out);
		j->last_out = strdup(display(out));
	}
	if (owned)
		free((void *)out);
	return r;
}

static void be16_to_host(uint16_t *dst, const uint8_t *src, size_t n)
{
	size_t i;

	for (i = 0; i < n; i++)
		dst[i] = (uint16_t)(src[2 * i] << 8 | src[2 * i + 1]);
}

static uint32_t frame_capacity(uint32_t src_size)
{
	uint32_t cap = cmp_compress_bound(src_size);

	if (cmp_is_error(cap)) {
		log_msg(LOG_WARNING, "Can't calculating compressed data buffer size, use maximum size");
		cap = (1u << 24) - 1u;
	}
	return cap;
}

/* A run of same-size files [i0, i1) as one GPU batch (frames at a 16-byte
 * stride in stage), written out in order. */
static int compress_run(struct job *j, struct dev *d, struct cmp_context *ctx, int i0, int i1, uint32_t size,
			uint16_t *stage)
{
	const uint32_t nf = (uint32_t)(i1 - i0);
	const uint32_t cap = frame_capacity(size);
	const uint64_t dstride = ((uint64_t)cap + 7u) & ~7ull;
	const uint64_t sstride = ((uint64_t)size + 15u) & ~15ull;
	struct cmp_gpu_batch b;
	uint32_t *sizes, e;
	uint8_t *frame;
	int i, r = 0;

	if (dev_open(d) || dev_reserve(&d->src, &d->src_cap, sstride * nf) ||
	    dev_reserve(&d->dst, &d->dst_cap, dstride * nf) || dev_reserve(&d->sizes, &d->sizes_cap, 4u * nf))
		return -1;
	if (hipMemcpy(d->src, stage, sstride * nf, hipMemcpyHostToDevice) != hipSuccess) {
		log_msg(LOG_ERROR, "Copy to the GPU failed");
		return -1;
	}
	memset(&b, 0, sizeof(b));
	b.type = CMP_GPU_U16;
	b.src = d->src;
	b.src_stride = sstride;
	b.src_size = size;
	b.dst = d->dst;
	b.dst_stride = dstride;
	b.dst_capacity = cap;
	b.sizes = d->sizes;
	e = cmp_gpu_compress(d->eng, ctx, 1, nf, &b);
	if (!cmp_is_error(e))
		e = cmp_gpu_synchronize(d->eng);
	if (cmp_is_error(e)) {
		log_cmp(e, "Compression failed for %s", display(j->in[i0]));
		return -1;
	}
	sizes = xmalloc(4u * nf);
	frame = xmalloc(cap);
	if (hipMemcpy(sizes, d->sizes, 4u * nf, hipMemcpyDeviceToHost) != hipSuccess) {
		log_msg(LOG_ERROR, "Copy from the GPU failed");
		r = -1;
	}
	for (i = 0; !r && i < (int)nf; i++) {
		if (cmp_is_error(sizes[i])) {
			log_cmp(sizes[i], "Compression failed for %s", display(j->in[i0 + i]));
			r = -1;
		} else if (hipMemcpy(frame, (uint8_t *)d->dst + dstride * i, sizes[i], hipMemcpyDeviceToHost) !=
			   hipSuccess) {
			log_msg(LOG_ERROR, "Copy from the GPU failed");
			r = -1;
		} else {
			r = emit(j, i0 + i, frame, sizes[i], size);
		}
	}
	free(frame);
	free(sizes);
	return r;
}

static int compress_files(struct job *j, const struct cmp_params *par)
{
	struct cmp_context ctx;
	struct dev d;
	void *wb = NULL;
	uint32_t wbs, e;
	uint8_t *raw;
	size_t size;
	int owned, r = -1, i;

	memset(&d, 0, sizeof(d));
	if (probe_size(j->in[0], &size))
		return -1;
	wbs = cmp_cal_work_buf_size(par, (uint32_t)size);
	if (cmp_is_error(wbs)) {
		log_cmp(wbs, "Error calculating work buffer size");
		return -1;
	}
	if (wbs) {
		/* the work buffer on the device (cmp_gpu_compress reads and writes it there) */
		if (dev_open(&d) || hipMalloc(&wb, ((size_t)wbs + 15u) & ~(size_t)15u) != hipSuccess) {
			log_msg(LOG_ERROR, "GPU allocation of the work buffer failed");
			wb = NULL;
			goto done;
		}
	}
	e = cmp_initialise(&ctx, par, wb, wbs);
	if (cmp_is_error(e)) {
		log_cmp(e, "Compression initialization failed");
		goto done;
	}

	{
		/* batches of consecutive same-size files */
		uint16_t *stage = NULL;
		size_t stage_cap = 0;
		int i0 = 0, nrun = 0;
		uint32_t run_size = 0;

		for (i = 0; i <= j->n_in; i++) {
			int load_failed = 0;
			uint64_t sstride;

			if (i < j->n_in) {
				if (load_file(j->in[i], &raw, &size, &owned)) {
					load_failed = 1;
				} else if (size % 2u) {
					log_msg(LOG_ERROR, "%s: file size not a multiple of 2", display(j->in[i]));
					if (owned)
						free(raw);
					load_failed = 1;
				}
			}
			sstride = ((uint64_t)run_size + 15u) & ~15ull;
			if (nrun && (i == j->n_in || load_failed || size != run_size ||
				     sstride * (uint64_t)(nrun + 1) > BATCH_BYTES)) {
				if (compress_run(j, &d, &ctx, i0, i0 + nrun, run_size, stage)) {
					if (i < j->n_in && !load_failed && owned)
						free(raw);
					free(stage);
					goto done;
				}
				nrun = 0;
			}
			if (i == j->n_in || load_failed) {
				if (load_failed) {
					free(stage);
					goto done;
				}
				break;
			}
			if (!nrun) {
				i0 = i;
				run_size = (uint32_t)size;
			}
			sstride = ((uint64_t)run_size + 15u) & ~15ull;
			if (sstride * (uint64_t)(nrun + 1) > stage_cap) {
				size_t want = (size_t)(sstride * (uint64_t)(nrun + 1));

				want = want < 2 * stage_cap ? 2 * stage_cap : want;
				stage = realloc(stage, want);
				if (!stage) {
					log_errno("Memory allocation failed");
					goto done;
				}
				stage_cap = want;
			}
			be16_to_host((uint16_t *)((uint8_t *)stage + sstride * nrun), raw, size / 2u);
			if (owned)
				free(raw);
			nrun++;
		}
		free(stage);
	}
	log_summary("compressed", j->in, j->n_in, j->sum_in, j->last_out ? j->last_out : "", j->sum_out);
	r = 0;
done:
	if (wb)
		hipFree(wb);
	dev_close(&d);
	return r;
}

/* ---- decompression (extension) ------------------------------------------ */
static uint32_t be24(const uint8_t *p)
{
	return (uint32_t)p[0] << 16 | (uint32_t)p[1] << 8 | p[2];
}

/* model after a frame: the samples (primary pass) or the weighted update
 * of the u16 model (reference cmp.c:304-311, is_unsigned) */
static void next_model(uint16_t *model, const uint16_t *x, size_t n, int is_model_frame, uint32_t rate)
{
	size_t i;

	if (!is_model_frame) {
		memcpy(model, x, 2 * n);
		return;
	}
	for (i = 0; i < n; i++)
		model[i] = (uint16_t)(((uint32_t)model[i] * rate + (uint32_t)x[i] * (16u - rate)) >> 4);
}

static int decompress_file(struct job *j, struct dev *d, int fi)
{
	uint8_t *raw, *out = NULL;
	size_t size, pos, total = 0;
	int owned, r = -1;
	uint16_t *model = NULL;
	size_t model_n = 0;
	void *d_model = NULL;

	if (load_file(j->in[fi], &raw, &size, &owned))
		return -1;
	/* walk the frames: compressed size at bytes 2-4, original size at 5-7 */
	for (pos = 0; pos < size;) {
		uint32_t fs;

		if (size - pos < HDR_MIN || (fs = be24(raw + pos + 2)) < HDR_MIN || fs > size - pos ||
		    be24(raw + pos + 5) % 2u) {
			log_msg(LOG_ERROR, "%s: not a valid AIRSPACE frame at byte %lu", display(j->in[fi]),
				(unsigned long)pos);
			goto out;
		}
		total += be24(raw + pos + 5);
		pos += fs;
	}
	out = xmalloc(total);
	if (dev_open(d))
		goto out;
	if (dev_reserve(&d->sizes, &d->sizes_cap, 64))
		goto out;
	{
		size_t o = 0;

		for (pos = 0; pos < size;) {
			/* a run: one MODEL frame (it needs the frame before it), or
			 * consecutive other frames, decoded as one batch */
			const uint32_t pre0 = raw[pos + 15] >> 4;
			size_t q = pos, nrun = 0, cap = 24, nmax = 1, dstride, i;
			struct cmp_gpu_decode_batch b;
			uint8_t *stage;
			uint16_t *x;
			uint32_t *st, e;

			for (;;) {
				const uint32_t fs = be24(raw + q + 2), n = be24(raw + q + 5) / 2u;
				const size_t c = fs < 24u ? 24u : ((size_t)fs + 7u) & ~(size_t)7u;
				const size_t ncap = c > cap ? c : cap, nn = n > nmax ? n : nmax;

				if (nrun && ((nrun + 1u) * (ncap + 2u * nn + 16u) > BATCH_BYTES || nrun == 65535u))
					break;
				cap = ncap;
				nmax = nn;
				nrun++;
				q += fs;
				if (pre0 == CMP_PREPROCESS_MODEL || q >= size || (raw[q + 15] >> 4) == CMP_PREPROCESS_MODEL)
					break;
			}
			dstride = (2u * nmax + 15u) & ~(size_t)15u; /* 16-byte rows: vector stores */
			if (dev_reserve(&d->src, &d->src_cap, nrun * cap) ||
			    dev_reserve(&d->dst, &d->dst_cap, nrun * dstride) ||
			    dev_reserve(&d->sizes, &d->sizes_cap, 4u * nrun))
				goto out;
			stage = calloc(nrun, cap);
			if (!stage) {
				log_errno("Memory allocation failed");
				goto out;
			}
			for (i = 0, q = pos; i < nrun; i++) {
				const uint32_t fs = be24(raw + q + 2);

				memcpy(stage + i * cap, raw + q, fs);
				q += fs;
			}
			e = hipMemcpy(d->src, stage, nrun * cap, hipMemcpyHostToDevice) == hipSuccess;
			free(stage);
			if (!e)
				goto gpu_fail;
			memset(&b, 0, sizeof(b));
			b.src = d->src;
			b.src_stride = cap;
			b.src_capacity = (uint32_t)cap;
			b.num_frames = (uint32_t)nrun;
			b.dst = d->dst;
			b.dst_stride = dstride;
			b.dst_samples = (uint32_t)nmax;
			b.status = d->sizes;
			if (pre0 == CMP_PREPROCESS_MODEL) {
				const uint32_t n = be24(raw + pos + 5) / 2u;

				if (model_n != n) {
					log_msg(LOG_ERROR, "%s: MODEL frame without a preceding frame of its size",
						display(j->in[fi]));
					goto out;
				}
				if (!d_model && hipMalloc(&d_model, 2u * (size_t)n + 16u) != hipSuccess)
					goto gpu_fail;
				if (hipMemcpy(d_model, model, 2u * (size_t)n, hipMemcpyHostToDevice) != hipSuccess)
					goto gpu_fail;
				b.model = d_model;
				b.model_stride = 2u * (uint64_t)n + 16u;
			}
			e = cmp_gpu_decompress(d->eng, &b);
			if (!cmp_is_error(e))
				e = cmp_gpu_synchronize(d->eng);
			if (cmp_is_error(e)) {
				log_cmp(e, "Decompression failed for %s", display(j->in[fi]));
				goto out;
			}
			st = xmalloc(4u * nrun);
			x = xmalloc(nrun * dstride);
			if (hipMemcpy(st, d->sizes, 4u * nrun, hipMemcpyDeviceToHost) != hipSuccess ||
			    hipMemcpy(x, d->dst, nrun * dstride, hipMemcpyDeviceToHost) != hipSuccess) {
				free(st);
				free(x);
				goto gpu_fail;
			}
			for (i = 0; i < nrun; i++) {
				const uint32_t n = be24(raw + pos + 5) / 2u;
				const uint16_t *xi = (const uint16_t *)((const uint8_t *)x + i * dstride);
				uint32_t k;

				if (cmp_is_error(st[i]) || st[i] != n) {
					log_cmp(cmp_is_error(st[i]) ? st[i] : (uint32_t) - (int32_t)CMP_ERR_INT_BITSTREAM,
						"Decompression failed for %s", display(j->in[fi]));
					free(st);
					free(x);
					goto out;
				}
				for (k = 0; k < n; k++) {
					out[o + 2u * k] = (uint8_t)(xi[k] >> 8);
					out[o + 2u * k + 1u] = (uint8_t)xi[k];
				}
				o += 2u * (size_t)n;
				if (i + 1u == nrun) { /* the model the next frame may need */
					if (model_n != n) {
						free(model);
						model = xmalloc(2u * (size_t)n + 2u);
						model_n = n;
						if (d_model) {
							hipFree(d_model);
							d_model = NULL;
						}
					}
					next_model(model, xi, n, pre0 == CMP_PREPROCESS_MODEL, raw[pos + 16]);
				}
				pos += be24(raw + pos + 2);
			}
			free(st);
			free(x);
		}
	}
	{
		const char *name = j->in[fi];
		size_t ln = strlen(name);
		char *oname = NULL;
		const char *target = j->out_name;

		if (!target) {
			if (ln <= strlen(AIR_EXT) || strcmp(name + ln - strlen(AIR_EXT), AIR_EXT) != 0) {
				log_msg(LOG_ERROR, "%s: unknown suffix (expected %s)", display(name), AIR_EXT);
				goto out;
			}
			oname = xmalloc(ln);
			memcpy(oname, name, ln - strlen(AIR_EXT));
			oname[ln - strlen(AIR_EXT)] = '\0';
			target = oname;
		}
		r = save_file(target, out, total);
		if (!r) {
			log_ratio(LOG_DEBUG, display(name), size, display(target), total);
			j->sum_in += size;
			j->sum_out += total;
			free(j->last_out);
			j->last_out = strdup(display(target));
		}
		free(oname);
	}
	goto out;
gpu_fail:
	log_msg(LOG_ERROR, "GPU copy failed");
out:
	if (d_model)
		hipFree(d_model);
	free(model);
	free(out);
	if (owned)
		free(raw);
	return r;
}

static int decompress_files(struct job *j)
{
	struct dev d;
	int i, r = 0;

	memset(&d, 0, sizeof(d));
	for (i = 0; i < j->n_in && !r; i++)
		r = decompress_file(j, &d, i);
	dev_close(&d);
	if (!r)
		log_summary("decompressed", j->in, j->n_in, j->sum_in, j->last_out ? j->last_out : "", j->sum_out);
	return r;
}

/* ---- command line (reference airspacecli.c:290-433) ------------------------ */
static void usage(FILE *f, const char *prog)
{
	fprintf(f, "Usage: %s [OPTIONS...] [FILE... | -] [-o OUTPUT]\n", prog);
	fprintf(f, "(De)compress AIRS science data FILE(s).\n\n");
	fprintf(f, "With no FILE, or when FILE is -, read standard input.\n");
	fprintf(f, "\nOptions:\n");
	fprintf(f, "  -c, --compress    Compress input files\n");
	fprintf(f, "  -d, --decompress  Decompress input files (default)\n");
	fprintf(f, "  --params=K=V,...  Compression parameters (see DESIGN.md)\n");
	fprintf(f, "  -o OUTPUT         Write output to OUTPUT\n");
	fprintf(f, "  --stdout          Write output to standard output\n");
	fprintf(f, "  -q, --quiet       Decrease verbosity\n");
	fprintf(f, "  -v, --verbose     Increase verbosity\n");
	fprintf(f, "  --[no-]color      Print color codes in output\n");
	fprintf(f, "  -V, --version     Display version\n");
	fprintf(f, "  -h, --help        Display this help\n");
	fprintf(f, "\nExamples:\n");
	fprintf(f, "# Compressing file1 and file2 to file1.air and file2.air\n");
	fprintf(f, "airspace -c file1 file2\n");
	fprintf(f, "# Decompressing file1.air back to file1\n");
	fprintf(f, "airspace file1.air\n");
}

static void version(void)
{
	if (log_level() < LOG_DEFAULT_LEVEL)
		printf("%s\n", CMP_VERSION_STRING);
	else
		printf("*** %s (%d-bit) v%s, MI355X build ***\n", PROGRAM_NAME, (int)(sizeof(size_t) * 8),
		       CMP_VERSION_STRING);
}

int main(int argc, char **argv)
{
	enum { OPT_STDOUT = CHAR_MAX + 1, OPT_COLOR, OPT_NO_COLOR, OPT_DBG_STDIN, OPT_DBG_STDOUT };
	static const struct option longs[] = {
		{ "compress", no_argument, NULL, 'c' },
		{ "decompress", no_argument, NULL, 'd' },
		{ "params", required_argument, NULL, 'p' },
		{ "stdout", no_argument, NULL, OPT_STDOUT },
		{ "verbose", no_argument, NULL, 'v' },
		{ "quiet", no_argument, NULL, 'q' },
		{ "color", no_argument, NULL, OPT_COLOR },
		{ "no-color", no_argument, NULL, OPT_NO_COLOR },
		{ "version", no_argument, NULL, 'V' },
		{ "help", no_argument, NULL, 'h' },
		{ "debug-stdin-is-consol", no_argument, NULL, OPT_DBG_STDIN },
		{ "debug-stdout-is-consol", no_argument, NULL, OPT_DBG_STDOUT },
		{ NULL, 0, NULL, 0 },
	};
	struct cmp_params par;
	struct job j;
	const char **files;
	int compress = 0, ch, i, from_stdin = 0, rc = EXIT_FAILURE;
	const char *out = NULL;

	memset(&par, 0, sizeof(par));
	memset(&j, 0, sizeof(j));
	log_color_from_env();
	while ((ch = getopt_long(argc, argv, "Vvqhcdo:", longs, NULL)) != -1) {
		switch (ch) {
		case 'c':
			compress = 1;
			break;
		case 'd':
			compress = 0;
			break;
		case 'p':
			if (cmp_params_parse(optarg, &par) != CMP_PARSE_OK) {
				log_msg(LOG_ERROR, "Incorrect parameter option: %s", argv[optind - 1]);
				return EXIT_FAILURE;
			}
			break;
		case 'o':
			out = optarg;
			break;
		case OPT_STDOUT:
			out = STDOUT_NAME;
			break;
		case 'v':
			log_more();
			break;
		case 'q':
			log_less();
			break;
		case OPT_COLOR:
			log_set_color(1);
			break;
		case OPT_NO_COLOR:
			log_set_color(0);
			break;
		case 'V':
			version();
			return EXIT_SUCCESS;
		case 'h':
			usage(stdout, argv[0]);
			return EXIT_SUCCESS;
		case OPT_DBG_STDIN:
			g_stdin_console = 1;
			break;
		case OPT_DBG_STDOUT:
			g_stdout_console = 1;
			break;
		default:
			usage(stderr, argv[0]);
			return EXIT_FAILURE;
		}
	}
	argv += optind;
	argc -= optind;
	log_plain(LOG_DEBUG, "*** %s (%d-bit) v%s, MI355X build ***\n", PROGRAM_NAME, (int)(sizeof(size_t) * 8),
		  CMP_VERSION_STRING);

	/* the input list: stdin when empty, "-" means stdin */
	j.n_in = argc ? argc : 1;
	files = xmalloc(sizeof(*files) * (size_t)j.n_in);
	for (i = 0; i < j.n_in; i++) {
		const int is_stdin = !argc || strcmp(argv[i], "-") == 0;

		files[i] = is_stdin ? STDIN_NAME : argv[i];
		from_stdin |= is_stdin;
	}
	j.in = files;
	if (from_stdin) {
		if (is_console(stdin)) {
			log_msg(LOG_ERROR, "stdin is a terminal, aborting");
			goto end;
		}
		log_msg(LOG_DEBUG, "Using stdin as an input");
		if (!out) {
			if (is_console(stdout)) {
				log_msg(LOG_ERROR, "stdout is a terminal, aborting");
				goto end;
			}
			log_msg(LOG_DEBUG, "Using stdout as output");
			out = STDOUT_NAME;
		}
	}
	/* no summary by default when the data goes to stdout */
	if (out && strcmp(out, STDOUT_NAME) == 0 && log_level() == LOG_DEFAULT_LEVEL)
		log_less();
	j.out_name = out;
	if (compress)
		rc = compress_files(&j, &par) ? EXIT_FAILURE : EXIT_SUCCESS;
	else
		rc = decompress_files(&j) ? EXIT_FAILURE : EXIT_SUCCESS;
end:
	free(j.last_out);
	free(files);
	return rc;
}
