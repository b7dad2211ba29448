/* log.c -- see log.h */
#include "log.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "cmp.h"
#include "cmp_errors.h"

static int g_level = LOG_DEFAULT_LEVEL;
static int g_color;

void log_set_level(int level)
{
	g_level = level;
}

int log_level(void)
{
	return g_level;
}

void log_more(void)
{
	if (g_level < LOG_TRACE)
		g_level++;
}

void log_less(void)
{
	if (g_level > LOG_QUIET)
		g_level--;
}

void log_set_color(int on)
{
	g_color = on;
}

void log_color_from_env(void)
{
	const char *no = getenv("NO_COLOR"), *force = getenv("CLICOLOR_FORCE"), *cli = getenv("CLICOLOR");

	if (no && no[0])
		g_color = 0;
	else if (force && force[0])
		g_color = 1;
	else if (cli && cli[0] == '0')
		g_color = 0;
	else
		g_color = isatty(fileno(stderr));
}

static void prefix(int level)
{
	static const char *const kind[] = { "", "error", "warning", "info", "debug", "trace" };
	static const char *const col[] = { "", "\033[1;31m", "\033[1;33m", "\033[1;33m", "\033[1;30m", "\033[1;30m" };

	fprintf(stderr, "airspace: %s%s%s: ", g_color ? col[level] : "", kind[level], g_color ? "\033[0m" : "");
}

/* info messages go out at warning level, as in the reference (log.h LOG_INFO) */
static int gate(int level)
{
	return level == LOG_INFO ? LOG_WARNING : level;
}

void log_msg(int level, const char *fmt, ...)
{
	va_list ap;

	if (g_level < gate(level))
		return;
	prefix(level);
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
	fputc('\n', stderr);
}

void log_errno(const char *fmt, ...)
{
	va_list ap;
	int e = errno;

	if (g_level < LOG_ERROR)
		return;
	prefix(LOG_ERROR);
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
	fprintf(stderr, ": %s (os error: %d)\n", strerror(e), e);
}

void log_cmp(unsigned int code, const char *fmt, ...)
{
	va_list ap;

	if (g_level < LOG_ERROR)
		return;
	prefix(LOG_ERROR);
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
	fprintf(stderr, ": %s (compression error: %d)\n", cmp_get_error_message(code), (int)cmp_get_error_code(code));
}

void log_plain(int level, const char *fmt, ...)
{
	va_list ap;

	if (g_level < level)
		return;
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
}
