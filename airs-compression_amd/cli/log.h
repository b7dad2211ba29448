/*
 * log.h -- leveled, optionally coloured messages of the airspace CLI on
 * stderr.  Levels and message shapes follow the reference's programs/log.h
 * (quiet < error < warning < info < debug < trace; "airspace: error: ..."),
 * colour set up from NO_COLOR / CLICOLOR_FORCE / CLICOLOR and whether stderr
 * is a terminal (programs/log.c:27-56).
 */
#ifndef AIRS_CLI_LOG_H
#define AIRS_CLI_LOG_H

#include <stdarg.h>
#include <stdio.h>

enum log_level { LOG_QUIET = 0, LOG_ERROR, LOG_WARNING, LOG_INFO, LOG_DEBUG, LOG_TRACE };
#define LOG_DEFAULT_LEVEL LOG_INFO

void log_set_level(int level);
int log_level(void);
void log_more(void);
void log_less(void);
void log_color_from_env(void);
void log_set_color(int on);

/* "airspace: <kind>: <message>\n" on stderr if the level is enabled */
void log_msg(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
/* the same, followed by ": <strerror(errno)> (os error: N)" */
void log_errno(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
/* the same, followed by ": <library message> (compression error: N)" */
void log_cmp(unsigned int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
/* unprefixed text on stderr if the level is enabled */
void log_plain(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#endif /* AIRS_CLI_LOG_H */
