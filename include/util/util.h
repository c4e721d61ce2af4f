/*
 * util/util.h -- the reference's utility macro (reference include/util/util.h:22), kept so code
 * that includes it against this library compiles unchanged.
 */
#ifndef RS_AMD_UTIL_UTIL_H
#define RS_AMD_UTIL_UTIL_H

/* Minimum of two values (arguments are evaluated twice, as in the reference). */
#define MIN(_x, _y) (((_x) < (_y)) ? (_x) : (_y))

#endif
