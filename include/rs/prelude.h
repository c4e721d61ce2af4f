/*
 * rs/prelude.h -- code-length constants (reference include/rs/prelude.h:16,21).
 */
#ifndef RS_AMD_PRELUDE_H
#define RS_AMD_PRELUDE_H

/* Reed-Solomon code length 2^16 - 1: k + r must not exceed it. */
#define N 65535

/* Symbol size used by the reference's tools (run_enc_dec.c:209, compare_codes.c:242). */
#define SYMBOL_SIZE 1300

#endif
