/*
 * rs/reed_solomon.h -- drop-in Reed-Solomon codec over GF(2^16), executed on MI355X (librs_amd.so).
 *
 * Same entry points, argument meaning and return codes as reference include/rs/reed_solomon.h:29-74.
 * Host buffers (symbol_seq_t) are gathered into pinned staging, coded by HIP kernels on the GPU
 * and scattered back; results are bit-identical to the reference CPU path.
 *
 * Threading: a context may be shared by threads; calls on one context are serialised internally.
 * Without a usable GPU rs_create() prints the HIP error to stderr and returns NULL: there is no
 * CPU fallback.
 */
#ifndef RS_AMD_REED_SOLOMON_H
#define RS_AMD_REED_SOLOMON_H

#include <stdbool.h>
#include <stdint.h>

#include "cyclotomic_coset.h"
#include "gf65536.h"
#include <memory/seq.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_COSET_LOCATOR_MAX_LEN (CC_MAX_COSET_SIZE + 1)

/* reference :29 */
#define RS_ERR_CANNOT_RESTORE 100
/* additions of this implementation (the reference asserts these preconditions instead) */
#define RS_ERR_INVALID 2   /* k + r > N, size mismatch, erasure count != t (rsg_*: also odd symbol sizes) */
#define RS_ERR_DEVICE 3    /* HIP runtime / kernel error */

/* reference :34-37; the first two members keep the reference's layout */
typedef struct {
    GF_t* gf;
    CC_t* cc;
    void* impl; /* device state of this implementation */
} RS_t;

/* reference :44 -- NULL on failure (allocation, or no usable GPU) */
RS_t* rs_create(void);
/* reference :51 */
void rs_destroy(RS_t* rs);
/* reference :61 -- 0 on success, 1 on allocation failure, RS_ERR_INVALID / RS_ERR_DEVICE. An odd symbol size
 * behaves as the reference's Release build: the even prefix is coded and each repair symbol's last byte
 * is 0 (restores likewise: restored symbols end in a zero byte). */
int rs_generate_repair_symbols(RS_t* rs, const symbol_seq_t* inf_symbols, symbol_seq_t* rep_symbols);
/* reference :74 -- erased slots must be zero on entry; restores erased information symbols in place
 * (erased repair slots are left untouched, as in the reference). 0, 1, RS_ERR_CANNOT_RESTORE (t > r),
 * RS_ERR_INVALID, RS_ERR_DEVICE. Bit-identical to the reference under its zeroed-erased-slots
 * contract; erased slots are not read, so non-zero garbage there still yields the true symbols here,
 * where the reference would return c XOR garbage-dependent values. */
int rs_restore_symbols(RS_t* rs, uint16_t k, uint16_t r, symbol_seq_t* rcv_symbols, const bool* is_erased,
                       uint16_t t);

#ifdef __cplusplus
}
#endif
#endif
