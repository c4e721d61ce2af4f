/*
 * rs/gf65536.h -- GF(2^16) scalar helpers of the drop-in API (host side).
 *
 * Field GF(2)[x]/(x^16 + x^5 + x^3 + x^2 + 1), primitive element alpha = x (reference
 * include/rs/gf65536.h:21-27). Scalar entry points match reference :85-137. The reference's
 * symbol-wide loops (gf_add/gf_mul/gf_madd, :146-167) and its DFT helpers (rs/fft.h) are internal
 * stages of the CPU algorithm that the GPU engine replaces wholesale; they are not exported.
 */
#ifndef RS_AMD_GF65536_H
#define RS_AMD_GF65536_H

#include <stdint.h>

#include "cyclotomic_coset.h"
#include "prelude.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GF_FIELD_SIZE 65536
#define GF_PRIMITIVE_POLY 65581
#define GF_NORMAL_BASES_ELEMENTS 31

typedef uint16_t element_t;
typedef uint32_t poly_t;

/* Tables: pow_table[i] = alpha^i for i < 2N-1, log_table[alpha^i] = i (log_table[0] unused);
 * the first two members keep the reference's names and layout (reference :49-60). */
typedef struct {
    element_t pow_table[(N << 1) - 1];
    uint16_t log_table[GF_FIELD_SIZE];
    element_t normal_bases[GF_NORMAL_BASES_ELEMENTS];
} GF_t;

GF_t* gf_create(void);                                          /* reference :85 */
void gf_destroy(GF_t* gf);                                      /* reference :92 */
element_t gf_get_normal_basis_element(GF_t* gf, uint8_t m, uint8_t i); /* reference :103 */
uint16_t gf_get_normal_repr(GF_t* gf, uint8_t m, uint16_t d);   /* reference :113 */
element_t gf_mul_ee(GF_t* gf, element_t a, element_t b);        /* reference :125 */
element_t gf_div_ee(GF_t* gf, element_t a, element_t b);        /* reference :137 (b != 0) */

#ifdef __cplusplus
}
#endif
#endif
