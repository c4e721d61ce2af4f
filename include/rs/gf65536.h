/*
 * rs/gf65536.h -- GF(2^16) helpers of the drop-in API.
 *
 * Field GF(2)[x]/(x^16 + x^5 + x^3 + x^2 + 1), primitive element alpha = x (reference
 * include/rs/gf65536.h:21-27). GF_t has the reference's full member list and layout (:49-78), so
 * sizeof(GF_t) and the table members read the same. Scalar entry points match reference :85-137;
 * the symbol-wide operations gf_add / gf_mul / gf_madd (:146-167) keep their signatures and
 * semantics (little-endian 16-bit words, zero-skip, coefficient 0 / 1 shortcuts) and run on the GPU:
 * the symbols are staged through pinned memory, coded by a HIP kernel and copied back.
 */
#ifndef RS_AMD_GF65536_H
#define RS_AMD_GF65536_H

#include <stddef.h>
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

/* Tables (reference :49-78): pow_table[i] = alpha^i for i < 2N-1, log_table[alpha^i] = i
 * (log_table[0] unused), the normal bases of GF(2^m) for m = 1, 2, 4, 8, 16 (m - 1 elements before
 * the first of subfield m), and normal_repr_by_subfield[m][d] = bits of alpha^d in the normal basis of
 * GF(2^m) (0 when alpha^d is not in GF(2^m)); entries m = 1, 2, 4, 8, 16 point into
 * _normal_repr_by_subfield_memory, the others are NULL. */
typedef struct {
    element_t pow_table[(N << 1) - 1];
    uint16_t log_table[GF_FIELD_SIZE];
    element_t normal_bases[GF_NORMAL_BASES_ELEMENTS];
    uint16_t* normal_repr_by_subfield[CC_MAX_COSET_SIZE + 1];
    uint16_t _normal_repr_by_subfield_memory[CC_COSET_SIZES_CNT * N];
} GF_t;

GF_t* gf_create(void);                                          /* reference :85 */
void gf_destroy(GF_t* gf);                                      /* reference :92 */
element_t gf_get_normal_basis_element(GF_t* gf, uint8_t m, uint8_t i); /* reference :103 */
uint16_t gf_get_normal_repr(GF_t* gf, uint8_t m, uint16_t d);   /* reference :113 */
element_t gf_mul_ee(GF_t* gf, element_t a, element_t b);        /* reference :125 */
element_t gf_div_ee(GF_t* gf, element_t a, element_t b);        /* reference :137 (b != 0) */

/* Symbol-wide operations over symbol_size / 2 little-endian words (symbol_size even; the reference
 * asserts it). Host memory in and out; computed on the GPU (no CPU path). */
void gf_add(void* a, const void* b, size_t symbol_size);                               /* reference :146, a ^= b */
void gf_mul(GF_t* gf, void* a, element_t coef, size_t symbol_size);                   /* reference :156, a = coef * a */
void gf_madd(GF_t* gf, void* a, element_t coef, const void* b, size_t symbol_size);   /* reference :167, a ^= coef * b */

#ifdef __cplusplus
}
#endif
#endif
