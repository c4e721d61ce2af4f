/*
 * rs/fft.h -- discrete Fourier transforms over symbol sequences (reference include/rs/fft.h:29-65).
 *
 * Same signatures and results as the reference, computed on the GPU: each call forms the transform's
 * GF(2^16) matrix on the host (the DFT coefficients alpha^(position * j); for the cyclotomic partial
 * transform the reference's normal-basis combination, src/rs/fft.c:142-169, entry by entry) and
 * applies it to the sequence with the engine's matrix kernels, staging the symbols through pinned
 * memory. The cyclotomic variants equal the plain ones on every input (the cyclotomic FFT is an
 * evaluation order, not a different map); they keep their return codes. Host memory in and out.
 * Parity holds where the reference's int products (positions[i] * j, s * positions[i], s * i,
 * i * j; fft.c:33,69,120,152) do not overflow, i.e. below 2^31.
 */
#ifndef RS_AMD_FFT_H
#define RS_AMD_FFT_H

#include <stdint.h>

#include <memory/seq.h>
#include <memory/symbol.h>

#include "gf65536.h"

#ifdef __cplusplus
extern "C" {
#endif

/* res[j] = sum_i f[i] * alpha^(positions[i] * j), j < res->length (reference :29, fft.c:18-37). */
void fft_transform(GF_t* gf, const symbol_seq_t* f, const uint16_t* positions, symbol_seq_t* res);
/* Same components by the cyclotomic FFT in the reference (fft.c:39-100). Returns 0, 1 on allocation
 * failure, RS_ERR_INVALID (2) on bad arguments, RS_ERR_DEVICE (3) on a HIP error. */
int fft_transform_cycl(GF_t* gf, const symbol_seq_t* f, const uint16_t* positions, symbol_seq_t* res);
/* res[idx] = f(alpha^-components[idx]) = sum_i f[i] * alpha^(i * (N - components[idx])) (reference :53,
 * fft.c:103-124). */
void fft_partial_transform(GF_t* gf, const symbol_seq_t* f, const uint16_t* components, symbol_seq_t* res);
/* res = f evaluated at alpha^-(leader * 2^j), j < size, coset by coset (reference :65, fft.c:126-177);
 * res->length must equal the sum of the coset sizes. Return codes as fft_transform_cycl. */
int fft_partial_transform_cycl(GF_t* gf, const symbol_seq_t* f, const coset_t* cosets, uint16_t cosets_cnt,
                               symbol_seq_t* res);

#ifdef __cplusplus
}
#endif
#endif
