/*
 * rs_oracle.h -- CPU restatement of the reference Reed-Solomon path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the checker, never the product. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it. The product path (reed-solomon_amd/, librs_amd.so)
 * never links or calls anything here.
 *
 * It restates the algorithm of /root/reference/src/rs (Vergil645/reed-solomon @ v2):
 *   - GF(2^16) over x^16+x^5+x^3+x^2+1 (reference include/rs/gf65536.h:27, src/rs/gf65536.c:59-111)
 *   - 2-cyclotomic coset selection of code positions (src/rs/cyclotomic_coset.c:154-230)
 *   - syndromes by the cyclotomic FFT with normal-basis XOR accumulators (src/rs/fft.c:39-100)
 *   - locator / evaluator / Forney (src/rs/reed_solomon.c:83-336)
 *   - encode (src/rs/reed_solomon.c:338-441) and restore (src/rs/reed_solomon.c:443-559)
 *
 * Parity pinning: checked against golden vectors produced by the compiled reference itself
 * (tests/golden/, generator oracle/gen_golden.c) and against the reference's own KATs.
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_N 65535u
#define ORC_ERR_CANNOT_RESTORE 100

/* Builds the process-wide tables once (thread-safe). Returns 0. */
int orc_init(void);

uint16_t orc_mul(uint16_t a, uint16_t b);
uint16_t orc_div(uint16_t a, uint16_t b);
uint16_t orc_pow(uint32_t e); /* alpha^(e mod N) */
uint16_t orc_log(uint16_t a);
uint8_t orc_coset_size(uint16_t leader);
uint16_t orc_normal_repr(uint8_t m, uint16_t d);

/* Coset selection (restates cc_estimate_cosets_cnt + cc_select_cosets). Arrays must hold
 * orc_cosets_upper(k) / orc_cosets_upper(r) entries. */
uint16_t orc_cosets_upper(uint16_t n);
void orc_select_cosets(uint16_t k, uint16_t r, uint16_t* inf_leader, uint8_t* inf_size, uint16_t* n_inf,
                       uint16_t* rep_leader, uint8_t* rep_size, uint16_t* n_rep);
/* positions[0..k) = information positions, positions[k..k+r) = repair positions. */
void orc_positions(uint16_t k, uint16_t r, uint16_t* positions);

/* Encode: info[k] -> rep[r], symbols of S bytes (S even). Returns 0, or 1 on allocation failure. */
int orc_encode(uint16_t k, uint16_t r, size_t S, const uint8_t* const* info, uint8_t* const* rep);
/* Restore erased information symbols in place. rcv[k+r], erased slots must be zero.
 * Returns 0, 1 on allocation failure, ORC_ERR_CANNOT_RESTORE if t > r. */
int orc_decode(uint16_t k, uint16_t r, size_t S, uint8_t* const* rcv, const bool* erased, uint16_t t);

/* Contiguous-stripe conveniences: stripe = [k+r][S] bytes. */
int orc_encode_stripe(uint16_t k, uint16_t r, size_t S, uint8_t* stripe);
int orc_decode_stripe(uint16_t k, uint16_t r, size_t S, uint8_t* stripe, const bool* erased, uint16_t t);
/* Encode/decode n_stripes contiguous stripes on n_threads pthreads (CPU baseline). Returns 0 on success. */
int orc_encode_many(uint16_t k, uint16_t r, size_t S, uint8_t* stripes, size_t n_stripes, int n_threads);
int orc_decode_many(uint16_t k, uint16_t r, size_t S, uint8_t* stripes, size_t n_stripes, const bool* erased,
                    uint16_t t, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
