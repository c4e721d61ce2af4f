/*
 * rs/cyclotomic_coset.h -- 2-cyclotomic cosets modulo N = 65535 (host-side helpers).
 *
 * Same entry points and selection rule as reference include/rs/cyclotomic_coset.h:18-172; the
 * code positions they produce define the code, so the GPU engine derives its coding matrices from
 * exactly these positions.
 */
#ifndef RS_AMD_CYCLOTOMIC_COSET_H
#define RS_AMD_CYCLOTOMIC_COSET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CC_COSET_SIZES_CNT 5      /* sizes 1, 2, 4, 8, 16 */
#define CC_COSETS_CNT 4115
#define CC_MAX_COSET_SIZE 16
#define CC_LEADERS_1_CNT 1
#define CC_LEADERS_2_CNT 1
#define CC_LEADERS_4_CNT 3
#define CC_LEADERS_8_CNT 30
#define CC_LEADERS_16_CNT 4080
#define CC_THRESHOLD_1 0          /* a size-2^i coset is taken while the remainder exceeds these */
#define CC_THRESHOLD_2 1
#define CC_THRESHOLD_4 3
#define CC_THRESHOLD_8 15
#define CC_THRESHOLD_16 255

/* s -> 2s mod N (reference cyclotomic_coset.h:87) */
#define NEXT_COSET_ELEMENT(_s) ((uint16_t)(((uint32_t)(_s) << 1) % 65535))

/* reference cyclotomic_coset.h:92-95 */
typedef struct {
    uint16_t leader;
    uint8_t size;
} coset_t;

/* Leaders grouped by size (ascending). Layout compatible with reference :100-113. */
typedef struct {
    uint16_t* leaders[CC_COSET_SIZES_CNT];
    uint16_t _leaders_memory[CC_COSETS_CNT];
} CC_t;

CC_t* cc_create(void);                      /* reference :120 */
void cc_destroy(CC_t* cc);                  /* reference :127 */
uint8_t cc_get_coset_size(uint16_t leader); /* reference :135 */
/* reference :145 -- upper bounds for the coset arrays of cc_select_cosets */
void cc_estimate_cosets_cnt(uint16_t k, uint16_t r, uint16_t* inf_max_cnt, uint16_t* rep_max_cnt);
/* reference :161 */
void cc_select_cosets(CC_t* cc, uint16_t k, uint16_t r, coset_t* inf_cosets, uint16_t inf_max_cnt,
                      uint16_t* inf_cosets_cnt, coset_t* rep_cosets, uint16_t rep_max_cnt, uint16_t* rep_cosets_cnt);
/* reference :172 */
void cc_cosets_to_positions(const coset_t* cosets, uint16_t cosets_cnt, uint16_t* positions, uint16_t positions_cnt);

#ifdef __cplusplus
}
#endif
#endif
