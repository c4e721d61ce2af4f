/*
 * memory/seq.h -- symbol sequences of the drop-in API (librs_amd.so).
 *
 * Replaces reference include/memory/seq.h:21-68 with the same layout and entry points.
 * Sequences hold an array of individually allocated symbols; views are built by pointer
 * arithmetic on `symbols` (reference src/example.c:87-95).
 */
#ifndef RS_AMD_MEMORY_SEQ_H
#define RS_AMD_MEMORY_SEQ_H

#include <stdbool.h>
#include <stddef.h>

#include "symbol.h"

#ifdef __cplusplus
extern "C" {
#endif

/* reference seq.h:21-36 */
typedef struct {
    size_t length;
    size_t symbol_size;
    symbol_t** symbols;
} symbol_seq_t;

/* reference seq.h:45 -- `length` zero-filled symbols, NULL on allocation failure.
 * With a GPU present the symbols' data are page-locked, one block per sequence at a stride of
 * symbol_size rounded up to 16 bytes (own block from 1 MiB, a shared slab below), so
 * rs_generate_repair_symbols / rs_restore_symbols work on them in place (zero-copy kernels or DMA).
 * Free them only through symbol_destroy / seq_destroy (as the reference's callers do). The
 * environment variable RS_AMD_PINNED_SEQ=0 restores one heap allocation per symbol. */
symbol_seq_t* seq_create(size_t length, size_t symbol_size);
/* reference seq.h:52 */
void seq_destroy(symbol_seq_t* seq);
/* reference seq.h:61 */
bool seq_eq(const symbol_seq_t* a, const symbol_seq_t* b);
/* reference seq.h:68 */
void seq_printf(const symbol_seq_t* seq);

#ifdef __cplusplus
}
#endif
#endif
