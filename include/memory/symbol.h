/*
 * memory/symbol.h -- symbol type of the drop-in API (librs_amd.so).
 *
 * Replaces reference include/memory/symbol.h:20-58 with the same layout and entry points:
 * a symbol is a caller-owned byte array of `symbol_size` bytes, read as little-endian uint16
 * GF(2^16) words by the codec.
 */
#ifndef RS_AMD_MEMORY_SYMBOL_H
#define RS_AMD_MEMORY_SYMBOL_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference symbol.h:20-25 */
typedef struct {
    uint8_t* data;
} symbol_t;

/* reference symbol.h:33 -- zero-filled symbol, NULL on allocation failure */
symbol_t* symbol_create(size_t symbol_size);
/* reference symbol.h:40 */
void symbol_destroy(symbol_t* s);
/* reference symbol.h:50 -- false if either is NULL */
bool symbol_eq(const symbol_t* a, const symbol_t* b, size_t symbol_size);
/* reference symbol.h:58 -- "[b0, b1, ...]" to stdout */
void symbol_printf(const symbol_t* s, size_t symbol_size);

#ifdef __cplusplus
}
#endif
#endif
