#define _POSIX_C_SOURCE 199309L
/* Drop-in per-call rate through the reference API exactly as a reference caller uses it
 * (include/rs/reed_solomon.h, include/memory/seq.h): one stripe per call, host symbol_t buffers.
 * usage: bench_dropin [k r S calls]   (defaults: C3 shape 128 32 65536, 32 calls)
 * Prints one JSON line: encode / decode GB/s of algorithmic bytes ((k+r)S and (k+t)S per call).
 * build: gcc -O2 -std=c11 -Iinclude scripts/bench_dropin.c -Lreed-solomon_amd -lrs_amd \
 *            -Wl,-rpath,'$ORIGIN/../reed-solomon_amd' -o scripts/bench_dropin */
#include <memory/seq.h>
#include <rs/reed_solomon.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
    int k = argc > 1 ? atoi(argv[1]) : 128, r = argc > 2 ? atoi(argv[2]) : 32;
    size_t S = argc > 3 ? (size_t)atol(argv[3]) : 65536;
    int calls = argc > 4 ? atoi(argv[4]) : 32;
    RS_t* rs = rs_create();
    if (!rs) return 2;
    symbol_seq_t** st = malloc(sizeof(*st) * calls);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int c = 0; c < calls; ++c) {
        st[c] = seq_create(k + r, S);
        for (int i = 0; i < k; ++i)
            for (size_t b = 0; b < S; ++b) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                st[c]->symbols[i]->data[b] = (uint8_t)x;
            }
    }
    bool* er = calloc(k + r, 1);
    int t = 0;
    for (int i = 0; i < r; ++i) er[i * (k / r)] = true, ++t;  /* bench pattern: r information erasures */
    symbol_seq_t inf = {k, S, st[0]->symbols}, rep = {r, S, st[0]->symbols + k};
    for (int w = 0; w < 2; ++w)
        if (rs_generate_repair_symbols(rs, &inf, &rep)) return 3;
    double t0 = now();
    for (int c = 0; c < calls; ++c) {
        symbol_seq_t a = {k, S, st[c]->symbols}, b = {r, S, st[c]->symbols + k};
        if (rs_generate_repair_symbols(rs, &a, &b)) return 3;
    }
    double te = now() - t0;
    /* keep a copy of the information symbols of every stripe, erase, restore */
    uint8_t* keep = malloc((size_t)calls * k * S);
    for (int c = 0; c < calls; ++c)
        for (int i = 0; i < k; ++i) memcpy(keep + ((size_t)c * k + i) * S, st[c]->symbols[i]->data, S);
    for (int w = 0; w < 10; ++w) { /* warm: plan, then its specialised kernel (a decode plan is specialised at its 3rd call, dec_jit_uses) */
        for (int i = 0; i < k + r; ++i)
            if (er[i]) memset(st[0]->symbols[i]->data, 0, S);
        if (rs_restore_symbols(rs, k, r, st[0], er, t)) return 4;
    }
    for (int c = 0; c < calls; ++c)
        for (int i = 0; i < k + r; ++i)
            if (er[i]) memset(st[c]->symbols[i]->data, 0, S);
    t0 = now();
    for (int c = 0; c < calls; ++c)
        if (rs_restore_symbols(rs, k, r, st[c], er, t)) return 4;
    double td = now() - t0;
    int bad = 0;
    for (int c = 0; c < calls; ++c)
        for (int i = 0; i < k; ++i) bad |= memcmp(keep + ((size_t)c * k + i) * S, st[c]->symbols[i]->data, S) != 0;
    /* a different pattern every call (r erasures anywhere, as stripes lose different symbols): each
     * call builds its decode plan; erased repair slots are zeroed and stay so (only info is restored) */
    bool* ers = calloc((size_t)calls * (k + r), 1);
    int* perm = malloc(sizeof(int) * (k + r));
    double alg_new = 0;
    for (int c = 0; c < calls; ++c) {
        for (int i = 0; i < k + r; ++i) perm[i] = i;
        for (int i = 0; i < r; ++i) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            int j = i + (int)(x % (uint64_t)(k + r - i)), tmp = perm[i];
            perm[i] = perm[j], perm[j] = tmp;
            ers[(size_t)c * (k + r) + perm[i]] = true;
        }
        int ti = 0;
        for (int i = 0; i < k; ++i) ti += ers[(size_t)c * (k + r) + i];
        alg_new += (double)(k + ti) * S;  /* survivors (k) read + erased information written */
        for (int i = 0; i < k + r; ++i)
            if (ers[(size_t)c * (k + r) + i]) memset(st[c]->symbols[i]->data, 0, S);
    }
    t0 = now();
    for (int c = 0; c < calls; ++c)
        if (rs_restore_symbols(rs, k, r, st[c], ers + (size_t)c * (k + r), r)) return 4;
    double tn = now() - t0;
    for (int c = 0; c < calls; ++c)
        for (int i = 0; i < k; ++i) bad |= memcmp(keep + ((size_t)c * k + i) * S, st[c]->symbols[i]->data, S) != 0;
    printf("{\"k\": %d, \"r\": %d, \"S\": %zu, \"calls\": %d, \"dropin_encode_GBps\": %.2f, \"dropin_decode_GBps\": %.2f, "
           "\"encode_ms_per_call\": %.3f, \"decode_ms_per_call\": %.3f, \"decode_new_pattern_ms_per_call\": %.3f, "
           "\"decode_new_pattern_GBps\": %.2f, \"roundtrip\": \"%s\"}\n",
           k, r, S, calls, (double)calls * (k + r) * S / te / 1e9, (double)calls * (k + t) * S / td / 1e9,
           1e3 * te / calls, 1e3 * td / calls, 1e3 * tn / calls, alg_new / tn / 1e9, bad ? "MISMATCH" : "ok");
    free(ers);
    free(perm);
    for (int c = 0; c < calls; ++c) seq_destroy(st[c]);
    rs_destroy(rs);
    return bad;
}
